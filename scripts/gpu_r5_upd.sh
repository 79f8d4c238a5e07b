#!/bin/bash
# A/B: CR level update GEMM with 1 / 4 / 8 waves per workgroup (same items, same bits)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/upd_${1:-r5g}.log
: > $out
for rep in 1 2; do
for shape in "278 112" "9 112" "4 64"; do
  for b in cr_bench_u1 cr_bench cr_bench_u8; do
    echo -n "$b $shape " >> $out
    CRB_NO_LEVELS=1 timeout -k 10 60 ./tools/$b $shape 30 > gpurun_out/crb_tmp.log 2>&1
    rc=$?
    grep '"x_hash"' gpurun_out/crb_tmp.log >> $out
    [ $rc -eq 0 ] || { echo "rc=$rc" >> $out; tail -5 gpurun_out/crb_tmp.log >> $out; exit 1; }
  done
done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/updprof -o run -- ./tools/cr_bench 278 112 5 > /dev/null 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/updprof1 -o run -- ./tools/cr_bench_u1 278 112 5 > /dev/null 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/updprofs -o run -- ./tools/cr_bench_ts 278 112 5 > /dev/null 2>&1 || exit 1
timeout -k 5 60 ./tools/mfma_probe > gpurun_out/mfma_probe_r5.log 2>&1 || exit 1
echo done
