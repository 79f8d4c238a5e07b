#!/bin/bash
# A/B: the CR solve compiled with -mllvm -amdgpu-mfma-vgpr-form (MFMA
# accumulators in VGPRs, no AGPR copies) vs the default heuristics; same bits.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/vf_${1:-r5f}.log
: > $out
for rep in 1 2; do
for shape in "278 112" "9 112" "4 64" "17 96"; do
  for b in cr_bench cr_bench_vf; do
    echo -n "$b $shape " >> $out
    CRB_NO_LEVELS=1 timeout -k 10 60 ./tools/$b $shape 30 > gpurun_out/crb_tmp.log 2>&1
    rc=$?
    grep '"x_hash"' gpurun_out/crb_tmp.log >> $out
    [ $rc -eq 0 ] || { echo "rc=$rc" >> $out; tail -5 gpurun_out/crb_tmp.log >> $out; exit 1; }
  done
done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/vfprof -o run -- ./tools/cr_bench_vf 278 112 5 > /dev/null 2>&1 || exit 1
echo done
