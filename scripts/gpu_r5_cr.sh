#!/bin/bash
# CR solve A/B on MI355X: the one-launch back substitution (k_cr_back_all)
# against one launch per level (CRB_LEVELS=1) -- same x_hash required -- then
# the CR/parity GPU tests and the default bench line, and a kernel trace.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5b}
out=gpurun_out/cr_ab_$tag.log
: > $out
for shape in "278 112" "4 64" "9 112" "2 112" "17 96" "3 48"; do
  for v in all levels; do
    if [ $v = levels ]; then export CRB_LEVELS=1; else unset CRB_LEVELS; fi
    echo -n "$v $shape " >> $out
    CRB_NO_LEVELS=1 timeout -k 10 60 ./tools/cr_bench $shape 30 > gpurun_out/crb_tmp.log 2>&1
    rc=$?
    grep '"x_hash"' gpurun_out/crb_tmp.log >> $out
    [ $rc -eq 0 ] || { echo "rc=$rc" >> $out; tail -5 gpurun_out/crb_tmp.log >> $out; exit 1; }
  done
done
unset CRB_LEVELS
cat $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_cr_fuse.py tests/test_gpu_fail_loud.py tests/test_gpu_spec.py tests/test_gpu_loop.py tests/test_gpu_sharded.py \
  > gpurun_out/pytest_cr_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_cr_$tag.log; exit 1; }
tail -2 gpurun_out/pytest_cr_$tag.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run -- python3 bench.py --no-cpu-baseline --no-extras --steps 20 > gpurun_out/prof_bench_$tag.json 2> gpurun_out/prof_$tag.err || exit 1
echo done
