#!/bin/bash
# GPU-box helper: CR microbenchmark A/B, full -m gpu suite, default bench line.
# usage: gpurun --timeout 1200 -- 'bash scripts/gpu_round.sh TAG'
set -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 5 60 ./tools/cr_bench 278 112 20 > gpurun_out/cr_${tag}.log 2>&1 || exit $?
SQLM_CR_LEGACY=1 timeout -k 5 60 ./tools/cr_bench 278 112 20 >> gpurun_out/cr_${tag}.log 2>&1 || exit $?
grep '"p"' gpurun_out/cr_${tag}.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_${tag}.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_${tag}.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err
rc=$?
tail -c 1500 gpurun_out/bench_${tag}.json
exit $rc
