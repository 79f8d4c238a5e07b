#!/bin/bash
# GPU-box helper: full -m gpu suite, then an interleaved A/B of library builds
# on config 2 (local BA) and config 4 (global BA).
# usage: gpurun --timeout 1200 -- 'bash scripts/gpu_ab_round.sh TAG base.so new.so'
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_${tag}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_${tag}.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  AB_ARGS="--config lba" timeout -k 10 200 python -u scripts/ab_bench.py "$@" >> gpurun_out/ab_lba_${tag}.log 2>&1 || exit $?
  timeout -k 10 200 python -u scripts/ab_bench.py "$@" >> gpurun_out/ab_gba_${tag}.log 2>&1 || exit $?
done
cat gpurun_out/ab_lba_${tag}.log gpurun_out/ab_gba_${tag}.log
