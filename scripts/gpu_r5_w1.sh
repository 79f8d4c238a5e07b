#!/bin/bash
# A/B: one lane per landmark for the shortest tracks (w1) vs two: parity
# tests on it, interleaved pairs (config 4, loop-closed, local BA).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_w1.log
: > $out
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_w1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_schedules.py >> $out 2>&1 || exit 1
timeout -k 10 800 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_w1.so libsqrtlm.so libsqrtlm_w1.so libsqrtlm.so libsqrtlm_w1.so >> $out 2>&1 || exit 1
AB_ARGS="--config gba_loop" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_w1.so libsqrtlm.so libsqrtlm_w1.so >> $out 2>&1 || exit 1
AB_ARGS="--config lba" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_w1.so libsqrtlm.so libsqrtlm_w1.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
