#!/bin/bash
# The half-lane landmark buckets as the product path: whole GPU suite, then
# A/B vs a quarter-lane variant for W >= 8 (uq): parity tests on it,
# interleaved pairs (config 4, local BA).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_uq.log
: > $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ >> $out 2>&1 || exit 1
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_uq.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_spec.py >> $out 2>&1 || exit 1
timeout -k 10 800 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_uq.so libsqrtlm.so libsqrtlm_uq.so libsqrtlm.so libsqrtlm_uq.so >> $out 2>&1 || exit 1
AB_ARGS="--config gba_loop" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_uq.so libsqrtlm.so libsqrtlm_uq.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
