#!/bin/bash
# A/B: tile windows capped at 21 cameras (libsqrtlm_mc21.so: no 9-tile class)
# vs 24; interleaved bench pairs, then the GPU parity tests on the variant.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_mc.log
: > $out
timeout -k 10 700 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_mc21.so libsqrtlm.so libsqrtlm_mc21.so libsqrtlm.so libsqrtlm_mc21.so >> $out 2>&1 || exit 1
AB_ARGS="--config gba_loop" timeout -k 10 400 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_mc21.so libsqrtlm.so libsqrtlm_mc21.so >> $out 2>&1 || exit 1
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_mc21.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_loop.py >> $out 2>&1 || exit 1
echo "all ok" >> $out
