#!/bin/bash
# A/B: the pose update folded into the back-substitution launch
# (libsqrtlm_pf.so): bitwise check, the launch-schedule test on it,
# interleaved bench pairs (config 4).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_pf2.log
: > $out
timeout -k 10 400 python -u scripts/ab_bits.py libsqrtlm_pf.so 0.2 >> $out 2>&1 || exit 1
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_pf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_schedules.py >> $out 2>&1 || exit 1
timeout -k 10 900 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_pf.so libsqrtlm.so libsqrtlm_pf.so libsqrtlm.so libsqrtlm_pf.so libsqrtlm.so libsqrtlm_pf.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
