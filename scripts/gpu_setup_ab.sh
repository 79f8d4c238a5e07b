#!/bin/bash
# Host-setup change check: results bitwise equal to libsqrtlm_old.so, setup
# phase times, and the GPU tests that build plans from shuffled / multi-level
# edge lists.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/setup_ab.log
: > $out
timeout -k 10 300 python -u scripts/ab_bits.py libsqrtlm_old.so 0.05 >> $out 2>&1 || exit 1
SQLM_PREP_TIMING=1 timeout -k 10 300 python -u scripts/e2e_timing.py > gpurun_out/e2e_prep_r4c.log 2>&1 || exit 1
grep "^rep" gpurun_out/e2e_prep_r4c.log >> $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_sharded.py tests/test_gpu_spec.py tests/test_capture.py tests/test_stereo.py tests/test_gpu_loop.py >> $out 2>&1 || exit 1
echo "all ok" >> $out
