#!/bin/bash
# Host-setup change check: bitwise equal results against the round's first
# library (same plan, same kernels but the camera / landmark changes, which are
# themselves bit-identical), setup phases, and the GPU tests that build plans.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5l}
out=gpurun_out/setup_ab_$tag.log
: > $out
timeout -k 10 300 python -u scripts/ab_bits.py libsqrtlm_base.so 0.05 >> $out 2>&1 || exit 1
SQLM_PREP_TIMING=1 REPS=4 timeout -k 10 300 python -u scripts/e2e_timing.py > gpurun_out/e2e_prep_$tag.log 2>&1 || exit 1
grep "^rep\|median" gpurun_out/e2e_prep_$tag.log >> $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_sharded.py tests/test_gpu_spec.py tests/test_capture.py tests/test_stereo.py tests/test_gpu_loop.py >> $out 2>&1 || exit 1
echo "all ok" >> $out
