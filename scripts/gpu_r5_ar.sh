#!/bin/bash
# Setup: small uploads through one arena copy (libsqrtlm_ar.so) vs the current
# library: bitwise check, LBA and GBA drop-in call timing (interleaved), the
# GPU tests that build plans (with the arena library as the product one).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_ar.log
: > $out
timeout -k 10 300 python -u scripts/ab_bits.py libsqrtlm_ar.so 0.05 >> $out 2>&1 || exit 1
for rep in 1 2; do
for lib in libsqrtlm.so libsqrtlm_ar.so; do
  echo "== $lib lba" >> $out
  SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/$lib REPS=6 timeout -k 10 120 python -u scripts/e2e_lba_timing.py 2>&1 | grep median >> $out || exit 1
  echo "== $lib gba" >> $out
  SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/$lib REPS=4 timeout -k 10 200 python -u scripts/e2e_timing.py 2>&1 | grep median >> $out || exit 1
done
done
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_ar.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_sharded.py tests/test_gpu_spec.py tests/test_capture.py tests/test_stereo.py tests/test_gpu_loop.py tests/test_gpu_schedules.py >> $out 2>&1 || exit 1
echo "all ok" >> $out
