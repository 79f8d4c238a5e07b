#!/bin/bash
# A/B: kernels read DevProblem through its device copy (libsqrtlm_dp.so) vs by
# value: bitwise check, interleaved bench pairs (config 4, local BA), the LBA
# drop-in call, and the GPU tests that exercise every schedule (arena library).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_dp.log
: > $out
timeout -k 10 300 python -u scripts/ab_bits.py libsqrtlm_dp.so 0.2 >> $out 2>&1 || exit 1
timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_dp.so libsqrtlm.so libsqrtlm_dp.so libsqrtlm.so libsqrtlm_dp.so >> $out 2>&1 || exit 1
AB_ARGS="--config lba" timeout -k 10 300 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_dp.so libsqrtlm.so libsqrtlm_dp.so libsqrtlm.so libsqrtlm_dp.so >> $out 2>&1 || exit 1
for lib in libsqrtlm.so libsqrtlm_dp.so libsqrtlm.so libsqrtlm_dp.so; do
  echo "== $lib lba call" >> $out
  SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/$lib REPS=6 timeout -k 10 120 python -u scripts/e2e_lba_timing.py 2>&1 | grep median >> $out || exit 1
done
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_dp.so timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ >> $out 2>&1 || exit 1
echo "all ok" >> $out
