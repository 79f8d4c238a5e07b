#!/bin/bash
# A/B: CR level update with two waves per workgroup (u2w: a D tile's two
# products at once; bitwise equal expected) and the landmark kernels at half
# the lanes per landmark (uh: slot order unchanged, new Givens tree: parity
# tests instead of bits), interleaved pairs (config 4, local BA).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_u2.log
: > $out
timeout -k 10 400 python -u scripts/ab_bits.py libsqrtlm_u2w.so 0.2 >> $out 2>&1 || exit 1
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_uh.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_schedules.py >> $out 2>&1 || exit 1
timeout -k 10 1000 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_u2w.so libsqrtlm_uh.so libsqrtlm_ol4.so libsqrtlm.so libsqrtlm_u2w.so libsqrtlm_uh.so libsqrtlm_ol4.so libsqrtlm.so libsqrtlm_u2w.so libsqrtlm_uh.so libsqrtlm_ol4.so >> $out 2>&1 || exit 1
AB_ARGS="--config lba" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_u2w.so libsqrtlm_uh.so libsqrtlm.so libsqrtlm_u2w.so libsqrtlm_uh.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
