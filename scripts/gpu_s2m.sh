#!/bin/bash
# GPU-box helper (round 3): full -m gpu suite, bitwise A/B of the top-fused CR
# solve against the previous build, interleaved bench A/B (config 4, config 2
# with forced superblock widths), then the PMC passes of config 4.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_s2m.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s2m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_bits.py libsqrtlm_base.so 1.0 > gpurun_out/ab_bits_top.log 2>&1 || exit 1
tail -2 gpurun_out/ab_bits_top.log
timeout -k 10 300 python -u scripts/ab_bench.py libsqrtlm_base.so libsqrtlm.so > gpurun_out/ab_top_gba.log 2>&1 || exit 1
AB_ARGS="--config lba" timeout -k 10 400 python -u scripts/ab_bench.py libsqrtlm_base.so libsqrtlm.so libsqrtlm.so:SQLM_CR_B=8 \
  libsqrtlm.so:SQLM_CR_B=12 libsqrtlm.so:SQLM_CR_B=16 libsqrtlm.so:SQLM_CR_B=18 libsqrtlm.so > gpurun_out/ab_top_lba.log 2>&1 || exit 1
cut -c1-220 gpurun_out/ab_top_gba.log gpurun_out/ab_top_lba.log
bash scripts/gpu_pmc.sh --no-extras
