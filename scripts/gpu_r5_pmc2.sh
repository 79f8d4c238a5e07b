#!/bin/bash
# PMC passes of the final tree (roofline traffic), then A/B: the mono
# landmark kernels compiled for 3 waves per SIMD instead of 4 (uo3).
set -o pipefail
bash scripts/gpu_pmc.sh || exit 1
out=gpurun_out/ab_uo3.log
: > $out
timeout -k 10 800 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_uo3.so libsqrtlm.so libsqrtlm_uo3.so libsqrtlm.so libsqrtlm_uo3.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
