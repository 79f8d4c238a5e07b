#!/bin/bash
# A/B with the merged landmark update: observations per lane 3 (default) vs
# 4 / 2, and 1 observation preloaded instead of 2: interleaved pairs (config 4).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_ol.log
: > $out
timeout -k 10 1000 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_ol4.so libsqrtlm_pl1.so libsqrtlm_ol2.so libsqrtlm.so libsqrtlm_ol4.so libsqrtlm_pl1.so libsqrtlm_ol2.so libsqrtlm.so libsqrtlm_ol4.so libsqrtlm_pl1.so libsqrtlm_ol2.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
