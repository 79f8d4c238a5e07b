#!/bin/bash
# A/B: tile classes on the three streams: default (8 | 6 | 9,4,3), to1
# (8 | 6,4 | 9,3), to2 (8,4 | 6 | 9,3): interleaved pairs (config 4, loop).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_to.log
: > $out
timeout -k 10 900 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_to1.so libsqrtlm_to2.so libsqrtlm.so libsqrtlm_to1.so libsqrtlm_to2.so libsqrtlm.so libsqrtlm_to1.so libsqrtlm_to2.so >> $out 2>&1 || exit 1
AB_ARGS="--config gba_loop" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_to1.so libsqrtlm_to2.so libsqrtlm.so libsqrtlm_to1.so libsqrtlm_to2.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
