#!/bin/bash
# A/B: per-bucket block cap of the per-landmark kernels 2048 (default) vs
# 4096 / 8192 now that the buckets share one launch: interleaved pairs.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_mg.log
: > $out
timeout -k 10 900 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_mg4k.so libsqrtlm_mg8k.so libsqrtlm.so libsqrtlm_mg4k.so libsqrtlm_mg8k.so libsqrtlm.so libsqrtlm_mg4k.so libsqrtlm_mg8k.so >> $out 2>&1 || exit 1
AB_ARGS="--config gba_loop" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_mg8k.so libsqrtlm.so libsqrtlm_mg8k.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
