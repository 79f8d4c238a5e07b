#!/bin/bash
# A/B: merged landmark-update buckets ordered by observations per block tile
# (uob) instead of by segment width: bitwise check, interleaved pairs.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_uob.log
: > $out
timeout -k 10 400 python -u scripts/ab_bits.py libsqrtlm_uob.so 0.2 >> $out 2>&1 || exit 1
timeout -k 10 900 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_uob.so libsqrtlm.so libsqrtlm_uob.so libsqrtlm.so libsqrtlm_uob.so libsqrtlm.so libsqrtlm_uob.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
