#!/bin/bash
# A/B: tile class 8 launched on the context stream before the side streams'
# fork waits are enqueued (libsqrtlm_f8.so): bitwise check, interleaved pairs.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_f8.log
: > $out
timeout -k 10 400 python -u scripts/ab_bits.py libsqrtlm_f8.so 0.2 >> $out 2>&1 || exit 1
timeout -k 10 900 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_f8.so libsqrtlm.so libsqrtlm_f8.so libsqrtlm.so libsqrtlm_f8.so libsqrtlm.so libsqrtlm_f8.so >> $out 2>&1 || exit 1
AB_ARGS="--config gba_loop" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_f8.so libsqrtlm.so libsqrtlm_f8.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
