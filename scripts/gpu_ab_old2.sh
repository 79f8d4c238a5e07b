#!/bin/bash
# A/B of the working tree's libsqrtlm.so against libsqrtlm_old.so (HEAD):
# bitwise results, then interleaved config-4 benches.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_old2.log
: > $out
timeout -k 10 300 python -u scripts/ab_bits.py libsqrtlm_old.so 0.05 >> $out 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_old.so >> $out 2>&1 || exit 1
done
echo "all ok" >> $out
