#!/bin/bash
# A/B: every landmark-update bucket in one launch, the pose update fused in on
# small problems (libsqrtlm_um2.so): bitwise check (config 4 band / loop,
# config 2 local BA), interleaved bench pairs (local BA, config 4).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_um2.log
: > $out
timeout -k 10 400 python -u scripts/ab_bits.py libsqrtlm_um2.so 0.2 >> $out 2>&1 || exit 1
AB_ARGS="--config lba" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_um2.so libsqrtlm.so libsqrtlm_um2.so libsqrtlm.so libsqrtlm_um2.so libsqrtlm.so libsqrtlm_um2.so >> $out 2>&1 || exit 1
timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_um2.so libsqrtlm.so libsqrtlm_um2.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
