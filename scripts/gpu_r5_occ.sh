#!/bin/bash
# A/B: camera pass compiled for 6 waves per SIMD (cam6), tile classes 5..6
# for 5 (tm5): interleaved pairs (config 4).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_occ.log
: > $out
timeout -k 10 900 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_cam6.so libsqrtlm_tm5.so libsqrtlm.so libsqrtlm_cam6.so libsqrtlm_tm5.so libsqrtlm.so libsqrtlm_cam6.so libsqrtlm_tm5.so >> $out 2>&1 || exit 1
echo "all ok" >> $out
