#!/bin/bash
# A/B: k_reduce with 8 strides of loads in flight and the published words
# requested up front (libsqrtlm_kr.so, same arithmetic order): bitwise check,
# interleaved pairs (config 4, local BA), kernel stats of the variant.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_kr.log
: > $out
timeout -k 10 400 python -u scripts/ab_bits.py libsqrtlm_kr.so 0.2 >> $out 2>&1 || exit 1
timeout -k 10 900 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_kr.so libsqrtlm.so libsqrtlm_kr.so libsqrtlm.so libsqrtlm_kr.so libsqrtlm.so libsqrtlm_kr.so >> $out 2>&1 || exit 1
AB_ARGS="--config lba" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_kr.so libsqrtlm.so libsqrtlm_kr.so libsqrtlm.so libsqrtlm_kr.so >> $out 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_kr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/krprof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > /dev/null 2>&1 || exit 1
echo "all ok" >> $out
