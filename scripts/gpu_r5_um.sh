#!/bin/bash
# A/B: every landmark-update bucket in one launch (libsqrtlm_um.so, heaviest
# bucket first) vs one launch per bucket: bitwise check, interleaved bench
# pairs (config 4, loop-closed), a kernel trace of the variant.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_um.log
: > $out
timeout -k 10 300 python -u scripts/ab_bits.py libsqrtlm_um.so 0.2 >> $out 2>&1 || exit 1
timeout -k 10 800 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_um.so libsqrtlm.so libsqrtlm_um.so libsqrtlm.so libsqrtlm_um.so libsqrtlm.so libsqrtlm_um.so >> $out 2>&1 || exit 1
AB_ARGS="--config gba_loop" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_um.so libsqrtlm.so libsqrtlm_um.so >> $out 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_um.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/umprof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > /dev/null 2>&1 || exit 1
echo "all ok" >> $out
