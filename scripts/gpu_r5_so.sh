#!/bin/bash
# A/B: S partials stored in reduction order (libsqrtlm_so.so) vs per tile:
# bitwise check, interleaved bench pairs (config 4, loop-closed), kernel
# stats of the variant, then the whole GPU suite on it.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_so.log
: > $out
timeout -k 10 300 python -u scripts/ab_bits.py libsqrtlm_so.so 0.2 >> $out 2>&1 || exit 1
timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_so.so libsqrtlm.so libsqrtlm_so.so libsqrtlm.so libsqrtlm_so.so >> $out 2>&1 || exit 1
AB_ARGS="--config gba_loop" timeout -k 10 400 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_so.so libsqrtlm.so libsqrtlm_so.so >> $out 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_so.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/soprof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > /dev/null 2>&1 || exit 1
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_so.so timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ >> $out 2>&1 || exit 1
echo "all ok" >> $out
