#!/bin/bash
# A/B: the trial mailbox published after a vmcnt wait (libsqrtlm_mb.so) vs
# after __threadfence_system (libsqrtlm.so); bitwise check and bench pairs.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_mb.log
: > $out
timeout -k 10 300 python -u scripts/ab_bits.py libsqrtlm_mb.so 0.2 >> $out 2>&1 || exit 1
timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_mb.so libsqrtlm.so libsqrtlm_mb.so libsqrtlm.so libsqrtlm_mb.so >> $out 2>&1 || exit 1
AB_ARGS="--config lba" timeout -k 10 300 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_mb.so libsqrtlm.so libsqrtlm_mb.so >> $out 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_mb.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mbprof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > /dev/null 2>&1 || exit 1
echo done
