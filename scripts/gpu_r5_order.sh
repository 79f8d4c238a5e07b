#!/bin/bash
# A/B: tile chain (9, 4, 3) on the context stream (ml), k_reduce before the
# camera-pass fork (rf), both (mlrf): bitwise check, interleaved bench pairs
# (config 4, loop-closed), a kernel trace of the best guess.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_order.log
: > $out
for v in ml rf mlrf; do
  timeout -k 10 300 python -u scripts/ab_bits.py libsqrtlm_$v.so 0.2 >> $out 2>&1 || exit 1
done
timeout -k 10 800 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_ml.so libsqrtlm_rf.so libsqrtlm_mlrf.so libsqrtlm.so libsqrtlm_ml.so libsqrtlm_rf.so libsqrtlm_mlrf.so libsqrtlm.so libsqrtlm_ml.so libsqrtlm_rf.so libsqrtlm_mlrf.so >> $out 2>&1 || exit 1
AB_ARGS="--config gba_loop" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_mlrf.so libsqrtlm.so libsqrtlm_mlrf.so >> $out 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_mlrf.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/orderprof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > /dev/null 2>&1 || exit 1
echo "all ok" >> $out
