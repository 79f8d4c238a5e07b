#!/bin/bash
# A/B: the tile streams' fork recorded while the host waits for the previous
# trial's scalars (libsqrtlm_pf.so) vs at the trial's start (libsqrtlm.so).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_pf.log
: > $out
timeout -k 10 300 python -u scripts/ab_bits.py libsqrtlm_pf.so 0.2 >> $out 2>&1 || exit 1
timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_pf.so libsqrtlm.so libsqrtlm_pf.so libsqrtlm.so libsqrtlm_pf.so >> $out 2>&1 || exit 1
AB_ARGS="--config lba" timeout -k 10 300 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm_pf.so libsqrtlm.so libsqrtlm_pf.so >> $out 2>&1 || exit 1
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_pf.so SQLM_HOST_TRACE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 3 > /dev/null 2>> $out || exit 1
echo done
