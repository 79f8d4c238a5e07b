#!/bin/bash
# Host launch cost vs kernel-argument size (tools/launch_probe), and the host
# trace of a local-BA trial (SQLM_HOST_TRACE=1: host us per trial phase).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/launch_probe.log
: > $out
timeout -k 10 60 ./tools/launch_probe >> $out 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 60 ./tools/launch_probe >> $out 2>&1 || exit 1
SQLM_HOST_TRACE=1 timeout -k 10 300 python -u bench.py --config lba --no-cpu-baseline --no-extras --steps 20 --warmup 3 >> $out 2>&1 || exit 1
SQLM_HOST_TRACE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 3 >> $out 2>&1 || exit 1
echo "all ok" >> $out
