#!/bin/bash
# The merged landmark update as the product path: bitwise vs the previous tree
# (libsqrtlm_head.so), kernel arguments in host memory (HIP_FORCE_DEV_KERNARG=0)
# vs the default device-memory kernargs, interleaved (local BA, config 4),
# then the whole GPU suite.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_ka.log
: > $out
timeout -k 10 400 python -u scripts/ab_bits.py libsqrtlm_head.so 0.2 >> $out 2>&1 || exit 1
AB_ARGS="--config lba" timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm.so libsqrtlm.so:HIP_FORCE_DEV_KERNARG=0 libsqrtlm.so libsqrtlm.so:HIP_FORCE_DEV_KERNARG=0 libsqrtlm.so libsqrtlm.so:HIP_FORCE_DEV_KERNARG=0 >> $out 2>&1 || exit 1
timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm_head.so libsqrtlm.so libsqrtlm.so:HIP_FORCE_DEV_KERNARG=0 libsqrtlm_head.so libsqrtlm.so libsqrtlm.so:HIP_FORCE_DEV_KERNARG=0 >> $out 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ >> $out 2>&1 || exit 1
echo "all ok" >> $out
