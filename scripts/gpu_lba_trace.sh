#!/bin/bash
# GPU-box helper: kernel trace of the config-2 local-BA bench and one trial's
# kernels / idle gaps (scripts/trial_trace.py), plus the host-side trace.
# usage: gpurun -- 'bash scripts/gpu_lba_trace.sh TAG'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1
mkdir -p gpurun_out/lbatr_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lbatr_$tag -o run \
  -- python -u bench.py --config lba --no-cpu-baseline --no-extras --steps 20 --warmup 3 \
  > gpurun_out/lbatr_$tag/bench.json 2> gpurun_out/lbatr_$tag/bench.err || exit $?
tr=$(find gpurun_out/lbatr_$tag -name '*kernel_trace.csv' | head -1)
python scripts/trial_trace.py "$tr" > gpurun_out/lbatr_$tag/trial.txt && cat gpurun_out/lbatr_$tag/trial.txt
SQLM_HOST_TRACE=1 timeout -k 10 120 python -u bench.py --config lba --no-cpu-baseline --no-extras --steps 20 --warmup 3 \
  > gpurun_out/lbatr_$tag/host.json 2> gpurun_out/lbatr_$tag/host.err
grep "host trace" gpurun_out/lbatr_$tag/host.err | tail -3
