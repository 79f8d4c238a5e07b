#!/bin/bash
# GPU-box helper: rocprofv3 kernel trace + stats of a short bench run.
# usage: gpurun -- 'bash scripts/gpu_prof.sh TAG [bench args]'
# -> gpurun_out/prof_TAG/ (csv), gpurun_out/kstats_TAG.csv (per-kernel stats)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run \
  -- python -u bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 1 "$@" \
  > gpurun_out/prof_$tag/bench.json 2> gpurun_out/prof_$tag/bench.err || exit $?
st=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1)
cp "$st" gpurun_out/kstats_$tag.csv
head -30 gpurun_out/kstats_$tag.csv | cut -c1-160
