#!/bin/bash
# End-of-round validation of the committed tree plus a kernel trace of the
# default bench (profiles/r05).
set -o pipefail
tag=${1:-r5n}
bash scripts/gpu_r5_validate.sh $tag || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof_$tag -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/kprof_bench_$tag.json 2> gpurun_out/kprof_bench_$tag.err || exit 1
echo done
