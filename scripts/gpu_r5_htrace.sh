#!/bin/bash
# Host-side cost of a trial's launches: the tile-launch sequence timed call by
# call (libsqrtlm_htr.so, -DSQLM_TILE_HTRACE), then a HIP API trace of a short
# bench with per-API statistics.
set -o pipefail
mkdir -p gpurun_out
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_htr.so SQLM_HOST_TRACE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 3 > gpurun_out/htr.json 2> gpurun_out/htr.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/hipprof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/hipprof.json 2> gpurun_out/hipprof.err || exit 1
echo done
