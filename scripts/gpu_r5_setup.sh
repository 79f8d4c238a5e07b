#!/bin/bash
# Setup phases of the drop-in GBA call (config 4), current library.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5j}
SQLM_PREP_TIMING=1 REPS=4 timeout -k 10 300 python -u scripts/e2e_timing.py > gpurun_out/e2e_prep_$tag.log 2>&1 || exit 1
echo done
