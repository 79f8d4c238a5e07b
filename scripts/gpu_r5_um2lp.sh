#!/bin/bash
set -o pipefail
bash scripts/gpu_r5_lp.sh || exit 1
bash scripts/gpu_r5_um2.sh || exit 1
