#!/bin/bash
# End of round 5: validation of the committed tree (GPU suite, smoke, bench,
# 2-rank rehearsal, kernel trace), then the PMC passes for the roofline's
# traffic (profiles/r05/pmc_gba.json).
set -o pipefail
tag=${1:-r5r}
bash scripts/gpu_r5_final.sh $tag || exit 1
bash scripts/gpu_pmc.sh || exit 1
echo end ok
