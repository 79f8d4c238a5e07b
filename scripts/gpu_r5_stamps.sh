#!/bin/bash
# Factor-chain stamps (cr_bench: per wave / step, and wave 0's diagonal groups)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/stamps_${1:-r5c}.log
: > $out
CRB_NO_LEVELS=1 timeout -k 10 60 ./tools/cr_bench 9 112 5 >> $out 2>&1 || exit 1
echo done
