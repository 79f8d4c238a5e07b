#!/bin/bash
# Interleaved config-4 A/B of library builds: scripts/gpu_ab_libs.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_libs.log
: > $out
for r in 1 2 3; do
  timeout -k 10 400 python -u scripts/ab_bench.py "$@" >> $out 2>&1 || exit 1
done
echo "all ok" >> $out
