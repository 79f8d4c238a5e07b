#!/bin/bash
# cr_bench (working tree) vs cr_bench_base (HEAD): same solution hash, time.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/cr_ab2.log
: > $out
for r in 1 2; do
  for shape in "278 112" "139 112" "9 112"; do
    for b in cr_bench cr_bench_base; do
      printf "%-14s %-8s " $b "$shape" >> $out
      CRB_NO_LEVELS=1 timeout -k 5 60 ./tools/$b $shape 30 2>&1 | grep '"p"' >> $out || exit 1
    done
  done
done
echo "all ok" >> $out
