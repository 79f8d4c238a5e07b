#!/bin/bash
# CR factor A/B (tools/cr_bench builds of the same source): solution hash must
# match; best / average ms per solve, two interleaved rounds; stamps.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/cr_ab.log
: > $out
for r in 1 2; do
  for shape in "278 112" "4 64" "9 112" "2 112"; do
    for b in cr_bench cr_bench_nosleep cr_bench_solo; do
      printf "%-18s %-8s " $b "$shape" >> $out
      CRB_NO_LEVELS=1 timeout -k 5 60 ./tools/$b $shape 30 2>&1 | grep '"p"' >> $out || exit 1
    done
  done
done
CRB_NO_LEVELS=1 timeout -k 5 60 ./tools/cr_bench 9 112 5 > gpurun_out/crb_stamps3.log 2>&1 || exit 1
timeout -k 5 60 ./tools/cr_bench_tmo 9 112 2 2>&1 | grep '"p"' >> $out; echo "tmo rc=$?" >> $out
echo "all ok" >> $out
