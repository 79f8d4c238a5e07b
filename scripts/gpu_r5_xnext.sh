#!/bin/bash
# A/B of the diagonal wave's next pivot block (SQLM_AUG_XNEXT 1 vs 0), interleaved
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/xnext_${1:-r5e}.log
: > $out
for rep in 1 2; do
for shape in "278 112" "9 112" "4 64" "2 112" "17 96"; do
  for b in cr_bench cr_bench_x0; do
    echo -n "$b $shape " >> $out
    CRB_NO_LEVELS=1 timeout -k 10 60 ./tools/$b $shape 30 > gpurun_out/crb_tmp.log 2>&1
    rc=$?
    grep '"x_hash"' gpurun_out/crb_tmp.log >> $out
    if [ $rep = 1 ] && [ "$shape" = "9 112" ]; then grep "w0_groups_2\|aug_phase_cycles_level_wg0\"" gpurun_out/crb_tmp.log >> $out; fi
    [ $rc -eq 0 ] || { echo "rc=$rc" >> $out; tail -5 gpurun_out/crb_tmp.log >> $out; exit 1; }
  done
done
done
echo done
