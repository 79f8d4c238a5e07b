#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/cr_debug.log
: > $out
echo "== A: persist only p=1 reps 3, no levels" >> $out
SQLM_CR_PERSIST=1 CRB_VERBOSE=1 CRB_NO_LEVELS=1 timeout -k 5 20 ./tools/cr_bench 1 112 3 >> $out 2>&1; echo "rc=$?" >> $out
echo "== B: persist p=1 reps 3 with levels after" >> $out
SQLM_CR_PERSIST=1 CRB_VERBOSE=1 timeout -k 5 20 ./tools/cr_bench 1 112 3 >> $out 2>&1; echo "rc=$?" >> $out
echo "== C: persist p=3 reps 3, no levels" >> $out
SQLM_CR_PERSIST=1 CRB_VERBOSE=1 CRB_NO_LEVELS=1 timeout -k 5 20 ./tools/cr_bench 3 112 3 >> $out 2>&1; echo "rc=$?" >> $out
echo "== D: persist p=278 reps 3, no levels" >> $out
SQLM_CR_PERSIST=1 CRB_VERBOSE=1 CRB_NO_LEVELS=1 timeout -k 5 20 ./tools/cr_bench 278 112 3 >> $out 2>&1; echo "rc=$?" >> $out
exit 0
