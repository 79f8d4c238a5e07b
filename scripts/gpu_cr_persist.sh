#!/bin/bash
# Persistent cyclic-reduction solve on MI355X: bit-identity with the per-level
# launches, residual, timing (tools/cr_bench), and the forced-timeout build.
set -o pipefail
export SQLM_CR_PERSIST=1
mkdir -p gpurun_out
out=gpurun_out/cr_persist.log
: > $out
for pn in "1 112" "2 112" "3 112" "4 64" "5 112" "7 48" "8 112" "9 112" "16 112" "33 112" "4 112" "278 112"; do
  set -- $pn
  echo "== p=$1 n=$2" >> $out
  timeout -k 10 60 ./tools/cr_bench $1 $2 10 >> $out 2>&1 || { echo "FAILED rc=$? p=$1 n=$2" >> $out; exit 1; }
done
echo "== levels A/B p=278" >> $out
SQLM_CR_PERSIST=0 timeout -k 10 60 ./tools/cr_bench 278 112 20 >> $out 2>&1 || exit 1
timeout -k 10 60 ./tools/cr_bench 278 112 20 >> $out 2>&1 || exit 1
echo "== forced timeout" >> $out
timeout -k 10 60 ./tools/cr_bench_tmo 9 112 2 >> $out 2>&1; echo "tmo rc=$?" >> $out

# focused GPU tests of this change (persistent solve inside the LM loop)
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_cr_fuse.py \
  "tests/test_eg_gpu.py::test_eg_bench_size_first_iteration" > gpurun_out/pytest_persist.log 2>&1
echo "pytest rc=$?" >> $out
