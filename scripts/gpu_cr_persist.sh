#!/bin/bash
# Persistent cyclic-reduction solve + device-side LM loop on MI355X:
# bit-identity with the per-level launches, residual, timing (tools/cr_bench),
# the forced-timeout build, focused GPU tests, and short benches.
set -o pipefail
export SQLM_CR_PERSIST=1
mkdir -p gpurun_out
out=gpurun_out/cr_persist.log
: > $out
for pn in "1 112" "2 112" "3 112" "4 64" "5 112" "7 48" "8 112" "9 112" "16 112" "33 112" "4 112" "278 112"; do
  set -- $pn
  echo "== p=$1 n=$2" >> $out
  timeout -k 10 60 ./tools/cr_bench $1 $2 10 > gpurun_out/crb.tmp 2>&1; rc=$?
  grep -v "aug_wave\|aug_phase\|top_phase" gpurun_out/crb.tmp >> $out
  [ $rc -eq 0 ] || { echo "FAILED rc=$rc p=$1 n=$2" >> $out; exit 1; }
done
echo "== levels A/B p=278" >> $out
SQLM_CR_PERSIST=0 timeout -k 10 60 ./tools/cr_bench 278 112 20 2>&1 | grep -v "aug_wave\|aug_phase\|top_phase" >> $out || exit 1
timeout -k 10 60 ./tools/cr_bench 278 112 20 2>&1 | grep -v "aug_wave\|aug_phase\|top_phase" >> $out || exit 1
echo "== forced timeout" >> $out
timeout -k 10 60 ./tools/cr_bench_tmo 9 112 2 2>&1 | grep -v "aug_wave\|aug_phase\|top_phase" >> $out; echo "tmo rc=$?" >> $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_schedules.py tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_cr_fuse.py tests/test_gpu_concurrent.py \
  "tests/test_eg_gpu.py::test_eg_bench_size_first_iteration" > gpurun_out/pytest_persist.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --config lba --steps 200 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/bench_lba.json 2> gpurun_out/bench_lba.err || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/bench_gba.json 2> gpurun_out/bench_gba.err || exit 1
SQLM_CR_PERSIST=0 SQLM_NO_DLM=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/bench_gba_base.json 2>> gpurun_out/bench_gba.err || exit 1
SQLM_CR_PERSIST=0 SQLM_NO_DLM=1 timeout -k 10 200 python -u bench.py --config lba --steps 200 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/bench_lba_base.json 2>> gpurun_out/bench_lba.err || exit 1
echo "all ok" >> $out
