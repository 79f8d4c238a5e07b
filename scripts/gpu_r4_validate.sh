#!/bin/bash
# Round-4 validation on MI355X: forced-timeout build, focused GPU tests
# (schedules bit for bit, parity, spec, concurrent, EG vs glibc), and short
# A/B benches of the device-side LM loop + pose fusion.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r4_validate.log
: > $out
echo "== forced timeout (expect flag 0, dev_err 1, rc 3)" >> $out
timeout -k 10 60 ./tools/cr_bench_tmo 9 112 2 2>&1 | grep -v "aug_wave\|aug_phase\|top_phase" >> $out; echo "tmo rc=$?" >> $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_schedules.py tests/test_gpu_spec.py tests/test_gpu_parity.py tests/test_gpu_concurrent.py tests/test_gpu_sharded.py \
  "tests/test_eg_gpu.py::test_eg_bench_size_first_iteration" > gpurun_out/pytest_r4.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out
tail -5 gpurun_out/pytest_r4.log >> $out
[ $rc -eq 0 ] || exit 1
for v in new base; do
  if [ $v = base ]; then export SQLM_NO_DLM=1 SQLM_NO_POSE_FUSE=1; fi
  timeout -k 10 200 python -u bench.py --config lba --steps 200 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/bench_lba_$v.json 2> gpurun_out/bench_lba_$v.err || exit 1
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/bench_gba_$v.json 2> gpurun_out/bench_gba_$v.err || exit 1
done
echo "all ok" >> $out
