#!/bin/bash
# Round-4 validation on MI355X: the factor with its pipe wave against the
# one-wave chain (same bits, cycles), forced-timeout build, focused GPU tests
# (schedules bit for bit, parity, spec, concurrent, EG vs glibc), and short
# A/B benches of the device-side LM loop + pose fusion.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r4_validate.log
: > $out
echo "== factor: pipe wave vs solo (x_hash must match)" >> $out
for shape in "278 112" "4 112" "9 112" "2 112" "17 96"; do
  for b in cr_bench cr_bench_solo cr_bench_nodeep; do
    echo "-- $b $shape" >> $out
    exe=$b; extra=""
    if [ $b = cr_bench_nodeep ]; then exe=cr_bench; extra="SQLM_NO_DEEP_BACK=1"; fi
    env $extra CRB_NO_LEVELS=1 timeout -k 10 60 ./tools/$exe $shape 20 > gpurun_out/crb_tmp.log 2>&1
    rc=$?
    grep -v "aug_wave\|aug_phase\|top_phase" gpurun_out/crb_tmp.log >> $out
    echo "rc=$rc" >> $out
    [ $rc -eq 0 ] || exit 1
  done
done
echo "== small bands: sequential one-launch solve vs cyclic reduction" >> $out
for shape in "4 64" "5 80" "3 48"; do
  for seqoff in 0 1; do
    echo "-- cr_bench $shape no_seq=$seqoff" >> $out
    if [ $seqoff = 1 ]; then export SQLM_NO_CR_SEQ=1; else unset SQLM_NO_CR_SEQ; fi
    CRB_NO_LEVELS=1 timeout -k 10 60 ./tools/cr_bench $shape 50 > gpurun_out/crb_tmp.log 2>&1
    rc=$?
    grep -v "aug_wave\|aug_phase\|top_phase" gpurun_out/crb_tmp.log >> $out
    echo "rc=$rc" >> $out
    [ $rc -eq 0 ] || exit 1
  done
done
unset SQLM_NO_CR_SEQ
timeout -k 10 60 ./tools/group_probe >> $out 2>&1 || exit 1
echo "== persistent all-levels CR (opt-in, SQLM_CR_PERSIST=1) on config 4's band" >> $out
SQLM_CR_PERSIST=1 timeout -k 10 120 ./tools/cr_bench 278 112 20 > gpurun_out/crb_tmp.log 2>&1
rc=$?
grep -v "aug_wave\|aug_phase\|top_phase" gpurun_out/crb_tmp.log >> $out
echo "rc=$rc" >> $out
echo "== forced timeout (expect flag 0, dev_err 1, rc 3)" >> $out
timeout -k 10 60 ./tools/cr_bench_tmo 9 112 2 2>&1 | grep -v "aug_wave\|aug_phase\|top_phase" >> $out; echo "tmo rc=$?" >> $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_cr_fuse.py "tests/test_gpu_parity.py::test_small_rcs_superblock_counts" tests/test_gpu_schedules.py tests/test_gpu_spec.py tests/test_gpu_parity.py \
  tests/test_gpu_concurrent.py tests/test_gpu_sharded.py \
  "tests/test_eg_gpu.py::test_eg_bench_size_first_iteration" > gpurun_out/pytest_r4.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out
tail -5 gpurun_out/pytest_r4.log >> $out
[ $rc -eq 0 ] || exit 1
for v in new base; do
  if [ $v = base ]; then export SQLM_DLM=1 SQLM_NO_POSE_FUSE=1; fi
  timeout -k 10 200 python -u bench.py --config lba --steps 200 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/bench_lba_$v.json 2> gpurun_out/bench_lba_$v.err || exit 1
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/bench_gba_$v.json 2> gpurun_out/bench_gba_$v.err || exit 1
done
unset SQLM_DLM SQLM_NO_POSE_FUSE
echo "all ok" >> $out
SQLM_PREP_TIMING=1 timeout -k 10 120 python -u bench.py --config lba --steps 50 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/bench_lba_prep.json 2> gpurun_out/bench_lba_prep.err || exit 1
SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/libsqrtlm_lm256.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/bench_gba_lm256.json 2> gpurun_out/bench_gba_lm256.err || exit 1
echo "lm256 done" >> $out
