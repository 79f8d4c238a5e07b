#!/bin/bash
# The one GPU-box driver (run from this container through gpurun):
#   gpurun --timeout 1200 -- 'bash scripts/gpu.sh MODE [args]'
# Every GPU step runs under its own time limit and the steps are chained so
# that the first failure ends the call. Output goes under gpurun_out/.
#
# modes
#   validate TAG        full -m gpu suite, smoke, the default bench line, a
#                       2-rank host-transport rehearsal of bench.py --gpus 2
#   prof TAG            rocprofv3 kernel trace + stats of the config-4 bench
#                       (--no-extras), the kernel stats as CSV and one trial's
#                       timeline
#   pmc                 the PMC passes of scripts/gpu_pmc.sh (config 4 only)
#   ab LIB[:VAR=V]...   interleaved config-4 A/B of library builds
#                       (scripts/ab_bench.py; AB_ARGS passes bench arguments,
#                       REPS the number of interleaved rounds, default 3)
#   bits LIB [SCALE]    bitwise A/B of a library build against the in-tree one
#   tests PYTEST_ARGS   a pytest -m gpu selection
#   lbatrace TAG        kernel trace of the config-2 local-BA bench, one trial
#   cr SHAPE...         tools/cr_bench on "p n" shapes (e.g. "278 112" "7 48")
set -o pipefail
mkdir -p gpurun_out
mode=$1
shift
prof_env() { cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1; }
case "$mode" in
validate)
  tag=${1:-run}
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$tag.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu_$tag.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit 1
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit 1
  timeout -k 10 300 python -u bench.py --gpus 2 --comm host --scale 0.2 --steps 10 --warmup 2 \
    > gpurun_out/bench_n2host_$tag.json 2> gpurun_out/bench_n2host_$tag.err || exit 1
  python scripts/bench_summary.py gpurun_out/bench_$tag.json
  ;;
prof)
  tag=${1:-run}
  prof_env
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof_$tag -o run \
    -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras \
    > gpurun_out/kprof_bench_$tag.json 2> gpurun_out/kprof_bench_$tag.err || exit 1
  db=$(find gpurun_out/kprof_$tag -name '*.db' | head -1)
  if [ -n "$db" ]; then
    python scripts/rocpd_stats.py "$db" gpurun_out/kstats_$tag.csv && \
      python scripts/trial_timeline.py "$db" > gpurun_out/trial_timeline_$tag.txt
  fi
  head -12 gpurun_out/kstats_$tag.csv 2>/dev/null
  ;;
pmc)
  bash scripts/gpu_pmc.sh "$@" || exit 1
  ;;
ab)
  out=gpurun_out/ab_${AB_TAG:-libs}.log
  : > $out
  for r in $(seq 1 ${REPS:-3}); do
    timeout -k 10 400 python -u scripts/ab_bench.py "$@" >> $out 2>&1 || { tail -20 $out; exit 1; }
  done
  cat $out
  ;;
e2e)
  # drop-in GBA call timing per library (setup phases on stderr), interleaved
  out=gpurun_out/e2e_${E2E_TAG:-ab}.log
  : > $out
  for r in $(seq 1 ${REPS:-2}); do
    for lib in "$@"; do
      echo "== $lib" >> $out
      SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/$lib SQLM_PREP_TIMING=1 REPS=4 \
        timeout -k 10 300 python -u scripts/e2e_timing.py >> $out 2>&1 || { tail -20 $out; exit 1; }
    done
  done
  grep -E "^==|^rep|median|obs\+camcsr|active\+sort" $out
  ;;
bits)
  timeout -k 10 400 python -u scripts/ab_bits.py "$@" > gpurun_out/ab_bits.log 2>&1 || { tail -20 gpurun_out/ab_bits.log; exit 1; }
  tail -20 gpurun_out/ab_bits.log
  ;;
tests)
  timeout -k 10 ${SQLM_TEST_TIMEOUT:-840} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -25 gpurun_out/pytest_gpu.log
  exit $rc
  ;;
lbatrace)
  tag=${1:-run}
  prof_env
  mkdir -p gpurun_out/lbatr_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lbatr_$tag -o run \
    -- python -u bench.py --config lba --no-cpu-baseline --no-extras --steps 20 --warmup 3 \
    > gpurun_out/lbatr_$tag/bench.json 2> gpurun_out/lbatr_$tag/bench.err || exit 1
  tr=$(find gpurun_out/lbatr_$tag -name '*kernel_trace.csv' | head -1)
  python scripts/trial_trace.py "$tr" > gpurun_out/lbatr_$tag/trial.txt && cat gpurun_out/lbatr_$tag/trial.txt
  ;;
cr)
  out=gpurun_out/cr_bench.log
  : > $out
  for shape in "$@"; do
    timeout -k 5 60 ./tools/cr_bench $shape 20 >> $out 2>&1 || { tail -20 $out; exit 1; }
  done
  grep '"p"' $out
  ;;
*)
  echo "unknown mode '$mode'" >&2
  exit 2
  ;;
esac
