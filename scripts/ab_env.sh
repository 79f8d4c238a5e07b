#!/bin/bash
# GPU-box helper: the default bench line without and with each environment
# setting given (e.g. SQLM_PSTREAM=1), interleaved twice, one JSON line each
# under gpurun_out/abenv_<i>_<rep>.json.
# usage: gpurun -- 'bash scripts/ab_env.sh SQLM_PSTREAM=1' [extra bench.py args via BENCH_ARGS]
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for setting in "" "$@"; do
    env $setting timeout -k 10 200 python -u bench.py --no-cpu-baseline $BENCH_ARGS \
      > gpurun_out/abenv_${i}_${rep}.json 2> gpurun_out/abenv_${i}_${rep}.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/abenv_${i}_${rep}.json')); print('[${setting:-base}]', round(d['value'],1), {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()})"
    i=$((i+1))
  done
done
