#!/bin/bash
# GPU-box helper: the default bench line for the in-tree library and for every
# A/B variant libsqrtlm_<tag>.so given on the command line (SQLM_LIB_PATH),
# interleaved twice, one JSON line each under gpurun_out/ab_<tag>_<rep>.json.
# usage: gpurun -- 'bash scripts/ab_bench.sh pre3 opl2' [extra bench.py args via BENCH_ARGS]
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for tag in base "$@"; do
    lib=sqrtlm-slam_amd/sqrtlm/libsqrtlm.so
    [ "$tag" != base ] && lib=sqrtlm-slam_amd/sqrtlm/libsqrtlm_$tag.so
    SQLM_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline $BENCH_ARGS \
      > gpurun_out/ab_${tag}_${rep}.json 2> gpurun_out/ab_${tag}_${rep}.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${tag}_${rep}.json')); print('$tag', round(d['value'],1), {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()})"
  done
done
