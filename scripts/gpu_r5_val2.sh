#!/bin/bash
# Round-5 validation of the current tree, then the tile camera-row padding A/B
# (libsqrtlm_nopad.so: rows of 16) against it and the round's first library
# (libsqrtlm_base.so), and a kernel trace of a short default bench.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5i}
bash scripts/gpu_r5_validate.sh $tag || exit 1
echo "bits nopad" > gpurun_out/ab_$tag.log
timeout -k 10 240 python -u scripts/ab_bits.py libsqrtlm_nopad.so 0.2 >> gpurun_out/ab_$tag.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/ab_bench.py libsqrtlm_base.so libsqrtlm_nopad.so libsqrtlm.so \
  libsqrtlm_base.so libsqrtlm_nopad.so libsqrtlm.so >> gpurun_out/ab_$tag.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof_$tag -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/kprof_bench_$tag.json 2> gpurun_out/kprof_bench_$tag.err || exit 1
echo done
