#!/bin/bash
# Round-5 validation on MI355X: the full GPU suite (incl. the forced-timeout
# library), smoke, the default bench line, and a self-launched 2-rank
# host-transport rehearsal of bench.py --gpus 2 (all ranks on GPU 0).
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5a}
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_$tag.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$tag.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$tag.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --comm host --scale 0.2 --steps 10 --warmup 2 \
  > gpurun_out/bench_n2host_$tag.json 2> gpurun_out/bench_n2host_$tag.err || exit 1
echo done
