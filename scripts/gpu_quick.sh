# GPU tests then the N=1 bench summary line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --no-cpu-baseline > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err; rc=$?; python3 -c "
import json; d=json.load(open('gpurun_out/bench_n1.json')); print(d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()})"; exit $rc
