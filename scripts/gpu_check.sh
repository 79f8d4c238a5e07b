set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK
timeout -k 10 600 python -m pytest tests/ -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -30 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --config lba --no-cpu-baseline > gpurun_out/bench_lba.json 2> gpurun_out/bench_lba.err; echo "lba rc=$?"
timeout -k 10 400 python bench.py --config gba --no-cpu-baseline > gpurun_out/bench_gba.json 2> gpurun_out/bench_gba.err; echo "gba rc=$?"
cat gpurun_out/bench_lba.json gpurun_out/bench_gba.json; tail -5 gpurun_out/bench_gba.err
