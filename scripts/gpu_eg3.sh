set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_eg_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_eg.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_eg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config eg > gpurun_out/bench_eg.json 2> gpurun_out/bench_eg.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench_eg.json')); print(d['value'], d['ms_per_step'], d['cpu_baseline'])"
