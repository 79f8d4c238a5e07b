set -o pipefail
mkdir -p gpurun_out/prof_eg
timeout -k 10 600 python -u -m pytest tests/test_eg_gpu.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_eg.log 2>&1; rc=$?
grep -E "passed|failed|FAIL" gpurun_out/pytest_eg.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config eg > gpurun_out/bench_eg.json 2> gpurun_out/bench_eg.err || exit 1
cat gpurun_out/bench_eg.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_eg -o eg -- python3 bench.py --config eg --no-cpu-baseline --steps 20 --warmup 1 > gpurun_out/prof_eg/bench.json 2> gpurun_out/prof_eg/err.log
