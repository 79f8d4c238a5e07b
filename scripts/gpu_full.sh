# Smoke, GPU test suite, then the default bench line; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err; rc=$?
cat gpurun_out/bench_n1.json; tail -3 gpurun_out/bench_n1.err; exit $rc
