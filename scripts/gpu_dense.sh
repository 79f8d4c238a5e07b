set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_stereo.py tests/test_capture.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_dense.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/pytest_dense.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config lba > gpurun_out/bench_lba.json 2> gpurun_out/bench_lba.err; rc=$?
cat gpurun_out/bench_lba.json; tail -2 gpurun_out/bench_lba.err; exit $rc
