set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py::test_config4_full_size_two_iterations tests/test_eg_gpu.py::test_eg_bench_size_first_iteration -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|^E " gpurun_out/pytest_new.log | head -20; exit $rc
