# Full GPU suite with per-test lines (evidence log for profiles/).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_final.log; exit $rc
