set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -40 gpurun_out/pytest_gpu.log
