# ORB GPU parity tests, then the ORB bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_orb_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_orb.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_orb.log; exit $rc
