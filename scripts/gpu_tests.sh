#!/bin/bash
# GPU-box helper: pytest selection "$@" under a time limit, log under gpurun_out/.
# usage (from this container):
#   gpurun --timeout 900 -- 'bash scripts/gpu_tests.sh tests/test_gpu_loop.py -k small'
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${SQLM_TEST_TIMEOUT:-840} python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu "$@" \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
exit $rc
