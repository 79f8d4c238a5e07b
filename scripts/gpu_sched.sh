#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_schedules.py > gpurun_out/pytest_sched.log 2>&1
echo "rc=$?" >> gpurun_out/pytest_sched.log
exit 0
