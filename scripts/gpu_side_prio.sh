#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_concurrent.py tests/test_gpu_spec.py > gpurun_out/pytest_side_prio.log 2>&1 || { tail -5 gpurun_out/pytest_side_prio.log; exit 1; }
tail -2 gpurun_out/pytest_side_prio.log
bash scripts/gpu_ab_libs.sh libsqrtlm.so libsqrtlm.so:SQLM_SIDE_PRIO=normal
