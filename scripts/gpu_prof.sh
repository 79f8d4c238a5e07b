set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/ -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/gba -o gba -- python3 bench.py --config gba --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_gba.log 2>&1
echo rc=$?
grep -o '"value": [0-9.]*' gpurun_out/prof_gba.log
