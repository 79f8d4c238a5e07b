# Kernel trace of a short bench run (timestamps) to measure inter-kernel gaps.
set -o pipefail
mkdir -p gpurun_out/trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o tr -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/trace/log.txt 2>&1
echo rc=$?
find gpurun_out/trace -name "*.csv" | head
