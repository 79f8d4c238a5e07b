set -o pipefail
mkdir -p gpurun_out/trace_lba
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_lba -o tr -- python3 bench.py --config lba --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/trace_lba/log.txt 2>&1
echo rc=$?
