set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --config lba --steps 20 --warmup 3 > gpurun_out/bench_lba.json 2> gpurun_out/bench_lba.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/lba -o lba -- python3 bench.py --config lba --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_lba.log 2>&1
echo rc=$?
cat gpurun_out/bench_lba.json
