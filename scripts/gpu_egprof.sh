set -o pipefail
mkdir -p gpurun_out/prof_eg2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_eg2 -o eg -- python3 bench.py --config eg --no-cpu-baseline --steps 20 --warmup 1 > gpurun_out/prof_eg2/bench.json 2> gpurun_out/prof_eg2/err.log
