# EG bench line (with CPU baseline) + rocprofv3 kernel stats of the same workload.
set -o pipefail
mkdir -p gpurun_out/prof_eg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 bench.py --config eg > gpurun_out/prof_eg/bench_full.json 2> gpurun_out/prof_eg/bench_full.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_eg -o eg -- python3 bench.py --config eg --no-cpu-baseline --steps 20 --warmup 1 > gpurun_out/prof_eg/bench.json 2> gpurun_out/prof_eg/err.log
rc=$?; cat gpurun_out/prof_eg/bench_full.json; find gpurun_out/prof_eg -name "*kernel_stats.csv"; exit $rc
