# Kernel stats of the default bench command (with the CR first-level fusion) + one bench line with the CPU baseline.
set -o pipefail
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2/gba -o gba -- python3 bench.py --no-cpu-baseline > gpurun_out/prof2_gba.log 2>&1 || { echo "rocprof rc=$?"; tail -5 gpurun_out/prof2_gba.log; exit 1; }
find gpurun_out/prof2 -name "*kernel_stats.csv" | head -3
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -5 gpurun_out/bench_final.err; exit 1; }
cat gpurun_out/bench_final.json
