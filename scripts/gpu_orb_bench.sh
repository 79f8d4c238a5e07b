# ORB bench line + rocprof kernel stats of the same command.
set -o pipefail
mkdir -p gpurun_out/prof_orb
timeout -k 10 300 python -u bench.py --config orb > gpurun_out/bench_orb.json 2> gpurun_out/bench_orb.err; rc=$?
cat gpurun_out/bench_orb.json; tail -3 gpurun_out/bench_orb.err; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_orb -o orb -- python3 bench.py --config orb --no-cpu-baseline > gpurun_out/prof_orb/bench.json 2> gpurun_out/prof_orb/err.log; rc=$?
find gpurun_out/prof_orb -name "*stats*" | head; exit $rc
