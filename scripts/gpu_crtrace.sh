set -o pipefail
mkdir -p gpurun_out/crtrace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 ./tools/cr_bench 1 112 3 | head -1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/crtrace -o cr -- ./tools/cr_bench 278 112 5 > gpurun_out/crtrace/log.txt 2>&1; rc=$?; tail -1 gpurun_out/crtrace/log.txt; exit $rc
