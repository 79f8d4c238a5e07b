set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/cr_bench 1 112 5 > gpurun_out/cr_prof.json 2>&1; rc=$?; cat gpurun_out/cr_prof.json; exit $rc
