#!/bin/bash
# PMC passes over the CR solve alone (tools/cr_bench 278 112): the wide-level
# update GEMM and TRSM, the factor, back substitution. One counter group per run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/crpmc
run() {
  local pass=$1; shift
  CRB_NO_LEVELS=1 timeout -s KILL 60 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/crpmc/$pass -o run \
    -- ./tools/cr_bench 278 112 5 > gpurun_out/crpmc/$pass.log 2>&1 || { echo "pass $pass failed"; exit 1; }
  echo "pass $pass done"
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
run fetch FETCH_SIZE TCC_HIT_sum
run miss TCC_MISS_sum WRITE_SIZE
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/crpmc/trace -o run -- ./tools/cr_bench 278 112 5 > gpurun_out/crpmc/trace.log 2>&1 || exit 1
echo done
