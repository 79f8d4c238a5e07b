#!/bin/bash
# GPU-box helper: rocprofv3 PMC passes of the config-4 bench (one counter group
# per run, as the hardware collects them), CSV under gpurun_out/pmc/<pass>/,
# then the per-kernel summary (scripts/pmc_summary.py) into gpurun_out/pmc_gba.json.
# usage: gpurun -- 'bash scripts/gpu_pmc.sh [bench args]'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
ARGS="--no-cpu-baseline --no-extras --steps 5 --warmup 1 $*"
run() {  # pass counters...
  local pass=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/$pass -o run \
    -- python -u bench.py $ARGS > gpurun_out/pmc/$pass.log 2>&1 || { echo "pass $pass failed"; exit 1; }
  echo "pass $pass done"
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY
n_obs=$(python -c "import sys; sys.path[:0]=['sqrtlm-slam_amd']; from sqrtlm import synth; print(synth.config4(seed=4).n_obs)")
python scripts/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_gba.json --workload gba --n-obs $n_obs
