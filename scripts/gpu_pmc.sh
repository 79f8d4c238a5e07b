# Full bench line + rocprofv3 evidence for profiles/: stats pass, then the PMC
# passes kept separate (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err && echo bench_ok && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/stats -o stats -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/pmc/stats.log 2>&1 && echo stats_ok && \
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o fetch -- $B > gpurun_out/pmc/fetch.log 2>&1 && echo fetch_ok && \
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o write -- $B > gpurun_out/pmc/write.log 2>&1 && echo write_ok && \
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc/mfma -o mfma -- $B > gpurun_out/pmc/mfma.log 2>&1 && echo mfma_ok && \
NOBS=$(python3 -c "import json;print(json.load(open('gpurun_out/bench_full.json'))['config']['n_obs'])") && \
python3 scripts/pmc_summary.py gpurun_out/pmc gpurun_out/pmc/pmc_gba.json --workload gba --n-obs $NOBS
cat gpurun_out/bench_full.json
