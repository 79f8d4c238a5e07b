# Landmarks per RCS tile sweep: GBA parity tests at the default, then bench at several caps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tilelm_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/tilelm_pytest.log; [ $rc -eq 0 ] || exit $rc
for lm in 128 192 256 384 512; do
  SQLM_TILE_LM=$lm timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/tilelm_$lm.json 2> gpurun_out/tilelm_$lm.err || { tail -5 gpurun_out/tilelm_$lm.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/tilelm_$lm.json')); k=d['kernel_ms_per_step']; print('LM $lm', round(d['value'],2), round(d['ms_per_step'],4), 'tile', round(k['k_rcs_tile'],3), 'reduce', round(k['k_rcs_reduce'],3), 'frac', round(d['roofline']['frac'],3))"
done
