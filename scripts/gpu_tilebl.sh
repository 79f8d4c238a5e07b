# RCS tile batch width A/B: GBA parity tests, then the default bench with BL=8 (auto) and BL=4.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tilebl_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/tilebl_pytest.log; [ $rc -eq 0 ] || exit $rc
for bl in 8 4; do
  SQLM_TILE_BL=$bl timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/tilebl_$bl.json 2> gpurun_out/tilebl_$bl.err || { tail -5 gpurun_out/tilebl_$bl.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/tilebl_$bl.json')); print('BL $bl', round(d['value'],2), round(d['ms_per_step'],4), {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()}, d['roofline']['frac'])"
done
