# Essential graph by cyclic reduction: EG GPU tests, then the EG bench with CR (default) and the arrow Cholesky.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_eg_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/egcr_pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error" gpurun_out/egcr_pytest.log | tail -25; tail -3 gpurun_out/egcr_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  SQLM_EG_CR=$v timeout -k 10 300 python -u bench.py --config eg --no-cpu-baseline > gpurun_out/egcr_$v.json 2> gpurun_out/egcr_$v.err || { tail -5 gpurun_out/egcr_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/egcr_$v.json')); print('EG_CR=$v', round(d['value'],2), round(d['ms_per_step'],4))"
done
