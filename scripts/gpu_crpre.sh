# k_cr_factor_elim with the first E strip loaded before the factor: parity tests, then three bench runs (k_solve, chi2_last).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cr_fuse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/crp_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/crp_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in a b c; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/crp_$v.json 2> gpurun_out/crp_$v.err || { tail -5 gpurun_out/crp_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/crp_$v.json')); k=d['kernel_ms_per_step']; print('$v', round(d['value'],2), round(d['ms_per_step'],4), repr(d['chi2_last']), round(k['k_solve'],4))"
done
