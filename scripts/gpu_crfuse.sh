# CR factor+elimination fusion: GBA parity / sharded / EG tests, then the bench fused vs unfused (A/B twice).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/crf_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/crf_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in fused unfused fused2 unfused2; do
  case $v in unfused*) export SQLM_CR_UNFUSED=1;; *) unset SQLM_CR_UNFUSED;; esac
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/crf_$v.json 2> gpurun_out/crf_$v.err || { tail -5 gpurun_out/crf_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/crf_$v.json')); k=d['kernel_ms_per_step']; print('$v', round(d['value'],2), round(d['ms_per_step'],4), d['chi2_last'], {a: round(b,3) for a,b in k.items()})"
done
