# Speculative linearization: bitwise spec/plain tests, GBA parity, sharded tests, then the bench with and without.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -v --timeout 120 --timeout-method thread > gpurun_out/spec_pytest.log 2>&1; rc=$?
tail -30 gpurun_out/spec_pytest.log | grep -E "PASS|FAIL|Error|error|passed|failed" ; [ $rc -eq 0 ] || { tail -40 gpurun_out/spec_pytest.log; exit $rc; }
for ns in 0 1; do
  SQLM_NO_SPEC=$ns timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/spec_$ns.json 2> gpurun_out/spec_$ns.err || { tail -5 gpurun_out/spec_$ns.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/spec_$ns.json')); k=d['kernel_ms_per_step']; print('NO_SPEC=$ns', round(d['value'],2), round(d['ms_per_step'],4), {a: round(b,3) for a,b in k.items()})"
done
