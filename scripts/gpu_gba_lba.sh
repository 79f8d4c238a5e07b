# GBA parity/spec/sharded/stereo/capture tests, then the GBA and LBA bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_stereo.py tests/test_capture.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gl_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/gl_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|^E " gpurun_out/gl_pytest.log | head; exit $rc; }
for c in gba lba; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/gl_$c.json 2> gpurun_out/gl_$c.err || { tail -5 gpurun_out/gl_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/gl_$c.json')); k=d['kernel_ms_per_step']; print('$c', round(d['value'],2), round(d['ms_per_step'],4), {a: round(b,3) for a,b in k.items()})"
done
