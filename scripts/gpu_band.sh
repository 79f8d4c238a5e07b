set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_capture.py tests/test_stereo.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_band.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_band.log; [ $rc -eq 0 ] || { grep -E "FAIL|^E " gpurun_out/pytest_band.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --config lba --no-cpu-baseline > gpurun_out/bench_lba.json 2> gpurun_out/bench_lba.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/bench_lba.json')); print(d['value'], d['ms_per_step'], {k: round(v,4) for k,v in d['kernel_ms_per_step'].items()})"
