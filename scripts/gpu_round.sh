# Full GPU suite, then the GBA / LBA / EG / ORB bench lines (one call).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
for cfg in gba lba eg orb; do
  timeout -k 10 600 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { tail -5 gpurun_out/bench_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_$cfg.json')); print('$cfg', round(d['value'],2), d['unit'], round(d['ms_per_step'],4))"
done
