set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_gba.json 2> gpurun_out/bench_gba.err || { tail -5 gpurun_out/bench_gba.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_gba.json')); print(round(d['value'],2), round(d['ms_per_step'],4), {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()})"
