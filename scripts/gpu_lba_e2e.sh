set -o pipefail
mkdir -p gpurun_out
SQLM_PREP_TIMING=1 timeout -k 10 300 python -u bench.py --config lba --no-cpu-baseline > gpurun_out/lba_e2e.json 2> gpurun_out/lba_e2e.err || { tail -5 gpurun_out/lba_e2e.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/lba_e2e.json')); print(round(d['value'],1), d.get('end_to_end'))"
grep prepare gpurun_out/lba_e2e.err | tail -8
