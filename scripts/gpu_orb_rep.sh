# ORB bench twice (host-side variance check).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python -u bench.py --config orb --no-cpu-baseline > gpurun_out/orb_rep_$i.json 2> gpurun_out/orb_rep_$i.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/orb_rep_$i.json')); print(round(d['value'],1), round(d['stereo_two_extractors_frames_per_s'],1), {k: round(v*1000,1) for k,v in d['stage_ms'].items()})"
done
nproc; cat /proc/loadavg
