#!/bin/bash
# Round-4 A/B on MI355X: device-side LM loop and pose fusion, local BA and
# config 4, interleaved (two rounds), after the build under test.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r4_ab.log
: > $out
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || return 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['value'],1), 'it/s', round(d['ms_per_step']*1e3,1), 'us/step', d.get('trials_per_step'), 'trials/step', {k: round(v*1e3,1) for k,v in d.get('kernel_ms_per_step',{}).items()})" >> $out
}
B="timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras"
for r in 1 2; do
  run lba_def$r $B --config lba --steps 300 --warmup 20 || exit 1
  run lba_dlm$r SQLM_DLM=1 $B --config lba --steps 300 --warmup 20 || exit 1
  run lba_nofuse$r SQLM_NO_POSE_FUSE=1 $B --config lba --steps 300 --warmup 20 || exit 1
  run lba_none$r SQLM_DLM=1 SQLM_NO_POSE_FUSE=1 $B --config lba --steps 300 --warmup 20 || exit 1
done
for r in 1 2; do
  run gba_def$r $B --steps 20 --warmup 3 || exit 1
  run gba_dlm$r SQLM_DLM=1 $B --steps 20 --warmup 3 || exit 1
done
echo "all ok" >> $out
