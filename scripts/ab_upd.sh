#!/bin/bash
# GPU-box helper: k_landmark_update time (sum of its buckets, rocprof) for library variants.
# usage: bash scripts/ab_upd.sh lib1.so lib2.so ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for lib in "$@"; do
  out=gpurun_out/abupd_${lib%.so}
  mkdir -p $out
  SQLM_LIB_PATH=$PWD/sqrtlm-slam_amd/sqrtlm/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
    -- python -u bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 1 > $out/bench.json 2> $out/bench.err || exit 1
  st=$(find $out -name '*kernel_stats.csv' | head -1)
  python - "$st" "$lib" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = {}
for r in rows:
    n = r["Name"]
    for k in ("k_landmark_update", "k_rcs_tile", "k_linearize", "k_camera_pass"):
        if k in n:
            tot[k] = tot.get(k, 0.0) + float(r["TotalDurationNs"]) / int(r["Calls"]) * 1e-3
print(sys.argv[2], {k: round(v, 1) for k, v in tot.items()}, "(us per call summed over buckets)")
PY
done
