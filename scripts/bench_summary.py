"""Key numbers of a bench.py JSON line: value, end-to-end, per-workload extras.
usage: python scripts/bench_summary.py gpurun_out/bench_X.json"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ex = d.pop("extra_workloads", {})
km = d.get("kernel_ms_per_step", {})
print("gba", round(d["value"], 1), "it/s | e2e", d.get("end_to_end"), "| tile", round(km.get("k_rcs_tile", 0), 4),
      "solve", round(km.get("k_solve", 0), 4), "lm_upd", round(km.get("k_landmark_update", 0), 4),
      "| roofline", round(d["roofline"]["frac"], 4))
for k, v in ex.items():
    kk = v.get("kernel_ms_per_step", {})
    print(k, round(v["value"], 1), "| e2e", v.get("end_to_end"), "| solve", round(kk.get("k_solve", 0), 4))
