"""One reduced-camera solve's kernel sequence from a rocprofv3 kernel trace
(csv): start offset, duration (us), kernel, grid -- from the k_rcs_reduce before
the second-to-last k_cr_gather to that gather.
usage: python scripts/solve_trace.py gpurun_out/prof_TAG/run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_cr_gather" in r["Kernel_Name"]]
last = idx[-2] if len(idx) > 1 else idx[-1]
start = last
while "k_rcs_reduce" not in rows[start]["Kernel_Name"]:
    start -= 1
t0 = int(rows[start]["Start_Timestamp"])
tot = {}
for r in rows[start:last + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("sqlm::", "").replace("void ", "")
    tot[name] = tot.get(name, 0.0) + (e - s) / 1000
    print(f"{(s - t0) / 1000:8.2f} {(e - s) / 1000:7.2f}  {name:32s} grid={r['Grid_Size_X']}")
print("solve span (after reduce): %.1f us" % ((int(rows[last]["End_Timestamp"]) - int(rows[start]["End_Timestamp"])) / 1000))
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {k:32s} {v:8.2f} us")
