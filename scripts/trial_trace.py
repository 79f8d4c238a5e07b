"""One LM trial's kernels from a rocprofv3 kernel trace (csv), every stream
merged by start time: start offset, duration, idle gap before it (us) -- from
the k_reduce (scalars for the host's decision) of one trial to the next
one's. Shows the host turnaround between trials (the gap after k_reduce). usage: python scripts/trial_trace.py run_kernel_trace.csv [k = index of the k_reduce, default -4]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_reduce(" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else -4
a, b = idx[k], idx[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
busy_end = t0
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("sqlm::", "").replace("void ", "")[:40]
    print(f"{(s - t0) / 1000:8.2f} {(e - s) / 1000:7.2f} gap {(s - busy_end) / 1000:6.2f}  {name}")
    busy_end = max(busy_end, e)
print(f"trial span {(int(rows[b]['Start_Timestamp']) - t0) / 1000:.1f} us")
