"""Per-kernel durations of the last full CR solve in a rocprofv3 kernel trace of tools/cr_bench."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/crtrace/cr_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
names = [r['Kernel_Name'].split('(')[0].replace('sqlm::', '') for r in rows]
facs = [i for i, n in enumerate(names) if n.startswith('k_cr_factor')]
# start of the last solve: the first factor after the second-to-last k_cr_top
tops = [i for i, n in enumerate(names) if n.startswith('k_cr_top')]
s = min(i for i in facs if i > tops[-2])
e = max(i for i, n in enumerate(names) if n.startswith('k_cr_back'))
tot = defaultdict(float)
for i in range(s, e + 1):
    d = (int(rows[i]['End_Timestamp']) - int(rows[i]['Start_Timestamp'])) / 1000
    tot[names[i]] += d
    print(f"{names[i][:22]:22s} {d:7.2f} us")
print({k: round(v, 1) for k, v in tot.items()}, 'span us',
      (int(rows[e]['End_Timestamp']) - int(rows[s]['Start_Timestamp'])) / 1000)
