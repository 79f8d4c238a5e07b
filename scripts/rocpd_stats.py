"""Kernel statistics from a rocprofv3 SQLite database (rocpd format, the
default output of rocprofv3 on ROCm 7): one CSV row per kernel name with
calls, total / average / min / max duration (ns) and the VGPR / LDS usage,
sorted by total time -- the same columns as rocprofv3's kernel_stats.csv.

usage: python scripts/rocpd_stats.py <run_results.db> [out.csv]
       python scripts/rocpd_stats.py <db> --trace FIRST LAST   (dispatch order)
"""
import csv
import sqlite3
import sys


def short(name: str) -> str:
    return name.split("(")[0].replace("sqlm::", "")


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, start, end, vgpr_count, accum_vgpr_count, lds_size, grid_x, workgroup_x "
                      "from kernels order by start").fetchall()
    if len(sys.argv) > 2 and sys.argv[2] == "--trace":
        a, b = int(sys.argv[3]), int(sys.argv[4])
        t0 = rows[a][1]
        for r in rows[a:b]:
            print(f"{(r[1] - t0) / 1000:9.2f} us  {(r[2] - r[1]) / 1000:8.2f} us  {short(r[0])}")
        return
    agg = {}
    for name, s, e, vg, ag, lds, gx, wx in rows:
        a = agg.setdefault(name, {"calls": 0, "total": 0, "min": None, "max": 0, "vgpr": vg, "agpr": ag,
                                  "lds": lds, "wg": gx // max(1, wx)})
        d = e - s
        a["calls"] += 1
        a["total"] += d
        a["min"] = d if a["min"] is None else min(a["min"], d)
        a["max"] = max(a["max"], d)
    tot = sum(a["total"] for a in agg.values()) or 1
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage", "VGPR", "AGPR",
                "LDS", "Workgroups"])
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["total"]):
        w.writerow([name, a["calls"], a["total"], round(a["total"] / a["calls"], 1), a["min"], a["max"],
                    round(100.0 * a["total"] / tot, 2), a["vgpr"], a["agpr"], a["lds"], a["wg"]])


if __name__ == "__main__":
    main()
