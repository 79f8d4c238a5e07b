#!/usr/bin/env python3
"""Fold rocprofv3 --pmc passes into a per-kernel, per-launch summary.

Usage: pmc_summary.py <pmc_dir> <out.json> [--workload NAME --n-obs N]

<pmc_dir> holds the separate passes written by scripts/gpu_pmc.sh
(fetch/, write/, mfma/ each with *_counter_collection.csv). Corrections
follow MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE (KB) is doubled on
gfx950 (128-B requests tallied at 64 B); WRITE_SIZE (KB) is taken as is.
Both count memory-side L2 requests, Infinity-Cache hits included.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def _short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name.strip('"'))
    return name.replace("void ", "").replace("sqlm::", "")


def _read(pass_dir: str):
    files = glob.glob(os.path.join(pass_dir, "*counter_collection.csv"))
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> dispatch -> counter -> value
    for f in files:
        for r in csv.DictReader(open(f)):
            k = _short(r["Kernel_Name"])
            d = int(r["Dispatch_Id"])
            c = r["Counter_Name"]
            per[k][d][c] = per[k][d].get(c, 0.0) + float(r["Counter_Value"])
            per[k][d]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per


def summarize(pmc_dir: str) -> dict:
    out: dict = {}
    for pname in ("fetch", "write", "mfma", "sq"):
        pdir = os.path.join(pmc_dir, pname)
        if not os.path.isdir(pdir):
            continue
        for k, disp in _read(pdir).items():
            e = out.setdefault(k, {})
            n = len(disp)
            counters = sorted({c for v in disp.values() for c in v if c != "_ns"})
            for c in counters:
                e[c] = sum(v.get(c, 0.0) for v in disp.values()) / n
            e.setdefault("dispatches", n)
    for k, e in out.items():
        if "FETCH_SIZE" in e:
            e["fetch_bytes_corrected"] = 2.0 * e["FETCH_SIZE"] * 1024.0
        if "WRITE_SIZE" in e:
            e["write_bytes"] = e["WRITE_SIZE"] * 1024.0
        if "fetch_bytes_corrected" in e and "write_bytes" in e:
            e["traffic_bytes"] = e["fetch_bytes_corrected"] + e["write_bytes"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in e and "GRBM_GUI_ACTIVE" in e and e["GRBM_GUI_ACTIVE"] > 0:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA busy over 1024 SIMDs
            e["mfma_util"] = e["SQ_VALU_MFMA_BUSY_CYCLES"] / (e["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0)
    return out


def main():
    pmc_dir, dst = sys.argv[1], sys.argv[2]
    meta = {}
    a = sys.argv[3:]
    for i in range(0, len(a) - 1, 2):
        meta[a[i].lstrip("-").replace("-", "_")] = a[i + 1]
    res = {"meta": dict(meta, correction="FETCH_SIZE x2 (gfx950), KB x1024; per-launch averages"),
           "kernels": summarize(pmc_dir)}
    with open(dst, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k, e in sorted(res["kernels"].items(), key=lambda kv: -kv[1].get("traffic_bytes", 0))[:12]:
        print(f"{k:40s} n={e.get('dispatches')} traffic={e.get('traffic_bytes', 0)/1e6:9.1f} MB "
              f"fetch2x={e.get('fetch_bytes_corrected', 0)/1e6:9.1f} write={e.get('write_bytes', 0)/1e6:9.1f}")


if __name__ == "__main__":
    main()
