#!/usr/bin/env python3
"""Dispatch-size profile of each ai-benchmark test (rocprofv3 kernel traces):
the GPU-time-weighted distribution of workgroups per dispatch, i.e. how much of
a workload's GPU time runs in kernels too small to fill the 256 CUs of an
MI355X.  Input: one directory per test id, as written by scripts/kernel_sizes.sh.

    python scripts/kernel_sizes.py gpurun_out/ksize [--tail 0.5]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def dims(row: dict, prefix: str) -> int:
    if prefix in row and row[prefix]:
        return int(float(row[prefix]))
    v = 1
    for ax in ("X", "Y", "Z"):
        k = f"{prefix}_{ax}"
        if row.get(k):
            v *= max(1, int(float(row[k])))
    return v


def summarize(files: list[str], tail: float) -> dict:
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    if not rows:
        return {}
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[int(len(rows) * (1 - tail)):]
    tot = 0.0
    small = {64: 0.0, 256: 0.0, 512: 0.0, 1024: 0.0}
    cnt_small = {64: 0, 256: 0, 512: 0, 1024: 0}
    wg_small = {64: 0, 256: 0, 512: 0, 1024: 0}
    wsum = 0.0
    wg_tot = 0
    sizes = []
    for r in rows:
        dt = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        wg_items = dims(r, "Workgroup_Size")
        grid = dims(r, "Grid_Size")
        wgs = max(1, grid // max(wg_items, 1))
        sizes.append(wgs)
        tot += dt
        wsum += dt * wgs
        wg_tot += wgs
        for k in small:
            if wgs < k:
                small[k] += dt
                cnt_small[k] += 1
                wg_small[k] += wgs
    sizes.sort()
    n = max(len(rows), 1)
    return {"dispatches": len(rows), "busy_ms": round(tot / 1e6, 2),
            "time_weighted_mean_workgroups": round(wsum / max(tot, 1), 1),
            "mean_workgroups": round(wg_tot / n, 1), "median_workgroups": sizes[len(sizes) // 2] if sizes else 0,
            **{f"time_frac_below_{k}_wg": round(v / max(tot, 1), 3) for k, v in small.items()},
            **{f"count_frac_below_{k}_wg": round(v / n, 3) for k, v in cnt_small.items()},
            **{f"wg_frac_below_{k}_wg": round(v / max(wg_tot, 1), 4) for k, v in wg_small.items()},
            "mean_us": round(tot / n / 1e3, 2)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--tail", type=float, default=0.5)
    a = ap.parse_args()
    out = {}
    for d in sorted(glob.glob(os.path.join(a.dir, "*"))):
        files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        if files:
            out[os.path.basename(d)] = summarize(files, a.tail)
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
