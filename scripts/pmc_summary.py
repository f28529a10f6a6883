#!/usr/bin/env python3
"""Join the PMC passes and the kernel trace of scripts/pmc_flagship.sh per
dispatch (matched by position counted from the end of each run: the runs
execute the same program) and summarise per kernel family over the last
forward pass(es):

    python scripts/pmc_summary.py gpurun_out/pmc_flagship [--last N]

Columns: µs per dispatch (trace run, unprofiled counters), MFMA busy
(SQ_VALU_MFMA_BUSY_CYCLES ÷ (4 SIMDs × 256 CUs × GRBM_GUI_ACTIVE/8)), wave
time split (active / issue-stalled / parked), LDS bank conflicts per LDS
instruction, HBM-side bytes (FETCH_SIZE×2 + WRITE_SIZE: gfx950 FETCH_SIZE
tallies wide streaming reads at half their bytes, MI355X_MICROARCH.md §HBM)
and the bandwidth those bytes imply over the dispatch time.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import family  # noqa: E402


def load_counters(d: str) -> list[dict]:
    """Per dispatch (ordered by dispatch id): {'name', counter: value...}."""
    per: dict[int, dict] = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = (int(r.get("Process_Id", 0) or 0), int(r["Dispatch_Id"]))
            e = per.setdefault(k, {"name": r["Kernel_Name"]})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def load_trace(d: str) -> list[dict]:
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return [{"name": r["Kernel_Name"], "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])}
            for r in rows]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=0,
                    help="dispatches to aggregate from the end (default: a third of the trace)")
    args = ap.parse_args()
    trace = load_trace(os.path.join(args.dir, "trace"))
    passes = [load_counters(p) for p in sorted(glob.glob(os.path.join(args.dir, "p[0-9]*")))
              if os.path.isdir(p)]
    n = args.last or len(trace) // 3
    fam_ns = collections.Counter()
    fam_cnt = collections.Counter()
    fam_ctr: dict[str, collections.Counter] = collections.defaultdict(collections.Counter)
    mismatched = 0
    for i in range(1, n + 1):
        t = trace[-i]
        fam = family(t["name"])
        fam_ns[fam] += t["ns"]
        fam_cnt[fam] += 1
        for p in passes:
            if i > len(p):
                continue
            e = p[-i]
            if family(e["name"]) != fam:
                mismatched += 1
                continue
            for k, v in e.items():
                if k != "name":
                    fam_ctr[fam][k] += v
    tot = sum(fam_ns.values())
    print(f"{n} dispatches from the end, busy {tot / 1e6:.2f} ms"
          + (f", {mismatched} pass rows not aligned (skipped)" if mismatched else "") + "\n")
    print("| % time | n | us/disp | MFMA busy | active/stall/parked | LDS confl/inst | HBM MB/disp | GB/s | family |")
    print("|---|---|---|---|---|---|---|---|---|")
    all_c = collections.Counter()
    for fam, ns in fam_ns.most_common():
        c = fam_ctr[fam]
        all_c.update(c)
        k = fam_cnt[fam]
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (4 * 256 * cyc) if cyc else float("nan")
        w = c.get("SQ_WAVE_CYCLES", 0) or float("nan")
        split = (f"{c.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f}/{c.get('SQ_WAIT_INST_ANY', 0) / w:.2f}/"
                 f"{c.get('SQ_WAIT_ANY', 0) / w:.2f}")
        lds = c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_INSTS_LDS", 0), 1)
        hbm = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024
        print(f"| {100 * ns / tot:.1f} | {k} | {ns / k / 1e3:.1f} | {100 * mfma:.0f}% | {split} | "
              f"{lds:.2f} | {hbm / k / 1e6:.1f} | {hbm / ns:.0f} | {fam} |")
    cyc = all_c.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc:
        hbm = (2 * all_c.get("FETCH_SIZE", 0) + all_c.get("WRITE_SIZE", 0)) * 1024
        print(f"\nwhole window: MFMA busy {100 * all_c['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * cyc):.1f}%, "
              f"HBM-side {hbm / 1e9:.2f} GB over {tot / 1e6:.2f} ms = {hbm / tot:.0f} GB/s, "
              f"effective clock {cyc / (tot / 1e9) / 1e9 * 1:.2f} GHz (GRBM_GUI_ACTIVE/8 over trace time)")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
