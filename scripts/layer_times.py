#!/usr/bin/env python3
"""Per-dispatch times of one flagship forward next to the roofline plan.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lt -o run -- \\
        python3 -m vgpu.bench.pod --workload 1.1 --steps 3 --warmup 1 --no-wait
    python scripts/layer_times.py gpurun_out/lt [--batch 50 --size 346]

The last forward's dispatches (as many as scripts/roofline.py plans, counted
from the end of the trace) are listed in order with their kernel family, µs,
the plan's compulsory bytes and FLOPs, the bound at 8 TB/s / 2.5 PFLOP/s and
the achieved fraction of it (the bound's µs over the measured µs).
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import family  # noqa: E402
from roofline import HBM_TBPS, MFMA_PFLOPS, plan  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--batch", type=int, default=50)
    ap.add_argument("--size", type=int, default=346)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    p = plan(a.batch, a.size)
    # the stem is two dispatches (space-to-depth, then conv + max pool): one plan row
    recs = []
    for r in reversed(rows):
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if "s2d_stem" in r["Kernel_Name"] and recs:
            recs[-1] = (recs[-1][0], recs[-1][1] + ns)
            continue
        if len(recs) == len(p):
            break
        recs.append((r, ns))
    last = list(reversed(recs))
    tot_ns = tot_bound = 0.0
    print("| # | plan kernel | dispatch | us | GFLOP | MB | bound us | of bound |")
    print("|---|---|---|---|---|---|---|---|")
    for i, ((name, flops, nbytes), (r, ns)) in enumerate(zip(p, last)):
        bound = max(nbytes / (HBM_TBPS * 1e12), flops / (MFMA_PFLOPS * 1e15)) * 1e9
        tot_ns += ns
        tot_bound += bound
        print(f"| {i} | {name} | {family(r['Kernel_Name'])[:48]} | {ns / 1e3:.1f} | {flops / 1e9:.1f} | "
              f"{nbytes / 1e6:.1f} | {bound / 1e3:.1f} | {bound / max(ns, 1):.2f} |")
    print(f"\nforward: {tot_ns / 1e3:.1f} us of kernels, bound {tot_bound / 1e3:.1f} us "
          f"({tot_bound / max(tot_ns, 1):.2f} of speed-of-light)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
