#!/usr/bin/env python3
"""Summarise rocprofv3 kernel traces (CSV) per process: time share per kernel
family over the steady-state tail, plus the per-dispatch sequence of one step.

    python scripts/prof_summary.py gpurun_out/prof_native [--tail 0.5] [--step-dispatches N]

The tail fraction skips warmup / MIOpen find / graph capture; each pod process is
one vGPU container.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re


def family(name: str) -> str:
    m = re.search(r"conv_gemm_kernelILi(\d)ELi(\d+)ELi(\d+)ELb(\d)", name)
    if m:
        ks, bm, bn, pro = m.groups()
        return f"vgpu conv_gemm {ks}x{ks} BM{bm} BN{bn}{' +prologue' if pro == '1' else ''}"
    m = re.search(r"bn_reduce_kernel(?:ILi|<)(\d)", name)
    if m:
        return "vgpu BN " + ("fwd" if m.group(1) == "0" else "bwd") + " reduce"
    for key, fam in (("bn_fwd_finalize", "vgpu BN finalize"), ("bn_bwd_finalize", "vgpu BN finalize"),
                     ("bn_bwd_apply", "vgpu BN bwd apply"), ("bn_apply_kernel", "vgpu BN+act apply"),
                     ("maxpool_kernel", "vgpu maxpool"), ("ssr_mean", "vgpu BN+ReLU+mean"),
                     ("add_scale_shift", "vgpu add+BN+ReLU"), ("bias_act", "vgpu bias+act"),
                     ("scale_shift_act", "vgpu BN+act"), ("igemm", "MIOpen igemm conv"),
                     ("kernel_grouped_conv", "MIOpen CK grouped conv"), ("Cijk", "hipBLASLt/Tensile GEMM"),
                     ("max_pool", "torch maxpool"), ("wgrad_reduce", "vgpu wgrad reduce"),
                     ("splitk_reduce", "vgpu split-K reduce"), ("at::native::reduce_kernel", "torch reduce")):
        if key in name:
            return fam
    return name[:60]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--tail", type=float, default=0.5)
    ap.add_argument("--step-dispatches", type=int, default=0, help="print the last N dispatches")
    ap.add_argument("--last", type=int, default=0, help="aggregate only the last N dispatches")
    ap.add_argument("--last-ms", type=float, default=0.0,
                    help="aggregate only dispatches starting in the last T ms of the trace (steady state)")
    args = ap.parse_args()
    files = sorted(glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True))
    for f in files:
        rows = list(csv.DictReader(open(f)))
        if not rows:
            continue
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        tail = rows[-args.last:] if args.last else rows[int(len(rows) * (1 - args.tail)):]
        if args.last_ms:
            t_end = int(rows[-1]["End_Timestamp"])
            tail = [r for r in rows if int(r["Start_Timestamp"]) >= t_end - args.last_ms * 1e6]
        busy = collections.Counter()
        count = collections.Counter()
        for r in tail:
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            fam = family(r["Kernel_Name"])
            busy[fam] += d
            count[fam] += 1
        tot = sum(busy.values())
        span = int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])
        print(f"## {os.path.relpath(f, args.dir)}: {len(tail)} dispatches, busy {tot / 1e6:.1f} ms, "
              f"span {span / 1e6:.1f} ms\n")
        print("| % of busy | dispatches | avg us | family |\n|---|---|---|---|")
        for fam, t in busy.most_common():
            print(f"| {100 * t / tot:.1f} | {count[fam]} | {t / count[fam] / 1e3:.1f} | {fam} |")
        print()
        if args.step_dispatches:
            print("```")
            for r in tail[-args.step_dispatches:]:
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                print(f"{d:8.1f} us  grid {r.get('Grid_Size_X', r.get('Grid_Size', '?')):>8}  "
                      f"{family(r['Kernel_Name'])}")
            print("```\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
