#!/usr/bin/env python3
"""Per-family wait breakdown of the flagship forward (scripts/pmc_waits.sh):

    python scripts/pmc_waits_summary.py gpurun_out/pmc_waits [--last 88]

Per family, over the last forward's dispatches (matched by position from the
end, as scripts/pmc_summary.py does): µs per dispatch (trace run), waves
resident per SIMD (SQ_LEVEL_WAVES / SQ_BUSY_CYCLES / 4 SIMDs... normalised by
the family's busy cycles), and what a wave-cycle was spent on —
issuing (SQ_ACTIVE_INST_ANY), waiting on an outstanding dependency
(SQ_WAIT_INST_ANY: vmcnt / lgkmcnt / MFMA results), of which LDS
(SQ_WAIT_INST_LDS), and otherwise waiting (SQ_WAIT_ANY - SQ_WAIT_INST_ANY:
barriers, issue arbitration) — plus VMEM instruction mix and the mean cycles a
vector memory instruction is in flight (SQ_INST_LEVEL_VMEM / SQ_INSTS_VMEM,
Little's law) and MFMA-busy share.
"""
from __future__ import annotations

import argparse
import collections
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load_counters, load_trace  # noqa: E402
from prof_summary import family  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=88)
    a = ap.parse_args()
    trace = load_trace(os.path.join(a.dir, "trace"))
    passes = [load_counters(p) for p in sorted(glob.glob(os.path.join(a.dir, "p[0-9]*"))) if os.path.isdir(p)]
    ns, cnt = collections.Counter(), collections.Counter()
    ctr: dict[str, collections.Counter] = collections.defaultdict(collections.Counter)
    for i in range(1, a.last + 1):
        t = trace[-i]
        f = family(t["name"])
        ns[f] += t["ns"]
        cnt[f] += 1
        for p in passes:
            if i <= len(p) and family(p[-i]["name"]) == f:
                for k, v in p[-i].items():
                    if k != "name":
                        ctr[f][k] += v
    tot = sum(ns.values())
    print(f"{a.last} dispatches from the end, busy {tot / 1e6:.2f} ms\n")
    print("| % time | n | us/disp | waves/SIMD | issue | dep-wait | of which LDS | other wait | "
          "VMEM rd/wr per wave | cycles in flight per VMEM | MFMA busy | family |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for f, v in ns.most_common(12):
        c = ctr[f]
        wc = c["SQ_WAVE_CYCLES"] or 1
        busy = c["SQ_BUSY_CYCLES"] or 1
        waves = c["SQ_LEVEL_WAVES"] / busy / 4 if c["SQ_LEVEL_WAVES"] else 0  # per SIMD (4 per CU)
        nw = c["SQ_WAVES"] or 0
        vmem = c["SQ_INSTS_VMEM_RD"] + c["SQ_INSTS_VMEM_WR"]
        inflight = c["SQ_INST_LEVEL_VMEM"] / vmem if vmem else 0
        print(f"| {100 * v / tot:.1f} | {cnt[f]} | {v / cnt[f] / 1e3:.1f} | {waves:.2f} | "
              f"{c['SQ_ACTIVE_INST_ANY'] / wc:.2f} | {c['SQ_WAIT_INST_ANY'] / wc:.2f} | "
              f"{c['SQ_WAIT_INST_LDS'] / wc:.2f} | {(c['SQ_WAIT_ANY'] - c['SQ_WAIT_INST_ANY']) / wc:.2f} | "
              f"{c['SQ_INSTS_VMEM_RD']:.3g}/{c['SQ_INSTS_VMEM_WR']:.3g} | {inflight:.0f} | "
              f"{c['SQ_VALU_MFMA_BUSY_CYCLES'] / busy / 4 if busy > 1 else 0:.2f} | {f[:58]} |")
    print("\nRatios are per wave-cycle (SQ_WAVE_CYCLES); `other wait` = SQ_WAIT_ANY - SQ_WAIT_INST_ANY "
          "(barriers, arbitration).  waves/SIMD = SQ_LEVEL_WAVES / SQ_BUSY_CYCLES / 4.")
    return 0


if __name__ == "__main__":
    sys.exit(main())
