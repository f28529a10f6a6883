#!/usr/bin/env python3
"""Per kernel family over the last flagship forward: L2 requests (TCC_REQ,
128-B lines on gfx950), hit rate, and the L2 bandwidth those requests imply
over the dispatch time (scripts/pmc_l2.sh).

    python scripts/pmc_l2.py gpurun_out/pmc_l2 [--last 43]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load_counters, load_trace  # noqa: E402
from prof_summary import family  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=43)
    a = ap.parse_args()
    cnt = load_counters(os.path.join(a.dir, "p1"))[-a.last:]
    tr = load_trace(os.path.join(a.dir, "trace"))[-a.last:]
    agg = collections.OrderedDict()
    for c, t in zip(cnt, tr):
        f = family(c["name"])[:60]
        e = agg.setdefault(f, [0, 0.0, 0.0, 0.0, 0.0])
        e[0] += 1
        e[1] += t["ns"]
        e[2] += c.get("TCC_REQ_sum", 0.0)
        e[3] += c.get("TCC_HIT_sum", 0.0)
        e[4] += c.get("TCC_MISS_sum", 0.0)
    print("| family | n | us | L2 req (M) | hit % | L2 GB | L2 TB/s |")
    print("|---|---|---|---|---|---|---|")
    for f, (n, ns, req, hit, miss) in agg.items():
        gb = req * 128 / 1e9
        print(f"| {f} | {n} | {ns / 1e3:.1f} | {req / 1e6:.2f} | {100 * hit / max(hit + miss, 1):.1f} | "
              f"{gb:.2f} | {gb / max(ns, 1) * 1e6:.2f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
