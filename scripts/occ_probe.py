#!/usr/bin/env python3
"""KFD cu_occupancy as a marker-independent busy signal:
how much does one sysfs read cost, and does the value track GPU work?

    python scripts/occ_probe.py [--seconds 3] [--period-us 1000]

A child process keeps the GPU busy (bf16 GEMMs in a captured hipGraph,
replayed back to back) for `--busy` seconds after a `--idle` lead; the parent
samples /sys/class/kfd/kfd/proc/<child pid>/stats_<gpu id>/cu_occupancy every
`--period-us` and prints one JSON line: read cost percentiles, the fraction of
samples > 0 in the idle lead and in the busy window, and value percentiles.
Run it as is and under `rocprofv3 --kernel-trace -- python3 scripts/occ_probe.py`
(the child inherits the profiler) to see whether the signal survives it.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import time

CHILD = r"""
import sys, time, torch
idle, busy = float(sys.argv[1]), float(sys.argv[2])
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
c = a @ b
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(8):
        c = a @ b
print("READY", flush=True)
time.sleep(idle)
t0 = time.monotonic()
n = 0
while time.monotonic() - t0 < busy:
    g.replay(); n += 1
    if n % 4 == 0:
        torch.cuda.synchronize()
torch.cuda.synchronize()
print("DONE", n, time.monotonic() - t0, flush=True)
"""


def pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--idle", type=float, default=1.0)
    ap.add_argument("--busy", type=float, default=3.0)
    ap.add_argument("--period-us", type=float, default=1000.0)
    a = ap.parse_args()
    kfd = "/sys/class/kfd/kfd/proc"
    before = set(os.listdir(kfd)) if os.path.isdir(kfd) else set()
    p = subprocess.Popen([sys.executable, "-c", CHILD, str(a.idle), str(a.busy)], stdout=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    if not line.startswith("READY"):
        print(json.dumps({"error": "child did not start", "line": line}))
        return 1
    # KFD names processes by host pid; inside a container the child's pid
    # differs, so take the entry that appeared with it.
    new = sorted(set(os.listdir(kfd)) - before) if os.path.isdir(kfd) else []
    cands = [str(p.pid)] + new
    files = []
    for c in cands:
        files = glob.glob(f"{kfd}/{c}/stats_*/cu_occupancy")
        if files:
            break
    if not files:
        p.wait()
        print(json.dumps({"error": "no cu_occupancy file", "new_kfd_entries": new,
                          "listing": {c: os.listdir(f"{kfd}/{c}") for c in new if os.path.isdir(f"{kfd}/{c}")}}))
        return 1
    fds = [os.open(f, os.O_RDONLY) for f in files]
    t_start = time.monotonic()
    samples = []  # (t, [values], read_ns)
    while p.poll() is None:
        t = time.monotonic()
        vals = []
        t0 = time.perf_counter_ns()
        for fd in fds:
            vals.append(int(os.pread(fd, 64, 0).split()[0] or 0))
        cost = time.perf_counter_ns() - t0
        samples.append((t - t_start, vals, cost))
        time.sleep(max(0.0, a.period_us * 1e-6 - (time.monotonic() - t)))
    out = p.stdout.read()
    idle = [s for s in samples if s[0] < a.idle * 0.9]
    busy = [s for s in samples if a.idle * 1.1 + 0.2 < s[0] < a.idle + a.busy * 0.9]
    costs = [s[2] / 1e3 for s in samples]
    bvals = [max(s[1]) for s in busy]
    res = {"files": files, "samples": len(samples), "period_us": a.period_us,
           "read_us_p50": pct(costs, 0.5), "read_us_p99": pct(costs, 0.99),
           "idle_nonzero": round(sum(1 for s in idle if max(s[1]) > 0) / max(len(idle), 1), 3),
           "busy_nonzero": round(sum(1 for v in bvals if v > 0) / max(len(bvals), 1), 3),
           "busy_value_p10": pct(bvals, 0.1), "busy_value_p50": pct(bvals, 0.5), "busy_value_max": max(bvals or [0]),
           "child": out.strip().splitlines()[-1] if out.strip() else None}
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
