#!/usr/bin/env python3
"""A two-stream captured graph (fork onto a side stream, join before the end)
replayed under the enforcement library — the shape of a training step whose
weight gradients run on a side stream (vgpu.ops.bnconv).  Prints one JSON line.

    python scripts/multistream_graph_probe.py          # parent: runs the child under libvgpu.so
    python scripts/multistream_graph_probe.py --child  # the workload itself

Set VGPU_CRASH_TRACE=1 for a native stack if the child dies on a signal.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys


def child() -> int:
    import torch
    dev = "cuda"
    a = torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16)
    b = torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16)
    side = torch.cuda.Stream()

    def body():
        main = torch.cuda.current_stream()
        y = a @ b
        side.wait_stream(main)
        with torch.cuda.stream(side):
            z = (a * 2) @ b
        main.wait_stream(side)
        return y + z

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            ref = body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = body()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    ok = bool(torch.equal(out, ref))
    print("MULTISTREAM " + json.dumps({"ok": ok, "replays": 5}), flush=True)
    return 0 if ok else 1


def main() -> int:
    if "--child" in sys.argv:
        return child()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    from vgpu.native import ensure_built, preload_env
    ensure_built()
    env = preload_env()
    env.setdefault("VGPU_DEVICE_MEMORY_LIMIT_0", "100000m")
    env["PYTHONPATH"] = repo
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                       text=True, timeout=300)
    line = [l for l in r.stdout.splitlines() if l.startswith("MULTISTREAM ")]
    res = json.loads(line[-1][12:]) if line else {"ok": False}
    res["rc"] = r.returncode
    if r.returncode:
        res["stderr"] = r.stderr[-4000:]
    print(json.dumps(res), flush=True)
    return 0 if res.get("ok") else 1


if __name__ == "__main__":
    raise SystemExit(main())
