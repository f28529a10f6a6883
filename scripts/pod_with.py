#!/usr/bin/env python3
"""Run a bench pod with a kernel-library setter applied first (in-process A/B
of knobs that have no environment variable):

    python scripts/pod_with.py splitk=0 -- --workload 4.2 --steps 20 --warmup 5 --graph --no-wait
"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sep = sys.argv.index("--")
for kv in sys.argv[1:sep]:
    k, v = kv.split("=")
    if k == "splitk":
        from vgpu.ops import conv as C
        C.set_splitk(int(v))
    else:
        raise SystemExit(f"unknown setter {k}")
sys.argv = [sys.argv[0]] + sys.argv[sep + 1:]
runpy.run_module("vgpu.bench.pod", run_name="__main__")
