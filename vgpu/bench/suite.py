"""ai-benchmark-equivalent suite on one MI355X: every test id the reference
publishes (BASELINE.md rows 1.1–5.2) in three scenarios, mirroring the
reference's comparison (README.md:234-257):

  exclusive          — one pod, whole GPU, no enforcement library
  vgpu               — 2 pods × gpucores=50, gpumem=144000 (BASELINE.json config 2),
                       device-plugin default share policy (auto: a share-board A/B
                       of time sharing vs CUs of their own; 12 s of warmup let it settle)
  vgpu-temporal      — the same, policy named explicitly
  vgpu-mask          — the same 2 pods, one CU mask each
  vgpu-cu25          — 4 pods × gpucores=25 (BASELINE.json config 3), default policy (auto)
  vgpu-cu25-temporal — the same 4 pods, policy named explicitly
  vgpu-cu25-mask     — the same 4 pods, one CU mask each
  vgpu-cu25-hybrid   — 2 CU masks + a temporal pool for the other two
  vgpu-cu25-auto     — the 4 pods under the adaptive policy: pool members that
                       claim CUs of their own when their dispatches are small
  vgpu-auto          — 2 pods, adaptive policy
  vgpu-cu25-k2       — the 4 pods in the temporal pool, at most 2 running at a time
                       (device plugin --pool-concurrency 2)
  vgpu-vmem          — the reference's "vGPU + virtual device memory" column:
                       2 pods per GPU on a plugin with --device-memory-scaling=1.8,
                       each capped at 230000 MiB (together 1.7 x the physical HBM,
                       so the caps oversubscribe it) and no compute limit (reference benchmarks/ai-benchmark/
                       vGPU-device-plugin(virtual device memory)/ai-benchmark.yml)

Prints one JSON line per (test, scenario) and a markdown table at the end.
    python -m vgpu.bench.suite [--tests 1.1,1.2,...] [--steps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SCENARIOS = {
    "exclusive": ["--pods", "1", "--no-shim", "--gpucores", "100", "--gpumem", "0"],
    "vgpu": ["--pods", "2", "--gpucores", "50", "--gpumem", "144000", "--warmup-seconds", "12"],
    "vgpu-temporal": ["--pods", "2", "--gpucores", "50", "--gpumem", "144000", "--cu-share", "temporal"],
    "vgpu-mask": ["--pods", "2", "--gpucores", "50", "--gpumem", "144000", "--cu-share", "mask"],
    "vgpu-cu25-hybrid": ["--pods", "4", "--gpucores", "25", "--gpumem", "70000", "--cu-share", "hybrid"],
    "vgpu-cu25": ["--pods", "4", "--gpucores", "25", "--gpumem", "70000", "--warmup-seconds", "12"],
    "vgpu-cu25-temporal": ["--pods", "4", "--gpucores", "25", "--gpumem", "70000", "--cu-share", "temporal"],
    "vgpu-cu25-mask": ["--pods", "4", "--gpucores", "25", "--gpumem", "70000", "--cu-share", "mask"],
    "vgpu-cu25-auto": ["--pods", "4", "--gpucores", "25", "--gpumem", "70000", "--cu-share", "auto",
                       "--warmup-seconds", "12"],
    "vgpu-auto": ["--pods", "2", "--gpucores", "50", "--gpumem", "144000", "--cu-share", "auto",
                  "--warmup-seconds", "12"],
    "vgpu-vmem": ["--pods", "2", "--gpucores", "0", "--gpumem", "230000", "--oversubscribe",
                  "--memory-scaling", "1.8"],
    "vgpu-cu25-k2": ["--pods", "4", "--gpucores", "25", "--gpumem", "70000", "--cu-share", "temporal",
                     "--pool-concurrency", "2"],
    "vgpu-cu25-temporal-q0": ["--pods", "4", "--gpucores", "25", "--gpumem", "70000", "--cu-share", "temporal",
                              "--hw-queues", "0"],
}


def run(test: str, scen: str, steps: int, warmup: int, timeout: int) -> dict:
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--workload", test, "--steps", str(steps),
           "--warmup", str(warmup), "--no-cap-probe", *SCENARIOS[scen]]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=REPO)
    except subprocess.TimeoutExpired:
        return {"test": test, "scenario": scen, "error": "timeout"}
    if os.environ.get("VGPU_SUITE_LOGDIR"):  # keep each run's pod / shim log
        d = os.environ["VGPU_SUITE_LOGDIR"]
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"{test}_{scen}.err"), "w") as f:
            f.write(r.stderr)
    js = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not js:
        return {"test": test, "scenario": scen, "error": r.stderr[-1500:]}
    d = json.loads(js[-1])
    return {"test": test, "scenario": scen, "images_s": d["value"], "per_pod": d["per_pod_images_s"],
            "ms_per_step": d["ms_per_step"], "share": d.get("per_pod_share"), "final_cus": d.get("per_pod_final_cus")}


def main(argv=None) -> int:
    from vgpu.models import WORKLOADS
    ap = argparse.ArgumentParser()
    ap.add_argument("--tests", default=",".join(WORKLOADS))
    ap.add_argument("--scenarios", default="exclusive,vgpu,vgpu-cu25,vgpu-vmem")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--timeout", type=int, default=900)
    a = ap.parse_args(argv)
    rows = []
    for t in a.tests.split(","):
        for s in a.scenarios.split(","):
            res = run(t, s, a.steps, a.warmup, a.timeout)
            print("SUITE " + json.dumps(res), flush=True)
            rows.append(res)
    print("\n| test | workload | " + " | ".join(a.scenarios.split(",")) + " | reference 2xV100 (excl / vGPU) |")
    print("|---|---|" + "---|" * len(a.scenarios.split(",")) + "---|")
    for t in a.tests.split(","):
        w = WORKLOADS[t]
        cells = []
        for s in a.scenarios.split(","):
            r = next((x for x in rows if x["test"] == t and x["scenario"] == s), {})
            cells.append(f"{r.get('images_s', 'err')}")
        print(f"| {t} | {w.name} {'train' if w.train else 'inf'} b={w.batch} | " + " | ".join(cells)
              + f" | {w.baseline_exclusive} / {w.baseline_vgpu} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
