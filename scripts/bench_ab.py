#!/usr/bin/env python3
"""Named A/B recipes of bench.py on one GPU box (replaces the round-1/2 one-off
gpu_*.sh scripts; their results live in profiles/).

    python scripts/bench_ab.py <recipe> [--reps N] [--out gpurun_out/ab]
    python scripts/bench_ab.py --list

Every variant is one bench.py run under its own `timeout -k 10`, with the
variant's env and flags on top of the recipe's base flags.  The runner stops
at the first failing variant (a GPU fault, abort or time limit must not be
followed by more GPU work), writes each run's log to <out>/<recipe>/<tag>.log
and prints one summary line per variant: images/s, ms/step, per-pod images/s,
the pods' share policy.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

EXCL = ["--pods", "1", "--gpucores", "100", "--gpumem", "0"]
P4 = ["--pods", "4", "--gpucores", "25", "--gpumem", "72000"]

# recipe -> (base flags, [(tag, env, extra flags)], per-run seconds)
RECIPES: dict[str, tuple[list, list, int]] = {
    # Flagship under the plugin's share policies (profiles/r2/flag).
    "flagship": (["--steps", "30", "--warmup", "10"], [
        ("temporal", {}, ["--cu-share", "temporal"]),
        ("hybrid", {}, ["--cu-share", "hybrid"]),
        ("mask", {}, ["--cu-share", "mask"]),
        ("exclusive", {}, EXCL),
    ], 300),
    # Flagship knobs under the default temporal share policy.
    "temporal-knobs": (["--steps", "30", "--warmup", "10"], [
        ("base", {}, []),
        ("q2", {}, ["--hw-queues", "2"]),
        ("q0", {}, ["--hw-queues", "0"]),
        ("split2_q1", {"VGPU_POD_SPLIT": "2"}, []),
        ("split2_q2", {"VGPU_POD_SPLIT": "2"}, ["--hw-queues", "2"]),
        ("cus256", {"VGPU_CONV_CUS": "256"}, []),
        ("dryrun", {"VGPU_LIMITER_DRYRUN": "1"}, []),
        ("noshim", {}, ["--no-shim"]),
        ("base_again", {}, []),
    ], 300),
    # ResNet-152 training at 4 x 25 %: where does the temporal pool lose to masks?
    "share4-r152t": (P4 + ["--workload", "2.2", "--steps", "40", "--warmup", "5"], [
        ("temporal", {}, ["--cu-share", "temporal"]),
        ("temporal_dryrun", {"VGPU_LIMITER_DRYRUN": "1"}, ["--cu-share", "temporal"]),
        ("noshim", {}, ["--no-shim"]),
        ("mask", {}, ["--cu-share", "mask"]),
        ("temporal_cus256", {"VGPU_CONV_CUS": "256"}, ["--cu-share", "temporal"]),
        ("temporal_again", {}, ["--cu-share", "temporal"]),
    ], 300),
    # Concurrency gate of the temporal pool (VGPU_POOL_CONCURRENCY) at 4 x 25 %.
    "pool-gate": (P4 + ["--steps", "40", "--warmup", "5", "--cu-share", "temporal"], [
        ("w2.2_free", {}, ["--workload", "2.2"]),
        ("w2.2_k2", {"VGPU_POOL_CONCURRENCY": "2"}, ["--workload", "2.2"]),
        ("w2.1_free", {}, ["--workload", "2.1"]),
        ("w2.1_k2", {"VGPU_POOL_CONCURRENCY": "2"}, ["--workload", "2.1"]),
        ("w1.1_free", {}, ["--workload", "1.1"]),
        ("w1.1_k2", {"VGPU_POOL_CONCURRENCY": "2"}, ["--workload", "1.1"]),
        ("w5.1_free", {}, ["--workload", "5.1"]),
        ("w5.1_k2", {"VGPU_POOL_CONCURRENCY": "2"}, ["--workload", "5.1"]),
        ("w2.2_k2_q100", {"VGPU_POOL_CONCURRENCY": "2", "VGPU_POOL_QUANTUM_MS": "100"}, ["--workload", "2.2"]),
    ], 300),
    # Pool gate with conv tiles sized for the CUs a running pod actually shares (256 / k).
    "pool-gate-cus": (P4 + ["--steps", "40", "--warmup", "5", "--cu-share", "temporal"], [
        ("w2.2_free", {}, ["--workload", "2.2"]),
        ("w2.2_k2_c128", {"VGPU_POOL_CONCURRENCY": "2", "VGPU_CONV_CUS": "128"}, ["--workload", "2.2"]),
        ("w2.2_free_c128", {"VGPU_CONV_CUS": "128"}, ["--workload", "2.2"]),
        ("w1.2_free", {}, ["--workload", "1.2"]),
        ("w1.2_k2_c128", {"VGPU_POOL_CONCURRENCY": "2", "VGPU_CONV_CUS": "128"}, ["--workload", "1.2"]),
        ("w2.1_free", {}, ["--workload", "2.1"]),
        ("w2.1_k2_c128", {"VGPU_POOL_CONCURRENCY": "2", "VGPU_CONV_CUS": "128"}, ["--workload", "2.1"]),
        ("w2.2_free_again", {}, ["--workload", "2.2"]),
    ], 300),
    # Conv dispatch knobs re-checked under the default temporal policy.
    "conv-knobs": (["--steps", "30", "--warmup", "10"], [
        ("base", {}, []),
        ("big_all", {"VGPU_CONV_BIG": "1"}, []),
        ("big_off", {"VGPU_CONV_BIG": "0"}, []),
        ("1x1_big", {"VGPU_CONV_1X1_BIG": "1"}, []),
        ("base_again", {}, []),
    ], 300),
    # Temporal limiter accuracy and fair share (profiles/temporal_r2.md).
    "temporal": (["--steps", "150"], [
        ("excl", {}, EXCL),
        ("t1x25", {}, ["--pods", "1", "--gpucores", "25", "--cu-share", "temporal", "--core-policy", "force"]),
        ("t1x50", {}, ["--pods", "1", "--gpucores", "50", "--cu-share", "temporal", "--core-policy", "force"]),
        ("t1x25_default", {}, ["--pods", "1", "--gpucores", "25", "--cu-share", "temporal"]),
        ("t2x50", {}, ["--pods", "2", "--gpucores", "50", "--cu-share", "temporal"]),
        ("t4x25", {}, P4 + ["--cu-share", "temporal"]),
        ("m4x25", {}, P4 + ["--cu-share", "mask"]),
    ], 400),
    # Limiter internals with the shim's own trace (VGPU_TRACE, gpu_time/throttle events).
    "temporal-trace": (["--steps", "150", "--pods", "1", "--cu-share", "temporal"], [
        ("t25", {"VGPU_TRACE": "{out}/t25"}, ["--gpucores", "25"]),
        ("t99", {"VGPU_TRACE": "{out}/t99"}, ["--gpucores", "99"]),
    ], 300),
    # 4 x 25 % share-policy comparison (profiles/sharing_4way_r1.md, profiles/r2).
    "share4": (P4, [
        ("mask", {}, ["--cu-share", "mask"]),
        ("temporal", {}, ["--cu-share", "temporal"]),
        ("hybrid", {}, ["--cu-share", "hybrid"]),
        ("group2", {}, ["--cu-share", "group2"]),
        ("group2i", {}, ["--cu-share", "group2i"]),
        ("nomask", {}, ["--gpucores", "100"]),
        ("mask_q0", {}, ["--cu-share", "mask", "--hw-queues", "0"]),
    ], 300),
    # Limiter marker spacing on a dispatch-heavy and a graph workload (profiles/r2/weak).
    "markers": (P4 + ["--steps", "40", "--warmup", "5", "--cu-share", "temporal"], [
        ("w4.2_dryrun", {"VGPU_LIMITER_DRYRUN": "1"}, ["--workload", "4.2"]),
        ("w4.2_noshim", {}, ["--workload", "4.2", "--no-shim"]),
    ], 300),
    # Conv tile choice vs the CUs a pod owns (profiles/conv_cus_r1.md).
    "conv-cus": (["--steps", "30", "--warmup", "10"], [
        ("flag", {}, []),
        ("flag_c256", {"VGPU_CONV_CUS": "256"}, []),
        ("excl", {}, EXCL),
        ("excl_c128", {"VGPU_CONV_CUS": "128"}, EXCL),
    ], 300),
    # Micro-batch split and HW-queue budget per pod (profiles/pmc_flagship_r1.md).
    "split": (["--steps", "30", "--warmup", "10"], [
        ("base", {}, []),
        ("s2q1", {"VGPU_POD_SPLIT": "2"}, []),
        ("s2q2", {"VGPU_POD_SPLIT": "2"}, ["--hw-queues", "2"]),
        ("baseq2", {}, ["--hw-queues", "2"]),
    ], 300),
    # Training workloads, one exclusive pod (profiles/bn_train_r1.md, wgrad_r1.md).
    "train": (["--steps", "20", "--warmup", "5"] + EXCL, [
        ("1.2", {}, ["--workload", "1.2"]),
        ("2.2", {}, ["--workload", "2.2"]),
        ("3.2", {}, ["--workload", "3.2"]),
    ], 300),
    # cost of the ROCr tools-lib intercept (HSA_TOOLS_LIB=libvgpu.so,
    # intercept queues on) on the flagship and on 1.2 training (profiles/r6/toolslib).
    "tools-lib": (["--steps", "30", "--warmup", "10"], [
        ("flag_base", {}, []),
        ("flag_tools", {"VGPU_HSA_TOOLS_INTERCEPT": "1"}, []),
        ("t12_base", {}, EXCL + ["--workload", "1.2", "--steps", "20", "--warmup", "5"]),
        ("t12_tools", {"VGPU_HSA_TOOLS_INTERCEPT": "1"}, EXCL + ["--workload", "1.2", "--steps", "20", "--warmup", "5"]),
        ("flag_base_again", {}, []),
        ("flag_tools_again", {"VGPU_HSA_TOOLS_INTERCEPT": "1"}, []),
    ], 400),
    # Virtual device memory column of the reference's chart, one workload.
    "vmem": (["--steps", "20", "--warmup", "5"], [
        ("vgpu", {}, ["--pods", "2", "--gpucores", "50", "--gpumem", "144000"]),
        ("vmem", {}, ["--pods", "2", "--gpucores", "0", "--gpumem", "230000", "--oversubscribe",
                      "--memory-scaling", "1.8"]),
    ], 300),
}


def run_variant(out: str, tag: str, env: dict, flags: list, secs: int) -> dict | None:
    e = dict(os.environ)
    e.setdefault("TMPDIR", "/tmp")
    for k, v in env.items():
        e[k] = v.format(out=out)
        if k == "VGPU_TRACE":
            os.makedirs(e[k], exist_ok=True)
    log = os.path.join(out, f"{tag}.log")
    cmd = ["timeout", "-k", "10", str(secs), sys.executable, os.path.join(REPO, "bench.py"),
           "--no-cap-probe", *flags]
    with open(log, "w") as f:
        rc = subprocess.call(cmd, stdout=f, stderr=subprocess.STDOUT, env=e, cwd=REPO)
    lines = [ln for ln in open(log, errors="replace") if ln.startswith("{")]
    if rc != 0 or not lines:
        print(f"{tag} FAILED rc={rc}; tail of {log}:")
        print("".join(open(log, errors="replace").readlines()[-8:]))
        return None
    d = json.loads(lines[-1])
    print(f"{tag} {d['value']} img/s, {d['ms_per_step']} ms/step, per pod {d['per_pod_images_s']}, "
          f"share {d.get('per_pod_share')}", flush=True)
    return d


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("recipe", nargs="?")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "ab"))
    ap.add_argument("--only", default="", help="comma-separated variant tags")
    ap.add_argument("--list", action="store_true")
    a = ap.parse_args(argv)
    if a.list or not a.recipe:
        for name, (base, vs, _) in RECIPES.items():
            print(f"{name}: base {' '.join(base) or '-'}; variants {', '.join(v[0] for v in vs)}")
        return 0
    base, variants, secs = RECIPES[a.recipe]
    out = os.path.join(a.out, a.recipe)
    os.makedirs(out, exist_ok=True)
    only = set(filter(None, a.only.split(",")))
    results = []
    for rep in range(1, a.reps + 1):
        for tag, env, flags in variants:
            if only and tag not in only:
                continue
            t = f"{tag}_{rep}" if a.reps > 1 else tag
            d = run_variant(out, t, env, base + flags, secs)
            if d is None:
                return 1
            results.append({"tag": t, "value": d["value"], "ms_per_step": d["ms_per_step"],
                            "per_pod": d["per_pod_images_s"], "share": d.get("per_pod_share"),
                            "config": d["config"]})
    with open(os.path.join(out, "summary.jsonl"), "w") as f:
        for r in results:
            f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
