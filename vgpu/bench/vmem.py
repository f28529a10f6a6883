"""Virtual device memory benchmark (BASELINE.json config 5): one pod requests
`amd.com/gpumem=400000` (MiB) on a 288 GB MI355X.

Part A — oversubscribed cap (runs as a capped vGPU child under libvgpu.so with
VGPU_OVERSUBSCRIBE=true): torch sees a 400000 MiB device; allocating past the
physical HBM succeeds (the enforcement library backs the excess with pinned,
device-mapped host memory), GPU kernels read/write those bytes correctly (K3
fill/verify), and the cap still refuses anything beyond 400000 MiB.

Part B — Llama-3-8B (random init, bf16) decode with its 32 layers paged through
a bounded HBM working set by the HostPager (side-stream prefetch, LRU) versus
fully resident; reports tokens/s and host→HBM GB/s.

Part C — transparent migration, no application changes: an unmodified PyTorch
Llama-3-8B decode in a gpumem=400000 pod while a neighbour process holds all
but --leave-gib of the HBM, so part of the model spills at load time.  The
neighbour then exits; the shim's pager (native/shim/vmem.cpp) promotes the
spilled weights it sees in kernel arguments back into HBM.  Run once with the
pager and once with VGPU_VMEM_MIGRATE=0 (the round-1 zero-copy spill, which
never moves back).  Reports tokens/s per window, swap-in bytes and migrations.

    python -m vgpu.bench.vmem [--spill-gib 8] [--budget-gib 8] [--tokens 16] [--part-c]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

GiB = 1 << 30


def part_a_child(spill_gib: int) -> dict:
    import ctypes

    import torch
    from vgpu.ops import kernels as K
    free, total = torch.cuda.mem_get_info()
    lib = ctypes.CDLL(None)
    host_bytes = getattr(lib, "vgpu_self_host_bytes", None)
    if host_bytes is not None:
        host_bytes.restype = ctypes.c_uint64
    # physical HBM as the runtime reports it (the cap reports the virtual size)
    phys = torch.cuda.get_device_properties(0).total_memory
    blocks = []
    target = None
    t0 = time.time()
    try:
        while True:
            blocks.append(torch.empty(4 * GiB, dtype=torch.uint8, device="cuda"))
            spilled = host_bytes(0) if host_bytes else 0
            if target is None and spilled:
                target = len(blocks) + max(spill_gib // 4 - 1, 0)
            if target is not None and len(blocks) >= target:
                break
    except torch.OutOfMemoryError:
        pass
    spilled = host_bytes(0) if host_bytes else 0
    # touch the last (host-backed) blocks from the GPU
    errs = 0
    for i, b in enumerate(blocks[-2:]):
        K.fill_pattern(b, 100 + i)
        errs += K.verify_pattern(b, 100 + i)
    torch.cuda.synchronize()
    # bandwidth of a GPU kernel streaming a spilled block
    b = blocks[-1]
    t1 = time.time()
    K.verify_pattern(b, 101)
    torch.cuda.synchronize()
    zc_gbs = b.numel() / (time.time() - t1) / 1e9
    allocated = len(blocks) * 4 * GiB
    del blocks
    torch.cuda.empty_cache()
    # beyond the cap: must fail
    over_ok = False
    try:
        torch.empty(401000 << 20, dtype=torch.uint8, device="cuda")
    except torch.OutOfMemoryError:
        over_ok = True
    return {"reported_total": total, "reported_free": free, "allocated": allocated,
            "host_spilled": spilled, "verify_errors": errs, "zero_copy_read_GBps": round(zc_gbs, 1),
            "beyond_cap_refused": over_ok, "alloc_s": round(time.time() - t0, 1), "prop_total": phys}


def part_b(budget_gib: float, tokens: int, ctx: int) -> dict:
    import torch
    from vgpu.models.llama import Llama, LlamaConfig
    from vgpu.models.streamed import StreamedLlama
    cfg = LlamaConfig.llama3_8b()
    dev = torch.device("cuda")
    res = {}
    # paged
    sm = StreamedLlama.random_init(cfg, budget_bytes=int(budget_gib * GiB), device=dev, lookahead=2)
    kv = _kv(cfg, ctx, dev)
    tok = torch.randint(0, cfg.vocab, (1, 1), device=dev)
    sm(tok, kv, 0)
    torch.cuda.synchronize()
    s0 = sm.pager.stats.swap_in_bytes
    t0 = time.time()
    for p in range(1, tokens + 1):
        sm(tok, kv, p)
    torch.cuda.synchronize()
    dt = time.time() - t0
    moved = sm.pager.stats.swap_in_bytes - s0
    res["paged"] = {"budget_gib": budget_gib, "tokens_per_s": round(tokens / dt, 2),
                    "swap_in_GBps": round(moved / dt / 1e9, 1), "layer_bytes": sm.layer_bytes(),
                    "evictions": sm.pager.stats.evictions}
    model_bytes = sm.layer_bytes() * cfg.layers
    del sm, kv
    torch.cuda.empty_cache()
    # fully resident reference
    with torch.device("meta"):
        m = Llama(cfg)
    m = m.to_empty(device=dev).to(torch.bfloat16)
    with torch.no_grad():
        for p_ in m.parameters():
            p_.normal_(0, 0.02)
    m.eval()
    kv = _kv(cfg, ctx, dev)
    with torch.inference_mode():
        m(tok, kv, 0)
        torch.cuda.synchronize()
        t0 = time.time()
        for p in range(1, tokens + 1):
            m(tok, kv, p)
        torch.cuda.synchronize()
    dt = time.time() - t0
    res["resident"] = {"tokens_per_s": round(tokens / dt, 2)}
    res["model_bytes"] = model_bytes
    return res


def part_c_child(tokens: int, ctx: int, windows: int) -> dict:
    """Runs under libvgpu.so (oversubscribed pod).  stdin/stdout protocol with
    the parent: prints LOADED after the model is on the device, waits for a
    line on stdin (the neighbour has exited), then decodes `windows` windows."""
    import ctypes

    import torch
    from vgpu.models.llama import Llama, LlamaConfig
    lib = ctypes.CDLL(None)
    vstats = getattr(lib, "vgpu_self_vmem_stats", None)
    host_bytes = getattr(lib, "vgpu_self_host_bytes", None)
    if host_bytes is not None:
        host_bytes.restype = ctypes.c_uint64

    def stats():
        v = (ctypes.c_uint64 * 5)()
        if vstats is not None:
            vstats(v)
        return {"swap_in": v[0], "swap_out": v[1], "moves": v[2], "spill_in_hbm": v[3], "spilled_ranges": v[4],
                "host_bytes": host_bytes(0) if host_bytes else 0}

    cfg = LlamaConfig.llama3_8b()
    with torch.device("meta"):
        m = Llama(cfg)
    m = m.to(torch.bfloat16).to_empty(device="cuda")  # bf16 storage only: no fp32 copy to spill
    with torch.no_grad():
        for p_ in m.parameters():
            p_.normal_(0, 0.02)
    m.eval()
    kv = _kv(cfg, ctx, torch.device("cuda"))
    tok = torch.randint(0, cfg.vocab, (1, 1), device="cuda")
    torch.cuda.synchronize()
    out = {"after_load": stats()}

    def window(pos0):
        t0 = time.time()
        with torch.inference_mode():
            for p in range(pos0, pos0 + tokens):
                m(tok, kv, p % ctx)
            torch.cuda.synchronize()
        return round(tokens / (time.time() - t0), 2)

    out["spilled_tok_s"] = window(0)
    out["spilled_stats"] = stats()
    print("LOADED", flush=True)
    sys.stdin.readline()
    t_rel = time.time()
    series = []
    for w in range(windows):
        series.append([round(time.time() - t_rel, 2), window((w + 1) * tokens)])
    out["after_release"] = series
    out["final_stats"] = stats()
    return out


def part_c(leave_gib: float, tokens: int, ctx: int, windows: int, migrate: bool) -> dict:
    """Neighbour (plain process, no shim) fills HBM, the pod loads and decodes,
    the neighbour exits, the pod keeps decoding."""
    from vgpu.native import ensure_built, preload_env
    ensure_built()
    repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    nb_code = ("import sys, torch; f, t = torch.cuda.mem_get_info(); "
               f"n = max(0, f - int({leave_gib} * (1 << 30))); "
               "b = torch.empty(n, dtype=torch.uint8, device='cuda'); torch.cuda.synchronize(); "
               "print('HELD', n, flush=True); sys.stdin.readline()")
    nb = subprocess.Popen([sys.executable, "-c", nb_code], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    held = nb.stdout.readline().split()
    env = preload_env()
    env.update({"VGPU_DEVICE_MEMORY_LIMIT_0": "400000m", "VGPU_OVERSUBSCRIBE": "true", "PYTHONPATH": repo,
                "VGPU_LOG_LEVEL": env.get("VGPU_LOG_LEVEL", "3"),
                "VGPU_VMEM_MIGRATE": "1" if migrate else "0"})
    if os.environ.get("VGPU_TRACE") and migrate:
        env["VGPU_TRACE"] = os.environ["VGPU_TRACE"]
        env.setdefault("VGPU_TRACE_EVENTS", "1000000")
    import tempfile
    errf = tempfile.NamedTemporaryFile(mode="w+", prefix="vmem_c_", suffix=".log",
                                       dir=os.environ.get("VGPU_VMEM_LOG_DIR") or None, delete=False)
    pod = subprocess.Popen([sys.executable, "-m", "vgpu.bench.vmem", "--child-c", "--tokens", str(tokens),
                            "--ctx", str(ctx), "--windows", str(windows)], env=env, stdin=subprocess.PIPE,
                           stdout=subprocess.PIPE, stderr=errf, text=True)

    def err_tail():
        errf.seek(0)
        return errf.read()[-2000:]
    line = pod.stdout.readline()
    res: dict = {"migrate": migrate, "neighbour_held_bytes": int(held[1]) if len(held) > 1 else None}
    if not line.startswith("LOADED"):
        nb.stdin.write("\n")
        nb.stdin.flush()
        nb.wait(timeout=60)
        pod.communicate(timeout=60)
        res["error"] = line + err_tail()
        return res
    nb.stdin.write("\n")  # the neighbour frees its HBM and exits
    nb.stdin.flush()
    nb.wait(timeout=60)
    pod.stdin.write("\n")
    pod.stdin.flush()
    outs, _ = pod.communicate(timeout=900)
    js = [l for l in outs.splitlines() if l.startswith("VMEM_C ")]
    res.update(json.loads(js[-1][7:]) if js else {"error": err_tail()})
    return res


def _kv(cfg, ctx, dev):
    import torch
    hd = cfg.dim // cfg.heads
    return [(torch.zeros(1, cfg.kv_heads, ctx, hd, dtype=torch.bfloat16, device=dev),
             torch.zeros(1, cfg.kv_heads, ctx, hd, dtype=torch.bfloat16, device=dev))
            for _ in range(cfg.layers)]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--spill-gib", type=int, default=8)
    ap.add_argument("--budget-gib", type=float, default=8.0)
    ap.add_argument("--tokens", type=int, default=16)
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--child-a", action="store_true")
    ap.add_argument("--child-c", action="store_true")
    ap.add_argument("--part-c", action="store_true", help="only part C (transparent migration A/B)")
    ap.add_argument("--leave-gib", type=float, default=8.0)
    ap.add_argument("--windows", type=int, default=6)
    ap.add_argument("--modes", default="pager,zero_copy")
    ap.add_argument("--skip-a", action="store_true")
    ap.add_argument("--skip-b", action="store_true")
    a = ap.parse_args(argv)
    if a.child_a:
        print("VMEM_A " + json.dumps(part_a_child(a.spill_gib)), flush=True)
        return 0
    if a.child_c:
        print("VMEM_C " + json.dumps(part_c_child(a.tokens, a.ctx, a.windows)), flush=True)
        return 0
    if a.part_c:
        out = {"config": "amd.com/gpumem=400000 (MiB), VGPU_OVERSUBSCRIBE=true, Llama-3-8B bf16 decode, "
                         f"neighbour holds all but {a.leave_gib} GiB of HBM during load"}
        for mode in a.modes.split(","):
            out[mode] = part_c(a.leave_gib, a.tokens, a.ctx, a.windows, mode == "pager")
            print("VMEM_C_RUN " + json.dumps(out[mode]), flush=True)
        print(json.dumps(out), flush=True)
        return 0
    out = {"config": "amd.com/gpumem=400000 (MiB) on one MI355X, VGPU_OVERSUBSCRIBE=true"}
    if not a.skip_a:
        from vgpu.native import ensure_built, preload_env
        ensure_built()
        env = preload_env()
        env.update({"VGPU_DEVICE_MEMORY_LIMIT_0": "400000m", "VGPU_OVERSUBSCRIBE": "true",
                    "PYTHONPATH": os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})
        r = subprocess.run([sys.executable, "-m", "vgpu.bench.vmem", "--child-a", "--spill-gib",
                            str(a.spill_gib)], env=env, capture_output=True, text=True, timeout=1200)
        line = [l for l in r.stdout.splitlines() if l.startswith("VMEM_A ")]
        out["oversubscription"] = json.loads(line[-1][7:]) if line else {"error": r.stderr[-2000:]}
    if not a.skip_b:
        out["llama3_8b_decode"] = part_b(a.budget_gib, a.tokens, a.ctx)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
