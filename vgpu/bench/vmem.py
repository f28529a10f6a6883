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

    python -m vgpu.bench.vmem [--spill-gib 8] [--budget-gib 8] [--tokens 16]
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
    ap.add_argument("--skip-a", action="store_true")
    ap.add_argument("--skip-b", action="store_true")
    a = ap.parse_args(argv)
    if a.child_a:
        print("VMEM_A " + json.dumps(part_a_child(a.spill_gib)), flush=True)
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
