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

Part D — model switch under a physical HBM budget, decode as hipGraph replay
(VERDICT r2 item 1).  One pod, cap 400000 MiB, physical budget --budget-gib
(VGPU_DEVICE_MEMORY_PHYSICAL_0, what the device plugin sets on an
oversubscribed node), two Llama-3-8B instances (2 x 15 GiB: footprint >=
1.3 x the budget), no neighbour process.  Model A is loaded, its decode step
captured as a graph and replayed; A idles, model B is loaded, captured and
served; then traffic switches back to A.  With the pager, B's load demotes
the idle A, and A's graph replays (whose kernels the shim saw at capture
time) bring A back while the now idle B gives way.  VGPU_VMEM_MIGRATE=0
(zero-copy) keeps whatever did not fit at load time in host memory for good.

Part E — one Llama-3-8B whose weights alone exceed the budget (a hot set
larger than the budget, read cyclically every token): no pager can beat the
host link here; the pager must simply not do worse than zero-copy.  The
budget is the pod's whole HBM, runtime context included: the context grows
after the weights are placed (queues' context-save areas, code objects), which
the pager answers by demoting managed bytes while zero-copy cannot, so a
zero-copy pod ends up over its budget by that growth (1.19 GB in
profiles/r4/vmem/part_e_books.log).  --context-charge books the context up
front for both modes (VGPU_CONTEXT_CHARGE), so both hold the same HBM.

    python -m vgpu.bench.vmem [--spill-gib 8] [--budget-gib 8] [--tokens 16] [--part-c]
    python -m vgpu.bench.vmem --part-d [--budget-gib 22] [--modes pager,zero_copy]
    python -m vgpu.bench.vmem --part-e [--budget-gib 11.5] [--context-charge-mib 0]
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


def _stats_fn():
    import ctypes
    lib = ctypes.CDLL(None)
    vstats = getattr(lib, "vgpu_self_vmem_stats", None)
    host_bytes = getattr(lib, "vgpu_self_host_bytes", None)
    if host_bytes is not None:
        host_bytes.restype = ctypes.c_uint64

    books_fn = getattr(lib, "vgpu_self_vmem_budget", None)

    def stats():
        v = (ctypes.c_uint64 * 5)()
        if vstats is not None:
            vstats(v)
        out = {"swap_in": v[0], "swap_out": v[1], "moves": v[2], "managed_in_hbm": v[3], "managed_ranges": v[4],
               "host_bytes": host_bytes(0) if host_bytes else 0}
        if books_fn is not None:
            b = (ctypes.c_uint64 * 8)()
            books_fn(ctypes.c_int(0), b)
            out["books"] = dict(zip(("budget", "pod_resident", "managed_in_hbm", "plain", "plain_reserve",
                                     "managed_on_host", "partial_ranges", "hbm_free"), [int(x) for x in b]))
        return out
    return stats


class GraphDecoder:
    """A Llama-3-8B instance with its decode step captured as one hipGraph."""

    def __init__(self, cfg, ctx: int, seed: int):
        import torch
        from vgpu.models.llama import Llama
        torch.manual_seed(seed)
        with torch.device("meta"):
            m = Llama(cfg)
        self.m = m.to(torch.bfloat16).to_empty(device="cuda")
        with torch.no_grad():
            for p_ in self.m.parameters():
                p_.normal_(0, 0.02)
        self.m.eval()
        self.kv = _kv(cfg, ctx, torch.device("cuda"))
        self.tok = torch.randint(0, cfg.vocab, (1, 1), device="cuda")
        self.pos = torch.zeros(1, dtype=torch.long, device="cuda")
        self.ctx = ctx
        self.n = 0
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.inference_mode():
            for _ in range(2):
                self.out = self.m.decode_static(self.tok, self.kv, self.pos)
        torch.cuda.current_stream().wait_stream(s)
        self.g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g), torch.inference_mode():
            self.out = self.m.decode_static(self.tok, self.kv, self.pos)
        torch.cuda.synchronize()

    def window(self, tokens: int) -> float:
        import torch
        t0 = time.time()
        for _ in range(tokens):
            self.pos.fill_(self.n % self.ctx)
            self.g.replay()
            self.n += 1
        torch.cuda.synchronize()
        return round(tokens / (time.time() - t0), 2)


def part_d_child(tokens: int, ctx: int, windows: int, idle_s: float) -> dict:
    """Runs in the pod (libvgpu.so, oversubscribed, physical budget)."""
    import torch
    from vgpu.models.llama import LlamaConfig
    stats = _stats_fn()
    cfg = LlamaConfig.llama3_8b()
    out = {}
    t0 = time.time()
    a = GraphDecoder(cfg, ctx, 1)
    out["load_a_s"] = round(time.time() - t0, 2)
    out["a_first"] = [a.window(tokens) for _ in range(2)]
    out["after_a"] = stats()
    time.sleep(idle_s)  # A idles: its ranges go cold
    t0 = time.time()
    b = GraphDecoder(cfg, ctx, 2)
    out["load_b_s"] = round(time.time() - t0, 2)
    out["after_load_b"] = stats()
    series = []
    t_rel = time.time()
    for _ in range(windows):
        series.append([round(time.time() - t_rel, 2), b.window(tokens)])
    out["b_serving"] = series
    out["after_b"] = stats()
    series = []
    t_rel = time.time()
    for _ in range(windows):  # traffic switches back to A
        series.append([round(time.time() - t_rel, 2), a.window(tokens)])
    out["a_again"] = series
    out["final"] = stats()
    out["torch_mem_total"] = torch.cuda.mem_get_info()[1]
    return out


def part_e_child(tokens: int, ctx: int, windows: int) -> dict:
    from vgpu.models.llama import LlamaConfig
    stats = _stats_fn()
    a = GraphDecoder(LlamaConfig.llama3_8b(), ctx, 1)
    out = {"after_load": stats()}
    t_rel = time.time()
    out["serving"] = [[round(time.time() - t_rel, 2), a.window(tokens)] for _ in range(windows)]
    out["final"] = stats()
    return out


def run_pod_child(part: str, budget_gib: float, migrate: bool, args: list[str], timeout: float = 1500,
                  context_mib: int = 0) -> dict:
    from vgpu.native import ensure_built, preload_env
    ensure_built()
    repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = preload_env()
    env.update({"VGPU_DEVICE_MEMORY_LIMIT_0": "400000m", "VGPU_OVERSUBSCRIBE": "true", "PYTHONPATH": repo,
                "VGPU_DEVICE_MEMORY_PHYSICAL_0": f"{int(budget_gib * 1024)}m",
                **({"VGPU_CONTEXT_CHARGE": f"{context_mib}m"} if context_mib else {}),
                "VGPU_LOG_LEVEL": env.get("VGPU_LOG_LEVEL", "3"), "VGPU_VMEM_MIGRATE": "1" if migrate else "0"})
    if os.environ.get("VGPU_TRACE") and migrate:
        env["VGPU_TRACE"] = os.path.join(os.environ["VGPU_TRACE"], f"part_{part}")
        os.makedirs(env["VGPU_TRACE"], exist_ok=True)
        env.setdefault("VGPU_TRACE_EVENTS", "1000000")
    import tempfile
    errf = tempfile.NamedTemporaryFile(mode="w+", prefix=f"vmem_{part}_", suffix=".log",
                                       dir=os.environ.get("VGPU_VMEM_LOG_DIR") or None, delete=False)
    r = subprocess.run([sys.executable, "-m", "vgpu.bench.vmem", f"--child-{part}", *args], env=env,
                       stdout=subprocess.PIPE, stderr=errf, text=True, timeout=timeout)
    tag = f"VMEM_{part.upper()} "
    js = [l for l in r.stdout.splitlines() if l.startswith(tag)]
    res = {"migrate": migrate, "budget_gib": budget_gib, "context_charge_mib": context_mib}
    if js:
        res.update(json.loads(js[-1][len(tag):]))
    else:
        errf.seek(0)
        res["error"] = f"rc={r.returncode} " + errf.read()[-3000:]
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
    ap.add_argument("--child-d", action="store_true")
    ap.add_argument("--child-e", action="store_true")
    ap.add_argument("--part-d", action="store_true", help="model switch under a physical budget (graph decode)")
    ap.add_argument("--part-e", action="store_true", help="hot set beyond the budget (graph decode)")
    ap.add_argument("--idle-s", type=float, default=3.0)
    ap.add_argument("--context-charge-mib", type=int, default=0,
                    help="book this much runtime context at first use (both modes; see Part E)")
    ap.add_argument("--skip-a", action="store_true")
    ap.add_argument("--skip-b", action="store_true")
    a = ap.parse_args(argv)
    if a.child_a:
        print("VMEM_A " + json.dumps(part_a_child(a.spill_gib)), flush=True)
        return 0
    if a.child_c:
        print("VMEM_C " + json.dumps(part_c_child(a.tokens, a.ctx, a.windows)), flush=True)
        return 0
    if a.child_d:
        print("VMEM_D " + json.dumps(part_d_child(a.tokens, a.ctx, a.windows, a.idle_s)), flush=True)
        return 0
    if a.child_e:
        print("VMEM_E " + json.dumps(part_e_child(a.tokens, a.ctx, a.windows)), flush=True)
        return 0
    if a.part_d or a.part_e:
        part = "d" if a.part_d else "e"
        out = {"config": f"amd.com/gpumem=400000 (MiB), VGPU_OVERSUBSCRIBE=true, physical budget {a.budget_gib} GiB, "
                         + ("two Llama-3-8B bf16 (model switch)" if a.part_d else "one Llama-3-8B bf16")
                         + ", decode step as one hipGraph replay, ctx " + str(a.ctx)}
        for mode in a.modes.split(","):
            out[mode] = run_pod_child(part, a.budget_gib, mode == "pager",
                                      ["--tokens", str(a.tokens), "--ctx", str(a.ctx), "--windows", str(a.windows),
                                       "--idle-s", str(a.idle_s)], context_mib=a.context_charge_mib)
            print(f"VMEM_{part.upper()}_RUN " + json.dumps(out[mode]), flush=True)
        print(json.dumps(out), flush=True)
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
