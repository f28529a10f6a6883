"""Device-side probes run inside a (capped) vGPU process; each prints one JSON
line.  Used by the GPU tests and by the accuracy benchmarks.

  python -m vgpu.bench.probes census [blocks] [spin_ticks]
      which physical CUs (XCD, SE, SH, CU) the process's workgroups ran on
  python -m vgpu.bench.probes busy [blocks] [iters] [reps]
      wall time of a fixed amount of VALU work (compute-share accuracy)
  python -m vgpu.bench.probes cap [chunk_mib]
      reported total + how many bytes torch could allocate before OOM
  python -m vgpu.bench.probes graph [blocks_a] [blocks_b]
      capture two busy kernels into a hipGraph and replay it (the library
      charges a graph launch by its kernel nodes' workgroups; see VGPU_TRACE)
  python -m vgpu.bench.probes arrays [cap_mib]
      hipMalloc3D / hipMallocArray / hipArray3DCreate past the cap, and
      hipModuleLoadData of a gfx950 code object (module charge class)
  python -m vgpu.bench.probes smi [alloc_mib]
      what amdsmi (python bindings over libamd_smi, the amd-smi CLI's path)
      reports for VRAM total / used after torch allocates alloc_mib
Every probe also reports the enforcement library's own view ("shim") when
the library is loaded in the process.
"""
from __future__ import annotations

import glob
import json
import os
import sys
import time


def shim_stats(dev: int = 0) -> dict | None:
    """Per-class charge of this process and the HSA interception mode, read
    through the preloaded enforcement library's C ABI (None when not loaded)."""
    import ctypes
    try:
        lib = ctypes.CDLL(None)
        fn = lib.vgpu_self_usage
    except (OSError, AttributeError):
        return None
    fn.restype = ctypes.c_uint64
    fn.argtypes = [ctypes.c_int, ctypes.c_int]
    names = ("context", "module", "buffer", "host", "total")
    out = {k: int(fn(dev, i)) for i, k in enumerate(names)}
    out["hsa_table_mode"] = int(lib.vgpu_self_hsa_table_mode())
    lib.vgpu_self_hsa_dispatches.restype = ctypes.c_uint64
    out["hsa_dispatches"] = int(lib.vgpu_self_hsa_dispatches())
    out["hsa_intercepted_queues"] = int(lib.vgpu_self_hsa_intercepted_queues())
    return out


def smi(alloc_mib: int = 1024) -> dict:
    import torch
    x = torch.empty(alloc_mib << 20, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    try:
        import amdsmi
        amdsmi.amdsmi_init()
    except Exception as e:  # no amdsmi bindings / no access on this host
        return {"error": repr(e)}
    h = amdsmi.amdsmi_get_processor_handles()[0]
    res: dict = {"torch_total": int(torch.cuda.mem_get_info()[1])}
    calls = {
        "total": lambda: int(amdsmi.amdsmi_get_gpu_memory_total(h, amdsmi.AmdSmiMemoryType.VRAM)),
        "used": lambda: int(amdsmi.amdsmi_get_gpu_memory_usage(h, amdsmi.AmdSmiMemoryType.VRAM)),
        "vram_usage": lambda: amdsmi.amdsmi_get_gpu_vram_usage(h),
        "vram_info": lambda: int(amdsmi.amdsmi_get_gpu_vram_info(h)["vram_size"]),
    }
    for k, fn in calls.items():
        try:
            v = fn()
        except Exception as e:  # not every query is supported on every host/partition mode
            res.setdefault("errors", {})[k] = repr(e)[:200]
            continue
        if k == "vram_usage":
            res["vram_total_mb"], res["vram_used_mb"] = int(v["vram_total"]), int(v["vram_used"])
        else:
            res[k] = v
    amdsmi.amdsmi_shut_down()
    del x
    return res


def census(blocks: int = 4096, spin: int = 200000) -> dict:
    import torch
    from vgpu.ops import kernels as K
    K.census(64, 100)  # warm the code object
    torch.cuda.synchronize()
    xh, ticks = K.census(blocks, spin)
    torch.cuda.synchronize()
    xcc = xh[:, 0].cpu()
    f = K.decode_hw_id(xh[:, 1].cpu())
    tuples = set(zip(xcc.tolist(), f["se"].tolist(), f["sh"].tolist(), f["cu"].tolist()))
    per_xcc: dict[int, int] = {}
    for x, *_ in tuples:
        per_xcc[x] = per_xcc.get(x, 0) + 1
    per_se: dict[str, int] = {}
    for x, se, sh, cu in tuples:
        k = f"{x}.{se}"
        per_se[k] = per_se.get(k, 0) + 1
    return {"distinct_cus": len(tuples), "per_xcc": {str(k): v for k, v in sorted(per_xcc.items())},
            "per_se": per_se, "blocks": blocks,
            "cus_prop": torch.cuda.get_device_properties(0).multi_processor_count}


def busy(blocks: int = 8192, iters: int = 20000, reps: int = 5) -> dict:
    import torch
    from vgpu.ops import kernels as K
    K.busy(blocks, 100)
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        K.busy(blocks, iters)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    return {"blocks": blocks, "iters": iters, "times": times, "median_s": sorted(times)[len(times) // 2]}


def busyvia(blocks: int = 8192, iters: int = 20000, reps: int = 5, path: int = 1, launches: int = 1) -> dict:
    """busy() through another launch entry point (kernels.busy_via); each rep
    is `launches` back-to-back launches."""
    import torch
    from vgpu.ops import kernels as K
    K.busy_via(blocks, 100, path)
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for _ in range(launches):
            K.busy_via(blocks, iters, path)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    return {"blocks": blocks, "iters": iters, "path": path, "launches": launches, "times": times,
            "median_s": sorted(times)[len(times) // 2]}


def pitch(chunk_mib: int = 1024) -> dict:
    """hipMemAllocPitch (the driver-style pitched allocation, reference
    cuMemAllocPitch_v2) in chunk_mib pieces until the runtime refuses."""
    import ctypes
    import torch
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemAllocPitch.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint]
    ptrs, last = [], 0
    for _ in range(4096):
        p, pt = ctypes.c_void_p(), ctypes.c_size_t()
        last = hip.hipMemAllocPitch(ctypes.byref(p), ctypes.byref(pt), 1 << 20, chunk_mib, 4)
        if last != 0:
            break
        ptrs.append(p)
    hip.hipGetLastError()
    res = {"allocated": len(ptrs) * (chunk_mib << 20), "chunks": len(ptrs), "last_error": last,
           "usage": shim_stats()}
    for p in ptrs:
        hip.hipFree(p)
    return res


def cap(chunk_mib: int = 1024) -> dict:
    import torch
    free, total = torch.cuda.mem_get_info()
    props = torch.cuda.get_device_properties(0)
    blocks = []
    try:
        while True:
            blocks.append(torch.empty(chunk_mib << 20, dtype=torch.uint8, device="cuda"))
    except torch.OutOfMemoryError:
        pass
    res = {"free": free, "total": total, "prop_total": props.total_memory,
           "allocated": len(blocks) * (chunk_mib << 20), "reserved": torch.cuda.memory_reserved()}
    # release one chunk so the verification's own small buffers fit under the cap
    if blocks:
        blocks.pop()
        torch.cuda.empty_cache()
    # touch everything: prove the bytes are real
    from vgpu.ops import kernels as K
    errs = 0
    for i, b in enumerate(blocks):
        K.fill_pattern(b, i + 1)
    for i, b in enumerate(blocks):
        errs += K.verify_pattern(b, i + 1)
    res["verify_errors"] = errs
    return res


def graph(blocks_a: int = 1000, blocks_b: int = 3000) -> dict:
    import torch
    from vgpu.ops import kernels as K
    K.busy(blocks_a, 10)  # load the module / warm up outside the capture
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            K.busy(blocks_a, 10)
            K.busy(blocks_b, 10)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    return {"blocks": [blocks_a, blocks_b], "replays": 2}


def forkjoin(replays: int = 5, width: int = 1024) -> dict:
    """A two-stream training step captured as one graph and replayed: the
    forward and the data-gradient chain on the capture stream, the weight
    gradients of the first layer on a side stream (a parallel branch of the
    graph), joined before the SGD update.  Returns the replayed parameters'
    max deviation from the same steps run eagerly.  Under GPU_MAX_HW_QUEUES=1
    the HIP runtime's multi-stream executor crashes on such a graph unless the
    enforcement library chains it (hooks_hip.cpp chain_graph)."""
    import torch
    torch.manual_seed(0)
    dev = torch.device("cuda")
    x = torch.randn(512, width, device=dev)
    w1 = torch.randn(width, width, device=dev) / width ** 0.5
    w2 = torch.randn(width, width, device=dev) / width ** 0.5
    lr = 1e-3

    def step(w1, w2, side):
        main = torch.cuda.current_stream()
        h = torch.relu(x @ w1)
        y = h @ w2
        dy = 2 * y / y.numel()
        g2 = h.t() @ dy
        dh = (dy @ w2.t()) * (h > 0)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            g1 = x.t() @ dh          # the branch: weight gradient of layer 1
        w2.sub_(lr * g2)
        main.wait_stream(side)
        w1.sub_(lr * g1)

    ref1, ref2 = w1.clone(), w2.clone()
    side = torch.cuda.Stream()
    for _ in range(2 + replays):  # eager reference: the warmup steps + the replays
        step(ref1, ref2, side)
    torch.cuda.synchronize()
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        for _ in range(2):  # warmup on the capture stream, as torch requires
            step(w1, w2, side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        step(w1, w2, side)
    for _ in range(replays - 1):
        g.replay()
    torch.cuda.synchronize()
    # capture does not run the step: 2 warmup + (replays - 1) replays so far
    g.replay()
    torch.cuda.synchronize()
    err = max((w1 - ref1).abs().max().item(), (w2 - ref2).abs().max().item())
    return {"replays": replays, "max_err": err, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "")}


def arrays(cap_mib: int = 8192) -> dict:
    """Array-class allocations through the real HIP runtime (ctypes): under a
    cap of `cap_mib`, the second 6 GiB hipMalloc3D and a 4 GiB hipMallocArray
    must fail; a code object must land in the module class."""
    import ctypes
    from pathlib import Path
    import torch
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")  # the runtime torch already loaded

    class Extent(ctypes.Structure):
        _fields_ = [("width", ctypes.c_size_t), ("height", ctypes.c_size_t), ("depth", ctypes.c_size_t)]

    class Pitched(ctypes.Structure):
        _fields_ = [("ptr", ctypes.c_void_p), ("pitch", ctypes.c_size_t), ("xsize", ctypes.c_size_t),
                    ("ysize", ctypes.c_size_t)]

    class ChanDesc(ctypes.Structure):
        _fields_ = [("x", ctypes.c_int), ("y", ctypes.c_int), ("z", ctypes.c_int), ("w", ctypes.c_int),
                    ("f", ctypes.c_int)]

    class Arr3D(ctypes.Structure):
        _fields_ = [("Width", ctypes.c_size_t), ("Height", ctypes.c_size_t), ("Depth", ctypes.c_size_t),
                    ("Format", ctypes.c_int), ("NumChannels", ctypes.c_uint), ("Flags", ctypes.c_uint)]

    hip.hipMalloc3D.argtypes = [ctypes.POINTER(Pitched), Extent]
    res: dict = {}
    a, b = Pitched(), Pitched()
    six = Extent(6 << 30, 1, 1)
    res["malloc3d_a"] = hip.hipMalloc3D(ctypes.byref(a), six)
    res["malloc3d_b"] = hip.hipMalloc3D(ctypes.byref(b), six)
    hip.hipGetLastError()
    fd = ChanDesc(32, 0, 0, 0, 2)  # hipChannelFormatKindFloat
    arr, arr2, arr3 = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    hip.hipMallocArray.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ChanDesc), ctypes.c_size_t,
                                   ctypes.c_size_t, ctypes.c_uint]
    res["array_a"] = hip.hipMallocArray(ctypes.byref(arr), ctypes.byref(fd), 8192, 8192, 0)    # 256 MiB
    res["array_b"] = hip.hipMallocArray(ctypes.byref(arr2), ctypes.byref(fd), 32768, 32768, 0)  # 4 GiB
    hip.hipGetLastError()
    d3 = Arr3D(1024, 1024, 1024, 0x20, 1, 0)  # HIP_AD_FORMAT_FLOAT: 4 GiB
    res["array3d"] = hip.hipArray3DCreate(ctypes.byref(arr3), ctypes.byref(d3))
    hip.hipGetLastError()
    image = (Path(__file__).resolve().parents[1] / "_lib" / "module_probe.hsaco").read_bytes()
    mod = ctypes.c_void_p()
    buf = ctypes.create_string_buffer(image, len(image))
    res["module"] = hip.hipModuleLoadData(ctypes.byref(mod), buf)
    res["image_bytes"] = len(image)
    res["usage"] = shim_stats()
    hip.hipModuleUnload(mod)
    if res["array_a"] == 0:
        hip.hipFreeArray(arr)
    if res["malloc3d_a"] == 0:
        hip.hipFree(ctypes.c_void_p(a.ptr))
    res["usage_after_free"] = shim_stats()
    return res


def progress(seconds: int = 10, blocks: int = 256, iters: int = 2000) -> dict:
    """Launch small busy kernels back to back for `seconds`, printing
    `PROGRESS <launches> <t>` lines (priority-feedback tests watch them)."""
    import torch
    from vgpu.ops import kernels as K
    torch.cuda.init()
    t0 = time.time()
    n = 0
    while time.time() - t0 < seconds:
        K.busy(blocks, iters)
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
            print(f"PROGRESS {n} {time.time():.3f}", flush=True)
    torch.cuda.synchronize()
    return {"launches": n}


def capheld(chunk_mib: int = 256) -> dict:
    """Allocate chunks until the cap refuses one, print `HELD <bytes>`, and keep
    them until a line arrives on stdin (two of these race for one region)."""
    import torch
    torch.cuda.init()
    torch.empty(1, device="cuda")
    print("READY", flush=True)
    sys.stdin.readline()  # start line: both processes allocate at the same time
    n = chunk_mib << 20
    held = []
    while True:
        try:
            held.append(torch.empty(n, dtype=torch.uint8, device="cuda"))
        except torch.OutOfMemoryError:
            break
        if len(held) > 4096:
            break
        time.sleep(0.005)  # interleave with the other process
    torch.cuda.synchronize()
    print(f"HELD {len(held) * n}", flush=True)
    sys.stdin.readline()
    return {"held": len(held) * n, "usage": shim_stats()}


def vmem(block_gib: int = 4, wait_s: int = 20) -> dict:
    """Transparent migration on the device (oversubscribed pod): fill HBM with
    plain blocks until one spills, use the spilled block from kernels (read
    bandwidth in place), free two plain blocks, keep using the spilled block
    until the shim's pager has moved it into HBM, then read it again."""
    import ctypes

    import torch
    from vgpu.ops import kernels as K
    lib = ctypes.CDLL(None)
    host_bytes = lib.vgpu_self_host_bytes
    host_bytes.restype = ctypes.c_uint64

    def vstats():
        v = (ctypes.c_uint64 * 5)()
        lib.vgpu_self_vmem_stats(v)
        return {"swap_in": v[0], "swap_out": v[1], "moves": v[2], "spill_in_hbm": v[3], "ranges": v[4]}

    def read_gbps(t, seed, reps=3):
        K.verify_pattern(t, seed)
        torch.cuda.synchronize()
        t0 = time.time()
        errs = 0
        for _ in range(reps):
            errs += K.verify_pattern(t, seed)
        torch.cuda.synchronize()
        return round(reps * t.numel() / (time.time() - t0) / 1e9, 1), errs

    import faulthandler
    faulthandler.dump_traceback_later(30, repeat=True)

    def note(msg):
        print(f"VMEM_PROBE {time.time():.3f} {msg} {vstats()}", file=sys.stderr, flush=True)

    n = block_gib << 30
    blocks = []
    while True:
        blocks.append(torch.empty(n, dtype=torch.uint8, device="cuda"))
        if host_bytes(0):
            break
        if len(blocks) > 400:
            return {"error": "no spill"}
    spilled = blocks.pop()
    note(f"spilled after {len(blocks)} plain blocks")
    res = {"plain_blocks": len(blocks), "host_bytes": host_bytes(0), "after_spill": vstats()}
    K.fill_pattern(spilled, 42)
    torch.cuda.synchronize()
    res["in_place_GBps"], res["in_place_errors"] = read_gbps(spilled, 42, 2)
    res["after_use_full"] = vstats()
    note("used in place")
    del blocks[-2:]
    torch.cuda.empty_cache()
    note("freed two blocks")
    t0 = time.time()
    while time.time() - t0 < wait_s:
        K.verify_pattern(spilled, 42)
        torch.cuda.synchronize()
        if vstats()["spill_in_hbm"] >= spilled.numel():
            break
        time.sleep(0.05)
    res["promote_wait_s"] = round(time.time() - t0, 2)
    note("promoted")
    faulthandler.cancel_dump_traceback_later()
    res["after_room"] = vstats()
    res["promoted_GBps"], res["promoted_errors"] = read_gbps(spilled, 42)
    res["host_bytes_after"] = host_bytes(0)
    del spilled, blocks
    torch.cuda.empty_cache()
    res["final"] = vstats()
    return res


def vmemcopy(mib: int = 512) -> dict:
    """Host copies into and out of managed ranges (physical budget set, so a
    large allocation is a managed range from the start).  Without the shim's
    staging KFD moves every page such a copy touches to system memory and the
    GPU reads it over the host link afterwards (native/probes/managed_access.hip).
    Reads each range after: D2H from it, sync H2D into it, async H2D from
    pinned memory into it."""
    import ctypes

    import torch
    from vgpu.ops import kernels as K
    lib = ctypes.CDLL(None)

    def ranges():
        v = (ctypes.c_uint64 * 5)()
        lib.vgpu_self_vmem_stats(v)
        return int(v[4])

    def read_gbps(t, seed, reps=5):
        K.verify_pattern(t, seed)
        torch.cuda.synchronize()
        t0 = time.time()
        errs = 0
        for _ in range(reps):
            errs += K.verify_pattern(t, seed)
        torch.cuda.synchronize()
        return round(reps * t.numel() / (time.time() - t0) / 1e9, 1), errs

    n = mib << 20
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    K.fill_pattern(src, 7)
    torch.cuda.synchronize()
    res = {"ranges": ranges()}
    res["fresh_GBps"], e0 = read_gbps(src, 7)
    t0 = time.time()
    h = src.cpu()  # D2H out of a managed range
    res["d2h_ms"] = round((time.time() - t0) * 1e3, 1)
    res["after_d2h_GBps"], e1 = read_gbps(src, 7)
    dst = torch.empty(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t0 = time.time()
    dst.copy_(h)  # sync H2D into a managed range
    torch.cuda.synchronize()
    res["h2d_ms"] = round((time.time() - t0) * 1e3, 1)
    res["after_h2d_GBps"], e2 = read_gbps(dst, 7)
    hp = h.pin_memory()
    dst2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    dst2.copy_(hp, non_blocking=True)  # async H2D from pinned memory
    torch.cuda.synchronize()
    res["after_async_h2d_GBps"], e3 = read_gbps(dst2, 7)
    # 2-D copies and memsets.  hipMemcpy2D host -> range
    # (4 KiB rows: the pattern survives, pitch = width), then hipMemset over
    # the first half of another range and the pattern refilled on the GPU.
    # The process-wide symbols, as an application's own calls resolve them (the
    # shim's hooks first when it is preloaded): a handle on libamdhip64.so would
    # call the runtime directly, and a memset the shim never sees races its pager
    # (the runtime's memset of a managed range moved pages to host memory).
    hip = ctypes.CDLL(None)
    if not hasattr(hip, "hipMemset"):
        hip = ctypes.CDLL("libamdhip64.so")
    dst3 = torch.empty(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    w = 4096
    rc2 = hip.hipMemcpy2D(ctypes.c_void_p(dst3.data_ptr()), ctypes.c_size_t(w), ctypes.c_void_p(hp.data_ptr()),
                          ctypes.c_size_t(w), ctypes.c_size_t(w), ctypes.c_size_t(n // w), 1)  # HostToDevice
    torch.cuda.synchronize()
    res["memcpy2d_rc"] = rc2
    res["after_memcpy2d_GBps"], e4 = read_gbps(dst3, 7)
    rc3 = hip.hipMemset(ctypes.c_void_p(dst2.data_ptr()), 0, ctypes.c_size_t(n // 2))
    torch.cuda.synchronize()
    res["memset_rc"] = rc3
    res["memset_zeroed"] = bool(int(dst2[: n // 2].count_nonzero()) == 0)
    K.fill_pattern(dst2, 7)
    torch.cuda.synchronize()
    res["after_memset_GBps"], e5 = read_gbps(dst2, 7)
    res["errors"] = e0 + e1 + e2 + e3 + e4 + e5
    res["ranges_end"] = ranges()
    return res


def rcclloop(iters: int = 200, mib: int = 64, port: int = 0) -> dict:
    """A world-size-1 RCCL process group all-reducing `mib` MiB `iters` times
    (the collective path of a DDP pod), timed; the sum is checked."""
    import datetime
    import socket

    import torch
    import torch.distributed as dist
    if not port:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=120), device_id=dev)
    x = torch.full(((mib << 20) // 4,), 3.0, device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    t0 = time.time()
    for i in range(iters):
        dist.all_reduce(x)
        if i % 20 == 0:
            torch.cuda.synchronize()
            print(f"PROGRESS {i} {time.time():.3f}", flush=True)
    torch.cuda.synchronize()
    dt = time.time() - t0
    ok = bool(torch.all(x == 3.0).item())
    dist.destroy_process_group()
    return {"iters": iters, "seconds": round(dt, 3), "ms_per_allreduce": round(1e3 * dt / iters, 3), "sum_ok": ok}


def _vram_used_files() -> dict[str, int]:
    import glob
    out = {}
    for f in glob.glob("/sys/bus/pci/devices/*/mem_info_vram_used"):
        try:
            out[f] = int(open(f).read())
        except (OSError, ValueError):
            pass
    return out


def asynccap(cap_mib: int = 8192, graph_mib: int = 1024) -> dict:
    """Stream-ordered allocations under the cap: run with
    PYTORCH_HIP_ALLOC_CONF=backend:hipMallocAsync.  Alloc / free / re-alloc
    cycles of varying sizes up to OOM, then captured graphs whose temporaries
    are graph alloc nodes.  amdgpu's own VRAM counter (mem_info_vram_used) is
    sampled throughout; the peak over the pre-init baseline is reported."""
    import random
    base = _vram_used_files()  # before this process touches the GPU
    import torch
    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    path = f"/sys/bus/pci/devices/{bdf}/mem_info_vram_used"
    if path not in base:
        return {"error": f"no VRAM counter at {path}", "candidates": sorted(base)}
    baseline = base[path]
    peak = 0
    samples = 0
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    pool = ctypes.c_void_p()
    hip.hipDeviceGetMemPool(ctypes.byref(pool), 0)
    phases: dict[str, dict] = {}
    phase = "cycles"

    def pool_attr(a: int) -> int:
        v = ctypes.c_uint64(0)
        hip.hipMemPoolGetAttribute(pool, a, ctypes.byref(v))
        return v.value

    # KFD's own per-process VRAM counter (/sys/class/kfd/kfd/proc/<host pid>/vram_<gpu id>):
    # updated when a buffer object is created or destroyed, unlike amdgpu's
    # device-wide mem_info_vram_used, which lags frees and counts other processes.
    selfpid = ctypes.CDLL(None).vgpu_self_host_pid  # int vgpu_self_host_pid(int* src)
    src = ctypes.c_int(0)
    hp = selfpid(ctypes.byref(src)) or os.getpid()
    kfd_files = glob.glob(f"/sys/class/kfd/kfd/proc/{hp}/vram_*") or \
        glob.glob(f"/sys/class/kfd/kfd/proc/{os.getpid()}/vram_*")
    kfd_procs = sorted(os.listdir("/sys/class/kfd/kfd/proc")) if os.path.isdir("/sys/class/kfd/kfd/proc") else None
    kfd_diag = {"host_pid": hp, "host_pid_src": src.value, "pid": os.getpid(),
                "kfd_proc_entries": None if kfd_procs is None else len(kfd_procs)}
    kfd_peak = 0

    def kfd_vram() -> int:
        tot = 0
        for f in kfd_files:
            try:
                tot += int(open(f).read())
            except (OSError, ValueError):
                pass
        return tot

    def sample():
        nonlocal peak, samples, kfd_peak
        torch.cuda.synchronize()
        v = int(open(path).read()) - baseline
        peak = max(peak, v)
        k = kfd_vram()
        kfd_peak = max(kfd_peak, k)
        samples += 1
        ph = phases.setdefault(phase, {"kfd_peak": 0})
        if k >= ph["kfd_peak"]:
            st = shim_stats() or {}
            ph.update({"kfd_peak": k, "vram_used_over_baseline": v, "pool_reserved": pool_attr(5),
                       "pool_used": pool_attr(7), "shim_total": st.get("total"),
                       "torch_reserved": torch.cuda.memory_reserved()})

    rng = random.Random(0)
    MiB = 1 << 20
    reached = 0
    ooms = 0
    for rnd in range(3):
        live = []
        while True:
            n = rng.choice([64, 256, 512, 768, 1024, 1536]) * MiB
            try:
                live.append(torch.empty(n, dtype=torch.uint8, device="cuda").fill_(rnd))
            except torch.OutOfMemoryError:
                ooms += 1
                break
            sample()
        reached = max(reached, sum(t.numel() for t in live))
        del live[::2]
        sample()
        while True:  # re-allocate other sizes into the holes and past them
            n = rng.choice([96, 384, 640, 1280]) * MiB
            try:
                live.append(torch.empty(n, dtype=torch.uint8, device="cuda").fill_(rnd + 1))
            except torch.OutOfMemoryError:
                ooms += 1
                break
            sample()
        del live
        sample()
    # graphs whose temporaries are stream-ordered allocations (graph alloc nodes)
    phase = "graphs"
    x = torch.randn(graph_mib * MiB // 4, device="cuda")
    graph_ok = 0
    for k in (1, 2, 3):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            y = (x * k + 1).relu().sum()  # warm-up outside the capture
        torch.cuda.current_stream().wait_stream(s)
        try:
            with torch.cuda.graph(g):
                y = ((x * k + 1).relu() * (x - k)).sum()
            for _ in range(3):
                g.replay()
                sample()
            graph_ok += 1
        except (torch.OutOfMemoryError, RuntimeError) as e:
            print("graph", k, "refused:", str(e)[:200], flush=True)
        del g
        sample()
    return {"cap": cap_mib * MiB, "baseline": baseline, "peak_over_baseline": peak, "samples": samples,
            "kfd_vram_peak": kfd_peak, "kfd_files": kfd_files, "kfd_diag": kfd_diag,
            "max_live_reached": reached, "ooms": ooms, "graphs_replayed": graph_ok, "y": float(y),
            "backend": os.environ.get("PYTORCH_HIP_ALLOC_CONF", ""), "phases": phases}


def _sysfs_vram(dev: int = 0) -> tuple[int, int] | None:
    """(total, used) bytes from amdgpu's VRAM counters (they count KFD SVM pages,
    which hipMemGetInfo does not); None when unreadable."""
    import ctypes
    buf = ctypes.create_string_buffer(64)
    if ctypes.CDLL("libamdhip64.so").hipDeviceGetPCIBusId(buf, 64, dev) != 0:
        return None
    base = f"/sys/bus/pci/devices/{buf.value.decode().lower()}"
    try:
        with open(f"{base}/mem_info_vram_total") as f:
            total = int(f.read())
        with open(f"{base}/mem_info_vram_used") as f:
            used = int(f.read())
        return total, used
    except OSError:
        return None


def vmemfull(gib: int = 4) -> dict:
    """The full-HBM migration case (native/probes/svm_probe.hip
    part F): an application-managed range of `gib` GiB, filled and moved to host
    memory; a plain balloon then leaves gib/2 GiB of HBM free; the application
    prefetches the whole range back into HBM.  Under the shim the prefetch is cut
    to the free HBM beyond VGPU_VMEM_HEADROOM_MB, so KFD is never asked to
    migrate into a full device.  Reports the prefetch time, the data check, the
    read bandwidth and physical free HBM before and after."""
    import ctypes

    import torch
    from vgpu.native import load_kernels
    import faulthandler
    faulthandler.dump_traceback_later(60, repeat=True)
    hip = ctypes.CDLL("libamdhip64.so")
    kl = load_kernels()
    n = gib << 30
    vr = _sysfs_vram()
    if vr is None:
        return {"error": "sysfs VRAM counters unreadable"}
    torch.empty(1, device="cuda")
    ptr = ctypes.c_void_p()
    rc = hip.hipMallocManaged(ctypes.byref(ptr), ctypes.c_size_t(n), ctypes.c_uint(1))
    if rc:
        return {"error": f"hipMallocManaged {rc}"}
    s0 = ctypes.c_void_p(0)
    kl.vgpu_fill_pattern(ptr, n, 77, s0)
    torch.cuda.synchronize()
    hip.hipMemPrefetchAsync(ptr, ctypes.c_size_t(n), ctypes.c_int(-1), s0)
    torch.cuda.synchronize()
    # Device-wide counters: memory another process is still releasing (the
    # test before this one may have just exited with 255 GB) shows up here, so
    # wait until the counter settles, then top the balloon up until only
    # `leave` is free.
    prev, t_end = None, time.time() + 20
    while time.time() < t_end:
        used = _sysfs_vram()[1]
        if prev is not None and abs(used - prev) < (256 << 20):
            break
        prev = used
        time.sleep(0.5)
    leave = n // 2
    balloon = []
    for _ in range(8):
        total, used = _sysfs_vram()
        extra = total - used - leave
        if extra < (512 << 20):
            break
        balloon.append(torch.empty(extra, dtype=torch.uint8, device="cuda"))
        torch.cuda.synchronize()
        time.sleep(0.2)
    balloon_bytes = sum(b.numel() for b in balloon)
    free_before = (lambda t: t[0] - t[1])(_sysfs_vram())
    t0 = time.time()
    rc = hip.hipMemPrefetchAsync(ptr, ctypes.c_size_t(n), ctypes.c_int(0), s0)
    torch.cuda.synchronize()
    dt = time.time() - t0
    free_after = (lambda t: t[0] - t[1])(_sysfs_vram())
    err = torch.zeros(1, dtype=torch.int64, device="cuda")
    kl.vgpu_verify_pattern(ptr, n, 77, ctypes.c_void_p(err.data_ptr()), s0)
    torch.cuda.synchronize()
    errors = int(err.item())
    t1 = time.time()
    for _ in range(3):
        kl.vgpu_verify_pattern(ptr, n, 77, ctypes.c_void_p(err.data_ptr()), s0)
    torch.cuda.synchronize()
    gbps = round(3 * n / (time.time() - t1) / 1e9, 1)
    del balloon
    torch.cuda.empty_cache()
    hip.hipFree(ptr)
    faulthandler.cancel_dump_traceback_later()
    return {"bytes": n, "total": total, "used_at_start": used, "balloon": balloon_bytes,
            "free_before": free_before, "free_after": free_after,
            "prefetch_rc": rc, "prefetch_s": round(dt, 3), "errors": errors, "read_GBps": gbps,
            "headroom_mb": int(os.environ.get("VGPU_VMEM_HEADROOM_MB", "2048"))}


def evictee(gib: int = 64, block_gib: int = 4) -> dict:
    """The low-priority side of an evicting suspend.  Allocates
    `gib` GiB in `block_gib` blocks (managed ranges under VGPU_SUSPEND_EVICT),
    fills each with the K3 pattern, prints `READY {json}` and then serves
    commands read from stdin: `STATS` (one `STATS {json}` line: vmem counters,
    host bytes), `VERIFY` (check every block, report errors and read GB/s) and
    `EXIT`.  The driver suspends / resumes it with SIGUSR2 / SIGUSR1 in between."""
    import ctypes

    import torch
    from vgpu.ops import kernels as K
    lib = ctypes.CDLL(None)
    host_bytes = lib.vgpu_self_host_bytes
    host_bytes.restype = ctypes.c_uint64

    def stats():
        v = (ctypes.c_uint64 * 5)()
        lib.vgpu_self_vmem_stats(v)
        m = (ctypes.c_uint64 * 8)()
        lib.vgpu_self_vmm_stats(m)  # the VMM vehicle (VGPU_SUSPEND_VMM, default with VGPU_SUSPEND_EVICT)
        return {"swap_in": v[0], "swap_out": v[1], "moves": v[2], "in_hbm": v[3], "ranges": v[4],
                "host_bytes": int(host_bytes(0)), "vmm_ranges": m[0], "vmm_bytes": m[1], "vmm_evicted": m[2],
                "vmm_suspend_s": round(m[3] / 1e9, 3), "vmm_resume_s": round(m[4] / 1e9, 3), "vmm_cycles": m[5],
                "vmm_pin_s": round(m[6] / 1e9, 3), "vmm_map_s": round(m[7] / 1e9, 3)}

    blocks = []
    for i in range(gib // block_gib):
        t = torch.empty(block_gib << 30, dtype=torch.uint8, device="cuda")
        K.fill_pattern(t, 100 + i)
        blocks.append(t)
    torch.cuda.synchronize()
    print("READY " + json.dumps(stats()), flush=True)
    res = {}
    for line in sys.stdin:
        cmd = line.strip()
        if cmd == "STATS":
            print("STATS " + json.dumps(stats()), flush=True)
        elif cmd == "VERIFY":
            t0 = time.time()
            errs = sum(K.verify_pattern(b, 100 + i) for i, b in enumerate(blocks))
            torch.cuda.synchronize()
            first = time.time() - t0
            t0 = time.time()
            errs += sum(K.verify_pattern(b, 100 + i) for i, b in enumerate(blocks))
            torch.cuda.synchronize()
            res = {"errors": errs, "first_pass_s": round(first, 3),
                   "second_pass_GBps": round(gib * (1 << 30) / (time.time() - t0) / 1e9, 1), **stats()}
            print("VERIFIED " + json.dumps(res), flush=True)
        elif cmd == "EXIT":
            break
    return res


def _ipc_child(q_in, q_out) -> None:
    """ipcshare's consumer process: sum the shared tensor, write element 0."""
    import torch
    try:
        t = q_in.get(timeout=120)
        s = int(t.sum().item())
        t[0] = -1
        torch.cuda.synchronize()
        q_out.put({"sum": s})
        del t
    except Exception as e:  # report, never hang the parent
        q_out.put({"error": repr(e)[:400]})


def ipcshare(mib: int = 64) -> dict:
    """share a CUDA tensor with another process of the container
    (torch.multiprocessing, CUDA IPC) while allocations of >= 32 MiB are VMM
    mappings (VGPU_SUSPEND_EVICT).  Reports whether the export worked, what the
    consumer read, whether its write is visible here, and the shim's VMM /
    IPC state of the range."""
    import ctypes

    import torch
    import torch.multiprocessing as mp
    lib = ctypes.CDLL(None)
    n = (mib << 20) // 4
    x = torch.arange(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    m = (ctypes.c_uint64 * 8)()
    if hasattr(lib, "vgpu_self_vmm_stats"):
        lib.vgpu_self_vmm_stats(m)
    out = {"vmm_ranges": int(m[0]), "vmm_bytes": int(m[1]), "expected_sum": n * (n - 1) // 2}
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    p = ctx.Process(target=_ipc_child, args=(q_in, q_out))
    p.start()
    try:
        try:
            # pickle here, not in the queue's feeder thread, so an export error
            # surfaces in this thread (and the child still gets something)
            from multiprocessing.reduction import ForkingPickler
            ForkingPickler.dumps(x)
            q_in.put(x)
            out["exported"] = True
        except Exception as e:
            out["exported"] = False
            out["export_error"] = repr(e)[:400]
            q_in.put(torch.zeros(1, device="cuda"))  # let the child finish
        r = q_out.get(timeout=180)
        out.update({"child_" + k: v for k, v in r.items()})
        p.join(60)
        out["child_rc"] = p.exitcode
    finally:
        if p.is_alive():
            p.kill()
    torch.cuda.synchronize()
    out["parent_sees_write"] = bool(int(x[0].item()) == -1)
    out["child_sum_ok"] = out.get("child_sum") == out["expected_sum"]
    return out


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = argv.pop(0) if argv else "census"
    nums = [int(a) for a in argv]
    out = {"census": census, "busy": busy, "cap": cap, "smi": smi, "graph": graph, "arrays": arrays,
           "progress": progress, "forkjoin": forkjoin, "vmem": vmem, "vmemcopy": vmemcopy, "capheld": capheld, "asynccap": asynccap, "rcclloop": rcclloop,
           "vmemfull": vmemfull, "evictee": evictee, "busyvia": busyvia, "pitch": pitch,
           "ipcshare": ipcshare}[cmd](*nums)
    out["shim"] = shim_stats()
    print("PROBE " + json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
