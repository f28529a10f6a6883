"""Does KFD's per-process VRAM follow a stream-ordered pool's reserved size?

Plain HIP through ctypes (run with or without the shim): grow the default pool
with hipMallocAsync, free half, trim, re-grow, and after every step print the
pool's reserved/used bytes next to /sys/class/kfd/kfd/proc/<pid>/vram_*.
Used to explain the gap between the shim's pool charge and KFD's count in
tests/test_gpu_caps.py.
"""
import ctypes
import glob
import json
import os
import sys
import time

MiB = 1 << 20


def main() -> int:
    if os.environ.get("PROBE_TORCH"):
        import torch
        torch.empty(1, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipSetDevice(0)
    hip.hipFree(ctypes.c_void_p(0))  # context
    if os.environ.get("PROBE_MALLOC_FIRST"):
        q = ctypes.c_void_p()
        print("hipMalloc first:", hip.hipMalloc(ctypes.byref(q), ctypes.c_size_t(2 << 20)), flush=True)
    pid = os.getpid()
    try:
        selfpid = ctypes.CDLL(None).vgpu_self_host_pid
        src = ctypes.c_int(0)
        pid = selfpid(ctypes.byref(src)) or pid
    except AttributeError:
        pass
    files = glob.glob(f"/sys/class/kfd/kfd/proc/{pid}/vram_*")
    pool = ctypes.c_void_p()
    hip.hipDeviceGetMemPool(ctypes.byref(pool), 0)
    stream = ctypes.c_void_p(0)

    def attr(a):
        v = ctypes.c_uint64(0)
        hip.hipMemPoolGetAttribute(pool, a, ctypes.byref(v))
        return v.value

    def kfd():
        return sum(int(open(f).read()) for f in files)

    free, total = ctypes.c_size_t(0), ctypes.c_size_t(0)
    hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total))
    print("memgetinfo", free.value, total.value, flush=True)
    base = kfd()
    rows = []

    def row(tag, sleep=0.0):
        hip.hipDeviceSynchronize()
        if sleep:
            time.sleep(sleep)
        k = kfd() - base
        rows.append({"step": tag, "kfd_mib": k // MiB, "reserved_mib": attr(5) // MiB, "used_mib": attr(7) // MiB,
                     "gap_mib": (k - attr(5)) // MiB})
        print(json.dumps(rows[-1]), flush=True)

    sizes = [int(a) for a in sys.argv[1:]] or [64, 256, 512, 768, 1024, 1536, 96, 384, 640, 1280]
    ptrs = []
    row("start")
    for s in sizes:
        p = ctypes.c_void_p()
        rc = hip.hipMallocAsync(ctypes.byref(p), ctypes.c_size_t(s * MiB), stream)
        ptrs.append(p)
        row(f"alloc {s} rc={rc}")
    for p in ptrs[::2]:
        hip.hipFreeAsync(p, stream)
    row("freed half")
    hip.hipMemPoolTrimTo(pool, ctypes.c_size_t(0))
    row("trim")
    row("trim +0.5s", 0.5)
    for s in sizes[:4]:
        p = ctypes.c_void_p()
        rc = hip.hipMallocAsync(ctypes.byref(p), ctypes.c_size_t(s * MiB), stream)
        ptrs.append(p)
        row(f"realloc {s} rc={rc}")
    for p in ptrs[1::2] + ptrs[len(sizes):]:
        hip.hipFreeAsync(p, stream)
    row("freed all")
    hip.hipMemPoolTrimTo(pool, ctypes.c_size_t(0))
    row("trim all")
    row("trim all +0.5s", 0.5)
    print("MAXGAP", max(r["gap_mib"] for r in rows), "files", files, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
