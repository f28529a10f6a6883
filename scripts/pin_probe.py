#!/usr/bin/env python3
"""Design probe for the VMM suspend-evict vehicle: how fast
can a process get G GiB of pinned host memory, and how fast does D2H fill it?

    python scripts/pin_probe.py [G] [threads...]

For each thread count T: T threads hipHostMalloc G/T GiB each (the runtime's
pinned allocation, page zeroing included); then T threads mmap(MAP_POPULATE)
+ hipHostRegister their share; then D2H copies of G GiB from one device
buffer on 1 and on 4 streams into the pinned memory.  One JSON line.
"""
import ctypes
import json
import mmap
import os
import sys
import threading
import time

import torch

G = int(sys.argv[1]) if len(sys.argv) > 1 else 64
TS = [int(a) for a in sys.argv[2:]] or [1, 4, 8]
n = G << 30
torch.cuda.init()
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
out = {"gib": G}


def par(T, fn):
    res = [None] * T
    ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, fn(i))) for i in range(T)]
    t0 = time.time()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return time.time() - t0, res


for T in TS:
    share = n // T
    ptrs = [ctypes.c_void_p() for _ in range(T)]
    dt, rcs = par(T, lambda i: hip.hipHostMalloc(ctypes.byref(ptrs[i]), ctypes.c_size_t(share), 0))
    out[f"hostmalloc_t{T}_s"] = round(dt, 3)
    out[f"hostmalloc_t{T}_rc"] = sorted(set(rcs))
    for p in ptrs:
        hip.hipHostFree(p)
    maps = [None] * T

    def populate(i):
        maps[i] = mmap.mmap(-1, share, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS | mmap.MAP_POPULATE)
        return 0
    dt, _ = par(T, populate)
    out[f"populate_t{T}_s"] = round(dt, 3)
    addrs = [ctypes.addressof(ctypes.c_char.from_buffer(m)) for m in maps]
    dt, rcs = par(T, lambda i: hip.hipHostRegister(ctypes.c_void_p(addrs[i]), ctypes.c_size_t(share), 0))
    out[f"register_t{T}_s"] = round(dt, 3)
    out[f"register_t{T}_rc"] = sorted(set(rcs))
    if T == TS[-1]:
        x = torch.empty(n, dtype=torch.uint8, device="cuda")
        x.fill_(5)
        torch.cuda.synchronize()
        for ns in (1, 4):
            streams = [torch.cuda.Stream() for _ in range(ns)]
            torch.cuda.synchronize()
            t0 = time.time()
            for i in range(T):
                s = streams[i % ns]
                hip.hipMemcpyAsync(ctypes.c_void_p(addrs[i]), ctypes.c_void_p(x.data_ptr() + i * share),
                                   ctypes.c_size_t(share), 2, ctypes.c_void_p(s.cuda_stream))  # D2H
            torch.cuda.synchronize()
            out[f"d2h_streams{ns}_s"] = round(time.time() - t0, 3)
        t0 = time.time()
        for i in range(T):
            s = streams[i % 4]
            hip.hipMemcpyAsync(ctypes.c_void_p(x.data_ptr() + i * share), ctypes.c_void_p(addrs[i]),
                               ctypes.c_size_t(share), 1, ctypes.c_void_p(s.cuda_stream))  # H2D
        torch.cuda.synchronize()
        out["h2d_streams4_s"] = round(time.time() - t0, 3)
        out["check"] = bool(ctypes.c_ubyte.from_address(addrs[-1] + share - 1).value == 5)
        del x
    t0 = time.time()
    for a in addrs:
        hip.hipHostUnregister(ctypes.c_void_p(a))
    out[f"unregister_t{T}_s"] = round(time.time() - t0, 3)
    del addrs
    for m in maps:
        m.close()
    print("PIN " + json.dumps(out), flush=True)
print("PIN " + json.dumps(out), flush=True)
