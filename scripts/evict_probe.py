#!/usr/bin/env python3
"""Design probe for the suspend-evict vehicle: what it costs
to move G GiB of HBM to host memory and back on this MI355X, per vehicle.

    python scripts/evict_probe.py [G]

1. pinned: hipHostMalloc of G GiB (pinning cost) + D2H + H2D copies;
2. pageable: malloc'd host memory + D2H + H2D (the runtime stages);
3. VMM: a device handle mapped into a reserved VA, released and re-created
   at the same VA (the HBM really goes back: hipMemGetInfo before/after).
Prints one JSON line.
"""
import ctypes
import json
import sys
import time

import torch

G = int(sys.argv[1]) if len(sys.argv) > 1 else 16
n = G << 30
out = {"gib": G}
torch.cuda.init()
dev = torch.device("cuda", 0)
x = torch.empty(n, dtype=torch.uint8, device=dev)
x.fill_(7)
torch.cuda.synchronize()


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.time()
    fn()
    torch.cuda.synchronize()
    return round(time.time() - t0, 3)


t0 = time.time()
hp = torch.empty(n, dtype=torch.uint8, pin_memory=True)
out["pin_alloc_s"] = round(time.time() - t0, 3)
out["pinned_d2h_s"] = timed(lambda: hp.copy_(x, non_blocking=True))
out["pinned_h2d_s"] = timed(lambda: x.copy_(hp, non_blocking=True))
del hp
t0 = time.time()
pg = torch.empty(n, dtype=torch.uint8)
pg[:: 4096] = 0  # touch every page
out["pageable_alloc_touch_s"] = round(time.time() - t0, 3)
out["pageable_d2h_s"] = timed(lambda: pg.copy_(x))
out["pageable_h2d_s"] = timed(lambda: x.copy_(pg))
del pg
del x
torch.cuda.empty_cache()

# VMM: reserve + create + map + access, release and re-create at the same VA
import os  # noqa: E402
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))  # torch's runtime


class Loc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]


class Prop(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("handleType", ctypes.c_int), ("location", Loc),
                ("win32", ctypes.c_void_p), ("ctype", ctypes.c_ubyte), ("rdma", ctypes.c_ubyte),
                ("usage", ctypes.c_ushort)]


class Access(ctypes.Structure):
    _fields_ = [("location", Loc), ("flags", ctypes.c_int)]


prop = Prop()
prop.type = 1  # pinned
prop.location = Loc(1, 0)  # device 0
gran = ctypes.c_size_t(0)
out["gran_rc"] = hip.hipMemGetAllocationGranularity(ctypes.byref(gran), ctypes.byref(prop), 1)  # recommended
out["gran"] = gran.value
va = ctypes.c_void_p()
free0, tot = ctypes.c_size_t(), ctypes.c_size_t()
hip.hipMemGetInfo(ctypes.byref(free0), ctypes.byref(tot))
t0 = time.time()
out["reserve_rc"] = hip.hipMemAddressReserve(ctypes.byref(va), ctypes.c_size_t(n), ctypes.c_size_t(0),
                                             ctypes.c_void_p(0), ctypes.c_ulonglong(0))
h = ctypes.c_void_p()
out["create_rc"] = hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(n), ctypes.byref(prop), ctypes.c_ulonglong(0))
out["map_rc"] = hip.hipMemMap(va, ctypes.c_size_t(n), ctypes.c_size_t(0), h, ctypes.c_ulonglong(0))
acc = Access(Loc(1, 0), 3)
out["access_rc"] = hip.hipMemSetAccess(va, ctypes.c_size_t(n), ctypes.byref(acc), ctypes.c_size_t(1))
out["vmm_setup_s"] = round(time.time() - t0, 3)
free1 = ctypes.c_size_t()
hip.hipMemGetInfo(ctypes.byref(free1), ctypes.byref(tot))
out["vmm_hbm_taken_gib"] = round((free0.value - free1.value) / (1 << 30), 2)
hip.hipMemsetD8(va, ctypes.c_ubyte(9), ctypes.c_size_t(n))
hip.hipDeviceSynchronize()
t0 = time.time()
out["unmap_rc"] = hip.hipMemUnmap(va, ctypes.c_size_t(n))
out["release_rc"] = hip.hipMemRelease(h)
out["vmm_release_s"] = round(time.time() - t0, 3)
free2 = ctypes.c_size_t()
hip.hipMemGetInfo(ctypes.byref(free2), ctypes.byref(tot))
out["vmm_hbm_back_gib"] = round((free2.value - free1.value) / (1 << 30), 2)
t0 = time.time()
h2 = ctypes.c_void_p()
out["recreate_rc"] = hip.hipMemCreate(ctypes.byref(h2), ctypes.c_size_t(n), ctypes.byref(prop), ctypes.c_ulonglong(0))
out["remap_rc"] = hip.hipMemMap(va, ctypes.c_size_t(n), ctypes.c_size_t(0), h2, ctypes.c_ulonglong(0))
out["reaccess_rc"] = hip.hipMemSetAccess(va, ctypes.c_size_t(n), ctypes.byref(acc), ctypes.c_size_t(1))
out["vmm_recreate_s"] = round(time.time() - t0, 3)
hip.hipMemsetD8(va, ctypes.c_ubyte(3), ctypes.c_size_t(n))
out["memset_after_remap_rc"] = hip.hipDeviceSynchronize()
hip.hipMemUnmap(va, ctypes.c_size_t(n))
hip.hipMemRelease(h2)
hip.hipMemAddressFree(va, ctypes.c_size_t(n))
print("EVICT " + json.dumps(out), flush=True)
