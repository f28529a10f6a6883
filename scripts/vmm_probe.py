"""What the HIP virtual-memory API can do on this MI355X (design probe for the
shim's VA-stable oversubscription, native/shim/vmem.cpp):

1. a device-located physical handle mapped into a reserved VA range;
2. a host-located physical handle (hipMemLocationTypeHost) mapped the same way,
   and GPU kernels reading it (bandwidth);
3. moving a chunk: same VA, device handle -> host handle -> device handle, data intact.
"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

torch.cuda.init()
torch.empty(1, device="cuda")
hip = ctypes.CDLL("libamdhip64.so")
from vgpu.native import load_kernels  # noqa: E402

K = load_kernels()


class Loc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]


class Prop(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("handleType", ctypes.c_int), ("location", Loc),
                ("win32", ctypes.c_void_p), ("ctype", ctypes.c_ubyte), ("rdma", ctypes.c_ubyte),
                ("usage", ctypes.c_ushort)]


class Access(ctypes.Structure):
    _fields_ = [("location", Loc), ("flags", ctypes.c_int)]


DEV, HOST = 1, 2
out = {}
size = 1 << 30


def prop(loc):
    p = Prop()
    p.type = 1  # pinned
    p.location = Loc(loc, 0)
    return p


gran = ctypes.c_size_t()
out["granularity_dev"] = hip.hipMemGetAllocationGranularity(ctypes.byref(gran), ctypes.byref(prop(DEV)), 0), gran.value
g2 = ctypes.c_size_t()
out["granularity_host"] = hip.hipMemGetAllocationGranularity(ctypes.byref(g2), ctypes.byref(prop(HOST)), 0), g2.value
hd, hh = ctypes.c_uint64(), ctypes.c_uint64()
out["create_dev"] = hip.hipMemCreate(ctypes.byref(hd), ctypes.c_size_t(size), ctypes.byref(prop(DEV)), ctypes.c_ulonglong(0))
out["create_host"] = hip.hipMemCreate(ctypes.byref(hh), ctypes.c_size_t(size), ctypes.byref(prop(HOST)), ctypes.c_ulonglong(0))
hip.hipGetLastError()
va = ctypes.c_void_p()
out["reserve"] = hip.hipMemAddressReserve(ctypes.byref(va), ctypes.c_size_t(size), ctypes.c_size_t(0),
                                          ctypes.c_void_p(0), ctypes.c_ulonglong(0))
acc_dev = Access(Loc(DEV, 0), 3)


def verify(ptr, seed):
    err = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    K.vgpu_verify_pattern(ptr, size, seed,
                          err.data_ptr(), s)
    torch.cuda.synchronize()
    return int(err.item())


def fill(ptr, seed):
    s = torch.cuda.current_stream().cuda_stream
    K.vgpu_fill_pattern(ptr, size, seed, s)
    torch.cuda.synchronize()


def read_gbps(ptr):
    verify(ptr, 5)
    t0 = time.time()
    for _ in range(3):
        verify(ptr, 5)
    return round(3 * size / (time.time() - t0) / 1e9, 1)


if out["create_dev"] == 0 and out["reserve"] == 0:
    out["map_dev"] = hip.hipMemMap(va, ctypes.c_size_t(size), ctypes.c_size_t(0), hd, ctypes.c_ulonglong(0))
    out["access_dev"] = hip.hipMemSetAccess(va, ctypes.c_size_t(size), ctypes.byref(acc_dev), ctypes.c_size_t(1))
    fill(va.value, 5)
    out["verify_dev"] = verify(va.value, 5)
    out["dev_read_GBps"] = read_gbps(va.value)
    if out["create_host"] == 0:
        # second VA for the host handle, copy device -> host, then swap mappings
        va2 = ctypes.c_void_p()
        hip.hipMemAddressReserve(ctypes.byref(va2), ctypes.c_size_t(size), ctypes.c_size_t(0), ctypes.c_void_p(0),
                                 ctypes.c_ulonglong(0))
        out["map_host"] = hip.hipMemMap(va2, ctypes.c_size_t(size), ctypes.c_size_t(0), hh, ctypes.c_ulonglong(0))
        out["access_host"] = hip.hipMemSetAccess(va2, ctypes.c_size_t(size), ctypes.byref(acc_dev), ctypes.c_size_t(1))
        t0 = time.time()
        out["copy_d2h"] = hip.hipMemcpy(va2, va, ctypes.c_size_t(size), 3)  # hipMemcpyDeviceToDevice
        hip.hipDeviceSynchronize()
        out["copy_d2h_GBps"] = round(size / (time.time() - t0) / 1e9, 1)
        out["verify_host_copy"] = verify(va2.value, 5)
        out["host_read_GBps"] = read_gbps(va2.value)
        hip.hipMemUnmap(va2, ctypes.c_size_t(size))
        out["unmap_dev"] = hip.hipMemUnmap(va, ctypes.c_size_t(size))
        out["remap_host_at_va"] = hip.hipMemMap(va, ctypes.c_size_t(size), ctypes.c_size_t(0), hh, ctypes.c_ulonglong(0))
        out["access_host_at_va"] = hip.hipMemSetAccess(va, ctypes.c_size_t(size), ctypes.byref(acc_dev),
                                                       ctypes.c_size_t(1))
        out["verify_after_swap_out"] = verify(va.value, 5)
        # and back in
        hip.hipMemMap(va2, ctypes.c_size_t(size), ctypes.c_size_t(0), hd, ctypes.c_ulonglong(0))
        hip.hipMemSetAccess(va2, ctypes.c_size_t(size), ctypes.byref(acc_dev), ctypes.c_size_t(1))
        fill(va2.value, 9)
        t0 = time.time()
        out["copy_h2d"] = hip.hipMemcpy(va2, va, ctypes.c_size_t(size), 3)
        hip.hipDeviceSynchronize()
        out["copy_h2d_GBps"] = round(size / (time.time() - t0) / 1e9, 1)
        hip.hipMemUnmap(va2, ctypes.c_size_t(size))
        hip.hipMemUnmap(va, ctypes.c_size_t(size))
        out["remap_dev_at_va"] = hip.hipMemMap(va, ctypes.c_size_t(size), ctypes.c_size_t(0), hd, ctypes.c_ulonglong(0))
        hip.hipMemSetAccess(va, ctypes.c_size_t(size), ctypes.byref(acc_dev), ctypes.c_size_t(1))
        out["verify_after_swap_in"] = verify(va.value, 5)
print("VMM " + json.dumps(out), flush=True)
