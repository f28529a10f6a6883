"""How HIP's stream-ordered pool gives physical VRAM back (ctypes, no torch).
Prints amdgpu mem_info_vram_used - baseline and the pool's reserved/used
attributes after each step.  python scripts/mempool_probe.py"""
import ctypes
import glob
import json

base = {f: int(open(f).read()) for f in glob.glob("/sys/bus/pci/devices/*/mem_info_vram_used")}
hip = ctypes.CDLL("libamdhip64.so")
hip.hipSetDevice(0)
hip.hipFree(None)
bus = ctypes.create_string_buffer(64)
hip.hipDeviceGetPCIBusId(bus, 64, 0)
path = f"/sys/bus/pci/devices/{bus.value.decode().lower()}/mem_info_vram_used"
b0 = base[path]
pool = ctypes.c_void_p()
hip.hipDeviceGetMemPool(ctypes.byref(pool), 0)
stream = ctypes.c_void_p()
hip.hipStreamCreate(ctypes.byref(stream))
G = 1 << 30
out = []


def attr(a):
    v = ctypes.c_uint64()
    hip.hipMemPoolGetAttribute(pool, a, ctypes.byref(v))
    return v.value


def note(tag):
    hip.hipDeviceSynchronize()
    out.append({"step": tag, "vram_over_GB": round((int(open(path).read()) - b0) / G, 2),
                "pool_reserved_GB": round(attr(5) / G, 2), "pool_used_GB": round(attr(7) / G, 2)})


note("init")
ptrs = []
for sz in (1, 2, 3):
    p = ctypes.c_void_p()
    rc = hip.hipMallocAsync(ctypes.byref(p), ctypes.c_size_t(sz * G), stream)
    ptrs.append(p)
    note(f"mallocAsync {sz}G rc={rc}")
for p in ptrs:
    hip.hipFreeAsync(p, stream)
note("freeAsync all")
hip.hipStreamSynchronize(stream)
note("stream sync")
hip.hipMemPoolTrimTo(pool, ctypes.c_size_t(0))
note("trimTo 0")
thr = ctypes.c_uint64(2 ** 64 - 1)
hip.hipMemPoolSetAttribute(pool, 4, ctypes.byref(thr))  # release threshold: max (what PyTorch sets)
ptrs = []
for i in range(6):
    p = ctypes.c_void_p()
    hip.hipMallocAsync(ctypes.byref(p), ctypes.c_size_t((i % 3 + 1) * G), stream)
    hip.hipFreeAsync(p, stream)
    note(f"cycle {i}: malloc+free {(i % 3 + 1)}G (threshold max)")
hip.hipMemPoolTrimTo(pool, ctypes.c_size_t(0))
note("trimTo 0")
p = ctypes.c_void_p()
hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(2 * G))
note("hipMalloc 2G")
hip.hipFree(p)
note("hipFree")
print(json.dumps(out, indent=0))
