"""xGMI / NUMA-aware GPU-set selection for GetPreferredAllocation and for
multi-GPU vGPU placement.

Reference analogues: the NVIDIA plugin's gpuallocator best-effort policy
(pkg/device-plugin/nvidiadevice/nvinternal/rm/allocate.go:26-121, NVLink
aware, but disabled in practice because GetPreferredAllocation returns empty,
server.go:262-277) and the MLU ring allocators that prefer sets with the most
non-conflicting MLULink rings (pkg/device-plugin/mlu/allocator/board.go:35-194,
spider.go:34-136).

MI355X: an 8-GPU node is a fully connected xGMI mesh (7 links per GPU), so any
pair inside one hive is one hop; RCCL rings are per-link bound, so the score
counts xGMI-connected pairs (all pairs for a full hive), then prefers one NUMA
node (host-side staging, CPU affinity), then keeps devices that are already
partially used together (leave whole GPUs free).
"""
from __future__ import annotations

import ctypes
import itertools
import os

from .discovery import LINK_XGMI, Backend, Device


def link_matrix(backend: Backend, devs: list[Device]) -> list[list[int]]:
    n = len(devs)
    m = [[0] * n for _ in range(n)]
    for a in range(n):
        for b in range(n):
            if a != b:
                _, t = backend.link(devs[a].index, devs[b].index)
                m[a][b] = t
    return m


def score_set(idx: tuple[int, ...], devs: list[Device], links: list[list[int]], used: dict[int, int]) -> tuple:
    xgmi_pairs = sum(1 for a, b in itertools.combinations(idx, 2) if links[a][b] == LINK_XGMI)
    numas = len({devs[i].numa for i in idx})
    hives = len({devs[i].xgmi_hive for i in idx})
    busy = sum(used.get(i, 0) for i in idx)
    return (xgmi_pairs, -hives, -numas, busy, tuple(-i for i in idx))


_NATIVE = None


def _native():
    """vgpu_topo_preferred from libvgpu_smi.so (native/smi/topo.cpp), or None."""
    global _NATIVE
    if _NATIVE is None:
        _NATIVE = False
        if os.environ.get("VGPU_TOPO_NATIVE", "1") != "0":
            from vgpu.native import lib_path
            p = lib_path("libvgpu_smi.so")
            if p.exists():
                fn = ctypes.CDLL(str(p)).vgpu_topo_preferred
                fn.restype = ctypes.c_int
                _NATIVE = fn
    return _NATIVE or None


def preferred(available: list[int], must: list[int], size: int, devs: list[Device],
              links: list[list[int]], used: dict[int, int] | None = None, limit: int = 20000) -> list[int]:
    """Pick `size` device positions from `available` (positions into `devs`),
    always including `must`.  Runs the native solver (native/smi/topo.cpp) when
    libvgpu_smi is built; preferred_py below is its executable specification."""
    fn = _native()
    if fn is None:
        return preferred_py(available, must, size, devs, links, used, limit)
    used = used or {}
    n = len(devs)
    I = ctypes.c_int
    arr = lambda xs: (I * max(1, len(xs)))(*xs)  # noqa: E731
    flat = [links[a][b] for a in range(n) for b in range(n)]
    out = (I * max(1, size + len(must) + len(available)))()
    dense = lambda vals: [sorted(set(vals)).index(v) for v in vals]  # noqa: E731  (64-bit hive ids)
    k = fn(I(n), arr(flat), arr(dense([d.numa for d in devs])), arr(dense([d.xgmi_hive for d in devs])),
           arr([used.get(i, 0) for i in range(n)]), arr(list(available)), I(len(available)),
           arr(list(must)), I(len(must)), I(size), ctypes.c_longlong(limit), out)
    if k < 0:
        raise ValueError("vgpu_topo_preferred: bad arguments")
    return list(out[:k])


def preferred_py(available: list[int], must: list[int], size: int, devs: list[Device],
                 links: list[list[int]], used: dict[int, int] | None = None, limit: int = 20000) -> list[int]:
    """Reference implementation of `preferred` (exhaustive for the ≤8-GPU node,
    capped otherwise)."""
    used = used or {}
    must = [m for m in must if m in available]
    rest = [a for a in available if a not in must]
    need = size - len(must)
    if need <= 0:
        return must[:size]
    if need > len(rest):
        return must + rest
    best, best_s = None, None
    for n, combo in enumerate(itertools.combinations(rest, need)):
        if n >= limit:
            break
        cand = tuple(sorted(must + list(combo)))
        s = score_set(cand, devs, links, used)
        if best_s is None or s > best_s:
            best, best_s = cand, s
    return list(best)
