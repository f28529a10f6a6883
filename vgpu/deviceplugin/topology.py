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

import itertools

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


def preferred(available: list[int], must: list[int], size: int, devs: list[Device],
              links: list[list[int]], used: dict[int, int] | None = None, limit: int = 20000) -> list[int]:
    """Pick `size` device positions from `available` (positions into `devs`),
    always including `must`.  Exhaustive for the ≤8-GPU node, capped otherwise."""
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
