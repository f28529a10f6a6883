"""XCD-balanced CU-mask allocator for MI355X (256 CUs = 8 XCDs × 32 CUs).

Reference analogue: the Hygon DCU plugin's hex-string CU bitmap
(pkg/device-plugin/hygon/dcu/corealloc.go:8-77: `allocCoreUsage` greedily takes
free bits, `addCoreUsage` ORs masks, `reqcores = pct*totalcores/100`).  Taking
arbitrary free bits is wrong on MI355X: workgroups are dealt round-robin to the
8 XCDs, so a mask that gives one XCD fewer CUs than the others makes that XCD
the straggler of every kernel.

Here the unit of allocation is a *granule* = one CU on every XCD.  With the
gfx950 queue-mask mapping (logical bit i → XCD i % 8, verified on hardware by
tests/test_gpu_shim.py::test_cu_mask_census) granule g is logical bits
[8g, 8g+8); within an XCD consecutive granules land on different shader
engines (local CU j → SE j % 4), so low granules are also SE-balanced.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class CULayout:
    total_cus: int = 256
    num_xcc: int = 8
    interleaved: bool = True   # bit i -> XCD i % num_xcc (gfx950); False: blocked
    num_se: int = 4            # shader engines per XCD (local CU j -> SE j % num_se)

    @property
    def granules(self) -> int:
        return self.total_cus // self.num_xcc

    def granule_mask(self, g: int) -> int:
        if self.interleaved:
            return ((1 << self.num_xcc) - 1) << (g * self.num_xcc)
        per = self.total_cus // self.num_xcc
        m = 0
        for x in range(self.num_xcc):
            m |= 1 << (x * per + g)
        return m

    def full_mask(self) -> int:
        return (1 << self.total_cus) - 1

    def cus_for_percent(self, pct: int) -> int:
        """CUs granted for a percentage: ceil to whole granules."""
        if pct <= 0:
            return 0
        pct = min(pct, 100)
        n = -(-self.total_cus * pct // 100)
        g = -(-n // self.num_xcc)
        return min(g * self.num_xcc, self.total_cus)

    def per_xcd_counts(self, mask: int) -> list[int]:
        counts = [0] * self.num_xcc
        per = self.total_cus // self.num_xcc
        for bit in range(self.total_cus):
            if mask >> bit & 1:
                x = bit % self.num_xcc if self.interleaved else bit // per
                counts[x] += 1
        return counts


MI355X = CULayout()


def popcount(m: int) -> int:
    return bin(m).count("1")


PACKINGS = ("spread", "se")


def resolve_packing(pack: str | None = None, layout: CULayout = MI355X) -> str:
    """Validate a packing name (default: VGPU_CU_PACK, else "spread") and return
    the packing that takes effect on `layout`.  "se" needs whole SE groups of
    granules and degrades to "spread" otherwise.  Callers resolve this once at
    start-up, so a bad value fails there and not inside Allocate."""
    pack = pack or os.environ.get("VGPU_CU_PACK", "spread")
    if pack not in PACKINGS:
        raise ValueError(f"unknown CU packing {pack!r} (one of {PACKINGS})")
    if pack == "se" and not (layout.num_se > 1 and layout.granules % layout.num_se == 0):
        return "spread"
    return pack


def granule_order(layout: CULayout, pack: str | None = None) -> list[int]:
    """Order in which free granules are taken.

    spread: 0, 1, 2, ... — a pod's CUs are spread over every shader engine.
    se:     all granules of SE 0, then SE 1, ... — a pod owns whole shader
            engines where its share allows, so no two pods feed the same SE's
            workgroup dispatcher."""
    if resolve_packing(pack, layout) == "se":
        return [g for se in range(layout.num_se) for g in range(se, layout.granules, layout.num_se)]
    return list(range(layout.granules))


def alloc_cu_mask(used: int, pct: int, layout: CULayout = MI355X, pack: str | None = None) -> int | None:
    """Allocate an XCD-balanced mask for `pct` percent of the device's CUs from
    the granules not set in `used` (taken in `granule_order`).  Returns None when
    not enough free granules remain (the caller then falls back to sharing +
    temporal limiting)."""
    need = layout.cus_for_percent(pct) // layout.num_xcc
    if need == 0:
        return 0
    mask = 0
    for g in granule_order(layout, pack):
        gm = layout.granule_mask(g)
        if used & gm:
            continue
        mask |= gm
        need -= 1
        if need == 0:
            return mask
    return None


def add_usage(used: int, mask: int) -> int:
    return used | mask


def free_usage(used: int, mask: int) -> int:
    return used & ~mask


def parse_mask(s: str) -> int:
    s = s.strip().lower().replace(",", "").replace("_", "")
    if s.startswith("0x"):
        s = s[2:]
    return int(s, 16) if s else 0
