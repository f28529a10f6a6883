"""Node-local compute-share state: which containers hold a CU mask on which
device, persisted next to each container's shared region so it survives
device-plugin restarts.

Reference analogue: the Hygon plugin rebuilds its CU-mask occupancy from
per-container directory names and garbage-collects dead pods
(pkg/device-plugin/hygon/dcu/server.go:258-336, RefreshContainerDevices); its
allocator takes free CU bits greedily (corealloc.go:60-77).

Each container dir holds `grant.json`: {device uuid: {"mask": hex, "mode":
"mask"|"pool"}} (a bare hex string is read as mode "mask", the round-1 format).

Share policies (DevicePluginConfig.cu_share; measurements in
profiles/sharing_4way_r1.md and profiles/temporal_r2.md):

* ``mask``: every fractional container gets its own XCD-balanced CU mask.
  When no granules are free, the container gets the pool instead.
* ``temporal``: no per-container masks. Every fractional container
  is a pool member: the shim's GPU-time limiter, charged through the per-GPU
  fair-share board. It throttles only under contention (work-conserving) and
  is the reference's time-sliced SM limit. On MI355X, 4 x 25 % temporal pods
  run at >= 0.97 x the exclusive GPU on 9 of 10 ai-benchmark tests, against
  0.65 x with four masks on ResNet-50; ResNet-152 training is the exception
  (0.83-0.96 x; four masks 1.01 x). 2 x 50 % pods match or beat two masks on
  9 of 10 tests; the flagship goes from 24.2k to 25.4k images/s.

A pod may override the node's policy for its own containers with the
annotation ``amd.com/cu-share: mask|temporal|hybrid`` (e.g. a training job
that wants exclusive CUs on a temporal node).
* ``hybrid``: the first ``max_mask_slots`` fractional containers on a GPU get
  masks, which is exact spatial isolation at equal throughput for two sharers.
  Later containers join the pool.
* ``auto``: every fractional container starts as a pool member (like
  ``temporal``); once two or more are busy, the pods of the GPU measure a
  window time-shared and a window with each on an XCD-balanced claim of its
  share's CUs (share-board A/B, native/shim/limiter.cpp auto_step) and keep
  whichever ran their dispatches faster.  Spatial where it pays, temporal
  where it does not; re-measured when the set of busy pods changes.

The pool of a device is every CU not held by a masked container; pool members
share it in time. The shim scales a pool member's time limit by
(device CUs / pool CUs).
"""
from __future__ import annotations

import json
import logging
import os
import shutil
import threading
import time
from dataclasses import dataclass
from pathlib import Path

from vgpu.device.cualloc import MI355X, CULayout, alloc_cu_mask, resolve_packing

log = logging.getLogger("vgpu.deviceplugin.custate")

GRANT_FILE = "grant.json"
REGION_FILE = "vgpu.cache"  # the container's shared region (allocate.py: VGPU_SHARED_REGION)
MODE_MASK = "mask"
MODE_POOL = "pool"
POLICIES = ("mask", "temporal", "hybrid", "auto")


@dataclass
class ShareGrant:
    mask: int = 0          # CU mask handed to the container (0 = all CUs / none)
    mode: str = MODE_MASK  # MODE_MASK: exclusive CUs; MODE_POOL: shared CUs + temporal limiter

    @property
    def temporal(self) -> bool:
        return self.mode == MODE_POOL


class CUMaskState:
    def __init__(self, containers_dir: str, layout: CULayout = MI355X, policy: str = "auto",
                 max_mask_slots: int = 2, pack: str | None = None):
        if policy not in POLICIES:
            raise ValueError(f"cu_share policy must be one of {POLICIES}, got {policy!r}")
        # CU packing order (VGPU_CU_PACK), validated once here rather than per Allocate.
        self.pack = resolve_packing(pack, layout)
        requested = pack or os.environ.get("VGPU_CU_PACK", "spread")
        if requested != self.pack:
            log.warning("CU packing %r does not fit the %d-CU layout; using %r", requested,
                        layout.total_cus, self.pack)
        self.dir = Path(containers_dir)
        self.layout = layout
        self.policy = policy
        self.max_mask_slots = max(0, int(max_mask_slots))
        self._lock = threading.Lock()

    def _grants(self) -> dict[str, dict[str, ShareGrant]]:
        out: dict[str, dict[str, ShareGrant]] = {}
        if not self.dir.exists():
            return out
        for d in self.dir.iterdir():
            g = d / GRANT_FILE
            if not g.exists():
                continue
            try:
                raw = json.loads(g.read_text())
                out[d.name] = {k: (ShareGrant(int(v, 16), MODE_MASK) if isinstance(v, str)
                                   else ShareGrant(int(v.get("mask", "0x0"), 16), v.get("mode", MODE_MASK)))
                               for k, v in raw.items()}
            except (OSError, ValueError, AttributeError):
                continue
        return out

    def used(self, uuid: str) -> int:
        """CUs of `uuid` held exclusively by masked containers."""
        m = 0
        for g in self._grants().values():
            sg = g.get(uuid)
            if sg and sg.mode == MODE_MASK:
                m |= sg.mask
        return m

    def pool_members(self, uuid: str) -> int:
        return sum(1 for g in self._grants().values() if uuid in g and g[uuid].mode == MODE_POOL)

    def allocate(self, container_key: str, requests: list[tuple[str, int]],
                 layouts: dict[str, CULayout] | None = None, policy: str | None = None) -> dict[str, ShareGrant]:
        """requests: [(device uuid, cores %)] → {uuid: ShareGrant}.  Whole-device
        and best-effort requests (cores 0 or >= 100) get ShareGrant(0, "mask"):
        no mask, no limiter.  `layouts` gives each device's CU/XCD geometry (a CPX
        compute partition is one XCD of 32 CUs; SPX is 8 × 32).  `policy`
        overrides the node's share policy for this container (pod annotation
        amd.com/cu-share)."""
        layouts = layouts or {}
        pol = policy if policy in POLICIES else self.policy
        with self._lock:
            grants = self._grants()
            grants.pop(container_key, None)  # re-allocation of the same container
            res: dict[str, ShareGrant] = {}
            for uuid, cores in requests:
                if cores <= 0 or cores >= 100:
                    res[uuid] = ShareGrant(0, MODE_MASK)
                    continue
                lay = layouts.get(uuid, self.layout)
                full = (1 << lay.total_cus) - 1
                masked = 0      # CUs held by masked containers
                occupied = 0    # CUs of any grant (pool masks included)
                n_masked = 0
                for g in list(grants.values()) + [res]:
                    sg = g.get(uuid)
                    if not sg:
                        continue
                    occupied |= sg.mask
                    if sg.mode == MODE_MASK and sg.mask:
                        masked |= sg.mask
                        n_masked += 1
                want_mask = pol == "mask" or (pol == "hybrid" and n_masked < self.max_mask_slots)
                m = alloc_cu_mask(occupied, cores, lay, resolve_packing(self.pack, lay)) if want_mask else None
                if m:
                    res[uuid] = ShareGrant(m, MODE_MASK)
                else:
                    pool = full & ~masked
                    res[uuid] = ShareGrant(0 if pool == full else pool, MODE_POOL)
            self._write_grant(container_key, res)
            grants[container_key] = res
            for uuid, sg in res.items():
                if sg.mode == MODE_MASK and sg.mask:
                    lay = layouts.get(uuid, self.layout)
                    self._reshape_pool(uuid, grants, (1 << lay.total_cus) - 1)
            return res

    def _write_grant(self, container_key: str, res: dict[str, ShareGrant]) -> None:
        d = self.dir / container_key
        d.mkdir(parents=True, exist_ok=True)
        tmp = d / (GRANT_FILE + ".tmp")
        tmp.write_text(json.dumps({k: {"mask": hex(v.mask), "mode": v.mode} for k, v in res.items()
                                   if v.mask or v.mode == MODE_POOL}))
        os.replace(tmp, d / GRANT_FILE)

    def _reshape_pool(self, uuid: str, grants: dict[str, dict[str, ShareGrant]], full: int) -> None:
        """A masked grant took CUs of `uuid`: every pool member of that device
        shrinks to the CUs no masked container holds, so the new container's CUs
        are exclusive even when pool members were admitted before it (a pool
        member with mask 0 runs on every CU).  The grant file is rewritten and,
        when the container is running, its shared region's CU mask too: the
        shim re-applies region masks to its live queues within ~10 ms
        (limiter.cpp) and rescales its time share to the smaller pool."""
        masked = 0
        for g in grants.values():
            sg = g.get(uuid)
            if sg and sg.mode == MODE_MASK:
                masked |= sg.mask
        pool = full & ~masked
        want = 0 if pool == full else pool
        for key, g in grants.items():
            sg = g.get(uuid)
            if not sg or sg.mode != MODE_POOL or sg.mask == want:
                continue
            g[uuid] = ShareGrant(want, MODE_POOL)
            self._write_grant(key, g)
            self._update_region(key, uuid, want)
            log.info("container %s: pool of %s reshaped to %d CUs", key, uuid, bin(want or full).count("1"))

    def _update_region(self, container_key: str, uuid: str, mask: int) -> None:
        path = self.dir / container_key / REGION_FILE
        if not path.exists():
            return
        try:
            from vgpu.monitor.region import AttachedRegion
            r = AttachedRegion(str(path))
        except (OSError, RuntimeError) as e:
            log.warning("cannot reshape live region %s: %s", path, e)
            return
        try:
            for d in r.devices():
                if d.uuid == uuid:
                    r.set_cu_mask(d.index, mask)
        finally:
            r.close()

    def gc(self, live_pod_uids: set[str], grace_s: float = 300.0) -> list[str]:
        """Remove container dirs whose pod UID is gone for longer than `grace_s`
        (reference monitor GC: cmd/vGPUmonitor/pathmonitor.go:88-99)."""
        removed = []
        if not self.dir.exists():
            return removed
        now = time.time()
        for d in self.dir.iterdir():
            uid = d.name.split("_", 1)[0]
            if uid in live_pod_uids:
                continue
            try:
                age = now - d.stat().st_mtime
            except OSError:
                continue
            if age >= grace_s:
                shutil.rmtree(d, ignore_errors=True)
                removed.append(d.name)
        return removed
