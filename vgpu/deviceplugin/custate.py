"""Node-local CU-mask occupancy, persisted next to each container's shared
region so it survives device-plugin restarts.

Reference analogue: the Hygon plugin rebuilds its CU-mask occupancy from
per-container directory names and garbage-collects dead pods
(pkg/device-plugin/hygon/dcu/server.go:258-336, RefreshContainerDevices).
Here each container dir holds `grant.json` ({device uuid: mask hex}); the
occupancy of a device is the OR over live containers.
"""
from __future__ import annotations

import json
import os
import shutil
import threading
import time
from pathlib import Path

from vgpu.device.cualloc import MI355X, CULayout, alloc_cu_mask

GRANT_FILE = "grant.json"


class CUMaskState:
    def __init__(self, containers_dir: str, layout: CULayout = MI355X):
        self.dir = Path(containers_dir)
        self.layout = layout
        self._lock = threading.Lock()

    def _grants(self) -> dict[str, dict[str, int]]:
        out = {}
        if not self.dir.exists():
            return out
        for d in self.dir.iterdir():
            g = d / GRANT_FILE
            if not g.exists():
                continue
            try:
                out[d.name] = {k: int(v, 16) for k, v in json.loads(g.read_text()).items()}
            except (OSError, ValueError):
                continue
        return out

    def used(self, uuid: str) -> int:
        m = 0
        for g in self._grants().values():
            m |= g.get(uuid, 0)
        return m

    def allocate(self, container_key: str, requests: list[tuple[str, int]],
                 layouts: dict[str, CULayout] | None = None) -> dict[str, int]:
        """requests: [(device uuid, cores %)] → {uuid: mask} (0 = no spatial mask:
        exclusive, best-effort, or not enough free granules → temporal limiting).
        `layouts` gives each device's CU/XCD geometry (a CPX compute partition
        is one XCD of 32 CUs; SPX is 8 × 32)."""
        layouts = layouts or {}
        with self._lock:
            grants = self._grants()
            grants.pop(container_key, None)  # re-allocation of the same container
            res: dict[str, int] = {}
            for uuid, cores in requests:
                if cores <= 0 or cores >= 100:
                    res[uuid] = 0
                    continue
                used = 0
                for g in grants.values():
                    used |= g.get(uuid, 0)
                used |= res.get(uuid, 0)
                m = alloc_cu_mask(used, cores, layouts.get(uuid, self.layout))
                res[uuid] = m or 0
            d = self.dir / container_key
            d.mkdir(parents=True, exist_ok=True)
            tmp = d / (GRANT_FILE + ".tmp")
            tmp.write_text(json.dumps({k: hex(v) for k, v in res.items() if v}))
            os.replace(tmp, d / GRANT_FILE)
            return res

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
