"""Discover container shared regions on the host and garbage-collect the ones
whose pods are gone.

Reference: cmd/vGPUmonitor/pathmonitor.go:21-26 (containers dir), :30-63
(dir name → pod), :74-121 (monitorpath: mmap new .cache files, delete dirs
whose pod UID is gone after 300 s).  Differences: pods are listed with a
spec.nodeName field selector (not cluster-wide), and the region file name is
fixed (`vgpu.cache`) instead of a random UUID per container.
"""
from __future__ import annotations

import logging
import os
import shutil
import time
from dataclasses import dataclass

from vgpu.k8s import objects as O

from .region import AttachedRegion

log = logging.getLogger("vgpu.monitor.path")

REGION_FILE = "vgpu.cache"
GC_GRACE_S = 300.0


@dataclass
class ContainerRegion:
    key: str            # "<podUID>_<container>"
    pod_uid: str
    ctr_name: str
    region: AttachedRegion
    pod_name: str = ""
    namespace: str = ""


class PathMonitor:
    def __init__(self, containers_dir: str, client=None, node: str = ""):
        self.dir = containers_dir
        self.client = client
        self.node = node
        self.regions: dict[str, ContainerRegion] = {}
        self._gone_since: dict[str, float] = {}

    def _pods(self) -> dict[str, dict] | None:
        if self.client is None:
            return None
        sel = f"spec.nodeName={self.node}" if self.node else None
        try:
            return {O.uid(p): p for p in self.client.list_pods(field_selector=sel)}
        except Exception as e:
            log.error("list pods failed: %s", e)
            return None

    def scan(self, now: float | None = None) -> dict[str, ContainerRegion]:
        now = now or time.time()
        pods = self._pods()
        try:
            entries = sorted(os.listdir(self.dir))
        except FileNotFoundError:
            entries = []
        seen = set()
        for key in entries:
            path = os.path.join(self.dir, key, REGION_FILE)
            uid, _, ctr = key.partition("_")
            if pods is not None and uid not in pods:
                first = self._gone_since.setdefault(key, now)
                if now - first >= GC_GRACE_S:
                    log.info("removing stale container dir %s", key)
                    cr = self.regions.pop(key, None)
                    if cr:
                        cr.region.close()
                    shutil.rmtree(os.path.join(self.dir, key), ignore_errors=True)
                    self._gone_since.pop(key, None)
                    continue
            else:
                self._gone_since.pop(key, None)
            if not os.path.exists(path):
                continue
            seen.add(key)
            if key not in self.regions:
                try:
                    r = AttachedRegion(path)
                except (FileNotFoundError, RuntimeError) as e:
                    log.debug("skip %s: %s", path, e)
                    continue
                self.regions[key] = ContainerRegion(key, uid, ctr, r)
            cr = self.regions[key]
            if pods is not None and uid in pods:
                cr.pod_name, cr.namespace = O.name(pods[uid]), O.namespace(pods[uid])
        for key in list(self.regions):
            if key not in seen:
                self.regions.pop(key).region.close()
        return self.regions
