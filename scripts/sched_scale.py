"""/filter latency at cluster scale: N nodes x 8 MI355X, P pods already placed.

    python scripts/sched_scale.py [--nodes 1000] [--pods 8000] [--calls 50] [--register-every 10]

The scheduler runs in-process with a stub API client (the annotation patch of
the chosen node is a no-op), so the number is the extender's own work:
usage snapshot, scoring and node choice (reference hot path
pkg/scheduler/scheduler.go:249-310 getNodesUsage + score.go:183-214 calcScore).

Registration churn: the nodes are registered through their
device-plugin annotations, and every --register-every calls a registration
pass runs (reference RegisterFromNodeAnnotations, scheduler.go:135-229, every
15 s in production); on every third pass one node's GPU flips health, and
halfway through a new node joins.  The filter calls right after a pass are
part of the latency sample; the pass itself runs between calls, as on the
registration thread.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vgpu import config  # noqa: E402
from vgpu.api import resources as R  # noqa: E402
from vgpu.api.codec import encode_node_devices  # noqa: E402
from vgpu.api.resources import ContainerDevice, DeviceInfo  # noqa: E402
from vgpu.device.base import init_default_devices, known_devices  # noqa: E402
from vgpu.scheduler.core import NodeInfo, Scheduler  # noqa: E402


class StubClient:
    """Nodes with device-plugin register annotations; patches are no-ops."""

    def __init__(self):
        self.nodes: dict[str, list[DeviceInfo]] = {}

    def patch_pod_annotations(self, ns, name, annos):
        return {}

    def patch_node_annotations(self, name, annos):
        return {}

    def list_nodes(self):
        (hs_key, reg_key), = known_devices().items()
        return [{"metadata": {"name": n, "annotations": {
            reg_key: encode_node_devices(devs), hs_key: R.HANDSHAKE_REPORTED + "2026.01.01 00:00:00"}}}
            for n, devs in self.nodes.items()]


def node_devices(n: int) -> list[DeviceInfo]:
    return [DeviceInfo(id=f"GPU-{n:04d}-{i}", index=i, count=10, devmem=294912, devcore=100,
                       type="AMD-MI355X", numa=i // 4, health=True) for i in range(8)]


def build(nodes: int, pods: int) -> Scheduler:
    init_default_devices()
    config.SCHEDULER = config.SchedulerConfig()
    client = StubClient()
    s = Scheduler(client)
    for n in range(nodes):
        client.nodes[f"node-{n:04d}"] = node_devices(n)
    s.register_from_node_annotations_once()
    for p in range(pods):
        n = p % nodes
        i = (p // nodes) % 8
        pod = {"metadata": {"name": f"p{p}", "namespace": "default", "uid": f"u{p}"}}
        s.add_pod(pod, f"node-{n:04d}", [[ContainerDevice(uuid=f"GPU-{n:04d}-{i}", type=R.VENDOR,
                                                         usedmem=18000, usedcores=10)]])
    return s


def measure(s: Scheduler, nodes: int, calls: int, register_every: int = 0) -> dict:
    names = [f"node-{n:04d}" for n in range(nodes)]
    lat = []
    passes = 0
    reg_s = []
    for c in range(calls):
        if register_every and c and c % register_every == 0:
            passes += 1
            if passes % 3 == 0:  # one GPU's health flips
                d = s.client.nodes[names[passes % nodes]][passes % 8]
                d.health = not d.health
            if c == (calls // (2 * register_every)) * register_every:  # a node joins
                s.client.nodes[f"node-{nodes:04d}"] = node_devices(nodes)
            t0 = time.perf_counter()
            s.register_from_node_annotations_once()
            reg_s.append(time.perf_counter() - t0)
        pod = {"metadata": {"name": f"new{c}", "namespace": "default", "uid": f"new{c}", "annotations": {}},
               "spec": {"containers": [{"name": "c", "resources": {"limits": {
                   R.RESOURCE_COUNT: "1", R.RESOURCE_MEM: "36000", R.RESOURCE_CORES: "25"}}}]}}
        t0 = time.perf_counter()
        r = s.filter({"pod": pod, "nodenames": names})
        lat.append(time.perf_counter() - t0)
        assert r["nodenames"], r
        s.del_pod(pod)  # keep the cluster state fixed between calls
    lat.sort()
    return {"nodes": nodes, "gpus": nodes * 8, "calls": calls, "median_ms": 1e3 * statistics.median(lat),
            "p90_ms": 1e3 * lat[int(0.9 * (len(lat) - 1))], "p99_ms": 1e3 * lat[int(0.99 * (len(lat) - 1))],
            "max_ms": 1e3 * lat[-1], "registration_passes": passes,
            "registration_pass_ms_max": round(1e3 * max(reg_s), 1) if reg_s else None}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--pods", type=int, default=8000)
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--register-every", type=int, default=10)
    a = ap.parse_args()
    s = build(a.nodes, a.pods)
    res = measure(s, a.nodes, a.calls, a.register_every)
    res["pods"] = a.pods
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
