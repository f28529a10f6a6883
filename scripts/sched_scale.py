"""/filter latency at cluster scale: N nodes x 8 MI355X, P pods already placed.

    python scripts/sched_scale.py [--nodes 1000] [--pods 8000] [--calls 50]

The scheduler runs in-process with a stub API client (the annotation patch of
the chosen node is a no-op), so the number is the extender's own work:
usage snapshot, scoring and node choice (reference hot path
pkg/scheduler/scheduler.go:249-310 getNodesUsage + score.go:183-214 calcScore).
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
from vgpu.api.resources import ContainerDevice, DeviceInfo  # noqa: E402
from vgpu.device.base import init_default_devices  # noqa: E402
from vgpu.scheduler.core import NodeInfo, Scheduler  # noqa: E402


class StubClient:
    def patch_pod_annotations(self, ns, name, annos):
        return {}


def build(nodes: int, pods: int) -> Scheduler:
    init_default_devices()
    config.SCHEDULER = config.SchedulerConfig()
    s = Scheduler(StubClient())
    for n in range(nodes):
        devs = [DeviceInfo(id=f"GPU-{n:04d}-{i}", index=i, count=10, devmem=294912, devcore=100,
                           type="AMD-MI355X", numa=i // 4, health=True) for i in range(8)]
        s.add_node(f"node-{n:04d}", NodeInfo(id=f"node-{n:04d}", devices=devs))
    for p in range(pods):
        n = p % nodes
        i = (p // nodes) % 8
        pod = {"metadata": {"name": f"p{p}", "namespace": "default", "uid": f"u{p}"}}
        s.add_pod(pod, f"node-{n:04d}", [[ContainerDevice(uuid=f"GPU-{n:04d}-{i}", type=R.VENDOR,
                                                         usedmem=18000, usedcores=10)]])
    return s


def measure(s: Scheduler, nodes: int, calls: int) -> dict:
    names = [f"node-{n:04d}" for n in range(nodes)]
    lat = []
    for c in range(calls):
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
            "p90_ms": 1e3 * lat[int(0.9 * (len(lat) - 1))], "max_ms": 1e3 * lat[-1]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--pods", type=int, default=8000)
    ap.add_argument("--calls", type=int, default=50)
    a = ap.parse_args()
    s = build(a.nodes, a.pods)
    res = measure(s, a.nodes, a.calls)
    res["pods"] = a.pods
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
