#!/usr/bin/env python3
"""Generate docs/gpu-dashboard.json: a Grafana dashboard over the scheduler
(:9395) and node monitor (:9394) metrics.

Reference: docs/gpu-dashboard.json + docs/dashboard.md (a DCGM-based board
plus the vGPU series).  Here every panel queries a series this framework
exports (vgpu/scheduler/metrics.py, vgpu/monitor/metrics.py) — tests/
test_monitor.py checks that each expression names one of them.

    python scripts/gen_dashboard.py > docs/gpu-dashboard.json
"""
from __future__ import annotations

import json

PANELS = [
    # (title, unit, [(expr, legend)])
    ("Node HBM allocated by vGPUs", "bytes",
     [("sum by (nodeid, deviceidx) (GPUDeviceMemoryAllocated)", "{{nodeid}} gpu{{deviceidx}}")]),
    ("Node HBM allocatable", "bytes",
     [("GPUDeviceMemoryLimit", "{{nodeid}} gpu{{deviceidx}}")]),
    ("vGPUs per physical GPU", "short",
     [("GPUDeviceSharedNum", "{{nodeid}} gpu{{deviceidx}}")]),
    ("CU share allocated (%)", "percent",
     [("GPUDeviceCoreAllocated", "{{nodeid}} gpu{{deviceidx}}")]),
    ("Node HBM allocated (fraction)", "percentunit",
     [("nodeGPUMemoryPercentage", "{{nodeid}} gpu{{deviceidx}}")]),
    ("Pod HBM share of device (fraction)", "percentunit",
     [("vGPUMemoryPercentage", "{{namespace}}/{{podname}}")]),
    ("Pod CU share of device (%)", "percent",
     [("vGPUCorePercentage", "{{namespace}}/{{podname}}")]),
    ("Container HBM usage vs cap", "bytes",
     [("vGPU_device_memory_usage_in_bytes", "{{podname}}/{{ctrname}} used"),
      ("vGPU_device_memory_limit_in_bytes", "{{podname}}/{{ctrname}} cap")]),
    ("Container CU mask size", "short",
     [("vGPU_cu_mask_cus", "{{podname}}/{{ctrname}}")]),
    ("Host-resident (oversubscribed) bytes", "bytes",
     [("vGPU_host_memory_bytes", "{{podname}}/{{ctrname}}")]),
    ("Pager traffic", "Bps",
     [("rate(vGPU_swap_in_bytes[1m])", "{{podname}} in"),
      ("rate(vGPU_swap_out_bytes[1m])", "{{podname}} out")]),
    ("Limiter wait (s/s)", "short",
     [("rate(vGPU_throttle_wait_seconds[1m])", "{{podname}}/{{ctrname}}")]),
    ("Cap refusals (OOM) per minute", "short",
     [("increase(vGPU_oom_events_total[1m])", "{{podname}}/{{ctrname}}")]),
    ("GPU utilization (host)", "percent",
     [("HostCoreUtilization", "gpu{{deviceidx}}")]),
    ("GPU HBM used (host)", "bytes",
     [("HostGPUMemoryUsage", "gpu{{deviceidx}}")]),
]


def dashboard() -> dict:
    panels = []
    for i, (title, unit, targets) in enumerate(PANELS):
        panels.append({
            "id": i + 1,
            "type": "timeseries",
            "title": title,
            "datasource": {"type": "prometheus", "uid": "${DS_PROMETHEUS}"},
            "gridPos": {"h": 8, "w": 12, "x": 12 * (i % 2), "y": 8 * (i // 2)},
            "fieldConfig": {"defaults": {"unit": unit}, "overrides": []},
            "targets": [{"expr": e, "legendFormat": lg, "refId": chr(ord("A") + j)}
                        for j, (e, lg) in enumerate(targets)],
        })
    return {
        "__inputs": [{"name": "DS_PROMETHEUS", "label": "Prometheus", "type": "datasource",
                      "pluginId": "prometheus"}],
        "title": "vGPU on MI355X",
        "uid": "vgpu-amd-mi355x",
        "schemaVersion": 38,
        "time": {"from": "now-1h", "to": "now"},
        "refresh": "30s",
        "tags": ["vgpu", "amd", "mi355x"],
        "panels": panels,
    }


if __name__ == "__main__":
    print(json.dumps(dashboard(), indent=1))
