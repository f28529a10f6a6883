"""Node monitor Prometheus collector (:9394).

Reference: cmd/vGPUmonitor/metrics.go:61-91 (descriptors), :140-246
(Collect: NVML host stats + per-container regions).  Same names and labels:
HostGPUMemoryUsage, HostCoreUtilization, vGPU_device_memory_usage_in_bytes,
vGPU_device_memory_limit_in_bytes, Device_memory_desc_of_container.
MI355X additions: vGPU_cu_mask_cus (CUs in the container's mask, mask as a
label), vGPU_throttle_wait_seconds, vGPU_oom_events_total,
vGPU_host_memory_bytes / vGPU_swap_{in,out}_bytes (virtual device memory),
HostGPUProcessCUOccupancy (KFD per-process CU occupancy).
"""
from __future__ import annotations

from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily


class MonitorCollector:
    def __init__(self, pathmon, backend=None):
        self.pm = pathmon
        self.backend = backend

    def collect(self):
        host_mem = GaugeMetricFamily("HostGPUMemoryUsage", "GPU device memory usage",
                                     labels=["deviceidx", "deviceuuid"])
        host_util = GaugeMetricFamily("HostCoreUtilization", "GPU core utilization",
                                      labels=["deviceidx", "deviceuuid"])
        occ = GaugeMetricFamily("HostGPUProcessCUOccupancy", "CUs occupied by a process (KFD)",
                                labels=["deviceidx", "deviceuuid", "pid"])
        if self.backend is not None:
            try:
                for d in self.backend.devices():
                    host_mem.add_metric([str(d.index), d.uuid], d.vram_used)
                    host_util.add_metric([str(d.index), d.uuid], d.gfx_activity)
                    for p in self.backend.processes(d.index):
                        occ.add_metric([str(d.index), d.uuid, str(p.pid)], p.cu_occupancy)
            except Exception:
                pass
        yield from (host_mem, host_util, occ)

        lab = ["podnamespace", "podname", "ctrname", "vdeviceid", "deviceuuid"]
        usage = GaugeMetricFamily("vGPU_device_memory_usage_in_bytes", "vGPU device usage", labels=lab)
        limit = GaugeMetricFamily("vGPU_device_memory_limit_in_bytes", "vGPU device limit", labels=lab)
        desc = CounterMetricFamily("Device_memory_desc_of_container", "Container device meory description",
                                   labels=lab + ["context", "module", "data", "offset"])
        cus = GaugeMetricFamily("vGPU_cu_mask_cus", "CUs in the container's CU mask (0 = whole device)",
                                labels=lab + ["mask"])
        hostb = GaugeMetricFamily("vGPU_host_memory_bytes", "Oversubscribed bytes resident in host memory",
                                  labels=lab)
        swin = CounterMetricFamily("vGPU_swap_in_bytes", "Pager host->HBM bytes", labels=lab)
        swout = CounterMetricFamily("vGPU_swap_out_bytes", "Pager HBM->host bytes", labels=lab)
        wait = CounterMetricFamily("vGPU_throttle_wait_seconds", "Time dispatches waited in the limiter",
                                   labels=["podnamespace", "podname", "ctrname"])
        ooms = CounterMetricFamily("vGPU_oom_events_total", "Allocations refused by the vGPU cap",
                                   labels=["podnamespace", "podname", "ctrname"])
        for cr in list(self.pm.regions.values()):
            base = [cr.namespace, cr.pod_name, cr.ctr_name]
            slots = cr.region.live_slots()
            for d in cr.region.devices():
                if not d.uuid and not d.mem_limit:
                    continue
                l = base + [str(d.index), d.uuid]
                usage.add_metric(l, d.used)
                limit.add_metric(l, d.mem_limit)
                desc.add_metric(l + [str(d.context), str(d.module), str(d.buffer), "0"], d.used)
                cus.add_metric(l + [hex(d.cu_mask)], bin(d.cu_mask).count("1"))
                hostb.add_metric(l, d.host_used)
                swin.add_metric(l, d.swap_in)
                swout.add_metric(l, d.swap_out)
            wait.add_metric(base, sum(s.throttle_wait_ns for s in slots) / 1e9)
            ooms.add_metric(base, sum(s.oom_events for s in slots))
        yield from (usage, limit, desc, cus, hostb, swin, swout, wait, ooms)
