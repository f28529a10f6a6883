"""Node monitor Prometheus collector (:9394).

Reference: cmd/vGPUmonitor/metrics.go:61-91 (descriptors), :140-246
(Collect: NVML host stats + per-container regions).  Same names and labels:
HostGPUMemoryUsage, HostCoreUtilization, vGPU_device_memory_usage_in_bytes,
vGPU_device_memory_limit_in_bytes, Device_memory_desc_of_container.
MI355X additions: vGPU_cu_mask_cus (CUs in the container's mask, mask as a
label), vGPU_throttle_wait_seconds, vGPU_oom_events_total,
vGPU_host_memory_bytes / vGPU_swap_{in,out}_bytes (virtual device memory),
HostGPUProcessCUOccupancy (KFD per-process CU occupancy), host telemetry
HostGPUPowerWatts, HostGPUTemperatureCelsius{sensor}, HostGPUECCErrors{type},
HostXGMIReadBytes / HostXGMIWriteBytes (amdsmi gpu_metrics accumulators), and
the shim's per-container GPU-time share vGPU_gpu_time_share (0..1, last 120 ms).
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
        dl = ["deviceidx", "deviceuuid"]
        power = GaugeMetricFamily("HostGPUPowerWatts", "GPU socket power", labels=dl)
        temp = GaugeMetricFamily("HostGPUTemperatureCelsius", "GPU temperature", labels=dl + ["sensor"])
        ecc = CounterMetricFamily("HostGPUECCErrors", "Accumulated ECC errors (RAS)", labels=dl + ["type"])
        xrd = CounterMetricFamily("HostXGMIReadBytes", "Bytes read over all xGMI links", labels=dl)
        xwr = CounterMetricFamily("HostXGMIWriteBytes", "Bytes written over all xGMI links", labels=dl)
        if self.backend is not None:
            try:
                for d in self.backend.devices():
                    lab = [str(d.index), d.uuid]
                    host_mem.add_metric(lab, d.vram_used)
                    host_util.add_metric(lab, d.gfx_activity)
                    for p in self.backend.processes(d.index):
                        occ.add_metric(lab + [str(p.pid)], p.cu_occupancy)
                    t = self.backend.telemetry(d.index)
                    if t is None:
                        continue
                    if t.valid & 2:
                        power.add_metric(lab, t.power_w)
                    if t.valid & 4:
                        for sensor, v in (("edge", t.temp_edge_c), ("hotspot", t.temp_hotspot_c),
                                          ("memory", t.temp_mem_c)):
                            temp.add_metric(lab + [sensor], v)
                    if t.valid & 1:
                        ecc.add_metric(lab + ["correctable"], t.ecc_correctable)
                        ecc.add_metric(lab + ["uncorrectable"], t.ecc_uncorrectable)
                    if t.valid & 8:
                        xrd.add_metric(lab, t.xgmi_read_bytes)
                        xwr.add_metric(lab, t.xgmi_write_bytes)
            except Exception:
                pass
        yield from (host_mem, host_util, occ, power, temp, ecc, xrd, xwr)

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
        share = GaugeMetricFamily("vGPU_gpu_time_share", "Fair-share GPU time of the container (temporal limiter)",
                                  labels=lab)
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
                if d.busy_ns:
                    share.add_metric(l, d.busy_permille / 1000.0)
            wait.add_metric(base, sum(s.throttle_wait_ns for s in slots) / 1e9)
            ooms.add_metric(base, sum(s.oom_events for s in slots))
        yield from (usage, limit, desc, cus, hostb, swin, swout, wait, ooms, share)
