"""Scheduler Prometheus collector (same metric names as the reference so its
Grafana dashboard keeps working).

Reference: cmd/scheduler/metrics.go:65-207 (Collect over the ledger), :223-242
(served on :9395).  The reference's `vGPUCorePercentage` carries a typo'd
label ("nmodename"); we export the intended "nodename".  Added:
`vGPUSchedulerFilterLatencySeconds` (filter latency summary).
"""
from __future__ import annotations

from prometheus_client.core import GaugeMetricFamily, SummaryMetricFamily

MIB = 1024 * 1024


class SchedulerCollector:
    def __init__(self, scheduler):
        self.s = scheduler

    def collect(self):
        usage, _ = self.s.nodes_usage(None)
        lim = GaugeMetricFamily("GPUDeviceMemoryLimit", "Device memory limit for a certain GPU",
                                labels=["nodeid", "deviceuuid", "deviceidx"])
        core_lim = GaugeMetricFamily("GPUDeviceCoreLimit", "Device memory core limit for a certain GPU",
                                     labels=["nodeid", "deviceuuid", "deviceidx"])
        mem_alloc = GaugeMetricFamily("GPUDeviceMemoryAllocated", "Device memory allocated for a certain GPU",
                                      labels=["nodeid", "deviceuuid", "deviceidx", "devicecores"])
        shared = GaugeMetricFamily("GPUDeviceSharedNum", "Number of containers sharing this GPU",
                                   labels=["nodeid", "deviceuuid", "deviceidx"])
        core_alloc = GaugeMetricFamily("GPUDeviceCoreAllocated", "Device core allocated for a certain GPU",
                                       labels=["nodeid", "deviceuuid", "deviceidx"])
        overview = GaugeMetricFamily("nodeGPUOverview", "GPU overview on a certain node",
                                     labels=["nodeid", "deviceuuid", "deviceidx", "devicecores",
                                             "sharedcontainers", "devicememorylimit", "devicetype"])
        mem_pct = GaugeMetricFamily("nodeGPUMemoryPercentage",
                                    "GPU Memory Allocated Percentage on a certain GPU",
                                    labels=["nodeid", "deviceuuid", "deviceidx"])
        totals = {}
        for nid, nu in sorted(usage.items()):
            for d in nu.devices:
                idx = str(d.index)
                totals[d.id] = d.totalmem
                lim.add_metric([nid, d.id, idx], d.totalmem * MIB)
                core_lim.add_metric([nid, d.id, idx], d.totalcore)
                mem_alloc.add_metric([nid, d.id, idx, str(d.usedcores)], d.usedmem * MIB)
                shared.add_metric([nid, d.id, idx], d.used)
                core_alloc.add_metric([nid, d.id, idx], d.usedcores)
                overview.add_metric([nid, d.id, idx, str(d.usedcores), str(d.used), str(d.totalmem), d.type],
                                    d.usedmem * MIB)
                mem_pct.add_metric([nid, d.id, idx], d.usedmem / d.totalmem if d.totalmem else 0.0)
        yield from (lim, core_lim, mem_alloc, shared, core_alloc, overview, mem_pct)

        pod_dev = GaugeMetricFamily("vGPUPodsDeviceAllocated", "vGPU Allocated from pods",
                                    labels=["namespace", "nodename", "podname", "containeridx",
                                            "deviceuuid", "deviceusedcore"])
        pod_mem = GaugeMetricFamily("vGPUMemoryPercentage", "vGPU memory percentage allocated from a container",
                                    labels=["namespace", "nodename", "podname", "containeridx", "deviceuuid"])
        pod_core = GaugeMetricFamily("vGPUCorePercentage", "vGPU core allocated from a container",
                                     labels=["namespace", "nodename", "podname", "containeridx", "deviceuuid"])
        for p in self.s.scheduled_pods().values():
            for ci, ctr in enumerate(p.devices):
                for cd in ctr:
                    lab = [p.namespace, p.node_id, p.name, str(ci), cd.uuid]
                    pod_dev.add_metric(lab + [str(cd.usedcores)], cd.usedmem * MIB)
                    if totals.get(cd.uuid):
                        pod_mem.add_metric(lab, cd.usedmem / totals[cd.uuid])
                    pod_core.add_metric(lab, cd.usedcores)
        yield from (pod_dev, pod_mem, pod_core)

        lat = list(self.s.filter_latency_s)
        sm = SummaryMetricFamily("vGPUSchedulerFilterLatencySeconds", "Extender filter latency",
                                 count_value=len(lat), sum_value=float(sum(lat)))
        yield sm
