"""kubelet device-plugin gRPC server for `amd.com/gpu` vGPUs.

Reference: pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:54-68
(struct), :114-145 (Start: serve + register + health + node registration),
:162-209 (Serve with a crash-restart budget: >5 crashes within an hour is
fatal), :212-234 (Register with kubelet), :237-259 (GetDevicePluginOptions,
ListAndWatch streaming unhealthy updates), :262-277 (GetPreferredAllocation,
empty in the reference), :280-403 (Allocate), :405-434 (response devices),
:549-575 (PreStartContainer); rm/devices.go:144-167 (each GPU fanned out into
`splitCount` IDs "<uuid>-<i>"); rm/health.go:42-189 (health events).

Differences: GetPreferredAllocation is implemented (it steers kubelet to the
fake IDs of the physical GPUs the scheduler already chose, falling back to an
xGMI/NUMA-aware set), and a device that comes back after a GPU reset is marked
healthy again (the reference has no recovery path, server.go:253).
"""
from __future__ import annotations

import logging
import os
import queue
import threading
import time
from concurrent import futures

import grpc

from vgpu.api import resources as R
from vgpu.config import DevicePluginConfig
from vgpu.k8s.client import KubeClient

from . import api
from .allocate import AllocateError, allocate, get_pending_pod, next_device_request
from . import cdi
from .custate import CUMaskState
from .discovery import (EVT_POST_RESET, EVT_PRE_RESET, EVT_THERMAL, EVT_VMFAULT, TELEM_ECC, Backend,
                        Device)
from .topology import link_matrix, preferred

log = logging.getLogger("vgpu.deviceplugin")

MAX_RESTARTS_PER_HOUR = 5


def fake_ids(dev: Device, split: int) -> list[str]:
    return [f"{dev.uuid}-{i}" for i in range(split)]


def physical_of(fake_id: str) -> str:
    return fake_id.rsplit("-", 1)[0]


class VGPUDevicePlugin:
    def __init__(self, cfg: DevicePluginConfig, backend: Backend, client: KubeClient, node: str,
                 socket_name: str = "amd-vgpu.sock", devices: list[Device] | None = None,
                 resource_name: str | None = None, unhealthy: dict[str, str] | None = None):
        """`devices` / `resource_name`: the subset this server advertises and its
        extended resource (partition strategies, partitions.py); by default every
        device the backend finds, under cfg.resource_name."""
        self.cfg = cfg
        self.backend = backend
        self.client = client
        self.node = node
        self.socket_path = os.path.join(cfg.socket_dir, socket_name)
        self.resource_name = resource_name or cfg.resource_name
        self.devices = backend.devices() if devices is None else devices
        self.by_uuid = {d.uuid: d for d in self.devices}
        self.policy_unhealthy = dict(unhealthy or {})
        self.health: dict[str, bool] = {d.uuid: d.health and not self._partition_mismatch(d)
                                        and d.uuid not in self.policy_unhealthy for d in self.devices}
        for u, why in self.policy_unhealthy.items():
            if u in self.by_uuid:
                log.warning("device %s advertised unhealthy: %s", u, why)
        for d in self.devices:
            if self._partition_mismatch(d):
                log.warning("device %s is in compute partition %s, expected %s: advertised unhealthy",
                            d.uuid, d.compute_partition, cfg.partition_mode)
        self._ecc_baseline: dict[str, int] = {}   # uncorrectable ECC count at the last healthy point
        self.vm_faults: dict[str, int] = {}
        self.thermal_events: dict[str, int] = {}
        self.cu_state = CUMaskState(os.path.join(cfg.host_lib_dir, "containers"), policy=cfg.cu_share,
                                    max_mask_slots=cfg.max_mask_slots)
        log.info("compute share policy %s (max %d masked vGPUs per GPU), CU packing %s", cfg.cu_share,
                 cfg.max_mask_slots, self.cu_state.pack)
        self._links = None
        self._server: grpc.Server | None = None
        self._watchers: list[queue.Queue] = []
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._restarts: list[float] = []

    # ---- device list ----------------------------------------------------------------
    def plugin_devices(self) -> list:
        out = []
        for d in self.devices:
            st = api.HEALTHY if self.health.get(d.uuid, True) else api.UNHEALTHY
            for fid in fake_ids(d, self.cfg.device_split_count):
                dv = api.Device(ID=fid, health=st)
                dv.topology.nodes.add(ID=max(d.numa, 0))
                out.append(dv)
        return out

    def _partition_mismatch(self, d) -> bool:
        """--partition-mode pins the compute partition (SPX/DPX/QPX/CPX) this node is
        expected to run in; a device found in another mode (re-partitioned under a
        running plugin, or a node prepared with the wrong amd-smi profile) would
        hand out vGPUs sized for the wrong CU/HBM share, so it is advertised
        unhealthy until it is back in the expected mode."""
        want = (self.cfg.partition_mode or "").upper()
        return bool(want) and (d.compute_partition or "SPX").upper() != want

    def set_health(self, uuid: str, healthy: bool, reason: str = "") -> None:
        with self._lock:
            if self.health.get(uuid) == healthy:
                return
            self.health[uuid] = healthy
            watchers = list(self._watchers)
        log.warning("device %s is now %s %s", uuid, "healthy" if healthy else "UNHEALTHY", reason)
        for q in watchers:
            q.put(True)

    # ---- gRPC: DevicePlugin ------------------------------------------------------------
    def GetDevicePluginOptions(self, request, context):
        return api.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=True)

    def ListAndWatch(self, request, context):
        q: queue.Queue = queue.Queue()
        with self._lock:
            self._watchers.append(q)
        try:
            yield api.ListAndWatchResponse(devices=self.plugin_devices())
            while not self._stop.is_set() and context.is_active():
                try:
                    q.get(timeout=1.0)
                except queue.Empty:
                    continue
                yield api.ListAndWatchResponse(devices=self.plugin_devices())
        finally:
            with self._lock:
                if q in self._watchers:
                    self._watchers.remove(q)

    def GetPreferredAllocation(self, request, context):
        resp = api.PreferredAllocationResponse()
        for creq in request.container_requests:
            avail = list(creq.available_deviceIDs)
            chosen = self._preferred_for(avail, list(creq.must_include_deviceIDs), creq.allocation_size)
            resp.container_responses.add(deviceIDs=chosen)
        return resp

    def _preferred_for(self, avail: list[str], must: list[str], size: int) -> list[str]:
        by_phys: dict[str, list[str]] = {}
        for fid in avail:
            by_phys.setdefault(physical_of(fid), []).append(fid)
        # 1) the scheduler's choice for the pending pod
        try:
            pod = get_pending_pod(self.client, self.node)
            if pod is not None:
                _, devreq = next_device_request(R.VENDOR, pod)
                picks = []
                for d in devreq:
                    ids = [f for f in by_phys.get(d.uuid, []) if f not in picks]
                    if ids:
                        picks.append(ids[0])
                if len(picks) == size:
                    return picks
        except (AllocateError, Exception) as e:  # advisory only
            log.debug("preferred allocation without annotation: %s", e)
        # 2) xGMI/NUMA-aware choice over distinct physical devices
        phys = [u for u in by_phys if u in self.by_uuid]
        pos = {u: i for i, u in enumerate(d.uuid for d in self.devices)}
        cand = [pos[u] for u in phys]
        mustp = [pos[physical_of(m)] for m in must if physical_of(m) in pos]
        if self._links is None:
            self._links = link_matrix(self.backend, self.devices)
        used = {pos[u]: self.cfg.device_split_count - len(by_phys[u]) for u in phys}
        sel = preferred(cand, mustp, min(size, len(cand)), self.devices, self._links, used)
        out = [m for m in must]
        for p in sel:
            for f in by_phys[self.devices[p].uuid]:
                if f not in out:
                    out.append(f)
                    break
        for f in avail:  # more fake IDs than physical devices requested: fill up
            if len(out) >= size:
                break
            if f not in out:
                out.append(f)
        return out[:size]

    def Allocate(self, request, context):
        reqs = [list(c.devices_ids) for c in request.container_requests]
        for ids in reqs:
            for fid in ids:
                u = physical_of(fid)
                if u not in self.by_uuid:
                    context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unknown device {fid}")
        try:
            grants = allocate(self.client, self.cfg, R.VENDOR, reqs, self.by_uuid, self.cu_state, self.node)
        except Exception as e:
            context.abort(grpc.StatusCode.UNKNOWN, str(e))
        resp = api.AllocateResponse()
        for g in grants:
            cr = resp.container_responses.add()
            for k, v in g.envs.items():
                cr.envs[k] = v
            for cp, hp, ro in g.mounts:
                cr.mounts.add(container_path=cp, host_path=hp, read_only=ro)
            for cp, hp, perm in g.devices:
                cr.devices.add(container_path=cp, host_path=hp, permissions=perm)
            for k, v in g.annotations.items():
                cr.annotations[k] = v
            for name in g.cdi_devices:
                cr.cdi_devices.add(name=name)
        return resp

    def PreStartContainer(self, request, context):
        return api.PreStartContainerResponse()

    # ---- lifecycle ---------------------------------------------------------------------------
    def serve(self) -> None:
        os.makedirs(self.cfg.socket_dir, exist_ok=True)
        if os.path.exists(self.socket_path):
            os.unlink(self.socket_path)
        srv = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
        srv.add_generic_rpc_handlers((api.service_handler("DevicePlugin", self),))
        srv.add_insecure_port(api.unix_target(self.socket_path))
        srv.start()
        self._server = srv
        # wait until the socket answers (reference dials with a 5 s timeout)
        ch = grpc.insecure_channel(api.unix_target(self.socket_path))
        grpc.channel_ready_future(ch).result(timeout=5)
        ch.close()

    def register(self) -> None:
        kubelet = os.path.join(self.cfg.socket_dir, api.KUBELET_SOCKET)
        with grpc.insecure_channel(api.unix_target(kubelet)) as ch:
            stub = api.Stub(ch, "Registration")
            stub.Register(api.RegisterRequest(
                version=api.VERSION, endpoint=os.path.basename(self.socket_path),
                resource_name=self.resource_name,
                options=api.DevicePluginOptions(get_preferred_allocation_available=True)), timeout=5)

    def start(self) -> None:
        if self.cfg.device_list_strategy.startswith("cdi"):
            cdi.write_spec(self.devices, self.cfg.cdi_dir)
        self.serve()
        self.register()
        threading.Thread(target=self._health_loop, daemon=True, name="vgpu-health").start()
        log.info("device plugin serving %s: %d devices x %d vGPUs on %s", self.resource_name, len(self.devices),
                 self.cfg.device_split_count, self.socket_path)

    def stop(self) -> None:
        self._stop.set()
        if self._server is not None:
            self._server.stop(grace=1).wait()
            self._server = None
        if os.path.exists(self.socket_path):
            try:
                os.unlink(self.socket_path)
            except OSError:
                pass

    def note_crash(self) -> bool:
        """Crash-restart budget: False once > MAX_RESTARTS_PER_HOUR in the last hour."""
        now = time.time()
        self._restarts = [t for t in self._restarts if now - t < 3600] + [now]
        return len(self._restarts) <= MAX_RESTARTS_PER_HOUR

    # ---- health ---------------------------------------------------------------------------------
    def health_step(self, timeout_ms: int = 1000) -> None:
        """One poll (reference rm/health.go:42-189: XID/ECC event set):
        * device events: reset → unhealthy, post-reset → healthy again (the
          reference has no recovery path, server.go:253 FIXME); VM faults and
          thermal throttling are counted and logged but leave the device
          healthy (an application fault, like the XIDs 13/31/43/45/68 the
          reference skips);
        * uncorrectable ECC: any increase of the device's RAS uncorrectable
          count since the last healthy baseline → unhealthy until a reset;
        * the device list itself: a vanished device → unhealthy."""
        if os.environ.get("DP_DISABLE_HEALTHCHECKS", "").lower() in ("all", "true", "1"):
            return
        by_index = {d.index: d for d in self.devices}  # backend index -> our device (a subset per resource)
        for dev, typ, msg in self.backend.events(timeout_ms):
            if dev not in by_index:
                continue
            uuid = by_index[dev].uuid
            if typ == EVT_PRE_RESET:
                self.set_health(uuid, False, f"GPU reset: {msg}")
            elif typ == EVT_POST_RESET:
                self._ecc_baseline.pop(uuid, None)  # counters restart with the device
                if not self._partition_mismatch(by_index[dev]) and uuid not in self.policy_unhealthy:
                    self.set_health(uuid, True, f"GPU reset done: {msg}")
            elif typ == EVT_VMFAULT:
                self.vm_faults[uuid] = self.vm_faults.get(uuid, 0) + 1
                log.warning("device %s: VM fault (%s); device stays healthy", uuid, msg)
            elif typ == EVT_THERMAL:
                self.thermal_events[uuid] = self.thermal_events.get(uuid, 0) + 1
                log.warning("device %s: thermal throttling (%s)", uuid, msg)
        for d in self.devices:
            t = self.backend.telemetry(d.index)
            if t is None or not t.valid & TELEM_ECC:
                continue
            base = self._ecc_baseline.setdefault(d.uuid, t.ecc_uncorrectable)
            if t.ecc_uncorrectable > base and self.health.get(d.uuid, True):
                self.set_health(d.uuid, False,
                                f"uncorrectable ECC errors: {t.ecc_uncorrectable - base} new")
        present = {d.uuid: d for d in self.backend.devices()}
        for d in self.devices:
            if d.uuid not in present:
                self.set_health(d.uuid, False, "device disappeared")
            elif not present[d.uuid].health:
                self.set_health(d.uuid, False, "driver reports unhealthy")
            elif d.uuid in self.policy_unhealthy:
                continue
            elif self.cfg.partition_mode:
                pd = present[d.uuid]
                was_bad, d.compute_partition = self._partition_mismatch(d), pd.compute_partition
                if self._partition_mismatch(d):
                    self.set_health(d.uuid, False, f"compute partition {d.compute_partition}, "
                                    f"expected {self.cfg.partition_mode}")
                elif was_bad:
                    self.set_health(d.uuid, True, f"compute partition {d.compute_partition} restored")

    def _health_loop(self) -> None:
        while not self._stop.is_set():
            try:
                self.health_step(1000)
            except Exception as e:
                log.error("health check failed: %s", e)
                self._stop.wait(5.0)
