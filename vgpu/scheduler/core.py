"""Scheduler extender core: node registry + handshake, pod usage ledger,
Filter and Bind.

Reference: pkg/scheduler/scheduler.go:41-53 (struct), :72-109 (pod informer
handlers), :135-229 (RegisterFromNodeAnnotations: handshake state machine,
device merge), :249-310 (getNodesUsage), :312-352 (Bind), :354-402 (Filter);
pkg/scheduler/nodes.go:59-114 (node manager), pkg/scheduler/pods.go:28-74
(pod manager).

Differences:
  * every shared map is accessed under one lock and readers get copies (the
    reference's ListNodes / GetScheduledPods return live maps unlocked);
  * Bind fails the binding when the node lock cannot be taken;
  * the pod informer is LIST + WATCH (resourceVersion, bookmarks, relist on
    410 Gone or any stream error; reference: client-go informer with
    add/update/delete handlers, scheduler.go:72-129), so a deleted pod frees
    its vGPU slot as soon as the delete event arrives.  The annotations stay
    the source of truth: a restart (or a relist) rebuilds the ledger.
"""
from __future__ import annotations

import copy
import datetime as dt
import logging
import threading
import time
from dataclasses import dataclass, field

from vgpu import config
from vgpu.api import resources as R
from vgpu.api.codec import (CodecError, apply_node_devices_ext, decode_node_devices,
                            decode_pod_devices, encode_pod_devices, NODE_REGISTER_EXT)
from vgpu.api.resources import ContainerDevice, DeviceInfo, DeviceUsage
from vgpu.device.base import get_devices, known_devices, resource_reqs
from vgpu.k8s import objects as O
from vgpu.k8s.client import ApiError, KubeClient
from vgpu.k8s.nodelock import NodeLockError, lock_node

from . import native as N
from .score import FitError, NodeUsage, calc_score, check_type, pick_node

log = logging.getLogger("vgpu.scheduler")

HANDSHAKE_TIME_FMT = "%Y.%m.%d %H:%M:%S"


@dataclass
class NodeInfo:
    id: str
    devices: list[DeviceInfo] = field(default_factory=list)


@dataclass
class PodInfo:
    namespace: str
    name: str
    uid: str
    node_id: str
    devices: list[list[ContainerDevice]]


class Scheduler:
    def __init__(self, client: KubeClient, cfg: config.SchedulerConfig | None = None):
        self.client = client
        self.cfg = cfg or config.SCHEDULER
        self._lock = threading.RLock()
        self.nodes: dict[str, NodeInfo] = {}
        self.pods: dict[str, PodInfo] = {}
        # per vendor handshake key → NodeInfo last registered (for removal)
        self._registered: dict[tuple[str, str], NodeInfo] = {}
        self.overview: dict[str, NodeUsage] = {}
        self._stop = threading.Event()
        self.filter_latency_s: list[float] = []
        # Flat per-device state for the native scorer, kept current on pod
        # add/remove, updated in place when a device's attributes change, and
        # rebuilt -- by the registration pass, off the /filter path -- only
        # when devices appear or vanish (_flat_stale).
        self._flat: N.FlatState | None = None
        self._flat_stale = False
        self._node_gen = 0
        self.informer_synced = threading.Event()
        self.informer_events = 0
        self.informer_relists = 0

    # ---- pod ledger (C4) ----------------------------------------------------------------
    def add_pod(self, pod: dict, node_id: str, devices: list[list[ContainerDevice]]) -> None:
        with self._lock:
            old = self.pods.get(O.uid(pod))
            self.pods[O.uid(pod)] = PodInfo(O.namespace(pod), O.name(pod), O.uid(pod), node_id, devices)
            if self._flat is not None:
                if old is not None:
                    self._flat.apply(old.node_id, old.devices, -1)
                self._flat.apply(node_id, devices, +1)

    def del_pod(self, pod: dict) -> None:
        with self._lock:
            old = self.pods.pop(O.uid(pod), None)
            if old is not None and self._flat is not None:
                self._flat.apply(old.node_id, old.devices, -1)

    def scheduled_pods(self) -> dict[str, PodInfo]:
        with self._lock:
            return copy.deepcopy(self.pods)

    def on_pod(self, pod: dict, deleted: bool = False) -> None:
        """Informer handler (reference onAddPod/onUpdatePod/onDelPod)."""
        annos = O.annotations(pod)
        node_id = annos.get(R.ASSIGNED_NODE)
        if node_id is None:
            return
        if deleted or O.is_terminated(pod):
            self.del_pod(pod)
            return
        ids = annos.get(R.ASSIGNED_IDS)
        if ids is None:
            return
        self.add_pod(pod, node_id, decode_pod_devices(ids))

    def resync_pods(self, pods: list[dict] | None = None) -> None:
        """Rebuild the ledger from pod annotations (restart recovery / relist)."""
        if pods is None:
            pods = self.client.list_pods()
        seen = set()
        for p in pods:
            if R.ASSIGNED_NODE in O.annotations(p):
                self.on_pod(p)
                seen.add(O.uid(p))
        with self._lock:
            for uid in list(self.pods):
                if uid not in seen:
                    old = self.pods.pop(uid)
                    if self._flat is not None:
                        self._flat.apply(old.node_id, old.devices, -1)

    # ---- node registry (C3) ---------------------------------------------------------------
    def add_node(self, node_id: str, info: NodeInfo) -> None:
        with self._lock:
            cur = self.nodes.get(node_id)
            if cur is None:
                self.nodes[node_id] = copy.deepcopy(info)
            else:
                known = {d.id for d in cur.devices}
                new = [copy.deepcopy(d) for d in info.devices if d.id not in known]
                if not new:
                    return
                cur.devices.extend(new)
            self._structure_changed()

    def _structure_changed(self) -> None:
        """Devices appeared or vanished (caller holds the lock)."""
        self._flat_stale = True
        self._node_gen += 1

    def rebuild_flat(self) -> None:
        """Rebuild the flat state after a structural change.  The registration
        thread is the only writer of the node registry, so it builds the new
        device table without the lock (readers never mutate it) and takes the
        lock only to add the pods' usage and swap it in."""
        with self._lock:
            if not self._flat_stale and self._flat is not None:
                return
            gen = self._node_gen
        flat = N.FlatState(self.nodes, {})
        with self._lock:
            if gen != self._node_gen:
                return  # changed again meanwhile: the next pass (or /filter) rebuilds
            flat.apply_all(self.pods)
            self._flat = flat
            self._flat_stale = False

    def rm_node_devices(self, node_id: str, info: NodeInfo) -> None:
        with self._lock:
            self._structure_changed()
            cur = self.nodes.get(node_id)
            if cur is None:
                return
            gone = {d.id for d in info.devices}
            cur.devices = [d for d in cur.devices if d.id not in gone]
            if not cur.devices:
                self.nodes.pop(node_id)

    def list_nodes(self) -> dict[str, NodeInfo]:
        with self._lock:
            return copy.deepcopy(self.nodes)

    def _now(self) -> dt.datetime:
        return dt.datetime.now()

    def register_from_node_annotations_once(self) -> None:
        """One pass of the handshake state machine (reference scheduler.go:135-229):
        Reported/absent → write Requesting_<now> and (re)register devices;
        Requesting older than the timeout → drop the devices, write Deleted_<now>;
        Deleted → ignore until the device plugin reports again."""
        kd = known_devices()
        for node in self.client.list_nodes():
            name = O.name(node)
            annos = O.annotations(node)
            for hs_key, reg_key in kd.items():
                if reg_key not in annos:
                    continue
                try:
                    devs = decode_node_devices(annos[reg_key])
                except CodecError:
                    continue
                if not devs:
                    continue
                apply_node_devices_ext(devs, annos.get(NODE_REGISTER_EXT))
                hs = annos.get(hs_key, "")
                if hs.startswith(R.HANDSHAKE_REQUESTING):
                    try:
                        t = dt.datetime.strptime(hs[len(R.HANDSHAKE_REQUESTING):], HANDSHAKE_TIME_FMT)
                    except ValueError:
                        t = self._now()
                    if self._now() > t + dt.timedelta(seconds=self.cfg.handshake_timeout_s):
                        prev = self._registered.get((name, hs_key))
                        if prev is not None:
                            self.rm_node_devices(name, prev)
                            self._registered.pop((name, hs_key), None)
                            log.warning("node %s devices %s left (handshake timeout)", name, hs_key)
                            try:
                                self.client.patch_node_annotations(
                                    name, {hs_key: R.HANDSHAKE_DELETED + self._now().strftime(HANDSHAKE_TIME_FMT)})
                            except ApiError as e:
                                log.error("patch node %s failed: %s", name, e)
                        continue
                    # Not expired yet: keep (or, after a scheduler restart, adopt)
                    # the devices without re-arming the handshake.  The reference
                    # skips the node here, leaving a restarted scheduler blind
                    # until the next plugin report.
                elif hs.startswith(R.HANDSHAKE_DELETED):
                    continue
                else:
                    try:
                        self.client.patch_node_annotations(
                            name, {hs_key: R.HANDSHAKE_REQUESTING + self._now().strftime(HANDSHAKE_TIME_FMT)})
                    except ApiError as e:
                        log.error("patch node %s failed: %s", name, e)
                info = NodeInfo(id=name)
                with self._lock:
                    cur = self.nodes.get(name)
                    byid = {x.id: x for x in cur.devices} if cur is not None else {}
                    for i, d in enumerate(devs):
                        if not d.index:
                            d.index = i
                        m = byid.get(d.id)
                        if m is None:
                            info.devices.append(d)
                            continue
                        attrs = (d.devmem, d.devcore, d.count, d.health, d.cus, d.xgmi_hive, d.resource)
                        if attrs == (m.devmem, m.devcore, m.count, m.health, m.cus, m.xgmi_hive, m.resource):
                            continue  # unchanged: nothing to invalidate
                        m.devmem, m.devcore, m.count, m.health, m.cus, m.xgmi_hive, m.resource = attrs
                        if self._flat is not None and not self._flat.update_device(name, m):
                            self._structure_changed()
                if info.devices:
                    self.add_node(name, info)
                self._registered[(name, hs_key)] = NodeInfo(id=name, devices=copy.deepcopy(devs))
        self.rebuild_flat()

    def run_loops(self) -> None:
        """Background registration + ledger resync (daemon threads)."""
        def reg():
            while not self._stop.is_set():
                try:
                    self.register_from_node_annotations_once()
                except Exception as e:  # keep the loop alive across API errors
                    log.error("registration pass failed: %s", e)
                self._stop.wait(self.cfg.register_interval_s)

        threading.Thread(target=reg, daemon=True, name="vgpu-register").start()
        threading.Thread(target=self.run_informer, daemon=True, name="vgpu-informer").start()

    def run_informer(self, watch_timeout_s: float = 300.0) -> None:
        """Pod informer: LIST (ledger rebuilt from annotations) then WATCH from
        the list's resourceVersion; relist after 410 Gone or a broken stream."""
        backoff = 0.5
        while not self._stop.is_set():
            try:
                items, rv = self.client.list_pods_rv()
                self.resync_pods(items)
                self.informer_synced.set()
                backoff = 0.5
                while not self._stop.is_set():
                    for typ, obj in self.client.watch_pods(rv, timeout_s=watch_timeout_s):
                        rv = (obj.get("metadata") or {}).get("resourceVersion", rv)
                        if typ == "BOOKMARK":
                            continue
                        if R.ASSIGNED_NODE in O.annotations(obj) or typ == "DELETED":
                            self.on_pod(obj, deleted=typ == "DELETED")
                        self.informer_events += 1
                        if self._stop.is_set():
                            break
            except Exception as e:  # 410 Gone, connection loss, decode errors: relist
                if self._stop.is_set():
                    break
                log.warning("pod informer: %s; relisting", e)
                self.informer_relists += 1
                self._stop.wait(backoff)
                backoff = min(backoff * 2, 10.0)

    def stop(self) -> None:
        self._stop.set()

    # ---- usage (getNodesUsage) -----------------------------------------------------------
    def nodes_usage(self, node_names: list[str] | None) -> tuple[dict[str, NodeUsage], dict[str, str]]:
        with self._lock:
            overall: dict[str, NodeUsage] = {}
            for nid, n in self.nodes.items():
                overall[nid] = NodeUsage(devices=[
                    DeviceUsage(id=d.id, index=d.index, used=0, count=d.count, usedmem=0,
                                totalmem=d.devmem, usedcores=0, totalcore=d.devcore, type=d.type,
                                numa=d.numa, health=d.health, cus=d.cus, xgmi_hive=d.xgmi_hive,
                                resource=d.resource)
                    for d in n.devices])
            for p in self.pods.values():
                node = overall.get(p.node_id)
                if node is None:
                    continue
                byid = {d.id: d for d in node.devices}
                for ctr in p.devices:
                    for cd in ctr:
                        d = byid.get(cd.uuid)
                        if d is not None:
                            d.used += 1
                            d.usedmem += cd.usedmem
                            d.usedcores += cd.usedcores
                            d.pods.append(p.uid)
            self.overview = overall
            failed: dict[str, str] = {}
            if node_names is None:
                return copy.deepcopy(overall), failed
            out = {}
            for nid in node_names:
                if nid in overall:
                    out[nid] = copy.deepcopy(overall[nid])
                else:
                    failed[nid] = "node unregistered"
            return out, failed

    # ---- extender verbs -------------------------------------------------------------------
    def filter(self, args: dict) -> dict:
        t0 = time.perf_counter()
        try:
            return self._filter(args)
        finally:
            self.filter_latency_s.append(time.perf_counter() - t0)
            if len(self.filter_latency_s) > 10000:
                del self.filter_latency_s[:5000]

    def _filter(self, args: dict) -> dict:
        pod = _ci(args, "pod") or {}
        node_names = _ci(args, "nodenames")
        if node_names is None:
            nl = _ci(args, "nodes")
            if nl:
                node_names = [O.name(n) for n in nl.get("items", [])]
        nums = resource_reqs(pod)
        if sum(k.nums for n in nums for k in n) == 0:
            return {"nodenames": node_names, "failedNodes": {}, "error": ""}
        annos = O.annotations(pod)
        self.del_pod(pod)  # re-scheduling is idempotent
        if N.load_lib() is not None:
            best, failed = self._filter_native(node_names, nums, annos)
            if isinstance(best, str):
                return {"nodenames": [], "failedNodes": failed, "error": best}
        else:
            usage, failed = self.nodes_usage(node_names)
            try:
                scores = calc_score(usage, nums, annos)
            except FitError as e:
                return {"nodenames": [], "failedNodes": failed, "error": str(e)}
            best = pick_node(scores)
            if best is None:
                for nid in usage:
                    failed.setdefault(nid, "no device fits the request")
        if best is None:
            return {"nodenames": [], "failedNodes": failed, "error": ""}
        enc = encode_pod_devices(best.devices)
        patch = {R.ASSIGNED_NODE: best.node_id, R.ASSIGNED_TIME: str(int(time.time())),
                 R.ASSIGNED_IDS: enc, R.ASSIGNED_IDS_TO_ALLOCATE: enc}
        self.add_pod(pod, best.node_id, best.devices)
        try:
            self.client.patch_pod_annotations(O.namespace(pod), O.name(pod), patch)
        except ApiError as e:
            self.del_pod(pod)
            return {"nodenames": [], "failedNodes": failed, "error": f"patch pod failed: {e}"}
        log.info("schedule %s/%s to %s %s", O.namespace(pod), O.name(pod), best.node_id, enc)
        return {"nodenames": [best.node_id], "failedNodes": failed, "error": ""}

    def _filter_native(self, node_names, nums, annos):
        """Score on the flat device state (native/sched/score.cpp).  Returns
        (NodeScore | None | error string, failed nodes)."""
        from vgpu.device.amd import assert_xgmi
        from .score import NodeScore
        with self._lock:
            if self._flat is None or self._flat_stale:  # first call, or a change the registration pass has not folded in
                self._flat = N.FlatState(self.nodes, self.pods)
                self._flat_stale = False
            res, failed = self._flat.filter(
                node_names, nums, check_type, annos, assert_xgmi(annos), config.SCHEDULER.xgmi_weight,
                binpack_devices=config.SCHEDULER.gpu_scheduler_policy != "spread",
                spread_nodes=config.SCHEDULER.node_scheduler_policy == "spread")
        if res.error:
            return res.error, failed
        if res.node is None:
            return None, failed
        return NodeScore(node_id=res.node, score=res.score, devices=res.devices), failed

    def bind(self, args: dict) -> dict:
        ns = _ci(args, "podNamespace")
        name = _ci(args, "podName")
        uid = _ci(args, "podUID")
        node = _ci(args, "node")
        try:
            lock_node(self.client, node)
        except (NodeLockError, ApiError) as e:
            log.warning("bind %s/%s: lock node %s failed: %s", ns, name, node, e)
            return {"error": f"node lock: {e}"}
        try:
            self.client.patch_pod_annotations(ns, name, {R.BIND_PHASE: R.BIND_ALLOCATING,
                                                         R.BIND_TIME: str(int(time.time()))})
            self.client.bind_pod(ns, name, uid, node)
        except ApiError as e:
            from vgpu.k8s.nodelock import release_node_lock
            try:
                release_node_lock(self.client, node)
            except Exception:
                pass
            try:
                self.client.patch_pod_annotations(ns, name, {R.BIND_PHASE: R.BIND_FAILED})
            except ApiError:
                pass
            return {"error": str(e)}
        return {"error": ""}


def _ci(d: dict, key: str):
    """Case-insensitive field lookup (Go's encoding/json matches names that way)."""
    if key in d:
        return d[key]
    lk = key.lower()
    for k, v in d.items():
        if k.lower() == lk:
            return v
    return None
