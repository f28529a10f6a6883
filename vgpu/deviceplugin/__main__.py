"""Device plugin daemon: serve + register with kubelet, publish node
annotations, restart when kubelet restarts (its socket is recreated) or on
SIGHUP, garbage-collect per-container state.

Reference: cmd/device-plugin/nvidia/main.go:38-127 (flags/env), :154-238
(start: fsnotify on kubelet.sock → restart, SIGHUP → restart, 30 s retry when
starting fails), :240-306 (startPlugins), watchers.go:26-48; vgpucfg.go:15-133
(split count, memory/cores scaling, disable core limit, per-node JSON).

    NODE_NAME=<node> python -m vgpu.deviceplugin --device-split-count 10 --backend auto
"""
from __future__ import annotations

import argparse
import logging
import os
import shutil
import signal
import sys
import threading
import time

from vgpu.config import DevicePluginConfig, add_dataclass_args, from_namespace
from vgpu.k8s.client import KubeClient

from .discovery import load_backend
from .register import Registrar
from .server import VGPUDevicePlugin

log = logging.getLogger("vgpu.deviceplugin.main")


def install_host_files(cfg: DevicePluginConfig) -> None:
    """Copy the enforcement library + ld.so.preload into the host dir that
    Allocate mounts into containers (reference docker/entrypoint.sh:17-21)."""
    from vgpu.native import shim_path
    os.makedirs(os.path.join(cfg.host_lib_dir, "containers"), exist_ok=True)
    src = shim_path()
    if src.exists():
        dst = os.path.join(cfg.host_lib_dir, "libvgpu.so")
        tmp = dst + ".tmp"
        shutil.copyfile(src, tmp)
        os.replace(tmp, dst)
    with open(os.path.join(cfg.host_lib_dir, "ld.so.preload"), "w") as f:
        f.write("/usr/local/vgpu/libvgpu.so\n")


def socket_id(path: str):
    try:
        st = os.stat(path)
        return (st.st_ino, st.st_ctime_ns)
    except OSError:
        return None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="vgpu-device-plugin")
    add_dataclass_args(ap, DevicePluginConfig)
    ap.add_argument("-v", "--verbose", action="count", default=0)
    ns = ap.parse_args(argv)
    logging.basicConfig(level=logging.DEBUG if ns.verbose else logging.INFO,
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    cfg = from_namespace(DevicePluginConfig, ns)
    cfg.node_name = cfg.node_name or os.environ.get("NODE_NAME") or os.environ.get("NodeName", "")
    cfg.apply_node_overrides()
    if not cfg.node_name:
        log.error("NODE_NAME is required")
        return 2
    install_host_files(cfg)
    backend = load_backend(cfg.backend)
    client = KubeClient.from_env()

    restart = threading.Event()
    signal.signal(signal.SIGHUP, lambda *_: restart.set())
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())

    plugins: list[VGPUDevicePlugin] = []
    registrar = None
    crashes = CrashBudget()
    kubelet_sock = os.path.join(cfg.socket_dir, "kubelet.sock")
    while not stop.is_set():
        if not plugins:
            try:
                plugins = build_plugins(cfg, backend, client)
                for p in plugins:
                    p.start()
                registrar = Registrar(client, cfg.node_name, lambda: [d for p in plugins for d in p.devices], cfg,
                                      get_health=lambda: {u: h for p in plugins for u, h in p.health.items()})
                registrar.start()
                sock_id = socket_id(kubelet_sock)
            except Exception as e:
                log.error("could not start plugin: %s; retrying in 30s", e)
                for p in plugins:
                    p.stop()
                plugins = []
                if not crashes.note():
                    log.critical("crash budget exhausted")
                    return 1
                stop.wait(30.0)
                continue
        stop.wait(1.0)
        cur = socket_id(kubelet_sock)
        if restart.is_set() or cur != sock_id:
            log.info("kubelet restarted or SIGHUP: restarting plugin")
            restart.clear()
            registrar.stop()
            for p in plugins:
                p.stop()
            plugins = []
    if plugins:
        registrar.stop()
        for p in plugins:
            p.stop()
    return 0


class CrashBudget:
    """More than MAX_RESTARTS_PER_HOUR failed starts within an hour is fatal
    (reference plugin/server.go:171-199)."""

    def __init__(self):
        self._t: list[float] = []

    def note(self) -> bool:
        from .server import MAX_RESTARTS_PER_HOUR
        now = time.time()
        self._t = [t for t in self._t if now - t < 3600] + [now]
        return len(self._t) <= MAX_RESTARTS_PER_HOUR


def build_plugins(cfg: DevicePluginConfig, backend, client) -> list[VGPUDevicePlugin]:
    """One device-plugin server per extended resource of the node's partition
    strategy (vgpu/deviceplugin/partitions.py): amd.com/gpu, and with `mixed`
    amd.com/gpu-dpx / -qpx / -cpx, each on its own socket.  Several servers
    share the backend's device-event stream through an EventFanout: reading
    events consumes them (amdsmi's notification queue), so each server gets
    every event on a queue of its own and keeps those of its devices."""
    from .discovery import EventFanout
    from .partitions import plan, socket_name
    groups, bad = plan(backend.devices(), cfg.partition_strategy, cfg.resource_name, cfg.partition_memory)
    groups = {res: devs for res, devs in groups.items() if devs}
    fan = EventFanout(backend) if len(groups) > 1 else None
    out = []
    for res, devs in sorted(groups.items()):
        out.append(VGPUDevicePlugin(cfg, fan.view() if fan else backend, client, cfg.node_name,
                                    socket_name=socket_name(res, cfg.resource_name),
                                    devices=devs, resource_name=res, unhealthy=bad))
    if not out:
        raise RuntimeError(f"no device to advertise under partition strategy {cfg.partition_strategy}")
    return out


if __name__ == "__main__":
    sys.exit(main())
