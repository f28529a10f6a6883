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

    plugin = None
    registrar = None
    kubelet_sock = os.path.join(cfg.socket_dir, "kubelet.sock")
    while not stop.is_set():
        if plugin is None:
            try:
                plugin = VGPUDevicePlugin(cfg, backend, client, cfg.node_name)
                plugin.start()
                registrar = Registrar(client, cfg.node_name, lambda: plugin.devices, cfg,
                                      get_health=lambda: dict(plugin.health))
                registrar.start()
                sock_id = socket_id(kubelet_sock)
            except Exception as e:
                log.error("could not start plugin: %s; retrying in 30s", e)
                if plugin is not None and not plugin.note_crash():
                    log.critical("crash budget exhausted")
                    return 1
                plugin = None
                stop.wait(30.0)
                continue
        stop.wait(1.0)
        cur = socket_id(kubelet_sock)
        if restart.is_set() or cur != sock_id:
            log.info("kubelet restarted or SIGHUP: restarting plugin")
            restart.clear()
            registrar.stop()
            plugin.stop()
            plugin = None
    if plugin is not None:
        registrar.stop()
        plugin.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
