"""Publish this node's device inventory to the scheduler through node
annotations, and answer the scheduler's handshake.

Reference: pkg/device-plugin/nvidiadevice/nvinternal/plugin/register.go:55-100
(devices: memory × scaling, Count = split count, Devcore = coresScaling × 100,
type "NVIDIA-<model>", NUMA), :102-120 (patch register + "Reported <ts>"
handshake), :122-133 (every 30 s, 5 s after an error); Hygon register.go:34-88.
Differences: NUMA / xGMI hive / CU count come from amdsmi or KFD sysfs (no
`nvidia-smi topo -m` parsing, no hard-coded Count:30 / Numa:0).
"""
from __future__ import annotations

import datetime as dt
import logging
import threading

from vgpu.api import resources as R
from vgpu.api.codec import NODE_REGISTER_EXT, encode_node_devices, encode_node_devices_ext
from vgpu.api.resources import DeviceInfo
from vgpu.config import DevicePluginConfig
from vgpu.k8s.client import KubeClient

from .discovery import Device

log = logging.getLogger("vgpu.deviceplugin.register")

HANDSHAKE_TIME_FMT = "%Y.%m.%d %H:%M:%S"


def api_devices(devs: list[Device], cfg: DevicePluginConfig, health: dict[str, bool] | None = None
                ) -> list[DeviceInfo]:
    out = []
    for d in devs:
        ok = d.health and (health or {}).get(d.uuid, True)
        out.append(DeviceInfo(id=d.uuid, count=cfg.device_split_count,
                              devmem=int((d.vram_total >> 20) * cfg.device_memory_scaling),
                              devcore=int(100 * cfg.device_cores_scaling), type=d.type,
                              numa=d.numa, health=ok, cus=d.cus,
                              xgmi_hive=f"{d.xgmi_hive:x}" if d.xgmi_hive else "", index=d.index,
                              resource=d.resource))
    return out


def register_once(client: KubeClient, node: str, devs: list[Device], cfg: DevicePluginConfig,
                  health: dict[str, bool] | None = None, now: dt.datetime | None = None) -> None:
    infos = api_devices(devs, cfg, health)
    now = now or dt.datetime.now()
    client.patch_node_annotations(node, {
        R.NODE_REGISTER: encode_node_devices(infos),
        NODE_REGISTER_EXT: encode_node_devices_ext(infos),
        R.NODE_HANDSHAKE: R.HANDSHAKE_REPORTED + now.strftime(HANDSHAKE_TIME_FMT),
    })


class Registrar:
    def __init__(self, client: KubeClient, node: str, get_devices, cfg: DevicePluginConfig,
                 get_health=None):
        self.client = client
        self.node = node
        self.get_devices = get_devices
        self.get_health = get_health or (lambda: {})
        self.cfg = cfg
        self._stop = threading.Event()

    def run(self) -> None:
        while not self._stop.is_set():
            try:
                register_once(self.client, self.node, self.get_devices(), self.cfg, self.get_health())
                wait = self.cfg.register_interval_s
            except Exception as e:
                log.error("register on %s failed: %s", self.node, e)
                wait = 5.0
            self._stop.wait(wait)

    def start(self) -> threading.Thread:
        t = threading.Thread(target=self.run, daemon=True, name="vgpu-registrar")
        t.start()
        return t

    def stop(self) -> None:
        self._stop.set()
