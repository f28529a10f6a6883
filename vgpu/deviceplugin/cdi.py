"""Container Device Interface (CDI) spec for AMD GPUs (optional delivery path
instead of AllocateResponse.devices).

Reference: pkg/device-plugin/nvidiadevice/nvinternal/cdi/cdi.go:32-173
(nvidia-container-toolkit generated specs, used only with
device-list-strategy=cdi-annotations).  AMD needs no hook binaries: a device is
/dev/kfd plus its /dev/dri render and card nodes.
"""
from __future__ import annotations

import json
import os

from .discovery import Device

CDI_KIND = "amd.com/gpu"
CDI_VERSION = "0.6.0"


def spec(devs: list[Device]) -> dict:
    return {
        "cdiVersion": CDI_VERSION,
        "kind": CDI_KIND,
        "containerEdits": {"deviceNodes": [{"path": "/dev/kfd", "permissions": "rw"}]},
        "devices": [{
            "name": d.uuid,
            "containerEdits": {"deviceNodes": [
                {"path": f"/dev/dri/renderD{d.render_minor}", "permissions": "rw"},
                {"path": f"/dev/dri/card{d.card}", "permissions": "rw"}]},
        } for d in devs] + [{"name": "all", "containerEdits": {"deviceNodes": [
            {"path": f"/dev/dri/renderD{d.render_minor}", "permissions": "rw"} for d in devs]}}],
    }


def device_names(uuids: list[str]) -> list[str]:
    return [f"{CDI_KIND}={u}" for u in uuids]


def write_spec(devs: list[Device], directory: str = "/var/run/cdi") -> str:
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, "amd.com-gpu.json")
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(spec(devs), f, indent=2)
    os.replace(tmp, path)
    return path
