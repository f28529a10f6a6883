"""Annotation codecs — byte-compatible with the reference's text formats so a
mixed fleet (or a Go rewrite) interoperates.

Reference: pkg/util/util.go:68-108 (node devices "id,count,mem,core,type,numa,health:"),
:110-119 (container devices "uuid,type,mem,cores:"), :121-128 (pod devices,
';'-joined per container), :130-172 (decoders).

MI355X extension: per-device fields that the 7-field node record cannot carry
(CU count, xGMI hive, PCI index, partition mode) travel in a separate JSON
annotation (`NODE_REGISTER_EXT`), so the core record stays reference-compatible.
"""
from __future__ import annotations

import json

from .resources import ContainerDevice, DeviceInfo

NODE_REGISTER_EXT = "4pd.io/node-amd-register-ext"


class CodecError(ValueError):
    pass


def _bool(s: str) -> bool:
    # Go strconv.ParseBool accepts 1,t,T,TRUE,true,True,0,f,F,FALSE,false,False
    if s in ("1", "t", "T", "TRUE", "true", "True"):
        return True
    if s in ("0", "f", "F", "FALSE", "false", "False"):
        return False
    return False


def _atoi(s: str) -> int:
    try:
        return int(s)
    except ValueError:
        return 0


def encode_node_devices(devs: list[DeviceInfo]) -> str:
    return "".join(f"{d.id},{d.count},{d.devmem},{d.devcore},{d.type},{d.numa},"
                   f"{'true' if d.health else 'false'}:" for d in devs)


def decode_node_devices(s: str) -> list[DeviceInfo]:
    if ":" not in s:
        raise CodecError("node annotations not decode successfully")
    out = []
    for val in s.split(":"):
        if "," not in val:
            continue
        items = val.split(",")
        if len(items) != 7:
            raise CodecError("node annotations not decode successfully")
        out.append(DeviceInfo(id=items[0], count=_atoi(items[1]), devmem=_atoi(items[2]),
                              devcore=_atoi(items[3]), type=items[4], numa=_atoi(items[5]),
                              health=_bool(items[6])))
    return out


def encode_node_devices_ext(devs: list[DeviceInfo]) -> str:
    def ext(d: DeviceInfo) -> dict:
        e = {"cus": d.cus, "hive": d.xgmi_hive, "index": d.index}
        if d.resource != DeviceInfo.resource:  # a partition under its own resource (mixed strategy)
            e["res"] = d.resource
        return e
    return json.dumps({d.id: ext(d) for d in devs}, sort_keys=True, separators=(",", ":"))


def apply_node_devices_ext(devs: list[DeviceInfo], s: str | None) -> list[DeviceInfo]:
    if not s:
        return devs
    try:
        ext = json.loads(s)
    except ValueError:
        return devs
    for d in devs:
        e = ext.get(d.id)
        if e:
            d.cus = int(e.get("cus", d.cus))
            d.xgmi_hive = str(e.get("hive", d.xgmi_hive))
            d.index = int(e.get("index", d.index))
            d.resource = str(e.get("res", d.resource))
    return devs


def encode_container_devices(cd: list[ContainerDevice]) -> str:
    return "".join(f"{d.uuid},{d.type},{d.usedmem},{d.usedcores}:" for d in cd)


def encode_pod_devices(pd: list[list[ContainerDevice]]) -> str:
    return ";".join(encode_container_devices(cd) for cd in pd)


def decode_container_devices(s: str) -> list[ContainerDevice]:
    if not s:
        return []
    out = []
    for val in s.split(":"):
        if "," not in val:
            continue
        t = val.split(",")
        if len(t) < 4:
            raise CodecError("pod annotation format error; information missing, "
                             "please do not use nodeName field in task")
        out.append(ContainerDevice(uuid=t[0], type=t[1], usedmem=_atoi(t[2]), usedcores=_atoi(t[3])))
    return out


def decode_pod_devices(s: str) -> list[list[ContainerDevice]]:
    if not s:
        return []
    out = []
    for part in s.split(";"):
        try:
            out.append(decode_container_devices(part))
        except CodecError:
            return []  # reference returns an empty PodDevices on any container error
    return out
