"""Helpers over plain-JSON Kubernetes objects (dicts as returned by the API
server): resource quantities, container limits, pod phase.

Reference: k8s.io/apimachinery resource.Quantity.AsInt64 (used by
pkg/device/nvidia/device.go:114-175) and pkg/k8sutil/pod.go:42-48
(IsPodInTerminatedState).
"""
from __future__ import annotations

import re
from decimal import Decimal

_SUFFIX = {
    "": 1, "k": 10**3, "M": 10**6, "G": 10**9, "T": 10**12, "P": 10**15, "E": 10**18,
    "Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60,
}
_Q = re.compile(r"^([+-]?[0-9.]+(?:[eE][+-]?[0-9]+)?)(Ki|Mi|Gi|Ti|Pi|Ei|m|k|M|G|T|P|E)?$")


def parse_quantity(v) -> int | None:
    """Kubernetes quantity → integer value (None when not an integer, like AsInt64)."""
    if v is None:
        return None
    if isinstance(v, (int, float)):
        return int(v) if float(v).is_integer() else None
    s = str(v).strip()
    m = _Q.match(s)
    if not m:
        return None
    num, suf = m.group(1), m.group(2) or ""
    if suf == "m":
        val = Decimal(num) / 1000
    else:
        val = Decimal(num) * _SUFFIX[suf]
    if val != val.to_integral_value():
        return None
    return int(val)


def containers(pod: dict) -> list[dict]:
    return pod.get("spec", {}).get("containers", []) or []


def limit_or_request(ctr: dict, name: str):
    res = ctr.get("resources", {}) or {}
    lim = res.get("limits", {}) or {}
    if name in lim:
        return lim[name]
    req = res.get("requests", {}) or {}
    return req.get(name)


def annotations(obj: dict) -> dict:
    return obj.get("metadata", {}).get("annotations", {}) or {}


def labels(obj: dict) -> dict:
    return obj.get("metadata", {}).get("labels", {}) or {}


def name(obj: dict) -> str:
    return obj.get("metadata", {}).get("name", "")


def namespace(obj: dict) -> str:
    return obj.get("metadata", {}).get("namespace", "default")


def uid(obj: dict) -> str:
    return obj.get("metadata", {}).get("uid", "")


def is_terminated(pod: dict) -> bool:
    return pod.get("status", {}).get("phase") in ("Failed", "Succeeded")


def is_privileged(ctr: dict) -> bool:
    sc = ctr.get("securityContext") or {}
    return bool(sc.get("privileged"))
