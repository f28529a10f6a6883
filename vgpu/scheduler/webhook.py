"""Mutating admission webhook (AdmissionReview v1).

Reference: pkg/scheduler/webhook.go:52-88 — skip privileged containers, let
every vendor mutate each container (the AMD policy injects the task-priority
env from the `priority` limit), and when any vendor resource is present set
`spec.schedulerName` so the pod goes through our scheduler; answer with a JSON
patch.  Pods labelled `4pd.io/webhook: ignore` are passed through (the chart's
objectSelector normally filters them before they reach us).
"""
from __future__ import annotations

import base64
import copy
import json

from vgpu import config
from vgpu.api.resources import ANN_WEBHOOK_IGNORE_LABEL
from vgpu.device.base import get_devices
from vgpu.k8s.objects import is_privileged, labels


def _escape(k) -> str:
    return str(k).replace("~", "~0").replace("/", "~1")


def json_patch(old, new, path: str = "") -> list[dict]:
    """Minimal RFC 6902 diff (dict keys recursively; lists element-wise when the
    length is unchanged, else replaced wholesale)."""
    if type(old) is not type(new):
        return [{"op": "replace", "path": path or "/", "value": new}]
    if isinstance(old, dict):
        ops = []
        for k in old:
            if k not in new:
                ops.append({"op": "remove", "path": f"{path}/{_escape(k)}"})
        for k, v in new.items():
            p = f"{path}/{_escape(k)}"
            if k not in old:
                ops.append({"op": "add", "path": p, "value": v})
            else:
                ops.extend(json_patch(old[k], v, p))
        return ops
    if isinstance(old, list):
        if len(old) != len(new):
            return [{"op": "replace", "path": path, "value": new}]
        ops = []
        for i, (a, b) in enumerate(zip(old, new)):
            ops.extend(json_patch(a, b, f"{path}/{i}"))
        return ops
    return [] if old == new else [{"op": "replace", "path": path, "value": new}]


def handle_admission(review: dict, scheduler_name: str | None = None) -> dict:
    req = review.get("request") or {}
    uid = req.get("uid", "")
    api_version = review.get("apiVersion", "admission.k8s.io/v1")

    def resp(allowed: bool, patch: list | None = None, message: str = "", code: int = 200) -> dict:
        r = {"uid": uid, "allowed": allowed}
        if message:
            r["status"] = {"message": message, "code": code}
        if patch:
            r["patchType"] = "JSONPatch"
            r["patch"] = base64.b64encode(json.dumps(patch).encode()).decode()
        return {"apiVersion": api_version, "kind": "AdmissionReview", "response": r}

    pod = req.get("object")
    if not isinstance(pod, dict):
        return resp(False, message="could not decode pod", code=400)
    containers = (pod.get("spec") or {}).get("containers") or []
    if not containers:
        return resp(False, message="pod has no containers", code=403)
    if labels(pod).get(ANN_WEBHOOK_IGNORE_LABEL) == "ignore":
        return resp(True, message="webhook ignored by label")
    new = copy.deepcopy(pod)
    has = False
    for ctr in new["spec"]["containers"]:
        if is_privileged(ctr):
            continue
        for dev in get_devices().values():
            has = dev.mutate_admission(ctr) or has
    if not has:
        return resp(True, message="no resource found")
    name = config.SCHEDULER.scheduler_name if scheduler_name is None else scheduler_name
    if name:
        new["spec"]["schedulerName"] = name
    return resp(True, json_patch(pod, new))
