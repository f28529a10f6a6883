"""Node-level allocation lock in a node annotation.

Reference: pkg/util/nodelock/nodelock.go:14-15 (key `4pd.io/mutex.lock`,
5-minute expiry), :18-47 (set with optimistic Update, 5 retries × 100 ms),
:49-79 (release), :81-104 (LockNode: refuse if held and not expired, break an
expired lock).  Scheduler Bind takes it; the device plugin releases it after
Allocate (pkg/device/devices.go:54-91).

Difference: the reference logs and ignores a failed LockNode in Bind
(scheduler.go:324-327); our Bind fails the binding instead.
"""
from __future__ import annotations

import datetime as dt
import time

from vgpu.api.resources import NODE_LOCK, NODE_LOCK_EXPIRE_S

from .client import ApiError, KubeClient

RETRIES = 5
RETRY_SLEEP_S = 0.1


class NodeLockError(Exception):
    pass


def _now() -> dt.datetime:
    return dt.datetime.now(dt.timezone.utc).replace(microsecond=0)


def _fmt(t: dt.datetime) -> str:
    return t.strftime("%Y-%m-%dT%H:%M:%SZ")


def _parse(s: str) -> dt.datetime | None:
    try:
        return dt.datetime.strptime(s, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=dt.timezone.utc)
    except ValueError:
        try:
            return dt.datetime.fromisoformat(s.replace("Z", "+00:00"))
        except ValueError:
            return None


def _set(client: KubeClient, node_name: str, value: str | None) -> None:
    last = None
    for _ in range(RETRIES):
        node = client.get_node(node_name)
        annos = node.setdefault("metadata", {}).setdefault("annotations", {})
        if value is None:
            if NODE_LOCK not in annos:
                return
            annos.pop(NODE_LOCK)
        else:
            annos[NODE_LOCK] = value
        try:
            client.update_node(node)  # resourceVersion → optimistic concurrency
            return
        except ApiError as e:
            last = e
            if e.status != 409:
                raise
            time.sleep(RETRY_SLEEP_S)
    raise NodeLockError(f"could not update lock on {node_name}: {last}")


def lock_node(client: KubeClient, node_name: str, now: dt.datetime | None = None) -> None:
    """Check-and-set in one optimistic Update: a concurrent locker makes our
    Update fail with 409 and we re-read (and then see its lock)."""
    now = now or _now()
    last = None
    for _ in range(RETRIES):
        node = client.get_node(node_name)
        annos = node.setdefault("metadata", {}).setdefault("annotations", {})
        held = annos.get(NODE_LOCK)
        if held:
            t = _parse(held)
            if t is not None and now < t + dt.timedelta(seconds=NODE_LOCK_EXPIRE_S):
                raise NodeLockError(f"node {node_name} has been locked within {NODE_LOCK_EXPIRE_S}s")
            # expired (or unparsable): overwrite it
        annos[NODE_LOCK] = _fmt(now)
        try:
            client.update_node(node)
            return
        except ApiError as e:
            last = e
            if e.status != 409:
                raise
            time.sleep(RETRY_SLEEP_S)
    raise NodeLockError(f"could not lock {node_name}: {last}")


def release_node_lock(client: KubeClient, node_name: str) -> None:
    _set(client, node_name, None)
