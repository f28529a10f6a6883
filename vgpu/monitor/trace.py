"""Reader for the enforcement library's event trace (VGPU_TRACE=<dir>).

Layout: native/include/vgpu/trace.h (mirrored here with ctypes; sizes are
checked against the header's own header_size / event_size fields).  SURVEY.md
§5 "Tracing / profiling" — the reference has debug logs only.

    python -m vgpu.monitor.trace <dir-or-file> [--events]
"""
from __future__ import annotations

import argparse
import collections
import ctypes
import glob
import json
import mmap
import os

MAGIC = 0x56545243
TYPES = {1: "alloc", 2: "free", 3: "oom", 4: "launch", 5: "throttle", 6: "suspend",
         7: "priority_block", 8: "queue", 9: "gpu_time", 10: "migrate", 11: "copy"}


class Event(ctypes.Structure):
    _fields_ = [("ts_ns", ctypes.c_uint64), ("type", ctypes.c_uint32), ("dev", ctypes.c_int32),
                ("a", ctypes.c_uint64), ("b", ctypes.c_uint64)]


class Header(ctypes.Structure):
    _fields_ = [("magic", ctypes.c_uint32), ("version", ctypes.c_uint32),
                ("header_size", ctypes.c_uint32), ("event_size", ctypes.c_uint32),
                ("capacity", ctypes.c_uint64), ("head", ctypes.c_uint64),
                ("pid", ctypes.c_int32), ("host_pid", ctypes.c_int32),
                ("start_ns", ctypes.c_uint64), ("reserved", ctypes.c_uint64 * 2)]


assert ctypes.sizeof(Event) == 32 and ctypes.sizeof(Header) == 64


def read(path: str) -> tuple[Header, list[dict]]:
    """Events of one trace file in claim order (oldest surviving first)."""
    with open(path, "rb") as f:
        buf = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    try:
        h = Header.from_buffer_copy(buf, 0)
        if h.magic != MAGIC or h.header_size != ctypes.sizeof(Header) or h.event_size != ctypes.sizeof(Event):
            raise ValueError(f"{path}: not a vgpu trace (or layout mismatch)")
        n = min(h.head, h.capacity)
        first = h.head - n
        out = []
        for k in range(first, h.head):
            e = Event.from_buffer_copy(buf, ctypes.sizeof(Header) + (k % h.capacity) * ctypes.sizeof(Event))
            if e.ts_ns == 0:  # claimed but not yet published
                continue
            out.append({"t_ns": e.ts_ns - h.start_ns, "type": TYPES.get(e.type, str(e.type)),
                        "dev": e.dev, "a": e.a, "b": e.b})
        return h, out
    finally:
        buf.close()


def summarize(events: list[dict]) -> dict:
    cnt = collections.Counter(e["type"] for e in events)
    s = {"events": dict(cnt)}
    s["alloc_bytes"] = sum(e["a"] for e in events if e["type"] == "alloc")
    s["free_bytes"] = sum(e["a"] for e in events if e["type"] == "free")
    s["launch_workgroups"] = sum(e["a"] for e in events if e["type"] == "launch")
    s["exempt_launches"] = sum(1 for e in events if e["type"] == "launch" and e["b"])
    s["throttle_wait_ms"] = sum(e["a"] for e in events if e["type"] == "throttle") / 1e6
    s["blocked_ms"] = sum(e["a"] for e in events if e["type"] in ("suspend", "priority_block")) / 1e6
    mig = [e for e in events if e["type"] == "migrate"]
    if mig:  # b = (ns << 1) | to_hbm
        up = [e for e in mig if e["b"] & 1]
        down = [e for e in mig if not e["b"] & 1]
        s["migrate_to_hbm_bytes"] = sum(e["a"] for e in up)
        s["migrate_to_host_bytes"] = sum(e["a"] for e in down)
        busy = sum(e["b"] >> 1 for e in mig)
        s["migrate_busy_ms"] = busy / 1e6
        s["migrate_GBps"] = round(sum(e["a"] for e in mig) / busy, 2) if busy else None
        s["migrate_window_ms"] = [mig[0]["t_ns"] / 1e6, (mig[-1]["t_ns"]) / 1e6]
    return s


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--events", action="store_true", help="print every event")
    a = ap.parse_args(argv)
    files = sorted(glob.glob(os.path.join(a.path, "vgpu-trace-*.bin"))) if os.path.isdir(a.path) else [a.path]
    for f in files:
        h, ev = read(f)
        print(json.dumps({"file": f, "pid": h.pid, "host_pid": h.host_pid, "claimed": h.head,
                          **summarize(ev)}))
        if a.events:
            for e in ev:
                print(json.dumps(e))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
