"""Device discovery for the node agents: ctypes over libvgpu_smi.so (amdsmi or
KFD sysfs), plus a static backend for tests / fixtures.

Reference equivalents: NVML enumeration in the NVIDIA plugin
(pkg/device-plugin/nvidiadevice/nvinternal/rm/nvml_devices.go:48-168,
plugin/register.go:55-100 incl. NUMA from `nvidia-smi topo -m`), Hygon's
`hy-smi` scraping + libdrm_amdgpu cgo (pkg/device-plugin/hygon/dcu/server.go:50-175,
amdgpu/amdgpu.go) and hwloc NUMA lookup (hygon/dcu/hwloc/hwloc.go:69-97).
"""
from __future__ import annotations

import ctypes
import json
import threading
from dataclasses import asdict, dataclass, field

from vgpu.native import LIB_DIR, NativeMissing

STR = 64


class _SmiDevice(ctypes.Structure):
    _fields_ = [("uuid", ctypes.c_char * STR), ("bdf", ctypes.c_char * STR), ("name", ctypes.c_char * STR),
                ("compute_partition", ctypes.c_char * 16), ("memory_partition", ctypes.c_char * 16),
                ("vram_total", ctypes.c_uint64), ("vram_used", ctypes.c_uint64),
                ("xgmi_hive", ctypes.c_uint64), ("device_id", ctypes.c_uint64),
                ("vendor_id", ctypes.c_uint32), ("cus", ctypes.c_uint32), ("num_xcc", ctypes.c_uint32),
                ("numa_node", ctypes.c_int32), ("render_minor", ctypes.c_uint32), ("card", ctypes.c_uint32),
                ("kfd_gpu_id", ctypes.c_uint32), ("index", ctypes.c_uint32), ("health", ctypes.c_uint32),
                ("gfx_activity", ctypes.c_uint32), ("umc_activity", ctypes.c_uint32),
                ("partition_id", ctypes.c_uint32), ("reserved", ctypes.c_uint32 * 6)]


class _SmiProc(ctypes.Structure):
    _fields_ = [("pid", ctypes.c_uint32), ("cu_occupancy", ctypes.c_uint32),
                ("vram_bytes", ctypes.c_uint64), ("gfx_ns", ctypes.c_uint64)]


class _SmiTelemetry(ctypes.Structure):
    _fields_ = [("ecc_correctable", ctypes.c_uint64), ("ecc_uncorrectable", ctypes.c_uint64),
                ("ecc_deferred", ctypes.c_uint64), ("xgmi_read_kb", ctypes.c_uint64),
                ("xgmi_write_kb", ctypes.c_uint64), ("power_w", ctypes.c_uint32),
                ("temp_edge_c", ctypes.c_int32), ("temp_hotspot_c", ctypes.c_int32),
                ("temp_mem_c", ctypes.c_int32), ("valid", ctypes.c_uint32), ("reserved", ctypes.c_uint32 * 7)]


TELEM_ECC, TELEM_POWER, TELEM_TEMP, TELEM_XGMI = 1, 2, 4, 8


@dataclass
class Telemetry:
    """Health / host counters of one device (native vgpu_smi_telemetry)."""
    ecc_correctable: int = 0
    ecc_uncorrectable: int = 0
    ecc_deferred: int = 0
    xgmi_read_bytes: int = 0
    xgmi_write_bytes: int = 0
    power_w: int = 0
    temp_edge_c: int = 0
    temp_hotspot_c: int = 0
    temp_mem_c: int = 0
    valid: int = 0


class _SmiEvent(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("type", ctypes.c_int32), ("message", ctypes.c_char * (STR * 2))]


# AMDSMI_EVT_NOTIF_* values we act on
EVT_VMFAULT, EVT_THERMAL, EVT_PRE_RESET, EVT_POST_RESET = 1, 2, 3, 4
LINK_UNKNOWN, LINK_PCIE, LINK_XGMI = 0, 1, 2


@dataclass
class Device:
    uuid: str
    index: int
    bdf: str = ""
    name: str = "AMD Instinct MI355X"
    vram_total: int = 288 << 30
    vram_used: int = 0
    cus: int = 256
    num_xcc: int = 8
    numa: int = 0
    render_minor: int = 128
    card: int = 0
    kfd_gpu_id: int = 0
    xgmi_hive: int = 0
    compute_partition: str = "SPX"
    memory_partition: str = "NPS1"
    health: bool = True
    gfx_activity: int = 0
    umc_activity: int = 0
    vendor_id: int = 0x1002
    partition_id: int = 0          # compute partition of its physical GPU (0 in SPX)
    resource: str = "amd.com/gpu"  # extended resource it is advertised under (partitions.py)
    memory_shared_by: int = 1      # partitions sharing its NPS memory domain (partitions.py)

    @property
    def model(self) -> str:
        """Short model for the device type string, e.g. 'MI355X'."""
        for tok in self.name.replace("(", " ").split():
            if tok.upper().startswith("MI") and any(c.isdigit() for c in tok):
                return tok.upper()
        return self.name.split()[-1] if self.name else "GPU"

    @property
    def type(self) -> str:
        t = f"AMD-{self.model}"
        if self.compute_partition and self.compute_partition.upper() != "SPX":
            t += f"-{self.compute_partition.upper()}"
        return t


@dataclass
class Proc:
    pid: int
    vram_bytes: int
    cu_occupancy: int = 0
    gfx_ns: int = 0


# XCDs per compute partition of an 8-XCD part (MI355X / MI300X), for backends
# that report the partition but not its XCD count (amdsmi).
XCC_PER_PARTITION = {"SPX": 8, "DPX": 4, "QPX": 2, "CPX": 1}


def xcc_of_partition(mode: str) -> int:
    return XCC_PER_PARTITION.get((mode or "SPX").upper(), 8)


class Backend:
    name = "base"

    def devices(self) -> list[Device]:
        raise NotImplementedError

    def link(self, a: int, b: int) -> tuple[int, int]:
        return 0, LINK_UNKNOWN

    def processes(self, index: int) -> list[Proc]:
        return []

    def events(self, timeout_ms: int = 1000) -> list[tuple[int, int, str]]:
        return []

    def telemetry(self, index: int) -> Telemetry | None:
        return None


class SmiBackend(Backend):
    def __init__(self, mode: str = "auto"):
        p = LIB_DIR / "libvgpu_smi.so"
        if not p.exists():
            raise NativeMissing(f"{p} not built")
        lib = ctypes.CDLL(str(p))
        lib.vgpu_smi_open.argtypes = [ctypes.c_char_p]
        lib.vgpu_smi_get.argtypes = [ctypes.c_int, ctypes.POINTER(_SmiDevice)]
        lib.vgpu_smi_link.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_int32)]
        lib.vgpu_smi_processes.argtypes = [ctypes.c_int, ctypes.POINTER(_SmiProc), ctypes.c_int]
        lib.vgpu_smi_events.argtypes = [ctypes.POINTER(_SmiEvent), ctypes.c_int, ctypes.c_int]
        lib.vgpu_smi_backend.restype = ctypes.c_char_p
        lib.vgpu_smi_telemetry.argtypes = [ctypes.c_int, ctypes.POINTER(_SmiTelemetry)]
        self.lib = lib
        n = lib.vgpu_smi_open(mode.encode())
        if n < 0:
            raise RuntimeError(f"vgpu_smi_open({mode}) failed")
        self.count = n
        self.name = lib.vgpu_smi_backend().decode()

    def devices(self) -> list[Device]:
        out = []
        for i in range(self.lib.vgpu_smi_count()):
            d = _SmiDevice()
            if self.lib.vgpu_smi_get(i, ctypes.byref(d)) != 0:
                continue
            out.append(Device(
                uuid=d.uuid.decode() or f"GPU-{i}", index=i, bdf=d.bdf.decode(), name=d.name.decode(),
                vram_total=d.vram_total, vram_used=d.vram_used, cus=d.cus or 256,
                num_xcc=d.num_xcc or xcc_of_partition(d.compute_partition.decode()), numa=max(d.numa_node, 0), render_minor=d.render_minor,
                card=d.card, kfd_gpu_id=d.kfd_gpu_id, xgmi_hive=d.xgmi_hive,
                compute_partition=d.compute_partition.decode() or "SPX",
                memory_partition=d.memory_partition.decode() or "NPS1", health=bool(d.health),
                gfx_activity=d.gfx_activity, umc_activity=d.umc_activity, vendor_id=d.vendor_id,
                partition_id=d.partition_id))
        return out

    def link(self, a: int, b: int) -> tuple[int, int]:
        hops, t = ctypes.c_uint64(0), ctypes.c_int32(0)
        self.lib.vgpu_smi_link(a, b, ctypes.byref(hops), ctypes.byref(t))
        return hops.value, t.value

    def processes(self, index: int) -> list[Proc]:
        buf = (_SmiProc * 256)()
        n = self.lib.vgpu_smi_processes(index, buf, 256)
        return [Proc(buf[i].pid, buf[i].vram_bytes, buf[i].cu_occupancy, buf[i].gfx_ns)
                for i in range(max(n, 0))]

    def telemetry(self, index: int) -> Telemetry | None:
        t = _SmiTelemetry()
        if self.lib.vgpu_smi_telemetry(index, ctypes.byref(t)) != 0:
            return None
        return Telemetry(t.ecc_correctable, t.ecc_uncorrectable, t.ecc_deferred, t.xgmi_read_kb * 1024,
                         t.xgmi_write_kb * 1024, t.power_w, t.temp_edge_c, t.temp_hotspot_c, t.temp_mem_c,
                         t.valid)

    def events(self, timeout_ms: int = 1000) -> list[tuple[int, int, str]]:
        buf = (_SmiEvent * 32)()
        n = self.lib.vgpu_smi_events(buf, 32, timeout_ms)
        return [(buf[i].device, buf[i].type, buf[i].message.decode(errors="replace")) for i in range(n)]


class EventFanout:
    """One consumer of `backend.events()` for several device-plugin servers
    (mixed partition strategy).  The backend's events are consumed
    by reading them, so per-server polling lost a reset to whichever server
    read it first and dropped it as not its device.  Each server polls through
    a view with its own queue; a poll of an empty queue reads the backend once
    (one reader at a time) and appends what it got to every queue."""

    def __init__(self, backend):
        self.backend = backend
        self._lock = threading.Lock()
        self._queues: list[list[tuple[int, int, str]]] = []

    def view(self) -> "_FanoutView":
        q: list[tuple[int, int, str]] = []
        with self._lock:
            self._queues.append(q)
        return _FanoutView(self, q)

    def _events(self, q: list, timeout_ms: int) -> list[tuple[int, int, str]]:
        with self._lock:
            if not q:
                ev = self.backend.events(timeout_ms)
                for other in self._queues:
                    other.extend(ev)
            out = list(q)
            q.clear()
            return out


class _FanoutView:
    """The backend as one server sees it: everything but events() passes through."""

    def __init__(self, fan: EventFanout, q: list):
        self._fan, self._q = fan, q

    def events(self, timeout_ms: int = 1000) -> list[tuple[int, int, str]]:
        return self._fan._events(self._q, timeout_ms)

    def __getattr__(self, name):
        return getattr(self._fan.backend, name)


class StaticBackend(Backend):
    """Fixed device list (tests, dry runs, `--backend fake:<file.json>`)."""
    name = "static"

    def __init__(self, devices: list[Device], xgmi: bool = True, procs: dict | None = None):
        self._devs = devices
        self.xgmi = xgmi
        self._procs = procs or {}
        self.pending_events: list[tuple[int, int, str]] = []
        self.telemetry_by_index: dict[int, Telemetry] = {}

    def devices(self) -> list[Device]:
        return [Device(**asdict(d)) for d in self._devs]

    def link(self, a: int, b: int) -> tuple[int, int]:
        da, db = self._devs[a], self._devs[b]
        if self.xgmi and da.xgmi_hive == db.xgmi_hive:
            return 1, LINK_XGMI
        return 2, LINK_PCIE

    def processes(self, index: int) -> list[Proc]:
        return list(self._procs.get(index, []))

    def events(self, timeout_ms: int = 1000) -> list[tuple[int, int, str]]:
        ev, self.pending_events = self.pending_events, []
        return ev

    def telemetry(self, index: int) -> Telemetry | None:
        return self.telemetry_by_index.get(index)


def mi355x_node(n: int = 8, hive: int = 0x1111) -> list[Device]:
    """A synthetic 8 × MI355X node (one xGMI hive, two NUMA nodes)."""
    return [Device(uuid=f"GPU-{hive:x}-{i:02d}", index=i, bdf=f"0000:{0x05 + 0x10 * i:02x}:00.0",
                   numa=i // 4, render_minor=128 + i, card=i, kfd_gpu_id=1000 + i, xgmi_hive=hive)
            for i in range(n)]


def load_backend(spec: str = "auto") -> Backend:
    if spec.startswith("fake:"):
        data = json.load(open(spec[5:]))
        return StaticBackend([Device(**d) for d in data["devices"]], xgmi=data.get("xgmi", True))
    if spec == "synthetic":
        return StaticBackend(mi355x_node())
    return SmiBackend(spec)
