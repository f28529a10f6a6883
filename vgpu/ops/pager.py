"""Explicit HBM ↔ pinned-host pager for virtual device memory.

The reference's "virtual device memory" (deviceMemoryScaling > 1 →
CUDA_OVERSUBSCRIBE, cuMemAllocManaged in libvgpu.so; SURVEY.md §5 row
"Long-context") relies on CUDA unified-memory page faults.  MI355X pools here run
with XNACK off, so there is no demand paging: the enforcement library backs
allocations beyond physical HBM with pinned, device-mapped host memory
(zero-copy, correct but PCIe-bound), and this module is the performance path on
top: named chunks (layer weights, KV-cache blocks) live in pinned host memory
and are staged into a bounded HBM working set on a side HIP stream, ahead of
use, with LRU eviction and write-back of dirty chunks.

* `prefetch(names)` issues host→HBM copies on the pager stream (SDMA via
  hipMemcpyAsync) and records an event per chunk;
* `get(name)` makes the compute stream wait on that event only (no device-wide
  sync), then returns the HBM tensor;
* scattered page sets are gathered with the K2 kernel straight from pinned host
  memory (`gather_pages`);
* bytes moved are charged to this process's slot in the shared region
  (swap_in / swap_out), so the node monitor exports them.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict
from dataclasses import dataclass

import torch


def _shim_swap_hook():
    try:
        lib = ctypes.CDLL(None)
        f = lib.vgpu_self_add_swap
        f.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        return f
    except (AttributeError, OSError):
        return None


@dataclass
class PagerStats:
    hits: int = 0
    misses: int = 0
    swap_in_bytes: int = 0
    swap_out_bytes: int = 0
    evictions: int = 0


class HostPager:
    def __init__(self, budget_bytes: int, device: torch.device | str = "cuda", *,
                 stream_priority: int = -1):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.budget = int(budget_bytes)
        self.host: dict[str, torch.Tensor] = {}
        self.resident: OrderedDict[str, torch.Tensor] = OrderedDict()  # LRU → MRU
        self.ready: dict[str, object] = {}
        self.dirty: set[str] = set()
        self.pinned: set[str] = set()
        self.used = 0
        self.stats = PagerStats()
        self._free: dict[tuple, list[torch.Tensor]] = {}
        self.stream = torch.cuda.Stream(self.device, priority=stream_priority) if self.cuda else None
        self._hook = _shim_swap_hook() if self.cuda else None
        self._dev_index = self.device.index or 0 if self.cuda else 0

    # ---- registration -----------------------------------------------------------------
    def register(self, name: str, t: torch.Tensor) -> None:
        """Take ownership of a chunk; its home is pinned host memory."""
        t = t.detach()
        if self.cuda:
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h.copy_(t)
        else:
            h = t.to("cpu")
        self.host[name] = h

    def nbytes(self, name: str) -> int:
        h = self.host[name]
        return h.numel() * h.element_size()

    # ---- residency ----------------------------------------------------------------------
    def _account(self, inb: int, outb: int) -> None:
        self.stats.swap_in_bytes += inb
        self.stats.swap_out_bytes += outb
        if self._hook is not None:
            self._hook(self._dev_index, inb, outb)

    def _evict_one(self) -> bool:
        for name in self.resident:
            if name in self.pinned:
                continue
            buf = self.resident.pop(name)
            ev = self.ready.pop(name, None)
            if name in self.dirty:
                # write back before the buffer is reused
                if self.cuda:
                    with torch.cuda.stream(self.stream):
                        self.stream.wait_stream(torch.cuda.current_stream(self.device))
                        self.host[name].copy_(buf, non_blocking=True)
                else:
                    self.host[name].copy_(buf)
                self.dirty.discard(name)
                self._account(0, self.nbytes(name))
            key = (tuple(buf.shape), buf.dtype)
            if self.cuda:
                # the buffer may still be read by queued compute: make the pager
                # stream (which will overwrite it) wait for the compute stream
                self.stream.wait_stream(torch.cuda.current_stream(self.device))
            self._free.setdefault(key, []).append(buf)
            self.used -= buf.numel() * buf.element_size()
            self.stats.evictions += 1
            return True
        return False

    def _alloc(self, name: str) -> torch.Tensor:
        h = self.host[name]
        need = self.nbytes(name)
        if need > self.budget:
            raise MemoryError(f"chunk {name} ({need} B) exceeds the pager budget ({self.budget} B)")
        while self.used + need > self.budget:
            if not self._evict_one():
                raise MemoryError("pager budget exhausted by pinned chunks")
        key = (tuple(h.shape), h.dtype)
        lst = self._free.get(key)
        buf = lst.pop() if lst else torch.empty_like(h, device=self.device)
        self.used += need
        return buf

    def prefetch(self, names) -> None:
        for name in names:
            if name in self.resident or name not in self.host:
                continue
            buf = self._alloc(name)
            if self.cuda:
                with torch.cuda.stream(self.stream):
                    buf.copy_(self.host[name], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                self.ready[name] = ev
            else:
                buf.copy_(self.host[name])
            self.resident[name] = buf
            self.stats.misses += 1
            self._account(self.nbytes(name), 0)

    def get(self, name: str, write: bool = False) -> torch.Tensor:
        if name in self.resident:
            self.stats.hits += 1
        else:
            self.prefetch([name])
        self.resident.move_to_end(name)
        ev = self.ready.pop(name, None)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
        if write:
            self.dirty.add(name)
        return self.resident[name]

    def pin(self, name: str) -> None:
        self.pinned.add(name)

    def unpin(self, name: str) -> None:
        self.pinned.discard(name)

    def flush(self) -> None:
        """Write every dirty resident chunk back to host memory."""
        for name in list(self.dirty):
            buf = self.resident[name]
            if self.cuda:
                torch.cuda.current_stream(self.device).synchronize()
            self.host[name].copy_(buf)
            self._account(0, self.nbytes(name))
        self.dirty.clear()

    # ---- scattered pages -----------------------------------------------------------------------
    def gather_pages(self, name: str, page_ids: torch.Tensor, page_bytes: int,
                     out: torch.Tensor | None = None) -> torch.Tensor:
        """Gather selected pages of a host-resident chunk into a packed HBM
        buffer with the K2 kernel reading pinned host memory directly."""
        from vgpu.ops.kernels import gather_pages
        h = self.host[name]
        n = page_ids.numel()
        if out is None:
            out = torch.empty(n * page_bytes, dtype=torch.uint8, device=self.device)
        gather_pages(out, h, page_ids.to(self.device, torch.int64), page_bytes)
        self._account(n * page_bytes, 0)
        return out
