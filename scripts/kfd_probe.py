"""Probe what the KFD sysfs exposes to a process inside the GPU box's PID namespace.

Prints: NSpid, amdgpu scheduler parameters, this process's KFD proc entry found by
diffing /sys/class/kfd/kfd/proc around the first /dev/kfd open (the shim's
host-PID resolution, native/shim/hostpid.cpp), and cu_occupancy samples while
one-wave workgroups spin on 64 / 128 / 256 / 1024 CUs' worth of grid.
"""
from __future__ import annotations

import glob
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KFD = "/sys/class/kfd/kfd/proc"


def entries() -> set[int]:
    return {int(os.path.basename(p)) for p in glob.glob(KFD + "/*") if os.path.basename(p).isdigit()}


def read(p: str) -> str:
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError as e:
        return f"<{e.__class__.__name__}: {e.strerror}>"


def main() -> None:
    out: dict = {}
    out["nspid"] = [l for l in read("/proc/self/status").splitlines() if l.startswith(("NSpid", "Pid"))]
    out["params"] = {k: read(f"/sys/module/amdgpu/parameters/{k}")
                     for k in ("hws_max_conc_proc", "sched_policy", "mes", "cwsr_enable",
                               "hws_gws_support", "compute_multipipe", "no_system_mem_limit")}
    out["vgpulock_env"] = os.environ.get("VGPU_LOCK_DIR")
    before = entries()
    import torch
    torch.cuda.init()
    torch.empty(1, device="cuda")
    after = entries()
    new = sorted(after - before)
    out["kfd_before"] = len(before)
    out["kfd_new"] = new
    me = new[0] if len(new) == 1 else None
    out["me"] = me
    if me is None:
        print(json.dumps(out, indent=1))
        return
    d = f"{KFD}/{me}"
    out["files"] = sorted(os.listdir(d))
    for s in glob.glob(d + "/stats_*"):
        out[os.path.basename(s)] = {f: read(f"{s}/{f}") for f in os.listdir(s)}
    out["queues"] = {q: {f: read(f"{d}/queues/{q}/{f}") for f in os.listdir(f"{d}/queues/{q}")}
                     for q in os.listdir(d + "/queues")} if os.path.isdir(d + "/queues") else None
    stats = glob.glob(d + "/stats_*/cu_occupancy")
    from vgpu.ops import kernels as K
    res = {}
    for blocks in (64, 128, 256, 1024, 4096):
        samples: list[int] = []
        stop = threading.Event()

        def sampler():
            while not stop.is_set():
                for s in stats:
                    try:
                        samples.append(int(read(s)))
                    except ValueError:
                        pass
                time.sleep(0.005)

        th = threading.Thread(target=sampler)
        t0 = time.time()
        th.start()
        n = 0
        while time.time() - t0 < 1.5:
            K.census(blocks, spin_ticks=200000)
            n += 1
            if n % 4 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        stop.set()
        th.join()
        nz = [x for x in samples if x]
        res[blocks] = {"n": len(samples), "mean": sum(samples) / max(1, len(samples)),
                       "max": max(samples or [0]), "mean_nonzero": sum(nz) / max(1, len(nz)),
                       "launches": n}
    # idle
    time.sleep(0.3)
    res["idle"] = [int(read(s)) for s in stats]
    out["cu_occupancy"] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
