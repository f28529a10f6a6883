"""GPU-box check of the shim's host-PID resolution: run under LD_PRELOAD of
libvgpu.so, initialise HIP, and compare the pid the shim resolved with the KFD
process entries that exist afterwards."""
import ctypes
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgpu.native import shim_path  # noqa: E402

KFD = "/sys/class/kfd/kfd/proc"
before = {int(os.path.basename(p)) for p in glob.glob(KFD + "/*")}
import torch  # noqa: E402

torch.empty(1, device="cuda")
after = {int(os.path.basename(p)) for p in glob.glob(KFD + "/*")}
lib = ctypes.CDLL(str(shim_path()))
src = ctypes.c_int(-1)
hp = lib.vgpu_self_host_pid(ctypes.byref(src))
print(json.dumps({"getpid": os.getpid(), "host_pid": hp, "src": src.value,
                  "new_kfd_entries_over_torch_init": sorted(after - before),
                  "resolved_entry_exists": os.path.isdir(f"{KFD}/{hp}"),
                  "queues": sorted(os.listdir(f"{KFD}/{hp}/queues")) if os.path.isdir(f"{KFD}/{hp}/queues") else None}))
