"""Robustness of the enforcement library: ThreadSanitizer / AddressSanitizer
builds of the shim (host code only) under concurrent alloc/free/launch, and
recovery of the shared-region robust mutex when a holder is SIGKILLed
(SURVEY.md §5 race detection + failure detection)."""
import os
import signal
import subprocess
import sys
import time

import pytest

from vgpu.native import FAKES_DIR, LIB_DIR, shim_path

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gcc_runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def _run_threads(preload, env_extra=None):
    env = {k: v for k, v in os.environ.items() if not k.startswith(("VGPU_", "HIP_"))}
    env.update({"LD_LIBRARY_PATH": str(FAKES_DIR), "LD_PRELOAD": preload,
                "VGPU_DEVICE_MEMORY_LIMIT_0": "64g", "VGPU_DEVICE_CU_LIMIT_0": "50"})
    env.update(env_extra or {})
    return subprocess.run([str(FAKES_DIR / "shim_driver"), "threads", "8", "200"], env=env,
                          capture_output=True, text=True, timeout=300)


def test_concurrent_hooks_plain(native_build):
    r = _run_threads(str(shim_path()))
    assert r.returncode == 0, r.stderr
    assert "thread_fails=0" in r.stdout and "region_used=0" in r.stdout


@pytest.mark.parametrize("san,rt", [("thread", "libtsan.so"), ("address", "libasan.so")])
def test_sanitizer_builds(native_build, san, rt):
    runtime = _gcc_runtime(rt)
    if runtime is None:
        pytest.skip(f"{rt} not available")
    from vgpu.native import build
    lib = build.build_shim(sanitize=san)
    env = {"TSAN_OPTIONS": "halt_on_error=1 report_signal_unsafe=0",
           "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1"}
    r = _run_threads(f"{runtime} {lib}", env)
    assert r.returncode == 0, r.stderr[-5000:]
    assert "ThreadSanitizer" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-5000:]
    assert "thread_fails=0" in r.stdout


def test_region_lock_recovers_from_dead_owner(native_build, tmp_path):
    path = str(tmp_path / "r.cache")
    holder = (
        "import ctypes,sys,time;"
        f"lib=ctypes.CDLL({str(shim_path())!r});"
        "lib.vgpu_region_create.restype=ctypes.c_void_p;"
        "lib.vgpu_region_lock.argtypes=[ctypes.c_void_p];"
        f"r=lib.vgpu_region_create({path!r}.encode());"
        "assert lib.vgpu_region_lock(r)==0;print('locked',flush=True);time.sleep(60)")
    env = dict(os.environ, VGPU_DEVICE_MEMORY_LIMIT_0="1g")
    p = subprocess.Popen([sys.executable, "-c", holder], stdout=subprocess.PIPE, text=True, env=env)
    assert p.stdout.readline().strip() == "locked"
    os.kill(p.pid, signal.SIGKILL)
    p.wait()
    taker = (
        "import ctypes;"
        f"lib=ctypes.CDLL({str(shim_path())!r});"
        "lib.vgpu_region_attach.restype=ctypes.c_void_p;"
        "lib.vgpu_region_lock.argtypes=[ctypes.c_void_p];lib.vgpu_region_unlock.argtypes=[ctypes.c_void_p];"
        f"r=lib.vgpu_region_attach({path!r}.encode());"
        "print(lib.vgpu_region_lock(r));lib.vgpu_region_unlock(r)")
    r = subprocess.run([sys.executable, "-c", taker], capture_output=True, text=True, timeout=30, env=env)
    assert r.stdout.strip() == "0", r.stderr


def _forkjoin(preload, env_extra=None):
    env = {k: v for k, v in os.environ.items() if not k.startswith(("VGPU_", "HIP_", "GPU_MAX"))}
    env.update({"LD_LIBRARY_PATH": str(FAKES_DIR), "GPU_MAX_HW_QUEUES": "1"})
    if preload:
        env["LD_PRELOAD"] = preload
    env.update(env_extra or {})
    r = subprocess.run([str(FAKES_DIR / "shim_driver"), "forkjoin"], env=env, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr[-3000:]
    return dict(l.split("=", 1) for l in r.stdout.splitlines() if "=" in l), r.stderr


@pytest.mark.parametrize("san", ["", "address"])
def test_fork_join_graph_replays_under_one_hw_queue(native_build, san):
    """the bench pod's two-stream training graph died with
    SIGSEGV on its first replay.  The native stack (profiles/r5/side_stream)
    puts the fault in the HIP runtime, hip::Graph::UpdateStreams: under
    GPU_MAX_HW_QUEUES=1 (the device plugin's default for a fractional vGPU) its
    walk for a parallel stream on another hardware queue runs past the list.
    The fake runtime refuses such a launch.  A fork/join graph (A -> {B, C} ->
    D) replays under the shim, whose instantiate hook chains the nodes (one
    branch: the single queue serialises them anyway); plain and ASan builds."""
    raw, _ = _forkjoin(None)
    assert raw["launch"] != "0" and raw["branchy_refused"] == "5"  # the runtime bug, modelled
    if san:
        runtime = _gcc_runtime("libasan.so")
        if runtime is None:
            pytest.skip("libasan.so not available")
        from vgpu.native import build
        preload = f"{runtime} {build.build_shim(sanitize=san)}"
        extra = {"ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1"}
    else:
        preload, extra = str(shim_path()), {}
    o, err = _forkjoin(preload, extra)
    assert "AddressSanitizer" not in err, err[-3000:]
    assert (o["instantiate"], o["launch"], o["branchy_refused"], o["fake_launches"]) == ("0", "0", "0", "5")
    assert (o["edges"], o["max_out"], o["max_in"]) == ("3", "1", "1")  # a chain
    # the chain is a clone's; the application's graph keeps its fork/join
    assert (o["app_edges"], o["app_max_out"], o["app_max_in"]) == ("4", "2", "2")
