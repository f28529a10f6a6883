"""Cap holes closed in round 3, on a real MI355X:
stream-ordered pools (PyTorch's hipMallocAsync backend) and graph alloc nodes
never let physical VRAM use pass the container's cap."""
import json
import os

import pytest

from test_gpu_shim import probe

pytestmark = pytest.mark.gpu


def test_hipmallocasync_backend_never_exceeds_the_cap(gpu_build):
    cap_mib = 8192
    res = probe(["asynccap", cap_mib, 1024], {"VGPU_DEVICE_MEMORY_LIMIT_0": f"{cap_mib}m",
                                             "PYTORCH_HIP_ALLOC_CONF": "backend:cudaMallocAsync"}, timeout=900)
    assert "error" not in res, res
    cap = cap_mib << 20
    # KFD's per-process VRAM counter: every buffer object of this process, the
    # runtime's own included (amdgpu's device-wide mem_info_vram_used lags frees
    # by seconds and counts other processes: scripts/mempool_probe.py)
    assert res["kfd_files"], res
    assert res["kfd_vram_peak"] <= cap * 1.01, res
    assert res["max_live_reached"] >= 0.75 * cap, res  # the cap is reachable
    assert res["ooms"] >= 6 and res["graphs_replayed"] >= 1, res


def test_rccl_in_a_temporal_pod_does_not_stall_beside_a_busy_sibling(gpu_build, tmp_path):
    """an RCCL all-reduce loop (world size 1) inside a
    temporal 25 % pod keeps running while a 75 % sibling on the same GPU keeps
    the fair-share board busy: RCCL kernels are exempt from the limiter
    (limiter.cpp exempt_kernel), so a collective can never wait on a throttled
    rank.  Both pods share the node-wide lock dir (one share board)."""
    import subprocess
    import sys
    import time
    from vgpu.native import preload_env
    from test_gpu_shim import REPO
    lock = tmp_path / "lock"
    lock.mkdir()

    def pod_env(limit):
        env = preload_env(dict(os.environ))
        env.update({"VGPU_DEVICE_MEMORY_LIMIT_0": "65536m", "VGPU_DEVICE_CU_LIMIT_0": str(limit),
                    "VGPU_CU_SHARE": "temporal", "VGPU_CU_MASK_FROM_LIMIT": "false", "VGPU_LOCK_DIR": str(lock),
                    "VGPU_DEVICE_UUID_0": "GPU-rccl-test", "GPU_CORE_UTILIZATION_POLICY": "force",
                    "PYTHONPATH": REPO + os.pathsep + env.get("PYTHONPATH", "")})
        return env
    busy = subprocess.Popen([sys.executable, "-m", "vgpu.bench.probes", "progress", "40"], env=pod_env(75),
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=REPO)
    try:
        line = busy.stdout.readline()  # the sibling is launching
        assert line.startswith("PROGRESS"), line
        t0 = time.time()
        r = subprocess.run([sys.executable, "-m", "vgpu.bench.probes", "rcclloop", "300", "64"], env=pod_env(25),
                           capture_output=True, text=True, timeout=240, cwd=REPO)
        assert r.returncode == 0, r.stderr[-3000:]
        res = json.loads([l for l in r.stdout.splitlines() if l.startswith("PROBE ")][-1][6:])
        print("rccl under contention:", res, "wall", time.time() - t0)
        assert res["sum_ok"] and res["iters"] == 300
        assert busy.poll() is None  # the sibling was busy the whole time
    finally:
        busy.kill()
        busy.wait()
