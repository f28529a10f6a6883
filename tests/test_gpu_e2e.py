"""MI355X end-to-end tests through the control plane.

* Admission: a fake API server, the real scheduler extender (filter/bind), and
  the real device-plugin Allocate. The plugin discovers the GPU with
  SmiBackend (amdsmi on the box). Two 50 % pods get their envs. Each env then
  runs a real process with the enforcement library preloaded, standing in for
  /etc/ld.so.preload. The test checks the HBM cap, disjoint XCD-balanced
  128-CU sets, and the cap as amd-smi shows it.
  Reference flow: pkg/scheduler/scheduler.go:312-402,
  pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:280-403.
* Priority: one low-priority and one high-priority pod run on the GPU, and the
  node monitor's feedback pass runs over both regions. The low-priority pod's
  launches block while the high-priority pod is active. They resume once it
  has left. Reference: cmd/vGPUmonitor/feedback.go:197-255.
"""
import json
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _probe(env, *args, timeout=300):
    from vgpu.native import preload_env
    e = preload_env(dict(os.environ))
    e.update(env)
    e["PYTHONPATH"] = REPO + os.pathsep + e.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-m", "vgpu.bench.probes", *map(str, args)], env=e, capture_output=True,
                       text=True, timeout=timeout, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("PROBE ")][-1][6:])


def test_allocate_envs_enforced_on_the_gpu(gpu_build, tmp_path):
    from vgpu.bench.control import admit_pods
    from vgpu.bench.launch import PodSpec
    from vgpu.deviceplugin.discovery import SmiBackend
    dev = SmiBackend("auto").devices()[0]
    pods = admit_pods([PodSpec(cores=50, mem_mib=8192), PodSpec(cores=50, mem_mib=8192)], dev.index,
                      str(tmp_path), policy="hybrid", device=dev)
    assert [p.share for p in pods] == ["mask", "mask"]
    envs = []
    for p in pods:
        e = dict(p.env)
        e["HIP_VISIBLE_DEVICES"] = str(dev.index)
        envs.append(e)
        assert e["VGPU_DEVICE_UUID_0"] == dev.uuid and e["VGPU_DEVICE_MEMORY_LIMIT_0"] == "8192m"
    census = [_probe(e, "census", 4096, 200000) for e in envs]
    assert [c["distinct_cus"] for c in census] == [128, 128]
    for c in census:
        assert sorted(c["per_xcc"].values()) == [16] * 8, c
    caps = [_probe(e, "cap", 512) for e in envs]
    for c in caps:
        assert c["total"] == 8192 << 20 and c["reserved"] <= 8192 << 20
    smi = _probe(envs[0], "smi", 1024)
    if "error" not in smi:
        assert smi["total"] == 8192 << 20, smi


def _start_progress(env, seconds):
    from vgpu.native import preload_env
    e = preload_env(dict(os.environ))
    e.update(env)
    e["PYTHONPATH"] = REPO + os.pathsep + e.get("PYTHONPATH", "")
    return subprocess.Popen([sys.executable, "-u", "-m", "vgpu.bench.probes", "progress", str(seconds)], env=e,
                            stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, cwd=REPO)


class _Progress:
    """Reads PROGRESS lines of one process in a thread."""

    def __init__(self, proc):
        import threading
        self.proc = proc
        self.last = (0, 0.0)
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        for line in self.proc.stdout:
            if line.startswith("PROGRESS "):
                _, n, t = line.split()
                self.last = (int(n), float(t))


def test_priority_feedback_blocks_low_priority_pod(gpu_build, tmp_path):
    from vgpu.monitor.feedback import observe
    from vgpu.monitor.region import AttachedRegion
    base = {"VGPU_DEVICE_UUID_0": "GPU-prio-test", "VGPU_DEVICE_MEMORY_LIMIT_0": "8192m",
            "HIP_VISIBLE_DEVICES": os.environ.get("HIP_VISIBLE_DEVICES", "0")}
    lo_env = dict(base, VGPU_SHARED_REGION=str(tmp_path / "lo.cache"), VGPU_TASK_PRIORITY="1")
    hi_env = dict(base, VGPU_SHARED_REGION=str(tmp_path / "hi.cache"), VGPU_TASK_PRIORITY="0")
    lo = _Progress(_start_progress(lo_env, 40))
    hi_proc = None
    try:
        t0 = time.time()
        while lo.last[0] < 16 and time.time() - t0 < 120:
            time.sleep(0.2)
        assert lo.last[0] >= 16, "low-priority pod never started"
        hi = _Progress(_start_progress(hi_env, 8))
        hi_proc = hi.proc
        t0 = time.time()
        while hi.last[0] < 8 and time.time() - t0 < 120:
            time.sleep(0.2)
        regions = {"lo": AttachedRegion(str(tmp_path / "lo.cache")), "hi": AttachedRegion(str(tmp_path / "hi.cache"))}
        for _ in range(3):  # monitor passes while both run
            observe(regions)
            time.sleep(0.2)
        assert regions["lo"].recent_kernel < 0
        n0 = lo.last[0]
        h0 = hi.last[0]
        time.sleep(2.0)
        observe(regions)
        blocked_progress = lo.last[0] - n0
        assert hi.last[0] - h0 > 16, "high-priority pod must keep running"
        assert blocked_progress <= 8, blocked_progress  # at most the launches in flight when blocked
        hi.proc.wait(timeout=60)
        for _ in range(4):  # high-priority pod gone: its recent_kernel decays, low is released
            observe(regions)
            time.sleep(0.2)
        assert regions["lo"].recent_kernel >= 0
        n1 = lo.last[0]
        time.sleep(1.5)
        assert lo.last[0] - n1 > 16, "low-priority pod must resume"
    finally:
        for p in (lo.proc, hi_proc):
            if p is not None and p.poll() is None:
                p.kill()
