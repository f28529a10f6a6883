"""Node monitor: region layout mirror, priority feedback, path discovery/GC,
metrics, and the shim obeying the monitor's blocking word."""
import os
import subprocess
import time

import pytest

from vgpu.api import resources as R
from vgpu.k8s.client import KubeClient
from vgpu.k8s.fakeapi import FakeApiServer
from vgpu.monitor.feedback import observe
from vgpu.monitor.metrics import MonitorCollector
from vgpu.monitor.pathmonitor import PathMonitor
from vgpu.monitor.region import AttachedRegion, check_layout
from vgpu.native import FAKES_DIR, shim_path

GiB = 1 << 30


def make_region(path, monkeypatch, uuid="GPU-0", limit="8g", prio=1, cu=0, evict=False):
    for k in list(os.environ):
        if k.startswith("VGPU_"):
            monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("VGPU_DEVICE_MEMORY_LIMIT_0", limit)
    monkeypatch.setenv("VGPU_DEVICE_UUID_0", uuid)
    monkeypatch.setenv("VGPU_TASK_PRIORITY", str(prio))
    if cu:
        monkeypatch.setenv("VGPU_DEVICE_CU_LIMIT_0", str(cu))
    if evict:
        monkeypatch.setenv("VGPU_SUSPEND_EVICT", "true")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    return AttachedRegion(str(path), create=True)


def test_layout_matches_c(native_build):
    check_layout()


def test_region_roundtrip(native_build, tmp_path, monkeypatch):
    r = make_region(tmp_path / "a" / "vgpu.cache", monkeypatch, cu=50)
    devs = r.devices()
    assert devs[0].uuid == "GPU-0" and devs[0].mem_limit == 8 * GiB and devs[0].cu_limit == 50
    assert r.priority == 1
    r.set_cu_mask(0, 0xFF)
    assert r.devices()[0].cu_mask == 0xFF
    r.close()


def test_feedback_blocks_low_priority(native_build, tmp_path, monkeypatch):
    hi = make_region(tmp_path / "hi" / "vgpu.cache", monkeypatch, prio=0)
    lo = make_region(tmp_path / "lo" / "vgpu.cache", monkeypatch, prio=1)
    other = make_region(tmp_path / "ot" / "vgpu.cache", monkeypatch, uuid="GPU-1", prio=1)
    for r in (hi, lo, other):
        r.set_recent_kernel(2)
    observe({"hi": hi, "lo": lo, "ot": other})
    assert lo.recent_kernel == -1          # high-priority task active on GPU-0
    assert hi.recent_kernel == 1 and hi.utilization_switch == 0
    assert lo.utilization_switch == 1
    assert other.recent_kernel == 1 and other.utilization_switch == 0  # alone on GPU-1
    # the high-priority task goes idle: two passes later the low one is released
    observe({"hi": hi, "lo": lo, "ot": other})
    observe({"hi": hi, "lo": lo, "ot": other})
    assert lo.recent_kernel == 0
    for r in (hi, lo, other):
        r.close()


def test_shim_obeys_blocking_word(native_build, tmp_path, monkeypatch):
    path = tmp_path / "c" / "vgpu.cache"
    r = make_region(path, monkeypatch, limit="1g")
    r.set_recent_kernel(-1)
    env = {k: v for k, v in os.environ.items() if not k.startswith("HIP_")}
    env.update({"LD_PRELOAD": str(shim_path()), "LD_LIBRARY_PATH": str(FAKES_DIR),
                "VGPU_SHARED_REGION": str(path)})
    p = subprocess.Popen([str(FAKES_DIR / "shim_driver"), "launch", "5"], env=env, stdout=subprocess.PIPE,
                         text=True)
    time.sleep(1.0)
    assert p.poll() is None  # held back by the monitor
    r.set_recent_kernel(0)
    out, _ = p.communicate(timeout=20)
    assert "fake_launches=7" in out
    assert r.recent_kernel == 2
    r.close()


def test_pathmonitor_discovery_gc_and_metrics(native_build, tmp_path, monkeypatch):
    from prometheus_client import CollectorRegistry, generate_latest
    srv = FakeApiServer()
    c = KubeClient(srv.start())
    srv.add_node("n1")
    srv.add_pod({"metadata": {"name": "p", "namespace": "ns1", "uid": "uidA"},
                 "spec": {"nodeName": "n1", "containers": [{"name": "main"}]}})
    cdir = tmp_path / "containers"
    ra = make_region(cdir / "uidA_main" / "vgpu.cache", monkeypatch, uuid="GPU-7", limit="4g")
    rb = make_region(cdir / "uidGone_x" / "vgpu.cache", monkeypatch)
    # a live process of container A holds 1 GiB
    env = {k: v for k, v in os.environ.items() if not k.startswith("HIP_")}
    env.update({"LD_PRELOAD": str(shim_path()), "LD_LIBRARY_PATH": str(FAKES_DIR),
                "VGPU_SHARED_REGION": str(cdir / "uidA_main" / "vgpu.cache"),
                "VGPU_DEVICE_MEMORY_LIMIT_0": "4g", "VGPU_DEVICE_UUID_0": "GPU-7"})
    holder = subprocess.Popen([str(FAKES_DIR / "shim_driver"), "hold", str(GiB), "5"], env=env,
                              stdout=subprocess.PIPE, text=True)
    assert holder.stdout.readline().strip() == "hold_rc=0"
    pm = PathMonitor(str(cdir), c, "n1")
    t0 = time.time()
    regs = pm.scan(now=t0)
    assert set(regs) == {"uidA_main", "uidGone_x"}
    assert regs["uidA_main"].pod_name == "p" and regs["uidA_main"].namespace == "ns1"
    reg = CollectorRegistry()
    reg.register(MonitorCollector(pm))
    text = generate_latest(reg).decode()
    line = [l for l in text.splitlines() if l.startswith("vGPU_device_memory_usage_in_bytes{") and "GPU-7" in l]
    assert line and float(line[0].split()[-1]) == GiB
    assert 'vGPU_device_memory_limit_in_bytes{ctrname="main",deviceuuid="GPU-7"' in text
    holder.wait(timeout=20)
    # GC after the grace period removes the dead pod's directory
    regs = pm.scan(now=t0 + 400)
    assert set(regs) == {"uidA_main"} and not (cdir / "uidGone_x").exists()
    ra.close()
    rb.close()
    srv.stop()


def test_dashboard_queries_exported_series():
    """docs/gpu-dashboard.json is generated (scripts/gen_dashboard.py) and only
    queries series the scheduler / monitor collectors export."""
    import json
    import pathlib
    import re
    import runpy
    root = pathlib.Path(__file__).resolve().parents[1]
    gen = runpy.run_path(str(root / "scripts" / "gen_dashboard.py"))
    assert json.loads((root / "docs" / "gpu-dashboard.json").read_text()) == gen["dashboard"]()
    src = (root / "vgpu" / "monitor" / "metrics.py").read_text() + (root / "vgpu" / "scheduler" / "metrics.py").read_text()
    exported = set(re.findall(r'MetricFamily\(\s*"([A-Za-z_]+)"', src))
    for p in gen["dashboard"]()["panels"]:
        for t in p["targets"]:
            names = set(re.findall(r"[A-Za-z_][A-Za-z_]+", t["expr"])) - {"sum", "by", "rate", "increase", "m",
                                                                        "nodeid", "deviceidx"}
            assert names and names <= exported, (t["expr"], names - exported)


def test_nodeinfo_endpoint(native_build, tmp_path, monkeypatch):
    """V6: the reference's NodeVGPUInfo gRPC is unimplemented; ours serves the
    same per-container view as JSON over HTTP."""
    import json
    import urllib.request
    from vgpu.monitor.__main__ import serve_nodeinfo
    srv = FakeApiServer()
    c = KubeClient(srv.start())
    srv.add_node("n1")
    srv.add_pod({"metadata": {"name": "p", "namespace": "ns1", "uid": "uidA"},
                 "spec": {"nodeName": "n1", "containers": [{"name": "main"}]}})
    cdir = tmp_path / "containers"
    ra = make_region(cdir / "uidA_main" / "vgpu.cache", monkeypatch, uuid="GPU-3", limit="2g", prio=0)
    pm = PathMonitor(str(cdir), c, "n1")
    pm.scan()
    http = serve_nodeinfo(pm, 0, host="127.0.0.1")
    try:
        base = f"http://127.0.0.1:{http.server_address[1]}"
        info = json.loads(urllib.request.urlopen(base + "/nodeinfo", timeout=10).read())
        assert set(info) == {"uidA_main"}
        e = info["uidA_main"]
        assert (e["pod"], e["namespace"], e["container"], e["priority"]) == ("p", "ns1", "main", 0)
        assert [d["uuid"] for d in e["devices"]] == ["GPU-3"]
        assert json.loads(urllib.request.urlopen(base + "/healthz", timeout=10).read()) == {"status": "ok"}
        with pytest.raises(urllib.error.HTTPError):
            urllib.request.urlopen(base + "/other", timeout=10)
    finally:
        http.shutdown()
        ra.close()
        srv.stop()


def test_host_telemetry_metrics():
    """V5 host series (reference HostGPUMemoryUsage / HostCoreUtilization,
    cmd/vGPUmonitor/metrics.go:113-129) plus MI355X power, temperature, ECC
    and xGMI traffic."""
    from prometheus_client import CollectorRegistry, generate_latest
    from vgpu.deviceplugin.discovery import StaticBackend, Telemetry, mi355x_node

    class NoRegions:
        regions = {}

    be = StaticBackend(mi355x_node(2))
    be.telemetry_by_index = {0: Telemetry(ecc_correctable=4, ecc_uncorrectable=1, xgmi_read_bytes=1 << 30,
                                          xgmi_write_bytes=2 << 30, power_w=1050, temp_edge_c=50,
                                          temp_hotspot_c=80, temp_mem_c=70, valid=15)}
    reg = CollectorRegistry()
    reg.register(MonitorCollector(NoRegions(), be))
    text = generate_latest(reg).decode()
    assert 'HostGPUPowerWatts{deviceidx="0",deviceuuid="GPU-1111-00"} 1050.0' in text
    assert 'HostGPUTemperatureCelsius{deviceidx="0",deviceuuid="GPU-1111-00",sensor="hotspot"} 80.0' in text
    assert 'HostGPUECCErrors_total{deviceidx="0",deviceuuid="GPU-1111-00",type="uncorrectable"} 1.0' in text
    assert 'HostXGMIReadBytes_total{deviceidx="0",deviceuuid="GPU-1111-00"} 1.073741824e+09' in text
    assert 'GPU-1111-01"} 1050' not in text  # device 1 reports no telemetry


def test_monitor_resolves_ambiguous_host_pids_then_purges(native_build, tmp_path, monkeypatch):
    """slots the shim left unverified (ambiguous KFD diff)
    get their host pid from the monitor (NSpid + the pod's cgroup, the closest
    start before the slot's claim when a container pid repeats across the
    pod's containers), src = MONITOR; the host-side purge then frees a slot
    once its process is gone (reference feedback.go:83-162 setHostPid)."""
    import subprocess
    import time
    from vgpu.monitor import pids
    from vgpu.monitor.region import HOSTPID_MONITOR, HOSTPID_UNVERIFIED
    r = make_region(tmp_path / "c" / "vgpu.cache", monkeypatch)
    lib = r.lib
    s7 = lib.vgpu_region_claim(r.ptr, 7, 7, 1)   # container pids, unverified
    s9 = lib.vgpu_region_claim(r.ptr, 9, 9, 1)
    assert r.r.procs[s7].host_pid_src == HOSTPID_UNVERIFIED
    claim_ns = r.r.procs[s7].start_ns
    live = [subprocess.Popen(["sleep", "60"]) for _ in range(2)]
    a, b = live[0].pid, live[1].pid  # real host pids of the pod's two processes
    uid = "1a2b3c4d-0000-1111-2222-333344445555"
    proc = tmp_path / "proc"
    tick = 1_000_000_000 // pids.CLK_TCK

    def fake(pid, nspid, cgroup, start_ns):
        d = proc / str(pid)
        d.mkdir(parents=True)
        (d / "status").write_text(f"Name:\tpython\nNSpid:\t{pid}\t{nspid}\n")
        (d / "cgroup").write_text(f"0::/kubepods.slice/kubepods-burstable-{cgroup}.slice/cri-containerd-x.scope\n")
        fields = ["S"] + ["0"] * 18 + [str(start_ns // tick)] + ["0"] * 10
        (d / "stat").write_text(f"{pid} (python) " + " ".join(fields) + "\n")

    pod = "pod" + uid.replace("-", "_")  # systemd cgroup driver form
    fake(a, 7, pod, claim_ns - 2_000_000_000)        # container pid 7, started before the claim
    fake(99991, 7, pod, claim_ns + 5_000_000_000)    # pid 7 of another container of the pod, started later
    fake(b, 9, pod, claim_ns - 1_000_000_000)
    fake(99992, 9, "podffffffff_0000", claim_ns)      # pid 9 of some other pod
    assert pids.resolve_region(r, uid, str(proc)) == 2
    assert (r.r.procs[s7].host_pid, r.r.procs[s7].host_pid_src) == (a, HOSTPID_MONITOR)
    assert (r.r.procs[s9].host_pid, r.r.procs[s9].host_pid_src) == (b, HOSTPID_MONITOR)
    assert pids.resolve_region(r, uid, str(proc)) == 0  # nothing left to resolve
    assert r.purge(host_ns=True) == 0  # both alive
    live[0].kill()
    live[0].wait()
    time.sleep(0.05)
    assert r.purge(host_ns=True) == 1
    assert r.r.procs[s7].status == 0 and r.r.procs[s9].status != 0
    live[1].kill()
    live[1].wait()
    r.close()


def test_feedback_evicting_suspend_with_hysteresis(native_build, tmp_path, monkeypatch):
    """a low-priority container that opted into suspend-with-
    eviction (VGPU_SUSPEND_EVICT) and stays blocked by a high-priority task
    for SUSPEND_AFTER observations gets SIGUSR2 (its shim then moves its
    managed ranges to host memory); once unblocked it gets SIGUSR1.  A
    container without the opt-in is only blocked, never signalled."""
    from vgpu.monitor import feedback
    monkeypatch.setattr(feedback, "SIGNAL_HOST_NS", False)
    hi = make_region(tmp_path / "hi" / "vgpu.cache", monkeypatch, prio=0)
    lo_path = tmp_path / "lo" / "vgpu.cache"
    lo = make_region(lo_path, monkeypatch, prio=1, evict=True)
    plain_path = tmp_path / "pl" / "vgpu.cache"
    plain = make_region(plain_path, monkeypatch, prio=1)
    assert lo.suspend_evict and not plain.suspend_evict and not hi.suspend_evict
    env = {k: v for k, v in os.environ.items() if not k.startswith(("VGPU_", "CUDA_", "HIP_"))}
    env.update(LD_LIBRARY_PATH=str(FAKES_DIR), LD_PRELOAD=str(shim_path()), VGPU_DEVICE_MEMORY_LIMIT_0="8g",
               VGPU_DEVICE_UUID_0="GPU-0", VGPU_TASK_PRIORITY="1")
    procs = {}
    for name, path, ev in (("lo", lo_path, "true"), ("pl", plain_path, "false")):
        procs[name] = subprocess.Popen([str(FAKES_DIR / "shim_driver"), "idle", "4"],
                                       env={**env, "VGPU_SHARED_REGION": str(path), "VGPU_SUSPEND_EVICT": ev},
                                       stdout=subprocess.PIPE, text=True)
    deadline = time.time() + 20
    while time.time() < deadline and not (lo.live_slots() and plain.live_slots()):
        time.sleep(0.05)
    regions = {"hi": hi, "lo": lo, "pl": plain}
    hi.set_recent_kernel(2)
    observe(regions)                       # blocked once: not yet suspended
    time.sleep(0.2)
    assert not lo.suspended()
    hi.set_recent_kernel(2)
    observe(regions)                       # blocked twice: SIGUSR2
    time.sleep(0.3)
    assert lo.suspended() and not plain.suspended()
    observe(regions)                       # high-priority task idle (decayed): still blocked this pass
    observe(regions)
    observe(regions)                       # unblocked: SIGUSR1
    time.sleep(0.3)
    assert not lo.suspended() and lo.recent_kernel >= 0
    outs = {n: dict(l.split("=", 1) for l in p.communicate(timeout=30)[0].splitlines() if "=" in l)
            for n, p in procs.items()}
    assert outs["lo"]["saw_suspend"] == "1" and outs["lo"]["saw_resume"] == "1", outs
    assert outs["pl"]["saw_suspend"] == "0", outs
    for r in regions.values():
        r.close()
