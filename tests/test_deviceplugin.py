"""Device plugin: discovery through libvgpu_smi (fake amdsmi fixture and a fake
KFD sysfs tree), node registration, and the kubelet gRPC surface end to end with
a fake kubelet + fake API server + the real scheduler extender."""
import json
import os
import threading
from concurrent import futures

import grpc
import pytest

from vgpu import config
from vgpu.api import resources as R
from vgpu.api.codec import decode_node_devices
from vgpu.config import DevicePluginConfig
from vgpu.device.base import init_default_devices
from vgpu.device.cualloc import MI355X, parse_mask
from vgpu.deviceplugin import api
from vgpu.deviceplugin.custate import CUMaskState, ShareGrant
from vgpu.deviceplugin.discovery import (EVT_POST_RESET, EVT_PRE_RESET, LINK_XGMI, SmiBackend,
                                         StaticBackend, mi355x_node)
from vgpu.deviceplugin.register import register_once
from vgpu.deviceplugin.server import VGPUDevicePlugin
from vgpu.k8s.client import KubeClient
from vgpu.k8s.fakeapi import FakeApiServer
from vgpu.native import FAKES_DIR
from vgpu.scheduler.core import Scheduler

from test_scheduler import pod as mkpod


# ---- discovery ------------------------------------------------------------------------
def _smi_subprocess(env, code):
    import subprocess
    import sys
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=60,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


DISCOVER = ("import json; from vgpu.deviceplugin.discovery import SmiBackend; b=SmiBackend('{mode}');"
            "d=b.devices(); print(json.dumps({{'backend': b.name, 'devs': [x.__dict__ for x in d],"
            "'link': b.link(0, 1) if len(d) > 1 else None, 'procs': [p.__dict__ for p in b.processes(0)],"
            "'events': b.events(10)}}))")


def test_discovery_fake_amdsmi(native_build, tmp_path):
    fx = {"gpus": [{"uuid": f"GPU-{i}", "bdf": f"0000:{5 + i:02x}:00.0", "name": "AMD Instinct MI355X",
                    "vram": 309220868096, "cus": 256, "numa": i // 2, "render": 128 + i, "card": i,
                    "hive": 77, "partition": "SPX", "mem_partition": "NPS1", "gfx": 30,
                    "processes": [{"pid": 42, "vram": 1 << 30, "cu": 64}] if i == 0 else []}
                   for i in range(4)],
          "link": "xgmi", "events": [{"gpu": 1, "type": 3, "message": "reset"}]}
    f = tmp_path / "fx.json"
    f.write_text(json.dumps(fx))
    out = _smi_subprocess({"VGPU_AMDSMI_LIB": str(FAKES_DIR / "libamd_smi.so"),
                           "VGPU_FAKE_AMDSMI_JSON": str(f)}, DISCOVER.format(mode="amdsmi"))
    assert out["backend"] == "amdsmi"
    devs = out["devs"]
    assert len(devs) == 4
    assert devs[2]["numa"] == 1 and devs[3]["render_minor"] == 131 and devs[0]["bdf"] == "0000:05:00.0"
    assert devs[0]["vram_total"] == 309220868096 and devs[0]["cus"] == 256 and devs[0]["gfx_activity"] == 30
    assert out["link"][1] == LINK_XGMI
    assert out["procs"] == [{"pid": 42, "vram_bytes": 1 << 30, "cu_occupancy": 64, "gfx_ns": 0}]
    assert out["events"] == [[1, 3, "reset"]]


def make_sysfs(root, n=2):
    for i in range(n + 1):  # node 0 = CPU
        nd = root / f"sys/class/kfd/kfd/topology/nodes/{i}"
        nd.mkdir(parents=True)
        if i == 0:
            (nd / "gpu_id").write_text("0\n")
            (nd / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
            continue
        (nd / "gpu_id").write_text(f"{4000 + i}\n")
        loc = (0x10 * i) << 8
        (nd / "properties").write_text(
            f"simd_count 1024\nsimd_per_cu 4\nnum_xcc 8\nvendor_id 4098\ndevice_id 30115\n"
            f"drm_render_minor {127 + i}\nhive_id 555\nunique_id {0xabc0 + i}\nlocation_id {loc}\ndomain 0\n")
        mb = nd / "mem_banks/0"
        mb.mkdir(parents=True)
        (mb / "properties").write_text(f"heap_type 1\nsize_in_bytes {288 << 30}\n")
        il = nd / "io_links/0"
        il.mkdir(parents=True)
        other = 2 if i == 1 else 1
        (il / "properties").write_text(f"type 11\nnode_from {i}\nnode_to {other}\nweight 15\n")
        pci = root / f"sys/bus/pci/devices/0000:{0x10 * i:02x}:00.0"
        pci.mkdir(parents=True)
        (pci / "numa_node").write_text(f"{i - 1}\n")
        (pci / "current_compute_partition").write_text("SPX\n")
        (pci / "current_memory_partition").write_text("NPS1\n")
        (pci / "product_name").write_text("AMD Instinct MI355X\n")
        (pci / "mem_info_vram_used").write_text("1048576\n")
        ras = pci / "ras"
        ras.mkdir()
        (ras / "umc_err_count").write_text(f"ue: {i}\nce: {10 * i}\n")
        (ras / "gfx_err_count").write_text("ue: 0\nce: 1\n")
        hw = pci / "hwmon/hwmon3"
        hw.mkdir(parents=True)
        (hw / "power1_average").write_text(f"{(700 + i) * 1000000}\n")
        (hw / "temp1_input").write_text("51000\n")
        (hw / "temp2_input").write_text("73500\n")


def test_discovery_sysfs(native_build, tmp_path):
    make_sysfs(tmp_path)
    out = _smi_subprocess({"VGPU_SYSFS_ROOT": str(tmp_path)}, DISCOVER.format(mode="sysfs"))
    assert out["backend"] == "sysfs"
    d0, d1 = out["devs"]
    assert d0["cus"] == 256 and d0["num_xcc"] == 8 and d0["vram_total"] == 288 << 30
    assert d0["uuid"] == f"GPU-{0xabc1:016x}" and d1["numa"] == 1 and d1["render_minor"] == 129
    assert d0["bdf"] == "0000:10:00.0" and d0["vram_used"] == 1048576
    assert out["link"][1] == LINK_XGMI


# ---- CU-mask state ------------------------------------------------------------------------
def test_cumask_state_disjoint_and_gc(tmp_path):
    st = CUMaskState(str(tmp_path), policy="mask")
    a = st.allocate("uid1_c", [("GPU-0", 50)])["GPU-0"]
    b = st.allocate("uid2_c", [("GPU-0", 50)])["GPU-0"]
    assert a.mask and b.mask and a.mask & b.mask == 0 and MI355X.per_xcd_counts(a.mask) == [16] * 8
    c = st.allocate("uid3_c", [("GPU-0", 25)])["GPU-0"]
    assert c.temporal and c.mask == 0  # device fully partitioned: temporal pool (no CUs left to pin)
    e = st.allocate("uid4_c", [("GPU-1", 100)])["GPU-1"]
    assert e.mask == 0 and not e.temporal  # exclusive: no mask, no limiter
    assert st.used("GPU-0") == a.mask | b.mask
    removed = st.gc({"uid2"}, grace_s=0)
    assert "uid1_c" in removed and st.used("GPU-0") == b.mask


def test_cumask_state_hybrid_policy_pools_after_two_masks(tmp_path):
    """hybrid: two masked pods per GPU, later fractional pods share the rest in time."""
    st = CUMaskState(str(tmp_path), policy="hybrid", max_mask_slots=2)
    g = [st.allocate(f"u{i}_c", [("GPU-0", 25)])["GPU-0"] for i in range(4)]
    assert [x.mode for x in g] == ["mask", "mask", "pool", "pool"]
    assert g[0].mask & g[1].mask == 0 and bin(g[0].mask).count("1") == 64
    pool = ((1 << 256) - 1) & ~(g[0].mask | g[1].mask)
    assert g[2].mask == pool and g[3].mask == pool and bin(pool).count("1") == 128
    assert st.pool_members("GPU-0") == 2
    # a freed mask slot goes to the next pod, outside the pool's CUs
    st.gc({"u0", "u2", "u3"}, grace_s=0)
    n = st.allocate("u4_c", [("GPU-0", 25)])["GPU-0"]
    assert n.mode == "mask" and n.mask & pool == 0 and n.mask & g[0].mask == 0


def test_cumask_state_temporal_policy_never_masks(tmp_path):
    st = CUMaskState(str(tmp_path), policy="temporal")
    for i in range(3):
        sg = st.allocate(f"u{i}_c", [("GPU-0", 25)])["GPU-0"]
        assert sg.temporal and sg.mask == 0
    assert st.used("GPU-0") == 0


def test_mask_after_pool_members_shrinks_the_pool(native_build, tmp_path, monkeypatch):
    """a temporal pod admitted BEFORE a mask pod runs on every CU
    (mask 0).  The mask pod's CUs must still be exclusive: the earlier pool
    member's grant and its live shared region shrink to the remaining pool."""
    import os
    from vgpu.monitor.region import AttachedRegion
    st = CUMaskState(str(tmp_path), policy="temporal")
    a = st.allocate("ua_c", [("GPU-0", 25)])["GPU-0"]
    assert a.temporal and a.mask == 0
    for k in list(os.environ):
        if k.startswith("VGPU_"):
            monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("VGPU_DEVICE_MEMORY_LIMIT_0", "8g")
    monkeypatch.setenv("VGPU_DEVICE_UUID_0", "GPU-0")
    live = AttachedRegion(str(tmp_path / "ua_c" / "vgpu.cache"), create=True)  # pool member is running
    assert live.devices()[0].cu_mask == 0
    m = st.allocate("um_c", [("GPU-0", 25)], policy="mask")["GPU-0"]
    assert m.mode == "mask" and bin(m.mask).count("1") == 64
    pool = ((1 << 256) - 1) & ~m.mask
    assert st._grants()["ua_c"]["GPU-0"] == ShareGrant(pool, "pool")
    assert live.devices()[0].cu_mask == pool
    # later pool members get the same pool
    b = st.allocate("ub_c", [("GPU-0", 25)])["GPU-0"]
    assert b.temporal and b.mask == pool
    live.close()


def test_cumask_state_reads_round1_grant_format(tmp_path):
    (tmp_path / "old_c").mkdir()
    (tmp_path / "old_c" / "grant.json").write_text(json.dumps({"GPU-0": "0xff"}))
    st = CUMaskState(str(tmp_path))
    assert st.used("GPU-0") == 0xFF


# ---- end to end ------------------------------------------------------------------------------
class FakeKubelet:
    def __init__(self, sock):
        self.registrations = []
        self.srv = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        self.srv.add_generic_rpc_handlers((api.service_handler("Registration", self),))
        self.srv.add_insecure_port(api.unix_target(sock))
        self.srv.start()

    def Register(self, request, context):
        self.registrations.append(request)
        return api.Empty()


@pytest.fixture
def cluster(tmp_path):
    init_default_devices()
    config.SCHEDULER = config.SchedulerConfig()
    srv = FakeApiServer()
    url = srv.start()
    client = KubeClient(url)
    sockdir = tmp_path / "dp"
    sockdir.mkdir()
    kubelet = FakeKubelet(str(sockdir / "kubelet.sock"))
    cfg = DevicePluginConfig(node_name="n1", device_split_count=4, socket_dir=str(sockdir),
                             host_lib_dir=str(tmp_path / "host"), config_file="", cu_share="mask")
    srv.add_node("n1")
    backend = StaticBackend(mi355x_node(8))
    plugin = VGPUDevicePlugin(cfg, backend, client, "n1")
    plugin.start()
    register_once(client, "n1", plugin.devices, cfg)
    sched = Scheduler(client)
    sched.register_from_node_annotations_once()
    ch = grpc.insecure_channel(api.unix_target(plugin.socket_path))
    stub = api.Stub(ch, "DevicePlugin")
    yield dict(srv=srv, client=client, plugin=plugin, sched=sched, stub=stub, kubelet=kubelet,
               backend=backend, cfg=cfg)
    ch.close()
    plugin.stop()
    kubelet.srv.stop(0)
    srv.stop()


def test_registration_and_list(cluster):
    reg = cluster["kubelet"].registrations
    assert len(reg) == 1 and reg[0].resource_name == "amd.com/gpu" and reg[0].version == "v1beta1"
    assert reg[0].options.get_preferred_allocation_available
    first = next(iter(cluster["stub"].ListAndWatch(api.Empty(), timeout=5)))
    assert len(first.devices) == 8 * 4
    assert all(d.health == api.HEALTHY for d in first.devices)
    node = cluster["client"].get_node("n1")
    devs = decode_node_devices(node["metadata"]["annotations"][R.NODE_REGISTER])
    assert len(devs) == 8 and devs[0].count == 4 and devs[0].devmem == 294912 and devs[0].type == "AMD-MI355X"
    assert {d.numa for d in devs} == {0, 1}


def schedule_and_allocate(c, name, mem, cores, n=1):
    p = mkpod(name, n=n, mem=mem, cores=cores, uid=f"uid-{name}")
    c["srv"].add_pod(p)
    r = c["sched"].filter({"pod": c["client"].get_pod("default", name), "nodenames": ["n1"]})
    assert r["nodenames"] == ["n1"], r
    assert c["sched"].bind({"podName": name, "podNamespace": "default", "podUID": f"uid-{name}",
                            "node": "n1"})["error"] == ""
    lw = next(iter(c["stub"].ListAndWatch(api.Empty(), timeout=5)))
    ids = [d.ID for d in lw.devices]
    pref = c["stub"].GetPreferredAllocation(api.PreferredAllocationRequest(container_requests=[
        dict(available_deviceIDs=ids, allocation_size=n)]), timeout=5)
    chosen = list(pref.container_responses[0].deviceIDs)
    resp = c["stub"].Allocate(api.AllocateRequest(container_requests=[dict(devices_ids=chosen)]), timeout=10)
    return chosen, resp.container_responses[0]


def test_allocate_two_pods_share_one_gpu(cluster):
    c = cluster
    c["sched"].cfg.gpu_scheduler_policy = "binpack"
    config.SCHEDULER.gpu_scheduler_policy = "binpack"
    ch1, r1 = schedule_and_allocate(c, "a", 144000, 50)
    ch2, r2 = schedule_and_allocate(c, "b", 144000, 50)
    # binpack: same physical GPU; preferred allocation steered kubelet to it
    assert ch1[0].rsplit("-", 1)[0] == ch2[0].rsplit("-", 1)[0]
    for r in (r1, r2):
        e = dict(r.envs)
        assert e["VGPU_DEVICE_MEMORY_LIMIT_0"] == "144000m" and e["VGPU_DEVICE_CU_LIMIT_0"] == "50"
        assert e["VGPU_SHARED_REGION"] == "/var/run/vgpu/vgpu.cache"
        assert e["GPU_MAX_HW_QUEUES"] == "1"
        paths = {m.container_path for m in r.mounts}
        assert {"/usr/local/vgpu/libvgpu.so", "/var/run/vgpu", "/tmp/vgpulock", "/etc/ld.so.preload"} <= paths
        devs = {d.container_path for d in r.devices}
        assert "/dev/kfd" in devs and any(p.startswith("/dev/dri/renderD") for p in devs)
    m1, m2 = parse_mask(dict(r1.envs)["VGPU_CU_MASK_0"]), parse_mask(dict(r2.envs)["VGPU_CU_MASK_0"])
    assert m1 & m2 == 0 and bin(m1).count("1") == 128 and bin(m2).count("1") == 128
    # the same masks for ROCr's own queues (HSA_CU_MASK list syntax)
    for r, m in ((r1, m1), (r2, m2)):
        dev, _, spec = dict(r.envs)["HSA_CU_MASK"].partition(":")
        bits = 0
        for part in spec.split(","):
            lo, _, hi = part.partition("-")
            for b in range(int(lo), int(hi or lo) + 1):
                bits |= 1 << b
        assert dev == "0" and bits == m
    for name in ("a", "b"):
        a = c["client"].get_pod("default", name)["metadata"]["annotations"]
        assert a[R.BIND_PHASE] == R.BIND_SUCCESS
        assert a[R.ASSIGNED_IDS_TO_ALLOCATE] == ""
    assert R.NODE_LOCK not in c["client"].get_node("n1")["metadata"]["annotations"]


def test_allocate_multi_gpu_prefers_one_numa(cluster):
    c = cluster
    chosen, r = schedule_and_allocate(c, "big", 0, 100, n=4)
    e = dict(r.envs)
    assert sorted(k for k in e if k.startswith("VGPU_DEVICE_MEMORY_LIMIT_")) == \
        [f"VGPU_DEVICE_MEMORY_LIMIT_{i}" for i in range(4)]
    assert "VGPU_DEVICE_CU_LIMIT_0" not in e and "GPU_MAX_HW_QUEUES" not in e
    renders = [d.container_path for d in r.devices if "renderD" in d.container_path]
    assert len(renders) == 4
    by_render = {f"/dev/dri/renderD{d.render_minor}": d for d in c["plugin"].devices}
    assert len({by_render[p].numa for p in renders}) == 1  # one NUMA node, one xGMI hive
    # container ordinal i follows physical (KFD) order
    uuids = [e[f"VGPU_DEVICE_UUID_{i}"] for i in range(4)]
    idx = [next(d.index for d in c["plugin"].devices if d.uuid == u) for u in uuids]
    assert idx == sorted(idx)
    # each ordinal's PCI address: the shim's smi hooks list only these GPUs
    bdfs = [e[f"VGPU_DEVICE_BDF_{i}"] for i in range(4)]
    assert bdfs == [next(d.bdf for d in c["plugin"].devices if d.uuid == u) for u in uuids] and all(bdfs)


def test_allocate_hsa_tools_intercept_knob(cluster):
    c = cluster
    _, r = schedule_and_allocate(c, "plain", 1000, 25)
    assert "HSA_TOOLS_LIB" not in dict(r.envs)
    c["cfg"].hsa_tools_intercept = True
    try:
        _, r = schedule_and_allocate(c, "tools", 1000, 25)
    finally:
        c["cfg"].hsa_tools_intercept = False
    assert dict(r.envs)["HSA_TOOLS_LIB"] == "/usr/local/vgpu/libvgpu.so"


def test_allocate_without_pending_pod_fails(cluster):
    with pytest.raises(grpc.RpcError) as ei:
        cluster["stub"].Allocate(api.AllocateRequest(container_requests=[dict(devices_ids=["x-0"])]), timeout=5)
    assert ei.value.code() in (grpc.StatusCode.INVALID_ARGUMENT, grpc.StatusCode.UNKNOWN)


def test_allocate_count_mismatch_marks_failed(cluster):
    c = cluster
    p = mkpod("m", n=1, mem=1000, cores=10, uid="uid-m")
    c["srv"].add_pod(p)
    c["sched"].filter({"pod": c["client"].get_pod("default", "m"), "nodenames": ["n1"]})
    c["sched"].bind({"podName": "m", "podNamespace": "default", "podUID": "uid-m", "node": "n1"})
    ids = [d.ID for d in next(iter(c["stub"].ListAndWatch(api.Empty(), timeout=5))).devices][:2]
    with pytest.raises(grpc.RpcError):
        c["stub"].Allocate(api.AllocateRequest(container_requests=[dict(devices_ids=ids)]), timeout=5)
    assert c["client"].get_pod("default", "m")["metadata"]["annotations"][R.BIND_PHASE] == R.BIND_FAILED
    assert R.NODE_LOCK not in c["client"].get_node("n1")["metadata"]["annotations"]


def test_health_reset_and_recovery(cluster):
    c = cluster
    stream = c["stub"].ListAndWatch(api.Empty(), timeout=10)
    first = next(stream)
    assert all(d.health == api.HEALTHY for d in first.devices)
    c["backend"].pending_events.append((2, EVT_PRE_RESET, "mode1 reset"))
    c["plugin"].health_step(10)
    upd = next(stream)
    bad = {d.ID.rsplit("-", 1)[0] for d in upd.devices if d.health == api.UNHEALTHY}
    assert bad == {c["plugin"].devices[2].uuid}
    c["backend"].pending_events.append((2, EVT_POST_RESET, "done"))
    c["plugin"].health_step(10)
    upd = next(stream)
    assert all(d.health == api.HEALTHY for d in upd.devices)
    stream.cancel()


def test_cdi_spec(tmp_path):
    """N10: CDI spec — /dev/kfd shared, per-GPU render + card nodes, an 'all'
    device, atomic write; qualified names are kind=uuid."""
    import json
    from vgpu.deviceplugin import cdi
    from vgpu.deviceplugin.discovery import Device
    devs = [Device(uuid=f"GPU-{i}", index=i, render_minor=128 + 8 * i, card=i) for i in range(2)]
    path = cdi.write_spec(devs, str(tmp_path / "cdi"))
    spec = json.load(open(path))
    assert spec["kind"] == "amd.com/gpu" and spec["cdiVersion"] == cdi.CDI_VERSION
    assert spec["containerEdits"]["deviceNodes"] == [{"path": "/dev/kfd", "permissions": "rw"}]
    by_name = {d["name"]: d["containerEdits"]["deviceNodes"] for d in spec["devices"]}
    assert [n["path"] for n in by_name["GPU-1"]] == ["/dev/dri/renderD136", "/dev/dri/card1"]
    assert [n["path"] for n in by_name["all"]] == ["/dev/dri/renderD128", "/dev/dri/renderD136"]
    assert not os.path.exists(path + ".tmp")
    assert cdi.device_names(["GPU-0"]) == ["amd.com/gpu=GPU-0"]


def test_allocate_cdi_strategies(cluster):
    """device-list-strategy: cdi-cri returns CDI names instead of device nodes,
    cdi-annotations puts them in the container annotation."""
    from vgpu.deviceplugin.allocate import CDI_ANNOTATION
    c = cluster
    c["cfg"].device_list_strategy = "cdi-cri"
    _, r = schedule_and_allocate(c, "cri", 1000, 25)
    assert len(r.devices) == 0
    names = [d.name for d in r.cdi_devices]
    assert len(names) == 1 and names[0].startswith("amd.com/gpu=")
    assert dict(r.envs)["VGPU_DEVICE_MEMORY_LIMIT_0"] == "1000m"
    c["cfg"].device_list_strategy = "cdi-annotations"
    _, r = schedule_and_allocate(c, "ann", 1000, 25)
    assert len(r.devices) == 0 and len(r.cdi_devices) == 0
    assert dict(r.annotations)[CDI_ANNOTATION].startswith("amd.com/gpu=")
    c["cfg"].device_list_strategy = "envvar"


# ---- health: ECC / VM fault / thermal + host telemetry ------------------------------------
TELEM = ("import json; from vgpu.deviceplugin.discovery import SmiBackend; b=SmiBackend('{mode}');"
         "print(json.dumps([b.telemetry(i).__dict__ for i in range(len(b.devices()))]))")


def test_telemetry_fake_amdsmi(native_build, tmp_path):
    fx = {"gpus": [{"uuid": f"GPU-{i}", "hive": 1} for i in range(2)], "link": "xgmi"}
    (tmp_path / "fx.json").write_text(json.dumps(fx))
    (tmp_path / "t.json").write_text(json.dumps({"1": {"ecc_ue": 3, "ecc_ce": 40, "power": 1120, "temp_edge": 55,
                                                       "temp_hotspot": 81, "temp_mem": 70,
                                                       "xgmi_read_kb": 5, "xgmi_write_kb": 7}}))
    out = _smi_subprocess({"VGPU_AMDSMI_LIB": str(FAKES_DIR / "libamd_smi.so"),
                           "VGPU_FAKE_AMDSMI_JSON": str(tmp_path / "fx.json"),
                           "VGPU_FAKE_AMDSMI_TELEMETRY": str(tmp_path / "t.json")}, TELEM.format(mode="amdsmi"))
    t0, t1 = out
    assert t0["ecc_uncorrectable"] == 0 and t0["valid"] & 1
    assert (t1["ecc_uncorrectable"], t1["ecc_correctable"], t1["power_w"]) == (3, 40, 1120)
    assert (t1["temp_edge_c"], t1["temp_hotspot_c"], t1["temp_mem_c"]) == (55, 81, 70)
    assert (t1["xgmi_read_bytes"], t1["xgmi_write_bytes"]) == (5 * 1024, 7 * 1024)


def test_telemetry_sysfs_ras_and_hwmon(native_build, tmp_path):
    make_sysfs(tmp_path, 2)
    out = _smi_subprocess({"VGPU_SYSFS_ROOT": str(tmp_path)}, TELEM.format(mode="sysfs"))
    assert [t["ecc_uncorrectable"] for t in out] == [1, 2]
    assert [t["ecc_correctable"] for t in out] == [11, 21]
    assert [t["power_w"] for t in out] == [701, 702]
    assert out[0]["temp_edge_c"] == 51 and out[0]["temp_hotspot_c"] == 73


def test_health_uncorrectable_ecc_then_reset_recovers(cluster):
    """reference rm/health.go:42-189 (ECC events → unhealthy); the reference
    never recovers (server.go:253 FIXME) — here a GPU reset clears it."""
    from vgpu.deviceplugin.discovery import EVT_THERMAL, EVT_VMFAULT, Telemetry
    c = cluster
    plugin, backend = c["plugin"], c["backend"]
    stream = c["stub"].ListAndWatch(api.Empty(), timeout=10)
    next(stream)
    backend.telemetry_by_index = {i: Telemetry(ecc_uncorrectable=5, valid=1) for i in range(8)}
    plugin.health_step(10)  # baseline: pre-existing errors do not count
    assert all(plugin.health.values())
    backend.telemetry_by_index[3] = Telemetry(ecc_uncorrectable=7, valid=1)
    plugin.health_step(10)
    upd = next(stream)
    bad = {d.ID.rsplit("-", 1)[0] for d in upd.devices if d.health == api.UNHEALTHY}
    assert bad == {plugin.devices[3].uuid}
    # application faults and throttling are counted, device health unchanged
    backend.pending_events += [(1, EVT_VMFAULT, "page fault"), (1, EVT_THERMAL, "hot")]
    plugin.health_step(10)
    assert plugin.vm_faults[plugin.devices[1].uuid] == 1 and plugin.thermal_events[plugin.devices[1].uuid] == 1
    assert plugin.health[plugin.devices[1].uuid]
    # reset: pre → still unhealthy, post → healthy with a new ECC baseline
    backend.pending_events.append((3, EVT_PRE_RESET, "mode1"))
    plugin.health_step(10)
    backend.pending_events.append((3, EVT_POST_RESET, "done"))
    plugin.health_step(10)
    assert plugin.health[plugin.devices[3].uuid]
    upd = next(stream)
    while any(d.health == api.UNHEALTHY for d in upd.devices):
        upd = next(stream)
    stream.cancel()


def test_mask_ranges_syntax():
    from vgpu.deviceplugin.allocate import mask_ranges
    assert mask_ranges(0b1110011) == "0-1,4-6"
    assert mask_ranges(1 << 255) == "255"
    assert mask_ranges((1 << 256) - 1) == "0-255"


def test_partition_mode_mismatch_is_unhealthy_until_restored():
    """--partition-mode pins the expected compute partition: a device found in
    another mode is advertised unhealthy, and healthy again once it is back."""
    from vgpu.config import DevicePluginConfig
    from vgpu.deviceplugin.discovery import StaticBackend, mi355x_node
    from vgpu.deviceplugin.server import VGPUDevicePlugin
    devs = mi355x_node(2)
    devs[1].compute_partition = "CPX"
    backend = StaticBackend(devs)
    cfg = DevicePluginConfig(node_name="n1", partition_mode="SPX", host_lib_dir="/tmp/vgpu-pm-test")
    plugin = VGPUDevicePlugin(cfg, backend, None, "n1")
    assert plugin.health == {devs[0].uuid: True, devs[1].uuid: False}
    plugin.health_step(1)
    assert not plugin.health[devs[1].uuid]
    backend._devs[1].compute_partition = "SPX"
    plugin.health_step(1)
    assert plugin.health[devs[1].uuid]
    backend._devs[0].compute_partition = "DPX"
    plugin.health_step(1)
    assert not plugin.health[devs[0].uuid] and plugin.health[devs[1].uuid]
    # no expectation configured: any mode is fine
    cfg2 = DevicePluginConfig(node_name="n1", host_lib_dir="/tmp/vgpu-pm-test")
    assert all(VGPUDevicePlugin(cfg2, backend, None, "n1").health.values())


def test_allocate_pool_concurrency_env(tmp_path):
    """--pool-concurrency reaches every temporal-pool member as the shim's
    VGPU_POOL_CONCURRENCY / VGPU_POOL_QUANTUM_MS; masked pods never get it."""
    from vgpu.bench.control import admit_pods
    from vgpu.bench.launch import PodSpec
    pods = admit_pods([PodSpec(cores=25, mem_mib=70000)] * 4, 0, str(tmp_path / "a"), pool_concurrency=2)
    for p in pods:
        assert p.share == "temporal"
        assert p.env["VGPU_POOL_CONCURRENCY"] == "2" and p.env["VGPU_POOL_QUANTUM_MS"] == "50"
    pods = admit_pods([PodSpec(cores=25, mem_mib=70000)] * 2, 0, str(tmp_path / "b"))
    assert all("VGPU_POOL_CONCURRENCY" not in p.env for p in pods)
    pods = admit_pods([PodSpec(cores=25, mem_mib=70000)] * 2, 0, str(tmp_path / "c"), policy="mask",
                      pool_concurrency=2)
    assert all(p.share == "mask" and "VGPU_POOL_CONCURRENCY" not in p.env for p in pods)


def test_pod_annotation_overrides_share_policy(tmp_path):
    """amd.com/cu-share on a pod overrides the node's policy for its containers:
    a 'mask' pod on a temporal node gets exclusive CUs, the pool shares the rest."""
    from vgpu.bench.control import admit_pods
    from vgpu.bench.launch import PodSpec
    specs = [PodSpec(cores=25, mem_mib=70000, cu_share="mask"), PodSpec(cores=25, mem_mib=70000),
             PodSpec(cores=25, mem_mib=70000, cu_share="bogus")]
    pods = admit_pods(specs, 0, str(tmp_path), policy="temporal")
    assert pods[0].share == "mask" and pods[0].cu_mask_bits == 64
    assert pods[1].share == "temporal" and pods[2].share == "temporal"
    pool = int(pods[1].env["VGPU_CU_MASK_0"], 16)
    mask = int(pods[0].env["VGPU_CU_MASK_0"], 16)
    assert pool & mask == 0 and bin(pool).count("1") == 192


def test_oversubscribed_node_hands_out_physical_budgets(tmp_path):
    """on a node with --device-memory-scaling 1.8 every
    container gets a physical HBM budget of cap / 1.8 (the shim's virtual
    device memory keeps at most that much resident), so co-located pods split
    the HBM in proportion to their caps instead of first come, first served."""
    from vgpu.bench.control import admit_pods
    from vgpu.bench.launch import PodSpec
    pods = admit_pods([PodSpec(cores=0, mem_mib=230000)] * 2, 0, str(tmp_path / "a"), memory_scaling=1.8)
    for p in pods:
        assert p.env["VGPU_OVERSUBSCRIBE"] == "true"
        assert p.env["VGPU_DEVICE_MEMORY_LIMIT_0"] == "230000m"
        assert p.env["VGPU_DEVICE_MEMORY_PHYSICAL_0"] == f"{int(230000 / 1.8)}m"
    pods = admit_pods([PodSpec(cores=0, mem_mib=100000)], 0, str(tmp_path / "b"))
    assert "VGPU_DEVICE_MEMORY_PHYSICAL_0" not in pods[0].env and "VGPU_OVERSUBSCRIBE" not in pods[0].env


def test_suspend_evict_flag_reaches_the_container(tmp_path):
    """--suspend-evict (chart devicePlugin.suspendEvict) hands
    every container VGPU_SUSPEND_EVICT, which the shim records in its region
    so the monitor knows a suspend frees that container's HBM."""
    from vgpu.bench.control import admit_pods
    from vgpu.bench.launch import PodSpec
    pods = admit_pods([PodSpec(cores=50, mem_mib=100000)], 0, str(tmp_path / "a"), suspend_evict=True)
    assert pods[0].env["VGPU_SUSPEND_EVICT"] == "true"
    pods = admit_pods([PodSpec(cores=50, mem_mib=100000)], 0, str(tmp_path / "b"))
    assert "VGPU_SUSPEND_EVICT" not in pods[0].env
