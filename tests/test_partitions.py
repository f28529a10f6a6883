"""Compute / memory partitions as the MIG analogue.

Reference: the NVIDIA plugin's MIG strategies none|single|mixed
(pkg/device-plugin/nvidiadevice/nvinternal/mig/mig.go:17-86,
rm/device_map.go:121-183).  Fixture: an 8 x MI355X node in CPX / NPS2 mode
(64 devices, 32 CUs and one XCD each; every NPS domain of 144 GiB is shared
by 4 partitions) discovered through the fake libamd_smi.
"""
import json
import os
import pathlib

import grpc
import pytest
import yaml

from vgpu import config
from vgpu.api import resources as R
from vgpu.api.codec import NODE_REGISTER_EXT, apply_node_devices_ext, decode_node_devices, decode_pod_devices
from vgpu.config import DevicePluginConfig
from vgpu.device.base import init_default_devices
from vgpu.deviceplugin import api
from vgpu.deviceplugin.__main__ import build_plugins
from vgpu.deviceplugin.discovery import Device, StaticBackend
from vgpu.deviceplugin.partitions import plan, socket_name
from vgpu.deviceplugin.register import register_once
from vgpu.k8s.client import KubeClient
from vgpu.k8s.fakeapi import FakeApiServer
from vgpu.native import FAKES_DIR
from vgpu.scheduler.core import Scheduler

from test_deviceplugin import DISCOVER, FakeKubelet, _smi_subprocess

GiB = 1 << 30
REPO = pathlib.Path(__file__).resolve().parents[1]


def cpx_nps2_fixture(gpus=8, spx=()):
    """8 physical GPUs; GPU g in CPX/NPS2 yields 8 partitions (bdf function =
    partition id) that each report their NPS domain (144 GiB) as VRAM."""
    out = []
    for g in range(gpus):
        parts = 1 if g in spx else 8
        for p in range(parts):
            out.append({"uuid": f"GPU-{g:02d}-{p}", "bdf": f"0000:{0x05 + 0x10 * g:02x}:00.{p}",
                        "name": "AMD Instinct MI355X", "vram": 288 * GiB if parts == 1 else 144 * GiB,
                        "cus": 256 if parts == 1 else 32, "numa": g // 4, "render": 128 + 8 * g + p,
                        "card": 8 * g + p, "hive": 77, "partition": "SPX" if parts == 1 else "CPX",
                        "mem_partition": "NPS1" if parts == 1 else "NPS2", "partition_id": p})
    return out


def devices_of(fx) -> list[Device]:
    from vgpu.deviceplugin.discovery import xcc_of_partition
    return [Device(uuid=g["uuid"], index=i, bdf=g["bdf"], vram_total=g["vram"], cus=g["cus"],
                   num_xcc=xcc_of_partition(g["partition"]), numa=g["numa"], render_minor=g["render"],
                   card=g["card"], xgmi_hive=g["hive"], compute_partition=g["partition"],
                   memory_partition=g["mem_partition"], partition_id=g["partition_id"])
            for i, g in enumerate(fx)]


def test_discovery_of_a_cpx_nps2_node_through_fake_amdsmi(native_build, tmp_path):
    f = tmp_path / "fx.json"
    f.write_text(json.dumps({"gpus": cpx_nps2_fixture(), "link": "xgmi"}))
    out = _smi_subprocess({"VGPU_AMDSMI_LIB": str(FAKES_DIR / "libamd_smi.so"),
                           "VGPU_FAKE_AMDSMI_JSON": str(f)}, DISCOVER.format(mode="amdsmi"))
    devs = out["devs"]
    assert len(devs) == 64
    assert {d["compute_partition"] for d in devs} == {"CPX"} and {d["memory_partition"] for d in devs} == {"NPS2"}
    assert [d["partition_id"] for d in devs[:8]] == list(range(8))
    assert all(d["cus"] == 32 and d["num_xcc"] == 1 for d in devs)


def test_plan_single_splits_nps_domains_between_partitions():
    devs = devices_of(cpx_nps2_fixture())
    groups, bad = plan(devs, "single")
    assert list(groups) == ["amd.com/gpu"] and len(groups["amd.com/gpu"]) == 64 and not bad
    # 288 GB / 2 NPS domains / 4 CPX partitions per domain
    assert {d.vram_total for d in devs} == {36 * GiB} and {d.memory_shared_by for d in devs} == {4}
    assert {d.type for d in devs} == {"AMD-MI355X-CPX"}


def test_plan_reported_memory_is_left_alone():
    devs = devices_of(cpx_nps2_fixture(gpus=1))
    plan(devs, "single", memory="reported")
    assert {d.vram_total for d in devs} == {144 * GiB}


def test_plan_strategies_on_a_mixed_node():
    fx = cpx_nps2_fixture(gpus=8, spx=(0, 1, 2, 3))  # 4 whole GPUs + 4 x 8 CPX partitions
    groups, bad = plan(devices_of(fx), "mixed")
    assert sorted(groups) == ["amd.com/gpu", "amd.com/gpu-cpx"] and not bad
    assert len(groups["amd.com/gpu"]) == 4 and len(groups["amd.com/gpu-cpx"]) == 32
    assert {d.vram_total for d in groups["amd.com/gpu"]} == {288 * GiB}
    assert socket_name("amd.com/gpu-cpx") == "amd-vgpu-cpx.sock" and socket_name("amd.com/gpu") == "amd-vgpu.sock"
    groups, bad = plan(devices_of(fx), "none")
    assert list(groups) == ["amd.com/gpu"] and [d.compute_partition for d in groups["amd.com/gpu"]] == ["SPX"] * 4
    groups, bad = plan(devices_of(fx), "single")
    # single needs a uniform node: the 4 SPX GPUs are the minority
    assert len(groups["amd.com/gpu"]) == 36 and sorted(bad) == [f"GPU-{g:02d}-0" for g in range(4)]
    with pytest.raises(ValueError):
        plan(devices_of(fx), "bogus")


@pytest.fixture
def cpx_cluster(tmp_path):
    def make(fx, strategy):
        init_default_devices()
        config.SCHEDULER = config.SchedulerConfig()
        srv = FakeApiServer()
        client = KubeClient(srv.start())
        sockdir = tmp_path / f"dp-{strategy}"
        sockdir.mkdir()
        kubelet = FakeKubelet(str(sockdir / "kubelet.sock"))
        cfg = DevicePluginConfig(node_name="n1", device_split_count=4, socket_dir=str(sockdir),
                                 host_lib_dir=str(tmp_path / f"host-{strategy}"), config_file="", cu_share="mask",
                                 partition_strategy=strategy)
        srv.add_node("n1")
        plugins = build_plugins(cfg, StaticBackend(devices_of(fx)), client)
        for p in plugins:
            p.start()
        register_once(client, "n1", [d for p in plugins for d in p.devices], cfg)
        sched = Scheduler(client)
        sched.register_from_node_annotations_once()
        made.append((srv, kubelet, plugins))
        return dict(srv=srv, client=client, plugins={p.resource_name: p for p in plugins}, sched=sched,
                    kubelet=kubelet, cfg=cfg)
    made = []
    yield make
    for srv, kubelet, plugins in made:
        for p in plugins:
            p.stop()
        kubelet.srv.stop(0)
        srv.stop()


def _schedule(c, pod, resource="amd.com/gpu"):
    c["srv"].add_pod(pod)
    name, uid = pod["metadata"]["name"], pod["metadata"]["uid"]
    r = c["sched"].filter({"pod": c["client"].get_pod("default", name), "nodenames": ["n1"]})
    assert r["nodenames"] == ["n1"], r
    assert c["sched"].bind({"podName": name, "podNamespace": "default", "podUID": uid, "node": "n1"})["error"] == ""
    plugin = c["plugins"][resource]
    with grpc.insecure_channel(api.unix_target(plugin.socket_path)) as ch:
        stub = api.Stub(ch, "DevicePlugin")
        lw = next(iter(stub.ListAndWatch(api.Empty(), timeout=5)))
        ids = [d.ID for d in lw.devices]
        pref = stub.GetPreferredAllocation(api.PreferredAllocationRequest(container_requests=[
            dict(available_deviceIDs=ids, allocation_size=1)]), timeout=5)
        chosen = list(pref.container_responses[0].deviceIDs)
        resp = stub.Allocate(api.AllocateRequest(container_requests=[dict(devices_ids=chosen)]), timeout=10)
    assigned = decode_pod_devices(c["client"].get_pod("default", name)["metadata"]["annotations"][R.ASSIGNED_IDS])
    return assigned[0][0], dict(resp.container_responses[0].envs), len(ids)


def test_cpx_nps2_node_registers_schedules_and_allocates(cpx_cluster):
    """64 CPX partitions under `single`: registered with NPS-scaled memory and a
    32-CU layout; examples/compute-partition.yaml lands on a partition and its
    CU mask stays inside the partition's single XCD."""
    c = cpx_cluster(cpx_nps2_fixture(), "single")
    reg = c["kubelet"].registrations
    assert [r.resource_name for r in reg] == ["amd.com/gpu"]
    annos = c["client"].get_node("n1")["metadata"]["annotations"]
    devs = apply_node_devices_ext(decode_node_devices(annos[R.NODE_REGISTER]), annos[NODE_REGISTER_EXT])
    assert len(devs) == 64 and {d.type for d in devs} == {"AMD-MI355X-CPX"}
    assert {d.devmem for d in devs} == {36 * 1024} and {d.cus for d in devs} == {32}
    example = yaml.safe_load((REPO / "examples" / "compute-partition.yaml").read_text())
    example["metadata"].update({"namespace": "default", "uid": "uid-cpx"})
    cd, env, n_ids = _schedule(c, example)
    assert n_ids == 64 * 4
    assert cd.uuid.startswith("GPU-") and cd.usedmem == 16384
    mask = int(env["VGPU_CU_MASK_0"], 16)
    assert mask < (1 << 32) and bin(mask).count("1") == 16  # 50 % of the partition's 32 CUs
    assert env["VGPU_DEVICE_MEMORY_LIMIT_0"] == "16384m"


def test_mixed_node_serves_partitions_under_their_own_resource(cpx_cluster):
    c = cpx_cluster(cpx_nps2_fixture(gpus=8, spx=(0, 1, 2, 3)), "mixed")
    assert sorted(r.resource_name for r in c["kubelet"].registrations) == ["amd.com/gpu", "amd.com/gpu-cpx"]
    from test_scheduler import pod as mkpod
    p = mkpod("cpxpod", mem=8192, cores=25)
    lim = p["spec"]["containers"][0]["resources"]["limits"]
    lim["amd.com/gpu-cpx"] = lim.pop(R.RESOURCE_COUNT)
    cd, env, n_ids = _schedule(c, p, "amd.com/gpu-cpx")
    assert n_ids == 32 * 4 and cd.uuid.split("-")[1] in ("04", "05", "06", "07")
    assert int(env["VGPU_CU_MASK_0"], 16) < (1 << 32)
    cd2, env2, n2 = _schedule(c, mkpod("spxpod", mem=8192, cores=25), "amd.com/gpu")
    assert n2 == 4 * 4 and cd2.uuid.split("-")[1] in ("00", "01", "02", "03")
    assert bin(int(env2["VGPU_CU_MASK_0"], 16)).count("1") == 64  # 25 % of a whole 256-CU GPU


def test_mixed_node_reset_event_reaches_the_partition_plugin(cpx_cluster):
    """ADVICE r3 (server.py health_step): under `mixed` every resource's server
    polls the one backend; a GPU pre-reset event for a CPX partition read first
    by the amd.com/gpu server must still reach the amd.com/gpu-cpx server (and
    its post-reset bring the partition back)."""
    from vgpu.deviceplugin.server import EVT_POST_RESET, EVT_PRE_RESET
    c = cpx_cluster(cpx_nps2_fixture(gpus=8, spx=(0, 1, 2, 3)), "mixed")
    gpu, cpx = c["plugins"]["amd.com/gpu"], c["plugins"]["amd.com/gpu-cpx"]
    for p in (gpu, cpx):  # the servers' own health threads must not race the test
        p._stop.set()
    target = cpx.devices[3]
    backend = gpu.backend._fan.backend
    backend.pending_events.append((target.index, EVT_PRE_RESET, "pre-reset"))
    gpu.health_step(0)  # reads the backend first: the event is not one of its devices
    cpx.health_step(0)
    assert cpx.health[target.uuid] is False
    assert all(gpu.health.get(d.uuid, True) for d in gpu.devices)
    backend.pending_events.append((target.index, EVT_POST_RESET, "post-reset"))
    cpx.health_step(0)
    gpu.health_step(0)
    assert cpx.health[target.uuid] is True
