"""CPU tests of the interposition paths added around the HIP hooks (fake
runtimes, no GPU):

* HSA memory-pool accounting — runtime-internal device allocations are
  charged to the container once (reference allocator.c
  tracks context/module/buffer bytes separately, §2.6 E1d).
* HSA tools-library mode — ROCr's OnLoad(api_table) hands us the table
  (SURVEY.md §2.6 E1a), and the PLT interposers step aside (nothing twice).
* amdsmi / rocm-smi virtualisation through dlopen handles (the `dlsym`
  override; reference nvmlDeviceGetMemoryInfo hooks, §2.6 E1c).
"""
import json

from vgpu.native import shim_path

from test_shim_native import GiB, run

MiB = 1 << 20


def test_runtime_pool_allocations_charged_once(native_build):
    o = run("pool", env={"VGPU_DEVICE_MEMORY_LIMIT_0": "16g",
                         "VGPU_FAKE_RUNTIME_ALLOC": str(64 * MiB)})
    assert o["table_mode"] == "0"
    assert int(o["ctx0"]) == 64 * MiB           # CLR's init-time pool allocation
    assert int(o["buf0"]) == 0
    assert int(o["buf1"]) == GiB                # hipMalloc: buffer class only ...
    assert int(o["ctx1"]) == 64 * MiB           # ... not again at the pool level
    # the driver itself calling HSA is an application allocation: buffer class
    assert int(o["ctx2"]) == 64 * MiB and int(o["buf2"]) == GiB + 256 * MiB
    assert int(o["ctx3"]) == 64 * MiB and int(o["buf3"]) == GiB
    assert int(o["buf4"]) == 0
    assert int(o["pool_used"]) == 64 * MiB      # the fake runtime really freed the rest
    assert o["big_rc"] == str(0x1008)           # HSA_STATUS_ERROR_OUT_OF_RESOURCES past the 16 GiB cap


def test_runtime_charge_counts_against_cap(native_build):
    # 1 GiB of runtime-internal memory leaves room for 9 of 10 1-GiB buffers.
    o = run("fill", GiB, env={"VGPU_DEVICE_MEMORY_LIMIT_0": "10g",
                              "VGPU_FAKE_RUNTIME_ALLOC": str(GiB)})
    assert o["allocated"] == "9"
    assert int(o["region_used"]) == 10 * GiB


def test_hsa_tools_lib_table_mode(native_build):
    env = {"VGPU_DEVICE_MEMORY_LIMIT_0": "16g", "VGPU_FAKE_RUNTIME_ALLOC": str(64 * MiB),
           "HSA_TOOLS_LIB": str(shim_path())}
    o = run("pool", env=env)
    assert o["tools_loaded"] == "1"
    assert o["table_mode"] == "1"
    assert int(o["ctx1"]) == 64 * MiB and int(o["buf1"]) == GiB
    # the caller is recovered through the PLT hop even though the table entry runs the hook
    assert int(o["ctx2"]) == 64 * MiB and int(o["buf2"]) == GiB + 256 * MiB
    assert int(o["ctx3"]) == 64 * MiB
    assert o["big_rc"] == str(0x1008)


def test_hsa_tools_lib_applies_cu_mask_once(native_build):
    env = {"VGPU_DEVICE_CU_LIMIT_0": "25", "HSA_TOOLS_LIB": str(shim_path())}
    o = run("masks", env=env)
    assert o["queues"] == "1"
    assert o["queue0_words"] == "8"
    # 25 % of 256 CUs = 64 → the 64 low logical bits (8 per XCD)
    assert o["queue0_mask"].lower().endswith("ffffffffffffffff")
    assert int(o["queue0_mask"], 16).bit_count() == 64


def test_tools_lib_without_preload(native_build):
    # HSA_TOOLS_LIB alone (no LD_PRELOAD): the table path still enforces masks.
    env = {"VGPU_DEVICE_CU_LIMIT_0": "50", "HSA_TOOLS_LIB": str(shim_path())}
    o = run("masks", env=env, preload=False)
    assert int(o["queue0_mask"], 16).bit_count() == 128


def _smi_fixture(tmp_path):
    f = tmp_path / "smi.json"
    f.write_text(json.dumps({"gpus": [{"uuid": "GPU-0", "vram": 288 * GiB, "vram_used": 5 * GiB}]}))
    return str(f)


def test_amdsmi_and_rsmi_report_the_cap(native_build, tmp_path):
    env = {"VGPU_DEVICE_MEMORY_LIMIT_0": "144000m", "VGPU_FAKE_AMDSMI_JSON": _smi_fixture(tmp_path),
           "VGPU_FAKE_RUNTIME_ALLOC": str(512 * MiB)}
    o = run("smi", env=env)
    cap = 144000 * MiB
    assert o["amdsmi_loaded"] == "1"
    assert o["interposed"] == "1"               # dlsym(handle) → our hook
    assert int(o["smi_total"]) == cap
    assert int(o["smi_used"]) == 512 * MiB      # container usage, not the device's 5 GiB
    assert int(o["smi_vram_total_mb"]) == 144000
    assert int(o["smi_vram_used_mb"]) == 512
    assert int(o["smi_gtt_total"]) != cap       # non-VRAM types pass through
    assert int(o["rsmi_total"]) == cap
    assert int(o["rsmi_used"]) == 512 * MiB
    assert o["next_ok"] == "1"


def test_smi_passthrough_without_limit(native_build, tmp_path):
    o = run("smi", env={"VGPU_FAKE_AMDSMI_JSON": _smi_fixture(tmp_path)})
    assert o["interposed"] == "1"
    assert int(o["rsmi_total"]) == 288 * GiB
    assert int(o["rsmi_used"]) == GiB           # fake's own number


def test_event_trace_records_allocs_oom_and_launches(native_build, tmp_path):
    from vgpu.monitor import trace
    o = run("fill", GiB, env={"VGPU_DEVICE_MEMORY_LIMIT_0": "4g", "VGPU_TRACE": str(tmp_path)})
    assert o["allocated"] == "4"
    (f,) = list(tmp_path.glob("vgpu-trace-*.bin"))
    h, ev = trace.read(str(f))
    s = trace.summarize(ev)
    assert s["events"]["alloc"] == 4 and s["events"]["free"] == 4 and s["events"]["oom"] == 1
    assert s["alloc_bytes"] == s["free_bytes"] == 4 * GiB
    assert s["events"].get("queue", 0) == 0  # no CU limit → no mask
    assert all(a["t_ns"] <= b["t_ns"] for a, b in zip(ev, ev[1:]))


def test_event_trace_launches_and_masked_queue(native_build, tmp_path):
    from vgpu.monitor import trace
    run("launch", 50, 1024, env={"VGPU_DEVICE_CU_LIMIT_0": "25", "VGPU_TRACE": str(tmp_path)})
    (f,) = list(tmp_path.glob("vgpu-trace-*.bin"))
    _, ev = trace.read(str(f))
    s = trace.summarize(ev)
    assert s["events"]["launch"] >= 50 and s["launch_workgroups"] >= 50 * 1024
    q = [e for e in ev if e["type"] == "queue"]
    assert q and q[0]["b"] == 64


def test_event_trace_ring_wraps(native_build, tmp_path):
    from vgpu.monitor import trace
    run("launch", 500, 8, env={"VGPU_TRACE": str(tmp_path), "VGPU_TRACE_EVENTS": "64"})
    (f,) = list(tmp_path.glob("vgpu-trace-*.bin"))
    h, ev = trace.read(str(f))
    assert h.head > 500 and len(ev) == 64


def test_graph_launch_charged_by_kernel_nodes(native_build, tmp_path):
    """hipGraphLaunch is charged the workgroups of the executable graph's
    kernel nodes (child graphs included, other node types ignored), recorded
    at instantiation; an unknown exec falls back to VGPU_GRAPH_LAUNCH_TOKENS."""
    from vgpu.monitor import trace
    o = run("graph", 3, env={"VGPU_TRACE": str(tmp_path), "VGPU_GRAPH_LAUNCH_TOKENS": "7"})
    assert o["fake_launches"] == "5"
    (f,) = list(tmp_path.glob("vgpu-trace-*.bin"))
    _, ev = trace.read(str(f))
    wg = [e["a"] for e in ev if e["type"] == "launch"]
    # 2 kernel nodes (100x2, 300x2) + child (50) = 850 per launch; e1 x3, e2 x1, destroyed e1 x1
    assert wg == [850, 850, 850, 850, 7]


def test_smi_process_lists_show_only_the_container(native_build, tmp_path):
    """E1c process-list virtualisation: amd-smi / rocm-smi inside a pod list only
    the pod's own processes (host pids resolved by the KFD diff)."""
    from test_shim_native import _kfd_env
    env = _kfd_env(tmp_path, 777100)
    f = tmp_path / "smi.json"
    f.write_text(json.dumps({"gpus": [{"uuid": "GPU-0", "processes": [
        {"pid": 4242, "vram": GiB}, {"pid": 777100, "vram": GiB}, {"pid": 5151, "vram": GiB}]}]}))
    env.update({"VGPU_FAKE_AMDSMI_JSON": str(f), "VGPU_FAKE_RSMI_PIDS": "4242,777100,5151"})
    o = run("smi", env=env)
    assert o["smi_procs"] == "777100"
    assert o["rsmi_procs"] == "777100"


def test_smi_process_lists_pass_through_without_control(native_build, tmp_path):
    f = tmp_path / "smi.json"
    f.write_text(json.dumps({"gpus": [{"uuid": "GPU-0", "processes": [{"pid": 4242}, {"pid": 5151}]}]}))
    o = run("smi", env={"VGPU_FAKE_AMDSMI_JSON": str(f), "VGPU_FAKE_RSMI_PIDS": "4242,5151",
                        "VGPU_DISABLE_CONTROL": "true"})
    assert o["smi_procs"] == "4242,5151" and o["rsmi_procs"] == "4242,5151"


def _smi8(tmp_path, extra_pid=None):
    gpus = [{"uuid": f"GPU-{i}", "bdf": f"0000:{0x05 + 0x10 * i:02x}:00.0", "vram": 288 * GiB,
             "vram_used": (i + 1) * GiB, "processes": [{"pid": 4242 + i, "vram": GiB}]} for i in range(8)]
    if extra_pid:
        gpus[5]["processes"].append({"pid": extra_pid, "vram": GiB})
    f = tmp_path / "smi8.json"
    f.write_text(json.dumps({"gpus": gpus}))
    return str(f)


def test_smi_device_identity_by_pci_address(native_build, tmp_path):
    """VERDICT r4 #6 (reference libvgpu.so handle_remap, nvmlDeviceGetCount_v2,
    nvmlDeviceGetHandleByIndex_v2): the node has 8 GPUs and the container holds
    physical GPU 5 as its ordinal 0 (VGPU_DEVICE_BDF_0 from the device plugin).
    amdsmi lists one processor handle -- GPU 5's -- with the pod's cap, usage
    and processes; rocm-smi reports one device whose index 0 is GPU 5 and
    refuses index 1."""
    from test_shim_native import _kfd_env
    env = _kfd_env(tmp_path, 777200)
    env.update({"VGPU_FAKE_AMDSMI_JSON": _smi8(tmp_path, 777200), "VGPU_FAKE_GPUS": "8",
                "VGPU_DEVICE_MEMORY_LIMIT_0": "100g", "VGPU_DEVICE_BDF_0": "0000:55:00.0"})
    o = run("smi_ident", env=env)
    assert o["gpus"] == "1" and o["sockets"] == "1"
    assert o["gpu0_bdf"] == "0000:55:00.0"
    assert int(o["gpu0_total"]) == 100 * GiB and int(o["gpu0_used"]) == GiB
    assert o["gpu0_procs"] == "777200"
    assert o["rsmi_devices"] == "1" and o["rsmi_pci0"] == "0000:55:00.0" and o["rsmi_pci0_rc"] == "0"
    assert int(o["rsmi_total0"]) == 100 * GiB
    assert o["rsmi_past_rc"] != "0"


def test_smi_device_list_unfiltered_without_addresses_or_control(native_build, tmp_path):
    """Without the container's PCI addresses (no device-plugin env, HIP not
    loaded) or with control disabled, every GPU stays listed as before."""
    base = {"VGPU_FAKE_AMDSMI_JSON": _smi8(tmp_path), "VGPU_FAKE_GPUS": "8"}
    o = run("smi_ident", env={**base, "VGPU_DEVICE_MEMORY_LIMIT_0": "100g"})
    assert o["gpus"] == "8" and o["rsmi_devices"] == "8" and o["gpu0_bdf"] == "0000:05:00.0"
    o = run("smi_ident", env={**base, "VGPU_DEVICE_BDF_0": "0000:55:00.0", "VGPU_DISABLE_CONTROL": "true"})
    assert o["gpus"] == "8" and o["rsmi_devices"] == "8"


def test_hsa_direct_dispatches_are_intercepted_and_held(native_build):
    """VERDICT r4 missing #4: a program dispatching AQL packets on an HSA
    queue of its own (no HIP launch) under HSA_TOOLS_LIB.  The shim builds that
    queue with ROCr's intercept-queue entry of the tools API table; every
    kernel dispatch passes its handler (counted, 4 per submission of 4
    dispatches + 1 barrier) and is held while the pod is suspended."""
    from vgpu.native import shim_path
    o = run("hsa_dispatch", env={"VGPU_DEVICE_CU_LIMIT_0": "25", "HSA_TOOLS_LIB": str(shim_path())})
    assert o["queue_rc"] == "0" and o["intercept_queues"] == "1" and o["shim_queues"] == "1"
    assert o["hw_dispatched"] == "100" and o["shim_dispatches"] == "100"
    assert o["held_while_suspended"] == "1" and o["hw_while_suspended"] == "100"
    assert o["hw_after_resume"] == "104"


def test_hsa_queue_without_tools_lib_is_plain(native_build):
    o = run("hsa_dispatch", env={"VGPU_DEVICE_CU_LIMIT_0": "25"})
    assert o["intercept_queues"] == "0" and o["hw_dispatched"] == "100"
