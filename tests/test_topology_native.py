"""Native topology solver (native/smi/topo.cpp) against its executable spec
(vgpu/deviceplugin/topology.py:preferred_py) on random nodes — the reference's
allocator tables (pkg/device-plugin/mlu/allocator/board_test.go, spider_test.go)
pin hand-written cases; here every random node is a case."""
import random

import pytest
from hypothesis import given, settings, strategies as st

from vgpu.deviceplugin import topology as T
from vgpu.deviceplugin.discovery import LINK_PCIE, LINK_XGMI, Device


def _node(rnd, n):
    devs = [Device(index=i, uuid=f"GPU-{i}", numa=rnd.randrange(2), xgmi_hive=rnd.choice([0, 1 << 40, 7]))
            for i in range(n)]
    links = [[0] * n for _ in range(n)]
    for a in range(n):
        for b in range(a + 1, n):
            t = LINK_XGMI if devs[a].xgmi_hive == devs[b].xgmi_hive and rnd.random() < 0.9 else LINK_PCIE
            links[a][b] = links[b][a] = t
    return devs, links


@pytest.fixture(scope="module")
def native(native_build):
    T._NATIVE = None
    fn = T._native()
    assert fn is not None, "libvgpu_smi.so not built"
    return fn


@settings(max_examples=300, deadline=None)
@given(seed=st.integers(0, 1 << 30), n=st.integers(1, 12), size=st.integers(0, 8),
       limit=st.sampled_from([5, 20000]))
def test_native_matches_reference(native, seed, n, size, limit):
    rnd = random.Random(seed)
    devs, links = _node(rnd, n)
    avail = sorted(rnd.sample(range(n), rnd.randrange(n + 1)))
    must = rnd.sample(range(n), rnd.randrange(min(3, n) + 1))
    used = {i: rnd.randrange(4) for i in range(n) if rnd.random() < 0.5}
    got = T.preferred(avail, must, size, devs, links, used, limit)
    want = T.preferred_py(avail, must, size, devs, links, used, limit)
    assert got == want


def test_full_hive_prefers_one_numa(native):
    devs = [Device(index=i, uuid=f"G{i}", numa=i // 4, xgmi_hive=1) for i in range(8)]
    links = [[0 if a == b else LINK_XGMI for b in range(8)] for a in range(8)]
    assert T.preferred(list(range(8)), [], 4, devs, links) in ([0, 1, 2, 3], [4, 5, 6, 7])
    # a partially used device is kept in the set (whole GPUs stay free)
    got = T.preferred(list(range(8)), [], 2, devs, links, {5: 2})
    assert 5 in got


def test_cpx_node_is_fast(native):
    import time
    rnd = random.Random(1)
    devs, links = _node(rnd, 64)  # 8 GPUs x CPX = 64 logical devices
    t0 = time.perf_counter()
    got = T.preferred(list(range(64)), [], 4, devs, links, limit=20000)
    assert len(got) == 4 and time.perf_counter() - t0 < 1.0
