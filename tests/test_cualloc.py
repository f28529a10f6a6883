"""XCD-balanced CU-mask allocator (port of the reference's CU-mask cases,
pkg/device-plugin/hygon/dcu/corealloc_test.go:10-36, re-targeted to granules of
one CU per XCD)."""
from vgpu.deviceplugin.custate import CUMaskState
from vgpu.device.cualloc import MI355X, CULayout, alloc_cu_mask, free_usage, parse_mask, popcount


def test_cus_for_percent_rounds_to_granules():
    assert MI355X.cus_for_percent(50) == 128
    assert MI355X.cus_for_percent(25) == 64
    assert MI355X.cus_for_percent(30) == 80       # 76.8 → 77 → 80
    assert MI355X.cus_for_percent(1) == 8          # at least one CU per XCD
    assert MI355X.cus_for_percent(100) == 256
    assert MI355X.cus_for_percent(0) == 0


def test_alloc_balanced_and_disjoint():
    used = 0
    masks = []
    for pct in (50, 25, 25):
        m = alloc_cu_mask(used, pct)
        assert m is not None and m & used == 0
        assert MI355X.per_xcd_counts(m) == [popcount(m) // 8] * 8
        used |= m
        masks.append(m)
    assert used == MI355X.full_mask()
    assert alloc_cu_mask(used, 10) is None
    used = free_usage(used, masks[1])
    assert alloc_cu_mask(used, 25) == masks[1]


def test_blocked_layout():
    lay = CULayout(total_cus=256, num_xcc=8, interleaved=False)
    m = alloc_cu_mask(0, 25, lay)
    assert lay.per_xcd_counts(m) == [8] * 8
    assert m & 0xFF == 0xFF  # first 8 CUs of XCD 0


def test_cpx_partition_layout():
    cpx = CULayout(total_cus=32, num_xcc=1)
    m = alloc_cu_mask(0, 50, cpx)
    assert m == (1 << 16) - 1


def test_state_uses_per_device_layout(tmp_path):
    st = CUMaskState(str(tmp_path), policy="mask")
    got = st.allocate("u_c", [("CPX-0", 50), ("SPX-0", 50)],
                      {"CPX-0": CULayout(32, 1), "SPX-0": MI355X})
    assert popcount(got["CPX-0"].mask) == 16 and popcount(got["SPX-0"].mask) == 128


def test_parse_mask():
    assert parse_mask("0xff00") == 0xFF00
    assert parse_mask("ff,00") == 0xFF00
    assert parse_mask("") == 0


def test_se_packed_order_gives_whole_shader_engines():
    """VGPU_CU_PACK=se: a 25 % pod owns one SE on every XCD (local CUs j with
    j % 4 == se), a 50 % pod two; masks stay disjoint and XCD-balanced."""
    from vgpu.device.cualloc import MI355X, alloc_cu_mask, granule_order, popcount
    order = granule_order(MI355X, "se")
    assert sorted(order) == list(range(32)) and order[:8] == list(range(0, 32, 4))
    used = 0
    for se in range(4):
        m = alloc_cu_mask(used, 25, MI355X, "se")
        assert popcount(m) == 64 and MI355X.per_xcd_counts(m) == [8] * 8
        local = {bit // 8 for bit in range(256) if m >> bit & 1}
        assert {j % 4 for j in local} == {se}
        used |= m
    assert alloc_cu_mask(used, 25, MI355X, "se") is None
    assert granule_order(MI355X, "spread") == list(range(32))
    import pytest
    with pytest.raises(ValueError):
        granule_order(MI355X, "bogus")
