"""MFMA implicit-GEMM convolution (native/kernels/conv_gemm.hip), stem max-pool and
the fused BN+ReLU+mean against plain-PyTorch fp32 references; the native ResNet
runner against the module."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CL = torch.channels_last


@pytest.fixture(scope="module")
def C(gpu_build):
    from vgpu.ops import conv
    return conv


def _t(shape, seed, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(torch.bfloat16).cuda().contiguous(memory_format=CL)


def _f(shape, seed, lo=-0.5, hi=0.5):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(shape, generator=g) * (hi - lo) + lo).cuda().contiguous()


CASES = [
    # n, c, h, w, cout, ks, stride, pad, bias, act, pro, res
    (2, 64, 9, 11, 64, 1, 1, 0, False, "none", False, False),
    (2, 256, 9, 11, 64, 1, 1, 0, True, "relu", True, False),     # conv1: BN+ReLU prologue
    (2, 64, 9, 11, 256, 1, 1, 0, False, "none", False, True),    # conv3: residual
    (3, 256, 13, 13, 512, 1, 2, 0, False, "none", True, False),  # strided projection shortcut
    (2, 64, 9, 11, 64, 3, 1, 1, True, "relu", False, False),     # conv2
    (2, 128, 15, 15, 128, 3, 2, 1, True, "relu", False, False),  # strided conv2
    (1, 192, 7, 5, 320, 3, 1, 1, True, "none", True, True),      # everything, odd sizes
    (5, 512, 6, 6, 2048, 1, 1, 0, False, "none", False, True),   # stage-4 conv3, M % 128 != 0
    (1, 2048, 3, 3, 512, 1, 1, 0, True, "relu", True, False),    # deep K
    (16, 64, 64, 64, 256, 3, 1, 1, True, "relu", False, False),  # BM=128 LDS-DMA 3x3 tiles
    (16, 64, 64, 63, 64, 3, 1, 1, False, "none", False, True),   # BM=128 x BN=64, ragged M
    (16, 64, 64, 64, 256, 1, 1, 0, False, "none", False, True),  # BM=128 1x1 + residual
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:8])))
def test_conv_matches_fp32(C, case):
    n, c, h, w, cout, ks, stride, pad, has_bias, act, has_pro, has_res = case
    x = _t((n, c, h, w), 1)
    wt = _t((cout, c, ks, ks), 2, scale=(2.0 / (c * ks * ks)) ** 0.5)
    bias = _f((cout,), 3) if has_bias else None
    pro = (_f((c,), 4, 0.5, 1.5), _f((c,), 5)) if has_pro else None
    oh, ow = C.out_hw(h, w, ks, stride, pad)
    res = _t((n, cout, oh, ow), 6) if has_res else None
    got = C.conv2d(x, wt, bias, stride=stride, padding=pad, act=act, pro=pro, residual=res)
    ref = C.conv2d_ref(x, wt, bias, stride=stride, padding=pad, act=act, pro=pro, residual=res)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=CL)
    torch.testing.assert_close(got.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("splits", [-1, 0, 3, 7])
@pytest.mark.parametrize("kind", ["3x3_relu6", "1x1_res"])
def test_conv_splitk_and_bf16_bias(C, splits, kind):
    """Split-K (vgpu_conv2d_workspace / splitk_reduce_kernel): VGG's 14² layer
    at batch 2 and a 1x1 with residual, heuristic / off / forced split counts,
    with a bf16 bias read by the epilogue directly (act | 256)."""
    if kind == "3x3_relu6":
        n, c, h, cout, ks, pad, act, has_res = 2, 512, 14, 512, 3, 1, "relu6", False
    else:
        n, c, h, cout, ks, pad, act, has_res = 3, 1024, 7, 256, 1, 0, "relu", True
    x = _t((n, c, h, h), 21)
    wt = _t((cout, c, ks, ks), 22, scale=(2.0 / (c * ks * ks)) ** 0.5)
    bias = _f((cout,), 23).to(torch.bfloat16)
    res = _t((n, cout, h, h), 24) if has_res else None
    C.set_splitk(splits)
    try:
        got = C.conv2d(x, wt, bias, padding=pad, act=act, residual=res)
        need = C.load_kernels().vgpu_conv2d_workspace(n, h, h, c, cout, ks, 1, pad, 0)
    finally:
        C.set_splitk(-1)
    assert (need > 0) == (splits != 0), need
    ref = C.conv2d_ref(x, wt, bias, padding=pad, act=act, residual=res)
    torch.testing.assert_close(got.float(), ref, atol=3e-2, rtol=2e-2)


BIG_CASES = [
    # 256x256-tile kernel (1x1, stride 1, no prologue, Cout % 256 == 0), forced on
    (4, 256, 32, 33, 512, True, "relu", True),    # M = 4224: ragged last M tile, bias+act+residual
    (2, 1024, 16, 16, 256, False, "none", False),  # deep K (16 steps), one N tile
    (1, 128, 7, 9, 768, True, "none", True),       # M = 63 < one tile, three N tiles
    (16, 128, 64, 64, 512, True, "relu", True),    # 512 tiles: each workgroup walks several (persistent ring)
    (9, 192, 33, 35, 256, False, "none", False),   # K = 192 (6 steps of 32), ragged M across tiles
]


@pytest.mark.parametrize("case", BIG_CASES, ids=lambda c: "x".join(map(str, c[:5])))
def test_conv_big_tile_matches_fp32(C, case):
    from vgpu.native import load_kernels
    n, c, h, w, cout, has_bias, act, has_res = case
    x = _t((n, c, h, w), 11)
    wt = _t((cout, c, 1, 1), 12, scale=(2.0 / c) ** 0.5)
    bias = _f((cout,), 13) if has_bias else None
    res = _t((n, cout, h, w), 14) if has_res else None
    lib = load_kernels()
    lib.vgpu_conv_set_big(1)
    try:
        got = C.conv2d(x, wt, bias, act=act, residual=res)
    finally:
        lib.vgpu_conv_set_big(-1)
    ref = C.conv2d_ref(x, wt, bias, act=act, residual=res)
    torch.testing.assert_close(got.float(), ref, atol=3e-2, rtol=2e-2)


HALO_CASES = [
    # 3x3 / stride 1 on the halo-tile kernel: n, c, h, w, cout, bias, act, tile (2: BM 256, 3: BM 128)
    (2, 64, 11, 11, 128, True, "relu", 3),      # one channel block, tiles span two images
    (5, 512, 11, 11, 512, False, "none", 3),    # ResNet stage 4 (N-major placement: 4.7 MB filter)
    (3, 256, 22, 22, 256, True, "relu", 2),     # ResNet stage 3 on 256-row tiles, ragged last tile
    (2, 128, 16, 16, 256, True, "none", 2),     # ResNet-152 stage 3, M < one 256-row tile
    (7, 128, 8, 8, 128, False, "relu", 3),      # two images per tile
    (3, 64, 9, 1, 128, True, "none", 3),        # W = 1: every kw != 1 tap is padding
    (9, 64, 1, 16, 128, False, "none", 2),      # H = 1: every kh != 1 tap is padding
    (1, 192, 5, 7, 384, True, "relu", 1),       # heuristic tile, M = 35 < one tile, three N tiles
]


@pytest.mark.parametrize("case", HALO_CASES, ids=lambda c: "x".join(map(str, c[:5])) + f"-t{c[7]}")
def test_conv_halo_matches_fp32(C, case):
    from vgpu.native import load_kernels
    n, c, h, w, cout, has_bias, act, tile = case
    x = _t((n, c, h, w), 41)
    wt = _t((cout, c, 3, 3), 42, scale=(2.0 / (9 * c)) ** 0.5)
    bias = _f((cout,), 43) if has_bias else None
    lib = load_kernels()
    lib.vgpu_conv_set_halo(tile)
    before = lib.vgpu_conv_halo_launches()
    try:
        got = C.conv2d(x, wt, bias, stride=1, padding=1, act=act)
    finally:
        lib.vgpu_conv_set_halo(-1)
    assert lib.vgpu_conv_halo_launches() == before + 1, "the halo kernel did not run"  # no silent fallback
    ref = C.conv2d_ref(x, wt, bias, stride=1, padding=1, act=act)
    torch.testing.assert_close(got.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("tile", [2, 3])
def test_conv_halo_integer_exact(C, tile):
    """Integer data through the halo kernel: any tap / row / slot mix-up is visible."""
    from vgpu.native import load_kernels
    g = torch.Generator(device="cpu").manual_seed(tile)
    x = torch.randint(-2, 3, (6, 128, 7, 9), generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=CL)
    wt = torch.randint(-2, 3, (256, 128, 3, 3), generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=CL)
    lib = load_kernels()
    lib.vgpu_conv_set_halo(tile)
    before = lib.vgpu_conv_halo_launches()
    try:
        got = C.conv2d(x, wt, stride=1, padding=1)
    finally:
        lib.vgpu_conv_set_halo(-1)
    assert lib.vgpu_conv_halo_launches() == before + 1
    # fp32 sums of these integers are exact; the kernel rounds them once to bf16
    assert torch.equal(got.float(), C.conv2d_ref(x, wt, stride=1, padding=1).to(torch.bfloat16).float())


DEEP_CASES = [
    # deep-K 1x1 convs with a BN+ReLU prologue (conv_pro_kernel / register path)
    (3, 256, 13, 13, 512, 2, True, "none", False),   # strided projection shortcut, K = 4 steps
    (1, 2048, 3, 3, 512, 1, True, "relu", False),    # deep K (32 steps), M = 9 < one tile
    (4, 1024, 11, 11, 256, 1, False, "relu", False), # K = 16 steps, ragged M
    (2, 192, 7, 9, 256, 1, True, "relu", True),      # K = 3 steps (the minimum), residual
    (5, 320, 9, 7, 128, 1, True, "none", True),      # K = 5 steps: main loop + 2-step remainder
    # persistent 1x1 prologue kernel: thousands of tiles, several per workgroup,
    # the A loads running across tile boundaries (conv1x1_pro_kernel)
    (64, 256, 64, 64, 256, 1, True, "relu", True),   # 4096 tiles, K = 4 steps, residual
    (32, 256, 64, 64, 512, 2, False, "none", False), # strided projection shortcut, 1024 tiles
    (48, 128, 48, 47, 256, 1, True, "relu", True),   # K = 2 steps, ragged M
    (24, 1024, 22, 22, 256, 1, True, "relu", False), # stage-3 conv1 shape (BM 64 tiles), K = 16 steps
]


@pytest.mark.parametrize("case", DEEP_CASES, ids=lambda c: "x".join(map(str, c[:6])))
def test_conv_prologue_deep_k_matches_fp32(C, case):
    n, c, h, w, cout, stride, has_bias, act, has_res = case
    x = _t((n, c, h, w), 21)
    wt = _t((cout, c, 1, 1), 22, scale=(2.0 / c) ** 0.5)
    bias = _f((cout,), 23) if has_bias else None
    pro = (_f((c,), 24, 0.5, 1.5), _f((c,), 25))
    oh, ow = C.out_hw(h, w, 1, stride, 0)
    res = _t((n, cout, oh, ow), 26) if has_res else None
    got = C.conv2d(x, wt, bias, stride=stride, act=act, pro=pro, residual=res)
    ref = C.conv2d_ref(x, wt, bias, stride=stride, act=act, pro=pro, residual=res)
    torch.testing.assert_close(got.float(), ref, atol=3e-2, rtol=2e-2)


def test_conv_asymmetric_exact(C):
    """Integer data (exact in bf16/fp32): catches any row/col or k-order swap."""
    n, c, h, w, cout = 1, 64, 4, 5, 128
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randint(-2, 3, (n, c, h, w), generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=CL)
    wt = torch.randint(-2, 3, (cout, c, 3, 3), generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=CL)
    got = C.conv2d(x, wt, stride=1, padding=1)
    ref = C.conv2d_ref(x, wt, stride=1, padding=1)
    assert torch.equal(got.float(), ref)


def test_conv_rejects_unsupported(C):
    x = _t((1, 3, 8, 8), 0)
    with pytest.raises(ValueError):
        C.conv2d(x, _t((64, 3, 7, 7), 1))
    with pytest.raises(ValueError):
        C.conv2d(_t((1, 64, 8, 8), 0).contiguous(), _t((64, 64, 1, 1), 1).contiguous())


@pytest.mark.parametrize("kpad", [(3, 2, 1), (2, 2, 0), (3, 1, 1)])
def test_maxpool(C, kpad):
    x = _t((2, 64, 13, 12), 7)
    torch.testing.assert_close(C.maxpool(x, *kpad).float(), C.maxpool_ref(x, *kpad), atol=0, rtol=0)


@pytest.mark.parametrize("shape", [(2, 64, 112, 112), (1, 64, 173, 173)])
def test_maxpool_stem_shape(C, shape):
    """The ResNet stem pooling shape: a row (OW x C = 56 x 64 = 3 584 values)
    is far wider than the kernel's 256 threads, so the strided row loop and
    the mix of the K=3 fast path and the edge path inside one row run
    (ADVICE r1).  Bit-exact against the reference."""
    x = _t(shape, 17)
    torch.testing.assert_close(C.maxpool(x, 3, 2, 1).float(), C.maxpool_ref(x, 3, 2, 1), atol=0, rtol=0)


def test_scale_shift_relu_mean(C):
    x = _t((3, 2048, 5, 7), 8)
    s, b = _f((2048,), 9, 0.5, 1.5), _f((2048,), 10)
    torch.testing.assert_close(C.scale_shift_relu_mean(x, s, b).float(),
                               C.scale_shift_relu_mean_ref(x, s, b), atol=1e-2, rtol=1e-2)


def test_native_resnet_matches_module(gpu_build):
    from vgpu.models.resnet import FusedResNetV2Inference, resnet_v2_50
    torch.manual_seed(0)
    m = resnet_v2_50().cuda().eval()
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.1, 0.1)
            mod.running_var.uniform_(0.5, 1.5)
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.1, 0.1)
    x = torch.randn(2, 3, 128, 128, device="cuda")
    with torch.no_grad():
        ref = m.float()(x.contiguous(memory_format=CL))
    mb = m.to(torch.bfloat16).to(memory_format=CL)
    fm = FusedResNetV2Inference(mb, conv="native")
    got = fm(x.to(torch.bfloat16).contiguous(memory_format=CL)).float()
    rel = (got - ref).norm() / ref.norm()
    assert rel < 0.05, float(rel)


def test_native_vgg_matches_module(gpu_build):
    from vgpu.models.vision import VGG16, NativeVGG16Inference
    torch.manual_seed(0)
    m = VGG16().cuda().eval()
    x = torch.randn(2, 3, 64, 64, device="cuda")
    with torch.no_grad():
        ref = m.float()(x.contiguous(memory_format=CL))
    mb = m.to(torch.bfloat16).to(memory_format=CL)
    got = NativeVGG16Inference(mb)(x.to(torch.bfloat16)).float()
    rel = (got - ref).norm() / ref.norm()
    assert rel < 0.05, float(rel)


@pytest.mark.parametrize("hw", [(346, 346), (64, 61), (9, 10)])
def test_stem_space_to_depth_conv(C, hw):
    h, w = hw
    x = _t((2, 3, h, w), 11)
    wt = _t((64, 3, 7, 7), 12, scale=(2.0 / 147) ** 0.5)
    got = C.stem_conv(x, C.stem_weight_s2d(wt))
    ref = torch.nn.functional.conv2d(x.float(), wt.float(), stride=2, padding=3)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=CL)
    torch.testing.assert_close(got.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("nhw", [(2, 346, 346), (3, 64, 61), (1, 9, 10), (2, 351, 339)])
def test_stem_pool_matches_conv_then_maxpool(C, nhw):
    """Fused stem conv + 3x3/s2 max pool: bit-identical to the two kernels
    (same K order and MFMA sequence; the stem row is rounded to bf16 before the
    pool exactly where the unfused conv stores it)."""
    n, h, w = nhw
    x = _t((n, 3, h, w), 41)
    ws2d = C.stem_weight_s2d(_t((64, 3, 7, 7), 42, scale=(2.0 / 147) ** 0.5))
    got = C.stem_pool(x, ws2d)
    ref = C.maxpool3s2(C.stem_conv(x, ws2d))
    assert got.shape == ref.shape and got.is_contiguous(memory_format=CL)
    torch.testing.assert_close(got, ref, atol=0, rtol=0)


@pytest.mark.parametrize("case", [(2, 64, 19, 17, 1), (2, 128, 21, 19, 2), (3, 128, 9, 9, 1),
                                  (4, 64, 64, 64, 1), (2, 128, 40, 37, 1)])
def test_conv23_matches_unfused(C, case):
    n, c, h, w, stride = case
    x = _t((n, c, h, w), 21)
    w2 = _t((c, c, 3, 3), 22, scale=(2.0 / (9 * c)) ** 0.5)
    b2 = _f((c,), 23)
    w3 = _t((4 * c, c, 1, 1), 24, scale=(2.0 / c) ** 0.5)
    oh, ow = C.out_hw(h, w, 3, stride, 1)
    res = _t((n, 4 * c, oh, ow), 25)
    got = C.conv23(x, w2, b2, w3, res, stride=stride)
    h2 = C.conv2d_ref(x, w2, b2, stride=stride, padding=1, act="relu").to(torch.bfloat16)
    ref = C.conv2d_ref(h2.contiguous(memory_format=CL), w3, residual=res)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=CL)
    torch.testing.assert_close(got.float(), ref, atol=3e-2, rtol=2e-2)
    # and bit-for-bit against the unfused native pair on the per-tap kernel
    # (same K order; the halo kernel sums channel-block major, tap minor)
    from vgpu.native import load_kernels
    lib = load_kernels()
    lib.vgpu_conv_set_halo(0)
    try:
        h2n = C.conv2d(x, w2, b2, stride=stride, padding=1, act="relu")
    finally:
        lib.vgpu_conv_set_halo(-1)
    unf = C.conv2d(h2n, w3, residual=res)
    torch.testing.assert_close(got, unf, atol=0, rtol=0)


@pytest.mark.parametrize("case", [(2, 64, 19, 17, 1), (2, 128, 21, 19, 2), (3, 128, 9, 9, 1),
                                  (4, 64, 64, 64, 1), (1, 64, 7, 5, 1), (2, 128, 40, 37, 1)])
def test_conv231_matches_conv23_then_conv1(C, case):
    """Tail + next block's BN+ReLU+conv1 in one kernel: bit-for-bit equal to
    conv23 followed by the prologue conv1 (same roundings, same K order)."""
    n, c, h, w, stride = case
    x = _t((n, c, h, w), 31)
    w2 = _t((c, c, 3, 3), 32, scale=(2.0 / (9 * c)) ** 0.5)
    b2 = _f((c,), 33)
    w3 = _t((4 * c, c, 1, 1), 34, scale=(2.0 / c) ** 0.5)
    w1n = _t((c, 4 * c, 1, 1), 35, scale=(2.0 / (4 * c)) ** 0.5)
    b1n = _f((c,), 36)
    pro = (_f((4 * c,), 37, 0.5, 1.5), _f((4 * c,), 38))
    oh, ow = C.out_hw(h, w, 3, stride, 1)
    res = _t((n, 4 * c, oh, ow), 39)
    y, h1 = C.conv231(x, w2, b2, w3, res, w1n, b1n, pro, stride=stride)
    y_ref = C.conv23(x, w2, b2, w3, res, stride=stride)
    h1_ref = C.conv2d(y_ref, w1n, b1n, act="relu", pro=pro)
    assert y.is_contiguous(memory_format=CL) and h1.is_contiguous(memory_format=CL)
    torch.testing.assert_close(y, y_ref, atol=0, rtol=0)
    torch.testing.assert_close(h1, h1_ref, atol=0, rtol=0)
    # and against fp32
    ref = C.conv2d_ref(y_ref, w1n, b1n, act="relu", pro=pro)
    torch.testing.assert_close(h1.float(), ref, atol=3e-2, rtol=2e-2)


TRAIN_CASES = [
    # n, c, h, w, cout, ks, stride, pad, residual
    (2, 64, 12, 10, 256, 1, 1, 0, True),     # conv3 + residual
    (2, 256, 12, 10, 64, 1, 1, 0, False),    # conv1
    (2, 64, 12, 10, 64, 3, 1, 1, False),     # conv2
    (2, 128, 12, 10, 128, 3, 2, 1, False),   # strided conv2: MIOpen gradients
    (2, 256, 12, 10, 512, 1, 2, 0, False),   # projection shortcut
]


@pytest.mark.parametrize("n,c,h,w,cout,ks,stride,pad,res", TRAIN_CASES)
def test_conv_train_fwd_bwd_matches_fp32(C, n, c, h, w, cout, ks, stride, pad, res):
    conv = torch.nn.Conv2d(c, cout, ks, stride=stride, padding=pad, bias=False).cuda().to(torch.bfloat16)
    conv = conv.to(memory_format=CL)
    assert C.train_eligible(_t((n, c, h, w), 1), conv)
    x = _t((n, c, h, w), 1).requires_grad_()
    oh, ow = C.out_hw(h, w, ks, stride, pad)
    r = _t((n, cout, oh, ow), 2).requires_grad_() if res else None
    y = C.conv_train(x, conv, residual=r)
    xr = x.detach().float().requires_grad_()
    wr = conv.weight.detach().float().requires_grad_()
    rr = r.detach().float().requires_grad_() if res else None
    yr = torch.nn.functional.conv2d(xr, wr, stride=stride, padding=pad)
    if res:
        yr = yr + rr
    assert y.is_contiguous(memory_format=CL)
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    dy = _t((n, cout, oh, ow), 3)
    y.backward(dy)
    yr.backward(dy.float())
    for got, ref in ((x.grad, xr.grad), (conv.weight.grad, wr.grad)) + (((r.grad, rr.grad),) if res else ()):
        scale = ref.abs().max().item()
        torch.testing.assert_close(got.float(), ref, atol=2e-2 * scale, rtol=2e-2)


WGRAD_CASES = [
    # n, c, h, w, cout, ks, stride, pad — covers the 4 tile shapes, split-K, padding taps, strides
    (2, 64, 12, 10, 64, 3, 1, 1),       # BM=64 x BN=64
    (2, 128, 12, 10, 128, 3, 2, 1),     # BM=128 x BN=128, strided
    (4, 64, 33, 31, 256, 1, 1, 0),      # BM=128 x BN=64, ragged pixel tail
    (3, 256, 13, 13, 64, 1, 2, 0),      # BM=64 x BN=128, strided 1x1
    (20, 64, 87, 87, 64, 3, 1, 1),      # ResNet-V2-50 stage-1 conv2 at ai-benchmark 1.2 (b=20, 346²)
    (20, 256, 87, 87, 64, 1, 1, 0),     # stage-1 conv1: hundreds of splits
    (3, 64, 9, 9, 64, 1, 1, 0),         # one split, odd step count
    (2, 512, 11, 11, 512, 3, 1, 1),     # deep columns, few pixels
    (2, 128, 40, 37, 192, 3, 1, 1),     # tap-fused 3x3: ragged 32-pixel row segments
    (2, 64, 33, 35, 128, 3, 2, 1),      # tap-fused 3x3, stride 2, odd sizes
    (20, 1024, 22, 22, 256, 1, 1, 0),   # stage-3 conv1 (LDS-DMA kernel, 1x1 fast path)
    (4, 256, 22, 22, 256, 3, 1, 1),     # stage-3 3x3 per tap (LDS-DMA kernel, im2col path, padding)
    (3, 128, 9, 7, 256, 1, 2, 0),       # strided 1x1 on the LDS-DMA kernel, ragged pixel tail
]


@pytest.mark.parametrize("n,c,h,w,cout,ks,stride,pad", WGRAD_CASES)
def test_conv_wgrad_matches_fp32(C, n, c, h, w, cout, ks, stride, pad):
    x = _t((n, c, h, w), 11)
    oh, ow = C.out_hw(h, w, ks, stride, pad)
    dy = _t((n, cout, oh, ow), 12)
    dw = C.conv2d_wgrad(dy, x, ks, stride=stride, padding=pad)
    assert dw.shape == (cout, c, ks, ks) and dw.is_contiguous(memory_format=CL)
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, c, ks, ks), dy.float(), stride=stride, padding=pad)
    scale = ref.abs().max().item()
    torch.testing.assert_close(dw.float(), ref, atol=1e-2 * scale, rtol=1e-2)
    # deterministic: split-K partials are reduced in a fixed order
    assert torch.equal(dw, C.conv2d_wgrad(dy, x, ks, stride=stride, padding=pad))


def test_dgrad_filters_batched_flip_matches_torch(C):
    """One launch builds every stride-1 conv's data-gradient filter
    (native/kernels/weights.hip): w'[c][kh][kw][co] = w[co][2-kh][2-kw][c],
    bit-exact against transpose + flip, and _ConvTrainFn picks it up."""
    from torch import nn
    convs = [nn.Conv2d(64, 128, 3, padding=1, bias=False), nn.Conv2d(256, 64, 1, bias=False),
             nn.Conv2d(128, 128, 3, padding=1, bias=False), nn.Conv2d(512, 1024, 1, bias=False),
             nn.Conv2d(128, 128, 3, stride=2, padding=1, bias=False)]  # strided: not part of the set
    for m in convs:
        m.to("cuda", torch.bfloat16).to(memory_format=CL)
    d = C.DgradFilters(convs)
    assert len(d.convs) == 4
    d.refresh()
    torch.cuda.synchronize()
    for m, wt in zip(d.convs, d.bufs):
        ref = m.weight.transpose(0, 1)
        if m.kernel_size[0] > 1:
            ref = ref.flip(2, 3)
        assert torch.equal(wt, ref.contiguous(memory_format=CL))
        assert C._dgrad_filter(m.weight) is wt
    with torch.no_grad():
        convs[0].weight.add_(1)  # a changed weight is not served stale
    assert C._dgrad_filter(convs[0].weight) is not d.bufs[0]
