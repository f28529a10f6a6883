"""BatchNorm statistics from the conv epilogues (vgpu.ops.bnconv;
native/kernels/conv_gemm.hip vgpu_conv2d_nhwc_bn, bn_nhwc.hip *_partials):
the epilogue's per-64-row pairs against fp32 sums of the stored values, the
fused BN→act→conv node against the fp32 PyTorch reference in both directions,
and a ResNet-V2 training step fused vs unfused."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CL = torch.channels_last


@pytest.fixture(scope="module")
def F(gpu_build):
    from vgpu.ops import bnconv
    return bnconv


def _x(shape, seed, offset=0.0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return ((torch.randn(shape, generator=g) * scale) + offset).to(torch.bfloat16).cuda().contiguous(memory_format=CL)


def _group_sums(v: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
    """[G, C, 2] = per 64-row group (Σ v, Σ v·q) of NHWC rows, fp64."""
    c = v.shape[1]
    v = v.permute(0, 2, 3, 1).reshape(-1, c).double()
    q = q.permute(0, 2, 3, 1).reshape(-1, c).double()
    m = v.shape[0]
    g = (m + 63) // 64
    pad = g * 64 - m
    v = torch.nn.functional.pad(v, (0, 0, 0, pad)).view(g, 64, c)
    q = torch.nn.functional.pad(q, (0, 0, 0, pad)).view(g, 64, c)
    return torch.stack([v.sum(1), (v * q).sum(1)], dim=-1)


def _lib():
    from vgpu.native import load_kernels
    return load_kernels()


def _ptr(t):
    import ctypes
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    import ctypes
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


FWD = [
    # n, c, h, w, cout, ks, stride, pad, residual, tile_m, halo
    (2, 64, 9, 11, 64, 1, 1, 0, False, 64, 0),
    (2, 64, 9, 11, 128, 1, 1, 0, True, 128, 0),
    (3, 128, 17, 13, 256, 1, 1, 0, True, 64, 0),
    (2, 256, 15, 15, 128, 1, 2, 0, False, 128, 0),   # projection-style 1x1/s2
    (2, 64, 23, 21, 64, 3, 1, 1, False, 64, 0),
    (2, 128, 29, 29, 128, 3, 2, 1, False, 128, 0),   # 3x3/s2
    (4, 128, 16, 16, 128, 3, 1, 1, False, 0, 1),     # halo, 128-row tiles
    (20, 256, 11, 11, 256, 3, 1, 1, False, 0, 1),
]


@pytest.mark.parametrize("n,c,h,w,cout,ks,stride,pad,res,tile_m,halo", FWD)
def test_forward_statistics_match_the_stored_output(F, n, c, h, w, cout, ks, stride, pad, res, tile_m, halo):
    from vgpu.ops import conv as C
    lib = _lib()
    x = _x((n, c, h, w), 1)
    wt = _x((cout, c, ks, ks), 2, scale=0.05)
    oh, ow = C.out_hw(h, w, ks, stride, pad)
    r = _x((n, cout, oh, ow), 3) if res else None
    lib.vgpu_conv_set_tile_m(tile_m)
    lib.vgpu_conv_set_halo(halo if halo else 0)
    try:
        before = lib.vgpu_conv_halo_launches()
        z, st = F._conv_out(x, wt, stride, pad, r, True)
        torch.cuda.synchronize()
        ran_halo = lib.vgpu_conv_halo_launches() > before
    finally:
        lib.vgpu_conv_set_tile_m(0)
        lib.vgpu_conv_set_halo(-1)
    assert st is not None and tuple(st.shape) == ((n * oh * ow + 63) // 64, cout, 2)
    assert ran_halo == bool(halo)
    # output identical to the plain kernel of the same tiling
    ref = C.conv2d_ref(x, wt, stride=stride, padding=pad, residual=r)
    torch.testing.assert_close(z.float(), ref, atol=3e-2 * ref.abs().max().item(), rtol=2e-2)
    want = _group_sums(z, z)
    torch.testing.assert_close(st.double(), want, atol=1e-3 * want.abs().max().item() + 1e-4, rtol=1e-4)


@pytest.mark.parametrize("n,c,h,w,ks,act,tile_m,halo", [
    (2, 64, 9, 11, 1, 1, 64, 0), (3, 128, 17, 13, 1, 1, 128, 0), (2, 256, 8, 8, 1, 2, 0, 0),
    (2, 64, 23, 21, 3, 1, 64, 0), (2, 128, 15, 15, 3, 1, 128, 0), (2, 128, 11, 11, 3, 0, 0, 0),
    (4, 128, 15, 15, 3, 1, 0, 1), (20, 256, 11, 11, 3, 1, 0, 1), (3, 128, 16, 16, 3, 2, 0, 1)])
def test_backward_statistics_mask_and_sum_the_data_gradient(F, n, c, h, w, ks, act, tile_m, halo):
    """dgrad epilogue with the BN's x: stores dy·act'(x·s + t) and (Σ, Σ·x̂)
    (halo 1: the 3x3 data gradient on the 32x32 halo kernel)."""
    from vgpu.ops import conv as C
    lib = _lib()
    cout = 128
    pad = ks // 2
    dz = _x((n, cout, h, w), 4)
    wgt = _x((cout, c, ks, ks), 5, scale=0.05)
    wt = C._dgrad_filter(wgt)
    x = _x((n, c, h, w), 6)
    g = torch.Generator(device="cpu").manual_seed(7)
    coef = torch.cat([torch.rand(c, generator=g) + 0.5, torch.rand(c, generator=g) - 0.5,
                      torch.randn(c, generator=g) * 0.1, torch.rand(c, generator=g) + 0.5]).cuda()
    out = torch.empty_like(x)
    st = torch.empty(((n * h * w + 63) // 64, c, 2), dtype=torch.float32, device="cuda")
    lib.vgpu_conv_set_tile_m(tile_m)
    lib.vgpu_conv_set_halo(halo)   # the same kernel family for the fused and the plain data gradient
    try:
        before = lib.vgpu_conv_halo_launches()
        rc = lib.vgpu_conv2d_nhwc_bn(_ptr(dz), _ptr(wt), _ptr(out), None, n, h, w, cout, c, ks, 1, ks - 1 - pad,
                                     _ptr(st), _ptr(x), _ptr(coef), act, 1, _stream())
        ran_halo = lib.vgpu_conv_halo_launches() > before
        dy = C.conv2d(dz, wt, stride=1, padding=ks - 1 - pad)   # the plain data gradient, same kernel
        torch.cuda.synchronize()
    finally:
        lib.vgpu_conv_set_tile_m(0)
        lib.vgpu_conv_set_halo(-1)
    assert rc == 0
    assert ran_halo == bool(halo)
    s, t, mu, inv = (coef[i * c:(i + 1) * c].view(1, c, 1, 1) for i in range(4))
    pre = x.float() * s + t
    mask = (pre > 0).float() if act == 1 else (((pre > 0) & (pre < 6)).float() if act == 2 else torch.ones_like(pre))
    want = (dy.float() * mask).to(torch.bfloat16)
    # the fused kernel stores the masked value of its own fp32 accumulation: equal
    # to masking the bf16 dy except where the mask flips on a rounding tie
    bad = (out.float() != want.float()).float().mean().item()
    assert bad < 1e-3, bad
    ref = _group_sums(out, (x.float() - mu) * inv)
    torch.testing.assert_close(st.double(), ref, atol=1e-3 * ref.abs().max().item() + 1e-4, rtol=1e-4)


def _bn_conv_ref(x, bn, weight, stride, padding, act, residual):
    xf = x.float()
    y = torch.nn.functional.batch_norm(xf, None, None, bn.weight.float(), bn.bias.float(), training=True,
                                       eps=bn.eps)
    y = y.clamp_min(0) if act == "relu" else y
    z = torch.nn.functional.conv2d(y, weight, stride=stride, padding=padding)
    return z + residual.float() if residual is not None else z


@pytest.mark.parametrize("fuse_small", [1, 0])
@pytest.mark.parametrize("c,cout,ks,stride,res,stats_in", [
    (64, 256, 1, 1, True, False), (256, 64, 1, 1, False, True), (64, 64, 3, 1, False, True),
    (128, 128, 3, 2, False, True)])
def test_bn_conv_node_matches_fp32_reference(F, c, cout, ks, stride, res, stats_in, fuse_small):
    """bn_conv: z, running stats, dx, dγ, dβ, dw against fp32 PyTorch; with
    stats_in the BN's statistics come from a producing conv's epilogue.
    fuse_small 1: finalize + apply in one launch (these layers are small), 0:
    the separate finalize kernels."""
    import copy
    from torch import nn
    _lib().vgpu_bn_set_fuse_small(fuse_small)
    torch.manual_seed(0)
    n, h, w = 4, 19, 17
    bn = nn.BatchNorm2d(c).cuda().train()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv = nn.Conv2d(c, cout, ks, stride=stride, padding=ks // 2, bias=False).cuda()
    conv = conv.to(torch.bfloat16).to(memory_format=CL)
    bn_r = copy.deepcopy(bn)
    x0 = _x((n, 64, h, w), 11)
    pre_conv = nn.Conv2d(64, c, 1, bias=False).cuda().to(torch.bfloat16).to(memory_format=CL)
    x_leaf = x0.clone().requires_grad_()
    if stats_in:
        x, st = F.conv_stats(x_leaf, pre_conv)
        assert st is not None
    else:
        x, st = pre_conv(x_leaf).contiguous(memory_format=CL), None
    from vgpu.ops.conv import out_hw
    oh, ow = out_hw(h, w, ks, stride, ks // 2)
    r = _x((n, cout, oh, ow), 12).requires_grad_() if res else None
    x.retain_grad()
    F.set_enabled(True)
    try:
        z, st_out = F.bn_conv(x, bn, conv, residual=r, stats_in=st)
    finally:
        F.set_enabled(False)
    xr = x.detach().float().requires_grad_()
    wr = conv.weight.detach().float().requires_grad_()
    rr = r.detach().float().requires_grad_() if res else None
    zr = _bn_conv_ref(xr, bn_r, wr, conv.stride, conv.padding, "relu", rr)
    torch.testing.assert_close(z.float(), zr, atol=3e-2 * zr.abs().max().item(), rtol=3e-2)
    # running stats (momentum 0.1) from the epilogue / reduction statistics
    with torch.no_grad():
        xm = x.float().mean(dim=(0, 2, 3))
        xv = x.float().var(dim=(0, 2, 3), unbiased=True)
    torch.testing.assert_close(bn.running_mean, 0.9 * 0 + 0.1 * xm, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(bn.running_var, 0.9 * 1 + 0.1 * xv, atol=1e-3, rtol=1e-3)
    assert int(bn.num_batches_tracked) == 1
    if st_out is not None:
        want = _group_sums(z, z)
        torch.testing.assert_close(st_out.double(), want, atol=1e-3 * want.abs().max().item() + 1e-4, rtol=1e-4)
    gz = _x(tuple(z.shape), 13)
    torch.autograd.backward([z], [gz])
    zr.backward(gz.float())
    assert bn.weight.grad is not None and conv.weight.grad is not None
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=3e-2 * xr.grad.abs().max().item(), rtol=5e-2)
    for got, ref in ((bn.weight.grad, bn_r.weight.grad), (bn.bias.grad, bn_r.bias.grad),
                     (conv.weight.grad, wr.grad)):
        tol = 3e-2 * ref.abs().max().item() + 1e-3
        torch.testing.assert_close(got.float(), ref.float(), atol=tol, rtol=5e-2)
    if res:
        torch.testing.assert_close(r.grad.float(), gz.float())
    assert x_leaf.grad is not None and torch.isfinite(x_leaf.grad.float()).all()
    _lib().vgpu_bn_set_fuse_small(-1)


def test_resnet_training_step_fused_matches_unfused(F):
    """ResNet-V2 (identity and projection blocks, 3x3/s2 convs) one training
    step, fused BN statistics vs the unfused native path, each against an fp32
    copy of the model: the fused path's gradients are no further from fp32
    than the unfused path's (both are bf16; early-layer gradients of a deep
    random-init net carry a few % of bf16 noise, so the paths are not compared
    with each other directly), and the running statistics agree."""
    import copy
    from vgpu.models import resnet as R
    torch.manual_seed(0)
    m32 = R.ResNetV2([2, 2, 1, 1]).cuda().to(memory_format=CL).train()
    m = copy.deepcopy(m32).to(torch.bfloat16)
    m2 = copy.deepcopy(m)
    x = _x((4, 3, 96, 96), 9)

    def step(model, inp, fused):
        F.set_enabled(fused)
        try:
            model.zero_grad(set_to_none=True)
            out = model(inp).float()
            out.logsumexp(-1).sum().backward()
        finally:
            F.set_enabled(False)
        return out.detach(), {k: p.grad.float().clone() for k, p in model.named_parameters()}

    out_f, g_f = step(m, x, True)
    out_u, g_u = step(m2, x, False)
    out_r, g_r = step(m32, x.float(), False)
    cos = lambda a, b: torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()  # noqa: E731
    assert cos(out_f, out_r) > 0.99 and cos(out_f, out_u) > 0.995
    bad = []
    for k in g_r:
        nr = g_r[k].norm()
        if nr == 0:
            continue
        ef, eu = ((g_f[k] - g_r[k]).norm() / nr).item(), ((g_u[k] - g_r[k]).norm() / nr).item()
        if ef > 1.5 * eu + 0.02:
            bad.append((k, round(ef, 3), round(eu, 3)))
    assert not bad, bad
    for (k, b1), b2 in zip(m.named_buffers(), m2.buffers()):
        if b1.dtype.is_floating_point:
            torch.testing.assert_close(b1.float(), b2.float(), atol=2e-2, rtol=2e-2, msg=k)


@pytest.mark.parametrize("c,width,sc_stride,h", [(64, 64, 1, 18), (256, 128, 2, 18), (128, 64, 2, 19)])
def test_bn_conv_with_projection_shortcut_matches_fp32_reference(F, c, width, sc_stride, h):
    """A projection block's entry: pre = relu(bn(x)) feeds conv1 and the
    shortcut; the shortcut's data gradient joins conv1's in the fused epilogue
    (stride 2: as a compact 1x1 GEMM result added at the even pixels)."""
    import copy
    from torch import nn
    torch.manual_seed(1)
    n, w = 4, h
    bn = nn.BatchNorm2d(c).cuda().train()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv1 = nn.Conv2d(c, width, 1, bias=False).cuda().to(torch.bfloat16).to(memory_format=CL)
    sc = nn.Conv2d(c, 4 * width, 1, stride=sc_stride, bias=False).cuda().to(torch.bfloat16).to(memory_format=CL)
    bn_r = copy.deepcopy(bn)
    x = _x((n, c, h, w), 31).requires_grad_()
    F.set_enabled(True)
    try:
        z, st, s_out = F.bn_conv(x, bn, conv1, shortcut=sc)
    finally:
        F.set_enabled(False)
    xr = x.detach().float().requires_grad_()
    w1r = conv1.weight.detach().float().requires_grad_()
    wsr = sc.weight.detach().float().requires_grad_()
    pre = torch.nn.functional.batch_norm(xr, None, None, bn_r.weight, bn_r.bias, training=True).clamp_min(0)
    zr = torch.nn.functional.conv2d(pre, w1r)
    sr = torch.nn.functional.conv2d(pre, wsr, stride=sc_stride)
    for got, ref in ((z, zr), (s_out, sr)):
        torch.testing.assert_close(got.float(), ref, atol=3e-2 * ref.abs().max().item(), rtol=3e-2)
    gz, gs = _x(tuple(z.shape), 32), _x(tuple(s_out.shape), 33)
    torch.autograd.backward([z, s_out], [gz, gs])
    torch.autograd.backward([zr, sr], [gz.float(), gs.float()])
    for got, ref in ((x.grad, xr.grad), (bn.weight.grad, bn_r.weight.grad), (bn.bias.grad, bn_r.bias.grad),
                     (conv1.weight.grad, w1r.grad), (sc.weight.grad, wsr.grad)):
        tol = 3e-2 * ref.abs().max().item() + 1e-3
        torch.testing.assert_close(got.float(), ref.float(), atol=tol, rtol=5e-2)


@pytest.mark.parametrize("n,c,h,w,k,s,p", [(4, 64, 37, 41, 3, 2, 1), (2, 128, 16, 16, 2, 2, 0), (3, 64, 9, 9, 3, 1, 1)])
def test_training_maxpool_matches_pytorch(gpu_build, n, c, h, w, k, s, p):
    """Native training max pool (winning-tap bytes + gather backward) against
    torch's max_pool2d on the same bf16 tensors: forward and dx bit-exact."""
    from vgpu.ops.conv import maxpool_train
    x = _x((n, c, h, w), 41)
    x[0, :, 0, 0] = x[0, :, 0, 1]          # ties: the first maximum wins in both
    pool = torch.nn.MaxPool2d(k, s, p)
    xa = x.clone().requires_grad_()
    xb = x.clone().requires_grad_()
    ya = maxpool_train(xa, pool)
    yb = pool(xb)
    assert ya.is_contiguous(memory_format=CL)
    torch.testing.assert_close(ya, yb, atol=0, rtol=0)
    g = _x(tuple(ya.shape), 42)
    ya.backward(g)
    yb.backward(g)
    torch.testing.assert_close(xa.grad, xb.grad, atol=0, rtol=0)
