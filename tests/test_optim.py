"""vgpu.ops.optim.SGD against torch.optim.SGD: the PyTorch fallback path on
CPU (bit-exact), the native bf16 kernel (native/kernels/optim.hip) on the GPU
against PyTorch's fused SGD over several steps, first step included."""
import pytest
import torch

from vgpu.ops.optim import SGD


def _params(device, dtype, seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 3, 3, 3), (64,), (4096, 25088 // 49), (1000,), (7, 5)]  # (7, 5): odd size, fallback
    ps = [torch.nn.Parameter((torch.randn(s, generator=g) * 0.1).to(device=device, dtype=dtype)) for s in shapes]
    # a channels_last conv weight (the models' layout): dense, not contiguous
    ps.append(torch.nn.Parameter((torch.randn(128, 64, 3, 3, generator=g) * 0.1).to(device=device, dtype=dtype)
                                 .contiguous(memory_format=torch.channels_last)))
    return ps


def _run(opt_cls, params, steps, **kw):
    opt = opt_cls(params, **kw)
    g = torch.Generator().manual_seed(1)
    for _ in range(steps):
        for p in params:
            p.grad = torch.empty_like(p).copy_((torch.randn(p.shape, generator=g) * 0.01))
        opt.step()
    return [p.detach().float().cpu() for p in params]


@pytest.mark.parametrize("kw", [dict(lr=0.1, momentum=0.9), dict(lr=0.05, momentum=0.9, weight_decay=1e-2),
                                dict(lr=0.05, momentum=0.8, nesterov=True), dict(lr=0.1),
                                dict(lr=0.1, momentum=0.9, dampening=0.3)])
def test_sgd_fallback_matches_torch_cpu(kw):
    a = _run(SGD, _params("cpu", torch.float32), 4, **kw)
    b = _run(torch.optim.SGD, _params("cpu", torch.float32), 4, **kw)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(lr=0.1, momentum=0.9), dict(lr=0.05, momentum=0.9, weight_decay=1e-2),
                                dict(lr=0.05, momentum=0.8, nesterov=True),
                                dict(lr=0.1, momentum=0.9, dampening=0.3)])
def test_sgd_native_bf16_matches_torch_fused(gpu_build, kw):
    calls = []
    import vgpu.ops.optim as O
    orig = O.sgd_bf16_
    O.sgd_bf16_ = lambda *a, **k: (calls.append(len(a[0])), orig(*a, **k))[1]
    try:
        a = _run(SGD, _params("cuda", torch.bfloat16), 4, **kw)
    finally:
        O.sgd_bf16_ = orig
    assert calls and sum(calls) == 4 * 5, calls  # 5 eligible tensors per step, natively
    b = _run(torch.optim.SGD, _params("cuda", torch.bfloat16), 4, fused=True, **kw)
    for x, y in zip(a, b):
        # fp32 math, bf16 storage on both sides; fma vs mul+add rounding moves a
        # rare element by a bf16 ulp, which later steps carry along
        if x.numel() >= 4096:  # the (7, 5) fallback tensor runs PyTorch's foreach SGD here
            assert (x != y).float().mean().item() < 1e-3
        torch.testing.assert_close(x, y, atol=1e-3, rtol=1.6e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,c", [(2, 1000), (50, 1000), (7, 2), (3, 4097), (100, 1000)])
def test_cross_entropy_matches_torch(gpu_build, dtype, rows, c):
    """vgpu.ops.loss.cross_entropy (native/kernels/loss.hip): the mean loss and
    dlogits against F.cross_entropy on the fp32 logits."""
    from vgpu.ops.loss import cross_entropy
    g = torch.Generator().manual_seed(rows * c)
    x = (torch.randn(rows, c, generator=g) * 3).to(dtype).cuda().requires_grad_()
    t = torch.randint(0, c, (rows,), generator=g).cuda()
    loss = cross_entropy(x, t)
    (loss * 2.0).backward()
    xr = x.detach().float().requires_grad_()
    lr = torch.nn.functional.cross_entropy(xr, t)
    (lr * 2.0).backward()
    torch.testing.assert_close(loss, lr, atol=1e-4, rtol=1e-4)
    tol = dict(atol=2e-3, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,c,ignore", [(50, 1000, -100), (100, 1000, 7), (300, 21, 255), (7, 2, -100)])
def test_cross_entropy_ignore_index_matches_torch(gpu_build, dtype, rows, c, ignore):
    """targets equal to ignore_index (or outside [0, C)) drop their
    row from the loss, the mean and the gradient, as in F.cross_entropy."""
    from vgpu.ops.loss import cross_entropy
    g = torch.Generator().manual_seed(rows + c)
    x = (torch.randn(rows, c, generator=g) * 3).to(dtype).cuda().requires_grad_()
    t = torch.randint(0, c, (rows,), generator=g)
    t[::3] = ignore if ignore >= c or ignore < 0 else t[::3]
    if 0 <= ignore < c:
        t[1::4] = ignore
    t = t.cuda()
    loss = cross_entropy(x, t, ignore_index=ignore)
    (loss * 2.0).backward()
    xr = x.detach().float().requires_grad_()
    lr = torch.nn.functional.cross_entropy(xr, t, ignore_index=ignore)
    (lr * 2.0).backward()
    torch.testing.assert_close(loss, lr, atol=1e-4, rtol=1e-4)
    tol = dict(atol=2e-3, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["channels_last", "nchw"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_pixelwise_cross_entropy_matches_torch(gpu_build, layout, dtype):
    """DeepLab's per-pixel loss (nll_loss2d was ~224 us a step)
    read in place from [B, 21, H, W] logits in either layout, with PyTorch's
    ignore_index=255 convention for void pixels: loss and gradient against
    F.cross_entropy on the fp32 logits."""
    from vgpu.ops.loss import cross_entropy
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(2, 21, 33, 40, generator=g) * 2).to(dtype).cuda()
    if layout == "channels_last":
        x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    t = torch.randint(0, 21, (2, 33, 40), generator=g)
    t[:, ::5, ::7] = 255
    t = t.cuda()
    loss = cross_entropy(x, t, ignore_index=255)
    loss.backward()
    assert x.grad.stride() == x.stride()
    xr = x.detach().float().requires_grad_()
    lr = torch.nn.functional.cross_entropy(xr, t, ignore_index=255)
    lr.backward()
    torch.testing.assert_close(loss, lr, atol=1e-4, rtol=1e-4)
    tol = dict(atol=1e-4, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-7, rtol=1e-4)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)


def _mlp(device, seed=0):
    torch.manual_seed(seed)
    m = torch.nn.Sequential(torch.nn.Linear(1032, 512), torch.nn.Linear(512, 200))
    return m.to(device)


def test_fuse_into_backward_registers_linear_weights_cpu():
    """fp32 CPU: the registered weights never take the skinny kernels, so the
    step is PyTorch's SGD exactly (gradients stay ordinary)."""
    a, b = _mlp("cpu"), _mlp("cpu")
    oa = SGD(a.parameters(), lr=0.1, momentum=0.9)
    assert oa.fuse_into_backward(a) == 2
    ob = torch.optim.SGD(b.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(2, 1032)
    for _ in range(3):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad(set_to_none=True)
            m(x).square().sum().backward()
            o.step()
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(lr=0.1, momentum=0.9), dict(lr=0.05, momentum=0.9, weight_decay=1e-2),
                                dict(lr=0.05, momentum=0.8, nesterov=True),
                                dict(lr=0.1, momentum=0.9, dampening=0.3)])
def test_sgd_in_skinny_backward_bit_exact(gpu_build, kw):
    """native/kernels/skinny.hip SgdJob: the FC weights stepped inside their
    backward give the same bf16 weights, momentum buffers and input gradient
    as the unfused native SGD over a materialised dW, over four steps (the
    first initialises the buffers), and the fused weights' .grad stays None."""
    from vgpu.ops.linear import linear_act
    nets = [_mlp("cuda").to(torch.bfloat16) for _ in range(2)]
    opts = [SGD(n.parameters(), **kw) for n in nets]
    assert opts[1].fuse_into_backward(nets[1]) == 2
    torch.manual_seed(1)
    xs = [torch.randn(2, 1032, device="cuda", dtype=torch.bfloat16) for _ in range(4)]
    dys = [torch.randn(2, 200, device="cuda", dtype=torch.bfloat16) for _ in range(4)]
    for net, opt in zip(nets, opts):
        net.dx = []
        for x, dy in zip(xs, dys):
            opt.zero_grad(set_to_none=True)
            xi = x.clone().requires_grad_()
            y = linear_act(linear_act(xi, net[0], "relu"), net[1])
            y.backward(dy)
            net.dx.append(xi.grad)
            if opt is opts[1]:
                assert net[0].weight.grad is None and net[1].weight.grad is None
                assert net[0].bias.grad is not None
            opt.step()
    for (pa, pb) in zip(nets[0].parameters(), nets[1].parameters()):
        assert torch.equal(pa, pb)
        assert torch.equal(opts[0].state[pa]["momentum_buffer"], opts[1].state[pb]["momentum_buffer"])
    for da, db in zip(nets[0].dx, nets[1].dx):
        assert torch.equal(da, db)
