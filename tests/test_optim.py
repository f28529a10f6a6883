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
