"""Numerics of the hand-written gfx950 kernels against plain PyTorch / CPU
references (K2 page gather/scatter, K3 fill/verify, K1 census)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K(gpu_build):
    from vgpu.ops import kernels
    return kernels


def test_fill_matches_cpu_reference(K):
    n = 4096
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    K.fill_pattern(t, 42)
    torch.cuda.synchronize()
    got = t.view(torch.int32).cpu().to(torch.int64) & 0xFFFFFFFF
    ref = K.pattern_reference(n, 42)
    assert torch.equal(got, ref)


def test_verify_detects_corruption(K):
    t = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    K.fill_pattern(t, 3)
    assert K.verify_pattern(t, 3) == 0
    t[12345] ^= 0xFF
    assert K.verify_pattern(t, 3) == 1


@pytest.mark.parametrize("page_bytes,npages,src_pages", [(4096, 100, 1000), (2 << 20, 16, 64)])
def test_gather_scatter_vs_torch(K, page_bytes, npages, src_pages):
    g = torch.Generator(device="cpu").manual_seed(0)
    src = torch.randint(0, 255, (src_pages * page_bytes,), dtype=torch.uint8, generator=g).cuda()
    idx = torch.randperm(src_pages, generator=g)[:npages].cuda()
    dst = torch.empty(npages * page_bytes, dtype=torch.uint8, device="cuda")
    K.gather_pages(dst, src, idx, page_bytes)
    ref = src.view(src_pages, page_bytes)[idx].reshape(-1)
    assert torch.equal(dst, ref)
    back = torch.zeros_like(src)
    K.scatter_pages(back, dst, idx, page_bytes)
    torch.cuda.synchronize()
    assert torch.equal(back.view(src_pages, page_bytes)[idx], src.view(src_pages, page_bytes)[idx])


def test_gather_from_pinned_host(K):
    page = 64 << 10
    host = torch.randint(0, 255, (32 * page,), dtype=torch.uint8).pin_memory()
    idx = torch.tensor([5, 1, 31, 0], dtype=torch.int64, device="cuda")
    dst = torch.empty(4 * page, dtype=torch.uint8, device="cuda")
    K.gather_pages(dst, host, idx, page)
    ref = host.view(32, page)[idx.cpu()].reshape(-1)
    assert torch.equal(dst.cpu(), ref)


def test_census_reports_valid_ids(K):
    xh, ticks = K.census(2048, 1000)
    torch.cuda.synchronize()
    assert int(xh[:, 0].max()) <= 7
    assert bool((ticks >= 1000).all())


@pytest.mark.parametrize("wave", ["1", "0"])
@pytest.mark.parametrize("b,t,e,layers", [(37, 64, 300, 2), (100, 48, 128, 1), (140, 33, 300, 2)])
def test_fused_lstm_matches_fp32(gpu_build, monkeypatch, wave, b, t, e, layers):
    """native/kernels/lstm.hip (+ input-projection GEMM) against torch.nn.LSTM in
    fp32 on the same bf16-rounded weights and inputs; B = 37 leaves a partial
    16-row slice, B = 140 spans two wavefront placement groups (9 row blocks).
    wave=1: a 2-layer stack as one wavefront launch (layer 2 a few steps behind
    layer 1, its input projection inside the kernel); wave=0: layer by layer."""
    import torch
    monkeypatch.setenv("VGPU_LSTM_WAVE", wave)
    from vgpu.ops import lstm as fused
    torch.manual_seed(0)
    ref = torch.nn.LSTM(e, 128, num_layers=layers, batch_first=True).cuda()
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_((p * 2.0).to(torch.bfloat16).float())
    x = (torch.randn(b, t, e, device="cuda") * 0.5).to(torch.bfloat16)
    with torch.no_grad():
        want = ref(x.float())[0][:, -1]
        got = fused.lstm_last_hidden(ref.to(torch.bfloat16), x).float()
    torch.testing.assert_close(got, want, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("wave", ["1", "0"])
def test_fused_lstm_training_grads_match_fp32(gpu_build, monkeypatch, wave):
    """Forward + backward-through-time kernels (LSTM2Fn wavefront, or
    LSTMLayerFn per layer) against torch.nn.LSTM in fp32 on the same
    bf16-rounded weights: every weight / bias gradient, and the input gradient
    of a 2-layer stack."""
    import torch
    monkeypatch.setenv("VGPU_LSTM_WAVE", wave)
    from vgpu.ops import lstm as fused
    torch.manual_seed(1)
    b, t, e = 10, 40, 300
    ref = torch.nn.LSTM(e, 128, num_layers=2, batch_first=True).cuda()
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_((p * 2.0).to(torch.bfloat16).float())
    x = (torch.randn(b, t, e, device="cuda") * 0.5).to(torch.bfloat16)
    head = torch.randn(128, device="cuda")
    xr = x.float().requires_grad_(True)
    (ref(xr)[0][:, -1] @ head).sum().backward()
    mod = torch.nn.LSTM(e, 128, num_layers=2, batch_first=True).cuda().to(torch.bfloat16)
    with torch.no_grad():
        for p, q in zip(mod.parameters(), ref.parameters()):
            p.copy_(q.to(torch.bfloat16))
    xb = x.clone().requires_grad_(True)
    (fused.lstm_forward_train(mod, xb)[:, -1].float() @ head).sum().backward()
    errs = {}
    for (name, p), q in zip(mod.named_parameters(), ref.parameters()):
        scale = q.grad.abs().max().item() + 1e-6
        errs[name] = (p.grad.float() - q.grad).abs().max().item() / scale
    print("max-norm relative gradient error vs fp32:", {k: round(v, 4) for k, v in errs.items()})
    assert max(errs.values()) < 0.05, errs
    err = (xb.grad.float() - xr.grad).abs().max().item() / (xr.grad.abs().max().item() + 1e-6)
    assert err < 0.05, ("x", err)
