"""Fused NHWC epilogue kernels vs fp32 PyTorch references, and the fused
ResNet-V2 inference runner vs the plain module."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fused(gpu_build):
    from vgpu.ops import fused
    return fused


def _x(shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(shape, generator=g).to(torch.bfloat16).cuda().contiguous(
        memory_format=torch.channels_last)


@pytest.mark.parametrize("shape", [(2, 64, 9, 9), (3, 256, 5, 7), (1, 2048, 3, 3)])
@pytest.mark.parametrize("act", ["none", "relu", "relu6"])
def test_bias_act(fused, shape, act):
    x = _x(shape)
    bias = torch.randn(shape[1]).cuda()
    ref = fused.bias_act_ref(x, bias, act)
    got = fused.bias_act_(x.clone(), bias, act)
    torch.testing.assert_close(got.float(), ref.float(), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("shape", [(2, 64, 9, 9), (4, 512, 3, 5)])
def test_scale_shift_act(fused, shape):
    x = _x(shape, 1)
    sc, sh = torch.rand(shape[1]).cuda() + 0.5, torch.randn(shape[1]).cuda()
    torch.testing.assert_close(fused.scale_shift_act(x, sc, sh).float(),
                               fused.scale_shift_act_ref(x, sc, sh).float(), atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("shape", [(2, 256, 11, 11), (1, 1024, 4, 4)])
def test_add_scale_shift_act(fused, shape):
    a, b = _x(shape, 2), _x(shape, 3)
    sc, sh = torch.rand(shape[1]).cuda() + 0.5, torch.randn(shape[1]).cuda()
    s, y = fused.add_scale_shift_act(a, b, sc, sh)
    s_ref, y_ref = fused.add_scale_shift_act_ref(a, b, sc, sh)
    torch.testing.assert_close(s.float(), s_ref.float(), atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(y.float(), y_ref.float(), atol=2e-2, rtol=1e-2)


def test_rejects_bad_layout(fused):
    x = torch.randn(2, 64, 4, 4, dtype=torch.bfloat16, device="cuda")  # NCHW contiguous
    with pytest.raises(ValueError):
        fused.bias_act_(x, torch.zeros(64, device="cuda"))


def test_fused_resnet_matches_module(gpu_build):
    from vgpu.models.resnet import FusedResNetV2Inference, resnet_v2_50
    torch.manual_seed(0)
    m = resnet_v2_50().cuda().eval()
    # non-trivial BN statistics
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.1, 0.1)
            mod.running_var.uniform_(0.5, 1.5)
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.1, 0.1)
    x = torch.randn(2, 3, 128, 128, device="cuda")
    with torch.no_grad():
        ref = m.float()(x.contiguous(memory_format=torch.channels_last))
    mb = m.to(torch.bfloat16).to(memory_format=torch.channels_last)
    fm = FusedResNetV2Inference(mb)
    got = fm(x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)).float()
    rel = (got - ref).norm() / ref.norm()
    assert rel < 0.05, float(rel)
