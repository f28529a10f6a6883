"""Model definitions on the CPU: the BN+activation entry point keeps the
module semantics off the native path, and every ai-benchmark workload builds
and runs a (shrunken) forward/backward."""
import pytest
import torch
import torch.nn.functional as F


def test_bn_act_cpu_fallback_matches_module():
    from vgpu.ops.bn import bn_act, native_eligible
    bn = torch.nn.BatchNorm2d(16).train()
    ref = torch.nn.BatchNorm2d(16).train()
    x = torch.randn(2, 16, 5, 5)
    assert not native_eligible(x, bn)
    for act, f in (("relu", F.relu), ("relu6", F.relu6), ("none", lambda t: t)):
        torch.testing.assert_close(bn_act(x, bn, act), f(ref(x)))
    torch.testing.assert_close(bn.running_mean, ref.running_mean)
    assert int(bn.num_batches_tracked) == int(ref.num_batches_tracked) == 3
    with pytest.raises(ValueError):
        bn_act(x, bn, "gelu")


def test_conv_bn_act_keeps_sequential_layout():
    from vgpu.models.vision import _conv_bn
    m = _conv_bn(8, 16, 3)
    assert [k for k in m.state_dict()][:2] == ["0.weight", "1.weight"]
    x = torch.randn(1, 8, 6, 6)
    torch.testing.assert_close(m(x), F.relu6(m[1](m[0](x))))
    m2 = _conv_bn(8, 16, 1, act=False).eval()
    torch.testing.assert_close(m2(x), m2[1](m2[0](x)))


def test_resnet_v2_training_step_cpu():
    from vgpu.models.resnet import ResNetV2
    m = ResNetV2([1, 1, 1, 1], num_classes=10).train()
    x = torch.randn(2, 3, 64, 64)
    loss = F.cross_entropy(m(x), torch.tensor([1, 2]))
    loss.backward()
    assert all(p.grad is not None for p in m.parameters())
    assert int(m.blocks[0].bn_in.num_batches_tracked) == 1


def test_batched_step_counters_match_per_layer_updates():
    """num_batches_tracked deferred to one multi-tensor add per forward: same
    values as the per-layer update, nested blocks flush once."""
    import torch
    from torch import nn
    from vgpu.ops import bn as B

    mods = [nn.BatchNorm2d(8) for _ in range(3)]
    with B.batched_step_counters():
        for m in mods:
            B._counters.pending.append(m.num_batches_tracked)
        with B.batched_step_counters():
            B._counters.pending.append(mods[0].num_batches_tracked)
        assert all(int(m.num_batches_tracked) == 0 for m in mods)  # deferred
    assert [int(m.num_batches_tracked) for m in mods] == [2, 1, 1]
    assert getattr(B._counters, "pending", None) is None


def test_deeplab_channel_padding_is_exact():
    """DeepLab's MobileNet-V2 stores its channel dims padded to multiples of 64
    (so every 1x1 conv runs on the native MFMA kernels).  The padded model with
    an unpadded model's weights computes the same output and loss, gives every
    real parameter the same gradient, gives the padding exactly zero gradient,
    and keeps the padding at zero through SGD steps (fp32, CPU)."""
    import torch
    import torch.nn.functional as F
    from vgpu.models.vision import DeepLabV3
    torch.manual_seed(0)
    ref = DeepLabV3(num_classes=5, pad_channels=1).train()
    pad = DeepLabV3(num_classes=5).train()
    pad.load_unpadded(ref)
    x = torch.randn(2, 3, 64, 64)
    tgt = torch.randint(0, 5, (2, 64, 64))
    opt_r = torch.optim.SGD(ref.parameters(), lr=0.01, momentum=0.9)
    opt_p = torch.optim.SGD(pad.parameters(), lr=0.01, momentum=0.9)
    for step in range(3):
        for o in (opt_r, opt_p):
            o.zero_grad()
        lr_, lp = F.cross_entropy(ref(x), tgt), F.cross_entropy(pad(x), tgt)
        # step 0 strict; after an SGD step the padded convs' different summation
        # order (1e-7) is amplified by the batch-norms over 4x4 maps (see below)
        torch.testing.assert_close(lp, lr_, rtol=1e-2 if step else 1e-5, atol=1e-6)
        lr_.backward()
        lp.backward()
        pp = dict(pad.named_parameters())
        for name, p in ref.named_parameters():
            q = pp[name]
            sl = tuple(slice(0, n) for n in p.shape)
            if step == 0:
                # (later steps are not compared: the 1e-7 summation-order differences of
                # the padded convs, amplified by 50 batch-norms over 4x4 maps, reach ~1e-2)
                torch.testing.assert_close(q.grad[sl], p.grad, rtol=1e-4, atol=1e-6, msg=f"{step} {name}")
            if q.shape != p.shape:
                mask = torch.ones_like(q, dtype=torch.bool)
                mask[sl] = False
                assert float(q.grad[mask].abs().max()) == 0.0, (step, name)
        opt_r.step()
        opt_p.step()
    for name, p in ref.named_parameters():
        q = pp[name]
        if q.shape != p.shape:
            mask = torch.ones_like(q, dtype=torch.bool)
            mask[tuple(slice(0, n) for n in p.shape)] = False
            assert float(q.detach()[mask].abs().max()) == 0.0, name


def test_space_to_batch_dilated_conv_identity():
    """DeepLab's ASPP training path (vgpu.models.vision._atrous_conv): a 3x3
    conv with dilation = padding = d equals a plain 3x3 / padding 1 conv on the
    d x d space-to-batch sub-images, for maps that d divides and maps it does
    not (zero-padded up), channels-last in and out (fp32, CPU)."""
    import torch
    import torch.nn.functional as F
    from vgpu.models.vision import _batch_to_space, _space_to_batch
    g = torch.Generator().manual_seed(0)
    for n, c, h, w, d in [(1, 8, 24, 24, 6), (2, 8, 24, 24, 12), (1, 8, 24, 24, 18), (2, 4, 32, 30, 18),
                          (1, 4, 7, 9, 2)]:
        x = torch.randn(n, c, h, w, generator=g).contiguous(memory_format=torch.channels_last)
        wt = torch.randn(5, c, 3, 3, generator=g)
        ref = F.conv2d(x, wt, padding=d, dilation=d)
        xs = _space_to_batch(x, d)
        assert xs.is_contiguous(memory_format=torch.channels_last)
        assert xs.shape == (d * d * n, c, -(-h // d), -(-w // d))
        y = F.conv2d(xs, wt, padding=1).contiguous(memory_format=torch.channels_last)
        got = _batch_to_space(y, d, n, h, w)
        assert got.is_contiguous(memory_format=torch.channels_last)
        torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)
