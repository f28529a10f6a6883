"""vgpu.ops.interp: the interpolation matrices reproduce PyTorch's bilinear
resize (align_corners=False) forward and backward exactly (CPU, fp64)."""
import pytest
import torch
import torch.nn.functional as F

from vgpu.ops.interp import interp_matrix


@pytest.mark.parametrize("ih,iw,oh,ow", [(24, 24, 384, 384), (1, 1, 24, 24), (7, 5, 20, 13), (16, 16, 8, 8)])
def test_interp_matrices_match_pytorch(ih, iw, oh, ow):
    g = torch.Generator().manual_seed(ih * 100 + ow)
    x = torch.randn(2, 3, ih, iw, dtype=torch.float64, generator=g)
    ah = interp_matrix(oh, ih, "cpu").double()
    aw = interp_matrix(ow, iw, "cpu").double()
    y = F.interpolate(x, size=(oh, ow), mode="bilinear", align_corners=False)
    torch.testing.assert_close(ah @ x @ aw.t(), y, atol=1e-6, rtol=1e-6)
    xr = x.clone().requires_grad_(True)
    dy = torch.randn(y.shape, dtype=torch.float64, generator=g)
    F.interpolate(xr, size=(oh, ow), mode="bilinear", align_corners=False).backward(dy)
    torch.testing.assert_close(ah.t() @ dy @ aw, xr.grad, atol=1e-5, rtol=1e-6)
