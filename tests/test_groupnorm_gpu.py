"""rmbx_groupnorm_act (the DiffusionPolicy / DP3 UNet Conv1dBlock's GroupNorm + Mish in one pass)
against torch's group_norm + mish in f64 on the same f32 inputs: within the f32 error class (the register-resident path for spans up to 2,048 values and the three-pass one above)
(1e-5 absolute on unit-scale outputs; torch's own f32 ops measured ~1e-6), with and without the
Mish, in place, and at the UNet's shapes (B = 2048, C 256-1024, T 16 / 8 / 4)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("B,C,T,G", [(2048, 256, 16, 8), (2048, 1024, 4, 8), (2048, 512, 8, 8), (7, 64, 5, 8),
                                     (3, 96, 33, 4), (2, 64, 300, 2)])
@pytest.mark.parametrize("mish", [True, False])
def test_groupnorm_act_vs_f64(B, C, T, G, mish):
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator().manual_seed(B + C + T)
    x = (3.0 * torch.randn(B, C, T, generator=g) + 0.5).to(DEV)
    w = (0.5 + torch.rand(C, generator=g)).to(DEV)
    b = (0.2 * torch.randn(C, generator=g)).to(DEV)
    got = K.groupnorm_act(x, w, b, G, 1e-5, mish=mish)
    ref = F.group_norm(x.double(), G, w.double(), b.double(), 1e-5)
    if mish:
        ref = F.mish(ref)
    err = (got.double() - ref).abs().max().item()
    assert err < 1e-5, err
    t32 = F.group_norm(x, G, w, b, 1e-5)
    t32 = F.mish(t32) if mish else t32
    assert err <= 4 * (t32.double() - ref).abs().max().item() + 2e-6


@pytest.mark.parametrize("B,C,T,G", [(2048, 256, 16, 8), (2048, 1024, 4, 8), (2, 64, 300, 2)])
def test_groupnorm_act_time_major_input(B, C, T, G):
    """The conv GEMM's [B, T, C] rows in, [B, C, T] out: the same values as the [B, C, T] input."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator().manual_seed(B + T)
    x = (2.0 * torch.randn(B, C, T, generator=g)).to(DEV)
    w = (0.5 + torch.rand(C, generator=g)).to(DEV)
    b = (0.2 * torch.randn(C, generator=g)).to(DEV)
    got = K.groupnorm_act(x.transpose(1, 2).contiguous(), w, b, G, 1e-5, time_major=True)
    assert got.shape == (B, C, T)
    ref = F.mish(F.group_norm(x.double(), G, w.double(), b.double(), 1e-5))
    assert (got.double() - ref).abs().max().item() < 1e-5


def test_groupnorm_act_in_place_and_checks():
    from robomanipbaselines_amd import kernels as K

    x = torch.randn(16, 128, 16, device=DEV)
    w = torch.rand(128, device=DEV) + 0.5
    b = torch.randn(128, device=DEV)
    want = K.groupnorm_act(x.clone(), w, b, 8)
    y = x.clone()
    out = K.groupnorm_act(y, w, b, 8, out=y)
    assert out.data_ptr() == y.data_ptr() and torch.equal(out, want)
    with pytest.raises(ValueError):
        K.groupnorm_act(torch.randn(2, 12, 4, device=DEV), torch.ones(12, device=DEV), torch.zeros(12, device=DEV), 8)
    # a caller-supplied out of the wrong shape, dtype or layout is rejected before the launch
    for bad in (torch.empty(16, 128, 8, device=DEV), torch.empty(16, 128, 16, device=DEV, dtype=torch.float64),
                torch.empty(16, 16, 128, device=DEV).transpose(1, 2)):
        with pytest.raises(ValueError):
            K.groupnorm_act(x, w, b, 8, out=bad)
