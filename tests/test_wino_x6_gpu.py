"""The explicit Winograd F(4x4, 3x3) conv of the 256/512-channel fp32 trunk layers (input transform
pass, 36 fp32-accurate bf16x6 position GEMMs, output transform + epilogue pass) against an f64
F.conv2d, beside the fused F(4x4) f32-MFMA kernel it replaces at those widths.  Bar: the fused
kernel's class, |err| <= 4e-5 * max |ref| (F(4x4)'s transform coefficients up to 8 amplify the f32
rounding; measured ~1e-5 for both)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@torch.no_grad()
@pytest.mark.parametrize("n,C,H,W,res,relu", [(2, 256, 30, 40, True, True), (3, 512, 15, 20, False, True),
                                              (1, 256, 7, 9, True, False), (2, 512, 13, 18, True, True)])
def test_wino4_x6_vs_f64(n, C, H, W, res, relu):
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device="cpu").manual_seed(C + H)
    x = torch.randn(n, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / (9 * C) ** 0.5
    b = torch.randn(C, generator=g)
    r = torch.randn(n, C, H, W, generator=g) if res else None
    cl = torch.channels_last
    got = K.conv3x3_wino4_x6(x.to(DEV).contiguous(memory_format=cl), K.pack_wino4_x6(w.to(DEV)), b.to(DEV),
                             relu=relu, res=None if r is None else r.to(DEV).contiguous(memory_format=cl))
    assert got.shape == x.shape and got.is_contiguous(memory_format=cl)
    ref = F.conv2d(x.double(), w.double(), b.double(), 1, 1)
    if r is not None:
        ref = ref + r.double()
    if relu:
        ref = ref.clamp_min(0)
    fused = K.conv3x3_winograd4_f32(x.to(DEV).contiguous(memory_format=cl), K.pack_winograd4_f32(w.to(DEV)), b.to(DEV),
                                    relu=relu, res=None if r is None else r.to(DEV).contiguous(memory_format=cl))
    scale = ref.abs().max()
    e = ((got.cpu().double() - ref).abs().max() / scale).item()
    ef = ((fused.cpu().double() - ref).abs().max() / scale).item()
    print(f"\nC={C} {H}x{W}: explicit x6 {e:.2e}, fused f32 {ef:.2e}")
    assert e <= 4e-5, (e, ef)
