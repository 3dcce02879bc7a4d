"""rmbx_linear_f32x6 (fp32-accurate GEMM on the bf16 matrix cores: both operands split into three
bf16 pieces, six piece products accumulated in f32) against an f64 product of the same f32
operands, beside the device's own f32 GEMM (hipBLASLt, the path it replaces in the fp32 ACT
transformer).  The bar is the f32 GEMM error class: max |err| <= 4e-6 * max |ref| and no worse
than 2x hipBLASLt's f32 GEMM error on the same inputs (measured ~0.3-0.8e-6 vs 1-2e-6)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _err(got, ref):
    return ((got.double() - ref).abs().max() / ref.abs().max()).item()


@torch.no_grad()
def test_split_bf16x3_exact():
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device="cpu").manual_seed(0)
    w = torch.randn(4096, generator=g) * torch.logspace(-30, 30, 4096)
    w[:4] = torch.tensor([0.0, -0.0, 1.0, -3.0])
    p = K.split_bf16x3(w.to(DEV)).cpu()
    assert p.shape == (3, 4096) and p.dtype == torch.bfloat16
    s = p[0].double() + p[1].double() + p[2].double()
    torch.testing.assert_close(s, w.double(), rtol=0, atol=0)
    # each level rounded to nearest: |x1| <= 2^-8 |x0|, |x2| <= 2^-8 |x1| (normal range)
    nz = p[0].float().abs() > 1e-30
    assert (p[1].float().abs()[nz] <= p[0].float().abs()[nz] * 2.0 ** -8).all()


@torch.no_grad()
@pytest.mark.parametrize("M,N,K,relu,bias", [(1, 128, 32, False, False), (1000, 384, 512, True, True),
                                             (257, 3200, 512, True, True), (3000, 512, 3200, False, True),
                                             (5000, 1536, 512, False, True)])
def test_linear_f32x6_vs_f64(M, N, K, relu, bias):
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    b = torch.randn(N, generator=g).to(DEV) if bias else None
    got = K_.linear_f32x6(x, K_.split_bf16x3(w), b, relu=relu)
    ref = x.double() @ w.double().t()
    if bias:
        ref = ref + b.double()
    if relu:
        ref = ref.clamp_min(0)
    base = F.linear(x, w, b)
    if relu:
        base = base.clamp_min(0)
    e, e32 = _err(got, ref), _err(base, ref)
    assert got.shape == (M, N) and torch.isfinite(got).all()
    assert e <= 4e-6 and e <= 2 * e32 + 1e-7, (e, e32)


@torch.no_grad()
def test_linear_f32x6_strided_rows_and_plane_slice():
    """x as a column slice of a wider activation (row stride > K) and W as a row slice of a split
    in_proj_weight, as the fused MHA uses them."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(7)
    big = torch.randn(700, 1536, generator=g).to(DEV)
    x = big[:, 512:1024]
    w = (torch.randn(1536, 512, generator=g) / 512 ** 0.5).to(DEV)
    b = torch.randn(1536, generator=g).to(DEV)
    planes = K_.split_bf16x3(w)
    got = K_.linear_f32x6(x, planes[:, 512:1024], b[512:1024])
    ref = x.double() @ w[512:1024].double().t() + b[512:1024].double()
    assert _err(got, ref) <= 4e-6


@torch.no_grad()
def test_linear_f32x6_rejects_bad_shapes():
    from robomanipbaselines_amd import kernels as K_

    x = torch.randn(8, 48, device=DEV)
    with pytest.raises((ValueError, RuntimeError)):
        K_.linear_f32x6(x, K_.split_bf16x3(torch.randn(128, 48, device=DEV)))
    with pytest.raises((ValueError, RuntimeError)):
        K_.linear_f32x6(torch.randn(8, 64, device=DEV), K_.split_bf16x3(torch.randn(100, 64, device=DEV)))
