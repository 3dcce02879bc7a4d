"""The fp32-accurate GEMMs on the matrix cores against an f64 product of the same f32 operands,
beside the device's own f32 GEMM (hipBLASLt, the path they replace in the fp32 ACT transformer):
rmbx_linear_f32x6 (bf16x6: both operands split into three bf16 pieces, six piece products
accumulated in f32) and rmbx_linear_f16x3 (f16x3: two f16 pieces, the low one scaled by 2^11, three
products; per-row power-of-two weight scales and a per-block re-run on a scaled copy for
activations outside f16's comfortable range).  The bar is the f32 GEMM error class: max |err| <=
4e-6 * max |ref|, and for the linear layers no worse than 2x hipBLASLt's f32 GEMM error on the same
inputs (measured ~0.3-0.8e-6 vs 1-2e-6).  The implicit-GEMM convolutions (rmbx_conv2d_f16x3, the
default packing, and rmbx_conv2d_f32x6) are held to the 4e-6 bar against an f64 F.conv2d."""

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


def _pack(form):
    from robomanipbaselines_amd import kernels as K_

    return K_.split_bf16x3 if form == "bf16x6" else K_.split_f16x2


@torch.no_grad()
def test_split_f16x2_pieces_and_scales():
    """W[n] = scale[n] (hi + lo) to 2^-22 of each element (2^-36 of the row max for elements below
    2^-16 of it, whose low piece is an f16 subnormal), scale[n] a power of two with the scaled row
    max in [2^13, 2^14); zero rows keep scale 1."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(1)
    w = torch.randn(64, 300, generator=g) * torch.logspace(-20, 20, 64)[:, None]
    w[5] = 0.0
    w[6, :7] = torch.tensor([0.0, -0.0, 1e-30, 65504.0, -1e-5, 3.0, 1e-12])
    p = K_.split_f16x2(w.to(DEV))
    assert p.planes.shape == (2, 64, 300) and p.planes.dtype == torch.float16 and p.scale.shape == (64,)
    hi, lo, sc = p.planes[0].double().cpu(), p.planes[1].double().cpu(), p.scale.double().cpu()
    rec = sc[:, None] * (hi + lo)
    wd = w.double()
    rowmax = wd.abs().amax(1, keepdim=True)
    assert ((rec - wd).abs() <= wd.abs() * 2.0 ** -22 + rowmax * 2.0 ** -36).all()
    assert torch.equal(torch.log2(sc).round(), torch.log2(sc))  # powers of two
    m = (hi.abs().amax(1))[rowmax[:, 0] > 0]
    assert ((m >= 2 ** 13) & (m <= 2 ** 14)).all()
    assert sc[5] == 1.0 and (rec[5] == 0).all()


@torch.no_grad()
@pytest.mark.parametrize("form", ["bf16x6", "f16x3"])
@pytest.mark.parametrize("M,N,K,relu,bias", [(1, 128, 32, False, False), (1000, 384, 512, True, True),
                                             (257, 3200, 512, True, True), (3000, 512, 3200, False, True),
                                             (5000, 1536, 512, False, True)])
def test_linear_f32x6_vs_f64(form, M, N, K, relu, bias):
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    b = torch.randn(N, generator=g).to(DEV) if bias else None
    got = K_.linear_f32x6(x, _pack(form)(w), b, relu=relu)
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
@pytest.mark.parametrize("form", ["bf16x6", "f16x3"])
def test_linear_f32x6_strided_rows_and_plane_slice(form):
    """x as a column slice of a wider activation (row stride > K) and W as a row slice of a split
    in_proj_weight, as the fused MHA uses them."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(7)
    big = torch.randn(700, 1536, generator=g).to(DEV)
    x = big[:, 512:1024]
    w = (torch.randn(1536, 512, generator=g) / 512 ** 0.5).to(DEV)
    b = torch.randn(1536, generator=g).to(DEV)
    planes = _pack(form)(w)
    got = K_.linear_f32x6(x, planes[:, 512:1024], b[512:1024])
    ref = x.double() @ w[512:1024].double().t() + b[512:1024].double()
    assert _err(got, ref) <= 4e-6


@torch.no_grad()
@pytest.mark.parametrize("form", ["bf16x6", "f16x3"])
def test_linear_f32x6_rejects_bad_shapes(form):
    from robomanipbaselines_amd import kernels as K_

    x = torch.randn(8, 48, device=DEV)
    with pytest.raises((ValueError, RuntimeError)):
        K_.linear_f32x6(x, _pack(form)(torch.randn(128, 48, device=DEV)))
    with pytest.raises((ValueError, RuntimeError)):
        K_.linear_f32x6(torch.randn(8, 64, device=DEV), _pack(form)(torch.randn(100, 64, device=DEV)))


@torch.no_grad()
@pytest.mark.parametrize("case", ["huge", "tiny", "mixed_blocks", "near_f16_max", "zero_rows"])
def test_linear_f16x3_activation_range(case):
    """f16's range is handled exactly: a row whose |a| max lies outside [2^-6, 2^15] is re-run on a
    power-of-two-scaled copy.  Every 256-row block of rows stays in the f32 GEMM error class
    relative to that block's own result scale, including activations far beyond f16's max
    (65504) and far below its normal range."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(11)
    M, N, K = 1024, 256, 512
    x = torch.randn(M, K, generator=g)
    scale = {"huge": torch.full((M, 1), 1e7), "tiny": torch.full((M, 1), 1e-9),
             "mixed_blocks": torch.tensor([1e6, 1e-7, 1.0, 3e4]).repeat_interleave(256)[:, None],
             "near_f16_max": torch.full((M, 1), 32000.0 / 4.5), "zero_rows": torch.ones(M, 1)}[case]
    x = x * scale
    if case == "zero_rows":
        x[::3] = 0.0
    w = torch.randn(N, K, generator=g) / K ** 0.5
    got = K_.linear_f32x6(x.to(DEV), K_.split_f16x2(w.to(DEV))).cpu().double()
    ref = x.double() @ w.double().t()
    assert torch.isfinite(got).all()
    for blk in range(M // 256):
        r = slice(256 * blk, 256 * blk + 256)
        den = ref[r].abs().max()
        if den == 0:
            assert (got[r] == 0).all()
            continue
        assert ((got[r] - ref[r]).abs().max() / den).item() <= 4e-6, (case, blk)


@torch.no_grad()
def test_linear_f16x3_rows_independent_of_their_block():
    """A row's f16x3 result is bitwise the same whether its 256-row block holds rows that need the
    range re-run (1e8, 1e-9) or not: the re-run keeps in-range rows at scale 1."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(13)
    x = torch.randn(512, 512, generator=g)
    x[5] *= 1e8
    x[300] *= 1e-9
    w = K_.split_f16x2((torch.randn(384, 512, generator=g) / 512 ** 0.5).to(DEV))
    xd = x.to(DEV)
    full = K_.linear_f32x6(xd, w)
    keep = [i for i in range(512) if i not in (5, 300)]
    alone = K_.linear_f32x6(xd[keep].contiguous(), w)
    assert torch.equal(full[keep], alone)
    for r in (5, 300):
        one = K_.linear_f32x6(xd[r:r + 1].contiguous(), w)
        assert torch.equal(full[r:r + 1], one)


@torch.no_grad()
def test_linear_f16x3_weight_range_and_non_finite_inputs():
    """Weight rows from 1e-12 to 1e12 (per-row power-of-two scales) stay in the f32 error class per
    output column; an inf / NaN activation makes its own output row non-finite as f32 does, and
    leaves the other rows exact to the f32 class."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(12)
    M, N, K = 600, 256, 256
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) * torch.logspace(-12, 12, N)[:, None]
    got = K_.linear_f32x6(x.to(DEV), K_.split_f16x2(w.to(DEV))).cpu().double()
    ref = x.double() @ w.double().t()
    colmax = ref.abs().amax(0)
    assert ((got - ref).abs().amax(0) / colmax).max().item() <= 4e-6
    x[3, 7] = float("inf")
    x[400, 9] = float("nan")
    got = K_.linear_f32x6(x.to(DEV), K_.split_f16x2(w.to(DEV))).cpu().double()
    base = (x @ w.t()).double()
    assert torch.equal(torch.isfinite(got).all(1), torch.isfinite(base).all(1))
    ok = torch.isfinite(base).all(1)
    ref = x[ok].double() @ w.double().t()
    assert ((got[ok] - ref).abs().amax(0) / ref.abs().amax(0)).max().item() <= 4e-6


def _conv_ref(x, w, b, stride, pad, relu, res):
    ref = F.conv2d(x.double(), w.double(), None if b is None else b.double(), stride, pad)
    if res is not None:
        ref = ref + res.double()
    return ref.clamp_min(0) if relu else ref


@torch.no_grad()
@pytest.mark.parametrize("n,C,H,W,Cout,k,stride,pad,relu,res,bias", [
    (2, 64, 17, 23, 128, 3, 2, 1, True, False, True),     # layer-2 c1 shape class, odd sizes
    (3, 128, 15, 20, 256, 1, 2, 0, False, False, False),  # 1x1 downsample
    (2, 256, 9, 11, 512, 3, 2, 1, True, False, True),
    (2, 64, 12, 16, 128, 3, 1, 1, True, True, True),      # stride 1 with a residual
])
@pytest.mark.parametrize("form", ["bf16x6", "f16x3"])
def test_conv2d_f32x6_vs_f64(monkeypatch, form, n, C, H, W, Cout, k, stride, pad, relu, res, bias):
    from robomanipbaselines_amd import kernels as K_

    monkeypatch.setattr(K_, "F32_PIECES", form)
    g = torch.Generator(device="cpu").manual_seed(n * 1000 + C + k)
    x = torch.randn(n, C, H, W, generator=g)
    w = torch.randn(Cout, C, k, k, generator=g) / (C * k * k) ** 0.5
    b = torch.randn(Cout, generator=g) if bias else None
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    r = torch.randn(n, Cout, Ho, Wo, generator=g) if res else None
    cl = torch.channels_last
    got = K_.conv2d_f32x6(x.to(DEV).contiguous(memory_format=cl), K_.pack_conv_f32x6(w.to(DEV)),
                          None if b is None else b.to(DEV), k, stride, pad, relu=relu,
                          res=None if r is None else r.to(DEV).contiguous(memory_format=cl))
    assert got.shape == (n, Cout, Ho, Wo) and got.is_contiguous(memory_format=cl)
    ref = _conv_ref(x, w, b, stride, pad, relu, r)
    base = F.conv2d(x.to(DEV), w.to(DEV), None if b is None else b.to(DEV), stride, pad).cpu()
    if r is not None:
        base = base + r
    if relu:
        base = base.clamp_min(0)
    e, e32 = _err(got.cpu(), ref), _err(base, ref)
    # the f32-GEMM error class (sequential f32 accumulation over K = KH*KW*C up to 2304; MIOpen's
    # direct fp32 conv sums in a different order and can land lower, ~2e-7 here)
    assert e <= 4e-6, (e, e32)


@torch.no_grad()
def test_conv2d_f32x6_trunk_shape_8_frames():
    """The layer-2 stride-2 conv at the policy's 120x160 feature size (8 frames), f64 reference."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(8, 64, 120, 160, generator=g).clamp_min(0)
    w = torch.randn(128, 64, 3, 3, generator=g) / (64 * 9) ** 0.5
    b = torch.randn(128, generator=g)
    got = K_.conv2d_f32x6(x.to(DEV).contiguous(memory_format=torch.channels_last), K_.pack_conv_f32x6(w.to(DEV)),
                          b.to(DEV), 3, 2, 1, relu=True)
    assert _err(got.cpu(), _conv_ref(x, w, b, 2, 1, True, None)) <= 4e-6


@torch.no_grad()
@pytest.mark.parametrize("n,C,H,W,Cout,k,stride,pad,bias", [(3, 3, 37, 45, 64, 7, 2, 3, False),
                                                          (2, 3, 216, 288, 64, 7, 2, 3, True),
                                                          (2, 4, 9, 11, 32, 3, 1, 1, True)])
def test_conv2d_direct_f32_vs_f64(n, C, H, W, Cout, k, stride, pad, bias):
    """rmbx_conv2d_direct_f32 (the diffusion policy's 3-channel stem): f32 FMA in a fixed order,
    deterministic, vs an f64 F.conv2d (bar 1e-5 relative; K <= 196 terms)."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(H * W)
    x = torch.randn(n, C, H, W, generator=g)
    w = torch.randn(Cout, C, k, k, generator=g) / (C * k * k) ** 0.5
    b = torch.randn(Cout, generator=g) if bias else None
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    got = K_.conv2d_direct_f32(xd, w.to(DEV), None if b is None else b.to(DEV), stride, pad)
    again = K_.conv2d_direct_f32(xd, w.to(DEV), None if b is None else b.to(DEV), stride, pad)
    assert torch.equal(got, again)
    ref = F.conv2d(x.double(), w.double(), None if b is None else b.double(), stride, pad)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=torch.channels_last)
    assert _err(got.cpu(), ref) <= 1e-5


@torch.no_grad()
@pytest.mark.parametrize("M,N,K", [(5000, 3200, 512), (3000, 512, 3200), (257, 384, 96)])
def test_gemm_profiling_variants_equal_default(monkeypatch, M, N, K):
    """The RMBX_GEMM_VAR schedule variants that keep the arithmetic (stagger 80, groups of 16 row
    tiles 18, scalar epilogue 0) give the default's output bit for bit."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(M + 5 * N)
    x = torch.randn(M, K, generator=g).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    planes = K_.split_bf16x3(w)
    want = K_.linear_f32x6(x, planes, b, relu=True)
    for var in ("80", "18", "0"):
        monkeypatch.setenv("RMBX_GEMM_VAR", var)
        got = K_.linear_f32x6(x, planes, b, relu=True)
        torch.cuda.synchronize()
        assert torch.equal(got, want), var


@torch.no_grad()
@pytest.mark.parametrize("form", ["bf16x6", "f16x3"])
@pytest.mark.parametrize("n,C,H,W,Cout,res,relu", [(2, 256, 30, 40, 256, True, True), (3, 512, 15, 20, 512, False, True)])
def test_winograd4_explicit_position_gemms_vs_f64(monkeypatch, form, n, C, H, W, Cout, res, relu):
    """The explicit Winograd F(4x4) conv of the 256/512-channel layers (input transform, 36 batched
    position GEMMs, output transform) in both piece forms against an f64 F.conv2d."""
    from robomanipbaselines_amd import kernels as K_

    monkeypatch.setattr(K_, "F32_PIECES", form)
    g = torch.Generator(device="cpu").manual_seed(C + H)
    x = torch.randn(n, C, H, W, generator=g).clamp_min(0)
    w = torch.randn(Cout, C, 3, 3, generator=g) / (C * 9) ** 0.5
    b = torch.randn(Cout, generator=g)
    r = torch.randn(n, Cout, H, W, generator=g) if res else None
    cl = torch.channels_last
    planes = K_.pack_wino4_x6(w.to(DEV))
    assert isinstance(planes, K_.F16x3Planes) == (form == "f16x3")
    got = K_.conv3x3_wino4_x6(x.to(DEV).contiguous(memory_format=cl), planes, b.to(DEV), relu=relu,
                              res=None if r is None else r.to(DEV).contiguous(memory_format=cl))
    # Winograd's transforms add their own f32 rounding (~1e-6 relative at these sizes)
    assert _err(got.cpu(), _conv_ref(x, w, b, 1, 1, relu, r)) <= 1e-5


@torch.no_grad()
@pytest.mark.parametrize("M,N,K,relu", [(700, 64, 576, True), (1000, 192, 512, False), (257, 320, 96, True)])
def test_linear_f16x3_narrow_tile_vs_f64(M, N, K, relu):
    """The f16x3 form's 64-column tile (N % 128 != 0) against an f64 product, beside hipBLASLt f32."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(M + N)
    x = torch.randn(M, K, generator=g).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    got = K_.linear_f32x6(x, K_.split_f16x2(w), b, relu=relu)
    ref = x.double() @ w.double().t() + b.double()
    base = F.linear(x, w, b)
    if relu:
        ref, base = ref.clamp_min(0), base.clamp_min(0)
    e, e32 = _err(got, ref), _err(base, ref)
    assert got.shape == (M, N) and (e <= 4e-6 and e <= 2 * e32 + 1e-7), (e, e32)


@torch.no_grad()
@pytest.mark.parametrize("n,H,W,res", [(3, 30, 41, True), (2, 120, 160, True), (4, 17, 23, False)])
def test_conv2d_f16x3_64_channels_vs_f64(monkeypatch, n, H, W, res):
    """The ResNet layer-1 conv shape (64 -> 64, 3x3, stride 1, bias + residual + ReLU) on the f16x3
    implicit GEMM's 64-column tile against an f64 F.conv2d."""
    from robomanipbaselines_amd import kernels as K_

    monkeypatch.setattr(K_, "F32_PIECES", "f16x3")
    g = torch.Generator(device="cpu").manual_seed(H * W)
    x = torch.randn(n, 64, H, W, generator=g).clamp_min(0)
    w = torch.randn(64, 64, 3, 3, generator=g) / (64 * 9) ** 0.5
    b = torch.randn(64, generator=g)
    r = torch.randn(n, 64, H, W, generator=g) if res else None
    cl = torch.channels_last
    got = K_.conv2d_f32x6(x.to(DEV).contiguous(memory_format=cl), K_.pack_conv_f32x6(w.to(DEV)), b.to(DEV), 3, 1, 1,
                          relu=True, res=None if r is None else r.to(DEV).contiguous(memory_format=cl))
    assert _err(got.cpu(), _conv_ref(x, w, b, 1, 1, True, r)) <= 4e-6


@torch.no_grad()
@pytest.mark.parametrize("M,N,K", [(5000, 3200, 512), (3000, 512, 3200), (257, 384, 96)])
def test_gemm_f16x3_three_stage_variant_equals_default(monkeypatch, M, N, K):
    """The f16x3 kernel's three-LDS-stage schedule (RMBX_GEMM_VAR=1040, profiling) gives the default
    two-stage schedule's output bit for bit."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(M + 7 * N)
    x = torch.randn(M, K, generator=g).to(DEV)
    p = K_.split_f16x2((torch.randn(N, K, generator=g) / K ** 0.5).to(DEV))
    b = torch.randn(N, generator=g).to(DEV)
    monkeypatch.setenv("RMBX_GEMM_WIDE", "0")  # the variants are forms of the 128-wide tile
    want = K_.linear_f32x6(x, p, b, relu=True)
    monkeypatch.setenv("RMBX_GEMM_VAR", "1040")
    got = K_.linear_f32x6(x, p, b, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(got, want)


@torch.no_grad()
@pytest.mark.parametrize("M,N,K,relu,scale", [(5000, 3200, 512, True, 1.0), (3000, 512, 3200, False, 1.0),
                                              (257, 384, 96, True, 1.0), (700, 256, 512, False, 1e6)])
def test_gemm_f16x3_producer_consumer_equals_default(monkeypatch, M, N, K, relu, scale):
    """The producer / consumer f16x3 kernel (RMBX_GEMM_PC=1: 8 MFMA waves, 4 waves loading,
    splitting and moving W) gives the default kernel's output bit for bit, the range re-run
    included (scale 1e6)."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(M + 3 * N)
    x = (torch.randn(M, K, generator=g) * scale).to(DEV)
    p = K_.split_f16x2((torch.randn(N, K, generator=g) / K ** 0.5).to(DEV))
    b = torch.randn(N, generator=g).to(DEV)
    monkeypatch.setenv("RMBX_GEMM_WIDE", "0")  # the producer / consumer kernel is a 128-wide form
    monkeypatch.setenv("RMBX_GEMM_PC", "0")
    want = K_.linear_f32x6(x, p, b, relu=relu)
    monkeypatch.setenv("RMBX_GEMM_PC", "1")
    got = K_.linear_f32x6(x, p, b, relu=relu)
    torch.cuda.synchronize()
    assert torch.equal(got, want)


@torch.no_grad()
def test_conv2d_f16x3_producer_consumer_equals_default(monkeypatch):
    from robomanipbaselines_amd import kernels as K_

    monkeypatch.setattr(K_, "F32_PIECES", "f16x3")
    g = torch.Generator(device="cpu").manual_seed(5)
    cl = torch.channels_last
    x = torch.randn(3, 64, 37, 45, generator=g).clamp_min(0).to(DEV).contiguous(memory_format=cl)
    w = K_.pack_conv_f32x6((torch.randn(128, 64, 3, 3, generator=g) / 24.0).to(DEV))
    b = torch.randn(128, generator=g).to(DEV)
    r = torch.randn(3, 128, 19, 23, generator=g).to(DEV).contiguous(memory_format=cl)
    monkeypatch.setenv("RMBX_GEMM_WIDE", "0")
    monkeypatch.setenv("RMBX_GEMM_PC", "0")
    want = K_.conv2d_f32x6(x, w, b, 3, 2, 1, relu=True, res=r)
    monkeypatch.setenv("RMBX_GEMM_PC", "1")
    got = K_.conv2d_f32x6(x, w, b, 3, 2, 1, relu=True, res=r)
    torch.cuda.synchronize()
    assert torch.equal(got, want)


@torch.no_grad()
@pytest.mark.parametrize("M,N,K,relu,scale", [(5000, 3200, 512, True, 1.0), (3000, 512, 3200, False, 1.0),
                                              (1000, 1024, 512, True, 1.0), (700, 768, 96, False, 1e6)])
def test_gemm_f16x3_wide_tile_equals_default(monkeypatch, M, N, K, relu, scale):
    """The f16x3 kernel's 256-column tile (the default; N = 3200 as a 3072-column wide launch plus a
    128-column one) gives the 128-column tile's output (RMBX_GEMM_WIDE=0) bit for bit, the range
    re-run included."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator(device="cpu").manual_seed(M + 11 * N)
    x = (torch.randn(M, K, generator=g) * scale).to(DEV)
    p = K_.split_f16x2((torch.randn(N, K, generator=g) / K ** 0.5).to(DEV))
    b = torch.randn(N, generator=g).to(DEV)
    monkeypatch.setenv("RMBX_GEMM_WIDE", "0")
    want = K_.linear_f32x6(x, p, b, relu=relu)
    monkeypatch.setenv("RMBX_GEMM_WIDE", "1")
    got = K_.linear_f32x6(x, p, b, relu=relu)
    torch.cuda.synchronize()
    assert torch.equal(got, want)


@torch.no_grad()
@pytest.mark.parametrize("n,C,H,W,Cout", [(2, 256, 30, 40, 256), (3, 128, 15, 21, 384)])
def test_gemm_f16x3_wide_tile_batched_equals_narrow(monkeypatch, n, C, H, W, Cout):
    """The batched f16x3 GEMM (the 36 Winograd position GEMMs) on the 256-wide tile -- with a
    128-column remainder launch per item for Cout = 384 -- equals the 128-wide tile bit for bit."""
    from robomanipbaselines_amd import kernels as K_

    monkeypatch.setattr(K_, "F32_PIECES", "f16x3")
    g = torch.Generator(device="cpu").manual_seed(n * C + Cout)
    cl = torch.channels_last
    x = torch.randn(n, C, H, W, generator=g).clamp_min(0).to(DEV).contiguous(memory_format=cl)
    wt = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV)
    u = K_.pack_wino4_x6(wt)
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("RMBX_GEMM_WIDE", v)
        outs.append(K_.conv3x3_wino4_x6(x, u, b, relu=True))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = _conv_ref(x, wt, b, 1, 1, True, None)
    assert _err(outs[1], ref) <= 1e-5  # the Winograd F(4x4) transforms' rounding, as the explicit test


@torch.no_grad()
@pytest.mark.parametrize("n,C,H,W,Cout,k,stride,res", [(2, 128, 30, 40, 256, 3, 2, True), (3, 256, 15, 20, 512, 3, 2, False),
                                                       (2, 64, 20, 24, 384, 1, 1, True)])
def test_conv2d_f16x3_wide_tile_equals_narrow(monkeypatch, n, C, H, W, Cout, k, stride, res):
    """Implicit-GEMM convs with Cout >= 256 on the 256-wide tile (the layer-3/4 stride-2 and 1x1
    downsample convs; Cout = 384 adds a 128-column remainder launch with its residual offset) equal
    the 128-wide tile bit for bit and the f64 conv to f32 accuracy."""
    from robomanipbaselines_amd import kernels as K_

    monkeypatch.setattr(K_, "F32_PIECES", "f16x3")
    g = torch.Generator(device="cpu").manual_seed(n * C + Cout)
    cl = torch.channels_last
    pad = k // 2
    x = torch.randn(n, C, H, W, generator=g).clamp_min(0).to(DEV).contiguous(memory_format=cl)
    wt = (torch.randn(Cout, C, k, k, generator=g) / (C * k * k) ** 0.5).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV)
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    r = torch.randn(n, Cout, Ho, Wo, generator=g).to(DEV).contiguous(memory_format=cl) if res else None
    w = K_.pack_conv_f32x6(wt)
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("RMBX_GEMM_WIDE", v)
        outs.append(K_.conv2d_f32x6(x, w, b, k, stride, pad, relu=True, res=r))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = _conv_ref(x, wt, b, stride, pad, True, r)
    assert _err(outs[1], ref) < 2e-6


@pytest.mark.parametrize("M,N,K", [(32768, 256, 2560), (4096, 512, 1024), (1024, 192, 256)])
def test_linear_f16x3_small_grid_tiles_bitwise(monkeypatch, M, N, K):
    """Grids with fewer wide tiles than CUs run the 128- / 64-wide tile (launch_f16x3); the per-element
    K order is the tile width's invariant, so the outputs equal the wide-tile rule's bitwise
    (RMBX_GEMM_FILL=0) and stay within the f16x3 bar against f64."""
    from robomanipbaselines_amd import kernels as K_

    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    planes = K_.split_f16x2(w)
    got = K_.linear_f32x6(x, planes, b)
    monkeypatch.setenv("RMBX_GEMM_FILL", "0")
    ref = K_.linear_f32x6(x, planes, b)
    assert torch.equal(got, ref)
    want = x.double() @ w.double().t() + b.double()
    err = _err(got, want)  # max |err| / max |ref|: the file's f32 GEMM bar
    assert err < 4e-6, err
