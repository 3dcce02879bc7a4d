"""rmbx_conv3x3_f16x3_patch (3x3 / stride 1 conv in the f16x3 form, each input pixel split once per
output tile) vs an f64 reference of the same op, beside the implicit-GEMM f16x3 conv it can
replace; f16's range handled by the per-(tile, chunk) power-of-two scale; every image's result
independent of the batch it runs in."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref(x, w, b, relu, res):
    r = F.conv2d(x.double(), w.double(), None if b is None else b.double(), 1, 1)
    if res is not None:
        r = r + res.double()
    return r.clamp_min(0) if relu else r


def _err(got, ref):
    return ((got.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-300)).item()


def _case(n, C, H, W, Cout, res, relu, seed, bias=True):
    g = torch.Generator(device="cpu").manual_seed(seed)
    cl = torch.channels_last
    x = torch.randn(n, C, H, W, generator=g).clamp_min(0).to(DEV).contiguous(memory_format=cl)
    w = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV) if bias else None
    r = torch.randn(n, Cout, H, W, generator=g).to(DEV).contiguous(memory_format=cl) if res else None
    return x, w, b, r


@torch.no_grad()
@pytest.mark.parametrize("n,C,H,W,Cout,res,relu,bias", [
    (2, 64, 120, 160, 64, True, True, True),    # layer-1 shape (16 x 32 tiles, 512 x 64 per block)
    (3, 64, 37, 45, 64, False, True, True),     # ragged tiles
    (2, 128, 60, 80, 128, True, True, True),    # layer-2 shape (16 x 16 tiles, 256 x 128 per block)
    (2, 128, 19, 23, 128, False, False, False),
    (2, 64, 30, 40, 128, True, True, True),
    (1, 96, 17, 33, 192, True, False, True),    # 3 chunks, 3 channel blocks of 64
    (1, 32, 5, 7, 64, False, True, True),       # one tile, mostly padding
])
def test_conv3x3_patch_vs_f64(n, C, H, W, Cout, res, relu, bias):
    from robomanipbaselines_amd import kernels as K

    x, w, b, r = _case(n, C, H, W, Cout, res, relu, n * 1000 + C + H + Cout)
    p = K.pack_conv_f32x6(w) if K.F32_PIECES == "f16x3" else None
    if p is None:
        pytest.skip("f16x3 form disabled")
    got = K.conv3x3_f16x3_patch(x, p, b, relu=relu, res=r)
    gemm = K.conv2d_f32x6(x, p, b, 3, 1, 1, relu=relu, res=r)
    torch.cuda.synchronize()
    assert got.shape == (n, Cout, H, W) and got.is_contiguous(memory_format=torch.channels_last)
    ref = _ref(x, w, b, relu, r)
    e, eg = _err(got, ref), _err(gemm, ref)
    print(f"\npatch {e:.2e}  implicit GEMM {eg:.2e}")
    assert e <= 2e-6, (e, eg)


@torch.no_grad()
@pytest.mark.parametrize("case", ["huge", "tiny", "zero", "chunks_apart", "mixed_images"])
def test_conv3x3_patch_range_and_batch_independence(case):
    """Images scaled by 1e6 / 1e-7, an all-zero image, channel chunks 2^40 apart within a tile (the
    accumulator rescale), and a batch mixing all of them: each image within f32 accuracy of f64 on
    its own scale, and bitwise equal to the same image run alone."""
    from robomanipbaselines_amd import kernels as K

    x, w, b, r = _case(4, 64, 33, 40, 64, True, True, 77)
    if case == "huge":
        x[1] *= 1e6
    elif case == "tiny":
        x[1] *= 1e-7
    elif case == "zero":
        x[1] = 0.0
    elif case == "chunks_apart":
        x[1, :32] *= 2.0 ** -20
        x[1, 32:] *= 2.0 ** 20
    else:
        x[0] *= 1e6
        x[1] *= 1e-7
        x[2] = 0.0
    x = x.contiguous(memory_format=torch.channels_last)
    p = K.pack_conv_f32x6(w)
    got = K.conv3x3_f16x3_patch(x, p, b, relu=False, res=None)
    ref = _ref(x, w, b, False, None)
    for i in range(4):
        e = _err(got[i], ref[i])
        assert e <= 2e-6, (case, i, e)
        alone = K.conv3x3_f16x3_patch(x[i:i + 1].contiguous(memory_format=torch.channels_last), p, b)
        assert torch.equal(alone[0], got[i]), (case, i)


@torch.no_grad()
def test_conv3x3_patch_nan_propagates_and_rejects_bad_shapes():
    from robomanipbaselines_amd import kernels as K

    x, w, b, _ = _case(1, 64, 20, 20, 64, False, False, 5)
    x[0, 3, 10, 10] = float("nan")
    p = K.pack_conv_f32x6(w)
    got = K.conv3x3_f16x3_patch(x, p, b)
    torch.cuda.synchronize()
    assert torch.isnan(got[0, :, 9:12, 9:12]).all()
    assert not torch.isnan(got[0, :, :5, :5]).any()
    with pytest.raises(ValueError):
        K.conv3x3_f16x3_patch(x[:, :48].contiguous(memory_format=torch.channels_last), p, b)
    w2 = torch.randn(96, 64, 3, 3, device=DEV)
    with pytest.raises(ValueError):
        K.conv3x3_f16x3_patch(x, K.pack_conv_f32x6(w2), None)
