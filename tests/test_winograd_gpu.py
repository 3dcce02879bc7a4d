"""rmbx_conv3x3_winograd_f32 (Winograd F(2x2, 3x3) on f32 MFMA, fused bias / residual / ReLU)
against the direct convolution: F.conv2d in f64 on the CPU for small cases, in f32 on the device
for sizes with several tile blocks per persistent block.  The bar is f32 rounding of the
transform adds: |err| <= 1e-5 * max(1, max |ref|) (measured ~1e-6)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _case(n, C, H, W, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(n, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / (9 * C) ** 0.5
    b = torch.randn(C, generator=g)
    r = torch.randn(n, C, H, W, generator=g)
    return x, w, b, r


def _run(x, w, b, r, relu):
    from robomanipbaselines_amd import kernels as K

    u = K.pack_winograd_f32(w.to(DEV))
    xd = _cl(x.to(DEV))
    rd = None if r is None else _cl(r.to(DEV))
    got = K.conv3x3_winograd_f32(xd, u, b.to(DEV), relu=relu, res=rd)
    assert got.shape == x.shape and got.is_contiguous(memory_format=torch.channels_last)
    return got


@torch.no_grad()
@pytest.mark.parametrize("n,C,H,W,res,relu", [(2, 64, 7, 9, True, True), (3, 128, 15, 20, False, True),
                                              (2, 256, 8, 6, True, False), (2, 512, 15, 20, True, True),
                                              (1, 64, 1, 1, True, True), (1, 512, 3, 2, False, False)])
def test_winograd_matches_f64_conv(n, C, H, W, res, relu):
    x, w, b, r = _case(n, C, H, W, seed=C + H * W)
    r = r if res else None
    ref = F.conv2d(x.double(), w.double(), b.double(), 1, 1)
    if r is not None:
        ref = ref + r.double()
    if relu:
        ref = F.relu(ref)
    got = _run(x, w, b, r, relu).cpu().double()
    err = (got - ref).abs().max().item()
    assert err <= 1e-5 * max(1.0, ref.abs().max().item()), err


@torch.no_grad()
@pytest.mark.parametrize("n,C,H,W", [(32, 64, 64, 64), (16, 512, 30, 40), (24, 128, 33, 47)])
def test_winograd_multi_unit_matches_device_conv(n, C, H, W):
    """Several tile blocks per persistent block (the chunk pipeline runs across units), ragged last
    block and odd sizes; reference F.conv2d f32 on the device."""
    x, w, b, r = _case(n, C, H, W, seed=n * C)
    xd, wd, bd, rd = (t.to(DEV) for t in (x, w, b, r))
    ref = F.relu(F.conv2d(xd, wd, bd, 1, 1) + rd)
    got = _run(x, w, b, r, relu=True)
    err = (got - ref).abs().max().item()
    assert err <= 1e-5 * max(1.0, ref.abs().max().item()), err


def test_winograd_rejects_bad_arguments():
    from robomanipbaselines_amd import kernels as K

    with pytest.raises(ValueError):
        K.pack_winograd_f32(torch.randn(96, 96, 3, 3))
    x = _cl(torch.randn(1, 64, 8, 8, device=DEV))
    u = K.pack_winograd_f32(torch.randn(64, 64, 3, 3, device=DEV))
    with pytest.raises(ValueError):  # bf16 input
        K.conv3x3_winograd_f32(x.to(torch.bfloat16), u, torch.zeros(64, device=DEV))
    with pytest.raises(ValueError):  # packed filter of another width
        K.conv3x3_winograd_f32(x, K.pack_winograd_f32(torch.randn(128, 128, 3, 3, device=DEV)),
                               torch.zeros(64, device=DEV))


@torch.no_grad()
def test_winograd_batch_slices_equal_one_launch(monkeypatch):
    """Batches beyond the kernel's 32-bit offsets run as slices of whole images: same output."""
    from robomanipbaselines_amd import kernels as K

    x, w, b, r = _case(5, 64, 12, 10, seed=3)
    whole = _run(x, w, b, r, relu=True)
    monkeypatch.setattr(K, "WINOGRAD_MAX_ELEMS", 2 * 12 * 10 * 64)  # two images per launch
    sliced = _run(x, w, b, r, relu=True)
    assert torch.equal(whole, sliced)


def _run4(x, w, b, r, relu):
    from robomanipbaselines_amd import kernels as K

    u = K.pack_winograd4_f32(w.to(DEV))
    xd = _cl(x.to(DEV))
    rd = None if r is None else _cl(r.to(DEV))
    got = K.conv3x3_winograd4_f32(xd, u, b.to(DEV), relu=relu, res=rd)
    assert got.shape == x.shape and got.is_contiguous(memory_format=torch.channels_last)
    return got


@torch.no_grad()
@pytest.mark.parametrize("n,C,H,W,res,relu", [(2, 64, 7, 9, True, True), (3, 128, 15, 20, False, True),
                                              (2, 256, 8, 6, True, False), (2, 512, 15, 20, True, True),
                                              (1, 64, 1, 1, True, True), (1, 512, 3, 2, False, False),
                                              (5, 64, 30, 40, True, True)])
def test_winograd4_matches_f64_conv(n, C, H, W, res, relu):
    """F(4x4, 3x3): the larger transform constants cost a few bits more than F(2x2); bar 2e-5 relative."""
    x, w, b, r = _case(n, C, H, W, seed=C + H * W + 1)
    r = r if res else None
    ref = F.conv2d(x.double(), w.double(), b.double(), 1, 1)
    if r is not None:
        ref = ref + r.double()
    if relu:
        ref = F.relu(ref)
    got = _run4(x, w, b, r, relu).cpu().double()
    err = (got - ref).abs().max().item()
    assert err <= 2e-5 * max(1.0, ref.abs().max().item()), err


@torch.no_grad()
@pytest.mark.parametrize("n,C,H,W", [(32, 64, 64, 64), (16, 512, 30, 40), (24, 128, 33, 47), (40, 256, 30, 40)])
def test_winograd4_multi_unit_matches_device_conv(n, C, H, W):
    x, w, b, r = _case(n, C, H, W, seed=7 * C + W)
    xd, wd, bd, rd = _cl(x.to(DEV)), w.to(DEV), b.to(DEV), _cl(r.to(DEV))
    ref = F.relu(F.conv2d(xd, wd, bd, 1, 1) + rd)
    got = _run4(x, w, b, r, True)
    err = (got - ref).abs().max().item()
    assert err <= 2e-5 * max(1.0, ref.abs().max().item()), err
