"""Vision-trunk epilogue kernels (rmbx_nhwc_bias_act / rmbx_nhwc_bias_relu_maxpool) vs the
unfused PyTorch sequence they replace (bias add -> [residual add] -> ReLU [-> max-pool]), and the
fused ResNet-18 trunk vs the fp32 FrozenBN reference module."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _torch_epilogue(x, b, res=None, rb=None, relu=True):
    y = x + b.to(x.dtype).reshape(1, -1, 1, 1)
    if res is not None:
        r = res if rb is None else res + rb.to(x.dtype).reshape(1, -1, 1, 1)
        y = y + r
    return F.relu(y) if relu else y


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("mode", ["bias", "bias_relu", "res_relu", "res_bias_relu", "res_bias"])
def test_bias_act_bit_exact(dtype, mode):
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(1)
    x = _cl(torch.randn(3, 64, 9, 13, device=DEV, generator=g).to(dtype))
    b = torch.randn(64, device=DEV, generator=g).to(dtype).float()
    res = _cl(torch.randn(3, 64, 9, 13, device=DEV, generator=g).to(dtype)) if "res" in mode else None
    rb = torch.randn(64, device=DEV, generator=g).to(dtype).float() if "res_bias" in mode else None
    relu = "relu" in mode
    ref = _torch_epilogue(x, b, res, rb, relu)
    got = K.nhwc_bias_act(x, b, res, rb, relu=relu)
    assert torch.equal(got, ref)
    # in place
    x2 = x.clone(memory_format=torch.channels_last)
    K.nhwc_bias_act(x2, b, res, rb, relu=relu, out=x2)
    assert torch.equal(x2, ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("hw", [(17, 23), (16, 16), (240, 320), (1, 1)])
def test_bias_relu_maxpool_bit_exact(dtype, hw):
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(2)
    H, W = hw
    x = _cl(torch.randn(2, 64, H, W, device=DEV, generator=g).to(dtype))
    b = torch.randn(64, device=DEV, generator=g).to(dtype).float()
    ref = F.max_pool2d(_torch_epilogue(x, b), 3, 2, 1)
    got = K.nhwc_bias_relu_maxpool(x, b)
    assert got.shape == ref.shape
    assert torch.equal(got, ref)


def test_epilogue_rejects_bad_layout():
    from robomanipbaselines_amd import kernels as K

    x = torch.randn(2, 64, 5, 5, device=DEV)  # NCHW-contiguous, not channels_last
    with pytest.raises(ValueError):
        K.nhwc_bias_act(x, torch.zeros(64, device=DEV))
    y = _cl(torch.randn(2, 12, 5, 5, device=DEV, dtype=torch.bfloat16))  # C not a multiple of 8
    with pytest.raises(ValueError):
        K.nhwc_bias_act(y, torch.zeros(12, device=DEV))


def _trunk_pair(seed=0):
    from robomanipbaselines_amd.policy.backbone import FusedResNet18Trunk, ResNet18Trunk

    torch.manual_seed(seed)
    ref = ResNet18Trunk().eval().requires_grad_(False)
    for m in ref.modules():  # non-trivial frozen BN statistics
        if hasattr(m, "running_var"):
            m.weight.uniform_(0.5, 1.5)
            m.bias.uniform_(-0.2, 0.2)
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 2.0)
    fused = FusedResNet18Trunk(ref)
    return ref, fused


@torch.no_grad()
def test_fused_trunk_fp32_matches_reference():
    ref, fused = _trunk_pair()
    x = torch.rand(2, 3, 96, 128)
    want = ref(x)
    fused = fused.to(DEV).to(memory_format=torch.channels_last)
    got = fused(_cl(x.to(DEV))).cpu()
    assert got.shape == want.shape == (2, 512, 3, 4)
    err = (got - want).abs().max().item()
    assert err <= 1e-3 * max(1.0, want.abs().max().item()), err


@pytest.mark.parametrize("cin,cout,k,stride,res,relu", [(64, 64, 3, 1, True, True), (64, 128, 3, 2, False, True),
                                                       (64, 128, 1, 2, False, False), (128, 128, 3, 1, True, True),
                                                       (256, 512, 3, 2, False, False)])
@torch.no_grad()
def test_conv2d_nhwc_matches_fp32(cin, cout, k, stride, res, relu):
    """rmbx implicit-GEMM conv (bf16 in, f32 accumulate, fused bias/residual/ReLU, one bf16
    rounding) vs F.conv2d in fp32 on the same bf16 operands: within one bf16 rounding."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(cin + cout + k)
    x = _cl(torch.randn(3, cin, 17, 23, device=DEV, generator=g).to(torch.bfloat16))
    w = _cl((torch.randn(cout, cin, k, k, device=DEV, generator=g) / (cin * k * k) ** 0.5).to(torch.bfloat16))
    b = torch.randn(cout, device=DEV, generator=g).to(torch.bfloat16).float()
    pad = k // 2
    ref = F.conv2d(x.float(), w.float(), b, stride, pad)
    r = None
    if res:
        r = _cl(torch.randn(ref.shape, device=DEV, generator=g).to(torch.bfloat16))
        ref = ref + r.float()
    if relu:
        ref = F.relu(ref)
    got = K.conv2d_nhwc(x, w, b, stride, pad, relu=relu, res=r)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=torch.channels_last)
    err = (got.float() - ref).abs()
    assert (err <= 2 ** -8 * ref.abs() + 1e-3).all(), err.max().item()


@torch.no_grad()
@pytest.mark.parametrize("n,H,W,res,relu", [(5, 37, 45, True, True), (2, 16, 32, False, True), (3, 9, 17, True, False),
                                            (1, 120, 160, True, True)])
def test_conv2d_nhwc_f32_matches_fp32(n, H, W, res, relu):
    """rmbx_conv2d_nhwc_f32 (layer-1 conv, f32 MFMA, fused bias/residual/ReLU) vs F.conv2d in fp32:
    within f32 accumulation-order rounding (ragged tiles, several tiles per persistent block)."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(n * 1000 + H)
    x = _cl(torch.randn(n, 64, H, W, device=DEV, generator=g))
    w = _cl(torch.randn(64, 64, 3, 3, device=DEV, generator=g) / 24)
    b = torch.randn(64, device=DEV, generator=g)
    ref = F.conv2d(x, w, b, 1, 1)
    r = None
    if res:
        r = _cl(torch.randn(ref.shape, device=DEV, generator=g))
        ref = ref + r
    if relu:
        ref = F.relu(ref)
    got = K.conv2d_nhwc(x, w, b, 1, 1, relu=relu, res=r)
    assert got.dtype == torch.float32 and got.shape == ref.shape
    assert got.is_contiguous(memory_format=torch.channels_last)
    err = (got - ref).abs().max().item()
    assert err <= 2e-5 * max(1.0, ref.abs().max().item()), err


def test_conv2d_nhwc_f32_rejects_other_shapes():
    from robomanipbaselines_amd import kernels as K

    x = _cl(torch.randn(1, 128, 8, 8, device=DEV))
    w = _cl(torch.randn(128, 128, 3, 3, device=DEV))
    with pytest.raises(ValueError):
        K.conv2d_nhwc(x, w, torch.zeros(128, device=DEV), 1, 1)


@torch.no_grad()
def test_conv3x3_c64_resident_equals_streaming_kernel(monkeypatch):
    """The persistent resident-filter kernel (Cin = Cout = 64) walks several 16x16 tiles per block
    (768 tiles > CU count, ragged edges) and must equal the per-tile streaming kernel bit for bit
    (same MFMA order), and the fp32 reference within one bf16 rounding."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(7)
    x = _cl(torch.randn(64, 64, 40, 57, device=DEV, generator=g).to(torch.bfloat16))
    w = _cl((torch.randn(64, 64, 3, 3, device=DEV, generator=g) / 24).to(torch.bfloat16))
    b = torch.randn(64, device=DEV, generator=g)
    r = _cl(torch.randn(64, 64, 40, 57, device=DEV, generator=g).to(torch.bfloat16))
    got = K.conv2d_nhwc(x, w, b, 1, 1, relu=True, res=r)
    monkeypatch.setenv("RMBX_CONV_NO_RESIDENT", "1")
    alt = K.conv2d_nhwc(x, w, b, 1, 1, relu=True, res=r)
    assert torch.equal(got, alt)
    ref = F.relu(F.conv2d(x.float(), w.float(), b, 1, 1) + r.float())
    err = (got.float() - ref).abs()
    assert (err <= 2 ** -8 * ref.abs() + 1e-3).all(), err.max().item()


@torch.no_grad()
def test_fused_trunk_bf16_epilogues_equal_unfused_sequence():
    """Walk the trunk with each conv evaluated ONCE; the HIP epilogues and the torch ops applied
    to the same conv outputs must agree bit for bit at every block (real trunk shapes)."""
    ref, fused = _trunk_pair(1)
    fused = fused.to(DEV, torch.bfloat16).to(memory_format=torch.channels_last)
    from robomanipbaselines_amd import kernels as K

    x = _cl(torch.rand(2, 3, 96, 128, device=DEV).to(torch.bfloat16))
    # (the MIOpen + rmbx-epilogue form, which the f32 trunk and the stem use)
    s = fused.stem.conv_nobias(x)
    h = K.nhwc_bias_relu_maxpool(s, fused.stem.bias_f32())
    assert torch.equal(h, F.max_pool2d(_torch_epilogue(s, fused.stem.bias_f32()), 3, 2, 1))
    for blk in fused.blocks:
        c1 = blk.c1.conv_nobias(h)
        y = K.nhwc_bias_act(c1, blk.c1.bias_f32(), relu=True)
        assert torch.equal(y, _torch_epilogue(c1, blk.c1.bias_f32()))
        z = blk.c2.conv_nobias(y)
        if blk.down is None:
            out = K.nhwc_bias_act(z, blk.c2.bias_f32(), res=h, relu=True)
            want = _torch_epilogue(z, blk.c2.bias_f32(), h)
        else:
            d = blk.down.conv_nobias(h)
            out = K.nhwc_bias_act(z, blk.c2.bias_f32(), res=d, res_bias=blk.down.bias_f32(), relu=True)
            want = _torch_epilogue(z, blk.c2.bias_f32(), d, blk.down.bias_f32())
        assert torch.equal(out, want)
        h = out


@torch.no_grad()
def test_fused_trunk_bf16_close_to_fp32_reference():
    ref, fused = _trunk_pair(2)
    x = torch.rand(2, 3, 96, 128)
    want = ref(x)
    fused = fused.to(DEV, torch.bfloat16).to(memory_format=torch.channels_last)
    got = fused(_cl(x.to(DEV).to(torch.bfloat16))).float().cpu()
    rel = (got - want).norm() / want.norm()
    assert rel < 3e-2, rel.item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_add_layernorm(dtype):
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(4)
    x = (torch.randn(301, 512, device=DEV, generator=g) * 3).to(dtype)
    r = torch.randn(301, 512, device=DEV, generator=g).to(dtype)
    w = torch.randn(512, device=DEV, generator=g).to(dtype)
    b = torch.randn(512, device=DEV, generator=g).to(dtype)
    s = (x + r).float()  # the rounded sum, as the unfused add produces it
    want = F.layer_norm(s, (512,), w.float(), b.float(), 1e-5)
    got = K.add_layernorm(x, r, w.float(), b.float(), 1e-5).float()
    tol = 1e-5 if dtype == torch.float32 else 2 ** -7  # one bf16 ulp of the output
    assert ((got - want).abs() <= tol * (1 + want.abs())).all()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_add_layernorm_pos_equals_separate_add(dtype):
    """rmbx_add_layernorm_pos: out is rmbx_add_layernorm's, out_pos == (out + pos) as torch adds
    them in the storage dtype, bit for bit (pos broadcast per sequence position)."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(5)
    x = (torch.randn(3, 302, 512, device=DEV, generator=g) * 3).to(dtype)
    r = torch.randn(3, 302, 512, device=DEV, generator=g).to(dtype)
    w = torch.randn(512, device=DEV, generator=g)
    b = torch.randn(512, device=DEV, generator=g)
    pos = torch.randn(1, 302, 512, device=DEV, generator=g).to(dtype)
    y, yp = K.add_layernorm_pos(x, r, w, b, pos, 1e-5)
    assert torch.equal(y, K.add_layernorm(x, r, w, b, 1e-5))
    assert torch.equal(yp, y + pos)


@torch.no_grad()
def test_act_device_inference_form_matches_fp32_reference():
    from robomanipbaselines_amd.policy.act.act_model import ActModel

    torch.manual_seed(0)
    ref = ActModel(enc_layers=2, dec_layers=2).eval().requires_grad_(False)
    dev = ActModel(enc_layers=2, dec_layers=2).eval().requires_grad_(False)
    dev.load_state_dict(ref.state_dict())
    dev.fuse_backbone()
    dev = dev.to(DEV)
    dev._fused = dev._fused.to(memory_format=torch.channels_last)
    dev.fuse_transformer()
    q = torch.randn(2, 7)
    img = torch.rand(2, 1, 3, 96, 128)
    want = ref(q, img)
    got = dev(q.to(DEV), img.to(DEV)).cpu()
    assert got.shape == (2, 100, 7)
    assert (got - want).abs().max().item() <= 2e-3 * max(1.0, want.abs().max().item())


@torch.no_grad()
def test_stem_s2d_conv_matches_fp32():
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(2, 3, 48, 64, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(64, 3, 7, 7, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    b = torch.randn(64, device=DEV, generator=g)
    ref = F.relu(F.conv2d(x.float(), w.float(), b, 2, 3))
    got = K.stem_s2d_conv(K.image_to_s2d(x), K.pack_stem_s2d(w), b)
    assert got.shape == ref.shape == (2, 64, 24, 32)
    err = (got.float() - ref).abs()
    assert (err <= 2 ** -8 * ref.abs() + 1e-3).all(), err.max().item()


@torch.no_grad()
@pytest.mark.parametrize("n,H,W,band_rows", [(2, 48, 64, 0), (3, 480, 640, 0), (2, 480, 640, 7),
                                             (2, 46, 630, 5), (1, 34, 90, 1), (5, 20, 40, 0)])
def test_stem_conv_maxpool_fused_equals_unfused(n, H, W, band_rows):
    """rmbx_stem_s2d_conv_maxpool == rmbx_stem_s2d_conv + rmbx_nhwc_bias_relu_maxpool bit for bit
    (full 480x640 frames, pool-row bands that split images, widths not a multiple of 32, odd
    stem-map sizes)."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(11)
    x = (torch.rand(n, 3, H, W, device=DEV, generator=g) * 4 - 2).to(torch.bfloat16)
    w = (torch.randn(64, 3, 7, 7, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    b = torch.randn(64, device=DEV, generator=g) * 0.5
    xs, wp = K.image_to_s2d(x), K.pack_stem_s2d(w)
    want = K.nhwc_bias_relu_maxpool(K.stem_s2d_conv(xs, wp, b), torch.zeros(64, device=DEV))
    got = K.stem_s2d_conv_maxpool(xs, wp, b, band_rows=band_rows)
    torch.cuda.synchronize()
    assert got.shape == want.shape
    assert torch.equal(got, want), (got.float() - want.float()).abs().max().item()


def test_stem_conv_maxpool_rejects_wide_images():
    from robomanipbaselines_amd import kernels as K

    x = torch.zeros(1, 8, 322, 16, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(ValueError):
        K.stem_s2d_conv_maxpool(x, torch.zeros(64, 4, 4, 16, dtype=torch.bfloat16, device=DEV),
                                torch.zeros(64, device=DEV))


@torch.no_grad()
def test_trunk_s2d_matches_standard_layout():
    ref, fused = _trunk_pair(3)
    fused = fused.to(DEV, torch.bfloat16).to(memory_format=torch.channels_last)
    from robomanipbaselines_amd import kernels as K

    x = torch.rand(2, 3, 96, 128, device=DEV).to(torch.bfloat16)
    a = fused(_cl(x)).float()
    b = fused.forward_s2d(K.image_to_s2d(x)).float()
    assert (a - b).norm() / a.norm() < 2e-2


def test_render_s2d_layout_equals_standard():
    from robomanipbaselines_amd import kernels as K
    from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv

    env = BatchedMujocoUR5eCableEnv(3, DEV)
    env.reset()
    H, W = env.renderer.height, env.renderer.width
    std = torch.empty((3, 3, H, W), dtype=torch.bfloat16, device=DEV)
    s2d = torch.empty((3, H // 2, W // 2, 16), dtype=torch.bfloat16, device=DEV)
    env.render_images("front", policy=std)
    env.render_images("front", policy=s2d)
    assert torch.equal(K.image_to_s2d(std), s2d)


@torch.no_grad()
@pytest.mark.parametrize("n,H,W,band_rows", [(2, 48, 64, 0), (3, 480, 640, 0), (2, 480, 640, 7), (2, 46, 630, 5),
                                             (1, 34, 90, 1)])
def test_stem_conv_maxpool_f32_matches_fp32_reference(n, H, W, band_rows):
    """rmbx_stem_s2d_conv_maxpool_f32 (f32 MFMA) vs F.conv2d + bias + ReLU + max_pool2d in fp32 on
    the same image: within f32 accumulation-order rounding."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(13)
    x = torch.rand(n, 3, H, W, device=DEV, generator=g) * 4 - 2
    w = torch.randn(64, 3, 7, 7, device=DEV, generator=g) * 0.1
    b = torch.randn(64, device=DEV, generator=g) * 0.5
    want = F.max_pool2d(F.relu(F.conv2d(x, w, b, 2, 3)), 3, 2, 1)
    got = K.stem_s2d_conv_maxpool(K.image_to_s2d(x), K.pack_stem_s2d(w), b, band_rows=band_rows)
    torch.cuda.synchronize()
    assert got.shape == want.shape and got.dtype == torch.float32
    assert got.is_contiguous(memory_format=torch.channels_last)
    err = (got - want).abs().max().item()
    assert err <= 2e-5 * max(1.0, want.abs().max().item()), err


@torch.no_grad()
@pytest.mark.parametrize("pieces", ["f16", "bf16"])
@pytest.mark.parametrize("n,H,W,band_rows", [(2, 48, 64, 0), (3, 480, 640, 0), (2, 480, 640, 7), (2, 46, 630, 5),
                                             (1, 34, 90, 1), (2, 6, 8, 0)])
def test_stem_conv_maxpool_u8_matches_fp32_reference(pieces, n, H, W, band_rows):
    """The u8 stem (normalisation folded into the stem, integer pixels x the weight pieces:
    rmbx_stem_s2d_conv_maxpool_u8h with two f16 pieces of the power-of-two-scaled bank, the default,
    and rmbx_stem_s2d_conv_maxpool_u8 with three exact bf16 pieces) vs F.conv2d + bias + ReLU +
    max_pool2d in fp32 on the normalised image x = (u / 255 - mean) / std the renderer would hand
    over (the border taps exercise the edge table): within f32 rounding, and no worse than the f32
    MFMA kernel against an f64 reference on the CPU."""
    from robomanipbaselines_amd import kernels as K

    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    g = torch.Generator(device=DEV).manual_seed(17)
    u = torch.randint(0, 256, (n, 3, H, W), device=DEV, generator=g, dtype=torch.int32).to(torch.uint8)
    w = torch.randn(64, 3, 7, 7, device=DEV, generator=g) * 0.1
    b = torch.randn(64, device=DEV, generator=g) * 0.5
    m3 = torch.tensor(mean, device=DEV).reshape(1, 3, 1, 1)
    s3 = torch.tensor(std, device=DEV).reshape(1, 3, 1, 1)
    x = (u.float() / 255.0 - m3) / s3
    us2d = K.image_to_s2d(u)
    torch.testing.assert_close(K.s2d_u8_normalize(us2d, mean, std), K.image_to_s2d(x), rtol=0, atol=1e-6)
    want = F.max_pool2d(F.relu(F.conv2d(x, w, b, 2, 3)), 3, 2, 1)
    ops = K.pack_stem_u8(w, b, mean, std, pieces=pieces)
    assert ops[0].dtype == (torch.float16 if pieces == "f16" else torch.bfloat16)
    got = K.stem_s2d_conv_maxpool_u8(us2d, *ops, band_rows=band_rows)
    torch.cuda.synchronize()
    assert got.shape == want.shape and got.dtype == torch.float32
    assert got.is_contiguous(memory_format=torch.channels_last)
    scale = max(1.0, want.abs().max().item())
    err = (got - want).abs().max().item()
    print(f"\nu8 stem ({pieces} pieces) vs f32 conv: max |d| {err:.3e} = {err / scale:.2e} relative")
    # the centred form: within 5e-6 of the f32 conv (the uncentred form needed 2e-5)
    assert err <= 5e-6 * scale, err
    if n * H * W <= 2 * 48 * 64:  # f64 CPU reference: the u8 form is as close as the f32 kernel
        want64 = F.max_pool2d(F.relu(F.conv2d(x.cpu().double(), w.cpu().double(), b.cpu().double(), 2, 3)), 3, 2, 1)
        f32k = K.stem_s2d_conv_maxpool(K.image_to_s2d(x), K.pack_stem_s2d(w), b, band_rows=band_rows)
        e_u8 = (got.cpu().double() - want64).abs().max().item()
        e_f32 = (f32k.cpu().double() - want64).abs().max().item()
        print(f"vs f64: u8 stem {e_u8:.3e}, f32 MFMA stem {e_f32:.3e}")
        assert e_u8 <= 1.5 * e_f32 + 1e-7 * scale, (e_u8, e_f32)


def test_stem_conv_maxpool_u8_rejects_bad_operands():
    from robomanipbaselines_amd import kernels as K

    x = torch.zeros(1, 8, 8, 16, dtype=torch.uint8, device=DEV)
    ops = K.pack_stem_u8(torch.zeros(64, 3, 7, 7, device=DEV), torch.zeros(64, device=DEV), (0, 0, 0), (1, 1, 1))
    with pytest.raises(ValueError):
        K.stem_s2d_conv_maxpool_u8(x.float(), *ops)
    with pytest.raises(ValueError):
        K.stem_s2d_conv_maxpool_u8(torch.zeros(1, 8, 400, 16, dtype=torch.uint8, device=DEV), *ops)


def test_render_s2d_u8_layout_equals_rgb():
    """rmbx_render policy_dtype 4 holds the rgb image's 8-bit values in the space-to-depth layout."""
    from robomanipbaselines_amd import kernels as K
    from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv

    env = BatchedMujocoUR5eCableEnv(2, DEV)
    env.reset()
    H, W = env.renderer.height, env.renderer.width
    rgb = torch.empty((2, H, W, 3), dtype=torch.uint8, device=DEV)
    s2d = torch.empty((2, H // 2, W // 2, 16), dtype=torch.uint8, device=DEV)
    f32 = torch.empty((2, H // 2, W // 2, 16), dtype=torch.float32, device=DEV)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    env.render_images("front", rgb=rgb, policy=s2d, mean=mean, std=std)
    env.render_images("front", policy=f32, mean=mean, std=std)
    assert torch.equal(K.image_to_s2d(rgb.permute(0, 3, 1, 2)), s2d)
    # the host restatement of the renderer's normalisation agrees to rounding (torch divides a
    # tensor by a scalar through the reciprocal, the kernel divides)
    torch.testing.assert_close(K.s2d_u8_normalize(s2d, mean, std), f32, rtol=0, atol=1e-6)


def test_render_s2d_f32_layout_equals_standard():
    from robomanipbaselines_amd import kernels as K
    from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv

    env = BatchedMujocoUR5eCableEnv(2, DEV)
    env.reset()
    H, W = env.renderer.height, env.renderer.width
    std = torch.empty((2, 3, H, W), dtype=torch.float32, device=DEV)
    s2d = torch.empty((2, H // 2, W // 2, 16), dtype=torch.float32, device=DEV)
    env.render_images("front", policy=std, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225))
    env.render_images("front", policy=s2d, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225))
    assert torch.equal(K.image_to_s2d(std), s2d)
