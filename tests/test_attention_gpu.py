"""rmbx_attention_bf16 (the ACT transformer's attention) vs a plain PyTorch fp32 reference of the
same op on the same bf16 q/k/v: softmax(q k^T / 8) v per head.  The kernel rounds the
probabilities to bf16 for the P.V product and the output to bf16, so the bar is 1e-2 of the
output scale (|v| <= 4 here) plus one bf16 rounding."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref(q, k, v, heads):
    B, Lq, D = q.shape
    Lk = k.shape[1]
    qh = q.float().reshape(B, Lq, heads, 64).transpose(1, 2)
    kh = k.float().reshape(B, Lk, heads, 64).transpose(1, 2)
    vh = v.float().reshape(B, Lk, heads, 64).transpose(1, 2)
    p = torch.softmax(qh @ kh.transpose(-1, -2) / 8.0, dim=-1)
    return (p @ vh).transpose(1, 2).reshape(B, Lq, D)


@torch.no_grad()
@pytest.mark.parametrize("B,H,Lq,Lk", [(3, 8, 302, 302), (4, 8, 100, 100), (2, 8, 100, 302), (1, 8, 1, 1),
                                       (2, 2, 257, 33), (1, 1, 130, 320)])
def test_attention_matches_fp32(B, H, Lq, Lk):
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(Lq * 31 + Lk)
    D = H * 64
    q = (torch.randn(B, Lq, D, device=DEV, generator=g) * 2).to(torch.bfloat16)
    k = (torch.randn(B, Lk, D, device=DEV, generator=g) * 2).to(torch.bfloat16)
    v = (torch.randn(B, Lk, D, device=DEV, generator=g)).clamp(-4, 4).to(torch.bfloat16)
    got = K.attention_bf16(q, k, v, H).float()
    want = _ref(q, k, v, H)
    torch.cuda.synchronize()
    err = (got - want).abs()
    assert (err <= 1e-2 * 4 + 2 ** -8 * want.abs()).all(), err.max().item()


@torch.no_grad()
def test_attention_strided_qkv_views():
    """q/k/v as slices of one fused projection output (row stride 3 D), as the MHA module feeds them."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(9)
    qkv = torch.randn(2, 150, 3 * 512, device=DEV, generator=g).to(torch.bfloat16)
    q, k, v = qkv.split(512, dim=-1)
    got = K.attention_bf16(q, k, v, 8).float()
    want = _ref(q, k, v, 8)
    assert (got - want).abs().max().item() <= 5e-2


def test_attention_rejects_long_sequences():
    from robomanipbaselines_amd import kernels as K

    x = torch.zeros(1, 321, 64, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        K.attention_bf16(x, x, x, 1)


@torch.no_grad()
@pytest.mark.parametrize("B,H,Lq,Lk", [(3, 8, 302, 302), (4, 8, 100, 100), (2, 8, 100, 302), (1, 8, 1, 1),
                                       (2, 2, 257, 33), (1, 1, 130, 650)])
def test_attention_f32_matches_fp32(B, H, Lq, Lk):
    """rmbx_attention_f32 (f32 MFMA, f32 online softmax) vs the fp32 reference: within f32
    accumulation-order rounding (1e-5 of the output scale), ragged query groups and key tiles."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(Lq * 37 + Lk)
    D = H * 64
    q = torch.randn(B, Lq, D, device=DEV, generator=g) * 2
    k = torch.randn(B, Lk, D, device=DEV, generator=g) * 2
    v = torch.randn(B, Lk, D, device=DEV, generator=g).clamp(-4, 4)
    got = K.attention_f32(q, k, v, H)
    want = _ref(q, k, v, H)
    torch.cuda.synchronize()
    assert (got - want).abs().max().item() <= 1e-5 * 4


@torch.no_grad()
def test_attention_f32_strided_qkv_views():
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(11)
    qkv = torch.randn(2, 150, 3 * 512, device=DEV, generator=g)
    q, k, v = qkv.split(512, dim=-1)
    got = K.attention_f32(q, k, v, 8)
    want = _ref(q, k, v, 8)
    assert (got - want).abs().max().item() <= 1e-5 * 4


def _ref64(q, k, v, heads):
    B, Lq, D = q.shape
    Lk = k.shape[1]
    qh = q.double().reshape(B, Lq, heads, 64).transpose(1, 2)
    kh = k.double().reshape(B, Lk, heads, 64).transpose(1, 2)
    vh = v.double().reshape(B, Lk, heads, 64).transpose(1, 2)
    p = torch.softmax(qh @ kh.transpose(-1, -2) / 8.0, dim=-1)
    return (p @ vh).transpose(1, 2).reshape(B, Lq, D)


@torch.no_grad()
@pytest.mark.parametrize("B,H,Lq,Lk", [(3, 8, 302, 302), (4, 8, 100, 100), (2, 8, 100, 302), (1, 8, 1, 1),
                                       (2, 2, 257, 33), (1, 1, 130, 650)])
def test_attention_f32x6_matches_f64(B, H, Lq, Lk):
    """rmbx_attention_f32x6 (Q, K, V, P split into three bf16 pieces, six piece products per
    product on the bf16 matrix cores, f32 accumulation and softmax) vs an f64 reference, beside the
    f32-MFMA kernel it replaces: both within 1e-5 of the output scale (|v| <= 4)."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(Lq * 41 + Lk)
    D = H * 64
    q = torch.randn(B, Lq, D, device=DEV, generator=g) * 2
    k = torch.randn(B, Lk, D, device=DEV, generator=g) * 2
    v = torch.randn(B, Lk, D, device=DEV, generator=g).clamp(-4, 4)
    want = _ref64(q, k, v, H)
    e6 = (K.attention_f32(q, k, v, H, x6=True).double() - want).abs().max().item()
    e32 = (K.attention_f32(q, k, v, H).double() - want).abs().max().item()
    print(f"\nB={B} H={H} Lq={Lq} Lk={Lk}: x6 {e6:.2e}  f32 {e32:.2e}")
    assert e6 <= 1e-5 * 4, (e6, e32)


@torch.no_grad()
def test_attention_f32x6_strided_qkv_views():
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(13)
    qkv = torch.randn(2, 150, 3 * 512, device=DEV, generator=g)
    q, k, v = qkv.split(512, dim=-1)
    got = K.attention_f32(q, k, v, 8, x6=True)
    assert (got.double() - _ref64(q, k, v, 8)).abs().max().item() <= 1e-5 * 4


@torch.no_grad()
@pytest.mark.parametrize("B,H,Lq,Lk", [(3, 8, 302, 302), (4, 8, 100, 100), (2, 8, 100, 302), (1, 8, 1, 1),
                                       (2, 2, 257, 33), (1, 1, 130, 650)])
def test_attention_f16x3_matches_f64(B, H, Lq, Lk):
    """rmbx_attention_f16x3 (K, V split as h + 2^-11 l, Q and 2^14 P as h + l, three f16 piece
    products per product, f32 accumulation and softmax) vs an f64 reference, beside the bf16x6
    kernel: within 1e-5 of the output scale (|v| <= 4), no block re-run at these ranges."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(Lq * 43 + Lk)
    D = H * 64
    q = torch.randn(B, Lq, D, device=DEV, generator=g) * 2
    k = torch.randn(B, Lk, D, device=DEV, generator=g) * 2
    v = torch.randn(B, Lk, D, device=DEV, generator=g).clamp(-4, 4)
    want = _ref64(q, k, v, H)
    e3 = (K.attention_f32(q, k, v, H, form="f16x3").double() - want).abs().max().item()
    e6 = (K.attention_f32(q, k, v, H, form="x6").double() - want).abs().max().item()
    print(f"\nB={B} H={H} Lq={Lq} Lk={Lk}: f16x3 {e3:.2e}  x6 {e6:.2e}")
    assert e3 <= 1e-5 * 4, (e3, e6)


@torch.no_grad()
def test_attention_f16x3_strided_qkv_views():
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(17)
    qkv = torch.randn(2, 150, 3 * 512, device=DEV, generator=g)
    q, k, v = qkv.split(512, dim=-1)
    got = K.attention_f32(q, k, v, 8, form="f16x3")
    assert (got.double() - _ref64(q, k, v, 8)).abs().max().item() <= 1e-5 * 4


@torch.no_grad()
@pytest.mark.parametrize("shape", [(3, 2, 100, 90), (4, 2, 302, 90)])  # 1 / 2 query parts per head
@pytest.mark.parametrize("case", ["huge_q", "huge_k", "huge_v", "tiny_v_dim", "tiny_all", "zero_v_dim", "tiny_q",
                                  "tiny_k"])
def test_attention_f16x3_range_and_block_independence(case, shape):
    """Out-of-f16-range inputs in ONE batch item (|k| or |v| >= 2^15, a max |k| or a head dimension
    of V whose max is below 2^-6, everything scaled by 1e-6) re-run that item's blocks on the bf16x6
    kernel: the result stays within f32 accuracy of f64 relative to each item's own output scale, the
    re-run blocks equal the bf16x6 kernel bit for bit, and the other items are bit-identical to a run
    without the odd item.  Queries of any magnitude stay on the f16x3 kernel (each query is scaled by
    a power of two before the split): tiny queries against large keys (S of order 1, so the
    softmax sees the queries' low bits) keep f32 accuracy without a re-run."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(7)
    B, H, Lq, Lk = shape
    D = H * 64
    q = torch.randn(B, Lq, D, device=DEV, generator=g)
    k = torch.randn(B, Lk, D, device=DEV, generator=g)
    v = torch.randn(B, Lk, D, device=DEV, generator=g)
    base = K.attention_f32(q, k, v, H, form="f16x3")
    if case == "huge_q":
        q[1] *= 1e5
        k[1] *= 1e-5
    elif case == "huge_k":
        k[1, :, :64] *= 4e4
        q[1, :, :64] *= 1e-4
    elif case == "huge_v":
        v[1, 5, 70] = 1e6
    elif case == "tiny_v_dim":
        v[1, :, 3] *= 1e-4
    elif case == "tiny_all":
        q[1] *= 1e-6
        k[1] *= 1e-6
        v[1] *= 1e-6
    elif case == "zero_v_dim":
        v[1, :, 3] = 0.0
    elif case == "tiny_q":  # every |q| < 2^-3: an unscaled low piece would be subnormal
        q[1] *= 1e-3
        k[1] *= 100.0
    elif case == "tiny_k":  # |k| ~ 1e-6 against large queries: re-run (kh would be subnormal)
        k[1] *= 1e-6
        q[1] *= 1e5
    got = K.attention_f32(q, k, v, H, form="f16x3")
    x6 = K.attention_f32(q, k, v, H, form="x6")
    want = _ref64(q, k, v, H)
    torch.cuda.synchronize()
    for b in range(B):
        scale = want[b].abs().max().item()
        err = (got[b].double() - want[b]).abs().max().item() / scale
        assert err < 1e-6, (case, b, err)
    for b in range(B):
        if b != 1:
            assert torch.equal(got[b], base[b])
    if case in ("huge_q", "tiny_all", "tiny_k"):
        assert torch.equal(got[1], x6[1]), case  # every block of item 1 re-ran on bf16x6 (tiny |k|)
    if case == "tiny_q":  # no re-run: item 1 is the f16x3 kernel's own result
        assert not torch.equal(got[1], x6[1])
    if case in ("huge_k", "tiny_v_dim"):  # head 0 re-ran, head 1 kept its f16x3 result
        assert torch.equal(got[1, :, :64], x6[1, :, :64])
        assert torch.equal(got[1, :, 64:], base[1, :, 64:])
    if case == "huge_v":  # head 1 re-ran, head 0 kept its f16x3 result
        assert torch.equal(got[1, :, 64:], x6[1, :, 64:])
        assert torch.equal(got[1, :, :64], base[1, :, :64])
    if case == "tiny_v_dim":  # the small dimension itself to f32 accuracy
        d3 = (got[1, :, 3].double() - want[1, :, 3]).abs().max().item() / want[1, :, 3].abs().max().item()
        assert d3 < 1e-6, d3
    if case == "zero_v_dim":  # no re-run; the zero dimension stays exactly zero
        assert torch.equal(got[1, :, 3], torch.zeros_like(got[1, :, 3]))


@torch.no_grad()
@pytest.mark.parametrize("B,H,Lq,Lk,case", [(3, 8, 302, 302, None), (2, 8, 100, 302, None), (4, 8, 100, 100, None),
                                             (1, 2, 1, 1, None), (2, 2, 257, 33, None), (1, 1, 130, 650, None),
                                             (3, 2, 302, 90, "huge_k"), (3, 2, 100, 90, "tiny_v_dim")])
@pytest.mark.parametrize("form", ["1", "2", "3", "1x", "2x", "3x"])
def test_attention_f16x3_dma_staging_equals_register_staging(monkeypatch, B, H, Lq, Lk, case, form):
    """The LDS-DMA-staged f16x3 kernel (the default, RMBX_ATTN_DMA=1: raw tiles by LDS-DMA, pieces
    split once per block, V^T read through ds_read_b64_tr_b16; form 2 also runs K one tile ahead of V
    so S^T of the next tile overlaps the softmax; form 3: one raw stage, three blocks per CU; "x": the
    parts of a head on one XCD) computes the register-staged kernel's
    pieces in the same MFMA order: bitwise-equal outputs, including ragged key tiles, query parts
    past Lq, long key sequences and re-run (flagged) blocks."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(Lq * 7 + Lk)
    D = H * 64
    q = torch.randn(B, Lq, D, device=DEV, generator=g) * 2
    k = torch.randn(B, Lk, D, device=DEV, generator=g) * 2
    v = torch.randn(B, Lk, D, device=DEV, generator=g)
    if case == "huge_k":
        k[1, :, :64] *= 4e4
    elif case == "tiny_v_dim":
        v[1, :, 3] *= 1e-4
    monkeypatch.setenv("RMBX_ATTN_DMA", form[0])
    monkeypatch.setenv("RMBX_ATTN_XCD", "1" if form.endswith("x") else "0")
    dma = K.attention_f32(q, k, v, H, form="f16x3")
    monkeypatch.setenv("RMBX_ATTN_DMA", "0")
    reg = K.attention_f32(q, k, v, H, form="f16x3")
    torch.cuda.synchronize()
    assert torch.equal(dma, reg)
    if case is not None:  # item 1's first head re-ran on bf16x6
        assert torch.equal(dma[1, :, :64], K.attention_f32(q, k, v, H, form="x6")[1, :, :64])


@torch.no_grad()
def test_attention_f16x3_non_finite_inputs():
    """A NaN in V propagates to the outputs that use it (as in f32); an inf in K re-runs the block on
    bf16x6 and gives that kernel's result."""
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(9)
    q = torch.randn(2, 40, 64, device=DEV, generator=g)
    k = torch.randn(2, 40, 64, device=DEV, generator=g)
    v = torch.randn(2, 40, 64, device=DEV, generator=g)
    v[0, 3, 5] = float("nan")
    k[1, 2, 7] = float("inf")
    got = K.attention_f32(q, k, v, 1, form="f16x3")
    x6 = K.attention_f32(q, k, v, 1, form="x6")
    assert torch.isnan(got[0, :, 5]).all()
    assert torch.equal(got[1].isnan(), x6[1].isnan())
    assert torch.equal(torch.nan_to_num(got[1]), torch.nan_to_num(x6[1]))
