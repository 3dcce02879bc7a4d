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
