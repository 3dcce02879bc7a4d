"""CPU check of the Winograd F(2x2, 3x3) data path of rmbx_conv3x3_winograd_f32: the packed filter
transform (kernels.pack_winograd_f32) and the kernel's input / output transform formulas,
emulated in numpy f64 and compared with the direct convolution (no GPU needed)."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F


def _emulate(x, up, bias, res, relu):
    """The kernel's arithmetic in f64: V = B^T d B per window (tmp rows, then columns, as the
    kernel's store pieces), M = sum_c U V from the packed layout, Y = A^T M A + bias (+ res)."""
    n, C, H, W = x.shape
    ty_n, tx_n = (H + 1) // 2, (W + 1) // 2
    xp = np.zeros((n, C, 2 * ty_n + 2, 2 * tx_n + 2))
    xp[:, :, 1:H + 1, 1:W + 1] = x
    # unpack U[p][co][ci] from [ncb][nk][16][64][8]
    ncb, nk = C // 64, C // 8
    U = np.zeros((16, C, C))
    for cb in range(ncb):
        for k in range(nk):
            U[:, cb * 64:(cb + 1) * 64, k * 8:(k + 1) * 8] = up[cb, k]
    out = np.zeros((n, C, H, W))
    for ty in range(ty_n):
        for tx in range(tx_n):
            d = xp[:, :, 2 * ty:2 * ty + 4, 2 * tx:2 * tx + 4]  # [n, C, 4, 4]
            t = np.stack([d[..., 0, :] - d[..., 2, :], d[..., 1, :] + d[..., 2, :],
                          d[..., 2, :] - d[..., 1, :], d[..., 1, :] - d[..., 3, :]], axis=-2)
            v = np.stack([t[..., 0] - t[..., 2], t[..., 1] + t[..., 2],
                          t[..., 2] - t[..., 1], t[..., 1] - t[..., 3]], axis=-1).reshape(n, C, 16)
            m = np.einsum("poc,ncp->nop", U, v).reshape(n, C, 4, 4)
            t0 = m[:, :, 0] + m[:, :, 1] + m[:, :, 2]
            t1 = m[:, :, 1] - m[:, :, 2] - m[:, :, 3]
            y = np.stack([np.stack([t0[..., 0] + t0[..., 1] + t0[..., 2], t0[..., 1] - t0[..., 2] - t0[..., 3]], -1),
                          np.stack([t1[..., 0] + t1[..., 1] + t1[..., 2], t1[..., 1] - t1[..., 2] - t1[..., 3]], -1)], -2)
            hh, ww = min(2, H - 2 * ty), min(2, W - 2 * tx)
            out[:, :, 2 * ty:2 * ty + hh, 2 * tx:2 * tx + ww] = y[:, :, :hh, :ww]
    out += bias[None, :, None, None]
    if res is not None:
        out += res
    return np.maximum(out, 0) if relu else out


@pytest.mark.parametrize("C,H,W,relu", [(64, 5, 7, True), (128, 4, 3, False)])
def test_packed_winograd_equals_direct_conv(C, H, W, relu):
    from robomanipbaselines_amd import kernels as K

    g = torch.Generator().manual_seed(C + H)
    x = torch.randn(2, C, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(C, C, 3, 3, generator=g, dtype=torch.float64) / (9 * C) ** 0.5
    b = torch.randn(C, generator=g, dtype=torch.float64)
    r = torch.randn(2, C, H, W, generator=g, dtype=torch.float64)
    up = K.pack_winograd_f32(w).double().numpy()
    assert up.shape == (C // 64, C // 8, 16, 64, 8)
    got = _emulate(x.numpy(), up, b.numpy(), r.numpy(), relu)
    ref = F.conv2d(x, w, b, 1, 1) + r
    ref = (F.relu(ref) if relu else ref).numpy()
    # the packed U is rounded to f32; everything else here is f64
    assert np.abs(got - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())
