"""TEST INFRASTRUCTURE ONLY (the oracle; never imported by the product path).

numpy restatement of the OpenCV resize the reference applies to policy images
(cv2.resize(image, image_size) with the default INTER_LINEAR: policy/diffusion_policy/
RolloutDiffusionPolicy.py:112, policy/diffusion_policy_3d/RolloutDiffusionPolicy3d.py:140-141),
following OpenCV's published algorithm: an exact 2x down-scale goes to the area-fast path
(2x2 mean, u8 rounding (s + 2) >> 2, f32 mean * 0.25); otherwise fx = (x + 0.5) * scale - 0.5
clamped at the borders, u8 with 11-bit fixed-point weights and (sum + 2^21) >> 22 (the scalar
vertical pass), f32 with float weights.  OpenCV is not installed here: parity vs cv2 itself is
UNPINNED.  Then ToDtype(float32, scale=True) (v * (1/255)) and the affine / centre crop.
"""

import numpy as np


def _coords(dsize, ssize):
    scale = ssize / dsize
    d = np.arange(dsize)
    fx = ((d + 0.5) * scale - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx).astype(np.float32)
    lo = sx < 0
    fx[lo], sx[lo] = 0, 0
    hi = sx >= ssize - 1
    fx[hi], sx[hi] = 0, ssize - 1
    s1 = np.minimum(sx + 1, ssize - 1)
    c0 = np.rint((np.float32(1) - fx) * np.float32(2048)).astype(np.int64)
    return sx, s1, fx, c0, 2048 - c0


def resize_u8(img, size):
    """img u8 [H, W, C], size = (rw, rh) -> u8 [rh, rw, C]."""
    H, W, C = img.shape
    rw, rh = size
    x = img.astype(np.int64)
    if W == 2 * rw and H == 2 * rh:
        return ((x[0::2, 0::2] + x[0::2, 1::2] + x[1::2, 0::2] + x[1::2, 1::2] + 2) >> 2).astype(np.uint8)
    sx0, sx1, _, cx0, cx1 = _coords(rw, W)
    sy0, sy1, _, cy0, cy1 = _coords(rh, H)
    h = x[:, sx0] * cx0[None, :, None] + x[:, sx1] * cx1[None, :, None]
    v = (h[sy0] * cy0[:, None, None] + h[sy1] * cy1[:, None, None] + (1 << 21)) >> 22
    return np.clip(v, 0, 255).astype(np.uint8)


def resize_f32(img, size):
    """img f32 [H, W] -> [rh, rw]."""
    H, W = img.shape
    rw, rh = size
    f = np.float32
    if W == 2 * rw and H == 2 * rh:
        return (((img[0::2, 0::2] + img[0::2, 1::2]) + img[1::2, 0::2]) + img[1::2, 1::2]) * f(0.25)
    sx0, sx1, fx, _, _ = _coords(rw, W)
    sy0, sy1, fy, _, _ = _coords(rh, H)
    h = img[:, sx0] * (f(1) - fx)[None] + img[:, sx1] * fx[None]
    return h[sy0] * (f(1) - fy)[:, None] + h[sy1] * fy[:, None]


def policy_image(img, size, crop, a, b):
    """u8 HWC frame -> f32 CHW policy input: resize, crop (y0, x0, ch, cw), v/255*a+b."""
    r = resize_u8(img, size)
    y0, x0, ch, cw = crop
    r = r[y0:y0 + ch, x0:x0 + cw]
    v = r.astype(np.float32) * np.float32(1.0 / 255.0)
    v = v * np.float32(a) + np.float32(b)
    return np.moveaxis(v, -1, 0)
