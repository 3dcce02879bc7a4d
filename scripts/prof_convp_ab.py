"""Patch-staged f16x3 conv at the backbone's 64 / 128-channel shapes, 1024 frames, with and without
the residual: one line per case for the library this process loaded (RMBX_LIB_VARIANT selects a
build_variant.py build; run once per variant, interleaved, for an A/B), plus a checksum of the
outputs so variants can be compared bitwise."""
import os
import sys

import torch

sys.path.insert(0, ".")
from robomanipbaselines_amd import kernels as K  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)


def timeit(f, reps=5):
    f()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


tag = os.environ.get("RMBX_LIB_VARIANT") or "default"
with torch.no_grad():
    for C, H, W in ((64, 120, 160), (128, 60, 80)):
        n = 1024
        x = torch.randn(n, C, H, W, device=dev, generator=g).clamp_min(0).contiguous(memory_format=torch.channels_last)
        w = torch.randn(C, C, 3, 3, device=dev, generator=g) / (9 * C) ** 0.5
        b = torch.randn(C, device=dev, generator=g)
        r = torch.randn(n, C, H, W, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        p = K.pack_conv_f32x6(w)
        for res in (r, None):
            y = K.conv3x3_f16x3_patch(x, p, b, relu=True, res=res)
            torch.cuda.synchronize()
            ck = float(y.double().sum())
            del y
            t = timeit(lambda: K.conv3x3_f16x3_patch(x, p, b, relu=True, res=res))
            ex = 3 * 2.0 * n * H * W * C * C * 9
            print(f"[{tag}] C={C} {H}x{W} {'res' if res is not None else 'nores'}: {t:.3f} ms ({ex / t / 1e9 / 2500:.3f})"
                  f" checksum {ck:.10e}", flush=True)
        del x, r
