"""Phase skips of the patch-staged f16x3 conv at the backbone's shapes, 1024 frames: RMBX_CONVP_VAR
= 0 (default), 1 (no epilogue), 2 (no patch re-staging), 4 (no W staging), 7 (MFMA loop + barriers
only); wrong results except 0, timing only (HIP events, rounds interleaved in one process)."""
import os
import sys

import torch

sys.path.insert(0, ".")
from robomanipbaselines_amd import kernels as K  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)


def timeit(f, reps=3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


VARS = ("0", "1", "2", "4", "7")
with torch.no_grad():
    for C, H, W in ((64, 120, 160), (128, 60, 80)):
        n = 1024
        x = torch.randn(n, C, H, W, device=dev, generator=g).clamp_min(0).contiguous(memory_format=torch.channels_last)
        w = torch.randn(C, C, 3, 3, device=dev, generator=g) / (9 * C) ** 0.5
        b = torch.randn(C, device=dev, generator=g)
        r = torch.randn(n, C, H, W, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        p = K.pack_conv_f32x6(w)
        ts = {v: [] for v in VARS}
        for _ in range(3):
            for v in VARS:
                os.environ["RMBX_CONVP_VAR"] = v
                K.conv3x3_f16x3_patch(x, p, b, relu=True, res=r)
                torch.cuda.synchronize()
                ts[v].append(timeit(lambda: K.conv3x3_f16x3_patch(x, p, b, relu=True, res=r)))
        os.environ.pop("RMBX_CONVP_VAR")
        ex = 3 * 2.0 * n * H * W * C * C * 9
        print(f"C={C} {H}x{W}: " + " | ".join(f"{v}: {min(t):.3f} ms ({ex / min(t) / 1e9 / 2500:.3f})"
                                              for v, t in ts.items()), flush=True)
        del x, r
