"""(A/B probe: the forms it selects were measured slower or no faster and removed from
csrc/rmbx_convp.hip; DESIGN.md, not-adopted list)  Patch-staged f16x3 conv forms at the backbone's 64 / 128-channel shapes, 1024 frames, with and
without the residual: RMBX_CONVP_CFG 0 (8-wave blocks, one per CU) vs 2 (4-wave 16 x 16 x 64 blocks,
two per CU), each with and without a start stagger (RMBX_CONVP_STAGGER); outputs compared with cfg 0
(HIP events, rounds interleaved in one process)."""
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


FORMS = {64: (("0", ""), ("0", "2:1750"), ("2", ""), ("2", "2:1750"), ("2", "2:900"), ("3", "")),
         128: (("0", ""), ("0", "2:2950"), ("2", ""), ("2", "2:3500"), ("2", "2:1750"))}
with torch.no_grad():
    for C, H, W in ((64, 120, 160), (128, 60, 80)):
        n = 1024
        x = torch.randn(n, C, H, W, device=dev, generator=g).clamp_min(0).contiguous(memory_format=torch.channels_last)
        w = torch.randn(C, C, 3, 3, device=dev, generator=g) / (9 * C) ** 0.5
        b = torch.randn(C, device=dev, generator=g)
        r = torch.randn(n, C, H, W, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        p = K.pack_conv_f32x6(w)
        for res in (r, None):
            ts = {f: [] for f in FORMS[C]}
            diff = {}
            ref = None
            for _ in range(3):
                for f in FORMS[C]:
                    os.environ["RMBX_CONVP_CFG"], os.environ["RMBX_CONVP_STAGGER"] = f
                    y = K.conv3x3_f16x3_patch(x, p, b, relu=True, res=res)
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = y.clone()
                    d = (y - ref).abs()
                    diff[f] = (int((y != ref).sum()), float(d.max()))
                    del y, d
                    ts[f].append(timeit(lambda: K.conv3x3_f16x3_patch(x, p, b, relu=True, res=res)))
            os.environ.pop("RMBX_CONVP_CFG")
            os.environ.pop("RMBX_CONVP_STAGGER")
            ex = 3 * 2.0 * n * H * W * C * C * 9
            tag = "res" if res is not None else "nores"
            for f, t in ts.items():
                print(f"C={C} {H}x{W} {tag} cfg {f[0]} stagger '{f[1]}': {min(t):.3f} ms ({ex / min(t) / 1e9 / 2500:.3f})"
                      f"  vs cfg 0: {diff[f][0]} differing, max {diff[f][1]:.2e}", flush=True)
        del x, r
