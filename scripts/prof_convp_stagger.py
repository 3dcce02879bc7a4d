"""(A/B probe: the forms it selects were measured slower or no faster and removed from
csrc/rmbx_convp.hip; DESIGN.md, not-adopted list)  Start-phase stagger of the patch-staged f16x3 conv (RMBX_CONVP_STAGGER="n:ticks": the persistent
blocks start in n phases ticks x 10 ns apart, so their epilogues' residual reads / output writes
do not all hit HBM at once), 1024 frames at the backbone's 64 / 128-channel shapes, with and
without the residual; outputs compared bitwise with the unstaggered run (HIP events, rounds
interleaved in one process)."""
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


CASES = {64: ("", "2:1750", "4:875", "2:900", "8:440"), 128: ("", "2:2950", "4:1475", "8:740")}
with torch.no_grad():
    for C, H, W in ((64, 120, 160), (128, 60, 80)):
        n = 1024
        x = torch.randn(n, C, H, W, device=dev, generator=g).clamp_min(0).contiguous(memory_format=torch.channels_last)
        w = torch.randn(C, C, 3, 3, device=dev, generator=g) / (9 * C) ** 0.5
        b = torch.randn(C, device=dev, generator=g)
        r = torch.randn(n, C, H, W, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        p = K.pack_conv_f32x6(w)
        for res in (r, None):
            ts = {v: [] for v in CASES[C]}
            ref = None
            same = {}
            for _ in range(3):
                for v in CASES[C]:
                    os.environ["RMBX_CONVP_STAGGER"] = v
                    y = K.conv3x3_f16x3_patch(x, p, b, relu=True, res=res)
                    torch.cuda.synchronize()
                    if v == "":
                        ref = y.clone()
                    same[v] = bool(torch.equal(y, ref))
                    del y
                    ts[v].append(timeit(lambda: K.conv3x3_f16x3_patch(x, p, b, relu=True, res=res)))
            os.environ.pop("RMBX_CONVP_STAGGER")
            ex = 3 * 2.0 * n * H * W * C * C * 9
            tag = "res" if res is not None else "nores"
            print(f"C={C} {H}x{W} {tag}: " + " | ".join(
                f"'{v}': {min(t):.3f} ms ({ex / min(t) / 1e9 / 2500:.3f}){'' if same[v] else ' DIFF'}"
                for v, t in ts.items()), flush=True)
        del x, r
