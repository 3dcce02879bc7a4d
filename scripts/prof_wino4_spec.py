"""A/B of the F(4x4) Winograd conv's producer/consumer form (RMBX_WINO4_SPEC=1: operand prefetch 4
positions, =2: 1) against the default kernel, at ACT's trunk shapes over 1024 frames, interleaved
rounds in one process (HIP events), with the outputs compared bit for bit."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(0)


def timed(fn, reps=4):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


for C, H, W in ((64, 120, 160), (128, 60, 80), (256, 30, 40), (512, 15, 20)):
    x = torch.randn(n, C, H, W, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    r = torch.randn(n, C, H, W, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    w = torch.randn(C, C, 3, 3, device=dev, generator=g) / (9 * C) ** 0.5
    b = torch.randn(C, device=dev, generator=g)
    u = K.pack_winograd4_f32(w)
    fn = lambda: K.conv3x3_winograd4_f32(x, u, b, relu=True, res=r)  # noqa: E731
    outs, times = {}, {m: [] for m in ("0", "1", "2")}
    for m in times:
        os.environ["RMBX_WINO4_SPEC"] = m
        outs[m] = fn()
    torch.cuda.synchronize()
    for _ in range(4):
        for m in times:
            os.environ["RMBX_WINO4_SPEC"] = m
            times[m].append(timed(fn))
    fl = 2.0 * 36 * C * C * n * ((H + 3) // 4) * ((W + 3) // 4)
    line = f"C={C:3d} {H}x{W}:"
    for m, label in (("0", "default"), ("1", "spec pd4"), ("2", "spec pd1")):
        t = statistics.median(times[m])
        line += f"  {label} {t:6.3f} ms ({fl / t / 1e9 / 157.3:.3f} of f32 peak)"
    d1 = (outs["1"] - outs["0"]).abs().max().item()
    d2 = (outs["2"] - outs["0"]).abs().max().item()
    print(line + f"  | max |d| spec vs default {d1:.2e} / {d2:.2e}", flush=True)
    del x, r, outs
    torch.cuda.empty_cache()
os.environ["RMBX_WINO4_SPEC"] = "0"
