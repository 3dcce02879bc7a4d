"""The patch-staged f16x3 3x3 conv (rmbx_conv3x3_f16x3_patch) vs the current paths at the ACT
backbone's stride-1 shapes, 1024 frames: 64 channels at 120 x 160 vs the fused f32 Winograd
F(4x4) and the f16x3 implicit GEMM; 128 channels at 60 x 80 vs the implicit GEMM.  Rounds
interleaved in one process, HIP events; error of each vs f64 on 2 frames."""
import os
import sys

import torch
import torch.nn.functional as F

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


with torch.no_grad():
    for C, H, W in ((64, 120, 160), (128, 60, 80)):
        n = 1024
        x = torch.randn(n, C, H, W, device=dev, generator=g).clamp_min(0).contiguous(memory_format=torch.channels_last)
        w = torch.randn(C, C, 3, 3, device=dev, generator=g) / (9 * C) ** 0.5
        b = torch.randn(C, device=dev, generator=g)
        r = torch.randn(n, C, H, W, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        p = K.pack_conv_f32x6(w)
        def patch_cfg(cfg):
            def f():
                os.environ["RMBX_CONVP_CFG"] = cfg
                return K.conv3x3_f16x3_patch(x, p, b, relu=True, res=r)
            return f
        ops = {"patch": patch_cfg("0"), "patch2": patch_cfg("1"),
               "gemm": lambda: K.conv2d_f32x6(x, p, b, 3, 1, 1, relu=True, res=r)}
        if C == 64:
            u = K.pack_winograd4_f32(w) if hasattr(K, "pack_winograd4_f32") else None
            if u is not None:
                ops["winograd4"] = lambda: K.conv3x3_winograd4_f32(x, u, b, relu=True, res=r)
        ref = F.conv2d(x[:2].double(), w.double(), b.double(), 1, 1) + r[:2].double()
        ref = ref.clamp_min(0)
        errs = {k: ((f()[:2].double() - ref).abs().max() / ref.abs().max()).item() for k, f in ops.items()}
        ts = {k: [] for k in ops}
        for _ in range(3):
            for k, f in ops.items():
                f()
                torch.cuda.synchronize()
                ts[k].append(timeit(f))
        fl = 2.0 * n * H * W * C * C * 9
        print(f"C={C} {H}x{W} x{n}: " + " | ".join(
            f"{k} {min(t):.3f} ms ({fl / min(t) / 1e9:.0f} TF/s direct, err {errs[k]:.1e})" for k, t in ts.items()),
            flush=True)
        del x, r
