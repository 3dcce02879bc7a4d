"""Per-layer timing of the f32 Winograd convs at ACT's trunk shapes (1024 frames of 480x640):
F(2x2, 3x3) (rmbx_conv3x3_winograd_f32) vs F(4x4, 3x3) (rmbx_conv3x3_winograd4_f32), with each one's error against the device's direct f32 conv on the first
two frames, and F(4x4) phase skips (RMBX_WINO_DBG: 1 no MFMAs, 2 no window loads, 4 no V
transform/stores, 8 no U loads, 14 = 2|4|8 the MFMA + LDS-read skeleton).

F(4x4) schedule variants (RMBX_WINO4_VAR bits: 1 split, 2 early window loads, 4 deep LDS prefetch,
16 buffer-load window gathers)
are timed side by side with --vars 0,2,4,6.

usage: python scripts/prof_winograd4.py [n_frames] [--dbg] [--vars 0,1]"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1024
dbg = "--dbg" in sys.argv
VARS = sys.argv[sys.argv.index("--vars") + 1].split(",") if "--vars" in sys.argv else ["0", "1"]
dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(0)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
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
    u2, u4 = K.pack_winograd_f32(w), K.pack_winograd4_f32(w)
    ref = F.relu(F.conv2d(x[:2].float(), w, b, 1, 1) + r[:2])
    flops = 2.0 * n * H * W * C * C * 9
    out = {}
    def f4(v):  # v: RMBX_WINO4_VAR value
        return lambda: K.conv3x3_winograd4_f32(x, u4, b, relu=True, res=r)

    for name, groups, fn in [("F2", None, lambda: K.conv3x3_winograd_f32(x, u2, b, relu=True, res=r))] + \
            [(f"F4v{v}", v, f4(v)) for v in VARS]:
        if groups:
            os.environ["RMBX_WINO4_VAR"] = groups
        y = fn()
        err = ((y[:2] - ref).abs().max() / ref.abs().max()).item()
        ms = timed(fn)
        ex = 2.0 * C * C * n * ((H + 1) // 2) * ((W + 1) // 2) * 16 if name == "F2" else \
            2.0 * C * C * n * ((H + 3) // 4) * ((W + 3) // 4) * 36
        out[name] = ms
        line = (f"C={C:3d} {H}x{W} {name}: {ms:7.3f} ms  direct-equiv {flops / ms / 1e9:7.1f} TF/s  "
                f"executed {ex / ms / 1e9:6.1f} TF/s ({ex / ms / 1e9 / 157.3:.2f} of f32 peak)  rel err {err:.2e}")
        if dbg and groups == "0":
            parts = []
            for d in ("1", "2", "4", "8", "14"):
                os.environ["RMBX_WINO_DBG"] = d
                parts.append(f"dbg{d} {timed(fn, 3):.3f}")
            os.environ["RMBX_WINO_DBG"] = "0"
            line += "  [" + ", ".join(parts) + "]"
        print(line, flush=True)
    print("  speedup vs F2: " + ", ".join(f"{k} {out['F2'] / v:.2f}x" for k, v in out.items() if k != "F2"), flush=True)
    del x, r
