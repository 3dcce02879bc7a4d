"""The ResNet layer-1 conv (64 -> 64, 3x3 / stride 1, 120 x 160, 1024 frames, bias + residual +
ReLU): the fused f32 Winograd F(4x4) kernel vs the f16x3 implicit GEMM on its 64-column tile, HIP
events, rounds interleaved; error of each against the other."""
import sys

import torch

sys.path.insert(0, ".")
from robomanipbaselines_amd import kernels as K  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
cl = torch.channels_last
x = torch.randn(n, 64, 120, 160, device="cuda").clamp_min(0).contiguous(memory_format=cl)
r = torch.randn(n, 64, 120, 160, device="cuda").contiguous(memory_format=cl)
w = torch.randn(64, 64, 3, 3, device="cuda") / 24.0
b = torch.randn(64, device="cuda")
pw = K.pack_winograd4_f32(w)
pg = K.pack_conv_f32x6(w)
fns = {"winograd4_f32": lambda: K.conv3x3_winograd4_f32(x, pw, b, relu=True, res=r),
       "f16x3_gemm_bn64": lambda: K.conv2d_f32x6(x, pg, b, 3, 1, 1, relu=True, res=r)}
a, c = fns["winograd4_f32"](), fns["f16x3_gemm_bn64"]()
torch.cuda.synchronize()
print(f"max rel diff {((a - c).abs().max() / a.abs().max()).item():.2e}", flush=True)
ts = {k: [] for k in fns}
for _ in range(3):
    for k, f in fns.items():
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        ts[k].append(e0.elapsed_time(e1) / 5)
fl = 2.0 * n * 120 * 160 * 64 * 64 * 9
print(" | ".join(f"{k}: {min(t):.3f} ms ({fl / min(t) / 1e9:.1f} TF/s direct)" for k, t in ts.items()), flush=True)
