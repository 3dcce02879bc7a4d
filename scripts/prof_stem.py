"""Diagnostic: the ResNet-18 stem at batch B on 480x640 frames — unfused (rmbx_stem_s2d_conv +
rmbx_nhwc_bias_relu_maxpool) vs fused (rmbx_stem_s2d_conv_maxpool), bf16, and the fused f32 form
(rmbx_stem_s2d_conv_maxpool_f32, the fp32 policy's stem) against the f32 MFMA peak, timed with
HIP events."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = "cuda:0"


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


with torch.no_grad():
    xs = torch.rand(B, 240, 320, 16, device=dev).to(torch.bfloat16)
    wp = (torch.randn(64, 4, 4, 16, device=dev) * 0.1).to(torch.bfloat16)
    b = torch.randn(64, device=dev)
    z = torch.zeros(64, device=dev)
    flop = 2.0 * B * 240 * 320 * 64 * 7 * 7 * 3  # algorithmic (7x7x3 taps)
    ms_conv = timed(lambda: K.stem_s2d_conv(xs, wp, b))
    s = K.stem_s2d_conv(xs, wp, b)
    ms_pool = timed(lambda: K.nhwc_bias_relu_maxpool(s, z))
    del s
    ms_fused = timed(lambda: K.stem_s2d_conv_maxpool(xs, wp, b))
    io = B * (240 * 320 * 16 + 120 * 160 * 64) * 2
    print(json.dumps({"B": B, "unfused_conv_ms": round(ms_conv, 3), "unfused_pool_ms": round(ms_pool, 3),
                      "fused_ms": round(ms_fused, 3), "fused_tflops_alg": round(flop / ms_fused / 1e9, 1),
                      "fused_io_gbs": round(io / ms_fused / 1e6, 1)}), flush=True)
    del xs
    xf = torch.rand(B, 240, 320, 16, device=dev)
    wf = K.pack_stem_s2d(torch.randn(64, 3, 7, 7, device=dev) * 0.1)
    ms_f32 = timed(lambda: K.stem_s2d_conv_maxpool(xf, wf, b))
    print(json.dumps({"B": B, "f32_fused_ms": round(ms_f32, 3), "f32_tflops_alg": round(flop / ms_f32 / 1e9, 1),
                      "f32_frac_of_157": round(flop / ms_f32 / 1e9 / 157.3, 3)}), flush=True)

