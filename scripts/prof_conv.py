"""Diagnostic: ResNet-18 block conv shapes at rollout batch size, rmbx implicit-GEMM conv (fused
epilogue) vs MIOpen conv + rmbx epilogue; ms and TFLOP/s per layer shape."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

torch.backends.cudnn.benchmark = True
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = "cuda:0"
shapes = [  # (cin, cout, H, W, k, stride)
    (64, 64, 120, 160, 3, 1), (64, 128, 120, 160, 3, 2), (128, 128, 60, 80, 3, 1), (64, 128, 120, 160, 1, 2),
    (128, 256, 60, 80, 3, 2), (256, 256, 30, 40, 3, 1), (256, 512, 30, 40, 3, 2), (512, 512, 15, 20, 3, 1)]


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


out = []
with torch.no_grad():
    for cin, cout, H, W, k, s in shapes:
        x = torch.randn(B, cin, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        bias = torch.randn(cout, device=dev)
        pad = k // 2
        ho, wo = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
        flop = 2.0 * B * ho * wo * cout * cin * k * k
        t_r = timeit(lambda: K.conv2d_nhwc(x, w, bias, s, pad, relu=True))
        def miopen():
            y = F.conv2d(x, w, None, s, pad)
            return K.nhwc_bias_act(y, bias, relu=True, out=y)
        t_m = timeit(miopen)
        t_c = timeit(lambda: F.conv2d(x, w, None, s, pad))
        out.append({"shape": [cin, cout, H, W, k, s], "rmbx_ms": round(t_r, 3), "miopen_epi_ms": round(t_m, 3),
                    "miopen_conv_ms": round(t_c, 3), "rmbx_tflops": round(flop / t_r / 1e9, 1),
                    "miopen_tflops": round(flop / t_c / 1e9, 1)})
        print(json.dumps(out[-1]), flush=True)
    # stem: 7x7/s2 over the 480x640 image (MIOpen on NCHW->NHWC) vs rmbx s2d kernel
    img = torch.randn(B, 3, 480, 640, device=dev).to(torch.bfloat16)
    w = (torch.randn(64, 3, 7, 7, device=dev) * 0.1).to(torch.bfloat16)
    bias = torch.randn(64, device=dev)
    x_cl = img.contiguous(memory_format=torch.channels_last)
    w_cl = w.contiguous(memory_format=torch.channels_last)
    s2d = K.image_to_s2d(img)
    wp = K.pack_stem_s2d(w)
    flop = 2.0 * B * 240 * 320 * 64 * 147
    t_m = timeit(lambda: F.conv2d(x_cl, w_cl, None, 2, 3))
    t_r = timeit(lambda: K.stem_s2d_conv(s2d, wp, bias))
    print(json.dumps({"shape": "stem 7x7/2 3->64 480x640", "rmbx_s2d_ms": round(t_r, 3), "miopen_conv_ms": round(t_m, 3),
                      "rmbx_tflops": round(flop / t_r / 1e9, 1), "miopen_tflops": round(flop / t_m / 1e9, 1)}), flush=True)
