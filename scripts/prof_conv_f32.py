"""Diagnostic: the ResNet-18 layer-1 conv (64 -> 64, 3x3, 120 x 160) in f32 at batch B: the fused
rmbx_conv2d_nhwc_f32 vs MIOpen's conv + the rmbx bias/residual/ReLU pass (the f32 path it
replaces), timed with HIP events; TF/s on the algorithmic 2 * 9 * 64 * 64 FLOP per pixel."""
import json
import os
import sys

import torch
import torch.nn.functional as F

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
    torch.backends.cudnn.benchmark = True
    torch.backends.cudnn.allow_tf32 = False
    cl = torch.channels_last
    x = torch.randn(B, 64, 120, 160, device=dev).contiguous(memory_format=cl)
    r = torch.randn(B, 64, 120, 160, device=dev).contiguous(memory_format=cl)
    w = (torch.randn(64, 64, 3, 3, device=dev) / 24).contiguous(memory_format=cl)
    b = torch.randn(64, device=dev)
    flop = 2.0 * B * 120 * 160 * 64 * 64 * 9
    out = {"B": B}
    for name, res in (("relu", None), ("res_relu", r)):
        ms_r = timed(lambda: K.conv2d_nhwc(x, w, b, 1, 1, relu=True, res=res))

        def miopen():
            y = F.conv2d(x, w, None, 1, 1)
            return K.nhwc_bias_act(y, b, res=res, relu=True, out=y)

        ms_m = timed(miopen)
        ms_mc = timed(lambda: F.conv2d(x, w, None, 1, 1))
        out[name] = {"rmbx_f32_ms": round(ms_r, 3), "rmbx_tflops": round(flop / ms_r / 1e9, 1),
                     "rmbx_frac_of_157": round(flop / ms_r / 1e9 / 157.3, 3),
                     "miopen_conv_plus_epi_ms": round(ms_m, 3), "miopen_conv_ms": round(ms_mc, 3)}
    for dbg in ("1", "2", "3", "6"):  # phase skips: no MFMAs / no patch loads / neither / MFMAs + barriers only
        os.environ["RMBX_CONV_DBG"] = dbg
        out["dbg" + dbg + "_ms"] = round(timed(lambda: K.conv2d_nhwc(x, w, b, 1, 1, relu=True, res=r)), 3)
    os.environ.pop("RMBX_CONV_DBG")
    print(json.dumps(out), flush=True)
