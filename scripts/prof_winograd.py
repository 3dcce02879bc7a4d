"""Diagnostic: the fp32 stride-1 3x3 convs of the ResNet-18 trunk at rollout batch B (480 x 640
images: 64ch 120x160, 128ch 60x80, 256ch 30x40, 512ch 15x20) with bias + residual + ReLU:
rmbx_conv3x3_winograd_f32 vs the direct paths it replaces (rmbx_conv2d_nhwc_f32 for 64 channels,
MIOpen conv + the rmbx epilogue pass otherwise), timed with HIP events; TF/s on the direct
algorithm's 2 * 9 * C * C FLOP per pixel (the Winograd kernel executes 4/9 of them on MFMA)."""
import json
import os
import sys

os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

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
    shapes = ((64, 120, 160), (128, 60, 80), (256, 30, 40), (512, 15, 20))
    only = os.environ.get("WINO_C")
    for C, H, W in shapes:
        if only and str(C) not in only.split(","):
            continue
        x = torch.randn(B, C, H, W, device=dev).contiguous(memory_format=cl)
        r = torch.randn(B, C, H, W, device=dev).contiguous(memory_format=cl)
        w = (torch.randn(C, C, 3, 3, device=dev) / (9 * C) ** 0.5).contiguous(memory_format=cl)
        b = torch.randn(C, device=dev)
        u = K.pack_winograd_f32(w)
        flop = 2.0 * B * H * W * C * C * 9
        ms_w = timed(lambda: K.conv3x3_winograd_f32(x, u, b, relu=True, res=r))
        if C == 64:
            ms_d = timed(lambda: K.conv2d_nhwc(x, w, b, 1, 1, relu=True, res=r))
            direct = "rmbx_conv2d_nhwc_f32"
        else:
            def miopen():
                y = F.conv2d(x, w, None, 1, 1)
                return K.nhwc_bias_act(y, b, res=r, relu=True, out=y)
            ms_d = timed(miopen)
            direct = "miopen+epilogue"
        ref = F.relu(F.conv2d(x[:8], w, b, 1, 1) + r[:8])
        got = K.conv3x3_winograd_f32(x[:8].contiguous(memory_format=cl), u, b, relu=True,
                                     res=r[:8].contiguous(memory_format=cl))
        err = (got - ref).abs().max().item() / max(1.0, ref.abs().max().item())
        dbg = {}
        for stg in os.environ.get("WINO_STAGGERS", "").split(","):
            if stg:
                os.environ["RMBX_WINO_STAGGER"] = stg
                dbg["stagger" + stg] = round(timed(lambda: K.conv3x3_winograd_f32(x, u, b, relu=True, res=r)), 3)
        os.environ.pop("RMBX_WINO_STAGGER", None)
        for d in os.environ.get("WINO_DBGS", "2,4,6,15").split(","):  # phase skips (RMBX_WINO_DBG bits)
            os.environ["RMBX_WINO_DBG"] = d
            dbg["dbg" + d] = round(timed(lambda: K.conv3x3_winograd_f32(x, u, b, relu=True, res=r)), 3)
        os.environ.pop("RMBX_WINO_DBG")
        print(json.dumps({"B": B, "C": C, "H": H, "W": W, "winograd_ms": round(ms_w, 3), **dbg,
                          "winograd_tflops_direct_equiv": round(flop / ms_w / 1e9, 1),
                          "winograd_mfma_frac_of_157": round(flop * 4 / 9 / ms_w / 1e9 / 157.3, 3),
                          "direct": direct, "direct_ms": round(ms_d, 3), "speedup": round(ms_d / ms_w, 2),
                          "max_rel_err_vs_miopen": err}), flush=True)
        del x, r
