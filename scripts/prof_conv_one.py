"""Diagnostic: the layer1 3x3 conv (64 -> 64, 120x160, batch 1024) under each rmbx kernel variant
and diagnostic phase skip (RMBX_CONV_DBG bits: 1 no MFMA phase, 2 no epilogue, 4 no global
loads), timed with events; also usable under rocprofv3 --pmc."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = "cuda:0"
with torch.no_grad():
    x = torch.randn(B, 64, 120, 160, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 64, 3, 3, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    bias = torch.randn(64, device=dev)
    r = torch.randn(B, 64, 120, 160, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for variant, dbg, res in [("resident", 0, None), ("resident", 0, r), ("resident", 1, None), ("resident", 2, None),
                              ("resident", 4, None), ("resident", 3, None), ("resident", 6, None),
                              ("resident", 5, None), ("streaming", 0, None)]:
        os.environ["RMBX_CONV_DBG"] = str(dbg)
        if variant == "streaming":
            os.environ["RMBX_CONV_NO_RESIDENT"] = "1"
        K.conv2d_nhwc(x, w, bias, 1, 1, relu=True, res=res)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            K.conv2d_nhwc(x, w, bias, 1, 1, relu=True, res=res)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"variant": variant, "dbg": dbg, "res": res is not None, "ms": round(e0.elapsed_time(e1) / 5, 3)}), flush=True)
    os.environ["RMBX_CONV_DBG"] = "0"
