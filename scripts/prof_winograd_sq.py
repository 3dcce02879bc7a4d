"""SQ counter driver for the Winograd F(4x4) conv: 3 launches at each of the 512- and 64-channel
ACT trunk shapes (1024 frames) per RMBX_WINO4_VAR value given, in that order; run under
`rocprofv3 --pmc <8 SQ counters>` passes (scripts/gpurun/wino_sq.sh).

    python3 scripts/prof_winograd_sq.py 0,16
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

VARS = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0"]
cl = torch.channels_last
with torch.no_grad():
    for C, H, W in ((512, 15, 20), (64, 120, 160)):
        x = torch.randn(1024, C, H, W, device="cuda").contiguous(memory_format=cl)
        r = torch.randn(1024, C, H, W, device="cuda").contiguous(memory_format=cl)
        w = torch.randn(C, C, 3, 3, device="cuda") / (9 * C) ** 0.5
        b = torch.randn(C, device="cuda")
        for v in VARS:
            os.environ["RMBX_WINO4_VAR"] = v
            u = K.pack_winograd4_f32(w)
            torch.cuda.synchronize()
            for _ in range(3):
                K.conv3x3_winograd4_f32(x, u, b, relu=True, res=r)
            torch.cuda.synchronize()
            print(f"C={C} var={v}: 3 launches", flush=True)
        del x, r
