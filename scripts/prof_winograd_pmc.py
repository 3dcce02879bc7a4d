"""PMC driver: calibration copies (scripts/pmc_calib.hip, 512 MiB read + written per launch) then the
Winograd f32 conv (bias + residual + ReLU) at the four ResNet-18 stride-1 layer shapes of the ACT
trunk (64ch 120x160, 128ch 60x80, 256ch 30x40, 512ch 15x20), 1024 frames, 3 launches each, in that
order -- run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes
(scripts/gpurun/wino_pmc.sh) to measure its HBM traffic per launch against the algorithmic bytes
(input + residual + output, each N*H*W*C*4 B, + the packed filter transform);
tools/pmc_traffic.py --winograd reduces the two passes.

    python3 scripts/prof_winograd_pmc.py [--tile f4|f2]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

SHAPES = ((64, 120, 160), (128, 60, 80), (256, 30, 40), (512, 15, 20))

ap = argparse.ArgumentParser()
ap.add_argument("--tile", choices=["f4", "f2"], default="f4")
ap.add_argument("--frames", type=int, default=1024)
a = ap.parse_args()
pack, conv = ((K.pack_winograd4_f32, K.conv3x3_winograd4_f32) if a.tile == "f4"
              else (K.pack_winograd_f32, K.conv3x3_winograd_f32))

cal = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libpmc_calib.so"))
cal.pmc_calib.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
nb = 512 << 20
x = torch.zeros(nb // 8, dtype=torch.float64, device="cuda")
y = torch.empty_like(x)
for wide in (0, 1, 0, 1):
    assert cal.pmc_calib(x.data_ptr(), y.data_ptr(), nb, wide, None) == 0
torch.cuda.synchronize()
del x, y
cl = torch.channels_last
with torch.no_grad():
    for C, H, W in SHAPES:
        B = a.frames
        xin = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=cl)
        r = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=cl)
        u = pack(torch.randn(C, C, 3, 3, device="cuda") / (9 * C) ** 0.5)
        b = torch.randn(C, device="cuda")
        torch.cuda.synchronize()
        for _ in range(3):
            conv(xin, u, b, relu=True, res=r)
        torch.cuda.synchronize()
        print(f"{a.tile} C={C} {H}x{W}: algorithmic bytes per launch {3 * B * H * W * C * 4 + u.numel() * 4}",
              flush=True)
        del xin, r
