"""Diagnostic for the round-2 DP capture crash (profiles/r2_dp_capture_1024_fp32_100steps_segv.log):
that log's last line ("[87.1s] eager loop") is printed after a device synchronize, so the eager
100-step loop had finished and the process died in conditional_sample(use_graph=True): the
warm-up loop outside the capture or torch.cuda.graph capturing the UNet's f32 F.conv1d calls,
which then went to MIOpen (deterministic mode, as RolloutDiffusionPolicy set it).  This script
isolates ONE such call: an f32 Conv1d(512 -> 512, k 5) on [B, 512, 16] under the same cudnn flags,
run eagerly, then again, then inside a HIP stream capture.  Each stage prints before it starts.

usage: MIOPEN_ENABLE_LOGGING=1 python scripts/diag_conv1d_capture.py 1024"""

import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
torch.backends.cudnn.benchmark = False
torch.backends.cudnn.deterministic = True
t0 = time.time()


def log(m):
    print(f"[{time.time() - t0:6.1f}s] {m}", flush=True)


dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(B, 512, 16, device=dev, generator=g)
w = torch.randn(512, 512, 5, device=dev, generator=g) * 0.02
b = torch.zeros(512, device=dev)
log(f"B={B}: eager F.conv1d")
y0 = F.conv1d(x, w, b, padding=2)
torch.cuda.synchronize()
log("eager again")
y1 = F.conv1d(x, w, b, padding=2)
torch.cuda.synchronize()
log(f"eager repeat equal: {bool(torch.equal(y0, y1))}; capturing")
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    y2 = F.conv1d(x, w, b, padding=2)
log("captured; replaying")
graph.replay()
torch.cuda.synchronize()
log(f"replay equal to eager: {bool(torch.equal(y2, y0))}")

if len(sys.argv) > 2 and sys.argv[2] == "--unet":
    # the round-2 path itself: the production-width UNet with every conv through MIOpen (the GEMM
    # device form switched off), one evaluation eagerly, then captured
    from robomanipbaselines_amd.policy.diffusion import unet1d

    unet1d._device_form = lambda x: False
    torch.manual_seed(0)
    m = unet1d.ConditionalUnet1D(7, global_cond_dim=2 * (64 + 7), down_dims=(512, 1024, 2048), kernel_size=5,
                                 cond_predict_scale=True).eval().requires_grad_(False).to(dev)
    xs = torch.randn(B, 16, 7, device=dev, generator=g)
    gc = torch.randn(B, 2 * (64 + 7), device=dev, generator=g)
    ts = torch.tensor(50, device=dev)
    with torch.no_grad():
        log("UNet eager")
        u0 = m(xs, ts, gc)
        torch.cuda.synchronize()
        log("UNet eager again")
        m(xs, ts, gc)
        torch.cuda.synchronize()
        log("UNet capturing")
        ug = torch.cuda.CUDAGraph()
        with torch.cuda.graph(ug):
            u1 = m(xs, ts, gc)
        log("UNet captured; replaying")
        ug.replay()
        torch.cuda.synchronize()
        log(f"UNet replay equal to eager: {bool(torch.equal(u0, u1))}")
