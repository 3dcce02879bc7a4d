"""SQ counter driver for rmbx_linear_f32x6: 3 launches each of the ffn1 (K 512, N 3200) and ffn2
(K 3200, N 512) shapes at M = 1024 x 302; run under `rocprofv3 --pmc <counters>` passes
(scripts/gpurun/gemm_sq.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

M = 1024 * 302
with torch.no_grad():
    for Kd, Nd in ((512, 3200), (3200, 512)):
        x = torch.randn(M, Kd, device="cuda")
        p = K.split_bf16x3(torch.randn(Nd, Kd, device="cuda") / Kd ** 0.5)
        out = torch.empty(M, Nd, device="cuda")
        for _ in range(3):
            K.linear_f32x6(x, p, None, out=out)
        torch.cuda.synchronize()
        print(f"K={Kd} N={Nd}: 3 launches", flush=True)
        del x, out
