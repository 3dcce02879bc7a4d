"""SQ counter driver for the fp32-accurate GEMM: 3 launches each of the ffn1 (K 512, N 3200) and
ffn2 (K 3200, N 512) shapes at M = 1024 x 302, in the piece form of env RMBX_SQ_FORM (bf16x6,
the default, or f16x3); run under `rocprofv3 --pmc <counters>` passes (scripts/gpurun/gemm_sq.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

M = 1024 * 302
with torch.no_grad():
    for Kd, Nd in ((512, 3200), (3200, 512)):
        x = torch.randn(M, Kd, device="cuda")
        w = torch.randn(Nd, Kd, device="cuda") / Kd ** 0.5
        p = K.split_f16x2(w) if os.environ.get("RMBX_SQ_FORM") == "f16x3" else K.split_bf16x3(w)
        out = torch.empty(M, Nd, device="cuda")
        for _ in range(3):
            K.linear_f32x6(x, p, None, out=out)
        torch.cuda.synchronize()
        print(f"K={Kd} N={Nd}: 3 launches", flush=True)
        del x, out
