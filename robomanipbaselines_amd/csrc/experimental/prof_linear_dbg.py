"""Diagnostic: rmbx_linear_bf16 phase skips (RMBX_GEMM_DBG: 1 no K-loop DMA, 2 no MFMA) on the
encoder FFN shapes at 1024 envs."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

M = 1024 * 302
for N, Kd in [(3200, 512), (512, 3200)]:
    x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, Kd, device="cuda") / Kd ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    for dbg in (0, 1, 2, 3):
        os.environ["RMBX_GEMM_DBG"] = str(dbg)
        K.linear_bf16(x, w, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            K.linear_bf16(x, w, b)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(json.dumps({"N": N, "K": Kd, "dbg": dbg, "ms": round(ms, 3), "tflops": round(2 * M * N * Kd / ms / 1e9, 1)}), flush=True)
    os.environ["RMBX_GEMM_DBG"] = "0"
