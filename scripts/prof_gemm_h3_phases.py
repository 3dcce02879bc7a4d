"""Phase skips of the f16x3 GEMM (RMBX_GEMM_VAR; wrong results, timing only) on the ACT ffn1 /
ffn2 / v-out shapes at 1024 envs, rounds interleaved in one process: 16 = default, 48 = no split
VALU, 272 = no A loads, 528 = no W DMA, 784 = no A loads and no W DMA, 816 = none of the three,
1040 = the three-LDS-stage schedule (same results)."""
import os
import sys

os.environ.setdefault("RMBX_GEMM_WIDE", "0")  # the variants compared are forms of the 128-wide tile
import torch

sys.path.insert(0, ".")
from robomanipbaselines_amd import kernels as K  # noqa: E402

M = 1024 * 302
VARS = ["16", "1040", "48", "272", "528", "784", "816"]
for name, Kd, Nd in (("ffn1", 512, 3200), ("ffn2", 3200, 512), ("v/out", 512, 512)):
    x = torch.randn(M, Kd, device="cuda")
    p = K.split_f16x2(torch.randn(Nd, Kd, device="cuda") / Kd ** 0.5)
    out = torch.empty(M, Nd, device="cuda")
    ts = {v: [] for v in VARS}
    for _ in range(3):
        for v in VARS:
            os.environ["RMBX_GEMM_VAR"] = v
            K.linear_f32x6(x, p, None, out=out)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                K.linear_f32x6(x, p, None, out=out)
            e.record()
            torch.cuda.synchronize()
            ts[v].append(s.elapsed_time(e) / 5)
    os.environ.pop("RMBX_GEMM_VAR")
    fl = 2.0 * M * Kd * Nd
    print(name, " | ".join(f"{v}: {min(t):.3f} ms ({3 * fl / min(t) / 1e9 / 2500:.3f})" for v, t in ts.items()), flush=True)
    del x, out
    torch.cuda.empty_cache()
