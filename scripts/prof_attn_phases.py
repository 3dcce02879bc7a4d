"""Phase skips of the default f16x3 attention kernel (RMBX_ATTN_DMA=2, RMBX_ATTN_F16_DBG): encoder
self-attention, 1024 envs, 8 heads, 302 x 302.  Wrong results for every skip; timing only.
1 = no K / V splits in the loop, 2 = no softmax, 4 = no DMA in the loop, 8 = no S^T MFMAs,
16 = no PV MFMAs, 24 = neither product, 5 = neither DMA nor split.

    python scripts/prof_attn_phases.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

os.environ["RMBX_ATTN_DMA"] = "2"
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn(1024, 302, 512, device="cuda", generator=g) * 2
k = torch.randn(1024, 302, 512, device="cuda", generator=g) * 2
v = torch.randn(1024, 302, 512, device="cuda", generator=g)
SKIPS = (0, 1, 2, 4, 8, 16, 24, 5)


def timeit(reps=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        K.attention_f32(q, k, v, 8, form="f16x3")
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


ts = {d: [] for d in SKIPS}
with torch.no_grad():
    for _ in range(3):
        for d in SKIPS:
            os.environ["RMBX_ATTN_F16_DBG"] = str(d)
            K.attention_f32(q, k, v, 8, form="f16x3")
            torch.cuda.synchronize()
            ts[d].append(timeit())
os.environ.pop("RMBX_ATTN_F16_DBG")
for d in SKIPS:
    print(f"skip {d:2d}: {min(ts[d]):.3f} ms", flush=True)
