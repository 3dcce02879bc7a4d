"""Driver for counter passes over the f16x3 attention kernels: encoder self-attention (1024 envs,
8 heads, 302 x 302), RMBX_ATTN_DMA from the environment, a few launches.

    rocprofv3 --pmc <counters> --kernel-trace -- python scripts/prof_attn_pmc.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn(1024, 302, 512, device="cuda", generator=g) * 2
k = torch.randn(1024, 302, 512, device="cuda", generator=g) * 2
v = torch.randn(1024, 302, 512, device="cuda", generator=g)
with torch.no_grad():
    for _ in range(4):
        K.attention_f32(q, k, v, 8, form="f16x3")
torch.cuda.synchronize()
print("done", flush=True)
