"""Diagnostic driver: the encoder self-attention shape (1024 envs x 8 heads x 302) a few times
(for rocprofv3 --pmc runs)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

B, L = 1024, 302
q = torch.randn(B, L, 512, device="cuda").to(torch.bfloat16)
kv = torch.randn(B, L, 1024, device="cuda").to(torch.bfloat16)
k, v = kv.split(512, dim=-1)
for _ in range(3):
    K.attention_bf16(q, k, v, 8)
torch.cuda.synchronize()
print("done")
