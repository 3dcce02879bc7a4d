"""Diagnostic: whole ACT forward (device inference form, bf16, 1024 envs) with the decoder's
cross-attention keys/values of all layers as one GEMM each vs one GEMM pair per layer."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.policy.act.act_model import ActModel  # noqa: E402


def timeit(fn, iters=6, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


dev = "cuda:0"
torch.manual_seed(0)
m = ActModel().eval().requires_grad_(False)
m.fuse_backbone()
m = m.to(dev, torch.bfloat16)
m._fused = m._fused.to(memory_format=torch.channels_last)
m.fuse_transformer()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
s2d = torch.rand(B, 1, 240, 320, 16, device=dev).to(torch.bfloat16)
q = torch.randn(B, 7, device=dev, dtype=torch.bfloat16)
res = {}
with torch.no_grad():
    m.batch_cross_kv = False
    ref = m(q, s2d)
    m.batch_cross_kv = True
    got = m(q, s2d)
    res["max_abs_diff"] = (got.float() - ref.float()).abs().max().item()
    for rep in range(2):
        for flag in (False, True):
            m.batch_cross_kv = flag
            res[f"forward_ms_batched_{flag}_{rep}"] = round(timeit(lambda: m(q, s2d)), 3)
print(json.dumps(res), flush=True)
