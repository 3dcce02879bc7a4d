"""Diagnostic: the encoder FFN GEMMs (M = 1024 envs x 302 tokens) token-major (x W^T, as now) vs
feature-major (W x^T), with PyTorch TunableOp tuning each shape (hipBLASLt/rocBLAS solutions)."""
import json
import os
import sys

import torch
import torch.cuda.tunable as tun
import torch.nn.functional as F

tun.enable(True)
tun.tuning_enable(True)
tun.set_max_tuning_duration(20)
tun.set_filename("/tmp/ffn_layout_tunable.csv")


def timeit(fn, iters=10, warm=3):
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
M, D, H = 1024 * 302, 512, 3200
bf = torch.bfloat16
x = torch.randn(M, D, device=dev, dtype=bf)
w1 = torch.randn(H, D, device=dev, dtype=bf) * 0.02
b1 = torch.randn(H, device=dev, dtype=bf)
w2 = torch.randn(D, H, device=dev, dtype=bf) * 0.02
b2 = torch.randn(D, device=dev, dtype=bf)
h = torch.relu(F.linear(x, w1, b1))
xT = x.t().contiguous()
hT = h.t().contiguous()
res = {}
res["ffn1_token_major_ms"] = timeit(lambda: torch._addmm_activation(b1, x, w1.t()))
res["ffn1_feature_major_ms"] = timeit(lambda: torch.addmm(b1[:, None], w1, xT))
res["ffn2_token_major_ms"] = timeit(lambda: F.linear(h, w2, b2))
res["ffn2_feature_major_ms"] = timeit(lambda: torch.addmm(b2[:, None], w2, hT))
res["transpose_x_ms"] = timeit(lambda: x.t().contiguous())
for k in list(res):
    if k.startswith("ffn"):
        res[k.replace("_ms", "_tflops")] = round(2 * M * D * H / (res[k] * 1e-3) / 1e12, 1)
print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in res.items()}), flush=True)
