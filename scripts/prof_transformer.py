"""Diagnostic: ACT transformer (4 enc + 7 dec, d 512, ff 3200) at rollout batch size, GPU-event
timing, default hipBLASLt heuristics vs PyTorch TunableOp (GEMM solution search), plus the FFN
GEMM with a separate ReLU vs the fused-activation addmm.

python scripts/prof_transformer.py [batch] [tunable_csv]
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.policy.act.act_model import ActModel  # noqa: E402


def timeit(fn, iters=5, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
csv = sys.argv[2] if len(sys.argv) > 2 else None
dev = "cuda:0"
torch.manual_seed(0)
m = ActModel().eval().requires_grad_(False).to(dev, torch.bfloat16)
S, D = 302, 512
src = torch.randn(B, S, D, device=dev, dtype=torch.bfloat16)
pos = torch.randn(1, S, D, device=dev, dtype=torch.bfloat16)
qe = m.query_embed.weight[None]


def transformer():
    mem = src
    for layer in m.encoder_layers:
        mem = layer(mem, pos)
    tgt = torch.zeros(B, 100, D, device=dev, dtype=torch.bfloat16)
    mp = mem + pos
    for layer in m.decoder_layers:
        tgt = layer(tgt, mem, pos, qe, mp)
    return tgt


lin1 = m.encoder_layers[0].linear1
x = src.reshape(-1, D)
res = {"batch": B}
with torch.no_grad():
    res["transformer_default_ms"] = timeit(transformer)
    res["ffn1_linear_relu_ms"] = timeit(lambda: F.relu(F.linear(x, lin1.weight, lin1.bias)))
    res["ffn1_addmm_act_ms"] = timeit(lambda: torch._addmm_activation(lin1.bias, x, lin1.weight.t()))
    res["ffn1_linear_only_ms"] = timeit(lambda: F.linear(x, lin1.weight, lin1.bias))
    if csv:
        import torch.cuda.tunable as tun

        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_filename(csv)
        tun.set_max_tuning_duration(30)
        res["transformer_tuning_pass_ms"] = timeit(transformer, iters=1, warm=0)
        tun.tuning_enable(False)
        res["transformer_tuned_ms"] = timeit(transformer)
        res["ffn1_linear_relu_tuned_ms"] = timeit(lambda: F.relu(F.linear(x, lin1.weight, lin1.bias)))
print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in res.items()}), flush=True)
