"""Diagnostic: rmbx_attention_bf16 vs torch scaled_dot_product_attention on the ACT transformer's
attention shapes at 1024 envs (encoder self 302x302, decoder self 100x100, cross 100x302)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


with torch.no_grad():
    for name, Lq, Lk in (("enc_self", 302, 302), ("dec_self", 100, 100), ("dec_cross", 100, 302)):
        q = torch.randn(B, Lq, 512, device="cuda").to(torch.bfloat16)
        kv = torch.randn(B, Lk, 1024, device="cuda").to(torch.bfloat16)
        k, v = kv.split(512, dim=-1)

        def sdpa():
            qh = q.view(B, Lq, 8, 64).transpose(1, 2)
            kh = k.view(B, Lk, 8, 64).transpose(1, 2)
            vh = v.view(B, Lk, 8, 64).transpose(1, 2)
            return F.scaled_dot_product_attention(qh, kh, vh).transpose(1, 2).reshape(B, Lq, 512)

        t_r = timed(lambda: K.attention_bf16(q, k, v, 8))
        os.environ["RMBX_ATTN_DBG"] = "1"
        t_stage = timed(lambda: K.attention_bf16(q, k, v, 8))
        os.environ["RMBX_ATTN_DBG"] = "0"
        t_t = timed(sdpa)
        err = (K.attention_bf16(q, k, v, 8).float() - sdpa().float()).abs().max().item()
        flops = 4.0 * B * 8 * Lq * Lk * 64
        io = B * (2 * Lq + 2 * Lk) * 512 * 2
        print(json.dumps({"shape": name, "rmbx_ms": round(t_r, 3), "rmbx_staging_only_ms": round(t_stage, 3),
                          "sdpa_ms": round(t_t, 3),
                          "rmbx_tflops": round(flops / t_r / 1e9, 1), "rmbx_gbs": round(io / t_r / 1e6, 1),
                          "max_abs_diff_vs_sdpa": err}), flush=True)
        del q, kv
