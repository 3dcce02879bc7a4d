"""Diagnostic: the ACT encoder self-attention (B x 8 heads x 302 x 302, head dim 64) and the
decoder cross-attention (100 x 302) in f32: rmbx_attention_f32 vs torch SDPA, HIP events;
TF/s on the algorithmic 4 * Lq * Lk * 64 FLOP per (batch, head)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = "cuda:0"


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
    out = {"B": B}
    for name, Lq, Lk in (("enc_self", 302, 302), ("dec_cross", 100, 302)):
        q = torch.randn(B, Lq, 512, device=dev)
        kv = torch.randn(B, Lk, 1024, device=dev)
        k, v = kv.split(512, dim=-1)
        flop = 4.0 * B * 8 * Lq * Lk * 64
        ms_r = timed(lambda: K.attention_f32(q, k, v, 8))
        ms_6 = timed(lambda: K.attention_f32(q, k, v, 8, x6=True))

        def sdpa():
            qh = q.view(B, Lq, 8, 64).transpose(1, 2)
            kh = k.reshape(B, Lk, 8, 64).transpose(1, 2)
            vh = v.reshape(B, Lk, 8, 64).transpose(1, 2)
            return F.scaled_dot_product_attention(qh, kh, vh)

        ms_t = timed(sdpa)
        dbg = {}
        for d in os.environ.get("ATTN_DBGS", "").split(","):
            if d:
                os.environ["RMBX_ATTN_F32_DBG"] = d
                dbg["dbg" + d] = round(timed(lambda: K.attention_f32(q, k, v, 8)), 3)
        os.environ.pop("RMBX_ATTN_F32_DBG", None)
        out[name] = {"rmbx_ms": round(ms_r, 3), "rmbx_x6_ms": round(ms_6, 3),
                     "rmbx_x6_bf16_mfma_frac": round(6 * flop / ms_6 / 1e9 / 2500, 3), **dbg, "rmbx_tflops": round(flop / ms_r / 1e9, 1),
                     "rmbx_frac_of_157": round(flop / ms_r / 1e9 / 157.3, 3), "sdpa_ms": round(ms_t, 3)}
    print(json.dumps(out), flush=True)
