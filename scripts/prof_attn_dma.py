"""A/B of the f16x3 attention's K / V staging: the register-staged kernel (RMBX_ATTN_DMA=0) vs the
LDS-DMA-staged kernel (RMBX_ATTN_DMA=1) and its software-pipelined form (RMBX_ATTN_DMA=2, S^T of the
next key tile beside the softmax), each with the parts of a head on one XCD (RMBX_ATTN_XCD=1), at the ACT shapes and 1024 envs, 8 heads:
encoder self-attention 302 x 302, decoder cross-attention 100 x 302, decoder self-attention
100 x 100.  Rounds interleaved in one process; min over rounds; the outputs of every variant are
checked bitwise against the register-staged kernel's.

    python scripts/prof_attn_dma.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
VARIANTS = (("register", {"RMBX_ATTN_DMA": "0", "RMBX_ATTN_XCD": "0"}),
            ("dma", {"RMBX_ATTN_DMA": "1", "RMBX_ATTN_XCD": "0"}),
            ("dma+xcd", {"RMBX_ATTN_DMA": "1", "RMBX_ATTN_XCD": "1"}),
            ("dma+pipe", {"RMBX_ATTN_DMA": "2", "RMBX_ATTN_XCD": "0"}),
            ("dma+pipe+xcd", {"RMBX_ATTN_DMA": "2", "RMBX_ATTN_XCD": "1"}),
            ("dma1stage", {"RMBX_ATTN_DMA": "3", "RMBX_ATTN_XCD": "0"}),
            ("dma1stage+xcd", {"RMBX_ATTN_DMA": "3", "RMBX_ATTN_XCD": "1"}))


def timeit(f, reps=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


with torch.no_grad():
    for name, Lq, Lk in (("encoder self 302x302", 302, 302), ("decoder cross 100x302", 100, 302),
                         ("decoder self 100x100", 100, 100)):
        q = torch.randn(1024, Lq, 512, device=dev, generator=g) * 2
        k = torch.randn(1024, Lk, 512, device=dev, generator=g) * 2
        v = torch.randn(1024, Lk, 512, device=dev, generator=g)
        ts = {n: [] for n, _ in VARIANTS}
        outs = {}
        for _ in range(3):
            for n, env in VARIANTS:
                os.environ.update(env)
                outs[n] = K.attention_f32(q, k, v, 8, form="f16x3")
                torch.cuda.synchronize()
                ts[n].append(timeit(lambda: K.attention_f32(q, k, v, 8, form="f16x3")))
        same = all(torch.equal(outs[n], outs["register"]) for n, _ in VARIANTS)
        print(f"{name}: " + " | ".join(f"{n}: {min(t):.3f} ms" for n, t in ts.items()) + f" | bitwise equal: {same}",
              flush=True)
        del q, k, v, outs
os.environ.pop("RMBX_ATTN_DMA", None)
os.environ.pop("RMBX_ATTN_XCD", None)
