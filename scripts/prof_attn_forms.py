"""ACT attention at 1024 envs (encoder self-attention 302 x 302 and decoder cross-attention 100 x 302,
8 heads): rmbx_attention_f16x3 vs rmbx_attention_f32x6, and the f16x3 kernel with 5-wave blocks
(RMBX_ATTN_WAVES=5, "f16x3-w5"); rounds interleaved in one process; error of each
vs an f64 reference on 16 envs."""
import os
import sys

import torch

sys.path.insert(0, ".")
from robomanipbaselines_amd import kernels as K  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)


def timeit(f, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def ref64(q, k, v, h):
    B, Lq, D = q.shape
    Lk = k.shape[1]
    qh = q.double().reshape(B, Lq, h, 64).transpose(1, 2)
    kh = k.double().reshape(B, Lk, h, 64).transpose(1, 2)
    vh = v.double().reshape(B, Lk, h, 64).transpose(1, 2)
    p = torch.softmax(qh @ kh.transpose(-1, -2) / 8.0, dim=-1)
    return (p @ vh).transpose(1, 2).reshape(B, Lq, D)


with torch.no_grad():
    for name, Lq, Lk in (("encoder self 302x302", 302, 302), ("decoder cross 100x302", 100, 302)):
        q = torch.randn(1024, Lq, 512, device=dev, generator=g) * 2
        k = torch.randn(1024, Lk, 512, device=dev, generator=g) * 2
        v = torch.randn(1024, Lk, 512, device=dev, generator=g)
        want = ref64(q[:16], k[:16], v[:16], 8)
        errs = {f: (K.attention_f32(q[:16], k[:16], v[:16], 8, form=f).double() - want).abs().max().item()
                for f in ("f16x3", "x6")}
        ts = {f: [] for f in ("f16x3", "f16x3-w5", "x6")}
        for _ in range(3):
            for f in ts:
                os.environ["RMBX_ATTN_WAVES"] = "5" if f == "f16x3-w5" else "4"
                ff = f.split("-")[0]
                K.attention_f32(q, k, v, 8, form=ff)
                torch.cuda.synchronize()
                ts[f].append(timeit(lambda: K.attention_f32(q, k, v, 8, form=ff)))
        os.environ.pop("RMBX_ATTN_WAVES")
        print(f"{name}: f16x3 {min(ts['f16x3']):.3f} ms (err {errs['f16x3']:.2e}) | f16x3-w5 "
              f"{min(ts['f16x3-w5']):.3f} ms | x6 {min(ts['x6']):.3f} ms (err {errs['x6']:.2e}) | "
              f"speedup {min(ts['x6']) / min(ts['f16x3']):.2f}x", flush=True)
        del q, k, v
