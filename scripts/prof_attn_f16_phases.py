"""Phase skips of the f16x3 attention kernel (RMBX_ATTN_F16_DBG: 1 = no V^T staging stores, 2 = no
S^T MFMAs, 4 = no softmax, 8 = no PV MFMAs, 16 = no K / V tile loads, 10 = neither MFMA product,
15 = staging loads + K stores + barriers only), encoder self-attention 302 x 302 and decoder
cross-attention 100 x 302 at 1024 envs, 8 heads; wrong results except 0, timing only (rounds
interleaved in one process)."""
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


DBGS = ("0", "1", "2", "4", "8", "16", "10", "15")
with torch.no_grad():
    for name, Lq, Lk in (("encoder self 302x302", 302, 302), ("decoder cross 100x302", 100, 302)):
        q = torch.randn(1024, Lq, 512, device=dev, generator=g) * 2
        k = torch.randn(1024, Lk, 512, device=dev, generator=g) * 2
        v = torch.randn(1024, Lk, 512, device=dev, generator=g)
        ts = {d: [] for d in DBGS}
        for _ in range(3):
            for d in DBGS:
                os.environ["RMBX_ATTN_F16_DBG"] = d
                K.attention_f32(q, k, v, 8, form="f16x3")
                torch.cuda.synchronize()
                ts[d].append(timeit(lambda: K.attention_f32(q, k, v, 8, form="f16x3")))
        os.environ.pop("RMBX_ATTN_F16_DBG")
        print(f"{name}: " + " | ".join(f"{d}: {min(t):.3f} ms" for d, t in ts.items()), flush=True)
        del q, k, v
