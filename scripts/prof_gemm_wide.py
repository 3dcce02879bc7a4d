"""f16x3 GEMM: the 256 x 128 tile (RMBX_GEMM_WIDE=0) vs the 256 x 256 tile (=1) on the ACT shapes
at 1024 envs, rounds interleaved in one process; outputs compared bitwise."""
import os
import sys

import torch

sys.path.insert(0, ".")
from robomanipbaselines_amd import kernels as K  # noqa: E402


def timeit(fn, it=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


M = 1024 * 302
for name, Kd, Nd in (("qk", 512, 1024), ("v/out", 512, 512), ("ffn1", 512, 3200), ("ffn2", 3200, 512)):
    x = torch.randn(M, Kd, device="cuda")
    if name == "ffn2":
        x = x.clamp_min(0)
    p = K.split_f16x2(torch.randn(Nd, Kd, device="cuda") / Kd ** 0.5)
    b = torch.randn(Nd, device="cuda")
    out = torch.empty(M, Nd, device="cuda")
    fn = lambda: K.linear_f32x6(x, p, b, out=out)  # noqa: E731
    outs, ts = {}, {"0": [], "1": []}
    for v in ("0", "1"):
        os.environ["RMBX_GEMM_WIDE"] = v
        outs[v] = fn().clone()
    torch.cuda.synchronize()
    same = torch.equal(outs["0"], outs["1"])
    for _ in range(3):
        for v in ("0", "1"):
            os.environ["RMBX_GEMM_WIDE"] = v
            fn()
            torch.cuda.synchronize()
            ts[v].append(timeit(fn))
    fl = 2.0 * M * Kd * Nd
    t0, t1 = min(ts["0"]), min(ts["1"])
    print(f"{name:6s}: 256x128 {t0:.3f} ms ({3 * fl / t0 / 1e9 / 2500:.3f} of peak) | 256x256 {t1:.3f} ms "
          f"({3 * fl / t1 / 1e9 / 2500:.3f}) | speedup {t0 / t1:.2f}x | bitwise equal {same}", flush=True)
    del x, out
    torch.cuda.empty_cache()
