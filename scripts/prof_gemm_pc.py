"""f16x3 GEMM: the default kernel (RMBX_GEMM_PC=0) vs the producer / consumer form (=1) on the ACT
shapes at 1024 envs and a trunk conv, rounds interleaved in one process; outputs compared bitwise."""
import os
import sys

os.environ.setdefault("RMBX_GEMM_WIDE", "0")  # the variants compared are forms of the 128-wide tile
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
cases = []
for name, Kd, Nd in (("qk", 512, 1024), ("v/out", 512, 512), ("ffn1", 512, 3200), ("ffn2", 3200, 512)):
    x = torch.randn(M, Kd, device="cuda")
    if name == "ffn2":
        x = x.clamp_min(0)
    p = K.split_f16x2(torch.randn(Nd, Kd, device="cuda") / Kd ** 0.5)
    b = torch.randn(Nd, device="cuda")
    out = torch.empty(M, Nd, device="cuda")
    cases.append((name, 2.0 * M * Kd * Nd, lambda x=x, p=p, b=b, out=out: K.linear_f32x6(x, p, b, out=out)))
xc = torch.randn(1024, 64, 120, 160, device="cuda").clamp_min(0).contiguous(memory_format=torch.channels_last)
pc_ = K.pack_conv_f32x6(torch.randn(128, 64, 3, 3, device="cuda") / 24.0)
bc = torch.randn(128, device="cuda")
cases.append(("conv 3x3/2 64->128", 2.0 * 1024 * 60 * 80 * 128 * 576, lambda: K.conv2d_f32x6(xc, pc_, bc, 3, 2, 1, relu=True)))
for name, fl, fn in cases:
    outs, ts = {}, {"0": [], "1": []}
    for v in ("0", "1"):
        os.environ["RMBX_GEMM_PC"] = v
        outs[v] = fn().clone()
    torch.cuda.synchronize()
    same = torch.equal(outs["0"], outs["1"])
    for _ in range(3):
        for v in ("0", "1"):
            os.environ["RMBX_GEMM_PC"] = v
            fn()
            torch.cuda.synchronize()
            ts[v].append(timeit(fn))
    t0, t1 = min(ts["0"]), min(ts["1"])
    print(f"{name:20s}: default {t0:.3f} ms ({3 * fl / t0 / 1e9 / 2500:.3f} of peak) | producer/consumer {t1:.3f} ms "
          f"({3 * fl / t1 / 1e9 / 2500:.3f}) | speedup {t0 / t1:.2f}x | bitwise equal {same}", flush=True)
