"""A/B of the bf16x6 GEMM's persistent form (RMBX_GEMM_PERSIST=1, the default) against the per-tile
kernel (=0) on the fp32 ACT shapes at 1024 envs, interleaved rounds in one process (HIP events).
Prints ms per call and the executed bf16 MFMA rate as a fraction of the 2.5 PF dense peak."""

import os
import statistics
import sys

import torch

sys.path.insert(0, ".")
from robomanipbaselines_amd import kernels as K  # noqa: E402


def timeit(fn, it=8):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    torch.manual_seed(0)
    M = 1024 * 302
    shapes = [("qk", M, 512, 1024), ("v/out", M, 512, 512), ("ffn1", M, 512, 3200), ("ffn2", M, 3200, 512),
              ("cross_kv", M, 512, 512), ("dec_ffn1", 1024 * 100, 512, 3200), ("dec_q", 1024 * 100, 512, 512)]
    for name, Mm, Kd, Nd in shapes:
        x = torch.rand(Mm, Kd, device="cuda") * 2 - 1
        w = (torch.rand(Nd, Kd, device="cuda") * 2 - 1) / Kd ** 0.5
        b = torch.rand(Nd, device="cuda")
        p = K.split_bf16x3(w)
        out = torch.empty(Mm, Nd, device="cuda")
        res = {"1": [], "0": []}
        for mode in ("1", "0"):  # warm-up
            os.environ["RMBX_GEMM_PERSIST"] = mode
            K.linear_f32x6(x, p, b, out=out)
        torch.cuda.synchronize()
        for _ in range(5):
            for mode in ("1", "0"):
                os.environ["RMBX_GEMM_PERSIST"] = mode
                res[mode].append(timeit(lambda: K.linear_f32x6(x, p, b, out=out)))
        fl = 2.0 * Mm * Kd * Nd
        line = f"{name:9s} M={Mm} K={Kd:5d} N={Nd:5d}:"
        for mode, label in (("1", "persistent"), ("0", "per-tile")):
            t = statistics.median(res[mode])
            line += f"  {label} {t:7.3f} ms ({6 * fl / t / 1e9 / 2500:5.3f} of bf16 peak, min {min(res[mode]):.3f})"
        print(line, flush=True)
        del x, w, out
        torch.cuda.empty_cache()
    os.environ["RMBX_GEMM_PERSIST"] = "1"


if __name__ == "__main__":
    main()
