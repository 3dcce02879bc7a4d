"""A/B of the bf16x6 GEMM forms on the fp32 ACT shapes at 1024 envs, interleaved rounds in one process
(HIP events): the per-tile kernel (default), with the wave-4-7 stagger (RMBX_GEMM_VAR=80), the
persistent form (RMBX_GEMM_PERSIST=1) and persistent + stagger (RMBX_GEMM_STAGGER=1).
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
        # (RMBX_GEMM_PERSIST, RMBX_GEMM_STAGGER, RMBX_GEMM_VAR, RMBX_GEMM_WIDE)
        modes = {"t": ("0", "0", None, "0"), "ts": ("0", "0", "80", "0"), "p": ("1", "0", None, "0"),
                 "ps": ("1", "1", None, "0"), "w": ("0", "0", None, "1"), "ws": ("0", "1", None, "1")}

        def setmode(m):
            pe, st, var, wide = modes[m]
            os.environ["RMBX_GEMM_PERSIST"], os.environ["RMBX_GEMM_STAGGER"] = pe, st
            os.environ["RMBX_GEMM_WIDE"] = wide
            if var is None:
                os.environ.pop("RMBX_GEMM_VAR", None)
            else:
                os.environ["RMBX_GEMM_VAR"] = var

        res = {m: [] for m in modes}
        for mode in modes:  # warm-up
            setmode(mode)
            K.linear_f32x6(x, p, b, out=out)
        torch.cuda.synchronize()
        for _ in range(5):
            for mode in modes:
                setmode(mode)
                res[mode].append(timeit(lambda: K.linear_f32x6(x, p, b, out=out)))
        fl = 2.0 * Mm * Kd * Nd
        line = f"{name:9s} M={Mm} K={Kd:5d} N={Nd:5d}:"
        for mode, label in (("t", "per-tile"), ("ts", "per-tile+stagger"), ("p", "persistent"),
                            ("ps", "persistent+stagger"), ("w", "wide 128x256"), ("ws", "wide+stagger")):
            t = statistics.median(res[mode])
            line += f"\n    {label:20s} {t:7.3f} ms ({6 * fl / t / 1e9 / 2500:5.3f} of bf16 peak, min {min(res[mode]):.3f})"
        print(line, flush=True)
        del x, w, out
        torch.cuda.empty_cache()
    os.environ["RMBX_GEMM_PERSIST"], os.environ["RMBX_GEMM_STAGGER"], os.environ["RMBX_GEMM_WIDE"] = "0", "0", "0"
    os.environ.pop("RMBX_GEMM_VAR", None)


if __name__ == "__main__":
    main()
