"""rmbx_linear_f32x6 vs hipBLASLt f32 (F.linear) on the fp32 ACT transformer shapes at 1024 envs:
time per call (HIP events), fp32-equivalent TF/s, bf16 MFMA utilisation, error vs f64."""

import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from robomanipbaselines_amd import kernels as K  # noqa: E402


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
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
    shapes = [("qk", 512, 1024), ("v/out", 512, 512), ("ffn1", 512, 3200), ("ffn2", 3200, 512), ("qkv", 512, 1536)]
    for name, Kd, Nd in shapes:
        x = torch.randn(M, Kd, device="cuda")
        w = torch.randn(Nd, Kd, device="cuda") / Kd ** 0.5
        b = torch.randn(Nd, device="cuda")
        p = K.split_bf16x3(w)
        ref = x[:4096].double() @ w.double().t() + b.double()
        e6 = ((K.linear_f32x6(x[:4096], p, b).double() - ref).abs().max() / ref.abs().max()).item()
        e32 = ((F.linear(x[:4096], w, b).double() - ref).abs().max() / ref.abs().max()).item()
        out = torch.empty(M, Nd, device="cuda")
        t6 = timeit(lambda: K.linear_f32x6(x, p, b, out=out))
        t32 = timeit(lambda: F.linear(x, w, b))
        fl = 2.0 * M * Kd * Nd
        print(f"{name:6s} M={M} K={Kd:5d} N={Nd:5d}: f32x6 {t6:7.3f} ms = {fl / t6 / 1e9:6.1f} TF/s fp32-equiv "
              f"(bf16 MFMA {6 * fl / t6 / 1e9 / 2500 * 100:5.1f} % of 2.5 PF) err {e6:.2e} | hipBLASLt f32 {t32:7.3f} ms "
              f"= {fl / t32 / 1e9:6.1f} TF/s err {e32:.2e} | speedup {t32 / t6:5.2f}x", flush=True)
        del x, w, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
