"""f16x3 (rmbx_linear_f16x3) vs bf16x6 (rmbx_linear_f32x6) vs hipBLASLt f32 on the fp32 ACT
transformer shapes at 1024 envs and the trunk's stride-2 convs: time per call (HIP events, rounds
interleaved), fp32-equivalent TF/s, executed MFMA fraction of the 2.5 PF bf16 peak, error vs f64."""

import sys

import torch
import torch.nn.functional as F

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


def err(got, ref):
    return ((got.double() - ref).abs().max() / ref.abs().max()).item()


def main():
    torch.manual_seed(0)
    M = 1024 * 302
    shapes = [("qk", 512, 1024), ("v/out", 512, 512), ("ffn1", 512, 3200), ("ffn2", 3200, 512)]
    for name, Kd, Nd in shapes:
        x = torch.randn(M, Kd, device="cuda")
        if name == "ffn2":
            x = x.clamp_min(0)
        w = torch.randn(Nd, Kd, device="cuda") / Kd ** 0.5
        b = torch.randn(Nd, device="cuda")
        p6, p3 = K.split_bf16x3(w), K.split_f16x2(w)
        ref = x[:4096].double() @ w.double().t() + b.double()
        e6, e3 = err(K.linear_f32x6(x[:4096], p6, b), ref), err(K.linear_f32x6(x[:4096], p3, b), ref)
        e32 = err(F.linear(x[:4096], w, b), ref)
        out = torch.empty(M, Nd, device="cuda")
        fns = {"x6": lambda: K.linear_f32x6(x, p6, b, out=out), "h3": lambda: K.linear_f32x6(x, p3, b, out=out)}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        ts = {k: [] for k in fns}
        for _ in range(3):
            for k, f in fns.items():
                ts[k].append(timeit(f))
        t6, t3 = min(ts["x6"]), min(ts["h3"])
        fl = 2.0 * M * Kd * Nd
        print(f"{name:6s} M={M} K={Kd:5d} N={Nd:5d}: bf16x6 {t6:7.3f} ms {fl / t6 / 1e9:6.1f} TF/s-eq "
              f"({6 * fl / t6 / 1e9 / 2500:.3f} of peak) err {e6:.2e} | f16x3 {t3:7.3f} ms {fl / t3 / 1e9:6.1f} TF/s-eq "
              f"({3 * fl / t3 / 1e9 / 2500:.3f} of peak) err {e3:.2e} | hipBLASLt f32 err {e32:.2e} | "
              f"f16x3 speedup {t6 / t3:5.2f}x", flush=True)
        del x, w, out, p6, p3
        torch.cuda.empty_cache()
    # implicit-GEMM convs of the trunk (1024 frames)
    for (n, C, H, W, Co, k, s, pd) in [(1024, 64, 120, 160, 128, 3, 2, 1), (1024, 128, 60, 80, 256, 3, 2, 1),
                                       (1024, 64, 120, 160, 64 * 2, 3, 1, 1)]:
        x = torch.randn(n, C, H, W, device="cuda").clamp_min(0).contiguous(memory_format=torch.channels_last)
        w = torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5
        b = torch.randn(Co, device="cuda")
        K.F32_PIECES = "bf16x6"
        p6 = K.pack_conv_f32x6(w)
        K.F32_PIECES = "f16x3"
        p3 = K.pack_conv_f32x6(w)
        ref = F.conv2d(x[:4].double(), w.double(), b.double(), s, pd)
        e6 = err(K.conv2d_f32x6(x[:4].contiguous(memory_format=torch.channels_last), p6, b, k, s, pd), ref)
        e3 = err(K.conv2d_f32x6(x[:4].contiguous(memory_format=torch.channels_last), p3, b, k, s, pd), ref)
        fns = {"x6": lambda: K.conv2d_f32x6(x, p6, b, k, s, pd), "h3": lambda: K.conv2d_f32x6(x, p3, b, k, s, pd)}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        ts = {kk: [] for kk in fns}
        for _ in range(3):
            for kk, f in fns.items():
                ts[kk].append(timeit(f, 4))
        t6, t3 = min(ts["x6"]), min(ts["h3"])
        Ho, Wo = (H + 2 * pd - k) // s + 1, (W + 2 * pd - k) // s + 1
        fl = 2.0 * n * Ho * Wo * Co * C * k * k
        print(f"conv {k}x{k}/{s} {C}->{Co} {H}x{W} x{n}: bf16x6 {t6:7.3f} ms {fl / t6 / 1e9:6.1f} TF/s-eq err {e6:.2e} | "
              f"f16x3 {t3:7.3f} ms {fl / t3 / 1e9:6.1f} TF/s-eq ({3 * fl / t3 / 1e9 / 2500:.3f} of peak) err {e3:.2e} | "
              f"speedup {t6 / t3:5.2f}x", flush=True)
        del x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
