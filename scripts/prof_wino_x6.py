"""Explicit Winograd F(4x4) with bf16x6 position GEMMs (kernels.conv3x3_wino4_x6) vs the fused f32
F(4x4) kernel on the ACT trunk's stride-1 conv shapes at 1024 frames; per-stage times."""
import sys

import torch

sys.path.insert(0, ".")
from robomanipbaselines_amd import _native as N  # noqa: E402
from robomanipbaselines_amd import kernels as K  # noqa: E402


def timeit(fn, it=5):
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
    cl = torch.channels_last
    for C, H, W in ((128, 60, 80), (256, 30, 40), (512, 15, 20)):
        x = torch.randn(1024, C, H, W, device="cuda").contiguous(memory_format=cl)
        r = torch.randn(1024, C, H, W, device="cuda").contiguous(memory_format=cl)
        w = torch.randn(C, C, 3, 3, device="cuda") / (9 * C) ** 0.5
        b = torch.randn(C, device="cuda")
        p6 = K.pack_wino4_x6(w)
        u4 = K.pack_winograd4_f32(w)
        t6 = timeit(lambda: K.conv3x3_wino4_x6(x, p6, b, relu=True, res=r))
        t4 = timeit(lambda: K.conv3x3_winograd4_f32(x, u4, b, relu=True, res=r))
        T = 1024 * ((H + 3) // 4) * ((W + 3) // 4)
        V = torch.empty(36, T, C, device="cuda")
        M = torch.empty(36, T, C, device="cuda")
        ti = timeit(lambda: N.call("rmbx_wino4_input_f32", N.ptr(x), 1024, H, W, C, N.ptr(V), N.stream_ptr()))
        tg = timeit(lambda: N.call("rmbx_linear_f32x6_batched", N.ptr(V), C, T * C, N.ptr(p6), p6.stride(1),
                                   p6.stride(0), C * C, None, N.ptr(M), C, T * C, 36, T, C, C, 0, N.stream_ptr()))
        out = torch.empty_like(x)
        to = timeit(lambda: N.call("rmbx_wino4_output_f32", N.ptr(M), 1024, H, W, C, N.ptr(b), N.ptr(r), N.ptr(out), 1,
                                   N.stream_ptr()))
        fl = 2.0 * 36 * T * C * C
        print(f"C={C:3d} {H}x{W}: explicit x6 {t6:6.3f} ms (input {ti:5.3f} + 36 GEMMs {tg:5.3f} = "
              f"{fl / tg / 1e9:5.1f} TF/s fp32-equiv + output {to:5.3f}) | fused f32 F(4x4) {t4:6.3f} ms | "
              f"speedup {t4 / t6:4.2f}x", flush=True)
        del x, r, V, M, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
