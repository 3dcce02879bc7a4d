"""Timing (GPU): the Winograd input transform f32 vs pre-split, the 36 position GEMMs in-register
vs pre-split, at the 1024-frame ACT layer-3 / layer-4 shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

dev = "cuda:0"


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for C, H, W in ((256, 30, 40), (512, 15, 20)):
    n = 1024
    x = torch.randn(n, C, H, W, device=dev).clamp_min(0).contiguous(memory_format=torch.channels_last)
    T = n * ((H + 3) // 4) * ((W + 3) // 4)
    V = torch.empty((36, T, C), device=dev)
    Vp = torch.empty((2, 36, T, C), dtype=torch.float16, device=dev)
    rinv = torch.empty(T, device=dev)
    t0 = timeit(lambda: K.N.call("rmbx_wino4_input_f32", K.N.ptr(x), n, H, W, C, K.N.ptr(V), K.N.stream_ptr()))
    t1 = timeit(lambda: K.N.call("rmbx_wino4_input_split", K.N.ptr(x), n, H, W, C, K.N.ptr(Vp), K.N.ptr(rinv),
                                 K.N.stream_ptr()))
    planes = K.pack_wino4_x6(torch.randn(C, C, 3, 3, device=dev) / (9 * C) ** 0.5)
    b = torch.zeros(C, device=dev)
    K.GEMM_PRESPLIT = False
    t2 = timeit(lambda: K.conv3x3_wino4_x6(x, planes, b, relu=True))
    K.GEMM_PRESPLIT = True
    t3 = timeit(lambda: K.conv3x3_wino4_x6(x, planes, b, relu=True))
    print(f"C={C} {H}x{W}: input transform f32 {t0:.3f} ms | pre-split {t1:.3f} ms ; whole conv in-register "
          f"{t2:.3f} ms | pre-split {t3:.3f} ms", flush=True)
