"""Calibration probe (not a product path): the library f16 GEMM's throughput at the ACT FFN /
projection shapes with K tripled (the f16x3 products written as one f16 GEMM over [ah | ah | al] x
[wh | wl | 2^-11 wh]), f16 and f32 outputs, hipBLASLt vs rocBLAS -- the ceiling a hand-written
f16x3 kernel is measured against (HIP events, best of 3)."""
import torch

dev = "cuda"
torch.manual_seed(0)


def timeit(f, reps=5):
    f()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


SHAPES = ((309248, 3200, 512), (309248, 512, 3200), (309248, 512, 512), (309248, 1024, 512))
for lib in ("cublaslt", "cublas"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:  # noqa: BLE001
        print(lib, "unavailable", e)
        continue
    for M, N, K in SHAPES:
        a = torch.randn(M, 3 * K, device=dev, dtype=torch.float16)
        w = torch.randn(N, 3 * K, device=dev, dtype=torch.float16)
        fl = 2.0 * M * N * 3 * K
        t16 = timeit(lambda: torch.mm(a, w.t()))
        try:
            t32 = timeit(lambda: torch.mm(a, w.t(), out_dtype=torch.float32))
            s32 = f"{t32:.3f} ms ({fl / t32 / 1e9 / 2500:.3f})"
        except Exception as e:  # noqa: BLE001
            s32 = f"n/a ({type(e).__name__}: {str(e)[:80]})"
        print(f"{lib} M={M} N={N} K=3x{K}: f16 out {t16:.3f} ms ({fl / t16 / 1e9 / 2500:.3f}) | f32 out {s32}", flush=True)
        del a, w
