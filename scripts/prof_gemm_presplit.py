"""GEMM timing (GPU): the f16x3 GEMM on f32 rows (split in registers, rmbx_linear_f16x3) vs the same
rows pre-split by the LayerNorm (rmbx_linear_f16x3_presplit), at the ACT shapes of one 1024-env
inference (M = 1024 x 302 encoder tokens).  Executed fraction = 3 x 2MNK / time / 2.5 PF."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

M = int(os.environ.get("GEMM_M", str(1024 * 302)))
dev = "cuda:0"
torch.manual_seed(0)
lw, lb = torch.ones(512, device=dev), torch.zeros(512, device=dev)
x = torch.randn(M, 512, device=dev)
a = K.add_layernorm_split(x, None, lw, lb)
a_plain = a.clone()


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


for name, N in (("qk", 1024), ("v/out", 512), ("ffn1", 3200)):
    w = torch.randn(N, 512, device=dev) / 512 ** 0.5
    b = torch.randn(N, device=dev)
    p = K.split_f16x2(w)
    out = torch.empty(M, N, device=dev)
    t0 = timeit(lambda: K.linear_f32x6(a_plain, p, b, out=out))
    os.environ["RMBX_PRESPLIT_FORM"] = "2"
    t1 = timeit(lambda: K.linear_f32x6(a, p, b, out=out))
    ref = out.clone()
    os.environ["RMBX_PRESPLIT_FORM"] = "3"
    t2 = timeit(lambda: K.linear_f32x6(a, p, b, out=out))
    eq = torch.equal(ref, out)
    os.environ["RMBX_PRESPLIT_FORM"] = "3"
    fl = 3 * 2.0 * M * N * 512
    print(f"{name:6s} M={M} N={N} K=512: in-register split {t0:.3f} ms ({fl / t0 / 1e9 / 2500:.3f}) | "
          f"pre-split 2 stages {t1:.3f} ms ({fl / t1 / 1e9 / 2500:.3f}) | 3 rings {t2:.3f} ms "
          f"({fl / t2 / 1e9 / 2500:.3f}) | equal {eq}", flush=True)
for grp in ("2", "4", "8", "16"):
    os.environ["RMBX_PRESPLIT_GROUP"] = grp
    for name, N in (("qk", 1024), ("ffn1", 3200)):
        w = torch.randn(N, 512, device=dev) / 512 ** 0.5
        p = K.split_f16x2(w)
        out = torch.empty(M, N, device=dev)
        t1 = timeit(lambda: K.linear_f32x6(a, p, None, out=out))
        print(f"group {grp:>2s} {name:5s}: pre-split {t1:.3f} ms ({3 * 2.0 * M * N * 512 / t1 / 1e9 / 2500:.3f})", flush=True)
os.environ["RMBX_PRESPLIT_GROUP"] = "8"
# phase skips (timing only, the three-ring form): 1 = no DMA after the prologue, 2 = no MFMAs, 4 = no stores;
# 8 = non-temporal output stores (same results)
for var in ("1", "2", "4", "5", "6", "8"):
    os.environ["RMBX_PRESPLIT_VAR"] = var
    for name, N in (("qk", 1024), ("ffn1", 3200)):
        w = torch.randn(N, 512, device=dev) / 512 ** 0.5
        p = K.split_f16x2(w)
        out = torch.empty(M, N, device=dev)
        t1 = timeit(lambda: K.linear_f32x6(a, p, None, out=out))
        print(f"skip {var} {name:5s}: {t1:.3f} ms ({3 * 2.0 * M * N * 512 / t1 / 1e9 / 2500:.3f})", flush=True)
os.environ["RMBX_PRESPLIT_VAR"] = "0"
t_ln = timeit(lambda: K.add_layernorm(x, None, lw, lb))
t_ls = timeit(lambda: K.add_layernorm_split(x, None, lw, lb))
t_lp = timeit(lambda: K.add_layernorm_split(x.view(1024, 302, 512), None, lw, lb, pos=torch.zeros(302, 512, device=dev)))
print(f"layernorm f32 {t_ln:.3f} ms | + split {t_ls:.3f} ms | + pos + both splits {t_lp:.3f} ms", flush=True)
