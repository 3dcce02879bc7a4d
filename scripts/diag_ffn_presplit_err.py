import sys, torch
sys.path.insert(0, '.')
import torch.nn.functional as F
from robomanipbaselines_amd import kernels as K_
sys.path.insert(0, 'tests')
import test_presplit_gpu as T
torch.set_grad_enabled(False)
for M, scale in ((1000, 1.0), (257, 1e-12), (300, 3e6)):
    x, r = T._rows(M, 512, M + 7)
    g = torch.Generator(device="cpu").manual_seed(5)
    lw = (scale * (0.5 + torch.rand(512, generator=g))).to(T.DEV)
    lb = (scale * 0.1 * torch.randn(512, generator=g)).to(T.DEV)
    a = K_.add_layernorm_split(x, r, lw, lb, 1e-5, y_norm=True)
    sp = a.rmbx_split
    w1 = (torch.randn(3200, 512, generator=g) / 512 ** 0.5).to(T.DEV)
    b1 = (0.1 * torch.randn(3200, generator=g)).to(T.DEV)
    w2 = (torch.randn(512, 3200, generator=g) / 3200 ** 0.5).to(T.DEV)
    b2 = (0.1 * torch.randn(512, generator=g)).to(T.DEV)
    hs = K_.linear_presplit_split(sp, K_.split_f16x2(w1), b1, K_.weight_bounds(w1, b1), relu=True)
    h_ref = (a.double() @ w1.double().t() + b1.double()).clamp_min(0)
    out = K_.linear_presplit(hs, K_.split_f16x2(w2), b2)
    ref = h_ref @ w2.double().t() + b2.double()
    for lib in ("cublaslt", "cublas"):
        torch.backends.cuda.preferred_blas_library(lib)
        base = F.linear(F.linear(a, w1, b1).clamp_min(0), w2, b2)
        print(M, scale, lib, "ours", T._err(out, ref), "blas", T._err(base, ref), flush=True)
