"""Prototype: fp32 GEMM emulated on bf16 MFMA by operand splitting (bf16x6 / bf16x9), measured
against hipBLASLt fp32 on the ACT transformer shapes (M = 1024 envs x 302 tokens).

a = a0 + a1 + a2 (three bf16 pieces, RNE), a.b ~ sum of the products a_i b_j with i + j <= 2 (6 terms)
or all 9.  Here each split product set is one bf16 GEMM with K-concatenated operands and an fp32
output (hipBLASLt via torch.mm(out_dtype=float32)) -- an upper-bound check of accuracy and of the
library's bf16 rate before a hand-written kernel."""

import time

import torch


def split3(x):
    x0 = x.to(torch.bfloat16)
    r = x - x0.float()
    x1 = r.to(torch.bfloat16)
    x2 = (r - x1.float()).to(torch.bfloat16)
    return x0, x1, x2


PAIRS6 = [(0, 0), (0, 1), (1, 0), (0, 2), (1, 1), (2, 0)]
PAIRS9 = PAIRS6 + [(1, 2), (2, 1), (2, 2)]
PAIRS3 = [(0, 0), (0, 1), (1, 0)]


def emul(a, w, pairs):
    As, Ws = split3(a), split3(w)
    # small terms first so the big one lands last in the K order
    pairs = pairs[::-1]
    A = torch.cat([As[i] for i, _ in pairs], dim=1)
    W = torch.cat([Ws[j] for _, j in pairs], dim=1)
    return torch.mm(A, W.t(), out_dtype=torch.float32)


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e3


def main():
    dev = "cuda"
    torch.manual_seed(0)
    M = 1024 * 302
    for K, N in [(512, 1536), (512, 3200), (3200, 512), (512, 512)]:
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        ref = (a[:8192].double() @ w.double().t())
        scale = ref.abs().max().item()
        r32 = a[:8192] @ w.t()
        e32 = (r32.double() - ref).abs().max().item() / scale
        line = f"K={K:5d} N={N:5d}  fp32 err {e32:.2e}"
        for name, pairs in (("x3", PAIRS3), ("x6", PAIRS6), ("x9", PAIRS9)):
            e = (emul(a[:8192], w, pairs).double() - ref).abs().max().item() / scale
            line += f"  {name} err {e:.2e}"
        print(line, flush=True)
        flop = 2 * M * K * N
        t32 = timeit(lambda: torch.mm(a, w.t()))
        ab = a.to(torch.bfloat16)
        a6 = torch.cat([ab] * 6, dim=1)
        w6 = torch.cat([w.to(torch.bfloat16)] * 6, dim=1)
        t6 = timeit(lambda: torch.mm(a6, w6.t(), out_dtype=torch.float32))
        tb = timeit(lambda: torch.mm(ab, w.to(torch.bfloat16).t(), out_dtype=torch.float32))
        tsplit = timeit(lambda: emul(a, w, PAIRS6), it=3)
        print(f"   fp32 {t32:7.3f} ms ({flop / t32 / 1e9:6.1f} TF/s)  bf16 K {tb:7.3f} ms ({flop / tb / 1e9:6.1f})"
              f"  bf16 6K {t6:7.3f} ms (fp32-equiv {flop / t6 / 1e9:6.1f} TF/s, bf16 {6 * flop / t6 / 1e9:6.1f})"
              f"  split+cat+6K {tsplit:7.3f} ms", flush=True)
        del a, w, a6, w6, ab
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
