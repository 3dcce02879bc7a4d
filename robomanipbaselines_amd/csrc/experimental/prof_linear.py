"""Diagnostic: rmbx_linear_bf16 vs torch (hipBLASLt, with the committed TunableOp table) on the
ACT transformer's GEMM shapes at 1024 envs, HIP-event timing; TFLOP/s per shape."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402
from robomanipbaselines_amd.common.tuning import enable_gemm_tuning  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
enc, dec = B * 302, B * 100
SHAPES = [("enc_qk", enc, 1024, 512), ("enc_v/out", enc, 512, 512), ("enc_ffn1", enc, 3200, 512),
          ("enc_ffn2", enc, 512, 3200), ("dec_qk", dec, 1024, 512), ("dec_512", dec, 512, 512),
          ("dec_ffn1", dec, 3200, 512), ("dec_ffn2", dec, 512, 3200)]


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


enable_gemm_tuning()
with torch.no_grad():
    for name, M, N, Kd in SHAPES:
        x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, Kd, device="cuda") / Kd ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device="cuda")
        bb = b.to(torch.bfloat16)
        relu = name.endswith("ffn1")
        t_r = timed(lambda: K.linear_bf16(x, w, b, relu=relu))
        if relu:
            t_t = timed(lambda: torch._addmm_activation(bb, x, w.t()))
        else:
            t_t = timed(lambda: F.linear(x, w, bb))
        fl = 2.0 * M * N * Kd
        print(json.dumps({"shape": name, "M": M, "N": N, "K": Kd, "rmbx_ms": round(t_r, 3), "torch_ms": round(t_t, 3),
                          "rmbx_tflops": round(fl / t_r / 1e9, 1), "torch_tflops": round(fl / t_t / 1e9, 1)}), flush=True)
        del x, w
