"""Diagnostic: capture the DiffusionPolicy denoising loop into a HIP graph at a given batch size and
precision, with the solver settings RolloutDiffusionPolicy uses, and report what fails.

usage: python scripts/diag_dp_capture.py <batch> <fp32|bf16> [--widths small|prod]
Each stage synchronises and prints; a failure inside the capture prints the exception text.
Run with MIOPEN_ENABLE_LOGGING=1 MIOPEN_LOG_LEVEL=5 to see MIOpen's calls around the capture."""

import argparse
import os
import sys
import time
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.policy.diffusion_policy.dp_model import DiffusionPolicyModel  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("batch", type=int)
p.add_argument("precision", choices=["fp32", "bf16"])
p.add_argument("--widths", choices=["small", "prod"], default="prod")
p.add_argument("--steps", type=int, default=100)
a = p.parse_args()
t0 = time.time()


def log(m):
    torch.cuda.synchronize()
    print(f"[{time.time() - t0:6.1f}s] {m}", flush=True)


dt = torch.float32 if a.precision == "fp32" else torch.bfloat16
torch.backends.cudnn.benchmark = dt == torch.bfloat16
torch.backends.cudnn.deterministic = dt != torch.bfloat16
widths = (512, 1024, 2048) if a.widths == "prod" else (64, 128, 256)
torch.manual_seed(0)
m = DiffusionPolicyModel(7, 7, 1, down_dims=widths, num_inference_steps=a.steps).eval().requires_grad_(False)
m = m.to("cuda:0", dt)
B = a.batch
g = torch.Generator(device="cuda:0").manual_seed(3)
gc = torch.randn(B, m.obs_feature_dim * 2, device="cuda:0", generator=g).to(dt)
x0 = torch.randn(B, 16, 7, device="cuda:0", generator=g)
noise = torch.randn(m._n_noise(), B, 16, 7, device="cuda:0", generator=g)
log(f"model {a.precision} widths {widths} batch {B}")
with torch.no_grad():
    eager = m.conditional_sample(gc, use_graph=False, x0=x0, noise=noise).clone()
    log("eager loop")
    m.graph_max_batch = 1 << 30
    try:
        graph = m.conditional_sample(gc, use_graph=True, x0=x0, noise=noise).clone()
        log("captured + replayed")
        print("replay == eager:", bool(torch.equal(graph, eager)),
              "max |d|:", (graph - eager).abs().max().item(), flush=True)
    except Exception:
        print("CAPTURE FAILED:", flush=True)
        traceback.print_exc()
        sys.stdout.flush()
        sys.exit(3)
