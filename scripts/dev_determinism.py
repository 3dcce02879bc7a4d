"""Diagnostic: run-to-run determinism of the DP denoising loop (eager / graph), with and
without torch.backends.cudnn.deterministic."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.policy.diffusion_policy.dp_model import DiffusionPolicyModel  # noqa: E402

DEV = "cuda:0"
for det in (False, True):
    torch.backends.cudnn.deterministic = det
    torch.manual_seed(0)
    m = DiffusionPolicyModel(7, 7, 1, crop_hw=(64, 96), down_dims=(64, 128, 256)).eval().requires_grad_(False).to(DEV)
    B = 5
    g = torch.Generator(device=DEV).manual_seed(3)
    gc = torch.randn(B, m.obs_feature_dim * 2, device=DEV, generator=g)
    x0 = torch.randn(B, 16, 7, device=DEV, generator=g)
    noise = torch.randn(m._n_noise(), B, 16, 7, device=DEV, generator=g)
    with torch.no_grad():
        e = [m.conditional_sample(gc, use_graph=False, x0=x0, noise=noise).clone() for _ in range(3)]
        u = [m.model(x0, m._tsteps[0], gc).clone() for _ in range(3)]
        gr = [m.conditional_sample(gc, use_graph=True, x0=x0, noise=noise).clone() for _ in range(3)]
    print("det", det, "eager eq", [torch.equal(e[0], x) for x in e[1:]], "unet eq", [torch.equal(u[0], x) for x in u[1:]],
          "graph eq", [torch.equal(gr[0], x) for x in gr[1:]], "graph-eager", (gr[0] - e[1]).abs().max().item(),
          "e0-e1", (e[0] - e[1]).abs().max().item(), flush=True)
