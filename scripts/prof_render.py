"""Diagnostic: renderer time per call at rollout batch size (policy tensor, bf16 s2d and CHW)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
env = BatchedMujocoUR5eCableEnv(n, "cuda:0")
env.reset()
H, W = env.renderer.height, env.renderer.width
s2d = torch.empty((n, H // 2, W // 2, 16), dtype=torch.bfloat16, device="cuda:0")
rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device="cuda:0")


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


s2d32 = torch.empty((n, H // 2, W // 2, 16), dtype=torch.float32, device="cuda:0")
res = {"n_env": n, "policy_s2d_ms": timeit(lambda: env.render_images("front", policy=s2d)),
       "policy_s2d_f32_ms": timeit(lambda: env.render_images("front", policy=s2d32)),
       "rgb_ms": timeit(lambda: env.render_images("front", rgb=rgb))}
for d in os.environ.get("RENDER_DBGS", "").split(","):  # phase skips (RMBX_RENDER_DBG bits)
    if d:
        os.environ["RMBX_RENDER_DBG"] = d
        res["f32_dbg" + d] = timeit(lambda: env.render_images("front", policy=s2d32))
os.environ.pop("RMBX_RENDER_DBG", None)
img = rgb.float().mean().item()
res["rgb_mean"] = img
print(json.dumps(res), flush=True)
