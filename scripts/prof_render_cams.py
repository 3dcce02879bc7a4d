"""Renderer time per 1024-env call of every camera (8-bit policy frame), the static-background cache
on (the default; world-fixed cameras only) and off (RMBX_RENDER_CACHE=0)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402

n = 1024
env = BatchedMujocoUR5eCableEnv(n, "cuda:0")
env.reset()
H, W = env.renderer.height, env.renderer.width
u8 = torch.empty((n, H // 2, W // 2, 16), dtype=torch.uint8, device="cuda:0")
for cam in env.renderer.cam_names:
    for cache in ("1", "0"):
        os.environ["RMBX_RENDER_CACHE"] = cache
        for _ in range(2):
            env.renderer.render(env.engine, cam, policy=u8)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            env.renderer.render(env.engine, cam, policy=u8)
        e1.record()
        torch.cuda.synchronize()
        print(f"{cam:8s} cache {cache}: {e0.elapsed_time(e1) / 5:8.3f} ms per {n}-env call", flush=True)
os.environ.pop("RMBX_RENDER_CACHE")
