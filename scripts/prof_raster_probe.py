"""Raster (visibility) pass probes for rocprofv3 --kernel-trace --stats: front camera, 1024 envs,
RMBX_RENDER_DBG from the environment (0 full, 16 per-block frames only, 32 + triangle set-up,
64 + ray tests without the visibility writes), 5 renders."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402

n = 1024
env = BatchedMujocoUR5eCableEnv(n, "cuda:0")
env.reset()
H, W = env.renderer.height, env.renderer.width
pol = torch.empty((n, H // 2, W // 2, 16), dtype=torch.uint8, device="cuda:0")
for _ in range(5):
    env.render_images("front", policy=pol)
torch.cuda.synchronize()
print("done", flush=True)
