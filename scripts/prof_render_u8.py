"""Renderer time per call at the bench's batch (1024 envs, the 8-bit space-to-depth policy image of
the fp32 rollout, policy_dtype 4); run once per library variant (RMBX_LIB_VARIANT) on one box."""
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
cam = env.renderer.cam_names[0]


def run():
    env.renderer.render(env.engine, cam, policy=u8)


run()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e9
for _ in range(3):
    a.record()
    for _ in range(5):
        run()
    b.record()
    torch.cuda.synchronize()
    best = min(best, a.elapsed_time(b) / 5)
print(f"variant {os.environ.get('RMBX_LIB_VARIANT', 'default')}: render u8 s2d {best:.3f} ms per 1024-env call "
      f"(checksum {int(u8.sum().item())})", flush=True)
