"""Diagnostic: renderer phase skips at 1024 envs (RMBX_RENDER_DBG: 1 no ray loop, 2 no stores), s2d
policy output; plus the per-tile primitive-list statistics the ray loop walks."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402

n = 1024
env = BatchedMujocoUR5eCableEnv(n, "cuda:0")
env.reset()
H, W = env.renderer.height, env.renderer.width
s2d = torch.empty((n, H // 2, W // 2, 16), dtype=torch.bfloat16, device="cuda:0")
for dbg in (0, 1, 2, 3):
    os.environ["RMBX_RENDER_DBG"] = str(dbg)
    env.render_images("front", policy=s2d)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        env.render_images("front", policy=s2d)
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"dbg": dbg, "ms": round(a.elapsed_time(b) / 3, 3)}), flush=True)
os.environ["RMBX_RENDER_DBG"] = "0"
# per-pixel ray-loop statistics (RMBX_RENDER_DBG=4 writes ntests + 1000 * tile list length as depth)
os.environ["RMBX_RENDER_DBG"] = "4"
depth = torch.empty((8, H, W), dtype=torch.float32, device="cuda:0")
env8 = BatchedMujocoUR5eCableEnv(8, "cuda:0")
env8.reset()
env8.render_images("front", depth=depth)
for cam in env8.camera_names:
    env8.render_images(cam, depth=depth)
    d = depth.cpu()
    ntest = d % 1000
    cnt = (d - ntest) / 1000
    print(json.dumps({"camera": cam, "tests_per_pixel_mean": round(float(ntest.mean()), 2),
                      "tests_per_pixel_p90": float(ntest.flatten().kthvalue(int(0.9 * ntest.numel())).values),
                      "tile_list_mean": round(float(cnt.mean()), 2), "tile_list_max": float(cnt.max())}), flush=True)
os.environ["RMBX_RENDER_DBG"] = "0"
