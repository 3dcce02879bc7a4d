"""Renderer phase skips on the rollout's own front-camera call (1024 envs, the 8-bit space-to-depth
policy output of the fp32 ACT path): RMBX_RENDER_DBG 0 (full), 1 (no primitive ray loop), 256 (no
texture sampling), 257 (neither), 16 (visibility pass: per-block frames only), 2 (no stores)."""
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
pol = torch.empty((n, H // 2, W // 2, 16), dtype=torch.uint8, device="cuda:0")
res = {}
for rnd in range(3):
    for dbg in (0, 1, 256, 257, 16, 2):
        os.environ["RMBX_RENDER_DBG"] = str(dbg)
        env.render_images("front", policy=pol)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            env.render_images("front", policy=pol)
        b.record()
        torch.cuda.synchronize()
        res.setdefault(dbg, []).append(a.elapsed_time(b) / 3)
os.environ["RMBX_RENDER_DBG"] = "0"
for dbg, t in res.items():
    print(json.dumps({"dbg": dbg, "ms": round(min(t), 3)}), flush=True)
os.environ["RMBX_RENDER_DBG"] = "4"
depth = torch.empty((n, H, W), dtype=torch.float32, device="cuda:0")
env.render_images("front", depth=depth)
d = depth[:64].cpu()
ntest = d % 1000
cnt = (d - ntest) / 1000
print(json.dumps({"tests_per_pixel_mean": round(float(ntest.mean()), 2), "tile_list_mean": round(float(cnt.mean()), 2)}))
os.environ["RMBX_RENDER_DBG"] = "0"
hg = torch.empty((n, H, W), dtype=torch.int32, device="cuda:0")
env.render_images("front", depth=depth)
env.renderer.render(env.engine, "front", hit_geom=hg)
u, c = torch.unique(hg[:64], return_counts=True)
print(json.dumps({"hit_geom_share": {int(k): round(int(v) / hg[:64].numel(), 4) for k, v in zip(u, c)}}))
