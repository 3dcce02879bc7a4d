"""A/B of the renderer's static-background cache on the rollout's front-camera call (1024 envs, the
8-bit space-to-depth policy output of the fp32 ACT path): RMBX_RENDER_CACHE=0 (every pixel in full)
vs the cache reused (clean) vs the call that rebuilds every env's cache (dirty); interleaved rounds,
min over rounds; outputs checked bitwise."""
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


def timed(fn, reps=3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


res = {"full": [], "cached": [], "rebuild": []}
for rnd in range(3):
    os.environ["RMBX_RENDER_CACHE"] = "0"
    env.render_images("front", policy=pol)
    res["full"].append(timed(lambda: env.render_images("front", policy=pol)))
    ref = pol.clone()
    os.environ["RMBX_RENDER_CACHE"] = "1"
    env.render_images("front", policy=pol)
    res["cached"].append(timed(lambda: env.render_images("front", policy=pol)))
    same = torch.equal(pol, ref)

    def rebuild():
        env.renderer._caches["front"][3].fill_(float("nan"))  # every snapshot invalid: all envs dirty
        env.render_images("front", policy=pol)
    res["rebuild"].append(timed(rebuild))
    print(json.dumps({"round": rnd, "bitwise_equal": same}), flush=True)
for k, v in res.items():
    print(json.dumps({"mode": k, "ms_per_call": round(min(v), 3)}), flush=True)
