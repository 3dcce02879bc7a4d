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
# back-face culling (default) vs the two-sided triangles of round 5 (RMBX_RENDER_DBG=1024): time of
# the full render and the share of pixels whose surface changes
os.environ["RMBX_RENDER_CACHE"] = "0"
hg = torch.empty((n, H, W), dtype=torch.int32, device="cuda:0")
rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device="cuda:0")
out = {}
for name, dbg in (("culled", "0"), ("two_sided", "1024")):
    os.environ["RMBX_RENDER_DBG"] = dbg
    env.render_images("front", policy=pol)
    t = min(timed(lambda: env.render_images("front", policy=pol)) for _ in range(3))
    env.renderer.render(env.engine, "front", rgb=rgb, hit_geom=hg)
    torch.cuda.synchronize()
    out[name] = (t, hg.clone(), rgb.clone())
os.environ["RMBX_RENDER_DBG"] = "0"
os.environ["RMBX_RENDER_CACHE"] = "1"
print(json.dumps({"full_ms_culled": round(out["culled"][0], 3), "full_ms_two_sided": round(out["two_sided"][0], 3),
                  "pixels_surface_changed": float((out["culled"][1] != out["two_sided"][1]).float().mean()),
                  "pixels_rgb_changed": float((out["culled"][2] != out["two_sided"][2]).any(-1).float().mean())}), flush=True)
