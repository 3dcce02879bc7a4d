"""Timing probe (GPU) of the mesh visibility pass: per camera, the raster kernel's time with
RMBX_RENDER_DBG probes -- 16: per-block frames only, 32: + triangle set-up, 64: + ray tests without
the visibility writes, 0: the full pass (frames wrong under a probe; timing only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402

n = int(os.environ.get("N_ENV", "1024"))
env = BatchedMujocoUR5eCableEnv(n, "cuda:0")
env.reset()
H, W = env.renderer.height, env.renderer.width
u8 = torch.empty((n, H // 2, W // 2, 16), dtype=torch.uint8, device="cuda:0")
for cam in env.renderer.cam_names:
    for dbg in ("16", "32", "64", "0"):
        os.environ["RMBX_RENDER_DBG"] = dbg
        env.renderer.render(env.engine, cam, policy=u8)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            env.renderer.render(env.engine, cam, policy=u8)
        b.record()
        torch.cuda.synchronize()
        print(f"{cam} dbg {dbg}: {a.elapsed_time(b) / 3:.3f} ms per call", flush=True)
    os.environ["RMBX_RENDER_DBG"] = "0"
