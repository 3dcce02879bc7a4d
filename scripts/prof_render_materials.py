"""Renderer time per 1024-env call of every camera with the scene's materials (textures, specular,
skybox: round 6) and without them (the round-5 flat shading), and the front / side frames of env 0
in both forms as PNGs (gpurun_out/), the 8-bit policy frame being the fp32 rollout's form."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.common.image_io import write_png  # noqa: E402
from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402
from robomanipbaselines_amd.render import Renderer  # noqa: E402

MAT_KEYS = ("geom_texid", "geom_matinfo", "tex_type", "tex_size", "tex_adr", "tex_rgb", "sky_rgb")
n = int(os.environ.get("N_ENV", "1024"))
out_dir = os.environ.get("OUT", "gpurun_out")
env = BatchedMujocoUR5eCableEnv(n, "cuda:0")
env.reset()
eng = env.engine
H, W = env.renderer.height, env.renderer.width
flat = Renderer({k: v for k, v in env.arrays.items() if k not in MAT_KEYS}, "cuda:0", width=W, height=H)
assert env.renderer.materials and not flat.materials
u8 = torch.empty((n, H // 2, W // 2, 16), dtype=torch.uint8, device="cuda:0")
rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device="cuda:0")
for cam in env.renderer.cam_names:
    for label, r in (("materials", env.renderer), ("flat", flat)):
        for _ in range(2):
            r.render(eng, cam, policy=u8)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            r.render(eng, cam, policy=u8)
        e1.record()
        torch.cuda.synchronize()
        print(f"{cam:8s} {label:10s} {e0.elapsed_time(e1) / 5:8.3f} ms per {n}-env call (8-bit policy frame)", flush=True)
        r.render(eng, cam, rgb=rgb)
        write_png(os.path.join(out_dir, f"r6_render_{cam}_{label}.png"), rgb[0].cpu().numpy())
