"""Renderer time per 1024-env call of the policy camera (8-bit space-to-depth frame, the fp32
rollout's form): the scene with its visual meshes (the asset's render meshes, 1 mm LOD), coarser
LODs from scripts/_build/rmesh_cable_cell*.npz (tools-generated, optional), and the round-4
primitive substitutes (no meshes).  Also the share of pixels whose surface is a mesh."""
import glob
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402
from robomanipbaselines_amd.render import Renderer  # noqa: E402

n = int(os.environ.get("N_ENV", "1024"))
env = BatchedMujocoUR5eCableEnv(n, "cuda:0")
env.reset()
H, W = env.renderer.height, env.renderer.width
u8 = torch.empty((n, H // 2, W // 2, 16), dtype=torch.uint8, device="cuda:0")
hit = torch.empty((n, H, W), dtype=torch.int32, device="cuda:0")
cam = env.renderer.cam_names[0]
base = {k: v for k, v in env.arrays.items() if not k.startswith("rmesh_")}
variants_only = os.environ.get("RENDER_ONLY_ASSET") == "1"
cams = env.renderer.cam_names if os.environ.get("RENDER_ALL_CAMS") == "1" else [cam]
variants = [("meshes 1 mm (asset)", env.renderer)]
if not variants_only:
    variants.append(("substitutes (no meshes)", Renderer(base, "cuda:0")))
for f in ([] if variants_only else sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "rmesh_cable_cell*.npz")))):
    with np.load(f) as z:
        arr = dict(base, **{k: z[k] for k in z.files})
    variants.append((os.path.basename(f), Renderer(arr, "cuda:0")))
mesh_geoms = torch.tensor(env.arrays["rmesh_geoms"], device="cuda:0")
for name, r, cam in [(nm, r, c) for nm, r in variants for c in cams]:
    def run():
        r.render(env.engine, cam, policy=u8)
    run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        a.record()
        for _ in range(3):
            run()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / 3)
    r.render(env.engine, cam, hit_geom=hit)
    frac = torch.isin(hit, mesh_geoms).float().mean().item()
    print(f"{name} [{cam}]: {best:.3f} ms per {n}-env call, mesh pixels {frac:.3f}, tris "
          f"{0 if r.mesh_tri is None else r.mesh_tri.shape[0]}", flush=True)
