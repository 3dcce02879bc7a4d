"""Diagnostic (GPU): is a rendered frame independent of the batch it is rendered in?  The same
states rendered in a 1024-env batch, in a 512-env batch (its first half) and twice in a row."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402

dev = "cuda:0"
big = BatchedMujocoUR5eCableEnv(1024, dev)
big.reset()
g = torch.Generator(device=dev).manual_seed(0)
for _ in range(20):
    act = big.engine.ctrl.clone()
    act[:, :6] += 0.05 * torch.randn(1024, 6, device=dev, dtype=torch.float64, generator=g)
    big.step(act)
small = BatchedMujocoUR5eCableEnv(512, dev)
small.reset()
for name in ("qpos", "qvel", "qacc_ws", "ctrl", "time", "body_pos"):
    getattr(small.engine, name).copy_(getattr(big.engine, name)[:512])
small.engine.forward()
big.engine.forward()
H, W = big.renderer.height, big.renderer.width
for cam in big.camera_names:
    out = {}
    for tag, env, n in (("b1", big, 1024), ("b2", big, 1024), ("s", small, 512)):
        rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device=dev)
        depth = torch.empty((n, H, W), dtype=torch.float32, device=dev)
        hit = torch.empty((n, H, W), dtype=torch.int32, device=dev)
        env.renderer.render(env.engine, cam, rgb=rgb, depth=depth, hit_geom=hit)
        out[tag] = (rgb[:512].clone(), depth[:512].clone(), hit[:512].clone())
    for a_, b_ in (("b1", "b2"), ("b1", "s")):
        dr = (out[a_][0] != out[b_][0]).any(-1)
        dd = out[a_][1] != out[b_][1]
        dh = out[a_][2] != out[b_][2]
        print(f"{cam} {a_} vs {b_}: rgb differs at {int(dr.sum())} px, depth {int(dd.sum())}, hit {int(dh.sum())}", flush=True)
        if dd.any():
            idx = dd.nonzero()[:5].tolist()
            for e, y, x in idx:
                print("   ", e, y, x, float(out[a_][1][e, y, x]), float(out[b_][1][e, y, x]), int(out[a_][2][e, y, x]),
                      int(out[b_][2][e, y, x]))
print("states equal:", torch.equal(small.engine.xpos, big.engine.xpos[:512]), torch.equal(small.engine.xquat, big.engine.xquat[:512]))
