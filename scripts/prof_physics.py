"""Diagnostic: per-stage shader-cycle breakdown and wall time of the physics kernel."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
env = BatchedMujocoUR5eCableEnv(n, "cuda:0")
env.reset()
a = env.engine.ctrl.clone()
a[:, 6] = 255.0
for _ in range(20):
    env.step(a)
torch.cuda.synchronize()
t = time.time()
for _ in range(5):
    env.step(a)
torch.cuda.synchronize()
dt = (time.time() - t) / 5
print(f"n_env {n}: {dt*1e3:.2f} ms per env-step -> {n/dt:.0f} env-steps/s")
st = env.engine.stats.cpu().numpy()
print("ncon mean", st[:, 0].mean(), "nefc mean", st[:, 1].mean(), "iters mean", st[:, 2].mean(), "bad", st[:, 3].sum())
p = env.engine.step_profiled(8)
tot = sum(v for k, v in p.items() if "." not in k)
for k, v in p.items():
    print(f"  {k:18s} {v/1e6:8.3f} Mcycles  {100*v/tot:5.1f}%")
