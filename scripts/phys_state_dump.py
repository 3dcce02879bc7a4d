"""Diagnostic: 10 physics env-steps of 1024 cable (or --env pick: 256 pick) envs from a seeded reset
with a fixed control, the final qpos / qvel saved to gpurun_out/phys_state_<tag>.npy, for a
bitwise comparison of two library builds (RMBX_LIB_VARIANT) on one box."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402
from robomanipbaselines_amd.envs.ur5e_pick import BatchedMujocoUR5ePickEnv  # noqa: E402

pick = "--env" in sys.argv and sys.argv[sys.argv.index("--env") + 1] == "pick"
env = (BatchedMujocoUR5ePickEnv(256, "cuda:0") if pick else BatchedMujocoUR5eCableEnv(1024, "cuda:0"))
env.reset()
a = env.engine.ctrl.clone()
a[:, 6] = 0.0 if pick else 255.0
for _ in range(10):
    env.step(a)
torch.cuda.synchronize()
tag = (os.environ.get("RMBX_LIB_VARIANT") or "default") + ("_pick" if pick else "_cable")
st = np.concatenate([env.engine.qpos.cpu().numpy(), env.engine.qvel.cpu().numpy()], axis=1)
os.makedirs("gpurun_out", exist_ok=True)
np.save(f"gpurun_out/phys_state_{tag}.npy", st)
print(tag, st.shape, float(np.abs(st).sum()))
