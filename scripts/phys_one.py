"""Diagnostic driver: a few physics env-steps of 1024 cable envs (for rocprofv3 --pmc runs)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402

env = BatchedMujocoUR5eCableEnv(1024, "cuda:0")
env.reset()
a = env.engine.ctrl.clone()
a[:, 6] = 255.0
for _ in range(4):
    env.step(a)
torch.cuda.synchronize()
print("done")
