"""Diagnostic: can the physics env-step (FP64, latency-bound, low occupancy) overlap the ACT
policy (MFMA, 1 block/CU) on two HIP streams?  Times at 1024 envs: physics alone, policy alone
(batch B), and both launched concurrently on separate streams."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable  # noqa: E402
from robomanipbaselines_amd.policy.act.rollout_act import RolloutAct  # noqa: E402


class Rollout(OperationMujocoUR5eCable, RolloutAct):
    pass


n = 1024
ro = Rollout(argv=["--num_envs", str(n), "--device", "cuda:0", "--world_idx_list", "0", "1", "2", "3", "4", "5"])
ro.reset()
ro._active = None
while ro.phase_idx < len(ro.pre_durations):
    ro.step_once()
for _ in range(4):
    ro.step_once()
eng = ro.env.engine
state = ro.get_state().to(ro.policy_dtype)
img = ro.get_images(ro.policy_dtype)
s_pol, s_phy = torch.cuda.Stream(), torch.cuda.Stream()
torch.cuda.synchronize()  # setup work on the default stream must finish before the side streams touch the engine


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    torch.cuda.current_stream().wait_stream(s_pol)
    torch.cuda.current_stream().wait_stream(s_phy)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def phys(nsteps=3):
    s_phy.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s_phy):
        for _ in range(nsteps):
            eng.step(8)


def pol(b):
    s_pol.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s_pol), torch.no_grad():
        ro.policy(state[:b], img[:b])


def both(b, nsteps=3):
    pol(b)
    phys(nsteps)


res = {"phys_3steps_ms": timed(phys)}
for b in (1024, 342):
    res[f"policy_b{b}_ms"] = timed(lambda: pol(b))
    res[f"both_b{b}_ms"] = timed(lambda: both(b))
print(json.dumps({k: round(v, 3) for k, v in res.items()}), flush=True)
