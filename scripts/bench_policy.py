"""Throughput of the batched rollout loop for the other policies of BASELINE.json's configs:
env-steps/s over K timed RolloutPhase steps after the scripted phases and W warm-up steps, plus GPU
ms per batched infer_policy call.

* configs[3]: DiffusionPolicy x2048 on MujocoUR5ePick (env_ur5e_pick.xml minus the absent YCB_sim
  objects, convex-hull contacts, dt 0.002 x 16; envs/ur5e_pick.py);
* configs[4]: DP3 x1024 on MujocoUR5ePick with the synthetic tactile channel computed every
  env-step (--tactile; the reference's tactile plugin is absent, envs/ur5e_pick.py);
* Mlp on the cable scene.

    python scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --steps 24 --warmup 8
    python scripts/bench_policy.py DiffusionPolicy3d --num_envs 1024 --tactile
"""
import argparse
import json
import os
import sys
import time

import numpy as np

# MIOpen Find at rollout batch sizes: skip timing the naive reference solver (as bench.py) -- except
# for the fp32 DiffusionPolicy, whose image encoder runs on MIOpen's deterministic solvers, where the
# naive solver is the one some shapes have
if not ("DiffusionPolicy" in sys.argv[1:2] and "fp32" in sys.argv):
    os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable  # noqa: E402
from robomanipbaselines_amd.envs.operation.OperationMujocoUR5ePick import OperationMujocoUR5ePick  # noqa: E402

ENVS = {"MujocoUR5eCable": OperationMujocoUR5eCable, "MujocoUR5ePick": OperationMujocoUR5ePick}
DEFAULT_ENV = {"DiffusionPolicy": "MujocoUR5ePick", "DiffusionPolicy3d": "MujocoUR5ePick", "Mlp": "MujocoUR5eCable"}

POLICIES = {
    "DiffusionPolicy": ("robomanipbaselines_amd.policy.diffusion_policy.rollout_diffusion_policy",
                        "RolloutDiffusionPolicy"),
    "DiffusionPolicy3d": ("robomanipbaselines_amd.policy.diffusion_policy_3d.rollout_diffusion_policy_3d",
                          "RolloutDiffusionPolicy3d"),
    "Mlp": ("robomanipbaselines_amd.policy.mlp.rollout_mlp", "RolloutMlp"),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("policy", choices=sorted(POLICIES))
    p.add_argument("--num_envs", type=int, default=1024)
    p.add_argument("--steps", type=int, default=24)
    p.add_argument("--warmup", type=int, default=8)
    p.add_argument("--precision", choices=["bf16", "fp32"], default="bf16")
    p.add_argument("--env", choices=sorted(ENVS), default=None, help="default: the BASELINE config's scene")
    p.add_argument("--tactile", action="store_true", help="synthetic tactile every env-step (Pick scene)")
    a = p.parse_args()
    a.env = a.env or DEFAULT_ENV[a.policy]
    import importlib

    mod, cls = POLICIES[a.policy]
    Pol = getattr(importlib.import_module(mod), cls)

    class Rollout(ENVS[a.env], Pol):
        pass

    argv = ["--num_envs", str(a.num_envs), "--device", "cuda:0", "--world_idx_list", *[str(i) for i in range(6)],
            "--world_random_scale", "0.01", "0.01", "0.0", "--seed", "0", "--precision", a.precision] + (["--tactile"] if a.tactile else [])
    t_start = time.time()

    def log(msg):
        print(f"[{time.time() - t_start:7.1f}s] {msg}", file=sys.stderr, flush=True)

    ro = Rollout(argv=argv)
    log("rollout constructed")
    ro.args.world_idx_list = [g % 6 for g in range(a.num_envs)]
    ro.reset()
    ro._active = None
    n_pre = len(ro.pre_durations)
    k = 0
    while ro.phase_idx < n_pre:
        ro.step_once()
        k += 1
        if k % 20 == 0:
            log(f"scripted phases: step {k}")
    for i in range(a.warmup):
        ro.step_once()
        log(f"warm-up step {i + 1}/{a.warmup}")
    ev = []
    orig = ro.infer_policy

    def timed():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig()
        e1.record()
        ev.append((e0, e1))

    ro.infer_policy = timed
    torch.cuda.synchronize()
    t0 = time.time()
    for i in range(a.steps):
        ro.step_once()
        if (i + 1) % 8 == 0:
            log(f"timed step {i + 1}/{a.steps}")
    torch.cuda.synchronize()
    dt = time.time() - t0
    ro.infer_policy = orig
    inf = [x.elapsed_time(y) for x, y in ev]
    print(json.dumps({"policy": a.policy, "num_envs": a.num_envs, "steps": a.steps, "warmup": a.warmup,
                      "precision": a.precision, "env_steps_per_s": round(a.num_envs * a.steps / dt, 1),
                      "ms_per_step": round(dt * 1e3 / a.steps, 3), "infer_calls": len(inf),
                      "infer_ms_per_call": round(float(np.mean(inf)), 3) if inf else None,
                      "scene": a.env + (" minus YCB_sim" if a.env == "MujocoUR5ePick" else ""),
                      "tactile": "synthetic, every env-step" if a.tactile else None,
                      "data": "synthetic (random-init weights)"}), flush=True)


if __name__ == "__main__":
    main()
