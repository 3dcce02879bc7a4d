"""Divergence curve of the batched engine against the C oracle (checker) from identical states:
per env-step, the max over envs of |qpos_gpu - qpos_oracle| for the arm, the gripper linkage and
the task's remaining joints (cable hinges + free joint; Pick objects), and the first step at which
each group exceeds 1e-4.  Sets the horizon of the all-qpos trajectory bars in
tests/test_engine_gpu.py / tests/test_pick_gpu.py.

    python scripts/diag_divergence.py --out gpurun_out/r6_divergence
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def curve(arrays, states, frame_skip, steps, dev="cuda:0"):
    from oracle.dyn import OracleEnv
    from robomanipbaselines_amd.engine import PhysicsEngine

    eng = PhysicsEngine(arrays, len(states), dev)
    eng.time.copy_(torch.tensor([s[0] for s in states], dtype=torch.float64))
    eng.qpos.copy_(torch.tensor(np.array([s[1] for s in states])))
    eng.qvel.copy_(torch.tensor(np.array([s[2] for s in states])))
    eng.qacc_ws.copy_(torch.tensor(np.array([s[3] for s in states])))
    eng.ctrl.copy_(torch.tensor(np.array([s[4] for s in states])))
    orcs = []
    for (t, qp, qv, qa, c) in states:
        o = OracleEnv(arrays)
        o.set_state(t, qp, qv, qa, c)
        orcs.append(o)
    groups = {"arm": slice(0, 6), "gripper": slice(6, 14), "task": slice(14, None)}
    rows = []
    for s in range(steps):
        eng.step(frame_skip)
        for o in orcs:
            assert o.step(frame_skip) == 0
        q = eng.qpos.cpu().numpy()
        qo = np.stack([o.state()[1] for o in orcs])
        d = np.abs(q - qo)
        rows.append({"env_step": s + 1, **{k: float(d[:, g].max()) for k, g in groups.items()},
                     "all": float(d.max()), "per_env_all": [float(x) for x in d.max(1)]})
    assert int(eng.stats[:, 3].sum()) == 0
    first = {k: next((r["env_step"] for r in rows if r[k] > 1e-4), None) for k in list(groups) + ["all"]}
    return {"n_env": len(states), "frame_skip": frame_skip, "first_step_above_1e-4": first, "curve": rows}


def cable_states(arrays, n):
    from test_engine_gpu import _states

    return _states(arrays, n, seed=2, warm_steps=(0, 5, 10, 40))


def pick_states(arrays, n):
    from test_pick_gpu import horizon_states

    return horizon_states(arrays, n)


def main():
    from robomanipbaselines_amd import model as MD

    p = argparse.ArgumentParser()
    p.add_argument("--out", default="gpurun_out/r6_divergence")
    p.add_argument("--n", type=int, default=16)
    p.add_argument("--cable_steps", type=int, default=100)
    p.add_argument("--pick_steps", type=int, default=50)
    a = p.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    for name, states_fn, fs, steps in (("cable", cable_states, 8, a.cable_steps),
                                      ("pick", pick_states, 16, a.pick_steps)):
        arrays = MD.load(f"ur5e_{name}")
        res = curve(arrays, states_fn(arrays, a.n), fs, steps)
        res["scene"] = f"ur5e_{name}"
        with open(f"{a.out}_{name}.json", "w") as f:
            json.dump(res, f, indent=1)
        print(name, "first env-step above 1e-4:", res["first_step_above_1e-4"], flush=True)
        for r in res["curve"][::5]:
            print(f"  {r['env_step']:4d} arm {r['arm']:.2e} gripper {r['gripper']:.2e} task {r['task']:.2e}", flush=True)


if __name__ == "__main__":
    main()
