"""Diagnostic (GPU): where the engine's Newton path leaves the oracle's.  The engine and the oracle
are run with the model's solver_iterations capped at k = 1, 2, ... on the same states; the first k
at which their qacc differ beyond rounding is the iteration that diverged.  Prints per state the
iteration counts and the deviation per cap."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import test_engine_gpu as T  # noqa: E402
from oracle.dyn import OracleEnv  # noqa: E402
from robomanipbaselines_amd import model as MD  # noqa: E402
from robomanipbaselines_amd.engine import PhysicsEngine  # noqa: E402

arrays = MD.load("ur5e_cable")
states = T._states(arrays, 8, seed=5, warm_steps=(0, 10, 40, 80))
rng = np.random.default_rng(12)
kicked = []
for (t, qp, qv, qa, c) in states:
    kick = np.zeros_like(qv)
    kick[14:62] = rng.normal(0, 0.3, 48)
    kicked.append((t, qp, qv + kick, qa, c))
states = states + kicked
for cap in (1, 2, 3, 4, 5, 8, 100):
    a = dict(arrays)
    a["_solver_iterations"] = np.int32(cap)
    eng = PhysicsEngine(a, len(states), "cuda:0")
    T._load(eng, states)
    eng.forward()
    torch.cuda.synchronize()
    qacc = eng.ws("qacc").cpu().numpy()
    it = eng.stats[:, 2].cpu().numpy()
    force = eng.ws("efc_force").cpu().numpy()
    row = []
    for i, (t, qp, qv, qa, c) in enumerate(states):
        o = OracleEnv(a)
        o.set_state(t, qp, qv, qa, c)
        o.forward()
        v = o.vecs()["qacc"]
        fo = o.efc_force()
        nact = int(np.sum((force[i, :len(fo)] != 0) != (fo != 0)))
        row.append(f"{i}:{it[i]}/{o.solver_iter()} d={np.abs(qacc[i] - v).max() / (np.abs(v).max() + 1):.1e} act{nact}")
    print(f"cap {cap}: " + "  ".join(row), flush=True)
for i in range(len(states)):
    t, qp, qv, qa, c = states[i]
    o = OracleEnv(arrays)
    o.set_state(t, qp, qv, qa, c)
    o.forward()
    print(i, [np.array2string(x, precision=2) for x in o.solver_trace()])
