"""Algorithmic FP64 FLOP count of one physics substep (SURVEY.md §8(d) "FP64 fraction").

Drives the op-counting build of the CPU restatement (oracle/flopcount.cpp; test infrastructure)
over a seeded trajectory of the cable scene and records, per substep, the FLOPs together with the
constraint-regime figures that drive them (contacts, constraint rows, Newton iterations).  A
least-squares model flops ~ c0 + c1*ncon + c2*nefc + c3*iters + c4*iters*nefc is fitted so that the
bench can price the regime it actually measured (its own contacts/rows/iterations means).  Also
checks that the counting build is bit-identical to the plain oracle along the trajectory.

    python tools/count_flops.py [--steps 150] [--out tests/golden/oracle_flops.json]
"""

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def trajectory(steps, seed=0):
    """Arm sweeps down over the cable with the gripper closing: free motion, cable-table contact,
    gripper-cable contact (same initial state as the scripted rollout, CABLE_INIT_QPOS)."""
    from oracle.dyn import OracleEnv
    from robomanipbaselines_amd import model as MD
    from robomanipbaselines_amd.envs.ur5e_cable import CABLE_INIT_QPOS

    arrays = MD.load("ur5e_cable")
    plain, counted = OracleEnv(arrays), OracleEnv(arrays, flops=True)
    qpos = arrays["qpos0"].copy()
    qpos[:14] = CABLE_INIT_QPOS
    rng = np.random.default_rng(seed)
    for e in (plain, counted):
        e.set_state(0.0, qpos, np.zeros(e.nv), np.zeros(e.nv), np.concatenate([CABLE_INIT_QPOS[:6], [0.0]]))
    lib = counted.lib
    rows = []
    for s in range(steps):
        frac = s / max(steps - 1, 1)
        ctrl = np.concatenate([CABLE_INIT_QPOS[:6] + [0.0, 0.35 * frac, 0.25 * frac, 0.3 * frac, 0.0, 0.0]
                               + rng.normal(0, 0.01, 6), [255.0 * min(1.0, 2 * frac)]])
        plain.set_ctrl(ctrl)
        counted.set_ctrl(ctrl)
        for _ in range(8):
            lib.orc_flops_reset()
            plain.step(1)
            counted.step(1)
            rows.append((lib.orc_flops(), lib.orc_special_ops(), counted.lib.orc_ncon(counted.h), counted.nefc(),
                         counted.solver_iter()))
        a, b = plain.state(), counted.state()
        for x, y in zip(a[1:], b[1:]):
            np.testing.assert_array_equal(x, y)
    return np.array(rows, dtype=np.float64)


def fit(rows):
    fl, _, ncon, nefc, it = rows.T
    X = np.stack([np.ones_like(ncon), ncon, nefc, it, it * nefc], 1)
    coef, *_ = np.linalg.lstsq(X, fl, rcond=None)
    pred = X @ coef
    return coef, float(np.max(np.abs(pred - fl) / fl))


def model_flops(coef, ncon, nefc, iters):
    return float(coef[0] + coef[1] * ncon + coef[2] * nefc + coef[3] * iters + coef[4] * iters * nefc)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=150)
    p.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "oracle_flops.json"))
    a = p.parse_args()
    rows = trajectory(a.steps)
    coef, rel = fit(rows)
    fl, sp, ncon, nefc, it = rows.T
    out = {
        "what": "algorithmic FP64 FLOPs per physics substep of the cable scene, counted by oracle/flopcount.cpp "
                "(+ - * / sqrt sin cos pow = 1 each) along tools/count_flops.py's seeded trajectory",
        "substeps": int(len(rows)),
        "flops_mean": float(fl.mean()), "flops_min": float(fl.min()), "flops_max": float(fl.max()),
        "special_mean": float(sp.mean()),
        "ncon_mean": float(ncon.mean()), "nefc_mean": float(nefc.mean()), "iters_mean": float(it.mean()),
        "fit": {"terms": ["1", "ncon", "nefc", "iters", "iters*nefc"], "coef": [float(c) for c in coef],
                "max_rel_err": rel},
        "samples": [[int(v) for v in r] for r in rows[:: max(1, len(rows) // 64)]],
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "samples"}, indent=1))


if __name__ == "__main__":
    main()
