"""The op-counting build of the dynamics restatement (oracle/flopcount.cpp) is bit-identical to the
plain oracle, and reproduces the committed FLOP-count fixture that bench.py prices its FP64
roofline with."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "oracle_flops.json")


def test_flop_fixture_reproduces():
    from tools.count_flops import fit, trajectory  # tools/ does not travel to the GPU box

    fx = json.load(open(GOLDEN))
    rows = trajectory(fx["substeps"] // 8)  # also asserts counted == plain state, bit for bit
    assert rows[:, 0].mean() == fx["flops_mean"]
    assert rows[:, 2].mean() == fx["ncon_mean"] and rows[:, 3].mean() == fx["nefc_mean"]
    coef, rel = fit(rows)
    np.testing.assert_allclose(coef, fx["fit"]["coef"], rtol=1e-9)
    # the fitted regime model is a sane predictor (95% of substeps within 10%)
    fl, _, ncon, nefc, it = rows.T
    pred = coef[0] + coef[1] * ncon + coef[2] * nefc + coef[3] * it + coef[4] * it * nefc
    assert np.percentile(np.abs(pred - fl) / fl, 95) < 0.1


def test_policy_flops_fixture():
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "policy_flops.json")))
    act = fx["act_480x640"]
    assert act["flops_per_inference"] == sum(act["per_op"].values())
    # ACT at 480x640 is ~42 GFLOP per inference
    assert 40e9 < act["flops_per_inference"] < 45e9
