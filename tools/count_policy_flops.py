"""FLOPs per inference of the restated policies (SURVEY.md §8(d) "Roofline: policy"), counted with
torch.utils.flop_counter.FlopCounterMode on the CPU fp32 modules at the benchmark input shapes
(batch 1).  Writes tests/golden/policy_flops.json, which bench.py reads to price the MFMA
roofline of the measured inference calls.

    python tools/count_policy_flops.py
"""

import json
import os
import sys

import torch
from torch.utils.flop_counter import FlopCounterMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def count(fn):
    with FlopCounterMode(display=False) as fc:
        fn()
    per_op = {str(k): int(v) for k, v in fc.get_flop_counts().get("Global", {}).items()}
    return fc.get_total_flops(), per_op


def main():
    from robomanipbaselines_amd.policy.act.act_model import ActModel

    torch.manual_seed(0)
    out = {}
    with torch.no_grad():
        act = ActModel().eval().requires_grad_(False)
        state, img = torch.zeros(1, 7), torch.rand(1, 1, 3, 480, 640)
        total, per_op = count(lambda: act(state, img))
        # FlopCounterMode has no formula for the CPU SDPA kernel: attention products added
        # analytically, 2 GEMMs (QK^T, PV) x 2 flops/MAC x Sq x Sk x d per attention
        S, Q, d = 2 + 15 * 20, 100, 512
        attn = 4 * (len(act.encoder_layers) * S * S + len(act.decoder_layers) * (Q * Q + Q * S)) * d
        per_op["attention (analytic)"] = attn
        out["act_480x640"] = {"flops_per_inference": total + attn, "per_op": per_op,
                              "config": "ACT (ResNet-18 to layer4, enc 4 / dec 7, d 512, ff 3200, chunk 100), 1 cam 480x640"}
        # the computation the output depends on: the DETRVAE reads decoder layer 0's normed
        # intermediate only, so layers 1..6 are dead (prune_dead_decoder; exact, tests/test_act_full_gpu.py)
        act.prune_dead_decoder = True
        total, per_op = count(lambda: act(state, img))
        attn = 4 * (len(act.encoder_layers) * S * S + (Q * Q + Q * S)) * d
        per_op["attention (analytic)"] = attn
        out["act_480x640_dec0"] = {"flops_per_inference": total + attn, "per_op": per_op,
                                   "config": "as act_480x640 with decoder layers 1..6 skipped (outputs unused)"}
    path = os.path.join(ROOT, "tests", "golden", "policy_flops.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
