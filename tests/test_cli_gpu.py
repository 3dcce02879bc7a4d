"""End-to-end CLI contract on the GPU: the command misc/AutoEval.py:362-435 builds
(`Rollout.py <Policy> <Env> --auto_exit --no_plot --no_render --save_last_image
--output_image_dir D --world_idx_list ... --result_filename F`) runs the batched engine, one env per
listed world, and leaves the YAML AutoEval parses (success / reward / duration, one entry per
world in order) plus one last-frame PNG per episode."""

import glob
import os

import numpy as np
import pytest
import yaml

pytestmark = pytest.mark.gpu


def test_autoeval_command_line(tmp_path, capsys):
    from robomanipbaselines_amd.bin.Rollout import main
    from robomanipbaselines_amd.common.image_io import decode_png

    res = os.path.join(tmp_path, "result.yaml")
    img_dir = os.path.join(tmp_path, "img")
    ro = main(["Mlp", "MujocoUR5eCable", "--auto_exit", "--no_plot", "--no_render", "--save_last_image",
               "--output_image_dir", img_dir, "--world_idx_list", "0", "3", "5", "--result_filename", res,
               "--max_duration", "1.5"])
    out = capsys.readouterr().out
    assert ro.n == 3  # one env per listed world
    # AutoEval passes no precision flag: the policy runs at the reference's precision (fp32)
    import torch

    assert ro.args.precision == "fp32" and ro.policy_dtype == torch.float32
    assert all(p.dtype == torch.float32 for p in ro.policy.parameters())
    with open(res) as f:
        data = yaml.safe_load(f)
    assert set(data) == {"success", "reward", "duration"}
    assert len(data["success"]) == len(data["reward"]) == len(data["duration"]) == 3
    assert list(map(int, data["success"])) == [int(s) for s in data["success"]]
    # no success with a random policy within 1.5 s: every episode ends at max_duration
    for d in data["duration"]:
        assert 1.5 < d <= 1.5 + 0.032 + 1e-9
    assert out.count("Rollout result: ") == 3
    pngs = sorted(glob.glob(os.path.join(img_dir, "RolloutMlp_MujocoUR5eCable_world*_*.png")))
    assert len(pngs) == 3
    assert {os.path.basename(p).split("_")[2] for p in pngs} == {"world0", "world3", "world5"}
    with open(pngs[0], "rb") as f:
        img = decode_png(f.read())
    H, W = ro.env.renderer.height, ro.env.renderer.width
    assert img.shape == (H, W * len(ro.env.camera_names), 3)
    assert img.std() > 0
    # every env was frozen at its transition: all three stopped at the same sim time
    t = ro.env.get_time().cpu().numpy()
    np.testing.assert_array_equal(t, t[0])
