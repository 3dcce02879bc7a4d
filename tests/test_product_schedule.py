"""Product-path parity of the rollout plugin (BatchedRolloutBase) against fixtures minted from
the reference's own Python (tools/gen_golden.py):

* state normalisation: BatchedRolloutBase.normalize_state vs normalize_data (DataUtils.py:9-24) and
  the f32 cast of RolloutBase.get_state (:463-477), bit-exact;
* the phase schedule as the product loop runs it: BatchedRolloutBase.step_once drives the real
  batched cable env (physics clock advanced by the engine, 8 x 0.004 s per env-step), with the
  reward forced from each golden case; the host phase mirror, the device schedule, the steps at
  which infer_policy fired and the final success / reward / duration must equal the reference's
  PhaseManager run (RolloutBase.py:28-132, 387-415) bit for bit."""

import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

NORM_CASES = {
    "gauss": lambda d: {"norm_config": {"type": "gaussian"}, "mean": d["mean"], "std": d["std"]},
    "gauss_noconfig": lambda d: {"mean": d["mean"], "std": d["std"]},
    "limits": lambda d: {"norm_config": {"type": "limits", "out_min": -1.0, "out_max": 1.0}, "min": d["min"],
                         "range": d["range"]},
    "limits01": lambda d: {"norm_config": {"type": "limits", "out_min": 0.0, "out_max": 1.0}, "min": d["min"],
                           "range": d["range"]},
}


def _get_state(device, case):
    from robomanipbaselines_amd.common.rollout_base import BatchedRolloutBase

    d = np.load(os.path.join(GOLDEN, "normalize.npz"))
    ro = object.__new__(BatchedRolloutBase)
    ro.device = torch.device(device)
    ro.model_meta_info = {"state": NORM_CASES[case](d)}
    ro._bind_state_stats()
    got = ro.normalize_state(torch.tensor(d["data"], dtype=torch.float64, device=device)).cpu().numpy()
    want = d[f"{case}_norm"].astype(np.float32)  # torch.tensor(state, dtype=float32)
    return got, want


@pytest.mark.parametrize("case", list(NORM_CASES))
def test_get_state_matches_normalize_data_cpu(case):
    got, want = _get_state("cpu", case)
    assert got.dtype == np.float32
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(NORM_CASES))
def test_get_state_matches_normalize_data_gpu(case):
    got, want = _get_state("cuda:0", case)
    np.testing.assert_array_equal(got, want)


def _phase_cases():
    d = np.load(os.path.join(GOLDEN, "phase_schedule.npz"))
    return [{k[len(f"c{i}_"):]: d[k] for k in d.files if k.startswith(f"c{i}_")} for i in range(int(d["n_cases"]))]


@pytest.mark.gpu
@pytest.mark.parametrize("md,skip", [(30.0, 3), (10.0, 1), (5.0, 4)])
def test_product_loop_schedule_matches_reference(md, skip):
    from robomanipbaselines_amd import kernels as K
    from robomanipbaselines_amd.common.rollout_base import BatchedRolloutBase
    from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable

    cases = [c for c in _phase_cases() if float(c["max_duration"]) == md and int(c["skip"]) == skip]
    assert len(cases) == 6
    n = len(cases)

    class _LogPolicy(BatchedRolloutBase):
        """Policy stub: records the host step of every infer_policy call and holds the command."""

        policy_name = "Log"

        def setup_policy(self):
            self.policy = None
            self.infer_log = []
            self.step_t = -1

        def infer_policy(self):
            self.infer_log.append(self.step_t)
            self.policy_action = torch.cat([self.q_cmd, self.grip_cmd], dim=1).clone()

    class Rollout(OperationMujocoUR5eCable, _LogPolicy):
        pass

    ro = Rollout(argv=["--num_envs", str(n), "--device", "cuda:0", "--skip", str(skip), "--max_duration", str(md)])
    T = max(int(c["n_steps"]) for c in cases)
    rew = np.zeros((T, n))
    for i, c in enumerate(cases):
        rew[: len(c["reward"]), i] = c["reward"]
    rew_dev = torch.tensor(rew, dtype=torch.float64, device="cuda:0")
    box = {"t": 0}
    ro.env._get_reward = lambda: rew_dev[box["t"]].clone()
    ro.reset()
    n_pre = len(ro.pre_durations)
    assert n_pre == 4
    dev_before, dev_after, host = [], [], []
    for t in range(T):
        box["t"] = t
        ro.step_t = t
        dev_before.append(K.sched_view(ro.sched)["phase"].copy())
        ro.step_once()
        host.append(ro.phase_idx)
        dev_after.append(K.sched_view(ro.sched)["phase"].copy())
    dev_before, dev_after, host = np.array(dev_before), np.array(dev_after), np.array(host)
    v = K.sched_view(ro.sched)
    infer = np.array(ro.infer_log)
    for i, c in enumerate(cases):
        ns = int(c["n_steps"])
        name = str(c["name"])
        np.testing.assert_array_equal(dev_after[:ns, i], c["phase"], err_msg=name)
        np.testing.assert_array_equal(host[:ns], np.minimum(c["phase"], n_pre), err_msg=name)
        fired = infer[dev_before[infer, i] == n_pre]
        np.testing.assert_array_equal(fired, c["infer_steps"], err_msg=name)
        assert v["done"][i] == 1, name
        assert bool(v["success"][i]) == bool(c["success"][0]), name
        assert v["result_reward"][i] == float(c["result_reward"][0]), name
        assert v["duration"][i] == float(c["duration"][0]), name
    # an env frozen at its end keeps its clock: its time is the golden duration's clock
    assert np.isfinite(ro.env.get_time().cpu().numpy()).all()


@pytest.mark.gpu
def test_reach_phases_follow_reference_ik():
    """Pre-motion reach phases (OperationMujocoUR5eCable.py:8-30, PhaseBase.py:41-56,
    ArmManager.py:148-153, 220-243) through the product loop: each reach phase's target is
    (diag(-1, 1, -1), cable_end xy of the env at the phase start, fixed z), and every env-step's
    command update is one DLS IK iteration from the previous command (oracle/arm_ik.py)."""
    from oracle import arm_ik
    from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable
    from robomanipbaselines_amd.policy.mlp.rollout_mlp import RolloutMlp

    class Rollout(OperationMujocoUR5eCable, RolloutMlp):
        pass

    n = 5
    ro = Rollout(argv=["--num_envs", str(n), "--device", "cuda:0", "--world_idx_list", "0", "1", "2", "3", "4",
                       "--world_random_scale", "0.01", "0.01", "0.0"])
    recs, targets = [], []
    ik, settgt = ro._ik_step, ro._set_reach_target

    def rec_ik():
        before = ro.q_cmd.cpu().numpy().copy()
        ik()
        recs.append((before, ro._tgt_R.cpu().numpy().copy(), ro._tgt_p.cpu().numpy().copy(),
                     ro.q_cmd.cpu().numpy().copy()))

    def rec_target(pos_z):
        end = ro.env.get_body_pose("cable_end")[:, :3].cpu().numpy().copy()
        settgt(pos_z)
        targets.append((pos_z, end, ro._tgt_R.cpu().numpy().copy(), ro._tgt_p.cpu().numpy().copy()))

    ro._ik_step, ro._set_reach_target = rec_ik, rec_target
    ro.reset()
    while ro.phase_idx < len(ro.pre_durations):
        ro.step_once()
    # Reach1 0.7 s and Reach2 0.3 s at 32 ms per env-step (transitions on the strict > of the clock)
    assert [t[0] for t in targets] == [1.02, 0.995]
    assert len(recs) == 22 + 10
    for pos_z, end, R, p in targets:
        np.testing.assert_array_equal(R.reshape(n, 3, 3), np.tile(np.diag([-1.0, 1.0, -1.0]), (n, 1, 1)))
        np.testing.assert_array_equal(p[:, :2], end[:, :2])
        assert np.all(p[:, 2] == pos_z)
    P = np.ascontiguousarray(ro.env.arrays["arm_placement"], dtype=np.float64)
    for before, R, p, after in recs:
        for e in range(n):
            want = arm_ik.ik_step(P, before[e], R[e].reshape(3, 3), p[e])
            np.testing.assert_allclose(after[e], want, rtol=0, atol=1e-8 * max(1.0, np.abs(want - before[e]).max()))
