"""Closed-loop rollout parity: the batched HIP rollout (RolloutAct on OperationMujocoUR5eCable, fp32
policy, the bench's device forms) runs in lockstep with the reference's loop restated on the CPU
(oracle/rollout.py: RolloutBase.run, the phases, ArmManager IK, RolloutAct's ensemble, routing,
reward, oracle physics) with the CPU fp32 ACT module (all seven decoder layers) on the frame the
GPU renders of the same env-step (the renderer is pinned separately, tests/test_render_gpu.py).

Through the whole episode -- Initial, Reach1, Reach2, Grasp, then RolloutPhase until
--max_duration ends it -- every env-step asserts:
* the phase schedule (host mirror and device record), reward and, at the end, the result records
  (success, reward, duration): bit-exact;
* the pre-motion commands (IK steps, gripper): 1e-9 (both are f64 restatements of one formula);
* the policy actions after the temporal ensemble: 1e-4 (north star);
* the arm joint positions: 1e-4 (north star); the whole qpos (gripper linkage, 48 cable hinges,
  the cable's free joint) is held to BAR_QPOS_ALL over this horizon, the bar the divergence curve
  of the engine against the oracle supports (profiles/r6_divergence_cable.json).

References: common/base/RolloutBase.py:387-426, policy/act/RolloutAct.py:68-101,
envs/mujoco/MujocoEnvBase.py:82-97."""

import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
N_ENV = 4
MAX_DURATION = 0.6  # RolloutPhase: 19 env-steps, 7 inferences at skip 3
BAR_ACTION = 1e-4
BAR_ARM = 1e-4
BAR_CMD = 1e-9
BAR_QPOS_ALL = 1e-4


def _rollout(monkeypatch):
    import robomanipbaselines_amd.policy.act.rollout_act as RA
    from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable

    captured = {}
    real = RA.ActModel

    def factory(*a, **k):
        m = real(*a, **k)
        captured["cpu"] = copy.deepcopy(m)  # the same random-init weights, before the device fusions
        return m

    monkeypatch.setattr(RA, "ActModel", factory)

    class Rollout(OperationMujocoUR5eCable, RA.RolloutAct):
        pass

    ro = Rollout(argv=["--num_envs", str(N_ENV), "--device", DEV, "--world_idx_list", "0", "1", "2", "3",
                       "--world_random_scale", "0.01", "0.01", "0.0", "--seed", "0", "--precision", "fp32",
                       "--max_duration", str(MAX_DURATION), "--act_prune_dead_decoder"])
    cpu = captured["cpu"].eval().requires_grad_(False).float()
    assert not cpu.prune_dead_decoder
    return ro, cpu


def _cpu_images(ro):
    """The policy camera's 8-bit frame of the current env-step (the same render the policy tensor
    is made from, tests/test_env_info_gpu.py), normalised as ACTPolicy does in f32."""
    from robomanipbaselines_amd.policy.act.act_model import IMAGENET_MEAN, IMAGENET_STD

    u = ro.info["rgb_images"][ro.camera_names[0]].cpu()  # [n, H, W, 3] u8
    x = u.permute(0, 3, 1, 2).float() / 255.0
    m = torch.tensor(IMAGENET_MEAN).reshape(1, 3, 1, 1)
    s = torch.tensor(IMAGENET_STD).reshape(1, 3, 1, 1)
    return ((x - m) / s)[:, None]


@torch.no_grad()
def test_closed_loop_rollout_matches_cpu_reference_loop(monkeypatch):
    from oracle.rollout import CableRolloutOracle
    from robomanipbaselines_amd import kernels as K

    ro, cpu = _rollout(monkeypatch)
    ro.reset()
    env = ro.env
    bp = env.engine.body_pos.cpu().numpy()
    orcs = [CableRolloutOracle(env.arrays, env.init_qpos_head, bp[e, env._world_body], ro.model_meta_info,
                               skip=ro.args.skip, max_duration=MAX_DURATION) for e in range(N_ENV)]
    n_pre = len(ro.pre_durations)
    assert n_pre == orcs[0].n_pre == 4
    arm_q = orcs[0].arm_q
    # the reset states agree before the first step
    np.testing.assert_array_equal(env.engine.qpos.cpu().numpy(), np.stack([o.qpos() for o in orcs]))
    dev = {"action": 0.0, "arm_qpos": 0.0, "qpos_all": 0.0, "cmd_pre": 0.0, "state": 0.0}
    curve = []
    inferences = policy_steps = 0
    for t in range(400):
        infer = [o.needs_inference() for o in orcs]
        assert len(set(infer)) == 1  # the pre-rollout schedule is env-independent
        chunks = [None] * N_ENV
        if infer[0]:
            state_cpu = np.stack([o.policy_state() for o in orcs])
            state_gpu = ro.get_state().cpu().numpy()
            dev["state"] = max(dev["state"], float(np.abs(state_gpu - state_cpu).max()))
            c = cpu(torch.from_numpy(state_cpu), _cpu_images(ro)).numpy()
            chunks = list(c)
            inferences += 1
        in_rollout = orcs[0].phase == n_pre
        ro.step_once()
        for e, o in enumerate(orcs):
            o.step(chunks[e])
        # schedule: host mirror, device record, reward -- bit-exact
        v = K.sched_view(ro.sched)
        phases = np.array([o.phase for o in orcs])
        np.testing.assert_array_equal(v["phase"], phases, err_msg=f"step {t}")
        assert ro.phase_idx == min(int(phases.max()), n_pre), t
        np.testing.assert_array_equal(ro.reward.cpu().numpy(), [o.reward for o in orcs], err_msg=f"step {t}")
        np.testing.assert_array_equal(env.get_time().cpu().numpy(), [o.time() for o in orcs])
        # commands and actions
        cmd_gpu = torch.cat([ro.q_cmd, ro.grip_cmd], 1).cpu().numpy()
        cmd_cpu = np.stack([np.concatenate([o.arm.q, o.arm.g]) for o in orcs])
        d_cmd = float(np.abs(cmd_gpu - cmd_cpu).max())
        if in_rollout:
            policy_steps += 1
            d_act = float(np.abs(ro.policy_action.cpu().numpy() - np.stack([o.policy_action for o in orcs])).max())
            dev["action"] = max(dev["action"], d_act, d_cmd)
            assert d_act <= BAR_ACTION and d_cmd <= BAR_ACTION, (t, d_act, d_cmd)
        else:
            dev["cmd_pre"] = max(dev["cmd_pre"], d_cmd)
            assert d_cmd <= BAR_CMD, (t, d_cmd)
        # trajectories
        q_gpu = env.engine.qpos.cpu().numpy()
        q_cpu = np.stack([o.qpos() for o in orcs])
        d_arm = float(np.abs(q_gpu[:, arm_q] - q_cpu[:, arm_q]).max())
        d_all = float(np.abs(q_gpu - q_cpu).max())
        curve.append((t, int(phases.max()), d_arm, d_all))
        dev["arm_qpos"] = max(dev["arm_qpos"], d_arm)
        dev["qpos_all"] = max(dev["qpos_all"], d_all)
        assert d_arm <= BAR_ARM, (t, d_arm)
        assert d_all <= BAR_QPOS_ALL, (t, d_all)
        if all(o.phase > n_pre for o in orcs):
            break
    else:
        pytest.fail("the episode did not end")
    print(f"\nclosed loop: {t + 1} env-steps ({policy_steps} in RolloutPhase, {inferences} inferences); max deviation "
          "GPU vs CPU reference loop: " + ", ".join(f"{k} {x:.2e}" for k, x in dev.items()))
    print("per env-step (step, phase, |d arm qpos|, |d qpos|): "
          + " ".join(f"{s}:{p}:{a:.1e}:{q:.1e}" for s, p, a, q in curve[::5]))
    assert policy_steps >= 12 and inferences >= 4
    # EndRolloutPhase: the GPU env is frozen at its transition step (the state its results were
    # recorded from); the episode is marked done on the next env-step (EndRolloutPhase.check_transition)
    frozen = env.engine.qpos.clone()
    ro.step_once()
    assert torch.equal(env.engine.qpos, frozen)
    # result records: bit-exact
    v = K.sched_view(ro.sched)
    for e, o in enumerate(orcs):
        succ, rew, dur = o.result
        assert v["done"][e] == 1
        assert bool(v["success"][e]) == succ
        assert v["result_reward"][e] == rew
        assert v["duration"][e] == dur
