"""BASELINE config C3's per-rank workload on the HIP path: results do not depend on the GPU count.

C3 runs MujocoUR5eCable x4096 with ACT over 8 GPUs, i.e. 512 envs per rank (bench.py
--total_envs 4096, distributed.shard_range).  Envs are independent and every per-env quantity is
keyed by the GLOBAL env index (world index, Philox placement noise), so a rank's shard must evolve
exactly as the same envs do inside one unsharded batch (SURVEY.md section 8e;
common/base/RolloutBase.py:417-422 for the per-env records).

Here the fp32 ACT Cable rollout runs once as one 1024-env batch and once as two 512-env shards
(--env_offset 0 / 512, C3's per-rank size) on the same device, through the scripted pre-rollout
phases, several policy inferences and a forced episode end (a short --max_duration, plus a success
forced on a fixed set of global envs part-way), and the test asserts bitwise equality of every env's
qpos, its action at every env-step and its schedule records (success / reward / duration / steps).
The two shards' packed records are then all-gathered over gloo (world size 2, CPU processes of
this box) with distributed.gather_results and must equal the unsharded records."""

import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOTAL = 1024
SHARD = 512
MAX_DURATION = 0.6  # s of RolloutPhase: 19 env-steps of policy control, then the episode ends
FORCE_STEP = 8  # RolloutPhase env-step from which the forced envs report reward 1.0


def _forced(g):
    """Global envs whose reward is forced to 1.0 (success latch, then +1 s to the episode end)."""
    return g % 7 == 3


def _run(n, offset):
    from robomanipbaselines_amd import kernels as K
    from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable
    from robomanipbaselines_amd.policy.act.rollout_act import RolloutAct

    class Rollout(OperationMujocoUR5eCable, RolloutAct):
        pass

    ro = Rollout(argv=["--num_envs", str(n), "--device", DEV, "--world_idx_list", *[str(i) for i in range(6)],
                       "--world_random_scale", "0.01", "0.01", "0.0", "--seed", "0", "--env_offset", str(offset),
                       "--max_duration", str(MAX_DURATION), "--act_prune_dead_decoder"])
    real_reward = ro.env._get_reward
    forced = torch.tensor(_forced(np.arange(offset, offset + n)), device=DEV)
    clock = {"rollout_steps": -1}

    def reward():
        r = real_reward()
        if clock["rollout_steps"] >= FORCE_STEP:
            r = torch.where(forced, torch.ones_like(r), r)
        return r

    ro.env._get_reward = reward
    ro.reset()
    actions, steps = [], 0
    while True:
        if ro.phase_idx >= len(ro.pre_durations):
            clock["rollout_steps"] += 1
        ro.step_once()
        steps += 1
        if ro.phase_idx >= len(ro.pre_durations):
            actions.append(ro.policy_action.clone())
        if steps % 8 == 0 and ro.phase_idx >= len(ro.pre_durations) and K.sched_view(ro.sched)["done"].all():
            break
        assert steps < 400
    torch.cuda.synchronize()
    v = K.sched_view(ro.sched)
    rec = {k: np.array(v[k]) for k in ("success", "result_reward", "duration", "rollout_time_idx", "done")}
    out = dict(qpos=ro.env.engine.qpos.cpu().numpy(), time=ro.env.get_time().cpu().numpy(),
               actions=torch.stack(actions, 1).cpu().numpy(), rec=rec, steps=steps,
               inferences=len(ro._infer_events) + len(ro.inference_duration_list))
    del ro
    torch.cuda.empty_cache()
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather_worker(rank, world, port, shard_files, out_dir):
    import torch.distributed as dist

    from robomanipbaselines_amd.distributed import gather_results

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    local = np.load(shard_files[rank])
    full = gather_results(local, "cpu")
    np.save(os.path.join(out_dir, f"gathered_r{rank}.npy"), full)
    dist.destroy_process_group()


@torch.no_grad()
def test_c3_shards_equal_the_unsharded_batch(tmp_path):
    import torch.multiprocessing as mp

    from robomanipbaselines_amd.distributed import pack_results, shard_range

    full = _run(TOTAL, 0)
    shards = []
    for r in range(TOTAL // SHARD):
        g0, g1 = shard_range(r, TOTAL // SHARD, TOTAL)
        assert (g0, g1) == (r * SHARD, (r + 1) * SHARD)
        shards.append(_run(SHARD, g0))
    rec = full["rec"]
    # the episode ran past several inferences and ended for every env: forced successes latched,
    # the others stopped at max_duration
    assert full["inferences"] >= 2, full["inferences"]
    assert rec["done"].all()
    g = np.arange(TOTAL)
    assert (rec["success"].astype(bool) == _forced(g)).all()
    assert len(np.unique(rec["duration"])) >= 2
    for r, sh in enumerate(shards):
        sl = slice(r * SHARD, (r + 1) * SHARD)
        assert sh["steps"] == full["steps"]
        assert np.array_equal(sh["qpos"], full["qpos"][sl]), f"shard {r}: qpos"
        assert np.array_equal(sh["time"], full["time"][sl]), f"shard {r}: time"
        assert np.array_equal(sh["actions"], full["actions"][sl]), f"shard {r}: actions"
        for k in rec:
            assert np.array_equal(sh["rec"][k], rec[k][sl]), f"shard {r}: {k}"
    # the end-of-episode all-gather of the two shards' records (world size 2, gloo on this box's CPU)
    files = []
    for r, sh in enumerate(shards):
        f = str(tmp_path / f"shard{r}.npy")
        np.save(f, pack_results(sh["rec"]["success"], sh["rec"]["result_reward"], sh["rec"]["duration"],
                                sh["rec"]["rollout_time_idx"]))
        files.append(f)
    mp.spawn(_gather_worker, args=(2, _free_port(), files, str(tmp_path)), nprocs=2, join=True)
    want = pack_results(rec["success"], rec["result_reward"], rec["duration"], rec["rollout_time_idx"])
    for r in range(2):
        assert np.array_equal(np.load(tmp_path / f"gathered_r{r}.npy"), want)
