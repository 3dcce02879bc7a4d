"""Host-side logic of the rollout plugins on CPU (no device calls): model meta info handling and
the env sharding of world placements across GPU counts."""

import types

import numpy as np
import pytest

from robomanipbaselines_amd.distributed import shard_range


def test_checkpoint_without_meta_info_fails(tmp_path):
    """RolloutBase.setup_model_meta_info (:289-293) opens model_meta_info.pkl next to the
    checkpoint unconditionally; a missing file must not fall back to synthetic statistics."""
    from robomanipbaselines_amd.common.data_utils import make_meta_info

    ck = tmp_path / "policy_last.ckpt"
    ck.write_bytes(b"")
    op = types.SimpleNamespace(args=types.SimpleNamespace(checkpoint=str(ck)), policy_name="Act",
                               env=types.SimpleNamespace(init_qpos=np.zeros(14)))
    with pytest.raises(FileNotFoundError):
        make_meta_info(op)


def test_synthetic_meta_info_without_checkpoint():
    from robomanipbaselines_amd.common.data_utils import make_meta_info

    op = types.SimpleNamespace(args=types.SimpleNamespace(checkpoint=None), policy_name="Act",
                               env=types.SimpleNamespace(init_qpos=np.arange(14.0)))
    meta = make_meta_info(op)
    assert meta["data"]["skip"] == 3 and meta["data"]["chunk_size"] == 100
    np.testing.assert_array_equal(meta["state"]["mean"], np.r_[np.arange(6.0), 0.0])


def _env_shard(cls, n, offset, seed=0, scale=(0.01, 0.01, 0.0)):
    env = object.__new__(cls)
    env.num_envs = n
    env.seed = seed
    env.env_offset = offset
    env.world_random_scale = np.array(scale)
    env.original_world_pos = np.array([0.1, -0.2, 0.8])
    return env


@pytest.mark.parametrize("world", [2, 3, 8])
def test_world_positions_independent_of_gpu_count(world):
    """Per-env placements (offset per world index + Philox(seed, GLOBAL env) noise) of the shards
    of `world` ranks, concatenated, equal those of one unsharded batch (distributed.py)."""
    from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv as Env

    total = 37
    wl = list(range(6))
    full_idx = np.array([wl[g % 6] for g in range(total)])
    w_full, p_full = _env_shard(Env, total, 0)._world_positions(full_idx, None)
    parts_w, parts_p = [], []
    for r in range(world):
        g0, g1 = shard_range(r, world, total)
        idx = np.array([wl[(g0 + e) % 6] for e in range(g1 - g0)])
        w, p = _env_shard(Env, g1 - g0, g0)._world_positions(idx, None)
        parts_w.append(w)
        parts_p.append(p)
    np.testing.assert_array_equal(np.concatenate(parts_w), w_full)
    np.testing.assert_array_equal(np.concatenate(parts_p), p_full)
    # and the noise really is per env (not one draw broadcast)
    assert len(np.unique(p_full[:, 0])) == total
