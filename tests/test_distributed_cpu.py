"""World-size-2 gloo test of the env sharding and the end-of-episode result all-gather
(the N>1 path of bench.py / the rollout, exercised on CPU)."""

import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from robomanipbaselines_amd.distributed import gather_results, pack_results, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = shard_range(rank, world, total)
    g = np.arange(a, b)
    local = pack_results(g % 2 == 0, (g % 3) / 2.0, 0.032 * g, g % 7)
    full = gather_results(local, "cpu")
    np.save(os.path.join(out_dir, f"r{rank}.npy"), full)
    dist.destroy_process_group()


def test_shard_range_covers_all():
    for total in (1, 7, 1024, 4096, 4097):
        for world in (1, 2, 3, 8):
            r = [shard_range(k, world, total) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == total
            assert all(r[k][1] == r[k + 1][0] for k in range(world - 1))
            sz = [b - a for a, b in r]
            assert max(sz) - min(sz) <= 1


def test_gather_results_gloo_world2(tmp_path):
    total, world = 13, 2
    mp.spawn(_worker, args=(world, _free_port(), total, str(tmp_path)), nprocs=world, join=True)
    g = np.arange(total)
    exp = pack_results(g % 2 == 0, (g % 3) / 2.0, 0.032 * g, g % 7)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"r{r}.npy"), exp)


def _finish_worker(rank, world, port, total, out_dir):
    """One shard of a --num_gpus rollout at its end: BatchedRolloutBase.finish() all-gathers the
    per-env records and rank 0 writes the YAML in global env order."""
    import types

    import yaml

    from robomanipbaselines_amd import _native as N
    from robomanipbaselines_amd.common.rollout_base import BatchedRolloutBase

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g0, g1 = shard_range(rank, world, total)
    rec = np.zeros(g1 - g0, dtype=N.SCHED_DTYPE)
    g = np.arange(g0, g1)
    rec["success"] = g % 3 == 0
    rec["result_reward"] = (g % 3 == 0).astype(np.float64)
    rec["duration"] = 0.032 * (g + 1)
    rec["rollout_time_idx"] = g
    ro = object.__new__(BatchedRolloutBase)
    ro.device = torch.device("cpu")
    ro.n = g1 - g0
    ro.sched = torch.from_numpy(rec.view(np.uint8).reshape(g1 - g0, N.SCHED_DTYPE.itemsize).copy())
    ro.result = {k: [] for k in ("success", "reward", "duration")}
    ro.inference_duration_list, ro._infer_events = [], []
    ro.args = types.SimpleNamespace(save_last_image=False, env_offset=g0,
                                    result_filename=os.path.join(out_dir, f"result_r{rank}.yaml"))
    ro.finish()
    dist.destroy_process_group()
    with open(os.path.join(out_dir, f"n_r{rank}.yaml"), "w") as f:
        yaml.dump({"n_result": len(ro.result["success"])}, f)


def test_rollout_finish_gathers_shards_gloo_world2(tmp_path):
    import yaml

    total, world = 11, 2
    mp.spawn(_finish_worker, args=(world, _free_port(), total, str(tmp_path)), nprocs=world, join=True)
    with open(tmp_path / "result_r0.yaml") as f:
        res = yaml.safe_load(f)
    g = np.arange(total)
    assert res["success"] == [bool(x) for x in g % 3 == 0]
    assert res["reward"] == [float(x) for x in (g % 3 == 0)]
    assert res["duration"] == [float(np.float64(0.032) * (x + 1)) for x in g]
    assert not (tmp_path / "result_r1.yaml").exists()  # only rank 0 writes


def test_bench_job_shards():
    """bench.py's rank plan: weak scaling keeps 1024 envs per GPU; configs[2] (--total_envs 4096
    on 8 GPUs) gives 512 per rank covering the global env range once."""
    import bench

    a = bench.parse(["--gpus", "2"])
    assert [bench.job_shard(a, r, 2) for r in range(2)] == [(False, 2048, 0, 1024), (False, 2048, 1024, 1024)]
    a = bench.parse(["--gpus", "8", "--total_envs", "4096"])
    plan = [bench.job_shard(a, r, 8) for r in range(8)]
    assert all(p[0] and p[1] == 4096 and p[3] == 512 for p in plan)
    assert [p[2] for p in plan] == list(range(0, 4096, 512))
