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
