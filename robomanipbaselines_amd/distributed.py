"""Multi-GPU sharding of the env batch (one process per GPU, torch.distributed over RCCL/xGMI).

Envs are independent, so the only exchange is ONE all-gather of per-env episode results at the
end: (success, reward, duration, rollout steps) per env, 4 f64 = 32 B/env.
The shard of rank r is the contiguous global env range [r*N/W, (r+1)*N/W); per-env seeds and
world indices derive from the GLOBAL env index, so results do not depend on the GPU count.
"""

import numpy as np
import torch


def shard_range(rank, world, total):
    """Contiguous global env range of `rank` (sizes differ by at most one)."""
    base, rem = divmod(int(total), int(world))
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def pack_results(success, reward, duration, steps):
    return np.stack([np.asarray(success, np.float64), np.asarray(reward, np.float64),
                     np.asarray(duration, np.float64), np.asarray(steps, np.float64)], axis=1)


def gather_results(local, device, group=None):
    """All-gather [n_local, 4] f64 result records from every rank (variable n_local allowed);
    returns the [n_total, 4] array in global env order."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    t = torch.as_tensor(np.ascontiguousarray(local), dtype=torch.float64, device=device)
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    m = int(max(int(s.item()) for s in sizes))
    pad = torch.zeros((m, 4), dtype=torch.float64, device=device)
    pad[: t.shape[0]] = t
    out = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(out, pad, group=group)
    return torch.cat([o[: int(s.item())] for o, s in zip(out, sizes)]).cpu().numpy()
