"""Meta CLI: `python -m robomanipbaselines_amd.bin.Rollout <Policy> <Env> [--num_envs N]
[--num_gpus G] ...`.

Same composition as bin/Rollout.py of the reference (:10-95): resolve Operation<Env> and
Rollout<Policy> by name and compose `class Rollout(Operation<Env>, Rollout<Policy>)` (the MRO
order matters, :82-86); remaining arguments go to the inner parser.

--num_gpus G > 1: one process per GPU (spawned here before any GPU call, or launched by
torch.distributed.run), each stepping the contiguous global env range of its rank
(distributed.shard_range; world index and noise stream per GLOBAL env), then one RCCL all-gather
of the per-env results; rank 0 prints them and writes the YAML in global env order.
"""

import argparse
import os
import importlib
import sys

import yaml

POLICIES = ["Mlp", "Act", "DiffusionPolicy", "DiffusionPolicy3d"]
ENVS = ["MujocoUR5eCable", "MujocoUR5eInsert", "MujocoUR5eDoor", "MujocoUR5eCabinet", "MujocoUR5eToolbox", "MujocoUR5ePick",
        "MujocoUR5eRing"]


def camel_to_snake(name):
    """common/utils/MiscUtils.py:20-32"""
    import re

    name = re.sub(r"([a-z0-9])([A-Z])", r"\1_\2", name)
    name = re.sub(r"([a-z])([0-9])", r"\1_\2", name)
    name = re.sub(r"([A-Z]+)([A-Z][a-z])", r"\1_\2", name)
    return (name[0].lower() + name[1:]).lower()


def main(argv=None):
    parser = argparse.ArgumentParser(fromfile_prefix_chars="@", add_help=False)
    parser.add_argument("policy", type=str, nargs="?", default=None, choices=POLICIES)
    parser.add_argument("env", type=str, nargs="?", default=None, choices=ENVS)
    parser.add_argument("--config", type=str)
    parser.add_argument("-h", "--help", action="store_true")
    args, remaining = parser.parse_known_args(argv)
    if args.policy is None or args.env is None:
        parser.print_help()
        return None
    gpus = argparse.ArgumentParser(add_help=False)
    gpus.add_argument("--num_gpus", type=int, default=1)
    if gpus.parse_known_args(remaining)[0].num_gpus > 1 and "WORLD_SIZE" not in os.environ and not args.help:
        # one process per GPU, started before anything here touches the GPU
        import socket

        import torch.multiprocessing as mp

        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        n = gpus.parse_known_args(remaining)[0].num_gpus
        mp.spawn(_rank_entry, args=(n, port, argv if argv is not None else sys.argv[1:]), nprocs=n, join=True)
        return None
    op_mod = importlib.import_module(f"robomanipbaselines_amd.envs.operation.Operation{args.env}")
    OperationEnvClass = getattr(op_mod, f"Operation{args.env}")
    pol_mod = importlib.import_module(f"robomanipbaselines_amd.policy.{camel_to_snake(args.policy)}.rollout_{camel_to_snake(args.policy)}")
    RolloutPolicyClass = getattr(pol_mod, f"Rollout{args.policy}")

    class Rollout(OperationEnvClass, RolloutPolicyClass):
        @property
        def policy_name(self):
            return args.policy

    config = {}
    if args.config is not None:
        with open(args.config) as f:
            config = yaml.safe_load(f) or {}
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--num_envs", type=int, default=None)
    pre.add_argument("--world_idx_list", type=int, nargs="*", default=None)
    pre.add_argument("--world_idx", type=int, default=0)
    ns, _ = pre.parse_known_args(remaining)
    n_envs = ns.num_envs or len(ns.world_idx_list or [ns.world_idx])
    if int(os.environ.get("WORLD_SIZE", 1)) > 1:
        shard, n_envs = _shard_args(n_envs)
        remaining = remaining + shard  # argparse takes the last --num_envs: this rank's shard
    if n_envs >= 256 and args.policy in ("Act", "Mlp"):
        # large conv batches: keep MIOpen Find from timing its naive reference solver (seconds per
        # shape, never selected); process-wide, read by MIOpen on first use
        os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
    rollout = Rollout(argv=remaining + (["--help"] if args.help else []), **config)
    rollout.run()
    if int(os.environ.get("WORLD_SIZE", 1)) > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return rollout


def _shard_args(total):
    """Join this rank's process group (RCCL); return the inner-parser overrides of its shard and
    the shard's env count."""
    import torch
    import torch.distributed as dist

    from ..distributed import shard_range

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    g0, g1 = shard_range(rank, world, total)
    return ["--num_envs", str(g1 - g0), "--env_offset", str(g0), "--device", f"cuda:{local}"], g1 - g0


def _rank_entry(local_rank, world, port, argv):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    main(argv)


if __name__ == "__main__":
    main(sys.argv[1:])
