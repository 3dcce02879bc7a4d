"""Meta CLI: `python -m robomanipbaselines_amd.bin.Rollout <Policy> <Env> [--num_envs N] ...`.

Same composition as bin/Rollout.py of the reference (:10-95): resolve Operation<Env> and
Rollout<Policy> by name and compose `class Rollout(Operation<Env>, Rollout<Policy>)` (the MRO
order matters, :82-86); remaining arguments go to the inner parser.
"""

import argparse
import os
import importlib
import sys

import yaml

POLICIES = ["Mlp", "Act", "DiffusionPolicy", "DiffusionPolicy3d"]
ENVS = ["MujocoUR5eCable", "MujocoUR5eInsert", "MujocoUR5eDoor", "MujocoUR5eCabinet", "MujocoUR5eToolbox"]


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
    ns, _ = pre.parse_known_args(remaining)
    n_envs = ns.num_envs or len(ns.world_idx_list or [0])
    if n_envs >= 256 and args.policy in ("Act", "Mlp"):
        # large conv batches: keep MIOpen Find from timing its naive reference solver (seconds per
        # shape, never selected); process-wide, read by MIOpen on first use
        os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
    rollout = Rollout(argv=remaining + (["--help"] if args.help else []), **config)
    rollout.run()
    return rollout


if __name__ == "__main__":
    main(sys.argv[1:])
