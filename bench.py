"""Headline benchmark: env-steps/s of the batched MujocoUR5eCable + ACT rollout hot path.

`python bench.py --gpus N --steps K --warmup W` (N > 1 under torch.distributed.run, one rank
per GPU, envs sharded per rank, results all-gathered over RCCL at the end).

Workload (BASELINE.json configs[1] at N = 1): 1024 MujocoUR5eCable envs per GPU, ACT policy
(ResNet-18 + 4/7-layer transformer, random init, bf16), synthetic episodes (world_idx = env % 6,
world_random_scale [0.01, 0.01, 0], seed 0).  Every env is first driven through the scripted
pre-rollout phases (Initial 1.0 s, Reach 0.7 + 0.3 s, Grasp 0.5 s; untimed), then W warm-up
and K timed env-steps of the RolloutPhase hot loop: render + ACT every `skip` = 3 steps,
temporal ensemble, command routing, 8 physics substeps, observation, success predicate and
phase bookkeeping, all on the device.  One `step` = one env-step of every env.

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (the fused physics
kernel: algorithmic bytes per env-step / measured kernel time) and the CPU baseline (oracle
physics + ACT in PyTorch-CPU on a bounded sample).
"""

import argparse
import json
import os
import sys
import time

import numpy as np

# MIOpen Find at 1024-env batch sizes: skip timing the naive reference solver (seconds per conv
# shape, never the one selected); must be set before MIOpen's first use in this process
os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (spec)
BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA dense (spec)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def physics_flops_per_substep(ncon, nefc, iters):
    """Algorithmic FP64 FLOPs of one substep at the measured constraint regime, from the op-count
    fixture (tools/count_flops.py over oracle/flopcount.cpp): fitted c0 + c1 ncon + c2 nefc +
    c3 iters + c4 iters*nefc."""
    with open(os.path.join(GOLDEN, "oracle_flops.json")) as f:
        c = json.load(f)["fit"]["coef"]
    return c[0] + c[1] * ncon + c[2] * nefc + c[3] * iters + c[4] * iters * nefc


def pmc_traffic_per_env_step():
    """Calibrated HBM-side bytes per env per env-step of the physics kernels from the latest committed
    counter profile (tools/pmc_traffic.py over two rocprofv3 --pmc passes); (bytes, file) or (None, None)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_physics_traffic_v*.json")),
                   key=lambda f: (os.path.basename(f).split("_")[0], int(f.rsplit("_v", 1)[1].split(".")[0])))
    if not files:
        return None, None
    with open(files[-1]) as f:
        return json.load(f)["bytes_per_env_step_per_env"], os.path.relpath(files[-1], ROOT)


def policy_flops_per_inference():
    """FLOPs of one ACT inference per env (tools/count_policy_flops.py, FlopCounterMode)."""
    with open(os.path.join(GOLDEN, "policy_flops.json")) as f:
        return json.load(f)["act_480x640"]["flops_per_inference"]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=6)
    p.add_argument("--num_envs", type=int, default=1024, help="environments per GPU")
    p.add_argument("--precision", choices=["bf16", "fp32"], default="bf16")
    p.add_argument("--no_cpu_baseline", action="store_true")
    p.add_argument("--cpu_sample_steps", type=int, default=600,
                   help="timed env-steps of the CPU baseline sample (about 10 s of host work)")
    p.add_argument("--act_prune_dead_decoder", action="store_true")
    return p.parse_args()


def algorithmic_bytes_per_env_step(nq, nv, nu, nsub):
    """per env-step the fused dynamics kernel must read qpos, qvel,
    qacc_warmstart, ctrl, time and write them back (ctrl read-only), plus obs (20 f64)
    and reward/flags: (nq + 2 nv + nu + 1) * 8 in + (nq + 2 nv + 1) * 8 out + 160 + 5."""
    return (nq + 2 * nv + nu + 1) * 8 + (nq + 2 * nv + 1) * 8 + 160 + 5


def cpu_baseline(sample_steps, skip=3):
    """Reference-path CPU baseline: the oracle's serial C physics (1 thread) + ACT in
    PyTorch-CPU (batch 1, all host threads) + numpy temporal ensemble, on `sample_steps`
    env-steps of one env (an inference every `skip` steps).  Rendering is not included (no
    CPU OpenGL renderer in this image)."""
    from oracle.dyn import OracleEnv
    from oracle import glue
    from robomanipbaselines_amd import model as MD
    from robomanipbaselines_amd.envs.ur5e_cable import CABLE_INIT_QPOS
    from robomanipbaselines_amd.policy.act.act_model import ActModel

    arrays = MD.load("ur5e_cable")
    env = OracleEnv(arrays)
    qpos = arrays["qpos0"].copy()
    qpos[:14] = CABLE_INIT_QPOS
    ctrl = np.concatenate([CABLE_INIT_QPOS[:6], [0.0]])
    env.set_state(0.0, qpos, np.zeros(env.nv), np.zeros(env.nv), ctrl)
    torch.manual_seed(0)
    threads = torch.get_num_threads()
    pol = ActModel().eval().requires_grad_(False)
    stats = {"norm_config": {"type": "gaussian"}, "mean": ctrl.copy(), "std": np.full(7, 0.1)}
    ens = glue.ActEnsembleOracle(100, stats)
    img = torch.rand(1, 1, 3, 480, 640)
    warm = 3  # untimed: first-call allocations of PyTorch-CPU
    t0 = time.time()
    for s in range(-warm, sample_steps):
        if s == 0:
            t0 = time.time()
        if s % skip == 0:
            state = torch.tensor(((qpos[:7] - ctrl) / 0.1)[None], dtype=torch.float32)
            with torch.no_grad():
                chunk = pol(state, img)[0].numpy()
            act = ens.step(lambda: chunk)
            env.set_ctrl(np.clip(act, -6.28, 255))
        env.step(8)
    dt = time.time() - t0
    return {"value": sample_steps / dt, "unit": "env-steps/s", "cores": int(threads), "kind": "port",
            "sample": f"{sample_steps} env-steps of 1 env (after {warm} untimed): C oracle physics (1 thread) + ACT "
                      f"fp32 PyTorch-CPU batch 1 every {skip} steps ({threads} threads) + numpy ensemble; "
                      f"rendering excluded", "seconds": round(dt, 2)}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    dist = world > 1
    if dist:
        import torch.distributed as tdist

        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    dev = f"cuda:{local_rank}"
    from robomanipbaselines_amd.bin.Rollout import main as rollout_main  # noqa: F401
    from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable
    from robomanipbaselines_amd.policy.act.rollout_act import RolloutAct
    from robomanipbaselines_amd import kernels as K

    class Rollout(OperationMujocoUR5eCable, RolloutAct):
        pass

    n = args.num_envs
    argv = ["--num_envs", str(n), "--device", dev, "--world_idx_list", *[str(i) for i in range(6)],
            "--world_random_scale", "0.01", "0.01", "0.0", "--seed", str(rank), "--precision", args.precision]
    if args.act_prune_dead_decoder:
        argv.append("--act_prune_dead_decoder")
    from robomanipbaselines_amd.distributed import gather_results, pack_results, shard_range

    ro = Rollout(argv=argv)
    # per-env world index from the GLOBAL env index so results do not depend on the GPU count
    g0, g1 = shard_range(rank, world, n * world)
    ro.args.world_idx_list = [g % 6 for g in range(g0, g1)]
    ro.reset()
    ro._active = None
    n_pre = len(ro.pre_durations)
    # scripted pre-rollout phases (untimed)
    while ro.phase_idx < n_pre:
        ro.step_once()
    # warm-up (also MIOpen/hipBLASLt algorithm selection)
    for _ in range(args.warmup):
        ro.step_once()

    # kernel timing: HIP events around every physics launch (same stream)
    phys_ms = []
    eng = ro.env.engine
    orig_step = eng.step

    def timed_step(nsub=8, active=None):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        orig_step(nsub, active)
        e1.record()
        phys_ms.append((e0, e1))

    eng.step = timed_step
    infer_ev = []
    orig_infer = ro.infer_policy

    def timed_infer():
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        orig_infer()
        e1.record()
        infer_ev.append((e0, e1))

    ro.infer_policy = timed_infer
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(args.steps):
        ro.step_once()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.time() - t0
    eng.step = orig_step
    ro.infer_policy = orig_infer
    phys = np.array([a.elapsed_time(b) for a, b in phys_ms])
    infer = np.array([a.elapsed_time(b) for a, b in infer_ev]) / 1e3  # seconds (GPU time)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
        # RCCL all-gather of per-env episode records (success, reward, duration, steps)
        v = K.sched_view(ro.sched)
        gathered = gather_results(pack_results(v["success"], v["result_reward"], v["duration"], v["rollout_time_idx"]), dev)
        assert gathered.shape[0] == n * world
    total_envs = n * world
    value = total_envs * args.steps / elapsed
    st = eng.stats.cpu().numpy()
    nq, nv, nu = eng.nq, eng.nv, eng.nu
    bytes_env_step = algorithmic_bytes_per_env_step(nq, nv, nu, 8)
    kern_s = float(phys.mean()) / 1e3
    achieved = n * bytes_env_step / kern_s / 1e9
    ncon, nefc, iters = float(st[:, 0].mean()), float(st[:, 1].mean()), float(st[:, 2].mean())
    fl_sub = physics_flops_per_substep(ncon, nefc, iters)
    fp64_tf = n * 8 * fl_sub / kern_s / 1e12
    traffic_env, traffic_src = pmc_traffic_per_env_step()
    result = {
        "metric": "env-steps/s (whole node) + policy-inference us/step, MujocoUR5eCable x N ACT",
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": f"f64 physics + {args.precision} policy",
        "data": "synthetic (random-init ACT weights, seeded worlds)",
        "config": {"workload": f"MujocoUR5eCable x{n} per GPU, ACT (ResNet-18 + transformer, chunk 100, skip 3, "
                               f"temporal ensembling), RolloutPhase hot loop", "num_envs_per_gpu": n,
                   "total_envs": total_envs, "parallelism": f"env-sharded x{world}, RCCL all-gather of results"},
        "policy_inference_us_per_call": round(1e6 * float(infer.mean()), 1) if len(infer) else None,
        "policy_inference_us_per_env_step": round(1e6 * float(infer.mean()) / (n * ro.args.skip), 3) if len(infer) else None,
        "physics_kernel_ms": round(float(phys.mean()), 3),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 4), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": round(traffic_env * n) if traffic_env else None,
                     "traffic_unit": "bytes per launch sequence (one env-step of all envs)",
                     "traffic_source": traffic_src,
                     "kernel": "physics env-step: 8 x (rmbx::front_kernel + rmbx::solver_kernel), one block per env",
                     "algorithmic_bytes_per_env_step": bytes_env_step},
        # the dynamics is not HBM-bound, so also its FP64 fraction on algorithmic FLOPs
        "roofline_fp64": {"bound": "fp64-valu", "achieved": round(fp64_tf, 4), "peak": FP64_PEAK_TFLOPS,
                          "unit": "TFLOP/s", "frac": fp64_tf / FP64_PEAK_TFLOPS,
                          "kernel": "physics env-step: 8 x (rmbx::front_kernel + rmbx::solver_kernel)",
                          "algorithmic_flops_per_substep": round(fl_sub)},
        "contacts_mean": ncon, "constraint_rows_mean": nefc, "newton_iters_mean": iters,
    }
    if len(infer):
        pol_tf = n * policy_flops_per_inference() / float(infer.mean()) / 1e12
        # whole batched infer_policy call (render + preprocessing + ACT), all kernels on the stream
        result["roofline_policy"] = {"bound": "mfma", "achieved": round(pol_tf, 2), "peak": BF16_PEAK_TFLOPS,
                                     "unit": "TFLOP/s", "frac": pol_tf / BF16_PEAK_TFLOPS,
                                     "algorithmic_flops_per_inference": policy_flops_per_inference(),
                                     "scope": "one batched infer_policy call over all envs"}
    if rank == 0 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(args.cpu_sample_steps)
        except Exception as exc:  # keep the GPU line even if the oracle is unavailable
            result["cpu_baseline"] = {"error": repr(exc)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
