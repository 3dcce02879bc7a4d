"""Headline benchmark: env-steps/s of the batched MujocoUR5eCable + ACT rollout hot path.

`python bench.py --gpus N --steps K --warmup W`.  Under torch.distributed.run (WORLD_SIZE set)
each process is one rank on one GPU; with --gpus N > 1 and no WORLD_SIZE, bench.py spawns the N
ranks itself (before any GPU call).  Envs are sharded per rank by global env index; results are
all-gathered over RCCL at the end.

Workload (BASELINE.json configs[1] at N = 1): 1024 MujocoUR5eCable envs per GPU (weak scaling;
--total_envs T fixes the whole-job count instead, e.g. configs[2]: --total_envs 4096 on 8 GPUs),
ACT policy (ResNet-18 + 4/7-layer transformer, random init) in **fp32, the reference's
precision** (the credited `value`), synthetic episodes (world_idx = global env % 6,
world_random_scale [0.01, 0.01, 0], seed 0).  Every env is first driven through the scripted
pre-rollout phases (Initial 1.0 s, Reach 0.7 + 0.3 s, Grasp 0.5 s; untimed), then W warm-up and
K timed env-steps of the RolloutPhase hot loop: render + ACT every `skip` = 3 steps, temporal
ensemble, command routing, 8 physics substeps, observation, success predicate and phase
bookkeeping, all on the device.  One `step` = one env-step of every env.  The ACT decoder runs
layer 0 only: the DETRVAE output reads that layer's normed intermediate, layers 1..6 are dead
(exact; tests/test_act_full_gpu.py; --act_full_decoder runs all seven); the JSON line also prices
the step with all seven computed (`all_decoder_layers`, from one isolated 7-layer call).

The same workload with the policy in bf16 (throughput mode) is reported as `secondary_bf16`
with its measured action error against fp32 on the same inputs; it is never `value`.

Prints ONE JSON line (rank 0) with the roofline of the physics kernels (algorithmic bytes per
env-step / HIP-event kernel time), FP64 and policy-MFMA fractions, and the CPU
baseline (the oracle's C physics + ACT in PyTorch-CPU: a throughput leg of single-threaded
1-env processes, a 1-env latency leg and the C1 MLP leg, on bounded samples).
"""

import argparse
import json
import os
import subprocess
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
MFMA_PEAK_TFLOPS = {"fp32": 157.3, "bf16": 2500.0}  # MI355X_MICROARCH.md: F32 / BF16 MFMA dense
GOLDEN = os.path.join(ROOT, "tests", "golden")
C3_PER_RANK = 512  # BASELINE.json configs[2]: 4096 envs over 8 GPUs
CPU_WORKERS_MAX = 16  # fallback CPU share per GPU when the box does not export OMP_NUM_THREADS
_T0 = time.time()


def progress(msg):
    """Progress on stderr (stdout carries only the JSON line)."""
    print(f"[bench {time.time() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


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


def winograd_flops_saved_per_inference(tile="f4", H=480, W=640):
    """Direct-algorithm MFMA FLOPs minus the FLOPs the Winograd kernels execute, per image, for the
    stride-1 3x3 convs of the fp32 ResNet-18 trunk: F(4x4, 3x3) (rmbx_conv3x3_winograd4_f32) runs
    36 products per 4x4 output tile and input channel, F(2x2, 3x3) (rmbx_conv3x3_winograd_f32) 16
    per 2x2 tile, the direct algorithm 9 per output; maps that are not a multiple of the tile pad
    the last tile row / column (30x40 -> 32x40, 15x20 -> 16x20 under F(4x4))."""
    saved = 0
    for c, n_conv, s in ((64, 4, 4), (128, 3, 8), (256, 3, 16), (512, 3, 32)):
        h, w = -(-H // s), -(-W // s)
        saved += n_conv * (2 * h * w * c * c * 9 - winograd_launch_flops((1, c, h, w), tile))
    return saved


def winograd_launch_flops(shape, tile):
    """MFMA FLOPs one Winograd conv call executes on an NCHW `shape` (all frames, all launches)."""
    n, c, h, w = shape
    t = 4 if tile == "f4" else 2
    return 2 * (t + 2) ** 2 * c * c * (-(-h // t)) * (-(-w // t)) * n


def winograd_kernel_launches(shape, tile):
    """Kernel launches of one call: kernels.py slices the frames at *_MAX_ELEMS elements."""
    from robomanipbaselines_amd import kernels as K

    n, c, h, w = shape
    per = max(1, (K.WINOGRAD4_MAX_ELEMS if tile == "f4" else K.WINOGRAD_MAX_ELEMS) // (h * w * c))
    return -(-n // per)


def winograd_pmc_traffic(tile):
    """HBM counter bytes per conv call at 1024 frames, per layer shape, from the committed PMC
    passes (scripts/gpurun/wino_pmc.sh + tools/pmc_traffic.py --winograd); ({}, None) if absent."""
    import glob

    pat = "r*_pmc_winograd4_traffic.json" if tile == "f4" else "r*_pmc_winograd_traffic_v*.json"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pat)),
                   key=lambda f: int(os.path.basename(f)[1:].split("_")[0]))
    if not files:
        return {}, None
    path = files[-1]
    with open(path) as f:
        d = json.load(f)
    layers = d.get("layers", {})
    return ({int(k[1:].split("_")[0]): v.get("traffic_bytes_per_call", v.get("traffic_bytes_per_launch"))
             for k, v in layers.items()}, os.path.relpath(path, ROOT))


def winograd_probe(ro):
    """One infer_policy call of `ro` with HIP events around every Winograd conv call (on the stream
    it is launched on, nothing else queued): the dominant policy kernel's executed MFMA rate."""
    from robomanipbaselines_amd.policy.backbone import _FusedConv

    _FusedConv.PROBE = probe = []
    try:
        ro.infer_policy()
        torch.cuda.synchronize()
    finally:
        _FusedConv.PROBE = None
    if not probe:
        return None
    tile = probe[0][1]
    ms = flops = launches = 0
    layers = {}
    for shape, t, e0, e1 in probe:
        dt = e0.elapsed_time(e1)
        fl = winograd_launch_flops(shape, t)
        ms += dt
        flops += fl
        launches += winograd_kernel_launches(shape, t)
        L = layers.setdefault(shape[1], {"calls": 0, "ms": 0.0, "flops": 0})
        L["calls"] += 1
        L["ms"] += dt
        L["flops"] += fl
    tf = flops / ms / 1e9
    traffic, src = winograd_pmc_traffic(tile)
    frames = probe[0][0][0]
    tr = None
    if traffic and all(c in traffic for c in layers):
        tr = round(sum(traffic[c] * L["calls"] for c, L in layers.items()) * frames / 1024 / len(probe))
    return {"bound": "mfma", "achieved": round(tf, 2), "peak": MFMA_PEAK_TFLOPS["fp32"], "unit": "TFLOP/s",
            "frac": tf / MFMA_PEAK_TFLOPS["fp32"], "traffic": tr,
            "traffic_unit": "HBM bytes per conv call (one layer over all frames), mean over the calls of one inference",
            "traffic_source": src,
            "algorithmic_bytes_per_call": round(sum(3 * 4 * s[0] * s[1] * s[2] * s[3] for s, *_ in probe) / len(probe)),
            "kernel": ("rmbx::wino4_f32_kernel (Winograd F(4x4,3x3) f32 MFMA, bias+res+ReLU fused)" if tile == "f4"
                       else "rmbx::wino_f32_kernel (Winograd F(2x2,3x3) f32 MFMA)"),
            "flops": "executed MFMA FLOPs (2*(m+2)^2*C^2 per output tile and frame)",
            "calls_per_inference": len(probe), "launches_per_inference": launches,
            "avg_launch_us": round(1e3 * ms / launches, 1), "frames": frames,
            "per_layer": {f"C{c}": {"calls": L["calls"], "ms_per_call": round(L["ms"] / L["calls"], 3),
                                    "TFLOPs": round(L["flops"] / L["ms"] / 1e9, 2)} for c, L in sorted(layers.items())}}


def convp_pmc_traffic():
    """HBM counter bytes of the patch-staged conv dispatches of one fp32 ACT inference at 1024 envs
    (the same gemm_pmc.sh passes, tools/pmc_traffic.py --convp); (None, None) if absent."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_conv3x3p_traffic.json")),
                   key=lambda f: int(os.path.basename(f)[1:].split("_")[0]))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return d["read_bytes_per_inference"] + d["write_bytes_per_inference"], os.path.relpath(files[-1], ROOT)


def gemm_pmc_traffic():
    """HBM counter bytes of the gemm_f32x6 dispatches of one fp32 ACT inference at 1024 envs, from the
    committed PMC passes (scripts/gpurun/gemm_pmc.sh + tools/pmc_traffic.py --gemm); (None, None) if
    absent."""
    import glob

    from robomanipbaselines_amd import kernels as K

    # the newest committed profile of the form in use (r<round>_pmc_gemm_<form>_traffic.json)
    form = "f16x3" if K.F32_PIECES == "f16x3" else "f32x6"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_gemm_{form}_traffic.json")),
                   key=lambda f: int(os.path.basename(f)[1:].split("_")[0]))
    if not files:
        return None, None
    path = files[-1]
    with open(path) as f:
        d = json.load(f)
    return d["read_bytes_per_inference"] + d["write_bytes_per_inference"], os.path.relpath(path, ROOT)


def gemm_probe(ro):
    """One infer_policy call of `ro` with HIP events around every fp32-accurate GEMM launch
    (rmbx_linear_f16x3 / _batched / rmbx_conv2d_f16x3, or their bf16x6 counterparts under
    RMBX_F32_PIECES=bf16x6: the dominant policy kernel) and every patch-staged 3x3 conv
    (rmbx_conv3x3_f16x3_patch): executed MFMA rate (three f16 or six bf16 products per f32 product,
    both at the bf16 rate) against the bf16 dense peak.  Returns (GEMM line, patch-conv line)."""
    from robomanipbaselines_amd import kernels as K

    K.GEMM_PROBE = probe = []
    try:
        ro.infer_policy()
        torch.cuda.synchronize()
    finally:
        K.GEMM_PROBE = None
    gemm = [e for e in probe if not e[0].startswith("conv3x3p")]
    patch = [e for e in probe if e[0].startswith("conv3x3p")]
    return _probe_line(gemm, True), _probe_line(patch, False)


def gemm_library_ceiling():
    """The vendor library's f16 GEMM running the same MFMA work as the f16x3 form (K tripled, f32 out)
    at the ACT shapes, from the latest committed calibration (scripts/prof_blas_f16_ceiling.py ->
    profiles/r<round>_blas_f16_ceiling.json): {"source", "hipblaslt_frac": {shape: fraction of the
    dense peak}} or None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_blas_f16_ceiling.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    lt = d.get("libraries", {}).get("hipblaslt", {})
    return {"source": os.path.relpath(files[-1], ROOT),
            "hipblaslt_frac": {k: v["frac_f32_out"] for k, v in lt.items()},
            "note": "hipBLASLt f16 GEMM over [ah, ah, al] x [wh, wl, 2^-11 wh] (the same MFMA work as f16x3), f32 out, "
                    "same chip; the per_shape table above is this kernel at those shapes"}


def mfma_utilisation(prefix):
    """Matrix-core utilisation at the clock the chip held, per kernel instance, from the latest
    committed counter pass over one fp32 ACT inference (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
    GRBM_GUI_ACTIVE / 8); scripts/gpurun/r6_j.sh -> scripts/mfma_util.py ->
    profiles/r<round>_mfma_util_act_inference.txt): {"source", "kernels": {name: {util, clock_GHz}}}
    for the kernels whose name starts with `prefix`, or None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_mfma_util_act_inference.txt")))
    if not files:
        return None
    out = {}
    with open(files[-1]) as f:
        for line in f:
            parts = [x.strip() for x in line.split("|")]
            if len(parts) == 5 and parts[0].startswith(prefix):
                out[parts[0]] = {"mfma_busy": float(parts[2]), "held_clock_GHz": float(parts[3]),
                                 "launches": int(parts[1])}
    return {"source": os.path.relpath(files[-1], ROOT), "kernels": out,
            "note": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction of the matrix "
                    "cores' cycles busy at the clock the chip held under this load (DVFS); `frac` above is "
                    "against the nominal 2.5 PF (2.4 GHz)"} if out else None


def _probe_line(probe, is_gemm):
    if not probe:
        return None
    ms = flops = nbytes = executed = 0.0
    shapes = {}
    kinds = set()
    for name, fl, nb, products, e0, e1 in probe:
        dt = e0.elapsed_time(e1)
        ms += dt
        flops += fl
        nbytes += nb
        executed += products * fl
        kinds.add(products)
        L = shapes.setdefault(name, {"launches": 0, "ms": 0.0, "flops": 0.0})
        L["launches"] += 1
        L["ms"] += dt
        L["flops"] += fl
    eq = flops / ms / 1e9      # fp32-equivalent TFLOP/s
    ex = executed / ms / 1e9   # executed MFMA TFLOP/s
    n = len(probe)
    traffic, src = gemm_pmc_traffic() if is_gemm else convp_pmc_traffic()
    if traffic is not None:
        traffic /= n  # per call (a GEMM call is one or two kernel dispatches: the 256-wide tile + a 128 remainder)
    form = ("f16x3: each f32 operand split into two f16 pieces (the low one scaled by 2^11), three piece products "
            "on v_mfma_f32_16x16x32_f16" if kinds == {3} else
            "bf16x6: each f32 operand split into three bf16 pieces, six piece products on v_mfma_f32_16x16x32_bf16"
            if kinds == {6} else "mixed f16x3 / bf16x6")
    kernel = (f"rmbx::gemm_f32x6_kernel + rmbx::gemm_f16x3_presplit3_kernel (fp32-accurate GEMM / implicit-GEMM conv, "
              f"{form}, f32 accumulation; the pre-split form loads the LayerNorm-split A pieces by LDS-DMA)" if is_gemm
              else f"rmbx::conv3x3p_f16x3_kernel (patch-staged 3x3 / stride-1 conv, {form}, f32 accumulation)")
    return {"bound": "mfma", "achieved": round(ex, 2), "peak": MFMA_PEAK_TFLOPS["bf16"], "unit": "TFLOP/s",
            "frac": ex / MFMA_PEAK_TFLOPS["bf16"], "traffic": None if traffic is None else round(traffic),
            "traffic_unit": ("HBM bytes per GEMM call (one op launch; N = 3200 on the in-register form runs as two kernel "
                             "dispatches), mean "
                             "over the calls of one fp32 ACT inference at 1024 envs" if is_gemm else
                             "HBM bytes per conv call, mean over the calls of one fp32 ACT inference at 1024 envs"),
            "traffic_source": src,
            "algorithmic_bytes_per_launch": round(nbytes / n),
            "kernel": kernel,
            "flops": "executed MFMA FLOPs = products x the f32 problem's 2*M*N*K (3 for f16x3, 6 for bf16x6)",
            "achieved_fp32_equivalent": round(eq, 2), "f32_mfma_peak": MFMA_PEAK_TFLOPS["fp32"],
            "launches_per_inference": n, "avg_launch_us": round(1e3 * ms / n, 1),
            "ms_per_inference": round(ms, 3),
            "per_shape": {k: {"launches": L["launches"], "ms": round(L["ms"], 3),
                              "fp32_equiv_TFLOPs": round(L["flops"] / L["ms"] / 1e9, 1)} for k, L in shapes.items()},
            "library_ceiling": gemm_library_ceiling() if is_gemm else None,
            "mfma_utilisation": mfma_utilisation("rmbx::gemm_f" if is_gemm else "rmbx::conv3x3p")}


def policy_flops_per_inference(full_decoder):
    """FLOPs of one ACT inference per env (tools/count_policy_flops.py, FlopCounterMode)."""
    with open(os.path.join(GOLDEN, "policy_flops.json")) as f:
        return json.load(f)["act_480x640" if full_decoder else "act_480x640_dec0"]["flops_per_inference"]


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=6)
    p.add_argument("--num_envs", type=int, default=1024, help="environments per GPU (weak scaling)")
    p.add_argument("--total_envs", type=int, default=None,
                   help="whole-job environment count, sharded over the GPUs (strong scaling)")
    p.add_argument("--precision", choices=["fp32", "bf16"], default="fp32", help="policy precision of `value`")
    p.add_argument("--groups", type=int, default=1,
                   help="env groups per GPU, each on its own HIP stream with its policy steps offset by one env-step "
                        "(measured: no gain at 1024 envs, DESIGN.md section 5)")
    p.add_argument("--no_bf16_secondary", action="store_true")
    p.add_argument("--no_cpu_baseline", action="store_true")
    p.add_argument("--no_c3_per_rank", action="store_true", help="skip the 512-env configs[2] per-rank line")
    p.add_argument("--act_full_decoder", action="store_true", help="also run the dead decoder layers 1..6")
    p.add_argument("--cpu_steps", type=int, default=60, help="timed env-steps per CPU throughput worker")
    p.add_argument("--cpu_latency_steps", type=int, default=150, help="timed env-steps of the 1-env latency leg")
    p.add_argument("--cpu_mlp_steps", type=int, default=150, help="timed env-steps of the C1 MLP leg")
    p.add_argument("--_cpu_worker", choices=["act", "mlp"], default=None, help=argparse.SUPPRESS)
    p.add_argument("--_threads", type=int, default=1, help=argparse.SUPPRESS)
    p.add_argument("--_sync", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args(argv)


def algorithmic_bytes_per_env_step(nq, nv, nu, nsub):
    """per env-step the fused dynamics kernel must read qpos, qvel,
    qacc_warmstart, ctrl, time and write them back (ctrl read-only), plus obs (20 f64)
    and reward/flags: (nq + 2 nv + nu + 1) * 8 in + (nq + 2 nv + 1) * 8 out + 160 + 5."""
    return (nq + 2 * nv + nu + 1) * 8 + (nq + 2 * nv + 1) * 8 + 160 + 5


# --------------------------------------------------------------------------------------------
# CPU baseline (the reference's CPU path, restated: oracle C physics + PyTorch-CPU policy)
# --------------------------------------------------------------------------------------------
def cpu_model_name():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_worker(kind, steps, threads, sync, skip=3, warm=3):
    """One env of the reference loop on the CPU: C oracle physics (8 substeps per env-step),
    policy in PyTorch-CPU fp32 batch 1 every `skip` steps (ACT + numpy temporal ensemble, or the
    C1 MLP), `threads` intra-op threads.  Prints one JSON line {steps, seconds}."""
    torch.set_num_threads(threads)
    from oracle import glue
    from oracle.dyn import OracleEnv
    from robomanipbaselines_amd import model as MD
    from robomanipbaselines_amd.envs.ur5e_cable import CABLE_INIT_QPOS

    arrays = MD.load("ur5e_cable")
    env = OracleEnv(arrays)
    qpos = arrays["qpos0"].copy()
    qpos[:14] = CABLE_INIT_QPOS
    ctrl = np.concatenate([CABLE_INIT_QPOS[:6], [0.0]])
    env.set_state(0.0, qpos, np.zeros(env.nv), np.zeros(env.nv), ctrl)
    torch.manual_seed(0)
    stats = {"norm_config": {"type": "gaussian"}, "mean": ctrl.copy(), "std": np.full(7, 0.1)}
    img = torch.rand(1, 1, 3, 480, 640)
    if kind == "act":
        from robomanipbaselines_amd.policy.act.act_model import ActModel

        pol = ActModel().eval().requires_grad_(False)
        ens = glue.ActEnsembleOracle(100, stats)

        def act(state):
            chunk = pol(state, img)[0].numpy()
            return ens.step(lambda: chunk)
    else:
        from robomanipbaselines_amd.policy.mlp.mlp_model import MlpModel

        pol = MlpModel(7, 7, 1).eval().requires_grad_(False)

        def act(state):
            return glue.denormalize(pol(state[:, None], img[:, :, None])[0, 0].numpy().astype(np.float64), stats)

    t0 = time.time()
    for s in range(-warm, steps):
        if s == 0:
            if sync:  # start together with the other workers
                print("ready", flush=True)
                sys.stdin.readline()
            t0 = time.time()
        if s % skip == 0:
            _, qp, _, _ = env.state()
            state = torch.tensor(((qp[:7] - ctrl) / 0.1)[None], dtype=torch.float32)
            with torch.no_grad():
                a = act(state)
            env.set_ctrl(np.clip(a, -6.28, 255))
        env.step(8)
    print(json.dumps({"steps": steps, "seconds": time.time() - t0}), flush=True)


def _spawn_workers(kind, count, steps, threads):
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    cmd = [sys.executable, os.path.abspath(__file__), "--_cpu_worker", kind, "--cpu_steps", str(steps),
           "--_threads", str(threads)] + (["--_sync"] if count > 1 else [])
    procs = [subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)
             for _ in range(count)]
    if count > 1:
        for p in procs:
            assert p.stdout.readline().strip() == "ready"
        for p in procs:
            p.stdin.write("go\n")
            p.stdin.flush()
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=600)
        if p.returncode != 0:
            raise RuntimeError(f"cpu worker exited with {p.returncode}")
        outs.append(json.loads(out.strip().splitlines()[-1]))
    return outs


def cpu_baseline(args, skip=3):
    """SURVEY §8(d) CPU baseline on the box's host cores (bounded samples, about 30 s in all):
    throughput = P single-threaded processes with 1 env each started together (P = the CPU share
    the harness allows a 1-GPU box, at most 16; the per-GPU share visible/8 and the whole host are
    reported as labelled linear extrapolations), latency = 1 env with P threads, C1 = 1 env with the MLP policy and P threads.
    Rendering is excluded (the reference renders 3 cameras with MuJoCo's OpenGL renderer; there
    is no CPU renderer in this image)."""
    cores = len(os.sched_getaffinity(0))
    # the box's CPU share: the GPU pool exports it to every command as OMP_NUM_THREADS / MAX_JOBS (16
    # on a 1-GPU box, recorded in the line below); without it, CPU_WORKERS_MAX
    share_env = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "MAX_JOBS")}
    cap = CPU_WORKERS_MAX
    if (share_env["OMP_NUM_THREADS"] or "").isdigit() and int(share_env["OMP_NUM_THREADS"]) > 0:
        cap = int(share_env["OMP_NUM_THREADS"])
    P = max(1, min(cores, cap))
    t0 = time.time()
    progress(f"CPU baseline: {P} workers")
    thr = _spawn_workers("act", P, args.cpu_steps, 1)
    thr_value = P * args.cpu_steps / max(o["seconds"] for o in thr)
    lat = _spawn_workers("act", 1, args.cpu_latency_steps, P)[0]
    mlp = _spawn_workers("mlp", 1, args.cpu_mlp_steps, P)[0]
    # the harness caps a 1-GPU box's worker pools at 16 processes (its CPU share); the node's
    # per-GPU share is visible / 8 and the whole host is `cores`: the independent single-threaded
    # workers scale linearly, so those two are reported as labelled extrapolations of the measured rate
    share = max(1, cores // 8)
    return {"value": thr_value, "unit": "env-steps/s", "cores": P, "kind": "port",
            "cpu_model": cpu_model_name(), "host_cpus_visible": cores,
            "cpu_share": {"workers": P, "env": share_env,
                          "source": "the box's OMP_NUM_THREADS" if (share_env["OMP_NUM_THREADS"] or "").isdigit()
                          else "CPU_WORKERS_MAX default"},
            "per_gpu_share": {"cores": share, "value": round(thr_value * share / P, 1),
                              "basis": f"linear extrapolation of the {P}-process measurement to visible/8 cores"},
            "whole_host": {"cores": cores, "value": round(thr_value * cores / P, 1),
                           "basis": f"linear extrapolation of the {P}-process measurement to every visible core"},
            "sample": f"throughput leg: {P} single-threaded processes x 1 env x {args.cpu_steps} env-steps (after 3 "
                      f"untimed, started together): C oracle physics (8 substeps) + ACT fp32 PyTorch-CPU batch 1 "
                      f"every {skip} steps + numpy temporal ensemble; rendering excluded",
            "latency_leg": {"value": lat["steps"] / lat["seconds"], "unit": "env-steps/s", "threads": P,
                            "sample": f"1 env x {lat['steps']} env-steps, ACT with {P} intra-op threads"},
            "c1_mlp_leg": {"value": mlp["steps"] / mlp["seconds"], "unit": "env-steps/s", "threads": P,
                           "sample": f"config C1: 1 env x {mlp['steps']} env-steps, MLP policy (ResNet-18 + "
                                     f"[512, 512]) fp32 every {skip} steps, {P} threads"},
            "seconds": round(time.time() - t0, 1)}


# --------------------------------------------------------------------------------------------
# GPU rollout
# --------------------------------------------------------------------------------------------
def make_rollout(args, dev, precision, n_local, g0):
    from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable
    from robomanipbaselines_amd.policy.act.rollout_act import RolloutAct

    class Rollout(OperationMujocoUR5eCable, RolloutAct):
        pass

    argv = ["--num_envs", str(n_local), "--device", dev, "--world_idx_list", *[str(i) for i in range(6)],
            "--world_random_scale", "0.01", "0.01", "0.0", "--seed", "0", "--env_offset", str(g0),
            "--precision", precision]
    if not args.act_full_decoder:
        argv.append("--act_prune_dead_decoder")
    ro = Rollout(argv=argv)
    ro.reset()
    ro._active = None
    progress(f"{precision} rollout of {n_local} envs built; scripted pre-rollout phases")
    while ro.phase_idx < len(ro.pre_durations):  # scripted pre-rollout phases (untimed)
        ro.step_once()
    return ro


def timed_run(groups, args, dist):
    """W warm-up + K timed env-steps of every group, group g on HIP stream g (its policy steps
    offset by g env-steps: group g takes g extra warm-up steps), then isolated probes: the physics
    launch sequence of every group and one infer_policy call of group 0, each bracketed by HIP
    events with nothing else queued (in-loop events would include the other groups' kernels)."""
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in groups[1:]]
    for i in range(args.warmup):  # also MIOpen / hipBLASLt algorithm selection
        for ro in groups:
            ro.step_once()
        torch.cuda.synchronize()
        progress(f"warm-up step {i + 1}/{args.warmup}")
    for g, ro in enumerate(groups):
        for _ in range(g % max(1, ro.args.skip)):
            ro.step_once()
    if dist:
        import torch.distributed as tdist

        tdist.barrier()
    markers = os.environ.get("RMBX_TRACE_MARKERS") == "1"  # scripts/trace_window.py --marker spin_kernel
    if markers:
        torch.cuda._sleep(1000)
    # per-phase split of the timed steps (one group: its marks are one stream's timeline)
    from robomanipbaselines_amd.common.phase_timer import PhaseTimer

    timer = PhaseTimer() if len(groups) == 1 else None
    if timer is not None:
        groups[0].attach_phase_timer(timer)
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(args.steps):
        for ro, st in zip(groups, streams):
            with torch.cuda.stream(st):
                ro.step_once()
    if timer is not None:
        timer.mark("end")
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.time() - t0
    phases = None
    if timer is not None:
        groups[0].attach_phase_timer(None)
        seg, window = timer.summary()
        seg.pop("end", None)
        infers = sum(1 for (lab, _), (nxt, _) in zip(timer.marks, timer.marks[1:]) if lab == "policy" and nxt == "render")
        phases = {"ms_per_env_step": {k: round(v / args.steps, 3) for k, v in sorted(seg.items())},
                  "gpu_window_ms_per_env_step": round(window / args.steps, 3),
                  "wall_ms_per_env_step": round(1e3 * elapsed / args.steps, 3),
                  "accounted_frac": round(window / (1e3 * elapsed), 4),
                  "inferences_in_window": infers,
                  "note": "HIP events at the phase boundaries of every timed env-step on the rollout's stream: "
                          "render = rmbx_render of the policy camera, policy = infer_policy minus the render "
                          "(state, ACT, temporal ensemble), physics = rmbx_engine_step (8 substeps), glue = "
                          "the rest (command routing, obs, reward, schedule); a window of K steps holds "
                          "ceil or floor of K/skip inferences depending on the phase of rollout_time_idx"}
    if markers:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    progress(f"timed {args.steps} steps: {elapsed:.3f} s")
    # isolated probes (after the timed region)
    phys = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for ro in groups:
            ro.env.engine.step(8, ro._active if ro._active is not None else ro._step_mask)
        e1.record()
        torch.cuda.synchronize()
        phys.append(e0.elapsed_time(e1))
    infer = []
    for _ in range(2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        groups[0].infer_policy()
        e1.record()
        torch.cuda.synchronize()
        infer.append(e0.elapsed_time(e1) / 1e3)
    # the same call with all 7 decoder layers computed (the dead layers 1..6 included), for the
    # sensitivity line `all_decoder_layers`: the second call is timed
    infer_full = []
    pol = getattr(groups[0], "policy", None)
    if pol is not None and getattr(pol, "prune_dead_decoder", False):
        pol.prune_dead_decoder = False
        for _ in range(2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            groups[0].infer_policy()
            e1.record()
            torch.cuda.synchronize()
            infer_full = [e0.elapsed_time(e1) / 1e3]
        pol.prune_dead_decoder = True
    if dist:
        import torch.distributed as tdist

        t = torch.tensor([elapsed], dtype=torch.float64, device=groups[0].device)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, np.array(phys), np.array(infer), np.array(infer_full), phases


@torch.no_grad()
def bf16_action_error(ro32, ro16, n=16):
    """Max |action| difference of the bf16 policy against the fp32 policy (same weights, same
    rendered frame and state of the first n envs), on the denormalised scale: std_a x |d chunk|,
    which bounds the ensembled action difference (the ensemble weights sum to 1)."""
    from robomanipbaselines_amd import kernels as K

    n = min(n, ro32.n)
    state = ro32.get_state()[:n]
    img32 = ro32.get_images(torch.float32)[:n]  # the renderer's f32 space-to-depth frame
    c32 = ro32.policy(state, img32).float()
    if img32.dtype == torch.uint8:  # the 8-bit frame of the f32 stem: the bf16 policy takes it normalised
        mean, std = ro32.image_norm
        img32 = K.s2d_u8_normalize(img32, mean, std)
    elif img32.shape[-1] != 16:
        img32 = K.image_to_s2d(img32[:, 0])[:, None]
    c16 = ro16.policy(state.to(torch.bfloat16), img32.to(torch.bfloat16)).float()
    std = torch.tensor(ro32.model_meta_info["action"]["std"], dtype=torch.float32, device=c32.device)
    return float(((c16 - c32).abs() * std).max().item()), float(((c16 - c32).norm() / c32.norm()).item())


def job_shard(args, rank, world):
    """(strong scaling?, whole-job env count, global index of this rank's first env, its env count):
    weak scaling keeps --num_envs per GPU, --total_envs shards a fixed job over the ranks."""
    from robomanipbaselines_amd.distributed import shard_range

    strong = args.total_envs is not None
    total = args.total_envs if strong else args.num_envs * world
    g0, g1 = shard_range(rank, world, total)
    return strong, total, g0, g1 - g0


def rank_main(args):
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    dist = world > 1
    if dist:
        import torch.distributed as tdist

        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    dev = f"cuda:{local_rank}"
    from robomanipbaselines_amd import kernels as K
    from robomanipbaselines_amd.distributed import gather_results, pack_results

    strong, total, g0, n = job_shard(args, rank, world)
    G = max(1, min(args.groups, n))
    bounds = [n * g // G for g in range(G + 1)]

    def make_groups(precision):
        return [make_rollout(args, dev, precision, bounds[g + 1] - bounds[g], g0 + bounds[g]) for g in range(G)]

    groups = make_groups(args.precision)
    ro = groups[0]
    elapsed, phys, infer, infer_full, phases = timed_run(groups, args, dist)
    value = total * args.steps / elapsed
    if dist:
        # RCCL all-gather of per-env episode records (success, reward, duration, steps)
        parts = []
        for r in groups:
            v = K.sched_view(r.sched)
            parts.append(pack_results(v["success"], v["result_reward"], v["duration"], v["rollout_time_idx"]))
        gathered = gather_results(np.concatenate(parts), dev)
        assert gathered.shape[0] == total
    eng = ro.env.engine
    st = np.concatenate([r.env.engine.stats.cpu().numpy() for r in groups])
    bytes_env_step = algorithmic_bytes_per_env_step(eng.nq, eng.nv, eng.nu, 8)
    kern_s = float(phys.mean()) / 1e3
    achieved = n * bytes_env_step / kern_s / 1e9
    ncon, nefc, iters = float(st[:, 0].mean()), float(st[:, 1].mean()), float(st[:, 2].mean())
    fl_sub = physics_flops_per_substep(ncon, nefc, iters)
    fp64_tf = n * 8 * fl_sub / kern_s / 1e12
    traffic_env, traffic_src = pmc_traffic_per_env_step()
    pol_flops = policy_flops_per_inference(args.act_full_decoder)
    result = {
        "metric": "env-steps/s (whole node) + policy-inference us/step, MujocoUR5eCable x N ACT",
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": f"f64 physics + {args.precision} policy",
        "data": "synthetic (random-init ACT weights, seeded worlds)",
        "config": {"workload": f"MujocoUR5eCable x{total} ({n} per GPU), ACT (ResNet-18 + transformer 4/7 layers, "
                               f"chunk 100, skip 3, temporal ensembling), {args.precision} policy, RolloutPhase hot loop",
                   "num_envs_per_gpu": n, "total_envs": total,
                   "parallelism": (f"env-sharded x{world}, RCCL all-gather of results" if world > 1
                                   else "single GPU (no collective)"),
                   "env_groups": G,
                   "act_decoder_layers_run": 7 if args.act_full_decoder else 1},
        "policy_inference_us_per_call": round(1e6 * float(infer.mean()), 1) if len(infer) else None,
        "policy_inference_batch": groups[0].n,
        "policy_inference_us_per_env_step": round(1e6 * float(infer.mean()) / (groups[0].n * ro.args.skip), 3) if len(infer) else None,
        "physics_kernel_ms": round(float(phys.mean()), 3),
        "physics_probe": f"isolated HIP-event time of one env-step of all {n} envs ({G} engine launch sequences back to back)",
        "roofline_physics": {"bound": "hbm", "achieved": round(achieved, 4), "peak": HBM_PEAK_GBS, "unit": "GB/s",
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
    if phases is not None:
        result["phases"] = phases
    if len(infer):
        pol_tf = groups[0].n * pol_flops / float(infer.mean()) / 1e12
        peak = MFMA_PEAK_TFLOPS[args.precision]
        # whole batched infer_policy call (render + preprocessing + ACT), all kernels on the stream
        # the whole batched infer_policy call (render + preprocessing + ACT) at the direct-algorithm
        # FLOPs of the f32 problem: informational, no roofline fraction -- the stride-1 convs run as
        # Winograd (fewer products) and the GEMMs / convs as f16x3 f32 emulation (three f16 products
        # per f32 product at 16x the f32 MFMA rate), so this rate can exceed the f32 MFMA peak; the
        # kernel-level fractions are roofline (f16x3 GEMM), roofline_conv3x3 (patch-staged convs),
        # roofline_winograd, roofline_physics
        result["roofline_policy"] = {"achieved_direct_fp32_equivalent": round(pol_tf, 2), "unit": "TFLOP/s",
                                     "f32_mfma_peak": MFMA_PEAK_TFLOPS["fp32"], "bf16_mfma_peak": MFMA_PEAK_TFLOPS["bf16"],
                                     "dtype": args.precision, "algorithmic_flops_per_inference": pol_flops,
                                     "scope": "one batched infer_policy call over all envs"}
        from robomanipbaselines_amd.policy.backbone import _FusedBlock

        if args.precision == "fp32" and _FusedBlock.F32_CONV == "winograd":
            wp = winograd_probe(groups[0])
            if wp is not None:
                result["roofline_winograd"] = wp
            gp, cp = gemm_probe(groups[0])
            if cp is not None:
                result["roofline_conv3x3"] = cp
            if gp is not None:
                # the dominant kernel of the step: the physics line stays as
                # roofline_physics, the fused Winograd conv as roofline_winograd
                result["roofline"] = gp
            elif wp is not None:
                result["roofline"] = wp
    if "roofline" not in result:  # bf16 policy / direct convs: the physics env-step line
        result["roofline"] = result["roofline_physics"]
    if len(infer) and len(infer_full):
        # exact either way (the DETRVAE output reads decoder layer 0 only); priced here so that the
        # credited line can be compared with a rollout that also computes the dead layers
        extra = (float(infer_full.mean()) - float(infer.mean())) / ro.args.skip
        result["all_decoder_layers"] = {
            "policy_inference_us_per_call": round(1e6 * float(infer_full.mean()), 1),
            "value_estimate": round(total / (elapsed / args.steps + extra), 1), "unit": "env-steps/s",
            "note": "the same step with decoder layers 1..6 computed too (their output is never read): "
                    "timed value with the per-env-step policy time replaced by the measured 7-layer call"}
    if world == 1 and not strong and args.precision == "fp32" and n > C3_PER_RANK and not args.no_c3_per_rank:
        # BASELINE.json configs[2] (4096 envs over 8 GPUs) runs 512 envs per rank with no data-path
        # collective: its per-rank workload measured here, same loop and window, on this one GPU
        del groups, ro, eng
        torch.cuda.empty_cache()
        g3 = [make_rollout(args, dev, "fp32", C3_PER_RANK, 0)]
        el3, ph3, inf3, _, phases3 = timed_run(g3, args, False)
        v3 = C3_PER_RANK * args.steps / el3
        result["c3_per_rank"] = {
            "value": round(v3, 1), "unit": "env-steps/s", "num_envs": C3_PER_RANK,
            "ms_per_step": round(1e3 * el3 / args.steps, 3),
            "physics_kernel_ms": round(float(ph3.mean()), 3),
            "policy_inference_us_per_call": round(1e6 * float(inf3.mean()), 1) if len(inf3) else None,
            "phases": phases3,
            "projection_8gpu": {"value": round(8 * v3, 1), "unit": "env-steps/s",
                                "basis": "8 x this per-rank rate: the ranks share no data-path collective (one "
                                         "all-gather of episode records after the loop), so configs[2] is 8 "
                                         "independent copies of this workload; an estimate, not a measurement"},
            "note": "BASELINE.json configs[2]'s per-rank workload (4096 envs / 8 GPUs): the same fp32 ACT loop, "
                    "steps and warm-up as `value`, 512 envs on one GPU; the physics solver runs two blocks per "
                    "CU at this size (csrc/rmbx_engine.hip solver_minb_for)"}
        del g3
        torch.cuda.empty_cache()
        groups = ro = eng = None
    if args.precision == "fp32" and not args.no_bf16_secondary:
        del groups, ro, eng
        torch.cuda.empty_cache()
        groups16 = make_groups("bf16")
        el16, _, inf16, _, phases16 = timed_run(groups16, args, dist)
        ro32 = make_rollout(args, dev, "fp32", 16, g0)  # same weights (seeded), its own 16-env frame
        err_abs, err_rel = bf16_action_error(ro32, groups16[0])
        result["secondary_bf16"] = {
            "value": round(total * args.steps / el16, 1), "unit": "env-steps/s",
            "ms_per_step": round(1e3 * el16 / args.steps, 3), "dtype": "f64 physics + bf16 policy",
            "policy_inference_us_per_call": round(1e6 * float(inf16.mean()), 1) if len(inf16) else None,
            "max_abs_action_err_vs_fp32": err_abs, "chunk_rel_l2_err_vs_fp32": err_rel,
            "phases_ms_per_env_step": None if phases16 is None else phases16["ms_per_env_step"],
            "note": "throughput mode, NOT reference precision: same workload with the ACT policy in bf16; "
                    "action error measured on the first 16 envs' frame (same weights, same inputs)"}
        if len(inf16):
            tf16 = groups16[0].n * pol_flops / float(inf16.mean()) / 1e12
            result["secondary_bf16"]["roofline_policy"] = {"bound": "mfma", "achieved": round(tf16, 2),
                                                           "peak": MFMA_PEAK_TFLOPS["bf16"], "unit": "TFLOP/s",
                                                           "frac": tf16 / MFMA_PEAK_TFLOPS["bf16"]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(args)
        except Exception as exc:  # keep the GPU line even if the oracle is unavailable
            result["cpu_baseline"] = {"error": repr(exc)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        import torch.distributed as tdist

        tdist.destroy_process_group()


def _spawned_rank(local_rank, world, port, argv):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    rank_main(parse(argv))


def _heartbeat(period=60.0):
    """A line on stderr every `period` s, so one long first call (MIOpen Find, kernel
    compilation) is not mistaken for a hang."""
    import threading

    def beat():
        while True:
            time.sleep(period)
            progress("alive")

    threading.Thread(target=beat, daemon=True).start()


def main(argv=None):
    args = parse(argv)
    if args._cpu_worker:
        _cpu_worker(args._cpu_worker, args.cpu_steps, args._threads, args._sync)
        return
    _heartbeat()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launch the N ranks here (nothing has touched the GPU yet in this process)
        import socket

        import torch.multiprocessing as mp

        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        mp.spawn(_spawned_rank, args=(args.gpus, port, sys.argv[1:] if argv is None else argv), nprocs=args.gpus,
                 join=True)
        return
    rank_main(args)


if __name__ == "__main__":
    main()
