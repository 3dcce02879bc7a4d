"""Torch-facing wrappers of the rmbx C ABI glue kernels (shape/dtype checks + launch).

All tensors must be CUDA (HIP) tensors, contiguous, with the dtypes named below; work is
enqueued on the current torch stream.  Shape errors raise ValueError, as the reference's
MotionManager/DataKey do for bad keys (common/manager/MotionManager.py:36-39).
"""

import os
import numpy as np
import torch

from . import _native as N


def _chk(t, dtype, shape=None, name="tensor"):
    if not isinstance(t, torch.Tensor):
        raise ValueError(f"{name} must be a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor (got {t.device})")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype} (got {t.dtype})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)} (got {tuple(t.shape)})")
    return t


# ------------------------------------------------------------------------------------------
# ACT temporal ensemble
# ------------------------------------------------------------------------------------------
def ensemble_weight_table(chunk, k=0.01):
    """w[n-1, i] for n = 1..chunk: the weights of RolloutAct.py:90-92, computed with numpy
    exactly as the reference does (np.exp then division by the pairwise np.sum)."""
    w = np.zeros((chunk, chunk), dtype=np.float64)
    for n in range(1, chunk + 1):
        e = np.exp(-k * np.arange(n))
        w[n - 1, :n] = e / e.sum()
    return w


def denorm_coeffs(stats):
    """(scale, sub, add) such that denormalize_data(a) == scale * (a - sub) + add bit-exactly
    (common/utils/DataUtils.py:26-40)."""
    norm_type = stats["norm_config"]["type"] if "norm_config" in stats else "gaussian"
    if norm_type == "gaussian":
        std = np.asarray(stats["std"], dtype=np.float64)
        return std, np.zeros_like(std), np.asarray(stats["mean"], dtype=np.float64)
    if norm_type == "limits":
        cfg = stats["norm_config"]
        rng = np.asarray(stats["range"], dtype=np.float64)
        scale = rng / (cfg["out_max"] - cfg["out_min"])
        return scale, np.full_like(rng, cfg["out_min"]), np.asarray(stats["min"], dtype=np.float64)
    raise ValueError(f"[denormalize_data] Invalid normalization type: {norm_type}")


def norm_coeffs(stats):
    """(scale, sub, add) with normalize_data(x) == (x - sub) * or / ... see DataUtils.py:9-24.
    Returned as the pair used by the device path: gaussian -> ((x - mean) / std),
    limits -> scale * (x - min) + out_min."""
    norm_type = stats["norm_config"]["type"] if "norm_config" in stats else "gaussian"
    if norm_type == "gaussian":
        return "gaussian", np.asarray(stats["mean"], np.float64), np.asarray(stats["std"], np.float64)
    if norm_type == "limits":
        cfg = stats["norm_config"]
        scale = (cfg["out_max"] - cfg["out_min"]) / np.asarray(stats["range"], np.float64)
        return "limits", np.asarray(stats["min"], np.float64), (scale, cfg["out_min"])
    raise ValueError(f"[normalize_data] Invalid normalization type: {norm_type}")


class ActEnsembleState:
    """Per-env chunk history ring for the batched RolloutAct.infer_policy."""

    def __init__(self, n_env, chunk, adim, stats, device, temporal_ensemble=True, k=0.01):
        self.n_env, self.chunk, self.adim = n_env, chunk, adim
        self.te = bool(temporal_ensemble)
        self.hist = torch.zeros((n_env, chunk if self.te else 1, chunk, adim), dtype=torch.float32, device=device)
        self.len = torch.zeros(n_env, dtype=torch.int32, device=device)
        self.head = torch.zeros(n_env, dtype=torch.int32, device=device)
        self.w = torch.tensor(ensemble_weight_table(chunk, k), device=device)
        sc, sb, ad = denorm_coeffs(stats)
        self.dn = [torch.tensor(x, dtype=torch.float64, device=device).contiguous() for x in (sc, sb, ad)]
        self.out = torch.zeros((n_env, adim), dtype=torch.float64, device=device)

    def reset(self, mask=None):
        if mask is None:
            self.len.zero_()
            self.head.zero_()
        else:
            m = mask.bool()
            self.len[m] = 0
            self.head[m] = 0

    def __call__(self, new_chunk, push=None, active=None):
        act_ensemble(
            new_chunk, push, active, self.hist, self.len, self.head, self.w, *self.dn, self.out,
            temporal_ensemble=self.te,
        )
        return self.out


def act_ensemble(new_chunk, push, active, hist, hist_len, hist_head, w_table, dn_scale, dn_sub,
                 dn_add, out, temporal_ensemble=True):
    n_env, adim = out.shape
    chunk = w_table.shape[0]
    _chk(out, torch.float64, name="out")
    if temporal_ensemble:
        _chk(hist, torch.float32, (n_env, chunk, chunk, adim), "hist")
    else:
        _chk(hist, torch.float32, (n_env, 1, chunk, adim), "hist")
    _chk(hist_len, torch.int32, (n_env,), "hist_len")
    _chk(hist_head, torch.int32, (n_env,), "hist_head")
    _chk(w_table, torch.float64, (chunk, chunk), "w_table")
    for t, nm in ((dn_scale, "dn_scale"), (dn_sub, "dn_sub"), (dn_add, "dn_add")):
        _chk(t, torch.float64, (adim,), nm)
    if new_chunk is not None:
        _chk(new_chunk, torch.float32, (n_env, chunk, adim), "new_chunk")
    if push is not None:
        _chk(push, torch.uint8, (n_env,), "push")
    if active is not None:
        _chk(active, torch.uint8, (n_env,), "active")
    if new_chunk is None and (push is None or bool(push.any())):
        raise ValueError("new_chunk is required when pushing")
    N.call(
        "rmbx_act_ensemble", N.ptr(new_chunk), N.ptr(push), N.ptr(active), N.ptr(hist),
        N.ptr(hist_len), N.ptr(hist_head), N.ptr(w_table), N.ptr(dn_scale), N.ptr(dn_sub),
        N.ptr(dn_add), N.ptr(out), n_env, chunk, adim, int(temporal_ensemble), N.stream_ptr(),
    )
    return out


# ------------------------------------------------------------------------------------------
# Cable success predicate, UR5e observation, depth linearisation
# ------------------------------------------------------------------------------------------
def cable_reward(cable_xpos, end_xpos, pole1, pole2, out=None):
    n, nc, _ = cable_xpos.shape
    _chk(cable_xpos, torch.float64, (n, nc, 3), "cable_xpos")
    for t, nm in ((end_xpos, "end_xpos"), (pole1, "pole1"), (pole2, "pole2")):
        _chk(t, torch.float64, (n, 3), nm)
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=cable_xpos.device)
    _chk(out, torch.float64, (n,), "reward")
    N.call("rmbx_cable_reward", N.ptr(cable_xpos), N.ptr(end_xpos), N.ptr(pole1), N.ptr(pole2),
           N.ptr(out), n, nc, N.stream_ptr())
    return out


def ring_reward(ring_xpos, pole_xpos, out=None):
    """MujocoUR5eRingEnv._get_reward for n envs (rmbx_ring_reward); ring_xpos [n, 11, 3] f64."""
    n, nr, _ = ring_xpos.shape
    _chk(ring_xpos, torch.float64, (n, nr, 3), "ring_xpos")
    _chk(pole_xpos, torch.float64, (n, 3), "pole_xpos")
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=ring_xpos.device)
    _chk(out, torch.float64, (n,), "reward")
    N.call("rmbx_ring_reward", N.ptr(ring_xpos), N.ptr(pole_xpos), N.ptr(out), n, nr, N.stream_ptr())
    return out


def toolbox_reward(toolbox_xpos, mat_xpos, xy_thre, z_offset, out=None):
    """MujocoUR5eToolboxEnv._get_reward for n envs (rmbx_toolbox_reward)."""
    n = toolbox_xpos.shape[0]
    _chk(toolbox_xpos, torch.float64, (n, 3), "toolbox_xpos")
    _chk(mat_xpos, torch.float64, (n, 3), "mat_xpos")
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=toolbox_xpos.device)
    _chk(out, torch.float64, (n,), "reward")
    N.call("rmbx_toolbox_reward", N.ptr(toolbox_xpos), N.ptr(mat_xpos), N.ptr(out), n, float(xy_thre),
           float(z_offset), N.stream_ptr())
    return out


CABINET_TASKS = {None: 0, "hinge": 1, "slide": 2}


def cabinet_reward(qpos, hinge_adr, slide_adr, hinge_thre, slide_thre, target_task=None, out=None):
    """MujocoUR5eCabinetEnv._get_reward for n envs (rmbx_cabinet_reward); qpos [n, nq] f64."""
    if target_task not in CABINET_TASKS:
        raise ValueError(f"[MujocoUR5eCabinetEnv] Invalid target task: {target_task}")
    n, nq = qpos.shape
    _chk(qpos, torch.float64, (n, nq), "qpos")
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=qpos.device)
    _chk(out, torch.float64, (n,), "reward")
    N.call("rmbx_cabinet_reward", N.ptr(qpos), nq, int(hinge_adr), int(slide_adr), float(hinge_thre),
           float(slide_thre), CABINET_TASKS[target_task], N.ptr(out), n, N.stream_ptr())
    return out


def door_reward(pinch_xpos, handle_xpos, door_angle, margin, target_angle, out=None):
    """MujocoUR5eDoorEnv._get_reward for n envs (rmbx_door_reward)."""
    n = pinch_xpos.shape[0]
    _chk(pinch_xpos, torch.float64, (n, 3), "pinch_xpos")
    _chk(handle_xpos, torch.float64, (n, 3), "handle_xpos")
    _chk(door_angle, torch.float64, (n,), "door_angle")
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=pinch_xpos.device)
    _chk(out, torch.float64, (n,), "reward")
    N.call("rmbx_door_reward", N.ptr(pinch_xpos), N.ptr(handle_xpos), N.ptr(door_angle), N.ptr(out), n,
           float(margin), float(target_angle), N.stream_ptr())
    return out


def insert_reward(peg_xpos, hole_xpos, peg_xquat, xy_thre, z_offset, cos_tilt, out=None):
    """MujocoUR5eInsertEnv._get_reward for n envs (rmbx_insert_reward)."""
    n = peg_xpos.shape[0]
    _chk(peg_xpos, torch.float64, (n, 3), "peg_xpos")
    _chk(hole_xpos, torch.float64, (n, 3), "hole_xpos")
    _chk(peg_xquat, torch.float64, (n, 4), "peg_xquat")
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=peg_xpos.device)
    _chk(out, torch.float64, (n,), "reward")
    N.call("rmbx_insert_reward", N.ptr(peg_xpos), N.ptr(hole_xpos), N.ptr(peg_xquat), N.ptr(out), n,
           float(xy_thre), float(z_offset), float(cos_tilt), N.stream_ptr())
    return out


def ur5e_obs(arm_qpos, arm_qvel, grip_qpos, force, torque):
    n = arm_qpos.shape[0]
    _chk(arm_qpos, torch.float64, (n, 6), "arm_qpos")
    _chk(arm_qvel, torch.float64, (n, 6), "arm_qvel")
    _chk(grip_qpos, torch.float64, (n, 4), "grip_qpos")
    _chk(force, torch.float64, (n, 3), "force")
    _chk(torque, torch.float64, (n, 3), "torque")
    dev = arm_qpos.device
    jp = torch.empty((n, 7), dtype=torch.float64, device=dev)
    jv = torch.empty((n, 7), dtype=torch.float64, device=dev)
    wr = torch.empty((n, 6), dtype=torch.float64, device=dev)
    N.call("rmbx_ur5e_obs", N.ptr(arm_qpos), N.ptr(arm_qvel), N.ptr(grip_qpos), N.ptr(force),
           N.ptr(torque), N.ptr(jp), N.ptr(jv), N.ptr(wr), n, N.stream_ptr())
    return jp, jv, wr


# ------------------------------------------------------------------------------------------
# DataKey routing (MotionManager / ArmManager on the device)
# ------------------------------------------------------------------------------------------
def _key_array(codes):
    return np.ascontiguousarray(np.asarray(codes, dtype=np.int32).reshape(-1))


def motion_state(placement, obs, q_cmd, grip_cmd, tgt_R, tgt_p, codes, dim, out=None):
    """Raw f64 state [n, dim] of the state keys (rmbx_motion_state)."""
    jp = obs["joint_pos"]
    n = jp.shape[0]
    _chk(placement, torch.float64, (6, 12), "placement")
    _chk(jp, torch.float64, (n, 7), "joint_pos")
    _chk(obs["joint_vel"], torch.float64, (n, 7), "joint_vel")
    _chk(obs["wrench"], torch.float64, (n, 6), "wrench")
    _chk(q_cmd, torch.float64, (n, 6), "q_cmd")
    _chk(grip_cmd, torch.float64, (n, 1), "grip_cmd")
    _chk(tgt_R, torch.float64, (n, 9), "target_R")
    _chk(tgt_p, torch.float64, (n, 3), "target_p")
    if out is None:
        out = torch.empty((n, dim), dtype=torch.float64, device=jp.device)
    _chk(out, torch.float64, (n, dim), "state")
    keys = _key_array(codes)
    N.call("rmbx_motion_state", N.ptr(placement), N.ptr(jp), N.ptr(obs["joint_vel"]), N.ptr(obs["wrench"]),
           N.ptr(q_cmd), N.ptr(grip_cmd), N.ptr(tgt_R), N.ptr(tgt_p), N.ptr(keys), len(keys), N.ptr(out), dim, n,
           N.stream_ptr())
    return out


def motion_command(placement, action, codes, is_skip, grip_low, grip_high, q_cmd, grip_cmd, tgt_R, tgt_p,
                   mask=None):
    """Apply the policy action to the command state in place (rmbx_motion_command)."""
    n = q_cmd.shape[0]
    _chk(placement, torch.float64, (6, 12), "placement")
    _chk(action, torch.float64, None, "action")
    if action.dim() != 2 or action.shape[0] != n:
        raise ValueError(f"action must be [{n}, action_dim] (got {tuple(action.shape)})")
    _chk(q_cmd, torch.float64, (n, 6), "q_cmd")
    _chk(grip_cmd, torch.float64, (n, 1), "grip_cmd")
    _chk(tgt_R, torch.float64, (n, 9), "target_R")
    _chk(tgt_p, torch.float64, (n, 3), "target_p")
    if mask is not None:
        _chk(mask, torch.uint8, (n,), "mask")
    keys = _key_array(codes)
    N.call("rmbx_motion_command", N.ptr(placement), N.ptr(action), action.shape[1], N.ptr(keys), len(keys),
           int(bool(is_skip)), float(grip_low), float(grip_high), N.ptr(q_cmd), N.ptr(grip_cmd), N.ptr(tgt_R),
           N.ptr(tgt_p), N.ptr(mask), n, N.stream_ptr())


def depth_linearize(zbuf, near, far, out=None):
    _chk(zbuf, torch.float32, None, "zbuf")
    if out is None:
        out = torch.empty_like(zbuf)
    _chk(out, torch.float32, tuple(zbuf.shape), "depth")
    N.call("rmbx_depth_linearize", N.ptr(zbuf), N.ptr(out), zbuf.numel(), float(near), float(far),
           N.stream_ptr())
    return out


# ------------------------------------------------------------------------------------------
# Phase schedule
# ------------------------------------------------------------------------------------------
def sched_alloc(n_env, device):
    return torch.zeros((n_env, N.SCHED_DTYPE.itemsize), dtype=torch.uint8, device=device)


def sched_view(sched_u8):
    """Host numpy structured view of a sched buffer (copies to host)."""
    return sched_u8.cpu().numpy().view(N.SCHED_DTYPE).reshape(-1)


def sched_reset(sched, time, mask=None):
    n = sched.shape[0]
    _chk(sched, torch.uint8, (n, N.SCHED_DTYPE.itemsize), "sched")
    _chk(time, torch.float64, (n,), "time")
    if mask is not None:
        _chk(mask, torch.uint8, (n,), "mask")
    N.call("rmbx_sched_reset", N.ptr(sched), N.ptr(time), N.ptr(mask), n, N.stream_ptr())


def sched_update(sched, time, reward, pre_durations, max_duration, post_success=1.0):
    n = sched.shape[0]
    _chk(sched, torch.uint8, (n, N.SCHED_DTYPE.itemsize), "sched")
    _chk(time, torch.float64, (n,), "time")
    _chk(reward, torch.float64, (n,), "reward")
    _chk(pre_durations, torch.float64, None, "pre_durations")
    N.call("rmbx_sched_update", N.ptr(sched), N.ptr(time), N.ptr(reward), N.ptr(pre_durations),
           pre_durations.numel(), float(max_duration), float(post_success), n, N.stream_ptr())


def sched_active(sched, n_pre, out=None):
    """uint8 [n] step mask: 1 until the env reaches EndRolloutPhase (rmbx_sched_active)."""
    n = sched.shape[0]
    _chk(sched, torch.uint8, (n, N.SCHED_DTYPE.itemsize), "sched")
    if out is None:
        out = torch.empty(n, dtype=torch.uint8, device=sched.device)
    _chk(out, torch.uint8, (n,), "out")
    N.call("rmbx_sched_active", N.ptr(sched), int(n_pre), N.ptr(out), n, N.stream_ptr())
    return out


# ------------------------------------------------------------------------------------------
# Vision-trunk epilogues (NHWC = torch channels_last)
# ------------------------------------------------------------------------------------------
_NN_DTYPES = {torch.bfloat16: 1, torch.float32: 0}


def _chk_nhwc(t, name):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.dtype not in _NN_DTYPES:
        raise ValueError(f"{name} must be bf16 or f32 (got {t.dtype})")
    if t.dim() != 4 or not t.is_contiguous(memory_format=torch.channels_last):
        raise ValueError(f"{name} must be a 4-D channels_last tensor")
    return t


def nhwc_bias_act(x, bias, res=None, res_bias=None, relu=True, out=None):
    """out = relu?(rnd(rnd(x + bias) + rnd(res + res_bias))) on channels_last [N, C, H, W]
    activations (rmbx_nhwc_bias_act); `bias`/`res_bias` f32 [C]. In place when out is x."""
    _chk_nhwc(x, "x")
    C = x.shape[1]
    _chk(bias, torch.float32, (C,), "bias")
    if res is not None:
        _chk_nhwc(res, "res")
        if res.shape != x.shape or res.dtype != x.dtype:
            raise ValueError("res must match x in shape and dtype")
    if res_bias is not None:
        if res is None:
            raise ValueError("res_bias needs res")
        _chk(res_bias, torch.float32, (C,), "res_bias")
    if out is None:
        out = torch.empty_like(x, memory_format=torch.channels_last)
    _chk_nhwc(out, "out")
    n_pix = x.numel() // C
    N.call("rmbx_nhwc_bias_act", N.ptr(x), N.ptr(bias), N.ptr(res), N.ptr(res_bias), N.ptr(out), n_pix, C,
           int(bool(relu)), _NN_DTYPES[x.dtype], N.stream_ptr())
    return out


def nhwc_bias_relu_maxpool(x, bias):
    """maxpool3x3/2/pad1(relu(rnd(x + bias))) of a channels_last [N, C, H, W] tensor."""
    _chk_nhwc(x, "x")
    n, C, H, W = x.shape
    _chk(bias, torch.float32, (C,), "bias")
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    out = torch.empty((n, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    N.call("rmbx_nhwc_bias_relu_maxpool", N.ptr(x), N.ptr(bias), N.ptr(out), n, H, W, C, _NN_DTYPES[x.dtype],
           N.stream_ptr())
    return out


# ------------------------------------------------------------------------------------------
# Policy-input image preprocessing
# ------------------------------------------------------------------------------------------
def resize_crop_u8(src, size, crop=None, a=1.0, b=0.0, dtype=torch.float32, out=None):
    """src u8 [n, H, W, C] -> [n, C, ch, cw] = cv2.resize(src, size=(rw, rh)) cropped at
    crop = (y0, x0, ch, cw) (None = full), scaled v / 255 * a + b (rmbx_resize_crop_u8)."""
    _chk(src, torch.uint8, name="src")
    if src.dim() != 4:
        raise ValueError("src must be [n, H, W, C]")
    n, H, W, C = src.shape
    rw, rh = int(size[0]), int(size[1])
    y0, x0, ch, cw = crop if crop is not None else (0, 0, rh, rw)
    if dtype == torch.uint8:  # the resized frame itself, [n, ch, cw, C]
        shape, code = (n, ch, cw, C), 2
    elif dtype in _NN_DTYPES:
        shape, code = (n, C, ch, cw), _NN_DTYPES[dtype]
    else:
        raise ValueError("dtype must be f32, bf16 or u8")
    if out is None:
        out = torch.empty(shape, dtype=dtype, device=src.device)
    _chk(out, dtype, shape, "out")
    N.call("rmbx_resize_crop_u8", N.ptr(src), n, H, W, C, rh, rw, y0, x0, ch, cw, float(a), float(b), N.ptr(out),
           code, N.stream_ptr())
    return out


def resize_f32(src, size, out=None):
    """cv2.resize of f32 [n, H, W] images to size = (rw, rh) (rmbx_resize_f32)."""
    _chk(src, torch.float32, name="src")
    n, H, W = src.shape
    rw, rh = int(size[0]), int(size[1])
    if out is None:
        out = torch.empty((n, rh, rw), dtype=torch.float32, device=src.device)
    _chk(out, torch.float32, (n, rh, rw), "out")
    N.call("rmbx_resize_f32", N.ptr(src), N.ptr(out), n, H, W, rh, rw, N.stream_ptr())
    return out


# ------------------------------------------------------------------------------------------
# Point-cloud observation (3D diffusion policy)
# ------------------------------------------------------------------------------------------
def focal_scaling(fovy_deg, height):
    """convert_depth_image_to_pointcloud's focal scaling (VisionUtils.py:59), NumPy f64."""
    return float((1.0 / np.tan(np.deg2rad(fovy_deg) / 2.0)) * height / 2.0)


def pointcloud_norm_coeffs(stats):
    """(norm_type, a, b, c) of normalize_data (DataUtils.py:9-24) for the 6-channel cloud."""
    t = stats["norm_config"]["type"] if "norm_config" in stats else "gaussian"
    if t == "gaussian":
        return 0, np.asarray(stats["mean"], np.float64), np.asarray(stats["std"], np.float64), None
    cfg = stats["norm_config"]
    scale = (cfg["out_max"] - cfg["out_min"]) / np.asarray(stats["range"], np.float64)
    return 1, np.asarray(stats["min"], np.float64), scale, np.full(6, float(cfg["out_min"]))


def pointcloud_fps(depth, rgb, fovy_deg, num_points, stats, min_bound=None, max_bound=None, raw=False):
    """depth f32 [n, H, W] + rgb u8 [n, H, W, 3] -> (normalised f32 [n, K, 6], count i32 [n],
    raw f64 [n, K, 6] or None) via rmbx_pointcloud_fps."""
    _chk(depth, torch.float32, name="depth")
    n, H, W = depth.shape
    _chk(rgb, torch.uint8, (n, H, W, 3), "rgb")
    nt, a, b, c = pointcloud_norm_coeffs(stats)
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    c = None if c is None else np.ascontiguousarray(c, np.float64)
    lo = None if min_bound is None else np.ascontiguousarray(min_bound, np.float64)
    hi = None if max_bound is None else np.ascontiguousarray(max_bound, np.float64)
    out = torch.empty((n, num_points, 6), dtype=torch.float32, device=depth.device)
    r = torch.empty((n, num_points, 6), dtype=torch.float64, device=depth.device) if raw else None
    cnt = torch.empty(n, dtype=torch.int32, device=depth.device)
    N.call("rmbx_pointcloud_fps", N.ptr(depth), N.ptr(rgb), n, H, W, focal_scaling(fovy_deg, H), N.ptr(lo),
           N.ptr(hi), int(num_points), nt, N.ptr(a), N.ptr(b), N.ptr(c), N.ptr(out), N.ptr(r), N.ptr(cnt),
           N.stream_ptr())
    return out, cnt, r


def add_layernorm(x, r, weight, bias, eps=1e-5, out=None):
    """LayerNorm(rnd(x + r)) over the last dim (rmbx_add_layernorm); x, r [..., D] contiguous
    bf16/f32 device tensors (r may be None), weight/bias f32 [D]."""
    if x.dtype not in _NN_DTYPES or not x.is_cuda or not x.is_contiguous():
        raise ValueError("x must be a contiguous bf16/f32 device tensor")
    D = x.shape[-1]
    if r is not None and (r.shape != x.shape or r.dtype != x.dtype or not r.is_contiguous()):
        raise ValueError("r must match x")
    _chk(weight, torch.float32, (D,), "weight")
    _chk(bias, torch.float32, (D,), "bias")
    if out is None:
        out = torch.empty_like(x)
    N.call("rmbx_add_layernorm", N.ptr(x), N.ptr(r), N.ptr(weight), N.ptr(bias), N.ptr(out), x.numel() // D, D,
           float(eps), _NN_DTYPES[x.dtype], N.stream_ptr())
    return out


def groupnorm_act(x, weight, bias, groups, eps=1e-5, mish=True, out=None, time_major=False):
    """GroupNorm(groups) over x [B, C, T] (contiguous f32 device tensor) with the affine, then Mish
    (rmbx_groupnorm_act): the UNet Conv1dBlock's norm + activation in one pass.  time_major: x is
    [B, T, C] (the conv GEMM's rows) and the result [B, C, T] (the transpose folded into the pass)."""
    if x.dtype != torch.float32 or not x.is_cuda or not x.is_contiguous() or x.dim() != 3:
        raise ValueError("x must be a contiguous f32 device tensor [B, C, T]")
    if time_major:
        B, T, C = x.shape
    else:
        B, C, T = x.shape
    if C % groups != 0:
        raise ValueError(f"C={C} is not a multiple of groups={groups}")
    _chk(weight, torch.float32, (C,), "weight")
    _chk(bias, torch.float32, (C,), "bias")
    if out is None:
        out = torch.empty((B, C, T), device=x.device, dtype=x.dtype)
    else:
        _chk(out, torch.float32, (B, C, T), "out")
        if out.device != x.device:
            raise ValueError(f"out must be on {x.device} (got {out.device})")
        if time_major and out.data_ptr() == x.data_ptr():
            raise ValueError("a time-major input cannot be normalised in place")
    N.call("rmbx_groupnorm_act", N.ptr(x), N.ptr(weight), N.ptr(bias), N.ptr(out), B, C, T, int(groups), float(eps),
           (1 if mish else 0) | (2 if time_major else 0), N.stream_ptr())
    return out


def add_layernorm_pos(x, r, weight, bias, pos, eps=1e-5):
    """(y, y + pos) with y = LayerNorm(rnd(x + r)) in one pass (rmbx_add_layernorm_pos); pos
    [P, D] (or [1, P, D]) in x's dtype, broadcast over the leading dims row-wise (row % P)."""
    if x.dtype not in _NN_DTYPES or not x.is_cuda or not x.is_contiguous():
        raise ValueError("x must be a contiguous bf16/f32 device tensor")
    D = x.shape[-1]
    if r is not None and (r.shape != x.shape or r.dtype != x.dtype or not r.is_contiguous()):
        raise ValueError("r must match x")
    _chk(weight, torch.float32, (D,), "weight")
    _chk(bias, torch.float32, (D,), "bias")
    pos2 = pos.reshape(-1, D)
    if pos2.dtype != x.dtype or not pos2.is_contiguous() or not pos2.is_cuda:
        raise ValueError("pos must be a contiguous device tensor of x's dtype")
    if x.dim() < 2 or x.shape[-2] % pos2.shape[0] != 0:
        raise ValueError("pos rows must divide the sequence length")
    out = torch.empty_like(x)
    out_pos = torch.empty_like(x)
    N.call("rmbx_add_layernorm_pos", N.ptr(x), N.ptr(r), N.ptr(weight), N.ptr(bias), N.ptr(out), N.ptr(pos2),
           pos2.shape[0], N.ptr(out_pos), x.numel() // D, D, float(eps), _NN_DTYPES[x.dtype], N.stream_ptr())
    return out, out_pos


class PresplitRows:
    """An f32 activation [M, K] in the pre-split A form of rmbx_linear_f16x3_presplit (written by
    rmbx_add_layernorm_split or rmbx_linear_f16x3_presplit_split): planes [2, M, K] f16, a[m] =
    rinv[m] * (planes[0, m] + planes[1, m]) to 2^-22 relative, rinv [M] f32 powers of two; norm [M]
    (optional) an upper bound of each row's |a|_2."""

    __slots__ = ("planes", "rinv", "norm", "_src")

    def __init__(self, planes, rinv, norm=None):
        self.planes, self.rinv, self.norm = planes, rinv, norm
        self._src = None

    def bind(self, t):
        """Record the f32 tensor these pieces were written beside (its storage and version)."""
        self._src = (t.data_ptr(), t._version)

    def valid_for(self, t):
        """True while `t` is that tensor (or a view of it) unchanged since the pieces were written: an
        in-place change of the f32 rows bumps the version and retires the pieces."""
        return self._src is not None and self._src == (t.data_ptr(), t._version)


def presplit_of(x):
    """The pre-split A form attached to x by its producer, if it still describes x's values."""
    sp = getattr(x, "rmbx_split", None)
    return sp if sp is not None and sp.valid_for(x) else None


# the pre-split A path (env RMBX_GEMM_PRESPLIT=0 turns it off: the LayerNorms then emit f32 only and
# every GEMM splits its A in registers)
GEMM_PRESPLIT = os.environ.get("RMBX_GEMM_PRESPLIT", "1") != "0"


def add_layernorm_split(x, r, weight, bias, eps=1e-5, pos=None, split_y=True, split_pos=True, y_norm=False):
    """add_layernorm(_pos) of f32 rows that also attaches the pre-split A form to its outputs:
    returns y (and y + pos when pos is given), each an f32 tensor carrying `.rmbx_split`
    (PresplitRows) when requested -- the form linear_f32x6 then reads (rmbx_add_layernorm_split)."""
    if x.dtype != torch.float32 or not x.is_cuda or not x.is_contiguous():
        raise ValueError("x must be a contiguous f32 device tensor")
    D = x.shape[-1]
    if r is not None and (r.shape != x.shape or r.dtype != x.dtype or not r.is_contiguous()):
        raise ValueError("r must match x")
    _chk(weight, torch.float32, (D,), "weight")
    _chk(bias, torch.float32, (D,), "bias")
    rows = x.numel() // D
    y = torch.empty_like(x)
    ys = PresplitRows(torch.empty((2, rows, D), dtype=torch.float16, device=x.device),
                      torch.empty(rows, dtype=torch.float32, device=x.device),
                      torch.empty(rows, dtype=torch.float32, device=x.device) if y_norm else None) if split_y else None
    yp = ps = pos2 = None
    if pos is not None:
        pos2 = pos.reshape(-1, D)
        if pos2.dtype != x.dtype or not pos2.is_contiguous() or not pos2.is_cuda:
            raise ValueError("pos must be a contiguous device tensor of x's dtype")
        if x.dim() < 2 or x.shape[-2] % pos2.shape[0] != 0:
            raise ValueError("pos rows must divide the sequence length")
        yp = torch.empty_like(x)
        if split_pos:
            ps = PresplitRows(torch.empty((2, rows, D), dtype=torch.float16, device=x.device),
                              torch.empty(rows, dtype=torch.float32, device=x.device))
    N.call("rmbx_add_layernorm_split", N.ptr(x), N.ptr(r), N.ptr(weight), N.ptr(bias), N.ptr(y),
           N.ptr(ys.planes if ys else None), N.ptr(ys.rinv if ys else None), N.ptr(ys.norm if ys else None), N.ptr(pos2),
           pos2.shape[0] if pos2 is not None else 0, N.ptr(yp), N.ptr(ps.planes if ps else None),
           N.ptr(ps.rinv if ps else None), rows, D, float(eps), N.stream_ptr())
    if ys is not None:
        ys.bind(y)
        y.rmbx_split = ys
    if ps is not None:
        ps.bind(yp)
        yp.rmbx_split = ps
    return (y, yp) if pos is not None else y


def weight_bounds(w, b):
    """(max_n |w_n|_2, max |b|) of an f32 weight [N, K] and bias [N], rounded up to f32 upper bounds
    (computed in f64): the output bound of linear_presplit_split."""
    wn = float(w.detach().double().norm(dim=1).max()) if w.numel() else 0.0
    bm = float(b.detach().double().abs().max()) if b is not None and b.numel() else 0.0
    up = 1.0 + 2.0 ** -20
    return wn * up, bm * up


def linear_presplit_split(xs, planes, bias, bounds, relu=False, out=None):
    """relu?(x @ W^T + bias) from pre-split rows xs (PresplitRows with norm bounds) to pre-split rows
    (rmbx_linear_f16x3_presplit_split): the FFN's first Linear, whose output only feeds the second.
    bounds = weight_bounds(W, bias); out (optional): the PresplitRows to write ([2, M, N] planes and
    [M] rinv, row-slice views allowed)."""
    Nn, K, h3 = _planes_nk(planes, "linear_presplit_split")
    if not h3 or xs.norm is None or xs.planes.shape[2] != K:
        raise ValueError("linear_presplit_split: f16x3 planes and pre-split rows with norm bounds of width K")
    M = xs.planes.shape[1]
    if bias is not None:
        _chk(bias, torch.float32, (Nn,), "bias")
    if out is None:
        out = PresplitRows(torch.empty((2, M, Nn), dtype=torch.float16, device=xs.planes.device),
                           torch.empty(M, dtype=torch.float32, device=xs.planes.device))
    elif (tuple(out.planes.shape) != (2, M, Nn) or out.planes.dtype != torch.float16 or out.planes.stride(2) != 1
          or tuple(out.rinv.shape) != (M,) or out.rinv.dtype != torch.float32 or not out.rinv.is_contiguous()):
        raise ValueError("linear_presplit_split: out must hold [2, M, N] f16 planes (unit column stride) and [M] f32 rinv")
    p, ap, op = planes.planes, xs.planes, out.planes
    _gemm_launch(f"linear M={M} N={Nn} K={K} presplit->split", 2.0 * M * Nn * K, 4 * M * K + 4 * Nn * K + 4 * M * Nn, 3,
                 "rmbx_linear_f16x3_presplit_split", N.ptr(ap), ap.stride(1), ap.stride(0), N.ptr(xs.rinv),
                 N.ptr(xs.norm), N.ptr(p), p.stride(1), p.stride(0), N.ptr(planes.scale), float(bounds[0]),
                 float(bounds[1]), N.ptr(bias), 1 if relu else 0, N.ptr(op), op.stride(1), op.stride(0),
                 N.ptr(out.rinv), M, Nn, K, N.stream_ptr())
    return out


def linear_presplit(xs, planes, bias=None, relu=False, out=None):
    """relu?(x @ W^T + bias) f32 [M, N] from pre-split rows xs (rmbx_linear_f16x3_presplit); out
    (optional): the f32 [M, N] rows to write (unit column stride)."""
    Nn, K, h3 = _planes_nk(planes, "linear_presplit")
    if not h3 or xs.planes.shape[2] != K or Nn % LINEAR_F32X6_BN != 0:
        raise ValueError("linear_presplit: f16x3 planes, N % 128 == 0 and pre-split rows of width K")
    M = xs.planes.shape[1]
    if bias is not None:
        _chk(bias, torch.float32, (Nn,), "bias")
    if out is None:
        out = torch.empty((M, Nn), dtype=torch.float32, device=xs.planes.device)
    elif tuple(out.shape) != (M, Nn) or out.dtype != torch.float32 or out.stride(1) != 1:
        raise ValueError("linear_presplit: out must be f32 [M, N] with unit column stride")
    p, ap = planes.planes, xs.planes
    _gemm_launch(f"linear M={M} N={Nn} K={K} presplit", 2.0 * M * Nn * K, 4 * M * K + 4 * Nn * K + 4 * M * Nn, 3,
                 "rmbx_linear_f16x3_presplit", N.ptr(ap), ap.stride(1), ap.stride(0), N.ptr(xs.rinv), N.ptr(p),
                 p.stride(1), p.stride(0), N.ptr(planes.scale), N.ptr(bias), None, N.ptr(out), out.stride(0), M, Nn, K,
                 1 if relu else 0, N.stream_ptr())
    return out


def conv2d_nhwc(x, weight, bias, stride=1, padding=0, relu=False, res=None):
    """relu?(conv2d(x, weight) + bias + res) by rmbx_conv2d_nhwc (bf16) / rmbx_conv2d_nhwc_f32
    (f32: the 3x3 / stride-1 / pad-1 conv with Cin = Cout = 64 only): x channels_last
    [N, Cin, H, W], weight channels_last [Cout, Cin, KH, KW] of the same dtype, bias f32 [Cout],
    res channels_last [N, Cout, Ho, Wo] or None -> channels_last [N, Cout, Ho, Wo]."""
    _chk_nhwc(x, "x")
    dt = x.dtype
    if dt not in (torch.bfloat16, torch.float32) or weight.dtype != dt:
        raise ValueError("conv2d_nhwc: x and weight must both be bf16 or both f32")
    if weight.dim() != 4 or not weight.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("weight must be a channels_last [Cout, Cin, KH, KW] tensor")
    n, cin, H, W = x.shape
    cout, cin_w, kh, kw = weight.shape
    if cin_w != cin:
        raise ValueError("weight/input channel mismatch")
    _chk(bias, torch.float32, (cout,), "bias")
    ho = (H + 2 * padding - kh) // stride + 1
    wo = (W + 2 * padding - kw) // stride + 1
    out = torch.empty((n, cout, ho, wo), dtype=dt, device=x.device, memory_format=torch.channels_last)
    if res is not None:
        _chk_nhwc(res, "res")
        if tuple(res.shape) != tuple(out.shape) or res.dtype != dt:
            raise ValueError("res must match the output")
    fn = "rmbx_conv2d_nhwc" if dt == torch.bfloat16 else "rmbx_conv2d_nhwc_f32"
    N.call(fn, N.ptr(x), N.ptr(weight), N.ptr(bias), N.ptr(res), N.ptr(out), n, H, W, cin, cout,
           kh, kw, int(stride), int(padding), int(bool(relu)), N.stream_ptr())
    return out


def conv2d_nhwc_f32_supported(cin, cout, kernel_size, stride, padding):
    """Whether rmbx_conv2d_nhwc_f32 implements this conv (ResNet-18 layer 1)."""
    return (cin, cout, tuple(kernel_size), stride, padding) == (64, 64, (3, 3), 1, 1)


_WINO_G = ((1.0, 0.0, 0.0), (0.5, 0.5, 0.5), (0.5, -0.5, 0.5), (0.0, 0.0, 1.0))
WINOGRAD_F32_CHANNELS = (64, 128, 256, 512)
WINOGRAD_MAX_ELEMS = (1 << 31) - 1  # per launch (32-bit element offsets in the kernel)
WINOGRAD4_MAX_ELEMS = (1 << 30) - 1024  # per launch (32-bit byte offsets + the buffer range of the F(4x4) loads)


def pack_winograd_f32(weight):
    """3x3 conv weight [C, C, 3, 3] -> the Winograd F(2x2, 3x3) filter transform U = G g G^T
    (computed in f64, rounded once to f32) in the LDS image rmbx_conv3x3_winograd_f32 stages per
    K chunk: [C/64 channel blocks][C/8 chunks][16 positions][64 output channels][8 input channels]."""
    C = weight.shape[0]
    if tuple(weight.shape) != (C, C, 3, 3) or C not in WINOGRAD_F32_CHANNELS:
        raise ValueError(f"pack_winograd_f32: weight {tuple(weight.shape)} is not [C, C, 3, 3] with C in {WINOGRAD_F32_CHANNELS}")
    w = weight.detach().to(torch.float64)
    G = torch.tensor(_WINO_G, dtype=torch.float64, device=w.device)
    U = torch.einsum("xa,oiab,yb->xyoi", G, w, G).reshape(16, C // 64, 64, C // 8, 8)  # [p][cb][co][k][c]
    return U.permute(1, 3, 0, 2, 4).contiguous().to(torch.float32)


def conv3x3_winograd_f32(x, u_packed, bias, relu=False, res=None):
    """relu?(conv2d(x, w, stride 1, pad 1) + bias + res) by rmbx_conv3x3_winograd_f32 (Winograd
    F(2x2, 3x3) on f32 MFMA): x channels_last f32 [N, C, H, W], u_packed = pack_winograd_f32(w),
    bias f32 [C], res channels_last [N, C, H, W] or None -> channels_last [N, C, H, W]."""
    _chk_nhwc(x, "x")
    n, C, H, W = x.shape
    if x.dtype != torch.float32 or C not in WINOGRAD_F32_CHANNELS:
        raise ValueError(f"conv3x3_winograd_f32: x must be f32 with C in {WINOGRAD_F32_CHANNELS}")
    _chk(u_packed, torch.float32, (C // 64, C // 8, 16, 64, 8), "u_packed")
    _chk(bias, torch.float32, (C,), "bias")
    if res is not None:
        _chk_nhwc(res, "res")
        if tuple(res.shape) != tuple(x.shape) or res.dtype != torch.float32:
            raise ValueError("res must match the output")
    out = torch.empty_like(x, memory_format=torch.channels_last)
    # the kernel indexes with 32-bit element offsets: larger batches run as slices of whole images
    per = max(1, WINOGRAD_MAX_ELEMS // (H * W * C))
    for i0 in range(0, n, per):
        i1 = min(n, i0 + per)
        xs, os_ = x[i0:i1], out[i0:i1]
        rs = None if res is None else res[i0:i1]
        N.call("rmbx_conv3x3_winograd_f32", N.ptr(xs), N.ptr(u_packed), N.ptr(bias), N.ptr(rs), N.ptr(os_),
               i1 - i0, H, W, C, int(bool(relu)), N.stream_ptr())
    return out


_WINO4_G = ((0.25, 0.0, 0.0), (-1 / 6, -1 / 6, -1 / 6), (-1 / 6, 1 / 6, -1 / 6), (1 / 24, 1 / 12, 1 / 6),
            (1 / 24, -1 / 12, 1 / 6), (0.0, 0.0, 1.0))


def pack_winograd4_f32(weight):
    """3x3 conv weight [C, C, 3, 3] -> the Winograd F(4x4, 3x3) filter transform U = G g G^T
    (computed in f64 on the host, rounded once to f32) in the LDS image rmbx_conv3x3_winograd4_f32
    stages per K chunk: [C/64 channel blocks][C/4 chunks][36 positions][64 output channels][4 input
    channels]."""
    C = weight.shape[0]
    if tuple(weight.shape) != (C, C, 3, 3) or C not in WINOGRAD_F32_CHANNELS:
        raise ValueError(f"pack_winograd4_f32: weight {tuple(weight.shape)} is not [C, C, 3, 3] with C in {WINOGRAD_F32_CHANNELS}")
    w = weight.detach().to("cpu", torch.float64)
    G = torch.tensor(_WINO4_G, dtype=torch.float64)
    U = torch.einsum("xa,oiab,yb->xyoi", G, w, G).reshape(36, C // 64, 64, C // 4, 4)  # [p][cb][co][kc][k]
    return U.permute(1, 3, 0, 2, 4).to(torch.float32).to(weight.device).contiguous()


def conv3x3_winograd4_f32(x, u_packed, bias, relu=False, res=None):
    """relu?(conv2d(x, w, stride 1, pad 1) + bias + res) by rmbx_conv3x3_winograd4_f32 (Winograd
    F(4x4, 3x3) on f32 MFMA): as conv3x3_winograd_f32 with u_packed = pack_winograd4_f32(w)."""
    _chk_nhwc(x, "x")
    n, C, H, W = x.shape
    if x.dtype != torch.float32 or C not in WINOGRAD_F32_CHANNELS:
        raise ValueError(f"conv3x3_winograd4_f32: x must be f32 with C in {WINOGRAD_F32_CHANNELS}")
    _chk(u_packed, torch.float32, (C // 64, C // 4, 36, 64, 4), "u_packed")
    _chk(bias, torch.float32, (C,), "bias")
    if res is not None:
        _chk_nhwc(res, "res")
        if tuple(res.shape) != tuple(x.shape) or res.dtype != torch.float32:
            raise ValueError("res must match the output")
    out = torch.empty_like(x, memory_format=torch.channels_last)
    # the kernel addresses the input with 32-bit byte offsets (buffer loads): slices of whole images
    per = max(1, WINOGRAD4_MAX_ELEMS // (H * W * C))
    for i0 in range(0, n, per):
        i1 = min(n, i0 + per)
        xs, os_ = x[i0:i1], out[i0:i1]
        rs = None if res is None else res[i0:i1]
        N.call("rmbx_conv3x3_winograd4_f32", N.ptr(xs), N.ptr(u_packed), N.ptr(bias), N.ptr(rs), N.ptr(os_),
               i1 - i0, H, W, C, int(bool(relu)), N.stream_ptr())
    return out


def pack_stem_s2d(weight):
    """conv1 weight [Cout, 3, 7, 7] -> [Cout, 4, 4, 16] for rmbx_stem_s2d_conv:
    W'[co][ky][kx][(dy*2+dx)*3+c] = W[co][c][2ky+dy-1][2kx+dx-1] (0 outside the 7x7 window)."""
    cout = weight.shape[0]
    w = torch.zeros((cout, 4, 4, 16), dtype=weight.dtype, device=weight.device)
    for ky in range(4):
        for dy in range(2):
            kh = 2 * ky + dy - 1
            if not 0 <= kh < 7:
                continue
            for kx in range(4):
                for dx in range(2):
                    kw = 2 * kx + dx - 1
                    if not 0 <= kw < 7:
                        continue
                    ch = (dy * 2 + dx) * 3
                    w[:, ky, kx, ch:ch + 3] = weight[:, :, kh, kw]
    return w.contiguous()


def image_to_s2d(img):
    """[n, 3, H, W] -> [n, H/2, W/2, 16] space-to-depth layout of rmbx_render policy_dtype 2."""
    n, c, H, W = img.shape
    x = img.reshape(n, c, H // 2, 2, W // 2, 2).permute(0, 2, 4, 3, 5, 1).reshape(n, H // 2, W // 2, 12)
    return torch.cat([x, x.new_zeros(n, H // 2, W // 2, 4)], dim=-1).contiguous()


def stem_s2d_conv(x_s2d, w_packed, bias, relu=True):
    """relu?(conv1(x) + bias) for the space-to-depth image: [n, Hs, Ws, 16] bf16 ->
    channels_last [n, Cout, Hs, Ws] bf16 (rmbx_stem_s2d_conv)."""
    _chk(x_s2d, torch.bfloat16, name="x_s2d")
    n, Hs, Ws, c16 = x_s2d.shape
    if c16 != 16:
        raise ValueError("x_s2d must be [n, Hs, Ws, 16]")
    cout = w_packed.shape[0]
    _chk(w_packed, torch.bfloat16, (cout, 4, 4, 16), "w_packed")
    _chk(bias, torch.float32, (cout,), "bias")
    out = torch.empty((n, cout, Hs, Ws), dtype=torch.bfloat16, device=x_s2d.device, memory_format=torch.channels_last)
    N.call("rmbx_stem_s2d_conv", N.ptr(x_s2d), N.ptr(w_packed), N.ptr(bias), N.ptr(out), n, Hs, Ws, cout,
           int(bool(relu)), N.stream_ptr())
    return out


STEM_POOL_MAX_WS = 320


def stem_s2d_conv_maxpool(x_s2d, w_packed, bias, band_rows=0):
    """maxpool3x3/2/pad1(relu(conv1(x) + bias)) for the space-to-depth image in one kernel:
    [n, Hs, Ws, 16] bf16 -> channels_last [n, 64, (Hs-1)//2+1, (Ws-1)//2+1] bf16
    (rmbx_stem_s2d_conv_maxpool; bit-identical to stem_s2d_conv + nhwc_bias_relu_maxpool);
    f32 in -> f32 out through rmbx_stem_s2d_conv_maxpool_f32."""
    if x_s2d.dtype == torch.float32:
        return _stem_s2d_conv_maxpool_f32(x_s2d, w_packed, bias, band_rows)
    _chk(x_s2d, torch.bfloat16, name="x_s2d")
    n, Hs, Ws, c16 = x_s2d.shape
    if c16 != 16:
        raise ValueError("x_s2d must be [n, Hs, Ws, 16]")
    if Ws > STEM_POOL_MAX_WS:
        raise ValueError(f"stem_s2d_conv_maxpool: Ws={Ws} exceeds {STEM_POOL_MAX_WS}")
    _chk(w_packed, torch.bfloat16, (64, 4, 4, 16), "w_packed")
    _chk(bias, torch.float32, (64,), "bias")
    Hp, Wp = (Hs - 1) // 2 + 1, (Ws - 1) // 2 + 1
    out = torch.empty((n, 64, Hp, Wp), dtype=torch.bfloat16, device=x_s2d.device, memory_format=torch.channels_last)
    N.call("rmbx_stem_s2d_conv_maxpool", N.ptr(x_s2d), N.ptr(w_packed), N.ptr(bias), N.ptr(out), n, Hs, Ws,
           int(band_rows), N.stream_ptr())
    return out


def _stem_s2d_conv_maxpool_f32(x_s2d, w_packed, bias, band_rows=0):
    _chk(x_s2d, torch.float32, name="x_s2d")
    n, Hs, Ws, c16 = x_s2d.shape
    if c16 != 16:
        raise ValueError("x_s2d must be [n, Hs, Ws, 16]")
    if Ws > STEM_POOL_MAX_WS:
        raise ValueError(f"stem_s2d_conv_maxpool: Ws={Ws} exceeds {STEM_POOL_MAX_WS}")
    _chk(w_packed, torch.float32, (64, 4, 4, 16), "w_packed")
    _chk(bias, torch.float32, (64,), "bias")
    Hp, Wp = (Hs - 1) // 2 + 1, (Ws - 1) // 2 + 1
    out = torch.empty((n, 64, Hp, Wp), dtype=torch.float32, device=x_s2d.device, memory_format=torch.channels_last)
    N.call("rmbx_stem_s2d_conv_maxpool_f32", N.ptr(x_s2d), N.ptr(w_packed), N.ptr(bias), N.ptr(out), n, Hs, Ws,
           int(band_rows), N.stream_ptr())
    return out


# piece form of the u8 stem's weights (env RMBX_STEM_U8_PIECES): "f16" = two f16 pieces of the
# power-of-two-scaled bank on the f16 matrix cores (rmbx_stem_s2d_conv_maxpool_u8h, 2 MFMAs per
# tap), "bf16" = three exact bf16 pieces (rmbx_stem_s2d_conv_maxpool_u8, 3 MFMAs per tap)
STEM_U8_PIECES = os.environ.get("RMBX_STEM_U8_PIECES", "f16")


def pack_stem_u8(weight, bias, mean, std, pieces=None):
    """Operands of the u8 stem for the folded stem conv (weight [64, 3, 7, 7], bias [64]) and the
    image normalisation x = (u / 255 - mean) / std = W'(u - 128) + c' (the kernel reads the
    centred pixels u - 128): (planes, bias_eff, edge, wscale) with planes the pieces of
    W / (255 std) (packed as pack_stem_s2d) -- "bf16": three exact bf16 pieces [3, 64, 16, 16],
    wscale 1; "f16": two f16 pieces [2, 64, 16, 16] of the bank times 2^s (max in [2^13, 2^14),
    hi = f16(x), lo = f16(x - hi), x represented to 2^-22) and wscale = 2^-s -- bias_eff = bias +
    sum W c' over every tap with c' = (128 / 255 - mean) / std, and the edge table [16, 16, 64]
    removing the c' term of the taps that fall outside the image (row mask of ky x column mask of
    kx).  Constants summed in f64."""
    pieces = STEM_U8_PIECES if pieces is None else pieces
    if pieces not in ("f16", "bf16"):
        raise ValueError(f"pack_stem_u8: pieces must be f16 or bf16, not {pieces!r}")
    dev = weight.device
    wp = pack_stem_s2d(weight.detach().double())  # [64, 4, 4, 16]
    mean = torch.tensor(mean, dtype=torch.float64, device=dev)
    std = torch.tensor(std, dtype=torch.float64, device=dev)
    ch = torch.arange(16, device=dev)
    valid = ch < 12
    inv = torch.where(valid, 1.0 / (255.0 * std[ch % 3]), torch.zeros((), dtype=torch.float64, device=dev))
    # -c' per channel: the constant of the centred pixels, negated (g below is subtracted)
    ms = torch.where(valid, mean[ch % 3] / std[ch % 3] - 128.0 / (255.0 * std[ch % 3]),
                     torch.zeros((), dtype=torch.float64, device=dev))
    if pieces == "bf16":
        wq = (wp * inv).float()
        p0 = wq.bfloat16()
        r = wq - p0.float()  # exact in f32
        p1 = r.bfloat16()
        p2 = (r - p1.float()).bfloat16()  # exact: <= 8 significant bits remain
        planes = torch.stack([p0, p1, p2]).reshape(3, 64, 16, 16).contiguous()
        wscale = 1.0
    else:
        wq = wp * inv  # f64
        m = float(wq.abs().max())
        e = int(np.frexp(m)[1]) if m > 0 else 14
        wq = wq * 2.0 ** (14 - e)  # exact; max in [2^13, 2^14)
        hi = wq.half()
        lo = (wq - hi.double()).half()
        planes = torch.stack([hi, lo]).reshape(2, 64, 16, 16).contiguous()
        wscale = 2.0 ** (e - 14)
    g = (wp * ms).sum(-1)  # [64, 4, 4] mean term per tap
    bias_eff = (bias.detach().double() - g.sum((1, 2))).float().contiguous()
    bits = torch.arange(16, device=dev)
    k4 = torch.arange(4, device=dev)
    out_k = ((bits[:, None] >> k4[None, :]) & 1).bool()  # [mask, k]
    sel = (out_k[:, None, :, None] | out_k[None, :, None, :]).double()  # [rm, cm, ky, kx]
    edge = torch.einsum("abyx,cyx->abc", sel, g).float().contiguous()
    return planes, bias_eff, edge, wscale


def s2d_u8_normalize(x_u8, mean, std):
    """The renderer's f32 space-to-depth policy image (policy_dtype 3) from its 8-bit form
    (policy_dtype 4): ((u / 255) - mean[c]) / std[c] in f32 per channel (dy*2+dx)*3+c, pad 0."""
    dev = x_u8.device
    ch = torch.arange(16, device=dev)
    m = torch.tensor(mean, dtype=torch.float32, device=dev)[ch % 3]
    sd = torch.tensor(std, dtype=torch.float32, device=dev)[ch % 3]
    x = (x_u8.float() / 255.0 - m) / sd
    return torch.where(ch < 12, x, torch.zeros((), device=dev)).contiguous()


def stem_s2d_conv_maxpool_u8(x_u8, planes, bias_eff, edge, wscale=1.0, band_rows=0):
    """maxpool3x3/2/pad1(relu(conv1(x) + bias)) for x = (u / 255 - mean) / std on the 8-bit
    space-to-depth image [n, Hs, Ws, 16] u8 (rmbx_render policy_dtype 4) -> channels_last
    [n, 64, Hp, Wp] f32 (rmbx_stem_s2d_conv_maxpool_u8h for f16 planes, rmbx_stem_s2d_conv_maxpool_u8
    for bf16 ones; operands from pack_stem_u8)."""
    _chk(x_u8, torch.uint8, name="x_u8")
    n, Hs, Ws, c16 = x_u8.shape
    if c16 != 16:
        raise ValueError("x_u8 must be [n, Hs, Ws, 16]")
    if Ws > STEM_POOL_MAX_WS:
        raise ValueError(f"stem_s2d_conv_maxpool_u8: Ws={Ws} exceeds {STEM_POOL_MAX_WS}")
    h2 = isinstance(planes, torch.Tensor) and planes.dtype == torch.float16
    if h2:
        _chk(planes, torch.float16, (2, 64, 16, 16), "planes")
    else:
        _chk(planes, torch.bfloat16, (3, 64, 16, 16), "planes")
    _chk(bias_eff, torch.float32, (64,), "bias_eff")
    _chk(edge, torch.float32, (16, 16, 64), "edge")
    Hp, Wp = (Hs - 1) // 2 + 1, (Ws - 1) // 2 + 1
    out = torch.empty((n, 64, Hp, Wp), dtype=torch.float32, device=x_u8.device, memory_format=torch.channels_last)
    if h2:
        N.call("rmbx_stem_s2d_conv_maxpool_u8h", N.ptr(x_u8), N.ptr(planes), float(wscale), N.ptr(bias_eff),
               N.ptr(edge), N.ptr(out), n, Hs, Ws, int(band_rows), N.stream_ptr())
    else:
        if wscale != 1.0:
            raise ValueError("stem_s2d_conv_maxpool_u8: bf16 planes take wscale 1")
        N.call("rmbx_stem_s2d_conv_maxpool_u8", N.ptr(x_u8), N.ptr(planes), N.ptr(bias_eff), N.ptr(edge), N.ptr(out),
               n, Hs, Ws, int(band_rows), N.stream_ptr())
    return out


# ------------------------------------------------------------------------------------------
# Transformer attention
# ------------------------------------------------------------------------------------------
ATTN_MAX_LK = 320


def attention_bf16(q, k, v, heads, scale=None):
    """softmax(scale * q k^T) v per head for bf16 [B, L, heads * 64] views (last dim contiguous,
    any row/batch strides, e.g. slices of a fused QKV projection) -> contiguous [B, Lq, heads * 64]
    (rmbx_attention_bf16; f32 softmax)."""
    for t, nm in ((q, "q"), (k, "k"), (v, "v")):
        if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.bfloat16 or t.dim() != 3:
            raise ValueError(f"{nm} must be a bf16 [B, L, D] device tensor")
        if t.stride(2) != 1 or t.shape[2] != heads * 64:
            raise ValueError(f"{nm} must have a contiguous last dim of heads * 64")
    B, Lq, D = q.shape
    Lk = k.shape[1]
    if k.shape != v.shape or k.shape[0] != B:
        raise ValueError("k and v must be [B, Lk, D] like q")
    if Lk > ATTN_MAX_LK:
        raise ValueError(f"attention_bf16: Lk={Lk} exceeds {ATTN_MAX_LK}")
    scale = 1.0 / 8.0 if scale is None else float(scale)
    out = torch.empty((B, Lq, D), dtype=torch.bfloat16, device=q.device)
    N.call("rmbx_attention_bf16", N.ptr(q), N.ptr(k), N.ptr(v), N.ptr(out), B, heads, Lq, Lk,
           q.stride(0), q.stride(1), k.stride(0), k.stride(1), v.stride(0), v.stride(1), scale, N.stream_ptr())
    return out


def attention_f32(q, k, v, heads, scale=None, x6=False, form=None):
    """attention_bf16 in f32: f32 [B, L, heads * 64] views with a contiguous last dim -> contiguous
    [B, Lq, heads * 64].  form "f32" (rmbx_attention_f32: exact f32 MFMA products, f32 online
    softmax), "x6" (rmbx_attention_f32x6: the same products fp32-accurate on the bf16 matrix cores by
    three-piece splits) or "f16x3" (rmbx_attention_f16x3: two f16 pieces, three products, blocks
    outside f16's range re-run as x6); x=True is form "x6"."""
    form = form or ("x6" if x6 else "f32")
    if form not in ("f32", "x6", "f16x3"):
        raise ValueError(f"attention_f32: unknown form {form!r}")
    for t, nm in ((q, "q"), (k, "k"), (v, "v")):
        if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.float32 or t.dim() != 3:
            raise ValueError(f"{nm} must be an f32 [B, L, D] device tensor")
        if t.stride(2) != 1 or t.shape[2] != heads * 64:
            raise ValueError(f"{nm} must have a contiguous last dim of heads * 64")
    B, Lq, D = q.shape
    Lk = k.shape[1]
    if k.shape != v.shape or k.shape[0] != B:
        raise ValueError("k and v must be [B, Lk, D] like q")
    scale = 1.0 / 8.0 if scale is None else float(scale)
    out = torch.empty((B, Lq, D), dtype=torch.float32, device=q.device)
    strides = (q.stride(0), q.stride(1), k.stride(0), k.stride(1), v.stride(0), v.stride(1), scale, N.stream_ptr())
    if form == "f16x3":
        # one re-run flag per block (blocks = B x heads x query parts <= B x heads x 32-query groups)
        redo = torch.empty(max(1, B * heads * ((Lq + 31) // 32)), dtype=torch.int32, device=q.device)
        N.call("rmbx_attention_f16x3", N.ptr(q), N.ptr(k), N.ptr(v), N.ptr(out), N.ptr(redo), B, heads, Lq, Lk,
               *strides)
    else:
        N.call("rmbx_attention_f32x6" if form == "x6" else "rmbx_attention_f32", N.ptr(q), N.ptr(k), N.ptr(v),
               N.ptr(out), B, heads, Lq, Lk, *strides)
    return out


# ------------------------------------------------------------------------------------------
# fp32-accurate linear layers / convolutions on the matrix cores: f16x3 (rmbx_linear_f16x3, the
# default) or bf16x6 (rmbx_linear_f32x6)
# ------------------------------------------------------------------------------------------
LINEAR_F32X6_BN, LINEAR_F32X6_BK = 128, 32

# the piece form pack_f32_weight produces (env RMBX_F32_PIECES): "f16x3" = two f16 pieces per
# operand, three products (half the MFMA work); "bf16x6" = three bf16 pieces, six products
F32_PIECES = os.environ.get("RMBX_F32_PIECES", "f16x3")
if F32_PIECES not in ("f16x3", "bf16x6"):
    raise ValueError(f"RMBX_F32_PIECES must be f16x3 or bf16x6, not {F32_PIECES!r}")

# bench.py's GEMM probe: a list to which every fp32-accurate GEMM / conv launch appends (name,
# fp32-equivalent FLOPs, algorithmic bytes, MFMA products per f32 product, HIP events around it on
# the current stream); None = no events
GEMM_PROBE = None


def _gemm_launch(name, flops, nbytes, products, fn, *args):
    """nbytes: the launch's algorithmic HBM bytes (f32 A in, the W pieces, f32 C out and the
    residual if any)."""
    if GEMM_PROBE is None:
        return N.call(fn, *args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    N.call(fn, *args)
    e1.record()
    GEMM_PROBE.append((name, flops, nbytes, products, e0, e1))


def split_bf16x3(w):
    """The three bf16 pieces of an f32 tensor, w = w0 + w1 + w2 exactly: [3, *w.shape] bf16
    (rmbx_split_bf16x3)."""
    _chk(w, torch.float32, name="w")
    planes = torch.empty((3,) + tuple(w.shape), dtype=torch.bfloat16, device=w.device)
    N.call("rmbx_split_bf16x3", N.ptr(w), N.ptr(planes), w.numel(), N.stream_ptr())
    return planes


class F16x3Planes:
    """An f32 weight [N, K] in the f16x3 form (rmbx_split_f16x2): planes [2, N, K] f16 with
    W[n] = scale[n] * (planes[0, n] + 2^-11 planes[1, n]) to 2^-22 relative, scale [N] f32 powers of
    two.  planes[:, a:b] row slices (the fused MHA's q / k / v rows of in_proj) are supported."""

    __slots__ = ("planes", "scale")

    def __init__(self, planes, scale):
        self.planes, self.scale = planes, scale

    @property
    def shape(self):
        return self.planes.shape

    @property
    def device(self):
        return self.planes.device

    def __getitem__(self, idx):
        if not (isinstance(idx, tuple) and len(idx) == 2 and idx[0] == slice(None) and isinstance(idx[1], slice)):
            raise IndexError("F16x3Planes takes [:, a:b] row slices only")
        return F16x3Planes(self.planes[idx], self.scale[idx[1]])


def split_f16x2(w):
    """w f32 [N, K] -> F16x3Planes (rmbx_split_f16x2: per-row power-of-two scale, f16 hi / lo)."""
    _chk(w, torch.float32, name="w")
    if w.dim() != 2:
        raise ValueError("split_f16x2: w must be [N, K]")
    w = w.contiguous()
    n, k = w.shape
    planes = torch.empty((2, n, k), dtype=torch.float16, device=w.device)
    scale = torch.empty(n, dtype=torch.float32, device=w.device)
    N.call("rmbx_split_f16x2", N.ptr(w), n, k, N.ptr(planes), N.ptr(scale), N.stream_ptr())
    return F16x3Planes(planes, scale)


def pack_f32_weight(w):
    """An f32 weight [N, K] in the piece form of F32_PIECES: F16x3Planes or split_bf16x3 planes,
    the W operand of linear_f32x6 / conv2d_f32x6."""
    return split_f16x2(w) if F32_PIECES == "f16x3" else split_bf16x3(w)


def _planes_nk(planes, what):
    """(N, K, f16x3?) of a packed weight; raises on anything else."""
    if isinstance(planes, F16x3Planes):
        p = planes.planes
        if p.dim() != 3 or p.shape[0] != 2 or p.dtype != torch.float16 or not p.is_cuda or p.stride(2) != 1:
            raise ValueError(f"{what}: bad F16x3Planes")
        return p.shape[1], p.shape[2], True
    if (not isinstance(planes, torch.Tensor) or planes.dim() != 3 or planes.shape[0] != 3
            or planes.dtype != torch.bfloat16 or not planes.is_cuda):
        raise ValueError(f"{what}: planes must be a [3, N, K] bf16 device tensor from split_bf16x3 or F16x3Planes")
    if planes.stride(2) != 1:
        raise ValueError(f"{what}: planes rows must be contiguous")
    return planes.shape[1], planes.shape[2], False


def _n_multiple(h3=None):
    """Output-width granule of the fp32-accurate GEMM: 128, or 64 for the f16x3 form (its narrow
    64-column tile)."""
    return 64 if (F32_PIECES == "f16x3" if h3 is None else h3) else LINEAR_F32X6_BN


def linear_f32x6_supported(x, n_out):
    """Shapes the fp32-accurate GEMM takes: f32 device input whose last dim (K) is a multiple of
    32, N a multiple of 128 (64 in the f16x3 form)."""
    return (x.is_cuda and x.dtype == torch.float32 and x.shape[-1] % LINEAR_F32X6_BK == 0
            and n_out % _n_multiple() == 0)


def linear_f32x6(x, planes, bias=None, relu=False, out=None):
    """relu?(x @ W^T + bias), fp32-accurate, with x f32 [..., K] and W = pack_f32_weight(W) (or a
    row slice planes[:, a:b] of one): F16x3Planes -> rmbx_linear_f16x3, split_bf16x3 planes [3, N, K]
    -> rmbx_linear_f32x6; f32 result [..., N].  x's rows may be strided (last dim contiguous, row
    stride a multiple of 4 elements)."""
    Nn, K, h3 = _planes_nk(planes, "linear_f32x6")
    if x.dtype != torch.float32 or not x.is_cuda or x.shape[-1] != K:
        raise ValueError(f"x must be an f32 device tensor [..., {K}]")
    x2 = x.reshape(-1, K)
    if x2.stride(1) != 1 or x2.stride(0) % 4 != 0 or x2.data_ptr() % 16 != 0:
        x2 = x2.contiguous()
    M = x2.shape[0]
    if bias is not None:
        _chk(bias, torch.float32, (Nn,), "bias")
    if out is None:
        out = torch.empty((M, Nn), dtype=torch.float32, device=x.device)
    elif out.dtype != torch.float32 or out.stride(-1) != 1 or out.shape != (M, Nn):
        raise ValueError("out must be an f32 [M, N] tensor with contiguous rows")
    name, flops = f"linear M={M} N={Nn} K={K}", 2.0 * M * Nn * K
    sp = presplit_of(x)
    if h3 and sp is not None and Nn % LINEAR_F32X6_BN == 0 and sp.planes.shape[1] == M and sp.planes.shape[2] == K:
        # the producer's pre-split rows (add_layernorm_split): both operands by LDS-DMA
        p, ap = planes.planes, sp.planes
        _gemm_launch(name + " presplit", flops, 4 * M * K + 4 * Nn * K + 4 * M * Nn, 3, "rmbx_linear_f16x3_presplit",
                     N.ptr(ap), ap.stride(1), ap.stride(0), N.ptr(sp.rinv), N.ptr(p), p.stride(1), p.stride(0),
                     N.ptr(planes.scale), N.ptr(bias), None, N.ptr(out), out.stride(0), M, Nn, K, 1 if relu else 0,
                     N.stream_ptr())
    elif h3:
        p = planes.planes
        _gemm_launch(name, flops, 4 * M * K + 4 * Nn * K + 4 * M * Nn, 3, "rmbx_linear_f16x3", N.ptr(x2), x2.stride(0),
                     N.ptr(p), p.stride(1), p.stride(0), N.ptr(planes.scale), N.ptr(bias), N.ptr(out), out.stride(0),
                     M, Nn, K, 1 if relu else 0, N.stream_ptr())
    else:
        _gemm_launch(name, flops, 4 * M * K + 6 * Nn * K + 4 * M * Nn, 6, "rmbx_linear_f32x6", N.ptr(x2), x2.stride(0),
                     N.ptr(planes), planes.stride(1), planes.stride(0), N.ptr(bias), N.ptr(out), out.stride(0), M, Nn,
                     K, 1 if relu else 0, N.stream_ptr())
    return out.view(*x.shape[:-1], Nn)


def pack_conv_f32x6(weight):
    """pack_f32_weight of a conv weight [Cout, C, KH, KW] laid out [Cout][KH][KW][C] (the k order of
    the implicit-GEMM conv): F16x3Planes or [3, Cout, KH*KW*C] bf16."""
    if weight.dim() != 4:
        raise ValueError("pack_conv_f32x6: weight must be [Cout, C, KH, KW]")
    w = weight.detach().float().permute(0, 2, 3, 1).reshape(weight.shape[0], -1).contiguous()
    return pack_f32_weight(w)


def conv2d_f32x6_supported(cin, cout, h3=None):
    return cin % LINEAR_F32X6_BK == 0 and cout % _n_multiple(h3) == 0


def conv2d_f32x6(x, planes, bias, kernel_size, stride=1, padding=0, relu=False, res=None):
    """relu?(conv2d(x, w, stride, padding) + bias + res) as one fp32-accurate implicit GEMM
    (rmbx_conv2d_f16x3 / rmbx_conv2d_f32x6 by the form of planes = pack_conv_f32x6(w)); x f32
    [N, C, H, W] channels_last; result channels_last [N, Cout, Ho, Wo]."""
    if x.dtype != torch.float32 or not x.is_cuda or x.dim() != 4:
        raise ValueError("conv2d_f32x6: x must be an f32 device tensor [N, C, H, W]")
    if not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv2d_f32x6: x must be channels_last")
    n, c, h, w_ = x.shape
    kh, kw = (kernel_size, kernel_size) if isinstance(kernel_size, int) else kernel_size
    cout, kk, h3 = _planes_nk(planes, "conv2d_f32x6")
    if kk != kh * kw * c:
        raise ValueError("conv2d_f32x6: planes must be pack_conv_f32x6(weight) for this input")
    pt = planes.planes if h3 else planes
    if not pt.is_contiguous():
        raise ValueError("conv2d_f32x6: planes must be contiguous")
    if not conv2d_f32x6_supported(c, cout, h3):
        raise ValueError(f"conv2d_f32x6: C={c} must be a multiple of 32 and Cout={cout} of {_n_multiple(h3)}")
    ho = (h + 2 * padding - kh) // stride + 1
    wo = (w_ + 2 * padding - kw) // stride + 1
    if bias is not None:
        _chk(bias, torch.float32, (cout,), "bias")
    out = torch.empty((n, cout, ho, wo), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    if res is not None:
        if res.shape != out.shape or res.dtype != torch.float32 or not res.is_contiguous(memory_format=torch.channels_last):
            raise ValueError("conv2d_f32x6: res must be a channels_last f32 tensor shaped like the output")
    name = f"conv {kh}x{kw}/{stride} {c}->{cout} {h}x{w_}"
    flops = 2.0 * n * ho * wo * cout * c * kh * kw
    nbytes = 4 * n * h * w_ * c + (4 if h3 else 6) * cout * c * kh * kw + 4 * n * ho * wo * cout * (1 if res is None else 2)
    if h3:
        _gemm_launch(name, flops, nbytes, 3, "rmbx_conv2d_f16x3", N.ptr(x), n, h, w_, c, N.ptr(pt), N.ptr(planes.scale),
                     N.ptr(bias), N.ptr(res), N.ptr(out), cout, kh, kw, stride, padding, 1 if relu else 0,
                     N.stream_ptr())
    else:
        _gemm_launch(name, flops, nbytes, 6, "rmbx_conv2d_f32x6", N.ptr(x), n, h, w_, c, N.ptr(pt), N.ptr(bias),
                     N.ptr(res), N.ptr(out), cout, kh, kw, stride, padding, 1 if relu else 0, N.stream_ptr())
    return out


def conv3x3_f16x3_patch(x, planes, bias, relu=False, res=None):
    """relu?(conv2d(x, w, stride 1, pad 1) + bias + res), fp32-accurate, by rmbx_conv3x3_f16x3_patch:
    the f16x3 form with each input pixel split once per output tile (16 x 16 or 16 x 32 pixels,
    the input patch of a 32-channel chunk staged in LDS for all nine taps) instead of once per tap.
    planes = pack_conv_f32x6(w) in the f16x3 form (F16x3Planes [2, Cout, 9 C]); x f32 channels_last
    [N, C, H, W] with C % 32 == 0, Cout % 64 == 0; result channels_last."""
    if x.dtype != torch.float32 or not x.is_cuda or x.dim() != 4:
        raise ValueError("conv3x3_f16x3_patch: x must be an f32 device tensor [N, C, H, W]")
    if not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv3x3_f16x3_patch: x must be channels_last")
    n, c, h, w_ = x.shape
    cout, kk, h3 = _planes_nk(planes, "conv3x3_f16x3_patch")
    if not h3:
        raise ValueError("conv3x3_f16x3_patch: planes must be in the f16x3 form")
    if kk != 9 * c or c % 32 or cout % 64:
        raise ValueError(f"conv3x3_f16x3_patch: C={c} (multiple of 32), Cout={cout} (multiple of 64), "
                         "planes = pack_conv_f32x6 of a 3x3 weight")
    pt = planes.planes
    if not pt.is_contiguous():
        raise ValueError("conv3x3_f16x3_patch: planes must be contiguous")
    if bias is not None:
        _chk(bias, torch.float32, (cout,), "bias")
    out = torch.empty((n, cout, h, w_), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    if res is not None:
        if res.shape != out.shape or res.dtype != torch.float32 or not res.is_contiguous(memory_format=torch.channels_last):
            raise ValueError("conv3x3_f16x3_patch: res must be a channels_last f32 tensor shaped like the output")
    name = f"conv3x3p {c}->{cout} {h}x{w_}"
    flops = 2.0 * n * h * w_ * cout * c * 9
    nbytes = 4 * n * h * w_ * c + 4 * cout * c * 9 + 4 * n * h * w_ * cout * (1 if res is None else 2)
    _gemm_launch(name, flops, nbytes, 3, "rmbx_conv3x3_f16x3_patch", N.ptr(x), n, h, w_, c, N.ptr(pt), pt.stride(0),
                 N.ptr(planes.scale), N.ptr(bias), N.ptr(res), N.ptr(out), cout, 1 if relu else 0, N.stream_ptr())
    return out


WINO_X6_CHANNELS = (256, 512)


def pack_wino4_x6(weight):
    """3x3 conv weight [Cout, C, 3, 3] -> pack_f32_weight of the Winograd F(4x4, 3x3) filter
    transform U = G g G^T (f64 on the host, rounded once to f32) laid out [36 positions][Cout][C]
    (the W operand of the 36 position GEMMs; rows [36 Cout, C])."""
    if weight.dim() != 4 or tuple(weight.shape[2:]) != (3, 3):
        raise ValueError("pack_wino4_x6: weight must be [Cout, C, 3, 3]")
    co, ci = weight.shape[0], weight.shape[1]
    w = weight.detach().to("cpu", torch.float64)
    G = torch.tensor(_WINO4_G, dtype=torch.float64)
    U = torch.einsum("xa,oiab,yb->xyoi", G, w, G).reshape(36 * co, ci)
    return pack_f32_weight(U.to(torch.float32).to(weight.device).contiguous())


def conv3x3_wino4_x6(x, planes, bias, relu=False, res=None):
    """relu?(conv2d(x, w, stride 1, pad 1) + bias + res) as the explicit Winograd F(4x4, 3x3): input
    transform pass (rmbx_wino4_input_f32), 36 fp32-accurate position GEMMs (rmbx_linear_f16x3_batched
    / rmbx_linear_f32x6_batched by the form of planes = pack_wino4_x6(w)), output transform pass
    with the epilogue (rmbx_wino4_output_f32).  x f32 channels_last [N, C, H, W]."""
    _chk_nhwc(x, "x")
    if x.dtype != torch.float32:
        raise ValueError("conv3x3_wino4_x6: x must be f32")
    n, C, H, W = x.shape
    rows, kk, h3 = _planes_nk(planes, "conv3x3_wino4_x6")
    if kk != C or rows % 36:
        raise ValueError("conv3x3_wino4_x6: planes must be pack_wino4_x6(weight) for this input")
    co = rows // 36
    if not conv2d_f32x6_supported(C, co, h3):
        raise ValueError(f"conv3x3_wino4_x6: C={C} must be a multiple of 32 and Cout={co} of {_n_multiple(h3)}")
    if bias is not None:
        _chk(bias, torch.float32, (co,), "bias")
    out = torch.empty((n, co, H, W), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    if res is not None:
        _chk_nhwc(res, "res")
        if tuple(res.shape) != tuple(out.shape) or res.dtype != torch.float32:
            raise ValueError("res must match the output")
    T = n * ((H + 3) // 4) * ((W + 3) // 4)
    M = torch.empty((36, T, co), dtype=torch.float32, device=x.device)
    name, flops = f"winograd x36 M={T} N={co} K={C}", 2.0 * 36 * T * co * C
    if h3 and GEMM_PRESPLIT and C <= 512 and co % LINEAR_F32X6_BN == 0:
        # the input transform writes the position GEMMs' A pre-split (one power-of-two scale per tile)
        Vp = torch.empty((2, 36, T, C), dtype=torch.float16, device=x.device)
        rinv = torch.empty(T, dtype=torch.float32, device=x.device)
        N.call("rmbx_wino4_input_split", N.ptr(x), n, H, W, C, N.ptr(Vp), N.ptr(rinv), N.stream_ptr())
        p = planes.planes
        _gemm_launch(name + " presplit", flops, 36 * (4 * T * C + 4 * co * C + 4 * T * co), 3,
                     "rmbx_linear_f16x3_presplit_batched", N.ptr(Vp), C, Vp.stride(0), T * C, N.ptr(rinv), 0, N.ptr(p),
                     p.stride(1), p.stride(0), co * C, N.ptr(planes.scale), co, None, N.ptr(M), co, T * co, 36, T, co, C,
                     0, N.stream_ptr())
        N.call("rmbx_wino4_output_f32", N.ptr(M), n, H, W, co, N.ptr(bias), N.ptr(res), N.ptr(out), 1 if relu else 0,
               N.stream_ptr())
        return out
    V = torch.empty((36, T, C), dtype=torch.float32, device=x.device)
    N.call("rmbx_wino4_input_f32", N.ptr(x), n, H, W, C, N.ptr(V), N.stream_ptr())
    if h3:
        p = planes.planes
        _gemm_launch(name, flops, 36 * (4 * T * C + 4 * co * C + 4 * T * co), 3, "rmbx_linear_f16x3_batched", N.ptr(V),
                     C, T * C, N.ptr(p), p.stride(1), p.stride(0), co * C, N.ptr(planes.scale), co, None, N.ptr(M), co,
                     T * co, 36, T, co, C, 0, N.stream_ptr())
    else:
        _gemm_launch(name, flops, 36 * (4 * T * C + 6 * co * C + 4 * T * co), 6, "rmbx_linear_f32x6_batched", N.ptr(V),
                     C, T * C, N.ptr(planes), planes.stride(1), planes.stride(0), co * C, None, N.ptr(M), co, T * co,
                     36, T, co, C, 0, N.stream_ptr())
    N.call("rmbx_wino4_output_f32", N.ptr(M), n, H, W, co, N.ptr(bias), N.ptr(res), N.ptr(out), 1 if relu else 0,
           N.stream_ptr())
    return out


def conv2d_direct_f32(x, weight, bias, stride=1, padding=0):
    """conv2d(x, weight, bias, stride, padding) for few input channels by rmbx_conv2d_direct_f32
    (deterministic f32 VALU kernel); x f32 channels_last [N, C, H, W], weight [Cout, C, KH, KW];
    result channels_last."""
    if x.dtype != torch.float32 or not x.is_cuda or not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv2d_direct_f32: x must be an f32 channels_last device tensor")
    n, c, h, w_ = x.shape
    co, ci, kh, kw = weight.shape
    if ci != c:
        raise ValueError("conv2d_direct_f32: channel mismatch")
    wp = weight.detach().float().permute(0, 2, 3, 1).contiguous()
    if bias is not None:
        _chk(bias, torch.float32, (co,), "bias")
    ho, wo = (h + 2 * padding - kh) // stride + 1, (w_ + 2 * padding - kw) // stride + 1
    out = torch.empty((n, co, ho, wo), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    N.call("rmbx_conv2d_direct_f32", N.ptr(x), n, h, w_, c, N.ptr(wp), N.ptr(bias), N.ptr(out), co, kh, kw, stride,
           padding, N.stream_ptr())
    return out
