"""ctypes binding of the C ABI declared in include/rmbx.h (librmbx.so, built in-tree for gfx950).

This is the only route from Python to the HIP kernels.  It fails loudly: if the library is
missing or a symbol is absent, importing a function raises; there is no CPU fallback on the
product path.
"""

import ctypes
import os

import numpy as np

# RMBX_LIB_VARIANT=<name> loads _lib/librmbx_<name>.so instead (profiling A/Bs of build options
# only; the product loads librmbx.so)
_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                         f"librmbx_{os.environ['RMBX_LIB_VARIANT']}.so" if os.environ.get("RMBX_LIB_VARIANT")
                         else "librmbx.so")

_c_int = ctypes.c_int
_c_p = ctypes.c_void_p
_c_sz = ctypes.c_size_t
_c_d = ctypes.c_double

# name -> (restype, argtypes).  Must list every function declared in include/rmbx.h.
SIGNATURES = {
    "rmbx_abi_version": (_c_int, []),
    "rmbx_last_error": (ctypes.c_char_p, []),
    "rmbx_device_count": (_c_int, [_c_p]),
    "rmbx_act_ensemble": (
        _c_int,
        [_c_p] * 11 + [_c_int, _c_int, _c_int, _c_int, _c_p],
    ),
    "rmbx_cable_reward": (_c_int, [_c_p] * 5 + [_c_int, _c_int, _c_p]),
    "rmbx_door_reward": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_int, _c_d, _c_d, _c_p]),
    "rmbx_toolbox_reward": (_c_int, [_c_p, _c_p, _c_p, _c_int, _c_d, _c_d, _c_p]),
    "rmbx_ring_reward": (_c_int, [_c_p, _c_p, _c_p, _c_int, _c_int, _c_p]),
    "rmbx_cabinet_reward": (_c_int, [_c_p, _c_int, _c_int, _c_int, _c_d, _c_d, _c_int, _c_p, _c_int, _c_p]),
    "rmbx_insert_reward": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_int, _c_d, _c_d, _c_d, _c_p]),
    "rmbx_ur5e_obs": (_c_int, [_c_p] * 8 + [_c_int, _c_p]),
    "rmbx_depth_linearize": (_c_int, [_c_p, _c_p, _c_sz, _c_d, _c_d, _c_p]),
    "rmbx_sched_reset": (_c_int, [_c_p, _c_p, _c_p, _c_int, _c_p]),
    "rmbx_sched_active": (_c_int, [_c_p, _c_int, _c_p, _c_int, _c_p]),
    "rmbx_sched_update": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_int, _c_d, _c_d, _c_int, _c_p]),
    "rmbx_engine_create": (_c_int, [_c_p, _c_int, _c_p]),
    "rmbx_engine_destroy": (_c_int, [_c_p]),
    "rmbx_engine_workspace_bytes": (_c_int, [_c_p, _c_p]),
    "rmbx_engine_ws_offset": (_c_int, [_c_p, ctypes.c_char_p, _c_p, _c_p]),
    "rmbx_engine_bind": (_c_int, [_c_p, _c_p]),
    "rmbx_engine_step": (_c_int, [_c_p, _c_int, _c_p, _c_p]),
    "rmbx_engine_forward": (_c_int, [_c_p, _c_p, _c_p]),
    "rmbx_engine_step_profiled": (_c_int, [_c_p, _c_int, _c_p, _c_p]),
    "rmbx_arm_ik": (_c_int, [_c_p] * 5 + [_c_int, _c_int, _c_p]),
    "rmbx_arm_fk": (_c_int, [_c_p] * 4 + [_c_int, _c_p]),
    "rmbx_motion_state": (_c_int, [_c_p] * 9 + [_c_int, _c_p, _c_int, _c_int, _c_p]),
    "rmbx_motion_command": (_c_int, [_c_p, _c_p, _c_int, _c_p, _c_int, _c_int, _c_d, _c_d] + [_c_p] * 5
                            + [_c_int, _c_p]),
    "rmbx_render": (_c_int, [_c_p, _c_p, _c_p, _c_int, _c_p, _c_p, _c_p, _c_p, _c_int, _c_int, _c_p, _c_p, _c_p,
                             _c_int, _c_p, _c_int, _c_p]),
    "rmbx_render_scene": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_int, _c_int, _c_p, _c_p, _c_p, _c_p,
                                   _c_int, _c_p, _c_int, _c_p]),
    "rmbx_render_scene_cached": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_int, _c_int, _c_p, _c_p, _c_p,
                                          _c_p, _c_int, _c_p, _c_int, _c_p, _c_p]),
    "rmbx_nhwc_bias_act": (_c_int, [_c_p] * 5 + [_c_sz, _c_int, _c_int, _c_int, _c_p]),
    "rmbx_nhwc_bias_relu_maxpool": (_c_int, [_c_p] * 3 + [_c_int] * 5 + [_c_p]),
    "rmbx_conv2d_nhwc": (_c_int, [_c_p] * 5 + [_c_int] * 10 + [_c_p]),
    "rmbx_conv2d_nhwc_f32": (_c_int, [_c_p] * 5 + [_c_int] * 10 + [_c_p]),
    "rmbx_conv3x3_winograd_f32": (_c_int, [_c_p] * 5 + [_c_int] * 5 + [_c_p]),
    "rmbx_conv3x3_winograd4_f32": (_c_int, [_c_p] * 5 + [_c_int] * 5 + [_c_p]),
    "rmbx_stem_s2d_conv": (_c_int, [_c_p] * 4 + [_c_int] * 5 + [_c_p]),
    "rmbx_stem_s2d_conv_maxpool": (_c_int, [_c_p] * 4 + [_c_int] * 4 + [_c_p]),
    "rmbx_stem_s2d_conv_maxpool_f32": (_c_int, [_c_p] * 4 + [_c_int] * 4 + [_c_p]),
    "rmbx_stem_s2d_conv_maxpool_u8": (_c_int, [_c_p] * 5 + [_c_int] * 4 + [_c_p]),
    "rmbx_stem_s2d_conv_maxpool_u8h": (_c_int, [_c_p, _c_p, ctypes.c_float] + [_c_p] * 3 + [_c_int] * 4 + [_c_p]),
    "rmbx_attention_bf16": (_c_int, [_c_p] * 4 + [_c_int] * 4 + [ctypes.c_longlong, _c_int] * 3 + [ctypes.c_float, _c_p]),
    "rmbx_attention_f32": (_c_int, [_c_p] * 4 + [_c_int] * 4 + [ctypes.c_longlong, _c_int] * 3 + [ctypes.c_float, _c_p]),
    "rmbx_attention_f32x6": (_c_int, [_c_p] * 4 + [_c_int] * 4 + [ctypes.c_longlong, _c_int] * 3 + [ctypes.c_float, _c_p]),
    "rmbx_attention_f16x3": (_c_int, [_c_p] * 5 + [_c_int] * 4 + [ctypes.c_longlong, _c_int] * 3 + [ctypes.c_float, _c_p]),
    "rmbx_linear_f32x6": (_c_int, [_c_p, ctypes.c_longlong, _c_p, ctypes.c_longlong, ctypes.c_longlong, _c_p, _c_p,
                                   ctypes.c_longlong, _c_int, _c_int, _c_int, _c_int, _c_p]),
    "rmbx_conv2d_f32x6": (_c_int, [_c_p] + [_c_int] * 4 + [_c_p] * 4 + [_c_int] * 6 + [_c_p]),
    "rmbx_linear_f32x6_batched": (_c_int, [_c_p, ctypes.c_longlong, ctypes.c_longlong, _c_p, ctypes.c_longlong,
                                           ctypes.c_longlong, ctypes.c_longlong, _c_p, _c_p, ctypes.c_longlong,
                                           ctypes.c_longlong] + [_c_int] * 5 + [_c_p]),
    "rmbx_wino4_input_f32": (_c_int, [_c_p] + [_c_int] * 4 + [_c_p, _c_p]),
    "rmbx_wino4_output_f32": (_c_int, [_c_p] + [_c_int] * 4 + [_c_p] * 3 + [_c_int, _c_p]),
    "rmbx_conv2d_direct_f32": (_c_int, [_c_p] + [_c_int] * 4 + [_c_p] * 3 + [_c_int] * 5 + [_c_p]),
    "rmbx_split_bf16x3": (_c_int, [_c_p, _c_p, ctypes.c_longlong, _c_p]),
    "rmbx_split_f16x2": (_c_int, [_c_p, _c_int, _c_int, _c_p, _c_p, _c_p]),
    "rmbx_linear_f16x3": (_c_int, [_c_p, ctypes.c_longlong, _c_p, ctypes.c_longlong, ctypes.c_longlong, _c_p, _c_p,
                                   _c_p, ctypes.c_longlong, _c_int, _c_int, _c_int, _c_int, _c_p]),
    "rmbx_linear_f16x3_batched": (_c_int, [_c_p, ctypes.c_longlong, ctypes.c_longlong, _c_p, ctypes.c_longlong,
                                           ctypes.c_longlong, ctypes.c_longlong, _c_p, ctypes.c_longlong, _c_p, _c_p,
                                           ctypes.c_longlong, ctypes.c_longlong] + [_c_int] * 5 + [_c_p]),
    "rmbx_conv3x3_f16x3_patch": (_c_int, [_c_p] + [_c_int] * 4 + [_c_p, ctypes.c_longlong] + [_c_p] * 4
                                 + [_c_int, _c_int, _c_p]),
    "rmbx_conv2d_f16x3": (_c_int, [_c_p] + [_c_int] * 4 + [_c_p] * 5 + [_c_int] * 6 + [_c_p]),
    "rmbx_add_layernorm": (_c_int, [_c_p] * 5 + [_c_int, _c_int, ctypes.c_float, _c_int, _c_p]),
    "rmbx_groupnorm_act": (_c_int, [_c_p] * 4 + [_c_int] * 4 + [ctypes.c_float, _c_int, _c_p]),
    "rmbx_add_layernorm_split": (_c_int, [_c_p] * 9 + [_c_int, _c_p, _c_p, _c_p, _c_int, _c_int, ctypes.c_float, _c_p]),
    "rmbx_linear_f16x3_presplit_split": (_c_int, [_c_p, ctypes.c_longlong, ctypes.c_longlong, _c_p, _c_p, _c_p,
                                                  ctypes.c_longlong, ctypes.c_longlong, _c_p, ctypes.c_float,
                                                  ctypes.c_float, _c_p, _c_int, _c_p, ctypes.c_longlong,
                                                  ctypes.c_longlong, _c_p, _c_int, _c_int, _c_int, _c_p]),
    "rmbx_linear_f16x3_presplit_batched": (_c_int, [_c_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_longlong, _c_p,
                                                    ctypes.c_longlong, _c_p, ctypes.c_longlong, ctypes.c_longlong,
                                                    ctypes.c_longlong, _c_p, ctypes.c_longlong, _c_p, _c_p,
                                                    ctypes.c_longlong, ctypes.c_longlong, _c_int, _c_int, _c_int, _c_int,
                                                    _c_int, _c_p]),
    "rmbx_wino4_input_split": (_c_int, [_c_p, _c_int, _c_int, _c_int, _c_int, _c_p, _c_p, _c_p]),
    "rmbx_linear_f16x3_presplit": (_c_int, [_c_p, ctypes.c_longlong, ctypes.c_longlong, _c_p, _c_p, ctypes.c_longlong,
                                            ctypes.c_longlong, _c_p, _c_p, _c_p, _c_p, ctypes.c_longlong, _c_int, _c_int,
                                            _c_int, _c_int, _c_p]),
    "rmbx_add_layernorm_pos": (_c_int, [_c_p] * 6 + [_c_int, _c_p, _c_int, _c_int, ctypes.c_float, _c_int, _c_p]),
    "rmbx_ddpm_step": (_c_int, [_c_p] * 4 + [_c_sz, _c_p, _c_p]),
    "rmbx_ddim_step": (_c_int, [_c_p] * 3 + [_c_sz, _c_p, _c_int, _c_p]),
    "rmbx_resize_crop_u8": (_c_int, [_c_p] + [_c_int] * 10 + [ctypes.c_float, ctypes.c_float, _c_p, _c_int, _c_p]),
    "rmbx_resize_f32": (_c_int, [_c_p, _c_p] + [_c_int] * 5 + [_c_p]),
    "rmbx_pointcloud_fps": (_c_int, [_c_p, _c_p, _c_int, _c_int, _c_int, _c_d, _c_p, _c_p, _c_int, _c_int,
                                     _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
}


class Camera(ctypes.Structure):
    """ctypes mirror of rmbx_camera (include/rmbx.h)."""

    _fields_ = [("body", ctypes.c_int32), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("fovy_deg", ctypes.c_float), ("pos", ctypes.c_double * 3), ("quat", ctypes.c_double * 4),
                ("znear", ctypes.c_float), ("zfar", ctypes.c_float), ("mean", ctypes.c_float * 3),
                ("std", ctypes.c_float * 3)]


class SceneTables(ctypes.Structure):
    """ctypes mirror of rmbx_scene_tables (include/rmbx.h)."""

    _fields_ = [("prim_i32", _c_p), ("prim_f32", _c_p), ("nprim", ctypes.c_int32), ("ntri", ctypes.c_int32),
                ("nmesh", ctypes.c_int32), ("mesh_tri", _c_p), ("mesh_body", _c_p), ("mesh_rad", _c_p), ("vis", _c_p),
                ("tflag", _c_p), ("geom_texid", _c_p), ("geom_matinfo", _c_p), ("tex_rgba", _c_p), ("tex_desc", _c_p),
                ("tex_level_adr", _c_p), ("ntex", ctypes.c_int32), ("sky_rgb", ctypes.c_float * 6)]


class RenderCache(ctypes.Structure):
    """ctypes mirror of rmbx_render_cache (include/rmbx.h)."""

    _fields_ = [("prim_static", _c_p), ("static_prims", _c_p), ("nstatic", ctypes.c_int32), ("cache", _c_p),
                ("snap", _c_p), ("dirty", _c_p)]


class EnvBuffers(ctypes.Structure):
    """ctypes mirror of rmbx_env_buffers (include/rmbx.h)."""

    _fields_ = [(n, _c_p) for n in ("time", "qpos", "qvel", "qacc_ws", "ctrl", "body_pos", "xpos", "xquat",
                                    "gxpos", "gxmat", "sensordata", "stats", "workspace")]

# numpy mirror of rmbx_sched_t (include/rmbx.h)
TEX_LEVELS = 16  # include/rmbx.h RMBX_TEX_LEVELS

SCHED_DTYPE = np.dtype(
    [
        ("phase", np.int32),
        ("rollout_time_idx", np.int32),
        ("done", np.uint8),
        ("success", np.uint8),
        ("has_success_time", np.uint8),
        ("pad_", np.uint8, 5),
        ("phase_start", np.float64),
        ("success_time", np.float64),
        ("result_reward", np.float64),
        ("duration", np.float64),
    ]
)
assert SCHED_DTYPE.itemsize == 48

_lib = None


class RmbxError(RuntimeError):
    pass


def lib_path():
    return _LIB_PATH


def load():
    """Load librmbx.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise RmbxError(
            f"{_LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(_LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if the symbol is missing: fail loudly
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status):
    if status != 0:
        msg = load().rmbx_last_error().decode(errors="replace")
        if status == -1:
            raise ValueError(msg)
        raise RmbxError(f"rmbx error {status}: {msg}")


def call(name, *args):
    check(getattr(load(), name)(*args))


def ptr(t):
    """Device (or host) pointer of a torch tensor / numpy array, or None."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return t.data_ptr()
    return t.ctypes.data


def stream_ptr(stream=None):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
