"""Model meta information and normalisation statistics.

The reference reads `model_meta_info.pkl` next to the checkpoint (RolloutBase.py:289-309) whose
schema TrainBase writes (common/base/TrainBase.py:190-217, 325-344).  For synthetic benchmarks
(no trained checkpoint exists offline, --checkpoint omitted) `make_meta_info` builds the same schema with gaussian
statistics mean = initial joint position, std = 0.1.  A meta file next to a
given checkpoint is read with a restricted unpickler that only reconstructs numpy arrays and
plain containers (nothing else in the file executes).
"""

import io
import os
import pickle

import numpy as np

from .data_key import DataKey

_ALLOWED = {
    ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"), ("builtins", "slice"),
}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name}")


def load_meta_info(path):
    with open(path, "rb") as f:
        return _SafeUnpickler(io.BytesIO(f.read())).load()


def _init_eef_pose(placement, q):
    """(t, qw, qx, qy, qz) of the arm at joint angles q: the URDF chain of the env's
    `arm_placement` and Eigen's matrix -> quaternion (MathUtils.get_pose_from_se3).  Used only
    to centre the synthetic normalisation statistics of the eef-pose keys."""
    R, p = np.eye(3), np.zeros(3)
    for k in range(6):
        c, s = np.cos(q[k]), np.sin(q[k])
        p = p + R @ placement[k, 9:12]
        R = R @ placement[k, :9].reshape(3, 3) @ np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])
    t = np.trace(R)
    if t > 0:
        r = np.sqrt(t + 1.0)
        quat = [0.5 * r, (R[2, 1] - R[1, 2]) * 0.5 / r, (R[0, 2] - R[2, 0]) * 0.5 / r, (R[1, 0] - R[0, 1]) * 0.5 / r]
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        r = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
        v = np.zeros(3)
        v[i], v[j], v[k] = 0.5 * r, (R[j, i] + R[i, j]) * 0.5 / r, (R[k, i] + R[i, k]) * 0.5 / r
        quat = [(R[k, j] - R[j, k]) * 0.5 / r, *v]
    return np.concatenate([p, quat])


def _synthetic_example(key, env):
    """The value of a data key at the env's initial pose (centre of the synthetic statistics)."""
    q0 = np.asarray(env.init_qpos[:6], dtype=np.float64)
    if key in (DataKey.MEASURED_JOINT_POS, DataKey.COMMAND_JOINT_POS):
        return np.concatenate([q0, [0.0]])
    if key in (DataKey.MEASURED_EEF_POSE, DataKey.COMMAND_EEF_POSE):
        return _init_eef_pose(np.asarray(env.arrays["arm_placement"], dtype=np.float64), q0)
    return np.zeros(DataKey.get_dim(key))


def _synthetic_stats(keys, env):
    """TrainBase-schema statistics (TrainBase.py:325-344) centred on the initial pose, std 0.1."""
    ex = np.concatenate([_synthetic_example(k, env) for k in keys]) if keys else np.zeros(0)
    return {"keys": list(keys), "norm_config": {"type": "gaussian"}, "mean": ex.copy(),
            "std": np.full(len(ex), 0.1), "min": ex - 1.0, "max": ex + 1.0, "range": np.full(len(ex), 2.0),
            "example": ex.copy()}


def make_meta_info(op):
    ck = getattr(op.args, "checkpoint", None)
    state_keys = getattr(op.args, "state_keys", None)
    action_keys = getattr(op.args, "action_keys", None)
    if ck:
        if state_keys is not None or action_keys is not None:
            raise ValueError("--state_keys / --action_keys configure synthetic runs only: a checkpoint's keys "
                             "come from its model_meta_info.pkl")
        # RolloutBase.setup_model_meta_info (:289-293) opens the file unconditionally: a trained
        # policy without its normalisation statistics / skip / chunk size must not run
        p = os.path.join(os.path.dirname(ck), "model_meta_info.pkl")
        if not os.path.exists(p):
            raise FileNotFoundError(f"model meta info not found next to the checkpoint: {p}")
        return load_meta_info(p)
    if state_keys is None:
        state_keys = [DataKey.MEASURED_JOINT_POS]
    if action_keys is None:
        action_keys = [DataKey.COMMAND_JOINT_POS]
    meta = {
        "data": {"name": "synthetic", "skip": 3, "chunk_size": 100, "n_obs_steps": 1, "n_action_steps": 1},
        "policy": {"name": op.policy_name, "args": {}},
        "state": _synthetic_stats(state_keys, op.env),
        "action": _synthetic_stats(action_keys, op.env),
        "image": {"camera_names": ["front"]},
    }
    return meta
