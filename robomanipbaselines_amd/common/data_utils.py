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


def make_meta_info(op):
    ck = getattr(op.args, "checkpoint", None)
    if ck:
        # RolloutBase.setup_model_meta_info (:289-293) opens the file unconditionally: a trained
        # policy without its normalisation statistics / skip / chunk size must not run
        p = os.path.join(os.path.dirname(ck), "model_meta_info.pkl")
        if not os.path.exists(p):
            raise FileNotFoundError(f"model meta info not found next to the checkpoint: {p}")
        return load_meta_info(p)
    init = np.concatenate([op.env.init_qpos[:6], [0.0]])
    stats = {"norm_config": {"type": "gaussian"}, "mean": init.copy(), "std": np.full(7, 0.1),
             "min": init - 1.0, "max": init + 1.0, "range": np.full(7, 2.0), "example": init.copy()}
    meta = {
        "data": {"name": "synthetic", "skip": 3, "chunk_size": 100, "n_obs_steps": 1, "n_action_steps": 1},
        "policy": {"name": op.policy_name, "args": {}},
        "state": {"keys": [DataKey.MEASURED_JOINT_POS], **{k: np.array(v) if not isinstance(v, dict) else v for k, v in stats.items()}},
        "action": {"keys": [DataKey.COMMAND_JOINT_POS], **{k: np.array(v) if not isinstance(v, dict) else v for k, v in stats.items()}},
        "image": {"camera_names": ["front"]},
    }
    return meta
