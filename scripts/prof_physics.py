"""Diagnostic: per-stage shader-cycle breakdown and wall time of the physics kernel."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv  # noqa: E402
from robomanipbaselines_amd.envs.ur5e_pick import BatchedMujocoUR5ePickEnv  # noqa: E402

# --env pick: the config-4/5 scene (dt 0.002 x 16, convex hulls), gripper open
PICK = "--env" in sys.argv and sys.argv[sys.argv.index("--env") + 1] == "pick"

_pos = [x for x in sys.argv[1:] if not x.startswith("--") and x != "pick"]
n = int(_pos[0]) if _pos else 1024
if "--calib" in sys.argv:
    # known-byte-count copies for calibrating FETCH_SIZE / WRITE_SIZE (scripts/pmc_calib.hip):
    # 512 MiB read + 512 MiB written per launch, past the 256 MiB Infinity Cache
    import ctypes

    cal = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libpmc_calib.so"))
    cal.pmc_calib.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    nb = 512 << 20
    x = torch.zeros(nb // 8, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    for wide in (0, 1, 0, 1):
        assert cal.pmc_calib(x.data_ptr(), y.data_ptr(), nb, wide, None) == 0
    torch.cuda.synchronize()
    del x, y
env = (BatchedMujocoUR5ePickEnv if PICK else BatchedMujocoUR5eCableEnv)(n, "cuda:0")
env.reset()
a = env.engine.ctrl.clone()
a[:, 6] = 0.0 if PICK else 255.0
for _ in range(20):
    env.step(a)
torch.cuda.synchronize()
t = time.time()
for _ in range(5):
    env.step(a)
torch.cuda.synchronize()
dt = (time.time() - t) / 5
print(f"n_env {n}: {dt*1e3:.2f} ms per env-step -> {n/dt:.0f} env-steps/s")
st = env.engine.stats.cpu().numpy()
print("ncon mean", st[:, 0].mean(), "nefc mean", st[:, 1].mean(), "iters mean", st[:, 2].mean(), "bad", st[:, 3].sum())
FS = env.frame_skip
p = env.engine.step_profiled(FS)
tot = sum(v for k, v in p.items() if "." not in k)
for k, v in p.items():
    print(f"  {k:34s} {v/1e6:8.3f} Mcycles  {100*v/tot:5.1f}%")
raw = env.engine.step_profiled(FS, raw=True).astype(np.float64)
front, solver = raw[:, 0:5].sum(1), raw[:, 5:8].sum(1)
for name, v in (("front stages", front), ("solver stages", solver)):
    print(f"  per-env {name:14s} mean {v.mean()/1e6:6.3f}  p50 {np.median(v)/1e6:6.3f}  p99 {np.percentile(v, 99)/1e6:6.3f}  max {v.max()/1e6:6.3f} Mcycles")
st = env.engine.stats.cpu().numpy()
print("  ncon max", st[:, 0].max(), "nefc max", st[:, 1].max(), "iters max", st[:, 2].max())
