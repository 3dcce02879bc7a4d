"""PMC driver for the dominant policy kernel (rmbx gemm_f32x6_kernel): calibration copies
(scripts/pmc_calib.hip, 512 MiB read + written per launch, 8-B and 16-B lanes), then two fp32 ACT
inferences of the bench workload (MujocoUR5eCable x1024, the bench's rollout and weights); run
under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes (scripts/gpurun/gemm_pmc.sh);
tools/pmc_traffic.py --gemm reduces the second inference's GEMM launches."""
import ctypes
import os
import sys
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

cal = ctypes.CDLL(os.path.join(ROOT, "scripts", "_build", "libpmc_calib.so"))
cal.pmc_calib.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
nb = 512 << 20
x = torch.zeros(nb // 8, dtype=torch.float64, device="cuda")
y = torch.empty_like(x)
for wide in (0, 1, 0, 1):
    assert cal.pmc_calib(x.data_ptr(), y.data_ptr(), nb, wide, None) == 0
torch.cuda.synchronize()
del x, y
ro = bench.make_rollout(SimpleNamespace(act_full_decoder=False), "cuda:0", "fp32", 1024, 0)
with torch.no_grad():
    for i in range(2):
        ro.infer_policy()
        torch.cuda.synchronize()
        print(f"inference {i} done", flush=True)
