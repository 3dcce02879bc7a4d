"""Phase skips of the u8 stem's f16 kernel at the production shape (1024 x 480 x 640 frames):
RMBX_STEM_VAR = 0 (default), 1 (no pool epilogue), 2 (no ring refill), 3 (neither: MFMA loop +
LDS reads), 4 (no MFMAs), 6 (no MFMAs, no refill); wrong results except 0, timing only (HIP events,
rounds interleaved in one process)."""
import os
import sys

import torch

sys.path.insert(0, ".")
from robomanipbaselines_amd import kernels as K  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = "cuda"
mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
g = torch.Generator(device=dev).manual_seed(0)
u = torch.randint(0, 256, (n, 240, 320, 16), device=dev, generator=g, dtype=torch.int32).to(torch.uint8)
u[..., 12:] = 0
w = torch.randn(64, 3, 7, 7, device=dev, generator=g) * 0.1
b = torch.randn(64, device=dev, generator=g) * 0.5
op = K.pack_stem_u8(w, b, mean, std, pieces="f16")


def timeit(f, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


VARS = ("0", "1", "2", "3", "4", "6")
ts = {v: [] for v in VARS}
for _ in range(3):
    for v in VARS:
        os.environ["RMBX_STEM_VAR"] = v
        K.stem_s2d_conv_maxpool_u8(u, *op)
        torch.cuda.synchronize()
        ts[v].append(timeit(lambda: K.stem_s2d_conv_maxpool_u8(u, *op)))
os.environ.pop("RMBX_STEM_VAR")
fl = 2.0 * n * 240 * 320 * 64 * 256 * 2  # executed: K = 16 taps x 16 s2d channels, 2 weight pieces
print(" | ".join(f"{v}: {min(t):.3f} ms ({fl / min(t) / 1e9 / 2500:.3f})" for v, t in ts.items()), flush=True)
