"""Production-shape timing of the ACT stem forms (1024 x 480 x 640 frames): the f32 MFMA kernel on
the f32 space-to-depth image vs the u8 kernel (normalisation folded, bf16 integer pixels x three
bf16 weight pieces), HIP events; and their max |difference|."""
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
x = K.s2d_u8_normalize(u, mean, std)
w = torch.randn(64, 3, 7, 7, device=dev, generator=g) * 0.1
b = torch.randn(64, device=dev, generator=g) * 0.5
wp = K.pack_stem_s2d(w)
ops = K.pack_stem_u8(w, b, mean, std)


def timeit(f, reps=5):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


a = K.stem_s2d_conv_maxpool(x, wp, b)
c = K.stem_s2d_conv_maxpool_u8(u, *ops)
torch.cuda.synchronize()
d = (a - c).abs().max().item() / max(1.0, a.abs().max().item())
t32 = timeit(lambda: K.stem_s2d_conv_maxpool(x, wp, b))
tu8 = timeit(lambda: K.stem_s2d_conv_maxpool_u8(u, *ops))
fl = 2.0 * n * 240 * 320 * 64 * 147
import os
print(f"stem n={n} layout={os.environ.get('RMBX_STEM_U8_LAYOUT', 4)} dpp={os.environ.get('RMBX_STEM_U8_DPP', 0)}: f32 kernel {t32:.3f} ms ({fl / t32 / 1e9:.1f} TF/s direct), u8 kernel {tu8:.3f} ms "
      f"({fl / tu8 / 1e9:.1f} TF/s direct, bf16 MFMA {3 * 2.0 * n * 240 * 320 * 64 * 256 / tu8 / 1e9:.0f} TF/s executed), "
      f"speedup {t32 / tu8:.2f}x, max rel diff {d:.2e}", flush=True)
