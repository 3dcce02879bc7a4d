"""Production-shape A/B of the u8 stem's weight forms (1024 x 480 x 640 frames, rounds interleaved in
one process): f16 (two f16 pieces, rmbx_stem_s2d_conv_maxpool_u8h) vs bf16 (three bf16 pieces,
rmbx_stem_s2d_conv_maxpool_u8), HIP events; max |difference| of each against the f32 MFMA stem."""
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
ops = {p: K.pack_stem_u8(w, b, mean, std, pieces=p) for p in ("f16", "bf16")}
ref = K.stem_s2d_conv_maxpool(K.s2d_u8_normalize(u[:64], mean, std), K.pack_stem_s2d(w), b)


def timeit(f, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for p in ops:
    c = K.stem_s2d_conv_maxpool_u8(u[:64].contiguous(), *ops[p])
    d = (ref - c).abs().max().item() / max(1.0, ref.abs().max().item())
    print(f"{p}: max rel diff vs the f32 MFMA stem {d:.2e}", flush=True)
ts = {p: [] for p in ops}
for _ in range(3):
    for p in ops:
        K.stem_s2d_conv_maxpool_u8(u, *ops[p])
        torch.cuda.synchronize()
        ts[p].append(timeit(lambda: K.stem_s2d_conv_maxpool_u8(u, *ops[p])))
fl = 2.0 * n * 240 * 320 * 64 * 147
print(" | ".join(f"{p}: {min(t):.3f} ms ({fl / min(t) / 1e9:.1f} TF/s direct)" for p, t in ts.items()),
      f"| f16 speedup {min(ts['bf16']) / min(ts['f16']):.2f}x", flush=True)
