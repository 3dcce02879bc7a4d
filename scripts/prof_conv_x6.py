"""rmbx_conv2d_f32x6 vs MIOpen fp32 (+ the rmbx bias/ReLU epilogue pass) on the fp32 ResNet-18
trunk's stride-2 3x3 and 1x1 downsample convs at 1024 frames (480x640 input)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from robomanipbaselines_amd import kernels as K  # noqa: E402


def timeit(fn, it=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    torch.backends.cudnn.benchmark = True
    torch.backends.cudnn.allow_tf32 = False
    cl = torch.channels_last
    for C, H, W, Co in ((64, 120, 160, 128), (128, 60, 80, 256), (256, 30, 40, 512)):
        x = torch.randn(1024, C, H, W, device="cuda").contiguous(memory_format=cl)
        for k, s, p in ((3, 2, 1), (1, 2, 0)):
            w = (torch.randn(Co, C, k, k, device="cuda") / (C * k * k) ** 0.5).contiguous(memory_format=cl)
            b = torch.randn(Co, device="cuda")
            pl = K.pack_conv_f32x6(w)
            y6 = K.conv2d_f32x6(x, pl, b, k, s, p, relu=(k == 3))
            ym = F.conv2d(x, w, None, s, p)
            ym = K.nhwc_bias_act(ym, b, relu=(k == 3), out=ym)
            rel = ((y6[:4].double() - ym[:4].double()).abs().max() / ym[:4].abs().max()).item()
            t6 = timeit(lambda: K.conv2d_f32x6(x, pl, b, k, s, p, relu=(k == 3)))
            tm = timeit(lambda: K.nhwc_bias_act(F.conv2d(x, w, None, s, p), b, relu=(k == 3)))
            Ho, Wo = y6.shape[2], y6.shape[3]
            fl = 2.0 * 1024 * Ho * Wo * Co * C * k * k
            print(f"C={C:3d}->{Co:3d} {H}x{W} k{k} s{s}: f32x6 {t6:6.3f} ms ({fl / t6 / 1e9:6.1f} TF/s, bf16 MFMA "
                  f"{6 * fl / t6 / 1e9 / 2500 * 100:4.1f} %) | MIOpen+epilogue {tm:6.3f} ms | speedup {tm / t6:4.2f}x "
                  f"| rel diff {rel:.2e}", flush=True)
        del x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
