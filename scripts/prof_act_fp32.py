"""Diagnostic: the fp32 ACT device form at rollout batch size, piece by piece, with progress lines.

python scripts/prof_act_fp32.py [--batch 1024] [--benchmark 0|1]
For every distinct conv of the fused ResNet-18 trunk: first-call time (MIOpen Find / solver
compile when benchmark is on) and steady ms per call with achieved TFLOP/s; then the
transformer (encoder 4 + decoder layer 0) and the whole forward."""

import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.policy.act.act_model import ActModel  # noqa: E402

T0 = time.time()


def log(msg):
    print(f"[{time.time() - T0:7.1f}s] {msg}", flush=True)


def timeit(fn, iters=3, warm=1):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--benchmark", type=int, default=1)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    dev = "cuda:0"
    torch.manual_seed(0)
    m = ActModel().eval().requires_grad_(False)
    m.fuse_backbone()
    m.prune_dead_decoder = True
    m = m.to(dev, torch.float32)
    m._fused = m._fused.to(memory_format=torch.channels_last)
    m.fuse_transformer()
    tr = m._fused
    B = a.batch
    log(f"batch {B} benchmark {a.benchmark}")
    x = torch.rand(B, 3, 480, 640, device=dev).contiguous(memory_format=torch.channels_last)
    total = 0.0
    with torch.no_grad():
        convs = [("stem", tr.stem, x)]
        h = F.max_pool2d(tr.stem.conv_nobias(x), 3, 2, 1)
        seen = {}
        for i, blk in enumerate(tr.blocks):
            convs.append((f"b{i}.c1", blk.c1, h))
            y = blk.c1.conv_nobias(h)
            convs.append((f"b{i}.c2", blk.c2, y))
            if blk.down is not None:
                convs.append((f"b{i}.down", blk.down, h))
            h = blk(h)
        torch.cuda.synchronize()
        log("shapes walked")
        for name, c, inp in convs:
            key = (tuple(inp.shape), tuple(c.conv.weight.shape), c.conv.stride)
            t1 = time.time()
            out = c.conv_nobias(inp)
            torch.cuda.synchronize()
            first = time.time() - t1
            ms = timeit(lambda: c.conv_nobias(inp))
            fl = 2 * out.numel() * c.conv.weight[0].numel()
            total += ms
            log(f"{name:8s} in {tuple(inp.shape)} w {tuple(c.conv.weight.shape)} s{c.conv.stride[0]}: first {first:6.2f}s "
                f"{ms:8.3f} ms  {fl / ms / 1e9:7.1f} TF/s{'  (repeat shape)' if key in seen else ''}")
            seen[key] = ms
        log(f"sum of conv times {total:.1f} ms")
        ms = timeit(lambda: tr(x))
        log(f"trunk (convs + rmbx epilogues) {ms:.1f} ms")
        from robomanipbaselines_amd import kernels as K

        xs = K.image_to_s2d(x.contiguous())
        log(f"fused f32 stem (rmbx)          {timeit(lambda: tr.forward_s2d(xs) if False else K.stem_s2d_conv_maxpool(xs, K.pack_stem_s2d(tr.stem.conv.weight), tr.stem.bias_f32())):.2f} ms")
        log(f"trunk via s2d f32 stem         {timeit(lambda: tr.forward_s2d(xs)):.1f} ms")
        # MIOpen in NCHW (Winograd-capable layouts) for two 3x3 shapes
        for name, c, inp in convs[1:2] + convs[-2:-1]:
            xin = inp.contiguous()
            wn = c.conv.weight.contiguous()
            F.conv2d(xin, wn, None, c.conv.stride, c.conv.padding)
            ms = timeit(lambda: F.conv2d(xin, wn, None, c.conv.stride, c.conv.padding))
            out = F.conv2d(xin, wn, None, c.conv.stride, c.conv.padding)
            log(f"NCHW {name:8s} {ms:8.3f} ms  {2 * out.numel() * wn[0].numel() / ms / 1e9:7.1f} TF/s")
        # transformer pieces (encoder layer 0 shapes: [B, 302, 512])
        from robomanipbaselines_amd import kernels as K

        L = m.encoder_layers[0]
        src = torch.randn(B, 302, 512, device=dev)
        pos = torch.randn(1, 302, 512, device=dev)
        qq = src + pos
        w, b = L.self_attn.in_proj_weight, L.self_attn.in_proj_bias
        log(f"qkv linear      {timeit(lambda: F.linear(qq, w, b)):8.3f} ms")
        qkv = F.linear(qq, w, b)
        qh, kh, vh = (t.reshape(B, 302, 8, 64).transpose(1, 2) for t in qkv.split(512, -1))
        log(f"sdpa            {timeit(lambda: F.scaled_dot_product_attention(qh, kh, vh)):8.3f} ms")
        for be in ("MATH", "EFFICIENT_ATTENTION", "FLASH_ATTENTION"):
            try:
                from torch.nn.attention import SDPBackend, sdpa_kernel

                with sdpa_kernel(getattr(SDPBackend, be)):
                    log(f"sdpa {be:14s} {timeit(lambda: F.scaled_dot_product_attention(qh, kh, vh)):8.3f} ms")
            except Exception as exc:
                log(f"sdpa {be}: {type(exc).__name__}: {str(exc)[:100]}")
        log(f"out_proj        {timeit(lambda: L.self_attn.out_proj(src)):8.3f} ms")
        log(f"attention (MHA) {timeit(lambda: L.self_attn(qq, qq, src)):8.3f} ms")
        nw, nb = L._norm_f32(L.norm1)
        log(f"add_layernorm   {timeit(lambda: K.add_layernorm(src, src, nw, nb, 1e-5)):8.3f} ms")
        log(f"ffn (fused)     {timeit(lambda: L.ffn(src)):8.3f} ms")
        x2 = src.reshape(-1, 512)
        log(f"ffn1 addmm_act  {timeit(lambda: torch._addmm_activation(L.linear1.bias, x2, L.linear1.weight.t())):8.3f} ms")
        log(f"ffn1 linear     {timeit(lambda: F.linear(x2, L.linear1.weight, L.linear1.bias)):8.3f} ms")
        h1 = F.linear(x2, L.linear1.weight, L.linear1.bias)
        log(f"ffn2 linear     {timeit(lambda: F.linear(h1, L.linear2.weight, L.linear2.bias)):8.3f} ms")
        log(f"encoder layer   {timeit(lambda: L.forward_q(src, qq, pos, True)):8.3f} ms")
        q = torch.randn(B, 7, device=dev)
        img = xs[:, None]
        ms = timeit(lambda: m(q, img), warm=2)
        log(f"whole ACT forward fp32 (s2d stem) {ms:.1f} ms -> {B * 34.93e9 / ms / 1e9:.1f} TF/s algorithmic")


if __name__ == "__main__":
    main()
