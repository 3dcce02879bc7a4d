"""Diagnostic: GPU-event timing of the ACT policy pieces at rollout batch size.

python scripts/prof_act.py [--batch 1024] [--benchmark]  (device cuda:0, bf16)
Prints ms per call for: trunk with HIP epilogues, trunk with torch epilogues, input proj +
transformer, whole forward; and the achieved TFLOP/s of the whole forward (41.8 GFLOP/sample).
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from robomanipbaselines_amd.policy.act.act_model import ActModel  # noqa: E402


def timeit(fn, iters=5, warm=2):
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


def torch_epi(x, b, res=None, rb=None, relu=True):
    y = x + b.to(x.dtype).reshape(1, -1, 1, 1)
    if res is not None:
        y = y + (res if rb is None else res + rb.to(x.dtype).reshape(1, -1, 1, 1))
    return F.relu(y) if relu else y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--benchmark", action="store_true")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = a.benchmark
    dev = "cuda:0"
    torch.manual_seed(0)
    m = ActModel().eval().requires_grad_(False)
    m.fuse_backbone()
    m = m.to(dev, torch.bfloat16)
    m._fused = m._fused.to(memory_format=torch.channels_last)
    tr = m._fused
    B = a.batch
    img = torch.rand(B, 1, 3, 480, 640, device=dev).to(torch.bfloat16)
    x = img[:, 0].contiguous(memory_format=torch.channels_last)
    q = torch.randn(B, 7, device=dev, dtype=torch.bfloat16)

    def trunk_torch():
        s = tr.stem.conv_nobias(x)
        h = F.max_pool2d(torch_epi(s, tr.stem.bias_f32()), 3, 2, 1)
        for blk in tr.blocks:
            y = torch_epi(blk.c1.conv_nobias(h), blk.c1.bias_f32())
            z = blk.c2.conv_nobias(y)
            h = torch_epi(z, blk.c2.bias_f32(), h) if blk.down is None else \
                torch_epi(z, blk.c2.bias_f32(), blk.down.conv_nobias(h), blk.down.bias_f32())
        return h

    def convs_only():
        s = tr.stem.conv_nobias(x)
        h = F.max_pool2d(s, 3, 2, 1)
        for blk in tr.blocks:
            y = blk.c1.conv_nobias(h)
            h = blk.c2.conv_nobias(y)
        return h

    res = {"batch": B, "cudnn_benchmark": a.benchmark}
    with torch.no_grad():
        res["trunk_hip_epilogue_ms"] = timeit(lambda: tr(x), a.iters)
        res["trunk_torch_epilogue_ms"] = timeit(trunk_torch, a.iters)
        res["trunk_convs_maxpool_only_ms"] = timeit(convs_only, a.iters)
        res["stem_conv_ms"] = timeit(lambda: tr.stem.conv_nobias(x), a.iters)
        res["forward_ms"] = timeit(lambda: m(q, img), a.iters)
        m.prune_dead_decoder = True
        res["forward_pruned_ms"] = timeit(lambda: m(q, img), a.iters)
    res["forward_tflops"] = 41.8e9 * B / (res["forward_ms"] * 1e-3) / 1e12
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
