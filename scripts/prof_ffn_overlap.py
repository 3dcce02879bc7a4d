"""A/B: the ACT FFN pair on pre-split rows (linear_presplit_split -> linear_presplit, M = 1024 x 302
tokens, 512 -> 3200 -> 512) run back to back vs in row chunks with FFN1 of chunk i + 1 on the main
stream beside FFN2 of chunk i on a side stream (so one kernel's epilogue stores overlap the other's
MFMAs).  Outputs checked bitwise (every row is computed independently)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
M, D, F = 1024 * 302, 512, 3200
x = torch.randn(M, D, device=dev, generator=g)
r = torch.randn(M, D, device=dev, generator=g)
lw, lb = torch.ones(D, device=dev), torch.zeros(D, device=dev)
y = K.add_layernorm_split(x, r, lw, lb, 1e-5, y_norm=True)
sp = K.presplit_of(y)
w1 = torch.randn(F, D, device=dev, generator=g) / D ** 0.5
b1 = torch.randn(F, device=dev, generator=g) * 0.1
w2 = torch.randn(D, F, device=dev, generator=g) / F ** 0.5
b2 = torch.randn(D, device=dev, generator=g) * 0.1
p1, p2 = K.pack_f32_weight(w1), K.pack_f32_weight(w2)
bnd = K.weight_bounds(w1, b1)
hid = K.PresplitRows(torch.empty((2, M, F), dtype=torch.float16, device=dev), torch.empty(M, dtype=torch.float32, device=dev))
side = torch.cuda.Stream()


def rows(ps, a, b):
    return K.PresplitRows(ps.planes[:, a:b], ps.rinv[a:b], ps.norm[a:b] if ps.norm is not None else None)


def sequential(out):
    K.linear_presplit_split(sp, p1, b1, bnd, relu=True, out=hid)
    K.linear_presplit(hid, p2, b2, out=out)


def chunked(out, C):
    main = torch.cuda.current_stream()
    edges = [((M // 256) * i // C) * 256 for i in range(C)] + [M]
    for i in range(C):
        a, b = edges[i], edges[i + 1]
        K.linear_presplit_split(rows(sp, a, b), p1, b1, bnd, relu=True, out=rows(hid, a, b))
        ev = torch.cuda.Event()
        ev.record(main)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            K.linear_presplit(rows(hid, a, b), p2, b2, out=out[a:b])
    done = torch.cuda.Event()
    done.record(side)
    main.wait_event(done)


def timed(fn, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


ref = torch.empty(M, D, device=dev)
got = torch.empty(M, D, device=dev)
res = {}
with torch.no_grad():
    for rnd in range(3):
        sequential(ref)
        res.setdefault("sequential", []).append(timed(lambda: sequential(ref)))
        for C in (2, 4, 8):
            got.zero_()
            chunked(got, C)
            torch.cuda.synchronize()
            assert torch.equal(got, ref), C
            res.setdefault(f"chunks{C}", []).append(timed(lambda: chunked(got, C)))
for k, v in res.items():
    print(json.dumps({"form": k, "ms_per_ffn_pair": round(min(v), 3)}), flush=True)
