"""ACT at the benchmarked production configuration (policy/act/TrainAct.py:46-58: ResNet-18,
hidden 512, feed-forward 3200, 8 heads, 4 encoder / 7 decoder layers, 100 queries; 480x640
front camera) on the device against the unfused fp32 CPU module, through the temporal ensemble
and denormalisation (rmbx_act_ensemble vs oracle/glue.ActEnsembleOracle).

* fp32 (the reference's precision, the credited bench mode): denormalised env actions within
  1e-4 of the CPU module's (BASELINE.json north star).  The device form skips decoder layers
  1..6 (the DETRVAE output reads layer 0's normed intermediate only); the CPU module computes
  all seven, so the test also proves the skip exact.
* bf16 (throughput mode, the bench's secondary line): its action error against fp32 is measured
  and bounded here; the bound is the documented accuracy of that mode, not parity."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
N_ENV = 8
CALLS = 3


def _models():
    from robomanipbaselines_amd.policy.act.act_model import ActModel

    torch.manual_seed(0)
    ref = ActModel().eval().requires_grad_(False)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for m in ref.modules():  # non-trivial frozen BN statistics
            if hasattr(m, "running_var"):
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
                m.bias.copy_(torch.rand(m.bias.shape, generator=g) * 0.4 - 0.2)
                m.running_mean.copy_(torch.rand(m.running_mean.shape, generator=g) * 0.4 - 0.2)
                m.running_var.copy_(torch.rand(m.running_var.shape, generator=g) * 1.5 + 0.5)
    return ref


def _device_form(ref, dtype):
    from robomanipbaselines_amd.policy.act.act_model import ActModel

    dev = ActModel().eval().requires_grad_(False)
    dev.load_state_dict(ref.state_dict())
    dev.fuse_backbone()
    dev.prune_dead_decoder = True
    dev = dev.to(DEV, dtype).requires_grad_(False)
    dev._fused = dev._fused.to(memory_format=torch.channels_last)
    dev.fuse_transformer()
    return dev


def _inputs():
    from robomanipbaselines_amd.policy.act.act_model import IMAGENET_MEAN, IMAGENET_STD

    g = torch.Generator().manual_seed(2)
    out = []
    for _ in range(CALLS):
        state = torch.randn(N_ENV, 7, generator=g)
        # 8-bit pixels as the renderer quantises them, normalised as it does (f32 ops)
        u = (torch.rand(N_ENV, 1, 3, 480, 640, generator=g) * 255.0 + 0.5).floor().to(torch.uint8)
        m = torch.tensor(IMAGENET_MEAN).reshape(1, 1, 3, 1, 1)
        s = torch.tensor(IMAGENET_STD).reshape(1, 1, 3, 1, 1)
        out.append((state, (u.float() / 255.0 - m) / s))
        _U8.append(u)
    return out


_U8 = []  # the 8-bit images of _inputs(), in call order


STATS = {"norm_config": {"type": "gaussian"}, "mean": np.linspace(-1.0, 1.0, 7), "std": np.full(7, 0.1)}


def _ensemble_actions(chunks_dev):
    from robomanipbaselines_amd import kernels as K

    st = K.ActEnsembleState(N_ENV, 100, 7, STATS, DEV)
    return [st(c.float().contiguous()).cpu().numpy().copy() for c in chunks_dev]


@torch.no_grad()
def test_act_production_config_fp32_within_1e4_and_bf16_error():
    from oracle import glue
    from robomanipbaselines_amd import kernels as K

    ref = _models()
    inputs = _inputs()
    want_chunks = [ref(s, im) for s, im in inputs]  # CPU fp32, all 7 decoder layers
    orcs = [glue.ActEnsembleOracle(100, STATS) for _ in range(N_ENV)]
    want = []
    for c in want_chunks:
        cn = c.numpy()
        want.append(np.stack([o.step(lambda e=e: cn[e]) for e, o in enumerate(orcs)]))
    want = np.array(want)

    dev32 = _device_form(ref, torch.float32)
    # the bench path: the renderer's f32 space-to-depth image into the fused f32 stem
    got_chunks = [dev32(s.to(DEV), K.image_to_s2d(im[:, 0].to(DEV))[:, None]) for s, im in inputs]
    std_form = dev32(inputs[0][0].to(DEV), inputs[0][1].to(DEV))  # CHW image: MIOpen stem
    assert (std_form.cpu() - want_chunks[0]).abs().max().item() <= 1e-4
    got = np.array(_ensemble_actions(got_chunks))
    chunk_err = max((g.cpu() - w).abs().max().item() for g, w in zip(got_chunks, want_chunks))
    err32 = np.abs(got - want).max()
    print(f"\nACT 4/7 480x640 fp32 device vs CPU: max |d chunk| {chunk_err:.3e}, max |d action| {err32:.3e}")
    assert err32 <= 1e-4, err32
    # the rollout's fp32 path: the renderer's 8-bit space-to-depth frame, normalisation folded into
    # the stem (rmbx_stem_s2d_conv_maxpool_u8)
    assert dev32.accepts_u8_s2d
    got_u8 = [dev32(s.to(DEV), K.image_to_s2d(u[:, 0].to(DEV))[:, None]) for (s, _), u in zip(inputs, _U8[-CALLS:])]
    act_u8 = np.array(_ensemble_actions(got_u8))
    err_u8 = np.abs(act_u8 - want).max()
    print(f"ACT fp32 device (u8 stem) vs CPU: max |d action| {err_u8:.3e}")
    assert err_u8 <= 1e-4, err_u8

    del dev32
    torch.cuda.empty_cache()
    dev16 = _device_form(ref, torch.bfloat16)
    # the bench path: the renderer's space-to-depth bf16 image into the fused stem
    got16 = [dev16(s.to(DEV, torch.bfloat16), K.image_to_s2d(im[:, 0].to(DEV, torch.bfloat16))[:, None])
             for s, im in inputs]
    act16 = np.array(_ensemble_actions(got16))
    err16 = np.abs(act16 - want).max()
    rel16 = max(((g.float().cpu() - w).norm() / w.norm()).item() for g, w in zip(got16, want_chunks))
    print(f"ACT bf16 device vs CPU fp32: max |d action| {err16:.3e} (std 0.1), chunk rel-L2 {rel16:.3e}")
    assert rel16 < 5e-2, rel16
