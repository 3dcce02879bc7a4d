"""rmbx_resize_crop_u8 / rmbx_resize_f32 vs the numpy restatement of OpenCV INTER_LINEAR
(oracle/image.py): bit-exact on the 2x area-fast path and on the fixed-point / float bilinear
path at non-integer scales (DP3's 84x84), including ragged crops."""

import numpy as np
import pytest
import torch

from oracle import image as OI

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("size,crop", [((320, 240), (12, 16, 216, 288)), ((84, 84), (0, 0, 84, 84)),
                                       ((100, 75), (3, 5, 60, 70)), ((640, 480), (0, 0, 480, 640))])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_resize_crop_u8(size, crop, dtype):
    from robomanipbaselines_amd import kernels as K

    rng = np.random.default_rng(0)
    src = rng.integers(0, 256, (3, 480, 640, 3), dtype=np.uint8)
    got = K.resize_crop_u8(torch.from_numpy(src).to(DEV), size, crop, a=2.0, b=-1.0, dtype=dtype).cpu()
    want = np.stack([OI.policy_image(s, size, crop, 2.0, -1.0) for s in src])
    if dtype == torch.float32:
        assert np.array_equal(got.numpy(), want)
    else:
        assert torch.equal(got, torch.from_numpy(want).to(torch.bfloat16))


@pytest.mark.parametrize("size", [(320, 240), (84, 84), (97, 61)])
def test_resize_f32(size):
    from robomanipbaselines_amd import kernels as K

    rng = np.random.default_rng(1)
    src = rng.uniform(0.1, 3.0, (2, 480, 640)).astype(np.float32)
    got = K.resize_f32(torch.from_numpy(src).to(DEV), size).cpu().numpy()
    want = np.stack([OI.resize_f32(s, size) for s in src])
    assert np.array_equal(got, want)


def test_resize_u8_frame():
    from robomanipbaselines_amd import kernels as K

    rng = np.random.default_rng(2)
    src = rng.integers(0, 256, (2, 480, 640, 3), dtype=np.uint8)
    got = K.resize_crop_u8(torch.from_numpy(src).to(DEV), (84, 84), dtype=torch.uint8).cpu().numpy()
    want = np.stack([OI.resize_u8(s, (84, 84)) for s in src])
    assert np.array_equal(got, want)


def test_render_depth_bounds_do_not_change_pixels(monkeypatch):
    """The per-primitive depth bound that lets rays stop before the far walls is exact: every
    camera renders the same rgb / depth bits with it (default) as with bounding spheres only
    (RMBX_RENDER_DBG=8)."""
    import numpy as np
    import torch

    from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv

    env = BatchedMujocoUR5eCableEnv(4, "cuda:0", world_random_scale=[0.01, 0.01, 0.0])
    env.modify_world(world_idx=np.arange(4))
    env.reset()
    H, W = env.renderer.height, env.renderer.width
    for cam in env.camera_names:
        out = {}
        for dbg in ("0", "8"):
            monkeypatch.setenv("RMBX_RENDER_DBG", dbg)
            rgb = torch.empty((4, H, W, 3), dtype=torch.uint8, device="cuda:0")
            depth = torch.empty((4, H, W), dtype=torch.float32, device="cuda:0")
            env.render_images(cam, rgb=rgb, depth=depth)
            out[dbg] = (rgb, depth)
        assert torch.equal(out["0"][0], out["8"][0]), cam
        assert torch.equal(out["0"][1], out["8"][1]), cam
