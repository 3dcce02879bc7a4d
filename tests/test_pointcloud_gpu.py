"""rmbx_pointcloud_fps vs the oracle pipeline (oracle/pointcloud.py: depth -> points -> crop,
pinned by tests/golden/depth_pointcloud.npz through oracle/glue.py, then the pytorch3d FPS
restatement): selected points, normalised f32 cloud and kept count bit-exact, including the
fewer-points-than-K and empty-cloud edge cases."""

import numpy as np
import pytest
import torch

from oracle import pointcloud as OP

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
LO, HI = [-0.4, -0.4, -0.4], [1.0, 1.0, 1.0]
STATS = {"norm_config": {"type": "limits", "out_min": -1.0, "out_max": 1.0},
         "min": np.array(LO + [0.0] * 3), "range": np.array([1.4] * 3 + [1.0] * 3)}


def _scene(n, H, W, seed, far_frac=0.0):
    rng = np.random.default_rng(seed)
    d = rng.uniform(0.2, 1.3, (n, H, W)).astype(np.float32)
    d[:, :3] = 0.0  # invalid rows
    d[:, -2:, :5] = np.inf
    if far_frac:
        d[rng.uniform(size=d.shape) < far_frac] = 5.0  # cropped by the max bound
    rgb = rng.integers(0, 256, (n, H, W, 3), dtype=np.uint8)
    return d, rgb


def _run(d, rgb, K, stats=STATS):
    from robomanipbaselines_amd import kernels as K_

    out, cnt, raw = K_.pointcloud_fps(torch.from_numpy(d).to(DEV), torch.from_numpy(rgb).to(DEV), 45.0, K, stats,
                                      LO, HI, raw=True)
    return out.cpu().numpy(), cnt.cpu().numpy(), raw.cpu().numpy()


@pytest.mark.parametrize("H,W,K", [(84, 84, 512), (48, 64, 256), (17, 23, 64)])
def test_fps_matches_oracle(H, W, K):
    d, rgb = _scene(3, H, W, seed=H)
    out, cnt, raw = _run(d, rgb, K)
    for e in range(3):
        n_ref, raw_ref, c_ref = OP.observation(d[e], rgb[e], 45.0, LO, HI, K, STATS)
        assert cnt[e] == c_ref
        assert np.array_equal(raw[e], raw_ref)
        assert np.array_equal(out[e], n_ref)


def test_fps_fewer_points_than_k_and_empty():
    d, rgb = _scene(3, 32, 32, seed=5, far_frac=0.97)
    d[2] = 0.0  # env 2: no valid depth at all
    out, cnt, raw = _run(d, rgb, 128)
    for e in range(2):
        n_ref, raw_ref, c_ref = OP.observation(d[e], rgb[e], 45.0, LO, HI, 128, STATS)
        assert c_ref < 128 and cnt[e] == c_ref
        assert np.array_equal(raw[e], raw_ref)  # trailing slots repeat the last kept point
    assert cnt[2] == 0 and not out[2].any()


def test_fps_gaussian_normalisation():
    d, rgb = _scene(1, 40, 40, seed=9)
    stats = {"mean": np.array([0.1, 0.0, 0.8, 0.5, 0.5, 0.5]), "std": np.array([0.3, 0.3, 0.4, 0.2, 0.2, 0.2])}
    out, cnt, raw = _run(d, rgb, 100, stats)
    n_ref, raw_ref, _ = OP.observation(d[0], rgb[0], 45.0, LO, HI, 100, stats)
    assert np.array_equal(out[0], n_ref)
