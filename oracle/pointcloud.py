"""TEST INFRASTRUCTURE ONLY (the oracle; never imported by the product path).

The 3D diffusion policy's observation pipeline (RolloutDiffusionPolicy3d.get_pointcloud,
policy/diffusion_policy_3d/RolloutDiffusionPolicy3d.py:132-160) on already-resized images:
convert_depth_image_to_pointcloud + crop_pointcloud_bb (restated in oracle/glue.py and pinned by
tests/golden/depth_pointcloud.npz), then downsample_pointcloud_fps (Vision3dUtils.py:17-25), whose
algorithm lives in pytorch3d (absent here; not pinned in pyproject): sample_farthest_points
converts the points to float32 and runs its CPU loop from start index 0 - squared distances
accumulated in f32 over every channel, running minimum, strict-greater argmax starting from
(0, index 0); indices beyond the number of points stay -1, which the reference then applies as
a NumPy index (the last point).  Parity of this FPS restatement vs pytorch3d: UNPINNED.
"""

import numpy as np

from . import glue


def fps_indices(points, K):
    """pytorch3d sample_farthest_points (CPU), one cloud: points [P, D] -> int64 [K]."""
    pts = np.asarray(points, dtype=np.float32)
    P = pts.shape[0]
    idx = np.full(K, -1, dtype=np.int64)
    dists = np.full(P, np.finfo(np.float32).max, dtype=np.float32)
    sel = 0
    for k in range(min(K, P)):
        idx[k] = sel
        diff = pts[sel][None, :] - pts  # f32
        d2 = np.zeros(P, dtype=np.float32)
        for d in range(pts.shape[1]):  # accumulation order over channels
            d2 = d2 + diff[:, d] * diff[:, d]
        dists = np.minimum(d2, dists)
        m = dists.max() if P else 0
        sel = int(np.argmax(dists)) if m > 0 else 0
    return idx


def observation(depth, rgb, fovy, min_bound, max_bound, K, stats):
    """depth f32 [H, W], rgb u8 [H, W, 3] -> (normalised f32 [K, 6], raw f64 [K, 6], count)."""
    xyz, col = glue.depth_to_pointcloud(depth, fovy, rgb)
    pc = np.concatenate((xyz, col), axis=1)
    pc = glue.crop_bb(pc, np.asarray(min_bound), np.asarray(max_bound))
    idx = fps_indices(pc, K)
    raw = pc[idx]
    t = stats["norm_config"]["type"] if "norm_config" in stats else "gaussian"
    if t == "gaussian":
        norm = (raw - stats["mean"]) / stats["std"]
    else:
        cfg = stats["norm_config"]
        scale = (cfg["out_max"] - cfg["out_min"]) / stats["range"]
        norm = scale * (raw - stats["min"]) + cfg["out_min"]
    return norm.astype(np.float32), raw, pc.shape[0]
