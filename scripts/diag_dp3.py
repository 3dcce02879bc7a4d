"""Diagnostic: the DP3 inference pieces one at a time at N envs, synchronising after each."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import kernels as K  # noqa: E402
from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable  # noqa: E402
from robomanipbaselines_amd.policy.diffusion_policy_3d.rollout_diffusion_policy_3d import \
    RolloutDiffusionPolicy3d  # noqa: E402

n = int(sys.argv[1])
t0 = time.time()


def log(m):
    torch.cuda.synchronize()
    print(f"[{time.time() - t0:6.1f}s] {m}", flush=True)


class Rollout(OperationMujocoUR5eCable, RolloutDiffusionPolicy3d):
    pass


ro = Rollout(argv=["--num_envs", str(n), "--device", "cuda:0", "--precision", "bf16"])
ro.reset()
log("reset")
H, W = ro.env.renderer.height, ro.env.renderer.width
rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device="cuda:0")
depth = torch.empty((n, H, W), dtype=torch.float32, device="cuda:0")
cam = ro.camera_names[0]
ro.env.render_images(cam, rgb=rgb, depth=depth)
log("render")
rw, rh = ro.image_size
rgb_s = K.resize_crop_u8(rgb, (rw, rh), None, dtype=torch.uint8)
log("resize rgb")
depth_s = K.resize_f32(depth, (rw, rh))
log("resize depth")
d = ro.model_meta_info["data"]
pc, cnt, _ = K.pointcloud_fps(depth_s, rgb_s, ro.env.get_camera_fovy(cam), ro.num_points,
                              ro.model_meta_info["pointcloud"], d["min_bound"], d["max_bound"])
log(f"fps {tuple(pc.shape)}")
state = ro.get_state()
log("state")
pcb = pc[:, None].repeat(1, ro.n_obs_steps, 1, 1)
out = ro.policy.predict_action(state, pcb, use_graph=False)
log(f"predict eager {tuple(out.shape)}")
ro.policy.graph_max_batch = 1 << 20  # capture at this batch too
out = ro.policy.predict_action(state, pcb, use_graph=True)
log(f"predict graph {tuple(out.shape)}")
for mode in (False, True):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        ro.policy.predict_action(state, pcb, use_graph=mode)
    e1.record()
    torch.cuda.synchronize()
    log(f"predict use_graph={mode}: {e0.elapsed_time(e1) / 5:.2f} ms")
