import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv
env = BatchedMujocoUR5eCableEnv(4, "cuda:0", world_random_scale=[0.01, 0.01, 0.0])
env.modify_world(world_idx=np.arange(4) % 6)
obs, _ = env.reset()
print("obs", obs["joint_pos"][0].cpu().numpy(), "reward", env.reward.cpu().numpy())
n = env.num_envs
rgb = torch.zeros((n, 480, 640, 3), dtype=torch.uint8, device="cuda:0")
depth = torch.zeros((n, 480, 640), dtype=torch.float32, device="cuda:0")
pol = torch.zeros((n, 3, 480, 640), dtype=torch.bfloat16, device="cuda:0")
os.makedirs("gpurun_out", exist_ok=True)
for cam in ["front", "side", "hand"]:
    env.render_images(cam, rgb=rgb, depth=depth, policy=pol)
    torch.cuda.synchronize()
    img = rgb[0].cpu().numpy()
    import matplotlib; matplotlib.use("agg"); import matplotlib.pyplot as plt
    plt.imsave(f"gpurun_out/render_{cam}.png", img)
    print(cam, img.mean(axis=(0, 1)), "depth range", float(depth[0].min()), float(depth[0].max()))
for i in range(20):
    obs, r, _, _, _ = env.step(env.engine.ctrl.clone())
torch.cuda.synchronize()
print("after 20 steps t", env.get_time()[0].item(), "stats", env.engine.stats[0].cpu().numpy())
# timing physics at 1024 envs
env2 = BatchedMujocoUR5eCableEnv(1024, "cuda:0")
env2.reset()
a = env2.engine.ctrl.clone()
for _ in range(3): env2.step(a)
torch.cuda.synchronize(); t = time.time()
for _ in range(10): env2.step(a)
torch.cuda.synchronize(); dt = (time.time() - t) / 10
print(f"physics 1024 envs: {dt*1e3:.2f} ms per env-step -> {1024/dt:.0f} env-steps/s")
rgb2 = torch.zeros((1024, 480, 640, 3), dtype=torch.uint8, device="cuda:0")
pol2 = torch.zeros((1024, 3, 480, 640), dtype=torch.bfloat16, device="cuda:0")
env2.render_images("front", policy=pol2); torch.cuda.synchronize(); t = time.time()
for _ in range(3): env2.render_images("front", policy=pol2)
torch.cuda.synchronize(); dt = (time.time() - t) / 3
print(f"render 1024 envs front 640x480 policy-bf16: {dt*1e3:.2f} ms")
