"""DiffusionPolicy (hybrid image policy, UNet-1D, DDPM) inference, batched over environments.

Restates the inference path of diffusion_policy's DiffusionUnetHybridImagePolicy (public
upstream diffusion_policy/policy/diffusion_unet_hybrid_image_policy.py; the reference's
third_party/diffusion_policy submodule is absent) with the reference's configuration
(policy/diffusion_policy/TrainDiffusionPolicy.py:97-138): obs encoder = robomimic VisualCore per
camera (ResNet-18 conv trunk with GroupNorm(C/16) in place of BatchNorm, SpatialSoftmax with 32
keypoints, Linear 64 -> 64) on the eval centre crop, low-dim state passed through; global
conditioning on n_obs_steps (2) encoded steps; ConditionalUnet1D(down [512, 1024, 2048], k 5,
8 groups, FiLM); DDPMScheduler with 100 inference steps; action = prediction[:, To-1 : To-1+8].
The LinearNormalizer of the upstream policy is the identity here (RoboManipBaselines feeds
already-normalised data, RolloutDiffusionPolicy.py:89-105).  Parity vs upstream: unpinned.

The denoising loop (100 UNet evaluations + the rmbx_ddpm_step kernel per step) is captured once
into a HIP graph (torch.cuda.CUDAGraph) per batch size and replayed on every inference; the
initial trajectory and the per-step noise are drawn into static buffers before each replay.
"""

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..diffusion.schedulers import DDIMSampler, DDPMSampler
from ..diffusion.unet1d import ConditionalUnet1D


def _conv(conv, x):
    """conv(x) (bias-free); f32 channels_last on the device through the rmbx kernels (deterministic,
    no MIOpen Find): rmbx_conv2d_f32x6 (fp32-accurate bf16x6 implicit GEMM) where C % 32 == 0 and
    Cout % 128 == 0, the fused Winograd F(4x4) f32 kernel for the 64-channel stride-1 3x3 convs,
    rmbx_conv2d_direct_f32 for the 3-channel stem (MIOpen's only deterministic solver for it is its
    naive kernel: 4.3 s per 4096-image call); MIOpen otherwise."""
    from ... import kernels as K

    if not (x.is_cuda and x.dtype == torch.float32):
        return conv(x)
    # (torch's GroupNorm hands back NCHW-contiguous tensors: re-lay them out, a memory-bound copy)
    x = x.contiguous(memory_format=torch.channels_last)
    w = conv.weight
    key = (w.data_ptr(), w._version)
    cache = conv.__dict__.get("_rmbx")
    if K.conv2d_f32x6_supported(conv.in_channels, conv.out_channels) and conv.stride[0] == conv.stride[1]:
        if cache is None or cache[0] != key:
            cache = (key, K.pack_conv_f32x6(w))
            conv.__dict__["_rmbx"] = cache
        return K.conv2d_f32x6(x, cache[1], None, conv.kernel_size, conv.stride[0], conv.padding[0])
    if (conv.in_channels == conv.out_channels == 64 and tuple(conv.kernel_size) == (3, 3) and conv.stride[0] == 1
            and conv.padding[0] == 1):
        if cache is None or cache[0] != key:
            cache = (key, (K.pack_winograd4_f32(w), torch.zeros(64, device=w.device)))
            conv.__dict__["_rmbx"] = cache
        return K.conv3x3_winograd4_f32(x, cache[1][0], cache[1][1])
    if conv.in_channels <= 4 and conv.out_channels % 16 == 0 and conv.stride[0] == conv.stride[1] \
            and conv.padding[0] == conv.padding[1]:
        return K.conv2d_direct_f32(x, w, conv.bias, conv.stride[0], conv.padding[0])
    return conv(x)


class GNBasicBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.GroupNorm(cout // 16, cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.GroupNorm(cout // 16, cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.GroupNorm(cout // 16, cout))

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample[1](_conv(self.downsample[0], x))
        y = F.relu(self.bn1(_conv(self.conv1, x)))
        return F.relu(self.bn2(_conv(self.conv2, y)) + idt)


class ResNet18GNConv(nn.Module):
    """robomimic ResNet18Conv (torchvision resnet18 children[:-2]) with GroupNorm."""

    def __init__(self):
        super().__init__()
        layers = [nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.GroupNorm(4, 64), nn.ReLU(), nn.MaxPool2d(3, 2, 1)]
        cin = 64
        for cout, stride in ((64, 1), (128, 2), (256, 2), (512, 2)):
            layers.append(nn.Sequential(GNBasicBlock(cin, cout, stride), GNBasicBlock(cout, cout, 1)))
            cin = cout
        self.nets = nn.Sequential(*layers)

    def forward(self, x):
        stem = self.nets[0]
        x = _conv(stem, x)
        for layer in list(self.nets)[1:]:
            x = layer(x)
        return x


class SpatialSoftmax(nn.Module):
    """robomimic SpatialSoftmax(num_kp=32, temperature 1, no noise): 1x1 conv to keypoint maps,
    softmax over pixels, expected (x, y) in [-1, 1]^2 -> [B, num_kp * 2]."""

    def __init__(self, in_c, h, w, num_kp=32):
        super().__init__()
        self.nets = nn.Conv2d(in_c, num_kp, kernel_size=1)
        self.num_kp, self.h, self.w = num_kp, h, w
        px, py = np.meshgrid(np.linspace(-1.0, 1.0, w), np.linspace(-1.0, 1.0, h))
        self.register_buffer("pos_x", torch.from_numpy(px.reshape(1, h * w)).float())
        self.register_buffer("pos_y", torch.from_numpy(py.reshape(1, h * w)).float())

    def _keypoint_maps(self, f):
        """the 1x1 keypoint conv; f32 channels_last on the device: one rmbx_linear_f32x6 over the NHWC
        pixels with the 32 keypoint rows zero-padded to the kernel's 128-column tile (deterministic)."""
        from ... import kernels as K

        c = self.nets
        if not (f.is_cuda and f.dtype == torch.float32 and c.in_channels % 32 == 0):
            return c(f)
        f = f.contiguous(memory_format=torch.channels_last)
        w = c.weight
        key = (w.data_ptr(), w._version)
        cache = self.__dict__.get("_x6")
        if cache is None or cache[0] != key:
            n_pad = -(-c.out_channels // 128) * 128
            wp = torch.zeros(n_pad, c.in_channels, dtype=torch.float32, device=w.device)
            wp[: c.out_channels] = w.detach().reshape(c.out_channels, -1)
            bp = torch.zeros(n_pad, dtype=torch.float32, device=w.device)
            bp[: c.out_channels] = c.bias.detach()
            cache = (key, K.pack_f32_weight(wp), bp)
            self.__dict__["_x6"] = cache
        B, C, H, W = f.shape
        y = K.linear_f32x6(f.permute(0, 2, 3, 1), cache[1], cache[2])[..., : c.out_channels]  # [B, H, W, kp]
        return y.permute(0, 3, 1, 2)

    def forward(self, f):
        f = self._keypoint_maps(f).reshape(-1, self.h * self.w)
        att = F.softmax(f.float(), dim=-1)
        ex = torch.sum(self.pos_x * att, dim=1, keepdim=True)
        ey = torch.sum(self.pos_y * att, dim=1, keepdim=True)
        return torch.cat([ex, ey], 1).view(-1, self.num_kp * 2)


class VisualCore(nn.Module):
    def __init__(self, crop_hw, feature_dim=64, num_kp=32):
        super().__init__()
        self.backbone = ResNet18GNConv()
        h = crop_hw[0]
        w = crop_hw[1]
        for _ in range(5):
            h, w = (h + 1) // 2, (w + 1) // 2
        self.pool = SpatialSoftmax(512, h, w, num_kp)
        self.linear = nn.Linear(num_kp * 2, feature_dim)

    def forward(self, x):
        return self.linear(self.pool(self.backbone(x)).to(x.dtype))


class DiffusionPolicyModel(nn.Module):
    """predict_action(state [B, To, S], images [B, ncam, To, 3, ch, cw]) -> [B, n_action, A]."""

    def __init__(self, state_dim, action_dim, num_cams, horizon=16, n_obs_steps=2, n_action_steps=8,
                 crop_hw=(216, 288), num_inference_steps=100, down_dims=(512, 1024, 2048), kernel_size=5,
                 n_groups=8, diffusion_step_embed_dim=128, feature_dim=64, scheduler="ddpm", eps_mode=0):
        super().__init__()
        self.horizon, self.n_obs_steps, self.n_action_steps = horizon, n_obs_steps, n_action_steps
        self.action_dim, self.state_dim = action_dim, state_dim
        self.obs_nets = nn.ModuleList([VisualCore(crop_hw, feature_dim) for _ in range(num_cams)])
        self.obs_feature_dim = state_dim + num_cams * feature_dim
        self.model = ConditionalUnet1D(action_dim, self.obs_feature_dim * n_obs_steps, diffusion_step_embed_dim,
                                       down_dims, kernel_size, n_groups, cond_predict_scale=True)
        if scheduler == "ddpm":
            self.sampler = DDPMSampler(num_train_timesteps=100, num_inference_steps=num_inference_steps)
        else:
            self.sampler = DDIMSampler(num_train_timesteps=100, num_inference_steps=num_inference_steps,
                                       eps_mode=eps_mode)
        self._graphs = {}

    def encode_obs(self, state, images):
        B, To = state.shape[:2]
        feats = [state[:, :To].reshape(B * To, -1).to(self.dtype)]
        for c, net in enumerate(self.obs_nets):
            x = images[:, c, :To].reshape(B * To, *images.shape[-3:]).to(self.dtype)
            feats.append(net(x.contiguous(memory_format=torch.channels_last)))
        return torch.cat(feats, dim=-1).reshape(B, -1)

    @property
    def dtype(self):
        return self.model.final_conv[1].weight.dtype

    def _n_noise(self):
        s = self.sampler
        return int(sum(1 for c in s.coeffs if c[5])) if isinstance(s, DDPMSampler) else 0

    def _sample_loop(self, global_cond, traj, noise):
        """The conditional_sample loop: UNet evaluation + scheduler-step kernel per timestep;
        `noise[k]` is the variance noise of the k-th step with t > 0 (DDPM)."""
        s = self.sampler
        k = 0
        for i in range(len(s.timesteps)):
            out = self.model(traj.to(self.dtype), self._tsteps[i], global_cond).float().contiguous()
            if isinstance(s, DDPMSampler):
                nz = None
                if s.coeffs[i][5]:
                    nz = noise[k]
                    k += 1
                traj = s.step(i, out, traj, nz)
            else:
                traj = s.step(i, out, traj)
        return traj

    # Graph replay removes launch overhead, which matters at small batches (at 1024 envs the DP3
    # loop takes 75.0 ms eager vs 75.4 ms replayed, scripts/diag_dp3.py).  Root cause of the
    # round-1 capture crash: the f32 UNet ran its Conv1d through MIOpen, whose first call at a new
    # rollout batch searched solvers (85 s at 1024 envs) and then segfaulted inside the capture
    # (profiles/r2_dp_capture_1024_fp32_100steps_segv.log).  Every UNet conv is now a hipBLASLt
    # GEMM in both precisions (unet1d._device_form), so the loop holds no MIOpen call and captures
    # at 1024 / 2048 envs with replay == eager bit for bit (profiles/r2_dp_capture_gemm_*.log,
    # tests/test_diffusion_policy_gpu.py): no batch cap.
    graph_max_batch = None

    def conditional_sample(self, global_cond, use_graph=True, x0=None, noise=None):
        """Sample [B, horizon, A].  x0 (initial trajectory) and noise ([n_noise, B, horizon, A])
        default to fresh torch.randn draws (the reference draws them with torch.randn too)."""
        B = global_cond.shape[0]
        dev = global_cond.device
        if getattr(self, "_tsteps", None) is None or self._tsteps[0].device != dev:
            self._tsteps = [torch.tensor(int(t), device=dev) for t in self.sampler.timesteps]
        shape = (B, self.horizon, self.action_dim)
        nn_ = self._n_noise()
        if x0 is None:
            x0 = torch.randn(shape, device=dev)
        if noise is None:
            noise = torch.randn((nn_,) + shape, device=dev) if nn_ else None
        if not use_graph or dev.type != "cuda" or (self.graph_max_batch is not None and B > self.graph_max_batch):
            return self._sample_loop(global_cond, x0.contiguous(), noise)
        key = (B, self.dtype)
        if key not in self._graphs:
            gc = torch.zeros_like(global_cond)
            xb = torch.zeros(shape, device=dev)
            nb = torch.zeros((nn_,) + shape, device=dev) if nn_ else None
            self._sample_loop(global_cond, x0.contiguous(), noise)  # warm-up: solver selection outside capture
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = self._sample_loop(gc, xb, nb)
            self._graphs[key] = (g, gc, xb, nb, out)
        g, gc, xb, nb, out = self._graphs[key]
        gc.copy_(global_cond)
        xb.copy_(x0)
        if nb is not None:
            nb.copy_(noise)
        g.replay()
        return out

    @torch.no_grad()
    def predict_action(self, state, images, use_graph=True, x0=None, noise=None):
        gcond = self.encode_obs(state, images)
        traj = self.conditional_sample(gcond, use_graph, x0, noise)
        start = self.n_obs_steps - 1
        return traj[:, start:start + self.n_action_steps]
