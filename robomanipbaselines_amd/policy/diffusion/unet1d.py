"""ConditionalUnet1D — the denoising network of DiffusionPolicy and 3D-DiffusionPolicy.

Restates the public diffusion_policy model (diffusion_policy/model/diffusion/conditional_unet1d.py;
the reference's third_party/diffusion_policy and third_party/3D-Diffusion-Policy submodules are
absent) as the reference configures it: down_dims [512, 1024, 2048], kernel 5, 8 groups,
diffusion_step_embed_dim 128, global conditioning, FiLM (`cond_predict_scale`)
(TrainDiffusionPolicy.py:114-129, TrainDiffusionPolicy3d.py:189-200).  Module names follow the
upstream ones so its state_dict loads.  Parity vs the upstream code is unpinned (absent).

Batched over environments; under rollout the 100 (DP) / 10 (DP3) evaluations per inference are
captured with the scheduler-step kernels in one HIP graph (see dp_model.DiffusionSampler).
"""

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F


class SinusoidalPosEmb(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, x):
        half = self.dim // 2
        emb = math.log(10000) / (half - 1)
        emb = torch.exp(torch.arange(half, device=x.device) * -emb)
        emb = x[:, None] * emb[None, :]
        return torch.cat((emb.sin(), emb.cos()), dim=-1)


def _gemm(owner, name, x2, w2, bias):
    """F.linear(x2, w2, bias) with w2 derived from owner.weight; f32 on the device through
    rmbx_linear_f32x6 (fp32-accurate bf16x6 GEMM) where the shape allows, with w2's bf16 pieces
    cached on `owner` per version of owner.weight."""
    from ... import kernels as K

    if x2.is_cuda and x2.dtype == torch.float32 and K.linear_f32x6_supported(x2, w2.shape[0]):
        src = owner.weight
        key = (src.data_ptr(), src._version, tuple(w2.shape))
        cache = owner.__dict__.setdefault("_x6", {})
        ent = cache.get(name)
        if ent is None or ent[0] != key:
            ent = (key, K.pack_f32_weight(w2.detach().contiguous()))
            cache[name] = ent
        return K.linear_f32x6(x2, ent[1], bias)
    return F.linear(x2, w2, bias)


def conv1d_gemm(x, conv, rows=False):
    """Conv1d as one GEMM: the k-tap windows of x [B, C, T] (padding, stride) unfolded to
    [B*To, C*k] rows times the weight viewed [Cout, C*k] (hipBLASLt), -> [B, Cout, To].  At
    rollout batch sizes the trajectories are short (T = horizon, 16) and wide (C up to 2048), a
    shape the library GEMM runs far better than the convolution solvers."""
    k, p, st = conv.kernel_size[0], conv.padding[0], conv.stride[0]
    B, C, T = x.shape
    cols = (F.pad(x, (p, p)) if p else x).unfold(2, k, st)
    To = cols.shape[2]
    cols = cols.permute(0, 2, 1, 3).reshape(B * To, C * k)
    y = _gemm(conv, "w", cols, conv.weight.reshape(conv.out_channels, C * k), conv.bias)
    if rows:  # [B, To, Cout] as the GEMM wrote it (the caller transposes)
        return y.view(B, To, -1)
    return y.view(B, To, -1).transpose(1, 2).contiguous()


def conv_transpose1d_gemm(x, conv):
    """ConvTranspose1d(k=4, stride=2, padding=1) as one GEMM: P_k = W_kᵀ x_i for the four taps,
    then y[2m] = P_1[m] + P_3[m-1], y[2m+1] = P_2[m] + P_0[m+1] (+ bias)."""
    B, C, T = x.shape
    Co = conv.weight.shape[1]
    wk = conv.weight.permute(2, 1, 0).reshape(4 * Co, C)
    P = _gemm(conv, "wt", x.transpose(1, 2).reshape(B * T, C), wk, None).view(B, T, 4, Co)
    even = P[:, :, 1] + F.pad(P[:, :-1, 3], (0, 0, 1, 0))
    odd = P[:, :, 2] + F.pad(P[:, 1:, 0], (0, 0, 0, 1))
    y = torch.stack([even, odd], dim=2).view(B, 2 * T, Co)
    if conv.bias is not None:
        y = y + conv.bias
    return y.transpose(1, 2).contiguous()


# the fp32 device UNet's GroupNorm + Mish as one rmbx pass (RMBX_UNET_FUSED_GN=0: torch's ops)
UNET_FUSED_GN = os.environ.get("RMBX_UNET_FUSED_GN", "1") != "0"
# ... reading the conv GEMM's [B, T, C] rows (RMBX_UNET_GN_ROWS=0: after the transpose copy, in place)
UNET_GN_ROWS = os.environ.get("RMBX_UNET_GN_ROWS", "1") != "0"


def _device_form(x):
    return x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32)


def run_conv(conv, x):
    """conv(x), through the GEMM forms above on the device (bf16: hipBLASLt; f32: rmbx_linear_f32x6
    where the shape allows, else hipBLASLt -- all deterministic, so the captured denoising loop
    holds no MIOpen call)."""
    if isinstance(conv, nn.Identity) or not _device_form(x):
        return conv(x)
    if isinstance(conv, nn.ConvTranspose1d):
        assert conv.kernel_size[0] == 4 and conv.stride[0] == 2 and conv.padding[0] == 1
        return conv_transpose1d_gemm(x, conv)
    return conv1d_gemm(x, conv)


class Conv1dBlock(nn.Module):
    """Conv1d -> GroupNorm -> Mish."""

    def __init__(self, inp, out, kernel_size, n_groups=8):
        super().__init__()
        self.block = nn.Sequential(nn.Conv1d(inp, out, kernel_size, padding=kernel_size // 2),
                                   nn.GroupNorm(n_groups, out), nn.Mish())

    def forward(self, x):
        conv, norm, act = self.block
        if (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3 and norm.affine and UNET_FUSED_GN
                and norm.weight.dtype == torch.float32 and isinstance(conv, nn.Conv1d)):
            from ... import kernels as K

            # the conv GEMM's [B, T, C] rows straight into GroupNorm + Mish (rmbx_groupnorm_act), which
            # writes [B, C, T]: no transpose copy, one pass for norm + activation
            if UNET_GN_ROWS:
                rows = conv1d_gemm(x, conv, rows=True).contiguous()
                return K.groupnorm_act(rows, norm.weight, norm.bias, norm.num_groups, norm.eps, mish=True,
                                       time_major=True)
            y = run_conv(conv, x)
            return K.groupnorm_act(y, norm.weight, norm.bias, norm.num_groups, norm.eps, mish=True, out=y)
        return act(norm(run_conv(conv, x)))


class ConditionalResidualBlock1D(nn.Module):
    def __init__(self, in_channels, out_channels, cond_dim, kernel_size=3, n_groups=8, cond_predict_scale=False):
        super().__init__()
        self.blocks = nn.ModuleList([Conv1dBlock(in_channels, out_channels, kernel_size, n_groups),
                                     Conv1dBlock(out_channels, out_channels, kernel_size, n_groups)])
        cond_channels = out_channels * 2 if cond_predict_scale else out_channels
        self.cond_predict_scale = cond_predict_scale
        self.out_channels = out_channels
        self.cond_encoder = nn.Sequential(nn.Mish(), nn.Linear(cond_dim, cond_channels))
        self.residual_conv = nn.Conv1d(in_channels, out_channels, 1) if in_channels != out_channels else nn.Identity()

    def forward(self, x, cond):
        out = self.blocks[0](x)
        embed = self.cond_encoder(cond).unsqueeze(-1)
        if self.cond_predict_scale:
            embed = embed.reshape(embed.shape[0], 2, self.out_channels, 1)
            out = embed[:, 0] * out + embed[:, 1]
        else:
            out = out + embed
        out = self.blocks[1](out)
        return out + run_conv(self.residual_conv, x)


class Downsample1d(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.conv = nn.Conv1d(dim, dim, 3, 2, 1)

    def forward(self, x):
        return run_conv(self.conv, x)


class Upsample1d(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.conv = nn.ConvTranspose1d(dim, dim, 4, 2, 1)

    def forward(self, x):
        return run_conv(self.conv, x)


class ConditionalUnet1D(nn.Module):
    def __init__(self, input_dim, global_cond_dim=None, diffusion_step_embed_dim=256, down_dims=(256, 512, 1024),
                 kernel_size=3, n_groups=8, cond_predict_scale=False):
        super().__init__()
        all_dims = [input_dim] + list(down_dims)
        start_dim = down_dims[0]
        dsed = diffusion_step_embed_dim
        self.diffusion_step_encoder = nn.Sequential(SinusoidalPosEmb(dsed), nn.Linear(dsed, dsed * 4), nn.Mish(),
                                                    nn.Linear(dsed * 4, dsed))
        cond_dim = dsed + (global_cond_dim or 0)
        in_out = list(zip(all_dims[:-1], all_dims[1:]))
        mid_dim = all_dims[-1]
        kw = dict(cond_dim=cond_dim, kernel_size=kernel_size, n_groups=n_groups, cond_predict_scale=cond_predict_scale)
        self.mid_modules = nn.ModuleList([ConditionalResidualBlock1D(mid_dim, mid_dim, **kw),
                                          ConditionalResidualBlock1D(mid_dim, mid_dim, **kw)])
        self.down_modules = nn.ModuleList()
        for ind, (dim_in, dim_out) in enumerate(in_out):
            is_last = ind >= len(in_out) - 1
            self.down_modules.append(nn.ModuleList([
                ConditionalResidualBlock1D(dim_in, dim_out, **kw), ConditionalResidualBlock1D(dim_out, dim_out, **kw),
                Downsample1d(dim_out) if not is_last else nn.Identity()]))
        self.up_modules = nn.ModuleList()
        for ind, (dim_in, dim_out) in enumerate(reversed(in_out[1:])):
            is_last = ind >= len(in_out) - 1
            self.up_modules.append(nn.ModuleList([
                ConditionalResidualBlock1D(dim_out * 2, dim_in, **kw), ConditionalResidualBlock1D(dim_in, dim_in, **kw),
                Upsample1d(dim_in) if not is_last else nn.Identity()]))
        self.final_conv = nn.Sequential(Conv1dBlock(start_dim, start_dim, kernel_size=kernel_size),
                                        nn.Conv1d(start_dim, input_dim, 1))

    def forward(self, sample, timestep, global_cond=None):
        """sample [B, T, input_dim], timestep [B] (or scalar) -> [B, T, input_dim]."""
        x = sample.transpose(1, 2)
        if not torch.is_tensor(timestep):
            timestep = torch.tensor([timestep], dtype=torch.long, device=sample.device)
        elif timestep.dim() == 0:
            timestep = timestep[None].to(sample.device)
        timestep = timestep.expand(sample.shape[0])
        # the sinusoidal embedding is computed in f32 and fed to the MLP in the weights' dtype
        enc = self.diffusion_step_encoder
        g = enc[0](timestep).to(enc[1].weight.dtype)
        for m in list(enc)[1:]:
            g = m(g)
        g = g.to(sample.dtype)
        if global_cond is not None:
            g = torch.cat([g, global_cond], dim=-1)
        h = []
        for resnet, resnet2, down in self.down_modules:
            x = resnet2(resnet(x, g), g)
            h.append(x)
            x = down(x)
        for mid in self.mid_modules:
            x = mid(x, g)
        for resnet, resnet2, up in self.up_modules:
            x = torch.cat((x, h.pop()), dim=1)
            x = up(resnet2(resnet(x, g), g))
        return run_conv(self.final_conv[1], self.final_conv[0](x)).transpose(1, 2)
