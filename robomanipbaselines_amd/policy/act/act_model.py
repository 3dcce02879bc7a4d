"""ACT (Action Chunking with Transformers) inference network, batched over environments.

Restates the inference path of ACT's DETRVAE + ACTPolicy (third_party/act, a git submodule that
is absent from the reference checkout; public upstream: tonyzhaozh/act detr/models/detr_vae.py,
transformer.py, backbone.py, position_encoding.py) with the hyper-parameters the reference
trains it with (policy/act/TrainAct.py:46-58): hidden 512, feed-forward 3200, 8 heads,
4 encoder / 7 decoder layers (post-norm), 100 queries, ResNet-18 backbone, latent 32.
At inference the latent is zero (no VAE encoder), the image is ImageNet-normalised inside
ACTPolicy.__call__, and the DETRVAE output uses the FIRST decoder layer's normed output
(`self.transformer(...)[0]`).  Every decoder layer is still computed here (as the reference
does); `prune_dead_decoder=True` is an opt-in that skips layers 1..6, which cannot change the
output.  Parity of this restatement with the upstream code is UNPINNED (submodule absent).
"""

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..backbone import FusedResNet18Trunk, ResNet18Trunk

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def sine_pos_embed(h, w, num_pos_feats=256, temperature=10000, device=None, dtype=torch.float32):
    """PositionEmbeddingSine(normalize=True, scale=2*pi) of ACT: [1, 2*num_pos_feats, h, w]."""
    scale = 2 * math.pi
    eps = 1e-6
    ones = torch.ones(1, h, w, device=device, dtype=torch.float32)
    y_embed = ones.cumsum(1)
    x_embed = ones.cumsum(2)
    y_embed = y_embed / (y_embed[:, -1:, :] + eps) * scale
    x_embed = x_embed / (x_embed[:, :, -1:] + eps) * scale
    dim_t = torch.arange(num_pos_feats, dtype=torch.float32, device=device)
    dim_t = temperature ** (2 * (dim_t // 2) / num_pos_feats)
    pos_x = x_embed[:, :, :, None] / dim_t
    pos_y = y_embed[:, :, :, None] / dim_t
    pos_x = torch.stack((pos_x[:, :, :, 0::2].sin(), pos_x[:, :, :, 1::2].cos()), dim=4).flatten(3)
    pos_y = torch.stack((pos_y[:, :, :, 0::2].sin(), pos_y[:, :, :, 1::2].cos()), dim=4).flatten(3)
    return torch.cat((pos_y, pos_x), dim=3).permute(0, 3, 1, 2).to(dtype)


# f32 GEMMs of the fused device form: "x6" = the fp32-accurate rmbx GEMMs (kernels.pack_f32_weight:
# f16x3 by default, two f16 pieces per operand and three products; or bf16x6, three bf16 pieces and six
# products; both at the bf16 MFMA rate with f32 accumulation, the f32 GEMM error class,
# tests/test_gemm_gpu.py), "blas" = hipBLASLt f32; env RMBX_F32_GEMM
F32_GEMM = os.environ.get("RMBX_F32_GEMM", "x6")
# f32 attention products: "f16x3" = rmbx_attention_f16x3 (two f16 pieces, three products; blocks
# outside f16's range re-run as x6), "x6" = rmbx_attention_f32x6 (bf16x6 pieces), "f32" =
# rmbx_attention_f32 (f32 MFMA); env RMBX_F32_ATTN
F32_ATTN = os.environ.get("RMBX_F32_ATTN", "f16x3")


def _x6_ok(x, n_out):
    if F32_GEMM != "x6":
        return False
    from ... import kernels as K

    return K.linear_f32x6_supported(x, n_out)


def _x6_planes(owner, name, w):
    """pack_f32_weight(w) (the f16x3 or bf16x6 pieces), cached on `owner` per weight storage and version."""
    from ... import kernels as K

    key = (w.data_ptr(), w._version, tuple(w.shape))
    cache = owner.__dict__.setdefault("_x6", {})
    ent = cache.get(name)
    if ent is None or ent[0] != key:
        ent = (key, K.pack_f32_weight(w.detach().contiguous()))
        cache[name] = ent
    return ent[1]


def _x6_linear(owner, name, x, w, b, relu=False):
    from ... import kernels as K

    return K.linear_f32x6(x, _x6_planes(owner, name, w), b, relu=relu)


def _x6_linear_padded(owner, name, x, w, b):
    """F.linear(x, w, b) on rmbx_linear_f32x6 for shapes it does not take directly (N not a multiple
    of 128, K not a multiple of 32: the proprio projection 7 -> 512, the action head 512 -> 7): W and
    b zero-padded once (cached per weight storage and version), x zero-padded along K when needed,
    the first N columns returned.  fp32-accurate like the other device GEMMs, and every row's
    result is independent of the batch size (hipBLASLt chooses its algorithm by the row count, so
    its last bits vary with the number of envs)."""
    from ... import kernels as K

    N, Kd = w.shape
    Np, Kp = -(-N // 128) * 128, -(-Kd // 32) * 32
    key = (w.data_ptr(), w._version, b.data_ptr(), b._version, Np, Kp)
    cache = owner.__dict__.setdefault("_x6p", {})
    ent = cache.get(name)
    if ent is None or ent[0] != key:
        wp = torch.zeros(Np, Kp, device=w.device, dtype=torch.float32)
        wp[:N, :Kd] = w.detach()
        bp = torch.zeros(Np, device=w.device, dtype=torch.float32)
        bp[:N] = b.detach()
        ent = (key, K.pack_f32_weight(wp), bp)
        cache[name] = ent
    shp = x.shape
    x2 = x.reshape(-1, Kd)
    if Kp != Kd:
        xp = torch.zeros(x2.shape[0], Kp, device=x.device, dtype=torch.float32)
        xp[:, :Kd] = x2
        x2 = xp
    return K.linear_f32x6(x2, ent[1], ent[2])[:, :N].reshape(*shp[:-1], N)


class MHA(nn.Module):
    """nn.MultiheadAttention-compatible parameters (in_proj_weight/bias, out_proj), batch-first
    compute through scaled_dot_product_attention."""

    fused_attention = False  # device inference form: rmbx_attention_bf16 / _f32 instead of SDPA

    def __init__(self, d, heads):
        super().__init__()
        self.d, self.h = d, heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d))
        self.out_proj = nn.Linear(d, d)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)

    def _in_proj(self, x, a, b):
        """x @ in_proj_weight[a:b]^T + in_proj_bias[a:b]."""
        w, bb = self.in_proj_weight, self.in_proj_bias
        if self.fused_attention and _x6_ok(x, b - a):
            from ... import kernels as K

            return K.linear_f32x6(x, _x6_planes(self, "in_proj", w)[:, a:b], bb[a:b])
        return F.linear(x, w[a:b], bb[a:b])

    def _out_proj(self, o):
        if self.fused_attention and _x6_ok(o, self.out_proj.out_features):
            return _x6_linear(self, "out_proj", o, self.out_proj.weight, self.out_proj.bias)
        return self.out_proj(o)

    def forward(self, q, k, v):
        D = q.shape[2]
        if q is k and k is v:
            qkv = self._in_proj(q, 0, 3 * D)
            qq, kk, vv = qkv.split(D, dim=-1)
        elif q is k:
            qk = self._in_proj(q, 0, 2 * D)
            qq, kk = qk.split(D, dim=-1)
            vv = self._in_proj(v, 2 * D, 3 * D)
        else:
            qq = self._in_proj(q, 0, D)
            kk = self._in_proj(k, D, 2 * D)
            vv = self._in_proj(v, 2 * D, 3 * D)
        return self._attend(qq, kk, vv)

    def attend_kv(self, q, kk, vv):
        """forward(q, k, v) with the key / value projections kk, vv already computed (e.g. column
        slices of one GEMM shared by several layers)."""
        D = q.shape[2]
        return self._attend(self._in_proj(q, 0, D), kk, vv)

    def _attend(self, qq, kk, vv):
        B, Lq, D = qq.shape
        Lk = kk.shape[1]
        hd = D // self.h
        if self.fused_attention and qq.dtype == torch.bfloat16 and hd == 64 and Lk <= 320 and qq.is_cuda:
            from ... import kernels as K

            # rmbx_attention_bf16 reads the head slices of the projections in place and writes the
            # [B, Lq, D] layout out_proj consumes
            return self._out_proj(K.attention_bf16(qq, kk, vv, self.h))
        if self.fused_attention and qq.dtype == torch.float32 and hd == 64 and qq.is_cuda:
            from ... import kernels as K

            return self._out_proj(K.attention_f32(qq, kk, vv, self.h, form=F32_ATTN))
        qq = qq.view(B, Lq, self.h, hd).transpose(1, 2)
        kk = kk.view(B, Lk, self.h, hd).transpose(1, 2)
        vv = vv.view(B, Lk, self.h, hd).transpose(1, 2)
        o = F.scaled_dot_product_attention(qq, kk, vv)
        return self.out_proj(o.transpose(1, 2).reshape(B, Lq, D))


class _LayerOps(nn.Module):
    """Feed-forward and residual+LayerNorm of a post-norm layer.  With `fused` (device inference)
    the FFN's first Linear carries its ReLU in the GEMM epilogue (hipBLASLt bias+ReLU) and each
    residual add + LayerNorm is one rmbx_add_layernorm pass; otherwise the plain module ops."""

    fused = False

    def ffn(self, x):
        from ... import kernels as K

        sp = K.presplit_of(x) if self.fused else None
        if (sp is not None and sp.norm is not None and _x6_ok(x, self.linear1.out_features)
                and self.linear1.out_features % 128 == 0 and self.linear2.out_features % 128 == 0
                and self.linear1.out_features % K.LINEAR_F32X6_BK == 0):
            # the LayerNorm's pre-split rows in, the hidden layer kept in the pre-split form (scaled per
            # row by a Cauchy-Schwarz bound of its values): neither GEMM splits in registers
            l1, l2 = self.linear1, self.linear2
            key = (l1.weight.data_ptr(), l1.weight._version, l1.bias.data_ptr(), l1.bias._version)
            cache = self.__dict__.get("_ffn_bounds")
            if cache is None or cache[0] != key:
                cache = (key, K.weight_bounds(l1.weight, l1.bias))
                self.__dict__["_ffn_bounds"] = cache
            hs = K.linear_presplit_split(sp, _x6_planes(self, "linear1", l1.weight), l1.bias, cache[1], relu=True)
            return K.linear_presplit(hs, _x6_planes(self, "linear2", l2.weight), l2.bias).view(*x.shape[:-1], -1)
        if self.fused and _x6_ok(x, self.linear1.out_features) and self.linear2.out_features % 128 == 0:
            h = _x6_linear(self, "linear1", x, self.linear1.weight, self.linear1.bias, relu=True)
            return _x6_linear(self, "linear2", h, self.linear2.weight, self.linear2.bias)
        if self.fused:
            shp = x.shape
            h = torch._addmm_activation(self.linear1.bias, x.reshape(-1, shp[-1]), self.linear1.weight.t())
            return self.linear2(h).view(*shp[:-1], -1)
        return self.linear2(F.relu(self.linear1(x)))

    @staticmethod
    def _norm_f32(norm):
        """The LayerNorm's weight/bias widened to f32 for the rmbx kernel (cached per storage)."""
        key = (norm.weight.data_ptr(), norm.weight.dtype)
        cache = norm.__dict__.get("_f32")
        if cache is None or cache[0] != key:
            cache = (key, norm.weight.detach().float().contiguous(), norm.bias.detach().float().contiguous())
            norm.__dict__["_f32"] = cache
        return cache[1], cache[2]

    @staticmethod
    def _presplit(x):
        """Emit the LayerNorm outputs in the pre-split A form too (f32 device rows feeding f16x3
        GEMMs): the QK / V / FFN1 / cross-attention projections then load pieces instead of
        splitting in registers (kernels.add_layernorm_split, rmbx_linear_f16x3_presplit)."""
        from ... import kernels as K

        # (the pieces feed only the f16x3 GEMMs, which take K % LINEAR_F32X6_BK == 0: other widths keep
        # the plain LayerNorm and the GEMM / library path that fits them)
        return (x.dtype == torch.float32 and F32_GEMM == "x6" and K.F32_PIECES == "f16x3" and K.GEMM_PRESPLIT
                and x.is_cuda and x.shape[-1] % K.LINEAR_F32X6_BK == 0)

    def addnorm(self, norm, x, r):
        if self.fused:
            from ... import kernels as K

            w, b = self._norm_f32(norm)
            if self._presplit(x):
                return K.add_layernorm_split(x.contiguous(), r.contiguous(), w, b, norm.eps, y_norm=True)
            return K.add_layernorm(x.contiguous(), r.contiguous(), w, b, norm.eps)
        return norm(x + r)

    def addnorm_pos(self, norm, x, r, pos):
        """(y, y + pos) with y = addnorm(norm, x, r): the layer output and the next attention's
        query input, one rmbx_add_layernorm_pos pass when fused."""
        if self.fused:
            from ... import kernels as K

            w, b = self._norm_f32(norm)
            if self._presplit(x):
                # (y + pos feeds the next QK / cross-attention projections; y itself only the V
                # projection, N = 512, whose gain does not pay for writing its pieces)
                return K.add_layernorm_split(x.contiguous(), r.contiguous(), w, b, norm.eps, pos=pos.contiguous(),
                                             split_y=False)
            return K.add_layernorm_pos(x.contiguous(), r.contiguous(), w, b, pos.contiguous(), norm.eps)
        y = norm(x + r)
        return y, y + pos


class EncoderLayer(_LayerOps):
    def __init__(self, d, heads, ff):
        super().__init__()
        self.self_attn = MHA(d, heads)
        self.linear1, self.linear2 = nn.Linear(d, ff), nn.Linear(ff, d)
        self.norm1, self.norm2 = nn.LayerNorm(d), nn.LayerNorm(d)

    def forward(self, src, pos):
        q = src + pos
        src = self.addnorm(self.norm1, src, self.self_attn(q, q, src))
        return self.addnorm(self.norm2, src, self.ffn(src))

    def forward_q(self, src, q, pos, want_next_q):
        """forward() with the query input q = src + pos given, returning (out, out + pos or None)."""
        src = self.addnorm(self.norm1, src, self.self_attn(q, q, src))
        if want_next_q:
            return self.addnorm_pos(self.norm2, src, self.ffn(src), pos)
        return self.addnorm(self.norm2, src, self.ffn(src)), None


class DecoderLayer(_LayerOps):
    def __init__(self, d, heads, ff):
        super().__init__()
        self.self_attn = MHA(d, heads)
        self.multihead_attn = MHA(d, heads)
        self.linear1, self.linear2 = nn.Linear(d, ff), nn.Linear(ff, d)
        self.norm1, self.norm2, self.norm3 = nn.LayerNorm(d), nn.LayerNorm(d), nn.LayerNorm(d)

    def forward(self, tgt, memory, pos, query_pos, mem_pos=None):
        q = tgt + query_pos
        tgt = self.addnorm(self.norm1, tgt, self.self_attn(q, q, tgt))
        mk = memory + pos if mem_pos is None else mem_pos
        tgt = self.addnorm(self.norm2, tgt, self.multihead_attn(tgt + query_pos, mk, memory))
        return self.addnorm(self.norm3, tgt, self.ffn(tgt))

    def forward_q(self, tgt, q, memory, query_pos, mem_pos, want_next_q, cross_kv=None):
        """forward() with q = tgt + query_pos given; both later `+ query_pos` adds are fused into
        the LayerNorm passes that produce their operands.  cross_kv: this layer's cross-attention
        key / value projections of the memory, when computed for all layers at once.  Returns
        (out, out + query_pos or None)."""
        tgt, q2 = self.addnorm_pos(self.norm1, tgt, self.self_attn(q, q, tgt), query_pos)
        if cross_kv is not None:
            ca = self.multihead_attn.attend_kv(q2, *cross_kv)
        else:
            ca = self.multihead_attn(q2, mem_pos, memory)
        tgt = self.addnorm(self.norm2, tgt, ca)
        if want_next_q:
            return self.addnorm_pos(self.norm3, tgt, self.ffn(tgt), query_pos)
        return self.addnorm(self.norm3, tgt, self.ffn(tgt)), None


class ActModel(nn.Module):
    """DETRVAE inference path. forward(qpos [B,S], image [B,ncam,3,H,W] normalised, or the
    space-to-depth form [B,ncam,H/2,W/2,16] on the device) -> [B,Q,A]."""

    def __init__(self, state_dim=7, action_dim=7, num_queries=100, hidden_dim=512, dim_feedforward=3200,
                 nheads=8, enc_layers=4, dec_layers=7, num_cams=1, latent_dim=32):
        super().__init__()
        d = hidden_dim
        self.num_queries, self.num_cams, self.latent_dim = num_queries, num_cams, latent_dim
        self.backbone = ResNet18Trunk()
        self.input_proj = nn.Conv2d(512, d, kernel_size=1)
        self.input_proj_robot_state = nn.Linear(state_dim, d)
        self.latent_out_proj = nn.Linear(latent_dim, d)
        self.query_embed = nn.Embedding(num_queries, d)
        self.additional_pos_embed = nn.Embedding(2, d)
        self.encoder_layers = nn.ModuleList([EncoderLayer(d, nheads, dim_feedforward) for _ in range(enc_layers)])
        self.decoder_layers = nn.ModuleList([DecoderLayer(d, nheads, dim_feedforward) for _ in range(dec_layers)])
        self.decoder_norm = nn.LayerNorm(d)
        self.action_head = nn.Linear(d, action_dim)
        self.is_pad_head = nn.Linear(d, 1)
        self.prune_dead_decoder = False
        # (mean, std) the 8-bit image path folds into its stem: the normalisation the float image
        # paths receive from the renderer (ACTPolicy's ImageNet statistics; the rollout sets its own
        # image_norm here, RolloutAct.setup_policy)
        self.u8_image_norm = (IMAGENET_MEAN, IMAGENET_STD)
        self._fused = None
        self._pos_cache = {}

    def fuse_backbone(self):
        self._fused = FusedResNet18Trunk(self.backbone)
        return self

    def fuse_transformer(self, on=True):
        """Device inference form of the transformer layers (see _LayerOps)."""
        for layer in list(self.encoder_layers) + list(self.decoder_layers):
            layer.fused = on
            for m in layer.modules():
                if isinstance(m, MHA):
                    m.fused_attention = on
        return self

    batch_cross_kv = True

    def _cross_kv(self, mem_pos, mem, n_dec):
        """Device inference: the memory's cross-attention keys (from mem + pos) and values (from
        mem) of all n_dec decoder layers as two GEMMs with N = n_dec * d instead of 2 * n_dec GEMMs
        with N = d (the memory is the same for every layer); per layer, column slices of them."""
        layers = self.decoder_layers[:n_dec]
        if not self.batch_cross_kv or n_dec < 2 or not all(getattr(l, "fused", False) for l in layers):
            return None
        D = mem.shape[2]
        ws = [l.multihead_attn.in_proj_weight for l in layers]
        bs = [l.multihead_attn.in_proj_bias for l in layers]
        key = tuple((w.data_ptr(), w.dtype) for w in ws)
        cache = self.__dict__.get("_cross_w")
        if cache is None or cache[0] != key:
            wk = torch.cat([w[D: 2 * D] for w in ws]).contiguous()
            bk = torch.cat([b[D: 2 * D] for b in bs]).contiguous()
            wv = torch.cat([w[2 * D:] for w in ws]).contiguous()
            bv = torch.cat([b[2 * D:] for b in bs]).contiguous()
            cache = (key, wk, bk, wv, bv)
            self.__dict__["_cross_w"] = cache
        _, wk, bk, wv, bv = cache
        if _x6_ok(mem, wk.shape[0]):
            k_all = _x6_linear(self, "cross_k", mem_pos, wk, bk)
            v_all = _x6_linear(self, "cross_v", mem, wv, bv)
        else:
            k_all = F.linear(mem_pos, wk, bk)
            v_all = F.linear(mem, wv, bv)
        return [(k_all[..., i * D: (i + 1) * D], v_all[..., i * D: (i + 1) * D]) for i in range(n_dec)]

    def _input_proj(self, feat):
        """input_proj (1x1 conv 512 -> d) of the trunk's features; on the device in f32 with
        channels_last features it is one rmbx_linear_f32x6 over the NHWC pixels (no layout copy)."""
        c = self.input_proj
        if (self._fused is not None and feat.is_contiguous(memory_format=torch.channels_last)
                and _x6_ok(feat.permute(0, 2, 3, 1), c.out_channels)):
            y = _x6_linear(self, "input_proj", feat.permute(0, 2, 3, 1), c.weight.view(c.out_channels, -1), c.bias)
            return y.permute(0, 3, 1, 2)
        return c(feat)

    def _pos(self, h, w, device, dtype):
        key = (h, w, str(device), dtype)
        if key not in self._pos_cache:
            self._pos_cache[key] = sine_pos_embed(h, w, self.input_proj.out_channels // 2, device=device, dtype=dtype)
        return self._pos_cache[key]

    @property
    def accepts_s2d(self):
        """The device inference form also takes the renderer's space-to-depth images
        [B, ncam, H/2, W/2, 16] (bf16) and runs the stem as an rmbx MFMA kernel."""
        return self._fused is not None

    @property
    def accepts_u8_s2d(self):
        """The fp32 device form also takes the renderer's 8-bit space-to-depth images
        [B, ncam, H/2, W/2, 16] u8 and folds the ImageNet normalisation into its f32 stem kernel
        (rmbx_stem_s2d_conv_maxpool_u8); RMBX_STEM_U8=0 selects the f32 image instead."""
        return (self._fused is not None and self._fused.stem.conv.weight.dtype == torch.float32
                and os.environ.get("RMBX_STEM_U8", "1") != "0")

    def forward(self, qpos, image):
        B = qpos.shape[0]
        trunk = self._fused if self._fused is not None else self.backbone
        s2d = image.dim() == 5 and image.shape[-1] == 16
        if image.dtype == torch.uint8 and not (s2d and self._fused is not None):
            raise ValueError("ActModel: 8-bit images must be the space-to-depth form of the fused device model")
        feats, poss = [], []
        for c in range(image.shape[1]):
            x = image[:, c]
            if image.dtype == torch.uint8:
                f = self._input_proj(trunk.forward_s2d_u8(x.contiguous(), *self.u8_image_norm))
            elif s2d:
                f = self._input_proj(trunk.forward_s2d(x.contiguous()))
            else:
                if self._fused is not None:
                    x = x.contiguous(memory_format=torch.channels_last)
                f = self._input_proj(trunk(x))  # [B, d, h, w]
            feats.append(f)
            poss.append(self._pos(f.shape[2], f.shape[3], f.device, f.dtype))
        # (one camera: no concatenation copy of the feature map)
        src = (feats[0] if len(feats) == 1 else torch.cat(feats, dim=3)).flatten(2).transpose(1, 2)  # [B, hw, d]
        pos = (poss[0] if len(poss) == 1 else torch.cat(poss, dim=3)).flatten(2).transpose(1, 2)  # [1, hw, d]
        # fp32 device form: the two small linears and the final norm on rmbx kernels too, so every
        # env's chunk is bit-identical whatever the batch (tests/test_act_batch_gpu.py)
        dev_f32 = self._fused is not None and src.is_cuda and src.dtype == torch.float32 and F32_GEMM == "x6"
        latent = self.latent_out_proj(torch.zeros(B, self.latent_dim, device=qpos.device, dtype=src.dtype))
        if dev_f32:
            p = self.input_proj_robot_state
            proprio = _x6_linear_padded(self, "proprio", qpos.to(src.dtype).contiguous(), p.weight, p.bias)
        else:
            proprio = self.input_proj_robot_state(qpos.to(src.dtype))
        src = torch.cat([latent[:, None], proprio[:, None], src], dim=1)
        pos = torch.cat([self.additional_pos_embed.weight[None].to(src.dtype), pos], dim=1)
        mem = src
        # each layer's query input (x + pos) comes out of the previous LayerNorm pass (same values
        # as the separate add: the sum of the rounded layer output and pos, rounded once)
        q = src + pos
        n_enc = len(self.encoder_layers)
        for i, layer in enumerate(self.encoder_layers):
            # the last layer's (out, out + pos) pass also yields the decoder's memory keys mem + pos
            mem, q = layer.forward_q(mem, q, pos, want_next_q=True)
        qe = self.query_embed.weight[None].to(src.dtype)
        tgt = torch.zeros(B, self.num_queries, mem.shape[2], device=mem.device, dtype=mem.dtype)
        mem_pos = q if q is not None else mem + pos
        q = tgt + qe
        first = None
        n_dec = 1 if self.prune_dead_decoder else len(self.decoder_layers)
        cross = self._cross_kv(mem_pos, mem, n_dec)
        for i in range(n_dec):
            tgt, q = self.decoder_layers[i].forward_q(tgt, q, mem, qe, mem_pos, want_next_q=i + 1 < n_dec,
                                                      cross_kv=cross[i] if cross else None)
            if i == 0:
                # intermediate[0] = norm(output of layer 0)
                if dev_f32:
                    from ... import kernels as K

                    w, b = _LayerOps._norm_f32(self.decoder_norm)
                    first = K.add_layernorm(tgt.contiguous(), None, w, b, self.decoder_norm.eps)
                else:
                    first = self.decoder_norm(tgt)
        if dev_f32:
            h = self.action_head
            return _x6_linear_padded(self, "action_head", first.contiguous(), h.weight, h.bias)
        return self.action_head(first)


def normalize_images(image):
    """transforms.Normalize(ImageNet) of ACTPolicy.__call__ on [B, ncam, 3, H, W] in [0, 1]."""
    m = torch.tensor(IMAGENET_MEAN, device=image.device, dtype=image.dtype).reshape(1, 1, 3, 1, 1)
    s = torch.tensor(IMAGENET_STD, device=image.device, dtype=image.dtype).reshape(1, 1, 3, 1, 1)
    return (image - m) / s
