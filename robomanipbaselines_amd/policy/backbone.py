"""ResNet-18 trunk with frozen batch norm (torchvision.models.resnet18 + FrozenBatchNorm2d, the
backbone of ACT's DETR (third_party/act, absent from the reference checkout) and of MlpPolicy
(policy/mlp/MlpPolicy.py:34-39)).  torchvision is not installed here, so the network is
restated; parameter names follow torchvision's (conv1, bn1, layer1.0.conv1, ...) so a reference
state_dict maps onto it.  `fuse()` folds each frozen BN into its conv for the MIOpen/MFMA
inference path (channels_last, bf16); the unfused module is the fp32 reference."""

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import kernels as K


class FrozenBatchNorm2d(nn.Module):
    """torchvision.ops.misc.FrozenBatchNorm2d: y = (x - rm) / sqrt(rv + eps) * w + b."""

    def __init__(self, n, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.register_buffer("weight", torch.ones(n))
        self.register_buffer("bias", torch.zeros(n))
        self.register_buffer("running_mean", torch.zeros(n))
        self.register_buffer("running_var", torch.ones(n))

    def scale_shift(self):
        scale = self.weight * (self.running_var + self.eps).rsqrt()
        return scale, self.bias - self.running_mean * scale

    def forward(self, x):
        s, b = self.scale_shift()
        return x * s.reshape(1, -1, 1, 1) + b.reshape(1, -1, 1, 1)


class BasicBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = FrozenBatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = FrozenBatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), FrozenBatchNorm2d(cout))

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return F.relu(y + idt)


class ResNet18Trunk(nn.Module):
    """conv1..layer4 (no avgpool/fc): [B,3,H,W] -> [B,512,H/32,W/32]."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = FrozenBatchNorm2d(64)
        self.layer1 = nn.Sequential(BasicBlock(64, 64, 1), BasicBlock(64, 64, 1))
        self.layer2 = nn.Sequential(BasicBlock(64, 128, 2), BasicBlock(128, 128, 1))
        self.layer3 = nn.Sequential(BasicBlock(128, 256, 2), BasicBlock(256, 256, 1))
        self.layer4 = nn.Sequential(BasicBlock(256, 512, 2), BasicBlock(512, 512, 1))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        x = F.max_pool2d(x, 3, 2, 1)
        return self.layer4(self.layer3(self.layer2(self.layer1(x))))


class _FusedConv(nn.Module):
    """conv + folded frozen BN.  The conv runs without bias (MIOpen, MFMA); bias, residual and
    ReLU are applied by the rmbx HIP epilogue in one pass over the output."""

    def __init__(self, conv, bn, relu):
        super().__init__()
        s, b = bn.scale_shift()
        w = conv.weight.detach() * s.reshape(-1, 1, 1, 1)
        self.conv = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding, bias=True)
        self.conv.weight.data.copy_(w)
        self.conv.bias.data.copy_(b.detach())
        self.relu = relu
        self._bias_key = None
        self._bias_f32 = None

    def conv_nobias(self, x):
        c = self.conv
        return F.conv2d(x, c.weight, None, c.stride, c.padding)

    def bias_f32(self):
        """The bias in the storage dtype, widened to f32 for the epilogue (cached)."""
        b = self.conv.bias
        key = (b.data_ptr(), b.dtype, b.device)
        if key != self._bias_key:
            self._bias_f32 = b.detach().float().contiguous()
            self._bias_key = key
        return self._bias_f32

    def forward(self, x):
        y = self.conv_nobias(x)
        return K.nhwc_bias_act(y, self.bias_f32(), relu=self.relu, out=y)

    def rmbx(self, x, relu, res=None):
        """conv + bias (+ res) (+ ReLU) in one rmbx implicit-GEMM launch (bf16, or f32 for the
        layer-1 shape)."""
        c = self.conv
        w = c.weight
        if not w.is_contiguous(memory_format=torch.channels_last):
            w = w.contiguous(memory_format=torch.channels_last)
        return K.conv2d_nhwc(x, w, self.bias_f32(), c.stride[0], c.padding[0], relu=relu, res=res)

    def rmbx_f32_ok(self):
        c = self.conv
        return K.conv2d_nhwc_f32_supported(c.in_channels, c.out_channels, c.kernel_size, c.stride[0], c.padding[0])

    def wino_ok(self):
        c = self.conv
        return (c.in_channels == c.out_channels and c.in_channels in K.WINOGRAD_F32_CHANNELS
                and tuple(c.kernel_size) == (3, 3) and c.stride[0] == 1 and c.padding[0] == 1)

    # Winograd tile of the f32 stride-1 convs: "f4" = F(4x4, 3x3) (rmbx_conv3x3_winograd4_f32: 2.25
    # instead of 4 products per output; the default: ACT call 240.5 -> 232.1 ms at 1024 envs,
    # profiles/r3_bench_f4b.json.log), "f2" = F(2x2, 3x3) (rmbx_conv3x3_winograd_f32); env
    # RMBX_WINO_TILE
    WINO_TILE = os.environ.get("RMBX_WINO_TILE", "f4")

    # the 256/512-channel stride-1 convs as the explicit Winograd F(4x4, 3x3) with the 36 position
    # GEMMs on rmbx_linear_f32x6 (kernels.conv3x3_wino4_x6); env RMBX_WINO_X6=0 keeps them on the
    # fused f32-MFMA kernel
    WINO_X6 = os.environ.get("RMBX_WINO_X6", "1") != "0"

    def wino(self, x, relu, res=None, bias=None):
        """f32 conv + bias (+ res) (+ ReLU) in one rmbx Winograd launch (or the explicit x6 form at
        256/512 channels); the packed filter transform is cached per weight storage."""
        w = self.conv.weight
        if self.WINO_X6 and w.shape[0] in K.WINO_X6_CHANNELS:
            key = (w.data_ptr(), w._version, w.device, "x6")
            cache = self.__dict__.get("_wino")
            if cache is None or cache[0] != key:
                cache = (key, K.pack_wino4_x6(w))
                self.__dict__["_wino"] = cache
            return K.conv3x3_wino4_x6(x, cache[1], self.bias_f32() if bias is None else bias, relu=relu, res=res)
        f4 = self.WINO_TILE == "f4"
        key = (w.data_ptr(), w.dtype, w.device, f4)
        cache = self.__dict__.get("_wino")
        if cache is None or cache[0] != key:
            cache = (key, K.pack_winograd4_f32(w) if f4 else K.pack_winograd_f32(w))
            self.__dict__["_wino"] = cache
        fn = K.conv3x3_winograd4_f32 if f4 else K.conv3x3_winograd_f32
        probe = _FusedConv.PROBE
        if probe is None:
            return fn(x, cache[1], self.bias_f32() if bias is None else bias, relu=relu, res=res)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn(x, cache[1], self.bias_f32() if bias is None else bias, relu=relu, res=res)
        e1.record()
        probe.append((tuple(x.shape), "f4" if f4 else "f2", e0, e1))
        return out

    def x6_ok(self):
        c = self.conv
        return (c.stride[0] == c.stride[1] and c.padding[0] == c.padding[1]
                and K.conv2d_f32x6_supported(c.in_channels, c.out_channels))

    # stride-1 3x3 convs whose output width is in this set run as the fp32-accurate implicit GEMM
    # (x6 below, f16x3 pieces) instead of the fused f32 Winograd: at 128 channels (60 x 80, 1024
    # frames) 5.1 vs 6.3 ms per conv, 18,559 vs 18,178 env-steps/s
    # (profiles/r4_bench_s1gemm128_ab.log); the 64-channel layer stays on the Winograd kernel: on
    # the GEMM's 64-column tile it is 9.1 vs 7.7 ms per conv (18,366 vs 18,826 env-steps/s,
    # profiles/r4_conv64_gemm_bn64_vs_winograd.log, r4_bench_s1gemm64_ab.log); env RMBX_S1_GEMM
    # ("" = none)
    S1_GEMM_CHANNELS = tuple(int(c) for c in os.environ.get("RMBX_S1_GEMM", "128").split(",") if c)

    def s1_gemm_ok(self):
        return (self.conv.out_channels in self.S1_GEMM_CHANNELS and K.F32_PIECES == "f16x3" and self.x6_ok())

    # stride-1 3x3 convs whose output width is in this set run on the patch-staged f16x3 conv
    # (rmbx_conv3x3_f16x3_patch: each input pixel split once per output tile instead of once per
    # tap) -- 64 channels at 120 x 160, 1024 frames: 6.86 ms vs 7.70 for the fused Winograd (and
    # 10x closer to f64); 128 channels at 60 x 80: 4.93 vs 5.34 ms for the implicit GEMM
    # (profiles/r4_conv3x3_patch_ab.log); env RMBX_S1_PATCH ("" = none)
    S1_PATCH_CHANNELS = tuple(int(c) for c in os.environ.get("RMBX_S1_PATCH", "64,128").split(",") if c)

    def s1_patch_ok(self):
        c = self.conv
        return (c.out_channels in self.S1_PATCH_CHANNELS and K.F32_PIECES == "f16x3" and c.in_channels % 32 == 0
                and c.out_channels % 64 == 0 and tuple(c.kernel_size) == (3, 3) and tuple(c.stride) == (1, 1)
                and tuple(c.padding) == (1, 1) and tuple(c.dilation) == (1, 1) and c.groups == 1)

    def x6(self, x, relu, res=None, bias=True):
        """f32 conv (+ bias) (+ res) (+ ReLU) as one fp32-accurate implicit-GEMM launch
        (rmbx_conv2d_f16x3 / rmbx_conv2d_f32x6 by kernels.F32_PIECES, epilogue fused); bias=False:
        no bias, a tensor: that bias.  The packed weight is cached per weight storage."""
        c = self.conv
        w = c.weight
        key = (w.data_ptr(), w._version, w.device)
        cache = self.__dict__.get("_x6")
        if cache is None or cache[0] != key:
            cache = (key, K.pack_conv_f32x6(w))
            self.__dict__["_x6"] = cache
        if isinstance(bias, torch.Tensor):
            b = bias
        else:
            b = self.bias_f32() if bias else None
        return K.conv2d_f32x6(x, cache[1], b, c.kernel_size, c.stride[0], c.padding[0], relu=relu, res=res)

    def s1(self, x, relu, res=None, bias=None):
        """A stride-1 3x3 conv of the f32 trunk: patch-staged f16x3 conv (s1_patch_ok), implicit
        GEMM (s1_gemm_ok) or fused Winograd."""
        if self.s1_patch_ok():
            w = self.conv.weight
            key = (w.data_ptr(), w._version, w.device)
            cache = self.__dict__.get("_x6")
            if cache is None or cache[0] != key:
                cache = (key, K.pack_conv_f32x6(w))
                self.__dict__["_x6"] = cache
            b = self.bias_f32() if bias is None else bias
            return K.conv3x3_f16x3_patch(x, cache[1], b, relu=relu, res=res)
        if self.s1_gemm_ok():
            return self.x6(x, relu, res=res, bias=True if bias is None else bias)
        return self.wino(x, relu, res=res, bias=bias)

    # bench.py's Winograd probe: a list to which wino() appends (shape, tile, HIP events around the
    # launch) on the current stream; None = no events
    PROBE = None


class _FusedBlock(nn.Module):
    def __init__(self, blk):
        super().__init__()
        self.c1 = _FusedConv(blk.conv1, blk.bn1, True)
        self.c2 = _FusedConv(blk.conv2, blk.bn2, False)
        self.down = None if blk.downsample is None else _FusedConv(blk.downsample[0], blk.downsample[1], False)

    # rmbx implicit-GEMM convs (fused epilogue) where they beat MIOpen + epilogue on MI355X
    # (scripts/prof_conv.py, profiles/r1_prof_conv_v3.log: layer1 2.7 vs 4.0 ms, layer2 2.0 vs
    # 2.6 ms per conv at 1024 envs); MIOpen's tuned solvers still win for the 256/512-channel
    # layers
    RMBX_CONV_MAX_COUT = 128

    # fp32 stride-1 3x3 convs: "winograd" (rmbx_conv3x3_winograd_f32, every layer) or "direct"
    # (layer 1 on rmbx_conv2d_nhwc_f32, layers 2-4 MIOpen + epilogue pass); env RMBX_F32_CONV
    F32_CONV = os.environ.get("RMBX_F32_CONV", "winograd")
    F32_CONV_S2 = os.environ.get("RMBX_F32_CONV_S2", "x6")

    def _bias_sum(self):
        """c2's bias + the downsample's (the residual's bias folded into c2's epilogue), cached."""
        key = (self.c2.bias_f32().data_ptr(), self.down.bias_f32().data_ptr())
        cache = self.__dict__.get("_bsum")
        if cache is None or cache[0] != key:
            cache = (key, (self.c2.bias_f32() + self.down.bias_f32()).contiguous())
            self.__dict__["_bsum"] = cache
        return cache[1]

    def forward(self, x):
        if x.dtype == torch.float32 and self.F32_CONV == "winograd" and self.c2.wino_ok():
            if self.down is None and self.c1.wino_ok():
                y = self.c1.s1(x, relu=True)
                return self.c2.s1(y, relu=True, res=x)
            if self.down is not None:
                # stride-2 c1 and the 1x1 downsample: rmbx_conv2d_f32x6 (RMBX_F32_CONV_S2 = "x6",
                # the default) or MIOpen + the epilogue pass ("miopen"); c2 (stride 1) adds the
                # downsample branch and both biases in its epilogue
                if self.F32_CONV_S2 == "x6" and self.c1.x6_ok() and self.down.x6_ok():
                    y = self.c1.x6(x, relu=True)
                    d = self.down.x6(x, relu=False, bias=False)
                else:
                    y = self.c1(x)
                    d = self.down.conv_nobias(x)
                return self.c2.s1(y, relu=True, res=d, bias=self._bias_sum())
        if x.dtype == torch.bfloat16 and self.c2.conv.out_channels <= self.RMBX_CONV_MAX_COUT:
            y = self.c1.rmbx(x, relu=True)
            idt = x if self.down is None else self.down.rmbx(x, relu=False)
            return self.c2.rmbx(y, relu=True, res=idt)
        if x.dtype == torch.float32 and self.down is None and self.c1.rmbx_f32_ok() and self.c2.rmbx_f32_ok():
            # f32 layer 1: rmbx f32 MFMA convs with the epilogue fused (the f32 MIOpen solvers
            # need a separate bias/residual/ReLU pass and a split-K zero fill per conv)
            y = self.c1.rmbx(x, relu=True)
            return self.c2.rmbx(y, relu=True, res=x)
        y = self.c1(x)
        z = self.c2.conv_nobias(y)
        if self.down is None:
            return K.nhwc_bias_act(z, self.c2.bias_f32(), res=x, relu=True, out=z)
        d = self.down.conv_nobias(x)
        return K.nhwc_bias_act(z, self.c2.bias_f32(), res=d, res_bias=self.down.bias_f32(), relu=True, out=z)


class FusedResNet18Trunk(nn.Module):
    """Inference form on the device: BN folded into conv weights/bias, channels_last
    activations.  bf16: the block convs are rmbx MFMA implicit-GEMM kernels with bias / residual /
    ReLU fused (rmbx_conv2d_nhwc); the 3-channel 7x7 stem is MIOpen + the rmbx bias/ReLU/max-pool
    epilogue.  f32: every stride-1 3x3 conv on rmbx_conv3x3_winograd_f32 (Winograd F(2x2, 3x3), epilogue
    fused; RMBX_F32_CONV=direct restores layer 1 on rmbx_conv2d_nhwc_f32), the stride-2 and 1x1
    convs MIOpen + one rmbx HIP epilogue per conv.  Same function as ResNet18Trunk; bit-identical to the unfused storage-dtype
    sequence on the same conv outputs (tests/test_nn_gpu.py)."""

    def __init__(self, trunk):
        super().__init__()
        self.stem = _FusedConv(trunk.conv1, trunk.bn1, True)
        blocks = []
        for layer in (trunk.layer1, trunk.layer2, trunk.layer3, trunk.layer4):
            blocks += [_FusedBlock(b) for b in layer]
        self.blocks = nn.Sequential(*blocks)

    def forward(self, x):
        s = self.stem.conv_nobias(x)
        return self.blocks(K.nhwc_bias_relu_maxpool(s, self.stem.bias_f32()))

    def forward_s2d_u8(self, x_u8, mean, std):
        """The f32 trunk on the renderer's 8-bit space-to-depth image [n, H/2, W/2, 16] u8
        (policy_dtype 4): the image normalisation x = (u / 255 - mean) / std is folded into the stem
        (rmbx_stem_s2d_conv_maxpool_u8: exact bf16 integer pixels x three exact bf16 pieces of
        W / (255 std), f32 accumulation, the mean term in the bias and the border edge table)."""
        w = self.stem.conv.weight
        if w.dtype != torch.float32 or w.shape[0] != 64 or x_u8.shape[2] > K.STEM_POOL_MAX_WS:
            raise ValueError("forward_s2d_u8: needs the f32 64-channel stem and Ws <= STEM_POOL_MAX_WS")
        b = self.stem.conv.bias
        key = (w.data_ptr(), w._version, b.data_ptr(), b._version, tuple(mean), tuple(std))
        if getattr(self, "_u8_key", None) != key:
            self._u8_ops = K.pack_stem_u8(w, self.stem.conv.bias, mean, std)
            self._u8_key = key
        return self.blocks(K.stem_s2d_conv_maxpool_u8(x_u8, *self._u8_ops))

    def forward_s2d(self, x_s2d):
        """Same function on the renderer's 2x2 space-to-depth image [B, H/2, W/2, 16] (bf16 or
        f32): conv + bias + ReLU + max-pool in one rmbx MFMA kernel (rmbx_stem_s2d_conv_maxpool
        / _f32); wider bf16 images: rmbx_stem_s2d_conv then the max-pool."""
        w = self.stem.conv.weight
        key = (w.data_ptr(), w.dtype)
        if getattr(self, "_s2d_key", None) != key:
            self._s2d_w = K.pack_stem_s2d(w.detach())
            self._s2d_zero = torch.zeros(w.shape[0], dtype=torch.float32, device=w.device)
            self._s2d_key = key
        if w.shape[0] == 64 and x_s2d.shape[2] <= K.STEM_POOL_MAX_WS:
            # conv + bias + ReLU + max-pool in one kernel: the full-resolution stem map stays on chip
            return self.blocks(K.stem_s2d_conv_maxpool(x_s2d, self._s2d_w, self.stem.bias_f32()))
        if x_s2d.dtype != torch.bfloat16:
            raise ValueError(f"forward_s2d: f32 images wider than {2 * K.STEM_POOL_MAX_WS} pixels are not supported")
        s = K.stem_s2d_conv(x_s2d, self._s2d_w, self.stem.bias_f32(), relu=True)
        return self.blocks(K.nhwc_bias_relu_maxpool(s, self._s2d_zero))
