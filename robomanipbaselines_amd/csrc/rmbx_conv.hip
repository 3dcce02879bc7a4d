// Implicit-GEMM convolution with a fused epilogue for the policy vision trunk (bf16, NHWC),
// MFMA 32x32x16 on gfx950.
//
// Replaces the conv -> FrozenBN -> (+ residual) -> ReLU sequence of the ResNet-18 BasicBlocks of
// the reference's backbones (torchvision resnet18 inside ACT's DETR, third_party/act [absent];
// policy/mlp/MlpPolicy.py:34-39) for the 3x3 (stride 1/2) and 1x1 (stride 2) convolutions: BN is
// folded into the weights on the host, and bias, residual add and ReLU are applied to the f32
// accumulators before the single bf16 store, so the activation makes one HBM round trip per
// conv instead of four.
//
// GEMM view: M = N*Ho*Wo output pixels, N = Cout, K = KH*KW*Cin ordered (tap, channel), so
// every K step of 64 is one filter tap over 64 contiguous input channels (16-byte loads of NHWC
// rows; out-of-image taps read zeros).  Block tile 128 pixels x 64 channels, 4 waves, each wave
// 32 pixels x 64 channels = two 32x32 accumulator tiles; A/B staged global -> registers -> LDS
// (rows padded to 72 bf16 against bank conflicts) with the next K step's loads in flight while
// the current one is multiplied.  Consecutive blocks walk the Cout tiles of one pixel tile, so
// the input tile is reused from L2; pixel tiles are spread over the 8 XCDs in contiguous ranges.

#include "rmbx_common.h"

#include <cstdint>
#include <cstdlib>

namespace rmbx {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int CBM = 128, CBN = 64, CBK = 64, CLD = CBK + 8;

struct ConvArgs {
  const uint16_t* in;   // [N][H][W][Cin]
  const uint16_t* w;    // [Cout][KH][KW][Cin]
  const float* bias;    // [Cout]
  const uint16_t* res;  // [N][Ho][Wo][Cout] or null
  uint16_t* out;        // [N][Ho][Wo][Cout]
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, relu;
  long long M;
  int n_ntiles;         // Cout / CBN
  int dbg;              // diagnostic phase skips (RMBX_CONV_DBG; 0 in production)
  long long n_mtiles;
};

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// bias (+ residual) (+ ReLU) on 8 consecutive channels of one pixel, rounded once to bf16
__device__ __forceinline__ uint4 epi_finish8(const float* c, const float* bv, uint4 rv, bool res, bool relu) {
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = c[k] + bv[k];
  if (res) {
    const uint32_t w4[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] += bf2f((uint16_t)(w4[k] & 0xffff));
      v[2 * k + 1] += bf2f((uint16_t)(w4[k] >> 16));
    }
  }
  if (relu)
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = v[k] > 0.f ? v[k] : 0.f;
  uint4 ov;
  ov.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  ov.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  ov.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
  ov.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
  return ov;
}

// MODE 0: KH x KW conv over [N][H][W][Cin], K step = one tap x 64 channels.
// MODE 1: the ResNet stem (7x7 / stride 2 / pad 3 over 3 channels) on a 2x2 space-to-depth
//   image [N][H/2][W/2][16] (channel (dy*2+dx)*3+c, 12..15 zero): a 4x4 / stride 1 conv with
//   pad 2 (before) whose K step is one filter row ky = 4 taps x 16 channels, i.e. the 64
//   contiguous values of s2d pixels X = ox-2 .. ox+1 of row Y = oy+ky-2; weights packed
//   [Cout][ky][kx][16] on the host.
constexpr int EPI_LD = 68;  // f32 row stride of the epilogue image [128 pixels][64 channels]
constexpr int GEN_LDS = (CBM * CLD + CBN * CLD) > (CBM * EPI_LD * 2) ? (CBM * CLD + CBN * CLD) : (CBM * EPI_LD * 2);

// epilogue shared by the conv kernels: the 128 x 64 f32 accumulator tile is written to LDS as
// [pixel][channel], then each thread finishes 8 consecutive channels of a pixel (bias, residual,
// ReLU) with 16-byte NHWC loads/stores.  out_off(pix) = element offset of the pixel's channel 0
// (or -1 when outside the output).
template <class OFF>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, float* sC, const f32x16& acc0, const f32x16& acc1,
                                              int n0, OFF out_off) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int row = 32 * wave + (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
    sC[row * EPI_LD + col] = acc0[j];
    sC[row * EPI_LD + 32 + col] = acc1[j];
  }
  __syncthreads();
  // this thread's 8 channels are the same in every pass (256 is a multiple of 8): bias once, and
  // all residual loads in flight before the first store
  const int c8 = (tid & 7) * 8;
  float bv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) bv[k] = a.bias[n0 + c8 + k];
  long long base[4];
  uint4 rv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    base[i] = out_off((tid + 256 * i) >> 3);
    rv[i] = (a.res && base[i] >= 0) ? *reinterpret_cast<const uint4*>(a.res + (size_t)base[i] + n0 + c8)
                                    : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (base[i] < 0) continue;
    const int pix = (tid + 256 * i) >> 3;
    *reinterpret_cast<uint4*>(a.out + (size_t)base[i] + n0 + c8) =
        epi_finish8(sC + pix * EPI_LD + c8, bv, rv[i], a.res != nullptr, a.relu != 0);
  }
}

template <int MODE>
__global__ void __launch_bounds__(256) conv_nhwc_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[GEN_LDS];
  uint16_t* sA = smem;
  uint16_t* sB = smem + CBM * CLD;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // block -> (pixel tile, channel tile); pixel tiles in contiguous ranges per XCD
  const long long nblk = (long long)gridDim.x;
  long long b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const long long mt = b / a.n_ntiles;
  const int nt = (int)(b - mt * a.n_ntiles);
  const long long m0 = mt * CBM;
  const int n0 = nt * CBN;

  // A loader: 128 pixels x 64 ch = 1024 16-byte chunks, 4 per thread (pixel = q >> 3, part = q & 7)
  int pn[4], ph[4], pw[4];
  bool pv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + 256 * i;
    const long long m = m0 + (q >> 3);
    pv[i] = m < a.M;
    const long long mm = pv[i] ? m : 0;
    const int wo = (int)(mm % a.Wo);
    const long long t = mm / a.Wo;
    const int ho = (int)(t % a.Ho);
    pn[i] = (int)(t / a.Ho);
    ph[i] = ho * a.stride - a.pad;
    pw[i] = wo * a.stride - a.pad;
  }
  const int cchunks = a.Cin / CBK;
  const int KT = a.KH * a.KW * cchunks;

  uint4 ra0, ra1, ra2, ra3, rb0, rb1;
  int kh_ = 0, kw_ = 0, c0_ = 0;
#define RMBX_A_LOAD(I, DST)                                                                              \
  if (MODE == 0) {                                                                                       \
    const int h_ = ph[I] + kh_, w_ = pw[I] + kw_;                                                        \
    DST = (pv[I] && h_ >= 0 && h_ < a.H && w_ >= 0 && w_ < a.W)                                          \
              ? *reinterpret_cast<const uint4*>(a.in + (((size_t)pn[I] * a.H + h_) * a.W + w_) * a.Cin + c0_ + \
                                                ((tid + 256 * (I)) & 7) * 8)                             \
              : make_uint4(0, 0, 0, 0);                                                                  \
  } else {                                                                                               \
    const int part_ = (tid + 256 * (I)) & 7;                                                             \
    const int h_ = ph[I] + kh_, w_ = pw[I] + (part_ >> 1);                                               \
    DST = (pv[I] && h_ >= 0 && h_ < a.H && w_ >= 0 && w_ < a.W)                                          \
              ? *reinterpret_cast<const uint4*>(a.in + (((size_t)pn[I] * a.H + h_) * a.W + w_) * 16 +    \
                                                (part_ & 1) * 8)                                         \
              : make_uint4(0, 0, 0, 0);                                                                  \
  }
#define RMBX_B_LOAD(I, DST)                                                                              \
  {                                                                                                      \
    const int q_ = tid + 256 * (I);                                                                      \
    DST = *reinterpret_cast<const uint4*>(a.w + (((size_t)(n0 + (q_ >> 3)) * a.KH + kh_) * a.KW + kw_) * a.Cin + \
                                          c0_ + (q_ & 7) * 8);                                           \
  }
#define RMBX_CONV_LOAD(KT)                    \
  {                                           \
    const int tap_ = (KT) / cchunks;          \
    c0_ = ((KT) - tap_ * cchunks) * CBK;      \
    kh_ = tap_ / a.KW;                        \
    kw_ = tap_ - kh_ * a.KW;                  \
    RMBX_A_LOAD(0, ra0)                       \
    RMBX_A_LOAD(1, ra1)                       \
    RMBX_A_LOAD(2, ra2)                       \
    RMBX_A_LOAD(3, ra3)                       \
    RMBX_B_LOAD(0, rb0)                       \
    RMBX_B_LOAD(1, rb1)                       \
  }
#define RMBX_ST(BUF, I, V) *reinterpret_cast<uint4*>(BUF + ((tid + 256 * (I)) >> 3) * CLD + ((tid + 256 * (I)) & 7) * 8) = V;

  f32x16 acc0 = {}, acc1 = {};
  RMBX_CONV_LOAD(0)
  for (int kt = 0; kt < KT; ++kt) {
    __syncthreads();
    RMBX_ST(sA, 0, ra0)
    RMBX_ST(sA, 1, ra1)
    RMBX_ST(sA, 2, ra2)
    RMBX_ST(sA, 3, ra3)
    RMBX_ST(sB, 0, rb0)
    RMBX_ST(sB, 1, rb1)
    __syncthreads();
    if (kt + 1 < KT) RMBX_CONV_LOAD(kt + 1)
    const int r = lane & 31, h8 = 8 * (lane >> 5);
    const uint16_t* arow = sA + (32 * wave + r) * CLD + h8;
    const uint16_t* brow0 = sB + r * CLD + h8;
    const uint16_t* brow1 = sB + (32 + r) * CLD + h8;
#pragma unroll
    for (int ks = 0; ks < CBK / 16; ++ks) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(arow + 16 * ks);
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(brow0 + 16 * ks);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(brow1 + 16 * ks);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b1, acc1, 0, 0, 0);
    }
  }
#undef RMBX_ST
#undef RMBX_A_LOAD
#undef RMBX_B_LOAD

  conv_epilogue(a, reinterpret_cast<float*>(smem), acc0, acc1, n0, [&](int pix) -> long long {
    const long long m = m0 + pix;
    return m < a.M ? m * a.Cout : -1;
  });
}
#undef RMBX_CONV_LOAD


// 3x3 / stride 1 / pad 1 conv with Cin = 64 k (the ResNet-18 stride-1 block convs): the block's
// output tile is 8 rows x 16 columns of one image; per 64-channel chunk its 10 x 18 input patch
// is loaded into LDS once and all 9 taps read their A fragments from it (the row-tiled kernel
// re-reads the input once per tap); weights stream per tap through a small LDS tile (keeping the
// block at 35 KiB of LDS, 4 blocks per CU).  The next chunk's patch is loaded into registers with
// all of its loads in flight together while the current chunk is multiplied.  Wave w owns output
// rows 2w, 2w+1.  The epilogue transposes the accumulators through LDS so bias, residual and ReLU
// are applied on 16-byte NHWC chunks.
constexpr int PT_H = 8, PT_W = 16, PP_H = PT_H + 2, PP_W = PT_W + 2, PLD = 72;
constexpr int P_CHUNKS = PP_H * PP_W * 8;                 // 16-byte chunks of one patch
constexpr int P_PER_THREAD = (P_CHUNKS + 255) / 256;      // 6
constexpr int PATCH_LDS = PP_H * PP_W * PLD + CBN * CLD;  // bf16 elements
static_assert(PATCH_LDS >= CBM * EPI_LD * 2, "epilogue image must fit the patch + B tiles");

__global__ void __launch_bounds__(256) conv3x3_c64_patch_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[PATCH_LDS];
  uint16_t* sP = smem;
  uint16_t* sB = smem + PP_H * PP_W * PLD;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_x = (a.Wo + PT_W - 1) / PT_W, tiles_y = (a.Ho + PT_H - 1) / PT_H;
  const long long nblk = (long long)gridDim.x;
  long long b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const int nt = (int)(b % a.n_ntiles);
  long long t = b / a.n_ntiles;
  const int tx = (int)(t % tiles_x);
  t /= tiles_x;
  const int ty = (int)(t % tiles_y);
  const int n = (int)(t / tiles_y);
  const int oy0 = ty * PT_H, ox0 = tx * PT_W, n0 = nt * CBN;

  const int r = lane & 31, h8 = 8 * (lane >> 5);
  // this lane's A row = output pixel (ly, lx); row 1 rotated by 2 columns (bank-conflict-free
  // ds_read_b128 groups with the 18-pixel patch pitch, see conv3x3_c64_resident_kernel)
  const int ly = 2 * wave + (r >> 4), lx = r < 16 ? r : ((r - 2) & 15);
  f32x16 acc0 = {}, acc1 = {};
  uint4 rb0, rb1;
  const int Cin = a.Cin;
  auto ldb = [&](int kk, uint4& x0, uint4& x1) {  // kk = chunk * 9 + tap
    const int ch = kk / 9, tap = kk - 9 * ch;
    const int kh = tap / 3, kw = tap - 3 * kh;
    const int q0 = tid, q1 = tid + 256;
    x0 = *reinterpret_cast<const uint4*>(a.w + (((size_t)(n0 + (q0 >> 3)) * 3 + kh) * 3 + kw) * Cin + 64 * ch + (q0 & 7) * 8);
    x1 = *reinterpret_cast<const uint4*>(a.w + (((size_t)(n0 + (q1 >> 3)) * 3 + kh) * 3 + kw) * Cin + 64 * ch + (q1 & 7) * 8);
  };
  // input patch rows oy0-1 .. oy0+8, cols ox0-1 .. ox0+16 of chunk ch (zero outside the image)
  uint4 pr[P_PER_THREAD];
  auto ldp = [&](int ch) {
#pragma unroll
    for (int i = 0; i < P_PER_THREAD; ++i) {
      const int q = tid + 256 * i;
      const int pix = q >> 3, part = q & 7;
      const int py = pix / PP_W, px = pix - py * PP_W;
      const int h = oy0 - 1 + py, w = ox0 - 1 + px;
      const bool ok = q < P_CHUNKS && h >= 0 && h < a.H && w >= 0 && w < a.W;
      pr[i] = *reinterpret_cast<const uint4*>(a.in + (ok ? (((size_t)n * a.H + h) * a.W + w) * Cin + 64 * ch + part * 8 : 0));
      if (!ok) pr[i] = make_uint4(0, 0, 0, 0);
    }
  };
  const int KK = 9 * (Cin / 64);
  ldp(0);
  ldb(0, rb0, rb1);
  for (int kk = 0; kk < KK; ++kk) {
    const int tap = kk % 9;
    __syncthreads();
    if (tap == 0) {
#pragma unroll
      for (int i = 0; i < P_PER_THREAD; ++i) {
        const int q = tid + 256 * i;
        if (q < P_CHUNKS) *reinterpret_cast<uint4*>(sP + (q >> 3) * PLD + (q & 7) * 8) = pr[i];
      }
      if (kk + 9 < KK) ldp(kk / 9 + 1);
    }
    *reinterpret_cast<uint4*>(sB + (tid >> 3) * CLD + (tid & 7) * 8) = rb0;
    *reinterpret_cast<uint4*>(sB + ((tid + 256) >> 3) * CLD + (tid & 7) * 8) = rb1;
    __syncthreads();
    if (kk + 1 < KK) ldb(kk + 1, rb0, rb1);
    const int kh = tap / 3, kw = tap - 3 * kh;
    const uint16_t* arow = sP + ((ly + kh) * PP_W + (lx + kw)) * PLD + h8;
    const uint16_t* brow0 = sB + r * CLD + h8;
    const uint16_t* brow1 = sB + (32 + r) * CLD + h8;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(arow + 16 * ks);
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(brow0 + 16 * ks);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(brow1 + 16 * ks);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b1, acc1, 0, 0, 0);
    }
  }
  conv_epilogue(a, reinterpret_cast<float*>(smem), acc0, acc1, n0, [&](int pix) -> long long {
    const int m = pix & 31;  // epilogue row 32 * wave + m = A row m of wave pix >> 5
    const int oy = oy0 + 2 * (pix >> 5) + (m >> 4), ox = ox0 + (m < 16 ? m : ((m - 2) & 15));
    return (oy < a.Ho && ox < a.Wo) ? ((((long long)n * a.Ho + oy) * a.Wo + ox) * a.Cout) : -1;
  });
}

// 3x3 / stride 1 / pad 1 conv with Cin = Cout = 64 (ResNet-18 layer1, the trunk's widest
// activations): the whole filter bank (9 taps x 64 x 64 bf16 = 72 KiB) stays resident in LDS for
// the life of a persistent block (one per CU) that walks a contiguous range of 8 x 32 output
// tiles.  Per tile only the 10 x 34 x 64 input patch moves (prefetched into registers while the
// previous tile is multiplied), so the L2 -> CU traffic per MFMA drops ~5x against the per-block
// weight streaming of conv3x3_c64_patch_kernel.  8 waves (2 per SIMD); wave w owns output row w
// of the tile (32 pixels x 64 channels = two 32x32 accumulators) and reads its A fragments for all
// 9 taps from the patch (8 x 32 tiles divide the 120 x 160 layer-1 map exactly).  The f32 epilogue image aliases the patch.
constexpr int RTH = 8, RTW = 32, RPH = RTH + 2, RPW = RTW + 2, RTHREADS = 512;
constexpr int RW_LDS = 9 * 64 * CLD;  // bf16 elements, [tap][cout][CLD]
constexpr int EPI_LDR = 72;  // f32 epilogue row stride: the two half-waves' ds_write_b32 hit disjoint banks
constexpr int RU_LDS = (RTH * RTW * EPI_LDR * 2 > RPH * RPW * PLD) ? RTH * RTW * EPI_LDR * 2 : RPH * RPW * PLD;
constexpr int RPATCH_CHUNKS = RPH * RPW * 8;
constexpr int RPATCH_PER_THREAD = (RPATCH_CHUNKS + RTHREADS - 1) / RTHREADS;
static_assert((RW_LDS + RU_LDS) * 2 <= 160 * 1024, "resident conv must fit the 160 KiB LDS");

__global__ void __launch_bounds__(RTHREADS) conv3x3_c64_resident_kernel(ConvArgs a, int tiles_x, int tiles_y,
                                                                         long long ntiles) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[RW_LDS + RU_LDS];
  uint16_t* sW = smem;
  uint16_t* sP = smem + RW_LDS;
  float* sC = reinterpret_cast<float*>(sP);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // filter bank [cout][kh][kw][c] -> sW[tap][cout][c]
  for (int q = tid; q < 9 * 64 * 8; q += RTHREADS) {
    const int part = q & 7, rest = q >> 3;  // rest = cout * 9 + tap
    const int co = rest / 9, tap = rest - 9 * co;
    *reinterpret_cast<uint4*>(sW + (tap * 64 + co) * CLD + part * 8) =
        *reinterpret_cast<const uint4*>(a.w + (size_t)rest * 64 + part * 8);
  }
  const long long t_begin = ntiles * blockIdx.x / gridDim.x;
  const long long t_end = ntiles * (blockIdx.x + 1) / gridDim.x;
  const int c8 = (tid & 7) * 8;  // this thread's epilogue channels (fixed: 512 % 8 == 0)
  float bv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) bv[k] = a.bias[c8 + k];
  const int r = lane & 31, h8 = 8 * (lane >> 5);
  // A row r -> output pixel (wave, r): 32 consecutive patch pixels at a 144-byte pitch, so every
  // 16-lane ds_read_b128 group touches 16 distinct 4-bank quads
  const int ly = wave, lx = r;
  uint4 pr[RPATCH_PER_THREAD];
  constexpr int EPASS = RTH * RTW * 8 / RTHREADS;  // epilogue 16-byte chunks per thread per tile
  uint4 rres[EPASS];                               // residual chunks of the current tile
#pragma unroll
  for (int i = 0; i < EPASS; ++i) rres[i] = make_uint4(0, 0, 0, 0);

#define RMBX_RES_TILE(T, N_, OY0, OX0)                     \
  {                                                        \
    long long t_ = (T);                                    \
    const int tx_ = (int)(t_ % tiles_x);                   \
    t_ /= tiles_x;                                         \
    OY0 = (int)(t_ % tiles_y) * RTH;                       \
    N_ = (int)(t_ / tiles_y);                              \
    OX0 = tx_ * RTW;                                       \
  }
#define RMBX_RES_LOAD(T)                                                                               \
  {                                                                                                    \
    int n_, oy0_, ox0_;                                                                                \
    RMBX_RES_TILE(T, n_, oy0_, ox0_)                                                                   \
    _Pragma("unroll") for (int i = 0; i < RPATCH_PER_THREAD; ++i) {                                    \
      const int q = tid + RTHREADS * i;                                                                \
      const int pix = q >> 3, part = q & 7;                                                            \
      const int py = pix / RPW, px = pix - py * RPW;                                                   \
      const int h = oy0_ - 1 + py, w = ox0_ - 1 + px;                                                  \
      pr[i] = (q < RPATCH_CHUNKS && h >= 0 && h < a.H && w >= 0 && w < a.W)                            \
                  ? *reinterpret_cast<const uint4*>(a.in + (((size_t)n_ * a.H + h) * a.W + w) * 64 + part * 8) \
                  : make_uint4(0, 0, 0, 0);                                                            \
    }                                                                                                  \
  }

  const int dbg = a.dbg;
#define RMBX_RESID_LOAD(T)                                                                             \
  if (a.res) {                                                                                         \
    int n_, oy0_, ox0_;                                                                                \
    RMBX_RES_TILE(T, n_, oy0_, ox0_)                                                                   \
    _Pragma("unroll") for (int i = 0; i < EPASS; ++i) {                                                \
      const int pix = (tid + RTHREADS * i) >> 3;                                                       \
      const int oy = oy0_ + (pix >> 5), ox = ox0_ + (pix & 31);                                        \
      if (oy < a.Ho && ox < a.Wo)                                                                      \
        rres[i] = *reinterpret_cast<const uint4*>(a.res + (((size_t)n_ * a.Ho + oy) * a.Wo + ox) * 64 + c8); \
    }                                                                                                  \
  }
  if (t_begin < t_end && !(dbg & 4)) {
    RMBX_RES_LOAD(t_begin)
    RMBX_RESID_LOAD(t_begin)
  }
  // finished bf16 chunks of the previous tile: stored only after the next patch is in LDS, so
  // the vmcnt wait in front of a patch store never waits on the output stores just issued
  uint4 ov[EPASS];
  int pn = -1, poy0 = 0, pox0 = 0;  // tile whose chunks are pending in ov (pn < 0: none)
#define RMBX_RES_STORE()                                                                               \
  if (pn >= 0) {                                                                                       \
    _Pragma("unroll") for (int i = 0; i < EPASS; ++i) {                                                \
      const int pix = (tid + RTHREADS * i) >> 3;                                                       \
      const int oy = poy0 + (pix >> 5), ox = pox0 + (pix & 31);                                        \
      if (oy < a.Ho && ox < a.Wo)                                                                      \
        *reinterpret_cast<uint4*>(a.out + (((size_t)pn * a.Ho + oy) * a.Wo + ox) * 64 + c8) = ov[i];   \
    }                                                                                                  \
  }
  for (long long t = t_begin; t < t_end; ++t) {
    int n, oy0, ox0;
    RMBX_RES_TILE(t, n, oy0, ox0)
    __syncthreads();  // previous epilogue done with the aliased region (and sW written)
#pragma unroll
    for (int i = 0; i < RPATCH_PER_THREAD; ++i) {
      const int q = tid + RTHREADS * i;
      if (q < RPATCH_CHUNKS) *reinterpret_cast<uint4*>(sP + (q >> 3) * PLD + (q & 7) * 8) = pr[i];
    }
    __syncthreads();
    RMBX_RES_STORE()
    if (t + 1 < t_end && !(dbg & 4)) RMBX_RES_LOAD(t + 1)
    f32x16 acc0 = {}, acc1 = {};
    if (!(dbg & 1)) {
    // A/B fragments double-buffered in registers by half-tap groups (2 k-steps: 6 LDS reads,
    // 4 MFMAs): group g + 1's reads are in flight while group g multiplies
    bf16x8 fa[2][2], fb0[2][2], fb1[2][2];
#define RMBX_RES_FRAGS(BUF, G)                                                                     \
  {                                                                                                \
    const int tap_ = (G) >> 1, k0_ = 32 * ((G) & 1);                                               \
    const int kh_ = tap_ / 3, kw_ = tap_ - 3 * kh_;                                                \
    const uint16_t* arow_ = sP + ((ly + kh_) * RPW + (lx + kw_)) * PLD + h8 + k0_;                 \
    const uint16_t* brow_ = sW + (tap_ * 64 + r) * CLD + h8 + k0_;                                 \
    _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) {                                             \
      fa[BUF][ks] = *reinterpret_cast<const bf16x8*>(arow_ + 16 * ks);                             \
      fb0[BUF][ks] = *reinterpret_cast<const bf16x8*>(brow_ + 16 * ks);                            \
      fb1[BUF][ks] = *reinterpret_cast<const bf16x8*>(brow_ + 32 * CLD + 16 * ks);                 \
    }                                                                                              \
  }
    RMBX_RES_FRAGS(0, 0)
#pragma unroll
    for (int g = 0; g < 18; ++g) {
      const int cur = g & 1;
      if (g < 17) RMBX_RES_FRAGS(cur ^ 1, g + 1)
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch above this group's MFMAs
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][ks], fb0[cur][ks], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][ks], fb1[cur][ks], acc1, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    }
#undef RMBX_RES_FRAGS
    // the next patch has landed in registers by now: consume the wait here so that the vmcnt
    // wait before the next patch store does not also wait for this tile's output stores
#pragma unroll
    for (int i = 0; i < RPATCH_PER_THREAD; ++i) asm volatile("" ::"v"(pr[i].x), "v"(pr[i].y), "v"(pr[i].z), "v"(pr[i].w));
    __syncthreads();  // every wave is done reading the patch
    if (dbg & 2) continue;
    const int col = lane & 31;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int row = 32 * wave + (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);  // = tile pixel
      sC[row * EPI_LDR + col] = acc0[j];
      sC[row * EPI_LDR + 32 + col] = acc1[j];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < EPASS; ++i) {
      const int pix = (tid + RTHREADS * i) >> 3;
      ov[i] = epi_finish8(sC + pix * EPI_LDR + c8, bv, rres[i], a.res != nullptr, a.relu != 0);
    }
    pn = n;
    poy0 = oy0;
    pox0 = ox0;
    if (t + 1 < t_end && !(dbg & 4)) RMBX_RESID_LOAD(t + 1)
  }
  RMBX_RES_STORE()
#undef RMBX_RES_STORE
#undef RMBX_RESID_LOAD
#undef RMBX_RES_LOAD
#undef RMBX_RES_TILE
}

// ---------------------------------------------------------------------------------------------
// f32 form of the layer-1 conv (3x3 / stride 1 / pad 1, Cin = Cout = 64; the reference's fp32
// policy) with the same fused epilogue, v_mfma_f32_32x32x2_f32 (exact f32 products, f32
// accumulation).  f32 MFMA issues at 64 cycles per instruction, so unlike the bf16 kernels this
// one is MFMA-bound and is laid out to keep the four SIMDs issuing:
//  * a persistent block per CU (8 waves, two per SIMD, so one wave's LDS reads hide under the
//    other's MFMAs) keeps the filter taps of its 32 output channels resident in LDS
//    (9 x 64 x 32 f32 = 72 KiB) and walks a contiguous range of 8 x 32 output tiles (120 x 160
//    splits exactly); wave w owns output row w of the tile (32 pixels) x the block's 32 channels:
//    one accumulator, 288 MFMAs per tile;
//  * the tile's 10 x 34 x 64 f32 input patch (85 KiB) is staged in LDS once for all 9 taps as two
//    channel halves: the MFMAs run over half 0 (all taps), then half 1, and the next tile's half 0
//    (prefetched into registers at the top of the tile) is written while half 1 is multiplied --
//    the patch traffic hides under the MFMAs instead of stalling every wave between tiles;
//  * the A rows (output channels) are permuted so that each lane finishes 16 consecutive channels
//    of ONE pixel: bias, residual and ReLU are applied in registers and leave as 16-byte stores
//    (no LDS transpose), and the barriers order LDS only, so the stores drain under the next
//    tile's MFMAs;
//  * the two channel halves of a tile run on blocks b and b + 8 (the same XCD under round-robin
//    dispatch), so each input patch is fetched from HBM once per XCD.
// ---------------------------------------------------------------------------------------------
constexpr int FC_TH = 8, FC_TW = 32, FC_PH = FC_TH + 2, FC_PW = FC_TW + 2, FC_COUT = 32, FC_THREADS = 512;
constexpr int FC_W_FLOATS = 9 * 32 * FC_COUT * 2;            // sW[tap][kpair][cout][2]
constexpr int FC_PKP = FC_PH * FC_PW * 2;                    // floats per k-pair plane of the patch
constexpr int FC_P_FLOATS = 32 * FC_PKP;                     // sP[kpair][py][px][2]
constexpr int FC_HCHUNKS = FC_PH * FC_PW * 8;                // float4 chunks of one channel half
constexpr int FC_PPT = (FC_HCHUNKS + FC_THREADS / 2 - 1) / (FC_THREADS / 2);  // per thread
static_assert((FC_W_FLOATS + FC_P_FLOATS) * 4 <= 160 * 1024, "f32 conv LDS must fit the 160 KiB of a CU");
static_assert(FC_THREADS % 16 == 0, "a thread's channel quad is the same in every patch chunk");
static_assert(FC_PPT <= 12, "three filter rows carry a thread's patch stores");

// workgroup barrier that orders LDS only: unlike __syncthreads() it does not wait for the
// wave's outstanding global stores (the previous tile's outputs drain under the next tile's MFMAs)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct ConvF32Args {
  const float* in;    // [N][H][W][64]
  const float* w;     // [64][3][3][64]
  const float* bias;  // [64]
  const float* res;   // [N][H][W][64] or null
  float* out;         // [N][H][W][64]
  int N, H, W, relu;
  int tiles_x, tiles_y;
  long long ntiles;
  int dbg;  // diagnostic phase skips (RMBX_CONV_DBG: 1 = no MFMAs, 2 = no patch loads, 4 = no patch
            // stores / residual loads / output stores; 0 in production)
};

// the 9 taps x 16 k-pairs of one channel half (KP0 = 0 or 16) into acc; hook(kh) runs after
// each filter row (the patch stores of the next tile are spread over the MFMA stream this way)
template <int KP0, class Hook>
__device__ __forceinline__ void fc_half(f32x16& acc, const float* wl, const float* pl, Hook&& hook) {
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const float* wt = wl + ((kh * 3 + kw) * 32 + KP0) * 64;
      const float* pt = pl + KP0 * FC_PKP + (kh * FC_PW + kw) * 2;
#pragma unroll
      for (int kp = 0; kp < 16; ++kp)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wt[kp * 64], pt[kp * FC_PKP], acc, 0, 0, 0);
    }
    hook(kh);
  }
}

__global__ void __launch_bounds__(FC_THREADS) conv3x3_c64_f32_kernel(ConvF32Args a) {
  __shared__ __attribute__((aligned(16))) float smem[FC_W_FLOATS + FC_P_FLOATS];
  float* sW = smem;
  float* sP = smem + FC_W_FLOATS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x;
  const int half = (b >> 3) & 1;              // output channels 32 half .. 32 half + 31
  const int G = gridDim.x >> 1;               // tile groups (gridDim.x % 16 == 0)
  const int g = (b & 7) + 8 * (b >> 4);
  const long long t_begin = a.ntiles * g / G, t_end = a.ntiles * (g + 1) / G;
  if (t_begin >= t_end) return;
  const int co0 = FC_COUT * half;

  // filter taps of the block's channels: global [cout][tap][cin] -> sW[tap][kp][cout_local][2]
  for (int q = tid; q < FC_COUT * 9 * 16; q += FC_THREADS) {
    const int quad = q & 15, rest = q >> 4;  // rest = cout_local * 9 + tap
    const int cl = rest / 9, tap = rest - 9 * cl;
    const float4 v = *reinterpret_cast<const float4*>(a.w + ((size_t)(co0 + cl) * 9 + tap) * 64 + 4 * quad);
    *reinterpret_cast<float2*>(sW + (((size_t)tap * 32 + 2 * quad) * FC_COUT + cl) * 2) = make_float2(v.x, v.y);
    *reinterpret_cast<float2*>(sW + (((size_t)tap * 32 + 2 * quad + 1) * FC_COUT + cl) * 2) = make_float2(v.z, v.w);
  }

  const int n = lane & 31, h = lane >> 5;
  const int sig = 16 * ((n >> 2) & 1) + (n & 3) + 4 * (n >> 3);  // A row n -> channel sig
  const float* wl = sW + sig * 2 + h;                    // + (tap * 32 + kp) * 64
  const float* pl = sP + (wave * FC_PW + n) * 2 + h;     // B column n = tile pixel (wave, n)
  float bv[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) bv[j] = a.bias[co0 + 16 * h + j];

  auto tile_of = [&](long long t, int& img, int& oy0, int& ox0) {
    const int tx = (int)(t % a.tiles_x);
    const long long r = t / a.tiles_x;
    oy0 = (int)(r % a.tiles_y) * FC_TH;
    img = (int)(r / a.tiles_y);
    ox0 = tx * FC_TW;
  };
  // Waves 0..3 stage channel half 0 of the patches (k-pairs 0..15), waves 4..7 half 1: chunk
  // c = (tid & 255) + 256 i of a half = pixel c >> 3 x channel quad (c & 7) + 8 hi.  A wave's
  // next-tile chunks are loaded into registers after it has stored the current ones, and stored
  // while the OTHER half is multiplied (hi waves during half 0, the others during half 1).
  const bool hi = wave >= 4;
  const int ht = tid & (FC_THREADS / 2 - 1);
  const int quad = (ht & 7) + 8 * hi;
  // loads are unconditional (clamped to a valid address) and the out-of-image chunks are zeroed
  // only when stored, so no wait on them is forced before the MFMAs they should hide under
  float4 pf[FC_PPT];
  uint32_t pf_ok = 0;
  auto load_patch = [&](long long t) {
    int img, oy0, ox0;
    tile_of(t, img, oy0, ox0);
    pf_ok = 0;
#pragma unroll
    for (int i = 0; i < FC_PPT; ++i) {
      const int c = ht + (FC_THREADS / 2) * i;
      const int pp = c >> 3;
      const int py = pp / FC_PW, px = pp - py * FC_PW;
      const int y = oy0 - 1 + py, x = ox0 - 1 + px;
      const bool ok = c < FC_HCHUNKS && y >= 0 && y < a.H && x >= 0 && x < a.W;
      const size_t off = ok ? (((size_t)img * a.H + y) * a.W + x) * 64 + 4 * quad : 0;
      pf[i] = *reinterpret_cast<const float4*>(a.in + off);
      pf_ok |= (uint32_t)ok << i;
    }
  };
  auto store_chunk = [&](int i) {
    const int c = ht + (FC_THREADS / 2) * i;
    if (c < FC_HCHUNKS) {
      const float4 v = ((pf_ok >> i) & 1u) ? pf[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      float* dst = sP + (size_t)(2 * quad) * FC_PKP + (c >> 3) * 2;
      *reinterpret_cast<float2*>(dst) = make_float2(v.x, v.y);
      *reinterpret_cast<float2*>(dst + FC_PKP) = make_float2(v.z, v.w);
    }
  };
  auto store_third = [&](int kh) {  // chunks 4 kh .. 4 kh + 3, after filter row kh
#pragma unroll
    for (int i = 4 * kh; i < 4 * kh + 4; ++i)
      if (i < FC_PPT) store_chunk(i);
  };
  load_patch(t_begin);
#pragma unroll
  for (int i = 0; i < FC_PPT; ++i) store_chunk(i);
  lds_barrier();  // sW and the first patch are in LDS

  for (long long t = t_begin; t < t_end; ++t) {
    int img, oy0, ox0;
    tile_of(t, img, oy0, ox0);
    const bool more = t + 1 < t_end;
    if (!hi && more && !(a.dbg & 2)) load_patch(t + 1);
    const int oy = oy0 + wave, ox = ox0 + n;
    const bool pix_ok = oy < a.H && ox < a.W;
    const size_t pix_off = (((size_t)img * a.H + oy) * a.W + ox) * 64 + co0 + 16 * h;
    float4 rv[4];
    if (a.res && !(a.dbg & 4)) {
      const float* rp = a.res + (pix_ok ? pix_off : 0);
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) rv[k4] = *reinterpret_cast<const float4*>(rp + 4 * k4);
    }

    // half 0 (P0 = k-pairs 0..15 of this tile); the hi waves write this tile's half 1 meanwhile
    const bool st1 = hi && t > t_begin && !(a.dbg & 4);
    f32x16 acc = {};
    if (!(a.dbg & 1)) fc_half<0>(acc, wl, pl, [&](int kh) { if (st1) store_third(kh); });
    lds_barrier();  // every wave is done with half 0 of this tile's patch, and half 1 is visible
    if (hi && more && !(a.dbg & 2)) load_patch(t + 1);
    // half 1; the other waves write the next tile's half 0 meanwhile
    const bool st0 = !hi && more && !(a.dbg & 4);
    if (!(a.dbg & 1)) fc_half<16>(acc, wl, pl, [&](int kh) { if (st0) store_third(kh); });
    lds_barrier();  // every wave is done with half 1; the next half 0 is visible
    if (pix_ok && !(a.dbg & 4)) {
      float o[16];
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const float r4[4] = {rv[k4].x, rv[k4].y, rv[k4].z, rv[k4].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = 4 * k4 + e;
          float v = acc[j] + bv[j];
          if (a.res) v += r4[e];
          if (a.relu) v = v > 0.f ? v : (v != v ? v : 0.f);
          o[j] = v;
        }
      }
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4)
        *reinterpret_cast<float4*>(a.out + pix_off + 4 * k4) = make_float4(o[4 * k4], o[4 * k4 + 1], o[4 * k4 + 2], o[4 * k4 + 3]);
    }
  }
}

int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 256;
  return cus > 0 ? cus : 256;
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_conv2d_nhwc(const void* in, const void* weight, const float* bias, const void* residual,
                                void* out, int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                int pad, int relu, void* stream) {
  RMBX_CHECK_ARG(in && weight && bias && out, "rmbx_conv2d_nhwc: null pointer");
  RMBX_CHECK_ARG(N >= 0 && H > 0 && W > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0,
                 "rmbx_conv2d_nhwc: bad geometry");
  RMBX_CHECK_ARG(Cin % rmbx::CBK == 0, "rmbx_conv2d_nhwc: Cin=%d must be a multiple of %d", Cin, rmbx::CBK);
  RMBX_CHECK_ARG(Cout % rmbx::CBN == 0, "rmbx_conv2d_nhwc: Cout=%d must be a multiple of %d", Cout, rmbx::CBN);
  RMBX_CHECK_ARG((((uintptr_t)in | (uintptr_t)weight) & 15) == 0, "rmbx_conv2d_nhwc: in/weight must be 16-byte aligned");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  RMBX_CHECK_ARG(Ho > 0 && Wo > 0, "rmbx_conv2d_nhwc: empty output");
  if (N == 0) return RMBX_OK;
  rmbx::ConvArgs a;
  a.in = (const uint16_t*)in;
  a.w = (const uint16_t*)weight;
  a.bias = bias;
  a.res = (const uint16_t*)residual;
  a.out = (uint16_t*)out;
  a.N = N;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.Ho = Ho;
  a.Wo = Wo;
  a.Cout = Cout;
  a.KH = KH;
  a.KW = KW;
  a.stride = stride;
  a.pad = pad;
  a.relu = relu;
  a.M = (long long)N * Ho * Wo;
  a.n_ntiles = Cout / rmbx::CBN;
  a.n_mtiles = (a.M + rmbx::CBM - 1) / rmbx::CBM;
  const char* dbg_env = std::getenv("RMBX_CONV_DBG");
  a.dbg = dbg_env ? std::atoi(dbg_env) : 0;
  if (KH == 3 && KW == 3 && stride == 1 && pad == 1 && Cin == 64 && Cout == 64 &&
      std::getenv("RMBX_CONV_NO_RESIDENT") == nullptr) {
    const int tiles_x = (Wo + rmbx::RTW - 1) / rmbx::RTW, tiles_y = (Ho + rmbx::RTH - 1) / rmbx::RTH;
    const long long ntiles = (long long)N * tiles_x * tiles_y;
    const int grid = (int)(ntiles < rmbx::device_cus() ? ntiles : rmbx::device_cus());
    hipLaunchKernelGGL(rmbx::conv3x3_c64_resident_kernel, dim3(grid), dim3(rmbx::RTHREADS), 0,
                       (hipStream_t)stream, a, tiles_x, tiles_y, ntiles);
    RMBX_CHECK_LAUNCH();
    return RMBX_OK;
  }
  if (KH == 3 && KW == 3 && stride == 1 && pad == 1) {
    const long long ntile = (long long)N * ((Ho + rmbx::PT_H - 1) / rmbx::PT_H) * ((Wo + rmbx::PT_W - 1) / rmbx::PT_W);
    const long long nb = ntile * a.n_ntiles;
    RMBX_CHECK_ARG(nb < (1ll << 31), "rmbx_conv2d_nhwc: grid too large");
    hipLaunchKernelGGL(rmbx::conv3x3_c64_patch_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, a);
    RMBX_CHECK_LAUNCH();
    return RMBX_OK;
  }
  const long long nblocks = a.n_mtiles * a.n_ntiles;
  RMBX_CHECK_ARG(nblocks < (1ll << 31), "rmbx_conv2d_nhwc: grid too large");
  hipLaunchKernelGGL(rmbx::conv_nhwc_kernel<0>, dim3((unsigned)nblocks), dim3(256), 0, (hipStream_t)stream, a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_stem_s2d_conv(const void* in, const void* weight, const float* bias, void* out, int N, int Hs,
                                  int Ws, int Cout, int relu, void* stream) {
  RMBX_CHECK_ARG(in && weight && bias && out, "rmbx_stem_s2d_conv: null pointer");
  RMBX_CHECK_ARG(N >= 0 && Hs > 0 && Ws > 0, "rmbx_stem_s2d_conv: bad geometry");
  RMBX_CHECK_ARG(Cout % rmbx::CBN == 0, "rmbx_stem_s2d_conv: Cout=%d must be a multiple of %d", Cout, rmbx::CBN);
  RMBX_CHECK_ARG((((uintptr_t)in | (uintptr_t)weight) & 15) == 0, "rmbx_stem_s2d_conv: unaligned");
  if (N == 0) return RMBX_OK;
  rmbx::ConvArgs a;
  a.dbg = 0;
  a.in = (const uint16_t*)in;
  a.w = (const uint16_t*)weight;
  a.bias = bias;
  a.res = nullptr;
  a.out = (uint16_t*)out;
  a.N = N;
  a.H = Hs;
  a.W = Ws;
  a.Cin = 64;  // K step = one filter row: 4 taps x 16 channels
  a.Ho = Hs;
  a.Wo = Ws;
  a.Cout = Cout;
  a.KH = 4;
  a.KW = 1;
  a.stride = 1;
  a.pad = 2;
  a.relu = relu;
  a.M = (long long)N * Hs * Ws;
  a.n_ntiles = Cout / rmbx::CBN;
  a.n_mtiles = (a.M + rmbx::CBM - 1) / rmbx::CBM;
  const long long nblocks = a.n_mtiles * a.n_ntiles;
  RMBX_CHECK_ARG(nblocks < (1ll << 31), "rmbx_stem_s2d_conv: grid too large");
  hipLaunchKernelGGL(rmbx::conv_nhwc_kernel<1>, dim3((unsigned)nblocks), dim3(256), 0, (hipStream_t)stream, a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_conv2d_nhwc_f32(const float* in, const float* weight, const float* bias, const float* residual,
                                    float* out, int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                    int pad, int relu, void* stream) {
  RMBX_CHECK_ARG(in && weight && bias && out, "rmbx_conv2d_nhwc_f32: null pointer");
  RMBX_CHECK_ARG(N >= 0 && H > 0 && W > 0, "rmbx_conv2d_nhwc_f32: bad geometry");
  RMBX_CHECK_ARG(Cin == 64 && Cout == 64 && KH == 3 && KW == 3 && stride == 1 && pad == 1,
                 "rmbx_conv2d_nhwc_f32: only the 3x3 / stride 1 / pad 1 conv with Cin = Cout = 64 is implemented");
  RMBX_CHECK_ARG((((uintptr_t)in | (uintptr_t)weight | (uintptr_t)out | (uintptr_t)residual) & 15) == 0,
                 "rmbx_conv2d_nhwc_f32: tensors must be 16-byte aligned");
  if (N == 0) return RMBX_OK;
  rmbx::ConvF32Args a;
  a.in = in;
  a.w = weight;
  a.bias = bias;
  a.res = residual;
  a.out = out;
  a.N = N;
  a.H = H;
  a.W = W;
  a.relu = relu;
  a.tiles_x = (W + rmbx::FC_TW - 1) / rmbx::FC_TW;
  a.tiles_y = (H + rmbx::FC_TH - 1) / rmbx::FC_TH;
  a.ntiles = (long long)N * a.tiles_x * a.tiles_y;
  const char* dbg_env = std::getenv("RMBX_CONV_DBG");
  a.dbg = dbg_env ? std::atoi(dbg_env) : 0;
  // one persistent block per CU, the two channel halves of a tile group on blocks b, b + 8
  int grid = rmbx::device_cus();
  grid = grid < 16 ? 16 : grid - grid % 16;
  hipLaunchKernelGGL(rmbx::conv3x3_c64_f32_kernel, dim3(grid), dim3(rmbx::FC_THREADS), 0, (hipStream_t)stream, a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
