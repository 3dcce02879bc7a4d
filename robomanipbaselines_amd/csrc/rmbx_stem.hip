// ResNet-18 stem fused end to end: conv1 (7x7 / stride 2 / pad 3, BN folded) + bias + ReLU +
// max-pool 3x3 / stride 2 / pad 1, from the renderer's 2x2 space-to-depth image straight to the
// pooled [N][Hp][Wp][64] bf16 activation that layer1 reads (MFMA 32x32x16 bf16, gfx950).
//
// Replaces the stem of the backbones' torchvision resnet18 (ACT's DETR backbone, third_party/act
// [absent]; policy/mlp/MlpPolicy.py:34-39): conv1 -> bn1 -> relu -> maxpool.  The unfused form
// (rmbx_stem_s2d_conv + rmbx_nhwc_bias_relu_maxpool) writes the 64-channel stem map at full
// resolution (240 x 320 x 64 bf16 = 9.8 MB per 480 x 640 image) and reads it back for the pool;
// here that map never leaves the CU: HBM sees the s2d image once (2.5 MB) and the pooled output
// once (2.5 MB).
//
// Mapping.  One block per (image, band of pool rows); wave w owns stem columns 32w .. 32w+31 for
// the whole band.  Per pool row py the block computes stem rows 2py and 2py+1 as a transposed
// implicit GEMM C^T[cout][pixel] = W[cout][k] * X[k][pixel] with k = (ky, kx, 16 s2d channels)
// in the order of rmbx_stem_s2d_conv (so the f32 accumulation chains, and therefore the bf16
// stem values, are identical to the unfused kernel's).  The A operand rows are the output
// channels permuted so that accumulator register j of lane-half h holds channel 16h + j of
// the 32-channel tile: after bias + ReLU + rounding each lane owns 16 consecutive channels of ONE
// stem pixel, so
//   * the vertical pool is a running max in registers (row 2py-1 carried from the previous row
//     pair; packed bf16 max as u16 is exact because every value is >= 0 after the ReLU),
//   * the horizontal pool is two lane shuffles (left/right neighbour pixel) plus one LDS edge
//     value from the wave on the left,
//   * the pooled pixel's 32 channels leave as two 16-byte stores.
// The filter bank (16 taps x 64 x 16 bf16 = 32 KiB) stays in LDS for the block's life; the input
// rows live in a 5-row LDS ring (rows 2py-2 .. 2py+2), the next two rows prefetched into
// registers while the current pair is multiplied.

#include "rmbx_common.h"

#include <cstdint>
#include <cstdlib>
#include <type_traits>

namespace rmbx {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8s __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2s __attribute__((ext_vector_type(2)));

constexpr int SP_MAX_WAVES = 10;               // stem columns <= 320
constexpr int SP_THREADS = 64 * SP_MAX_WAVES;  // launch bound
constexpr int SP_RING = 5;                     // s2d rows 2py-2 .. 2py+2
constexpr int SP_RC_MAX = 32 * SP_MAX_WAVES + 4;
constexpr int SP_LDS_U16 = 16 * 2 * 64 * 8 + SP_RING * 2 * SP_RC_MAX * 8 + 2 * 64 + SP_MAX_WAVES * 2 * 16 * 2;
static_assert(SP_LDS_U16 * 2 <= 160 * 1024, "stem+pool LDS must fit the 160 KiB of a CU");

__device__ __forceinline__ uint32_t sp_f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

typedef short i16x2 __attribute__((ext_vector_type(2)));
// per-half max of two packed bf16 pairs as signed 16-bit integers (v_pk_max_i16): for bf16 values
// >= +0 the integer order is the value order, and every negative value (sign bit set, -0 included)
// is below +0, so pk_max(x, 0) is the ReLU of a packed pair
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(i16x2, a), __builtin_bit_cast(i16x2, b)));
}

struct StemPoolArgs {
  const uint16_t* in;   // [N][Hs][Ws][16]
  const uint16_t* w;    // [64][16 taps][16]
  const float* bias;    // [64]
  uint16_t* out;        // [N][Hp][Wp][64]
  int N, Hs, Ws, Hp, Wp;
  int nct;              // column tiles (= waves per block)
  int rc;               // ring columns = 32 * nct + 4 (s2d cols -2 .. 32 * nct + 1)
  int bands, band_rows; // pool-row bands per image
};

__global__ void __launch_bounds__(SP_THREADS) stem_pool_kernel(StemPoolArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t sp_smem[SP_LDS_U16];
  uint16_t* sW = sp_smem;                          // [16 taps][2 halves][64 cout][8]
  uint16_t* sR = sW + 16 * 2 * 64 * 8;             // [5 slots][2 halves][rc][8]
  float* sBias = reinterpret_cast<float*>(sR + SP_RING * 2 * a.rc * 8);  // [64]
  uint32_t* sEdge = reinterpret_cast<uint32_t*>(sBias + 64);              // [nct][2][16]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nthreads = blockDim.x;
  const int img = blockIdx.x / a.bands, band = blockIdx.x - img * a.bands;
  const int py0 = band * a.band_rows;
  const int py1 = min(a.Hp, py0 + a.band_rows);
  if (py0 >= py1) return;
  const int pys = py0 > 0 ? py0 - 1 : 0;  // a compute-only row pair supplies the carried row
  const size_t row_elems = (size_t)a.Ws * 16;
  const uint16_t* in_img = a.in + (size_t)img * a.Hs * row_elems;

  // filter bank: global [cout][tap][16] -> sW[tap][half][cout][8]
  for (int q = tid; q < 64 * 16 * 2; q += nthreads) {
    const int half = q & 1, rest = q >> 1;  // rest = cout * 16 + tap
    const int co = rest >> 4, tap = rest & 15;
    *reinterpret_cast<uint4*>(sW + ((tap * 2 + half) * 64 + co) * 8) =
        *reinterpret_cast<const uint4*>(a.w + (size_t)rest * 16 + half * 8);
  }
  if (tid < 64) sBias[tid] = a.bias[tid];

  // 16-byte chunk q of s2d row y -> (half, ring col); zero outside the image
  const int row_chunks = 2 * a.rc;
  auto load_chunk = [&](int y, int q) -> uint4 {
    const int half = q / a.rc, c = q - half * a.rc;
    const int x = c - 2;
    if (y < 0 || y >= a.Hs || x < 0 || x >= a.Ws) return make_uint4(0, 0, 0, 0);
    return *reinterpret_cast<const uint4*>(in_img + (size_t)y * row_elems + (size_t)x * 16 + half * 8);
  };
  auto slot_of = [](int y) { return (y + 2 * SP_RING) % SP_RING; };
  // initial ring: rows 2pys-2 .. 2pys+2
  for (int q = tid; q < SP_RING * row_chunks; q += nthreads) {
    const int r = q / row_chunks, qq = q - r * row_chunks;
    const int y = 2 * pys - 2 + r;
    *reinterpret_cast<uint4*>(sR + ((size_t)slot_of(y) * row_chunks + qq) * 8) = load_chunk(y, qq);
  }

  const int n = lane & 31, h = lane >> 5;  // B: pixel column in the tile / k half; C: channel half
  const int X = 32 * wave + n;             // this lane's stem column
  const int m = lane & 31;                 // A row -> output channel sigma(m) of the tile
  const int sig = 16 * ((m >> 2) & 1) + (m & 3) + 4 * (m >> 3);
  const bool col_ok = X < a.Ws;

  // register prefetch of the next pair's two new rows (2 * row_chunks chunks over the block):
  // branch-free (clamped address, zero applied when the chunk is written to the ring)
  constexpr int PF_MAX = 3;  // (2 rows * 2 halves * 324 cols) / 640 threads, rounded up
  uint4 pf[PF_MAX];
  uint32_t pf_ok = 0;
  const int pf_chunks = 2 * row_chunks;
  int pf_r[PF_MAX], pf_q[PF_MAX];
#pragma unroll
  for (int i = 0; i < PF_MAX; ++i) {
    const int q = min(tid + nthreads * i, pf_chunks - 1);
    pf_r[i] = q / row_chunks;
    pf_q[i] = q - pf_r[i] * row_chunks;
  }

  uint32_t carry[2][8];  // stem row 2py-1 (bf16 pairs): [cout tile][channel pair]
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int k = 0; k < 8; ++k) carry[t][k] = 0;

  __syncthreads();
  for (int py = pys; py < py1; ++py) {
    const int Y0 = 2 * py;
    const bool more = py + 1 < py1;
    if (more) {
      pf_ok = 0;
#pragma unroll
      for (int i = 0; i < PF_MAX; ++i) {
        const int y = Y0 + 3 + pf_r[i];
        const int half = pf_q[i] / a.rc, x = pf_q[i] - half * a.rc - 2;
        const bool ok = tid + nthreads * i < pf_chunks && y < a.Hs && x >= 0 && x < a.Ws;
        const size_t off = ok ? (size_t)y * row_elems + (size_t)x * 16 + half * 8 : 0;
        pf[i] = *reinterpret_cast<const uint4*>(in_img + off);
        pf_ok |= (uint32_t)ok << i;
      }
    }
    f32x16 acc[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[r][t] = f32x16{};
    int slot[5];
#pragma unroll
    for (int d = 0; d < 5; ++d) slot[d] = slot_of(Y0 - 2 + d);
#pragma unroll
    for (int tap = 0; tap < 16; ++tap) {
      const int ky = tap >> 2, kx = tap & 3;
      bf16x8 bx[2], aw[2];
#pragma unroll
      for (int r = 0; r < 2; ++r)
        bx[r] = *reinterpret_cast<const bf16x8*>(sR + (((size_t)slot[r + ky] * 2 + h) * a.rc + X + kx) * 8);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        aw[t] = *reinterpret_cast<const bf16x8*>(sW + ((tap * 2 + h) * 64 + 32 * t + sig) * 8);
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[r][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aw[t], bx[r], acc[r][t], 0, 0, 0);
    }

    // bias + bf16 (round-to-nearest-even, v_cvt_pk_bf16_f32) + ReLU on the packed pair,
    // vertical max with the carried row, packed channel pairs
    const bool row1_ok = Y0 + 1 < a.Hs;
    uint32_t vm[2][8];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float4* bp = reinterpret_cast<const float4*>(sBias + 32 * t + 16 * h);
      float bv[16];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 b4 = bp[k];
        bv[4 * k] = b4.x;
        bv[4 * k + 1] = b4.y;
        bv[4 * k + 2] = b4.z;
        bv[4 * k + 3] = b4.w;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        f32x2 v0, v1;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          v0[e] = acc[0][t][2 * k + e] + bv[2 * k + e];
          v1[e] = acc[1][t][2 * k + e] + bv[2 * k + e];
        }
        // ReLU after rounding == rounding after ReLU (RNE keeps the sign; -0 and negatives -> +0)
        const uint32_t p0 = __builtin_bit_cast(uint32_t, __builtin_convertvector(v0, bf16x2));
        const uint32_t p1 = row1_ok ? pk_max(__builtin_bit_cast(uint32_t, __builtin_convertvector(v1, bf16x2)), 0u) : 0u;
        vm[t][k] = col_ok ? pk_max(pk_max(carry[t][k], p0), p1) : 0u;  // >= 0 through p1
        carry[t][k] = p1;
      }
    }
    // the tile's last column feeds the right neighbour wave's first pool window
    if (n == 31) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int k = 0; k < 8; ++k) sEdge[(wave * 2 + h) * 16 + 8 * t + k] = vm[t][k];
    }
    __syncthreads();  // edges visible; every wave is done with ring rows 2py-2, 2py-1

    // refill the ring first (the prefetch has landed long ago), so the wait for it never waits
    // on this row's output stores
    if (more) {
#pragma unroll
      for (int i = 0; i < PF_MAX; ++i) {
        if (tid + nthreads * i < pf_chunks) {
          const uint4 v = ((pf_ok >> i) & 1u) ? pf[i] : make_uint4(0, 0, 0, 0);
          const int dst_slot = pf_r[i] ? slot[1] : slot[0];  // row Y0+3+r replaces row Y0-2+r
          *reinterpret_cast<uint4*>(sR + ((size_t)dst_slot * row_chunks + pf_q[i]) * 8) = v;
        }
      }
    }
    if (py >= py0) {
      uint32_t o[2][8];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          uint32_t left = (uint32_t)__shfl_up((int)vm[t][k], 1);
          const uint32_t right = (uint32_t)__shfl_down((int)vm[t][k], 1);
          if (n == 0) left = wave > 0 ? sEdge[((wave - 1) * 2 + h) * 16 + 8 * t + k] : 0u;
          o[t][k] = pk_max(pk_max(left, vm[t][k]), right);
        }
      const int px = 16 * wave + (n >> 1);
      if ((n & 1) == 0 && px < a.Wp) {
        uint16_t* dst = a.out + (((size_t)img * a.Hp + py) * a.Wp + px) * 64 + 16 * h;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          *reinterpret_cast<uint4*>(dst + 32 * t) = make_uint4(o[t][0], o[t][1], o[t][2], o[t][3]);
          *reinterpret_cast<uint4*>(dst + 32 * t + 8) = make_uint4(o[t][4], o[t][5], o[t][6], o[t][7]);
        }
      }
    }
    __syncthreads();  // ring refilled; edge reads done before the next pair overwrites them
  }
}

// ---------------------------------------------------------------------------------------------
// f32 form (the reference's precision): the same fused stem on the renderer's f32 space-to-depth
// image [N][Hs][Ws][16] (12 channels used) with v_mfma_f32_32x32x2_f32 (exact f32 products,
// f32 accumulation), output [N][Hp][Wp][64] f32 (channels_last) for the layer-1 convs.
// K per tap = 12 s2d channels = 6 MFMA k-pairs; the 4 zero pad channels are skipped, and so are
// the k-pairs that are zero in every re-indexed 7x7 filter (pack_stem_s2d: ky = 0 has no dy = 0
// rows -> k-pairs 0..2; kx = 0 has no dx = 0 columns -> k-pairs 0 and 3): 77 of 96 k-pair steps.
// f32 MFMA issues at 64 cycles per 32x32x2 on each SIMD, so the kernel is MFMA-bound and the
// work is split evenly over the 4 SIMDs: 4 waves per block (one per SIMD), wave w owns output
// channel tile t = w & 1 (32 channels) of column tiles 5 (w >> 1) .. 5 (w >> 1) + 4 (32 stem
// columns each) for both stem rows of a pool row: 10 independent accumulators per wave.
// LDS: filter bank sW[tap][kpair][h][64 cout] (48 KiB), input ring sR[slot][kpair][324][2]
// (76 KiB), edges.  One block per (image, band) as in the bf16 kernel; Ws <= 320.
// ---------------------------------------------------------------------------------------------
constexpr int SF_WAVES = 4, SF_TILES = 5, SF_THREADS = 64 * SF_WAVES;
constexpr int SF_RC = SP_RC_MAX;  // ring columns: s2d cols -2 .. 321 (zeros beyond the image)
constexpr int SF_LDS_F32 = 16 * 6 * 2 * 64 + SP_RING * 6 * SF_RC * 2 + 64 + SF_WAVES * 2 * 16;
static_assert(SF_LDS_F32 * 4 <= 160 * 1024, "f32 stem+pool LDS must fit the 160 KiB of a CU");
static_assert(2 * SF_TILES * 32 == 32 * SP_MAX_WAVES, "the two wave pairs cover the 320 columns");

struct StemPoolF32Args {
  const float* in;   // [N][Hs][Ws][16]
  const float* w;    // [64][16 taps][16]
  const float* bias; // [64]
  float* out;        // [N][Hp][Wp][64]
  int N, Hs, Ws, Hp, Wp;
  int bands, band_rows;
};

// one filter row ky of the f32 stem: 4 taps x the k-pairs from KP_LO, minus the kx = 0 pairs that
// hold only dx = 0 channels; straight-line so that the next k-pair's LDS reads are issued under
// the current k-pair's 10 MFMAs
template <int KP_LO>
__device__ __forceinline__ void sf_filter_row(f32x16 (&acc)[SF_TILES][2], const float* row0, const float* row1,
                                              const float* wrow) {
#pragma unroll
  for (int kx = 0; kx < 4; ++kx) {
#pragma unroll
    for (int kp = KP_LO; kp < 6; ++kp) {
      if (kx == 0 && (kp == 0 || kp == 3)) continue;  // dx = 0 column of the 8x8 window
      const float aw = wrow[(kx * 6 + kp) * 128];
      float bx[SF_TILES][2];
#pragma unroll
      for (int i = 0; i < SF_TILES; ++i) {
        bx[i][0] = row0[(kp * SF_RC + 32 * i + kx) * 2];
        bx[i][1] = row1[(kp * SF_RC + 32 * i + kx) * 2];
      }
#pragma unroll
      for (int i = 0; i < SF_TILES; ++i)
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[i][r] = __builtin_amdgcn_mfma_f32_32x32x2f32(aw, bx[i][r], acc[i][r], 0, 0, 0);
    }
  }
}

__global__ void __launch_bounds__(SF_THREADS) stem_pool_f32_kernel(StemPoolF32Args a) {
  __shared__ __attribute__((aligned(16))) float sf_smem[SF_LDS_F32];
  float* sW = sf_smem;                            // [16 taps][6 kpairs][2 h][64 cout]
  float* sR = sW + 16 * 6 * 2 * 64;               // [5 slots][6 kpairs][SF_RC][2]
  float* sBias = sR + SP_RING * 6 * SF_RC * 2;    // [64]
  float* sEdge = sBias + 64;                      // [waves][2 h][16]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int img = blockIdx.x / a.bands, band = blockIdx.x - img * a.bands;
  const int py0 = band * a.band_rows;
  const int py1 = min(a.Hp, py0 + a.band_rows);
  if (py0 >= py1) return;
  const int pys = py0 > 0 ? py0 - 1 : 0;
  const size_t row_elems = (size_t)a.Ws * 16;
  const float* in_img = a.in + (size_t)img * a.Hs * row_elems;

  // filter bank: global [cout][tap][16] -> sW[tap][kp][h][cout] (channels 0..11)
  for (int q = tid; q < 64 * 16 * 12; q += SF_THREADS) {
    const int c = q % 12, rest = q / 12;  // rest = cout * 16 + tap
    const int co = rest >> 4, tap = rest & 15;
    sW[((tap * 6 + (c >> 1)) * 2 + (c & 1)) * 64 + co] = a.w[(size_t)rest * 16 + c];
  }
  if (tid < 64) sBias[tid] = a.bias[tid];

  // 16-byte chunk q (ring column c = q / 3, channel quad j = q % 3) of s2d row y
  constexpr int row_chunks = 3 * SF_RC;
  auto load_chunk = [&](int y, int q) -> float4 {
    const int c = q / 3, j = q - 3 * c;
    const int x = c - 2;
    if (y < 0 || y >= a.Hs || x < 0 || x >= a.Ws) return make_float4(0.f, 0.f, 0.f, 0.f);
    return *reinterpret_cast<const float4*>(in_img + (size_t)y * row_elems + (size_t)x * 16 + 4 * j);
  };
  auto store_chunk = [&](int slot, int q, float4 v) {
    const int c = q / 3, j = q - 3 * c;  // channels 4j..4j+3 = kpairs 2j, 2j+1
    float* base = sR + (size_t)slot * 6 * SF_RC * 2;
    *reinterpret_cast<float2*>(base + ((size_t)(2 * j) * SF_RC + c) * 2) = make_float2(v.x, v.y);
    *reinterpret_cast<float2*>(base + ((size_t)(2 * j + 1) * SF_RC + c) * 2) = make_float2(v.z, v.w);
  };
  auto slot_of = [](int y) { return (y + 2 * SP_RING) % SP_RING; };
  for (int q = tid; q < SP_RING * row_chunks; q += SF_THREADS) {
    const int r = q / row_chunks, qq = q - r * row_chunks;
    const int y = 2 * pys - 2 + r;
    store_chunk(slot_of(y), qq, load_chunk(y, qq));
  }

  const int n = lane & 31, h = lane >> 5;
  const int t = wave & 1;                  // output channel tile
  const int ct0 = SF_TILES * (wave >> 1);  // first column tile
  const int sig = 16 * ((n >> 2) & 1) + (n & 3) + 4 * (n >> 3);
  const float* wcol = sW + h * 64 + 32 * t + sig;  // + (tap * 6 + kp) * 128
  const int xcol = 32 * ct0 + n;                   // this lane's stem column in tile 0

  constexpr int PF_MAX = (2 * row_chunks + SF_THREADS - 1) / SF_THREADS;  // next two s2d rows
  float4 pf[PF_MAX];
  uint32_t pf_ok = 0;

  float carry[SF_TILES][16];
#pragma unroll
  for (int i = 0; i < SF_TILES; ++i)
#pragma unroll
    for (int k = 0; k < 16; ++k) carry[i][k] = 0.f;

  __syncthreads();
  for (int py = pys; py < py1; ++py) {
    const int Y0 = 2 * py;
    const bool more = py + 1 < py1;
    if (more) {
      pf_ok = 0;
#pragma unroll
      for (int i = 0; i < PF_MAX; ++i) {
        const int q = tid + SF_THREADS * i;
        const int r = q / row_chunks, qq = q - r * row_chunks;
        const int y = Y0 + 3 + r;
        const int c = qq / 3, j = qq - 3 * c, x = c - 2;
        const bool ok = q < 2 * row_chunks && y < a.Hs && x >= 0 && x < a.Ws;
        const size_t off = ok ? (size_t)y * row_elems + (size_t)x * 16 + 4 * j : 0;
        pf[i] = *reinterpret_cast<const float4*>(in_img + off);
        pf_ok |= (uint32_t)ok << i;
      }
    }
    f32x16 acc[SF_TILES][2];
#pragma unroll
    for (int i = 0; i < SF_TILES; ++i)
#pragma unroll
      for (int r = 0; r < 2; ++r) acc[i][r] = f32x16{};
    // ring rows of stem rows Y0 (r = 0) and Y0 + 1 (r = 1) for filter row ky
    auto ring_row = [&](int y) { return sR + (size_t)slot_of(y) * 6 * SF_RC * 2 + h + 2 * xcol; };
    sf_filter_row<3>(acc, ring_row(Y0 - 2), ring_row(Y0 - 1), wcol);  // ky = 0: no dy = 0 rows
#pragma unroll 1
    for (int ky = 1; ky < 4; ++ky) sf_filter_row<0>(acc, ring_row(Y0 - 2 + ky), ring_row(Y0 - 1 + ky), wcol + ky * 4 * 6 * 128);

    // bias + ReLU, vertical max with the carried row (all values >= 0, so 0 is the pool padding);
    // the window max overwrites acc[i][0] in place
    const bool row1_ok = Y0 + 1 < a.Hs;
#pragma unroll
    for (int i = 0; i < SF_TILES; ++i) {
      const bool col_ok = xcol + 32 * i < a.Ws;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float b = sBias[32 * t + 16 * h + k];
        const float p0 = fmaxf(acc[i][0][k] + b, 0.f);
        const float p1 = row1_ok ? fmaxf(acc[i][1][k] + b, 0.f) : 0.f;
        acc[i][0][k] = col_ok ? fmaxf(fmaxf(carry[i][k], p0), p1) : 0.f;
        carry[i][k] = p1;
      }
    }
    if (n == 31) {
#pragma unroll
      for (int k = 0; k < 16; ++k) sEdge[(wave * 2 + h) * 16 + k] = acc[SF_TILES - 1][0][k];
    }
    __syncthreads();

    if (more) {
#pragma unroll
      for (int i = 0; i < PF_MAX; ++i) {
        const int q = tid + SF_THREADS * i;
        if (q < 2 * row_chunks) {
          const int r = q / row_chunks, qq = q - r * row_chunks;
          const float4 v = ((pf_ok >> i) & 1u) ? pf[i] : make_float4(0.f, 0.f, 0.f, 0.f);
          store_chunk(slot_of(Y0 + 3 + r), qq, v);
        }
      }
    }
    if (py >= py0) {
      // horizontal window: stem columns 2px - 1, 2px, 2px + 1 around the even lanes; column
      // 32 ct - 1 comes from the previous tile's lane 31 (or the left wave pair's edge)
#pragma unroll
      for (int i = 0; i < SF_TILES; ++i) {
        const int px = 16 * (ct0 + i) + (n >> 1);
        const bool store = (n & 1) == 0 && px < a.Wp;
        float* dst = a.out + (((size_t)img * a.Hp + py) * a.Wp + px) * 64 + 32 * t + 16 * h;
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int k = 4 * k4 + e;
            float left = __shfl_up(acc[i][0][k], 1);
            const float right = __shfl_down(acc[i][0][k], 1);
            float prev;
            if (i > 0)
              prev = __shfl(acc[i - 1][0][k], (lane & 32) | 31);
            else
              prev = wave >= 2 ? sEdge[((wave - 2) * 2 + h) * 16 + k] : 0.f;
            if (n == 0) left = prev;
            o[e] = fmaxf(fmaxf(left, acc[i][0][k]), right);
          }
          if (store) *reinterpret_cast<float4*>(dst + 4 * k4) = make_float4(o[0], o[1], o[2], o[3]);
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// f32-accurate form on the quantised image (rmbx_render policy_dtype 4): the pixels the policy
// sees are x = (u / 255 - mean[c]) / std[c] with u an 8-bit integer (RolloutBase.py:479-490 +
// the backbone's ImageNet normalisation), i.e. x = W'(u - 128) + c' with W' = 1 / (255 std) and
// c' = (128 / 255 - mean) / std, so
//   conv(x)[co] = sum_in W[co][tap][ch] W'[ch] (u - 128)[tap][ch]  +  bias  +  sum_in W c'
// with "in" = the taps inside the image.  The pixels are CENTRED: the large mean term of the
// uncentred form (sum W mean/std, ~2 per tap) no longer cancels against sum W' u, the constant
// left (c' ~ 0.2) is 10x smaller and |u - 128| <= 128 is exact in bf16; W W' is split exactly
// into three bf16 pieces (RNE at each level, as rmbx_linear_f32x6), so the three piece products
// are exact in the f32 accumulator:
// v_mfma_f32_32x32x16_bf16, 3 MFMAs of 32 cycles per 16-channel tap against 8 of 64 cycles for
// the f32 kernel's 32x32x2_f32 (per k: 6 cycles vs 32).  The mean term is constant except where
// taps fall outside the image: bias_eff = bias - (the term of all 16 taps) and edge[rm][cm][co]
// adds back the term of the out-of-range taps (row mask rm of ky, column mask cm of kx).
// Mapping as the bf16 kernel: wave w = stem column tile w (32 columns), two stem rows x two
// 32-channel tiles = 4 accumulators; the three weight planes stay in LDS (96 KiB), the input
// rows in a 5-row LDS ring of bf16 integers converted from the u8 image (16 B per s2d pixel).
// ---------------------------------------------------------------------------------------------
constexpr int SQ_LDS_BYTES = 16 * 3 * 2 * 64 * 16 + SP_RING * 2 * SP_RC_MAX * 16 + 64 * 4 + SP_MAX_WAVES * 2 * 32 * 4;
static_assert(SQ_LDS_BYTES <= 160 * 1024, "u8 stem+pool LDS must fit the 160 KiB of a CU");

struct StemPoolU8Args {
  const uint8_t* in;    // [N][Hs][Ws][16] u8
  const uint16_t* w;    // [3 pieces][64][16 taps][16] bf16 bits (f16 form: [2 pieces] f16 bits)
  float wscale;         // f16 form: the factor undoing the weights' power-of-two scale
  const float* bias;    // [64] bias_eff
  const float* edge;    // [16 rm][16 cm][64]
  float* out;           // [N][Hp][Wp][64]
  int N, Hs, Ws, Hp, Wp;
  int nct, rc;
  int bands, band_rows;
};

// 16 u8 pixel channels -> two 16-B halves of the CENTRED bf16 integers u - 128 (exact: |u - 128|
// <= 128 holds <= 8 significant bits); ok = false (outside the image): zeros, the conv's padding
__device__ __forceinline__ void u8x16_to_bf16(uint4 v, bool ok, uint4& lo, uint4& hi) {
  uint32_t o[8];
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t b0 = __float_as_uint((float)((int)(w[i] & 0xffu) - 128));
    const uint32_t b1 = __float_as_uint((float)((int)((w[i] >> 8) & 0xffu) - 128));
    const uint32_t b2 = __float_as_uint((float)((int)((w[i] >> 16) & 0xffu) - 128));
    const uint32_t b3 = __float_as_uint((float)((int)(w[i] >> 24) - 128));
    o[2 * i] = (b0 >> 16) | (b1 & 0xffff0000u);
    o[2 * i + 1] = (b2 >> 16) | (b3 & 0xffff0000u);
  }
  lo = ok ? make_uint4(o[0], o[1], o[2], o[3]) : make_uint4(0, 0, 0, 0);
  hi = ok ? make_uint4(o[4], o[5], o[6], o[7]) : make_uint4(0, 0, 0, 0);
}

__global__ void __launch_bounds__(SP_THREADS) stem_pool_u8_kernel(StemPoolU8Args a) {
  __shared__ __attribute__((aligned(16))) unsigned char sq_smem[SQ_LDS_BYTES];
  uint16_t* sW = reinterpret_cast<uint16_t*>(sq_smem);       // [16 taps][3 pieces][2 halves][64 cout][8]
  uint16_t* sR = sW + 16 * 3 * 2 * 64 * 8;                   // [5 slots][2 halves][rc][8]
  float* sBias = reinterpret_cast<float*>(sR + SP_RING * 2 * a.rc * 8);  // [64]
  float* sEdge = sBias + 64;                                             // [nct][2 h][2 t][16]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nthreads = blockDim.x;
  const int img = blockIdx.x / a.bands, band = blockIdx.x - img * a.bands;
  const int py0 = band * a.band_rows;
  const int py1 = min(a.Hp, py0 + a.band_rows);
  if (py0 >= py1) return;
  const int pys = py0 > 0 ? py0 - 1 : 0;
  const size_t row_px = (size_t)a.Ws;
  const uint8_t* in_img = a.in + (size_t)img * a.Hs * row_px * 16;

  // weight planes: global [p][cout][tap][16] -> sW[tap][p][half][cout][8]
  for (int q = tid; q < 3 * 64 * 16 * 2; q += nthreads) {
    const int half = q & 1, rest = q >> 1;  // rest = (p * 64 + cout) * 16 + tap
    const int tap = rest & 15, pc = rest >> 4;
    const int co = pc & 63, p = pc >> 6;
    *reinterpret_cast<uint4*>(sW + (((tap * 3 + p) * 2 + half) * 64 + co) * 8) =
        *reinterpret_cast<const uint4*>(a.w + (size_t)rest * 16 + half * 8);
  }
  if (tid < 64) sBias[tid] = a.bias[tid];

  // s2d pixel (ring col c) of row y -> both halves; zero outside the image
  auto px_ok = [&](int y, int c) { return y >= 0 && y < a.Hs && c - 2 >= 0 && c - 2 < a.Ws; };
  auto load_px = [&](int y, int c) -> uint4 {
    if (!px_ok(y, c)) return make_uint4(0, 0, 0, 0);
    return *reinterpret_cast<const uint4*>(in_img + ((size_t)y * row_px + c - 2) * 16);
  };
  auto store_px = [&](int slot, int c, uint4 v, bool ok) {
    uint4 lo, hi;
    u8x16_to_bf16(v, ok, lo, hi);
    *reinterpret_cast<uint4*>(sR + ((size_t)(slot * 2) * a.rc + c) * 8) = lo;
    *reinterpret_cast<uint4*>(sR + ((size_t)(slot * 2 + 1) * a.rc + c) * 8) = hi;
  };
  auto slot_of = [](int y) { return (y + 2 * SP_RING) % SP_RING; };
  for (int q = tid; q < SP_RING * a.rc; q += nthreads) {
    const int r = q / a.rc, c = q - r * a.rc;
    const int y = 2 * pys - 2 + r;
    store_px(slot_of(y), c, load_px(y, c), px_ok(y, c));
  }

  const int n = lane & 31, h = lane >> 5;
  const int X = 32 * wave + n;
  const int m = lane & 31;
  const int sig = 16 * ((m >> 2) & 1) + (m & 3) + 4 * (m >> 3);
  const bool col_ok = X < a.Ws;
  // out-of-image kx taps of this lane's stem column (the mean term added back by the edge table)
  int cm = 0;
#pragma unroll
  for (int kx = 0; kx < 4; ++kx) cm |= (int)((unsigned)(X - 2 + kx) >= (unsigned)a.Ws) << kx;

  constexpr int PF_MAX = 2;  // (2 rows * 324 cols) / 640 threads, rounded up
  uint4 pf[PF_MAX];
  uint32_t pf_ok = 0;
  const int pf_px = 2 * a.rc;
  int pf_r[PF_MAX], pf_c[PF_MAX];
#pragma unroll
  for (int i = 0; i < PF_MAX; ++i) {
    const int q = min(tid + nthreads * i, pf_px - 1);
    pf_r[i] = q / a.rc;
    pf_c[i] = q - pf_r[i] * a.rc;
  }

  float carry[2][16];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int k = 0; k < 16; ++k) carry[t][k] = 0.f;

  __syncthreads();
  for (int py = pys; py < py1; ++py) {
    const int Y0 = 2 * py;
    const bool more = py + 1 < py1;
    if (more) {
      pf_ok = 0;
#pragma unroll
      for (int i = 0; i < PF_MAX; ++i) {
        const int y = Y0 + 3 + pf_r[i];
        const int x = pf_c[i] - 2;
        const bool ok = tid + nthreads * i < pf_px && y < a.Hs && x >= 0 && x < a.Ws;
        const size_t off = ok ? ((size_t)y * row_px + x) * 16 : 0;
        pf[i] = *reinterpret_cast<const uint4*>(in_img + off);
        pf_ok |= (uint32_t)ok << i;
      }
    }
    f32x16 acc[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[r][t] = f32x16{};
    int slot[5];
#pragma unroll
    for (int d = 0; d < 5; ++d) slot[d] = slot_of(Y0 - 2 + d);
#pragma unroll
    for (int tap = 0; tap < 16; ++tap) {
      const int ky = tap >> 2, kx = tap & 3;
      bf16x8 bx[2], aw[2][3];
#pragma unroll
      for (int r = 0; r < 2; ++r)
        bx[r] = *reinterpret_cast<const bf16x8*>(sR + (((size_t)slot[r + ky] * 2 + h) * a.rc + X + kx) * 8);
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          aw[t][p] = *reinterpret_cast<const bf16x8*>(sW + (((tap * 3 + p) * 2 + h) * 64 + 32 * t + sig) * 8);
      // small pieces first
#pragma unroll
      for (int p = 2; p >= 0; --p)
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int t = 0; t < 2; ++t)
            acc[r][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aw[t][p], bx[r], acc[r][t], 0, 0, 0);
    }

    // bias_eff (+ the edge term of the out-of-image taps) + ReLU, vertical max with the carried row
    const bool row1_ok = Y0 + 1 < a.Hs;
    int rm[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      rm[r] = 0;
#pragma unroll
      for (int ky = 0; ky < 4; ++ky) rm[r] |= (int)((unsigned)(Y0 + r - 2 + ky) >= (unsigned)a.Hs) << ky;
    }
    const float* ep0 = (rm[0] | cm) ? a.edge + (rm[0] * 16 + cm) * 64 + 16 * h : nullptr;
    const float* ep1 = (rm[1] | cm) ? a.edge + (rm[1] * 16 + cm) * 64 + 16 * h : nullptr;
    float vm[2][16];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float b = sBias[32 * t + 16 * h + k];
        float v0 = acc[0][t][k] + b, v1 = acc[1][t][k] + b;
        if (ep0) v0 += ep0[32 * t + k];  // border pixels only
        if (ep1) v1 += ep1[32 * t + k];
        const float p0 = fmaxf(v0, 0.f);
        const float p1 = row1_ok ? fmaxf(v1, 0.f) : 0.f;
        vm[t][k] = col_ok ? fmaxf(fmaxf(carry[t][k], p0), p1) : 0.f;
        carry[t][k] = p1;
      }
    }
    if (n == 31) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int k = 0; k < 16; ++k) sEdge[((wave * 2 + h) * 2 + t) * 16 + k] = vm[t][k];
    }
    __syncthreads();  // edges visible; every wave is done with ring rows 2py-2, 2py-1

    if (more) {
#pragma unroll
      for (int i = 0; i < PF_MAX; ++i) {
        if (tid + nthreads * i < pf_px) {
          // row Y0+3+r replaces row Y0-2+r
          store_px(pf_r[i] ? slot[1] : slot[0], pf_c[i], pf[i], (pf_ok >> i) & 1u);
        }
      }
    }
    if (py >= py0) {
      const int px = 16 * wave + (n >> 1);
      const bool store = (n & 1) == 0 && px < a.Wp;
      float* dst = a.out + (((size_t)img * a.Hp + py) * a.Wp + px) * 64 + 16 * h;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int k = 4 * k4 + e;
            float left = __shfl_up(vm[t][k], 1);
            const float right = __shfl_down(vm[t][k], 1);
            if (n == 0) left = wave > 0 ? sEdge[(((wave - 1) * 2 + h) * 2 + t) * 16 + k] : 0.f;
            o[e] = fmaxf(fmaxf(left, vm[t][k]), right);
          }
          if (store) *reinterpret_cast<float4*>(dst + 32 * t + 4 * k4) = make_float4(o[0], o[1], o[2], o[3]);
        }
    }
    __syncthreads();  // ring refilled; edge reads done before the next pair overwrites them
  }
}

// The same u8 stem in the f32 kernel's SIMD-balanced layout: 4 waves per block (one per SIMD;
// 10 waves would sit 3/3/2/2 on the SIMDs of an MFMA-bound kernel), wave w = 32-channel tile
// w & 1 of column tiles 5 (w >> 1) .. + 4 for both stem rows (10 accumulators, 512 registers).
// the value of lane l - 1 / l + 1 by a DPP wave shift (one VALU move instead of an LDS permute;
// gfx9 wave_shr:1 / wave_shl:1; the lanes without a neighbour are overridden by the caller)
// (bound_ctrl: a lane without a source reads 0 -- no separate zero-initialised destination)
__device__ __forceinline__ float dpp_from_left(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float dpp_from_right(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x130, 0xf, 0xf, true));
}

// 16 u8 pixel channels -> two 16-B halves of the CENTRED f16 integers u - 128 (exact)
// (two bytes at a time: v_perm_b32 places each byte under the f16 exponent of 1024 -- 0x6400 | u is
// 1024 + u exactly -- and one packed f16 subtract of 1152 leaves u - 128, exact; two instructions
// per pair instead of the extract / convert / round chain)
__device__ __forceinline__ void u8x16_to_f16(uint4 v, bool ok, uint4& lo, uint4& hi) {
  uint32_t o[8];
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  const f16x2s off = {(_Float16)1152.0f, (_Float16)1152.0f};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t e0 = __builtin_amdgcn_perm(0x64646464u, w[i], 0x04010400u);  // {0x64 b1, 0x64 b0}
    const uint32_t e1 = __builtin_amdgcn_perm(0x64646464u, w[i], 0x04030402u);  // {0x64 b3, 0x64 b2}
    o[2 * i] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2s, e0) - off);
    o[2 * i + 1] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2s, e1) - off);
  }
  lo = ok ? make_uint4(o[0], o[1], o[2], o[3]) : make_uint4(0, 0, 0, 0);
  hi = ok ? make_uint4(o[4], o[5], o[6], o[7]) : make_uint4(0, 0, 0, 0);
}

// H2 (the default): the f16 form -- the integer pixels (exact in f16) times two f16 pieces of
// W W' 2^s (hi = f16(x), lo = f16(x - hi), one power of two s for the whole filter bank putting
// its max in [2^13, 2^14)), both products in one accumulator on v_mfma_f32_32x32x16_f16 and the
// accumulator scaled by 2^-s before the bias: 2 MFMAs per tap and tile instead of 3, weights
// represented to 2^-22 (the f16x3 GEMM's weight split, csrc/rmbx_gemm.hip)
// VAR (profiling, RMBX_STEM_VAR; wrong results, timing only): bit 0 = no pool epilogue (one store
// per lane keeps the accumulators live), bit 1 = no ring refill (no prefetch loads / conversions),
// bit 2 = no MFMAs.  Round 4 (profiles/r4_stem_u8h_phase_skips.log -> ..._epilogue_v2.log): the
// pool epilogue cost more than the MFMAs (8.17 ms per 1024 frames, 3.55 without it); without its
// per-element branches (edge terms behind one wave-uniform test per tile, the column mask as a bit
// mask, the left neighbour by two readlanes instead of an LDS permute, DPP moves with bound_ctrl)
// the kernel runs 5.62 ms.
template <bool DPP, bool H2 = false, int VAR = 0>
__global__ void __launch_bounds__(SF_THREADS) stem_pool_u8w4_kernel(StemPoolU8Args a) {
  constexpr int NP = H2 ? 2 : 3;  // weight pieces
  __shared__ __attribute__((aligned(16))) unsigned char sq_smem[16 * NP * 2 * 64 * 16 + SP_RING * 2 * SF_RC * 16 +
                                                               64 * 4 + SF_WAVES * 2 * 16 * 4];
  uint16_t* sW = reinterpret_cast<uint16_t*>(sq_smem);  // [16 taps][NP pieces][2 halves][64 cout][8]
  uint16_t* sR = sW + 16 * NP * 2 * 64 * 8;             // [5 slots][2 halves][SF_RC][8]
  float* sBias = reinterpret_cast<float*>(sR + SP_RING * 2 * SF_RC * 8);  // [64]
  float* sEdge = sBias + 64;                                              // [waves][2 h][16]

  // (the wave index as a scalar: the tile / channel-half choices derived from it stay uniform)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int img = blockIdx.x / a.bands, band = blockIdx.x - img * a.bands;
  const int py0 = band * a.band_rows;
  const int py1 = min(a.Hp, py0 + a.band_rows);
  if (py0 >= py1) return;
  const int pys = py0 > 0 ? py0 - 1 : 0;
  const size_t row_px = (size_t)a.Ws;
  const uint8_t* in_img = a.in + (size_t)img * a.Hs * row_px * 16;

  for (int q = tid; q < NP * 64 * 16 * 2; q += SF_THREADS) {
    const int half = q & 1, rest = q >> 1;
    const int tap = rest & 15, pc = rest >> 4;
    const int co = pc & 63, p = pc >> 6;
    *reinterpret_cast<uint4*>(sW + (((tap * NP + p) * 2 + half) * 64 + co) * 8) =
        *reinterpret_cast<const uint4*>(a.w + (size_t)rest * 16 + half * 8);
  }
  if (tid < 64) sBias[tid] = a.bias[tid];

  auto store_px = [&](int slot, int c, uint4 v, bool ok) {
    uint4 lo, hi;
    if constexpr (H2)
      u8x16_to_f16(v, ok, lo, hi);
    else
      u8x16_to_bf16(v, ok, lo, hi);
    *reinterpret_cast<uint4*>(sR + ((size_t)(slot * 2) * SF_RC + c) * 8) = lo;
    *reinterpret_cast<uint4*>(sR + ((size_t)(slot * 2 + 1) * SF_RC + c) * 8) = hi;
  };
  auto slot_of = [](int y) { return (y + 2 * SP_RING) % SP_RING; };
  for (int q = tid; q < SP_RING * SF_RC; q += SF_THREADS) {
    const int r = q / SF_RC, c = q - r * SF_RC;
    const int y = 2 * pys - 2 + r, x = c - 2;
    uint4 v = make_uint4(0, 0, 0, 0);
    const bool ok = y >= 0 && y < a.Hs && x >= 0 && x < a.Ws;
    if (ok) v = *reinterpret_cast<const uint4*>(in_img + ((size_t)y * row_px + x) * 16);
    store_px(slot_of(y), c, v, ok);
  }

  const int n = lane & 31, h = lane >> 5;
  const int t = wave & 1;
  const int ct0 = SF_TILES * (wave >> 1);
  const int sig = 16 * ((n >> 2) & 1) + (n & 3) + 4 * (n >> 3);
  const int xcol = 32 * ct0 + n;

  constexpr int PF_MAX = (2 * SF_RC + SF_THREADS - 1) / SF_THREADS;
  uint4 pf[PF_MAX];
  uint32_t pf_ok = 0;

  float carry[SF_TILES][16];
#pragma unroll
  for (int i = 0; i < SF_TILES; ++i)
#pragma unroll
    for (int k = 0; k < 16; ++k) carry[i][k] = 0.f;

  __syncthreads();
  for (int py = pys; py < py1; ++py) {
    const int Y0 = 2 * py;
    const bool more = (VAR & 2) == 0 && py + 1 < py1;
    if (more) {
      pf_ok = 0;
#pragma unroll
      for (int i = 0; i < PF_MAX; ++i) {
        const int q = tid + SF_THREADS * i;
        const int r = q / SF_RC, c = q - r * SF_RC;
        const int y = Y0 + 3 + r, x = c - 2;
        const bool ok = q < 2 * SF_RC && y < a.Hs && x >= 0 && x < a.Ws;
        const size_t off = ok ? ((size_t)y * row_px + x) * 16 : 0;
        pf[i] = *reinterpret_cast<const uint4*>(in_img + off);
        pf_ok |= (uint32_t)ok << i;
      }
    }
    f32x16 acc[SF_TILES][2];
#pragma unroll
    for (int i = 0; i < SF_TILES; ++i)
#pragma unroll
      for (int r = 0; r < 2; ++r) acc[i][r] = f32x16{};
    int slot[5];
#pragma unroll
    for (int d = 0; d < 5; ++d) slot[d] = slot_of(Y0 - 2 + d);
#pragma unroll
    for (int tap = 0; tap < 16; ++tap) {
      const int ky = tap >> 2, kx = tap & 3;
      bf16x8 aw[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p)
        aw[p] = *reinterpret_cast<const bf16x8*>(sW + (((tap * NP + p) * 2 + h) * 64 + 32 * t + sig) * 8);
#pragma unroll
      for (int i = 0; i < SF_TILES; ++i) {
        bf16x8 bx[2];
#pragma unroll
        for (int r = 0; r < 2; ++r)
          bx[r] = *reinterpret_cast<const bf16x8*>(sR + (((size_t)slot[r + ky] * 2 + h) * SF_RC + xcol + 32 * i + kx) * 8);
#pragma unroll
        for (int p = NP - 1; p >= 0; --p)
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            if constexpr ((VAR & 4) != 0)
              acc[i][r][p] += __uint_as_float(__builtin_bit_cast(uint4, aw[p]).x ^ __builtin_bit_cast(uint4, bx[r]).y);
            else if constexpr (H2)
              acc[i][r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8s, aw[p]),
                                                                  __builtin_bit_cast(f16x8s, bx[r]), acc[i][r], 0, 0, 0);
            else
              acc[i][r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aw[p], bx[r], acc[i][r], 0, 0, 0);
          }
      }
    }

    if constexpr ((VAR & 1) != 0) {
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < SF_TILES; ++i)
#pragma unroll
        for (int k = 0; k < 16; ++k) sum += acc[i][0][k] + acc[i][1][k];
      a.out[(((size_t)img * a.Hp + py) * a.Wp) * 64 + tid] = sum;
      __syncthreads();
      if (more) {
#pragma unroll
        for (int i = 0; i < PF_MAX; ++i) {
          const int q = tid + SF_THREADS * i;
          if (q < 2 * SF_RC) {
            const int r = q / SF_RC, c = q - r * SF_RC;
            store_px(slot_of(Y0 + 3 + r), c, pf[i], (pf_ok >> i) & 1u);
          }
        }
      }
      __syncthreads();
      continue;
    }
    const bool row1_ok = Y0 + 1 < a.Hs;
    bool tile_edge[SF_TILES];  // wave-uniform: tile i holds a column within 2 of either image edge
#pragma unroll
    for (int i = 0; i < SF_TILES; ++i) {
      const int X0 = 32 * (ct0 + i);
      tile_edge[i] = X0 < 2 || X0 + 33 >= a.Ws;
    }
    int rm[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      rm[r] = 0;
#pragma unroll
      for (int ky = 0; ky < 4; ++ky) rm[r] |= (int)((unsigned)(Y0 + r - 2 + ky) >= (unsigned)a.Hs) << ky;
    }
#pragma unroll
    for (int i = 0; i < SF_TILES; ++i) {
      const int X = xcol + 32 * i;
      const bool col_ok = X < a.Ws;
      int cm = 0;
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) cm |= (int)((unsigned)(X - 2 + kx) >= (unsigned)a.Ws) << kx;
      // the mean term of the out-of-image taps: only rows near the image's top / bottom and the
      // first / last column tiles have any (a wave-uniform test, no per-element exec masking); the
      // edge table's entry (0, 0) is zero, so every lane reads a valid row
      const int col_mask = col_ok ? -1 : 0;
      const float* ep0 = a.edge + (rm[0] * 16 + cm) * 64 + 32 * t + 16 * h;
      const float* ep1 = a.edge + (rm[1] * 16 + cm) * 64 + 32 * t + 16 * h;
      auto pool_rows = [&](auto edge) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const float b = sBias[32 * t + 16 * h + k];
          float v0, v1;
          if constexpr (H2) {  // undo the weights' power of two (exact), then the bias
            v0 = fmaf(acc[i][0][k], a.wscale, b);
            v1 = fmaf(acc[i][1][k], a.wscale, b);
          } else {
            v0 = acc[i][0][k] + b;
            v1 = acc[i][1][k] + b;
          }
          if constexpr (decltype(edge)::value) {  // + 0 where no tap is outside
            v0 += ep0[k];
            v1 += ep1[k];
          }
          const float p0 = fmaxf(v0, 0.f);
          const float p1 = fmaxf(v1, 0.f);  // 0 for a missing second row (-inf, set above)
          // columns past the image: 0 (a bit mask, not a select the compiler turns into a branch)
          acc[i][0][k] = __int_as_float(__float_as_int(fmaxf(fmaxf(carry[i][k], p0), p1)) & col_mask);
          carry[i][k] = p1;
        }
      };
      if (!row1_ok) {  // odd stem height: the last pool row has one stem row; -inf pools as 0
#pragma unroll
        for (int k = 0; k < 16; ++k) acc[i][1][k] = -INFINITY;
      }
      if (rm[0] != 0 || rm[1] != 0 || tile_edge[i])
        pool_rows(std::true_type{});
      else
        pool_rows(std::false_type{});
    }
    if (n == 31) {
#pragma unroll
      for (int k = 0; k < 16; ++k) sEdge[(wave * 2 + h) * 16 + k] = acc[SF_TILES - 1][0][k];
    }
    __syncthreads();

    if (more) {
#pragma unroll
      for (int i = 0; i < PF_MAX; ++i) {
        const int q = tid + SF_THREADS * i;
        if (q < 2 * SF_RC) {
          const int r = q / SF_RC, c = q - r * SF_RC;
          store_px(slot_of(Y0 + 3 + r), c, pf[i], (pf_ok >> i) & 1u);
        }
      }
    }
    if (py >= py0) {
#pragma unroll
      for (int i = 0; i < SF_TILES; ++i) {
        const int px = 16 * (ct0 + i) + (n >> 1);
        const bool store = (n & 1) == 0 && px < a.Wp;
        float* dst = a.out + (((size_t)img * a.Hp + py) * a.Wp + px) * 64 + 32 * t + 16 * h;
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int k = 4 * k4 + e;
            float left = DPP ? dpp_from_left(acc[i][0][k]) : __shfl_up(acc[i][0][k], 1);
            const float right = DPP ? dpp_from_right(acc[i][0][k]) : __shfl_down(acc[i][0][k], 1);
            float prev;
            if (i > 0) {  // lane 31 / 63 of the tile on the left (same channel half): two readlanes
              const int x = __float_as_int(acc[i - 1][0][k]);
              const int l31 = __builtin_amdgcn_readlane(x, 31), l63 = __builtin_amdgcn_readlane(x, 63);
              prev = __int_as_float(l31 ^ ((l31 ^ l63) & -h));
            } else
              prev = wave >= 2 ? sEdge[((wave - 2) * 2 + h) * 16 + k] : 0.f;
            if (n == 0) left = prev;
            o[e] = fmaxf(fmaxf(left, acc[i][0][k]), right);
          }
          if (store) *reinterpret_cast<float4*>(dst + 4 * k4) = make_float4(o[0], o[1], o[2], o[3]);
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_stem_s2d_conv_maxpool(const void* in, const void* weight, const float* bias, void* out, int N,
                                          int Hs, int Ws, int band_rows, void* stream) {
  RMBX_CHECK_ARG(in && weight && bias && out, "rmbx_stem_s2d_conv_maxpool: null pointer");
  RMBX_CHECK_ARG(N >= 0 && Hs > 0 && Ws > 0, "rmbx_stem_s2d_conv_maxpool: bad geometry");
  RMBX_CHECK_ARG(Ws <= 32 * rmbx::SP_MAX_WAVES, "rmbx_stem_s2d_conv_maxpool: Ws=%d exceeds %d", Ws,
                 32 * rmbx::SP_MAX_WAVES);
  RMBX_CHECK_ARG((((uintptr_t)in | (uintptr_t)weight | (uintptr_t)out) & 15) == 0,
                 "rmbx_stem_s2d_conv_maxpool: in/weight/out must be 16-byte aligned");
  if (N == 0) return RMBX_OK;
  rmbx::StemPoolArgs a;
  a.in = (const uint16_t*)in;
  a.w = (const uint16_t*)weight;
  a.bias = bias;
  a.out = (uint16_t*)out;
  a.N = N;
  a.Hs = Hs;
  a.Ws = Ws;
  a.Hp = (Hs - 1) / 2 + 1;
  a.Wp = (Ws - 1) / 2 + 1;
  a.nct = (Ws + 31) / 32;
  a.rc = 32 * a.nct + 4;
  RMBX_CHECK_ARG(2 * 2 * a.rc <= 3 * 64 * a.nct, "rmbx_stem_s2d_conv_maxpool: prefetch does not fit");
  // bands: the whole image per block once there are enough images to fill the chip
  if (band_rows <= 0) {
    const int want_blocks = 512;
    int bands = (want_blocks + N - 1) / N;
    if (bands > a.Hp) bands = a.Hp;
    band_rows = (a.Hp + bands - 1) / bands;
  }
  a.band_rows = band_rows;
  a.bands = (a.Hp + band_rows - 1) / band_rows;
  const long long nblocks = (long long)N * a.bands;
  RMBX_CHECK_ARG(nblocks < (1ll << 31), "rmbx_stem_s2d_conv_maxpool: grid too large");
  hipLaunchKernelGGL(rmbx::stem_pool_kernel, dim3((unsigned)nblocks), dim3(64 * a.nct), 0, (hipStream_t)stream, a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

namespace rmbx {
int stem_u8_impl(const uint8_t* in, const void* w_planes, float wscale, bool h2, const float* bias, const float* edge,
                 float* out, int N, int Hs, int Ws, int band_rows, void* stream);
}  // namespace rmbx

extern "C" int rmbx_stem_s2d_conv_maxpool_u8(const uint8_t* in, const void* w_planes, const float* bias,
                                             const float* edge, float* out, int N, int Hs, int Ws, int band_rows,
                                             void* stream) {
  return rmbx::stem_u8_impl(in, w_planes, 1.f, false, bias, edge, out, N, Hs, Ws, band_rows, stream);
}

extern "C" int rmbx_stem_s2d_conv_maxpool_u8h(const uint8_t* in, const void* w_planes, float wscale, const float* bias,
                                              const float* edge, float* out, int N, int Hs, int Ws, int band_rows,
                                              void* stream) {
  RMBX_CHECK_ARG(wscale > 0.f, "rmbx_stem_s2d_conv_maxpool_u8h: wscale must be positive");
  return rmbx::stem_u8_impl(in, w_planes, wscale, true, bias, edge, out, N, Hs, Ws, band_rows, stream);
}

int rmbx::stem_u8_impl(const uint8_t* in, const void* w_planes, float wscale, bool h2, const float* bias,
                       const float* edge, float* out, int N, int Hs, int Ws, int band_rows, void* stream) {
  RMBX_CHECK_ARG(in && w_planes && bias && edge && out, "rmbx_stem_s2d_conv_maxpool_u8: null pointer");
  RMBX_CHECK_ARG(N >= 0 && Hs > 0 && Ws > 0, "rmbx_stem_s2d_conv_maxpool_u8: bad geometry");
  RMBX_CHECK_ARG(Ws <= 32 * rmbx::SP_MAX_WAVES, "rmbx_stem_s2d_conv_maxpool_u8: Ws=%d exceeds %d", Ws,
                 32 * rmbx::SP_MAX_WAVES);
  RMBX_CHECK_ARG((((uintptr_t)in | (uintptr_t)w_planes | (uintptr_t)edge | (uintptr_t)out) & 15) == 0,
                 "rmbx_stem_s2d_conv_maxpool_u8: in/w_planes/edge/out must be 16-byte aligned");
  if (N == 0) return RMBX_OK;
  rmbx::StemPoolU8Args a;
  a.in = in;
  a.w = (const uint16_t*)w_planes;
  a.wscale = wscale;
  a.bias = bias;
  a.edge = edge;
  a.out = out;
  a.N = N;
  a.Hs = Hs;
  a.Ws = Ws;
  a.Hp = (Hs - 1) / 2 + 1;
  a.Wp = (Ws - 1) / 2 + 1;
  a.nct = (Ws + 31) / 32;
  a.rc = 32 * a.nct + 4;
  RMBX_CHECK_ARG(2 * a.rc <= 2 * 64 * a.nct, "rmbx_stem_s2d_conv_maxpool_u8: prefetch does not fit");
  // layout: 4 SIMD-balanced waves (default) or one wave per column tile (RMBX_STEM_U8_LAYOUT=10)
  static const int layout = [] {
    const char* e = getenv("RMBX_STEM_U8_LAYOUT");
    return e ? atoi(e) : 4;
  }();
  // horizontal pool neighbours by DPP wave shifts (default: 8.53 vs 8.89 ms per 1024 frames,
  // profiles/r3_stem_dpp_prof.log) or LDS permutes (RMBX_STEM_U8_DPP=0)
  static const bool dpp = [] {
    const char* e = getenv("RMBX_STEM_U8_DPP");
    return !e || atoi(e) != 0;
  }();
  if (band_rows <= 0) {
    const int want_blocks = 512;
    int bands = (want_blocks + N - 1) / N;
    if (bands > a.Hp) bands = a.Hp;
    band_rows = (a.Hp + bands - 1) / bands;
  }
  a.band_rows = band_rows;
  a.bands = (a.Hp + band_rows - 1) / band_rows;
  const long long nblocks = (long long)N * a.bands;
  RMBX_CHECK_ARG(nblocks < (1ll << 31), "rmbx_stem_s2d_conv_maxpool_u8: grid too large");
  const char* ve = h2 ? getenv("RMBX_STEM_VAR") : nullptr;  // profiling phase skips (read per launch)
  const int var = ve ? atoi(ve) : 0;
  if (h2) {
    const dim3 grid((unsigned)nblocks), blk(rmbx::SF_THREADS);
    switch (var) {
      case 1: hipLaunchKernelGGL((rmbx::stem_pool_u8w4_kernel<true, true, 1>), grid, blk, 0, (hipStream_t)stream, a); break;
      case 2: hipLaunchKernelGGL((rmbx::stem_pool_u8w4_kernel<true, true, 2>), grid, blk, 0, (hipStream_t)stream, a); break;
      case 3: hipLaunchKernelGGL((rmbx::stem_pool_u8w4_kernel<true, true, 3>), grid, blk, 0, (hipStream_t)stream, a); break;
      case 4: hipLaunchKernelGGL((rmbx::stem_pool_u8w4_kernel<true, true, 4>), grid, blk, 0, (hipStream_t)stream, a); break;
      case 6: hipLaunchKernelGGL((rmbx::stem_pool_u8w4_kernel<true, true, 6>), grid, blk, 0, (hipStream_t)stream, a); break;
      default: hipLaunchKernelGGL((rmbx::stem_pool_u8w4_kernel<true, true>), grid, blk, 0, (hipStream_t)stream, a);
    }
  }
  else if (layout == 10)
    hipLaunchKernelGGL(rmbx::stem_pool_u8_kernel, dim3((unsigned)nblocks), dim3(64 * a.nct), 0, (hipStream_t)stream, a);
  else if (dpp)
    hipLaunchKernelGGL(rmbx::stem_pool_u8w4_kernel<true>, dim3((unsigned)nblocks), dim3(rmbx::SF_THREADS), 0,
                       (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(rmbx::stem_pool_u8w4_kernel<false>, dim3((unsigned)nblocks), dim3(rmbx::SF_THREADS), 0,
                       (hipStream_t)stream, a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_stem_s2d_conv_maxpool_f32(const float* in, const float* weight, const float* bias, float* out,
                                              int N, int Hs, int Ws, int band_rows, void* stream) {
  RMBX_CHECK_ARG(in && weight && bias && out, "rmbx_stem_s2d_conv_maxpool_f32: null pointer");
  RMBX_CHECK_ARG(N >= 0 && Hs > 0 && Ws > 0, "rmbx_stem_s2d_conv_maxpool_f32: bad geometry");
  RMBX_CHECK_ARG(Ws <= 32 * rmbx::SP_MAX_WAVES, "rmbx_stem_s2d_conv_maxpool_f32: Ws=%d exceeds %d", Ws,
                 32 * rmbx::SP_MAX_WAVES);
  RMBX_CHECK_ARG((((uintptr_t)in | (uintptr_t)out) & 15) == 0,
                 "rmbx_stem_s2d_conv_maxpool_f32: in/out must be 16-byte aligned");
  if (N == 0) return RMBX_OK;
  rmbx::StemPoolF32Args a;
  a.in = in;
  a.w = weight;
  a.bias = bias;
  a.out = out;
  a.N = N;
  a.Hs = Hs;
  a.Ws = Ws;
  a.Hp = (Hs - 1) / 2 + 1;
  a.Wp = (Ws - 1) / 2 + 1;
  if (band_rows <= 0) {
    const int want_blocks = 512;
    int bands = (want_blocks + N - 1) / N;
    if (bands > a.Hp) bands = a.Hp;
    band_rows = (a.Hp + bands - 1) / bands;
  }
  a.band_rows = band_rows;
  a.bands = (a.Hp + band_rows - 1) / band_rows;
  const long long nblocks = (long long)N * a.bands;
  RMBX_CHECK_ARG(nblocks < (1ll << 31), "rmbx_stem_s2d_conv_maxpool_f32: grid too large");
  hipLaunchKernelGGL(rmbx::stem_pool_f32_kernel, dim3((unsigned)nblocks), dim3(rmbx::SF_THREADS), 0, (hipStream_t)stream, a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
