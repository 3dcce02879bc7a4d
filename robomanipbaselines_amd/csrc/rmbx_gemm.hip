// fp32-accurate GEMM on the bf16 matrix cores: C = relu?(A . W^T + bias), A and C f32.
//
// Replaces the fp32 nn.Linear / nn.MultiheadAttention in-projections of ACT's transformer
// (third_party/act [absent]: detr/models/transformer.py; the reference runs the policy in fp32,
// policy/act/RolloutAct.py) for the fp32 policy path.  gfx950 runs f32-input MFMA at the f32
// vector rate (157 TF/s, no TF32) but bf16 MFMA at 2.5 PF/s, 16x more.  Every f32 operand is
// split exactly into three bf16 pieces, x = x0 + x1 + x2 (round-to-nearest-even at each level,
// so |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|; 3 x 8 significant bits hold all 24 of an f32), and the
// product is the sum of the six piece products with i + j <= 2:
//
//   a.b ~ a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0)        (dropped terms <= 2^-24 |ab|)
//
// Each piece product is exact in the f32 accumulator (8 x 8 significant bits), so the result
// differs from an exact dot product by the f32 accumulation rounding plus <= ~2^-23 relative per
// term: the same error class as an f32 GEMM (measured lower than hipBLASLt's f32 GEMM against an
// f64 product, tests/test_gemm_gpu.py).  Six bf16 MFMAs per f32 product step = 2.67x the f32
// MFMA rate at equal efficiency.
//
// W is split once per weight on the device (rmbx_split_bf16x3, planes [3][N][K]); A (the
// activations) is split once per block as it is staged into LDS.
//
// Mapping: block = 8 waves (2 per SIMD) owns a 256 x 128 output tile; wave (wm, wn) a 64 x 64
// sub-tile = 4 x 4 v_mfma_f32_16x16x32_bf16 accumulators (the 16x16x32 form holds a higher clock
// than 32x32x16 on random data under DVFS, MI355X_MICROARCH.md).  K runs in steps of 32 over two
// LDS stages of 72 KiB: the three W planes (3 x 128 x 32 bf16) arrive by LDS-DMA
// (global_load_lds_dwordx4); the A tile (256 x 32 f32) is loaded into registers two steps ahead,
// split into its three bf16 pieces (VALU) and stored as three planes (3 x 256 x 32 bf16) between
// the two MFMA halves of the step before it is used.  Every plane row (32 k) is four 16-B slots,
// XOR-swizzled by (row >> 2) & 2 so the fragment reads, the DMA pieces and the A stores are all
// LDS-bank-conflict-free.  Blocks are mapped XCD-contiguously and in groups of 8 row tiles x all
// column tiles, so the A rows and W columns an XCD streams stay in its L2.
//
// f16x3 form (PC = 2, rmbx_linear_f16x3 / _batched / rmbx_conv2d_f16x3): the same kernel with two
// f16 pieces per operand (11 significant bits each) and three products on
// v_mfma_f32_16x16x32_f16 (the bf16 rate), all accumulated in one f32 accumulator:
//
//   W row n scaled by a power of two s_n (max |w s_n| in [2^13, 2^14)):
//     w' = w s_n = hb + lb,          hb = f16(w'), lb = f16(w' - hb)
//   a = ha + 2^-11 la,               ha = f16(a),  la = f16((a - ha) 2^11)
//   a.w' ~ ha hb + ha lb + la (2^-11 hb)                         (dropped term <= 2^-22 |a w'|)
//
// a's low piece is carried scaled by 2^11 so it stays in f16's normal range (the split of Ootomo &
// Yokota, IJHPCA 2022), and the scale is undone on W's side: 2^-11 hb is formed in registers
// (v_pk_mul_f16, exact for |hb| >= 2^-3, i.e. every element above 2^-16 of its row's max; smaller
// ones round to f16 subnormals, 2^-38 of the row max), so the three products share one
// accumulator.  Each piece product is exact in f32 (11 x 11 bits): the error is the f32
// accumulation plus <= ~3 * 2^-22 relative per term, measured below hipBLASLt's f32 GEMM against
// an f64 product at every tested shape (tests/test_gemm_gpu.py).  Three products instead of six:
// half the MFMA work of bf16x6.  f16's exponent range is handled exactly: W by the row scales
// (packed once, rmbx_split_f16x2; 1 / s_n applied per output column in the epilogue), a by a
// per-row check: every block tracks the largest |a| of each of its rows, and a row whose max lies
// outside [2^-6, 2^15] (values that would overflow f16 or sit in its subnormal range) is split
// again as a 2^t with t putting its max in [2^13, 2^14), its result scaled back by 2^-t (powers
// of two: exact): the block re-runs its K loop with the other rows at scale 1 (bit-identical to
// the first pass), so every row's result depends on that row alone (batch invariance).
#include "rmbx_common.h"

#include <cstdint>
#include <cstdlib>
#include <type_traits>

namespace rmbx {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

constexpr int GM_BM = 256, GM_BN = 128, GM_BK = 32;
constexpr int GM_THREADS = 512;
constexpr int GM_A_PLANE = GM_BM * GM_BK * 2;            // 16 KiB per 16-bit piece plane
constexpr int GM_GROUP = 8;                              // row tiles per block group
// PC pieces per operand (3: bf16x6, 2: f16x3), BN output columns per block (128, or 64 for the
// f16x3 form's narrow layers): one K stage = PC A planes + PC W planes of BN x 32
template <int BN>
constexpr int gm_b_plane() { return BN * GM_BK * 2; }  // 8 KiB at BN = 128
template <int PC, int BN = 128>
constexpr int gm_stage() { return PC * (GM_A_PLANE + gm_b_plane<BN>()); }  // 72 / 48 / 40 KiB
// the LDS epilogue: eight 64-row wave tiles of min(BN / 2, 64) columns (+ 4 floats of row pitch;
// the 256-wide tile transposes its 128 wave columns in two passes)
template <int BN>
constexpr int gm_epi_bytes() { return 8 * 64 * ((BN / 2 < 64 ? BN / 2 : 64) + 4) * 4; }
// NS stages (2, or 3 for the f16x3 form: the W DMA two steps ahead), at least the epilogue tile;
// f16x3 adds the rows' range scales (1 KiB) and 8 flags
template <int PC, int BN = 128, int NS = 2>
constexpr int gm_smem() {
  return (NS * gm_stage<PC, BN>() > gm_epi_bytes<BN>() ? NS * gm_stage<PC, BN>() : gm_epi_bytes<BN>()) +
         (PC == 2 ? 1024 + 64 : 0);
}
static_assert(gm_smem<3>() <= 160 * 1024 && gm_smem<2, 128, 3>() <= 160 * 1024 && gm_smem<2, 64, 3>() <= 160 * 1024 &&
                  gm_smem<2, 256, 2>() <= 160 * 1024,
              "the LDS of a CU");

struct GemmArgs {
  const float* A;      // [M][lda]
  const uint16_t* W;   // plane p, row n at W + p * wps + n * ldw (bf16 bits)
  const float* bias;   // [N] or null
  float* C;            // [M][ldc]
  long long lda, ldc, ldw, wps;
  int M, N, K, relu;
  int tiles_m, tiles_n;
  const float* res;    // [M][ldc] added before the ReLU, or null
  // implicit-GEMM convolution (gemm_f32x6_kernel<true>): A = the NHWC input [img][ih][iw][ic], row
  // m = output pixel (img, oy, ox) of [img][oh][ow], k = (ky * kw + kx) * ic + c
  int ih, iw, ic, oh, ow, kw, stride, pad;
  // batched GEMM (rmbx_linear_f32x6_batched): batch item b uses A + b a_bs, W + b w_bs, C + b c_bs
  int batch;
  long long a_bs, w_bs, c_bs;
  // f16x3: per-output-column power-of-two weight scales [N] (item b: ws + b ws_bs)
  const float* ws;
  long long ws_bs;
};

__device__ __forceinline__ uint32_t pk_bf16(float x, float y) {
  f32x2v v = {x, y};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));  // v_cvt_pk_bf16_f32 (RNE)
}

// (x, y) -> three packed bf16 pairs with x = x0 + x1 + x2 exactly (each level rounded to nearest even)
__device__ __forceinline__ void split_pair(float x, float y, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
  p0 = pk_bf16(x, y);
  const float rx = x - __uint_as_float(p0 << 16), ry = y - __uint_as_float(p0 & 0xffff0000u);
  p1 = pk_bf16(rx, ry);
  const float sx = rx - __uint_as_float(p1 << 16), sy = ry - __uint_as_float(p1 & 0xffff0000u);
  p2 = pk_bf16(sx, sy);
}

__device__ __forceinline__ uint32_t pk_f16(float x, float y) {
  f32x2v v = {x, y};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2v));  // RNE
}

// (x, y) -> packed f16 pairs hi = f16(x), lo = f16((x - hi) 2^11): x = hi + 2^-11 lo to 2^-22 |x|
// for 2^-14 <= |x| <= 65504 (the activation split)
__device__ __forceinline__ void split_f16_pair(float x, float y, uint32_t& h, uint32_t& l) {
  h = pk_f16(x, y);
  const f16x2v hv = __builtin_bit_cast(f16x2v, h);
  l = pk_f16((x - (float)hv[0]) * 2048.f, (y - (float)hv[1]) * 2048.f);
}

// x -> hi = f16(x), lo = f16(x - hi) (the weight split, on rows scaled to max |x| in [2^13, 2^14))
__device__ __forceinline__ void split_f16_w(float x, uint16_t& h, uint16_t& l) {
  const _Float16 hv = (_Float16)x;
  h = __builtin_bit_cast(uint16_t, hv);
  l = __builtin_bit_cast(uint16_t, (_Float16)(x - (float)hv));
}

// LDS-DMA of 16 bytes per lane: the wave's 64 x 16 B land contiguously at the wave-uniform LDS
// address lds_dst (global_load_lds_dwordx4); completion is waited for by hand (vmcnt(0)) before
// the barrier that publishes the stage.
__device__ __forceinline__ void glds16(const void* gsrc, const void* lds_dst) {
  const uint32_t dst = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst;
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(dst))
               : "memory");
}

// s_waitcnt vmcnt(n) with n a compile-time count
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 16-byte global load hidden from hipcc's wait insertion: the A staging loads and the W LDS-DMA
// are all inline asm and counted by hand (hipcc does not count an asm LDS-DMA, and its own waits
// for the register loads around it either drained the DMA at the top of every K step or pulled
// the loads behind the MFMAs).  The destination is named "+v" by the wait that retires it
// (wait_vm_regs), so nothing reads it before the data has landed.
__device__ __forceinline__ void gload16(float4& r, const void* p) {
  f32x4v v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  r = __builtin_bit_cast(float4, v);
}
template <int N>
__device__ __forceinline__ void wait_vm_regs(float4 (&R)[4]) {
  f32x4v v0 = __builtin_bit_cast(f32x4v, R[0]), v1 = __builtin_bit_cast(f32x4v, R[1]);
  f32x4v v2 = __builtin_bit_cast(f32x4v, R[2]), v3 = __builtin_bit_cast(f32x4v, R[3]);
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "n"(N) : "memory");
  R[0] = __builtin_bit_cast(float4, v0);
  R[1] = __builtin_bit_cast(float4, v1);
  R[2] = __builtin_bit_cast(float4, v2);
  R[3] = __builtin_bit_cast(float4, v3);
}

// VAR (profiling, RMBX_GEMM_VAR): bit 0 = s_setprio(1) around each MFMA half-step, bits 1-2 = row
// tiles per block group 8 (0), 4 (1), 16 (2), bit 3 = no output stores (phase skip: the epilogue's
// cost; the result is not written), bit 4 = epilogue through LDS with 16-byte stores (needs
// ldc % 4 == 0 and 16-B aligned C / res / bias rows), bit 5 = no A split (phase skip: the split's
// VALU cost; truncated pieces, wrong values), bit 6 = stagger: waves 4-7 (the SIMD partners of
// waves 0-3) split + store the next A tile before their first MFMA half-step instead of between
// the halves (measured 3-7 % slower; so were a persistent one-block-per-CU form with the K pipeline
// running across tiles and a 128 x 256 tile, profiles/r4_gemm_forms_ab.log)
template <bool CONV, int VAR = 0, int PC = 3, int BN = 128>
__global__ void __launch_bounds__(GM_THREADS, 1) gemm_f32x6_kernel(GemmArgs g) {
  static_assert(PC == 3 || PC == 2, "bf16x6 (3 pieces) or f16x3 (2 pieces)");
  static_assert(BN == 128 || ((BN == 64 || BN == 256) && PC == 2), "BN = 64 / 256: the f16x3 form's tiles");
  static_assert(BN != 256 || (VAR & 1024) == 0, "the 256-wide tile runs two stages");
  constexpr int GROUP = ((VAR >> 1) & 3) == 1 ? 4 : ((VAR >> 1) & 3) == 2 ? 16 : GM_GROUP;
  constexpr int STAGE = gm_stage<PC, BN>(), A_BYTES = PC * GM_A_PLANE, B_PLANE = gm_b_plane<BN>();
  constexpr int NJ = BN / 32;             // 16-column accumulator tiles per wave (wave = 64 x BN / 2)
  constexpr int WP = PC * BN / 128;       // W DMA pieces (16 rows x 64 B) per wave and K step
  constexpr int PPP = BN / 16;            // pieces per W plane
  // Memory operations issued per K step, the counts every hand-written vmcnt below is derived from
  // (the A loads and the W LDS-DMA are inline asm, invisible to hipcc's own wait insertion): stage_b
  // issues W_OPS LDS-DMAs (one glds16 per W piece it owns), load_a issues A_OPS 16-byte loads (two
  // per staged row, two rows).  Both loops below run exactly to these bounds on every path (linear
  // and conv, BN 64 / 128 / 256, both range passes, the K tail, whose redundant copies keep the count
  // fixed), so a wait computed from them cannot drift from what was issued.
  constexpr int W_OPS = WP, A_OPS = 4, A_ROWS = 2;
  static_assert(A_OPS == 2 * A_ROWS, "two 16-byte loads (8 f32 of one k quarter) per staged row");
  // LDS stages: 2; VAR bit 10 (f16x3, profiling) = 3 stages, the W DMA of step kt + 2 issued at step
  // kt and left in flight across the barrier -- measured 1.02-1.08x slower than 2 stages
  // (profiles/r4_gemm_f16x3_phase_skips.log)
  constexpr int NS = (PC == 2 && (VAR & 1024) != 0) ? 3 : 2;
  constexpr int SMEM = gm_smem<PC, BN, NS>();
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 3, wn = wave >> 2;

  // block -> tile: XCD-contiguous ranges (blocks bid, bid + 8, ... run on one XCD), then groups of
  // GM_GROUP row tiles x all column tiles, row tile fastest
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  if (g.batch > 1) {  // consecutive tiles of an XCD stay inside one batch item
    const int per_item = g.tiles_m * g.tiles_n;
    const int item = lin / per_item;
    lin -= item * per_item;
    g.A += item * g.a_bs;
    g.W += item * g.w_bs;
    g.C += item * g.c_bs;
    if (g.ws) g.ws += item * g.ws_bs;
  }
  const int per_group = GROUP * g.tiles_n;
  const int first_m = (lin / per_group) * GROUP;
  const int gsize = min(g.tiles_m - first_m, GROUP);
  const int in_group = lin - (lin / per_group) * per_group;
  const int tm = first_m + in_group % gsize, tn = in_group / gsize;
  const int m0 = tm * GM_BM, n0 = tn * BN;

  // LDS images: every plane row is 32 k = four 16-B slots (8 k each), physical slot =
  // logical ^ ((row >> 2) & 2): conflict-free for the 16x16x32 fragment reads (lane l reads row
  // l%16, slot l/16), the LDS-DMA pieces and the A stores below.
  // A staging (registers): thread -> rows tid/4 and tid/4 + 128, k quarter tid%4 (8 f32 = 32 B
  // each); the pieces go to the PC LDS planes [256 rows][32 k].  Rows past M re-read row M-1
  // (their outputs are not stored).
  const int aq = tid & 3, arow = tid >> 2;
  const float* ag0 = g.A + (long long)min(m0 + arow, g.M - 1) * g.lda + 8 * aq;
  const float* ag1 = g.A + (long long)min(m0 + arow + 128, g.M - 1) * g.lda + 8 * aq;
  const int aoff0 = arow * 64 + ((aq ^ ((arow >> 2) & 2)) << 4);
  const int aoff1 = (arow + 128) * 64 + ((aq ^ (((arow + 128) >> 2) & 2)) << 4);
  // W: LDS-DMA of 8 WP pieces (PPP per plane) of 16 rows x 64 B, wave w copies pieces WP w..WP w+WP-1
  const uint16_t* bsrc[WP];
#pragma unroll
  for (int t = 0; t < WP; ++t) {
    const int i = wave * WP + t, p = i / PPP;
    const int row = (i % PPP) * 16 + (lane >> 2);
    const int sl = (lane & 3) ^ ((row >> 2) & 2);
    bsrc[t] = g.W + p * g.wps + (long long)(n0 + row) * g.ldw + sl * 8;
  }
  auto stage_b = [&](int kt, int buf) {
    if constexpr ((VAR & 512) != 0) {  // phase skip (timing only): no W DMA after the first stage
      if (kt > 0) return;
    }
    unsigned char* base = smem + buf * STAGE + A_BYTES;
#pragma unroll
    for (int t = 0; t < W_OPS; ++t) glds16(bsrc[t] + kt * GM_BK, base + (wave * WP + t) * 1024);
  };
  // convolution: each staged row's window origin (iy0, ix0) and its element offset in the input;
  // a K step of 32 lies inside one filter tap (C % 32 == 0), so a row's 8 channels are one
  // contiguous 32-B load, or zeros where the tap falls in the padding (the load then reads
  // element 0 and the values are dropped at the split)
  long long cbase[2] = {0, 0};
  int cy[2] = {0, 0}, cx[2] = {0, 0};
  if constexpr (CONV) {
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int m = min(m0 + arow + 128 * r2, g.M - 1);
      const int hw = g.oh * g.ow;
      const int img = m / hw, rem = m - img * hw;
      const int oy = rem / g.ow, ox = rem - oy * g.ow;
      cy[r2] = oy * g.stride - g.pad;
      cx[r2] = ox * g.stride - g.pad;
      cbase[r2] = ((long long)(img * g.ih + cy[r2]) * g.iw + cx[r2]) * g.ic + 8 * aq;
    }
  }
  // returns the in-image flags of the two rows (bit r)
  auto load_a = [&](float4 (&R)[4], int kt) -> int {
    if constexpr ((VAR & 256) != 0) {  // phase skip (timing only): no A loads after the first two
      if (kt > 1) return 3;
    }
    if constexpr (!CONV) {
      const float4* p[A_ROWS] = {(const float4*)(ag0 + kt * GM_BK), (const float4*)(ag1 + kt * GM_BK)};
#pragma unroll
      for (int j = 0; j < A_OPS; ++j) gload16(R[j], p[j >> 1] + (j & 1));
      return 3;
    } else {
      const int k0 = kt * GM_BK;
      const int tap = k0 / g.ic, c0 = k0 - tap * g.ic;
      const int ky = tap / g.kw, kx = tap - ky * g.kw;
      int ok = 0;
#pragma unroll
      for (int r2 = 0; r2 < A_ROWS; ++r2) {
        const bool v = (unsigned)(cy[r2] + ky) < (unsigned)g.ih && (unsigned)(cx[r2] + kx) < (unsigned)g.iw;
        const float4* p = (const float4*)(g.A + (v ? cbase[r2] + (long long)(ky * g.iw + kx) * g.ic + c0 : 0));
#pragma unroll
        for (int j = 0; j < A_OPS / A_ROWS; ++j) gload16(R[(A_OPS / A_ROWS) * r2 + j], p + j);
        ok |= (int)v << r2;
      }
      return ok;
    }
  };
  // f16x3: the largest |a| this thread split of its two rows (pass 0; as f32 bit patterns with the
  // sign cleared, whose unsigned order is the order of |a|, NaN above inf) and the rows' pass-1
  // scales
  uint32_t amax0 = 0, amax1 = 0;
  float as0 = 1.f, as1 = 1.f;
  auto store_a = [&](const float4 (&Rin)[4], int ok, int buf, auto scaled) {
    float4 R[4] = {Rin[0], Rin[1], Rin[2], Rin[3]};
    if constexpr (CONV) {
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!(ok & 1)) R[0] = R[1] = z;
      if (!(ok & 2)) R[2] = R[3] = z;
    }
    unsigned char* base = smem + buf * STAGE;
    if constexpr (PC == 2) {
      uint32_t h[8], l[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr ((VAR & 32) != 0) {  // phase skip (timing only): raw bits, no split, no range check
          h[2 * i] = __builtin_amdgcn_perm(__float_as_uint(R[i].y), __float_as_uint(R[i].x), 0x07060302u);
          h[2 * i + 1] = __builtin_amdgcn_perm(__float_as_uint(R[i].w), __float_as_uint(R[i].z), 0x07060302u);
          l[2 * i] = h[2 * i + 1];
          l[2 * i + 1] = h[2 * i];
          continue;
        }
        if constexpr (decltype(scaled)::value) {
          const float sc = i < 2 ? as0 : as1;
          R[i].x *= sc;
          R[i].y *= sc;
          R[i].z *= sc;
          R[i].w *= sc;
        } else {
          uint32_t& am = i < 2 ? amax0 : amax1;
          constexpr uint32_t ABS = 0x7fffffffu;
          am = max(am, max(__float_as_uint(R[i].x) & ABS, __float_as_uint(R[i].y) & ABS));
          am = max(am, max(__float_as_uint(R[i].z) & ABS, __float_as_uint(R[i].w) & ABS));
        }
        split_f16_pair(R[i].x, R[i].y, h[2 * i], l[2 * i]);
        split_f16_pair(R[i].z, R[i].w, h[2 * i + 1], l[2 * i + 1]);
      }
      *(uint4*)(base + aoff0) = make_uint4(h[0], h[1], h[2], h[3]);
      *(uint4*)(base + GM_A_PLANE + aoff0) = make_uint4(l[0], l[1], l[2], l[3]);
      *(uint4*)(base + aoff1) = make_uint4(h[4], h[5], h[6], h[7]);
      *(uint4*)(base + GM_A_PLANE + aoff1) = make_uint4(l[4], l[5], l[6], l[7]);
    } else {
      uint32_t p0[8], p1[8], p2[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr ((VAR & 32) != 0) {  // phase skip: truncated bf16 pieces (realistic values, no split VALU)
          p0[2 * i] = __builtin_amdgcn_perm(__float_as_uint(R[i].y), __float_as_uint(R[i].x), 0x07060302u);
          p0[2 * i + 1] = __builtin_amdgcn_perm(__float_as_uint(R[i].w), __float_as_uint(R[i].z), 0x07060302u);
          p1[2 * i] = p0[2 * i + 1];
          p1[2 * i + 1] = p0[2 * i];
          p2[2 * i] = p0[2 * i];
          p2[2 * i + 1] = p0[2 * i + 1];
        } else {
          split_pair(R[i].x, R[i].y, p0[2 * i], p1[2 * i], p2[2 * i]);
          split_pair(R[i].z, R[i].w, p0[2 * i + 1], p1[2 * i + 1], p2[2 * i + 1]);
        }
      }
      *(uint4*)(base + aoff0) = make_uint4(p0[0], p0[1], p0[2], p0[3]);
      *(uint4*)(base + GM_A_PLANE + aoff0) = make_uint4(p1[0], p1[1], p1[2], p1[3]);
      *(uint4*)(base + 2 * GM_A_PLANE + aoff0) = make_uint4(p2[0], p2[1], p2[2], p2[3]);
      *(uint4*)(base + aoff1) = make_uint4(p0[4], p0[5], p0[6], p0[7]);
      *(uint4*)(base + GM_A_PLANE + aoff1) = make_uint4(p1[4], p1[5], p1[6], p1[7]);
      *(uint4*)(base + 2 * GM_A_PLANE + aoff1) = make_uint4(p2[4], p2[5], p2[6], p2[7]);
    }
  };

  // wave (wm, wn) owns rows 64 wm.., columns 64 wn..: 4 x 4 accumulators of 16 x 16
  f32x4v acc[4][NJ];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4v){0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();

  // 16x16x32 fragments: lane l holds X_p[row l%16][k = 8 (l/16) + j], j = 0..7 (one 16-B slot)
  const int fr = lane & 15, fs = lane >> 4;
  auto frag_off = [&](int row) { return row * 64 + ((fs ^ ((row >> 2) & 2)) << 4); };
  // half h of a K step: m-tiles 2h, 2h+1 against all four n-tiles (bf16x6: 48 MFMAs, small
  // terms first; f16x3: 24)
  auto half_step = [&](int buf, int h, const bf16x8 (&b)[NJ][PC], const f16x8 (&bs)[NJ]) {
    const unsigned char* As = smem + buf * STAGE;
    bf16x8 a[2][PC];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int off = frag_off(wm * 64 + (2 * h + i) * 16 + fr);
#pragma unroll
      for (int p = 0; p < PC; ++p) a[i][p] = *(const bf16x8*)(As + p * GM_A_PLANE + off);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int nj = 0; nj < NJ; ++nj) {
        if constexpr (PC == 2) {
          const f16x8 ah = __builtin_bit_cast(f16x8, a[i][0]), al = __builtin_bit_cast(f16x8, a[i][1]);
          const f16x8 bh = __builtin_bit_cast(f16x8, b[nj][0]), bl = __builtin_bit_cast(f16x8, b[nj][1]);
          f32x4v c = acc[2 * h + i][nj];
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bs[nj], c, 0, 0, 0);  // small terms first
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
          acc[2 * h + i][nj] = c;
        } else {
          f32x4v c = acc[2 * h + i][nj];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][2], b[nj][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[nj][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[nj][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[nj][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[nj][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[nj][0], c, 0, 0, 0);
          acc[2 * h + i][nj] = c;
        }
      }
  };
  auto read_b = [&](bf16x8 (&b)[NJ][PC], int buf) {
    const unsigned char* Bs = smem + buf * STAGE + A_BYTES;
#pragma unroll
    for (int nj = 0; nj < NJ; ++nj) {
      const int off = frag_off(wn * (BN / 2) + nj * 16 + fr);
#pragma unroll
      for (int p = 0; p < PC; ++p) b[nj][p] = *(const bf16x8*)(Bs + p * B_PLANE + off);
    }
  };

  // K steps of 32 over NS LDS stages, one barrier per step.  Step kt computes stage kt while W of
  // kt + NS - 1 arrives by LDS-DMA, A of kt + 1 (loaded during step kt - 1) is split and stored
  // between the step's two MFMA halves, and A of kt + 2 is loaded into registers.  Issue order
  // per step: W DMA (WP pieces), then the 4 A loads; every step issues both (the last steps' are
  // redundant copies of the last K step into idle stages), so the hand counts are fixed: the split
  // waits for A of kt + 1 with vmcnt(WP + 4); the end of the step retires the DMA of stage kt + 1
  // with vmcnt(4) (2 stages: it was issued this step) or vmcnt(WP + 4) (3 stages: issued the step
  // before, so this step's DMA stays in flight across the barrier).
  const int KT = g.K / GM_BK;
  // The waits, from the per-step counts (vmcnt retires in issue order):
  //   SPLIT_WAIT: A of kt + 1 was loaded during the step before; issued after it are this step's W
  //     DMA and A loads, so <= W_OPS + A_OPS outstanding means it has landed (prologue likewise:
  //     Ra, then the stage-0 / stage-1 DMA and Rb);
  //   END_WAIT: the DMA of stage kt + 1 -- issued this step (2 stages: only this step's A loads
  //     follow it) or the step before (3 stages: this step's DMA and A loads follow it).
  // Round-4 fault (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION in gemm_f32x6_kernel<false, 528, 2,
  // 128>, gpurun_out/r4_l_gemm_phases.log): the VAR & 512 phase skip issues no W DMA after the first
  // stage, i.e. 4 operations per step where the literal waits assumed 6, so vmcnt(6) let the last two
  // A loads of Rcur still be in flight when store_a consumed Rcur; hipcc, which sees the asm outputs
  // as written at issue and Rcur dead after store_a, re-allocated those VGPRs -- to 64-bit load
  // addresses among others -- and the late data landing in them turned the next loads' addresses
  // out of range.  The phase-skip variants issue a varying count, so they wait for everything.
  constexpr bool SKIPS = (VAR & (256 | 512)) != 0;
  constexpr int LEAD = NS - 1;
  constexpr int SPLIT_WAIT = SKIPS ? 0 : W_OPS + A_OPS;
  constexpr int END_WAIT = SKIPS ? 0 : (NS == 3 ? W_OPS + A_OPS : A_OPS);
  static_assert(SPLIT_WAIT <= 63 && END_WAIT <= 63, "vmcnt holds 6 bits on gfx950");
  static_assert(SKIPS || (END_WAIT < SPLIT_WAIT || NS == 3), "a stage's DMA is retired after the A split");
  auto stage_of = [](int k) { return NS == 2 ? (k & 1) : k % 3; };
  auto k_loop = [&](auto scaled) {
    float4 Ra[4], Rb[4];
    int oka, okb;
    if constexpr (NS == 3) {
      stage_b(0, 0);
      oka = load_a(Ra, 0);
      stage_b(min(1, KT - 1), 1);
      okb = load_a(Rb, min(1, KT - 1));
    } else {
      oka = load_a(Ra, 0);
      stage_b(0, 0);
      okb = load_a(Rb, min(1, KT - 1));
    }
    wait_vm_regs<SPLIT_WAIT>(Ra);
    store_a(Ra, oka, 0, scaled);
    wait_vm<END_WAIT>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    auto step = [&](int kt, float4 (&Rcur)[4], int& okcur, float4 (&Rnext)[4], int& oknext) {
      const int buf = stage_of(kt), nbuf = stage_of(kt + 1);
      const bool more = kt + 1 < KT;
      stage_b(min(kt + LEAD, KT - 1), stage_of(kt + LEAD));
      oknext = load_a(Rnext, min(kt + 2, KT - 1));
      if constexpr (BN == 256) {
        // the 256-wide tile (wave = 64 x 128, 4 x 8 accumulators): the wave's four A fragment
        // pairs stay in registers for the step, the W fragments are read per column tile in two
        // halves of four, the A split between them (registers: acc 128 + A 32 + one W tile 12)
        const unsigned char* S = smem + buf * STAGE;
        f16x8 ah[4], al[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const int off = frag_off(wm * 64 + mi * 16 + fr);
          ah[mi] = __builtin_bit_cast(f16x8, *(const bf16x8*)(S + off));
          al[mi] = __builtin_bit_cast(f16x8, *(const bf16x8*)(S + GM_A_PLANE + off));
        }
        auto wide_half = [&](int hh) {
#pragma unroll
          for (int q = 0; q < NJ / 2; ++q) {
            const int nj = hh * (NJ / 2) + q;
            const int off = frag_off(wn * (BN / 2) + nj * 16 + fr);
            const f16x8 bh = __builtin_bit_cast(f16x8, *(const bf16x8*)(S + A_BYTES + off));
            const f16x8 bl = __builtin_bit_cast(f16x8, *(const bf16x8*)(S + A_BYTES + B_PLANE + off));
            const f16x8 bsc = bh * (_Float16)0.00048828125f;
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
              f32x4v c = acc[mi][nj];
              c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[mi], bsc, c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[mi], bl, c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[mi], bh, c, 0, 0, 0);
              acc[mi][nj] = c;
            }
          }
        };
        wide_half(0);
        wait_vm_regs<SPLIT_WAIT>(Rcur);
        store_a(Rcur, okcur, nbuf, scaled);
        wide_half(1);
        wait_vm<END_WAIT>();
        if (more) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        return;
      }
      bf16x8 b[NJ][PC];
      read_b(b, buf);
      f16x8 bs[NJ];  // f16x3: 2^-11 hb (exact above f16's subnormal range)
#pragma unroll
      for (int nj = 0; nj < NJ; ++nj) {
        if constexpr (PC == 2) bs[nj] = __builtin_bit_cast(f16x8, b[nj][0]) * (_Float16)0.00048828125f;
      }
      const bool late = (VAR & 64) == 0 || wave < 4;
      if (!late) {
        wait_vm_regs<SPLIT_WAIT>(Rcur);
        store_a(Rcur, okcur, nbuf, scaled);
      }
      if constexpr (VAR & 1) __builtin_amdgcn_s_setprio(1);
      half_step(buf, 0, b, bs);
      if constexpr (VAR & 1) __builtin_amdgcn_s_setprio(0);
      if (late) {
        wait_vm_regs<SPLIT_WAIT>(Rcur);
        store_a(Rcur, okcur, nbuf, scaled);
      }
      if constexpr (VAR & 1) __builtin_amdgcn_s_setprio(1);
      half_step(buf, 1, b, bs);
      if constexpr (VAR & 1) __builtin_amdgcn_s_setprio(0);
      wait_vm<END_WAIT>();
      if (more) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    for (int kt = 0; kt < KT; kt += 2) {
      step(kt, Rb, okb, Ra, oka);
      if (kt + 1 < KT) step(kt + 1, Ra, oka, Rb, okb);
    }
    // drain the last step's redundant loads (their registers are free after this) and DMA
    wait_vm_regs<0>(Ra);
    wait_vm_regs<0>(Rb);
  };
  k_loop(std::false_type{});

  if constexpr (PC == 2) {
    // per-row range check: a row whose |a| max lies outside [2^-6, 2^15] (f16 overflow / subnormal
    // range) is re-run on a * 2^s, max in [2^13, 2^14), and scaled back by 2^-s; a block with
    // such a row runs its K loop again with every other row at scale 1, i.e. bit-identical to
    // pass 0, so each row's result depends on its own values only.  A row holding a NaN or an
    // infinity is left to propagate them as in f32.
    uint32_t b0 = amax0, b1 = amax1;
    b0 = max(b0, (uint32_t)__shfl_xor((int)b0, 1));  // the 4 lanes of a row (tid % 4 = k quarter)
    b0 = max(b0, (uint32_t)__shfl_xor((int)b0, 2));
    b1 = max(b1, (uint32_t)__shfl_xor((int)b1, 1));
    b1 = max(b1, (uint32_t)__shfl_xor((int)b1, 2));
    const float m0 = __uint_as_float(b0), m1 = __uint_as_float(b1);  // NaN: no re-run
    float inv0 = 1.f, inv1 = 1.f;
    auto row_scale = [](float m, float& sc, float& inv) {
      if ((m > 32768.f || (m > 0.f && m < 0.015625f)) && m <= 3.4e38f) {
        int e;
        frexpf(m, &e);  // m = f 2^e, f in [0.5, 1)
        sc = ldexpf(1.f, 14 - e);
        inv = ldexpf(1.f, e - 14);
        return true;
      }
      return false;
    };
    const bool need = row_scale(m0, as0, inv0) | row_scale(m1, as1, inv1);
    float* rinv = reinterpret_cast<float*>(smem + SMEM - 1024 - 64);  // [256] rows' 2^-s
    int* flag = reinterpret_cast<int*>(smem + SMEM - 64);
    if (aq == 0) {
      rinv[arow] = inv0;
      rinv[arow + 128] = inv1;
    }
    const unsigned long long bal = __ballot(need);
    if (lane == 0) flag[wave] = bal != 0ull;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    int any = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) any |= flag[w];
    if (any) {
      zero_acc();
      k_loop(std::true_type{});
    }
    // undo the rows' pass-1 scales (powers of two)
    if (any) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float inv = rinv[wm * 64 + i * 16 + 4 * fs + e];
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j][e] *= inv;
        }
    }
  }

  if constexpr ((VAR & 16) != 0) {
    // epilogue through LDS: each wave writes its 64 x 64 accumulator tile row-major into its own
    // 16 KiB of the (now idle) stage buffers (row pitch 68 floats: the 16 lanes of a column group
    // write 16 consecutive floats, rows 4 apart land on different banks), then reads it back as
    // float4 rows so every lane stores 16 contiguous bytes (16 stores per lane instead of 64)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    constexpr int WC = BN / 2 < 64 ? BN / 2 : 64, PITCH = WC + 4;  // columns per pass, row pitch
    constexpr int LPR = WC / 4, RPI = 64 / LPR;  // lanes per row (4 columns each), rows per pass
    constexpr int NPASS = (BN / 2) / WC, NJP = NJ / NPASS;  // passes, accumulator columns per pass
    float* T = reinterpret_cast<float*>(smem) + wave * (64 * PITCH);
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
    if (pass > 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last pass's reads are done
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int q = 0; q < NJP; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) T[(mi * 16 + 4 * fs + e) * PITCH + q * 16 + fr] = acc[mi][pass * NJP + q][e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave reads only its own tile
    const int c4 = (lane % LPR) * 4;                     // 4 columns of the WC
    const int n = n0 + wn * (BN / 2) + pass * WC + c4;
    float4 bn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g.bias) bn = *(const float4*)(g.bias + n);
    float4 sn = make_float4(1.f, 1.f, 1.f, 1.f);
    if constexpr (PC == 2) sn = *(const float4*)(g.ws + n);
#pragma unroll
    for (int it = 0; it < 64 / RPI; ++it) {
      const int r = it * RPI + lane / LPR;
      const int m = m0 + wm * 64 + r;
      if (m < g.M) {
        float4 v = *(const float4*)(T + r * PITCH + c4);
        if constexpr (PC == 2) {  // the weight row scales (powers of two: exact)
          v.x *= sn.x; v.y *= sn.y; v.z *= sn.z; v.w *= sn.w;
        }
        v.x += bn.x; v.y += bn.y; v.z += bn.z; v.w += bn.w;
        if (g.res) {
          const float4 rv = *(const float4*)(g.res + (long long)m * g.ldc + n);
          v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
        }
        if (g.relu) {
          v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
        }
        *(float4*)(g.C + (long long)m * g.ldc + n) = v;
      }
    }
    }  // pass
    return;
  }
  // epilogue: accumulator register e of lane l is C[row 4 (l/16) + e][col l%16] of its tile
#pragma unroll
  for (int nj = 0; nj < NJ; ++nj) {
    const int n = n0 + wn * (BN / 2) + nj * 16 + fr;
    const float bn = g.bias ? g.bias[n] : 0.f;
    const float sn = PC == 2 ? g.ws[n] : 1.f;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int mb = m0 + wm * 64 + mi * 16 + 4 * fs;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = mb + e;
        if (!(VAR & 8) && m < g.M) {
          float v = acc[mi][nj][e];
          if constexpr (PC == 2) v *= sn;
          v += bn;
          if (g.res) v += g.res[(long long)m * g.ldc + n];
          if (g.relu) v = fmaxf(v, 0.f);
          g.C[(long long)m * g.ldc + n] = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Producer / consumer form of the f16x3 kernel (256 x 128 tile): 12 waves, 3 per SIMD.  Waves 0-7
// only read fragments and issue MFMAs (the layout above: 64 x 64 per wave, one accumulator set);
// waves 8-11 (one per SIMD) produce the K steps two ahead into a ring of three 48-KiB LDS stages:
// they load the A tile (thread -> rows r, r + 64, r + 128, r + 192 of k quarter q, 8 f32 each,
// loaded one step before its split), split it into the two f16 planes, track each row's max |a|,
// and move W by LDS-DMA (4 pieces per wave).  One barrier per K step for all 12 waves: after
// barrier j + 1 the stage of step j + 1 is complete (its A was stored and its DMA retired by the
// producers during step j), and the stage they write during step j (that of j + 2) was last read
// in step j - 1.  The per-row range check and the re-run pass are the PC = 2 kernel's.
constexpr int GP_THREADS = 768;
template <bool CONV, bool VEC>
__global__ void __launch_bounds__(GP_THREADS, 1) gemm_f16x3_pc_kernel(GemmArgs g) {
  constexpr int NS = 3, BN = 128, NJ = 4;
  constexpr int STAGE = gm_stage<2, BN>(), A_BYTES = 2 * GM_A_PLANE, B_PLANE = gm_b_plane<BN>();
  constexpr int SMEM = gm_smem<2, BN, NS>();
  constexpr int WPP = 4;  // W DMA pieces per producer wave and K step (16 per stage)
  constexpr int PA_OPS = 8;  // 16-byte A loads per producer thread and K step (load_a: 4 rows x 2)
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool producer = wave >= 8;

  // block -> tile (as gemm_f32x6_kernel)
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nblk >> 3, r8 = nblk & 7;
  int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  if (g.batch > 1) {
    const int per_item = g.tiles_m * g.tiles_n;
    const int item = lin / per_item;
    lin -= item * per_item;
    g.A += item * g.a_bs;
    g.W += item * g.w_bs;
    g.C += item * g.c_bs;
    if (g.ws) g.ws += item * g.ws_bs;
  }
  const int per_group = GM_GROUP * g.tiles_n;
  const int first_m = (lin / per_group) * GM_GROUP;
  const int gsize = min(g.tiles_m - first_m, GM_GROUP);
  const int in_group = lin - (lin / per_group) * per_group;
  const int tm = first_m + in_group % gsize, tn = in_group / gsize;
  const int m0 = tm * GM_BM, n0 = tn * BN;
  const int KT = g.K / GM_BK;
  auto stage_of = [](int k) { return k % 3; };

  // ---- producer state: thread pt -> k quarter aq, rows prow + 64 i (i = 0..3)
  const int pt = tid - 512, aq = pt & 3, prow = (pt >> 2) & 63;
  const float* arow[4];
  int aoff[4];
  long long cbase[4] = {0, 0, 0, 0};
  int cy[4] = {0, 0, 0, 0}, cx[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = prow + 64 * i, m = min(m0 + r, g.M - 1);
    arow[i] = g.A + (long long)m * g.lda + 8 * aq;
    aoff[i] = r * 64 + ((aq ^ ((r >> 2) & 2)) << 4);
    if constexpr (CONV) {
      const int hw = g.oh * g.ow;
      const int img = m / hw, rem = m - img * hw;
      const int oy = rem / g.ow, ox = rem - oy * g.ow;
      cy[i] = oy * g.stride - g.pad;
      cx[i] = ox * g.stride - g.pad;
      cbase[i] = ((long long)(img * g.ih + cy[i]) * g.iw + cx[i]) * g.ic + 8 * aq;
    }
  }
  const int pw = wave - 8;
  const uint16_t* bsrc[WPP];
#pragma unroll
  for (int t = 0; t < WPP; ++t) {
    const int i = pw * WPP + t, p = i >> 3;
    const int row = (i & 7) * 16 + (lane >> 2);
    const int sl = (lane & 3) ^ ((row >> 2) & 2);
    bsrc[t] = g.W + p * g.wps + (long long)(n0 + row) * g.ldw + sl * 8;
  }
  auto dma_w = [&](int kt, int buf) {
    unsigned char* base = smem + buf * STAGE + A_BYTES;
#pragma unroll
    for (int t = 0; t < WPP; ++t) glds16(bsrc[t] + kt * GM_BK, base + (pw * WPP + t) * 1024);
  };
  // 8 loads of 16 B: rows i = 0..3, two halves each; returns the rows' in-image flags (conv)
  auto load_a = [&](float4 (&R)[8], int kt) -> int {
    if constexpr (!CONV) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4* p = (const float4*)(arow[i] + kt * GM_BK);
        gload16(R[2 * i], p);
        gload16(R[2 * i + 1], p + 1);
      }
      return 15;
    } else {
      const int k0 = kt * GM_BK;
      const int tap = k0 / g.ic, c0 = k0 - tap * g.ic;
      const int ky = tap / g.kw, kx = tap - ky * g.kw;
      int ok = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool v = (unsigned)(cy[i] + ky) < (unsigned)g.ih && (unsigned)(cx[i] + kx) < (unsigned)g.iw;
        const float4* p = (const float4*)(g.A + (v ? cbase[i] + (long long)(ky * g.iw + kx) * g.ic + c0 : 0));
        gload16(R[2 * i], p);
        gload16(R[2 * i + 1], p + 1);
        ok |= (int)v << i;
      }
      return ok;
    }
  };
  static_assert(WPP + PA_OPS <= 63, "vmcnt holds 6 bits on gfx950");
  auto wait_regs8 = [&](float4 (&R)[8]) {  // vmcnt(WPP + PA_OPS): this step's DMA and loads stay in flight
    f32x4v v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = __builtin_bit_cast(f32x4v, R[i]);
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
                 : "n"(WPP + PA_OPS)
                 : "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) R[i] = __builtin_bit_cast(float4, v[i]);
  };
  auto drain_regs8 = [&](float4 (&R)[8]) {
    f32x4v v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = __builtin_bit_cast(f32x4v, R[i]);
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
                 :
                 : "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) R[i] = __builtin_bit_cast(float4, v[i]);
  };
  uint32_t amax[4] = {0, 0, 0, 0};
  float asc[4] = {1.f, 1.f, 1.f, 1.f};
  auto store_a = [&](const float4 (&Rin)[8], int ok, int buf, auto scaled) {
    unsigned char* base = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float4 R0 = Rin[2 * i], R1 = Rin[2 * i + 1];
      if constexpr (CONV) {
        if (!((ok >> i) & 1)) R0 = R1 = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if constexpr (decltype(scaled)::value) {
        const float sc = asc[i];
        R0.x *= sc; R0.y *= sc; R0.z *= sc; R0.w *= sc;
        R1.x *= sc; R1.y *= sc; R1.z *= sc; R1.w *= sc;
      } else {
        constexpr uint32_t ABS = 0x7fffffffu;
        uint32_t m = max(max(__float_as_uint(R0.x) & ABS, __float_as_uint(R0.y) & ABS),
                         max(__float_as_uint(R0.z) & ABS, __float_as_uint(R0.w) & ABS));
        m = max(m, max(max(__float_as_uint(R1.x) & ABS, __float_as_uint(R1.y) & ABS),
                       max(__float_as_uint(R1.z) & ABS, __float_as_uint(R1.w) & ABS)));
        amax[i] = max(amax[i], m);
      }
      uint32_t h[4], l[4];
      split_f16_pair(R0.x, R0.y, h[0], l[0]);
      split_f16_pair(R0.z, R0.w, h[1], l[1]);
      split_f16_pair(R1.x, R1.y, h[2], l[2]);
      split_f16_pair(R1.z, R1.w, h[3], l[3]);
      *(uint4*)(base + aoff[i]) = make_uint4(h[0], h[1], h[2], h[3]);
      *(uint4*)(base + GM_A_PLANE + aoff[i]) = make_uint4(l[0], l[1], l[2], l[3]);
    }
  };

  // ---- consumer state (waves 0-7): wave (wm, wn) owns rows 64 wm.., columns 64 wn..
  const int wm = wave & 3, wn = (wave >> 2) & 1;
  const int fr = lane & 15, fs = lane >> 4;
  auto frag_off = [&](int row) { return row * 64 + ((fs ^ ((row >> 2) & 2)) << 4); };
  f32x4v acc[4][NJ];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4v){0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();
  auto consume = [&](int buf) {
    const unsigned char* S = smem + buf * STAGE;
    bf16x8 b[NJ][2];
#pragma unroll
    for (int nj = 0; nj < NJ; ++nj) {
      const int off = frag_off(wn * 64 + nj * 16 + fr);
      b[nj][0] = *(const bf16x8*)(S + A_BYTES + off);
      b[nj][1] = *(const bf16x8*)(S + A_BYTES + B_PLANE + off);
    }
    f16x8 bs[NJ];
#pragma unroll
    for (int nj = 0; nj < NJ; ++nj) bs[nj] = __builtin_bit_cast(f16x8, b[nj][0]) * (_Float16)0.00048828125f;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int off = frag_off(wm * 64 + mi * 16 + fr);
      const f16x8 ah = __builtin_bit_cast(f16x8, *(const bf16x8*)(S + off));
      const f16x8 al = __builtin_bit_cast(f16x8, *(const bf16x8*)(S + GM_A_PLANE + off));
#pragma unroll
      for (int nj = 0; nj < NJ; ++nj) {
        f32x4v c = acc[mi][nj];
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bs[nj], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, __builtin_bit_cast(f16x8, b[nj][1]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, __builtin_bit_cast(f16x8, b[nj][0]), c, 0, 0, 0);
        acc[mi][nj] = c;
      }
    }
  };

  // one pass over K: KT + 1 barriers for every wave
  auto k_pass = [&](auto scaled) {
    if (producer) {
      float4 Ra[8], Rb[8];
      int oka, okb;
      // prologue: K steps 0 and 1 into stages 0 and 1, A of step 2 in flight
      dma_w(0, 0);
      oka = load_a(Ra, 0);
      dma_w(min(1, KT - 1), 1);
      okb = load_a(Rb, min(1, KT - 1));
      {
        // A(0): younger = DMA(1) + A(1)
        wait_regs8(Ra);
        store_a(Ra, oka, 0, scaled);
        drain_regs8(Rb);  // A(1) (and every DMA before it)
        store_a(Rb, okb, 1, scaled);
      }
      oka = load_a(Ra, min(2, KT - 1));  // A(2)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      // step j: produce K step j + 2 (A loaded last step into Rcur) and load A(j + 3)
      auto pstep = [&](int j, float4 (&Rcur)[8], int& okcur, float4 (&Rnext)[8], int& oknext) {
        const int p = min(j + 2, KT - 1);
        dma_w(p, stage_of(j + 2));
        oknext = load_a(Rnext, min(j + 3, KT - 1));
        wait_regs8(Rcur);  // A(j + 2): younger = DMA(j + 2) + A(j + 3)
        store_a(Rcur, okcur, stage_of(j + 2), scaled);
        // DMA(j + 1) (issued last step, older than A(j + 2)) retired by the same count
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      };
      for (int j = 0; j < KT; j += 2) {
        pstep(j, Ra, oka, Rb, okb);
        if (j + 1 < KT) pstep(j + 1, Rb, okb, Ra, oka);
      }
      drain_regs8(Ra);
      drain_regs8(Rb);
    } else {
      asm volatile("s_barrier" ::: "memory");
      for (int j = 0; j < KT; ++j) {
        consume(stage_of(j));
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
    }
  };
  k_pass(std::false_type{});

  // per-row range check (producers hold the rows' maxima) and the re-run pass
  float* rinv = reinterpret_cast<float*>(smem + SMEM - 1024 - 64);
  int* flag = reinterpret_cast<int*>(smem + SMEM - 64);
  {
    bool need = false;
    if (producer) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t b = amax[i];
        b = max(b, (uint32_t)__shfl_xor((int)b, 1));
        b = max(b, (uint32_t)__shfl_xor((int)b, 2));
        const float m = __uint_as_float(b);
        float inv = 1.f;
        if ((m > 32768.f || (m > 0.f && m < 0.015625f)) && m <= 3.4e38f) {
          int e;
          frexpf(m, &e);
          asc[i] = ldexpf(1.f, 14 - e);
          inv = ldexpf(1.f, e - 14);
          need = true;
        }
        if (aq == 0) rinv[prow + 64 * i] = inv;
      }
    }
    const unsigned long long bal = __ballot(need);
    if (lane == 0) flag[wave] = bal != 0ull;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    int any = 0;
#pragma unroll
    for (int w = 8; w < 12; ++w) any |= flag[w];
    if (any) {
      zero_acc();
      k_pass(std::true_type{});
      if (!producer) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float inv = rinv[wm * 64 + i * 16 + 4 * fs + e];
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j][e] *= inv;
          }
      }
    }
  }

  // epilogue (consumers; the producers only take part in the barrier)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (producer) return;
  if constexpr (VEC) {
    constexpr int PITCH = 68;
    float* T = reinterpret_cast<float*>(smem) + wave * (64 * PITCH);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < NJ; ++nj)
#pragma unroll
        for (int e = 0; e < 4; ++e) T[(mi * 16 + 4 * fs + e) * PITCH + nj * 16 + fr] = acc[mi][nj][e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int c4 = (lane & 15) * 4;
    const int n = n0 + wn * 64 + c4;
    float4 bn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g.bias) bn = *(const float4*)(g.bias + n);
    const float4 sn = *(const float4*)(g.ws + n);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int r = it * 4 + (lane >> 4);
      const int m = m0 + wm * 64 + r;
      if (m < g.M) {
        float4 v = *(const float4*)(T + r * PITCH + c4);
        v.x *= sn.x; v.y *= sn.y; v.z *= sn.z; v.w *= sn.w;
        v.x += bn.x; v.y += bn.y; v.z += bn.z; v.w += bn.w;
        if (g.res) {
          const float4 rv = *(const float4*)(g.res + (long long)m * g.ldc + n);
          v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
        }
        if (g.relu) {
          v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
        }
        *(float4*)(g.C + (long long)m * g.ldc + n) = v;
      }
    }
  } else {
#pragma unroll
    for (int nj = 0; nj < NJ; ++nj) {
      const int n = n0 + wn * 64 + nj * 16 + fr;
      const float bn = g.bias ? g.bias[n] : 0.f, sn = g.ws[n];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int mb = m0 + wm * 64 + mi * 16 + 4 * fs;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = mb + e;
          if (m < g.M) {
            float v = acc[mi][nj][e];
            v *= sn;  // as gemm_f32x6_kernel: scale, then bias (two roundings, no contraction)
            v += bn;
            if (g.res) v += g.res[(long long)m * g.ldc + n];
            if (g.relu) v = fmaxf(v, 0.f);
            g.C[(long long)m * g.ldc + n] = v;
          }
        }
      }
    }
  }
}

// planes[p * n + i] = piece p of x[i] (x = x0 + x1 + x2, bf16 bits)
__global__ void split_bf16x3_kernel(const float* __restrict__ x, uint16_t* __restrict__ planes, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    uint32_t p0, p1, p2;
    split_pair(x[i], 0.f, p0, p1, p2);
    planes[i] = (uint16_t)(p0 & 0xffff);
    planes[n + i] = (uint16_t)(p1 & 0xffff);
    planes[2 * n + i] = (uint16_t)(p2 & 0xffff);
  }
}

// one block per weight row n: s = 2^(14 - e) with max_k |w[n][k]| = f 2^e (f in [0.5, 1)), so the
// scaled row's max lies in [2^13, 2^14); planes [2][N][K] = f16 hi = f16(w s), lo = f16(w s - hi),
// scale[n] = 1 / s (an all-zero or non-finite row keeps s = 1)
__global__ void __launch_bounds__(256) split_f16x2_kernel(const float* __restrict__ w, int K, long long plane,
                                                          uint16_t* __restrict__ planes, float* __restrict__ scale) {
  __shared__ float red[4];
  const int n = blockIdx.x, tid = threadIdx.x;
  const float* row = w + (long long)n * K;
  float m = 0.f;
  for (int k = tid; k < K; k += 256) m = fmaxf(m, fabsf(row[k]));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  int e = 14;
  if (m > 0.f && m <= 3.4e38f) frexpf(m, &e);
  const float s = ldexpf(1.f, 14 - e);
  if (tid == 0) scale[n] = ldexpf(1.f, e - 14);
  for (int k = tid; k < K; k += 256) {
    uint16_t h, l;
    split_f16_w(row[k] * s, h, l);
    planes[(long long)n * K + k] = h;
    planes[plane + (long long)n * K + k] = l;
  }
}

// ---------------------------------------------------------------------------------------------
// Pre-split A form of the f16x3 kernel (rmbx_linear_f16x3_presplit): A arrives already split by its
// producer (rmbx_add_layernorm_split: each row scaled by a power of two 2^t_m with its max |a| in
// [2^13, 2^14), a' = a 2^t_m = ha + la, ha = f16(a'), la = f16(a' - ha) -- the weight rows' split),
// as two f16 planes [M][K] and the rows' 2^-t_m.  Both operands then move by LDS-DMA
// (global_load_lds_dwordx4, the W pieces' layout and swizzle for A too): no A registers, no split,
// no per-row range check or re-run pass (the producer chose each row's scale), and the three
// products take the raw pieces, a'.w' ~ ha hb + ha lb + la hb (dropped term <= 2^-22 |a' w'|,
// pieces below 2^-16 of their row's max are f16 subnormals, as for W).  The epilogue applies
// 2^-t_m 1 / s_n (powers of two: exact), then bias / residual / ReLU.  Two LDS stages: step kt
// computes stage kt while the DMA of kt + 1 is in flight, one barrier per step.  Tile 256 x BN,
// 8 waves (wave = 64 x BN / 2), the same XCD / group mapping as gemm_f32x6_kernel.
// N % 256 == 128 (FFN1's 3200 columns): the last column tile's second half is dead -- its waves
// skip the fragment reads and MFMAs, its W rows re-read row N - 1, nothing is stored -- so every
// column tile of a row band runs in one launch and the band's A is fetched once into the XCD's L2
// (a separate 128-wide launch re-read all of A for 4 % of the work).  GROUP row tiles per block
// group (the rasterisation: all column tiles of GROUP row tiles, row tile fastest).
// VAR (profiling phase skips, RMBX_PRESPLIT_VAR; wrong results, timing only): bit 0 = no DMA after
// the first stage, bit 1 = no fragment reads / MFMAs, bit 2 = no output stores
template <int BN, int GROUP, int VAR = 0>
__global__ void __launch_bounds__(GM_THREADS, 1) gemm_f16x3_presplit_kernel(GemmArgs g, const uint16_t* __restrict__ Ap,
                                                                           long long aps, long long ldah,
                                                                           const float* __restrict__ arinv) {
  static_assert(BN == 128 || BN == 256, "the 128- and 256-wide tiles");
  constexpr int NJ = BN / 32;                                 // 16-column accumulator tiles per wave
  constexpr int A_PIECES = 2 * (GM_BM / 16), B_PIECES = 2 * (BN / 16);  // 16 rows x 64 B per piece
  constexpr int PIECES = A_PIECES + B_PIECES, PW = PIECES / 8;          // per wave and K step
  static_assert(PIECES % 8 == 0, "pieces split evenly over the 8 waves");
  constexpr int A_BYTES = 2 * GM_A_PLANE, B_PLANE = gm_b_plane<BN>(), STAGE = A_BYTES + 2 * B_PLANE;
  constexpr int EPI = gm_epi_bytes<BN>();
  constexpr int SMEM = 2 * STAGE > EPI ? 2 * STAGE : EPI;
  static_assert(SMEM <= 160 * 1024, "the LDS of a CU");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 3, wn = wave >> 2;
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int per_group = GROUP * g.tiles_n;
  const int first_m = (lin / per_group) * GROUP;
  const int gsize = min(g.tiles_m - first_m, GROUP);
  const int in_group = lin - (lin / per_group) * per_group;
  const int tm = first_m + in_group % gsize, tn = in_group / gsize;
  const int m0 = tm * GM_BM, n0 = tn * BN;
  const bool dead = n0 + wn * (BN / 2) >= g.N;  // (wave-uniform) the half tile past N

  // the wave's DMA pieces: piece i < A_PIECES is A plane i / 16, rows 16 (i % 16)..; the rest W
  // plane, rows as in gemm_f32x6_kernel.  Lane l moves row (l / 4) of the piece, logical 8-k slot
  // (l % 4) ^ ((row >> 2) & 2) to physical slot l % 4 (the fragment reads' swizzle).  A rows past M
  // re-read row M - 1 (their outputs are not stored).
  const uint16_t* src[PW];
  int dst[PW];
#pragma unroll
  for (int t = 0; t < PW; ++t) {
    const int i = wave * PW + t;
    if (i < A_PIECES) {
      const int p = i / (GM_BM / 16), row = (i % (GM_BM / 16)) * 16 + (lane >> 2);
      const int sl = (lane & 3) ^ ((row >> 2) & 2);
      src[t] = Ap + p * aps + (long long)min(m0 + row, g.M - 1) * ldah + sl * 8;
      dst[t] = p * GM_A_PLANE + (i % (GM_BM / 16)) * 1024;
    } else {
      const int j = i - A_PIECES, p = j / (BN / 16), row = (j % (BN / 16)) * 16 + (lane >> 2);
      const int sl = (lane & 3) ^ ((row >> 2) & 2);
      src[t] = g.W + p * g.wps + (long long)min(n0 + row, g.N - 1) * g.ldw + sl * 8;
      dst[t] = A_BYTES + p * B_PLANE + (j % (BN / 16)) * 1024;
    }
  }
  auto stage = [&](int kt, int buf) {
#pragma unroll
    for (int t = 0; t < PW; ++t) glds16(src[t] + kt * GM_BK, smem + buf * STAGE + dst[t]);
  };

  f32x4v acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4v){0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fs = lane >> 4;
  auto frag_off = [&](int row) { return row * 64 + ((fs ^ ((row >> 2) & 2)) << 4); };

  const int KT = g.K / GM_BK;
  stage(0, 0);
  wait_vm<0>();
  asm volatile("s_barrier" ::: "memory");
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    // the next stage's DMA (its buffer was last read in step kt - 1, which the barrier closed)
    if (kt + 1 < KT && !(VAR & 1)) stage(kt + 1, buf ^ 1);
    const unsigned char* S = smem + buf * STAGE;
    f16x8 ah[4], al[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int off = frag_off(wm * 64 + mi * 16 + fr);
      ah[mi] = *(const f16x8*)(S + off);
      al[mi] = *(const f16x8*)(S + GM_A_PLANE + off);
    }
    if (!dead && !(VAR & 2))
#pragma unroll
    for (int nj = 0; nj < NJ; ++nj) {
      const int off = frag_off(wn * (BN / 2) + nj * 16 + fr);
      const f16x8 bh = *(const f16x8*)(S + A_BYTES + off);
      const f16x8 bl = *(const f16x8*)(S + A_BYTES + B_PLANE + off);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        f32x4v c = acc[mi][nj];
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[mi], bh, c, 0, 0, 0);  // small terms first
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[mi], bl, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[mi], bh, c, 0, 0, 0);
        acc[mi][nj] = c;
      }
    }
    wait_vm<0>();  // the next stage has landed
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

  // epilogue through LDS (each wave's 64 x BN/2 tile in passes of 64 columns, row pitch 68 floats),
  // then 16-byte stores: C = acc 2^-t_m / s_n + bias (+ res) (ReLU)
  constexpr int WC = 64, PITCH = WC + 4, LPR = WC / 4, RPI = 64 / LPR;
  constexpr int NPASS = (BN / 2) / WC, NJP = NJ / NPASS;
  float* T = reinterpret_cast<float*>(smem) + wave * (64 * PITCH);
  if (dead) return;  // (after the K loop's last barrier: no block-wide synchronisation follows)
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    if (pass > 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int qq = 0; qq < NJP; ++qq)
#pragma unroll
        for (int e = 0; e < 4; ++e) T[(mi * 16 + 4 * fs + e) * PITCH + qq * 16 + fr] = acc[mi][pass * NJP + qq][e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int c4 = (lane % LPR) * 4;
    const int n = n0 + wn * (BN / 2) + pass * WC + c4;
    float4 bn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g.bias) bn = *(const float4*)(g.bias + n);
    const float4 sn = *(const float4*)(g.ws + n);
#pragma unroll
    for (int it = 0; it < 64 / RPI; ++it) {
      const int rr = it * RPI + lane / LPR;
      const int m = m0 + wm * 64 + rr;
      if (m < g.M) {
        float4 v = *(const float4*)(T + rr * PITCH + c4);
        const float rs = arinv[m];
        v.x *= rs * sn.x; v.y *= rs * sn.y; v.z *= rs * sn.z; v.w *= rs * sn.w;
        v.x += bn.x; v.y += bn.y; v.z += bn.z; v.w += bn.w;
        if (g.res) {
          const float4 rv = *(const float4*)(g.res + (long long)m * g.ldc + n);
          v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
        }
        if (g.relu) {
          v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
        }
        if (!(VAR & 4)) *(float4*)(g.C + (long long)m * g.ldc + n) = v;
      }
    }
  }
}

// Three-ring form of the pre-split kernel (the default; RMBX_PRESPLIT_FORM=2 selects the two-stage
// form above): the 256 x 256 tile's K steps move by LDS-DMA into an A ring of three stages and a W
// ring of two (3 x 32 + 2 x 32 KiB = all 160 KiB of the CU's LDS), so the A pieces of step kt + 2 and
// the W pieces of step kt + 1 are in flight while step kt computes -- half again the bytes in
// flight of two full stages, and the DMA's L2 latency (~1.4 us per 64 KiB step measured with the
// MFMAs skipped) is what the two-stage form could not hide.  The eight DMA issues of a wave are
// spread over its eight column-tile MFMA groups instead of bunched at the step's start.  Per step,
// in issue order: W(kt + 1), then A(kt + 2); the step ends waiting until at most the A(kt + 2)
// pieces are outstanding, which retires A(kt + 1) (issued the step before) and W(kt + 1).
// SPLIT_OUT (rmbx_linear_f16x3_presplit_split): the outputs leave in the same pre-split form, for the
// next GEMM to load by DMA -- row m scaled by 2^u_m from a bound of its values, |c[m][n]| <=
// B_m = |a_m|_2 max_n |w_n|_2 + max |bias| (Cauchy-Schwarz on the f32 product; a_norm from the
// producing LayerNorm), 2^u_m putting B_m (1 + 2^-10) in [2^13, 2^14): hi = f16(c 2^u_m),
// lo = f16(c 2^u_m - hi), and out_rinv[m] = 2^-u_m.  The bound is loose by the ratio of B_m to the
// row's true max (a few bits for the ACT layers); elements below 2^-16 of B_m keep their low piece
// as an f16 subnormal, an absolute error <= 2^-38 B_m.
struct PresplitOut {
  uint16_t* planes;      // [2][M][ldo] f16 bits
  long long ldo, ps;     // row stride, plane stride (elements)
  float* rinv;           // [M]
  const float* a_norm;   // [M] upper bounds of the A rows' 2-norms
  float w_norm_max, b_abs_max;
};

template <int GROUP, int VAR = 0, bool SPLIT_OUT = false>
__global__ void __launch_bounds__(GM_THREADS, 1) gemm_f16x3_presplit3_kernel(GemmArgs g, const uint16_t* __restrict__ Ap,
                                                                            long long aps, long long ldah,
                                                                            const float* __restrict__ arinv,
                                                                            PresplitOut po = PresplitOut{},
                                                                            long long a_bs = 0, long long r_bs = 0) {
  constexpr int BN = 256, NJ = 8;
  constexpr int A_STAGE = 2 * GM_A_PLANE, B_PLANE = gm_b_plane<BN>(), W_STAGE = 2 * B_PLANE;  // 32 KiB each
  constexpr int W_RING = 3 * A_STAGE;
  constexpr int SMEM = 3 * A_STAGE + 2 * W_STAGE;
  static_assert(SMEM == 160 * 1024 && gm_epi_bytes<BN>() <= SMEM, "the LDS of a CU");
  constexpr int APW = 2 * (GM_BM / 16) / 8, WPW = 2 * (BN / 16) / 8;  // DMA pieces per wave and step
  static_assert(APW == 4 && WPW == 4 && APW + WPW == NJ, "one DMA issue per column-tile MFMA group");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 3, wn = wave >> 2;
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  if (g.batch > 1) {  // (rmbx_linear_f16x3_presplit_batched) consecutive tiles of an XCD stay in one item
    const int per_item = g.tiles_m * g.tiles_n;
    const int item = lin / per_item;
    lin -= item * per_item;
    Ap += item * a_bs;
    arinv += item * r_bs;
    g.W += item * g.w_bs;
    g.C += item * g.c_bs;
    g.ws += item * g.ws_bs;
  }
  const int per_group = GROUP * g.tiles_n;
  const int first_m = (lin / per_group) * GROUP;
  const int gsize = min(g.tiles_m - first_m, GROUP);
  const int in_group = lin - (lin / per_group) * per_group;
  const int tm = first_m + in_group % gsize, tn = in_group / gsize;
  const int m0 = tm * GM_BM, n0 = tn * BN;
  const bool dead = n0 + wn * (BN / 2) >= g.N;  // (wave-uniform) the half tile past N

  // the wave's pieces (16 rows x 64 B; lane l moves row l / 4, logical slot (l % 4) ^ ((row >> 2) & 2)
  // to physical slot l % 4): A pieces 4 wave .. 4 wave + 3 of the 32 (plane i / 16), W likewise
  const uint16_t* asrc[APW];
  const uint16_t* wsrc[WPW];
  int adst[APW], wdst[WPW];
#pragma unroll
  for (int t = 0; t < APW; ++t) {
    const int i = wave * APW + t, p = i / 16, rb = i % 16, row = rb * 16 + (lane >> 2);
    const int sl = (lane & 3) ^ ((row >> 2) & 2);
    asrc[t] = Ap + p * aps + (long long)min(m0 + row, g.M - 1) * ldah + sl * 8;
    adst[t] = p * GM_A_PLANE + rb * 1024;
  }
#pragma unroll
  for (int t = 0; t < WPW; ++t) {
    const int i = wave * WPW + t, p = i / 16, rb = i % 16, row = rb * 16 + (lane >> 2);
    const int sl = (lane & 3) ^ ((row >> 2) & 2);
    wsrc[t] = g.W + p * g.wps + (long long)min(n0 + row, g.N - 1) * g.ldw + sl * 8;
    wdst[t] = W_RING + p * B_PLANE + rb * 1024;
  }
  auto dma_a = [&](int t, int kt) {
    if constexpr ((VAR & 1) == 0) glds16(asrc[t] + kt * GM_BK, smem + (kt % 3) * A_STAGE + adst[t]);
  };
  auto dma_w = [&](int t, int kt) {
    if constexpr ((VAR & 1) == 0) glds16(wsrc[t] + kt * GM_BK, smem + (kt & 1) * W_STAGE + wdst[t]);
  };

  f32x4v acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4v){0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fs = lane >> 4;
  auto frag_off = [&](int row) { return row * 64 + ((fs ^ ((row >> 2) & 2)) << 4); };

  const int KT = g.K / GM_BK;
  // prologue: W(0), A(0), A(1)
#pragma unroll
  for (int t = 0; t < WPW; ++t) glds16(wsrc[t], smem + wdst[t]);
#pragma unroll
  for (int t = 0; t < APW; ++t) glds16(asrc[t], smem + adst[t]);
  if (KT > 1) {
#pragma unroll
    for (int t = 0; t < APW; ++t) glds16(asrc[t] + GM_BK, smem + A_STAGE + adst[t]);
    wait_vm<APW>();
  } else {
    wait_vm<0>();
  }
  asm volatile("s_barrier" ::: "memory");
  for (int kt = 0; kt < KT; ++kt) {
    const bool w_next = kt + 1 < KT, a_next = kt + 2 < KT;
    const unsigned char* SA = smem + (kt % 3) * A_STAGE;
    const unsigned char* SW = smem + W_RING + (kt & 1) * W_STAGE;
    f16x8 ah[4], al[4];
    if (!dead && !(VAR & 2)) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int off = frag_off(wm * 64 + mi * 16 + fr);
        ah[mi] = *(const f16x8*)(SA + off);
        al[mi] = *(const f16x8*)(SA + GM_A_PLANE + off);
      }
    }
#pragma unroll
    for (int nj = 0; nj < NJ; ++nj) {
      // one DMA issue per group: W(kt + 1) pieces first, then A(kt + 2)
      if (nj < WPW) {
        if (w_next) dma_w(nj, kt + 1);
      } else {
        if (a_next) dma_a(nj - WPW, kt + 2);
      }
      if (!dead && !(VAR & 2)) {
        const int off = frag_off(wn * (BN / 2) + nj * 16 + fr);
        const f16x8 bh = *(const f16x8*)(SW + off);
        const f16x8 bl = *(const f16x8*)(SW + B_PLANE + off);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          f32x4v c = acc[mi][nj];
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[mi], bh, c, 0, 0, 0);  // small terms first
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[mi], bl, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[mi], bh, c, 0, 0, 0);
          acc[mi][nj] = c;
        }
      }
    }
    if (a_next)
      wait_vm<APW>();  // A(kt + 2) may stay in flight
    else
      wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

  // epilogue through LDS (each wave's 64 x 128 tile in two passes of 64 columns, row pitch 68
  // floats), then 16-byte stores: C = acc 2^-t_m / s_n + bias (+ res) (ReLU)
  constexpr int WC = 64, PITCH = WC + 4, LPR = WC / 4, RPI = 64 / LPR;
  constexpr int NPASS = (BN / 2) / WC, NJP = NJ / NPASS;
  float* T = reinterpret_cast<float*>(smem) + wave * (64 * PITCH);
  if (dead) return;  // (after the K loop's last barrier: no block-wide synchronisation follows)
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    if (pass > 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int qq = 0; qq < NJP; ++qq)
#pragma unroll
        for (int e = 0; e < 4; ++e) T[(mi * 16 + 4 * fs + e) * PITCH + qq * 16 + fr] = acc[mi][pass * NJP + qq][e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (SPLIT_OUT) {
      // pre-split output: 8 columns per lane (16-byte stores of each piece plane), 8 rows per round
      const int c8 = (lane & 7) * 8;
      const int n = n0 + wn * (BN / 2) + pass * WC + c8;
      float sn8[8], bn8[8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 s4 = *(const float4*)(g.ws + n + 4 * h);
        const float4 b4 = g.bias ? *(const float4*)(g.bias + n + 4 * h) : make_float4(0.f, 0.f, 0.f, 0.f);
        sn8[4 * h] = s4.x; sn8[4 * h + 1] = s4.y; sn8[4 * h + 2] = s4.z; sn8[4 * h + 3] = s4.w;
        bn8[4 * h] = b4.x; bn8[4 * h + 1] = b4.y; bn8[4 * h + 2] = b4.z; bn8[4 * h + 3] = b4.w;
      }
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int rr = it * 8 + (lane >> 3);
        const int m = m0 + wm * 64 + rr;
        if (m < g.M) {
          const float4 v0 = *(const float4*)(T + rr * PITCH + c8), v1 = *(const float4*)(T + rr * PITCH + c8 + 4);
          const float vv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
          const float rs = arinv[m];
          const float B = (po.a_norm[m] * po.w_norm_max + po.b_abs_max) * (1.f + 0.0009765625f);
          int e = 14;
          if (B > 0.f && B <= 3.4e38f) frexpf(B, &e);  // B = f 2^e, f in [0.5, 1); NaN / inf: scale 1
          const float sc = ldexpf(1.f, 14 - e);
          if (n == 0) po.rinv[m] = ldexpf(1.f, e - 14);
          uint32_t hw[4], lw[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float x0 = vv[2 * k] * (rs * sn8[2 * k]) + bn8[2 * k];
            float x1 = vv[2 * k + 1] * (rs * sn8[2 * k + 1]) + bn8[2 * k + 1];
            if (g.relu) {
              x0 = fmaxf(x0, 0.f);
              x1 = fmaxf(x1, 0.f);
            }
            x0 *= sc;
            x1 *= sc;
            const _Float16 h0 = (_Float16)x0, h1 = (_Float16)x1;
            const _Float16 l0 = (_Float16)(x0 - (float)h0), l1 = (_Float16)(x1 - (float)h1);
            hw[k] = __builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
            lw[k] = __builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
          }
          uint16_t* o = po.planes + (long long)m * po.ldo + n;
          *(uint4*)o = make_uint4(hw[0], hw[1], hw[2], hw[3]);
          *(uint4*)(o + po.ps) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
        }
      }
      continue;
    }
    const int c4 = (lane % LPR) * 4;
    const int n = n0 + wn * (BN / 2) + pass * WC + c4;
    float4 bn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g.bias) bn = *(const float4*)(g.bias + n);
    const float4 sn = *(const float4*)(g.ws + n);
#pragma unroll
    for (int it = 0; it < 64 / RPI; ++it) {
      const int rr = it * RPI + lane / LPR;
      const int m = m0 + wm * 64 + rr;
      if (m < g.M) {
        float4 v = *(const float4*)(T + rr * PITCH + c4);
        const float rs = arinv[m];
        v.x *= rs * sn.x; v.y *= rs * sn.y; v.z *= rs * sn.z; v.w *= rs * sn.w;
        v.x += bn.x; v.y += bn.y; v.z += bn.z; v.w += bn.w;
        if (g.res) {
          const float4 rv = *(const float4*)(g.res + (long long)m * g.ldc + n);
          v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
        }
        if (g.relu) {
          v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
        }
        if constexpr ((VAR & 8) != 0) {  // (profiling) non-temporal output stores
          const f32x4v vv = {v.x, v.y, v.z, v.w};
          __builtin_nontemporal_store(vv, (f32x4v*)(g.C + (long long)m * g.ldc + n));
        } else if (!(VAR & 4)) {
          *(float4*)(g.C + (long long)m * g.ldc + n) = v;
        }
      }
    }
  }
}

// default: the LDS-transposed epilogue with 16-byte stores (VAR 16: 1.04-1.08x over 64 scalar
// stores per lane, profiles/r3_gemm_var_sweep.log) whenever the output / residual / bias rows allow
// 16-byte accesses; RMBX_GEMM_VAR overrides the bf16x6 form (profiling)
template <bool CONV, int PC>
void launch_gemm(long long blocks, const GemmArgs& g, hipStream_t st, int bn = 128) {
  const bool vec_ok = g.ldc % 4 == 0 &&
                      ((uintptr_t)g.C | (uintptr_t)g.res | (uintptr_t)g.bias | (uintptr_t)g.ws) % 16 == 0 &&
                      (g.batch <= 1 || (g.c_bs % 4 == 0 && g.ws_bs % 4 == 0));
  if constexpr (PC == 2) {
    if (bn == 64) {  // the narrow tile (N % 128 != 0): default epilogue forms only
      if (vec_ok)
        hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 16, 2, 64>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g);
      else
        hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 0, 2, 64>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g);
      return;
    }
    if (bn == 256) {  // the wide tile
      if (vec_ok)
        hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 16, 2, 256>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g);
      else
        hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 0, 2, 256>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g);
      return;
    }
    // producer / consumer form (RMBX_GEMM_PC=1; read per launch so a test can compare the forms)
    const char* pce = getenv("RMBX_GEMM_PC");
    const bool pc = pce && atoi(pce) != 0;
    if (pc) {
      if (vec_ok)
        hipLaunchKernelGGL((gemm_f16x3_pc_kernel<CONV, true>), dim3((unsigned)blocks), dim3(GP_THREADS), 0, st, g);
      else
        hipLaunchKernelGGL((gemm_f16x3_pc_kernel<CONV, false>), dim3((unsigned)blocks), dim3(GP_THREADS), 0, st, g);
      return;
    }
    // RMBX_GEMM_VAR (profiling, linear only): 16 | phase skips 32 (no split), 256 (no A loads),
    // 512 (no W DMA) -- wrong results, timing only; 1040 = three LDS stages (same results)
    const char* ve = CONV ? nullptr : getenv("RMBX_GEMM_VAR");
    const int var = ve && vec_ok ? atoi(ve) : (vec_ok ? 16 : 0);
    switch (var) {
      case 0: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 0, 2>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 48: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 48, 2>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 272: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 272, 2>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 528: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 528, 2>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 784: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 784, 2>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 816: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 816, 2>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 1040: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 1040, 2>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      default: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 16, 2>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g);
    }
    return;
  } else {
    // (the environment is read per launch, so a test or a profile can compare the forms in one process)
    const char* ve = getenv("RMBX_GEMM_VAR");
    const int env_var = ve ? atoi(ve) : -1;
    int var = env_var >= 0 ? env_var : 16;
    if (!vec_ok) var &= ~16;
    switch (var) {
      case 1: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 1>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 2: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 2>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 4: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 4>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 8: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 8>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 16: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 16>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 18: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 18>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 48: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 48>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      case 80: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 80>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g); break;
      default: hipLaunchKernelGGL((gemm_f32x6_kernel<CONV, 0>), dim3((unsigned)blocks), dim3(GM_THREADS), 0, st, g);
    }
  }
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_split_bf16x3(const float* x, void* planes, long long n, void* stream) {
  RMBX_CHECK_ARG(x && planes && n >= 0, "rmbx_split_bf16x3: bad arguments");
  if (n == 0) return RMBX_OK;
  const long long blocks = (n + 255) / 256;
  hipLaunchKernelGGL(rmbx::split_bf16x3_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0,
                     (hipStream_t)stream, x, (uint16_t*)planes, n);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

namespace rmbx {
namespace {
// shared argument checks and launch of the linear / batched / conv entry points of both forms
// f16x3 dispatch: the leading multiple of 256 output columns on the 256-wide tile (A split once
// per 256 columns instead of 128: 1.05-1.09x at the ACT shapes, bitwise equal,
// profiles/r4_gemm_wide_ab.log), the 128 columns left over (N = 3200 = 3072 + 128) by a second
// launch of the 128-wide tile; N % 128 != 0 runs the 64-wide tile.  RMBX_GEMM_WIDE=0 (read per
// launch) keeps everything on the 128-wide tile.
// Small grids (fewer blocks than CUs at one block per CU, e.g. the DiffusionPolicy UNet's
// 32,768 x 256 layers: 128 wide tiles) take the 128- or 64-wide tile instead, so every CU gets a
// block (same per-element K order: bitwise-equal results); RMBX_GEMM_FILL=0 (read per launch) keeps
// the width rule above.
static int gemm_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  return cus;
}
template <bool CONV>
void launch_f16x3(const GemmArgs& g, hipStream_t st, int bn) {
  const char* we = getenv("RMBX_GEMM_WIDE");
  const bool wide = !(we && atoi(we) == 0);
  const int n256 = g.N / 256 * 256;
  const long long items = g.batch > 1 ? g.batch : 1;
  const char* fe = getenv("RMBX_GEMM_FILL");
  if (!(fe && atoi(fe) == 0) && bn == GM_BN) {
    const long long cus = gemm_cus();
    const long long wide_blocks = (long long)g.tiles_m * (g.N / 256 + (g.N % 256 ? 1 : 0)) * items;
    if (wide_blocks < cus) {
      int nb = GM_BN;
      if ((long long)g.tiles_m * (g.N / GM_BN) * items < cus && g.N % 64 == 0) nb = 64;
      GemmArgs t = g;
      t.tiles_n = g.N / nb;
      launch_gemm<CONV, 2>((long long)t.tiles_m * t.tiles_n * items, t, st, nb);
      return;
    }
  }
  if (!wide || bn != GM_BN || n256 == 0) {
    launch_gemm<CONV, 2>((long long)g.tiles_m * g.tiles_n * items, g, st, bn);
    return;
  }
  GemmArgs w = g;
  w.N = n256;
  w.tiles_n = n256 / 256;
  launch_gemm<CONV, 2>((long long)w.tiles_m * w.tiles_n * items, w, st, 256);
  if (n256 == g.N) return;
  GemmArgs t = g;
  t.W = g.W + (long long)n256 * g.ldw;
  t.bias = g.bias ? g.bias + n256 : nullptr;
  t.C = g.C + n256;
  t.res = g.res ? g.res + n256 : nullptr;
  t.ws = g.ws + n256;
  t.N = g.N - n256;
  t.tiles_n = t.N / GM_BN;
  launch_gemm<CONV, 2>((long long)t.tiles_m * t.tiles_n * items, t, st, GM_BN);
}

template <int PC>
int linear_impl(const char* fn, const float* a, long long lda, long long a_bs, const void* w_planes, long long ldw,
                long long wps, long long w_bs, const float* ws, long long ws_bs, const float* bias, float* c,
                long long ldc, long long c_bs, int batch, int M, int N, int K, int relu, void* stream) {
  RMBX_CHECK_ARG(a && w_planes && c && (PC == 3 || ws), "%s: null pointer", fn);
  RMBX_CHECK_ARG(batch >= 1 && M >= 0 && N > 0 && K > 0, "%s: bad shape M=%d N=%d K=%d", fn, M, N, K);
  // output columns per block: 128, or 64 for f16x3 layers narrower than a multiple of 128 (the
  // f16x3 form runs the leading multiple of 256 columns on its 256-wide tile, launch_f16x3)
  const int bn = PC == 2 && N % GM_BN != 0 ? 64 : GM_BN;
  RMBX_CHECK_ARG(N % bn == 0, "%s: N=%d must be a multiple of %d", fn, N, PC == 2 ? 64 : GM_BN);
  RMBX_CHECK_ARG(K % GM_BK == 0, "%s: K=%d must be a multiple of %d", fn, K, GM_BK);
  RMBX_CHECK_ARG(lda >= K && lda % 4 == 0 && a_bs % 4 == 0 && ldc >= N && ldw >= K && ldw % 8 == 0 && wps % 8 == 0 &&
                     w_bs % 8 == 0,
                 "%s: bad strides lda=%lld ldc=%lld ldw=%lld wps=%lld", fn, lda, ldc, ldw, wps);
  RMBX_CHECK_ARG(((uintptr_t)a | (uintptr_t)w_planes) % 16 == 0, "%s: operands must be 16-B aligned", fn);
  if (M == 0) return RMBX_OK;
  GemmArgs g{a, (const uint16_t*)w_planes, bias, c, lda, ldc, ldw, wps, M, N, K, relu ? 1 : 0,
             (M + GM_BM - 1) / GM_BM, N / bn, nullptr};
  g.batch = batch;
  g.a_bs = a_bs;
  g.w_bs = w_bs;
  g.c_bs = c_bs;
  g.ws = ws;
  g.ws_bs = ws_bs;
  const long long blocks = (long long)g.tiles_m * g.tiles_n * batch;
  RMBX_CHECK_ARG(blocks < (1ll << 31), "%s: too many tiles", fn);
  if constexpr (PC == 2) {
    launch_f16x3<false>(g, (hipStream_t)stream, bn);
  } else {
    launch_gemm<false, PC>(blocks, g, (hipStream_t)stream, bn);
  }
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

template <int PC>
int conv_impl(const char* fn, const float* in, int N, int H, int W, int C, const void* w_planes, const float* ws,
              const float* bias, const float* res, float* out, int Cout, int KH, int KW, int stride, int pad, int relu,
              void* stream) {
  RMBX_CHECK_ARG(in && w_planes && out && (PC == 3 || ws), "%s: null pointer", fn);
  RMBX_CHECK_ARG(N >= 0 && H > 0 && W > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0, "%s: bad geometry", fn);
  RMBX_CHECK_ARG(C % GM_BK == 0, "%s: C=%d must be a multiple of %d", fn, C, GM_BK);
  const int bn = PC == 2 && Cout % GM_BN != 0 ? 64 : GM_BN;
  RMBX_CHECK_ARG(Cout % bn == 0, "%s: Cout=%d must be a multiple of %d", fn, Cout, PC == 2 ? 64 : GM_BN);
  RMBX_CHECK_ARG(((uintptr_t)in | (uintptr_t)w_planes) % 16 == 0, "%s: operands must be 16-B aligned", fn);
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  RMBX_CHECK_ARG(Ho > 0 && Wo > 0, "%s: empty output", fn);
  const long long M = (long long)N * Ho * Wo;
  RMBX_CHECK_ARG(M < (1ll << 31) && (long long)N * H * W < (1ll << 31), "%s: too many pixels", fn);
  if (M == 0) return RMBX_OK;
  const int K = KH * KW * C;
  GemmArgs g{in, (const uint16_t*)w_planes, bias, out, 0, Cout, K, (long long)Cout * K, (int)M, Cout, K,
             relu ? 1 : 0, (int)((M + GM_BM - 1) / GM_BM), Cout / bn, res, H, W, C, Ho, Wo, KW, stride, pad};
  g.ws = ws;
  const long long blocks = (long long)g.tiles_m * g.tiles_n;
  RMBX_CHECK_ARG(blocks < (1ll << 31), "%s: too many tiles", fn);
  if constexpr (PC == 2) {
    launch_f16x3<true>(g, (hipStream_t)stream, bn);
  } else {
    launch_gemm<true, PC>(blocks, g, (hipStream_t)stream, bn);
  }
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
}  // namespace
}  // namespace rmbx

extern "C" int rmbx_linear_f32x6(const float* a, long long lda, const void* w_planes, long long ldw,
                                 long long w_plane_stride, const float* bias, float* c, long long ldc, int M, int N,
                                 int K, int relu, void* stream) {
  return rmbx::linear_impl<3>("rmbx_linear_f32x6", a, lda, 0, w_planes, ldw, w_plane_stride, 0, nullptr, 0, bias, c,
                              ldc, 0, 1, M, N, K, relu, stream);
}

extern "C" int rmbx_linear_f32x6_batched(const float* a, long long lda, long long a_bs, const void* w_planes,
                                         long long ldw, long long w_plane_stride, long long w_bs, const float* bias,
                                         float* c, long long ldc, long long c_bs, int batch, int M, int N, int K,
                                         int relu, void* stream) {
  return rmbx::linear_impl<3>("rmbx_linear_f32x6_batched", a, lda, a_bs, w_planes, ldw, w_plane_stride, w_bs, nullptr,
                              0, bias, c, ldc, c_bs, batch, M, N, K, relu, stream);
}

extern "C" int rmbx_conv2d_f32x6(const float* in, int N, int H, int W, int C, const void* w_planes, const float* bias,
                                 const float* res, float* out, int Cout, int KH, int KW, int stride, int pad, int relu,
                                 void* stream) {
  return rmbx::conv_impl<3>("rmbx_conv2d_f32x6", in, N, H, W, C, w_planes, nullptr, bias, res, out, Cout, KH, KW,
                            stride, pad, relu, stream);
}

extern "C" int rmbx_split_f16x2(const float* w, int N, int K, void* planes, float* scale, void* stream) {
  RMBX_CHECK_ARG(w && planes && scale && N >= 0 && K > 0, "rmbx_split_f16x2: bad arguments");
  if (N == 0) return RMBX_OK;
  hipLaunchKernelGGL(rmbx::split_f16x2_kernel, dim3((unsigned)N), dim3(256), 0, (hipStream_t)stream, w, K,
                     (long long)N * K, (uint16_t*)planes, scale);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_linear_f16x3(const float* a, long long lda, const void* w_planes, long long ldw,
                                 long long w_plane_stride, const float* w_scale, const float* bias, float* c,
                                 long long ldc, int M, int N, int K, int relu, void* stream) {
  return rmbx::linear_impl<2>("rmbx_linear_f16x3", a, lda, 0, w_planes, ldw, w_plane_stride, 0, w_scale, 0, bias, c,
                              ldc, 0, 1, M, N, K, relu, stream);
}

extern "C" int rmbx_linear_f16x3_batched(const float* a, long long lda, long long a_bs, const void* w_planes,
                                         long long ldw, long long w_plane_stride, long long w_bs, const float* w_scale,
                                         long long ws_bs, const float* bias, float* c, long long ldc, long long c_bs,
                                         int batch, int M, int N, int K, int relu, void* stream) {
  return rmbx::linear_impl<2>("rmbx_linear_f16x3_batched", a, lda, a_bs, w_planes, ldw, w_plane_stride, w_bs, w_scale,
                              ws_bs, bias, c, ldc, c_bs, batch, M, N, K, relu, stream);
}

extern "C" int rmbx_conv2d_f16x3(const float* in, int N, int H, int W, int C, const void* w_planes,
                                 const float* w_scale, const float* bias, const float* res, float* out, int Cout,
                                 int KH, int KW, int stride, int pad, int relu, void* stream) {
  return rmbx::conv_impl<2>("rmbx_conv2d_f16x3", in, N, H, W, C, w_planes, w_scale, bias, res, out, Cout, KH, KW,
                            stride, pad, relu, stream);
}

extern "C" int rmbx_linear_f16x3_presplit(const void* a_planes, long long lda, long long a_plane_stride,
                                          const float* a_rinv, const void* w_planes, long long ldw,
                                          long long w_plane_stride, const float* w_scale, const float* bias,
                                          const float* res, float* c, long long ldc, int M, int N, int K, int relu,
                                          void* stream) {
  const char* fn = "rmbx_linear_f16x3_presplit";
  RMBX_CHECK_ARG(a_planes && a_rinv && w_planes && w_scale && c, "%s: null pointer", fn);
  RMBX_CHECK_ARG(M >= 0 && N > 0 && K > 0 && N % rmbx::GM_BN == 0 && K % rmbx::GM_BK == 0,
                 "%s: bad shape M=%d N=%d K=%d (N %% 128, K %% 32)", fn, M, N, K);
  RMBX_CHECK_ARG(lda >= K && lda % 8 == 0 && a_plane_stride % 8 == 0 && ldw >= K && ldw % 8 == 0 &&
                     w_plane_stride % 8 == 0 && ldc >= N && ldc % 4 == 0,
                 "%s: bad strides lda=%lld ldw=%lld ldc=%lld", fn, lda, ldw, ldc);
  RMBX_CHECK_ARG(((uintptr_t)a_planes | (uintptr_t)w_planes | (uintptr_t)c | (uintptr_t)bias | (uintptr_t)res |
                  (uintptr_t)w_scale) % 16 == 0,
                 "%s: operands must be 16-B aligned", fn);
  RMBX_CHECK_ARG((long long)M * lda + a_plane_stride < (1ll << 62), "%s: too large", fn);
  if (M == 0) return RMBX_OK;
  rmbx::GemmArgs g{nullptr, (const uint16_t*)w_planes, bias, c, 0, ldc, ldw, w_plane_stride, M, N, K, relu ? 1 : 0,
                   (M + rmbx::GM_BM - 1) / rmbx::GM_BM, 0, res};
  g.batch = 1;
  g.ws = w_scale;
  hipStream_t st = (hipStream_t)stream;
  const uint16_t* ap = (const uint16_t*)a_planes;
  // every column tile on the 256-wide tile (N % 256 == 128: the last one half dead); RMBX_PRESPLIT_GROUP
  // (profiling, read per launch) = row tiles per block group, 8 by default
  g.tiles_n = (N + 255) / 256;
  const long long blocks = (long long)g.tiles_m * g.tiles_n;
  RMBX_CHECK_ARG(blocks < (1ll << 31), "%s: too many tiles", fn);
  const char* ge = getenv("RMBX_PRESPLIT_GROUP");
  const int grp = ge ? atoi(ge) : 8;
  const char* ve = getenv("RMBX_PRESPLIT_VAR");
  const int var = ve ? atoi(ve) : 0;
  const char* fe = getenv("RMBX_PRESPLIT_FORM");
  const int form = fe ? atoi(fe) : 3;
  const bool form2 = form == 2;
  if (!form2) {  // the three-ring form (default)
    switch (var) {
      case 0: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit3_kernel<8, 0>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      case 1: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit3_kernel<8, 1>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      case 2: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit3_kernel<8, 2>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      case 4: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit3_kernel<8, 4>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      case 5: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit3_kernel<8, 5>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      case 6: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit3_kernel<8, 6>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      case 8: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit3_kernel<8, 8>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      default: RMBX_CHECK_ARG(false, "%s: RMBX_PRESPLIT_VAR %d", fn, var);
    }
    RMBX_CHECK_LAUNCH();
    return RMBX_OK;
  }
  if (var != 0) {  // profiling phase skips at the default group
    switch (var) {
      case 1: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit_kernel<256, 8, 1>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      case 2: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit_kernel<256, 8, 2>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      case 4: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit_kernel<256, 8, 4>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      case 5: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit_kernel<256, 8, 5>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      case 6: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit_kernel<256, 8, 6>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
      default: RMBX_CHECK_ARG(false, "%s: RMBX_PRESPLIT_VAR %d", fn, var);
    }
    RMBX_CHECK_LAUNCH();
    return RMBX_OK;
  }
  switch (grp) {
    case 2: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit_kernel<256, 2>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
    case 4: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit_kernel<256, 4>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
    case 16: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit_kernel<256, 16>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv); break;
    default: hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit_kernel<256, 8>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0, st, g, ap, a_plane_stride, lda, a_rinv);
  }
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_linear_f16x3_presplit_split(const void* a_planes, long long lda, long long a_plane_stride,
                                                const float* a_rinv, const float* a_norm, const void* w_planes,
                                                long long ldw, long long w_plane_stride, const float* w_scale,
                                                float w_norm_max, float b_abs_max, const float* bias, int relu,
                                                void* out_planes, long long ldo, long long out_plane_stride,
                                                float* out_rinv, int M, int N, int K, void* stream) {
  const char* fn = "rmbx_linear_f16x3_presplit_split";
  RMBX_CHECK_ARG(a_planes && a_rinv && a_norm && w_planes && w_scale && out_planes && out_rinv, "%s: null pointer", fn);
  RMBX_CHECK_ARG(M >= 0 && N > 0 && K > 0 && N % rmbx::GM_BN == 0 && K % rmbx::GM_BK == 0,
                 "%s: bad shape M=%d N=%d K=%d (N %% 128, K %% 32)", fn, M, N, K);
  RMBX_CHECK_ARG(lda >= K && lda % 8 == 0 && a_plane_stride % 8 == 0 && ldw >= K && ldw % 8 == 0 &&
                     w_plane_stride % 8 == 0 && ldo >= N && ldo % 8 == 0 && out_plane_stride % 8 == 0 &&
                     out_plane_stride >= (long long)M * ldo,
                 "%s: bad strides lda=%lld ldw=%lld ldo=%lld", fn, lda, ldw, ldo);
  RMBX_CHECK_ARG(((uintptr_t)a_planes | (uintptr_t)w_planes | (uintptr_t)bias | (uintptr_t)w_scale |
                  (uintptr_t)out_planes) % 16 == 0,
                 "%s: operands must be 16-B aligned", fn);
  RMBX_CHECK_ARG(w_norm_max >= 0.f && b_abs_max >= 0.f, "%s: bad bounds", fn);
  if (M == 0) return RMBX_OK;
  rmbx::GemmArgs g{nullptr, (const uint16_t*)w_planes, bias, nullptr, 0, 0, ldw, w_plane_stride, M, N, K,
                   relu ? 1 : 0, (M + rmbx::GM_BM - 1) / rmbx::GM_BM, (N + 255) / 256, nullptr};
  g.batch = 1;
  g.ws = w_scale;
  const long long blocks = (long long)g.tiles_m * g.tiles_n;
  RMBX_CHECK_ARG(blocks < (1ll << 31), "%s: too many tiles", fn);
  rmbx::PresplitOut po{(uint16_t*)out_planes, ldo, out_plane_stride, out_rinv, a_norm, w_norm_max, b_abs_max};
  hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit3_kernel<8, 0, true>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0,
                     (hipStream_t)stream, g, (const uint16_t*)a_planes, a_plane_stride, lda, a_rinv, po);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_linear_f16x3_presplit_batched(const void* a_planes, long long lda, long long a_plane_stride,
                                                  long long a_bs, const float* a_rinv, long long r_bs,
                                                  const void* w_planes, long long ldw, long long w_plane_stride,
                                                  long long w_bs, const float* w_scale, long long ws_bs,
                                                  const float* bias, float* c, long long ldc, long long c_bs,
                                                  int batch, int M, int N, int K, int relu, void* stream) {
  const char* fn = "rmbx_linear_f16x3_presplit_batched";
  RMBX_CHECK_ARG(a_planes && a_rinv && w_planes && w_scale && c && batch >= 1, "%s: null pointer / batch", fn);
  RMBX_CHECK_ARG(M >= 0 && N > 0 && K > 0 && N % rmbx::GM_BN == 0 && K % rmbx::GM_BK == 0,
                 "%s: bad shape M=%d N=%d K=%d (N %% 128, K %% 32)", fn, M, N, K);
  RMBX_CHECK_ARG(lda >= K && lda % 8 == 0 && a_plane_stride % 8 == 0 && a_bs % 8 == 0 && ldw >= K && ldw % 8 == 0 &&
                     w_plane_stride % 8 == 0 && w_bs % 8 == 0 && ws_bs % 4 == 0 && ldc >= N && ldc % 4 == 0 &&
                     c_bs % 4 == 0 && r_bs >= 0,
                 "%s: bad strides", fn);
  RMBX_CHECK_ARG(((uintptr_t)a_planes | (uintptr_t)w_planes | (uintptr_t)c | (uintptr_t)bias | (uintptr_t)w_scale) % 16 ==
                     0,
                 "%s: operands must be 16-B aligned", fn);
  if (M == 0) return RMBX_OK;
  rmbx::GemmArgs g{nullptr, (const uint16_t*)w_planes, bias, c, 0, ldc, ldw, w_plane_stride, M, N, K, relu ? 1 : 0,
                   (M + rmbx::GM_BM - 1) / rmbx::GM_BM, (N + 255) / 256, nullptr};
  g.batch = batch;
  g.w_bs = w_bs;
  g.c_bs = c_bs;
  g.ws = w_scale;
  g.ws_bs = ws_bs;
  const long long blocks = (long long)g.tiles_m * g.tiles_n * batch;
  RMBX_CHECK_ARG(blocks < (1ll << 31), "%s: too many tiles", fn);
  hipLaunchKernelGGL((rmbx::gemm_f16x3_presplit3_kernel<8, 0, false>), dim3((unsigned)blocks), dim3(rmbx::GM_THREADS), 0,
                     (hipStream_t)stream, g, (const uint16_t*)a_planes, a_plane_stride, lda, a_rinv, rmbx::PresplitOut{},
                     a_bs, r_bs);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
