// f32 3x3 / stride-1 / pad-1 convolution by Winograd F(2x2, 3x3) on f32 MFMA, with the
// bias / residual / ReLU epilogue fused (NHWC, Cin = Cout = C in {64, 128, 256, 512}).
//
// Replaces the stride-1 conv -> FrozenBN -> (+ residual) -> ReLU steps of the ResNet-18
// BasicBlocks in ACT's backbone (torchvision resnet18 inside third_party/act [absent]; the
// reference runs the policy in fp32, RolloutAct.py / ACTPolicy) for the fp32 policy path.  gfx950
// has no TF32, so f32 convs run on v_mfma_f32_32x32x2_f32 at the f32 vector rate (157 TF/s); the
// direct algorithm needs 9 products per output per input channel, F(2x2, 3x3) needs 16 per 2x2
// output tile = 4 per output (2.25x fewer MFMAs).  The transforms are additions and halvings
// (B, A: 0 / +-1; G: 0 / +-1/2), so the result is the same convolution up to f32 rounding of a
// few extra adds (measured against the direct fp32 conv in tests/test_winograd_gpu.py).
//
//   V = B^T d B  (4x4 input window d of a 2x2 output tile, per input channel)
//   U = G g G^T  (per filter; packed once on the host in f64, rounded to f32)
//   M[p] = sum_c U[p][co][c] V[p][c][tile]    p = 0..15: sixteen GEMMs with K = Cin
//   Y = A^T M A  (2x2 outputs per tile)
//
// Mapping (MI355X: 256 CUs in 8 XCDs, 160 KiB LDS, 512 registers per lane at one wave per SIMD):
//  * a block = 4 waves (one per SIMD) owns 64 output channels x 64 tiles; wave (cw, tw) keeps
//    32 channels x 32 tiles for ALL 16 positions in 16 accumulators (256 registers), so the output
//    transform runs in registers and each lane finishes 16 consecutive channels of one tile
//    (A rows permuted in the packed U), leaving as 16-byte stores;
//  * K runs in chunks of 8 input channels: U (32 KiB, pre-packed in the exact LDS image) and V
//    (32 KiB, computed from the gathered 4x4 windows) are double-buffered in LDS (128 KiB); the
//    next chunk's global loads are issued before this chunk's 64 MFMAs per wave and its LDS
//    stores are spread over the second half of the MFMA stream, one LDS-only barrier per chunk;
//  * persistent blocks, one per CU; the output-channel block is fixed per XCD (blockIdx % 8) so
//    each XCD's L2 holds the U slice it streams (2 MiB at C = 512), and the chunk pipeline runs
//    on across tile blocks (the next tile block's first chunk is staged under the last MFMAs of
//    the current one).
#include "rmbx_common.h"

#include <cstdint>
#include <cstdlib>

namespace rmbx {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int WG_THREADS = 512;
constexpr int WG_TILES = 64;                   // tiles per block unit
constexpr int WG_COUT = 64;                    // output channels per block unit
constexpr int WG_KC = 8;                       // input channels per K chunk
constexpr int WG_PLANE = 64 * WG_KC;           // floats per position plane: [64 rows][8 channels]
constexpr int WG_CHUNK = 16 * WG_PLANE;        // floats of one U or V chunk (32 KiB)
static_assert(4 * WG_CHUNK * 4 <= 160 * 1024, "double-buffered U and V must fit the LDS of a CU");

struct WinoArgs {
  const float* in;    // [N][H][W][C]
  const float* u;     // packed [C/64][C/8][16][64][8]
  const float* bias;  // [C]
  const float* res;   // [N][H][W][C] or null
  float* out;         // [N][H][W][C]
  int N, H, W, C, relu;
  int tiles_x, tiles_y;
  int ntiles;         // N * tiles_y * tiles_x (< 2^31, checked on the host)
  int ntb;            // tile blocks of WG_TILES
  int ncb, nk, nk_log2;  // C / 64, C / 8, log2(nk)
  int stagger;        // start delay per XCD-local block slot, in units of 4096 cycles
  int dbg;            // diagnostic phase skips (RMBX_WINO_DBG: 1 = no MFMAs, 2 = no window loads,
                      // 4 = no V transform / stores, 8 = no U loads; 0 in production)
};

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA of 16 bytes per lane (global_load_lds_dwordx4: the wave's 64 x 16 B land contiguously at
// the wave-uniform LDS byte address lds_dst).  Issued from inline asm so that hipcc does not insert
// its conservative vmcnt(0) before the next LDS read -- which would also make the loader waves wait
// for their in-flight window loads at the top of every chunk; completion is counted by hand
// (s_waitcnt vmcnt(0) of the U waves) before the barrier that publishes the chunk.
__device__ __forceinline__ void glds16(const float* gsrc, const float* lds_dst) {
  const uint32_t dst = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)lds_dst;
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(dst))
               : "memory");
}

template <int DBG>
__global__ void __launch_bounds__(WG_THREADS, 1) wino_f32_kernel(WinoArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[4 * WG_CHUNK];  // sU[2], sV[2]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cq = wave & 3, th = wave >> 2;  // MFMA work: channels 16 cq.. of the unit, tiles 32 th..
  const int li = lane & 15, lq = lane >> 4;  // 16x16x4 operand lane: row / column li, k group lq
  const bool loader = wave < 4;              // waves 0-3 gather and transform the windows, 4-7 move U

  // persistent schedule: output-channel block cb fixed per XCD (blockIdx % 8)
  const int G = gridDim.x;  // multiple of 8 (host)
  const int xcd = blockIdx.x & 7;
  const int cb = xcd % a.ncb;
  const int per_cb = G / a.ncb;
  const int r = (blockIdx.x >> 3) * (8 / a.ncb) + xcd / a.ncb;
  if (r >= a.ntb) return;
  const int nunits = (a.ntb - r + per_cb - 1) / per_cb;
  // stagger the blocks of an XCD by eighths of a unit so that their unit epilogues (residual loads
  // and output stores) do not hit HBM as one synchronised burst
  if (a.stagger > 0)
    for (int i = 0; i < ((blockIdx.x >> 3) & 7) * a.stagger; ++i) __builtin_amdgcn_s_sleep(64);
  const int nsteps = nunits << a.nk_log2;

  // ---- loader state: this thread's 4x4 window of 2 channels (loader waves)
  const int lt = (tid >> 2) & 63, cp = tid & 3;  // loader tile (0..63) and channel pair
  float2 xreg[16];
  uint32_t xok = 0;
  int ld_unit = -1, ld_o0 = 0;  // loader tile window origin (element offset, may be < 0 at the top-left
  uint32_t ld_mask = 0;         // halo; masked pixels read element 0) and in-image mask of ld_unit
  auto tile_pos = [&](int t, int& img, int& ty, int& tx) {
    const int q = t / a.tiles_x;
    tx = t - q * a.tiles_x;
    img = q / a.tiles_y;
    ty = q - img * a.tiles_y;
  };
  // step s: U waves copy the chunk's U image global -> LDS buffer (s & 1) by LDS-DMA (the packed U
  // is the exact LDS image: 8 KiB per wave as 8 lane-linear 1-KiB pieces); loader threads load
  // their window into registers
  auto load_u = [&](int s) {  // U waves
    const int k = s & (a.nk - 1);
    const float* ug = a.u + ((size_t)cb * a.nk + k) * WG_CHUNK + (wave - 4) * 2048 + lane * 4;
    float* ul = smem + (s & 1) * WG_CHUNK + (wave - 4) * 2048;
    if (!(DBG & 8))
#pragma unroll
      for (int j = 0; j < 8; ++j)
        glds16(ug + 256 * j, ul + 256 * j);
  };
  auto load_window = [&](int s) {  // loader threads
    const int unit = s >> a.nk_log2;
    const int k = s & (a.nk - 1);
    if (unit != ld_unit) {  // the loader tile's window origin and in-image mask, once per unit
      ld_unit = unit;
      const int t = (r + unit * per_cb) * WG_TILES + lt;
      const bool tok = t < a.ntiles;
      int img, ty, tx;
      tile_pos(tok ? t : a.ntiles - 1, img, ty, tx);
      const int y0 = 2 * ty - 1, x0 = 2 * tx - 1;
      ld_o0 = ((img * a.H + y0) * a.W + x0) * a.C + 2 * cp;
      ld_mask = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int y = y0 + (i >> 2), x = x0 + (i & 3);
        ld_mask |= (uint32_t)(tok && y >= 0 && y < a.H && x >= 0 && x < a.W) << i;
      }
    }
    xok = ld_mask;
    const int o = ld_o0 + k * WG_KC;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int off = ((ld_mask >> i) & 1u) ? o + ((i >> 2) * a.W + (i & 3)) * a.C : 0;
      xreg[i] = *reinterpret_cast<const float2*>(a.in + off);
    }
  };
  // ---- V = B^T d B of the loaded window into LDS buffer `buf` (loader threads), in 8 pieces
  // (hook(q), q = 0..7): piece 0 masks the window and forms tmp = B^T d (all four rows); piece q
  // writes V[q / 2][2 (q & 1) .. 2 (q & 1) + 1] = tmp row q / 2 times B
  float2 tmp[4][4];
  auto store_piece = [&](int buf, int q) {
    if (q == 0) {
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        float2 d[4];
#pragma unroll
        for (int y = 0; y < 4; ++y) d[y] = ((xok >> (y * 4 + x)) & 1u) ? xreg[y * 4 + x] : make_float2(0.f, 0.f);
        tmp[0][x] = make_float2(d[0].x - d[2].x, d[0].y - d[2].y);
        tmp[1][x] = make_float2(d[1].x + d[2].x, d[1].y + d[2].y);
        tmp[2][x] = make_float2(d[2].x - d[1].x, d[2].y - d[1].y);
        tmp[3][x] = make_float2(d[1].x - d[3].x, d[1].y - d[3].y);
      }
    }
    float* vb = smem + (2 + buf) * WG_CHUNK + lt * WG_KC + 2 * cp;
    const int xi = q >> 1;
    const float2* t = tmp[xi];
    if ((q & 1) == 0) {
      *reinterpret_cast<float2*>(vb + (xi * 4 + 0) * WG_PLANE) = make_float2(t[0].x - t[2].x, t[0].y - t[2].y);
      *reinterpret_cast<float2*>(vb + (xi * 4 + 1) * WG_PLANE) = make_float2(t[1].x + t[2].x, t[1].y + t[2].y);
    } else {
      *reinterpret_cast<float2*>(vb + (xi * 4 + 2) * WG_PLANE) = make_float2(t[2].x - t[1].x, t[2].y - t[1].y);
      *reinterpret_cast<float2*>(vb + (xi * 4 + 3) * WG_PLANE) = make_float2(t[1].x - t[3].x, t[1].y - t[3].y);
    }
  };

  // accumulators: position p x tile group g (16 tiles) of 16 channels; lane (li, lq) holds
  // channels 4 lq .. 4 lq + 3 of tile li
  f32x4 acc[16][2];
  // one K chunk: per position one A read and two B reads (float2 = the lane's 2 channels of the
  // chunk: k group lq holds channels 2 lq, 2 lq + 1), 4 MFMAs; operands of position p + 1 are read
  // while the MFMAs of position p run; loader threads store the next chunk's V over the second half
  // chunk s: MFMAs on LDS buffer s & 1.  U waves: the LDS-DMA of U(s + 1) into the other buffer is
  // issued first and retired (vmcnt(0)) before the closing barrier.  Loader waves: V(s + 1) is
  // transformed from the window registers over the last quarter of the MFMA stream, then the window
  // of step s + 2 is loaded; those loads stay in flight across the barrier (the loader waves'
  // barrier waits on LDS only) and have a whole chunk to land.
  auto chunk = [&](int s) {
    const int buf = s & 1;
    const bool more = s + 1 < nsteps;
    if (!loader && more) load_u(s + 1);
    const float* Ub = smem + buf * WG_CHUNK + (cq * 16 + li) * WG_KC + 2 * lq;
    const float* Vb = smem + (2 + buf) * WG_CHUNK + (th * 32 + li) * WG_KC + 2 * lq;
    float2 av = *reinterpret_cast<const float2*>(Ub);
    float2 b0 = *reinterpret_cast<const float2*>(Vb);
    float2 b1 = *reinterpret_cast<const float2*>(Vb + 16 * WG_KC);
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      float2 an = av, n0 = b0, n1 = b1;
      if (p < 15) {
        an = *reinterpret_cast<const float2*>(Ub + (p + 1) * WG_PLANE);
        n0 = *reinterpret_cast<const float2*>(Vb + (p + 1) * WG_PLANE);
        n1 = *reinterpret_cast<const float2*>(Vb + (p + 1) * WG_PLANE + 16 * WG_KC);
      }
      if (!(DBG & 1)) {
        acc[p][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, b0.x, acc[p][0], 0, 0, 0);
        acc[p][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, b1.x, acc[p][1], 0, 0, 0);
        acc[p][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, b0.y, acc[p][0], 0, 0, 0);
        acc[p][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, b1.y, acc[p][1], 0, 0, 0);
      } else {
        acc[p][0][0] += av.x * b0.x + av.y * b1.y;
      }
      // the window loads were issued at the top of the chunk: their stores wait for the last
      // quarter of the MFMA stream
      if (loader && p >= 12 && more && !(DBG & 4)) {
        store_piece(buf ^ 1, 2 * (p - 12));
        store_piece(buf ^ 1, 2 * (p - 12) + 1);
      }
      av = an;
      b0 = n0;
      b1 = n1;
    }
    if (loader && s + 2 < nsteps && !(DBG & 2)) load_window(s + 2);
    // U waves: the LDS-DMA of the next U chunk has landed; all: every wave is done with this buffer
    if (!loader) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
  };

  if (loader) {
    load_window(0);
#pragma unroll
    for (int q = 0; q < 8; ++q) store_piece(0, q);
    if (nsteps > 1) load_window(1);
  } else {
    load_u(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  lds_barrier();

  int s = 0;
  for (int unit = 0; unit < nunits; ++unit) {
#pragma unroll
    for (int p = 0; p < 16; ++p) acc[p][0] = acc[p][1] = f32x4{};
    for (int k = 0; k < a.nk; ++k, ++s) chunk(s);

    // Y = A^T M A per channel, + bias (+ residual), ReLU; per tile group: 4 pixels x 4 channels,
    // one 16-byte store per pixel
    const int co0 = cb * WG_COUT + cq * 16 + 4 * lq;
    const float4 b4 = *reinterpret_cast<const float4*>(a.bias + co0);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int t_out = (r + unit * per_cb) * WG_TILES + th * 32 + g * 16 + li;
      const bool t_ok = t_out < a.ntiles;
      int oimg, oty, otx;
      tile_pos(t_ok ? t_out : a.ntiles - 1, oimg, oty, otx);
      int off[4];
      bool pok[4];
      float4 rv[4];
#pragma unroll
      for (int px = 0; px < 4; ++px) {
        const int y = 2 * oty + (px >> 1), x = 2 * otx + (px & 1);
        pok[px] = t_ok && y < a.H && x < a.W;
        off[px] = pok[px] ? ((oimg * a.H + y) * a.W + x) * a.C + co0 : 0;
        if (a.res) rv[px] = *reinterpret_cast<const float4*>(a.res + off[px]);
      }
      float o[4][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t0[4], t1[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          t0[x] = acc[x][g][e] + acc[4 + x][g][e] + acc[8 + x][g][e];
          t1[x] = acc[4 + x][g][e] - acc[8 + x][g][e] - acc[12 + x][g][e];
        }
        const float bj = e == 0 ? b4.x : e == 1 ? b4.y : e == 2 ? b4.z : b4.w;
        o[0][e] = t0[0] + t0[1] + t0[2] + bj;
        o[1][e] = t0[1] - t0[2] - t0[3] + bj;
        o[2][e] = t1[0] + t1[1] + t1[2] + bj;
        o[3][e] = t1[1] - t1[2] - t1[3] + bj;
      }
#pragma unroll
      for (int px = 0; px < 4; ++px) {
        if (a.res) {
          o[px][0] += rv[px].x;
          o[px][1] += rv[px].y;
          o[px][2] += rv[px].z;
          o[px][3] += rv[px].w;
        }
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[px][e] = o[px][e] > 0.f ? o[px][e] : (o[px][e] != o[px][e] ? o[px][e] : 0.f);
        }
        if (pok[px]) *reinterpret_cast<float4*>(a.out + off[px]) = make_float4(o[px][0], o[px][1], o[px][2], o[px][3]);
      }
    }
  }
}

// =============================================================================================
// Winograd F(4x4, 3x3): 36 positions per 6x6 input window / 4x4 output tile = 2.25 products per
// output (F(2x2, 3x3): 4), points {0, +-1, +-2, inf}:
//   V = B^T d B (input, exact small-integer coefficients), U = G g G^T (packed once on the host in
//   f64 -> f32; G holds 1/4, 1/6, 1/12, 1/24), M[p] = sum_c U[p][co][c] V[p][c][tile],
//   Y = A^T M A (coefficients 0, +-1, +-2, 4, +-8).
// Mapping: a block = 8 waves owns 64 output channels x 32 tiles (512 output pixels); wave (cq, tg)
// keeps 16 channels x 16 tiles for all 36 positions in 36 accumulators (144 registers), one
// v_mfma_f32_16x16x4_f32 per position per K chunk of 4 input channels.  U (36 KiB per chunk,
// pre-packed LDS image) is moved by LDS-DMA from waves 4-7.  The windows (32 tiles x 4 channels
// per chunk, one whole 6x6 window per thread) are gathered and transformed by two loader groups
// (waves 0-1 and 2-3) that alternate chunks: group c & 1 issues the window loads of chunk c after
// its MFMA stream of chunk c - 2 (they stay in flight across the LDS-only barrier) and transforms
// them into V buffer c & 1 under the second half of the MFMA stream of chunk c - 1: B^T down the
// six columns in registers, then along the six rows with the LDS stores.  (Measured slower: the
// column and row passes split over two chunks so both groups transform in every chunk on
// complementary SIMDs, with the loads issued mid-stream -- 6.42 vs 5.71 ms at 512 channels; four
// groups including the U waves, 6.90 ms.)
// LDS: U and V double buffered, 108 KiB.  Persistent blocks and the per-XCD output-channel block
// as F(2x2).  Measured slower in round 4 (profiles/r4_wino4_padded_lds_ab.log,
// r4_wino4_producer_consumer_ab.log): bank-conflict-free padded U / V images (64 ch 8.17 vs 7.66
// ms: 33 % more U DMA per chunk, 150 KiB of LDS) and a 12-wave producer / consumer split (8 MFMA-only
// waves, 4 waves moving U and transforming the windows; 1.26-1.36x slower, bit-identical: at 3 waves
// per SIMD the 168-register budget spills the consumers and the U DMA of a chunk, issued by two
// waves, lands too late for the barrier that publishes it).
// =============================================================================================
__device__ float g_wino_zero[4];  // zero-initialised: the pixels outside the image
constexpr int W4_TILES = 32;
constexpr int W4_COUT = 64;
constexpr int W4_KC = 4;
constexpr int W4_UCH = 36 * W4_COUT * W4_KC;   // 9216 floats
constexpr int W4_VCH = 36 * W4_TILES * W4_KC;  // 4608 floats
constexpr int W4_DEFAULT_VAR = 0;
static_assert((2 * W4_UCH + 2 * W4_VCH) * 4 <= 160 * 1024, "W4 LDS");

// VAR bits: 1 = SPLIT schedule (above), 2 = the window loads of chunk c + 2 issued before (not
// after) the MFMA stream of chunk c, 4 = LDS operands prefetched 4 positions ahead, 16 = window
// gathers as buffer loads whose out-of-image pixels read 0 through the descriptor's range check
// (voffset past the end), the window column and the K chunk in the scalar offset: one v_or per
// pixel instead of a 64-bit address select.  Measured (profiles/r3_winograd4_variants.log): 6
// best at 64 / 128 channels, 16 at 256 / 512 (6 | 16 spills); position-quad LDS images (one
// ds_read_b128 per operand feeding 4 MFMAs) no faster than 6, and a one-wave-per-SIMD kernel
// (4 waves, accumulators in AGPRs) slower at every shape: its U waits also wait for the window
// gathers issued before them (vmcnt is in order), which the 8-wave split keeps in other waves
template <int DBG, int VAR>
__global__ void __launch_bounds__(WG_THREADS, 1) wino4_f32_kernel(WinoArgs a) {
  constexpr int SPLIT = VAR & 1;
  constexpr bool EARLY = (VAR & 2) != 0;
  constexpr bool DEEP = (VAR & 4) != 0;
  constexpr bool BUF = (VAR & 16) != 0;
  __shared__ __attribute__((aligned(16))) float smem[2 * W4_UCH + 2 * W4_VCH];  // sU[2], sV[2]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cq = wave & 3, tg = wave >> 2;
  const int li = lane & 15, lq = lane >> 4;
  const bool loader = wave < 4;  // waves 0-3: window loaders, waves 4-7: U LDS-DMA
  const int lgrp = wave >> 1;    // loader group: chunks c with c & 1 == lgrp

  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7;
  const int cb = xcd % a.ncb;
  const int per_cb = G / a.ncb;
  const int r = (blockIdx.x >> 3) * (8 / a.ncb) + xcd / a.ncb;
  if (r >= a.ntb) return;
  const int nunits = (a.ntb - r + per_cb - 1) / per_cb;
  const int nsteps = nunits << a.nk_log2;

  // loader thread: window of tile lt (0..31), channel lc (0..3) of the chunk; out-of-image pixels
  // read a device zero, so the transform needs no mask (measured slower: buffer loads with the
  // in-image mask applied in the column pass, 9.2 vs 8.1 ms at 64 channels)
  const int lt = (tid & 127) >> 2, lc = tid & 3;
  float xr[36];
  uint32_t ld_mlo = 0, ld_mhi = 0;  // in-image bits of the 36 window pixels
  int ld_unit = -1, ld_o0 = 0;
  auto tile_pos = [&](int t, int& img, int& ty, int& tx) {
    const int q = t / a.tiles_x;
    tx = t - q * a.tiles_x;
    img = q / a.tiles_y;
    ty = q - img * a.tiles_y;
  };
  auto load_u = [&](int s) {  // U waves: 9 KiB each as 9 lane-linear 1-KiB LDS-DMA pieces
    const int k = s & (a.nk - 1);
    const float* ug = a.u + ((size_t)cb * a.nk + k) * W4_UCH + (wave - 4) * 2304 + lane * 4;
    float* ul = smem + (s & 1) * W4_UCH + (wave - 4) * 2304;
    if (!(DBG & 8))
#pragma unroll
      for (int j = 0; j < 9; ++j) glds16(ug + 256 * j, ul + 256 * j);
  };
  // BUF: descriptor based one pixel before the input, so a window's first column (x0 = -1) has a
  // non-negative voffset; a pixel outside the image gets a voffset past the end (reads 0)
  const __amdgpu_buffer_rsrc_t in_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.in - a.C), 0, (int)(((long long)a.N * a.H * a.W * a.C + a.C) * 4), 0x00020000);
  constexpr uint32_t W4_PAST_END = 0xfffffff0u;
  uint32_t ld_base = 0;  // byte offset of pixel (y0, x0) (descriptor based one pixel early)
  uint32_t ld_ok = 0;    // bits 0-5: window row y in the image, bits 8-13: column x
  auto load_window_buf = [&](int s) {
    const int unit = s >> a.nk_log2;
    const int k = s & (a.nk - 1);
    if (unit != ld_unit) {
      ld_unit = unit;
      const int t = (r + unit * per_cb) * W4_TILES + lt;
      const bool tok = t < a.ntiles;
      int img, ty, tx;
      tile_pos(tok ? t : a.ntiles - 1, img, ty, tx);
      const int y0 = 4 * ty - 1, x0 = 4 * tx - 1;
      ld_base = (uint32_t)(((img * a.H + y0) * a.W + x0 + 1) * a.C + lc) * 4u;
      ld_ok = 0;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        ld_ok |= (uint32_t)(tok && y0 + j >= 0 && y0 + j < a.H) << j;
        ld_ok |= (uint32_t)(x0 + j >= 0 && x0 + j < a.W) << (8 + j);
      }
    }
    const int row_bytes = __builtin_amdgcn_readfirstlane(a.W * a.C * 4);
    uint32_t rv[6];  // row y's voffset, or past the end
#pragma unroll
    for (int y = 0; y < 6; ++y) rv[y] = (ld_base + y * row_bytes) | (((ld_ok >> y) & 1u) ? 0u : W4_PAST_END);
#pragma unroll
    for (int x = 0; x < 6; ++x) {
      const int soff = __builtin_amdgcn_readfirstlane((x * a.C + k * W4_KC) * 4);
      const uint32_t cmask = ((ld_ok >> (8 + x)) & 1u) ? 0u : W4_PAST_END;  // OR-ed in: past the end
#pragma unroll
      for (int y = 0; y < 6; ++y)
        xr[6 * y + x] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(in_rsrc, rv[y] | cmask, soff, 0));
    }
  };
  auto load_window = [&](int s) {
    if (DBG & 2) return;
    if (BUF) {
      load_window_buf(s);
      return;
    }
    const int unit = s >> a.nk_log2;
    const int k = s & (a.nk - 1);
    if (unit != ld_unit) {
      ld_unit = unit;
      const int t = (r + unit * per_cb) * W4_TILES + lt;
      const bool tok = t < a.ntiles;
      int img, ty, tx;
      tile_pos(tok ? t : a.ntiles - 1, img, ty, tx);
      const int y0 = 4 * ty - 1, x0 = 4 * tx - 1;
      ld_o0 = ((img * a.H + y0) * a.W + x0) * a.C + lc;
      ld_mlo = ld_mhi = 0;
#pragma unroll
      for (int i = 0; i < 36; ++i) {
        const int y = y0 + i / 6, x = x0 + i % 6;
        const uint32_t bit = (uint32_t)(tok && y >= 0 && y < a.H && x >= 0 && x < a.W);
        if (i < 32)
          ld_mlo |= bit << i;
        else
          ld_mhi |= bit << (i - 32);
      }
    }
    const float* base = a.in + ld_o0 + k * W4_KC;
#pragma unroll
    for (int i = 0; i < 36; ++i) {
      const uint32_t bit = i < 32 ? (ld_mlo >> i) & 1u : (ld_mhi >> (i - 32)) & 1u;
      const float* src = bit ? base + ((i / 6) * a.W + (i % 6)) * a.C : &g_wino_zero[0];
      xr[i] = *src;
    }
  };
  auto bt6 = [](float d0, float d1, float d2, float d3, float d4, float d5, float* v) {
    v[0] = 4.f * d0 - 5.f * d2 + d4;
    v[1] = (d3 + d4) - 4.f * (d1 + d2);
    v[2] = (d4 - d3) + 4.f * (d1 - d2);
    v[3] = (d4 - d2) + 2.f * (d3 - d1);
    v[4] = (d4 - d2) - 2.f * (d3 - d1);
    v[5] = 4.f * d1 - 5.f * d3 + d5;
  };
  auto col_piece = [&](int x) {  // B^T down window column x, in place
    if (DBG & 4) return;
    float v[6];
    bt6(xr[x], xr[6 + x], xr[12 + x], xr[18 + x], xr[24 + x], xr[30 + x], v);
#pragma unroll
    for (int y = 0; y < 6; ++y) xr[6 * y + x] = v[y];
  };
  auto row_piece = [&](int buf, int y) {  // B^T along row y, stored as positions 6 y .. 6 y + 5
    if (DBG & 4) return;
    float v[6];
    bt6(xr[6 * y], xr[6 * y + 1], xr[6 * y + 2], xr[6 * y + 3], xr[6 * y + 4], xr[6 * y + 5], v);
    float* vb = smem + 2 * W4_UCH + buf * W4_VCH + lt * W4_KC + lc;
#pragma unroll
    for (int x = 0; x < 6; ++x) vb[(6 * y + x) * (W4_TILES * W4_KC)] = v[x];
  };

  f32x4 acc[36];
  auto chunk = [&](int c) {
    const int buf = c & 1;
    const bool more = c + 1 < nsteps;
    if (!loader && more) load_u(c + 1);
    const bool tf = loader && lgrp == ((c + 1) & 1) && c + 1 < nsteps;  // V(c + 1) -> other buffer
    const bool cols2 = SPLIT && loader && lgrp == (c & 1) && c + 2 < nsteps;  // SPLIT: columns of V(c + 2)
    const float* Ub = smem + buf * W4_UCH + cq * 64 + li * 4 + lq;
    const float* Vb = smem + 2 * W4_UCH + buf * W4_VCH + tg * 64 + li * 4 + lq;
    if (!SPLIT && EARLY && loader && lgrp == (c & 1) && c + 2 < nsteps) load_window(c + 2);
    constexpr int PD = DEEP ? 4 : 1;  // operand prefetch distance (positions)
    float ar[PD], br[PD];
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      ar[j] = Ub[j * (W4_COUT * W4_KC)];
      br[j] = Vb[j * (W4_TILES * W4_KC)];
    }
#pragma unroll
    for (int p = 0; p < 36; ++p) {
      const float av = ar[p % PD], bv = br[p % PD];
      if (p + PD < 36) {
        ar[p % PD] = Ub[(p + PD) * (W4_COUT * W4_KC)];
        br[p % PD] = Vb[(p + PD) * (W4_TILES * W4_KC)];
      }
      if (!(DBG & 1))
        acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[p], 0, 0, 0);
      else
        acc[p][0] += av * bv;
      if (!SPLIT) {
        if (tf && p >= 8 && p <= 18 && (p & 1) == 0) col_piece((p - 8) >> 1);
        if (tf && p >= 20 && (p - 20) % 3 == 0) row_piece(buf ^ 1, (p - 20) / 3);
      } else {
        // rows of V(c + 1) over the first half, columns of V(c + 2) over the second
        if (tf && p >= 2 && p <= 17 && (p - 2) % 3 == 0) row_piece(buf ^ 1, (p - 2) / 3);
        if (cols2 && p >= 20 && (p - 20) % 3 == 0) col_piece((p - 20) / 3);
      }
    }
    if (!SPLIT && !EARLY && loader && lgrp == (c & 1) && c + 2 < nsteps) load_window(c + 2);
    if (SPLIT && tf && c + 3 < nsteps) load_window(c + 3);  // the group's next window
    // U waves: the LDS-DMA of U(c + 1) has landed (loader waves keep their window loads in flight
    // across the LDS-only barrier)
    if (!loader) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
  };

  // prologue: U(0); V(0) complete (group 0); the window of chunk 1 in flight (group 1)
  if (!loader) {
    load_u(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (lgrp < nsteps) {
    load_window(lgrp);
    if (lgrp == 0) {
#pragma unroll
      for (int x = 0; x < 6; ++x) col_piece(x);
#pragma unroll
      for (int y = 0; y < 6; ++y) row_piece(0, y);
      if (SPLIT && nsteps > 2) load_window(2);
    } else if (SPLIT) {
#pragma unroll
      for (int x = 0; x < 6; ++x) col_piece(x);
    }
  }
  lds_barrier();

  int s = 0;
  for (int unit = 0; unit < nunits; ++unit) {
#pragma unroll
    for (int p = 0; p < 36; ++p) acc[p] = f32x4{};
    for (int k = 0; k < a.nk; ++k, ++s) chunk(s);

    // Y = A^T M A (+ bias, + residual, ReLU): lane (li, lq) finishes channels 4 lq .. 4 lq + 3 of
    // tile li of its group, output row by row: 16 pixels, one 16-byte store each
    const int co0 = cb * W4_COUT + cq * 16 + 4 * lq;
    const float4 b4 = *reinterpret_cast<const float4*>(a.bias + co0);
    const int t_out = (r + unit * per_cb) * W4_TILES + tg * 16 + li;
    const bool t_ok = t_out < a.ntiles;
    int oimg, oty, otx;
    tile_pos(t_ok ? t_out : a.ntiles - 1, oimg, oty, otx);
    // row by row (output row i of the tile): t_i = (A^T M)[i] per channel, then its 4 pixels
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float y[4][4];  // [pixel q][channel e]
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t[6];
#pragma unroll
        for (int x = 0; x < 6; ++x) {
          const float m0 = acc[x][e], m1 = acc[6 + x][e], m2 = acc[12 + x][e], m3 = acc[18 + x][e],
                      m4 = acc[24 + x][e], m5 = acc[30 + x][e];
          const float s12 = m1 + m2, d12 = m1 - m2, s34 = m3 + m4, d34 = m3 - m4;
          t[x] = i == 0 ? m0 + s12 + s34 : i == 1 ? d12 + 2.f * d34 : i == 2 ? s12 + 4.f * s34 : d12 + 8.f * d34 + m5;
        }
        const float bj = e == 0 ? b4.x : e == 1 ? b4.y : e == 2 ? b4.z : b4.w;
        const float s12 = t[1] + t[2], d12 = t[1] - t[2], s34 = t[3] + t[4], d34 = t[3] - t[4];
        y[0][e] = t[0] + s12 + s34 + bj;
        y[1][e] = d12 + 2.f * d34 + bj;
        y[2][e] = s12 + 4.f * s34 + bj;
        y[3][e] = d12 + 8.f * d34 + t[5] + bj;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int yy = 4 * oty + i, xx = 4 * otx + q;
        const bool ok = t_ok && yy < a.H && xx < a.W;
        const int off = ok ? ((oimg * a.H + yy) * a.W + xx) * a.C + co0 : 0;
        float o0 = y[q][0], o1 = y[q][1], o2 = y[q][2], o3 = y[q][3];
        if (a.res) {
          const float4 rv = *reinterpret_cast<const float4*>(a.res + off);
          o0 += rv.x;
          o1 += rv.y;
          o2 += rv.z;
          o3 += rv.w;
        }
        if (a.relu) {
          o0 = o0 > 0.f ? o0 : (o0 != o0 ? o0 : 0.f);
          o1 = o1 > 0.f ? o1 : (o1 != o1 ? o1 : 0.f);
          o2 = o2 > 0.f ? o2 : (o2 != o2 ? o2 : 0.f);
          o3 = o3 > 0.f ? o3 : (o3 != o3 ? o3 : 0.f);
        }
        if (ok) *reinterpret_cast<float4*>(a.out + off) = make_float4(o0, o1, o2, o3);
      }
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

extern "C" int rmbx_conv3x3_winograd_f32(const float* in, const float* u_packed, const float* bias,
                                         const float* residual, float* out, int N, int H, int W, int C,
                                         int relu, void* stream) {
  RMBX_CHECK_ARG(in && u_packed && bias && out, "rmbx_conv3x3_winograd_f32: null pointer");
  RMBX_CHECK_ARG(N >= 0 && H > 0 && W > 0, "rmbx_conv3x3_winograd_f32: bad geometry");
  RMBX_CHECK_ARG(C == 64 || C == 128 || C == 256 || C == 512,
                 "rmbx_conv3x3_winograd_f32: C=%d (implemented: 64, 128, 256, 512)", C);
  RMBX_CHECK_ARG((((uintptr_t)in | (uintptr_t)u_packed | (uintptr_t)out | (uintptr_t)residual) & 15) == 0,
                 "rmbx_conv3x3_winograd_f32: tensors must be 16-byte aligned");
  RMBX_CHECK_ARG(in != out && (residual == nullptr || residual != out),
                 "rmbx_conv3x3_winograd_f32: the output must not alias the input or the residual");
  if (N == 0) return RMBX_OK;
  rmbx::WinoArgs a;
  a.in = in;
  a.u = u_packed;
  a.bias = bias;
  a.res = residual;
  a.out = out;
  a.N = N;
  a.H = H;
  a.W = W;
  a.C = C;
  a.relu = relu;
  a.tiles_x = (W + 1) / 2;
  a.tiles_y = (H + 1) / 2;
  const long long ntiles = (long long)N * a.tiles_x * a.tiles_y;
  RMBX_CHECK_ARG(ntiles + rmbx::WG_TILES < (1ll << 31) && (long long)N * H * W * C < (1ll << 31),
                 "rmbx_conv3x3_winograd_f32: tensor too large for 32-bit element offsets");
  a.ntiles = (int)ntiles;
  a.ntb = (a.ntiles + rmbx::WG_TILES - 1) / rmbx::WG_TILES;
  a.ncb = C / rmbx::WG_COUT;
  a.nk = C / rmbx::WG_KC;
  const char* stg_env = std::getenv("RMBX_WINO_STAGGER");
  // measured: 8.59 -> 8.40 ms at 64 channels (8 chunks per unit), no effect at 128-512 channels
  a.stagger = stg_env ? std::atoi(stg_env) : (C == 64 ? 2 : 0);
  const char* dbg_env = std::getenv("RMBX_WINO_DBG");
  a.dbg = dbg_env ? std::atoi(dbg_env) : 0;
  a.nk_log2 = 0;
  while ((1 << a.nk_log2) < a.nk) ++a.nk_log2;
  // one persistent block per CU (grid a multiple of 8: blockIdx % 8 is the XCD under round-robin
  // dispatch); blocks beyond the work exit at once
  int grid = rmbx::device_cus();
  grid = grid < 8 ? 8 : grid - grid % 8;
  const dim3 g(grid), blk(rmbx::WG_THREADS);
  hipStream_t st = (hipStream_t)stream;
  switch (a.dbg) {
    case 0: hipLaunchKernelGGL(rmbx::wino_f32_kernel<0>, g, blk, 0, st, a); break;
    case 1: hipLaunchKernelGGL(rmbx::wino_f32_kernel<1>, g, blk, 0, st, a); break;
    case 2: hipLaunchKernelGGL(rmbx::wino_f32_kernel<2>, g, blk, 0, st, a); break;
    case 4: hipLaunchKernelGGL(rmbx::wino_f32_kernel<4>, g, blk, 0, st, a); break;
    case 6: hipLaunchKernelGGL(rmbx::wino_f32_kernel<6>, g, blk, 0, st, a); break;
    case 8: hipLaunchKernelGGL(rmbx::wino_f32_kernel<8>, g, blk, 0, st, a); break;
    case 14: hipLaunchKernelGGL(rmbx::wino_f32_kernel<14>, g, blk, 0, st, a); break;
    case 15: hipLaunchKernelGGL(rmbx::wino_f32_kernel<15>, g, blk, 0, st, a); break;
    default: RMBX_CHECK_ARG(false, "rmbx_conv3x3_winograd_f32: RMBX_WINO_DBG=%d not instantiated", a.dbg);
  }
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_conv3x3_winograd4_f32(const float* in, const float* u_packed, const float* bias,
                                          const float* residual, float* out, int N, int H, int W, int C,
                                          int relu, void* stream) {
  RMBX_CHECK_ARG(in && u_packed && bias && out, "rmbx_conv3x3_winograd4_f32: null pointer");
  RMBX_CHECK_ARG(N >= 0 && H > 0 && W > 0, "rmbx_conv3x3_winograd4_f32: bad geometry");
  RMBX_CHECK_ARG(C == 64 || C == 128 || C == 256 || C == 512,
                 "rmbx_conv3x3_winograd4_f32: C=%d (implemented: 64, 128, 256, 512)", C);
  RMBX_CHECK_ARG((((uintptr_t)in | (uintptr_t)u_packed | (uintptr_t)out | (uintptr_t)residual) & 15) == 0,
                 "rmbx_conv3x3_winograd4_f32: tensors must be 16-byte aligned");
  RMBX_CHECK_ARG(in != out && (residual == nullptr || residual != out),
                 "rmbx_conv3x3_winograd4_f32: the output must not alias the input or the residual");
  if (N == 0) return RMBX_OK;
  rmbx::WinoArgs a;
  a.in = in;
  a.u = u_packed;
  a.bias = bias;
  a.res = residual;
  a.out = out;
  a.N = N;
  a.H = H;
  a.W = W;
  a.C = C;
  a.relu = relu;
  a.tiles_x = (W + 3) / 4;
  a.tiles_y = (H + 3) / 4;
  const long long ntiles = (long long)N * a.tiles_x * a.tiles_y;
  // 32-bit byte offsets, and the buffer descriptor's range (one pixel more, below a past-the-end
  // voffset of 2^32 - 16): at most 2^30 - 1024 elements per launch (kernels.WINOGRAD4_MAX_ELEMS)
  RMBX_CHECK_ARG(ntiles + rmbx::W4_TILES < (1ll << 31) && (long long)N * H * W * C <= (1ll << 30) - 1024,
                 "rmbx_conv3x3_winograd4_f32: tensor too large for 32-bit byte offsets");
  a.ntiles = (int)ntiles;
  a.ntb = (a.ntiles + rmbx::W4_TILES - 1) / rmbx::W4_TILES;
  a.ncb = C / rmbx::W4_COUT;
  a.nk = C / rmbx::W4_KC;
  a.stagger = 0;
  const char* dbg_env = std::getenv("RMBX_WINO_DBG");
  a.dbg = dbg_env ? std::atoi(dbg_env) : 0;
  a.nk_log2 = 0;
  while ((1 << a.nk_log2) < a.nk) ++a.nk_log2;
  int grid = rmbx::device_cus();
  grid = grid < 8 ? 8 : grid - grid % 8;
  const dim3 g(grid), blk(rmbx::WG_THREADS);
  hipStream_t st = (hipStream_t)stream;
  // schedule variant (RMBX_WINO4_VAR, wino4_f32_kernel's VAR bits); the phase-skip builds
  // (RMBX_WINO_DBG) exist for the default only
  // default by channel count (scripts/prof_winograd4.py, profiles/r3_winograd4_variants.log):
  // early window loads + deep LDS prefetch (6) at 64 / 128 channels, buffer-load window gathers
  // (16) at 256 / 512
  const char* var_env = std::getenv("RMBX_WINO4_VAR");
  const int var = var_env ? std::atoi(var_env) : (C >= 256 ? 16 : 6);
  RMBX_CHECK_ARG(a.dbg == 0 || var == rmbx::W4_DEFAULT_VAR,
                 "rmbx_conv3x3_winograd4_f32: RMBX_WINO_DBG needs RMBX_WINO4_VAR=%d", rmbx::W4_DEFAULT_VAR);
#define RMBX_W4_LAUNCH(D, V) hipLaunchKernelGGL((rmbx::wino4_f32_kernel<D, V>), g, blk, 0, st, a)
  if (a.dbg == 0) {
    switch (var) {
      case 0: RMBX_W4_LAUNCH(0, 0); break;
      case 1: RMBX_W4_LAUNCH(0, 1); break;
      case 2: RMBX_W4_LAUNCH(0, 2); break;
      case 4: RMBX_W4_LAUNCH(0, 4); break;
      case 6: RMBX_W4_LAUNCH(0, 6); break;
      case 16: RMBX_W4_LAUNCH(0, 16); break;
      default: RMBX_CHECK_ARG(false, "rmbx_conv3x3_winograd4_f32: RMBX_WINO4_VAR=%d not instantiated", var);
    }
  } else {
    switch (a.dbg) {
      case 1: RMBX_W4_LAUNCH(1, rmbx::W4_DEFAULT_VAR); break;
      case 2: RMBX_W4_LAUNCH(2, rmbx::W4_DEFAULT_VAR); break;
      case 4: RMBX_W4_LAUNCH(4, rmbx::W4_DEFAULT_VAR); break;
      case 8: RMBX_W4_LAUNCH(8, rmbx::W4_DEFAULT_VAR); break;
      case 14: RMBX_W4_LAUNCH(14, rmbx::W4_DEFAULT_VAR); break;
      default: RMBX_CHECK_ARG(false, "rmbx_conv3x3_winograd4_f32: RMBX_WINO_DBG=%d not instantiated", a.dbg);
    }
  }
#undef RMBX_W4_LAUNCH
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
