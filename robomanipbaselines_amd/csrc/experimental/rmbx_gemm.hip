// Dense bf16 linear layer for the ACT transformer: out[M][N] = act(x[M][K] . W[N][K]^T + bias[N]),
// f32 accumulation on MFMA 32x32x16 (gfx950), bf16 out.  Replaces the nn.Linear / MHA in_proj /
// out_proj / FFN GEMMs of ACT's transformer (third_party/act detr/models/transformer.py [absent];
// layer sizes policy/act/TrainAct.py:46-58: d 512, ff 3200) and their ReLU (fused, FFN1).
//
// Both operands are K-contiguous (nn.Linear layout), so both MFMA operands load as 16-byte rows.
// Block tile 256 x 256, BK = 64, 8 waves; global -> LDS by global_load_lds (16 B per lane, the
// DMA writes lane-linear LDS), two LDS stages so the next K tile streams in while the current one
// is multiplied.  The LDS image of a tile is [row][8 chunks of 16 B] with chunk c stored at
// c ^ ((row >> 1) & 7): the XOR is applied to the per-lane GLOBAL source address (the DMA
// destination cannot scatter), and it makes every ds_read_b128 lane group of the fragment reads
// hit 16 distinct bank quads.
//
// The product is computed transposed, C^T = W . x^T, with the W rows of each 32-row MFMA tile
// permuted (row i -> 16((i>>2)&1) + (i&3) + 4(i>>3)) so that accumulator register j of lane-half
// h holds output column 16h + j: every lane finishes 16 consecutive columns of one output row
// and writes them as two 16-byte stores (no LDS round trip in the epilogue).  Blocks are
// remapped so each XCD walks a contiguous range of (row tile, column tile) pairs, column tile
// fastest: an x row tile is read from HBM once per XCD and W stays L2-resident.

#include "rmbx_common.h"

#include <cstdint>
#include <cstdlib>

namespace rmbx {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int GBM = 256, GBN = 256, GBK = 64, GTHREADS = 512;
constexpr int G_TILE_BYTES = GBM * GBK * 2;  // 32 KiB per operand per stage

struct GemmArgs {
  const uint16_t* x;   // [M][K]
  const uint16_t* w;   // [N][K]
  const float* bias;   // [N] or null
  uint16_t* out;       // [M][N] (row stride ldo)
  int M, N, K, ldo, relu;
  int tiles_m, tiles_n;
  int dbg;  // diagnostic phase skips (RMBX_GEMM_DBG; 0 in production): 1 no K-loop DMA, 2 no MFMA
};

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// one operand tile (256 rows x 64 k) of K step kt into LDS: 4 glds per lane
__device__ __forceinline__ void load_tile(const uint16_t* src, int rows_total, int row0, int K, int k0,
                                          uint8_t* lds_tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = (wave * 4 + i) * 64 + lane;  // 16-byte chunk position in the tile image
    const int row = p >> 3, phys = p & 7;
    const int c = phys ^ ((row >> 1) & 7);
    const int grow = min(row0 + row, rows_total - 1);  // tail rows: any valid row, result unused
    const uint16_t* g = src + (size_t)grow * K + k0 + c * 8;
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(lds_tile + (wave * 4 + i) * 1024), 16, 0, 0);
  }
}

// epilogue of one 256 x 256 tile: lane (kh, r32) owns output rows m0+wm+32u+r32 and columns
// n0+wn+32t+16kh .. +15 (16 consecutive values -> two 16-byte stores per (t, u))
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& a, f32x16 (&acc)[2][4], int m0, int n0, int wm, int wn,
                                              int kh, int r32) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ncol = n0 + wn + 32 * t + 16 * kh;
    if (ncol >= a.N) continue;
    float bv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) bv[j] = 0.f;
    if (a.bias) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 b4 = *reinterpret_cast<const float4*>(a.bias + ncol + 4 * q);
        bv[4 * q] = b4.x;
        bv[4 * q + 1] = b4.y;
        bv[4 * q + 2] = b4.z;
        bv[4 * q + 3] = b4.w;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = m0 + wm + 32 * u + r32;
      if (row >= a.M) continue;
      uint32_t pk[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        f32x2 v;
        v[0] = acc[t][u][2 * q] + bv[2 * q];
        v[1] = acc[t][u][2 * q + 1] + bv[2 * q + 1];
        if (a.relu) {
          v[0] = v[0] > 0.f ? v[0] : 0.f;
          v[1] = v[1] > 0.f ? v[1] : 0.f;
        }
        pk[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
      }
      uint16_t* dst = a.out + (size_t)row * a.ldo + ncol;
      *reinterpret_cast<uint4*>(dst) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
      *reinterpret_cast<uint4*>(dst + 8) = make_uint4(pk[4], pk[5], pk[6], pk[7]);
    }
  }
}

// Persistent: one block per CU walks its tiles (strided over its XCD group) as ONE stream of K steps, so
// the DMA of the next tile's first K step is in flight while the current tile finishes, and a
// finished tile's epilogue (stores) overlaps the next tile's first MFMAs.
__global__ void __launch_bounds__(GTHREADS) gemm_bf16_tn_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[4 * G_TILE_BYTES];  // [stage][W, x]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // tile range of this block: each XCD (blocks b = x, x + 8, ...) gets a contiguous share of the
  // tile sequence (column tile fastest), split evenly among its blocks
  const int ntiles = a.tiles_m * a.tiles_n;
  const int nb = gridDim.x;
  const int G = nb < 8 ? nb : 8;  // XCD groups actually populated
  const int xcd = blockIdx.x % G, jx = blockIdx.x / G;
  const int nbx = (nb - xcd + G - 1) / G;  // blocks in this group
  const int xb = (int)((long long)ntiles * xcd / G), xe = (int)((long long)ntiles * (xcd + 1) / G);
  // strided within the group: at any moment the group's blocks work on consecutive tiles, so the
  // column tiles of one x row tile run together and share its L2 copy
  const int t_begin = xb + jx;
  if (t_begin >= xe) return;
  const int my_tiles = (xe - t_begin + nbx - 1) / nbx;
  const int KT = a.K / GBK;
  const int total = my_tiles * KT;

  // wave tile: 64 columns (n) x 128 rows (m): 2 n-tiles x 4 m-tiles of 32 x 32
  const int wn = (wave & 3) * 64, wm = (wave >> 2) * 128;
  const int r32 = lane & 31, kh = lane >> 5;
  const int sig = 16 * ((r32 >> 2) & 1) + (r32 & 3) + 4 * (r32 >> 3);
  int wrow[2], xrow[4];
#pragma unroll
  for (int t = 0; t < 2; ++t) wrow[t] = wn + 32 * t + sig;
#pragma unroll
  for (int u = 0; u < 4; ++u) xrow[u] = wm + 32 * u + r32;

  auto issue = [&](int s) {
    const int tile = t_begin + (s / KT) * nbx, kt = s - (s / KT) * KT;
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    uint8_t* st = smem + (s & 1) * 2 * G_TILE_BYTES;
    load_tile(a.w, a.N, tn * GBN, a.K, kt * GBK, st, wave, lane);
    load_tile(a.x, a.M, tm * GBM, a.K, kt * GBK, st + G_TILE_BYTES, wave, lane);
  };

  f32x16 acc[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[t][u] = f32x16{};

  issue(0);
  __syncthreads();
  for (int s = 0; s < total; ++s) {
    if (s + 1 < total && !(a.dbg & 1)) issue(s + 1);
    const int kt = s % KT;
    if (kt == 0 && s > 0) {
      const int tile = t_begin + (s / KT - 1) * nbx;
      const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
      gemm_epilogue(a, acc, tm * GBM, tn * GBN, wm, wn, kh, r32);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[t][u] = f32x16{};
    }
    const uint8_t* sw = smem + (s & 1) * 2 * G_TILE_BYTES;
    const uint8_t* sx = sw + G_TILE_BYTES;
    __builtin_amdgcn_s_setprio(1);
    if (!(a.dbg & 2)) {
      // fragments double-buffered by k-substep: substep ks + 1's six ds_read_b128 are in flight
      // while substep ks's eight MFMAs issue
      bf16x8 fw[2][2], fx[2][4];
#define RMBX_GEMM_FRAGS(BUF, KS)                                                                                 \
  {                                                                                                              \
    const int c_ = 2 * (KS) + kh;                                                                                \
    _Pragma("unroll") for (int t = 0; t < 2; ++t) fw[BUF][t] =                                                   \
        *reinterpret_cast<const bf16x8*>(sw + wrow[t] * 128 + swz(wrow[t], c_) * 16);                            \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) fx[BUF][u] =                                                   \
        *reinterpret_cast<const bf16x8*>(sx + xrow[u] * 128 + swz(xrow[u], c_) * 16);                            \
  }
      RMBX_GEMM_FRAGS(0, 0)
#pragma unroll
      for (int ks = 0; ks < GBK / 16; ++ks) {
        const int cb = ks & 1;
        if (ks + 1 < GBK / 16) RMBX_GEMM_FRAGS(cb ^ 1, ks + 1)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int u = 0; u < 4; ++u) acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[cb][t], fx[cb][u], acc[t][u], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
#undef RMBX_GEMM_FRAGS
    }
    __builtin_amdgcn_s_setprio(0);
    __syncthreads();  // the DMA into the other stage has landed (vmcnt(0)) and this stage is free
  }
  {
    const int tile = t_begin + (my_tiles - 1) * nbx;
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    gemm_epilogue(a, acc, tm * GBM, tn * GBN, wm, wn, kh, r32);
  }
}

int gemm_device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0)
      cus = c;
    else
      cus = 256;
  }
  return cus;
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_linear_bf16(const void* x, const void* weight, const float* bias, void* out, int M, int N, int K,
                                int ldo, int relu, void* stream) {
  RMBX_CHECK_ARG(x && weight && out, "rmbx_linear_bf16: null pointer");
  RMBX_CHECK_ARG(M >= 0 && N > 0 && K > 0, "rmbx_linear_bf16: bad shape M=%d N=%d K=%d", M, N, K);
  RMBX_CHECK_ARG(K % rmbx::GBK == 0, "rmbx_linear_bf16: K=%d must be a multiple of %d", K, rmbx::GBK);
  RMBX_CHECK_ARG(N % 16 == 0 && ldo >= N && ldo % 8 == 0, "rmbx_linear_bf16: N=%d must be a multiple of 16, ldo=%d", N, ldo);
  RMBX_CHECK_ARG((((uintptr_t)x | (uintptr_t)weight | (uintptr_t)out) & 15) == 0 && (!bias || ((uintptr_t)bias & 15) == 0),
                 "rmbx_linear_bf16: pointers must be 16-byte aligned");
  if (M == 0) return RMBX_OK;
  rmbx::GemmArgs a;
  a.x = (const uint16_t*)x;
  a.w = (const uint16_t*)weight;
  a.bias = bias;
  a.out = (uint16_t*)out;
  a.M = M;
  a.N = N;
  a.K = K;
  a.ldo = ldo;
  a.relu = relu;
  const char* dbg_env = std::getenv("RMBX_GEMM_DBG");
  a.dbg = dbg_env ? std::atoi(dbg_env) : 0;
  a.tiles_m = (M + rmbx::GBM - 1) / rmbx::GBM;
  a.tiles_n = (N + rmbx::GBN - 1) / rmbx::GBN;
  const long long ntiles = (long long)a.tiles_m * a.tiles_n;
  RMBX_CHECK_ARG(ntiles < (1ll << 31), "rmbx_linear_bf16: too many tiles");
  const int cus = rmbx::gemm_device_cus();
  const int nblocks = (int)(ntiles < cus ? ntiles : cus);
  hipLaunchKernelGGL(rmbx::gemm_bf16_tn_kernel, dim3((unsigned)nblocks), dim3(rmbx::GTHREADS), 0, (hipStream_t)stream, a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
