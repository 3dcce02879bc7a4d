// fp32-accurate 3x3 / stride-1 / pad-1 convolution in the f16x3 form with the input staged ONCE
// per spatial tile (gfx950): the implicit GEMM of rmbx_conv2d_f16x3 loads and splits every input
// pixel once per tap (nine times); here a block stages the (TH + 2) x (TW + 2) input patch of its
// output tile for one 32-channel chunk, split into its two f16 pieces, and all nine taps read
// their MFMA A fragments from that patch.
//
// Replaces the stride-1 3x3 conv -> FrozenBN -> (+ residual) -> ReLU steps of ACT's ResNet-18
// BasicBlocks (torchvision resnet18 inside third_party/act [absent]; the reference runs the
// policy in fp32, RolloutAct.py / ACTPolicy) at 64 and 128 channels.
//
// Arithmetic: the f16x3 scheme of csrc/rmbx_gemm.hip.  W rows come pre-split (rmbx_split_f16x2 of
// the [Cout][9 C] filter, tap-major K, per-row power-of-two scale ws[n]); the input pieces are
// h = f16(x 2^t), l = f16((x 2^t - h) 2^11) and acc += l (2^-11 hb) + h lb + h hb, one f32
// accumulator.  The power of two 2^t is chosen per (tile, chunk) from the chunk's max |x| (max in
// [2^13, 2^14)) and only ever decreases along a tile's chunks: the accumulator is rescaled by the
// (exact) ratio when it does, and the epilogue applies ws[n] 2^-t.  f16's range is thereby
// handled for any input; for values that are normal f16 numbers under both scalings the pieces are
// exact scalings of each other, so the result does not depend on the other pixels of the tile.
//
// Mapping: 512 threads = 8 waves, a block owns a 16 x TW output tile x BN output channels
// (TW = 16, BN = 128 or TW = 32, BN = 64: 256 x 128 or 512 x 64 outputs), wave = 64 pixels (four
// 16-pixel rows of the tile) x 64 channels, v_mfma_f32_16x16x32_f16.  Persistent blocks walk the
// (tile, channel block) units; one K step per tap (32 channels), nine per chunk, one barrier each;
// W of the next step is loaded into registers under this step's MFMAs and stored to the other W
// buffer after them; the next chunk's patch (a 32-channel chunk of the tile, or the next unit's
// first) is loaded under the chunk's first taps, its max reduced in LDS mid-chunk, and it is
// split and stored after the chunk's last MFMAs (one extra barrier per chunk; splitting it in
// registers during the chunk's last W group instead was slower: the VALU beside the MFMAs costs
// more than it hides, profiles/r4_conv3x3_patch_presplit_ab.log).
// LDS images: patch [2 pieces][pixel][4 x 16-B slots of 8 channels], W [2 buffers][2 pieces][BN
// rows][4 slots]; 16-B slot s of row / pixel r at s ^ ((r >> 1) & 3): the 16-lane groups of every
// fragment read cover all 64 banks.
#include "rmbx_common.h"

#include <cstdint>
#include <cstdlib>

namespace rmbx {
namespace {

typedef _Float16 cp_f16x8 __attribute__((ext_vector_type(8)));
typedef float cp_f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 cp_f16x2 __attribute__((ext_vector_type(2)));
typedef float cp_f32x2 __attribute__((ext_vector_type(2)));

constexpr int CP_THREADS = 512;
constexpr int CP_TH = 16;    // tile rows
constexpr int CP_KC = 32;    // channels per chunk (one MFMA K step)
constexpr int CP_TNONE = 1000;  // "no nonzero input yet" scale exponent

struct ConvPArgs {
  const float* in;        // [N][H][W][C]
  const uint16_t* w;      // f16 pieces: piece p, row n, k at w + p * wps + n * K + k (K = 9 C)
  const float* ws;        // [Cout] per-row power-of-two scales of the pieces
  const float* bias;      // [Cout] or null
  const float* res;       // [N][H][W][Cout] or null
  float* out;             // [N][H][W][Cout]
  long long wps;
  int N, H, W, C, Cout, relu;
  int tiles_x, tiles_y, ncb, units;
};

__device__ __forceinline__ uint32_t cp_pk(float x, float y) {
  cp_f32x2 v = {x, y};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, cp_f16x2));
}
// x -> h = f16(x), l = f16((x - h) 2^11) for a pair
__device__ __forceinline__ void cp_split(float x, float y, uint32_t& h, uint32_t& l) {
  h = cp_pk(x, y);
  const cp_f16x2 hv = __builtin_bit_cast(cp_f16x2, h);
  l = cp_pk((x - (float)hv[0]) * 2048.f, (y - (float)hv[1]) * 2048.f);
}
__device__ __forceinline__ int cp_slot(int r, int s) { return s ^ ((r >> 1) & 3); }

// VAR (profiling, RMBX_CONVP_VAR; wrong results, timing only): bit 0 = no epilogue (one store per
// lane keeps the accumulators live), bit 1 = no patch re-staging (the first patch is reused), bit 2
// = no W staging (the first W row is reused)
// Template: TW tile width, BN output channels per block, MI 16-pixel row segments per wave (a wave
// owns 16 MI pixels x 64 channels), WG taps per W staging group (3: one filter row per barrier, 1:
// one tap), MINB blocks per CU (2: 4 waves per SIMD, 128 registers).
template <int TW, int BN, int MI, int WG, int MINB, int VAR = 0>
__device__ __forceinline__ void conv3x3p_body(const ConvPArgs& a) {
  static_assert((TW / MI) * (BN / 64) == CP_THREADS / 64, "8 waves of 16 MI pixels x 64 channels");
  static_assert(WG == 1 || WG == 3, "a W group is one tap or one filter row");
  constexpr int NG = 9 / WG;  // W groups (barriers) per chunk
  constexpr int PW = TW + 2, PP = (CP_TH + 2) * PW;       // patch width, pixels
  constexpr int PLANE = PP * 64;                          // bytes of one patch piece
  constexpr int WPLANE = BN * 64;                         // bytes of one W piece
  constexpr int NPR = (PP * 8 + CP_THREADS - 1) / CP_THREADS;  // patch float4 loads per thread
  constexpr int NWR = (2 * BN * 4) / CP_THREADS;               // W 16-B loads per thread
  constexpr int WN = BN / 64;                                   // waves across the channels
  __shared__ __attribute__((aligned(16))) unsigned char sP[2 * PLANE];
  __shared__ __attribute__((aligned(16))) unsigned char sW[2 * WG * 2 * WPLANE];  // [buf][tap in group][piece][row]
  __shared__ unsigned int sMax;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - wm * WN;  // 16 MI-pixel slab, 64-channel column block
  const int fr = lane & 15, fs = lane >> 4;
  const int K = 9 * a.C, nchunk = a.C / CP_KC;

  // unit -> (image, tile origin, channel block)
  auto unit_geo = [&](int u, int& img, int& oy0, int& ox0, int& n0) {
    const int cb = u % a.ncb, t = u / a.ncb;
    const int tx = t % a.tiles_x, r = t / a.tiles_x;
    const int ty = r % a.tiles_y;
    img = r / a.tiles_y;
    oy0 = ty * CP_TH;
    ox0 = tx * TW;
    n0 = cb * BN;
  };

  // ---- patch staging of stage (unit u, chunk c): thread item q = tid + 512 i -> pixel q / 8,
  // channel quad q % 8
  float4 pr[NPR];
  auto load_patch = [&](int u, int c) {
    int img, oy0, ox0, n0;
    unit_geo(u, img, oy0, ox0, n0);
#pragma unroll
    for (int i = 0; i < NPR; ++i) {
      const int q = tid + CP_THREADS * i;
      const int p = q >> 3, q8 = q & 7;
      const int py = p / PW, px = p - py * PW;
      const int y = oy0 - 1 + py, x = ox0 - 1 + px;
      const bool ok = q < PP * 8 && (unsigned)y < (unsigned)a.H && (unsigned)x < (unsigned)a.W;
      pr[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ok)
        pr[i] = *reinterpret_cast<const float4*>(a.in + (((long long)img * a.H + y) * a.W + x) * a.C + c * CP_KC +
                                                 4 * q8);
    }
  };
  auto patch_max = [&]() {
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < NPR; ++i)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(pr[i].x), fabsf(pr[i].y)), fmaxf(fabsf(pr[i].z), fabsf(pr[i].w))));
    return m;
  };
  auto store_patch = [&](int t) {
#pragma unroll
    for (int i = 0; i < NPR; ++i) {
      const int q = tid + CP_THREADS * i;
      if (q >= PP * 8) break;
      const int p = q >> 3, q8 = q & 7;
      uint32_t h0, l0, h1, l1;
      cp_split(ldexpf(pr[i].x, t), ldexpf(pr[i].y, t), h0, l0);
      cp_split(ldexpf(pr[i].z, t), ldexpf(pr[i].w, t), h1, l1);
      const int off = p * 64 + cp_slot(p, q8 >> 1) * 16 + (q8 & 1) * 8;
      *reinterpret_cast<uint2*>(sP + off) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(sP + PLANE + off) = make_uint2(l0, l1);
    }
  };
  // scale exponent of a chunk from its max |x| (bits): max * 2^t in [2^13, 2^14)
  auto chunk_t = [](unsigned int mbits) {
    if (mbits == 0u) return CP_TNONE;
    int e;
    frexpf(__uint_as_float(mbits), &e);
    return 14 - e;
  };

  // ---- W of one staging group (unit u, chunk c, group g: taps WG g .. WG g + WG - 1): item
  // q = tid + 512 i -> (piece, row, 16-B slot) of each tap; named registers (not an array: hipcc
  // kept a captured uint4 array in scratch)
  static_assert(NWR == 1 || NWR == 2, "BN = 64 or 128");
  uint4 w00 = make_uint4(0, 0, 0, 0), w01 = w00, w10 = w00, w11 = w00, w20 = w00, w21 = w00;
  auto w_item = [&](int i, int& pc, int& n, int& sl) {
    const int q = tid + CP_THREADS * i;
    pc = q / (BN * 4);
    const int rem = q - pc * (BN * 4);
    n = rem >> 2;
    sl = rem & 3;
  };
  auto w_src = [&](int u, int c, int tap, int i) {
    int pc, n, sl;
    w_item(i, pc, n, sl);
    const int n0 = (u % a.ncb) * BN;
    return reinterpret_cast<const uint4*>(a.w + pc * a.wps + (long long)(n0 + n) * K + tap * a.C + c * CP_KC +
                                          8 * sl);
  };
  auto load_w = [&](int u, int c, int g) {
    w00 = *w_src(u, c, WG * g, 0);
    if constexpr (NWR == 2) w01 = *w_src(u, c, WG * g, 1);
    if constexpr (WG == 3) {
      w10 = *w_src(u, c, WG * g + 1, 0);
      w20 = *w_src(u, c, WG * g + 2, 0);
      if constexpr (NWR == 2) {
        w11 = *w_src(u, c, WG * g + 1, 1);
        w21 = *w_src(u, c, WG * g + 2, 1);
      }
    }
  };
  auto w_dst = [&](int buf, int k, int i) {
    int pc, n, sl;
    w_item(i, pc, n, sl);
    return reinterpret_cast<uint4*>(sW + ((buf * WG + k) * 2 + pc) * WPLANE + n * 64 + cp_slot(n, sl) * 16);
  };
  auto store_w = [&](int buf) {
    *w_dst(buf, 0, 0) = w00;
    if constexpr (NWR == 2) *w_dst(buf, 0, 1) = w01;
    if constexpr (WG == 3) {
      *w_dst(buf, 1, 0) = w10;
      *w_dst(buf, 2, 0) = w20;
      if constexpr (NWR == 2) {
        *w_dst(buf, 1, 1) = w11;
        *w_dst(buf, 2, 1) = w21;
      }
    }
  };

  cp_f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (cp_f32x4){0.f, 0.f, 0.f, 0.f};

  // MFMAs of one tap: A fragments from the patch at (ky, kx), B from W buffer wb
  auto mfma_tap = [&](int tap, int k, int wb) {  // tap (ky, kx); W at slot k of buffer wb
    const int ky = tap / 3, kx = tap - 3 * ky;
    cp_f16x8 ah[MI], al[MI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int p0 = wm * 16 * MI + mi * 16;  // first pixel of this 16-pixel row segment
      const int ty = p0 / TW, tx = p0 - ty * TW;
      const int pp = (ty + ky) * PW + tx + fr + kx;
      const int off = pp * 64 + cp_slot(pp, fs) * 16;
      ah[mi] = *reinterpret_cast<const cp_f16x8*>(sP + off);
      al[mi] = *reinterpret_cast<const cp_f16x8*>(sP + PLANE + off);
    }
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) {
      const int n = wn * 64 + nj * 16 + fr;
      const int off = n * 64 + cp_slot(n, fs) * 16;
      const cp_f16x8 bh = *reinterpret_cast<const cp_f16x8*>(sW + ((wb * WG + k) * 2) * WPLANE + off);
      const cp_f16x8 bl = *reinterpret_cast<const cp_f16x8*>(sW + ((wb * WG + k) * 2 + 1) * WPLANE + off);
      const cp_f16x8 bs = bh * (_Float16)0.00048828125f;  // 2^-11 hb (exact above f16's subnormals)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        cp_f32x4 c = acc[mi][nj];
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[mi], bs, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[mi], bl, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[mi], bh, c, 0, 0, 0);
        acc[mi][nj] = c;
      }
    }
  };

  // epilogue of a unit: each 4 x 4 block of an accumulator (4 pixels x 4 channels over 4 lanes) is
  // transposed across its lane quad by two DPP exchanges, so a lane holds 4 consecutive channels of
  // one pixel: 16-B residual loads and stores (past-the-image pixels read a clamped address and
  // skip the store)
  auto epilogue = [&](int u, int t) {
    if constexpr ((VAR & 1) != 0) {
      float sum = 0.f;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) sum += acc[mi][nj][0] + acc[mi][nj][1] + acc[mi][nj][2] + acc[mi][nj][3];
      a.out[(long long)(u % 4096) * CP_THREADS + tid] = sum;
      return;
    }
    int img, oy0, ox0, n0;
    unit_geo(u, img, oy0, ox0, n0);
    const int j = fr & 3, q = fr >> 2;  // lane in its quad, quad of 4 channels
    float4 sn[4], bb[4];
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) {
      const int n = n0 + wn * 64 + nj * 16 + 4 * q;
      sn[nj] = *reinterpret_cast<const float4*>(a.ws + n);
      bb[nj] = a.bias ? *reinterpret_cast<const float4*>(a.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    auto xchg = [](float x, int ctrl) {
      return __int_as_float(ctrl == 1 ? __builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xf, 0xf, false)
                                      : __builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xf, 0xf, false));
    };
    // the residual loads of two row segments at a time (two memory round trips per unit instead
    // of one per segment; all four at once spills the 16 x 32-pixel configuration)
#pragma unroll
    for (int m2 = 0; m2 < MI; m2 += 2) {
      long long pix[2];
      bool ok[2];
      float4 rv[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int p = wm * 16 * MI + (m2 + h) * 16 + 4 * fs + j;  // this lane's pixel after the transpose
        const int ty = p / TW, tx = p - ty * TW;
        const int y = oy0 + ty, x = ox0 + tx;
        ok[h] = y < a.H && x < a.W;
        pix[h] = ok[h] ? ((long long)img * a.H + y) * a.W + x : 0;
#pragma unroll
        for (int nj = 0; nj < 4; ++nj)
          rv[h][nj] = a.res ? *reinterpret_cast<const float4*>(a.res + pix[h] * a.Cout + n0 + wn * 64 + nj * 16 + 4 * q)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int mi = m2 + h;
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) {
          float v0 = acc[mi][nj][0], v1 = acc[mi][nj][1], v2 = acc[mi][nj][2], v3 = acc[mi][nj][3];
          {  // 2 x 2 blocks transposed with the lane j ^ 1
            const bool odd = j & 1;
            const float ra = xchg(odd ? v0 : v1, 1), rb = xchg(odd ? v2 : v3, 1);
            if (odd) { v0 = ra; v2 = rb; } else { v1 = ra; v3 = rb; }
          }
          {  // off-diagonal 2 x 2 blocks swapped with the lane j ^ 2
            const bool hi = j & 2;
            const float ra = xchg(hi ? v0 : v2, 2), rb = xchg(hi ? v1 : v3, 2);
            if (hi) { v0 = ra; v1 = rb; } else { v2 = ra; v3 = rb; }
          }
          const float sc[4] = {sn[nj].x, sn[nj].y, sn[nj].z, sn[nj].w};
          const float bs[4] = {bb[nj].x, bb[nj].y, bb[nj].z, bb[nj].w};
          const float rs[4] = {rv[h][nj].x, rv[h][nj].y, rv[h][nj].z, rv[h][nj].w};
          float o[4] = {v0, v1, v2, v3};
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            float v = t == CP_TNONE ? 0.f : ldexpf(o[c] * sc[c], -t);
            v += bs[c];
            v += rs[c];
            if (a.relu) v = fmaxf(v, 0.f);
            o[c] = v;
          }
          if (ok[h])
            *reinterpret_cast<float4*>(a.out + pix[h] * a.Cout + n0 + wn * 64 + nj * 16 + 4 * q) =
                make_float4(o[0], o[1], o[2], o[3]);
        }
      }
    }
  };

  // ---- persistent walk over the stages (unit, chunk) of this block's units
  const int G = gridDim.x;
  int u = blockIdx.x;
  if (u >= a.units) return;
  if (tid == 0) sMax = 0u;
  load_patch(u, 0);
  load_w(u, 0, 0);  // group 0
  __syncthreads();
  atomicMax(&sMax, __float_as_uint(patch_max()));
  __syncthreads();
  int t_cur = chunk_t(sMax);
  store_patch(t_cur == CP_TNONE ? 0 : t_cur);
  store_w(0);
  __syncthreads();
  if (tid == 0) sMax = 0u;  // (read by every thread before the barrier above)

  int c = 0, wb = 0;
  while (true) {
    // the stage after this one: the next chunk of this unit, or the next unit's first
    const bool last_chunk = c + 1 == nchunk;
    const int u_next = last_chunk ? u + G : u;
    const int c_next = last_chunk ? 0 : c + 1;
    const bool more = u_next < a.units;
#pragma unroll 1
    for (int g = 0; g < NG; ++g) {
      if ((VAR & 2) == 0 && g == 0 && more) load_patch(u_next, c_next);
      // W of the next group, loaded and stored unconditionally (after the last group: a redundant
      // copy of this group into the idle buffer) so the staging registers stay registers
      const int wu = g < NG - 1 || !more ? u : u_next, wc = g < NG - 1 || !more ? c : c_next;
      const int wg = g < NG - 1 ? g + 1 : (more ? 0 : g);
      if constexpr ((VAR & 4) == 0) load_w(wu, wc, wg);
      // keep the loads ahead of the MFMAs (left alone, the scheduler sinks them behind the MFMA
      // stream, and their latency is exposed at the end of every step)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < WG; ++k) mfma_tap(WG * g + k, k, wb);
      if (g == NG / 2 && more) atomicMax(&sMax, __float_as_uint(patch_max()));
      if constexpr ((VAR & 4) == 0) store_w(wb ^ 1);
      __syncthreads();
      wb ^= 1;
    }
    if (!more) {
      epilogue(u, t_cur);
      break;
    }
    // every wave is past the chunk's MFMAs: replace the patch with the next stage's
    const int tc = chunk_t(sMax);
    const int t_next = last_chunk ? tc : min(t_cur, tc);
    if constexpr ((VAR & 2) == 0) store_patch(t_next == CP_TNONE ? 0 : t_next);
    if (last_chunk) {
      epilogue(u, t_cur);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (cp_f32x4){0.f, 0.f, 0.f, 0.f};
    } else if (t_next != t_cur) {  // the chunk needs a smaller scale: rescale the sum so far (exact)
      const int d = t_cur == CP_TNONE ? -200 : t_next - t_cur;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][e] = ldexpf(acc[i][j][e], d);
    }
    t_cur = t_next;
    __syncthreads();                // the new patch is visible; sMax read by every thread
    if (tid == 0) sMax = 0u;        // (the next atomicMax comes after this stage's tap-4 barrier)
    u = u_next;
    c = c_next;
  }
}

// one block per CU (up to 256 registers per lane) / two blocks per CU (128: four waves per SIMD)
template <int TW, int BN, int MI, int WG, int VAR>
__global__ void __launch_bounds__(CP_THREADS, 1) conv3x3p_f16x3_kernel(ConvPArgs a) {
  conv3x3p_body<TW, BN, MI, WG, 1, VAR>(a);
}
template <int TW, int BN, int MI, int WG, int VAR>
__global__ void __launch_bounds__(CP_THREADS, 4)  // (hipcc: the second argument is waves per SIMD)
conv3x3p2_f16x3_kernel(ConvPArgs a) {
  conv3x3p_body<TW, BN, MI, WG, 2, VAR>(a);
}

template <int TW, int BN, int MI, int WG, int MINB>
int launch_convp(const ConvPArgs& base, hipStream_t st) {
  const char* ve = std::getenv("RMBX_CONVP_VAR");  // profiling phase skips (read per launch)
  const int var = ve ? std::atoi(ve) : 0;
  ConvPArgs a = base;
  a.tiles_x = (a.W + TW - 1) / TW;
  a.tiles_y = (a.H + CP_TH - 1) / CP_TH;
  a.ncb = a.Cout / BN;
  const long long units = (long long)a.N * a.tiles_x * a.tiles_y * a.ncb;
  RMBX_CHECK_ARG(units < (1ll << 31), "rmbx_conv3x3_f16x3_patch: too many tiles");
  a.units = (int)units;
  if (a.units == 0) return RMBX_OK;
  int dev = 0, cus = 0;
  RMBX_CHECK_HIP(hipGetDevice(&dev));
  RMBX_CHECK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = a.units < MINB * cus ? a.units : MINB * cus;
#define RMBX_CP_LAUNCH(V)                                                                                       \
  if constexpr (MINB == 2)                                                                                      \
    hipLaunchKernelGGL((conv3x3p2_f16x3_kernel<TW, BN, MI, WG, V>), dim3(grid), dim3(CP_THREADS), 0, st, a); \
  else                                                                                                          \
    hipLaunchKernelGGL((conv3x3p_f16x3_kernel<TW, BN, MI, WG, V>), dim3(grid), dim3(CP_THREADS), 0, st, a)
  switch (var) {
    case 1: RMBX_CP_LAUNCH(1); break;
    case 2: RMBX_CP_LAUNCH(2); break;
    case 4: RMBX_CP_LAUNCH(4); break;
    case 7: RMBX_CP_LAUNCH(7); break;
    default: RMBX_CP_LAUNCH(0);
  }
#undef RMBX_CP_LAUNCH
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_conv3x3_f16x3_patch(const float* in, int N, int H, int W, int C, const void* w_planes,
                                        long long w_plane_stride, const float* w_scale, const float* bias,
                                        const float* res, float* out, int Cout, int relu, void* stream) {
  RMBX_CHECK_ARG(in && w_planes && w_scale && out, "rmbx_conv3x3_f16x3_patch: null pointer");
  RMBX_CHECK_ARG(N >= 0 && H > 0 && W > 0, "rmbx_conv3x3_f16x3_patch: bad geometry");
  RMBX_CHECK_ARG(C > 0 && C % rmbx::CP_KC == 0, "rmbx_conv3x3_f16x3_patch: C=%d must be a multiple of 32", C);
  RMBX_CHECK_ARG(Cout > 0 && Cout % 64 == 0, "rmbx_conv3x3_f16x3_patch: Cout=%d must be a multiple of 64", Cout);
  RMBX_CHECK_ARG(w_plane_stride >= (long long)Cout * 9 * C && w_plane_stride % 8 == 0,
                 "rmbx_conv3x3_f16x3_patch: bad plane stride %lld", w_plane_stride);
  RMBX_CHECK_ARG((((uintptr_t)in | (uintptr_t)w_planes) & 15) == 0,
                 "rmbx_conv3x3_f16x3_patch: in / w_planes must be 16-byte aligned");
  // the epilogue reads w_scale / bias / res and writes out as float4 (no scalar fallback)
  RMBX_CHECK_ARG((((uintptr_t)out | (uintptr_t)res | (uintptr_t)bias | (uintptr_t)w_scale) & 15) == 0,
                 "rmbx_conv3x3_f16x3_patch: out / res / bias / w_scale must be 16-byte aligned");
  RMBX_CHECK_ARG((long long)N * H * W * (C > Cout ? C : Cout) < (1ll << 40), "rmbx_conv3x3_f16x3_patch: too large");
  if (N == 0) return RMBX_OK;
  rmbx::ConvPArgs a{};
  a.in = in;
  a.w = (const uint16_t*)w_planes;
  a.ws = w_scale;
  a.bias = bias;
  a.res = res;
  a.out = out;
  a.wps = w_plane_stride;
  a.N = N;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Cout = Cout;
  a.relu = relu ? 1 : 0;
  // RMBX_CONVP_CFG (read per launch): 0 = one block per CU (16 x 16 tiles x 128 channels, or 16 x
  // 32 x 64 when Cout % 128 != 0; a filter row of W per barrier), 1 = two blocks per CU (16 x 16 x 64,
  // 32 pixels x 64 channels per wave, one tap of W per barrier: one block's epilogue and patch
  // staging under the other's MFMAs)
  const char* ce = std::getenv("RMBX_CONVP_CFG");
  const int cfg = ce ? std::atoi(ce) : 0;
  if (cfg == 1) return rmbx::launch_convp<16, 64, 2, 1, 2>(a, (hipStream_t)stream);
  if (Cout % 128 == 0) return rmbx::launch_convp<16, 128, 4, 3, 1>(a, (hipStream_t)stream);
  return rmbx::launch_convp<32, 64, 4, 3, 1>(a, (hipStream_t)stream);
}
