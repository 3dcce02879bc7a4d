// Multi-head attention forward for the ACT transformer, bf16 in/out, f32 softmax/accumulation,
// head dim 64, no mask (MFMA 32x32x16, gfx950).  Replaces scaled_dot_product_attention inside
// nn.MultiheadAttention of ACT's encoder self-attention (S = 302), decoder self-attention (100)
// and decoder cross-attention (100 x 302) (third_party/act detr/models/transformer.py [absent];
// sizes policy/act/TrainAct.py:46-58: d 512, 8 heads).
//
// One block per (batch, head); its waves walk the 32-query groups.  The whole key/value sequence
// of the (batch, head) (<= 320 keys) is staged in LDS once for all queries: K row-major with the 16-byte
// chunk XOR swizzle of the GEMM kernels, V transposed so the P.V MFMA reads its A operand as
// 16-byte rows.  Scores are computed transposed, S^T = K . Q^T, so each lane owns ONE query and 16
// of the tile's keys: the online-softmax max and sum are in-lane except for one exchange with the
// partner half-wave (lane ^ 32), and the probabilities feed the P.V MFMA straight from registers
// (the key order inside a tile is permuted to match on the V side).  The output is computed as
// O^T = V^T . P^T with V's dims permuted so each lane finishes 16 consecutive dims of its query:
// the result leaves as 16-byte stores into [B][Lq][heads * 64] (the layout out_proj reads).

#include "rmbx_common.h"

#include <cstdint>
#include <cstdlib>

namespace rmbx {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int AT_MAX_WAVES = 5;  // waves per block (each walks 32-query groups)
constexpr int AT_LK_MAX = 320;   // keys staged per block
constexpr int AT_VT_LD = AT_LK_MAX;  // V^T row pitch (bf16); 16-byte chunk c of row d stored at c ^ ((d >> 1) & 7)

struct AttnArgs {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  uint16_t* o;
  long long q_bstride, k_bstride, v_bstride;  // elements between batches
  int q_rstride, k_rstride, v_rstride;        // elements between sequence rows
  int o_rstride;                              // = heads * 64
  int heads, Lq, Lk;
  float scale_log2;                           // softmax scale * log2(e)
  int dbg;                                    // diagnostic (RMBX_ATTN_DBG; 0 in production): 1 staging only
};

__device__ __forceinline__ int at_sigma(int i) { return 16 * ((i >> 2) & 1) + (i & 3) + 4 * (i >> 3); }
// position p (0..31) inside a 32-key tile of the transposed V image -> key offset it holds
__device__ __forceinline__ int at_key_of_pos(int p) {
  const int u = p >> 4, h = (p >> 3) & 1, m = p & 7;
  return 16 * u + 4 * h + (m & 3) + 8 * (m >> 2);
}

// column of position p in row d of the swizzled V^T image (the 16-byte chunk XOR of the K image:
// row pitch 640 B = 8 bank quads mod 16, so (d >> 1) & 7 spreads every read group over 16 quads)
__device__ __forceinline__ int vt_col(int d, int p) { return (((p >> 3) ^ ((d >> 1) & 7)) << 3) | (p & 7); }

__global__ void __launch_bounds__(64 * AT_MAX_WAVES) attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t sK[AT_LK_MAX * 64];
  __shared__ __attribute__((aligned(16))) uint16_t sVt[64 * AT_VT_LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.x;
  const int b = bh / a.heads, hd = bh - b * a.heads;
  const int Lk = a.Lk;
  const int nkt = (Lk + 31) >> 5;  // 32-key tiles
  const uint16_t* kb = a.k + b * a.k_bstride + hd * 64;
  const uint16_t* vb = a.v + b * a.v_bstride + hd * 64;

  // stage K ([key][8 chunks], chunk c at c ^ ((key >> 1) & 7)) and V^T (sVt[d][32 t + p] =
  // V[32 t + key_of_pos(p)][d]); keys >= Lk are zero.  All of this thread's global loads are issued
  // before the first LDS write, so the block pays one memory latency, not one per chunk.
  constexpr int ST = (AT_LK_MAX * 8 + 255) / 256;  // chunks per thread and operand (>= 256 threads)
  const int nchunk = nkt * 32 * 8, nthr = blockDim.x;
  uint4 kr[ST], vr[ST];
#pragma unroll
  for (int i = 0; i < ST; ++i) {
    const int q = tid + i * nthr;
    const int key = q >> 3, c = q & 7;
    const int p_all = key;  // V^T position of this chunk; its key is permuted inside the tile
    const int vkey = (p_all & ~31) + at_key_of_pos(p_all & 31);
    const bool okk = q < nchunk && key < Lk, okv = q < nchunk && vkey < Lk;
    kr[i] = *reinterpret_cast<const uint4*>(kb + (size_t)(okk ? key : 0) * a.k_rstride + c * 8);
    vr[i] = *reinterpret_cast<const uint4*>(vb + (size_t)(okv ? vkey : 0) * a.v_rstride + c * 8);
    if (!okk) kr[i] = make_uint4(0, 0, 0, 0);
    if (!okv) vr[i] = make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < ST; ++i) {
    const int q = tid + i * nthr;
    if (q >= nchunk) break;
    const int key = q >> 3, c = q & 7;
    *reinterpret_cast<uint4*>(sK + key * 64 + ((c ^ ((key >> 1) & 7)) * 8)) = kr[i];
    const uint32_t w[4] = {vr[i].x, vr[i].y, vr[i].z, vr[i].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int d0 = c * 8 + 2 * e, d1 = d0 + 1;
      sVt[d0 * AT_VT_LD + vt_col(d0, key)] = (uint16_t)(w[e] & 0xffff);
      sVt[d1 * AT_VT_LD + vt_col(d1, key)] = (uint16_t)(w[e] >> 16);
    }
  }

  const int r32 = lane & 31, kh = lane >> 5;
  const float c = a.scale_log2;
  const bool ragged = (Lk & 31) != 0;
  __syncthreads();
  if (a.dbg & 1) {
    if (tid == 0 && sK[0] == 0x7fff && sVt[1] == 0x7fff) a.o[0] = 0;  // keep the staging live
    return;
  }

  // wave w takes the 32-query groups w, w + nwaves, ... (K/V staged once for all of them)
  const int ngroups = (a.Lq + 31) >> 5, nwaves = blockDim.x >> 6;
  for (int grp = wave; grp < ngroups; grp += nwaves) {
    const int qi = grp * 32 + r32;  // this lane's query
    const bool q_ok = qi < a.Lq;
    // Q^T fragments (B operand of S^T = K Q^T): dims 16 s + 8 kh .. +7 of query qi
    bf16x8 fq[4];
    {
      const uint16_t* qrow = a.q + b * a.q_bstride + (size_t)(q_ok ? qi : 0) * a.q_rstride + hd * 64;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        uint4 val = *reinterpret_cast<const uint4*>(qrow + 16 * s + 8 * kh);
        if (!q_ok) val = make_uint4(0, 0, 0, 0);
        fq[s] = __builtin_bit_cast(bf16x8, val);
      }
    }
    f32x16 acc0 = {}, acc1 = {};  // O^T: dims sigma(i) (+32), query r32
    float m_run = -INFINITY;      // running max of the raw scores (scale > 0 commutes with max)
    float l_run = 0.f;            // this lane's partial softmax denominator
    // S^T tile t: rows = keys 32 t + (lane-row layout), cols = this wave's 32 queries
    auto score_tile = [&](int t) {
      f32x16 st = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int key = 32 * t + r32;
        const int cc = 2 * ks + kh;
        const bf16x8 fk = *reinterpret_cast<const bf16x8*>(sK + key * 64 + ((cc ^ ((key >> 1) & 7)) * 8));
        st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fk, fq[ks], st, 0, 0, 0);
      }
      return st;
    };
    // software pipeline: tile t + 1's score MFMAs are issued before tile t's softmax, so the
    // matrix core works while the wave's VALU does the exponentials
    f32x16 s_next = score_tile(0);
    for (int t = 0; t < nkt; ++t) {
      f32x16 s = s_next;
      if (t + 1 < nkt) s_next = score_tile(t + 1);
      __builtin_amdgcn_sched_barrier(0);
      // this lane's 16 keys: 32 t + 4 kh + (j & 3) + 8 (j >> 2); padding keys only in the last tile
      if (ragged && t == nkt - 1) {
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (32 * t + 4 * kh + (j & 3) + 8 * (j >> 2) >= Lk) s[j] = -INFINITY;
      }
      float mx = s[0];
#pragma unroll
      for (int j = 1; j < 16; ++j) mx = fmaxf(mx, s[j]);
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const float m_new = fmaxf(m_run, mx);
      // rescale only when some query's max moved (wave-uniform test)
      if (__any(m_new != m_run)) {
        const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * c);  // first tile: exp2(-inf) = 0
        l_run *= alpha;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          acc0[j] *= alpha;
          acc1[j] *= alpha;
        }
        m_run = m_new;
      }
      const float mc = m_run * c;
      // P (bf16) as the B operand of O^T += V^T P^T: k-step u takes registers 8 u .. 8 u + 7
      bf16x8 fp[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f32x2 pv;
          pv[0] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[8 * u + 2 * e], c, -mc));
          pv[1] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[8 * u + 2 * e + 1], c, -mc));
          l_run += pv[0] + pv[1];
          const bf16x2 pb = __builtin_convertvector(pv, bf16x2);
          fp[u][2 * e] = pb[0];
          fp[u][2 * e + 1] = pb[1];
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int d0 = at_sigma(r32), d1 = d0 + 32, p = 32 * t + 16 * u + 8 * kh;
        const bf16x8 fv0 = *reinterpret_cast<const bf16x8*>(sVt + d0 * AT_VT_LD + vt_col(d0, p));
        const bf16x8 fv1 = *reinterpret_cast<const bf16x8*>(sVt + d1 * AT_VT_LD + vt_col(d1, p));
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fv0, fp[u], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fv1, fp[u], acc1, 0, 0, 0);
      }
    }
    const float l_tot = l_run + __shfl_xor(l_run, 32);
    if (!q_ok) continue;
    const float inv = 1.f / l_tot;
    uint16_t* orow = a.o + (size_t)b * a.Lq * a.o_rstride + (size_t)qi * a.o_rstride + hd * 64 + 16 * kh;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const f32x16& acc = half ? acc1 : acc0;
      uint32_t pk[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        f32x2 ov;
        ov[0] = acc[2 * e] * inv;
        ov[1] = acc[2 * e + 1] * inv;
        pk[e] = __builtin_bit_cast(uint32_t, __builtin_convertvector(ov, bf16x2));
      }
      *reinterpret_cast<uint4*>(orow + 32 * half) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
      *reinterpret_cast<uint4*>(orow + 32 * half + 8) = make_uint4(pk[4], pk[5], pk[6], pk[7]);
    }
  }
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_attention_bf16(const void* q, const void* k, const void* v, void* out, int B, int heads, int Lq,
                                   int Lk, long long q_bstride, int q_rstride, long long k_bstride, int k_rstride,
                                   long long v_bstride, int v_rstride, float scale, void* stream) {
  RMBX_CHECK_ARG(q && k && v && out, "rmbx_attention_bf16: null pointer");
  RMBX_CHECK_ARG(B >= 0 && heads > 0 && Lq > 0 && Lk > 0, "rmbx_attention_bf16: bad shape");
  RMBX_CHECK_ARG(Lk <= rmbx::AT_LK_MAX, "rmbx_attention_bf16: Lk=%d exceeds %d", Lk, rmbx::AT_LK_MAX);
  RMBX_CHECK_ARG(q_rstride % 8 == 0 && k_rstride % 8 == 0 && v_rstride % 8 == 0 && q_bstride % 8 == 0 &&
                     k_bstride % 8 == 0 && v_bstride % 8 == 0,
                 "rmbx_attention_bf16: strides must be multiples of 8 elements");
  RMBX_CHECK_ARG((((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)out) & 15) == 0,
                 "rmbx_attention_bf16: pointers must be 16-byte aligned");
  if (B == 0) return RMBX_OK;
  rmbx::AttnArgs a;
  a.q = (const uint16_t*)q;
  a.k = (const uint16_t*)k;
  a.v = (const uint16_t*)v;
  a.o = (uint16_t*)out;
  a.q_bstride = q_bstride;
  a.k_bstride = k_bstride;
  a.v_bstride = v_bstride;
  a.q_rstride = q_rstride;
  a.k_rstride = k_rstride;
  a.v_rstride = v_rstride;
  a.o_rstride = heads * 64;
  a.heads = heads;
  a.Lq = Lq;
  a.Lk = Lk;
  a.scale_log2 = scale * 1.4426950408889634f;
  const char* dbg_env = std::getenv("RMBX_ATTN_DBG");
  a.dbg = dbg_env ? std::atoi(dbg_env) : 0;
  RMBX_CHECK_ARG(scale > 0.f, "rmbx_attention_bf16: scale must be positive");
  const long long nblocks = (long long)B * heads;
  RMBX_CHECK_ARG(nblocks < (1ll << 31), "rmbx_attention_bf16: grid too large");
  // waves: the fewest passes over the 32-query groups with at most AT_MAX_WAVES waves, then as
  // few waves as that many passes need (302 queries: 5 waves x 2 groups; 100: 4 x 1)
  const int ngroups = (Lq + 31) / 32;
  const int passes = (ngroups + rmbx::AT_MAX_WAVES - 1) / rmbx::AT_MAX_WAVES;
  const int waves = (ngroups + passes - 1) / passes;
  hipLaunchKernelGGL(rmbx::attn_fwd_kernel, dim3((unsigned)nblocks), dim3(64 * waves), 0, (hipStream_t)stream, a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
