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
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

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

// ---------------------------------------------------------------------------------------------
// f32 form (the reference's fp32 policy): exact f32 products and accumulation on
// v_mfma_f32_32x32x2_f32, f32 online softmax.  f32 MFMA is 16x slower than bf16, so this kernel is
// MFMA-bound and is laid out for occupancy rather than for LDS reuse: a block of 4-5 waves takes
// up to 5 32-query groups of one (batch, head) (302 queries: two blocks), the keys stream through
// a double-buffered LDS tile of 32 keys (K and V, 17 KiB each buffer, one barrier per tile, the
// next tile prefetched into registers under the current tile's MFMAs), so 3-4 blocks share a CU.
// Per wave and key tile: S^T = K Q^T (32 MFMAs, Q held in registers pre-scaled by scale*log2 e,
// dims 32h + kk on lane half h), the online softmax in-lane plus one exchange with lane ^ 32, and
// O^T += V^T P^T (2 x 16 MFMAs) with P fed straight from the S accumulator registers (MFMA t
// consumes key 8(t/4) + 4h + t%4 on half h, the key the S register t of that half holds) and
// V's dims permuted (at_sigma) so each lane finishes 16 consecutive dims of its query.
// ---------------------------------------------------------------------------------------------
constexpr int AF_MAX_WAVES = 5;
constexpr int AF_KP = 65;  // K tile row pitch (floats): lanes (key i, half h) at i*65 + 32h hit 64 banks
constexpr int AF_VP = 72;  // V tile row pitch: the halves' keys (4 apart) land 32 banks apart
constexpr int AF_TILE = 32 * AF_KP + 32 * AF_VP;  // floats of one K + V tile buffer

struct AttnF32Args {
  const float* q;
  const float* k;
  const float* v;
  float* o;
  long long q_bstride, k_bstride, v_bstride;
  int q_rstride, k_rstride, v_rstride;
  int o_rstride;
  int heads, Lq, Lk, parts;
  float scale_log2;
  // rmbx_attention_f16x3: per block, 1 = re-run on the bf16x6 kernel (written by the f16x3 kernel;
  // the bf16x6 kernel then runs only the flagged blocks); null for the other kernels
  int* redo = nullptr;
  int xcd_map = 0;  // f16x3 kernel: the parts of a head on one XCD (RMBX_ATTN_XCD=1; not faster)
};

template <int DBG>
__global__ void __launch_bounds__(64 * AF_MAX_WAVES) __attribute__((amdgpu_waves_per_eu(4))) attn_fwd_f32_kernel(AttnF32Args a) {
  __shared__ __attribute__((aligned(16))) float sT[2 * AF_TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nthreads = blockDim.x, nwaves = nthreads >> 6;
  const int bh = blockIdx.x / a.parts, part = blockIdx.x - bh * a.parts;
  const int b = bh / a.heads, head = bh - b * a.heads;
  const int n = lane & 31, h = lane >> 5;
  const int qrow = (part * nwaves + wave) * 32 + n;
  const bool qok = qrow < a.Lq;
  const float* kbase = a.k + (size_t)b * a.k_bstride + head * 64;
  const float* vbase = a.v + (size_t)b * a.v_bstride + head * 64;

  // this lane's query dims 32h .. 32h + 31, pre-scaled into the log2 domain
  float qv[32];
  {
    const float* qp = a.q + (size_t)b * a.q_bstride + (size_t)(qok ? qrow : 0) * a.q_rstride + head * 64 + 32 * h;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float4 x = *reinterpret_cast<const float4*>(qp + 4 * c);
      qv[4 * c] = x.x * a.scale_log2;
      qv[4 * c + 1] = x.y * a.scale_log2;
      qv[4 * c + 2] = x.z * a.scale_log2;
      qv[4 * c + 3] = x.w * a.scale_log2;
    }
  }

  // key tile jt -> registers in two halves (K rows, then V rows: 512 16-byte chunks each, at most
  // 2 per thread), each loaded one phase ahead of its store so that only 8 staging registers live
  const int nt = (a.Lk + 31) >> 5;
  constexpr int PF = 2;
  float4 pf[PF];
  auto load_half = [&](int jt, const float* base, int rstride) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int c = tid + nthreads * i;
      const int key = 32 * jt + (c >> 4), quad = c & 15;
      const bool ok = c < 512 && key < a.Lk;
      pf[i] = ok ? *reinterpret_cast<const float4*>(base + (size_t)key * rstride + 4 * quad) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_k = [&](float* buf) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int c = tid + nthreads * i;
      if (c >= 512) continue;
      float* d = buf + (c >> 4) * AF_KP + 4 * (c & 15);  // 4-byte aligned rows
      d[0] = pf[i].x;
      d[1] = pf[i].y;
      d[2] = pf[i].z;
      d[3] = pf[i].w;
    }
  };
  auto store_v = [&](float* buf) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int c = tid + nthreads * i;
      if (c < 512) *reinterpret_cast<float4*>(buf + 32 * AF_KP + (c >> 4) * AF_VP + 4 * (c & 15)) = pf[i];
    }
  };
  load_half(0, kbase, a.k_rstride);
  store_k(sT);
  load_half(0, vbase, a.v_rstride);
  store_v(sT);
  __syncthreads();

  const int sg = at_sigma(n);
  f32x16 o0 = {}, o1 = {};
  float m = -INFINITY, l = 0.f;
  for (int jt = 0; jt < nt; ++jt) {
    float* buf = sT + (jt & 1) * AF_TILE;
    float* nbuf = sT + ((jt + 1) & 1) * AF_TILE;  // read last in tile jt - 1
    const bool more = jt + 1 < nt;
    if (more && !(DBG & 8)) load_half(jt + 1, kbase, a.k_rstride);
    // S^T tile: rows = keys, cols = queries
    f32x16 s = {};
    const float* kr = buf + n * AF_KP + 32 * h;
    if (!(DBG & 1)) {
#pragma unroll
      for (int kk = 0; kk < 32; ++kk) s = __builtin_amdgcn_mfma_f32_32x32x2f32(kr[kk], qv[kk], s, 0, 0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) s[j] = kr[j] * qv[j];
    }
    if (more && !(DBG & 8)) {
      store_k(nbuf);
      load_half(jt + 1, vbase, a.v_rstride);
    }
    if (!(DBG & 2)) {
    float mx = -INFINITY;
    if (32 * jt + 32 > a.Lk) {  // the ragged last tile only (uniform branch)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int key = 32 * jt + 8 * (j >> 2) + 4 * h + (j & 3);
        if (key >= a.Lk) s[j] = -INFINITY;
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) mx = fmaxf(mx, s[j]);
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mn = fmaxf(m, mx);  // finite: every tile holds >= 1 key
    const float alpha = exp2f(m - mn);
    float ps = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      s[j] = exp2f(s[j] - mn);
      ps += s[j];
    }
    ps += __shfl_xor(ps, 32);
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      o0[j] *= alpha;
      o1[j] *= alpha;
    }
    } else {
      l += s[0];
    }
    // O^T += V^T P^T: MFMA t takes key 8(t/4) + 4h + t%4 of this tile on half h
    const float* vr = buf + 32 * AF_KP + sg;
    if (!(DBG & 4)) {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const float* vk = vr + (8 * (t >> 2) + 4 * h + (t & 3)) * AF_VP;
        o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(vk[0], s[t], o0, 0, 0, 0);
        o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(vk[32], s[t], o1, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) o0[t] += vr[t] * s[t];
    }
    if (more && !(DBG & 8)) store_v(nbuf);
    __syncthreads();
  }
  if (qok) {
    const float inv = 1.f / l;
    float* op = a.o + ((size_t)b * a.Lq + qrow) * a.o_rstride + head * 64 + 16 * h;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      *reinterpret_cast<float4*>(op + 4 * c) =
          make_float4(o0[4 * c] * inv, o0[4 * c + 1] * inv, o0[4 * c + 2] * inv, o0[4 * c + 3] * inv);
      *reinterpret_cast<float4*>(op + 32 + 4 * c) =
          make_float4(o1[4 * c] * inv, o1[4 * c + 1] * inv, o1[4 * c + 2] * inv, o1[4 * c + 3] * inv);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// fp32-accurate form on the bf16 matrix cores (rmbx_attention_f32x6; the reference's fp32 policy):
// every f32 operand of the two products (Q, K, V and the probabilities P) is split into three bf16
// pieces x = x0 + x1 + x2 and each product accumulates the six piece products with i + j <= 2 in f32
// (the rmbx_linear_f32x6 scheme, csrc/rmbx_gemm.hip): the f32 GEMM error class at 2.67x the f32
// MFMA rate.  Layout of the bf16 kernel above (S^T = K Q^T with each lane owning one query, P fed
// from the S accumulator registers, V's dims permuted so each lane finishes 16 consecutive dims),
// keys streamed through double-buffered 32-key LDS tiles as in the f32 kernel: per tile and buffer
// K [3 pieces][32 keys][64 dims] (16-byte chunk c of key row r at c ^ ((r >> 1) & 7)) and V^T
// [3 pieces][64 dims][32 positions] (position p holds key at_key_of_pos(p); chunk c of dim row d at
// c ^ ((d >> 2) & 3)), 24 KiB; the block's threads load the next tile into registers under this
// tile's MFMAs and split + store it after them; one barrier per tile.
// ---------------------------------------------------------------------------------------------
constexpr int AX_MAX_WAVES = 5;
constexpr int AX_PLANE = 32 * 64;               // bf16 elements of one piece of a K or V^T tile
constexpr int AX_BUF = 6 * AX_PLANE;            // K pieces then V^T pieces
constexpr int AX_CH = (1024 + 64 * 4 - 1) / (64 * 4);  // staged 16-byte chunks per thread (>= 256 threads)

__device__ __forceinline__ uint32_t ax_pk(float x, float y) {
  f32x2 v = {x, y};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
// (x, y) -> three packed bf16 pairs, x = x0 + x1 + x2 exactly (round-to-nearest-even at each level)
__device__ __forceinline__ void ax_split(float x, float y, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
  p0 = ax_pk(x, y);
  const float rx = x - __uint_as_float(p0 << 16), ry = y - __uint_as_float(p0 & 0xffff0000u);
  p1 = ax_pk(rx, ry);
  const float sx = rx - __uint_as_float(p1 << 16), sy = ry - __uint_as_float(p1 & 0xffff0000u);
  p2 = ax_pk(sx, sy);
}
// position of tile key k (0..31) in the V^T image (inverse of at_key_of_pos)
__device__ __forceinline__ int ax_pos_of_key(int k) {
  const int r = k & 15;
  return 16 * (k >> 4) + 8 * ((r >> 2) & 1) + (r & 3) + 4 * (r >> 3);
}

__global__ void __launch_bounds__(64 * AX_MAX_WAVES) attn_fwd_f32x6_kernel(AttnF32Args a) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[2 * AX_BUF];
  if (a.redo && a.redo[blockIdx.x] == 0) return;  // f16x3 re-run mode: only the flagged blocks
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nthreads = blockDim.x;
  const int bh = blockIdx.x / a.parts, part = blockIdx.x - bh * a.parts;
  const int b = bh / a.heads, hd = bh - b * a.heads;
  const int r32 = lane & 31, kh = lane >> 5;
  const int qi = (part * (nthreads >> 6) + wave) * 32 + r32;
  const bool q_ok = qi < a.Lq;
  const float* kbase = a.k + (size_t)b * a.k_bstride + hd * 64;
  const float* vbase = a.v + (size_t)b * a.v_bstride + hd * 64;
  const int nt = (a.Lk + 31) >> 5;

  // Q^T pieces (B operand of S^T = K Q^T): dims 16 s + 8 kh .. +7 of query qi
  bf16x8 fq[4][3];
  {
    const float* qp = a.q + (size_t)b * a.q_bstride + (size_t)(q_ok ? qi : 0) * a.q_rstride + hd * 64 + 8 * kh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float4 x0 = *reinterpret_cast<const float4*>(qp + 16 * s);
      const float4 x1 = *reinterpret_cast<const float4*>(qp + 16 * s + 4);
      uint32_t p0[4], p1[4], p2[4];
      ax_split(x0.x, x0.y, p0[0], p1[0], p2[0]);
      ax_split(x0.z, x0.w, p0[1], p1[1], p2[1]);
      ax_split(x1.x, x1.y, p0[2], p1[2], p2[2]);
      ax_split(x1.z, x1.w, p0[3], p1[3], p2[3]);
      fq[s][0] = __builtin_bit_cast(bf16x8, make_uint4(p0[0], p0[1], p0[2], p0[3]));
      fq[s][1] = __builtin_bit_cast(bf16x8, make_uint4(p1[0], p1[1], p1[2], p1[3]));
      fq[s][2] = __builtin_bit_cast(bf16x8, make_uint4(p2[0], p2[1], p2[2], p2[3]));
    }
  }

  // staging: chunk q < 512 = K[key q/16][4 (q%16) ..], q >= 512 = V[key (q-512)/16][...]
  float4 st[AX_CH];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int i = 0; i < AX_CH; ++i) {
      const int q = tid + nthreads * i;
      const int qq = q & 511, key = 32 * t + (qq >> 4), quad = qq & 15;
      const bool ok = q < 1024 && key < a.Lk;
      const float* src = q < 512 ? kbase + (size_t)key * a.k_rstride : vbase + (size_t)key * a.v_rstride;
      st[i] = ok ? *reinterpret_cast<const float4*>(src + 4 * quad) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_tile = [&](uint16_t* buf) {
#pragma unroll
    for (int i = 0; i < AX_CH; ++i) {
      const int q = tid + nthreads * i;
      if (q >= 1024) continue;
      const int qq = q & 511, key = qq >> 4, quad = qq & 15;
      uint32_t p0[2], p1[2], p2[2];
      ax_split(st[i].x, st[i].y, p0[0], p1[0], p2[0]);
      ax_split(st[i].z, st[i].w, p0[1], p1[1], p2[1]);
      if (q < 512) {  // K: 4 dims = half a 16-byte chunk of the key row
        const int off = key * 64 + (((quad >> 1) ^ ((key >> 1) & 7)) << 3) + 4 * (quad & 1);
        *reinterpret_cast<uint2*>(buf + off) = make_uint2(p0[0], p0[1]);
        *reinterpret_cast<uint2*>(buf + AX_PLANE + off) = make_uint2(p1[0], p1[1]);
        *reinterpret_cast<uint2*>(buf + 2 * AX_PLANE + off) = make_uint2(p2[0], p2[1]);
      } else {  // V^T: 4 dims of one key = one element in each of 4 rows
        const int pos = ax_pos_of_key(key);
        const uint32_t pk[3][2] = {{p0[0], p0[1]}, {p1[0], p1[1]}, {p2[0], p2[1]}};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int d = 4 * quad + e;
          const int off = 3 * AX_PLANE + d * 32 + ((((pos >> 3) ^ ((d >> 2) & 3))) << 3) + (pos & 7);
#pragma unroll
          for (int pc = 0; pc < 3; ++pc)
            buf[off + pc * AX_PLANE] = (uint16_t)((pk[pc][e >> 1] >> (16 * (e & 1))) & 0xffff);
        }
      }
    }
  };
  load_tile(0);
  store_tile(sA);
  __syncthreads();

  const float c = a.scale_log2;
  const bool ragged = (a.Lk & 31) != 0;
  const int d0 = at_sigma(r32), d1 = d0 + 32;
  f32x16 acc0 = {}, acc1 = {};
  float m_run = -INFINITY, l_run = 0.f;
  for (int t = 0; t < nt; ++t) {
    const uint16_t* buf = sA + (t & 1) * AX_BUF;
    const bool more = t + 1 < nt;
    if (more) load_tile(t + 1);
    // S^T tile: six piece products per 16-dim step
    f32x16 s = {};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int off = r32 * 64 + (((2 * ks + kh) ^ ((r32 >> 1) & 7)) << 3);
      const bf16x8 k0 = *reinterpret_cast<const bf16x8*>(buf + off);
      const bf16x8 k1 = *reinterpret_cast<const bf16x8*>(buf + AX_PLANE + off);
      const bf16x8 k2 = *reinterpret_cast<const bf16x8*>(buf + 2 * AX_PLANE + off);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k2, fq[ks][0], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k1, fq[ks][1], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k0, fq[ks][2], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k1, fq[ks][0], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k0, fq[ks][1], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k0, fq[ks][0], s, 0, 0, 0);
    }
    // this lane's 16 keys: 32 t + 4 kh + (j & 3) + 8 (j >> 2); padding keys only in the last tile
    if (ragged && t == nt - 1) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (32 * t + 4 * kh + (j & 3) + 8 * (j >> 2) >= a.Lk) s[j] = -INFINITY;
    }
    float mx = s[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) mx = fmaxf(mx, s[j]);
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float m_new = fmaxf(m_run, mx);
    if (__any(m_new != m_run)) {
      const float alpha = exp2f((m_run - m_new) * c);  // first tile: exp2(-inf) = 0
      l_run *= alpha;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        acc0[j] *= alpha;
        acc1[j] *= alpha;
      }
      m_run = m_new;
    }
    const float mc = m_run * c;
    // P pieces: the B operand of O^T += V^T P^T, k-step u from registers 8 u .. 8 u + 7
    bf16x8 fp[2][3];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      uint32_t p0[4], p1[4], p2[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pa = exp2f(fmaf(s[8 * u + 2 * e], c, -mc));
        const float pb = exp2f(fmaf(s[8 * u + 2 * e + 1], c, -mc));
        l_run += pa + pb;
        ax_split(pa, pb, p0[e], p1[e], p2[e]);
      }
      fp[u][0] = __builtin_bit_cast(bf16x8, make_uint4(p0[0], p0[1], p0[2], p0[3]));
      fp[u][1] = __builtin_bit_cast(bf16x8, make_uint4(p1[0], p1[1], p1[2], p1[3]));
      fp[u][2] = __builtin_bit_cast(bf16x8, make_uint4(p2[0], p2[1], p2[2], p2[3]));
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int cc = 2 * u + kh;
      const int o0 = 3 * AX_PLANE + d0 * 32 + ((cc ^ ((d0 >> 2) & 3)) << 3);
      const int o1 = 3 * AX_PLANE + d1 * 32 + ((cc ^ ((d1 >> 2) & 3)) << 3);
      bf16x8 v0[3], v1[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) {
        v0[pc] = *reinterpret_cast<const bf16x8*>(buf + o0 + pc * AX_PLANE);
        v1[pc] = *reinterpret_cast<const bf16x8*>(buf + o1 + pc * AX_PLANE);
      }
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v0[2], fp[u][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v1[2], fp[u][0], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v0[1], fp[u][1], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v1[1], fp[u][1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v0[0], fp[u][2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v1[0], fp[u][2], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v0[1], fp[u][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v1[1], fp[u][0], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v0[0], fp[u][1], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v1[0], fp[u][1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v0[0], fp[u][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v1[0], fp[u][0], acc1, 0, 0, 0);
    }
    if (more) store_tile(sA + ((t + 1) & 1) * AX_BUF);
    __syncthreads();
  }
  const float l_tot = l_run + __shfl_xor(l_run, 32);
  if (!q_ok) return;
  const float inv = 1.f / l_tot;
  // acc0 register e = dim 16 kh + e, acc1 = dim 32 + 16 kh + e
  float* op = a.o + ((size_t)b * a.Lq + qi) * a.o_rstride + hd * 64 + 16 * kh;
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) {
    *reinterpret_cast<float4*>(op + 4 * q4) =
        make_float4(acc0[4 * q4] * inv, acc0[4 * q4 + 1] * inv, acc0[4 * q4 + 2] * inv, acc0[4 * q4 + 3] * inv);
    *reinterpret_cast<float4*>(op + 32 + 4 * q4) =
        make_float4(acc1[4 * q4] * inv, acc1[4 * q4 + 1] * inv, acc1[4 * q4 + 2] * inv, acc1[4 * q4 + 3] * inv);
  }
}

// ---------------------------------------------------------------------------------------------
// f16x3 form (rmbx_attention_f16x3, the fp32 policy's default since round 4): the f16x3 GEMM's
// scheme (csrc/rmbx_gemm.hip) on the two products, three piece products each instead of six on
// the f16 matrix cores (bf16 rate):
//   S^T = K Q^T:  K (staged) = kh + 2^-11 kl with kh = f16(k), kl = f16((k - kh) 2^11); Q (registers)
//                 = qh + ql with ql = f16(q - qh): S = kh qh + kh ql + kl (2^-11 qh)
//   O^T += V^T P^T: V as K; P' = 2^14 exp2(...) (the power of two keeps every probability down to
//                 2^-28 in f16's normal range; l sums the same P', so O = acc / l is unchanged)
//                 = ph + pl: O' = vh ph + vh pl + vl (2^-11 ph)
// Each piece product is exact in f32; the dropped kl ql / vl pl terms are 2^-22 relative.  Q is
// scaled per query by a power of two 2^t putting the query's max |q| (over the head's 64 dims) in
// [2^13, 2^14) before the split, so its pieces stay in f16's normal range whatever the query's
// magnitude (an unscaled ql = f16(q - qh) is subnormal for every |q| < 2^-3, an absolute error floor
// of 2^-25 per element); the softmax undoes the scale exactly through the per-query log2 factor
// c 2^-t (S' = 2^t S, exp2((S' - m') c 2^-t) = exp2((S - m) c)).  f16's range of the staged
// operands is checked per block: any |k|, |v| >= 2^15 (f16 overflow), a max |k| over the block in
// (0, 2^-6), a head dimension whose max |v| over the keys is in (0, 2^-6) (their values would sit
// near f16's subnormal floor), or a non-finite query flags the block, and rmbx_attention_f16x3
// re-runs the flagged blocks on the bf16x6 kernel (f32's exponent range), so every query's result
// depends only on its own block (one head of one batch item).
// Layout of the bf16x6 kernel, two pieces per staged tile (16 KiB per buffer).
// ---------------------------------------------------------------------------------------------
constexpr int AH_PLANE = 32 * 64;      // f16 elements of one piece of a K or V^T tile
constexpr int AH_BUF = 4 * AH_PLANE;   // K pieces then V^T pieces
constexpr float AH_BIG = 32768.f;      // 2^15
constexpr float AH_TINY = 0.015625f;   // 2^-6

__device__ __forceinline__ uint32_t ah_pk(float x, float y) {
  f32x2 v = {x, y};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2));
}
__device__ __forceinline__ float ah_lo(uint32_t p) { return (float)__builtin_bit_cast(f16x2, p)[0]; }
__device__ __forceinline__ float ah_hi(uint32_t p) { return (float)__builtin_bit_cast(f16x2, p)[1]; }
// staged operand (K, V): h = f16(x), l = f16((x - h) 2^11)
__device__ __forceinline__ void ah_split_a(float x, float y, uint32_t& h, uint32_t& l) {
  h = ah_pk(x, y);
  l = ah_pk((x - ah_lo(h)) * 2048.f, (y - ah_hi(h)) * 2048.f);
}
// register operand (Q, P'): h = f16(x), l = f16(x - h)
__device__ __forceinline__ void ah_split_w(float x, float y, uint32_t& h, uint32_t& l) {
  h = ah_pk(x, y);
  l = ah_pk(x - ah_lo(h), y - ah_hi(h));
}

// DBG (profiling phase skips, RMBX_ATTN_F16_DBG; wrong results, timing only): 1 = no V^T staging
// stores, 2 = no S^T MFMAs, 4 = no softmax (fixed P'), 8 = no PV MFMAs, 16 = no K / V tile loads
template <int DBG>
__global__ void __launch_bounds__(64 * AX_MAX_WAVES) attn_fwd_f16x3_kernel(AttnF32Args a) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[2 * AH_BUF];
  __shared__ uint32_t sDim[64];  // per head dimension: max |v| over the keys (f32 bits)
  __shared__ uint32_t sKmax;     // max |k| over the block (f32 bits)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nthreads = blockDim.x;
  // block -> (head, query part): plain order, or (xcd_map) the parts of one head on one XCD, one
  // after the other (blocks bid and bid + 8 when parts = 2) so the second part's K / V reads could
  // hit that XCD's L2
  int bh, part;
  if (a.xcd_map && a.parts > 1 && (gridDim.x & (8 * a.parts - 1)) == 0 && (a.parts & (a.parts - 1)) == 0) {
    const int j = blockIdx.x >> 3;
    part = j & (a.parts - 1);
    bh = (j / a.parts) * 8 + (blockIdx.x & 7);
  } else {
    bh = blockIdx.x / a.parts;
    part = blockIdx.x - bh * a.parts;
  }
  const int b = bh / a.heads, hd = bh - b * a.heads;
  const int r32 = lane & 31, kh = lane >> 5;
  const int qi = (part * (nthreads >> 6) + wave) * 32 + r32;
  const bool q_ok = qi < a.Lq;
  const float* kbase = a.k + (size_t)b * a.k_bstride + hd * 64;
  const float* vbase = a.v + (size_t)b * a.v_bstride + hd * 64;
  const int nt = (a.Lk + 31) >> 5;
  if (tid < 64) sDim[tid] = 0u;
  if (tid == 0) sKmax = 0u;
  float big = 0.f;   // this thread's max |k|, |v| (and inf for a non-finite query)
  float kmx = 0.f;   // this thread's max |k|

  // Q pieces (B operand of S^T = K Q^T): dims 16 s + 8 kh .. +7 of query qi, scaled by the query's
  // power of two 2^t (max |q| into [2^13, 2^14)); fq[s][2] = 2^-11 qh
  f16x8 fq[4][3];
  float c = a.scale_log2;  // this query's log2-domain softmax factor: scale_log2 2^-t
  {
    const float* qp = a.q + (size_t)b * a.q_bstride + (size_t)(q_ok ? qi : 0) * a.q_rstride + hd * 64 + 8 * kh;
    float4 x[4][2];
    float qm = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      x[s][0] = *reinterpret_cast<const float4*>(qp + 16 * s);
      x[s][1] = *reinterpret_cast<const float4*>(qp + 16 * s + 4);
#pragma unroll
      for (int u = 0; u < 2; ++u)
        qm = fmaxf(qm, fmaxf(fmaxf(fabsf(x[s][u].x), fabsf(x[s][u].y)), fmaxf(fabsf(x[s][u].z), fabsf(x[s][u].w))));
    }
    qm = fmaxf(qm, __shfl_xor(qm, 32));  // the other 32 dims of the query
    int t = 0;
    if (qm > 0.f && qm < INFINITY) {
      int e;
      frexpf(qm, &e);  // qm in [2^(e-1), 2^e)
      t = 14 - e;
      t = t < -100 ? -100 : (t > 100 ? 100 : t);  // (keeps c 2^-t a normal f32)
    } else if (qm == INFINITY) {
      big = INFINITY;  // a non-finite query: the block re-runs on bf16x6
    }
    c = ldexpf(c, -t);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      uint32_t h[4], l[4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float4 y = make_float4(ldexpf(x[s][u].x, t), ldexpf(x[s][u].y, t), ldexpf(x[s][u].z, t),
                                     ldexpf(x[s][u].w, t));
        ah_split_w(y.x, y.y, h[2 * u], l[2 * u]);
        ah_split_w(y.z, y.w, h[2 * u + 1], l[2 * u + 1]);
      }
      fq[s][0] = __builtin_bit_cast(f16x8, make_uint4(h[0], h[1], h[2], h[3]));
      fq[s][1] = __builtin_bit_cast(f16x8, make_uint4(l[0], l[1], l[2], l[3]));
      fq[s][2] = fq[s][0] * (_Float16)0.00048828125f;
    }
  }

  // staging: chunk q < 512 = K[key q/16][4 (q%16) ..], q >= 512 = V[key (q-512)/16][...]; the
  // thread count is a multiple of 16, so a thread's V chunks all hold dims 4 (tid & 15) .. + 3
  float4 st[AX_CH];
  float vmax[4] = {0.f, 0.f, 0.f, 0.f};
  auto load_tile = [&](int t) {
#pragma unroll
    for (int i = 0; i < AX_CH; ++i) {
      const int q = tid + nthreads * i;
      const int qq = q & 511, key = 32 * t + (qq >> 4), quad = qq & 15;
      const bool ok = q < 1024 && key < a.Lk && ((DBG & 16) == 0 || t == 0);
      const float* src = q < 512 ? kbase + (size_t)key * a.k_rstride : vbase + (size_t)key * a.v_rstride;
      st[i] = ok ? *reinterpret_cast<const float4*>(src + 4 * quad) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_tile = [&](uint16_t* buf) {
#pragma unroll
    for (int i = 0; i < AX_CH; ++i) {
      const int q = tid + nthreads * i;
      if (q >= 1024) continue;
      const int qq = q & 511, key = qq >> 4, quad = qq & 15;
      const float ax = fabsf(st[i].x), ay = fabsf(st[i].y), az = fabsf(st[i].z), aw = fabsf(st[i].w);
      big = fmaxf(big, fmaxf(fmaxf(ax, ay), fmaxf(az, aw)));
      uint32_t h[2], l[2];
      ah_split_a(st[i].x, st[i].y, h[0], l[0]);
      ah_split_a(st[i].z, st[i].w, h[1], l[1]);
      if (q < 512) {  // K: 4 dims = half a 16-byte chunk of the key row
        kmx = fmaxf(kmx, fmaxf(fmaxf(ax, ay), fmaxf(az, aw)));
        const int off = key * 64 + (((quad >> 1) ^ ((key >> 1) & 7)) << 3) + 4 * (quad & 1);
        *reinterpret_cast<uint2*>(buf + off) = make_uint2(h[0], h[1]);
        *reinterpret_cast<uint2*>(buf + AH_PLANE + off) = make_uint2(l[0], l[1]);
      } else if ((DBG & 1) == 0) {  // V^T: 4 dims of one key = one element in each of 4 rows
        vmax[0] = fmaxf(vmax[0], ax);
        vmax[1] = fmaxf(vmax[1], ay);
        vmax[2] = fmaxf(vmax[2], az);
        vmax[3] = fmaxf(vmax[3], aw);
        const int pos = ax_pos_of_key(key);
        const uint32_t pk[2][2] = {{h[0], h[1]}, {l[0], l[1]}};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int d = 4 * quad + e;
          const int off = 2 * AH_PLANE + d * 32 + ((((pos >> 3) ^ ((d >> 2) & 3))) << 3) + (pos & 7);
#pragma unroll
          for (int pc = 0; pc < 2; ++pc)
            buf[off + pc * AH_PLANE] = (uint16_t)((pk[pc][e >> 1] >> (16 * (e & 1))) & 0xffff);
        }
      }
    }
  };
  load_tile(0);
  store_tile(sA);
  __syncthreads();

  const bool ragged = (a.Lk & 31) != 0;
  const int d0 = at_sigma(r32), d1 = d0 + 32;
  f32x16 acc0 = {}, acc1 = {};
  float m_run = -INFINITY, l_run = 0.f;
  for (int t = 0; t < nt; ++t) {
    const uint16_t* buf = sA + (t & 1) * AH_BUF;
    const bool more = t + 1 < nt;
    if (more) load_tile(t + 1);
    // S^T tile: three piece products per 16-dim step
    f32x16 s = {};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int off = r32 * 64 + (((2 * ks + kh) ^ ((r32 >> 1) & 7)) << 3);
      const f16x8 k0 = *reinterpret_cast<const f16x8*>(buf + off);
      const f16x8 k1 = *reinterpret_cast<const f16x8*>(buf + AH_PLANE + off);
      if constexpr ((DBG & 2) != 0) {
        s[ks] += (float)k0[0] + (float)k1[0];
      } else {
        s = __builtin_amdgcn_mfma_f32_32x32x16_f16(k1, fq[ks][2], s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0, fq[ks][1], s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0, fq[ks][0], s, 0, 0, 0);
      }
    }
    if (ragged && t == nt - 1) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (32 * t + 4 * kh + (j & 3) + 8 * (j >> 2) >= a.Lk) s[j] = -INFINITY;
    }
    float mx = s[0];
    if constexpr ((DBG & 4) == 0) {
#pragma unroll
      for (int j = 1; j < 16; ++j) mx = fmaxf(mx, s[j]);
      mx = fmaxf(mx, __shfl_xor(mx, 32));
    }
    const float m_new = fmaxf(m_run, mx);
    if ((DBG & 4) == 0 && __any(m_new != m_run)) {
      const float alpha = exp2f((m_run - m_new) * c);  // first tile: exp2(-inf) = 0
      l_run *= alpha;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        acc0[j] *= alpha;
        acc1[j] *= alpha;
      }
      m_run = m_new;
    }
    const float mc = m_run * c;
    // P' pieces: the B operand of O^T += V^T P'^T, k-step u from registers 8 u .. 8 u + 7
    f16x8 fp[2][3];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      uint32_t h[4], l[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if constexpr ((DBG & 4) != 0) {
          h[e] = __float_as_uint(s[8 * u + 2 * e]);
          l[e] = __float_as_uint(s[8 * u + 2 * e + 1]);
          continue;
        }
        // (v_exp_f32 alone: exp2f's denormal-result path only changes p' < 2^-112, which is zero
        // in the f16 pieces and below the ulp of l >= 2^14)
        const float pa = __builtin_amdgcn_exp2f(fmaf(s[8 * u + 2 * e], c, -mc)) * 16384.f;
        const float pb = __builtin_amdgcn_exp2f(fmaf(s[8 * u + 2 * e + 1], c, -mc)) * 16384.f;
        l_run += pa + pb;
        ah_split_w(pa, pb, h[e], l[e]);
      }
      fp[u][0] = __builtin_bit_cast(f16x8, make_uint4(h[0], h[1], h[2], h[3]));
      fp[u][1] = __builtin_bit_cast(f16x8, make_uint4(l[0], l[1], l[2], l[3]));
      fp[u][2] = fp[u][0] * (_Float16)0.00048828125f;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int cc = 2 * u + kh;
      const int o0 = 2 * AH_PLANE + d0 * 32 + ((cc ^ ((d0 >> 2) & 3)) << 3);
      const int o1 = 2 * AH_PLANE + d1 * 32 + ((cc ^ ((d1 >> 2) & 3)) << 3);
      f16x8 v0[2], v1[2];
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
        v0[pc] = *reinterpret_cast<const f16x8*>(buf + o0 + pc * AH_PLANE);
        v1[pc] = *reinterpret_cast<const f16x8*>(buf + o1 + pc * AH_PLANE);
      }
      if constexpr ((DBG & 8) != 0) {
        acc0[u] += (float)v0[1][0] + (float)v0[0][0] + (float)fp[u][0][0] + (float)fp[u][1][0] + (float)fp[u][2][0];
        acc1[u] += (float)v1[1][0] + (float)v1[0][0];
        continue;
      }
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v0[1], fp[u][2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1[1], fp[u][2], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v0[0], fp[u][1], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1[0], fp[u][1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v0[0], fp[u][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1[0], fp[u][0], acc1, 0, 0, 0);
    }
    if (more) store_tile(sA + ((t + 1) & 1) * AH_BUF);
    __syncthreads();
  }
  // range check: the block re-runs on the bf16x6 kernel if any operand left f16's range
#pragma unroll
  for (int e = 0; e < 4; ++e)  // (|v| as u32 bits orders like the value)
    if (vmax[e] > 0.f) atomicMax(&sDim[4 * (tid & 15) + e], __float_as_uint(vmax[e]));
  if (kmx > 0.f) atomicMax(&sKmax, __float_as_uint(kmx));
  __syncthreads();
  // (fmaxf skips NaNs: NaN inputs are not flagged and propagate through the f16 pieces)
  bool flag = big >= AH_BIG;
  if (tid < 64) {
    const float m = __uint_as_float(sDim[tid]);
    flag = flag || (m > 0.f && m < AH_TINY);
  }
  if (tid == 0) {
    const float km = __uint_as_float(sKmax);
    flag = flag || (km > 0.f && km < AH_TINY);
  }
  const int any = __syncthreads_or(flag ? 1 : 0);
  if (tid == 0) a.redo[bh * a.parts + part] = any;  // the bf16x6 kernel's block order
  if (any) return;
  const float l_tot = l_run + __shfl_xor(l_run, 32);
  if (!q_ok) return;
  const float inv = 1.f / l_tot;
  float* op = a.o + ((size_t)b * a.Lq + qi) * a.o_rstride + hd * 64 + 16 * kh;
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) {
    *reinterpret_cast<float4*>(op + 4 * q4) =
        make_float4(acc0[4 * q4] * inv, acc0[4 * q4 + 1] * inv, acc0[4 * q4 + 2] * inv, acc0[4 * q4 + 3] * inv);
    *reinterpret_cast<float4*>(op + 32 + 4 * q4) =
        make_float4(acc1[4 * q4] * inv, acc1[4 * q4 + 1] * inv, acc1[4 * q4 + 2] * inv, acc1[4 * q4 + 3] * inv);
  }
}

// ---------------------------------------------------------------------------------------------
// f16x3 form with the key / value tiles staged by LDS-DMA (rmbx_attention_f16x3's default since
// round 6: PIPE = false, ONE = true; RMBX_ATTN_DMA=0 selects the register-staged kernel above).  The register-staged kernel
// spends half its time staging (profiles/r5_attn_f16_phase_skips.log): the f32 tile loads into
// registers one tile ahead, the split, and the V^T image written as 2-byte transposing stores.
// Here, per 32-key tile:
//   * DMA: the raw f32 K and V rows go global -> LDS by global_load_lds_dwordx4 (no registers, no
//     LDS stores), two tiles ahead of the MFMAs; wave w moves rows 8 w .. 8 w + 7 of K and of V.
//   * split (once per block, one tile ahead): wave w reads its 8 raw rows back, splits them into
//     the staged-operand pieces (h = f16(x), l = f16((x - h) 2^11)), keeps the range statistics
//     and writes the pieces ROW-major with 16-byte stores: K as the register-staged kernel's image,
//     V key-major.
//   * MFMAs: K fragments as 16-byte row reads; the V^T fragments of O^T += V^T P'^T by
//     ds_read_b64_tr_b16 from the key-major V image (each 16-lane group reads a 4-key x 16-dim
//     block and receives it dim-major; two per fragment), so V is never stored transposed.
// One barrier per tile.  LDS per block: raw ring 2 x 16 KiB (row r = key 32 t + r, clamped to
// Lk - 1 so the masked keys of a ragged tile are real rows; 256-B rows, 16-byte chunk c' holding
// dims 4 (c' ^ (r & 15)) .. + 3) + pieces 2 x 16 KiB (K h, K l, V h, V l: 32 rows x 128 B; K chunk
// c at c ^ ((r >> 1) & 7), V chunk c at c ^ (((r >> 1) & 1) << 2): the K row reads, the transposed V
// reads and the piece stores are bank-conflict-free).  Same pieces and MFMA order as the
// register-staged kernel: bitwise-equal results; the range checks and the bf16x6 re-run of the
// flagged blocks are unchanged.  Waves whose 32 queries all lie past Lq only stage.
// ---------------------------------------------------------------------------------------------
constexpr int AD_WAVES = 4;
constexpr int AD_RAW_B = 2 * 32 * 256;  // one raw stage: K and V, 32 keys x 64 f32
constexpr int AD_PLANE_B = 32 * 128;    // one piece plane: 32 keys x 64 f16
constexpr int AD_PCS_B = 4 * AD_PLANE_B;

__device__ __forceinline__ void ad_glds16(const float* gsrc, const void* lds_dst) {
  const uint32_t dst = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst;
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(dst))
               : "memory");
}
// all of this wave's LDS-DMAs landed, then the block barrier (no __syncthreads: its fence is not
// needed for LDS and would be placed by the compiler without the DMAs in view)
__device__ __forceinline__ void ad_dma_barrier() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// x - f32(h) for the f16 in the low / high half of packed h, exactly (v_fma_mix_f32 reads the f16
// operand in place: one instruction instead of converting h back and subtracting)
__device__ __forceinline__ float ad_rem_lo(uint32_t h, float x) {
  float r;
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(x));
  return r;
}
__device__ __forceinline__ float ad_rem_hi(uint32_t h, float x) {
  float r;
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(x));
  return r;
}
// ah_split_a / ah_split_w with the remainders formed by v_fma_mix_f32 (the same bits)
__device__ __forceinline__ void ad_split_a(float x, float y, uint32_t& h, uint32_t& l) {
  h = ah_pk(x, y);
  l = ah_pk(ad_rem_lo(h, x) * 2048.f, ad_rem_hi(h, y) * 2048.f);
}
__device__ __forceinline__ void ad_split_w(float x, float y, uint32_t& h, uint32_t& l) {
  h = ah_pk(x, y);
  l = ah_pk(ad_rem_lo(h, x), ad_rem_hi(h, y));
}
__device__ __forceinline__ void ad_split8(float4 x0, float4 x1, f16x8& h, f16x8& l) {
  uint32_t hh[4], ll[4];
  ad_split_a(x0.x, x0.y, hh[0], ll[0]);
  ad_split_a(x0.z, x0.w, hh[1], ll[1]);
  ad_split_a(x1.x, x1.y, hh[2], ll[2]);
  ad_split_a(x1.z, x1.w, hh[3], ll[3]);
  h = __builtin_bit_cast(f16x8, make_uint4(hh[0], hh[1], hh[2], hh[3]));
  l = __builtin_bit_cast(f16x8, make_uint4(ll[0], ll[1], ll[2], ll[3]));
}
__device__ __forceinline__ float ad_amax4(float m, float4 x) {
  return fmaxf(m, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
}
// max(m, |x|, |y|) as one v_max3_f32 with source modifiers (fmaxf(m, fabsf(x)) also canonicalises
// each input first, one more instruction per element; the values are the same)
__device__ __forceinline__ float ad_max3abs(float m, float x, float y) {
  float r;
  asm("v_max3_f32 %0, |%1|, |%2|, %3" : "=v"(r) : "v"(x), "v"(y), "v"(m));
  return r;
}
__device__ __forceinline__ float ad_maxabs(float m, float x) {
  float r;
  asm("v_max_f32_e64 %0, %1, |%2|" : "=v"(r) : "v"(m), "v"(x));
  return r;
}
// s_waitcnt vmcnt(N) lgkmcnt(0), then the block barrier
template <int N>
__device__ __forceinline__ void ad_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
typedef short ad_s4 __attribute__((ext_vector_type(4)));
// 4 keys x 4 dims of a piece plane, delivered transposed across the 16-lane group (T10)
__device__ __forceinline__ ad_s4 ad_tr(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) ad_s4*)p);
}

// DBG (profiling phase skips of the PIPE form, RMBX_ATTN_F16_DBG with RMBX_ATTN_DMA=2; wrong results,
// timing only): 1 = no splits in the loop, 2 = no softmax (the tile's S^T is not read), 4 = no DMA in
// the loop, 8 = no S^T MFMAs, 16 = no PV MFMAs
// ONE (with PIPE = false): a single raw stage -- each wave splits tile t + 1 from it, then DMAs tile
// t + 2 into the rows it just read, so the DMA still lands under a tile of compute -- 48 KiB of LDS
// and at most 168 registers: three blocks (three waves per SIMD) per CU instead of two
template <bool PIPE, int DBG = 0, bool ONE = false>
__global__ void __launch_bounds__(64 * AD_WAVES) __attribute__((amdgpu_waves_per_eu(ONE ? 3 : 1)))
attn_fwd_f16x3d_kernel(AttnF32Args a) {
  // raw stages: 2, or 3 in the PIPE form (each DMA then has two key tiles of compute to land in);
  // 3 x 16 + 2 x 16 KiB = 80 KiB, two blocks per CU, so the range statistics (sDim: per head
  // dimension the max |v| over the keys, sKmax: the max |k|, f32 bits) take the raw ring's first
  // bytes once the loop is done
  static_assert(!(PIPE && ONE), "the single-stage form is the plain (PIPE = false) loop");
  constexpr int NR = PIPE ? 3 : (ONE ? 1 : 2);
  __shared__ __attribute__((aligned(16))) unsigned char sR[NR * AD_RAW_B];
  __shared__ __attribute__((aligned(16))) unsigned char sP[2 * AD_PCS_B];
  uint32_t* const sDim = reinterpret_cast<uint32_t*>(sR);
  uint32_t* const sKmax = sDim + 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // block -> (head, query part): plain order, or (xcd_map) the parts of a head on one XCD in
  // consecutive dispatch slots (block bid runs on XCD bid & 7), so the second and third parts'
  // K / V DMAs hit that XCD's L2 instead of HBM
  int bh, part;
  if (a.xcd_map) {
    const int j = blockIdx.x >> 3;
    part = j % a.parts;
    bh = (j / a.parts) * 8 + (blockIdx.x & 7);
  } else {
    bh = blockIdx.x / a.parts;
    part = blockIdx.x - bh * a.parts;
  }
  const int b = bh / a.heads, hd = bh - b * a.heads;
  const int r32 = lane & 31, kh = lane >> 5;
  const int q0 = (part * AD_WAVES + wave) * 32;  // the wave's first query (wave-uniform)
  const bool live = q0 < a.Lq;
  const int qi = q0 + r32;
  const bool q_ok = qi < a.Lq;
  const float* kbase = a.k + (size_t)b * a.k_bstride + hd * 64;
  const float* vbase = a.v + (size_t)b * a.v_bstride + hd * 64;
  const int nt = (a.Lk + 31) >> 5;
  auto stage = [](int t) { return PIPE ? t % 3 : (ONE ? 0 : t & 1); };

  const int dr = lane >> 4, dc = lane & 15;
  // DMA of one operand's raw rows (k = 0: K, 1: V) of tile t into its raw stage: lane -> row
  // 8 wave + 4 i + dr, 16-byte chunk dc ^ (row & 15); the per-lane offsets are formed once, the tile's
  // row offset is wave-uniform, and only a ragged last tile clamps its rows to Lk - 1
  long long doff[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 8 * wave + 4 * i + dr, c = dc ^ (r & 15);
    doff[0][i] = (long long)r * a.k_rstride + 4 * c;
    doff[1][i] = (long long)r * a.v_rstride + 4 * c;
  }
  auto dma_op = [&](int t, int k) {
    unsigned char* st = sR + stage(t) * AD_RAW_B + k * 32 * 256;
    const float* base = k ? vbase : kbase;
    const long long rs = k ? a.v_rstride : a.k_rstride;
    const bool clamp = 32 * t + 32 > a.Lk;  // (wave-uniform)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r0 = 8 * wave + 4 * i, r = r0 + dr;
      long long o = (long long)(32 * t) * rs + doff[k][i];
      if (clamp && 32 * t + r >= a.Lk) o = (long long)(a.Lk - 1) * rs + 4 * (dc ^ (r & 15));
      ad_glds16(base + o, st + r0 * 256);
    }
  };
  auto dma_tile = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r0 = 8 * wave + 4 * i, r = r0 + dr;
      int key = 32 * t + r;
      key = key < a.Lk ? key : a.Lk - 1;
      const int c = dc ^ (r & 15);
      unsigned char* st = sR + stage(t) * AD_RAW_B;
      ad_glds16(kbase + (size_t)key * a.k_rstride + 4 * c, st + r0 * 256);
      ad_glds16(vbase + (size_t)key * a.v_rstride + 4 * c, st + 32 * 256 + r0 * 256);
    }
  };
  // split of tile t: lane -> raw row rr = 8 wave + lane / 8, dims 8 jj .. 8 jj + 7 (the rows this
  // wave's DMAs wrote: the raw stages are wave-private)
  const int rr = 8 * wave + (lane >> 3), jj = lane & 7;
  float kmx = 0.f;      // max |k| of this lane's elements
  float vmx[8] = {};    // max |v| of dims 8 jj + e over this lane's keys
  auto split_k = [&](int t) {
    const unsigned char* raw = sR + stage(t) * AD_RAW_B + rr * 256;
    unsigned char* pcs = sP + (t & 1) * AD_PCS_B + rr * 128;
    const int sw = rr & 15;
    const float4 x0 = *reinterpret_cast<const float4*>(raw + (((2 * jj) ^ sw) << 4));
    const float4 x1 = *reinterpret_cast<const float4*>(raw + (((2 * jj + 1) ^ sw) << 4));
    kmx = ad_max3abs(ad_max3abs(ad_max3abs(ad_max3abs(kmx, x0.x, x0.y), x0.z, x0.w), x1.x, x1.y), x1.z, x1.w);
    f16x8 h, l;
    ad_split8(x0, x1, h, l);
    const int kc = jj ^ ((rr >> 1) & 7);
    *reinterpret_cast<f16x8*>(pcs + (kc << 4)) = h;
    *reinterpret_cast<f16x8*>(pcs + AD_PLANE_B + (kc << 4)) = l;
  };
  auto split_v = [&](int t) {
    const unsigned char* raw = sR + stage(t) * AD_RAW_B + rr * 256;
    unsigned char* pcs = sP + (t & 1) * AD_PCS_B + rr * 128;
    const int sw = rr & 15;
    const float4 y0 = *reinterpret_cast<const float4*>(raw + 32 * 256 + (((2 * jj) ^ sw) << 4));
    const float4 y1 = *reinterpret_cast<const float4*>(raw + 32 * 256 + (((2 * jj + 1) ^ sw) << 4));
    vmx[0] = ad_maxabs(vmx[0], y0.x);
    vmx[1] = ad_maxabs(vmx[1], y0.y);
    vmx[2] = ad_maxabs(vmx[2], y0.z);
    vmx[3] = ad_maxabs(vmx[3], y0.w);
    vmx[4] = ad_maxabs(vmx[4], y1.x);
    vmx[5] = ad_maxabs(vmx[5], y1.y);
    vmx[6] = ad_maxabs(vmx[6], y1.z);
    vmx[7] = ad_maxabs(vmx[7], y1.w);
    f16x8 h, l;
    ad_split8(y0, y1, h, l);
    const int vc = jj ^ (((rr >> 1) & 1) << 2);
    *reinterpret_cast<f16x8*>(pcs + 2 * AD_PLANE_B + (vc << 4)) = h;
    *reinterpret_cast<f16x8*>(pcs + 3 * AD_PLANE_B + (vc << 4)) = l;
  };

  dma_tile(0);
  if (!ONE && nt > 1) dma_tile(1);
  if (PIPE && nt > 2) dma_tile(2);

  // Q pieces as in the register-staged kernel (dims 16 s + 8 kh .. +7 of query qi, scaled by the
  // query's power of two 2^t; fq[s][2] = 2^-11 qh)
  f16x8 fq[4][3];
  float c = a.scale_log2;
  bool q_inf = false;
  {
    const float* qp = a.q + (size_t)b * a.q_bstride + (size_t)(q_ok ? qi : 0) * a.q_rstride + hd * 64 + 8 * kh;
    float4 x[4][2];
    float qm = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      x[s][0] = *reinterpret_cast<const float4*>(qp + 16 * s);
      x[s][1] = *reinterpret_cast<const float4*>(qp + 16 * s + 4);
      qm = ad_amax4(ad_amax4(qm, x[s][0]), x[s][1]);
    }
    qm = fmaxf(qm, __shfl_xor(qm, 32));
    int t = 0;
    if (qm > 0.f && qm < INFINITY) {
      int e;
      frexpf(qm, &e);
      t = 14 - e;
      t = t < -100 ? -100 : (t > 100 ? 100 : t);
    } else if (qm == INFINITY) {
      q_inf = true;
    }
    c = ldexpf(c, -t);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      uint32_t h[4], l[4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float4 y = make_float4(ldexpf(x[s][u].x, t), ldexpf(x[s][u].y, t), ldexpf(x[s][u].z, t),
                                     ldexpf(x[s][u].w, t));
        ah_split_w(y.x, y.y, h[2 * u], l[2 * u]);
        ah_split_w(y.z, y.w, h[2 * u + 1], l[2 * u + 1]);
      }
      fq[s][0] = __builtin_bit_cast(f16x8, make_uint4(h[0], h[1], h[2], h[3]));
      fq[s][1] = __builtin_bit_cast(f16x8, make_uint4(l[0], l[1], l[2], l[3]));
      fq[s][2] = fq[s][0] * (_Float16)0.00048828125f;
    }
  }

  const bool ragged = (a.Lk & 31) != 0;
  // transposed V reads: lane 4 q + p of its 16-lane group g supplies key row q, dims dv .. dv + 3
  // (the at_sigma order: lane i of the group, A row 16 (g & 1) + i, receives dim sigma(row))
  const int vq = (lane & 15) >> 2, vp = lane & 3;
  const int dv = 16 * (vp & 1) + 8 * ((lane >> 4) & 1) + 4 * (vp >> 1);
  f32x16 acc0 = {}, acc1 = {};
  float m_run = -INFINITY, l_run = 0.f;
  // S^T of tile t from the K pieces in piece stage t & 1
  auto s_tile = [&](int t) {
    const unsigned char* pc = sP + (t & 1) * AD_PCS_B;
    f32x16 s = {};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int off = r32 * 128 + (((2 * ks + kh) ^ ((r32 >> 1) & 7)) << 4);
      const f16x8 k0 = *reinterpret_cast<const f16x8*>(pc + off);
      const f16x8 k1 = *reinterpret_cast<const f16x8*>(pc + AD_PLANE_B + off);
      if constexpr (DBG & 8) {
        s[ks] += (float)k0[0] + (float)k1[1];
      } else {
        s = __builtin_amdgcn_mfma_f32_32x32x16_f16(k1, fq[ks][2], s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0, fq[ks][1], s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0, fq[ks][0], s, 0, 0, 0);
      }
    }
    return s;
  };
  // O^T += V^T P'^T from the V pieces at pc (V^T fragments of k-step u: elements 0-3 = keys
  // 16 u + 4 kh + 0..3, elements 4-7 = keys 16 u + 8 + 4 kh + 0..3, the keys the P' registers hold)
  auto pv_part = [&](const unsigned char* pc, const f16x8 (&fp)[2][3]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      ad_s4 w[2][2][2];  // [key block][dims d / d + 32][piece]
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const int key = 16 * u + 8 * k2 + 4 * kh + vq;
        const int fl = ((key >> 1) & 1) << 2;
#pragma unroll
        for (int dd = 0; dd < 2; ++dd) {
          const int d = dv + 32 * dd;
          const unsigned char* p = pc + 2 * AD_PLANE_B + key * 128 + ((((d >> 3) ^ fl) << 4) | ((d & 7) << 1));
          w[k2][dd][0] = ad_tr(p);
          w[k2][dd][1] = ad_tr(p + AD_PLANE_B);
        }
      }
      auto cat = [](ad_s4 lo, ad_s4 hi) {
        return __builtin_bit_cast(f16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      };
      const f16x8 v0h = cat(w[0][0][0], w[1][0][0]), v0l = cat(w[0][0][1], w[1][0][1]);
      const f16x8 v1h = cat(w[0][1][0], w[1][1][0]), v1l = cat(w[0][1][1], w[1][1][1]);
      if constexpr ((DBG & 16) != 0) {
        acc0[u] += (float)v0l[0] + (float)v1h[1] + (float)fp[u][2][0];
        continue;
      }
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v0l, fp[u][2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1l, fp[u][2], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v0h, fp[u][1], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1h, fp[u][1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v0h, fp[u][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1h, fp[u][0], acc1, 0, 0, 0);
    }
  };
  // online softmax of S^T (tile t) and O^T += V^T P'^T from the V pieces in piece stage t & 1
  // (next: S^T of tile t + 1 is issued after the max / rescale, beside this tile's exponentials)
  auto soft_pv = [&](f32x16 s, int t, bool next, f32x16& s_next) {
    const unsigned char* pc = sP + (t & 1) * AD_PCS_B;
    if constexpr ((DBG & 2) != 0) {
      if (next) s_next = s_tile(t + 1);
      f16x8 fp[2][3];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 3; ++i) fp[u][i] = fq[u][i];
      l_run += s[0];
      pv_part(pc, fp);
      return;
    }
    if (ragged && t == nt - 1) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (32 * t + 4 * kh + (j & 3) + 8 * (j >> 2) >= a.Lk) s[j] = -INFINITY;
    }
    float mx = s[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) mx = fmaxf(mx, s[j]);
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float m_new = fmaxf(m_run, mx);
    if (__any(m_new != m_run)) {
      const float alpha = exp2f((m_run - m_new) * c);
      l_run *= alpha;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        acc0[j] *= alpha;
        acc1[j] *= alpha;
      }
      m_run = m_new;
    }
    const float mc = m_run * c;
    if (next) s_next = s_tile(t + 1);
    f16x8 fp[2][3];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      uint32_t h[4], l[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // (v_exp_f32 alone: exp2f's denormal-result path only changes p' < 2^-112, which is zero
        // in the f16 pieces and below the ulp of l >= 2^14)
        const float pa = __builtin_amdgcn_exp2f(fmaf(s[8 * u + 2 * e], c, -mc)) * 16384.f;
        const float pb = __builtin_amdgcn_exp2f(fmaf(s[8 * u + 2 * e + 1], c, -mc)) * 16384.f;
        l_run += pa + pb;
        ad_split_w(pa, pb, h[e], l[e]);
      }
      fp[u][0] = __builtin_bit_cast(f16x8, make_uint4(h[0], h[1], h[2], h[3]));
      fp[u][1] = __builtin_bit_cast(f16x8, make_uint4(l[0], l[1], l[2], l[3]));
      fp[u][2] = fp[u][0] * (_Float16)0.00048828125f;
    }
    pv_part(pc, fp);
  };

  if constexpr (ONE) {
    ad_dma_barrier();  // tile 0 landed
    split_k(0);
    split_v(0);
    if (nt > 1) dma_tile(1);  // into the rows this wave's split just read
    for (int t = 0; t < nt; ++t) {
      ad_dma_barrier();  // tile t + 1 landed; tile t's pieces written; every wave is past tile t - 1
      if (t + 1 < nt) {
        split_k(t + 1);
        split_v(t + 1);
        if (t + 2 < nt) dma_tile(t + 2);
      }
      if (!live) continue;
      f32x16 unused;
      soft_pv(s_tile(t), t, false, unused);
    }
  } else if constexpr (!PIPE) {
    ad_dma_barrier();  // tile 0 (and 1) landed; sDim / sKmax cleared
    split_k(0);
    split_v(0);
    for (int t = 0; t < nt; ++t) {
      ad_dma_barrier();  // tile t + 1 landed; tile t's pieces written; every wave is past tile t - 1
      if (t + 2 < nt) dma_tile(t + 2);
      if (t + 1 < nt) {
        split_k(t + 1);
        split_v(t + 1);
      }
      if (!live) continue;
      f32x16 unused;
      soft_pv(s_tile(t), t, false, unused);
    }
  } else {
    // K runs one tile ahead of V, so S^T of tile t + 1 is on the matrix cores while the softmax of
    // tile t is on the vector ALUs, and the raw ring has three stages, so a DMA lands while two key
    // tiles compute.  Iteration t: DMA K(t + 4) and V(t + 3), split K(t + 2) and V(t + 1),
    // S^T(t + 1), softmax and PV of tile t.  The raw stages are wave-private (each wave splits the
    // rows its own DMAs wrote), so the wait at the top of iteration t covers only this wave's DMAs
    // of iteration t - 2 and older (those of t - 1 stay in flight); the barrier publishes the pieces
    // K(t + 1) / V(t) and retires every wave's reads of K(t) / V(t - 1), whose piece stages
    // iteration t overwrites.  Same pieces, same MFMA order: bitwise-equal to PIPE = false.
    ad_dma_barrier();  // K, V raw of tiles 0, 1, 2 landed
    split_k(0);
    split_v(0);
    if (nt > 1) split_k(1);
    if (nt > 3) {
      dma_op(3, 0);  // K(3) into stage 0 (this wave's own split of K(0) read it)
      ad_wait_barrier<2>();  // K pieces 0, 1 and V pieces 0 published; K(3) in flight
    } else {
      ad_wait_barrier<0>();
    }
    f32x16 s_cur = {};
    if (live) s_cur = s_tile(0);
    for (int t = 0; t < nt - 1; ++t) {
      // this wave's DMAs of iteration t - 1 (the prologue's K(3) for t = 0) may stay in flight
      const int inflight = t == 0 ? (nt > 3 ? 2 : 0) : (t + 3 < nt ? 2 : 0) + (t + 2 < nt ? 2 : 0);
      if (inflight == 4)
        ad_wait_barrier<4>();
      else if (inflight == 2)
        ad_wait_barrier<2>();
      else
        ad_wait_barrier<0>();
      if (!(DBG & 4)) {
        if (t + 4 < nt) dma_op(t + 4, 0);  // into stage (t + 1) % 3: K(t + 1) was split at t - 1
        if (t + 3 < nt) dma_op(t + 3, 1);  // into stage t % 3: V(t) was split at t - 1
      }
      if (!(DBG & 1)) {
        if (t + 2 < nt) split_k(t + 2);
        split_v(t + 1);
      }
      if (!live) continue;
      f32x16 s_next;
      soft_pv(s_cur, t, true, s_next);
      s_cur = s_next;
    }
    ad_dma_barrier();  // V pieces of the last tile published
    if (live) {
      f32x16 unused;
      soft_pv(s_cur, nt - 1, false, unused);
    }
  }
  // the raw ring is dead (every DMA retired, every split done): its first bytes hold the range
  // statistics
  if (tid < 64) sDim[tid] = 0u;
  if (tid < 2) sKmax[tid] = 0u;  // [0]: max |k|, [1]: the block's flag
  __syncthreads();
  // range check (the register-staged kernel's conditions): any |k|, |v| >= 2^15 or a non-finite
  // query, the block's max |k| in (0, 2^-6), a dimension's max |v| over the keys in (0, 2^-6)
  float vm = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float x = vmx[e];
    x = fmaxf(x, __shfl_xor(x, 8));
    x = fmaxf(x, __shfl_xor(x, 16));
    x = fmaxf(x, __shfl_xor(x, 32));
    vmx[e] = x;
    vm = fmaxf(vm, x);
  }
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (vmx[e] > 0.f) atomicMax(&sDim[8 * jj + e], __float_as_uint(vmx[e]));
  }
  if (kmx > 0.f) atomicMax(sKmax, __float_as_uint(kmx));
  __syncthreads();
  bool flag = q_inf || kmx >= AH_BIG || vm >= AH_BIG;
  if (tid < 64) {
    const float m = __uint_as_float(sDim[tid]);
    flag = flag || (m > 0.f && m < AH_TINY);
  }
  if (tid == 0) {
    const float km = __uint_as_float(*sKmax);
    flag = flag || (km > 0.f && km < AH_TINY);
  }
  // the block's OR of the flags through the LDS word sKmax[1] (__syncthreads_or would allocate
  // 256 B of LDS for its reduction: two 80-KiB blocks per CU leave none)
  if (__any(flag) && lane == 0) atomicOr(sKmax + 1, 1u);
  __syncthreads();
  const int any = sKmax[1] != 0u;
  if (tid == 0) a.redo[bh * a.parts + part] = any;  // (the bf16x6 kernel's block order)
  if (any) return;
  const float l_tot = l_run + __shfl_xor(l_run, 32);
  if (!q_ok) return;
  const float inv = 1.f / l_tot;
  float* op = a.o + ((size_t)b * a.Lq + qi) * a.o_rstride + hd * 64 + 16 * kh;
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) {
    *reinterpret_cast<float4*>(op + 4 * q4) =
        make_float4(acc0[4 * q4] * inv, acc0[4 * q4 + 1] * inv, acc0[4 * q4 + 2] * inv, acc0[4 * q4 + 3] * inv);
    *reinterpret_cast<float4*>(op + 32 + 4 * q4) =
        make_float4(acc1[4 * q4] * inv, acc1[4 * q4 + 1] * inv, acc1[4 * q4 + 2] * inv, acc1[4 * q4 + 3] * inv);
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

extern "C" int rmbx_attention_f32(const float* q, const float* k, const float* v, float* out, int B, int heads, int Lq,
                                  int Lk, long long q_bstride, int q_rstride, long long k_bstride, int k_rstride,
                                  long long v_bstride, int v_rstride, float scale, void* stream) {
  RMBX_CHECK_ARG(q && k && v && out, "rmbx_attention_f32: null pointer");
  RMBX_CHECK_ARG(B >= 0 && heads > 0 && Lq > 0 && Lk > 0, "rmbx_attention_f32: bad geometry");
  RMBX_CHECK_ARG(scale > 0.f, "rmbx_attention_f32: scale must be positive");
  RMBX_CHECK_ARG(q_rstride % 4 == 0 && k_rstride % 4 == 0 && v_rstride % 4 == 0 && q_bstride % 4 == 0 &&
                     k_bstride % 4 == 0 && v_bstride % 4 == 0,
                 "rmbx_attention_f32: strides must be multiples of 4 elements");
  RMBX_CHECK_ARG((((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)out) & 15) == 0,
                 "rmbx_attention_f32: pointers must be 16-byte aligned");
  if (B == 0) return RMBX_OK;
  rmbx::AttnF32Args a;
  a.q = q;
  a.k = k;
  a.v = v;
  a.o = out;
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
  // 4 or 5 waves (one 32-query group each; >= 256 threads stage a key tile in 4 chunks each)
  const int ngroups = (Lq + 31) / 32;
  const int waves = ngroups >= rmbx::AF_MAX_WAVES ? rmbx::AF_MAX_WAVES : 4;
  a.parts = (ngroups + waves - 1) / waves;
  const long long nblocks = (long long)B * heads * a.parts;
  RMBX_CHECK_ARG(nblocks < (1ll << 31), "rmbx_attention_f32: grid too large");
  const char* dbg_env = std::getenv("RMBX_ATTN_F32_DBG");
  const int dbg = dbg_env ? std::atoi(dbg_env) : 0;
  const dim3 g((unsigned)nblocks), blk(64 * waves);
  switch (dbg) {  // diagnostic phase skips: 1 = no S MFMAs, 2 = no softmax, 4 = no PV MFMAs, 8 = no tile loads
    case 0: hipLaunchKernelGGL(rmbx::attn_fwd_f32_kernel<0>, g, blk, 0, (hipStream_t)stream, a); break;
    case 1: hipLaunchKernelGGL(rmbx::attn_fwd_f32_kernel<1>, g, blk, 0, (hipStream_t)stream, a); break;
    case 2: hipLaunchKernelGGL(rmbx::attn_fwd_f32_kernel<2>, g, blk, 0, (hipStream_t)stream, a); break;
    case 4: hipLaunchKernelGGL(rmbx::attn_fwd_f32_kernel<4>, g, blk, 0, (hipStream_t)stream, a); break;
    case 8: hipLaunchKernelGGL(rmbx::attn_fwd_f32_kernel<8>, g, blk, 0, (hipStream_t)stream, a); break;
    case 5: hipLaunchKernelGGL(rmbx::attn_fwd_f32_kernel<5>, g, blk, 0, (hipStream_t)stream, a); break;
    case 10: hipLaunchKernelGGL(rmbx::attn_fwd_f32_kernel<10>, g, blk, 0, (hipStream_t)stream, a); break;
    default: RMBX_CHECK_ARG(false, "rmbx_attention_f32: RMBX_ATTN_F32_DBG=%d not instantiated", dbg);
  }
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_attention_f32x6(const float* q, const float* k, const float* v, float* out, int B, int heads,
                                    int Lq, int Lk, long long q_bstride, int q_rstride, long long k_bstride,
                                    int k_rstride, long long v_bstride, int v_rstride, float scale, void* stream) {
  RMBX_CHECK_ARG(q && k && v && out, "rmbx_attention_f32x6: null pointer");
  RMBX_CHECK_ARG(B >= 0 && heads > 0 && Lq > 0 && Lk > 0, "rmbx_attention_f32x6: bad geometry");
  RMBX_CHECK_ARG(scale > 0.f, "rmbx_attention_f32x6: scale must be positive");
  RMBX_CHECK_ARG(q_rstride % 4 == 0 && k_rstride % 4 == 0 && v_rstride % 4 == 0 && q_bstride % 4 == 0 &&
                     k_bstride % 4 == 0 && v_bstride % 4 == 0,
                 "rmbx_attention_f32x6: strides must be multiples of 4 elements");
  RMBX_CHECK_ARG((((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)out) & 15) == 0,
                 "rmbx_attention_f32x6: pointers must be 16-byte aligned");
  if (B == 0) return RMBX_OK;
  rmbx::AttnF32Args a;
  a.q = q;
  a.k = k;
  a.v = v;
  a.o = out;
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
  const int ngroups = (Lq + 31) / 32;
  const int waves = ngroups >= rmbx::AX_MAX_WAVES ? rmbx::AX_MAX_WAVES : 4;
  a.parts = (ngroups + waves - 1) / waves;
  const long long nblocks = (long long)B * heads * a.parts;
  RMBX_CHECK_ARG(nblocks < (1ll << 31), "rmbx_attention_f32x6: grid too large");
  hipLaunchKernelGGL(rmbx::attn_fwd_f32x6_kernel, dim3((unsigned)nblocks), dim3(64 * waves), 0, (hipStream_t)stream, a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_attention_f16x3(const float* q, const float* k, const float* v, float* out, int* redo, int B,
                                    int heads, int Lq, int Lk, long long q_bstride, int q_rstride, long long k_bstride,
                                    int k_rstride, long long v_bstride, int v_rstride, float scale, void* stream) {
  RMBX_CHECK_ARG(q && k && v && out && redo, "rmbx_attention_f16x3: null pointer");
  RMBX_CHECK_ARG(B >= 0 && heads > 0 && Lq > 0 && Lk > 0, "rmbx_attention_f16x3: bad geometry");
  RMBX_CHECK_ARG(scale > 0.f, "rmbx_attention_f16x3: scale must be positive");
  RMBX_CHECK_ARG(q_rstride % 4 == 0 && k_rstride % 4 == 0 && v_rstride % 4 == 0 && q_bstride % 4 == 0 &&
                     k_bstride % 4 == 0 && v_bstride % 4 == 0,
                 "rmbx_attention_f16x3: strides must be multiples of 4 elements");
  RMBX_CHECK_ARG((((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)out) & 15) == 0,
                 "rmbx_attention_f16x3: pointers must be 16-byte aligned");
  if (B == 0) return RMBX_OK;
  rmbx::AttnF32Args a;
  a.q = q;
  a.k = k;
  a.v = v;
  a.o = out;
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
  a.redo = redo;
  // RMBX_ATTN_XCD=1 (read per launch): the query parts of a head paired on one XCD -- measured no
  // faster (1.774 vs 1.756 ms encoder self-attention, profiles/r4_attention_xcd_pairing_ab.log):
  // the kernel is not bound by its K / V reads
  const char* xe = std::getenv("RMBX_ATTN_XCD");
  a.xcd_map = xe && std::atoi(xe) != 0;
  const int ngroups = (Lq + 31) / 32;
  // waves per block (RMBX_ATTN_WAVES, read per launch): 4 (default) = four 32-query groups per
  // block (302 queries: 3 parts; two 4-wave blocks per CU at 215 registers: two waves on every
  // SIMD), 5 = up to five groups (2 parts; one 5-wave block per CU, so one SIMD carries two waves
  // and three carry one): 1.41 vs 1.75 ms encoder self-attention at 1024 envs
  // (profiles/r4_attention_waves_ab.log)
  // RMBX_ATTN_DMA (read per launch): 3 (default) = the LDS-DMA-staged kernel with one raw stage
  // (48 KiB, <= 168 registers: three blocks per CU), 1 = the same with two raw stages (64 KiB, two
  // blocks per CU), 2 = two-stage with K one tile ahead of V (S^T of the next tile beside the
  // softmax) and a three-stage raw ring, 0 = the register-staged kernel.  Encoder self-attention at
  // 1024 envs, one box (profiles/r6_attn_dma_ab.log): 1.397 (0) / 1.227 (1) / 1.233 (2) / 1.095 ms (3),
  // each DMA form with XCD pairing -- the kernel is latency-bound (each phase skip saves 0.15-0.25 ms
  // of 1.24, profiles/r6_attn_phases.log), so the third block per CU pays and the skew does not.
  // The DMA forms pair the parts of a head on one XCD unless RMBX_ATTN_XCD=0 (their K / V DMAs then
  // hit L2 for the second and third parts)
  const char* me = std::getenv("RMBX_ATTN_DMA");
  const int dma_form = me ? std::atoi(me) : 3;
  if (dma_form != 0) {
    a.parts = (ngroups + rmbx::AD_WAVES - 1) / rmbx::AD_WAVES;
    const long long nb = (long long)B * heads * a.parts;
    a.xcd_map = (!xe || std::atoi(xe) != 0) && a.parts > 1 && ((long long)B * heads) % 8 == 0;
    RMBX_CHECK_ARG(nb < (1ll << 31), "rmbx_attention_f16x3: grid too large");
    const dim3 g((unsigned)nb), blk(64 * rmbx::AD_WAVES);
    const char* de = std::getenv("RMBX_ATTN_F16_DBG");  // profiling phase skips (read per launch)
    const int dbg = de ? std::atoi(de) : 0;
    if (dma_form == 2) {
      switch (dbg) {
        case 0: hipLaunchKernelGGL((rmbx::attn_fwd_f16x3d_kernel<true, 0>), g, blk, 0, (hipStream_t)stream, a); break;
        case 1: hipLaunchKernelGGL((rmbx::attn_fwd_f16x3d_kernel<true, 1>), g, blk, 0, (hipStream_t)stream, a); break;
        case 2: hipLaunchKernelGGL((rmbx::attn_fwd_f16x3d_kernel<true, 2>), g, blk, 0, (hipStream_t)stream, a); break;
        case 4: hipLaunchKernelGGL((rmbx::attn_fwd_f16x3d_kernel<true, 4>), g, blk, 0, (hipStream_t)stream, a); break;
        case 8: hipLaunchKernelGGL((rmbx::attn_fwd_f16x3d_kernel<true, 8>), g, blk, 0, (hipStream_t)stream, a); break;
        case 16: hipLaunchKernelGGL((rmbx::attn_fwd_f16x3d_kernel<true, 16>), g, blk, 0, (hipStream_t)stream, a); break;
        case 24: hipLaunchKernelGGL((rmbx::attn_fwd_f16x3d_kernel<true, 24>), g, blk, 0, (hipStream_t)stream, a); break;
        case 5: hipLaunchKernelGGL((rmbx::attn_fwd_f16x3d_kernel<true, 5>), g, blk, 0, (hipStream_t)stream, a); break;
        default: RMBX_CHECK_ARG(false, "rmbx_attention_f16x3: RMBX_ATTN_F16_DBG=%d not instantiated", dbg);
      }
    } else if (dma_form == 3) {
      hipLaunchKernelGGL((rmbx::attn_fwd_f16x3d_kernel<false, 0, true>), g, blk, 0, (hipStream_t)stream, a);
    } else {
      hipLaunchKernelGGL(rmbx::attn_fwd_f16x3d_kernel<false>, g, blk, 0, (hipStream_t)stream, a);
    }
    RMBX_CHECK_LAUNCH();
    hipLaunchKernelGGL(rmbx::attn_fwd_f32x6_kernel, g, blk, 0, (hipStream_t)stream, a);
    RMBX_CHECK_LAUNCH();
    return RMBX_OK;
  }
  const char* we = std::getenv("RMBX_ATTN_WAVES");
  const int wsel = we ? std::atoi(we) : 4;
  const int waves = (wsel == 5 && ngroups >= rmbx::AX_MAX_WAVES) ? rmbx::AX_MAX_WAVES : 4;
  a.parts = (ngroups + waves - 1) / waves;
  const long long nblocks = (long long)B * heads * a.parts;
  RMBX_CHECK_ARG(nblocks < (1ll << 31), "rmbx_attention_f16x3: grid too large");
  // the f16x3 pass, then the bf16x6 kernel over the same blocks: it returns at once for every block
  // the first pass did not flag (redo[block] = 0), so both write each query once
  const char* de = std::getenv("RMBX_ATTN_F16_DBG");  // profiling phase skips (read per launch)
  const int dbg = de ? std::atoi(de) : 0;
  const dim3 g((unsigned)nblocks), blk(64 * waves);
  switch (dbg) {
    case 0: hipLaunchKernelGGL(rmbx::attn_fwd_f16x3_kernel<0>, g, blk, 0, (hipStream_t)stream, a); break;
    case 1: hipLaunchKernelGGL(rmbx::attn_fwd_f16x3_kernel<1>, g, blk, 0, (hipStream_t)stream, a); break;
    case 2: hipLaunchKernelGGL(rmbx::attn_fwd_f16x3_kernel<2>, g, blk, 0, (hipStream_t)stream, a); break;
    case 4: hipLaunchKernelGGL(rmbx::attn_fwd_f16x3_kernel<4>, g, blk, 0, (hipStream_t)stream, a); break;
    case 8: hipLaunchKernelGGL(rmbx::attn_fwd_f16x3_kernel<8>, g, blk, 0, (hipStream_t)stream, a); break;
    case 16: hipLaunchKernelGGL(rmbx::attn_fwd_f16x3_kernel<16>, g, blk, 0, (hipStream_t)stream, a); break;
    case 10: hipLaunchKernelGGL(rmbx::attn_fwd_f16x3_kernel<10>, g, blk, 0, (hipStream_t)stream, a); break;
    case 15: hipLaunchKernelGGL(rmbx::attn_fwd_f16x3_kernel<15>, g, blk, 0, (hipStream_t)stream, a); break;
    default: RMBX_CHECK_ARG(false, "rmbx_attention_f16x3: RMBX_ATTN_F16_DBG=%d not instantiated", dbg);
  }
  RMBX_CHECK_LAUNCH();
  hipLaunchKernelGGL(rmbx::attn_fwd_f32x6_kernel, dim3((unsigned)nblocks), dim3(64 * waves), 0, (hipStream_t)stream, a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
