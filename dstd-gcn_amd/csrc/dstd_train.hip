// Training-path kernels (see dstd_train.h).  Everything here is generic over
// strides and small: the config-5 training batch is 32 sequences per GPU, so
// these kernels favour simple, deterministic reductions (fixed-order partials,
// no float atomics) over the hand-scheduled pipelines of the inference path.
#include <atomic>
#include "dstd_common.h"
#include "dstd_train.h"

#include <algorithm>
#include <type_traits>
#include <stdio.h>
#include <stdlib.h>

namespace dstd {
namespace train {
namespace {

constexpr int kRedThreads = 256;

template <typename F>
__device__ __forceinline__ F block_sum(F v, F* red) {
  // wave64 butterfly, then one value per wave through LDS
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  F t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

// ---------------------------------------------------------------------------
// Strided batched GEMM on v_mfma_f32_16x16x4_f32.
// Workgroup = 4 waves in a 2x2 grid over a TM x TN tile of C; each wave owns a
// (TM/2) x (TN/2) sub-tile = FM x FN MFMA fragments.  K advances 16 at a time
// through LDS tiles As[k][m], Bs[k][n] (k-major: a fragment read is 16
// consecutive floats per k row).  Global loads pick the thread->element map
// whose fastest index is the operand's unit stride, so row- and column-major
// operands both load in contiguous runs.
// ---------------------------------------------------------------------------
// final value of output (gm, gn): into C (with beta), or accumulated into
// its segment's destination (Gemm::nseg)
__device__ __forceinline__ void gemm_store(const Gemm& g, float* Cb, float* Db, int gm, int gn, float v) {
  if (Db) {
    float ac = g.d_A[gn];
    if (g.d_W) ac *= g.d_W[gn];
    if (g.d_R) ac += g.d_R[gn];
    Db[gm * g.c_m + gn * g.c_n] = fmaf(*g.d_alpha, v, ac);
  }
  if (g.nseg) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i < g.nseg && gm >= g.seg[i].row0 && gm < g.seg[i].row0 + g.seg[i].rows) {
        const int r = gm - g.seg[i].row0;
        float* d = gn < g.N - 1 ? g.seg[i].w + (size_t)r * (g.N - 1) + gn : g.seg[i].b + r;
        *d += v;
      }
    }
    return;
  }
  float* c = Cb + gm * g.c_m + gn * g.c_n;
  if (g.beta != 0.f) v += g.beta * *c;
  *c = v;
}

template <int TM, int TN>
__global__ __launch_bounds__(256) void k_gemm(Gemm g, int nsplit, int kch, int kc_len, float* partial) {
  constexpr int KT = 16;
  constexpr int LA = TM + 4, LB = TN + 4;
  constexpr int FM = TM / 32, FN = TN / 32;
  constexpr int EA = TM * KT / 256, EB = TN * KT / 256;
  __shared__ float As[KT * LA];
  __shared__ float Bs[KT * LB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  const int wm = (wave >> 1) * (TM / 2), wn = (wave & 1) * (TN / 2);
  const bool a_kfast = g.a_k < g.a_m;  // the smaller stride runs across lanes (unit stride when there is one)
  const bool b_kfast = g.b_k < g.b_n;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = zero4();

  // work units: (batch, K chunk); a reduce GEMM spreads units over nsplit
  // workgroups (split-K across and within batches), a batched one runs one
  // batch with the whole K per workgroup
  const int nbat = g.nb1 * g.nb2;
  int u_lo, u_hi;
  if (g.reduce) {
    const int units = nbat * kch, per = (units + nsplit - 1) / nsplit;
    u_lo = blockIdx.z * per;
    u_hi = min(units, u_lo + per);
  } else {
    u_lo = blockIdx.z;
    u_hi = u_lo + 1;
  }

  for (int u = u_lo; u < u_hi; ++u) {
    const int b = u / kch, kc = u - b * kch;
    const int b1 = b / g.nb2, b2 = b - b1 * g.nb2;
    const float* Ab = g.A + b1 * g.a_b1 + b2 * g.a_b2;
    const float* Bb = g.B + b1 * g.b_b1 + b2 * g.b_b2;
    const int k_end = min(g.K, (kc + 1) * kc_len);
    // register-staged k-tiles: the next tile's global loads are issued before
    // the current tile's MFMAs, so their latency hides behind the compute
    float ra[EA], rb[EB];
    auto gload = [&](int k0) {
#pragma unroll
      for (int e = 0; e < EA; ++e) {
        const int idx = tid + 256 * e;
        const int m = a_kfast ? idx / KT : idx % TM;
        const int k = a_kfast ? idx % KT : idx / TM;
        const int gm = m0 + m, gk = k0 + k;
        ra[e] = (gm < g.M && gk < k_end) ? Ab[gm * g.a_m + gk * g.a_k] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < EB; ++e) {
        const int idx = tid + 256 * e;
        const int n = b_kfast ? idx / KT : idx % TN;
        const int k = b_kfast ? idx % KT : idx / TN;
        const int gn = n0 + n, gk = k0 + k;
        rb[e] = (gn < g.N && gk < k_end) ? ((g.b_ones_last && gn == g.N - 1) ? 1.f : Bb[gk * g.b_k + gn * g.b_n])
                                         : 0.f;
      }
    };
    int k0 = kc * kc_len;
    if (k0 < k_end) gload(k0);
    for (; k0 < k_end; k0 += KT) {
      __syncthreads();  // the previous tile's fragment reads are done
#pragma unroll
      for (int e = 0; e < EA; ++e) {
        const int idx = tid + 256 * e;
        const int m = a_kfast ? idx / KT : idx % TM;
        const int k = a_kfast ? idx % KT : idx / TM;
        As[k * LA + m] = ra[e];
      }
#pragma unroll
      for (int e = 0; e < EB; ++e) {
        const int idx = tid + 256 * e;
        const int n = b_kfast ? idx / KT : idx % TN;
        const int k = b_kfast ? idx % KT : idx / TN;
        Bs[k * LB + n] = rb[e];
      }
      __syncthreads();
      if (k0 + KT < k_end) gload(k0 + KT);
#pragma unroll
      for (int kk = 0; kk < KT / 4; ++kk) {
        const int kr = kk * 4 + (lane >> 4);
        float av[FM], bv[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) av[i] = As[kr * LA + wm + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < FN; ++j) bv[j] = Bs[kr * LB + wn + j * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x4(av[i], bv[j], acc[i][j]);
      }
    }
  }

  // epilogue: C/D[row = (lane>>4)*4 + r][col = lane&15]
  if (partial) {
    float* P = partial + (size_t)blockIdx.z * g.M * g.N;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gm = m0 + wm + i * 16 + (lane >> 4) * 4 + r, gn = n0 + wn + j * 16 + (lane & 15);
          if (gm < g.M && gn < g.N) P[(size_t)gm * g.N + gn] = acc[i][j][r];
        }
    return;
  }
  const int b1 = g.reduce ? 0 : blockIdx.z / g.nb2, b2 = g.reduce ? 0 : blockIdx.z - b1 * g.nb2;
  float* Cb = g.C + b1 * g.c_b1 + b2 * g.c_b2;
  if (!g.d_out && !g.nseg) {  // plain store: one uniform branch, not one per element
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
        if (gm >= g.M) continue;
        float* row = Cb + gm * g.c_m;
        const float bm = g.bias_m ? g.bias_m[gm] : 0.f;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int gn = n0 + wn + j * 16 + (lane & 15);
          if (gn < g.N) {
            float* c = row + gn * g.c_n;
            float v = fmaf(g.alpha, acc[i][j][r], bm);
            if (g.beta != 0.f) v = fmaf(g.beta, *c, v);
            *c = v;
          }
        }
      }
    return;
  }
  float* Db = g.d_out ? g.d_out + b1 * g.c_b1 + b2 * g.c_b2 : nullptr;
  if (Db && !g.nseg) {
    // C and the adjacency D = d_alpha * C + (d_A (* d_W) (+ d_R)) per column:
    // a lane's columns are the same for all its 4 * FM rows, so the combine
    // is loaded once per column, not per element (gemm_store's order of
    // operations otherwise)
    const float ad = *g.d_alpha;
    float ac[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int gn = min(n0 + wn + j * 16 + (lane & 15), g.N - 1);
      ac[j] = g.d_A[gn];
      if (g.d_W) ac[j] *= g.d_W[gn];
      if (g.d_R) ac[j] += g.d_R[gn];
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
        if (gm >= g.M) continue;
        const float bm = g.bias_m ? g.bias_m[gm] : 0.f;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int gn = n0 + wn + j * 16 + (lane & 15);
          if (gn < g.N) {
            float v = g.alpha * acc[i][j][r];
            if (g.bias_m) v += bm;
            Db[gm * g.c_m + gn * g.c_n] = fmaf(ad, v, ac[j]);
            float* c = Cb + gm * g.c_m + gn * g.c_n;
            if (g.beta != 0.f) v += g.beta * *c;
            *c = v;
          }
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm + i * 16 + (lane >> 4) * 4 + r, gn = n0 + wn + j * 16 + (lane & 15);
        if (gm < g.M && gn < g.N) {
          float v = g.alpha * acc[i][j][r];
          if (g.bias_m) v += g.bias_m[gm];
          gemm_store(g, Cb, Db, gm, gn, v);
        }
      }
}

// C = alpha * sum_z partial[z] + bias + beta * C.  Workgroup = 16 outputs x
// 16 partial slices (slice s sums z = s, s + 16, ...), slices combined in LDS
// in a fixed order (deterministic).
__device__ __forceinline__ void gemm_finish_block(int blk, const Gemm& g, int nsplit, const float* partial) {
  __shared__ float red[16][17];
  const int el = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int idx = blk * 16 + el;
  const int MN = g.M * g.N;
  float s = 0.f;
  if (idx < MN)
#pragma unroll 8
    for (int z = sl; z < nsplit; z += 16) s += partial[(size_t)z * MN + idx];
  red[sl][el] = s;
  __syncthreads();
  if (sl != 0 || idx >= MN) return;
  float t = 0.f;
  for (int k = 0; k < 16; ++k) t += red[k][el];
  const int m = idx / g.N, n = idx - m * g.N;
  float v = g.alpha * t;
  if (g.bias_m) v += g.bias_m[m];
  gemm_store(g, g.C, g.d_out, m, n, v);
}
__global__ __launch_bounds__(256) void k_gemm_finish(Gemm g, int nsplit, const float* partial) {
  gemm_finish_block(blockIdx.x, g, nsplit, partial);
}

constexpr int kMaxSplit = 128;

// x / d for x < 2^16 by a multiply-high: m = ceil(2^32 / d) (m = 2^32, i.e.
// hi set, for d = 1); exact since x * (m - 2^32 / d) / 2^32 < 1 / d.
struct FastDiv {
  uint32_t m, hi;
  __device__ explicit FastDiv(uint32_t d) {
    const uint64_t M = 0xFFFFFFFFull / d + 1;
    m = (uint32_t)M;
    hi = (uint32_t)(M >> 32);
  }
  __device__ int operator()(int x) const { return (int)(__umulhi((uint32_t)x, m) + (hi ? (uint32_t)x : 0u)); }
};

// ---------------------------------------------------------------------------
// Streaming GEMM of the training step's 1x1 convolutions and conv_rm products:
// C[b][m][p] = alpha * sum_k A[m][k] B[b][k][p] + bias_m[m] (+ beta C) (+ the
// d_out adjacency), M, K <= 80, B and C rows contiguous.  The weight matrix
// stays in registers as MFMA A fragments for the whole launch (staged once
// per workgroup through LDS); each wave then streams 16-column items
// (b, column tile) with the next item's B fragments in flight during the
// current item's MFMAs -- no LDS round trip and no barrier per tile.  The
// panel kernels below staged both operands per workgroup and ran load,
// compute and store in lockstep (conv forward 20.4 us, conv dx 23.8 us at
// the config-5 batch against a 4 us copy of the panel, profiles/r03v).
// ---------------------------------------------------------------------------
constexpr int kCsMax = 80;  // M, K
constexpr uint32_t kCsOOB = 0x80000000u;
// a zero hipcc cannot see through: keeps the loop-invariant A-fragment LDS
// reads inside the item loop instead of hoisted into ~100 live registers
__device__ __forceinline__ int cs_opaque_zero() {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}  // buffer offset past any range: loads 0, stores dropped
__device__ __forceinline__ __amdgpu_buffer_rsrc_t cs_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float cs_ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void cs_st(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
#if defined(DSTD_CS_ABL) && (DSTD_CS_ABL & 2)  // (ablation builds: stores dropped)
  if (v != 12345.f) off = kCsOOB;
#endif
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, 0);
}
// Launch constants of k_conv_stream (byte strides of one batch's panels)
struct CsArgs {
  int ntile, nb2;
  uint32_t b_bytes, c_bytes;  // one batch's B / C extent (buffer ranges)
};
#ifndef DSTD_CS_NT  // 16-column tiles per item (experiments: 1, 2, 4)
#define DSTD_CS_NT 1
#endif
#ifndef DSTD_CS_PF  // next item's B fragments loaded during this item's MFMAs
#define DSTD_CS_PF 1
#endif
template <int MF, int KS>
__global__ __launch_bounds__(256) void k_conv_stream(Gemm g, CsArgs ca) {
  constexpr int NT = DSTD_CS_NT, PF = DSTD_CS_PF;
  // A in LDS in fragment order, four k-steps per lane per 16-byte read:
  // As[((x KS4 + s4) 64 + lane) 4 + j] = A[16x + lr][4 (4 s4 + j) + lk]
  constexpr int KS4 = (KS + 3) / 4;
  __shared__ float4 As[MF * KS4 * 64];
  __shared__ float bsl[MF * 16];  // bias_m (0 past M or without one)
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 15, lk = lane >> 4;
  float* Af = reinterpret_cast<float*>(As);
  if (tid < MF * 16) bsl[tid] = g.bias_m && tid < g.M ? g.bias_m[tid] : 0.f;
  for (int e = tid; e < MF * KS4 * 256; e += 256) {
    const int j = e & 3, l = (e >> 2) & 63, f = e >> 8, x = f / KS4, s4 = f - x * KS4;
    const int m = x * 16 + (l & 15), k = 4 * (4 * s4 + j) + (l >> 4);
    const bool in = m < g.M && k < g.K;
    const float v = g.A[in ? m * g.a_m + k * g.a_k : 0];
    Af[e] = in ? v : 0.f;
  }
  __syncthreads();

  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntile = ca.ntile, nw = gridDim.x * 4, items = g.nb1 * ca.nb2 * ntile;  // ntile: items per batch
  const int K = g.K, M = g.M, N = g.N;
  const int bk = (int)g.b_k, cm = (int)g.c_m;
  const uint32_t kstep = 16u * (uint32_t)bk;  // bytes between k-steps (4 rows)
  (void)K, (void)M;
  // the item's batch panels (wave-uniform) and this lane's first column
  auto panel = [&](int it, const float*& Bb, float*& Cb, float*& Db, int& p) {
    const int b = it / ntile, t = it - b * ntile;
    const int b1 = b / ca.nb2, b2 = b - b1 * ca.nb2;
    Bb = g.B + b1 * g.b_b1 + b2 * g.b_b2;
    Cb = g.C + b1 * g.c_b1 + b2 * g.c_b2;
    Db = g.d_out ? g.d_out + b1 * g.c_b1 + b2 * g.c_b2 : nullptr;
    p = t * 16 * NT + lr;
  };
  auto load = [&](int it, float (&v)[NT][KS]) {
    const float* Bb;
    float* Cb;
    float* Db;
    int p;
    panel(it, Bb, Cb, Db, p);
    const auto rb = cs_rsrc(Bb, ca.b_bytes);
    // one lane base per column tile; rows k >= K fall past the buffer range by
    // themselves (b_k >= N: row K starts at or after the range's end), columns
    // past N take an out-of-range base
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int pq = p + 16 * q;
      const uint32_t base = pq < N ? (uint32_t)(lk * bk + pq) * 4u : kCsOOB;
#pragma unroll
      for (int sk = 0; sk < KS; ++sk) v[q][sk] = cs_ld(rb, base + (uint32_t)sk * kstep);
    }
  };
  int it = blockIdx.x * 4 + wave;
  float bf[NT][KS];
  if (PF && it < items) load(it, bf);
  for (; it < items; it += nw) {
    float bn[NT][KS];
    if constexpr (PF) {
      const int nx = it + nw;
      load(nx < items ? nx : it, bn);  // the next item's fragments (the last reloads its own)
    } else {
      load(it, bf);
    }
    const float* Bb;
    float* Cb;
    float* Db;
    int p;
    panel(it, Bb, Cb, Db, p);
    const auto rc = cs_rsrc(Cb, ca.c_bytes);
    // beta: this item's C values, loaded before the MFMAs so they arrive under them
    float cv[NT][MF][4];
    if (g.beta != 0.f) {
#pragma unroll
      for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int x = 0; x < MF; ++x)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // (rows m >= M lie past the range: c_m >= N)
            const int pq = p + 16 * q;
            const uint32_t cb = pq < N ? (uint32_t)(lk * 4 * cm + pq) * 4u : kCsOOB;
            cv[q][x][r] = cs_ld(rc, cb + (uint32_t)((x * 16 + r) * cm) * 4u);
          }
    }
    f32x4 acc[NT][MF];
#pragma unroll
    for (int q = 0; q < NT; ++q)
#pragma unroll
      for (int x = 0; x < MF; ++x) acc[q][x] = zero4();
    const int lz = lane + cs_opaque_zero();
#if defined(DSTD_CS_ABL) && (DSTD_CS_ABL & 1)  // (ablation builds: no MFMAs)
#pragma unroll
    for (int sk = 0; sk < KS; ++sk) acc[0][sk % MF][sk & 3] += bf[0][sk];
    if (lz < 0)
#endif
#pragma unroll
    for (int s4 = 0; s4 < KS4; ++s4) {
      float4 a[MF];
#pragma unroll
      for (int x = 0; x < MF; ++x) a[x] = As[(x * KS4 + s4) * 64 + lz];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (4 * s4 + j >= KS) break;
#pragma unroll
        for (int q = 0; q < NT; ++q)
#pragma unroll
          for (int x = 0; x < MF; ++x)
            acc[q][x] = mfma16x16x4(j == 0 ? a[x].x : j == 1 ? a[x].y : j == 2 ? a[x].z : a[x].w, bf[q][4 * s4 + j],
                                    acc[q][x]);
      }
    }
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int pq = p + 16 * q;
      const bool pin = pq < N;
      // this lane's column base (rows m >= M lie past the range: c_m >= N)
      const uint32_t cbq = pin ? (uint32_t)(lk * 4 * cm + pq) * 4u : kCsOOB;
      if (Db) {  // C and D = d_alpha * C + (d_A (* d_W) (+ d_R)) of this column (k_gemm's order)
        const auto rd = cs_rsrc(Db, ca.c_bytes);
        const float ad = *g.d_alpha;
        const int pc = pin ? pq : 0;
        float ac = g.d_A[pc];
        if (g.d_W) ac *= g.d_W[pc];
        if (g.d_R) ac += g.d_R[pc];
#pragma unroll
        for (int x = 0; x < MF; ++x)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = x * 16 + lk * 4 + r;
            const uint32_t off = cbq + (uint32_t)((x * 16 + r) * cm) * 4u;
            float v = g.alpha * acc[q][x][r];
            if (g.bias_m) v += bsl[m];
            cs_st(rd, off, fmaf(ad, v, ac));
            if (g.beta != 0.f) v += g.beta * cv[q][x][r];
            cs_st(rc, off, v);
          }
      } else {
#pragma unroll
        for (int x = 0; x < MF; ++x)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = x * 16 + lk * 4 + r;
            float v = fmaf(g.alpha, acc[q][x][r], bsl[m]);
            if (g.beta != 0.f) v = fmaf(g.beta, cv[q][x][r], v);
            cs_st(rc, cbq + (uint32_t)((x * 16 + r) * cm) * 4u, v);
          }
      }
    }
    if constexpr (PF) {
#pragma unroll
      for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int sk = 0; sk < KS; ++sk) bf[q][sk] = bn[q][sk];
    }
  }
}

// ---------------------------------------------------------------------------
// Skinny GEMM of the training step's 1x1 convolutions: a small weight matrix
// (M, K <= 80) times a wide panel of contiguous rows.  gemm() routes the
// matching shapes here; the whole K extent of both operands sits in LDS.
// ---------------------------------------------------------------------------
constexpr int kSkMax = 80;     // M, K <= 5 fragments of 16
constexpr int kSkPT = 128;     // panel columns per workgroup
__host__ __device__ constexpr int sk_pitch(int n, int want) {  // >= n, = want mod 64
  int s = n;
  while ((s & 63) != want) ++s;
  return s;
}

// C[b][m][p] = alpha * sum_k A[m][k] B[b][k][p] (+ bias, beta, d_out, nseg:
// gemm_store), B and C rows contiguous (b_n = c_n = 1).  Workgroup = (batch,
// 128 columns): A (any strides) and the B panel in LDS, zero-padded to whole
// fragments; 4 waves x 32 columns x MF row fragments.
template <int MF>
__global__ __launch_bounds__(256) void k_skinny_panel(Gemm g, int KP, int BP, int vec) {
  extern __shared__ float sk_sm[];
  float* As = sk_sm;                   // [MF*16][KP]
  float* Bs = sk_sm + MF * 16 * KP;    // [K4][BP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lk = lane >> 4;
  const int ntile = cdiv(g.N, kSkPT);
  const int b = blockIdx.x / ntile, p0 = (blockIdx.x - b * ntile) * kSkPT;
  const int b1 = b / g.nb2, b2 = b - b1 * g.nb2;
  const int K = g.K, K4 = rup(K, 4);
  const float* Bb = g.B + b1 * g.b_b1 + b2 * g.b_b2;
  // every load of the staging in flight at once (clamped indices, no
  // branches): A (zero rows >= M, columns >= K), then the B panel
  constexpr int UA = cdiv(MF * 16 * kSkMax, 256);
  const int ta = MF * 16 * K4;
  const FastDiv div_k4(K4);
  float va[UA];
#pragma unroll
  for (int u = 0; u < UA; ++u) {
    const int e = min(tid + u * 256, ta - 1), m = div_k4(e), k = e - m * K4;
    const bool in = m < g.M && k < K;
    const float x = g.A[in ? m * g.a_m + k * g.a_k : 0];
    va[u] = in ? x : 0.f;
  }
  if (vec) {  // 16-byte loads: K4 rows x 32 float4 (b_k, N, batch strides 4-aligned)
    constexpr int UB = cdiv(kSkMax * kSkPT / 4, 256);
    const int tb = K4 * (kSkPT / 4);
    f32x4 vb[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int e = min(tid + u * 256, tb - 1), k = e >> 5, p = p0 + 4 * (e & 31);
      const bool in = k < K && p < g.N;
      const f32x4 x = *reinterpret_cast<const f32x4*>(Bb + (in ? k * g.b_k + p : 0));
      vb[u] = in ? x : zero4();
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int e = min(tid + u * 256, tb - 1);
      *reinterpret_cast<f32x4*>(Bs + (e >> 5) * BP + 4 * (e & 31)) = vb[u];
    }
  } else {
    constexpr int U = 20;
    const int tot = K4 * kSkPT;
    for (int e0 = tid; e0 < tot; e0 += U * 256) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = min(e0 + u * 256, tot - 1), k = e >> 7, p = p0 + (e & (kSkPT - 1));
        const bool in = k < K && p < g.N;
        const float x = Bb[in ? k * g.b_k + p : 0];
        v[u] = in ? x : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = min(e0 + u * 256, tot - 1);
        Bs[(e >> 7) * BP + (e & (kSkPT - 1))] = v[u];
      }
    }
  }
#pragma unroll
  for (int u = 0; u < UA; ++u) {
    const int e = min(tid + u * 256, ta - 1), m = div_k4(e);
    As[m * KP + e - m * K4] = va[u];
  }
  __syncthreads();
  f32x4 acc[MF][2];
#pragma unroll
  for (int x = 0; x < MF; ++x) acc[x][0] = acc[x][1] = zero4();
  const int cw = wave * 32;
  for (int k = lk; k < K4; k += 4) {
    float av[MF], bv[2];
#pragma unroll
    for (int x = 0; x < MF; ++x) av[x] = As[(x * 16 + lr) * KP + k];
#pragma unroll
    for (int y = 0; y < 2; ++y) bv[y] = Bs[k * BP + cw + y * 16 + lr];
#pragma unroll
    for (int x = 0; x < MF; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = mfma16x16x4(av[x], bv[y], acc[x][y]);
  }
  float* Cb = g.C + b1 * g.c_b1 + b2 * g.c_b2;
  if (!g.d_out && !g.nseg) {  // plain store: one uniform branch, not one per element
#pragma unroll
    for (int x = 0; x < MF; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = x * 16 + lk * 4 + r;
        if (m >= g.M) continue;
        float* row = Cb + m * g.c_m;
        const float bm = g.bias_m ? g.bias_m[m] : 0.f;
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          const int p = p0 + cw + y * 16 + lr;
          if (p < g.N) {
            float v = fmaf(g.alpha, acc[x][y][r], bm);
            if (g.beta != 0.f) v = fmaf(g.beta, row[p], v);
            row[p] = v;
          }
        }
      }
    return;
  }
  float* Db = g.d_out ? g.d_out + b1 * g.c_b1 + b2 * g.c_b2 : nullptr;
  if (Db && !g.nseg) {  // C and the adjacency D = alpha_d * C + (A (* W) (+ R)) per column
    const float ad = *g.d_alpha;
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int p = p0 + cw + y * 16 + lr;
      if (p >= g.N) continue;
      float ac = g.d_A[p];
      if (g.d_W) ac *= g.d_W[p];
      if (g.d_R) ac += g.d_R[p];
#pragma unroll
      for (int x = 0; x < MF; ++x)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = x * 16 + lk * 4 + r;
          if (m < g.M) {
            float v = g.alpha * acc[x][y][r];
            if (g.bias_m) v += g.bias_m[m];
            Db[m * g.c_m + p] = fmaf(ad, v, ac);
            float* c = Cb + m * g.c_m + p;
            if (g.beta != 0.f) v += g.beta * *c;
            *c = v;
          }
        }
    }
    return;
  }
#pragma unroll
  for (int x = 0; x < MF; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = x * 16 + lk * 4 + r, p = p0 + cw + y * 16 + lr;
        if (m < g.M && p < g.N) {
          float v = g.alpha * acc[x][y][r];
          if (g.bias_m) v += g.bias_m[m];
          gemm_store(g, Cb, Db, m, p, v);
        }
      }
}

// ---------------------------------------------------------------------------
// Per-sample aggregation over slabs: the DSTDGC products (model/dstdgcn.py:87
// spatial, :93 temporal) and their gradients,
//   fwd  y[c][(a,j)]  (+)= sum_i F[c][(a,i)] D[a][i][j]
//   bwd  dD[a][i][j]   (=) sum_c F[c][(a,i)] dy[c][(a,j)]
//        dF[c][(a,i)]  (=) sum_j dy[c][(a,j)] D[a][i][j]
// where (a,i) is frame-major a*V + i for the spatial op (a = t, i = v) and
// i*V + a for the temporal one (a = v, i = t).  Workgroup = (sample, chunk
// of AC consecutive a); the chunk's slab -- every channel's AC x NN values,
// contiguous runs of AC (temporal) or AC*NN (spatial) floats -- is staged in
// LDS with coalesced loads.  Each wave owns whole a's: it stages D[n][a]
// (zero padded, transposed for dF) in its own LDS region and runs the
// products on fp32 MFMA from LDS; outputs laid out like the slab overwrite
// the a's slots in place and leave as one coalesced store.  This replaces a
// one-batch-per-workgroup strided GEMM whose operand gathers (stride V for
// the temporal products) made it L2-request bound.
// ---------------------------------------------------------------------------
struct AggArgs {
  const float* X;  // fwd: F; bwd: F (rows [0, C) of the packed conv output)
  long long xs;
  const float* Y0;  // bwd: dy
  long long y0s;
  const float* Dm;  // [B][A][NN][NN]
  float* O;         // fwd: y; bwd: dF
  long long os;
  float* dD;  // bwd: [B][A][NN][NN]
  float beta;
  int C, A, NN, V, TV, AC, QP, RK, P;
  int vec;  // k_aggc: 16-byte loads / stores (T*V, strides and bases 4-aligned)
  int B;    // k_aggc_bwd: samples (stride of the dD partials)
  // k_aggc / k_aggc_bwd, spatial: the a's (frames) of one (sample, channel
  // chunk) split over asplit workgroups of apg frames each (their slab is a
  // contiguous [apg * V] run of every channel row); 1 / A: one workgroup
  int asplit, apg;
};
constexpr int kAggMaxC = 64, kAggMaxNN = 64;


template <bool TEMP, bool BWD, int MF, int JF, bool DF = true>  // DF: bwd also computes dF
__global__ __launch_bounds__(256) void k_agg(AggArgs g) {
  extern __shared__ float agg_sm[];
  constexpr int U = BWD ? 24 : 32;  // loads in flight per thread in the staging loops
  const int nth = blockDim.x, nw = nth >> 6, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int C = g.C, NN = g.NN, V = g.V, AC = g.AC, QP = g.QP, P = g.P;
  const int chunks = cdiv(g.A, AC);
  const int n = blockIdx.x / chunks, a0 = (blockIdx.x - n * chunks) * AC;
  const int ac = min(AC, g.A - a0);
  float* SX = agg_sm;                                // C x QP
  float* SY = agg_sm + C * QP;                       // bwd: dy slab
  float* DL = agg_sm + (BWD ? 2 : 1) * C * QP;       // ac x [RK][P]: D of the chunk's a
  const float* Xn = g.X + n * g.xs;
  const float* Yn = BWD ? g.Y0 + n * g.y0s : nullptr;
  // slab element e (memory order within each channel row) -> its offset in
  // the sample / its LDS slot
  const int per = ac * NN, tot = C * per;
  const FastDiv div_per(per), div_ac(ac), div_nn(NN), div_nn2(NN * NN);
  auto slot = [&](int e, int& go, int& q) __attribute__((always_inline)) {
    const int c = div_per(e), r = e - c * per;
    if (TEMP) {
      const int i = div_ac(r), al = r - i * ac;
      go = c * g.TV + i * V + a0 + al;
      q = c * QP + i * AC + al;
    } else {
      go = c * g.TV + a0 * V + r;
      q = c * QP + r;
    }
  };
  auto lq = [&](int al, int i) __attribute__((always_inline)) { return TEMP ? i * AC + al : al * NN + i; };

  // stage the slab(s) and D[n][a0 .. a0+ac) (contiguous): U loads per thread
  // in flight, then the LDS writes
  const int NN2 = NN * NN, dtot = (BWD && !DF) ? 0 : ac * NN2;
  const float* Dn = g.Dm + ((long long)n * g.A + a0) * NN2;
  for (int e0 = tid; e0 < tot; e0 += U * nth) {
    float vx[U], vy[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // (clamped: the last element is re-staged with its own value)
      int go, q;
      slot(min(e0 + u * nth, tot - 1), go, q);
      vx[u] = Xn[go];
      if (BWD) vy[u] = Yn[go];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {  // (slots recomputed: U loads in flight, not U addresses)
      int go, q;
      slot(min(e0 + u * nth, tot - 1), go, q);
      SX[q] = vx[u];
      if (BWD) SY[q] = vy[u];
    }
  }
  for (int e0 = tid; e0 < dtot; e0 += U * nth) {
    float vd[U];
#pragma unroll
    for (int u = 0; u < U; ++u) vd[u] = Dn[min(e0 + u * nth, dtot - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // Dl[i][j] (fwd: B operand rows i) or Dl[j][i] (dF: rows j)
      const int e = min(e0 + u * nth, dtot - 1);
      const int al = div_nn2(e), r = e - al * NN2, i = div_nn(r), j = r - i * NN;
      DL[al * g.RK * P + (BWD ? j * P + i : i * P + j)] = vd[u];
    }
  }
  // pad rows NN .. RK-1 of every D tile: zero (the K tail of the products)
  for (int e = tid; e < ((BWD && !DF) ? 0 : ac * (g.RK - NN) * P); e += nth) {
    const int al = e / ((g.RK - NN) * P), r = e - al * ((g.RK - NN) * P);
    DL[al * g.RK * P + NN * P + r] = 0.f;
  }
  __syncthreads();

  // Fragment rows / columns beyond C or NN hold garbage that only reaches
  // output rows / columns that are never stored; the K tail (k >= NN, or
  // c >= C for dD) is masked on the A side and zero on the B side.
  const int lr = lane & 15, lk = lane >> 4;
  for (int al = wave; al < ac; al += nw) {
    const float* Dl = DL + al * g.RK * P;
    if (BWD) {  // dD[a] = F^T dy over the channels: rows i, columns j
      f32x4 acc[JF][JF];
#pragma unroll
      for (int x = 0; x < JF; ++x)
#pragma unroll
        for (int y = 0; y < JF; ++y) acc[x][y] = zero4();
      int sl[JF];  // LDS slot of (a, i = x*16 + lr) within a channel row
#pragma unroll
      for (int x = 0; x < JF; ++x) sl[x] = lq(al, x * 16 + lr);
      for (int c = lk; c < C; c += 4) {
        float av[JF], bv[JF];
#pragma unroll
        for (int x = 0; x < JF; ++x) {
          av[x] = SX[c * QP + sl[x]];
          bv[x] = SY[c * QP + sl[x]];
        }
#pragma unroll
        for (int x = 0; x < JF; ++x)
#pragma unroll
          for (int y = 0; y < JF; ++y) acc[x][y] = mfma16x16x4(av[x], bv[y], acc[x][y]);
      }
      if (C & 3) {  // channel tail: lanes past C contribute zero
        const int c = (C & ~3) + lk;
        float av[JF], bv[JF];
#pragma unroll
        for (int x = 0; x < JF; ++x) {
          av[x] = c < C ? SX[c * QP + sl[x]] : 0.f;
          bv[x] = c < C ? SY[c * QP + sl[x]] : 0.f;
        }
#pragma unroll
        for (int x = 0; x < JF; ++x)
#pragma unroll
          for (int y = 0; y < JF; ++y) acc[x][y] = mfma16x16x4(av[x], bv[y], acc[x][y]);
      }
      float* dDa = g.dD + ((long long)n * g.A + a0 + al) * NN2;
#pragma unroll
      for (int x = 0; x < JF; ++x)
#pragma unroll
        for (int y = 0; y < JF; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = x * 16 + lk * 4 + r, j = y * 16 + lr;
            if (i < NN && j < NN) dDa[i * NN + j] = acc[x][y][r];
          }
      if (!DF) continue;
    }
    // out[c][(a, col)] = sum_k In[c][(a, k)] Dl[k][col]: In = F (fwd) / dy (dF)
    const float* In = BWD ? SY : SX;
    f32x4 acc[MF][JF];
#pragma unroll
    for (int x = 0; x < MF; ++x)
#pragma unroll
      for (int y = 0; y < JF; ++y) acc[x][y] = zero4();
    auto kstep = [&](int k, bool tail) __attribute__((always_inline)) {
      const int kq = lq(al, k);
      float av[MF], bv[JF];
#pragma unroll
      for (int x = 0; x < MF; ++x) {
        av[x] = In[(x * 16 + lr) * QP + kq];
        if (tail) av[x] = k < NN ? av[x] : 0.f;
      }
#pragma unroll
      for (int y = 0; y < JF; ++y) bv[y] = Dl[k * P + y * 16 + lr];
#pragma unroll
      for (int x = 0; x < MF; ++x)
#pragma unroll
        for (int y = 0; y < JF; ++y) acc[x][y] = mfma16x16x4(av[x], bv[y], acc[x][y]);
    };
    int k = lk;
    for (; k < (NN & ~3); k += 4) kstep(k, false);
    if (NN & 3) kstep(k, true);
    // in place: the a's slots of SX (its F values are no longer needed)
#pragma unroll
    for (int x = 0; x < MF; ++x)
#pragma unroll
      for (int y = 0; y < JF; ++y) {
        const int j = y * 16 + lr;
        if (j < NN) {
          const int q = lq(al, j);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = x * 16 + lk * 4 + r;
            if (c < C) SX[c * QP + q] = acc[x][y][r];
          }
        }
      }
  }
  if (BWD && !DF) return;
  __syncthreads();
  float* On = g.O + n * g.os;
  const bool acc_out = !BWD && g.beta != 0.f;
  for (int e0 = tid; e0 < tot; e0 += U * nth) {
    float old[U];
    int gos[U], qs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * nth;
      if (e < tot) {
        slot(e, gos[u], qs[u]);
        old[u] = acc_out ? On[gos[u]] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (e0 + u * nth < tot) On[gos[u]] = acc_out ? fmaf(g.beta, old[u], SX[qs[u]]) : SX[qs[u]];
  }
}

// Channel-chunk form of the per-a products without a channel reduction:
//   fwd  out[c][(a,j)] (+)= sum_i In[c][(a,i)] D[a][i][j]   (In = F)
//   dF   out[c][(a,i)]  (=) sum_j In[c][(a,j)] D[a][i][j]   (In = dy; TRANS)
// Workgroup = (sample, 16 channels) over ALL a: the slab is 16 whole channel
// rows, T*V contiguous floats, staged with 16-byte loads; each wave streams
// D[n][a] of its a's through its own LDS tile, the next a's D loaded into
// registers while the current a's MFMAs run.  Outputs overwrite the a's
// slots in place and leave as one contiguous store.  The LDS row pitch is
// = 4 mod 64 so the 16 rows x 4 k of an A fragment hit distinct banks for
// both k strides (1: spatial, V: temporal).
constexpr int kAggcThreads = 512;
template <bool TEMP, bool TRANS, int JF, int MF>
__global__ __launch_bounds__(kAggcThreads) void k_aggc(AggArgs g) {
  extern __shared__ float agg_sm[];
  constexpr int DR = JF * JF * 4;  // >= ceil(NN^2 / 64): D values per lane
  constexpr int NW = kAggcThreads / 64;
  constexpr int CW = 16 * MF;  // channels per chunk (MF row tiles)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lk = lane >> 4;
  const int C = g.C, NN = g.NN, V = g.V, TV = g.TV, TVP = g.QP, P = g.P, RK = g.RK;
  const int cch = cdiv(C, CW);
  const int blk = blockIdx.x / g.asplit, ag = blockIdx.x - blk * g.asplit;
  const int n = blk / cch, c0 = (blk - n * cch) * CW;
  const int cv = min(CW, C - c0);
  // this workgroup's a's [a_lo, a_hi) and their slab: W floats from sb of every channel row
  const int a_lo = TEMP ? 0 : ag * g.apg, a_hi = TEMP ? g.A : min(g.A, a_lo + g.apg);
  const int W = TEMP ? TV : (a_hi - a_lo) * V, sb = TEMP ? 0 : a_lo * V;
  float* S = agg_sm;  // [CW][TVP]
  float* Dl = agg_sm + CW * TVP + wave * RK * P;
  const float* In = g.X + n * g.xs + (long long)c0 * TV + sb;
  float* Out = g.O + n * g.os + (long long)c0 * TV + sb;
  const int NN2 = NN * NN;
  const FastDiv div_nn(NN);
  auto off = [&](int a, int i) __attribute__((always_inline)) { return TEMP ? i * V + a : (a - a_lo) * V + i; };

  // first D tile of this wave into registers (its latency overlaps the slab)
  float dv[DR];
  auto load_d = [&](int a) __attribute__((always_inline)) {
    const float* Da = g.Dm + ((long long)n * g.A + a) * NN2;
#pragma unroll
    for (int r = 0; r < DR; ++r) dv[r] = Da[min(lane + 64 * r, NN2 - 1)];
  };
  if (a_lo + wave < a_hi) load_d(a_lo + wave);
  // the 16 channel rows: runs of W floats, TV apart
  if (g.vec) {
    constexpr int U = 8;
    const int w4 = W >> 2, tv4 = TV >> 2, tot4 = cv * w4;
    const FastDiv div_w4(w4);
    const f32x4* In4 = reinterpret_cast<const f32x4*>(In);
    for (int e0 = tid; e0 < tot4; e0 += U * kAggcThreads) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // (clamped: no branch)
        const int e = min(e0 + u * kAggcThreads, tot4 - 1);
        const int c = div_w4(e);
        v[u] = In4[c * tv4 + e - c * w4];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {  // (a clamped element is rewritten with its own value)
        const int e = min(e0 + u * kAggcThreads, tot4 - 1);
        const int c = div_w4(e), q = e - c * w4;
        *reinterpret_cast<f32x4*>(S + c * TVP + 4 * q) = v[u];
      }
    }
  } else {
    constexpr int U = 16;
    const int tot = cv * W;
    const FastDiv div_w(W);
    for (int e0 = tid; e0 < tot; e0 += U * kAggcThreads) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = min(e0 + u * kAggcThreads, tot - 1);
        const int c = div_w(e);
        v[u] = In[c * TV + e - c * W];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = min(e0 + u * kAggcThreads, tot - 1);
        const int c = div_w(e);
        S[c * TVP + e - c * W] = v[u];
      }
    }
  }
  for (int e = lane; e < (RK - NN) * P; e += 64) Dl[NN * P + e] = 0.f;  // K-tail rows
  __syncthreads();

  for (int a = a_lo + wave; a < a_hi; a += NW) {
#pragma unroll
    for (int r = 0; r < DR; ++r) {  // D[a] -> Dl[i][j] (fwd) / Dl[j][i] (dF)
      const int e = min(lane + 64 * r, NN2 - 1);
      const int i = div_nn(e), j = e - i * NN;
      Dl[TRANS ? j * P + i : i * P + j] = dv[r];
    }
    if (a + NW < a_hi) load_d(a + NW);
    __builtin_amdgcn_wave_barrier();
    f32x4 acc[MF][JF];
#pragma unroll
    for (int m = 0; m < MF; ++m)
#pragma unroll
      for (int y = 0; y < JF; ++y) acc[m][y] = zero4();
    auto kstep = [&](int k, bool tail) __attribute__((always_inline)) {
      float av[MF];
#pragma unroll
      for (int m = 0; m < MF; ++m) {
        av[m] = S[(m * 16 + lr) * TVP + off(a, k)];
        if (tail) av[m] = k < NN ? av[m] : 0.f;
      }
      float bv[JF];
#pragma unroll
      for (int y = 0; y < JF; ++y) bv[y] = Dl[k * P + y * 16 + lr];
#pragma unroll
      for (int m = 0; m < MF; ++m)
#pragma unroll
        for (int y = 0; y < JF; ++y) acc[m][y] = mfma16x16x4(av[m], bv[y], acc[m][y]);
    };
    int k = lk;
    for (; k < (NN & ~3); k += 4) kstep(k, false);
    if (NN & 3) kstep(k, true);
#pragma unroll
    for (int y = 0; y < JF; ++y) {
      const int j = y * 16 + lr;
      if (j < NN) {
        const int q = off(a, j);
#pragma unroll
        for (int m = 0; m < MF; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) S[(m * 16 + lk * 4 + r) * TVP + q] = acc[m][y][r];
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  const bool acc_out = g.beta != 0.f;
  if (g.vec) {
    const int w4 = W >> 2, tv4 = TV >> 2, tot4 = cv * w4;
    const FastDiv div_w4(w4);
    f32x4* Out4 = reinterpret_cast<f32x4*>(Out);
    for (int e = tid; e < tot4; e += kAggcThreads) {
      const int c = div_w4(e), q = e - c * w4;
      f32x4 v = *reinterpret_cast<const f32x4*>(S + c * TVP + 4 * q);
      if (acc_out) v += g.beta * Out4[c * tv4 + q];
      Out4[c * tv4 + q] = v;
    }
  } else {
    const int tot = cv * W;
    const FastDiv div_w(W);
    for (int e = tid; e < tot; e += kAggcThreads) {
      const int c = div_w(e), q = e - c * W;
      float v = S[c * TVP + q];
      if (acc_out) v = fmaf(g.beta, Out[c * TV + q], v);
      Out[c * TV + q] = v;
    }
  }
}

// Channel-chunk backward of one op's aggregation in one pass over dy:
//   dF[c][(a,i)] (=) sum_j dy[c][(a,j)] D[a][i][j]
//   dD_p[a][i][j] (=) sum_{c in chunk p} F[c][(a,i)] dy[c][(a,j)]
// Workgroup = (sample, 16-channel chunk p) over all a, dy and F slabs of the
// chunk in LDS (16-byte loads); per a, the wave first forms the chunk's
// partial dD (K = 16 channels), then dF (D[a]^T through its LDS tile) in
// place of the a's dy slots.  The cdiv(C, CW) partials are summed in a fixed
// order by adj_bwd (deterministic).  CW = 16 MF channels: 16 (temporal), 64
// (spatial, MF = 4 row tiles of dF per a).
#ifndef DSTD_AGGCB_THREADS  // (experiments: waves per workgroup x 64)
#define DSTD_AGGCB_THREADS 512  // (spatial: 8 waves, B=32 step -1.3%, profiles/r05z_aggcb_waves_ab.txt)
#endif
// (the temporal instantiations keep 4 waves: at 8, JF = 3 spills)
__host__ __device__ constexpr int aggcb_threads(bool temporal) { return temporal ? 256 : DSTD_AGGCB_THREADS; }
template <bool TEMP, int JF, int MF>
__global__ __launch_bounds__(aggcb_threads(TEMP)) void k_aggc_bwd(AggArgs g) {
  constexpr int kAggcbThreads = aggcb_threads(TEMP);
  extern __shared__ float agg_sm[];
  constexpr int DR = JF * JF * 4;  // >= ceil(NN^2 / 64): D values per lane
  constexpr int NW = kAggcbThreads / 64;
  constexpr int CW = 16 * MF;  // channels per chunk (MF row tiles of dF)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lk = lane >> 4;
  const int C = g.C, NN = g.NN, V = g.V, TV = g.TV, TVP = g.QP, P = g.P, RK = g.RK;
  const int cch = cdiv(C, CW);
  const int blk = blockIdx.x / g.asplit, ag = blockIdx.x - blk * g.asplit;
  const int n = blk / cch, p = blk - n * cch, c0 = p * CW;
  const int cv = min(CW, C - c0);
  // this workgroup's a's [a_lo, a_hi) and their slab: W floats from sb of every channel row
  const int a_lo = TEMP ? 0 : ag * g.apg, a_hi = TEMP ? g.A : min(g.A, a_lo + g.apg);
  const int W = TEMP ? TV : (a_hi - a_lo) * V, sb = TEMP ? 0 : a_lo * V;
  float* SY = agg_sm;              // [CW][TVP] dy, then dF
  float* SF = agg_sm + CW * TVP;   // [CW][TVP] F
  float* Dl = agg_sm + 2 * CW * TVP + wave * RK * P;
  const float* Yn = g.Y0 + n * g.y0s + (long long)c0 * TV + sb;
  const float* Fn = g.X + n * g.xs + (long long)c0 * TV + sb;
  float* Out = g.O + n * g.os + (long long)c0 * TV + sb;
  const int NN2 = NN * NN;
  const FastDiv div_nn(NN);
  auto off = [&](int a, int i) __attribute__((always_inline)) { return TEMP ? i * V + a : (a - a_lo) * V + i; };

  float dv[DR];
  auto load_d = [&](int a) __attribute__((always_inline)) {
    const float* Da = g.Dm + ((long long)n * g.A + a) * NN2;
#pragma unroll
    for (int r = 0; r < DR; ++r) dv[r] = Da[min(lane + 64 * r, NN2 - 1)];
  };
  if (a_lo + wave < a_hi) load_d(a_lo + wave);
  if (g.vec) {
    constexpr int U = 8;
    const int w4 = W >> 2, tv4 = TV >> 2, tot4 = cv * w4;
    const FastDiv div_w4(w4);
    const f32x4* Y4 = reinterpret_cast<const f32x4*>(Yn);
    const f32x4* F4 = reinterpret_cast<const f32x4*>(Fn);
    for (int e0 = tid; e0 < tot4; e0 += U * kAggcbThreads) {
      f32x4 vy[U], vf[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = min(e0 + u * kAggcbThreads, tot4 - 1);
        const int c = div_w4(e), gi = c * tv4 + e - c * w4;
        vy[u] = Y4[gi];
        vf[u] = F4[gi];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {  // (a clamped element is rewritten with its own value)
        const int e = min(e0 + u * kAggcbThreads, tot4 - 1);
        const int c = div_w4(e), q = c * TVP + 4 * (e - c * w4);
        *reinterpret_cast<f32x4*>(SY + q) = vy[u];
        *reinterpret_cast<f32x4*>(SF + q) = vf[u];
      }
    }
  } else {
    constexpr int U = 8;
    const int tot = cv * W;
    const FastDiv div_w(W);
    for (int e0 = tid; e0 < tot; e0 += U * kAggcbThreads) {
      float vy[U], vf[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = min(e0 + u * kAggcbThreads, tot - 1);
        const int c = div_w(e), gi = c * TV + e - c * W;
        vy[u] = Yn[gi];
        vf[u] = Fn[gi];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = min(e0 + u * kAggcbThreads, tot - 1);
        const int c = div_w(e), q = c * TVP + e - c * W;
        SY[q] = vy[u];
        SF[q] = vf[u];
      }
    }
  }
  for (int e = lane; e < (RK - NN) * P; e += 64) Dl[NN * P + e] = 0.f;  // K-tail rows
  __syncthreads();

  float* dDp = g.dD + (long long)p * g.B * g.A * NN2;
  for (int a = a_lo + wave; a < a_hi; a += NW) {
    {  // partial dD[a] over the chunk's channels: rows i, columns j, K = c
      f32x4 acc[JF][JF];
#pragma unroll
      for (int x = 0; x < JF; ++x)
#pragma unroll
        for (int y = 0; y < JF; ++y) acc[x][y] = zero4();
#pragma unroll
      for (int ks = 0; ks < 4 * MF; ++ks) {
        const int c = ks * 4 + lk;
        float av[JF], bv[JF];
#pragma unroll
        for (int x = 0; x < JF; ++x) {
          const int q = c * TVP + off(a, x * 16 + lr);
          av[x] = c < cv ? SF[q] : 0.f;
          bv[x] = c < cv ? SY[q] : 0.f;
        }
#pragma unroll
        for (int x = 0; x < JF; ++x)
#pragma unroll
          for (int y = 0; y < JF; ++y) acc[x][y] = mfma16x16x4(av[x], bv[y], acc[x][y]);
      }
      float* dDa = dDp + ((long long)n * g.A + a) * NN2;
#pragma unroll
      for (int x = 0; x < JF; ++x)
#pragma unroll
        for (int y = 0; y < JF; ++y) {
          const int j = y * 16 + lr;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = x * 16 + lk * 4 + r;
            if (i < NN && j < NN) dDa[i * NN + j] = acc[x][y][r];
          }
        }
    }
#pragma unroll
    for (int r = 0; r < DR; ++r) {  // D[a]^T -> Dl[j][i]
      const int e = min(lane + 64 * r, NN2 - 1);
      const int i = div_nn(e), j = e - i * NN;
      Dl[j * P + i] = dv[r];
    }
    if (a + NW < a_hi) load_d(a + NW);
    __builtin_amdgcn_wave_barrier();
    f32x4 acc[MF][JF];
#pragma unroll
    for (int m = 0; m < MF; ++m)
#pragma unroll
      for (int y = 0; y < JF; ++y) acc[m][y] = zero4();
    auto kstep = [&](int k, bool tail) __attribute__((always_inline)) {
      float av[MF];
#pragma unroll
      for (int m = 0; m < MF; ++m) {
        av[m] = SY[(m * 16 + lr) * TVP + off(a, k)];
        if (tail) av[m] = k < NN ? av[m] : 0.f;
      }
      float bv[JF];
#pragma unroll
      for (int y = 0; y < JF; ++y) bv[y] = Dl[k * P + y * 16 + lr];
#pragma unroll
      for (int m = 0; m < MF; ++m)
#pragma unroll
        for (int y = 0; y < JF; ++y) acc[m][y] = mfma16x16x4(av[m], bv[y], acc[m][y]);
    };
    int k = lk;
    for (; k < (NN & ~3); k += 4) kstep(k, false);
    if (NN & 3) kstep(k, true);
#pragma unroll
    for (int y = 0; y < JF; ++y) {
      const int i = y * 16 + lr;
      if (i < NN) {
        const int q = off(a, i);
#pragma unroll
        for (int m = 0; m < MF; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) SY[(m * 16 + lk * 4 + r) * TVP + q] = acc[m][y][r];
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  if (g.vec) {
    const int w4 = W >> 2, tv4 = TV >> 2, tot4 = cv * w4;
    const FastDiv div_w4(w4);
    f32x4* Out4 = reinterpret_cast<f32x4*>(Out);
    for (int e = tid; e < tot4; e += kAggcbThreads) {
      const int c = div_w4(e), q = e - c * w4;
      Out4[c * tv4 + q] = *reinterpret_cast<const f32x4*>(SY + c * TVP + 4 * q);
    }
  } else {
    const int tot = cv * W;
    const FastDiv div_w(W);
    for (int e = tid; e < tot; e += kAggcbThreads) {
      const int c = div_w(e), q = e - c * W;
      Out[c * TV + q] = SY[c * TVP + q];
    }
  }
}

// ---------------------------------------------------------------------------
// tanh outer difference
// ---------------------------------------------------------------------------
constexpr int kTanhMaxNN = 128;  // the frame envelope (T <= 128; V <= 64)
__global__ void k_tanh_outer_fwd(const float* __restrict__ P, const float* __restrict__ Q, PQView v, int R, int A,
                                 int NN, float* __restrict__ M) {
  // one workgroup per (n, r, a); M block [NN][NN]
  const int blk = blockIdx.x;
  const int n = blk / (R * A), ra = blk - n * R * A, r = ra / A, a = ra - r * A;
  const float* p = P + n * v.sn + r * v.sr + a * v.sa;
  const float* q = Q + n * v.sn + r * v.sr + a * v.sa;
  float* m = M + (size_t)blk * NN * NN;
  // the block's P and Q rows (strided in the caller's layout) staged once in
  // LDS instead of two strided loads per output element
  __shared__ float ps[kTanhMaxNN], qs[kTanhMaxNN];
  for (int i = threadIdx.x; i < NN; i += blockDim.x) {
    ps[i] = p[i * v.si];
    qs[i] = q[i * v.si];
  }
  __syncthreads();
#pragma unroll 4
  for (int e = threadIdx.x; e < NN * NN; e += blockDim.x) {
    const int i = e / NN, j = e - i * NN;
    m[e] = tanhf(ps[i] - qs[j]);
  }
}

__global__ void k_tanh_outer_bwd(const float* __restrict__ M, const float* __restrict__ dM, PQView v, int R, int A,
                                 int NN, float* __restrict__ dP, float* __restrict__ dQ) {
  extern __shared__ float dz[];  // [NN][NN+1]
  const int blk = blockIdx.x;
  const int n = blk / (R * A), ra = blk - n * R * A, r = ra / A, a = ra - r * A;
  const float* m = M + (size_t)blk * NN * NN;
  const float* dm = dM + (size_t)blk * NN * NN;
#pragma unroll 4
  for (int e = threadIdx.x; e < NN * NN; e += blockDim.x) {
    const int i = e / NN, j = e - i * NN;
    const float t = m[e];
    dz[i * (NN + 1) + j] = dm[e] * (1.f - t * t);
  }
  __syncthreads();
  const size_t base = n * v.sn + r * v.sr + a * v.sa;
  for (int i = threadIdx.x; i < 2 * NN; i += blockDim.x) {
    float s = 0.f;
    if (i < NN) {
      for (int j = 0; j < NN; ++j) s += dz[i * (NN + 1) + j];
      dP[base + i * v.si] = s;
    } else {
      const int j = i - NN;
      for (int k = 0; k < NN; ++k) s += dz[k * (NN + 1) + j];
      dQ[base + j * v.si] = -s;
    }
  }
}


// Fused adjacency backward, stage 1: workgroup (row a, sample chunk); each
// thread owns entries ij and walks the chunk's samples (no atomics).
// stage 1: workgroup (a, sample chunk, column block): the chunk's samples 8
// at a time with every load in flight.  DSTD_ADJ_SPLIT (default): 256-column
// blocks, one (i, j) per thread; 0: one block per (a, chunk), a 3-trip
// column loop (profiles/r04u_train_switches_ab.txt)
__global__ __launch_bounds__(256) void k_adj_bwd_part(float* __restrict__ dD, const float* __restrict__ E,
                                                      const float* __restrict__ alpha, int B, int A, int NN2, int nch,
                                                      float* __restrict__ pdA, float* __restrict__ pbr,
                                                      double* __restrict__ pal, const float* __restrict__ dDp,
                                                      int np) {
  __shared__ float red[4];
  __shared__ double redd[4];
  constexpr int SG = 8;
  const int a = blockIdx.x, ch = blockIdx.y, nij = gridDim.z;
  const int per = (B + nch - 1) / nch, n0 = ch * per, n1 = min(B, n0 + per);
  const float al = *alpha;
  // dD, or the sum of its np <= 4 channel-chunk partials in chunk order
  const float* src = np > 1 ? dDp : dD;
  const int nq = np > 1 ? np : 1;
  const size_t qs = np > 1 ? (size_t)B * A * NN2 : 0;
  // d alpha = sum over every (n, a, i, j) of dD E: a global sum whose terms
  // cancel to ~1% of their magnitude on trained blocks, so its products and
  // partial sums are carried in fp64 (fp32 accumulation put it at ~3x the
  // fp32 torch error: scripts/grad_tail_bisect.py)
  float sbr = 0.f;
  double sal = 0.0;
  for (int ij = blockIdx.z * 256 + threadIdx.x; ij < NN2; ij += 256 * nij) {
    float sa = 0.f;
    for (int nb = n0; nb < n1; nb += SG) {  // SG samples' loads in flight, then use in order
      float dv[SG], ev[SG];
#pragma unroll
      for (int u = 0; u < SG; ++u) {  // (clamped sample: loads without branches)
        const size_t i = ((size_t)min(nb + u, n1 - 1) * A + a) * NN2 + ij;
        if (nq > 1) {
          float pv[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) pv[q] = src[min(q, nq - 1) * qs + i];
          float t = 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) t += q < nq ? pv[q] : 0.f;
          dv[u] = t;
        } else {
          dv[u] = src[i];
        }
        ev[u] = E[i];
      }
#pragma unroll
      for (int u = 0; u < SG; ++u) {
        if (nb + u >= n1) break;
        sa += dv[u];
        sal = fma((double)dv[u], (double)ev[u], sal);
        dD[((size_t)(nb + u) * A + a) * NN2 + ij] = al * dv[u];
      }
    }
    pdA[((size_t)ch * A + a) * NN2 + ij] = sa;
    sbr += sa;
  }
  sbr = block_sum(sbr, red);
  sal = block_sum(sal, redd);
  if (threadIdx.x == 0) {
    pbr[((size_t)ch * A + a) * nij + blockIdx.z] = al * sbr;
    pal[((size_t)ch * A + a) * nij + blockIdx.z] = sal;
  }
}

// stage 2: blocks [0, cdiv(NN2,16)) finish dA (16 outputs x 16 slices over the
// A*nch partial rows); the last block finishes dbrm and dalpha.
// dW2 (optional): also dW2[ij] += dA-contribution * Amul[ij] (the spatial
// adjacency A_s * W_s + R_s: dR_s = dA as dA itself, dW_s = dA * A_s)
struct AdjFinishArgs {
  const float* pdA;
  const float* pbr;
  const double* pal;
  int A, NN2, nch;
  float* dA;
  float* dbrm;
  float* dalpha;
  int assign_dA;
  float* dW2;
  const float* Amul;
  int nij;
};
__device__ __forceinline__ void adj_finish_block(int blk, const AdjFinishArgs& f) {
  const float* __restrict__ pdA = f.pdA;
  const float* __restrict__ pbr = f.pbr;
  const double* __restrict__ pal = f.pal;
  const int A = f.A, NN2 = f.NN2, nch = f.nch, assign_dA = f.assign_dA, nij = f.nij;
  float* __restrict__ dA = f.dA;
  float* __restrict__ dbrm = f.dbrm;
  float* __restrict__ dalpha = f.dalpha;
  float* __restrict__ dW2 = f.dW2;
  const float* __restrict__ Amul = f.Amul;
  __shared__ float lds[16][17];
  __shared__ double redd[4];
  const int nblk = (NN2 + 15) / 16;
  if (blk < nblk) {
    const int el = threadIdx.x & 15, sl = threadIdx.x >> 4;
    const int ij = blk * 16 + el;
    float s = 0.f;
    if (ij < NN2)
#pragma unroll 8
      for (int r = sl; r < A * nch; r += 16) s += pdA[(size_t)r * NN2 + ij];
    lds[sl][el] = s;
    __syncthreads();
    if (sl == 0 && ij < NN2) {
      float t = 0.f;
      for (int k = 0; k < 16; ++k) t += lds[k][el];
      dA[ij] = assign_dA ? t : dA[ij] + t;
      if (dW2) dW2[ij] += t * Amul[ij];
    }
    return;
  }
  // dbrm: S threads per row a, each summing every S-th (chunk, column block)
  // partial, combined in slice order (A <= 128: A * S <= 256)
  __shared__ float sp[256];
  const int n = nch * nij, S = max(1, (int)blockDim.x / A);
  const int ar = threadIdx.x / S, sl = threadIdx.x - ar * S;
  float tb = 0.f;
  if (ar < A) {
#pragma unroll 4
    for (int i = sl; i < n; i += S) {
      const int c = i / nij, z = i - c * nij;
      tb += pbr[((size_t)c * A + ar) * nij + z];
    }
  }
  sp[threadIdx.x] = tb;
  __syncthreads();
  if (ar < A && sl == 0) {
    float u = 0.f;
    for (int k = 0; k < S; ++k) u += sp[ar * S + k];
    dbrm[ar] += u;
  }
  double t = 0.0;
#pragma unroll 4
  for (int i = threadIdx.x; i < A * nch * nij; i += blockDim.x) t += pal[i];
  t = block_sum(t, redd);
  if (threadIdx.x == 0) dalpha[0] += (float)t;
}
__global__ __launch_bounds__(256) void k_adj_bwd_finish(AdjFinishArgs f) { adj_finish_block(blockIdx.x, f); }
// finish_set: blocks [0, na) the adjacency finish, then each GEMM finish's
struct FinishSetArgs {
  AdjFinishArgs adj;
  int na;
  Gemm g[2];
  int nsplit[2], nb[2];
  const float* part[2];
};
__global__ __launch_bounds__(256) void k_finish_set(FinishSetArgs a) {
  int b = blockIdx.x;  // (block-uniform branches: the finishes' barriers are safe)
  if (b < a.na) {
    adj_finish_block(b, a.adj);
    return;
  }
  b -= a.na;
  if (b < a.nb[0]) {
    gemm_finish_block(b, a.g[0], a.nsplit[0], a.part[0]);
    return;
  }
  b -= a.nb[0];
  if (b < a.nb[1]) gemm_finish_block(b, a.g[1], a.nsplit[1], a.part[1]);
}

__global__ void k_copy_jobs(CopyJobs js) {
  const CopyJob& j = js.j[blockIdx.y];
  const int tot = j.rows * j.cols;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += gridDim.x * blockDim.x) {
    const int r = e / j.cols, c = e - r * j.cols;
    const float v = j.src[(size_t)r * j.src_ld + c];
    float* d = j.dst + (size_t)r * j.dst_ld + c;
    *d = j.accumulate ? *d + v : v;
  }
}

__global__ void k_adj_param_grads(const float* dA, const float* A_s, float* dR_s, float* dW_s, size_t n) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const float d = dA[e];
    dR_s[e] += d;
    dW_s[e] += d * A_s[e];
  }
}

__global__ void k_scale_by(float* x, const float* alpha, size_t n) {
  const float al = *alpha;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
    x[e] *= al;
}

// ---------------------------------------------------------------------------
// Strided sums out[m] += scale * sum_{b, j} X[b*sb + m*sm + j*sj], two stages:
// (m, split) partials in a fixed order, then a per-m finish.  Stage 1 maps
// threads to whichever index is contiguous: j (bias / conv_rm-bias grads) or m
// (the adjacency gradient dA, summed over samples and rows).
// ---------------------------------------------------------------------------
constexpr int kRedSplit = 64;

__global__ void k_red_part_j(const float* X, int M, int nb, int nj, long long sb, long long sm, long long sj,
                             int splits, float* part) {
  __shared__ float red[kRedThreads / 64];
  const int m = blockIdx.x, sp = blockIdx.y;
  const long long tot = (long long)nb * nj, per = (tot + splits - 1) / splits;
  const long long lo = sp * per, hi = min(tot, lo + per);
  float s = 0.f;
  // int index math (tot < 2^31 here): a 64-bit divide per element costs more
  // than the load it addresses
#pragma unroll 4
  for (int e = (int)lo + threadIdx.x; e < (int)hi; e += blockDim.x) {
    const int b = e / nj, j = e - b * nj;
    s += X[b * sb + m * sm + j * sj];
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[(size_t)sp * M + m] = s;
}

__global__ void k_red_part_m(const float* X, int M, int nb, int nj, long long sb, long long sj, int splits,
                             float* part) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x, sp = blockIdx.y;
  if (m >= M) return;
  const long long tot = (long long)nb * nj, per = (tot + splits - 1) / splits;
  const long long lo = sp * per, hi = min(tot, lo + per);
  float s = 0.f;
  int b = (int)(lo / nj), j = (int)(lo - (long long)b * nj);  // (b, j) advance by carry
#pragma unroll 4
  for (long long e = lo; e < hi; ++e) {
    s += X[b * sb + m + j * sj];
    if (++j == nj) j = 0, ++b;
  }
  part[(size_t)sp * M + m] = s;
}

// out[m] += scale * sum_sp part[sp][m]; 16 outputs x 16 split slices per workgroup
__global__ __launch_bounds__(256) void k_red_finish(const float* part, int M, int splits, float* out, float scale) {
  __shared__ float red[16][17];
  const int el = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int m = blockIdx.x * 16 + el;
  float s = 0.f;
  if (m < M)
#pragma unroll 4
    for (int sp = sl; sp < splits; sp += 16) s += part[(size_t)sp * M + m];
  red[sl][el] = s;
  __syncthreads();
  if (sl != 0 || m >= M) return;
  float t = 0.f;
  for (int k = 0; k < 16; ++k) t += red[k][el];
  out[m] += scale * t;
}

constexpr int kDotBlocks = 256;

__global__ void k_dot_partial(const float* x, const float* y, size_t n, float* partials) {
  __shared__ float red[kRedThreads / 64];
  float s = 0.f;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
    s = fmaf(x[e], y[e], s);
  s = block_sum(s, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

__global__ void k_sum_into(const float* partials, int n, float* out) {
  __shared__ float red[kRedThreads / 64];
  float s = 0.f;
  for (int e = threadIdx.x; e < n; e += blockDim.x) s += partials[e];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] += s;
}


__global__ void k_acc_mul(const float* a, const float* b, const float* c, float* out, size_t n, int assign) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    float v = b ? a[e] * b[e] : a[e];
    if (c) v += c[e];
    out[e] = assign ? v : out[e] + v;
  }
}


// ---------------------------------------------------------------------------
// Train-mode BatchNorm, channel (c, v) of an NCTV tensor, statistics over the
// B*T rows (n, t).  Three launches each way so the work spreads over
// C x splits workgroups instead of C:
//   fwd: per-(c, split) chunk mean / M2 (two passes over the chunk), Chan
//        merge per channel (mean, rstd, running stats), element-wise apply;
//   bwd: per-(c, split) sums of dz and dz*xhat (+ the PReLU-slope partial),
//        merge (dgamma, dbeta), element-wise du.
// Inside a workgroup thread (slice s, joint v) walks the chunk's rows s,
// s + S, ... so a wave reads runs of V consecutive floats; slice sums are
// combined in LDS in a fixed order (deterministic).
// ---------------------------------------------------------------------------
struct BnChunk {  // blockIdx.y = group * splits + split; rows of the chunk [r0, r1) (absolute)
  int V, S, rows, r0, r1;
  __device__ BnChunk(int V_, int B, int T, int splits, int groups)
      : V(V_), S(kRedThreads / V_), rows(B / groups * T) {
    const int g = blockIdx.y / splits, sp = blockIdx.y - g * splits;
    const int per = (rows + splits - 1) / splits;
    r0 = g * rows + sp * per;
    r1 = g * rows + min(rows, sp * per + per);
  }
};

__device__ __forceinline__ float slice_sum(float v, float* lds, int V, int S) {
  // lds: [S][V]; returns the total over slices for this thread's v (all threads)
  const int tid = threadIdx.x;
  __syncthreads();
  if (tid < S * V) lds[tid] = v;
  __syncthreads();
  const int jv = tid % V;
  float t = 0.f;
  for (int s = 0; s < S; ++s) t += lds[s * V + jv];
  return t;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Rows are visited RB at a time with all RB loads issued before the first
// use (a row-at-a-time loop pays one memory latency per row, ~8 per chunk at
// the config-5 batch); the accumulation order is unchanged.
#ifndef DSTD_BN_RB  // (experiments)
#define DSTD_BN_RB 8
#endif
constexpr int kBnRB = DSTD_BN_RB;
struct BnRows {  // the rows row0, row0 + S, ... of one batch as (n, t)
  int n[kBnRB], t[kBnRB];
  bool ok[kBnRB];
  __device__ BnRows(int row0, int r1, int S, int T) {
    int nn = row0 / T, tt = row0 - nn * T;
#pragma unroll
    for (int j = 0; j < kBnRB; ++j) {
      ok[j] = row0 + j * S < r1;
      n[j] = nn, t[j] = tt;
      tt += S;
      while (tt >= T) tt -= T, ++nn;
    }
  }
  __device__ size_t at(int j, int c, int v, int C, int T, int V) const {
    return ((size_t)n[j] * C + c) * T * V + (size_t)t[j] * V + v;
  }
};

// part: [splits][C*V][2] = (chunk mean, chunk M2)
__global__ __launch_bounds__(kRedThreads) void k_bn_stats_part(BnFwd a, int B, int C, int T, int V, int splits,
                                                               float* part) {
  __shared__ float lds[kRedThreads];
  const int c = blockIdx.x, tid = threadIdx.x;
  const BnChunk G(V, B, T, splits, a.groups);
  const bool act = tid < G.S * V;
  const int v = tid % V, s0 = tid / V;
  const int cnt = max(G.r1 - G.r0, 0);
  auto u_of = [&](size_t i) { return a.x2 ? a.x[i] + a.x2[i] : a.x[i]; };
  // one batch covers the thread's rows when the chunk has <= RB * S rows:
  // its values stay in registers for the second pass
  const bool one = cnt <= kBnRB * G.S;
  float keep[kBnRB];
  float s = 0.f;
  if (act)
    for (int row0 = G.r0 + s0; row0 < G.r1; row0 += kBnRB * G.S) {
      const BnRows R(row0, G.r1, G.S, T);
#pragma unroll
      for (int j = 0; j < kBnRB; ++j) keep[j] = R.ok[j] ? u_of(R.at(j, c, v, C, T, V)) : 0.f;
#pragma unroll
      for (int j = 0; j < kBnRB; ++j)
        if (R.ok[j]) s += keep[j];
    }
  const float mean = cnt ? slice_sum(s, lds, V, G.S) / cnt : slice_sum(0.f, lds, V, G.S);
  float q = 0.f;
  if (act)
    for (int row0 = G.r0 + s0; row0 < G.r1; row0 += kBnRB * G.S) {
      const BnRows R(row0, G.r1, G.S, T);
      float u[kBnRB];
#pragma unroll
      for (int j = 0; j < kBnRB; ++j) u[j] = one ? keep[j] : (R.ok[j] ? u_of(R.at(j, c, v, C, T, V)) : 0.f);
#pragma unroll
      for (int j = 0; j < kBnRB; ++j)
        if (R.ok[j]) {
          const float d = u[j] - mean;
          q = fmaf(d, d, q);
        }
    }
  const float m2 = slice_sum(q, lds, V, G.S);
  if (tid < V) {
    float* p = part + ((size_t)blockIdx.y * C * V + c * V + v) * 2;
    p[0] = mean;
    p[1] = m2;
  }
}

// Merge + apply in one launch: workgroup (c, n) first merges the V channels
// (c, v) from the split partials (Chan merge in split order -- every
// workgroup of channel c computes the same values; the n == 0 one stores
// mean / rstd and updates the running statistics), then normalises the
// sample's contiguous [T][V] plane of channel c.
constexpr int kBnMaxV = 64;
constexpr int kBnMaxSplits = 16;  // bn_splits() never exceeds it
// rows: rows per group; g: the group whose split partials merge
// this rank's (mean, M2) of channel ch, group g: Chan merge of the split partials in split order
__device__ __forceinline__ void bn_local_merge(int cv, int ch, int rows, int splits, const float* part, int g,
                                               float& mean, float& m2) {
  const int per = (rows + splits - 1) / splits;
  part += (size_t)g * splits * cv * 2;
  float m = 0.f;
  for (int sp = 0; sp < splits; ++sp) {
    const int cnt = max(min(rows, (sp + 1) * per) - sp * per, 0);
    m += cnt * part[((size_t)sp * cv + ch) * 2];
  }
  m /= rows;
  float q = 0.f;
  for (int sp = 0; sp < splits; ++sp) {
    const int cnt = max(min(rows, (sp + 1) * per) - sp * per, 0);
    const float* p = part + ((size_t)sp * cv + ch) * 2;
    const float d = p[0] - m;
    q += p[1] + cnt * d * d;
  }
  mean = m;
  m2 = q;
}

// part: channel c's split partials [group][split][V][2] (staged in LDS by
// k_bn_apply_merged), v: the joint of ch = c * V + v
// (pcv, pch): the partials' channel count and this channel's index in them
__device__ __forceinline__ void bn_merge_stats(const BnFwd& a, int ch, int pch, int pcv, int rows, int splits,
                                               const float* part, int g, float& mean, float& rstd, bool store) {
  if (a.use_running) {
    mean = a.running_mean[ch];
    rstd = 1.f / sqrtf(a.running_var[ch] + a.eps);
  } else {
    float m, m2, n = (float)rows;
    if (a.gath) {
      // SyncBN: every rank's (mean, M2, count), Chan-merged in rank order
      // (every rank computes the same values)
      const size_t rs = (size_t)a.groups * a.cv * 3;
      const float* q = a.gath + ((size_t)g * a.cv + ch) * 3;
      n = 0.f;
      m = 0.f;
      for (int w = 0; w < a.world; ++w) {
        n += q[w * rs + 2];
        m += q[w * rs + 2] * q[w * rs];
      }
      m /= n;
      m2 = 0.f;
      for (int w = 0; w < a.world; ++w) {
        const float d = q[w * rs] - m;
        m2 += q[w * rs + 1] + q[w * rs + 2] * d * d;
      }
    } else {
      bn_local_merge(pcv, pch, rows, splits, part, g, m, m2);
    }
    const float var = m2 / n;
    mean = m;
    rstd = 1.f / sqrtf(var + a.eps);
    if (store && a.running_mean) {
      const float unb = n > 1.f ? m2 / (n - 1.f) : var;
      a.running_mean[ch] = (1.f - a.momentum) * a.running_mean[ch] + a.momentum * m;
      a.running_var[ch] = (1.f - a.momentum) * a.running_var[ch] + a.momentum * unb;
    }
  }
  if (store) {
    a.mean[g * a.cv + ch] = mean;
    a.rstd[g * a.cv + ch] = rstd;
  }
}

// SyncBN: this rank's (mean, M2, count) per (group, channel) into its slot of
// the gather buffer (dst = buf + rank * groups * C*V * 3)
__global__ __launch_bounds__(256) void k_bn_local_stats(int cv, int rows, int splits, const float* part, float* dst) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x, g = blockIdx.y;
  if (ch >= cv) return;
  float m, m2;
  bn_local_merge(cv, ch, rows, splits, part, g, m, m2);
  float* d = dst + ((size_t)g * cv + ch) * 3;
  d[0] = m;
  d[1] = m2;
  d[2] = (float)rows;
}

// Separate merge (bn_sep): the merge as a launch of its own (one thread per channel (c,
// v): every group's mean / rstd, the running statistics in group order, the
// apply's scale / shift in ss[group][C*V][2]), then a flat element-wise apply
__global__ __launch_bounds__(256) void k_bn_merge(BnFwd a, int rows, int splits, const float* part, float* ss, int C,
                                                  int V) {
  const int ch = blockIdx.x * 256 + threadIdx.x;
  if (ch >= a.cv) return;
  for (int g = 0; g < a.groups; ++g) {
    float mean, rstd;
    bn_merge_stats(a, ch, ch, a.cv, rows, splits, part, g, mean, rstd, true);
    const float sc = rstd * a.gamma[ch];
    ss[((size_t)g * a.cv + ch) * 2] = sc;
    ss[((size_t)g * a.cv + ch) * 2 + 1] = a.beta[ch] - mean * sc;
  }
}
__global__ __launch_bounds__(256) void k_bn_apply_flat(BnFwd a, int Bg, int C, int TV, int V, long long total,
                                                       const float* ss) {
  const float w = a.prelu ? *a.prelu : 0.f;
  const int stride = gridDim.x * 256 * 4, tot = (int)total;  // (the launcher keeps total < 2^31)
  for (int i0 = (blockIdx.x * 256 + threadIdx.x) * 4; i0 < tot; i0 += stride) {
    // TV % 4 == 0: the 4 elements share (n, c)
    const int nc = i0 / TV;
    const int e0 = i0 - nc * TV, n = nc / C, c = nc - n * C, g = n / Bg;
    float4 u = *reinterpret_cast<const float4*>(a.x + i0);
    if (a.x2) {
      const float4 u2 = *reinterpret_cast<const float4*>(a.x2 + i0);
      u.x += u2.x, u.y += u2.y, u.z += u2.z, u.w += u2.w;
    }
    const float4 r = a.res ? *reinterpret_cast<const float4*>(a.res + i0) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float uu[4] = {u.x, u.y, u.z, u.w}, rr[4] = {r.x, r.y, r.z, r.w};
    float zz[4], oo[4];
    int v = e0 % V;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* q = ss + ((size_t)g * a.cv + c * V + v) * 2;
      float z = fmaf(uu[j], q[0], q[1]);
      if (a.res) z += rr[j];
      zz[j] = z;
      oo[j] = a.prelu ? prelu_f(z, w) : z;
      v = v + 1 == V ? 0 : v + 1;
    }
    if (a.prelu) *reinterpret_cast<float4*>(a.zsave + i0) = make_float4(zz[0], zz[1], zz[2], zz[3]);
    *reinterpret_cast<float4*>(a.out + i0) = make_float4(oo[0], oo[1], oo[2], oo[3]);
  }
}

// workgroup (c, y) covers samples [ns*y, ns*y + ns) (one group: ns divides B/groups)
// VEC: T V % 4 == 0 and 16-byte aligned tensors -- the ns planes of channel c
// as one run of float4 items (the same arithmetic per element)
template <bool VEC>
__global__ __launch_bounds__(256) void k_bn_apply_merged(BnFwd a, int B, int C, int T, int V, int splits,
                                                         const float* part, int ns) {
  __shared__ float scl[kBnMaxV], shl[kBnMaxV];
  // channel c's split partials of the groups this workgroup merges, staged
  // with every load in flight at once (merging straight from memory chains
  // 2 x splits dependent loads per group)
  constexpr int kPl = 2 * kBnMaxSplits * 2 * kBnMaxV, kPlU = kPl / 256;
  __shared__ float pl[kPl];  // [group][split][V][2]
  const int c = blockIdx.x, n = blockIdx.y * ns, tid = threadIdx.x;
  const int Bg = B / a.groups, g = n / Bg;
  if (!a.use_running && !a.gath) {
    const int per = splits * 2 * V, g0 = n == 0 ? 0 : g, cnt = (n == 0 ? a.groups : 1) * per;
    float pv[kPlU];
#pragma unroll
    for (int u = 0; u < kPlU; ++u) {
      const int e = min(tid + 256 * u, cnt - 1), gs = e / (2 * V), q = e - gs * 2 * V;  // gs = (group - g0) * splits + sp
      pv[u] = part[((size_t)(g0 * splits + gs) * a.cv + c * V) * 2 + q];
    }
#pragma unroll
    for (int u = 0; u < kPlU; ++u)
      if (tid + 256 * u < cnt) pl[g0 * per + tid + 256 * u] = pv[u];
  }
  __syncthreads();
  if (tid < V) {
    const int ch = c * V + tid;
    float mean, rstd;
    // workgroup (c, 0) stores every group's mean / rstd and applies the
    // groups' running-statistics updates in group order
    if (n == 0)
      for (int gg = 1; gg < a.groups; ++gg) {
        float m_, r_;
        bn_merge_stats(a, ch, tid, V, Bg * T, splits, pl, gg - 1, m_, r_, true);
      }
    bn_merge_stats(a, ch, tid, V, Bg * T, splits, pl, n == 0 ? a.groups - 1 : g, mean, rstd, n == 0);
    if (n == 0 && a.groups > 1) bn_merge_stats(a, ch, tid, V, Bg * T, splits, pl, 0, mean, rstd, false);
    const float sc = rstd * a.gamma[ch];
    scl[tid] = sc;
    shl[tid] = a.beta[ch] - mean * sc;
  }
  __syncthreads();
  const float w = a.prelu ? *a.prelu : 0.f;
  if constexpr (VEC) {
    constexpr int EB = 2;  // float4 items per thread per batch, loads issued first
    const int tv4 = T * V / 4, tot = ns * tv4;
    const FastDiv divV(V);
    for (int i0 = tid; i0 < tot; i0 += EB * 256) {
      float4 u[EB], r[EB];
      size_t at[EB];
      int vv[EB];
#pragma unroll
      for (int j = 0; j < EB; ++j) {
        const int i = min(i0 + j * 256, tot - 1);  // (clamped: loads without branches)
        const int k = (i >= tv4) + (i >= 2 * tv4) + (i >= 3 * tv4), e = 4 * (i - k * tv4);
        at[j] = ((size_t)(n + k) * C + c) * T * V + e;
        vv[j] = e - divV(e) * V;
        u[j] = ld4(a.x + at[j]);
        if (a.x2) {
          const float4 u2 = ld4(a.x2 + at[j]);
          u[j].x += u2.x, u[j].y += u2.y, u[j].z += u2.z, u[j].w += u2.w;
        }
        r[j] = a.res ? ld4(a.res + at[j]) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < EB; ++j) {
        if (i0 + j * 256 >= tot) break;
        const float uu[4] = {u[j].x, u[j].y, u[j].z, u[j].w}, rr[4] = {r[j].x, r[j].y, r[j].z, r[j].w};
        float zz[4], oo[4];
        int v = vv[j];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float z = fmaf(uu[q], scl[v], shl[v]);
          if (a.res) z += rr[q];
          zz[q] = z;
          oo[q] = a.prelu ? prelu_f(z, w) : z;
          v = v + 1 == V ? 0 : v + 1;
        }
        if (a.prelu) *reinterpret_cast<float4*>(a.zsave + at[j]) = make_float4(zz[0], zz[1], zz[2], zz[3]);
        *reinterpret_cast<float4*>(a.out + at[j]) = make_float4(oo[0], oo[1], oo[2], oo[3]);
      }
    }
    return;
  }
#ifndef DSTD_BN_APPLY_EB
#define DSTD_BN_APPLY_EB 4
#endif
  constexpr int EB = DSTD_BN_APPLY_EB;  // elements per thread per batch, loads issued first
  for (int k = 0; k < ns; ++k)
  for (int e0 = tid; e0 < T * V; e0 += EB * 256) {
    const size_t base = ((size_t)(n + k) * C + c) * T * V;
    float u[EB], r[EB];
#pragma unroll
    for (int j = 0; j < EB; ++j) {
      const int e = e0 + j * 256;
      const size_t i = base + e;
      u[j] = e < T * V ? (a.x2 ? a.x[i] + a.x2[i] : a.x[i]) : 0.f;
      r[j] = (e < T * V && a.res) ? a.res[i] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < EB; ++j) {
      const int e = e0 + j * 256;
      if (e >= T * V) break;
      const size_t i = base + e;
      const int v = e % V;
      float z = fmaf(u[j], scl[v], shl[v]);
      if (a.res) z += r[j];
      if (a.prelu) {
        a.zsave[i] = z;
        a.out[i] = prelu_f(z, w);
      } else {
        a.out[i] = z;
      }
    }
  }
}

// part: [splits][C*V][2] = (sum dz, sum dz*xhat); wpart: [splits][C] PReLU slope partials
__global__ __launch_bounds__(kRedThreads) void k_bn_bwd_part(BnBwd a, int B, int C, int T, int V, int splits,
                                                             float* part, float* wpart) {
  __shared__ float lds[kRedThreads];
  const int c = blockIdx.x, tid = threadIdx.x;
  const BnChunk G(V, B, T, splits, a.groups);
  const bool act = tid < G.S * V;
  const int v = tid % V, s0 = tid / V;
  const int ch = c * V + v;
  const float w = a.prelu ? *a.prelu : 0.f;
  const int grp = blockIdx.y / splits;
  const float mean = act ? a.mean[grp * C * V + ch] : 0.f, rstd = act ? a.rstd[grp * C * V + ch] : 0.f;
  float sd = 0.f, sdx = 0.f, sw = 0.f;
  if (act)
    for (int row0 = G.r0 + s0; row0 < G.r1; row0 += kBnRB * G.S) {
      const BnRows R(row0, G.r1, G.S, T);
      float dv[kBnRB], zv[kBnRB], uv[kBnRB];
#pragma unroll
      for (int j = 0; j < kBnRB; ++j) {
        const size_t i = R.at(j, c, v, C, T, V);
        dv[j] = R.ok[j] ? a.dout[i] : 0.f;
        zv[j] = (R.ok[j] && a.prelu) ? a.zsave[i] : 0.f;
        uv[j] = R.ok[j] ? (a.x2 ? a.x[i] + a.x2[i] : a.x[i]) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < kBnRB; ++j) {
        if (!R.ok[j]) continue;
        const float d = dv[j];
        // PReLU' (torch convention: the slope for z <= 0)
        const float dz = (a.prelu && !(zv[j] > 0.f)) ? w * d : d;
        sd += dz;
        sdx = fmaf(dz, (uv[j] - mean) * rstd, sdx);
        if (a.prelu) sw = fmaf(d, fminf(zv[j], 0.f), sw);
      }
    }
  const float t0 = slice_sum(sd, lds, V, G.S);
  const float t1 = slice_sum(sdx, lds, V, G.S);
  if (tid < V) {
    float* p = part + ((size_t)blockIdx.y * C * V + ch) * 2;
    p[0] = t0;
    p[1] = t1;
  }
  if (a.prelu) {
    __shared__ float red[kRedThreads / 64];
    const float tw = block_sum(act ? sw : 0.f, red);
    if (tid == 0) wpart[(size_t)blockIdx.y * C + c] = tw;
  }
}

// SyncBN: this rank's (sum dz, sum dz*xhat) per (group, channel), split order,
// then the groups' row counts -- the buffer the all-reduce sums
__global__ __launch_bounds__(256) void k_bn_bwd_local_sums(int cv, int groups, int splits, int rows, const float* part,
                                                           float* dst) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x, g = blockIdx.y;
  if (ch == 0) dst[(size_t)groups * cv * 2 + g] = (float)rows;
  if (ch >= cv) return;
  float sd = 0.f, sdx = 0.f;
  for (int sp = 0; sp < splits; ++sp) {
    const float* p = part + ((size_t)(g * splits + sp) * cv + ch) * 2;
    sd += p[0];
    sdx += p[1];
  }
  dst[((size_t)g * cv + ch) * 2] = sd;
  dst[((size_t)g * cv + ch) * 2 + 1] = sdx;
}

// DSTD_BN_SEP backward: the merge as a launch of its own (one thread per
// channel: the group sums in split order into sx[group][C*V][2] -- SyncBN's
// all-reduced ones for the input gradient -- dgamma / dbeta, and workgroup 0
// the PReLU slope), then a flat float4 apply.  Same arithmetic as
// k_bn_bwd_apply_merged.
__global__ __launch_bounds__(256) void k_bn_bwd_merge(BnBwd a, int splits, int C, const float* part,
                                                      const float* wpart, float* dprelu, float* sx, int CV) {
  __shared__ float red[kRedThreads / 64];
  if (a.prelu && blockIdx.x == 0) {  // uniform per workgroup
    float t = 0.f;
    for (int e = threadIdx.x; e < splits * a.groups * C; e += blockDim.x) t += wpart[e];
    t = block_sum(t, red);
    if (threadIdx.x == 0) dprelu[0] += t;
  }
  const int ch = blockIdx.x * 256 + threadIdx.x;
  if (ch >= CV) return;
  float tb = 0.f, tg = 0.f;
  for (int gg = 0; gg < a.groups; ++gg) {
    float sd = 0.f, sdx = 0.f;
    for (int sp = 0; sp < splits; ++sp) {
      const float2 pv = *reinterpret_cast<const float2*>(part + ((size_t)(gg * splits + sp) * CV + ch) * 2);
      sd += pv.x;
      sdx += pv.y;
    }
    sx[((size_t)gg * CV + ch) * 2] = a.gsum ? a.gsum[((size_t)gg * CV + ch) * 2] : sd;
    sx[((size_t)gg * CV + ch) * 2 + 1] = a.gsum ? a.gsum[((size_t)gg * CV + ch) * 2 + 1] : sdx;
    tb += sd;
    tg += sdx;
  }
  a.dbeta[ch] += tb;
  a.dgamma[ch] += tg;
}
__global__ __launch_bounds__(256) void k_bn_bwd_apply_flat(BnBwd a, int Bg, int C, int TV, int V, int T,
                                                           long long total, const float* sx) {
  const float w = a.prelu ? *a.prelu : 0.f;
  const int CV = C * V;
  const int stride = gridDim.x * 256 * 4, tot = (int)total;  // (the launcher keeps total < 2^31)
  for (int i0 = (blockIdx.x * 256 + threadIdx.x) * 4; i0 < tot; i0 += stride) {
    const int nc = i0 / TV;
    const int e0 = i0 - nc * TV, n = nc / C, c = nc - n * C, g = n / Bg;
    const float inv = 1.f / (a.gsum ? a.gsum[(size_t)a.groups * CV * 2 + g] : (float)(Bg * T));
    const float4 d4 = *reinterpret_cast<const float4*>(a.dout + i0);
    const float4 z4 = a.prelu ? *reinterpret_cast<const float4*>(a.zsave + i0) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 u4 = *reinterpret_cast<const float4*>(a.x + i0);
    if (a.x2) {
      const float4 u2 = *reinterpret_cast<const float4*>(a.x2 + i0);
      u4.x += u2.x, u4.y += u2.y, u4.z += u2.z, u4.w += u2.w;
    }
    const float4 ad4 = a.dz_add ? *reinterpret_cast<const float4*>(a.dz_add + i0) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float dv[4] = {d4.x, d4.y, d4.z, d4.w}, zv[4] = {z4.x, z4.y, z4.z, z4.w}, uv[4] = {u4.x, u4.y, u4.z, u4.w};
    const float av[4] = {ad4.x, ad4.y, ad4.z, ad4.w};
    float du[4], dzo[4];
    int v = e0 % V;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ch = c * V + v;
      const float d = dv[j];
      const float dz = (a.prelu && !(zv[j] > 0.f)) ? w * d : d;
      const float mean = a.mean[g * CV + ch], rstd = a.rstd[g * CV + ch], gm = a.gamma[ch];
      const float xh = (uv[j] - mean) * rstd;
      const float sdl = sx[((size_t)g * CV + ch) * 2], sxl = sx[((size_t)g * CV + ch) * 2 + 1];
      du[j] = a.use_running ? gm * rstd * dz : gm * rstd * (dz - sdl * inv - xh * sxl * inv);
      dzo[j] = a.dz_add ? dz + av[j] : dz;
      v = v + 1 == V ? 0 : v + 1;
    }
    *reinterpret_cast<float4*>(a.du + i0) = make_float4(du[0], du[1], du[2], du[3]);
    if (a.dz_out) *reinterpret_cast<float4*>(a.dz_out + i0) = make_float4(dzo[0], dzo[1], dzo[2], dzo[3]);
  }
}

// Merge + apply of the backward in one launch: workgroup (c, n) sums the
// split partials of its V channels (split order), the n == 0 one accumulates
// dgamma / dbeta (and workgroup (0, 0) the PReLU slope: the partials in the
// order of the former sum_into pass), then writes du over the sample's plane.
template <bool VEC>
__global__ __launch_bounds__(256) void k_bn_bwd_apply_merged(BnBwd a, int B, int C, int T, int V, int splits,
                                                             const float* part, const float* wpart, float* dprelu,
                                                             int ns) {
  __shared__ float sdl[kBnMaxV], sxl[kBnMaxV], red[kRedThreads / 64];
  __shared__ float mnl[kBnMaxV], rsl[kBnMaxV], gml[kBnMaxV];  // the group's mean / rstd and gamma per v
  const int c = blockIdx.x, n = blockIdx.y * ns, tid = threadIdx.x;
  const int CV = C * V;
  const int Bg = B / a.groups, grp = n / Bg;
  if (tid < V) {
    const int ch = c * V + tid;
    mnl[tid] = a.mean[grp * CV + ch];
    rsl[tid] = a.rstd[grp * CV + ch];
    gml[tid] = a.gamma[ch];
    // group sums; workgroup (c, 0) adds every group's into dgamma / dbeta
    float tb = 0.f, tg = 0.f;
    for (int gg = 0; gg < a.groups; ++gg) {
      if (n != 0 && gg != grp) continue;
      float2 pv[kBnMaxSplits];  // loads first, then the split-order sums
#pragma unroll
      for (int sp = 0; sp < kBnMaxSplits; ++sp)
        if (sp < splits) pv[sp] = *reinterpret_cast<const float2*>(part + ((size_t)(gg * splits + sp) * CV + ch) * 2);
      float sd = 0.f, sdx = 0.f;
#pragma unroll
      for (int sp = 0; sp < kBnMaxSplits; ++sp)
        if (sp < splits) {
          sd += pv[sp].x;
          sdx += pv[sp].y;
        }
      if (gg == grp) {
        // SyncBN: the input gradient takes every rank's sums; dgamma / dbeta
        // (below) stay this rank's
        sdl[tid] = a.gsum ? a.gsum[((size_t)grp * CV + ch) * 2] : sd;
        sxl[tid] = a.gsum ? a.gsum[((size_t)grp * CV + ch) * 2 + 1] : sdx;
      }
      tb += sd;
      tg += sdx;
    }
    if (n == 0) {
      a.dbeta[ch] += tb;
      a.dgamma[ch] += tg;
    }
  }
  if (a.prelu && c == 0 && n == 0) {  // uniform per workgroup: block_sum's barriers are safe
    float t = 0.f;
    for (int e = tid; e < splits * a.groups * C; e += blockDim.x) t += wpart[e];
    t = block_sum(t, red);
    if (tid == 0) dprelu[0] += t;
  }
  __syncthreads();
  const float w = a.prelu ? *a.prelu : 0.f;
  const float inv = 1.f / (a.gsum ? a.gsum[(size_t)a.groups * CV * 2 + grp] : (float)(Bg * T));
  if constexpr (VEC) {  // (k_bn_apply_merged VEC: float4 items over the ns planes)
    constexpr int EB = 2;
    const int tv4 = T * V / 4, tot = ns * tv4;
    const FastDiv divV(V);
    for (int i0 = tid; i0 < tot; i0 += EB * 256) {
      float4 d4[EB], z4[EB], u4[EB], a4[EB];
      size_t at[EB];
      int vv[EB];
#pragma unroll
      for (int j = 0; j < EB; ++j) {
        const int i = min(i0 + j * 256, tot - 1);
        const int k = (i >= tv4) + (i >= 2 * tv4) + (i >= 3 * tv4), e = 4 * (i - k * tv4);
        at[j] = ((size_t)(n + k) * C + c) * T * V + e;
        vv[j] = e - divV(e) * V;
        d4[j] = ld4(a.dout + at[j]);
        z4[j] = a.prelu ? ld4(a.zsave + at[j]) : make_float4(0.f, 0.f, 0.f, 0.f);
        u4[j] = ld4(a.x + at[j]);
        if (a.x2) {
          const float4 u2 = ld4(a.x2 + at[j]);
          u4[j].x += u2.x, u4[j].y += u2.y, u4[j].z += u2.z, u4[j].w += u2.w;
        }
        a4[j] = a.dz_add ? ld4(a.dz_add + at[j]) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < EB; ++j) {
        if (i0 + j * 256 >= tot) break;
        const float dv[4] = {d4[j].x, d4[j].y, d4[j].z, d4[j].w}, zv[4] = {z4[j].x, z4[j].y, z4[j].z, z4[j].w};
        const float uv[4] = {u4[j].x, u4[j].y, u4[j].z, u4[j].w}, av[4] = {a4[j].x, a4[j].y, a4[j].z, a4[j].w};
        float du[4], dzo[4];
        int v = vv[j];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float d = dv[q];
          const float dz = (a.prelu && !(zv[q] > 0.f)) ? w * d : d;
          const float mean = mnl[v], rstd = rsl[v];
          const float xh = (uv[q] - mean) * rstd;
          du[q] = a.use_running ? gml[v] * rstd * dz : gml[v] * rstd * (dz - sdl[v] * inv - xh * sxl[v] * inv);
          dzo[q] = a.dz_add ? dz + av[q] : dz;
          v = v + 1 == V ? 0 : v + 1;
        }
        *reinterpret_cast<float4*>(a.du + at[j]) = make_float4(du[0], du[1], du[2], du[3]);
        if (a.dz_out) *reinterpret_cast<float4*>(a.dz_out + at[j]) = make_float4(dzo[0], dzo[1], dzo[2], dzo[3]);
      }
    }
    return;
  }
  constexpr int EB = 4;  // elements per thread per batch, loads issued first
  for (int k = 0; k < ns; ++k)
  for (int e0 = tid; e0 < T * V; e0 += EB * 256) {
    const size_t base = ((size_t)(n + k) * C + c) * T * V;
    float dv[EB], zv[EB], uv[EB];
#pragma unroll
    for (int j = 0; j < EB; ++j) {
      const int e = e0 + j * 256;
      const size_t i = base + e;
      const bool in = e < T * V;
      dv[j] = in ? a.dout[i] : 0.f;
      zv[j] = (in && a.prelu) ? a.zsave[i] : 0.f;
      uv[j] = in ? (a.x2 ? a.x[i] + a.x2[i] : a.x[i]) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < EB; ++j) {
      const int e = e0 + j * 256;
      if (e >= T * V) break;
      const size_t i = base + e;
      const int v = e % V;
      const float d = dv[j];
      const float dz = (a.prelu && !(zv[j] > 0.f)) ? w * d : d;
      const float mean = mnl[v], rstd = rsl[v];
      const float xh = (uv[j] - mean) * rstd;
      a.du[i] = a.use_running ? gml[v] * rstd * dz : gml[v] * rstd * (dz - sdl[v] * inv - xh * sxl[v] * inv);
      if (a.dz_out) a.dz_out[i] = a.dz_add ? dz + a.dz_add[i] : dz;
    }
  }
}

// ---------------------------------------------------------------------------
// model boundary, loss and metric
// ---------------------------------------------------------------------------
__global__ void k_prep_nctv(const float* x, int B, int T, int V, int C, float* X0) {
  const size_t tot = (size_t)B * 2 * C * T * V;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    size_t r = e;
    const int v = r % V; r /= V;
    const int t = r % T; r /= T;
    const int c = r % (2 * C);
    const int n = r / (2 * C);
    const float* xs = x + (size_t)n * T * V * C;
    const int cc = c < C ? c : c - C;
    const float val = xs[((size_t)t * V + v) * C + cc];
    X0[e] = c < C ? val : val - xs[((size_t)(T - 1) * V + v) * C + cc];
  }
}

__global__ void k_out_ntvc(const float* O, const float* x, int B, int T, int V, int C, float* y) {
  const size_t tot = (size_t)B * T * V * C;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    size_t r = e;
    const int c = r % C; r /= C;
    const int v = r % V; r /= V;
    const int t = r % T;
    const int n = r / T;
    y[e] = O[(((size_t)n * C + c) * T + t) * V + v] + x[(((size_t)n * T + T - 1) * V + v) * C + c];
  }
}

// one thread per (n, v, c): the T-long column, then the x[T-1] terms
__global__ void k_prep_nctv_bwd(const float* dX0, const float* dy, int B, int T, int V, int C, float* dx) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * V * C) return;
  const int c = e % C, v = (e / C) % V, n = e / (C * V);
  const size_t TV = (size_t)T * V;
  const float* d0 = dX0 + ((size_t)n * 2 * C + c) * TV + v;
  const float* d1 = d0 + (size_t)C * TV;
  float last = 0.f;
  for (int t = 0; t < T; ++t) {
    const size_t o = (((size_t)n * T + t) * V + v) * C + c;
    dx[o] = d0[t * V] + d1[t * V];
    last += dy[o] - d1[t * V];
  }
  dx[(((size_t)n * T + T - 1) * V + v) * C + c] += last;
}

__global__ void k_out_ntvc_bwd(const float* dy, int B, int T, int V, int C, float* dO) {
  const size_t tot = (size_t)B * T * V * C;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    size_t r = e;
    const int v = r % V; r /= V;
    const int t = r % T; r /= T;
    const int c = r % C;
    const int n = r / C;
    dO[e] = dy[(((size_t)n * T + t) * V + v) * C + c];
  }
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__global__ void k_dropout(const float* in, float* out, size_t n, float p, unsigned long long seed,
                          const unsigned long long* seedp) {
  if (seedp) seed = *seedp;  // DSTD_TRAIN_SEED_DEVICE (a seed drawn on the device: graph replays)
  const float keep_scale = 1.f / (1.f - p);
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const unsigned long long h = mix64(seed * 0x9e3779b97f4a7c15ULL + e);
    const float u = (float)(h >> 40) * (1.f / 16777216.f);  // [0, 1), 24 bits
    out[e] = u >= p ? in[e] * keep_scale : 0.f;
  }
}

constexpr int kLossBlocks = 128;

__global__ void k_mpjpe_partial(const float* p, const float* q, size_t npts, float* partials) {
  __shared__ float red[kRedThreads / 64];
  float s = 0.f;
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < npts; k += (size_t)gridDim.x * blockDim.x) {
    const float dx = p[3 * k] - q[3 * k], dy = p[3 * k + 1] - q[3 * k + 1], dz = p[3 * k + 2] - q[3 * k + 2];
    s += sqrtf(dx * dx + dy * dy + dz * dz);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

__global__ void k_mpjpe_final(const float* partials, int n, size_t npts, float* out) {
  __shared__ float red[kRedThreads / 64];
  float s = 0.f;
  for (int e = threadIdx.x; e < n; e += blockDim.x) s += partials[e];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = s / (float)npts;
}

__global__ void k_mpjpe_bwd(const float* p, const float* q, size_t npts, const float* gscale, float scale,
                            float* dp) {
  const float g = (gscale ? *gscale : 1.f) * scale / (float)npts;
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < npts; k += (size_t)gridDim.x * blockDim.x) {
    const float dx = p[3 * k] - q[3 * k], dy = p[3 * k + 1] - q[3 * k + 1], dz = p[3 * k + 2] - q[3 * k + 2];
    const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
    // torch.norm backward: 0 at the kink
    const float f = nrm > 0.f ? g / nrm : 0.f;
    dp[3 * k] = f * dx;
    dp[3 * k + 1] = f * dy;
    dp[3 * k + 2] = f * dz;
  }
}

// one workgroup per eval frame
__global__ void k_frame_mpjpe(const float* seqs, const float* outs, int B, int T, int D, int t_out0,
                              const int* used_pos, int n_used, const int* joint_src, const int* frames,
                              float* sums) {
  __shared__ float red[kRedThreads / 64];
  const int k = blockIdx.x, f = frames[k], J = D / 3;
  float s = 0.f;
  for (int e = threadIdx.x; e < B * J; e += blockDim.x) {
    const int n = e / J, j = e - n * J;
    const float* tg = seqs + ((size_t)n * T + f) * D;
    const int src = joint_src[j];
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int d = 3 * src + c;
      const int u = used_pos[d];
      const float pv = (u >= 0 && f >= t_out0) ? outs[((size_t)n * (T - t_out0) + (f - t_out0)) * n_used + u] : tg[d];
      const float df = tg[3 * j + c] - pv;
      acc = fmaf(df, df, acc);
    }
    s += sqrtf(acc);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) sums[k] += s / J;
}

int grid_for(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 4096); }

}  // namespace

// reduce GEMMs on 96-wide tiles split up to twice as far (one tile, e.g. the
// 68 x 65 packed-conv [W | b] gradient, must still fill the chip)
constexpr int kMaxSplit96 = 2 * kMaxSplit;
size_t gemm_scratch_floats(int M, int N) { return (size_t)kMaxSplit96 * M * N; }

namespace {
template <class K, class... Args>
void sk_go(K kern, int grid, size_t lds, hipStream_t s, Args... args) {
  static bool attr = false;  // (per instantiation) allow > 64 KB of dynamic LDS
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  kern<<<grid, 256, lds, s>>>(args...);
}
#ifndef DSTD_GEMM_STREAM  // (r04u: B=256 step 27.9 -> 25.2 ms, B=32 -0.5%; 0 = the panel / tile kernels)
#define DSTD_GEMM_STREAM 1
#endif
template <int MF, int KS>
hipError_t cs_go(const Gemm& g, int ntile, hipStream_t s) {
  static const int occ = [] {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k_conv_stream<MF, KS>, 256, 0) != hipSuccess ||
        nb < 1)
      nb = 1;
    (void)hipGetLastError();
    return nb;
  }();
  static const int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  const long items = (long)g.nb1 * g.nb2 * ntile;
  // A small product (the config-5 batch: ~3.7k items) takes half the resident
  // workgroups, leaving CUs to the weight-gradient stream's reductions that
  // run beside it (B=32 step -1.3%); a large one the whole chip (half of it
  // measured +2% at B=256; profiles/r04w_train_ab.txt)
#ifndef DSTD_CS_GRID_DIV  // (experiments: a fixed divisor)
  const int div = items < 16384 ? 2 : 1;
#else
  const int div = DSTD_CS_GRID_DIV;
#endif
  const int grid = (int)std::max(1L, std::min((long)cus * occ / div, (items + 3) / 4));
  CsArgs ca;
  ca.ntile = ntile;
  ca.nb2 = g.nb2;
  ca.b_bytes = (uint32_t)(((long long)(g.K - 1) * g.b_k + g.N) * 4);
  ca.c_bytes = (uint32_t)(((long long)(g.M - 1) * g.c_m + g.N) * 4);
  k_conv_stream<MF, KS><<<grid, 256, 0, s>>>(g, ca);
  return hipGetLastError();
}
template <int MF>
hipError_t cs_ks(const Gemm& g, int ntile, hipStream_t s) {
  const int ks = cdiv(g.K, 4);
  if (ks <= 4) return cs_go<MF, 4>(g, ntile, s);
  if (ks <= 6) return cs_go<MF, 6>(g, ntile, s);  // (K = 23: temporal dM at V = 23)
  if (ks <= 8) return cs_go<MF, 8>(g, ntile, s);
  if (ks <= 10) return cs_go<MF, 10>(g, ntile, s);  // (K = 40: conv_rm's transposed product, spatial)
  if (ks <= 12) return cs_go<MF, 12>(g, ntile, s);  // (K = 44 / 46: temporal conv_rm)
  if (ks <= 16) return cs_go<MF, 16>(g, ntile, s);
  if (ks <= 17) return cs_go<MF, 17>(g, ntile, s);
  return cs_go<MF, 20>(g, ntile, s);
}
// hipErrorNotSupported: not a streaming shape (nothing launched)
hipError_t gemm_stream(const Gemm& g, hipStream_t s) {
  // (one A shared by every batch: it is staged once per workgroup)
  if (!DSTD_GEMM_STREAM || g.reduce || g.a_b1 || g.a_b2 || g.b_n != 1 || g.c_n != 1 || g.b_ones_last || g.nseg || g.M > kCsMax ||
      g.K > kCsMax || g.K < 1 || g.N < 16)
    return hipErrorNotSupported;
  const long long nbat = (long long)g.nb1 * g.nb2;
  const int ntile = cdiv(g.N, 16 * DSTD_CS_NT);  // items per batch
  // 32-bit buffer offsets over one batch's panels
  // (rows past K / M are read / written at offsets past the buffer range: the
  // padded k-steps and row tiles must stay below 2^31 bytes too)
  if (nbat * ntile >= (1LL << 31) || g.b_k < g.N || g.c_m < g.N || ((long long)g.K + 84) * g.b_k * 4 >= (1LL << 31) ||
      ((long long)g.M + 16) * g.c_m * 4 >= (1LL << 31))
    return hipErrorNotSupported;
#ifdef DSTD_GEMM_LOG
  fprintf(stderr, "gemm stream M %d N %d K %d nb %lld beta %g bias %d d_out %d stream %p\n", g.M, g.N, g.K, nbat, g.beta,
          g.bias_m != nullptr, g.d_out != nullptr, (void*)s);
#endif
  switch (cdiv(g.M, 16)) {
    case 1: return cs_ks<1>(g, ntile, s);
    case 2: return cs_ks<2>(g, ntile, s);
    case 3: return cs_ks<3>(g, ntile, s);
    case 4: return cs_ks<4>(g, ntile, s);
    default: return cs_ks<5>(g, ntile, s);
  }
}
// hipErrorNotSupported: not a skinny shape (nothing launched)
hipError_t gemm_skinny(const Gemm& g, float* scratch, hipStream_t s) {
  const int nbat = g.nb1 * g.nb2;
  // Only the shape class where it measured faster than k_gemm (the 1x1-conv
  // forward, K = Cin = 64: 20.5 vs 25.5 us at the config-5 batch,
  // profiles/r03v_skinny_micro.txt); conv dx (K = 68, beta 1), conv_rm (d_out)
  // and its transposed product (K = A) stay on k_gemm.
  if (!g.reduce && !g.a_b1 && !g.a_b2 && g.b_n == 1 && g.c_n == 1 && !g.b_ones_last && !g.d_out && !g.nseg && g.beta == 0.f &&
      g.M <= kSkMax && g.K <= kSkMax && g.K >= 48 && g.N >= 64) {
    const int MF = cdiv(g.M, 16), K4 = rup(g.K, 4), KP = sk_pitch(K4, 4), BP = sk_pitch(kSkPT, 16);
    const size_t lds = sizeof(float) * ((size_t)MF * 16 * KP + (size_t)K4 * BP);
    const int grid = nbat * cdiv(g.N, kSkPT);
#ifdef DSTD_GEMM_LOG
    fprintf(stderr, "gemm skinny MF %d M %d N %d K %d nb %d beta %g bias %d stream %p\n", MF, g.M, g.N, g.K, nbat, g.beta,
            g.bias_m != nullptr, (void*)s);
#endif
    const int vec = g.N % 4 == 0 && g.b_k % 4 == 0 && g.b_b1 % 4 == 0 && g.b_b2 % 4 == 0 &&
                    ((uintptr_t)g.B & 15) == 0;
    switch (MF) {
      case 1: sk_go(k_skinny_panel<1>, grid, lds, s, g, KP, BP, vec); break;
      case 2: sk_go(k_skinny_panel<2>, grid, lds, s, g, KP, BP, vec); break;
      case 3: sk_go(k_skinny_panel<3>, grid, lds, s, g, KP, BP, vec); break;
      case 4: sk_go(k_skinny_panel<4>, grid, lds, s, g, KP, BP, vec); break;
      default: sk_go(k_skinny_panel<5>, grid, lds, s, g, KP, BP, vec); break;
    }
    return hipGetLastError();
  }
  return hipErrorNotSupported;
}
}  // namespace

hipError_t gemm(const Gemm& g, float* scratch, hipStream_t s, GemmFinish* defer) {
  if (defer) defer->nsplit = 0;
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  if (g.d_out && (g.reduce || !g.d_A || !g.d_alpha)) return hipErrorInvalidValue;
  {
    const hipError_t e = gemm_stream(g, s);
    if (e != hipErrorNotSupported) return e;
  }
  {
    const hipError_t e = gemm_skinny(g, scratch, s);
    if (e != hipErrorNotSupported) return e;
  }
  // tile edge per operand: 32 / 64, and 96 for a reduce GEMM's 65..96 extent
  // (the packed conv's [W | b] gradient is 68 x 65: one 96 x 96 tile instead
  // of four 64 x 64 ones, each operand read once instead of twice;
  // B=32 training step 5.95 -> 5.69 ms, profiles/r03y_gemm96_ab.txt)
  const bool t96 = g.reduce && scratch;
  auto edge = [&](int x) { return x <= 32 ? 32 : (x <= 64 || !t96 || x > 96) ? 64 : 96; };
  const int TM = edge(g.M), TN = edge(g.N);
  const int tiles = cdiv(g.M, TM) * cdiv(g.N, TN);
  const int nbat = g.nb1 * g.nb2;
  int nsplit = 1, kch = 1, kc_len = rup(std::max(g.K, 1), 16);
  if (g.reduce && scratch) {
    // ~1024 workgroups, each reducing >= 64 values of K: split the K range of
    // every batch into kch chunks so small batch counts still fill the chip
    const int ksteps = cdiv(g.K, 16);
    nsplit = std::max(1, std::min(TM == 96 || TN == 96 ? kMaxSplit96 : kMaxSplit, 512 / tiles));
    kch = std::max(1, std::min(cdiv(nsplit, nbat), cdiv(ksteps, 4)));
    kc_len = cdiv(ksteps, kch) * 16;
    kch = cdiv(g.K, kc_len);
    nsplit = std::min(nsplit, nbat * kch);
  }
  dim3 grid(cdiv(g.N, TN), cdiv(g.M, TM), g.reduce ? nsplit : nbat);
  float* part = nsplit > 1 ? scratch : nullptr;
#ifdef DSTD_GEMM_LOG  // (debug builds: the shape mix of a training step)
  fprintf(stderr, "gemm tile %dx%d M %d N %d K %d nb %d reduce %d nsplit %d a_m %lld a_k %lld b_k %lld b_n %lld c_m %lld "
          "c_n %lld d_out %d nseg %d bias %d beta %g stream %p\n", TM, TN, g.M, g.N, g.K, nbat, g.reduce, nsplit, g.a_m,
          g.a_k, g.b_k, g.b_n, g.c_m, g.c_n, g.d_out != nullptr, g.nseg, g.bias_m != nullptr, g.beta, (void*)s);
#endif
#define DSTD_GEMM_GO(tm, tn) \
  if (TM == tm && TN == tn) k_gemm<tm, tn><<<grid, 256, 0, s>>>(g, nsplit, kch, kc_len, part)
  DSTD_GEMM_GO(32, 32); else DSTD_GEMM_GO(32, 64); else DSTD_GEMM_GO(64, 32); else DSTD_GEMM_GO(64, 64);
  else DSTD_GEMM_GO(96, 96); else DSTD_GEMM_GO(96, 64); else DSTD_GEMM_GO(64, 96); else DSTD_GEMM_GO(96, 32);
  else DSTD_GEMM_GO(32, 96);
#undef DSTD_GEMM_GO
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || nsplit == 1) return e;
  if (defer) {  // the caller launches the finish (finish_set)
    defer->g = g;
    defer->nsplit = nsplit;
    defer->part = part;
    return hipSuccess;
  }
  k_gemm_finish<<<cdiv(g.M * g.N, 16), 256, 0, s>>>(g, nsplit, part);
  return hipGetLastError();
}

namespace {
// a-chunk per workgroup: the widest chunk (<= 4, one a per wave) whose slabs
// and D tiles fit 80 KB of LDS (two workgroups per CU)
constexpr size_t kAggLds = 80 * 1024;
void agg_tile(int NN, int& RK, int& P) {
  RK = rup(NN, 4);
  const int jf = cdiv(NN, 16);
  P = 16 * ((jf & 1) ? jf : jf + 1);  // 4 B-operand rows of 16 hit distinct banks
}
size_t agg_lds(bool bwd, bool df, int C, int NN, int ac, int& QP, int& RK, int& P) {
  QP = (ac * NN) | 1;
  agg_tile(NN, RK, P);
  return sizeof(float) * ((size_t)(bwd ? 2 : 1) * C * QP + (df ? (size_t)ac * RK * P : 0));
}
template <class K>
void agg_go(K kern, dim3 grid, dim3 block, size_t lds, const AggArgs& g, hipStream_t s) {
  static bool attr = false;  // (per instantiation) allow > 64 KB of dynamic LDS
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  kern<<<grid, block, lds, s>>>(g);
}
bool agg_ok(const AggArgs& g) {
  return g.C > 0 && g.C <= kAggMaxC && g.NN > 0 && g.NN <= kAggMaxNN && g.A > 0;
}
int agg_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}
// Channel-chunk kernels, spatial: below DSTD_AGG_SPLIT_WG (sample, chunk)
// workgroups per CU, the frames of each are split over several workgroups of
// apg frames (apg * V a multiple of 4: 16-byte runs stay aligned), so the
// config-5 batch (64 samples x 4 chunks: one workgroup and 4 waves per CU)
// gets ~per_cu workgroups per CU (2 each way: B=32 step 4.725 -> 4.671 ms;
// forward alone 4.698, backward alone 4.683, a forward target of 4: 4.739;
// profiles/r05q_agg_split_ab.txt); sets g.asplit / g.apg and returns the
// widest slab (floats per channel row)
#ifndef DSTD_AGG_SPLIT_WG  // forward (k_aggc); experiments: 0 = no split
#define DSTD_AGG_SPLIT_WG 2
#endif
#ifndef DSTD_AGGB_SPLIT_WG  // backward (k_aggc_bwd)
#define DSTD_AGGB_SPLIT_WG 2
#endif
int agg_split(AggArgs& g, int B, bool temporal, int per_cu, int cw = 16) {
  g.asplit = 1;
  g.apg = g.A;
  const int wgs = B * cdiv(g.C, cw), cus = agg_cus();
  if (temporal || per_cu <= 0 || wgs >= per_cu * cus) return g.TV;
  const int m = (g.V % 4 == 0) ? 1 : (g.V % 2 == 0) ? 2 : 4;
  const int want = std::min(g.A, cdiv(per_cu * cus, wgs));
  g.apg = std::min(g.A, rup(cdiv(g.A, want), m));
  g.asplit = cdiv(g.A, g.apg);
  return g.apg * g.V;
}
// a-chunk kernel: fwd, bwd dD + dF (df) or bwd dD only
hipError_t agg_launch_a(bool bwd, bool df, AggArgs g, int B, int temporal, hipStream_t s) {
  if (!agg_ok(g)) return hipErrorNotSupported;
  int ac = std::min(g.A, 4);
  size_t lds = agg_lds(bwd, df, g.C, g.NN, ac, g.QP, g.RK, g.P);
  while (ac > 1 && lds > kAggLds) lds = agg_lds(bwd, df, g.C, g.NN, --ac, g.QP, g.RK, g.P);
  if (lds > 160 * 1024) return hipErrorNotSupported;
  g.AC = ac;
  const dim3 grid(B * cdiv(g.A, ac)), block(64 * std::min(ac, 4));
  // channel fragments 1, 2, 4 (3 runs as 4); column fragments 1-4
  const int mf = cdiv(g.C, 16) == 3 ? 4 : cdiv(g.C, 16), jf = cdiv(g.NN, 16);
  auto pick_jf = [&](auto tb, auto bb, auto mfc, auto dfc) {
    constexpr bool T_ = decltype(tb)::value, B_ = decltype(bb)::value, D_ = decltype(dfc)::value;
    constexpr int M_ = decltype(mfc)::value;
    switch (jf) {
      case 1: agg_go(k_agg<T_, B_, M_, 1, D_>, grid, block, lds, g, s); break;
      case 2: agg_go(k_agg<T_, B_, M_, 2, D_>, grid, block, lds, g, s); break;
      case 3: agg_go(k_agg<T_, B_, M_, 3, D_>, grid, block, lds, g, s); break;
      default: agg_go(k_agg<T_, B_, M_, 4, D_>, grid, block, lds, g, s); break;
    }
  };
  using T1 = std::true_type;
  using F0 = std::false_type;
  auto pick_mf = [&](auto tb, auto bb, auto dfc) {
    if (mf == 1) pick_jf(tb, bb, std::integral_constant<int, 1>(), dfc);
    else if (mf == 2) pick_jf(tb, bb, std::integral_constant<int, 2>(), dfc);
    else pick_jf(tb, bb, std::integral_constant<int, 4>(), dfc);
  };
  if (!bwd) temporal ? pick_mf(T1(), F0(), T1()) : pick_mf(F0(), F0(), T1());
  else if (df) temporal ? pick_mf(T1(), T1(), T1()) : pick_mf(F0(), T1(), T1());
  else temporal ? pick_mf(T1(), T1(), F0()) : pick_mf(F0(), T1(), F0());
  return hipGetLastError();
}
// channel-chunk kernel: fwd (trans 0) or dF (trans 1)
hipError_t agg_launch_c(bool trans, AggArgs g, int B, int temporal, hipStream_t s) {
  if (!agg_ok(g)) return hipErrorNotSupported;
  // channels per chunk: 16; the spatial forward DSTD_AGG_CW_SP (16 or 64: a
  // wider chunk reads D once per chunk, but 64 measured +0.7% at B=32, +1.7%
  // at B=256 -- half its waves idle over 4 frames; profiles/r05jj_agg_cw_ab.txt)
#ifndef DSTD_AGG_CW_SP
#define DSTD_AGG_CW_SP 16
#endif
  // (row tiles 1 or 4: 2 and 3 run as 4, cv masking the rest)
  const int mfc = temporal || trans || DSTD_AGG_CW_SP < 64 || g.C <= 16 ? 1 : 4, cw = 16 * mfc;
  agg_tile(g.NN, g.RK, g.P);
  g.QP = agg_split(g, B, temporal, DSTD_AGG_SPLIT_WG, cw);
  while ((g.QP & 63) != 4) ++g.QP;
  const size_t lds = sizeof(float) * ((size_t)cw * g.QP + (size_t)(kAggcThreads / 64) * g.RK * g.P);
  if (lds > 160 * 1024) return hipErrorNotSupported;
  g.vec = (g.TV % 4 == 0 && g.xs % 4 == 0 && g.os % 4 == 0 && ((uintptr_t)g.X & 15) == 0 &&
           ((uintptr_t)g.O & 15) == 0);
  const dim3 grid(B * cdiv(g.C, cw) * g.asplit), block(kAggcThreads);
  const int jf = cdiv(g.NN, 16);
  auto pick = [&](auto tb, auto rb, auto mb) {
    constexpr bool T_ = decltype(tb)::value, R_ = decltype(rb)::value;
    constexpr int M_ = decltype(mb)::value;
    switch (jf) {
      case 1: agg_go(k_aggc<T_, R_, 1, M_>, grid, block, lds, g, s); break;
      case 2: agg_go(k_aggc<T_, R_, 2, M_>, grid, block, lds, g, s); break;
      case 3: agg_go(k_aggc<T_, R_, 3, M_>, grid, block, lds, g, s); break;
      default: agg_go(k_aggc<T_, R_, 4, M_>, grid, block, lds, g, s); break;
    }
  };
  using T1 = std::true_type;
  using F0 = std::false_type;
  using M1 = std::integral_constant<int, 1>;
  if (temporal) trans ? pick(T1(), T1(), M1()) : pick(T1(), F0(), M1());
  else if (trans) pick(F0(), T1(), M1());
  else if (mfc == 1) pick(F0(), F0(), M1());
#if DSTD_AGG_CW_SP >= 64
  else pick(F0(), F0(), std::integral_constant<int, 4>());
#endif
  return hipGetLastError();
}
AggArgs agg_geom(int C, int T, int V, int temporal) {
  AggArgs g{};
  g.C = C;
  g.A = temporal ? V : T;
  g.NN = temporal ? T : V;
  g.V = V;
  g.TV = T * V;
  return g;
}
}  // namespace

hipError_t agg_fwd(const float* F, long long fs, const float* D, float* y, long long ys, float beta, int B, int C,
                   int T, int V, int temporal, hipStream_t s) {
  AggArgs g = agg_geom(C, T, V, temporal);
  g.X = F, g.xs = fs, g.Dm = D, g.O = y, g.os = ys, g.beta = beta;
  return agg_launch_c(false, g, B, temporal, s);
}

// which kernel the last agg_bwd dispatched (dstd_debug_aggb_last): the
// channel-chunk kernel's chunk width, or 0 for the two-launch path
static std::atomic<int> g_aggb_last{-1};

hipError_t agg_bwd(const float* F, long long fs, const float* dy, long long dys, const float* D, float* dF,
                   long long dfs, float* dD, int B, int C, int T, int V, int temporal, hipStream_t s, float* dDpart,
                   int* nparts) {
  AggArgs g = agg_geom(C, T, V, temporal);
  g.X = F, g.xs = fs, g.Y0 = dy, g.y0s = dys, g.Dm = D, g.O = dF, g.os = dfs, g.dD = dD;
  *nparts = 0;
  if (!agg_ok(g)) return hipErrorNotSupported;
  // dF on the channel-chunk backward kernel, dD as its per-chunk partials
  // (dDpart; one chunk: dD itself); else dF on the channel-chunk kernel and
  // dD on the a-chunk kernel
  // channels per chunk: 16 (temporal); spatial DSTD_AGGB_CW_SP: one chunk
  // of all 64 channels reads D once and leaves one dD (no partials for
  // adj_bwd_part to sum): B=32 step -1.3%, profiles/r05gg_aggb_cw_ab.txt
#ifndef DSTD_AGGB_CW_SP
#define DSTD_AGGB_CW_SP 64
#endif
  // (row tiles 1, 2 or 4: 3 runs as 4, cv masking the fourth).  When the
  // preferred chunk's slab does not fit LDS (large batches split fewer frames
  // per workgroup: H36M / 3DPW at B=256 need 231-264 KB at 64 channels) the
  // 16-channel chunk is tried before the two-launch path (dF kernel + dD
  // a-chunk kernel)
  const int mf_pref = temporal ? 1 : std::min(DSTD_AGGB_CW_SP / 16, cdiv(C, 16));
  const int tries[2] = {mf_pref == 3 ? 4 : mf_pref, 1};
  for (int ti = 0; ti < (tries[0] == 1 ? 1 : 2); ++ti) {
    const int mfc = tries[ti], cw = 16 * mfc;
    const int cch = cdiv(C, cw);
    if (!(cch == 1 || dDpart)) continue;
    g.dD = cch > 1 ? dDpart : dD;
    g.B = B;
    agg_tile(g.NN, g.RK, g.P);
    g.QP = agg_split(g, B, temporal, DSTD_AGGB_SPLIT_WG, cw);
    while ((g.QP & 63) != 4) ++g.QP;
    const int nth = aggcb_threads(temporal);
    const size_t lds = sizeof(float) * ((size_t)2 * cw * g.QP + (size_t)(nth / 64) * g.RK * g.P);
    if (lds > 160 * 1024) continue;
    *nparts = cch;
    g_aggb_last.store(cw, std::memory_order_relaxed);
    g.vec = (g.TV % 4 == 0 && g.xs % 4 == 0 && g.os % 4 == 0 && g.y0s % 4 == 0 && ((uintptr_t)g.X & 15) == 0 &&
             ((uintptr_t)g.O & 15) == 0 && ((uintptr_t)g.Y0 & 15) == 0);
    const dim3 grid(B * cch * g.asplit), block(nth);
    const int jf = cdiv(g.NN, 16);
    auto pick = [&](auto tb, auto mb) {
      constexpr bool T_ = decltype(tb)::value;
      constexpr int M_ = decltype(mb)::value;
      switch (jf) {
        case 1: agg_go(k_aggc_bwd<T_, 1, M_>, grid, block, lds, g, s); break;
        case 2: agg_go(k_aggc_bwd<T_, 2, M_>, grid, block, lds, g, s); break;
        case 3: agg_go(k_aggc_bwd<T_, 3, M_>, grid, block, lds, g, s); break;
        default: agg_go(k_aggc_bwd<T_, 4, M_>, grid, block, lds, g, s); break;
      }
    };
    if (temporal) pick(std::true_type(), std::integral_constant<int, 1>());
    else if (mfc == 1) pick(std::false_type(), std::integral_constant<int, 1>());
#if DSTD_AGGB_CW_SP >= 32
    else if (mfc == 2) pick(std::false_type(), std::integral_constant<int, 2>());
#endif
#if DSTD_AGGB_CW_SP >= 64
    else pick(std::false_type(), std::integral_constant<int, 4>());
#endif
    return hipGetLastError();
  }
  *nparts = 1;
  g.dD = dD;
  g_aggb_last.store(0, std::memory_order_relaxed);
  AggArgs c = agg_geom(C, T, V, temporal);  // dF = dy . D^T per a
  c.X = dy, c.xs = dys, c.Dm = D, c.O = dF, c.os = dfs;
  const hipError_t e = agg_launch_c(true, c, B, temporal, s);
  if (e != hipSuccess) {
    *nparts = 0;  // (NotSupported: the caller runs both products)
    return e;
  }
  const hipError_t ed = agg_launch_a(true, false, g, B, temporal, s);  // dD
  if (ed == hipErrorNotSupported) *nparts = 0;  // (dF is done; the caller recomputes both)
  return ed;
}



}  // namespace train
}  // namespace dstd

extern "C" int dstd_debug_aggb_last(void) { return dstd::train::g_aggb_last.load(std::memory_order_relaxed); }

namespace dstd {
namespace train {

hipError_t tanh_outer_fwd(const float* P, const float* Q, PQView v, int B, int R, int A, int NN, float* M,
                          hipStream_t s) {
  if (NN > kTanhMaxNN) return hipErrorInvalidValue;
  k_tanh_outer_fwd<<<B * R * A, 256, 0, s>>>(P, Q, v, R, A, NN, M);
  return hipGetLastError();
}

hipError_t tanh_outer_bwd(const float* M, const float* dM, PQView v, int B, int R, int A, int NN, float* dP,
                          float* dQ, hipStream_t s) {
  const size_t lds = (size_t)NN * (NN + 1) * sizeof(float);  // 66 KB at the T = 128 envelope top
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k_tanh_outer_bwd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  k_tanh_outer_bwd<<<B * R * A, 256, lds, s>>>(M, dM, v, R, A, NN, dP, dQ);
  return hipGetLastError();
}


int adj_bwd_chunks(int B, int A) { return std::max(1, std::min(std::min(B, 16), cdiv(512, A))); }

size_t adj_bwd_scratch_floats(int B, int A, int NN2) {
  const int nch = adj_bwd_chunks(B, A);
  return (size_t)nch * A * NN2 + 3 * (size_t)nch * A * cdiv(NN2, 256) + 64;  // pal: doubles
}

#ifndef DSTD_ADJ_SPLIT  // (r04u: B=256 step 27.9 -> 27.0 ms, B=32 neutral; 0 = one column block)
#define DSTD_ADJ_SPLIT 1
#endif
namespace {
// the partials' layout in scratch (256-byte aligned workspace carve): pal
// (doubles), then pdA, then pbr
struct AdjBwdScratch {
  int nch, nij;
  double* pal;
  float *pdA, *pbr;
  AdjBwdScratch(float* scratch, int B, int A, int NN2)
      : nch(adj_bwd_chunks(B, A)), nij(DSTD_ADJ_SPLIT ? cdiv(NN2, 256) : 1) {
    pal = reinterpret_cast<double*>(scratch);
    pdA = scratch + 2 * (size_t)nch * A * nij;
    pbr = pdA + (size_t)nch * A * NN2;
  }
};
}  // namespace

hipError_t adj_bwd_part(float* dD, const float* E, const float* alpha, int B, int A, int NN2, float* scratch,
                        hipStream_t s, const float* dDpart, int nparts) {
  if (nparts > 1 && !dDpart) return hipErrorInvalidValue;
  if (A > 256) return hipErrorInvalidValue;  // (k_adj_bwd_finish: S threads per row, A * S <= 256)
  const AdjBwdScratch P(scratch, B, A, NN2);
  k_adj_bwd_part<<<dim3(A, P.nch, P.nij), 256, 0, s>>>(dD, E, alpha, B, A, NN2, P.nch, P.pdA, P.pbr, P.pal, dDpart,
                                                       nparts);
  return hipGetLastError();
}

hipError_t adj_bwd_finish(int B, int A, int NN2, float* dA, float* dbrm, float* dalpha, const float* scratch,
                          hipStream_t s, int assign_dA, float* dW2, const float* Amul) {
  if (dW2 && !Amul) return hipErrorInvalidValue;
  if (A > 256) return hipErrorInvalidValue;
  const AdjBwdScratch P(const_cast<float*>(scratch), B, A, NN2);
  const AdjFinishArgs f{P.pdA, P.pbr, P.pal, A, NN2, P.nch, dA, dbrm, dalpha, assign_dA, dW2, Amul, P.nij};
  k_adj_bwd_finish<<<cdiv(NN2, 16) + 1, 256, 0, s>>>(f);
  return hipGetLastError();
}

hipError_t finish_set(int B, int A, int NN2, float* dA, float* dbrm, float* dalpha, const float* adj_scratch,
                      int assign_dA, float* dW2, const float* Amul, const GemmFinish* f0, const GemmFinish* f1,
                      hipStream_t s) {
  if (dW2 && !Amul) return hipErrorInvalidValue;
  if (A > 256) return hipErrorInvalidValue;
  const AdjBwdScratch P(const_cast<float*>(adj_scratch), B, A, NN2);
  FinishSetArgs a{};
  a.adj = AdjFinishArgs{P.pdA, P.pbr, P.pal, A, NN2, P.nch, dA, dbrm, dalpha, assign_dA, dW2, Amul, P.nij};
  a.na = cdiv(NN2, 16) + 1;
  const GemmFinish* f[2] = {f0, f1};
  for (int i = 0; i < 2; ++i) {
    const bool on = f[i] && f[i]->nsplit > 1;
    if (on) a.g[i] = f[i]->g;
    a.nsplit[i] = on ? f[i]->nsplit : 0;
    a.part[i] = on ? f[i]->part : nullptr;
    a.nb[i] = on ? cdiv(f[i]->g.M * f[i]->g.N, 16) : 0;
  }
  k_finish_set<<<a.na + a.nb[0] + a.nb[1], 256, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t adj_bwd(float* dD, const float* E, const float* alpha, int B, int A, int NN2, float* dA, float* dbrm,
                   float* dalpha, float* scratch, hipStream_t s, int assign_dA, const float* dDpart, int nparts,
                   float* dW2, const float* Amul) {
  if (dW2 && !Amul) return hipErrorInvalidValue;
  const hipError_t e = adj_bwd_part(dD, E, alpha, B, A, NN2, scratch, s, dDpart, nparts);
  if (e != hipSuccess) return e;
  return adj_bwd_finish(B, A, NN2, dA, dbrm, dalpha, scratch, s, assign_dA, dW2, Amul);
}

hipError_t copy_jobs(const CopyJobs& js, hipStream_t s) {
  if (js.n == 0) return hipSuccess;
  int mx = 1;
  for (int i = 0; i < js.n; ++i) mx = std::max(mx, js.j[i].rows * js.j[i].cols);
  k_copy_jobs<<<dim3(std::min(cdiv(mx, 256), 64), js.n), 256, 0, s>>>(js);
  return hipGetLastError();
}

hipError_t adj_param_grads(const float* dA, const float* A_s, float* dR_s, float* dW_s, size_t n, hipStream_t s) {
  k_adj_param_grads<<<grid_for(n), 256, 0, s>>>(dA, A_s, dR_s, dW_s, n);
  return hipGetLastError();
}

hipError_t scale_by(float* x, const float* alpha, size_t n, hipStream_t s) {
  k_scale_by<<<grid_for(n), 256, 0, s>>>(x, alpha, n);
  return hipGetLastError();
}

size_t reduce_scratch_floats(int M) { return (size_t)kRedSplit * M; }

hipError_t reduce_rows(const float* X, int M, int nb, int nj, long long sb, long long sm, long long sj, float* out,
                       float scale, float* scratch, hipStream_t s) {
  const long long tot = (long long)nb * nj;
  if (tot >= (1LL << 31)) return hipErrorInvalidValue;  // k_red_part_j indexes in int
  const bool by_m = sm == 1 && M > 1;
  // ~1024 workgroups, each with a useful amount of work
  const long long want = by_m ? std::min(kRedSplit, 1024 / cdiv(M, kRedThreads)) : std::min(kRedSplit, std::max(1, 1024 / M));
  const int splits = (int)std::max<long long>(1, std::min<long long>(want, by_m ? (tot + 15) / 16 : (tot + 1023) / 1024));
  if (by_m)
    k_red_part_m<<<dim3(cdiv(M, kRedThreads), splits), kRedThreads, 0, s>>>(X, M, nb, nj, sb, sj, splits, scratch);
  else
    k_red_part_j<<<dim3(M, splits), kRedThreads, 0, s>>>(X, M, nb, nj, sb, sm, sj, splits, scratch);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  k_red_finish<<<cdiv(M, 16), 256, 0, s>>>(scratch, M, splits, out, scale);
  return hipGetLastError();
}

int dot_partials() { return kDotBlocks; }

hipError_t dot(const float* x, const float* y, size_t n, float* out, float* partials, hipStream_t s) {
  k_dot_partial<<<kDotBlocks, kRedThreads, 0, s>>>(x, y, n, partials);
  k_sum_into<<<1, kRedThreads, 0, s>>>(partials, kDotBlocks, out);
  return hipGetLastError();
}

hipError_t sum_into(const float* partial, int n, float* out, hipStream_t s) {
  k_sum_into<<<1, kRedThreads, 0, s>>>(partial, n, out);
  return hipGetLastError();
}


hipError_t acc_mul(const float* a, const float* b, float* out, size_t n, hipStream_t s, const float* c,
                   int assign) {
  k_acc_mul<<<grid_for(n), 256, 0, s>>>(a, b, c, out, n, assign);
  return hipGetLastError();
}

// samples per apply workgroup: more than one only while >= 4096 workgroups
// remain (measured: 4 per workgroup -2.7% at B=256, +1% at B=32 paired)
// Separate merge + flat apply for large batches only: at the config-5 batch
// (3.8M elements per BN) the 30 merge launches cost more than the re-merges
// they save (+4%), at B=256 they save 2% (profiles/r04y_bn_sep_ab.txt).
// DSTD_BN_SEP=0 / 1 forces it.
bool bn_sep(long long total) {
#ifdef DSTD_BN_SEP
  (void)total;
  return DSTD_BN_SEP;
#else
  return total >= (1LL << 24);
#endif
}
#ifndef DSTD_BN_NOVEC  // (A/B builds: the scalar element loops)
constexpr bool kBnVec = true;
#else
constexpr bool kBnVec = false;
#endif
int bn_apply_samples(int Bg, int B, int C) {
#ifdef DSTD_BN_NS  // (experiments: samples per apply workgroup)
  if (Bg % DSTD_BN_NS == 0) return DSTD_BN_NS;
#endif
  // (>= 1024 workgroups: 4 samples each at the config-5 batch, a quarter of
  // the per-workgroup merges; B=32 step -1.4%, profiles/r04ad_bn_ns_ab.txt)
  for (int ns : {4, 2})
    if (Bg % ns == 0 && (size_t)C * (B / ns) >= 1024) return ns;
  return 1;
}

int bn_splits(int B, int T) { return std::max(1, std::min(kBnMaxSplits, cdiv(B * T, 64))); }

size_t bn_scratch_floats(int B, int C, int T, int V) {  // sized for up to 2 groups (+ DSTD_BN_SEP's scale / shift)
  return 2 * ((size_t)bn_splits(B, T) * C * V * 2 + (size_t)bn_splits(B, T) * C) + (size_t)2 * C * V + (size_t)4 * C * V;
}

hipError_t bn_train_fwd(const BnFwd& a, int B, int C, int T, int V, float* scratch, hipStream_t s) {
  if (V > kBnMaxV) return hipErrorInvalidValue;
  if (a.use_running && (!a.running_mean || !a.running_var)) return hipErrorInvalidValue;
  if (a.groups < 1 || a.groups > 2 || B % a.groups) return hipErrorInvalidValue;
  const int splits = bn_splits(B / a.groups, T);
  BnFwd b = a;
  b.cv = C * V;
  if (!a.use_running)
    k_bn_stats_part<<<dim3(C, splits * a.groups), kRedThreads, 0, s>>>(b, B, C, T, V, splits, scratch);
  if (a.sync && !a.use_running) {  // SyncBN: gather every rank's statistics
    const dstd_bn_sync& y = *a.sync;
    const long long n = (long long)a.groups * b.cv * 3;
    k_bn_local_stats<<<dim3(cdiv(b.cv, 256), a.groups), 256, 0, s>>>(b.cv, (B / a.groups) * T, splits, scratch,
                                                                     y.buf + (size_t)y.rank * n);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (y.fn(y.ctx, DSTD_COLL_ALLGATHER, y.buf, n, (void*)s) != 0) return collective_failed();
    b.gath = y.buf;
    b.world = y.world;
  }
  const long long total = (long long)B * C * T * V;
  const bool al = ((uintptr_t)a.x | (uintptr_t)a.x2 | (uintptr_t)a.res | (uintptr_t)a.out | (uintptr_t)a.zsave) % 16 == 0;
  if (bn_sep(total) && (T * V) % 4 == 0 && al && total < (1LL << 31)) {
    float* ss = scratch + (size_t)a.groups * splits * b.cv * 2;
    k_bn_merge<<<cdiv(b.cv, 256), 256, 0, s>>>(b, (B / a.groups) * T, splits, scratch, ss, C, V);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const long long q = total / 4;
    const int grid = (int)std::min<long long>(cdiv(q, 256), 8192);
    k_bn_apply_flat<<<grid, 256, 0, s>>>(b, B / a.groups, C, T * V, V, total, ss);
    return hipGetLastError();
  }
  const int ns = bn_apply_samples(B / a.groups, B, C);
  if (kBnVec && (T * V) % 4 == 0 && al && ns <= 4)
    k_bn_apply_merged<true><<<dim3(C, B / ns), 256, 0, s>>>(b, B, C, T, V, splits, scratch, ns);
  else
    k_bn_apply_merged<false><<<dim3(C, B / ns), 256, 0, s>>>(b, B, C, T, V, splits, scratch, ns);
  return hipGetLastError();
}

hipError_t bn_train_bwd(const BnBwd& a, int B, int C, int T, int V, float* scratch, float* dprelu, hipStream_t s) {
  if (V > kBnMaxV) return hipErrorInvalidValue;
  if (a.groups < 1 || a.groups > 2 || B % a.groups) return hipErrorInvalidValue;
  const int splits = bn_splits(B / a.groups, T);
  float* part = scratch;
  float* wpart = part + (size_t)a.groups * splits * C * V * 2;
  k_bn_bwd_part<<<dim3(C, splits * a.groups), kRedThreads, 0, s>>>(a, B, C, T, V, splits, part, wpart);
  BnBwd b = a;
  if (a.sync && !a.use_running) {  // SyncBN: sum every rank's sums and row counts
    const dstd_bn_sync& y = *a.sync;
    const int cv = C * V;
    k_bn_bwd_local_sums<<<dim3(cdiv(cv, 256), a.groups), 256, 0, s>>>(cv, a.groups, splits, (B / a.groups) * T, part,
                                                                      y.buf);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (y.fn(y.ctx, DSTD_COLL_ALLREDUCE_SUM, y.buf, (long long)a.groups * cv * 2 + a.groups, (void*)s) != 0)
      return collective_failed();
    b.gsum = y.buf;
  }
  const bool al = ((uintptr_t)a.x | (uintptr_t)a.x2 | (uintptr_t)a.zsave | (uintptr_t)a.dout | (uintptr_t)a.du |
                   (uintptr_t)a.dz_out | (uintptr_t)a.dz_add) % 16 == 0;
  {
    const long long total = (long long)B * C * T * V;
    if (bn_sep(total) && (T * V) % 4 == 0 && al && total < (1LL << 31)) {
      const int cv = C * V;
      float* sx = wpart + (size_t)splits * a.groups * C;
      k_bn_bwd_merge<<<cdiv(cv, 256), 256, 0, s>>>(b, splits, C, part, wpart, dprelu, sx, cv);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      const int grid = (int)std::min<long long>(cdiv(total / 4, 256), 8192);
      k_bn_bwd_apply_flat<<<grid, 256, 0, s>>>(b, B / a.groups, C, T * V, V, T, total, sx);
      return hipGetLastError();
    }
  }
  const int ns = bn_apply_samples(B / a.groups, B, C);
  if (kBnVec && (T * V) % 4 == 0 && al && ns <= 4)
    k_bn_bwd_apply_merged<true><<<dim3(C, B / ns), 256, 0, s>>>(b, B, C, T, V, splits, part, wpart, dprelu, ns);
  else
    k_bn_bwd_apply_merged<false><<<dim3(C, B / ns), 256, 0, s>>>(b, B, C, T, V, splits, part, wpart, dprelu, ns);
  return hipGetLastError();
}

hipError_t prep_nctv(const float* x, int B, int T, int V, int C, float* X0, hipStream_t s) {
  k_prep_nctv<<<grid_for((size_t)B * 2 * C * T * V), 256, 0, s>>>(x, B, T, V, C, X0);
  return hipGetLastError();
}

hipError_t out_ntvc(const float* O, const float* x, int B, int T, int V, int C, float* y, hipStream_t s) {
  k_out_ntvc<<<grid_for((size_t)B * C * T * V), 256, 0, s>>>(O, x, B, T, V, C, y);
  return hipGetLastError();
}

hipError_t prep_nctv_bwd(const float* dX0, const float* dy, int B, int T, int V, int C, float* dx, hipStream_t s) {
  k_prep_nctv_bwd<<<cdiv(B * V * C, 256), 256, 0, s>>>(dX0, dy, B, T, V, C, dx);
  return hipGetLastError();
}

hipError_t out_ntvc_bwd(const float* dy, int B, int T, int V, int C, float* dO, hipStream_t s) {
  k_out_ntvc_bwd<<<grid_for((size_t)B * C * T * V), 256, 0, s>>>(dy, B, T, V, C, dO);
  return hipGetLastError();
}

hipError_t dropout(const float* in, float* out, size_t n, float p, unsigned long long seed, hipStream_t s,
                   bool seed_on_device) {
  const unsigned long long* seedp = seed_on_device ? reinterpret_cast<const unsigned long long*>(seed) : nullptr;
  k_dropout<<<grid_for(n), 256, 0, s>>>(in, out, n, p, seedp ? 0ULL : seed, seedp);
  return hipGetLastError();
}

int mpjpe_partials() { return kLossBlocks; }

hipError_t mpjpe_fwd(const float* p, const float* q, size_t npts, float* out, float* partials, hipStream_t s) {
  k_mpjpe_partial<<<kLossBlocks, kRedThreads, 0, s>>>(p, q, npts, partials);
  k_mpjpe_final<<<1, kRedThreads, 0, s>>>(partials, kLossBlocks, npts, out);
  return hipGetLastError();
}

hipError_t mpjpe_bwd(const float* p, const float* q, size_t npts, const float* gscale, float scale, float* dp,
                     hipStream_t s) {
  k_mpjpe_bwd<<<grid_for(npts), 256, 0, s>>>(p, q, npts, gscale, scale, dp);
  return hipGetLastError();
}

hipError_t frame_mpjpe(const float* all_seqs, const float* outputs, int B, int T, int D, int t_out0,
                       const int* used_pos, int n_used, const int* joint_src, const int* frames, int n_frames,
                       float* sums, hipStream_t s) {
  k_frame_mpjpe<<<n_frames, kRedThreads, 0, s>>>(all_seqs, outputs, B, T, D, t_out0, used_pos, n_used, joint_src,
                                                 frames, sums);
  return hipGetLastError();
}

}  // namespace train
}  // namespace dstd
