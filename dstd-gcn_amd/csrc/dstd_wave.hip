// Wave-independent DSTDGC kernels: every GC launch of the forward (spatial
// 64->64 of the encoders, 6->64 of conv_st_in and 64->3 of conv_st_out, both
// with their residual conv; temporal 64->64 and the 3->3 output tail).
//
// Why a second design (profiles/r01_*, scripts/ab_kernels.py): the persistent
// 8-wave kernels of round 1 (dstd_fast.hip, retired in round 3) spent ~60% of
// their time outside the MFMA pipe -- four barriers per tile, index arithmetic for the LDS staging, the
// conv output round trip through LDS.  Here every wave owns a whole unit of
// work and never meets a barrier after the prologue:
//
//  * the 1x1 conv is computed TRANSPOSED, D[p][c] = sum_k x[p][k] W[c][k] + b[c]
//    (positions p as MFMA rows, A operand = x rows loaded straight from HBM
//    into registers, B operand = W from LDS);
//  * its accumulator registers ARE the A operand of the aggregation: with the
//    16x16x4 f32 MFMA the accumulator register r of lane (kl, cl) holds
//    D[row 4kl + r][col cl], which is exactly A[i = cl][k = kl] of a k-step
//    that contracts over the rows {4kl + r}.  Rows are therefore ordered so
//    that each "r-slice" of a row tile holds four positions of ONE frame
//    (spatial) / four consecutive frames (temporal); the aggregation's
//    k-steps walk the r-slices and its B operand is the adjacency row block
//    of those four positions;
//  * the adjacency rows of the unit land in a wave-private LDS image by
//    LDS-DMA (global_load_lds_dwordx4), issued one unit ahead;
//  * epilogue (BatchNorm affine, residual, PReLU, 16-byte NTVC stores) and
//    the next DSTDGC's P/Q (an MFMA whose B operand is again the output
//    accumulator) run straight out of registers;
//  * units are strided over the waves statically.  (A global atomic work
//    ticket measured 1.1-1.7x SLOWER here: device-scope atomics on one
//    address from all eight XCDs serialise.)
//
// Spatial unit = (sample, 2 frames): 44 positions in 3 row tiles (48 rows,
// 12 k-slices of 4 joints: 6 per frame).  Temporal unit = (sample, joint):
// 35 frames in 3 row tiles (9 k-slices of 4 frames).
#include "dstd_common.h"
#include "dstd_kernels.h"

// Phase timers (debug builds only, -DDSTD_STAMPS): per wave, the s_memtime
// cycles spent in each phase summed over its units; read with
// dstd_debug_stamps().
#ifdef DSTD_STAMPS
__device__ unsigned long long g_stamps[2][4096 * 8];
#define STAMP_DECL                  \
  unsigned long long st_acc[8] = {}; \
  unsigned long long st_t = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                                \
  {                                                             \
    __builtin_amdgcn_sched_barrier(0);                          \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += t_ - st_t;                                     \
    st_t = t_;                                                  \
    __builtin_amdgcn_sched_barrier(0);                          \
  }
#define STAMP_FLUSH(k)                                                         \
  if ((threadIdx.x & 63) == 0 && gw < 4096)                                    \
    for (int i_ = 0; i_ < 8; ++i_) g_stamps[k][gw * 8 + i_] += st_acc[i_];
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_FLUSH(k)
#endif

namespace dstd {

namespace {

constexpr int WW = 4;        // waves per workgroup
constexpr int WT = WW * 64;  // threads per workgroup

// Channel blocking of a C-channel row.  MFMA k-step (j, s) of a conv with C
// input channels contracts channel 16j + 4kl + s (kl = lane >> 4): lane kl of
// a row holds the float4 chunks at 16j + 4kl, j < NJ -- for C = 64 each
// load instruction then reads 64 contiguous bytes per row.  Output channels
// come in NT tiles of 16.
template <int C>
struct Chan {
  static constexpr int NJ = cdiv(C, 16);
  static constexpr int NT = cdiv(C, 16);
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float comp(const float4& v, int s) { return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w; }
__device__ __forceinline__ float4 zf4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// channels c0 .. c0+3 of a row of C floats, zero past C (C % 4 != 0: scalar loads)
template <int C>
__device__ __forceinline__ float4 ld_chunk(const float* row, int c0) {
  if constexpr (C % 4 == 0) {
    return c0 < C ? ld4(row + c0) : zf4();
  } else {
    float e[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) e[i] = c0 + i < C ? row[c0 + i] : 0.f;
    return make_float4(e[0], e[1], e[2], e[3]);
  }
}
// store the channels c0 .. c0+3 that exist
template <int C>
__device__ __forceinline__ void st_chunk(float* row, int c0, const f32x4& v) {
  if constexpr (C % 4 == 0) {
    if (c0 < C) st4(row + c0, make_float4(v[0], v[1], v[2], v[3]));
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (c0 + i < C) row[c0 + i] = v[i];
  }
}

// 16-byte LDS-DMA (global_load_lds_dwordx4): lane l writes LDS byte address
// dst + 16*l (dst wave-uniform).  Issued from inline asm on purpose: with a
// compiler-visible LDS-DMA in flight hipcc turns every later wait for an
// ordinary load into vmcnt(0), which would serialise the epilogue's stores.
// hipcc does not count it, so its readers wait with adj_landed().
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)p);
}
__device__ __forceinline__ void glds16(const float* src, uint32_t dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(dst)
      : "memory");
}
// All of this wave's LDS-DMA has landed (vmcnt(0): covers every older VMEM
// operation; the image is staged one unit ahead, so by now it has landed and
// only the previous unit's stores can still be in flight).
__device__ __forceinline__ void adj_landed() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// LDS reads of the current wave may still be in flight when the next
// LDS-DMA into the same image is issued; retire them first (WAR).
__device__ __forceinline__ void lds_reads_done() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }


// Each wave takes a contiguous range of units: neighbouring units write
// neighbouring bytes, and a range keeps those writes in one wave -- one
// XCD's L2 -- instead of interleaving them across the eight XCDs.
__device__ __forceinline__ int unit_range(int nunits, int& uend, int& gw) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  gw = blockIdx.x * WW + wave;
  const long nw = (long)gridDim.x * WW;
  uend = (int)(((long)(gw + 1) * nunits) / nw);
  return (int)(((long)gw * nunits) / nw);
}

// Weight fragments in LDS, wl[(ct*NJ + j)*64 + lane] = W[16ct + cl][16j + 4kl .. +3]
// (zero outside [COUT][CIN]).  The same image serves as MFMA B operand of the
// transposed conv (lane (kl, cl)) and as A operand of a conv in output layout
// (lane (cl, kl)): both hold W[16ct + (lane & 15)][16j + 4(lane >> 4) + s].
template <int CIN, int COUT>
__device__ __forceinline__ void stage_frags(float4* wl, const float* w, int tid) {
  constexpr int NJ = Chan<CIN>::NJ, NT = Chan<COUT>::NT;
  for (int i = tid; i < NT * NJ * 64; i += WT) {
    const int l = i & 63, j = (i >> 6) % NJ, ct = (i >> 6) / NJ;
    const int c = 16 * ct + (l & 15), k0 = 16 * j + 4 * (l >> 4);
    float e[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) e[q] = (c < COUT && k0 + q < CIN) ? w[c * CIN + k0 + q] : 0.f;
    wl[i] = make_float4(e[0], e[1], e[2], e[3]);
  }
}

// P/Q weights of the next DSTDGC as MFMA A fragments: wq[ct*64 + lane], lane
// (cl = channel, kl) of k-step (ct, r) holds w[ch][16ct + 4kl + r]; channel
// ch = 2j + rr is row rr of conv_m* block j (C inputs).  bq[ch] = its bias.
template <int C>
__device__ __forceinline__ void stage_pq(float4* wq, float* bq, const float* const* pqw, const float* const* pqb,
                                         int nch, int tid) {
  constexpr int NT = Chan<C>::NT;
  for (int i = tid; i < NT * 64; i += WT) {
    const int l = i & 63, ct = i >> 6, ch = l & 15, c0 = 16 * ct + 4 * (l >> 4);
    float e[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) e[q] = (ch < nch && c0 + q < C) ? pqw[ch >> 1][(ch & 1) * C + c0 + q] : 0.f;
    wq[i] = make_float4(e[0], e[1], e[2], e[3]);
  }
  if (tid < 16) bq[tid] = tid < nch ? pqb[tid >> 1][tid & 1] : 0.f;
}

// folded BN vectors [V][C] -> LDS [c/4][v]: lanes (v) read consecutive float4
template <int C>
__device__ __forceinline__ void stage_bn(float4* dst, const float* src, int V, int tid) {
  constexpr int C4 = 4 * Chan<C>::NT;
  for (int i = tid; i < V * C4; i += WT) {
    const int v = i / C4, c4 = i % C4;
    dst[c4 * V + v] = ld_chunk<C>(src + v * C, 4 * c4);
  }
}

}  // namespace

// ===========================================================================
// Spatial GC (DSTDGCB.forward, model/dstdgcn.py:141-152, with DSTDGC.forward
// spatial :80-87), two graphs:
//   y[c][w] = sum_g sum_v (W_g x + b_g)[v][c] Adj_g[t][v][w]
//   EPI:  h = prelu(bn(y) + r),  r = x (CIN == COUT) or bn_r(W_r x + b_r) (RES)
//   + P_t/Q_t of h for the block's temporal DSTDGC ([B][T][V][4])
// ===========================================================================
template <int V>
struct SWGeom {
  static constexpr int KQ = cdiv(V, 4);          // k-slices per frame
  static constexpr int NQ = 2 * KQ;              // per unit
  static constexpr int MT = cdiv(NQ, 4);         // conv row tiles
  static constexpr int NWT = cdiv(V, 16);        // output column tiles
  static constexpr int NV4 = cdiv(V * V, 4);     // float4 per adjacency row
  static constexpr int IMG = rup(V * V + 48, 4);  // image floats (+ slack for the padded column reads)
};

// 64 -> 64: one wave per SIMD, 300+ registers hold the unit (conv tile, output,
// residual, prefetch).  The thinner 6 -> 64 / 64 -> 3 blocks have too little
// MFMA work per unit to hide a unit's load latency on their own: two waves.
// (A software-pipelined variant -- the epilogue of unit k interleaved with
// the first conv of unit k+1 through buffer stores and sched_group_barrier --
// measured 5-8% SLOWER at 430 registers.)
template <int CIN, int COUT>
constexpr int spatial_wpe() {
  return CIN == 64 && COUT == 64 ? 1 : 2;
}
template <int V, int CIN, int COUT, bool RES, bool EPI>
__global__ __launch_bounds__(WT) __attribute__((amdgpu_waves_per_eu(spatial_wpe<CIN, COUT>(),
                                                                    spatial_wpe<CIN, COUT>()))) void k_spatial_wave(
    SpatialArgs a) {
  using Gm = SWGeom<V>;
  constexpr int KQ = Gm::KQ, NQ = Gm::NQ, MT = Gm::MT, NWT = Gm::NWT, NV4 = Gm::NV4;
  constexpr int NJ = Chan<CIN>::NJ, NCO = Chan<COUT>::NT;
  static_assert(RES || CIN == COUT, "identity residual needs CIN == COUT");
  __shared__ float4 wl[2][NCO * NJ * 64];          // conv B fragments per graph
  __shared__ float4 wrl[RES ? NCO * NJ * 64 : 1];  // residual conv A fragments
  __shared__ float4 bnl[RES ? 4 : 2][4 * NCO * V]; // BN scale / shift (+ residual BN), [c/4][w]
  __shared__ float adjl[WW][2][2][Gm::IMG];        // per-wave adjacency images [g][frame]
  __shared__ float4 wql[NCO * 64];                 // P/Q A fragments
  __shared__ float bql[16];
  __shared__ float bfl[3][16 * NCO];               // conv biases (graphs, residual conv)

  const int tid = threadIdx.x, lane = tid & 63;
  const int kl = lane >> 4, cl = lane & 15;
  const int T = a.T;
  const int NP = cdiv(T, 2);
  const int nunits = a.B * NP;

  stage_frags<CIN, COUT>(wl[0], a.wf[0], tid);
  stage_frags<CIN, COUT>(wl[1], a.wf[1], tid);
  if constexpr (RES) stage_frags<CIN, COUT>(wrl, a.wf[2], tid);
  const int nch = a.pq ? 2 * a.npqw : 0;
  stage_pq<COUT>(wql, bql, a.pqw, a.pqb, nch, tid);
  for (int i = tid; i < (RES ? 3 : 2) * 16 * NCO; i += WT) {
    const int g = i / (16 * NCO), c = i % (16 * NCO);
    bfl[g][c] = c < COUT ? a.bf[g][c] : 0.f;
  }
  if constexpr (EPI) {
    stage_bn<COUT>(bnl[0], a.bn_s, V, tid);
    stage_bn<COUT>(bnl[1], a.bn_h, V, tid);
    if constexpr (RES) {
      stage_bn<COUT>(bnl[2], a.rbn_s, V, tid);
      stage_bn<COUT>(bnl[3], a.rbn_h, V, tid);
    }
  }
  __syncthreads();

  int gw, uend;
  int u = unit_range(nunits, uend, gw);
  const int wave = gw - blockIdx.x * WW;
  const float pw = EPI ? *a.prelu : 0.f;

  // row (m, i = cl) of the conv tiles -> (frame, joint): k-slice Q = 4m + (i & 3)
  // holds joints 4q .. 4q+3 (q = Q % KQ) of frame Q / KQ; row i is joint 4q + (i >> 2)
  int rowf[MT], rowv[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int Q = 4 * m + (cl & 3);
    const int f = Q < NQ ? Q / KQ : 0;
    const int v = 4 * (Q < NQ ? Q % KQ : 0) + (cl >> 2);
    rowf[m] = f;
    rowv[m] = v < V ? v : V - 1;  // padding rows read a real row; their adjacency rows are zero
  }

  float4 xa[MT][NJ];
  auto load_x = [&](int uu) {
    const int n = uu / NP, t0 = (uu - n * NP) * 2, nf = min(2, T - t0);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int f = min(rowf[m], nf - 1);
      const float* px = a.x + ((size_t)(n * T + t0 + f) * V + rowv[m]) * CIN;
#pragma unroll
      for (int j = 0; j < NJ; ++j) xa[m][j] = ld_chunk<CIN>(px, 16 * j + 4 * kl);
    }
  };
  auto stage_adj = [&](int uu) {
    const int n = uu / NP, t0 = (uu - n * NP) * 2, nf = min(2, T - t0);
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        if (f >= nf) continue;
        const float* src = a.adj + ((size_t)(n * 2 + g) * T + t0 + f) * a.adj_ld + 4 * lane;
        const uint32_t dst = lds_addr(adjl[wave][g][f]);
#pragma unroll
        for (int i = 0; i < NV4; i += 64)
          if (i + lane < NV4) glds16(src + 4 * i, dst + 16 * i);
      }
  };

  f32x4 D[MT][NCO];
  f32x4 O[2][NCO][NWT];
  auto conv = [&](int g) {
#pragma unroll
    for (int ct = 0; ct < NCO; ++ct) {
      const float b = bfl[g][16 * ct + cl];
#pragma unroll
      for (int m = 0; m < MT; ++m) D[m][ct] = f32x4{b, b, b, b};
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float4 wb[NCO];
#pragma unroll
      for (int ct = 0; ct < NCO; ++ct) wb[ct] = wl[g][(ct * NJ + j) * 64 + lane];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int ct = 0; ct < NCO; ++ct) D[m][ct] = mfma16x16x4(comp(xa[m][j], s), comp(wb[ct], s), D[m][ct]);
    }
  };
  auto agg = [&](int g, int nf) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      if (f >= nf) continue;
      const float* img = adjl[wave][g][f] + kl * V + cl;
      float b[KQ][NWT];  // B fragments: Adj[4q + kl][16wt + cl], rows >= V zero
#pragma unroll
      for (int q = 0; q < KQ; ++q)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) {
          b[q][wt] = img[4 * q * V + 16 * wt];
          if (4 * q + 3 >= V) b[q][wt] = 4 * q + kl < V ? b[q][wt] : 0.f;
        }
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        const int Q = f * KQ + q, m = Q >> 2, r = Q & 3;
#pragma unroll
        for (int ct = 0; ct < NCO; ++ct)
#pragma unroll
          for (int wt = 0; wt < NWT; ++wt) O[f][ct][wt] = mfma16x16x4(D[m][ct][r], b[q][wt], O[f][ct][wt]);
      }
    }
  };

  if (u < uend) {
    load_x(u);
    stage_adj(u);
  }
  STAMP_DECL
  while (u < uend) {
    const int n = u / NP, t0 = (u - n * NP) * 2, nf = min(2, T - t0);
    const int un = u + 1;
    // x at the output positions, issued first (it has the whole unit to land):
    // the identity residual, or the B operand of the residual conv
    float4 R[2][NWT][NJ];
    if constexpr (EPI) {
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        if (f >= nf) continue;
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) {
          const int w = min(16 * wt + cl, V - 1);
          const float* px = a.x + ((size_t)(n * T + t0 + f) * V + w) * CIN;
#pragma unroll
          for (int j = 0; j < NJ; ++j) R[f][wt][j] = ld_chunk<CIN>(px, 16 * j + 4 * kl);
        }
      }
    }
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int ct = 0; ct < NCO; ++ct)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) O[f][ct][wt] = zero4();
    conv(0);
    STAMP(0)
    adj_landed();
    STAMP(1)
    agg(0, nf);
    STAMP(2)
    conv(1);
    STAMP(3)
    __builtin_amdgcn_sched_barrier(0);
    if (un < uend) load_x(un);  // xa is dead after conv(1)
    STAMP(4)
    agg(1, nf);
    STAMP(5)
    lds_reads_done();
    if (un < uend) stage_adj(un);

    // ---- epilogue: h = prelu(bn(y) + r) -> NTVC, then P_t/Q_t of h ----
    if constexpr (EPI) {
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        if (f >= nf) continue;
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) {
          const int wc = min(16 * wt + cl, V - 1);
          f32x4 rc[NCO];  // residual conv, output layout: A = W_r fragments, B = x rows
          if constexpr (RES) {
#pragma unroll
            for (int ct = 0; ct < NCO; ++ct) {
              const float b = bfl[2][16 * ct + 4 * kl], b1 = bfl[2][16 * ct + 4 * kl + 1];
              const float b2 = bfl[2][16 * ct + 4 * kl + 2], b3 = bfl[2][16 * ct + 4 * kl + 3];
              rc[ct] = f32x4{b, b1, b2, b3};
#pragma unroll
              for (int j = 0; j < NJ; ++j) {
                const float4 wr = wrl[(ct * NJ + j) * 64 + lane];
#pragma unroll
                for (int s = 0; s < 4; ++s) rc[ct] = mfma16x16x4(comp(wr, s), comp(R[f][wt][j], s), rc[ct]);
              }
            }
          }
#pragma unroll
          for (int ct = 0; ct < NCO; ++ct) {
            f32x4& o = O[f][ct][wt];
            const int c4 = (4 * ct + kl) * V + wc;
            const float4 sc = bnl[0][c4], sh = bnl[1][c4];
            float r[4];
            if constexpr (RES) {
              const float4 rs = bnl[2][c4], rh = bnl[3][c4];
              r[0] = rc[ct][0] * rs.x + rh.x;
              r[1] = rc[ct][1] * rs.y + rh.y;
              r[2] = rc[ct][2] * rs.z + rh.z;
              r[3] = rc[ct][3] * rs.w + rh.w;
            } else {
              const float4 x4 = R[f][wt][ct];
              r[0] = x4.x;
              r[1] = x4.y;
              r[2] = x4.z;
              r[3] = x4.w;
            }
            o[0] = prelu_f(o[0] * sc.x + sh.x + r[0], pw);
            o[1] = prelu_f(o[1] * sc.y + sh.y + r[1], pw);
            o[2] = prelu_f(o[2] * sc.z + sh.z + r[2], pw);
            o[3] = prelu_f(o[3] * sc.w + sh.w + r[3], pw);
          }
        }
      }
    }
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      if (f >= nf) continue;
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) {
        const int w = 16 * wt + cl;
        if (w >= V) continue;
        float* py = a.y + ((size_t)(n * T + t0 + f) * V + w) * COUT;
#pragma unroll
        for (int ct = 0; ct < NCO; ++ct) st_chunk<COUT>(py, 16 * ct + 4 * kl, O[f][ct][wt]);
      }
    }
    // P_t/Q_t of h: out[ch][w] = sum_c wq[ch][c] h[c][w] + b, with h (the output
    // accumulators) as the B operand; the 2 x NWT chains interleave
    if (nch) {
      f32x4 acc[2][NWT];
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) acc[f][wt] = zero4();
#pragma unroll
      for (int ct = 0; ct < NCO; ++ct) {
        const float4 wq = wql[ct * 64 + lane];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int f = 0; f < 2; ++f)
#pragma unroll
            for (int wt = 0; wt < NWT; ++wt) acc[f][wt] = mfma16x16x4(comp(wq, r), O[f][ct][wt][r], acc[f][wt]);
      }
      // [B][T][V][4]: lane (0, cl) holds the 4 channels of joint w -> one 16-byte store
      if (kl == 0) {
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          if (f >= nf) continue;
#pragma unroll
          for (int wt = 0; wt < NWT; ++wt) {
            const int w = 16 * wt + cl;
            if (w >= V) continue;
            const f32x4 pv = acc[f][wt];
            st4(a.pq + ((size_t)(n * T + t0 + f) * V + w) * 4,
                make_float4(pv[0] + bql[0], pv[1] + bql[1], pv[2] + bql[2], pv[3] + bql[3]));
          }
        }
      }
    }
    STAMP(6)
    u = un;
  }
  STAMP_FLUSH(0)
}

// ===========================================================================
// Temporal GC, C -> C (DSTDGC.forward temporal, model/dstdgcn.py:88-93) with
// the DSTDGCB tail epilogues (:161-163 and DSTDGCN.forward :306-315):
//   y[c][u] = sum_t (W x + b)[t][c] Adj[v][t][u]
//   ENC: prelu(bn(y + xres));  IN: prelu(bn(y));  RAW: y
//   OUT: y + x_model[n][T-1][v][c]  (the model output, C = 3)
//   + P_s/Q_s (8 channels, [B][V][T][8]) of the output for the next block
// ===========================================================================
template <int T>
struct TWGeom {
  static constexpr int KT = cdiv(T, 4);       // k-slices (4 frames each)
  static constexpr int MT = cdiv(KT, 4);      // conv row tiles
  static constexpr int NUT = cdiv(T, 16);     // output column tiles
  static constexpr int NV4 = cdiv(T * T, 4);  // float4 per adjacency row
  static constexpr int IMG = rup(T * T + 48, 4);
};

template <int T, int WPE, int EPI, int C>
__global__ __launch_bounds__(WT) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_temporal_wave(
    TemporalArgs a) {
  using Gm = TWGeom<T>;
  constexpr int KT = Gm::KT, MT = Gm::MT, NUT = Gm::NUT, NV4 = Gm::NV4;
  constexpr int NJ = Chan<C>::NJ, NCO = Chan<C>::NT;
  constexpr int VMAX = 32;
  __shared__ float4 wl[NCO * NJ * 64];       // conv B fragments
  __shared__ float4 bnl[2][4 * NCO * VMAX];  // folded BN scale / shift, [c/4][v]
  __shared__ float adjl[WW][Gm::IMG];        // per-wave adjacency image
  __shared__ float4 wql[NCO * 64];           // P/Q A fragments
  __shared__ float bql[16];
  __shared__ float bfl[16 * NCO];            // conv bias

  const int tid = threadIdx.x, lane = tid & 63;
  const int kl = lane >> 4, cl = lane & 15;
  const int V = a.V;
  const int nunits = a.B * V;
  constexpr bool use_bn = EPI == TEPI_ENC || EPI == TEPI_IN;
  constexpr bool use_res = EPI == TEPI_ENC || EPI == TEPI_OUT;

  stage_frags<C, C>(wl, a.wf, tid);
  const int nch = a.pq ? 2 * a.npqw : 0;
  stage_pq<C>(wql, bql, a.pqw, a.pqb, nch, tid);
  if (tid < 16 * NCO) bfl[tid] = tid < C ? a.bf[tid] : 0.f;
  if constexpr (use_bn) {
    stage_bn<C>(bnl[0], a.bn_s, V, tid);
    stage_bn<C>(bnl[1], a.bn_h, V, tid);
  }
  __syncthreads();

  int gw, uend;
  int u = unit_range(nunits, uend, gw);
  const int wave = gw - blockIdx.x * WW;
  const float pw = use_bn ? *a.prelu : 0.f;

  // row (m, i = cl): k-slice Q = 4m + (i & 3) holds frames 4Q .. 4Q+3; row i is frame 4Q + (i >> 2)
  int rowt[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int t = 4 * (4 * m + (cl & 3)) + (cl >> 2);
    rowt[m] = t < T ? t : T - 1;
  }

  float4 xa[MT][NJ];
  auto load_x = [&](int uu) {
    const int n = uu / V, v = uu - n * V;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float* px = a.h + ((size_t)(n * T + rowt[m]) * V + v) * C;
#pragma unroll
      for (int j = 0; j < NJ; ++j) xa[m][j] = ld_chunk<C>(px, 16 * j + 4 * kl);
    }
  };
  auto stage_adj = [&](int uu) {
    const float* src = a.adj + (size_t)uu * a.adj_ld + 4 * lane;  // [B][V] rows: unit index == n*V + v
    const uint32_t dst = lds_addr(adjl[wave]);
#pragma unroll
    for (int i = 0; i < NV4; i += 64)
      if (i + lane < NV4) glds16(src + 4 * i, dst + 16 * i);
  };

  f32x4 D[MT][NCO];
  f32x4 O[NCO][NUT];
  if (u < uend) {
    load_x(u);
    stage_adj(u);
  }
  STAMP_DECL
  while (u < uend) {
    const int n = u / V, v = u - n * V;
    const int un = u + 1;
    // epilogue residual, issued first: it has the whole unit to land
    float4 R[NUT][NCO];
    if constexpr (use_res) {
#pragma unroll
      for (int ut = 0; ut < NUT; ++ut) {
        const int tr = EPI == TEPI_OUT ? T - 1 : min(16 * ut + cl, T - 1);
        const float* px = a.xres + ((size_t)(n * T + tr) * V + v) * C;
#pragma unroll
        for (int ct = 0; ct < NCO; ++ct) R[ut][ct] = ld_chunk<C>(px, 16 * ct + 4 * kl);
      }
    }
    // ---- conv: D[t][c] = sum_k x[t][k] W[c][k] + b[c] ----
#pragma unroll
    for (int ct = 0; ct < NCO; ++ct) {
      const float b = bfl[16 * ct + cl];
#pragma unroll
      for (int m = 0; m < MT; ++m) D[m][ct] = f32x4{b, b, b, b};
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float4 wb[NCO];
#pragma unroll
      for (int ct = 0; ct < NCO; ++ct) wb[ct] = wl[(ct * NJ + j) * 64 + lane];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int ct = 0; ct < NCO; ++ct) D[m][ct] = mfma16x16x4(comp(xa[m][j], s), comp(wb[ct], s), D[m][ct]);
    }
    STAMP(0)
    adj_landed();  // before the prefetch: the wait retires every older VMEM operation
    STAMP(1)
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch below the conv: xa is reloaded in place
    if (un < uend) load_x(un);
    // ---- aggregation: y[c][u] = sum_t D[t][c] Adj[t][u] ----
#pragma unroll
    for (int ct = 0; ct < NCO; ++ct)
#pragma unroll
      for (int ut = 0; ut < NUT; ++ut) O[ct][ut] = zero4();
    {
      const float* img = adjl[wave] + kl * T + cl;
#pragma unroll
      for (int Q0 = 0; Q0 < KT; Q0 += 4) {
        float b[4][NUT];  // B fragments of 4 k-slices: Adj[4Q + kl][16ut + cl], rows >= T zero
#pragma unroll
        for (int dq = 0; dq < 4; ++dq)
#pragma unroll
          for (int ut = 0; ut < NUT; ++ut) {
            const int Q = Q0 + dq;
            if (Q >= KT) continue;
            b[dq][ut] = img[4 * Q * T + 16 * ut];
            if (4 * Q + 3 >= T) b[dq][ut] = 4 * Q + kl < T ? b[dq][ut] : 0.f;
          }
#pragma unroll
        for (int dq = 0; dq < 4; ++dq) {
          const int Q = Q0 + dq;
          if (Q >= KT) continue;
          const int m = Q >> 2, r = Q & 3;
#pragma unroll
          for (int ct = 0; ct < NCO; ++ct)
#pragma unroll
            for (int ut = 0; ut < NUT; ++ut) O[ct][ut] = mfma16x16x4(D[m][ct][r], b[dq][ut], O[ct][ut]);
        }
      }
    }
    STAMP(2)
    lds_reads_done();
    if (un < uend) stage_adj(un);
    STAMP(3)

    // ---- epilogue ----
#pragma unroll
    for (int ut = 0; ut < NUT; ++ut) {
      const int uo = 16 * ut + cl;
      const int uc = uo < T ? uo : T - 1;
      float* py = a.y + ((size_t)(n * T + uc) * V + v) * C;
#pragma unroll
      for (int ct = 0; ct < NCO; ++ct) {
        f32x4& o = O[ct][ut];
        if constexpr (use_res) {
          o[0] += R[ut][ct].x;
          o[1] += R[ut][ct].y;
          o[2] += R[ut][ct].z;
          o[3] += R[ut][ct].w;
        }
        if constexpr (use_bn) {
          const float4 sc = bnl[0][(4 * ct + kl) * V + v], sh = bnl[1][(4 * ct + kl) * V + v];
          o[0] = prelu_f(o[0] * sc.x + sh.x, pw);
          o[1] = prelu_f(o[1] * sc.y + sh.y, pw);
          o[2] = prelu_f(o[2] * sc.z + sh.z, pw);
          o[3] = prelu_f(o[3] * sc.w + sh.w, pw);
        }
        if (uo < T) st_chunk<C>(py, 16 * ct + 4 * kl, o);
      }
    }
    STAMP(4)
    // next block's P_s/Q_s (8 channels) of the output, NUT interleaved chains
    if (nch) {
      f32x4 acc[NUT];
#pragma unroll
      for (int ut = 0; ut < NUT; ++ut) acc[ut] = zero4();
#pragma unroll
      for (int ct = 0; ct < NCO; ++ct) {
        const float4 wq = wql[ct * 64 + lane];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int ut = 0; ut < NUT; ++ut) acc[ut] = mfma16x16x4(comp(wq, r), O[ct][ut][r], acc[ut]);
      }
      STAMP(5)
      // [B][V][T][8]: lane (kl, cl), kl < 2, holds channels 4kl..4kl+3 of frame u
      if (kl < 2) {
#pragma unroll
        for (int ut = 0; ut < NUT; ++ut) {
          const int uo = 16 * ut + cl;
          if (uo >= T) continue;
          const f32x4 pv = acc[ut];
          st4(a.pq + ((size_t)u * T + uo) * 8 + 4 * kl,
              make_float4(pv[0] + bql[4 * kl], pv[1] + bql[4 * kl + 1], pv[2] + bql[4 * kl + 2], pv[3] + bql[4 * kl + 3]));
        }
      }
    }
    STAMP(6)
    u = un;
  }
  STAMP_FLUSH(1)
}

// ===========================================================================
// dispatch
// ===========================================================================
namespace {

int wave_num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

template <typename K>
int wave_occupancy(K k) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k, WT, 0) != hipSuccess || nb < 1) nb = 1;
  (void)hipGetLastError();
  return nb;
}

// (compile-time only: a -DDSTD_NO_WAVE build routes the exact-fp32 block
// launches to the generic kernels; no process-wide switch)
bool wave_disabled() {
#ifdef DSTD_NO_WAVE
  return true;
#else
  return false;
#endif
}

template <int V, int CIN, int COUT, bool RES>
hipError_t spatial_wave_launch(const SpatialArgs& a, hipStream_t s) {
  static const int occ = wave_occupancy(k_spatial_wave<V, CIN, COUT, RES, true>);
  const int units = a.B * cdiv(a.T, 2);
  int grid = wave_num_cus() * occ;
  grid = min(grid, cdiv(units, WW));
  hipLaunchKernelGGL((k_spatial_wave<V, CIN, COUT, RES, true>), dim3(grid), dim3(WT), 0, s, a);
  return hipGetLastError();
}
template <int V>
hipError_t spatial_wave_run(const SpatialArgs& a, hipStream_t s) {
  if (a.Cin == 64 && a.Cout == 64 && a.G == 2) return spatial_wave_launch<V, 64, 64, false>(a, s);
  if (a.Cin == 6 && a.Cout == 64 && a.G == 3) return spatial_wave_launch<V, 6, 64, true>(a, s);
  if (a.Cin == 64 && a.Cout == 3 && a.G == 3) return spatial_wave_launch<V, 64, 3, true>(a, s);
  return hipErrorNotSupported;
}

template <int T, int WPE, int EPI, int C>
hipError_t temporal_wave_launch(const TemporalArgs& a, hipStream_t s) {
  static const int occ = wave_occupancy(k_temporal_wave<T, WPE, EPI, C>);
  const int units = a.B * a.V;
  int grid = wave_num_cus() * occ;
  grid = min(grid, cdiv(units, WW));
  hipLaunchKernelGGL((k_temporal_wave<T, WPE, EPI, C>), dim3(grid), dim3(WT), 0, s, a);
  return hipGetLastError();
}
template <int T, int WPE>
hipError_t temporal_wave_run(const TemporalArgs& a, hipStream_t s) {
  if (a.Cin == 64 && a.Cout == 64) {
    switch (a.epi) {
      case TEPI_ENC: return temporal_wave_launch<T, WPE, TEPI_ENC, 64>(a, s);
      case TEPI_IN: return temporal_wave_launch<T, WPE, TEPI_IN, 64>(a, s);
      case TEPI_RAW: return temporal_wave_launch<T, WPE, TEPI_RAW, 64>(a, s);
      default: return hipErrorNotSupported;
    }
  }
  if (a.Cin == 3 && a.Cout == 3 && a.epi == TEPI_OUT && !a.pq) return temporal_wave_launch<T, WPE, TEPI_OUT, 3>(a, s);
  return hipErrorNotSupported;
}

}  // namespace

hipError_t launch_spatial_wave(const SpatialArgs& a, hipStream_t s) {
  if (wave_disabled()) return hipErrorNotSupported;
  if (a.NI != 2 || a.epi != 1) return hipErrorNotSupported;
  if (a.pq && (a.npqw != 2 || !pq_layout_eq(a.pql, pq_layout_tv(4, a.T, a.V)))) return hipErrorNotSupported;
  if (a.adj_ld % 4 != 0) return hipErrorNotSupported;
  switch (a.V) {
    case 22: return spatial_wave_run<22>(a, s);
    case 23: return spatial_wave_run<23>(a, s);
    case 25: return spatial_wave_run<25>(a, s);
    default: return hipErrorNotSupported;
  }
}

hipError_t launch_temporal_wave(const TemporalArgs& a, hipStream_t s) {
  if (wave_disabled()) return hipErrorNotSupported;
  if (a.V > 32) return hipErrorNotSupported;
  if (a.pq && (a.npqw != 4 || !pq_layout_eq(a.pql, pq_layout_vt(8, a.T, a.V)))) return hipErrorNotSupported;
  if (a.adj_ld % 4 != 0) return hipErrorNotSupported;
  switch (a.T) {
    case 35: return temporal_wave_run<35, 2>(a, s);
    case 40: return temporal_wave_run<40, 2>(a, s);
    case 75: return temporal_wave_run<75, 1>(a, s);
    default: return hipErrorNotSupported;
  }
}

}  // namespace dstd

#ifdef DSTD_STAMPS
extern "C" int dstd_debug_stamps(int which, unsigned long long* host, int n, int reset) {
  if (which < 0 || which > 1 || n > 4096 * 8) return 1;
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), n * sizeof(unsigned long long),
                                     which * 4096 * 8 * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    static unsigned long long zeros[4096 * 8];
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zeros, sizeof(zeros), which * 4096 * 8 * sizeof(unsigned long long));
  }
  return (int)e;
}
#endif
