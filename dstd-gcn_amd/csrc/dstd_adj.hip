// Dynamic-adjacency kernels (k_adj_fast): the J x J / T x T matrices of the
// DSTDGC, alpha * conv_rm(tanh(P_i - Q_j)) + A_stat, written to HBM in the
// fp32 layout of the generic GC kernels or the split-f16 (hi/lo) planes of
// the dstd_hilo.hip kernels.  Shape-specialised for (T, V) in {(35,22),
// (35,25), (40,23), (75,22)}; other shapes use the generic k_adj
// (dstd_kernels.hip).  The model forward builds the temporal planes inside
// k_temporal_fused and the spatial planes in its phase 3 (dstd_hilo.hip);
// these kernels serve the op and block entry points, T = 75 and the
// exact-fp32 arithmetic.
//
// (The exact-fp32 GC kernels k_spatial_fast / k_temporal_fast that once
// shared this file were retired in round 3: the block path runs on
// dstd_wave.hip, the op path on the generic kernels.)
#include "dstd_common.h"
#include "dstd_kernels.h"
#include "dstd_hilo.h"


// Workgroup timeline of the adjacency kernel (debug builds, -DDSTD_STAMPS):
// s_memrealtime (100 MHz, chip-wide) at entry, staging done, compute done, exit.
#ifdef DSTD_STAMPS
__device__ unsigned long long g_tl[2][2048][4];
#define TL(m, i) \
  if (threadIdx.x == 0 && blockIdx.x < 2048) g_tl[m][blockIdx.x][i] = __builtin_amdgcn_s_memrealtime();
#else
#define TL(m, i)
#endif

namespace dstd {

namespace {

constexpr int NWV = 8;                 // waves per workgroup
constexpr int NTHR = NWV * DSTD_WAVE;  // 512 threads

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// Register-staged cooperative copy: load() issues every global load of the
// thread (for the next tile), store() later writes them to LDS.
template <typename Val, int N>
struct Stager {
  static constexpr int IT = cdiv(N, NTHR);
  Val v[IT];
  template <typename Src>
  __device__ __forceinline__ void load(int tid, Src src) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = tid + it * NTHR;
      if (i < N) v[it] = src(i);
    }
  }
  template <typename Dst>
  __device__ __forceinline__ void store(int tid, Dst dst) const {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = tid + it * NTHR;
      if (i < N) dst(i, v[it]);
    }
  }
};

}  // namespace

// ===========================================================================
// Dynamic adjacency.  MODE 0: rows t (NROW = T), cols (v,w) (NA = V), K = 2T.
// MODE 1: rows v (NROW = V), cols (t,u) (NA = T), K = 2V.
//
// tanh of a difference, separably: with EP = 2^(c*P), EQ = 2^(-c*Q),
// c = 2*log2(e),   tanh(P - Q) = 1 - 2 / (EP*EQ + 1)
// -- per MFMA operand one LDS pair, one FMA, one v_rcp_f32 and one FMA.  The
// factors are formed once per workgroup.  While |c*P|, |c*Q| <= 120 they are
// normal floats (no 0*inf) and the product under/overflows only where tanh
// is -1/+1 to fp32 precision; a sample with a larger |P| or |Q| (never seen
// with trained or random weights) takes the direct tanh(P - Q) path.
// Padding rows/columns hold EP = EQ = 1 (tanh = 0) / P = Q = 0.
//
// Workgroup = (sample, graph, column chunk); grid = B * groups * NCHUNK.
// The prologue issues every global load it needs (P/Q, W_rm, A-stat, bias)
// before its first LDS write and meets ONE barrier: a workgroup timeline
// (scripts/timeline.py) showed the earlier load -> barrier -> load chain
// costing 3.4-5.4 us of a 16-24 us launch.  The temporal adjacency splits
// its columns in two so that B = 256 fills every CU with two workgroups
// (one round: all prologues start together, and a second round of
// workgroups would pay its prologue again rather than overlap it).
// ===========================================================================
template <int MODE, int NROW, int K, int NA, bool HL>
struct AdjGeom {
  static constexpr int RT = cdiv(NROW, 16), KSTEPS = cdiv(K, 4), KP = 4 * KSTEPS;
  // HL: columns (q, slot) with the slot order of the split-f16 GC kernels
  // (dstd_hilo.h): spatial joints interleaved, temporal frames sequential
  using SM = SlotMap<NA, MODE == 0>;
  static constexpr int SL = HL ? SM::SL : NA;
  static constexpr int NCOL = NA * SL, NCT = cdiv(NCOL, 16);
  static constexpr int NAA = NA * NA;  // A-stat entries
  static constexpr int SA = NA + 1;  // + one padding column
  static constexpr bool WREG = RT * KSTEPS <= 64;
  static constexpr int SR = stride_mod32(RT * 16, 16);
  static constexpr int OS = 20;                         // output staging row stride
  static constexpr int STG = NWV * RT * 16 * OS;        // per-wave output staging (also W staging)
  static constexpr int NCOLP = rup(NAA + 1, 4);         // astat (+ padding column)
  static constexpr int T = MODE == 0 ? NROW : NA;
  static constexpr int V = MODE == 0 ? NA : NROW;
  static constexpr int NCHUNK = MODE == 0 ? 1 : 2;      // column chunks per (sample, graph): one round of workgroups at B = 256
  static constexpr int CPC = cdiv(NCT, NCHUNK);         // column tiles per chunk
  static_assert(STG >= K * NROW, "W staging must fit the output staging area");
  static constexpr int LDS_FLOATS = 4 * KP * SA + (WREG ? 0 : KP * SR) + STG + NCOLP + 16 + 4;
};

template <int MODE, int NROW, int K, int NA, bool HL>
// 4 waves per SIMD (two 8-wave workgroups per CU): caps VGPRs at 128
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(4))) void k_adj_fast(AdjArgs a) {
  using Gm = AdjGeom<MODE, NROW, K, NA, HL>;
  constexpr int SL = Gm::SL, NAA = Gm::NAA;
  constexpr int RT = Gm::RT, KSTEPS = Gm::KSTEPS, KP = Gm::KP, NCOL = Gm::NCOL, NCT = Gm::NCT, SA = Gm::SA;
  constexpr bool WREG = Gm::WREG;
  constexpr int SR = Gm::SR, OS = Gm::OS;
  constexpr int T = Gm::T, V = Gm::V;
  constexpr float C2 = 2.8853900817779268f;  // 2*log2(e)
  extern __shared__ float lds[];
  float* Pl = lds;               // [KP][SA] raw P
  float* Ql = Pl + KP * SA;      // [KP][SA] raw Q
  float* El = Ql + KP * SA;      // [KP][SA] 2^(c*P)
  float* Fl = El + KP * SA;      // [KP][SA] 2^(-c*Q)
  float* Wl = Fl + KP * SA;      // [KP][SR] (only when !WREG)
  float* stg = Wl + (WREG ? 0 : KP * SR);   // W staging, then per-wave output staging
  float* asl = stg + Gm::STG;               // astat [NCOL] + zero padding column
  float* bsl = asl + Gm::NCOLP;             // bias rows [16 * RT]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kl = lane >> 4, cl = lane & 15;
  const int chunk = blockIdx.x % Gm::NCHUNK;
  const int g = (blockIdx.x / Gm::NCHUNK) % a.ngroups;
  const int n = blockIdx.x / (Gm::NCHUNK * a.ngroups);
  if (n >= a.B) return;
  TL(MODE, 0)

  // ---- prologue: every global load first ----
  // P/Q planes are channel-innermost (PQLayout sch == 1, Q right after P):
  // P_0, P_1, Q_0, Q_1 of one (frame, joint) are one float4, read in memory order
  const PQLayout L = a.pql;
  const float* pqb = a.pq + (size_t)n * L.sn + a.p_ch[g];
  Stager<float4, T * V> spq;
  spq.load(tid, [&](int i) {
    const int t = MODE == 0 ? i % T : i / V, v = MODE == 0 ? i / T : i % V;  // memory order
    return ld4(pqb + t * L.st + v * L.sv);
  });
  const float* W = a.W[g];
  Stager<float, NROW * K> sw;
  sw.load(tid, [&](int i) { return W[i]; });
  Stager<float, NAA> sas;
  sas.load(tid, [&](int i) { return a.astat[g][i]; });
  const float bias_v = tid < 16 * RT && tid < NROW ? a.bias[g][tid] : 0.f;
  const float alpha = *a.alpha;

  // LDS padding (no load dependence)
  for (int i = tid; i < KP * SA; i += NTHR) {
    const int k = i / SA, c = i - (i / SA) * SA;
    if (k >= K || c >= NA) {
      Pl[i] = 0.f;
      Ql[i] = 0.f;
      El[i] = 1.f;
      Fl[i] = 1.f;
    }
  }
  if (tid < Gm::NCOLP - NAA) asl[NAA + tid] = 0.f;
  if (tid < 16 * RT) bsl[tid] = bias_v;
  sw.store(tid, [&](int i, float v) { stg[i] = v; });
  sas.store(tid, [&](int i, float v) { asl[i] = v; });
  int bad = 0;
  spq.store(tid, [&](int i, float4 q) {
    const int t = MODE == 0 ? i % T : i / V, v = MODE == 0 ? i / T : i % V;
    const int k0 = MODE == 0 ? t : v, c = MODE == 0 ? v : t, kstep = MODE == 0 ? T : V;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int idx = (k0 + r * kstep) * SA + c;
      const float pv = r ? q.y : q.x, qv = r ? q.w : q.z;
      Pl[idx] = pv;
      Ql[idx] = qv;
      const float ep = C2 * pv, eq = -C2 * qv;
      bad |= !(fabsf(ep) <= 120.f && fabsf(eq) <= 120.f);
      El[idx] = __builtin_amdgcn_exp2f(ep);
      Fl[idx] = __builtin_amdgcn_exp2f(eq);
    }
  });
  const bool sep = __syncthreads_or(bad) == 0;
  TL(MODE, 1)

  float wr[WREG ? RT : 1][WREG ? KSTEPS : 1];
  if constexpr (WREG) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
        const int r = rt * 16 + cl, k = ks * 4 + kl;
        wr[rt][ks] = (r < NROW && k < K) ? stg[r * K + k] : 0.f;
      }
  } else {
    for (int i = tid; i < KP * SR; i += NTHR) {
      const int k = i / SR, r = i % SR;
      Wl[i] = (k < K && r < NROW) ? stg[r * K + k] : 0.f;
    }
  }
  float brow[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 4; ++j) brow[rt][j] = bsl[rt * 16 + kl * 4 + j];
  __syncthreads();  // stg (W staging) becomes the per-wave output staging

  float* so = stg + wave * (RT * 16 * OS);  // this wave's output staging
  float* out = a.out + (size_t)n * a.out_sN + (size_t)g * a.out_sG;
  const int ct_end = min(NCT, (chunk + 1) * Gm::CPC);
  for (int ct = chunk * Gm::CPC + wave; ct < ct_end; ct += NWV) {
    const int col = ct * 16 + cl;
    // ca: P index (contracted by the GC kernel), cb: Q index (its output column)
    int ca, cb;
    if constexpr (HL) {
      const int q = col / SL, pi = Gm::SM::slot_idx(col - q * SL);
      ca = col < NCOL && pi < NA ? pi : NA;
      cb = col < NCOL && pi < NA ? q : NA;
    } else {
      ca = col < NCOL ? col / NA : NA;
      cb = col < NCOL ? col - ca * NA : NA;
    }
    const bool cv = ca < NA;
    f32x4 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = zero4();
    if (sep) {
      const float* pw = El + kl * SA + ca;
      const float* qw = Fl + kl * SA + cb;
      float bv[KSTEPS];
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
        const float e = pw[ks * 4 * SA] * qw[ks * 4 * SA] + 1.f;
        bv[ks] = 1.f - 2.f * __builtin_amdgcn_rcpf(e);
      }
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          float av;
          if constexpr (WREG) av = wr[rt][ks];
          else av = Wl[(ks * 4 + kl) * SR + rt * 16 + cl];
          acc[rt] = mfma16x16x4(av, bv[ks], acc[rt]);
        }
      }
    } else {
      const float* pw = Pl + kl * SA + ca;
      const float* qw = Ql + kl * SA + cb;
      for (int ks = 0; ks < KSTEPS; ++ks) {
        const float bv = fast_tanh(pw[ks * 4 * SA] - qw[ks * 4 * SA]);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          float av;
          if constexpr (WREG) av = wr[rt][ks];
          else av = Wl[(ks * 4 + kl) * SR + rt * 16 + cl];
          acc[rt] = mfma16x16x4(av, bv, acc[rt]);
        }
      }
    }
    // epilogue: transpose the 16-column tile through this wave's LDS slot so
    // each lane stores 16 contiguous bytes of one row (1 KiB per store)
    const float as = asl[cv ? ca * NA + cb : NAA];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        so[(rt * 16 + kl * 4 + j) * OS + cl] = cv ? alpha * (acc[rt][j] + brow[rt][j]) + as : 0.f;
    if constexpr (HL) {
      // (row, 8-column group) per lane: 8 values -> hi / lo halves, one
      // 16-byte store per plane; row stride ldo and plane stride NCOL in halves
      uint16_t* oh = reinterpret_cast<uint16_t*>(out);
#pragma unroll
      for (int it = 0; it < cdiv(RT * 32, 64); ++it) {
        const int item = lane + 64 * it, row = item >> 1, c8 = ct * 16 + 8 * (item & 1);
        if (row < NROW && c8 < NCOL) {
          const float4 v0 = ld4(so + row * OS + 8 * (item & 1)), v1 = ld4(so + row * OS + 8 * (item & 1) + 4);
          uint4 hi, lo;
          split8(v0, v1, hi, lo);
          *reinterpret_cast<uint4*>(oh + (size_t)row * a.ldo + c8) = hi;
          *reinterpret_cast<uint4*>(oh + (size_t)row * a.ldo + NCOL + c8) = lo;
        }
      }
    } else {
      const int q = lane & 3;
      const int c4 = ct * 16 + 4 * q;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int row = rt * 16 + (lane >> 2);
        const float4 v = ld4(so + row * OS + 4 * q);
        if (row < NROW && c4 < NCOL) st4(out + (size_t)row * a.ldo + c4, v);
      }
    }
  }
  TL(MODE, 2)
  TL(MODE, 3)
}


// ===========================================================================
// dispatch
// ===========================================================================
namespace {

template <typename K>
int resident_per_cu(K k, size_t lds) {
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k, NTHR, lds) != hipSuccess || nb < 1) nb = 1;
  (void)hipGetLastError();
  return nb;
}

template <int MODE, int NROW, int K, int NA, bool HL>
hipError_t adj_fast_run_hl(const AdjArgs& a, hipStream_t s) {
  using Gm = AdjGeom<MODE, NROW, K, NA, HL>;
  constexpr size_t lds = (size_t)Gm::LDS_FLOATS * sizeof(float);
  static int occ = resident_per_cu(k_adj_fast<MODE, NROW, K, NA, HL>, lds);
  (void)occ;  // raises the LDS cap where needed
  if (HL ? (a.ldo != 2 * Gm::NCOL || a.ncol != Gm::NCOL) : a.ldo % 4 != 0) return hipErrorNotSupported;
  const int grid = a.B * a.ngroups * Gm::NCHUNK;
  hipLaunchKernelGGL((k_adj_fast<MODE, NROW, K, NA, HL>), dim3(grid), dim3(NTHR), lds, s, a);
  return hipGetLastError();
}
template <int MODE, int NROW, int K, int NA>
hipError_t adj_fast_run(const AdjArgs& a, hipStream_t s) {
  return a.hl ? adj_fast_run_hl<MODE, NROW, K, NA, true>(a, s) : adj_fast_run_hl<MODE, NROW, K, NA, false>(a, s);
}

}  // namespace

hipError_t launch_adj_fast(const AdjArgs& a, hipStream_t s, int) {
  // channel-innermost P/Q planes, Q right after P, 16-byte aligned (see the prologue)
  if (a.pql.sch != 1 || ((uintptr_t)a.pq & 15) || (a.pql.st & 3) || (a.pql.sv & 3) || (a.pql.sn & 3))
    return hipErrorNotSupported;
  for (int g = 0; g < a.ngroups; ++g)
    if (a.q_ch[g] != a.p_ch[g] + 2 || (a.p_ch[g] & 3)) return hipErrorNotSupported;
  if (a.mode == 0) {
    if (a.T == 35 && a.V == 22) return adj_fast_run<0, 35, 70, 22>(a, s);
    if (a.T == 35 && a.V == 25) return adj_fast_run<0, 35, 70, 25>(a, s);
    if (a.T == 40 && a.V == 23) return adj_fast_run<0, 40, 80, 23>(a, s);
    if (a.T == 75 && a.V == 22) return adj_fast_run<0, 75, 150, 22>(a, s);
  } else {
    if (a.T == 35 && a.V == 22) return adj_fast_run<1, 22, 44, 35>(a, s);
    if (a.T == 35 && a.V == 25) return adj_fast_run<1, 25, 50, 35>(a, s);
    if (a.T == 40 && a.V == 23) return adj_fast_run<1, 23, 46, 40>(a, s);
    if (a.T == 75 && a.V == 22) return adj_fast_run<1, 22, 44, 75>(a, s);
  }
  return hipErrorNotSupported;
}

}  // namespace dstd

#ifdef DSTD_STAMPS
extern "C" int dstd_debug_timeline(int mode, unsigned long long* host, int n) {
  if (mode < 0 || mode > 1 || n > 2048 * 4) return 1;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tl), n * sizeof(unsigned long long),
                                  mode * 2048 * 4 * sizeof(unsigned long long));
}
#endif
