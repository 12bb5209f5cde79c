// Shape-specialised DSTDGC kernels (the hot path for the shipped configs).
//
// Same math and data layouts as the generic kernels in dstd_kernels.hip, but
// every tile extent is a template constant, so LDS addressing folds into
// immediate offsets, divisions become multiply-shifts, operand tiles are
// zero-padded instead of guarded, global staging is 16 bytes per lane where
// the layout allows, and the P/Q reductions of the epilogues run on MFMA.
// Instantiated for (T, V) in {(35,22), (35,25), (40,23), (75,22)}; other
// shapes fall back to the generic kernels.
#include "dstd_common.h"
#include "dstd_kernels.h"

namespace dstd {

namespace {

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ void st2(float* p, float a, float b) { *reinterpret_cast<float2*>(p) = make_float2(a, b); }

// ---------------------------------------------------------------------------
// 1x1 conv GEMM out of LDS (see conv_gemm in dstd_kernels.hip):
//   Fs[g*CP + c][p] = sum_k wf[g][c][k] * xs[p][k] + bf[g][c]
// Work split: MT = G*CT row tiles.  MT >= 4: a wave owns rows mt = wave + 4m;
// MT < 4: waves split the column tiles of each row tile.
// ---------------------------------------------------------------------------
template <int KS, int CT, int G, int NT, int SX, int SP>
__device__ __forceinline__ void conv_fast(const float* const* wf, const float* const* bf, int Cin, int Cout,
                                          const float* xs, float* Fs, int wave, int lane) {
  constexpr int MT = G * CT;
  const int kl = lane >> 4, cl = lane & 15;
  if constexpr (MT >= 4) {
    // a wave owns row tiles mt = wave + 4m and sweeps every column tile
    constexpr int MTW = cdiv(MT, 4);
    float af[MTW][KS];
    float bias[MTW][4];
    bool live[MTW];
#pragma unroll
    for (int m = 0; m < MTW; ++m) {
      const int mt = wave + 4 * m;
      live[m] = mt < MT;
      const int g = live[m] ? mt / CT : 0;
      const int c = (mt % CT) * 16 + cl;
      const float* w = wf[g];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int k = ks * 4 + kl;
        af[m][ks] = (live[m] && c < Cout && k < Cin) ? w[c * Cin + k] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cr = (mt % CT) * 16 + kl * 4 + j;
        bias[m][j] = (live[m] && cr < Cout) ? bf[g][cr] : 0.f;
      }
    }
    for (int nt = 0; nt < NT; ++nt) {
      float bq[KS];
      const float* xr = xs + (nt * 16 + cl) * SX + kl;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) bq[ks] = xr[ks * 4];
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        if (!live[m]) continue;
        f32x4 acc = zero4();
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) acc = mfma16x16x4(af[m][ks], bq[ks], acc);
        float* fo = Fs + ((wave + 4 * m) * 16 + kl * 4) * SP + nt * 16 + cl;
#pragma unroll
        for (int j = 0; j < 4; ++j) fo[j * SP] = acc[j] + bias[m][j];
      }
    }
  } else {
    // few row tiles (Cout = 3 blocks): (mt, nt) units dealt round robin
    for (int u = wave; u < MT * NT; u += DSTD_WAVES) {
      const int mt = u % MT, nt = u / MT;
      const int g = mt / CT;
      const int c = (mt % CT) * 16 + cl;
      const float* w = wf[g];
      const float* xr = xs + (nt * 16 + cl) * SX + kl;
      f32x4 acc = zero4();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int k = ks * 4 + kl;
        const float av = (c < Cout && k < Cin) ? w[c * Cin + k] : 0.f;
        acc = mfma16x16x4(av, xr[ks * 4], acc);
      }
      float* fo = Fs + (mt * 16 + kl * 4) * SP + nt * 16 + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cr = (mt % CT) * 16 + kl * 4 + j;
        fo[j * SP] = acc[j] + (cr < Cout ? bf[g][cr] : 0.f);
      }
    }
  }
}

// P/Q of the next DSTDGC on MFMA: out[ch][p] = sum_c w[ch][c] * hs[c][p] + b[ch]
// hs = Fs rows [0, CT*16) (row stride SP); nch = 2*npqw <= 8 channels fill one
// 16-row tile.  store(ch, p, value) writes one result.
template <int CT, int NT, int SP, typename Store>
__device__ __forceinline__ void pq_fast(const float* const* pqw, const float* const* pqb, int npqw, int Cout,
                                        const float* hs, int P, int wave, int lane, Store store) {
  constexpr int KSO = CT * 4;
  const int kl = lane >> 4, cl = lane & 15;
  const int nch = 2 * npqw;
  float aw[KSO];
  {
    const int ch = cl;
    const float* w = ch < nch ? pqw[ch >> 1] + (ch & 1) * Cout : nullptr;
#pragma unroll
    for (int ks = 0; ks < KSO; ++ks) {
      const int c = ks * 4 + kl;
      aw[ks] = (ch < nch && c < Cout) ? w[c] : 0.f;
    }
  }
  for (int nt = wave; nt < NT; nt += DSTD_WAVES) {
    const float* hr = hs + kl * SP + nt * 16 + cl;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < KSO; ++ks) acc = mfma16x16x4(aw[ks], hr[ks * 4 * SP], acc);
    const int p = nt * 16 + cl;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ch = kl * 4 + j;
      if (ch < nch && p < P) store(ch, p, acc[j] + pqb[ch >> 1][ch & 1]);
    }
  }
}

}  // namespace

// ===========================================================================
// Dynamic adjacency, specialised.  MODE 0: rows t (NROW = T), cols (v,w)
// (NA = V), K = 2T.  MODE 1: rows v (NROW = V), cols (t,u) (NA = T), K = 2V.
// The W_rm fragments live in registers when they fit (RT*KSTEPS <= 64).
// ===========================================================================
template <int MODE, int NROW, int K, int NA>
__global__ __launch_bounds__(256) void k_adj_fast(AdjArgs a) {
  constexpr int RT = cdiv(NROW, 16), KSTEPS = cdiv(K, 4), KP = 4 * KSTEPS;
  constexpr int NCOL = NA * NA, NCT = cdiv(NCOL, 16);
  constexpr bool WREG = RT * KSTEPS <= 64;
  constexpr int SR = stride_mod32(RT * 16, 16);
  constexpr int T = MODE == 0 ? NROW : NA;
  constexpr int V = MODE == 0 ? NA : NROW;
  extern __shared__ float lds[];
  float* Pl = lds;              // [KP][NA]
  float* Ql = Pl + KP * NA;     // [KP][NA]
  float* Wl = Ql + KP * NA;     // [KP][SR] (only when !WREG)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kl = lane >> 4, cl = lane & 15;
  const int chunk = blockIdx.x % a.nchunks;
  const int g = (blockIdx.x / a.nchunks) % a.ngroups;
  const int n = blockIdx.x / (a.nchunks * a.ngroups);

  const float* P = a.pq + (size_t)n * a.pq_sN + a.p_off[g];
  const float* Q = a.pq + (size_t)n * a.pq_sN + a.q_off[g];
  for (int i = tid; i < KP * NA; i += DSTD_THREADS) {
    const int k = i / NA, c = i - (i / NA) * NA;
    float pv = 0.f, qv = 0.f;
    if (k < K) {
      const int src = MODE == 0 ? i : (k / V) * T * V + c * V + (k % V);
      pv = P[src];
      qv = Q[src];
    }
    Pl[i] = pv;
    Ql[i] = qv;
  }
  const float* W = a.W[g];
  float wr[WREG ? RT : 1][WREG ? KSTEPS : 1];
  if constexpr (WREG) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
        const int r = rt * 16 + cl, k = ks * 4 + kl;
        wr[rt][ks] = (r < NROW && k < K) ? W[r * K + k] : 0.f;
      }
  } else {
    for (int i = tid; i < KP * SR; i += DSTD_THREADS) {
      const int k = i / SR, r = i % SR;
      Wl[i] = (k < K && r < NROW) ? W[r * K + k] : 0.f;
    }
  }
  __syncthreads();

  const float alpha = *a.alpha;
  const float* bias = a.bias[g];
  const float* astat = a.astat[g];
  float* out = a.out + (size_t)n * a.out_sN + (size_t)g * a.out_sG;
  float brow[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = rt * 16 + kl * 4 + j;
      brow[rt][j] = row < NROW ? bias[row] : 0.f;
    }
  const int ct0 = chunk * a.ctiles_per_wg;
  const int ct1 = min(NCT, ct0 + a.ctiles_per_wg);
  for (int ct = ct0 + wave; ct < ct1; ct += DSTD_WAVES) {
    const int col = ct * 16 + cl;
    const bool cv = col < NCOL;
    const int ca = cv ? col / NA : 0;
    const int cb = cv ? col - ca * NA : 0;
    const float* pw = Pl + kl * NA + ca;
    const float* qw = Ql + kl * NA + cb;
    f32x4 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = zero4();
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      float bv = fast_tanh(pw[ks * 4 * NA] - qw[ks * 4 * NA]);
      bv = cv ? bv : 0.f;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        float av;
        if constexpr (WREG) av = wr[rt][ks];
        else av = Wl[(ks * 4 + kl) * SR + rt * 16 + cl];
        acc[rt] = mfma16x16x4(av, bv, acc[rt]);
      }
    }
    if (cv) {
      const float as = astat[col];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = rt * 16 + kl * 4 + j;
          if (row < NROW) out[row * NCOL + col] = alpha * (acc[rt][j] + brow[rt][j]) + as;
        }
    }
  }
}

// ===========================================================================
// Spatial GC, specialised: workgroup = (sample, TT frames), see k_spatial.
// ===========================================================================
template <int V, int KS, int CT, int G, int NI, int TT>
struct SpatialGeom {
  static constexpr int CINP = 4 * KS;
  static constexpr int SX = CINP + 2;           // == 2 (mod 4): conflict-free B reads
  static constexpr int NP16 = rup(TT * V, 16);
  static constexpr int NT = NP16 / 16;
  static constexpr int SP = NP16 + 2;
  static constexpr int CP = CT * 16;
  static constexpr int VP = rup(V, 4);
  static constexpr int KV = VP / 4;
  static constexpr int NW = cdiv(V, 16);
  static constexpr int ITEMS = TT * CT * NW;
  static constexpr int IPW = cdiv(ITEMS, DSTD_WAVES);
  static constexpr int ADJ = NI * TT * VP * V;
  static constexpr int LDS_FLOATS = NP16 * SX + G * CP * SP + ADJ + 32;
};

template <int V, int KS, int CT, int G, int NI, int TT>
__global__ __launch_bounds__(256) void k_spatial_fast(SpatialArgs a) {
  using Gm = SpatialGeom<V, KS, CT, G, NI, TT>;
  constexpr int SX = Gm::SX, SP = Gm::SP, CP = Gm::CP, VP = Gm::VP, NP16 = Gm::NP16;
  extern __shared__ float lds[];
  float* xs = lds;                        // [NP16][SX]
  float* Fs = xs + NP16 * SX;             // [G*CP][SP]
  float* adjs = Fs + G * CP * SP;         // [NI][TT][VP][V] + zero pad
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kl = lane >> 4, cl = lane & 15;
  const int T = a.T, Cin = a.Cin, Cout = a.Cout;
  constexpr int VV = V * V;
  const int ntb = cdiv(T, TT);
  const int n = blockIdx.x / ntb;
  const int t0 = (blockIdx.x - n * ntb) * TT;
  const int nf = min(TT, T - t0);
  const int P = nf * V;

  // ---- stage the x tile [p][k] and the adjacency tile ----------------------
  const float* xg = a.x + (size_t)(n * T + t0) * V * Cin;
  if (Cin == Gm::CINP) {
    for (int i = tid; i < NP16 * (Gm::CINP / 4); i += DSTD_THREADS) {
      const int p = i / (Gm::CINP / 4), c = (i % (Gm::CINP / 4)) * 4;
      const float4 v = p < P ? ld4(xg + p * Gm::CINP + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      st2(xs + p * SX + c, v.x, v.y);
      st2(xs + p * SX + c + 2, v.z, v.w);
    }
  } else {
    for (int i = tid; i < NP16 * Gm::CINP; i += DSTD_THREADS) {
      const int p = i / Gm::CINP, c = i % Gm::CINP;
      xs[p * SX + c] = (p < P && c < Cin) ? xg[p * Cin + c] : 0.f;
    }
  }
#pragma unroll
  for (int gi = 0; gi < NI; ++gi) {
    const float* ag = a.adj + (((size_t)n * NI + gi) * T + t0) * VV;
    float* ad = adjs + gi * TT * VP * V;
    for (int i = tid; i < TT * VP * V; i += DSTD_THREADS) {
      const int tt = i / (VP * V);
      const int r = i - tt * (VP * V);
      const int v = r / V;
      ad[i] = (tt < nf && v < V) ? ag[tt * VV + r] : 0.f;
    }
  }
  if (tid < 32) adjs[Gm::ADJ + tid] = 0.f;
  __syncthreads();

  conv_fast<KS, CT, G, Gm::NT, SX, SP>(a.wf, a.bf, Cin, Cout, xs, Fs, wave, lane);
  __syncthreads();

  // ---- aggregation: y[c][tt][w] = sum_(g,v) F[(g,c)][(tt,v)] Adj_g[tt][v][w]
  f32x4 res[Gm::IPW];
#pragma unroll
  for (int it = 0; it < Gm::IPW; ++it) {
    res[it] = zero4();
    const int item = wave + it * DSTD_WAVES;
    if (item >= Gm::ITEMS) continue;
    const int tt = item / (CT * Gm::NW);
    const int rem = item - tt * (CT * Gm::NW);
    const int mc = rem / Gm::NW, nw = rem - (rem / Gm::NW) * Gm::NW;
    f32x4 acc = zero4();
#pragma unroll
    for (int gi = 0; gi < NI; ++gi) {
      const float* fa = Fs + (gi * CP + mc * 16 + cl) * SP + tt * V + kl;
      const float* fb = adjs + ((gi * TT + tt) * VP + kl) * V + nw * 16 + cl;
#pragma unroll
      for (int ks = 0; ks < Gm::KV; ++ks) acc = mfma16x16x4(fa[ks * 4], fb[ks * 4 * V], acc);
    }
    res[it] = acc;
  }
  __syncthreads();  // Fs group-0 rows become the h tile below

  // ---- epilogue: h = prelu(bn(y) + r), store NTVC, keep h for P_t/Q_t ------
  const float pw = a.epi ? *a.prelu : 0.f;
  constexpr bool HAS_RES = G > NI;
#pragma unroll
  for (int it = 0; it < Gm::IPW; ++it) {
    const int item = wave + it * DSTD_WAVES;
    if (item >= Gm::ITEMS) continue;
    const int tt = item / (CT * Gm::NW);
    const int rem = item - tt * (CT * Gm::NW);
    const int mc = rem / Gm::NW, nw = rem - (rem / Gm::NW) * Gm::NW;
    const int w = nw * 16 + cl;
    const int c0 = mc * 16 + kl * 4;
    if (w >= V || tt >= nf || c0 >= Cout) continue;
    const int p = tt * V + w;
    float val[4] = {res[it][0], res[it][1], res[it][2], res[it][3]};
    float* yo = a.y + ((size_t)(n * T + t0 + tt) * V + w) * Cout + c0;
    if (Cout % 4 == 0) {
      if (a.epi) {
        const float4 s = ld4(a.bn_s + w * Cout + c0), h = ld4(a.bn_h + w * Cout + c0);
        float r[4];
        if constexpr (HAS_RES) {
          const float4 rs = ld4(a.rbn_s + w * Cout + c0), rh = ld4(a.rbn_h + w * Cout + c0);
          const float* fr = Fs + (NI * CP + c0) * SP + p;
          r[0] = fr[0] * rs.x + rh.x;
          r[1] = fr[SP] * rs.y + rh.y;
          r[2] = fr[2 * SP] * rs.z + rh.z;
          r[3] = fr[3 * SP] * rs.w + rh.w;
        } else {
          const float* xr = xs + p * SX + c0;
          r[0] = xr[0]; r[1] = xr[1]; r[2] = xr[2]; r[3] = xr[3];
        }
        val[0] = prelu_f(val[0] * s.x + h.x + r[0], pw);
        val[1] = prelu_f(val[1] * s.y + h.y + r[1], pw);
        val[2] = prelu_f(val[2] * s.z + h.z + r[2], pw);
        val[3] = prelu_f(val[3] * s.w + h.w + r[3], pw);
      }
      st4(yo, make_float4(val[0], val[1], val[2], val[3]));
#pragma unroll
      for (int j = 0; j < 4; ++j) Fs[(c0 + j) * SP + p] = val[j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + j;
        if (c >= Cout) continue;
        float v = val[j];
        if (a.epi) {
          const int cv = w * Cout + c;
          float r;
          if constexpr (HAS_RES) r = Fs[(NI * CP + c) * SP + p] * a.rbn_s[cv] + a.rbn_h[cv];
          else r = xs[p * SX + c];
          v = prelu_f(v * a.bn_s[cv] + a.bn_h[cv] + r, pw);
        }
        yo[j] = v;
        Fs[c * SP + p] = v;
      }
    }
  }
  if (a.pq) {
    __syncthreads();
    const int TV = T * V;
    float* pqn = a.pq + (size_t)n * 2 * a.npqw * TV + t0 * V;
    pq_fast<CT, Gm::NT, SP>(a.pqw, a.pqb, a.npqw, Cout, Fs, P, wave, lane,
                            [=](int ch, int p, float v) { pqn[(size_t)ch * TV + p] = v; });
  }
}

// ===========================================================================
// Temporal GC, specialised: workgroup = (sample, VT joints), see k_temporal.
// ===========================================================================
template <int T, int KS, int CT, int VT>
struct TemporalGeom {
  static constexpr int CINP = 4 * KS;
  static constexpr int SX = CINP + 2;
  static constexpr int NP16 = rup(VT * T, 16);
  static constexpr int NT = NP16 / 16;
  static constexpr int SP = NP16 + 2;
  static constexpr int CP = CT * 16;
  static constexpr int TP = rup(T, 4);
  static constexpr int KT = TP / 4;
  static constexpr int NU = cdiv(T, 16);
  static constexpr int ITEMS = VT * CT * NU;
  static constexpr int IPW = cdiv(ITEMS, DSTD_WAVES);
  static constexpr int ADJ = VT * TP * T;
  static constexpr int LDS_FLOATS = NP16 * SX + CP * SP + ADJ + 32;
};

template <int T, int KS, int CT, int VT>
__global__ __launch_bounds__(256) void k_temporal_fast(TemporalArgs a) {
  using Gm = TemporalGeom<T, KS, CT, VT>;
  constexpr int SX = Gm::SX, SP = Gm::SP, TP = Gm::TP, NP16 = Gm::NP16;
  constexpr int TT2 = T * T;
  extern __shared__ float lds[];
  float* hs = lds;                    // [NP16][SX]   column p = vv*T + t
  float* Fs = hs + NP16 * SX;         // [CP][SP]
  float* adjs = Fs + Gm::CP * SP;     // [VT][TP][T] + zero pad
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kl = lane >> 4, cl = lane & 15;
  const int V = a.V, Cin = a.Cin, Cout = a.Cout;
  const int nvb = cdiv(V, VT);
  const int n = blockIdx.x / nvb;
  const int v0 = (blockIdx.x - n * nvb) * VT;
  const int nv = min(VT, V - v0);
  const int P = nv * T;

  if (Cin == Gm::CINP) {
    for (int i = tid; i < NP16 * (Gm::CINP / 4); i += DSTD_THREADS) {
      const int p = i / (Gm::CINP / 4), c = (i % (Gm::CINP / 4)) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p < P) {
        const int vv = p / T, t = p - (p / T) * T;
        v = ld4(a.h + ((size_t)(n * T + t) * V + v0 + vv) * Gm::CINP + c);
      }
      st2(hs + p * SX + c, v.x, v.y);
      st2(hs + p * SX + c + 2, v.z, v.w);
    }
  } else {
    for (int i = tid; i < NP16 * Gm::CINP; i += DSTD_THREADS) {
      const int p = i / Gm::CINP, c = i % Gm::CINP;
      float v = 0.f;
      if (p < P && c < Cin) {
        const int vv = p / T, t = p - (p / T) * T;
        v = a.h[((size_t)(n * T + t) * V + v0 + vv) * Cin + c];
      }
      hs[p * SX + c] = v;
    }
  }
  {
    const float* ag = a.adj + ((size_t)n * V + v0) * TT2;
    for (int i = tid; i < VT * TP * T; i += DSTD_THREADS) {
      const int vv = i / (TP * T);
      const int r = i - vv * (TP * T);
      const int t = r / T;
      adjs[i] = (vv < nv && t < T) ? ag[vv * TT2 + r] : 0.f;
    }
    if (tid < 32) adjs[Gm::ADJ + tid] = 0.f;
  }
  __syncthreads();

  const float* wf[1] = {a.wf};
  const float* bf[1] = {a.bf};
  conv_fast<KS, CT, 1, Gm::NT, SX, SP>(wf, bf, Cin, Cout, hs, Fs, wave, lane);
  __syncthreads();

  f32x4 res[Gm::IPW];
#pragma unroll
  for (int it = 0; it < Gm::IPW; ++it) {
    res[it] = zero4();
    const int item = wave + it * DSTD_WAVES;
    if (item >= Gm::ITEMS) continue;
    const int vv = item / (CT * Gm::NU);
    const int rem = item - vv * (CT * Gm::NU);
    const int mc = rem / Gm::NU, nu = rem - (rem / Gm::NU) * Gm::NU;
    const float* fa = Fs + (mc * 16 + cl) * SP + vv * T + kl;
    const float* fb = adjs + (vv * TP + kl) * T + nu * 16 + cl;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < Gm::KT; ++ks) acc = mfma16x16x4(fa[ks * 4], fb[ks * 4 * T], acc);
    res[it] = acc;
  }
  __syncthreads();

  const int epi = a.epi;
  const float pw = (epi == TEPI_ENC || epi == TEPI_IN) ? *a.prelu : 0.f;
#pragma unroll
  for (int it = 0; it < Gm::IPW; ++it) {
    const int item = wave + it * DSTD_WAVES;
    if (item >= Gm::ITEMS) continue;
    const int vv = item / (CT * Gm::NU);
    const int rem = item - vv * (CT * Gm::NU);
    const int mc = rem / Gm::NU, nu = rem - (rem / Gm::NU) * Gm::NU;
    const int u = nu * 16 + cl;
    const int c0 = mc * 16 + kl * 4;
    if (u >= T || vv >= nv || c0 >= Cout) continue;
    const int v = v0 + vv;
    const size_t o = ((size_t)(n * T + u) * V + v) * Cout + c0;
    float val[4] = {res[it][0], res[it][1], res[it][2], res[it][3]};
    if (Cout % 4 == 0) {
      if (epi == TEPI_ENC || epi == TEPI_IN) {
        if (epi == TEPI_ENC) {
          const float4 r = ld4(a.xres + o);
          val[0] += r.x; val[1] += r.y; val[2] += r.z; val[3] += r.w;
        }
        const float4 s = ld4(a.bn_s + v * Cout + c0), h = ld4(a.bn_h + v * Cout + c0);
        val[0] = prelu_f(val[0] * s.x + h.x, pw);
        val[1] = prelu_f(val[1] * s.y + h.y, pw);
        val[2] = prelu_f(val[2] * s.z + h.z, pw);
        val[3] = prelu_f(val[3] * s.w + h.w, pw);
      } else if (epi == TEPI_OUT) {
        const float4 r = ld4(a.xres + ((size_t)(n * T + T - 1) * V + v) * Cout + c0);
        val[0] += r.x; val[1] += r.y; val[2] += r.z; val[3] += r.w;
      }
      st4(a.y + o, make_float4(val[0], val[1], val[2], val[3]));
#pragma unroll
      for (int j = 0; j < 4; ++j) Fs[(c0 + j) * SP + vv * T + u] = val[j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + j;
        if (c >= Cout) continue;
        float x = val[j];
        if (epi == TEPI_ENC) {
          x += a.xres[o + j];
          x = prelu_f(x * a.bn_s[v * Cout + c] + a.bn_h[v * Cout + c], pw);
        } else if (epi == TEPI_IN) {
          x = prelu_f(x * a.bn_s[v * Cout + c] + a.bn_h[v * Cout + c], pw);
        } else if (epi == TEPI_OUT) {
          x += a.xres[((size_t)(n * T + T - 1) * V + v) * Cout + c];
        }
        a.y[o + j] = x;
        Fs[c * SP + vv * T + u] = x;
      }
    }
  }
  if (a.pq) {
    __syncthreads();
    const int TV = T * V;
    float* pqn = a.pq + (size_t)n * 2 * a.npqw * TV + v0;
    pq_fast<CT, Gm::NT, SP>(a.pqw, a.pqb, a.npqw, Cout, Fs, P, wave, lane, [=](int ch, int p, float val) {
      const int vv = p / T, t = p - (p / T) * T;
      pqn[(size_t)ch * TV + t * V + vv] = val;
    });
  }
}

// ===========================================================================
// dispatch
// ===========================================================================
namespace {

template <typename K>
void allow_big_lds(K k) {
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <int MODE, int NROW, int K, int NA>
hipError_t adj_fast_run(const AdjArgs& a, hipStream_t s, int nblocks) {
  constexpr int KP = 4 * cdiv(K, 4);
  constexpr int RT = cdiv(NROW, 16);
  constexpr bool WREG = RT * cdiv(K, 4) <= 64;
  constexpr size_t lds = (size_t)(2 * KP * NA + (WREG ? 0 : KP * stride_mod32(RT * 16, 16))) * sizeof(float);
  static bool once = (allow_big_lds(k_adj_fast<MODE, NROW, K, NA>), true);
  (void)once;
  hipLaunchKernelGGL((k_adj_fast<MODE, NROW, K, NA>), dim3(nblocks), dim3(DSTD_THREADS), lds, s, a);
  return hipGetLastError();
}

template <int V, int KS, int CT, int G, int NI, int TT>
hipError_t spatial_fast_run(const SpatialArgs& a, hipStream_t s) {
  using Gm = SpatialGeom<V, KS, CT, G, NI, TT>;
  static_assert(Gm::LDS_FLOATS * 4 <= 160 * 1024, "spatial tile exceeds LDS");
  static bool once = (allow_big_lds(k_spatial_fast<V, KS, CT, G, NI, TT>), true);
  (void)once;
  const int nblocks = a.B * cdiv(a.T, TT);
  hipLaunchKernelGGL((k_spatial_fast<V, KS, CT, G, NI, TT>), dim3(nblocks), dim3(DSTD_THREADS),
                     (size_t)Gm::LDS_FLOATS * sizeof(float), s, a);
  return hipGetLastError();
}

template <int T, int KS, int CT, int VT>
hipError_t temporal_fast_run(const TemporalArgs& a, hipStream_t s) {
  using Gm = TemporalGeom<T, KS, CT, VT>;
  static_assert(Gm::LDS_FLOATS * 4 <= 160 * 1024, "temporal tile exceeds LDS");
  static bool once = (allow_big_lds(k_temporal_fast<T, KS, CT, VT>), true);
  (void)once;
  const int nblocks = a.B * cdiv(a.V, VT);
  hipLaunchKernelGGL((k_temporal_fast<T, KS, CT, VT>), dim3(nblocks), dim3(DSTD_THREADS),
                     (size_t)Gm::LDS_FLOATS * sizeof(float), s, a);
  return hipGetLastError();
}

// channel configurations: (KS, CT) from (Cin, Cout)
inline int chan_cfg(int cin, int cout) {
  const int ks = ks_for(cin), ct = cdiv(cout, 16);
  if (ks == 16 && ct == 4) return 0;  // 64 -> 64
  if (ks == 2 && ct == 4) return 1;   // 6 -> 64
  if (ks == 16 && ct == 1) return 2;  // 64 -> 3
  if (ks == 1 && ct == 1) return 3;   // 3 -> 3
  return -1;
}

template <int V>
hipError_t spatial_fast_v(const SpatialArgs& a, hipStream_t s) {
  constexpr int TT = 2;
  const int cfg = chan_cfg(a.Cin, a.Cout);
  if (a.NI == 2 && a.G == 2 && cfg == 0) return spatial_fast_run<V, 16, 4, 2, 2, TT>(a, s);
  if (a.NI == 2 && a.G == 3 && cfg == 1) return spatial_fast_run<V, 2, 4, 3, 2, TT>(a, s);
  if (a.NI == 2 && a.G == 3 && cfg == 2) return spatial_fast_run<V, 16, 1, 3, 2, TT>(a, s);
  if (a.NI == 1 && a.G == 1 && cfg == 0) return spatial_fast_run<V, 16, 4, 1, 1, TT>(a, s);
  if (a.NI == 1 && a.G == 1 && cfg == 1) return spatial_fast_run<V, 2, 4, 1, 1, TT>(a, s);
  if (a.NI == 1 && a.G == 1 && cfg == 2) return spatial_fast_run<V, 16, 1, 1, 1, TT>(a, s);
  return hipErrorNotSupported;
}

template <int T, int VT>
hipError_t temporal_fast_t(const TemporalArgs& a, hipStream_t s) {
  const int cfg = chan_cfg(a.Cin, a.Cout);
  if (cfg == 0) return temporal_fast_run<T, 16, 4, VT>(a, s);
  if (cfg == 3) return temporal_fast_run<T, 1, 1, VT>(a, s);
  return hipErrorNotSupported;
}

}  // namespace

hipError_t launch_adj_fast(const AdjArgs& a, hipStream_t s, int nblocks) {
  if (a.mode == 0) {
    if (a.T == 35 && a.V == 22) return adj_fast_run<0, 35, 70, 22>(a, s, nblocks);
    if (a.T == 35 && a.V == 25) return adj_fast_run<0, 35, 70, 25>(a, s, nblocks);
    if (a.T == 40 && a.V == 23) return adj_fast_run<0, 40, 80, 23>(a, s, nblocks);
    if (a.T == 75 && a.V == 22) return adj_fast_run<0, 75, 150, 22>(a, s, nblocks);
  } else {
    if (a.T == 35 && a.V == 22) return adj_fast_run<1, 22, 44, 35>(a, s, nblocks);
    if (a.T == 35 && a.V == 25) return adj_fast_run<1, 25, 50, 35>(a, s, nblocks);
    if (a.T == 40 && a.V == 23) return adj_fast_run<1, 23, 46, 40>(a, s, nblocks);
    if (a.T == 75 && a.V == 22) return adj_fast_run<1, 22, 44, 75>(a, s, nblocks);
  }
  return hipErrorNotSupported;
}

hipError_t launch_spatial_fast(const SpatialArgs& a, hipStream_t s) {
  if (a.epi != 0 && a.epi != 1) return hipErrorNotSupported;
  switch (a.V) {
    case 22: return spatial_fast_v<22>(a, s);
    case 23: return spatial_fast_v<23>(a, s);
    case 25: return spatial_fast_v<25>(a, s);
    default: return hipErrorNotSupported;
  }
}

hipError_t launch_temporal_fast(const TemporalArgs& a, hipStream_t s) {
  switch (a.T) {
    case 35: return temporal_fast_t<35, 2>(a, s);
    case 40: return temporal_fast_t<40, 2>(a, s);
    case 75: return temporal_fast_t<75, 1>(a, s);
    default: return hipErrorNotSupported;
  }
}

}  // namespace dstd
