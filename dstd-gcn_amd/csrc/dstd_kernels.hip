// DSTDGC hot-path kernels for MI355X (gfx950, CDNA4).
//
// One DSTDGCB (model/dstdgcn.py:141-163) runs as four launches:
//   k_adj (spatial)   Adj_s[n,i,t,v,w] = a_sm*(W_rm_i . tanh(P_i - Q_i) + b_rm_i)[t,(v,w)] + A_s*W_s+R_s
//   k_spatial         y = sum_i conv_f_i(x) . Adj_s_i per frame ; h = prelu(bn(y) + r) ; P_t,Q_t of h
//   k_adj (temporal)  Adj_t[n,v,t,u] = a_tm*(W_rm . tanh(P_t - Q_t) + b_rm)[v,(t,u)] + A_t + R_t
//   k_temporal        y = conv_f(h) . Adj_t per joint ; inter-block epilogue ; P_s,Q_s of next block
// Every contraction runs on the exact-fp32 MFMA (v_mfma_f32_16x16x4_f32).
// The tanh matrix M (2T x V^2 per sample, SURVEY §7 hard part 3) is never
// materialised: each wave generates its B-operand fragment in registers.
#include "dstd_common.h"
#include "dstd_kernels.h"

namespace dstd {

// ===========================================================================
// parameter folding
// ===========================================================================
__global__ void k_fold(FoldArgs a) {
  const FoldJob& j = a.jobs[blockIdx.y];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < j.n; i += gridDim.x * blockDim.x) {
    if (j.kind == FOLD_BN) {
      // BatchNorm1d eval: (x - m)/sqrt(v + eps)*w + b = x*s + (b - m*s)
      const float s = j.p0[i] / sqrtf(j.p3[i] + j.eps);
      const int c = i / j.V, v = i - c * j.V;
      j.o0[v * j.C + c] = s;
      j.o1[v * j.C + c] = j.p1[i] - j.p2[i] * s;
    } else if (j.kind == FOLD_AWR) {
      j.o0[i] = j.p0[i] * j.p1[i] + j.p2[i];
    } else {
      j.o0[i] = j.p0[i] + j.p1[i];
    }
  }
}

hipError_t launch_fold(const FoldArgs& a, hipStream_t s) {
  if (a.njobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fold, dim3(8, a.njobs), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ===========================================================================
// P / Q reduced embeddings from an NTVC activation (conv_m1 / conv_m2,
// model/dstdgcn.py:66-67, 82), optionally building the 6-channel model input.
// One thread per (n, t, v).
// ===========================================================================
__global__ __launch_bounds__(256) void k_pq(PQArgs a) {
  const int TV = a.T * a.V;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.B * TV) return;
  const int n = idx / TV, tv = idx % TV;
  const int v = tv % a.V;
  float xr[64];
  int cin = a.Cin;
  if (a.make_x6) {
    // x [B][T][V][3]; residual = x[:, -1:] (last frame), :298-302
    const float* xi = a.x + (size_t)idx * 3;
    const float* xl = a.x + ((size_t)(n * a.T + a.T - 1) * a.V + v) * 3;
    float* o = a.x6 + (size_t)idx * 6;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      xr[c] = xi[c];
      xr[3 + c] = xi[c] - xl[c];
      o[c] = xr[c];
      o[3 + c] = xr[3 + c];
    }
    cin = 6;
  } else {
    const float* xi = a.x + (size_t)idx * cin;
    for (int c = 0; c < cin; ++c) xr[c] = xi[c];
  }
  if (a.pq == nullptr) return;
  for (int j = 0; j < a.nw; ++j) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float* w = a.w[j] + r * cin;
      float s = a.b[j][r];
      for (int c = 0; c < cin; ++c) s += w[c] * xr[c];
      a.pq[(size_t)n * a.pql.sn + (2 * j + r) * a.pql.sch + (tv / a.V) * a.pql.st + v * a.pql.sv] = s;
    }
  }
}

hipError_t launch_pq(const PQArgs& a, hipStream_t s) {
  const int total = a.B * a.T * a.V;
  hipLaunchKernelGGL(k_pq, dim3(cdiv(total, 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ===========================================================================
// Dynamic adjacency (the tanh GEMM).  Per sample n and graph g:
//   D[row][col] = sum_k W[row][k] * tanh(Pl[k][col / NA] - Ql[k][col % NA])
//   out[row][col] = alpha * (D + bias[row]) + astat[col]
// spatial : row = t (T),  col = (v,w) (V*V), k = r*T + t'  (model/dstdgcn.py:84-86)
// temporal: row = v (V),  col = (t,u) (T*T), k = r*V + v'  (:89-92)
// Rows are RT 16-row MFMA tiles; each wave owns 16-column tiles and builds
// its B fragment (one tanh per lane per k-step) in registers, reused by all
// RT row tiles.  W (A operand) is staged transposed in LDS.
// ===========================================================================
template <int RT>
__global__ __launch_bounds__(256) void k_adj(AdjArgs a) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunk = blockIdx.x % a.nchunks;
  const int rg = (blockIdx.x / a.nchunks) % a.rgroups;
  const int g = (blockIdx.x / (a.nchunks * a.rgroups)) % a.ngroups;
  const int n = blockIdx.x / (a.nchunks * a.rgroups * a.ngroups);
  const int K = a.K, NA = a.NA, ncol = a.ncol;
  const int row0 = rg * RT * 16, nrow = min(a.nrow - row0, RT * 16);  // this group's rows
  const int Kp = rup(K, 4);
  const int SR = stride_mod32(RT * 16, 16);
  float* Wl = lds;              // [Kp][SR]   Wl[k][row] = W[row][k]
  float* Pl = Wl + Kp * SR;     // [Kp][NA]
  float* Ql = Pl + Kp * NA;     // [Kp][NA]

  const float* W = a.W[g] + (size_t)row0 * K;
  for (int i = tid; i < Kp * SR; i += 256) {
    const int k = i / SR, r = i % SR;
    Wl[i] = (k < K && r < nrow) ? W[r * K + k] : 0.f;
  }
  const float* P = a.pq + (size_t)n * a.pql.sn + a.p_ch[g] * a.pql.sch;
  const float* Q = a.pq + (size_t)n * a.pql.sn + a.q_ch[g] * a.pql.sch;
  for (int i = tid; i < Kp * NA; i += 256) {
    const int k = i / NA, c = i % NA;
    float pv = 0.f, qv = 0.f;
    if (k < K) {
      int src;
      if (a.mode == 0) {  // k = r*T + t', c = v
        src = (k / a.T) * a.pql.sch + (k % a.T) * a.pql.st + c * a.pql.sv;
      } else {            // k = r*V + v', c = t
        src = (k / a.V) * a.pql.sch + c * a.pql.st + (k % a.V) * a.pql.sv;
      }
      pv = P[src];
      qv = Q[src];
    }
    Pl[i] = pv;
    Ql[i] = qv;
  }
  __syncthreads();

  const float alpha = *a.alpha;
  const float* bias = a.bias[g] + row0;
  const float* astat = a.astat[g];
  float* out = a.out + (size_t)n * a.out_sN + (size_t)g * a.out_sG + (size_t)row0 * a.ldo;
  const int nct = cdiv(ncol, 16);
  const int ct0 = chunk * a.ctiles_per_wg;
  const int ct1 = min(nct, ct0 + a.ctiles_per_wg);
  const int KS = Kp / 4;
  const int kl = lane >> 4, cl = lane & 15;

  for (int ct = ct0 + wave; ct < ct1; ct += DSTD_WAVES) {
    const int col = ct * 16 + cl;
    const bool cv = col < ncol;
    const int ca = cv ? col / NA : 0;
    const int cb = cv ? col - ca * NA : 0;
    f32x4 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = zero4();
    const float* pw = Pl + ca;
    const float* qw = Ql + cb;
    const float* ww = Wl + cl;
    for (int ks = 0; ks < KS; ++ks) {
      const int k = ks * 4 + kl;
      const float bv = cv ? fast_tanh(pw[k * NA] - qw[k * NA]) : 0.f;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma16x16x4(ww[k * SR + rt * 16], bv, acc[rt]);
    }
    if (cv) {
      const float as = astat[col];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = rt * 16 + kl * 4 + j;
          if (row < nrow) out[(size_t)row * a.ldo + col] = alpha * (acc[rt][j] + bias[row]) + as;
        }
      }
    }
  }
}

static size_t adj_lds_bytes(int RT, int K, int NA) {
  const int Kp = rup(K, 4);
  return (size_t)(Kp * stride_mod32(RT * 16, 16) + 2 * Kp * NA) * sizeof(float);
}

template <int RT>
static hipError_t launch_adj_rt(const AdjArgs& a, hipStream_t s, int nblocks, size_t lds) {
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k_adj<RT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k_adj<RT>, dim3(nblocks), dim3(256), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_adj(AdjArgs a, hipStream_t s) {
  // rows split into the fewest groups whose W tile (Kp x RT*16) and P/Q planes fit in LDS;
  // each group re-evaluates the tanh operand (only T > 112 spatial needs more than one)
  const int RT_all = cdiv(a.nrow, 16);
  if (RT_all < 1 || a.ngroups < 1 || a.ngroups > 2) return hipErrorInvalidValue;
  a.rgroups = 1;
  while (a.rgroups <= RT_all &&
         (cdiv(RT_all, a.rgroups) > 8 || adj_lds_bytes(cdiv(RT_all, a.rgroups), a.K, a.NA) > 160 * 1024))
    ++a.rgroups;
  if (a.rgroups > RT_all) return hipErrorInvalidValue;
  const int RT = cdiv(RT_all, a.rgroups);
  a.rgroups = cdiv(RT_all, RT);
  const int nct = cdiv(a.ncol, 16);
  // enough workgroups to fill the chip (>= ~1024), each a multiple of 4 tiles
  int chunks = cdiv(1024, a.B * a.ngroups);
  chunks = chunks < 1 ? 1 : chunks;
  const int max_chunks = cdiv(nct, DSTD_WAVES);
  chunks = chunks > max_chunks ? max_chunks : chunks;
  a.ctiles_per_wg = rup(cdiv(nct, chunks), DSTD_WAVES);
  a.nchunks = cdiv(nct, a.ctiles_per_wg);
  {
    const hipError_t fe = launch_adj_fast(a, s, a.B * a.ngroups * a.nchunks);
    if (fe != hipErrorNotSupported || a.hl) return fe;  // the split-f16 layout has no generic writer
  }
  const int nblocks = a.B * a.ngroups * a.rgroups * a.nchunks;
  const size_t lds = adj_lds_bytes(RT, a.K, a.NA);
  switch (RT) {
    case 1: return launch_adj_rt<1>(a, s, nblocks, lds);
    case 2: return launch_adj_rt<2>(a, s, nblocks, lds);
    case 3: return launch_adj_rt<3>(a, s, nblocks, lds);
    case 4: return launch_adj_rt<4>(a, s, nblocks, lds);
    case 5: return launch_adj_rt<5>(a, s, nblocks, lds);
    case 6: return launch_adj_rt<6>(a, s, nblocks, lds);
    case 7: return launch_adj_rt<7>(a, s, nblocks, lds);
    case 8: return launch_adj_rt<8>(a, s, nblocks, lds);
    default: return hipErrorInvalidValue;
  }
}


// ===========================================================================
// Shared pieces of the two graph-convolution kernels.
// ===========================================================================
constexpr int kMaxItems = 8;              // aggregation tiles held per wave
constexpr size_t kGcLdsBudget = 78 * 1024;  // -> 2 workgroups per CU

// 1x1 conv as MFMA GEMM out of LDS:
//   Fs[g*Cp + c][p] = sum_ci wf[g][c][ci] * xs[p][ci] + bf[g][c]
// rows: G groups of Cp (Cout rounded to 16) output channels, cols: NP16
// positions, K = Cin.  Each wave keeps the A fragments (weights) of up to two
// 16-row tiles in registers and streams B (the activation tile) from LDS.
template <int KS>
__device__ __forceinline__ void conv_gemm(const float* const* wf, const float* const* bf, int G, int Cin,
                                          int Cout, int Cp, const float* xs, int SX, int NP16, float* Fs,
                                          int SP, int wave, int lane) {
  const int kl = lane >> 4, cl = lane & 15;
  const int CT = Cp / 16;
  const int MT = G * CT;
  const int NT = NP16 / 16;
  for (int mt0 = wave; mt0 < MT; mt0 += 2 * DSTD_WAVES) {
    float af[2][KS];
    bool live[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int mt = mt0 + m * DSTD_WAVES;
      live[m] = mt < MT;
      const int g = live[m] ? mt / CT : 0;
      const int c = (mt % CT) * 16 + cl;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int k = ks * 4 + kl;
        af[m][ks] = (live[m] && c < Cout && k < Cin) ? wf[g][c * Cin + k] : 0.f;
      }
    }
    for (int nt = 0; nt < NT; ++nt) {
      float bq[KS];
      const float* xr = xs + (nt * 16 + cl) * SX + kl;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) bq[ks] = xr[ks * 4];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        if (!live[m]) continue;
        const int mt = mt0 + m * DSTD_WAVES;
        f32x4 acc = zero4();
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) acc = mfma16x16x4(af[m][ks], bq[ks], acc);
        const int g = mt / CT;
        const int cbase = (mt % CT) * 16 + kl * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = cbase + j;
          const float bias = c < Cout ? bf[g][c] : 0.f;
          Fs[(mt * 16 + kl * 4 + j) * SP + nt * 16 + cl] = acc[j] + bias;
        }
      }
    }
  }
}

// P/Q of the next DSTDGC from an LDS tile zs[c][p] (stride SP):
//   pq[n][2j+r][t][v] = sum_c w[j][r][c] * zs[c][p] + b[j][r]
// pos(p) maps the tile column to (t*V + v) within the sample.
template <typename PosFn>
__device__ __forceinline__ void pq_from_tile(const float* const* pqw, const float* const* pqb, int npqw,
                                             int C, const float* zs, int SP, int P, float* pq_n, int sch,
                                             int tid, PosFn pos) {
  const int nch = 2 * npqw;
  for (int i = tid; i < nch * P; i += DSTD_THREADS) {
    const int ch = i / P, p = i % P;
    const int j = ch >> 1, r = ch & 1;
    const float* w = pqw[j] + r * C;
    float s = pqb[j][r];
    for (int c = 0; c < C; ++c) s += w[c] * zs[c * SP + p];
    pq_n[(size_t)ch * sch + pos(p)] = s;
  }
}

// ===========================================================================
// Spatial GC.  Workgroup = (sample n, Tt consecutive frames).
//   Fs[(i,c)][(tt,v)] = conv_f_i(x)       (model/dstdgcn.py:81)
//   y[c][t][w] = sum_i sum_v Fs[(i,c)][(tt,v)] * Adj_i[t][v][w]   (:87, :145-150)
// epi 1 (DSTDGCB mid-block, :151-154): h = prelu(bn(y) + r), r = x (Cin == Cout)
// or bn_r(conv_r(x)) (residual conv rows ride in the same GEMM as group NI).
// Optional: P_t/Q_t of h for the block's temporal DSTDGC.
// ===========================================================================
static __host__ __device__ inline void spatial_geom(int Tt, int V, int Cin, int Cout, int G, int NI, int* NP16,
                                                     int* SX, int* Cp, int* SP, int* lds_floats) {
  *NP16 = rup(Tt * V, 16);
  *SX = stride_2mod4(4 * ks_for(Cin));
  *Cp = rup(Cout, 16);
  *SP = stride_2mod4(*NP16);
  *lds_floats = (*NP16) * (*SX) + G * (*Cp) * (*SP) + NI * Tt * V * V;
}

template <int KS>
__global__ __launch_bounds__(256) void k_spatial(SpatialArgs a) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kl = lane >> 4, cl = lane & 15;
  const int T = a.T, V = a.V, Cin = a.Cin, Cout = a.Cout, NI = a.NI, Tt = a.Tt;
  const int ntb = cdiv(T, Tt);
  const int n = blockIdx.x / ntb;
  const int t0 = (blockIdx.x % ntb) * Tt;
  const int nf = min(Tt, T - t0);
  const int P = nf * V;
  int NP16, SX, Cp, SP, lf;
  spatial_geom(Tt, V, Cin, Cout, a.G, NI, &NP16, &SX, &Cp, &SP, &lf);
  float* xs = lds;                      // [NP16][SX]   x tile, position-major
  float* Fs = xs + NP16 * SX;           // [G*Cp][SP]   conv outputs
  float* adjs = Fs + a.G * Cp * SP;     // [NI][Tt][V][V]
  const int KX = 4 * KS;

  const float* xg = a.x + (size_t)(n * T + t0) * V * Cin;
  for (int i = tid; i < NP16 * KX; i += DSTD_THREADS) {
    const int p = i / KX, c = i % KX;
    xs[p * SX + c] = (p < P && c < Cin) ? xg[p * Cin + c] : 0.f;
  }
  const int VV = V * V;
  for (int gi = 0; gi < NI; ++gi) {
    const float* ag = a.adj + (((size_t)n * NI + gi) * T + t0) * a.adj_ld;
    float* ad = adjs + gi * Tt * VV;
    for (int i = tid; i < nf * VV; i += DSTD_THREADS) ad[i] = ag[(i / VV) * a.adj_ld + i % VV];
  }
  __syncthreads();

  conv_gemm<KS>(a.wf, a.bf, a.G, Cin, Cout, Cp, xs, SX, NP16, Fs, SP, wave, lane);
  __syncthreads();

  // aggregation: items (tt, mc, nw); K = (i, v) in 4-wide steps
  const int MC = Cp / 16, NW = cdiv(V, 16), KV = cdiv(V, 4);
  const int items = nf * MC * NW;
  f32x4 res[kMaxItems];
#pragma unroll
  for (int it = 0; it < kMaxItems; ++it) {
    res[it] = zero4();
    const int item = wave + it * DSTD_WAVES;
    if (item >= items) continue;
    const int tt = item / (MC * NW);
    const int rem = item % (MC * NW);
    const int mc = rem / NW, nw = rem % NW;
    const int w = nw * 16 + cl;
    f32x4 acc = zero4();
    for (int gi = 0; gi < NI; ++gi) {
      const float* fr = Fs + (gi * Cp + mc * 16 + cl) * SP + tt * V;
      const float* ar = adjs + (gi * Tt + tt) * VV + w;
      for (int vs = 0; vs < KV; ++vs) {
        const int v = vs * 4 + kl;
        const float av = v < V ? fr[v] : 0.f;
        const float bv = (v < V && w < V) ? ar[v * V] : 0.f;
        acc = mfma16x16x4(av, bv, acc);
      }
    }
    res[it] = acc;
  }
  __syncthreads();  // Fs group-0 rows are reused below as the h tile

  const float pw = a.epi ? *a.prelu : 0.f;
  const bool has_res = a.G > NI;
#pragma unroll
  for (int it = 0; it < kMaxItems; ++it) {
    const int item = wave + it * DSTD_WAVES;
    if (item >= items) continue;
    const int tt = item / (MC * NW);
    const int rem = item % (MC * NW);
    const int mc = rem / NW, nw = rem % NW;
    const int w = nw * 16 + cl;
    if (w >= V) continue;
    const int p = tt * V + w;
    float* yo = a.y + ((size_t)(n * T + t0 + tt) * V + w) * Cout;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = mc * 16 + kl * 4 + j;
      if (c >= Cout) continue;
      float val = res[it][j];
      if (a.epi) {
        const int cv = w * Cout + c;
        const float r = has_res ? Fs[(NI * Cp + c) * SP + p] * a.rbn_s[cv] + a.rbn_h[cv] : xs[p * SX + c];
        val = prelu_f(val * a.bn_s[cv] + a.bn_h[cv] + r, pw);
      }
      yo[c] = val;
      Fs[c * SP + p] = val;
    }
  }
  if (a.pq) {
    __syncthreads();
    const PQLayout L = a.pql;
    pq_from_tile(a.pqw, a.pqb, a.npqw, Cout, Fs, SP, P, a.pq + (size_t)n * L.sn, L.sch, tid,
                 [=](int p) { return (t0 + p / V) * L.st + (p % V) * L.sv; });
  }
}

// ===========================================================================
// Temporal GC.  Workgroup = (sample n, Vt consecutive joints); tile column
// p = vv*T + t (joint-major).
//   Fs[c][(vv,t)] = conv_f(h)                         (model/dstdgcn.py:81)
//   y[c][u][v] = sum_t Fs[c][(vv,t)] * Adj[v][t][u]     (:93)
// Epilogues: raw; ENC  z = prelu_e(bn_e(y + x_in))    (:247-248, 283-284)
//            IN   z = prelu(bn_in(y))                 (:306-308)
//            OUT  out[n][t][v][c] = y + x[n][T-1][v][c] (:314-315)
// Optional: P_s/Q_s of z for the next block's spatial DSTDGCs.
// ===========================================================================
static __host__ __device__ inline void temporal_geom(int Vt, int T, int Cin, int Cout, int* NP16, int* SX,
                                                      int* Cp, int* SP, int* lds_floats) {
  *NP16 = rup(Vt * T, 16);
  *SX = stride_2mod4(4 * ks_for(Cin));
  *Cp = rup(Cout, 16);
  *SP = stride_2mod4(*NP16);
  *lds_floats = (*NP16) * (*SX) + (*Cp) * (*SP) + Vt * T * T;
}

template <int KS>
__global__ __launch_bounds__(256) void k_temporal(TemporalArgs a) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kl = lane >> 4, cl = lane & 15;
  const int T = a.T, V = a.V, Cin = a.Cin, Cout = a.Cout, Vt = a.Vt;
  const int nvb = cdiv(V, Vt);
  const int n = blockIdx.x / nvb;
  const int v0 = (blockIdx.x % nvb) * Vt;
  const int nv = min(Vt, V - v0);
  const int P = nv * T;
  int NP16, SX, Cp, SP, lf;
  temporal_geom(Vt, T, Cin, Cout, &NP16, &SX, &Cp, &SP, &lf);
  float* hs = lds;                  // [NP16][SX]
  float* Fs = hs + NP16 * SX;       // [Cp][SP]
  float* adjs = Fs + Cp * SP;       // [Vt][T][T]
  const int KX = 4 * KS;

  // gather the joint tile: for each t, nv*Cin contiguous floats
  const int rowlen = nv * KX;
  for (int i = tid; i < NP16 * KX; i += DSTD_THREADS) {
    const int p = i / KX, c = i % KX;
    float val = 0.f;
    if (p < P && c < Cin) {
      const int vv = p / T, t = p % T;
      val = a.h[((size_t)(n * T + t) * V + v0 + vv) * Cin + c];
    }
    hs[p * SX + c] = val;
  }
  (void)rowlen;
  const int TT = T * T;
  const float* ag = a.adj + ((size_t)n * V + v0) * a.adj_ld;
  for (int i = tid; i < nv * TT; i += DSTD_THREADS) adjs[i] = ag[(i / TT) * a.adj_ld + i % TT];
  __syncthreads();

  const float* wf[1] = {a.wf};
  const float* bf[1] = {a.bf};
  conv_gemm<KS>(wf, bf, 1, Cin, Cout, Cp, hs, SX, NP16, Fs, SP, wave, lane);
  __syncthreads();

  const int MC = Cp / 16, NU = cdiv(T, 16), KT = cdiv(T, 4);
  const int items = nv * MC * NU;
  f32x4 res[kMaxItems];
#pragma unroll
  for (int it = 0; it < kMaxItems; ++it) {
    res[it] = zero4();
    const int item = wave + it * DSTD_WAVES;
    if (item >= items) continue;
    const int vv = item / (MC * NU);
    const int rem = item % (MC * NU);
    const int mc = rem / NU, nu = rem % NU;
    const int u = nu * 16 + cl;
    const float* fr = Fs + (mc * 16 + cl) * SP + vv * T;
    const float* ar = adjs + vv * TT + u;
    f32x4 acc = zero4();
    for (int ts = 0; ts < KT; ++ts) {
      const int t = ts * 4 + kl;
      const float av = t < T ? fr[t] : 0.f;
      const float bv = (t < T && u < T) ? ar[t * T] : 0.f;
      acc = mfma16x16x4(av, bv, acc);
    }
    res[it] = acc;
  }
  __syncthreads();  // Fs rows are reused below as the output tile

  const float pw = (a.epi == TEPI_ENC || a.epi == TEPI_IN) ? *a.prelu : 0.f;
#pragma unroll
  for (int it = 0; it < kMaxItems; ++it) {
    const int item = wave + it * DSTD_WAVES;
    if (item >= items) continue;
    const int vv = item / (MC * NU);
    const int rem = item % (MC * NU);
    const int mc = rem / NU, nu = rem % NU;
    const int u = nu * 16 + cl;
    if (u >= T) continue;
    const int v = v0 + vv;
    const size_t o = ((size_t)(n * T + u) * V + v) * Cout;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = mc * 16 + kl * 4 + j;
      if (c >= Cout) continue;
      float val = res[it][j];
      if (a.epi == TEPI_ENC) {
        val += a.xres[o + c];
        val = prelu_f(val * a.bn_s[v * Cout + c] + a.bn_h[v * Cout + c], pw);
      } else if (a.epi == TEPI_IN) {
        val = prelu_f(val * a.bn_s[v * Cout + c] + a.bn_h[v * Cout + c], pw);
      } else if (a.epi == TEPI_OUT) {
        val += a.xres[((size_t)(n * T + T - 1) * V + v) * Cout + c];
      }
      a.y[o + c] = val;
      Fs[c * SP + vv * T + u] = val;
    }
  }
  if (a.pq) {
    __syncthreads();
    const PQLayout L = a.pql;
    pq_from_tile(a.pqw, a.pqb, a.npqw, Cout, Fs, SP, P, a.pq + (size_t)n * L.sn, L.sch, tid,
                 [=](int p) { return (p % T) * L.st + (v0 + p / T) * L.sv; });
  }
}

// ---------------------------------------------------------------------------
int spatial_frames_per_wg(int T, int V, int Cin, int Cout, int G) {
  const int NI = G >= 2 ? 2 : 1;
  (void)NI;
  int best = 1;
  for (int Tt = 1; Tt <= 8 && Tt <= T; ++Tt) {
    int NP16, SX, Cp, SP, lf;
    spatial_geom(Tt, V, Cin, Cout, G, 2, &NP16, &SX, &Cp, &SP, &lf);
    const int items = Tt * (Cp / 16) * cdiv(V, 16);
    if ((size_t)lf * 4 <= kGcLdsBudget && items <= kMaxItems * DSTD_WAVES) best = Tt;
  }
  return best;
}

int temporal_joints_per_wg(int T, int V, int Cin, int Cout) {
  int best = 1;
  for (int Vt = 1; Vt <= 8 && Vt <= V; ++Vt) {
    int NP16, SX, Cp, SP, lf;
    temporal_geom(Vt, T, Cin, Cout, &NP16, &SX, &Cp, &SP, &lf);
    const int items = Vt * (Cp / 16) * cdiv(T, 16);
    if ((size_t)lf * 4 <= kGcLdsBudget && items <= kMaxItems * DSTD_WAVES) best = Vt;
  }
  return best;
}

template <typename Kern>
static void set_max_lds(Kern k, size_t lds) {
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

#define DSTD_KS_DISPATCH(KSV, KERNEL, ...)                 \
  switch (KSV) {                                            \
    case 1: KERNEL<1>(__VA_ARGS__); break;                  \
    case 2: KERNEL<2>(__VA_ARGS__); break;                  \
    case 4: KERNEL<4>(__VA_ARGS__); break;                  \
    case 8: KERNEL<8>(__VA_ARGS__); break;                  \
    case 16: KERNEL<16>(__VA_ARGS__); break;                \
    default: return hipErrorInvalidValue;                   \
  }

template <int KS>
static void run_spatial(const SpatialArgs& a, hipStream_t s, int nblocks, size_t lds) {
  set_max_lds(k_spatial<KS>, lds);
  hipLaunchKernelGGL(k_spatial<KS>, dim3(nblocks), dim3(DSTD_THREADS), lds, s, a);
}

template <int KS>
static void run_temporal(const TemporalArgs& a, hipStream_t s, int nblocks, size_t lds) {
  set_max_lds(k_temporal<KS>, lds);
  hipLaunchKernelGGL(k_temporal<KS>, dim3(nblocks), dim3(DSTD_THREADS), lds, s, a);
}

hipError_t launch_spatial(SpatialArgs a, hipStream_t s) {
  if (a.Tt <= 0) {
    const hipError_t we = launch_spatial_wave(a, s);
    if (we != hipErrorNotSupported) return we;
  }
  if (a.Tt <= 0) a.Tt = spatial_frames_per_wg(a.T, a.V, a.Cin, a.Cout, a.G);
  int NP16, SX, Cp, SP, lf;
  spatial_geom(a.Tt, a.V, a.Cin, a.Cout, a.G, a.NI, &NP16, &SX, &Cp, &SP, &lf);
  // every aggregation tile must have a register slot; LDS must fit one CU
  if (a.Tt * (Cp / 16) * cdiv(a.V, 16) > kMaxItems * DSTD_WAVES || (size_t)lf * 4 > 160 * 1024 || a.V > 32 ||
      a.Cin > 64 || a.Cout > 64 || a.NI < 1 || a.NI > 2 || a.G < a.NI || a.G > 3)
    return hipErrorInvalidValue;
  const size_t lds = (size_t)lf * sizeof(float);
  const int nblocks = a.B * cdiv(a.T, a.Tt);
  const int ks = ks_for(a.Cin);
  DSTD_KS_DISPATCH(ks, run_spatial, a, s, nblocks, lds);
  return hipGetLastError();
}

hipError_t launch_temporal(TemporalArgs a, hipStream_t s) {
  if (a.Vt <= 0) {
    const hipError_t we = launch_temporal_wave(a, s);
    if (we != hipErrorNotSupported) return we;
  }
  if (a.Vt <= 0) a.Vt = temporal_joints_per_wg(a.T, a.V, a.Cin, a.Cout);
  int NP16, SX, Cp, SP, lf;
  temporal_geom(a.Vt, a.T, a.Cin, a.Cout, &NP16, &SX, &Cp, &SP, &lf);
  if (a.Vt * (Cp / 16) * cdiv(a.T, 16) > kMaxItems * DSTD_WAVES || (size_t)lf * 4 > 160 * 1024 || a.Cin > 64 ||
      a.Cout > 64)
    return hipErrorInvalidValue;
  const size_t lds = (size_t)lf * sizeof(float);
  const int nblocks = a.B * cdiv(a.V, a.Vt);
  const int ks = ks_for(a.Cin);
  DSTD_KS_DISPATCH(ks, run_temporal, a, s, nblocks, lds);
  return hipGetLastError();
}

// ===========================================================================
// NCTV <-> NTVC layout change at the op / block boundary (32x32 LDS tiles).
// ===========================================================================
__global__ __launch_bounds__(256) void k_transpose(TransposeArgs a) {
  __shared__ float tile[32][33];
  // view: to_ntvc: src [B][C][TV] -> dst [B][TV][C]; else src [B][TV][C] -> dst [B][C][TV]
  const int R = a.to_ntvc ? a.C : a.TV;   // rows of the src matrix
  const int Cc = a.to_ntvc ? a.TV : a.C;  // cols of the src matrix
  const int tr = cdiv(R, 32), tc = cdiv(Cc, 32);
  const int b = blockIdx.x / (tr * tc);
  const int rem = blockIdx.x % (tr * tc);
  const int r0 = (rem / tc) * 32, c0 = (rem % tc) * 32;
  const float* src = a.src + (size_t)b * R * Cc;
  float* dst = a.dst + (size_t)b * R * Cc;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    if (r < R && c < Cc) tile[i][tx] = src[(size_t)r * Cc + c];
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (r < R && c < Cc) dst[(size_t)c * R + r] = tile[tx][i];
  }
}

hipError_t launch_transpose(const TransposeArgs& a, hipStream_t s) {
  const int R = a.to_ntvc ? a.C : a.TV;
  const int Cc = a.to_ntvc ? a.TV : a.C;
  const int nblocks = a.B * cdiv(R, 32) * cdiv(Cc, 32);
  hipLaunchKernelGGL(k_transpose, dim3(nblocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace dstd
