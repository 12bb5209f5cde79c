// Internal kernel interface (argument blocks + host launchers).  The public
// C ABI is include/dstd_gcn.h; dstd_capi.hip sequences these launches.
//
// Internal activation layout is NTVC ([B][T][V][C], channels innermost): a
// frame tile (spatial kernel) and a joint tile (temporal kernel) are then
// both runs of contiguous channel vectors, and the MFMA accumulator (4
// consecutive channels per lane) stores as one 16-byte write.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace dstd {

// ---- parameter folding (one launch per forward) --------------------------
enum FoldKind { FOLD_BN = 0, FOLD_AWR = 1, FOLD_AR = 2 };
struct FoldJob {
  int kind;   // FOLD_BN: o0 = w/sqrt(v+eps), o1 = b - m*o0, written transposed:
              //          input index c*V + v (BatchNorm1d channel) -> output v*C + c
              //          so an epilogue reads 4 consecutive channels as one float4
              // FOLD_AWR: o0 = p0*p1 + p2   (A_s*W_s + R_s, model/dstdgcn.py:146-149)
              // FOLD_AR:  o0 = p0 + p1      (A_t + R_t, :158-160)
  int n;
  int C, V;   // FOLD_BN only
  const float* p0;
  const float* p1;
  const float* p2;
  const float* p3;
  float eps;
  float* o0;
  float* o1;
};
constexpr int kMaxFoldJobs = 32;  // per launch; longer lists are split
struct FoldArgs {
  FoldJob jobs[kMaxFoldJobs];
  int njobs;
};

// ---- P/Q planes ------------------------------------------------------------
// The reduced embeddings of conv_m1 / conv_m2 (model/dstdgcn.py:66-67): element
// (sample n, channel ch, frame t, joint v) lives at n*sn + ch*sch + t*st + v*sv.
// The forward uses channel-innermost layouts so that a GC epilogue writes its
// P/Q as whole 16-byte vectors: the spatial P/Q of a block ([B][V][T][8], 8
// channels = P,Q of both spatial DSTDGCs) are written by the temporal kernel
// one joint at a time, the temporal P/Q ([B][T][V][4]) by the spatial kernel
// one frame at a time.
struct PQLayout {
  long sn;
  int sch, st, sv;
};
inline PQLayout pq_layout_vt(int nch, int T, int V) { return PQLayout{(long)nch * T * V, 1, nch, nch * T}; }
inline PQLayout pq_layout_tv(int nch, int T, int V) { return PQLayout{(long)nch * T * V, 1, nch * V, nch}; }
inline bool pq_layout_eq(const PQLayout& a, const PQLayout& b) {
  return a.sn == b.sn && a.sch == b.sch && a.st == b.st && a.sv == b.sv;
}

// ---- reduced embeddings P,Q (conv_m1 / conv_m2) ---------------------------
// pq(n, 2j+r, t, v) = sum_c w[j][r*Cin + c] * x[n][t][v][c] + b[j][r]
// (j indexes up to 4 two-row weight blocks).  With make_x6 the input is the
// model input [B][T][V][3] and the kernel also writes x6 = cat(x, x - x[:, -1])
// (model/dstdgcn.py:298-303) in NTVC.
struct PQArgs {
  const float* x;
  int B, T, V, Cin;
  int make_x6;
  float* x6;
  const float* w[4];
  const float* b[4];
  int nw;
  float* pq;
  PQLayout pql;
};

// ---- dynamic adjacency: Adj = alpha * (W_rm . tanh(P - Q) + b_rm) + Astat -
struct AdjArgs {
  const float* pq;
  PQLayout pql;
  int p_ch[2], q_ch[2];  // first P / Q channel of each graph (2 channels each)
  int mode;            // 0 spatial, 1 temporal (P/Q gather differs)
  int B, T, V;
  int nrow, K, NA, ncol;
  int ngroups;
  const float* W[2];
  const float* bias[2];
  const float* alpha;
  const float* astat[2];  // [ncol], row independent
  float* out;
  long out_sN, out_sG;
  int ldo;             // row stride of out (>= ncol, a multiple of 4 floats; hl: 2*ncol halves)
  int hl;              // 1: split-f16 planes in the slot order of dstd_hilo.h: out holds halves,
                       //    ldo counts halves (2 * ncol), out_sN / out_sG still count floats,
                       //    ncol = NA * SL
  int ctiles_per_wg, nchunks;
  int rgroups;         // generic writer: row groups of RT 16-row tiles per (n, g) (set by launch_adj)
};

// ---- spatial GC (both graphs) + DSTDGCB mid epilogue ----------------------
struct SpatialArgs {
  const float* x;       // NTVC [B][T][V][Cin]
  int B, T, V, Cin, Cout;
  int NI, G;            // NI graphs (1 or 2); G = NI + has residual conv
  const float* adj;     // [B][NI][T][adj_ld], row = V*V values (v, w)
  int adj_ld;
  const float* wf[3];
  const float* bf[3];
  int epi;              // 0 raw sum; 1 prelu(bn(y) + r)
  const float* bn_s;
  const float* bn_h;
  const float* rbn_s;
  const float* rbn_h;
  const float* prelu;
  float* y;             // NTVC [B][T][V][Cout]
  const float* pqw[4];
  const float* pqb[4];
  int npqw;
  float* pq;            // P/Q planes (2*npqw channels) or null
  PQLayout pql;
  int Tt;
};
// Folded BatchNorm vectors (bn_s, bn_h, rbn_s, rbn_h; temporal bn_s/bn_h) are
// in the transposed [V][C] layout produced by k_fold.

// ---- temporal GC + inter-block epilogue ----------------------------------
enum TemporalEpi { TEPI_RAW = 0, TEPI_ENC = 1, TEPI_IN = 2, TEPI_OUT = 3 };
struct TemporalArgs {
  const float* h;       // NTVC [B][T][V][Cin]
  int B, T, V, Cin, Cout;
  const float* adj;     // [B][V][adj_ld], row = T*T values (t, u)
  int adj_ld;
  const float* wf;
  const float* bf;
  int epi;
  const float* xres;
  const float* bn_s;
  const float* bn_h;
  const float* prelu;
  float* y;             // NTVC [B][T][V][Cout]
  const float* pqw[4];
  const float* pqb[4];
  int npqw;
  float* pq;
  PQLayout pql;
  int Vt;
};

struct TransposeArgs {
  const float* src;
  float* dst;
  int B, C, TV;
  int to_ntvc;  // 1: [B][C][TV] -> [B][TV][C]; 0: inverse
};

hipError_t launch_fold(const FoldArgs& a, hipStream_t s);
hipError_t launch_pq(const PQArgs& a, hipStream_t s);
hipError_t launch_adj(AdjArgs a, hipStream_t s);
hipError_t launch_spatial(SpatialArgs a, hipStream_t s);
hipError_t launch_temporal(TemporalArgs a, hipStream_t s);
hipError_t launch_transpose(const TransposeArgs& a, hipStream_t s);

// shape-specialised adjacency (dstd_adj.hip); hipErrorNotSupported when the
// shape has no instantiation and the generic kernel must run
hipError_t launch_adj_fast(const AdjArgs& a, hipStream_t s, int nblocks);
// exact-fp32 block kernels for the model's channel configurations
// (dstd_wave.hip), tried first; the generic kernels take every other shape
hipError_t launch_spatial_wave(const SpatialArgs& a, hipStream_t s);
hipError_t launch_temporal_wave(const TemporalArgs& a, hipStream_t s);

// Leading dimensions of the materialised adjacencies: rows padded to a
// multiple of 4 floats so the adjacency kernels store 16-byte vectors.
inline int adj_ld_spatial(int V) { return ((V * V + 3) / 4) * 4; }
inline int adj_ld_temporal(int T) { return ((T * T + 3) / 4) * 4; }

// tiling choices (host side, also used for workspace-free validation)
int spatial_frames_per_wg(int T, int V, int Cin, int Cout, int G);
int temporal_joints_per_wg(int T, int V, int Cin, int Cout);

}  // namespace dstd
