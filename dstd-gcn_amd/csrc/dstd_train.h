// Training-path primitives: a strided batched fp32-MFMA
// GEMM plus the element-wise / reduction kernels that the DSTDGC, BatchNorm
// and PReLU backward passes are composed of.  The fused inference kernels
// (dstd_wave.hip, dstd_hilo.hip) keep nothing for a backward pass; training
// instead materialises F, P, Q, M, E and D per op (a few MB per op at the
// config-5 batch of 32) and runs the backward as GEMMs over those saved
// tensors.  All launchers enqueue on the given stream and return the launch
// status.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "../../include/dstd_gcn_train.h"

namespace dstd {
namespace train {

// C[b] = alpha * A[b] . B[b] + beta * C[b] + bias_m[m]  for b over nb1 x nb2
// batches, or, with reduce != 0, C = alpha * sum_b A[b] . B[b] + beta*C + bias
// (batch strides of C ignored).  Every operand is addressed through explicit
// strides, so transposes and the spatial / temporal batch layouts need no
// copies.  beta == 0 never reads C.
struct Gemm {
  int M, N, K;
  int nb1 = 1, nb2 = 1;
  const float* A;
  long long a_b1 = 0, a_b2 = 0, a_m, a_k;
  const float* B;
  long long b_b1 = 0, b_b2 = 0, b_k, b_n;
  float* C;
  long long c_b1 = 0, c_b2 = 0, c_m, c_n;
  float alpha = 1.f, beta = 0.f;
  const float* bias_m = nullptr;
  int reduce = 0;
  int b_ones_last = 0;  // B(k, N-1) = 1: the last output column is sum_k A(m, k) (bias gradients)
  // nseg > 0: C is not written; output row m of segment i (row0 <= m <
  // row0 + rows) ACCUMULATES into seg[i].w[(m - row0) * (N - 1) + n] for
  // n < N - 1 and into seg[i].b[m - row0] for n = N - 1 (the [W | b]
  // gradient of packed convs lands in the parameters' own gradients)
  struct Seg {
    int row0, rows;
    float* w;
    float* b;
  };
  int nseg = 0;
  Seg seg[3];
  // d_out: also D = (*d_alpha) * C + (d_A[n] (* d_W[n]) + d_R[n]), same
  // layout as C (the DSTDGC adjacency alpha * conv_rm(M) + A_comb with the
  // block's A_s * W_s + R_s / A_t + R_t formed on the fly; d_W, d_R may be null)
  float* d_out = nullptr;
  const float* d_alpha = nullptr;
  const float* d_A = nullptr;
  const float* d_W = nullptr;
  const float* d_R = nullptr;
};

// Scratch (floats) a reduce-GEMM may need for its split-over-batches partials.
size_t gemm_scratch_floats(int M, int N);
// A reduce GEMM's split-K finish handed back instead of launched (gemm's
// defer argument; nsplit 0: the GEMM needed none), for finish_set.
struct GemmFinish {
  Gemm g;
  int nsplit = 0;
  const float* part = nullptr;
};
hipError_t gemm(const Gemm& g, float* scratch, hipStream_t s, GemmFinish* defer = nullptr);

// The DSTDGC aggregation products per sample n (model/dstdgcn.py:87 / :93),
// NCTV operands with channel stride T*V and per-sample strides fs / ys / dys /
// dfs; (a, i) = (t, v) for the spatial op, (v, t) for the temporal one;
// D [B][A][NN][NN] (A = T, NN = V spatial; A = V, NN = T temporal):
//   agg_fwd  y[c][(a,j)] (beta 0: = / 1: +=) sum_i F[c][(a,i)] D[a][i][j]
//   agg_bwd  dF[c][(a,i)] = sum_j dy[c][(a,j)] D[a][i][j]
//            dD[a][i][j] = sum_c F[c][(a,i)] dy[c][(a,j)]
// agg_bwd reports how dD was produced in *nparts: 1 -- in dD; k > 1 -- as k
// channel-chunk partials dDpart[p][B][A][NN][NN] (dDpart >= agg_parts(C) *
// B*A*NN*NN floats; pass them to adj_bwd); 0 -- not at all (the a-chunk
// kernel does not fit: the caller's strided GEMM).  hipErrorNotSupported (nothing launched)
// outside C <= 64, NN <= 64: the caller runs the strided GEMMs instead.
hipError_t agg_fwd(const float* F, long long fs, const float* D, float* y, long long ys, float beta, int B, int C,
                   int T, int V, int temporal, hipStream_t s);
hipError_t agg_bwd(const float* F, long long fs, const float* dy, long long dys, const float* D, float* dF,
                   long long dfs, float* dD, int B, int C, int T, int V, int temporal, hipStream_t s, float* dDpart,
                   int* nparts);
inline int agg_parts(int C) { return (C + 15) / 16; }

// P / Q element (n, r, a, i) lives at n*sn + r*sr + a*sa + i*si.
struct PQView {
  long long sn, sr, sa, si;
};

// M[n][r*A + a][i][j] = tanh(P(n,r,a,i) - Q(n,r,a,j)), r < R (red_channels).
hipError_t tanh_outer_fwd(const float* P, const float* Q, PQView v, int B, int R, int A, int NN, float* M,
                          hipStream_t s);
// dZ = dM * (1 - M^2);  dP(n,r,a,i) = sum_j dZ;  dQ(n,r,a,j) = -sum_i dZ.
hipError_t tanh_outer_bwd(const float* M, const float* dM, PQView v, int B, int R, int A, int NN, float* dP,
                          float* dQ, hipStream_t s);

// Backward of adj_combine + the conv_rm bias, fused: dD -> dE = alpha * dD in
// place, and dalpha += <dD, E>, dA[ij] += sum_{n,a} dD, dbrm[a] += sum_{n,ij} dE.
// scratch >= adj_bwd_scratch_floats(B, A, NN2).
size_t adj_bwd_scratch_floats(int B, int A, int NN2);
// assign_dA: dA (=) instead of (+=).  nparts > 1: dD is the fixed-order sum
// of the partials dDpart[p][B][A][NN2] (agg_bwd), dE written to dD.
// dW2 / Amul (optional): also dW2 += dA * Amul element-wise (the spatial
// adjacency's dW_s = dA * A_s, with dA itself accumulated into dR_s)
hipError_t adj_bwd(float* dD, const float* E, const float* alpha, int B, int A, int NN2, float* dA, float* dbrm,
                   float* dalpha, float* scratch, hipStream_t s, int assign_dA = 0, const float* dDpart = nullptr,
                   int nparts = 1, float* dW2 = nullptr, const float* Amul = nullptr);
// The same in two launches the caller can put on different streams: the
// part (dE in place, the partials in scratch) and the finish (dA, dbrm,
// dalpha, dW2 from the partials -- parameter gradients only, which nothing
// later in the backward reads).
hipError_t adj_bwd_part(float* dD, const float* E, const float* alpha, int B, int A, int NN2, float* scratch,
                        hipStream_t s, const float* dDpart, int nparts);
hipError_t adj_bwd_finish(int B, int A, int NN2, float* dA, float* dbrm, float* dalpha, const float* scratch,
                          hipStream_t s, int assign_dA, float* dW2, const float* Amul);
// One launch for an op's weight-gradient finishes (the model backward's
// second stream): the adjacency-backward finish above and up to two deferred
// split-K GEMM finishes (f0 / f1: null or nsplit 0 for none), each with the
// arithmetic of its own launch.
hipError_t finish_set(int B, int A, int NN2, float* dA, float* dbrm, float* dalpha, const float* adj_scratch,
                      int assign_dA, float* dW2, const float* Amul, const GemmFinish* f0, const GemmFinish* f1,
                      hipStream_t s);

// Batched strided 2-D copies in one launch: dst[r*dst_ld + c] (+)= src[r*src_ld + c].
struct CopyJob {
  const float* src;
  float* dst;
  int rows, cols, src_ld, dst_ld, accumulate;
};
constexpr int kMaxCopyJobs = 64;
struct CopyJobs {
  int n = 0;
  CopyJob j[kMaxCopyJobs];
  bool add(const float* src, float* dst, int rows, int cols, int src_ld, int dst_ld, int accumulate) {
    if (n >= kMaxCopyJobs) return false;
    j[n++] = CopyJob{src, dst, rows, cols, src_ld, dst_ld, accumulate};
    return true;
  }
};
hipError_t copy_jobs(const CopyJobs& js, hipStream_t s);
// dR_s += dA; dW_s += dA * A_s   (both graphs, n = 2*V*V)
hipError_t adj_param_grads(const float* dA, const float* A_s, float* dR_s, float* dW_s, size_t n, hipStream_t s);

// x[i] *= alpha (device scalar)
hipError_t scale_by(float* x, const float* alpha, size_t n, hipStream_t s);

// out[m] += scale * sum_{b < nb} sum_{j < nj} X[b*sb + m*sm + j*sj], m < M.
// scratch >= reduce_scratch_floats(M).
size_t reduce_scratch_floats(int M);
hipError_t reduce_rows(const float* X, int M, int nb, int nj, long long sb, long long sm, long long sj, float* out,
                       float scale, float* scratch, hipStream_t s);

// out[0] += sum_i x[i] * y[i]   (two-stage, deterministic; partials >= dot_partials())
int dot_partials();
hipError_t dot(const float* x, const float* y, size_t n, float* out, float* partials, hipStream_t s);

// out (+)= a (* b when b != null) (+ c when c != null); assign: '=' instead of '+='
hipError_t acc_mul(const float* a, const float* b, float* out, size_t n, hipStream_t s, const float* c = nullptr,
                   int assign = 0);

// Train-mode BatchNorm over an NCTV tensor, channel (c, v), statistics over
// (n, t) (reference model/dstdgcn.py:35-50, nn.BatchNorm1d semantics):
//   u = x (+ x2)                     x2: optional pre-add (encoder identity residual)
//   z = (u - mean) * rstd * gamma + beta (+ res)
//   out = prelu ? PReLU(z) : z       (z kept in zsave when prelu is set)
// mean / rstd ([C*V], index c*V + v) are saved for the backward; running
// stats are updated with `momentum` and the unbiased variance when
// running_mean != null.
// SyncBN (dstd_bn_sync, include/dstd_gcn_train.h): a collective that failed
// surfaces as DSTD_ECOLLECTIVE through the hipError_t paths (the C entry
// points return (int)error; -5 is outside hipError_t's own range, hence the
// representation copy instead of a cast)
static_assert(sizeof(hipError_t) == sizeof(int), "hipError_t carries the DSTD error code");
inline hipError_t collective_failed() {
  const int v = DSTD_ECOLLECTIVE;
  hipError_t e;
  __builtin_memcpy(&e, &v, sizeof e);
  return e;
}
struct BnFwd {
  const float* x;
  const float* x2 = nullptr;
  const float* res = nullptr;
  const float* gamma;
  const float* beta;
  float* running_mean = nullptr;
  float* running_var = nullptr;
  float momentum = 0.1f, eps = 1e-5f;
  const float* prelu = nullptr;
  float* out;
  float* zsave = nullptr;
  float* mean;
  float* rstd;
  int use_running = 0;  // eval-mode BN: mean / rstd from the running stats, no update
  int cv = 0;           // (set by bn_train_fwd: C * V)
  // groups > 1: the batch is `groups` independent BN batches of B / groups
  // samples (statistics per group; the running statistics take the groups'
  // updates in order; mean / rstd hold groups x C*V) -- the engine's forward
  // of a batch and of its time reversal as ONE launch sequence
  int groups = 1;
  // cross-rank statistics (null: this rank's batch only); gath / world are
  // set by bn_train_fwd from it: every rank's (mean, M2, count) per group
  const dstd_bn_sync* sync = nullptr;
  const float* gath = nullptr;
  int world = 1;
};
hipError_t bn_train_fwd(const BnFwd& a, int B, int C, int T, int V, float* scratch, hipStream_t s);

// Backward of BnFwd.  dout is d(out); with prelu set it is first mapped
// through PReLU' using zsave.  Writes du = d(u) (=), dz_out = dz (= , when
// non-null: the residual branch's gradient), accumulates dgamma, dbeta and,
// with prelu set, the slope gradient into *dprelu.
struct BnBwd {
  const float* x;
  const float* x2 = nullptr;
  const float* zsave = nullptr;
  const float* prelu = nullptr;
  const float* dout;
  const float* mean;
  const float* rstd;
  const float* gamma;
  float* du;
  float* dz_out = nullptr;
  const float* dz_add = nullptr;  // dz_out = dz + dz_add (an identity path's gradient joined in the same pass)
  float* dgamma;
  float* dbeta;
  int use_running = 0;  // mean / rstd are constants (eval-mode BN): du = gamma * rstd * dz
  int groups = 1;       // as BnFwd::groups (the forward's grouping)
  // cross-rank sums (null: this rank's); gsum is set by bn_train_bwd from it:
  // the all-reduced [groups][C*V][2] (sum dz, sum dz*xhat), then the groups' row counts
  const dstd_bn_sync* sync = nullptr;
  const float* gsum = nullptr;
};
// scratch (both directions) >= bn_scratch_floats(B, C, T, V) (any groups)
size_t bn_scratch_floats(int B, int C, int T, int V);
hipError_t bn_train_bwd(const BnBwd& a, int B, int C, int T, int V, float* scratch, float* dprelu, hipStream_t s);

// out[0] += sum_{i < n} partial[i]
hipError_t sum_into(const float* partial, int n, float* out, hipStream_t s);

// Model boundary in NCTV: X0[n][c][t][v] = c < C ? x[n][t][v][c] : x[n][t][v][c-C] - x[n][T-1][v][c-C]
hipError_t prep_nctv(const float* x, int B, int T, int V, int C, float* X0, hipStream_t s);
// y[n][t][v][c] = O[n][c][t][v] + x[n][T-1][v][c]
hipError_t out_ntvc(const float* O, const float* x, int B, int T, int V, int C, float* y, hipStream_t s);
// Input gradient of the model boundary (prep_nctv and the output residual
// y += x[:, T-1], model/dstdgcn.py:298-303, 315): dX0 [B][2C][T][V], dy
// [B][T][V][C] -> dx [B][T][V][C] (=):  dx[t] = dX0[c][t] + dX0[C+c][t], and
// dx[T-1] += sum_t (dy[t] - dX0[C+c][t]).
hipError_t prep_nctv_bwd(const float* dX0, const float* dy, int B, int T, int V, int C, float* dx, hipStream_t s);
// dO[n][c][t][v] = dy[n][t][v][c]
hipError_t out_ntvc_bwd(const float* dy, int B, int T, int V, int C, float* dO, hipStream_t s);

// Inverted dropout with a counter-based hash mask: out[i] = keep(seed, i) ? in[i] / (1 - p) : 0.
// Applying it to the upstream gradient with the same seed is the backward.
// seed_on_device: `seed` is the address of a device uint64 holding the seed
hipError_t dropout(const float* in, float* out, size_t n, float p, unsigned long long seed, hipStream_t s,
                   bool seed_on_device = false);

// mpjpe_error_3d (engine/utils/loss.py:52-65): loss = mean_k ||p_k - q_k||_2
// over K = n / 3 points.  fwd: out[0] (=); bwd: dp = g * (p - q) / ||p - q|| / K
// with g = *gscale (device scalar).
int mpjpe_partials();
hipError_t mpjpe_fwd(const float* p, const float* q, size_t npts, float* out, float* partials, hipStream_t s);
hipError_t mpjpe_bwd(const float* p, const float* q, size_t npts, const float* gscale, float scale, float* dp,
                     hipStream_t s);
// Per-frame test metric (engine/prediction.py:366-404) without host syncs.
// all_seqs [B][T][D] (D = 3J), outputs [B][T - t_out0][n_used] fill frames
// t_out0.. of the dims with used_pos[d] >= 0; joint j reads the filled value
// of joint joint_src[j] (the ignore <- equal copy).  For each k:
// sums[k] += (1/J) * sum_{n, j} ||all_seqs - pred|| at frame frames[k].
hipError_t frame_mpjpe(const float* all_seqs, const float* outputs, int B, int T, int D, int t_out0,
                       const int* used_pos, int n_used, const int* joint_src, const int* frames, int n_frames,
                       float* sums, hipStream_t s);

}  // namespace train
}  // namespace dstd
