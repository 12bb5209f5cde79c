// C ABI of the training path (include/dstd_gcn_train.h): saved-buffer and
// workspace carving plus the launch sequences of the train-mode forward and
// the backward of DSTDGC / DSTDGCB / DSTDGCN, and the engine's loss / metric.
//
// Index conventions shared by both DSTDGC modes ("rows" a = the adjacency
// index, "nodes" i, j = what the adjacency mixes):
//   spatial  (model/dstdgcn.py:83-87): a = t (A = T rows), i = v (NN = V)
//   temporal (model/dstdgcn.py:88-93): a = v (A = V rows), i = t (NN = T)
// An NCTV activation X[n][c][t][v] is addressed as n*C*TV + c*TV + a*ps_a +
// i*ps_i with (ps_a, ps_i) = (V, 1) spatial and (1, V) temporal, so every
// step below is one strided GEMM or element-wise kernel for either mode.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <initializer_list>
#include <mutex>
#include <vector>

#include "../../include/dstd_gcn_train.h"
#include "dstd_common.h"
#include "dstd_train.h"

using namespace dstd::train;

namespace {

constexpr int kMaxT = 128;  // same envelope as the forward (dstd_capi.hip)
constexpr int kMaxV = 32;
constexpr int kMaxC = 64;
constexpr int kMaxRed = 8;  // red_channels of one DSTDGC (P / Q channels each)
constexpr unsigned kTrainFlags = DSTD_TRAIN_RUNNING_STATS | DSTD_TRAIN_PAIRED;
constexpr unsigned kModelTrainFlags = kTrainFlags | DSTD_TRAIN_SEED_DEVICE | DSTD_TRAIN_ONE_STREAM;

struct Carver {
  char* base;
  size_t off = 0;
  float* take(size_t nfloats) {
    off = (off + 255) & ~size_t(255);
    float* p = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += nfloats * sizeof(float);
    return p;
  }
};

#define DSTD_TRY(expr)                    \
  do {                                    \
    hipError_t _e = (expr);               \
    if (_e != hipSuccess) return (int)_e; \
  } while (0)

#define DSTD_TRYH(expr)                  \
  do {                                   \
    hipError_t _e = (expr);              \
    if (_e != hipSuccess) return _e;     \
  } while (0)

bool shape_ok(int B, int T, int V) { return B > 0 && T > 1 && V > 0 && T <= kMaxT && V <= kMaxV; }
bool ch_ok(int c) { return c >= 1 && c <= kMaxC; }
bool gc_ok(const dstd_gc_weights* w) {
  return w && w->wf && w->bf && w->wm1 && w->bm1 && w->wm2 && w->bm2 && w->wrm && w->brm;
}
bool gg_ok(const dstd_gc_grads* g) {
  return g && g->wf && g->bf && g->wm1 && g->bm1 && g->wm2 && g->bm2 && g->wrm && g->brm;
}
bool bn_ok(const dstd_bn& b) { return b.weight && b.bias && b.running_mean && b.running_var; }
bool bng_ok(const dstd_bn_grads& b) { return b.weight && b.bias; }
bool block_ok(const dstd_block_params* p) {
  if (!p || !p->A_s || !p->W_s || !p->R_s || !p->A_t || !p->R_t || !p->alpha_sm || !p->alpha_tm || !p->prelu)
    return false;
  if (!ch_ok(p->cin) || !ch_ok(p->cout)) return false;
  if (!gc_ok(&p->conv_s[0]) || !gc_ok(&p->conv_s[1]) || !gc_ok(&p->conv_t) || !bn_ok(p->bn)) return false;
  if (p->cin != p->cout && (!p->res_w || !p->res_b || !bn_ok(p->res_bn))) return false;
  return true;
}
bool block_grads_ok(const dstd_block_params* p, const dstd_block_grads* g) {
  if (!g || !g->W_s || !g->R_s || !g->R_t || !g->alpha_sm || !g->alpha_tm || !g->prelu) return false;
  if (!gg_ok(&g->conv_s[0]) || !gg_ok(&g->conv_s[1]) || !gg_ok(&g->conv_t) || !bng_ok(g->bn)) return false;
  if (p->cin != p->cout && (!g->res_w || !g->res_b || !bng_ok(g->res_bn))) return false;
  return true;
}
bool model_ok(const dstd_model_params* p) {
  if (!p || p->num_layers < 0 || p->num_layers > DSTD_MAX_LAYERS || p->in_channels != 6) return false;
  if (!block_ok(&p->st_in) || !bn_ok(p->bn_in) || !p->prelu || !block_ok(&p->st_out)) return false;
  for (int i = 0; i < p->num_layers; ++i)
    if (!block_ok(&p->enc[i]) || !bn_ok(p->enc_bn[i]) || !p->enc_prelu[i]) return false;
  return true;
}

// ---------------------------------------------------------------------------
// one DSTDGC
// ---------------------------------------------------------------------------
// The aggregation products run on the slab kernels (agg_fwd / agg_bwd); the
// strided GEMMs take the shapes those do not support.
struct OpGeom {
  int B, cin, cout, T, V, TV;
  int R;  // red_channels: P / Q channels per op (2 in every block of the reference)
  int A, NN, NN2;
  long long ps_a, ps_i;
  int temporal;
  OpGeom(int mode, int B_, int cin_, int cout_, int T_, int V_, int R_ = 2)
      : B(B_), cin(cin_), cout(cout_), T(T_), V(V_), TV(T_ * V_), R(R_) {
    const bool sp = mode == DSTD_MODE_SPATIAL;
    A = sp ? T : V;
    NN = sp ? V : T;
    NN2 = NN * NN;
    ps_a = sp ? V : 1;
    ps_i = sp ? 1 : V;
    temporal = !sp;
  }
  int CG() const { return cout + 2 * R; }  // rows of the packed conv output G = [F; P; Q]
  // P (Q) rows of G: element (n, r, a, i) at n*CG*TV + r*TV + a*ps_a + i*ps_i
  PQView pq() const { return PQView{(long long)CG() * TV, (long long)TV, ps_a, ps_i}; }
};

// Saved state of one train-mode DSTDGC.  conv_f / conv_m1 / conv_m2 run as ONE
// GEMM with the packed weights Wp = [W_f; W_m1; W_m2] ([cout+4][cin]) into
// G = [F; P; Q] ([B][cout+4][T*V]); M, E, D as in the forward (§3.2).
struct OpSaved {
  float *Wp, *bp, *G, *M, *E, *D;
};
void carve_op_saved(Carver& cv, OpSaved& s, const OpGeom& g) {
  s.Wp = cv.take((size_t)g.CG() * g.cin);
  s.bp = cv.take(g.CG());
  s.G = cv.take((size_t)g.B * g.CG() * g.TV);
  s.M = cv.take((size_t)g.B * g.R * g.A * g.NN2);
  s.E = cv.take((size_t)g.B * g.A * g.NN2);
  s.D = cv.take((size_t)g.B * g.A * g.NN2);
}
// Copy jobs packing one op's conv weights into Wp / bp.
bool pack_jobs(CopyJobs& js, const dstd_gc_weights* w, const OpSaved& sv, const OpGeom& g) {
  const int R = g.R;
  return js.add(w->wf, sv.Wp, g.cout, g.cin, g.cin, g.cin, 0) &&
         js.add(w->wm1, sv.Wp + (size_t)g.cout * g.cin, R, g.cin, g.cin, g.cin, 0) &&
         js.add(w->wm2, sv.Wp + (size_t)(g.cout + R) * g.cin, R, g.cin, g.cin, g.cin, 0) &&
         js.add(w->bf, sv.bp, 1, g.cout, g.cout, g.cout, 0) && js.add(w->bm1, sv.bp + g.cout, 1, R, R, R, 0) &&
         js.add(w->bm2, sv.bp + g.cout + R, 1, R, R, R, 0);
}

struct OpWs {
  float *dG, *dD, *dM, *gW, *gs, *part, *red;
  float* dDp;  // channel-chunk partials of dD (agg_bwd), null when one chunk suffices
  // the second dG / dD set and the GEMM scratch of the weight-gradient stream
  // (WgradStream): consecutive ops alternate sets so that an op's weight
  // gradients can still read its dE / dG while the next op runs; adjp: the
  // adjacency backward's partials per set (its finish runs on that stream)
  float *dG2, *dD2, *gs2;
  float* adjp[2];
  float* gs3;  // the dW_rm reduction's partials (its finish waits for dWp's: finish_set)
};

// ---------------------------------------------------------------------------
// Weight-gradient stream of the model backward.  An op's two weight-gradient
// reductions -- dW_rm (reads dE, M) and [dW_f | dW_m1 | dW_m2 | db] (reads
// dG, x) -- feed nothing later in the backward, so they run on a second HIP
// stream, forked from the caller's stream by events, while the caller's
// stream goes on with the input-gradient chain (dM, tanh', dx and the next
// op).  Their 256..1152-workgroup launches leave most CUs idle at the
// config-5 batch (one workgroup per CU), which the two chains now share.
// Everything joins back into the caller's stream before the backward returns
// (also inside a HIP graph capture: the fork / join events pull the second
// stream into the capture).  Results are bit-identical to the one-stream
// order: every reduction keeps its own fixed order and no two concurrent
// kernels write the same memory.
// ---------------------------------------------------------------------------
struct WgradRes {
  int dev = -1;
  bool busy = false;  // held by a backward call (host side)
  hipStream_t st = nullptr;
  hipEvent_t fork, done[2], join;
};
// A free set of the current device's (created on first use -- in practice by
// an eager warm-up step, not inside a graph capture); concurrent host threads
// get different sets, consecutive calls share one.
std::mutex g_wgrad_mu;
WgradRes* wgrad_acquire() {
#ifdef DSTD_TRAIN_NO_WGRAD_STREAM
  return nullptr;
#else
  static std::vector<WgradRes*> pool;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_wgrad_mu);
  for (WgradRes* r : pool)
    if (r->dev == dev && !r->busy) {
      r->busy = true;
      return r;
    }
  WgradRes* r = new WgradRes;
  r->dev = dev;
  bool ok = hipStreamCreateWithFlags(&r->st, hipStreamNonBlocking) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&r->fork, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&r->done[0], hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&r->done[1], hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&r->join, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    (void)hipGetLastError();
    delete r;  // (a partly created set leaks its handles; creation failing means the device is gone)
    return nullptr;
  }
  r->busy = true;
  pool.push_back(r);
  return r;
#endif
}
void wgrad_release(WgradRes* r) {
  if (!r) return;
  std::lock_guard<std::mutex> lk(g_wgrad_mu);
  r->busy = false;
}

// One backward's use of the weight-gradient stream (null res: one stream).
struct Wgrad {
  WgradRes* res = nullptr;
  Wgrad() = default;
  explicit Wgrad(WgradRes* r) : res(r) {}
  // an error return between a fork and the success-path join() must not
  // leave side-stream work unordered before the caller's stream (it still
  // reads the workspace / saved state and writes the gradient arena), nor a
  // graph capture unjoined: the destructor joins whatever was forked
  ~Wgrad() {
    if (res && any) (void)join();
    wgrad_release(res);
  }
  Wgrad(const Wgrad&) = delete;
  Wgrad& operator=(const Wgrad&) = delete;
  hipStream_t main = nullptr;
  int next = 0;
  bool used[2] = {false, false};
  bool any = false;
  // the dG / dD set of the next op (waits until the op two back has released it)
  hipError_t take(const OpWs& w, float*& dG, float*& dD, int& slot) {
    if (!res) {
      dG = w.dG, dD = w.dD, slot = 0;
      return hipSuccess;
    }
    slot = next;
    next ^= 1;
    dG = slot ? w.dG2 : w.dG;
    dD = slot ? w.dD2 : w.dD;
    if (used[slot]) return hipStreamWaitEvent(main, res->done[slot], 0);
    return hipSuccess;
  }
  // the side stream continues after everything enqueued on main so far
  hipError_t fork() {
    any = true;  // from here on the side stream may hold work to join
    DSTD_TRYH(hipEventRecord(res->fork, main));
    return hipStreamWaitEvent(res->st, res->fork, 0);
  }
  hipError_t release(int slot) {
    used[slot] = any = true;
    return hipEventRecord(res->done[slot], res->st);
  }
  hipError_t join() {
    if (!res || !any) return hipSuccess;
    any = false;
    DSTD_TRYH(hipEventRecord(res->join, res->st));
    return hipStreamWaitEvent(main, res->join, 0);
  }
};
// Reduction / BatchNorm / adjacency-backward scratch for a geometry.
size_t red_floats(const OpGeom& g) {
  return std::max(std::max(reduce_scratch_floats(std::max(std::max(g.NN2, g.CG()), std::max(g.A, g.cin))),
                           bn_scratch_floats(g.B, std::max(g.cin, g.cout), g.T, g.V)),
                  adj_bwd_scratch_floats(g.B, g.A, g.NN2));
}
// Sized for the largest of the given op geometries (one workspace serves every
// op of a block / model in turn).
void carve_op_ws(Carver& cv, OpWs& w, const std::vector<OpGeom>& gl) {
  size_t nG = 0, nD = 0, nM = 0, nW = 0, nmn = 0, nred = 0, nDp = 0, nadj = 0;
  for (const OpGeom& g : gl) {
    nadj = std::max(nadj, adj_bwd_scratch_floats(g.B, g.A, g.NN2));
    nG = std::max(nG, (size_t)g.B * g.CG() * g.TV);
    nD = std::max(nD, (size_t)g.B * g.A * g.NN2);
    if (agg_parts(g.cout) > 1) nDp = std::max(nDp, (size_t)agg_parts(g.cout) * g.B * g.A * g.NN2);
    nM = std::max(nM, (size_t)g.B * g.R * g.A * g.NN2);
    nW = std::max(nW, (size_t)g.CG() * (g.cin + 1));
    nmn = std::max(nmn, (size_t)std::max(std::max(g.CG() * (g.cin + 1), g.R * g.A * g.A), g.cout * g.cin));
    nred = std::max(nred, red_floats(g));
  }
  w.dG = cv.take(nG);
  w.dD = cv.take(nD);
  w.dM = cv.take(nM);
  w.gW = cv.take(nW);
  w.gs = cv.take(gemm_scratch_floats((int)nmn, 1));
  w.part = cv.take(std::max(dot_partials(), mpjpe_partials()));
  w.red = cv.take(nred);
  w.dDp = nDp ? cv.take(nDp) : nullptr;
  w.dG2 = cv.take(nG);
  w.dD2 = cv.take(nD);
  w.gs2 = cv.take(gemm_scratch_floats((int)nmn, 1));
  w.adjp[0] = cv.take(nadj);
  w.adjp[1] = cv.take(nadj);
  w.gs3 = cv.take(gemm_scratch_floats((int)nmn, 1));
}

// 1x1 conv as GEMMs over NCTV (W [cout][cin]).
Gemm conv_fwd(const float* W, const float* bias, const float* X, float* Y, int B, int cin, int cout, int TV) {
  Gemm g;
  g.M = cout, g.N = TV, g.K = cin, g.nb1 = B;
  g.A = W, g.a_m = cin, g.a_k = 1;
  g.B = X, g.b_b1 = (long long)cin * TV, g.b_k = TV, g.b_n = 1;
  g.C = Y, g.c_b1 = (long long)cout * TV, g.c_m = TV, g.c_n = 1;
  g.bias_m = bias;
  return g;
}
Gemm conv_dx(const float* W, const float* dY, float* dX, int B, int cin, int cout, int TV) {
  Gemm g;
  g.M = cin, g.N = TV, g.K = cout, g.nb1 = B;
  g.A = W, g.a_m = 1, g.a_k = cin;
  g.B = dY, g.b_b1 = (long long)cout * TV, g.b_k = TV, g.b_n = 1;
  g.C = dX, g.c_b1 = (long long)cin * TV, g.c_m = TV, g.c_n = 1;
  g.beta = 1.f;
  return g;
}
Gemm conv_dw(const float* dY, const float* X, float* dW, int B, int cin, int cout, int TV) {
  Gemm g;
  g.M = cout, g.N = cin, g.K = TV, g.nb1 = B, g.reduce = 1;
  g.A = dY, g.a_b1 = (long long)cout * TV, g.a_m = TV, g.a_k = 1;
  g.B = X, g.b_b1 = (long long)cin * TV, g.b_k = 1, g.b_n = TV;
  g.C = dW, g.c_m = cin, g.c_n = 1;
  g.beta = 1.f;
  return g;
}
hipError_t conv_bwd(const float* W, const float* X, const float* dY, float* dX, float* dW, float* db, int B, int cin,
                    int cout, int TV, float* gs, hipStream_t s, float dx_beta = 1.f) {
  if (dX) {
    Gemm gx = conv_dx(W, dY, dX, B, cin, cout, TV);
    gx.beta = dx_beta;
    DSTD_TRYH(gemm(gx, gs, s));
  }
  // [dW | db] = sum dY [X; 1]^T in one reduce GEMM (the bias as the ones
  // column), accumulated into the parameters' gradients
  Gemm gw = conv_dw(dY, X, dW, B, cin + 1, cout, TV);
  gw.b_ones_last = 1;
  gw.b_b1 = (long long)cin * TV;
  gw.nseg = 1;
  gw.seg[0] = Gemm::Seg{0, cout, dW, db};
  return gemm(gw, gs, s);
}

// y (beta_y: 0 '=' / 1 '+=') = DSTDGC(x, Acomb, alpha); fills sv.  The packed
// weights sv.Wp / sv.bp must already hold the op's conv weights (pack_jobs).
// Acomb = A0 (* W0) (+ R0), formed by the conv_rm GEMM's epilogue (W0, R0 may be null).
// op_fwd in two parts: op_fwd_adj (the packed conv, M, E and D: everything up
// to the adjacency) and op_fwd_agg (the aggregation into y), so that a
// block's second spatial op can build its adjacency on another stream while
// the first runs (block_fwd)
hipError_t op_fwd_adj(const OpGeom& g, const float* x, const dstd_gc_weights* w, const float* A0, const float* W0,
                      const float* R0, const float* alpha, const OpSaved& sv, hipStream_t s) {
  // conv_f, conv_m1, conv_m2 in one GEMM                         :81-82
  DSTD_TRYH(gemm(conv_fwd(sv.Wp, sv.bp, x, sv.G, g.B, g.cin, g.CG(), g.TV), nullptr, s));
  const float* P = sv.G + (size_t)g.cout * g.TV;
  const float* Q = P + (size_t)g.R * g.TV;
  DSTD_TRYH(tanh_outer_fwd(P, Q, g.pq(), g.B, g.R, g.A, g.NN, sv.M, s));                   // :84 / :90
  Gemm e;  // E = conv_rm(M): [A x RA] . [RA x NN^2] + b_rm           :85 / :91
  e.M = g.A, e.N = g.NN2, e.K = g.R * g.A, e.nb1 = g.B;
  e.A = w->wrm, e.a_m = g.R * g.A, e.a_k = 1;
  e.B = sv.M, e.b_b1 = (long long)g.R * g.A * g.NN2, e.b_k = g.NN2, e.b_n = 1;
  e.C = sv.E, e.c_b1 = (long long)g.A * g.NN2, e.c_m = g.NN2, e.c_n = 1;
  e.bias_m = w->brm;
  e.d_out = sv.D;  // D = alpha * E + Acomb                          :86 / :92
  e.d_alpha = alpha;
  e.d_A = A0;
  e.d_W = W0;
  e.d_R = R0;
  return gemm(e, nullptr, s);
}
hipError_t op_fwd_agg(const OpGeom& g, float* y, float beta_y, const OpSaved& sv, hipStream_t s) {
  {  // y[c][(a,j)] = sum_i F[c][(a,i)] D[a][i][j]     :87 / :93
    const hipError_t e = agg_fwd(sv.G, (long long)g.CG() * g.TV, sv.D, y, (long long)g.cout * g.TV, beta_y, g.B,
                                 g.cout, g.T, g.V, g.temporal, s);
    if (e != hipErrorNotSupported) return e;
  }
  Gemm a;  // y[c][j] = sum_i F[c][i] D[i][j] per (n, a)               :87 / :93
  a.M = g.cout, a.N = g.NN, a.K = g.NN, a.nb1 = g.B, a.nb2 = g.A;
  a.A = sv.G, a.a_b1 = (long long)g.CG() * g.TV, a.a_b2 = g.ps_a, a.a_m = g.TV, a.a_k = g.ps_i;
  a.B = sv.D, a.b_b1 = (long long)g.A * g.NN2, a.b_b2 = g.NN2, a.b_k = g.NN, a.b_n = 1;
  a.C = y, a.c_b1 = (long long)g.cout * g.TV, a.c_b2 = g.ps_a, a.c_m = g.TV, a.c_n = g.ps_i;
  a.beta = beta_y;
  return gemm(a, nullptr, s);
}
hipError_t op_fwd(const OpGeom& g, const float* x, const dstd_gc_weights* w, const float* A0, const float* W0,
                  const float* R0, const float* alpha, float* y, float beta_y, const OpSaved& sv, hipStream_t s) {
  DSTD_TRYH(op_fwd_adj(g, x, w, A0, W0, R0, alpha, sv, s));
  return op_fwd_agg(g, y, beta_y, sv, s);
}

// dx_beta 0: dx (=) instead of (+=); assign_dA: dA likewise (block-internal
// buffers; the op entry point accumulates both)
hipError_t op_bwd(const OpGeom& g, const float* x, const dstd_gc_weights* w, const float* alpha, const OpSaved& sv,
                  const float* dy, float* dx, const dstd_gc_grads* gr, float* dA, float* dalpha, const OpWs& ws0,
                  hipStream_t s, float dx_beta = 1.f, int assign_dA = 0, Wgrad* wg = nullptr,
                  float* dW2 = nullptr, const float* Amul = nullptr) {
  const long long ldG = (long long)g.CG() * g.TV;
  OpWs ws = ws0;
  int slot = 0;
  Wgrad none;
  if (!wg) wg = &none;
  wg->main = s;
  DSTD_TRYH(wg->take(ws0, ws.dG, ws.dD, slot));
  // the weight-gradient reductions' stream and scratch
  const hipStream_t ws_s = wg->res ? wg->res->st : s;
  float* const ws_gs = wg->res ? ws.gs2 : ws.gs;
  // dF -> rows [0, cout) of dG; dD in place or as channel-chunk partials
  int nparts = 0;
  const hipError_t ae = agg_bwd(sv.G, ldG, dy, (long long)g.cout * g.TV, sv.D, ws.dG, ldG, ws.dD, g.B, g.cout, g.T, g.V,
                 g.temporal, s, ws.dDp, &nparts);
  if (ae != hipErrorNotSupported) DSTD_TRYH(ae);
  if (ae == hipErrorNotSupported) {
    Gemm f;  // dF[c][i] = sum_j dy[c][j] D[i][j]  -> rows [0, cout) of dG
    f.M = g.cout, f.N = g.NN, f.K = g.NN, f.nb1 = g.B, f.nb2 = g.A;
    f.A = dy, f.a_b1 = (long long)g.cout * g.TV, f.a_b2 = g.ps_a, f.a_m = g.TV, f.a_k = g.ps_i;
    f.B = sv.D, f.b_b1 = (long long)g.A * g.NN2, f.b_b2 = g.NN2, f.b_k = 1, f.b_n = g.NN;
    f.C = ws.dG, f.c_b1 = ldG, f.c_b2 = g.ps_a, f.c_m = g.TV, f.c_n = g.ps_i;
    DSTD_TRYH(gemm(f, nullptr, s));
  }
  if (nparts == 0) {
    Gemm d;  // dD[i][j] = sum_c F[c][i] dy[c][j]
    d.M = g.NN, d.N = g.NN, d.K = g.cout, d.nb1 = g.B, d.nb2 = g.A;
    d.A = sv.G, d.a_b1 = ldG, d.a_b2 = g.ps_a, d.a_m = g.ps_i, d.a_k = g.TV;
    d.B = dy, d.b_b1 = (long long)g.cout * g.TV, d.b_b2 = g.ps_a, d.b_k = g.TV, d.b_n = g.ps_i;
    d.C = ws.dD, d.c_b1 = (long long)g.A * g.NN2, d.c_b2 = g.NN2, d.c_m = g.NN, d.c_n = 1;
    DSTD_TRYH(gemm(d, nullptr, s));
    nparts = 1;
  }
  // Adj = alpha * (conv_rm(M)) + A:  dE = alpha dD in place (main stream);
  // dalpha, dA, d b_rm from the partials -- parameter gradients only, so on
  // the weight-gradient stream when there is one (B=32 step: 21 finishes off
  // the critical path), with the partials in the op's set
#ifndef DSTD_ADJ_FINISH_MAIN  // (A/B: 1 = the finish on the caller's stream, before the fork)
#define DSTD_ADJ_FINISH_MAIN 0
#endif
  // With the weight-gradient stream, this finish and the two reductions'
  // split-K finishes below run as ONE launch after dWp's reduction
  // (finish_set: 2 launches per op fewer; dW_rm's partials in gs3)
  float* const adjs = wg->res ? ws0.adjp[slot] : ws.red;
  DSTD_TRYH(adj_bwd_part(ws.dD, sv.E, alpha, g.B, g.A, g.NN2, adjs, s, ws.dDp, nparts));
  if (DSTD_ADJ_FINISH_MAIN || !wg->res)
    DSTD_TRYH(adj_bwd_finish(g.B, g.A, g.NN2, dA, gr->brm, dalpha, adjs, s, assign_dA, dW2, Amul));
  if (wg->res) DSTD_TRYH(wg->fork());
#ifndef DSTD_FINISH_SET  // (A/B: 0 = the three finishes as launches of their own on the side stream)
#define DSTD_FINISH_SET 1
#endif
  GemmFinish wrf, gwf;
  const bool fset = wg->res && !DSTD_ADJ_FINISH_MAIN && DSTD_FINISH_SET;
  if (wg->res && !DSTD_ADJ_FINISH_MAIN && !fset)
    DSTD_TRYH(adj_bwd_finish(g.B, g.A, g.NN2, dA, gr->brm, dalpha, adjs, ws_s, assign_dA, dW2, Amul));
  const float* dE = ws.dD;
  Gemm wr;  // dWrm[a][k] = sum_{n,ij} dE[n][a][ij] M[n][k][ij]
  wr.M = g.A, wr.N = g.R * g.A, wr.K = g.NN2, wr.nb1 = g.B, wr.reduce = 1;
  wr.A = dE, wr.a_b1 = (long long)g.A * g.NN2, wr.a_m = g.NN2, wr.a_k = 1;
  wr.B = sv.M, wr.b_b1 = (long long)g.R * g.A * g.NN2, wr.b_k = 1, wr.b_n = g.NN2;
  wr.C = gr->wrm, wr.c_m = g.R * g.A, wr.c_n = 1;
  wr.beta = 1.f;
  DSTD_TRYH(gemm(wr, fset ? ws.gs3 : ws_gs, ws_s, fset ? &wrf : nullptr));
  Gemm dm;  // dM[n][k][ij] = sum_a Wrm[a][k] dE[n][a][ij]
  dm.M = g.R * g.A, dm.N = g.NN2, dm.K = g.A, dm.nb1 = g.B;
  dm.A = w->wrm, dm.a_m = 1, dm.a_k = g.R * g.A;
  dm.B = dE, dm.b_b1 = (long long)g.A * g.NN2, dm.b_k = g.NN2, dm.b_n = 1;
  dm.C = ws.dM, dm.c_b1 = (long long)g.R * g.A * g.NN2, dm.c_m = g.NN2, dm.c_n = 1;
  DSTD_TRYH(gemm(dm, nullptr, s));
  // dP, dQ -> rows [cout, cout + 2R) of dG
  float* dP = ws.dG + (size_t)g.cout * g.TV;
  DSTD_TRYH(tanh_outer_bwd(sv.M, ws.dM, g.pq(), g.B, g.R, g.A, g.NN, dP, dP + (size_t)g.R * g.TV, s));
  // rows [0, cout) / [cout, cout+R) / [cout+R, cout+2R) of [dWp | dbp]
  // accumulate straight into the conv_f / conv_m1 / conv_m2 gradients
  Gemm gw = conv_dw(ws.dG, x, ws.gW, g.B, g.cin + 1, g.CG(), g.TV);
  gw.b_ones_last = 1;
  gw.b_b1 = (long long)g.cin * g.TV;
  gw.nseg = 3;
  gw.seg[0] = Gemm::Seg{0, g.cout, gr->wf, gr->bf};
  gw.seg[1] = Gemm::Seg{g.cout, g.R, gr->wm1, gr->bm1};
  gw.seg[2] = Gemm::Seg{g.cout + g.R, g.R, gr->wm2, gr->bm2};
  if (wg->res) {  // queued before dx, which then runs beside it
    DSTD_TRYH(wg->fork());
    DSTD_TRYH(gemm(gw, ws_gs, ws_s, fset ? &gwf : nullptr));
    if (fset)
      DSTD_TRYH(finish_set(g.B, g.A, g.NN2, dA, gr->brm, dalpha, adjs, assign_dA, dW2, Amul, &wrf, &gwf, ws_s));
    DSTD_TRYH(wg->release(slot));
  }
  // the three 1x1 convs at once: dx += Wp^T dG;  [dWp | dbp] = sum dG [x; 1]^T
  if (dx) {
    Gemm gx = conv_dx(sv.Wp, ws.dG, dx, g.B, g.cin, g.CG(), g.TV);
    gx.beta = dx_beta;
    DSTD_TRYH(gemm(gx, ws.gs, s));
  }
  return wg->res ? hipSuccess : gemm(gw, ws.gs, s);
}

// ---------------------------------------------------------------------------
// one DSTDGCB
// ---------------------------------------------------------------------------
struct BlockSaved {
  OpSaved op[3];
  float *ysp, *z, *h, *mean, *rstd;
  float *rc, *r, *rmean, *rrstd;
  float* red;  // BatchNorm statistics scratch of the forward
};
void carve_block_saved(Carver& cv, BlockSaved& s, int B, int cin, int cout, int T, int V) {
  const size_t act = (size_t)B * cout * T * V;
  for (int i = 0; i < 2; ++i) carve_op_saved(cv, s.op[i], OpGeom(DSTD_MODE_SPATIAL, B, cin, cout, T, V));
  carve_op_saved(cv, s.op[2], OpGeom(DSTD_MODE_TEMPORAL, B, cout, cout, T, V));
  s.ysp = cv.take(act);
  s.z = cv.take(act);
  s.h = cv.take(act);
  s.mean = cv.take(2 * cout * V);  // per BN group (DSTD_TRAIN_PAIRED: 2)
  s.rstd = cv.take(2 * cout * V);
  const bool res = cin != cout;
  s.rc = res ? cv.take(act) : nullptr;
  s.r = res ? cv.take(act) : nullptr;
  s.rmean = res ? cv.take(2 * cout * V) : nullptr;
  s.rrstd = res ? cv.take(2 * cout * V) : nullptr;
  s.red = cv.take(bn_scratch_floats(B, cout, T, V));
}

struct BlockWs {
  OpWs op;
  float *dh, *dysp, *dr, *drc, *pp;
};
struct Chans {
  int cin, cout;
};
// Sized for the largest of the given blocks.
void carve_block_ws(Carver& cv, BlockWs& w, int B, int T, int V, std::initializer_list<Chans> bl) {
  std::vector<OpGeom> gl;
  int cmax = 0;
  bool res = false;
  for (const Chans& c : bl) {
    gl.emplace_back(DSTD_MODE_SPATIAL, B, c.cin, c.cout, T, V);
    gl.emplace_back(DSTD_MODE_TEMPORAL, B, c.cout, c.cout, T, V);
    cmax = std::max(cmax, c.cout);
    res = res || c.cin != c.cout;
  }
  carve_op_ws(cv, w.op, gl);
  const size_t act = (size_t)B * cmax * T * V;
  w.dh = cv.take(act);
  w.dysp = cv.take(act);
  w.dr = cv.take(act);
  w.drc = res ? cv.take(act) : nullptr;
  w.pp = cv.take(cmax);
}

// conv weights of the block's three ops -> packed [W_f; W_m1; W_m2] (18 jobs)
constexpr int kBlockPackJobs = 18;
void pack_block(CopyJobs& js, const dstd_block_params* p, const BlockSaved& S, int B, int T, int V) {
  const OpGeom gs(DSTD_MODE_SPATIAL, B, p->cin, p->cout, T, V);
  const OpGeom gt(DSTD_MODE_TEMPORAL, B, p->cout, p->cout, T, V);
  pack_jobs(js, &p->conv_s[0], S.op[0], gs);
  pack_jobs(js, &p->conv_s[1], S.op[1], gs);
  pack_jobs(js, &p->conv_t, S.op[2], gt);
}

// packed: the caller already packed the block's weights (the model forward
// packs all blocks in two launches)
// side (optional): a second stream of the device (the backward's weight-
// gradient stream set): the second spatial op builds its adjacency there while
// the first runs on s; its aggregation then adds into y on s after the
// first's, so the result is bit-identical to the one-stream order.
hipError_t block_fwd(const dstd_block_params* p, const float* x, int B, int T, int V, float momentum, float* y,
                     const BlockSaved& S, hipStream_t s, int run = 0, const dstd_bn_sync* sync = nullptr,
                     bool packed = false, Wgrad* side = nullptr) {
  const int cin = p->cin, cout = p->cout, TV = T * V;
  const bool res = cin != cout;
  const OpGeom gs(DSTD_MODE_SPATIAL, B, cin, cout, T, V);
  const OpGeom gt(DSTD_MODE_TEMPORAL, B, cout, cout, T, V);
  if (!packed) {
    CopyJobs js;
    pack_block(js, p, S, B, T, V);
    DSTD_TRYH(copy_jobs(js, s));
  }
  // :145-150, A_s*W_s + R_s (:146-149)
  if (side && side->res) {
    side->main = s;
    DSTD_TRYH(side->fork());
    DSTD_TRYH(op_fwd_adj(gs, x, &p->conv_s[1], p->A_s + V * V, p->W_s + V * V, p->R_s + V * V, p->alpha_sm, S.op[1],
                         side->res->st));
    DSTD_TRYH(op_fwd(gs, x, &p->conv_s[0], p->A_s, p->W_s, p->R_s, p->alpha_sm, S.ysp, 0.f, S.op[0], s));
    DSTD_TRYH(side->join());
    DSTD_TRYH(op_fwd_agg(gs, S.ysp, 1.f, S.op[1], s));
  } else {
    for (int i = 0; i < 2; ++i)
      DSTD_TRYH(op_fwd(gs, x, &p->conv_s[i], p->A_s + i * V * V, p->W_s + i * V * V, p->R_s + i * V * V,
                       p->alpha_sm, S.ysp, i ? 1.f : 0.f, S.op[i], s));
  }
  const float* r = x;
  if (res) {  // residual Conv1x1 + BatchNorm (:117-121)
    DSTD_TRYH(gemm(conv_fwd(p->res_w, p->res_b, x, S.rc, B, cin, cout, TV), nullptr, s));
    BnFwd rb;
    rb.x = S.rc;
    rb.gamma = p->res_bn.weight;
    rb.beta = p->res_bn.bias;
    rb.running_mean = const_cast<float*>(p->res_bn.running_mean);
    rb.running_var = const_cast<float*>(p->res_bn.running_var);
    rb.momentum = momentum;
    rb.eps = p->res_bn.eps;
    rb.out = S.r;
    rb.mean = S.rmean;
    rb.rstd = S.rrstd;
    rb.use_running = (run & DSTD_TRAIN_RUNNING_STATS) != 0;
    rb.groups = (run & DSTD_TRAIN_PAIRED) ? 2 : 1;
    rb.sync = sync;
    DSTD_TRYH(bn_train_fwd(rb, B, cout, T, V, S.red, s));
    r = S.r;
  }
  BnFwd bb;  // h = PReLU(BN(y) + r)  (:151-154)
  bb.x = S.ysp;
  bb.res = r;
  bb.gamma = p->bn.weight;
  bb.beta = p->bn.bias;
  bb.running_mean = const_cast<float*>(p->bn.running_mean);
  bb.running_var = const_cast<float*>(p->bn.running_var);
  bb.momentum = momentum;
  bb.eps = p->bn.eps;
  bb.prelu = p->prelu;
  bb.out = S.h;
  bb.zsave = S.z;
  bb.mean = S.mean;
  bb.rstd = S.rstd;
  bb.use_running = (run & DSTD_TRAIN_RUNNING_STATS) != 0;
  bb.groups = (run & DSTD_TRAIN_PAIRED) ? 2 : 1;
  bb.sync = sync;
  DSTD_TRYH(bn_train_fwd(bb, B, cout, T, V, S.red, s));
  return op_fwd(gt, S.h, &p->conv_t, p->A_t, nullptr, p->R_t, p->alpha_tm, y, 0.f, S.op[2], s);  // :156-162
}

// dx_init: dx holds nothing yet -- the first contribution assigns (no
// memset); dx_extra (no residual conv only): also added to dx (the
// encoders' identity path of the model backward).
hipError_t block_bwd(const dstd_block_params* p, const float* x, int B, int T, int V, const BlockSaved& S,
                     const float* dy, float* dx, const dstd_block_grads* g, const BlockWs& W, hipStream_t s,
                     int run = 0, bool dx_init = false, const float* dx_extra = nullptr,
                     const dstd_bn_sync* sync = nullptr, Wgrad* wg = nullptr) {
  const int cin = p->cin, cout = p->cout, TV = T * V;
  const bool res = cin != cout;
  const size_t act = (size_t)B * cout * TV;
  const OpGeom gt(DSTD_MODE_TEMPORAL, B, cout, cout, T, V);
  // A_t + R_t: dR_t = dA; dh (=) the temporal op's input gradient
  DSTD_TRYH(op_bwd(gt, S.h, &p->conv_t, p->alpha_tm, S.op[2], dy, W.dh, &g->conv_t, g->R_t, g->alpha_tm, W.op, s,
                   0.f, 0, wg));
  BnBwd bb;
  bb.x = S.ysp;
  bb.zsave = S.z;
  bb.prelu = p->prelu;
  bb.dout = W.dh;
  bb.mean = S.mean;
  bb.rstd = S.rstd;
  bb.gamma = p->bn.weight;
  bb.du = W.dysp;
  bb.dz_out = W.dr;
  // identity residual, first contribution to dx: the BN backward writes
  // dx = dz (+ dx_extra) itself (no separate accumulate pass)
  const bool dz_to_dx = !res && dx && dx_init;
  if (dz_to_dx) {
    bb.dz_out = dx;
    bb.dz_add = dx_extra;
  }
  bb.dgamma = g->bn.weight;
  bb.dbeta = g->bn.bias;
  bb.use_running = (run & DSTD_TRAIN_RUNNING_STATS) != 0;
  bb.groups = (run & DSTD_TRAIN_PAIRED) ? 2 : 1;
  bb.sync = sync;
  DSTD_TRYH(bn_train_bwd(bb, B, cout, T, V, W.op.red, g->prelu, s));
  if (res) {
    BnBwd rb;
    rb.x = S.rc;
    rb.dout = W.dr;
    rb.mean = S.rmean;
    rb.rstd = S.rrstd;
    rb.gamma = p->res_bn.weight;
    rb.du = W.drc;
    rb.dgamma = g->res_bn.weight;
    rb.dbeta = g->res_bn.bias;
    rb.use_running = (run & DSTD_TRAIN_RUNNING_STATS) != 0;
    rb.groups = (run & DSTD_TRAIN_PAIRED) ? 2 : 1;
    rb.sync = sync;
    DSTD_TRYH(bn_train_bwd(rb, B, cout, T, V, W.op.red, nullptr, s));
    if (dx_extra) return hipErrorInvalidValue;
    DSTD_TRYH(conv_bwd(p->res_w, x, W.drc, dx, g->res_w, g->res_b, B, cin, cout, TV, W.op.gs, s,
                       dx_init ? 0.f : 1.f));
  } else if (dx && !dz_to_dx) {
    DSTD_TRYH(acc_mul(W.dr, nullptr, dx, act, s, dx_extra, dx_init ? 1 : 0));
  }
  const OpGeom gs(DSTD_MODE_SPATIAL, B, cin, cout, T, V);
  // A_s*W_s + R_s with A_s constant: each graph's dA accumulates straight into
  // its dR_s, and dW_s += dA * A_s, in the adjacency-backward finish
  for (int i = 0; i < 2; ++i)
    DSTD_TRYH(op_bwd(gs, x, &p->conv_s[i], p->alpha_sm, S.op[i], W.dysp, dx, &g->conv_s[i], g->R_s + i * V * V,
                     g->alpha_sm, W.op, s, 1.f, 0, wg, g->W_s + i * V * V, p->A_s + i * V * V));
  return hipSuccess;
}

// ---------------------------------------------------------------------------
// whole DSTDGCN
// ---------------------------------------------------------------------------
struct ModelSaved {
  float *X0, *y0, *z0, *hp0, *m0, *r0, *o;
  float* h[DSTD_MAX_LAYERS + 1];
  float *yb[DSTD_MAX_LAYERS], *ze[DSTD_MAX_LAYERS], *me[DSTD_MAX_LAYERS], *re[DSTD_MAX_LAYERS];
  BlockSaved st_in, st_out, enc[DSTD_MAX_LAYERS];
  float* red;
};
void carve_model_saved(Carver& cv, ModelSaved& s, int B, int T, int V, int C, int L) {
  const size_t act = (size_t)B * C * T * V;
  s.X0 = cv.take((size_t)B * 6 * T * V);
  carve_block_saved(cv, s.st_in, B, 6, C, T, V);
  s.y0 = cv.take(act);
  s.z0 = cv.take(act);
  s.hp0 = cv.take(act);
  s.m0 = cv.take(2 * C * V);  // per BN group (DSTD_TRAIN_PAIRED: 2)
  s.r0 = cv.take(2 * C * V);
  for (int i = 0; i <= L; ++i) s.h[i] = cv.take(act);
  for (int i = 0; i < L; ++i) {
    carve_block_saved(cv, s.enc[i], B, C, C, T, V);
    s.yb[i] = cv.take(act);
    s.ze[i] = cv.take(act);
    s.me[i] = cv.take(2 * C * V);
    s.re[i] = cv.take(2 * C * V);
  }
  carve_block_saved(cv, s.st_out, B, C, 3, T, V);
  s.o = cv.take((size_t)B * 3 * T * V);
  s.red = cv.take(bn_scratch_floats(B, C, T, V));
}

struct ModelWs {
  BlockWs blk;
  float *dO, *dha, *dhb, *du, *pp, *dX0;
};
void carve_model_ws(Carver& cv, ModelWs& w, int B, int T, int V, int C) {
  carve_block_ws(cv, w.blk, B, T, V, {{6, C}, {C, C}, {C, 3}});
  const size_t act = (size_t)B * C * T * V;
  w.dO = cv.take((size_t)B * 3 * T * V);
  w.dha = cv.take(act);
  w.dhb = cv.take(act);
  w.du = cv.take(act);
  w.pp = cv.take(C);
  w.dX0 = cv.take((size_t)B * 6 * T * V);
}

}  // namespace

extern "C" {

size_t dstd_dstdgc_train_saved_bytes_r(int mode, int B, int cin, int cout, int T, int V, int red) {
  Carver cv{nullptr};
  OpSaved s;
  carve_op_saved(cv, s, OpGeom(mode, B, cin, cout, T, V, red));
  return cv.off + 256;
}

size_t dstd_dstdgc_train_workspace_bytes_r(int mode, int B, int cin, int cout, int T, int V, int red) {
  Carver cv{nullptr};
  OpWs w;
  carve_op_ws(cv, w, {OpGeom(mode, B, cin, cout, T, V, red)});
  return cv.off + 256;
}

int dstd_dstdgc_train_fwd_r(int mode, const float* x, int B, int cin, int cout, int T, int V, int red,
                            const dstd_gc_weights* w, const float* A, const float* alpha, float* y, void* saved,
                            size_t saved_bytes, void* stream) {
  StreamDeviceGuard dev_guard_(stream, x);
  if (!x || !y || !A || !alpha || !gc_ok(w) || !saved) return DSTD_EINVAL;
  if (mode != DSTD_MODE_SPATIAL && mode != DSTD_MODE_TEMPORAL) return DSTD_EINVAL;
  if (B <= 0 || T <= 1 || V <= 0 || red <= 0) return DSTD_EINVAL;
  if (!shape_ok(B, T, V) || !ch_ok(cin) || !ch_ok(cout) || red > kMaxRed) return DSTD_ELIMIT;
  if (saved_bytes < dstd_dstdgc_train_saved_bytes_r(mode, B, cin, cout, T, V, red)) return DSTD_EWORKSPACE;
  const OpGeom g(mode, B, cin, cout, T, V, red);
  Carver cv{(char*)saved};
  OpSaved sv;
  carve_op_saved(cv, sv, g);
  CopyJobs js;
  pack_jobs(js, w, sv, g);
  DSTD_TRY(copy_jobs(js, (hipStream_t)stream));
  DSTD_TRY(op_fwd(g, x, w, A, nullptr, nullptr, alpha, y, 0.f, sv, (hipStream_t)stream));
  return DSTD_OK;
}

int dstd_dstdgc_train_bwd_r(int mode, const float* x, int B, int cin, int cout, int T, int V, int red,
                            const dstd_gc_weights* w, const float* alpha, const void* saved, size_t saved_bytes,
                            const float* dy, float* dx, const dstd_gc_grads* g, float* dA, float* dalpha,
                            void* workspace, size_t workspace_bytes, void* stream) {
  StreamDeviceGuard dev_guard_(stream, x);
  if (!x || !dy || !alpha || !gc_ok(w) || !gg_ok(g) || !dA || !dalpha || !saved || !workspace) return DSTD_EINVAL;
  if (mode != DSTD_MODE_SPATIAL && mode != DSTD_MODE_TEMPORAL) return DSTD_EINVAL;
  if (B <= 0 || T <= 1 || V <= 0 || red <= 0) return DSTD_EINVAL;
  if (!shape_ok(B, T, V) || !ch_ok(cin) || !ch_ok(cout) || red > kMaxRed) return DSTD_ELIMIT;
  if (saved_bytes < dstd_dstdgc_train_saved_bytes_r(mode, B, cin, cout, T, V, red)) return DSTD_EWORKSPACE;
  if (workspace_bytes < dstd_dstdgc_train_workspace_bytes_r(mode, B, cin, cout, T, V, red))
    return DSTD_EWORKSPACE;
  const OpGeom geo(mode, B, cin, cout, T, V, red);
  Carver cs{(char*)const_cast<void*>(saved)};
  OpSaved sv;
  carve_op_saved(cs, sv, geo);
  Carver cw{(char*)workspace};
  OpWs ws;
  carve_op_ws(cw, ws, {geo});
  DSTD_TRY(op_bwd(geo, x, w, alpha, sv, dy, dx, g, dA, dalpha, ws, (hipStream_t)stream));
  return DSTD_OK;
}

size_t dstd_dstdgc_train_saved_bytes(int mode, int B, int cin, int cout, int T, int V) {
  return dstd_dstdgc_train_saved_bytes_r(mode, B, cin, cout, T, V, 2);
}

size_t dstd_dstdgc_train_workspace_bytes(int mode, int B, int cin, int cout, int T, int V) {
  return dstd_dstdgc_train_workspace_bytes_r(mode, B, cin, cout, T, V, 2);
}

int dstd_dstdgc_train_fwd(int mode, const float* x, int B, int cin, int cout, int T, int V,
                          const dstd_gc_weights* w, const float* A, const float* alpha, float* y, void* saved,
                          size_t saved_bytes, void* stream) {
  return dstd_dstdgc_train_fwd_r(mode, x, B, cin, cout, T, V, 2, w, A, alpha, y, saved, saved_bytes, stream);
}

int dstd_dstdgc_train_bwd(int mode, const float* x, int B, int cin, int cout, int T, int V,
                          const dstd_gc_weights* w, const float* alpha, const void* saved, size_t saved_bytes,
                          const float* dy, float* dx, const dstd_gc_grads* g, float* dA, float* dalpha,
                          void* workspace, size_t workspace_bytes, void* stream) {
  return dstd_dstdgc_train_bwd_r(mode, x, B, cin, cout, T, V, 2, w, alpha, saved, saved_bytes, dy, dx, g, dA, dalpha,
                                 workspace, workspace_bytes, stream);
}

size_t dstd_block_train_saved_bytes(int B, int cin, int cout, int T, int V) {
  Carver cv{nullptr};
  BlockSaved s;
  carve_block_saved(cv, s, B, cin, cout, T, V);
  return cv.off + 256;
}

size_t dstd_block_train_workspace_bytes(int B, int cin, int cout, int T, int V) {
  Carver cv{nullptr};
  BlockWs w;
  carve_block_ws(cv, w, B, T, V, {{cin, cout}});
  return cv.off + 256;
}

int dstd_block_train_fwd_ex(const dstd_block_params* p, const float* x, int B, int T, int V, float momentum,
                            float* y, void* saved, size_t saved_bytes, void* stream, unsigned flags) {
  StreamDeviceGuard dev_guard_(stream, x);
  if (!block_ok(p) || !x || !y || !saved || (flags & ~kTrainFlags)) return DSTD_EINVAL;
  if ((flags & DSTD_TRAIN_PAIRED) && (B & 1)) return DSTD_EINVAL;
  if (B <= 0 || T <= 1 || V <= 0) return DSTD_EINVAL;
  if (!shape_ok(B, T, V)) return DSTD_ELIMIT;
  if (saved_bytes < dstd_block_train_saved_bytes(B, p->cin, p->cout, T, V)) return DSTD_EWORKSPACE;
  Carver cv{(char*)saved};
  BlockSaved S;
  carve_block_saved(cv, S, B, p->cin, p->cout, T, V);
  DSTD_TRY(block_fwd(p, x, B, T, V, momentum, y, S, (hipStream_t)stream, (int)flags));
  return DSTD_OK;
}

int dstd_block_train_fwd(const dstd_block_params* p, const float* x, int B, int T, int V, float momentum, float* y,
                         void* saved, size_t saved_bytes, void* stream) {
  return dstd_block_train_fwd_ex(p, x, B, T, V, momentum, y, saved, saved_bytes, stream, 0u);
}

int dstd_block_train_bwd_ex(const dstd_block_params* p, const float* x, int B, int T, int V, const void* saved,
                            size_t saved_bytes, const float* dy, float* dx, const dstd_block_grads* g,
                            void* workspace, size_t workspace_bytes, void* stream, unsigned flags) {
  StreamDeviceGuard dev_guard_(stream, x);
  if (!block_ok(p) || !block_grads_ok(p, g) || !x || !dy || !saved || !workspace) return DSTD_EINVAL;
  if (flags & ~kTrainFlags) return DSTD_EINVAL;
  if ((flags & DSTD_TRAIN_PAIRED) && (B & 1)) return DSTD_EINVAL;
  if (B <= 0 || T <= 1 || V <= 0) return DSTD_EINVAL;
  if (!shape_ok(B, T, V)) return DSTD_ELIMIT;
  if (saved_bytes < dstd_block_train_saved_bytes(B, p->cin, p->cout, T, V)) return DSTD_EWORKSPACE;
  if (workspace_bytes < dstd_block_train_workspace_bytes(B, p->cin, p->cout, T, V)) return DSTD_EWORKSPACE;
  Carver cs{(char*)const_cast<void*>(saved)};
  BlockSaved S;
  carve_block_saved(cs, S, B, p->cin, p->cout, T, V);
  Carver cw{(char*)workspace};
  BlockWs W;
  carve_block_ws(cw, W, B, T, V, {{p->cin, p->cout}});
  DSTD_TRY(block_bwd(p, x, B, T, V, S, dy, dx, g, W, (hipStream_t)stream, (int)flags));
  return DSTD_OK;
}

int dstd_block_train_bwd(const dstd_block_params* p, const float* x, int B, int T, int V, const void* saved,
                         size_t saved_bytes, const float* dy, float* dx, const dstd_block_grads* g,
                         void* workspace, size_t workspace_bytes, void* stream) {
  return dstd_block_train_bwd_ex(p, x, B, T, V, saved, saved_bytes, dy, dx, g, workspace, workspace_bytes, stream,
                                 0u);
}

size_t dstd_model_train_saved_bytes(int B, int T, int V, int num_feature, int num_layers) {
  Carver cv{nullptr};
  ModelSaved s;
  carve_model_saved(cv, s, B, T, V, num_feature, std::min(std::max(num_layers, 0), DSTD_MAX_LAYERS));
  return cv.off + 256;
}

size_t dstd_model_train_workspace_bytes(int B, int T, int V, int num_feature, int num_layers) {
  (void)num_layers;
  Carver cv{nullptr};
  ModelWs w;
  carve_model_ws(cv, w, B, T, V, num_feature);
  return cv.off + 256;
}

size_t dstd_bn_sync_buffer_floats(int world, int num_feature, int V) {
  // forward gather: world x (<= 2 groups) x C*V x (mean, M2, count); backward:
  // 2 x C*V x 2 sums + 2 counts
  const size_t cv = (size_t)std::max(num_feature, 6) * V;
  return std::max((size_t)std::max(world, 1) * 2 * cv * 3, 2 * cv * 2 + 2);
}

static bool sync_ok(const dstd_bn_sync* y, int C, int V) {
  return !y || (y->fn && y->buf && y->world >= 1 && y->rank >= 0 && y->rank < y->world &&
                y->buf_floats >= (long long)dstd_bn_sync_buffer_floats(y->world, C, V));
}

int dstd_model_train_fwd_ex(const dstd_model_params* p, const float* x, int B, float momentum, float dropout_p,
                            unsigned long long seed, float* y, void* saved, size_t saved_bytes, void* stream,
                            unsigned flags) {
  return dstd_model_train_fwd_sync(p, x, B, momentum, dropout_p, seed, y, saved, saved_bytes, stream, flags, nullptr);
}

int dstd_model_train_fwd_sync(const dstd_model_params* p, const float* x, int B, float momentum, float dropout_p,
                              unsigned long long seed, float* y, void* saved, size_t saved_bytes, void* stream,
                              unsigned flags, const dstd_bn_sync* sync) {
  StreamDeviceGuard dev_guard_(stream, x);
  if (!model_ok(p) || !x || !y || !saved || !(dropout_p >= 0.f && dropout_p < 1.f)) return DSTD_EINVAL;
  if (!sync_ok(sync, p->num_feature, p->V)) return DSTD_EINVAL;
  if (flags & ~kModelTrainFlags) return DSTD_EINVAL;
  if ((flags & DSTD_TRAIN_SEED_DEVICE) && dropout_p > 0.f && !seed) return DSTD_EINVAL;
  if ((flags & DSTD_TRAIN_PAIRED) && (B & 1)) return DSTD_EINVAL;
  const int run = (int)flags;
  const int T = p->T, V = p->V, C = p->num_feature, L = p->num_layers;
  if (B <= 0 || T <= 1 || V <= 0) return DSTD_EINVAL;
  if (!shape_ok(B, T, V) || !ch_ok(C)) return DSTD_ELIMIT;
  if (p->st_in.cin != 6 || p->st_in.cout != C || p->st_out.cin != C || p->st_out.cout != 3) return DSTD_EINVAL;
  if (saved_bytes < dstd_model_train_saved_bytes(B, T, V, C, L)) return DSTD_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  Carver cv{(char*)saved};
  ModelSaved S;
  carve_model_saved(cv, S, B, T, V, C, L);
  const size_t act = (size_t)B * C * T * V;
  // the blocks' second spatial ops build their adjacency on a second stream
  // (block_fwd); joined at each block and by the destructor on any return
#ifndef DSTD_FWD_SIDE  // (A/B: 0 = the forward on the caller's stream only)
#define DSTD_FWD_SIDE 1
#endif
  Wgrad side((flags & DSTD_TRAIN_ONE_STREAM) || !DSTD_FWD_SIDE ? nullptr : wgrad_acquire());
  side.main = s;
  DSTD_TRY(prep_nctv(x, B, T, V, 3, S.X0, s));                                   // :298-303
  {  // every block's packed conv weights, kMaxCopyJobs per launch
    CopyJobs js;
    auto add = [&](const dstd_block_params* bp, const BlockSaved& bs) -> hipError_t {
      if (js.n + kBlockPackJobs > kMaxCopyJobs) {
        DSTD_TRYH(copy_jobs(js, s));
        js.n = 0;
      }
      pack_block(js, bp, bs, B, T, V);
      return hipSuccess;
    };
    DSTD_TRY(add(&p->st_in, S.st_in));
    for (int i = 0; i < L; ++i) DSTD_TRY(add(&p->enc[i], S.enc[i]));
    DSTD_TRY(add(&p->st_out, S.st_out));
    DSTD_TRY(copy_jobs(js, s));
  }
  DSTD_TRY(block_fwd(&p->st_in, S.X0, B, T, V, momentum, S.y0, S.st_in, s, run, sync, true, &side));  // :305
  BnFwd b0;                                                                      // :306-308
  b0.x = S.y0;
  b0.gamma = p->bn_in.weight;
  b0.beta = p->bn_in.bias;
  b0.running_mean = const_cast<float*>(p->bn_in.running_mean);
  b0.running_var = const_cast<float*>(p->bn_in.running_var);
  b0.momentum = momentum;
  b0.eps = p->bn_in.eps;
  b0.prelu = p->prelu;
  b0.out = dropout_p > 0.f ? S.hp0 : S.h[0];
  b0.zsave = S.z0;
  b0.mean = S.m0;
  b0.rstd = S.r0;
  b0.use_running = (run & DSTD_TRAIN_RUNNING_STATS) != 0;
  b0.groups = (run & DSTD_TRAIN_PAIRED) ? 2 : 1;
  b0.sync = sync;
  DSTD_TRY(bn_train_fwd(b0, B, C, T, V, S.red, s));
  if (dropout_p > 0.f) DSTD_TRY(dropout(S.hp0, S.h[0], act, dropout_p, seed, s, (flags & DSTD_TRAIN_SEED_DEVICE) != 0));  // do_in
  for (int i = 0; i < L; ++i) {                                                  // :310-311
    DSTD_TRY(block_fwd(&p->enc[i], S.h[i], B, T, V, momentum, S.yb[i], S.enc[i], s, run, sync, true, &side));
    BnFwd be;  // BN(block(h) + h) -> PReLU  (:278-285, Identity residual :247-248)
    be.x = S.yb[i];
    be.x2 = S.h[i];
    be.gamma = p->enc_bn[i].weight;
    be.beta = p->enc_bn[i].bias;
    be.running_mean = const_cast<float*>(p->enc_bn[i].running_mean);
    be.running_var = const_cast<float*>(p->enc_bn[i].running_var);
    be.momentum = momentum;
    be.eps = p->enc_bn[i].eps;
    be.prelu = p->enc_prelu[i];
    be.out = S.h[i + 1];
    be.zsave = S.ze[i];
    be.mean = S.me[i];
    be.rstd = S.re[i];
    be.use_running = (run & DSTD_TRAIN_RUNNING_STATS) != 0;
    be.groups = (run & DSTD_TRAIN_PAIRED) ? 2 : 1;
    be.sync = sync;
    DSTD_TRY(bn_train_fwd(be, B, C, T, V, S.red, s));
  }
  DSTD_TRY(block_fwd(&p->st_out, S.h[L], B, T, V, momentum, S.o, S.st_out, s, run, sync, true, &side));  // :313
  DSTD_TRY(out_ntvc(S.o, x, B, T, V, 3, y, s));                                       // :314-315
  return DSTD_OK;
}

int dstd_model_train_fwd(const dstd_model_params* p, const float* x, int B, float momentum, float dropout_p,
                         unsigned long long seed, float* y, void* saved, size_t saved_bytes, void* stream) {
  return dstd_model_train_fwd_ex(p, x, B, momentum, dropout_p, seed, y, saved, saved_bytes, stream, 0u);
}

int dstd_model_train_bwd_ex(const dstd_model_params* p, const float* x, int B, float dropout_p,
                            unsigned long long seed, const void* saved, size_t saved_bytes, const float* dy,
                            const dstd_model_grads* g, float* dx, void* workspace, size_t workspace_bytes,
                            void* stream, unsigned flags) {
  return dstd_model_train_bwd_sync(p, x, B, dropout_p, seed, saved, saved_bytes, dy, g, dx, workspace,
                                   workspace_bytes, stream, flags, nullptr);
}

int dstd_model_train_bwd_sync(const dstd_model_params* p, const float* x, int B, float dropout_p,
                              unsigned long long seed, const void* saved, size_t saved_bytes, const float* dy,
                              const dstd_model_grads* g, float* dx, void* workspace, size_t workspace_bytes,
                              void* stream, unsigned flags, const dstd_bn_sync* sync) {
  StreamDeviceGuard dev_guard_(stream, x);
  if (!model_ok(p) || !g || !x || !dy || !saved || !workspace || !(dropout_p >= 0.f && dropout_p < 1.f))
    return DSTD_EINVAL;
  if (!sync_ok(sync, p->num_feature, p->V)) return DSTD_EINVAL;
  if (flags & ~kModelTrainFlags) return DSTD_EINVAL;
  if ((flags & DSTD_TRAIN_SEED_DEVICE) && dropout_p > 0.f && !seed) return DSTD_EINVAL;
  if ((flags & DSTD_TRAIN_PAIRED) && (B & 1)) return DSTD_EINVAL;
  const int run = (int)flags;
  const int T = p->T, V = p->V, C = p->num_feature, L = p->num_layers;
  if (B <= 0 || T <= 1 || V <= 0) return DSTD_EINVAL;
  if (!shape_ok(B, T, V) || !ch_ok(C)) return DSTD_ELIMIT;
  if (!block_grads_ok(&p->st_in, &g->st_in) || !block_grads_ok(&p->st_out, &g->st_out) || !bng_ok(g->bn_in) ||
      !g->prelu)
    return DSTD_EINVAL;
  for (int i = 0; i < L; ++i)
    if (!block_grads_ok(&p->enc[i], &g->enc[i]) || !bng_ok(g->enc_bn[i]) || !g->enc_prelu[i]) return DSTD_EINVAL;
  if (saved_bytes < dstd_model_train_saved_bytes(B, T, V, C, L)) return DSTD_EWORKSPACE;
  if (workspace_bytes < dstd_model_train_workspace_bytes(B, T, V, C, L)) return DSTD_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  Carver cs{(char*)const_cast<void*>(saved)};
  ModelSaved S;
  carve_model_saved(cs, S, B, T, V, C, L);
  Carver cw{(char*)workspace};
  ModelWs W;
  carve_model_ws(cw, W, B, T, V, C);
  const size_t act = (size_t)B * C * T * V;
  Wgrad wg((flags & DSTD_TRAIN_ONE_STREAM) ? nullptr : wgrad_acquire());
  wg.main = s;
  DSTD_TRY(out_ntvc_bwd(dy, B, T, V, 3, W.dO, s));
  float* dha = W.dha;
  float* dhb = W.dhb;
  DSTD_TRY(block_bwd(&p->st_out, S.h[L], B, T, V, S.st_out, W.dO, dha, &g->st_out, W.blk, s, run, true, nullptr,
                     sync, &wg));
  for (int i = L - 1; i >= 0; --i) {
    BnBwd be;
    be.x = S.yb[i];
    be.x2 = S.h[i];
    be.zsave = S.ze[i];
    be.prelu = p->enc_prelu[i];
    be.dout = dha;
    be.mean = S.me[i];
    be.rstd = S.re[i];
    be.gamma = p->enc_bn[i].weight;
    be.du = W.du;
    be.dgamma = g->enc_bn[i].weight;
    be.dbeta = g->enc_bn[i].bias;
    be.use_running = (run & DSTD_TRAIN_RUNNING_STATS) != 0;
    be.groups = (run & DSTD_TRAIN_PAIRED) ? 2 : 1;
    be.sync = sync;
    DSTD_TRY(bn_train_bwd(be, B, C, T, V, W.blk.op.red, g->enc_prelu[i], s));
    // u = block(h) + h: dh = du (identity path) + block backward
    DSTD_TRY(block_bwd(&p->enc[i], S.h[i], B, T, V, S.enc[i], W.du, dhb, &g->enc[i], W.blk, s, run, true, W.du,
                       sync, &wg));
    std::swap(dha, dhb);
  }
  if (dropout_p > 0.f) DSTD_TRY(dropout(dha, dha, act, dropout_p, seed, s, (flags & DSTD_TRAIN_SEED_DEVICE) != 0));
  BnBwd b0;
  b0.x = S.y0;
  b0.zsave = S.z0;
  b0.prelu = p->prelu;
  b0.dout = dha;
  b0.mean = S.m0;
  b0.rstd = S.r0;
  b0.gamma = p->bn_in.weight;
  b0.du = W.du;
  b0.dgamma = g->bn_in.weight;
  b0.dbeta = g->bn_in.bias;
  b0.use_running = (run & DSTD_TRAIN_RUNNING_STATS) != 0;
  b0.groups = (run & DSTD_TRAIN_PAIRED) ? 2 : 1;
  b0.sync = sync;
  DSTD_TRY(bn_train_bwd(b0, B, C, T, V, W.blk.op.red, g->prelu, s));
  DSTD_TRY(block_bwd(&p->st_in, S.X0, B, T, V, S.st_in, W.du, dx ? W.dX0 : nullptr, &g->st_in, W.blk, s, run, true,
                     nullptr, sync, &wg));
  if (dx) DSTD_TRY(prep_nctv_bwd(W.dX0, dy, B, T, V, 3, dx, s));  // :298-303, 315
  DSTD_TRY(wg.join());
  return DSTD_OK;
}

int dstd_model_train_bwd(const dstd_model_params* p, const float* x, int B, float dropout_p,
                         unsigned long long seed, const void* saved, size_t saved_bytes, const float* dy,
                         const dstd_model_grads* g, void* workspace, size_t workspace_bytes, void* stream) {
  return dstd_model_train_bwd_ex(p, x, B, dropout_p, seed, saved, saved_bytes, dy, g, nullptr, workspace,
                                 workspace_bytes, stream, 0u);
}

size_t dstd_loss_workspace_bytes(void) { return (size_t)mpjpe_partials() * sizeof(float) + 256; }

int dstd_mpjpe_fwd(const float* pred, const float* targ, size_t n_points, float* loss, void* workspace,
                   size_t workspace_bytes, void* stream) {
  StreamDeviceGuard dev_guard_(stream, pred);
  if (!pred || !targ || !loss || !workspace || n_points == 0) return DSTD_EINVAL;
  if (workspace_bytes < dstd_loss_workspace_bytes()) return DSTD_EWORKSPACE;
  DSTD_TRY(mpjpe_fwd(pred, targ, n_points, loss, (float*)workspace, (hipStream_t)stream));
  return DSTD_OK;
}

int dstd_mpjpe_bwd(const float* pred, const float* targ, size_t n_points, const float* grad_loss, float scale,
                   float* dpred, void* stream) {
  StreamDeviceGuard dev_guard_(stream, pred);
  if (!pred || !targ || !dpred || n_points == 0) return DSTD_EINVAL;
  DSTD_TRY(mpjpe_bwd(pred, targ, n_points, grad_loss, scale, dpred, (hipStream_t)stream));
  return DSTD_OK;
}

int dstd_frame_mpjpe(const float* all_seqs, const float* outputs, int B, int T, int D, int t_out0,
                     const int* used_pos, int n_used, const int* joint_src, const int* frames, int n_frames,
                     float* sums, void* stream) {
  StreamDeviceGuard dev_guard_(stream, all_seqs);
  if (!all_seqs || !outputs || !used_pos || !joint_src || !frames || !sums) return DSTD_EINVAL;
  if (B <= 0 || T <= 0 || D <= 0 || D % 3 || n_used <= 0 || n_frames <= 0 || t_out0 < 0 || t_out0 >= T)
    return DSTD_EINVAL;
  DSTD_TRY(frame_mpjpe(all_seqs, outputs, B, T, D, t_out0, used_pos, n_used, joint_src, frames, n_frames, sums,
                       (hipStream_t)stream));
  return DSTD_OK;
}

}  // extern "C"
