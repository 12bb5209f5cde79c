// C ABI (include/dstd_gcn.h): argument checking, workspace carving and the
// launch sequence of one DSTDGC / DSTDGCB / DSTDGCN forward.
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include <vector>

#include "../../include/dstd_gcn.h"
#include "dstd_common.h"
#include "dstd_hilo.h"
#include "dstd_kernels.h"

using namespace dstd;

#ifdef DSTD_SPRE_CHECK
#include <stdio.h>
// (debug builds: the planes phase 3 left in adj_s against a k_adj_hl<0> run
// of the same block into a private buffer -- mismatching halves and the first)
__global__ void k_cmp_u16(const uint16_t* a, const uint16_t* b, size_t n, unsigned* out) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (a[i] != b[i]) {
      atomicAdd(&out[0], 1u);
      atomicMin(&out[1], (unsigned)i);
    }
}
#endif
namespace {

constexpr int kMaxT = 128;  // the generic kernels cover T <= 128 (adjacency row groups past 112)
constexpr int kMaxV = 32;
constexpr int kMaxC = 64;

// Bump allocator over the caller's workspace.  With base == nullptr it only
// measures, so *_workspace_bytes and the forward share one layout.
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

#define DSTD_TRY(expr)                         \
  do {                                         \
    hipError_t _e = (expr);                    \
    if (_e != hipSuccess) return (int)_e;      \
  } while (0)

bool shape_ok(int B, int T, int V) { return B > 0 && T > 1 && V > 0; }
bool limits_ok(int T, int V, int cin, int cout) {
  return T <= kMaxT && V <= kMaxV && cin >= 1 && cin <= kMaxC && cout >= 1 && cout <= kMaxC;
}
bool gc_ok(const dstd_gc_weights* w) {
  return w && w->wf && w->bf && w->wm1 && w->bm1 && w->wm2 && w->bm2 && w->wrm && w->brm;
}
bool bn_ok(const dstd_bn& b) { return b.weight && b.bias && b.running_mean && b.running_var; }
bool block_ok(const dstd_block_params* p) {
  if (!p || !p->A_s || !p->W_s || !p->R_s || !p->A_t || !p->R_t || !p->alpha_sm || !p->alpha_tm || !p->prelu)
    return false;
  if (!gc_ok(&p->conv_s[0]) || !gc_ok(&p->conv_s[1]) || !gc_ok(&p->conv_t) || !bn_ok(p->bn)) return false;
  if (p->cin != p->cout && (!p->res_w || !p->res_b || !bn_ok(p->res_bn))) return false;
  return true;
}

// Optional per-launch event brackets (dstd_model_fwd_profiled).
struct Prof {
  dstd_profile* p = nullptr;
  int block = -1;
  int open = -1;
  void begin(int kind, hipStream_t s) {
    open = -1;
    if (!p || !(p->kind_mask & (1u << kind)) || p->count >= p->capacity) return;
    if (p->only_block >= 0 && p->only_block != block) return;
    open = p->count++;
    p->kinds[open] = kind;
    if (p->block) p->block[open] = block;
    (void)hipEventRecord((hipEvent_t)p->events[2 * open], s);
  }
  void end(hipStream_t s) {
    if (open >= 0) (void)hipEventRecord((hipEvent_t)p->events[2 * open + 1], s);
    open = -1;
  }
};

// Folded per-block constants (filled by k_fold).
struct BlockFold {
  float* bn_s;
  float* bn_h;
  float* rbn_s;
  float* rbn_h;
  float* astat_s;  // [2][V][V]
  float* astat_t;  // [T][T]
  // split-f16 weight images (k_hl_prep, dstd_hilo.h) of the 64 -> 64 GC kernels
  uint4* hl_ws[3];  // conv_s[g].conv_f, [2]: residual conv (cin != cout)
  uint4* hl_pqs;    // conv_t.conv_m1/m2 (P/Q written by the spatial kernel)
  uint4* hl_wt;     // conv_t.conv_f
  uint4* hl_pqt;    // next block's conv_s[*].conv_m1/m2 (P/Q written by the temporal kernel)
  uint4* hl_rms[2]; // conv_s[g].conv_rm (spatial adjacency)
  uint4* hl_rmt;    // conv_t.conv_rm (temporal adjacency)
  float* hl_scale;  // 9 scale slots (kHLSlot floats each, dstd_hilo.h): ws0, ws1, pqs, wt, pqt, rms0, rms1, rmt, ws2
  float* hl_rbias;  // [2T + V]: fused conv_rm biases (HLJob::bias_out) of rms0, rms1, rmt
};

// Which GC launches of a block run the split-f16 kernels; tf: the temporal
// one with its adjacency built in LDS (k_temporal_fused, no k_adj_hl<1>).
struct BlockHL {
  bool s, t, tf;
  bool s_pre = false;  // the spatial adjacency planes were built by the previous block's temporal launch
  bool bf = false;     // spatial + fused temporal GC in one launch (k_block_fused)
  bool adj0 = false;   // (conv_st_in with bf) its spatial planes from the model input in that launch
};

struct BlockScratch {
  float* adj_s;  // [B][2][T][V][V]
  float* adj_t;  // [B][V][T][T]
  float* pq_s;   // [B][8][T][V]
  float* pq_t;   // [B][4][T][V]
};

void carve_fold(Carver& cv, BlockFold& f, int T, int V, int cout, bool res) {
  f.bn_s = cv.take((size_t)cout * V);
  f.bn_h = cv.take((size_t)cout * V);
  f.rbn_s = res ? cv.take((size_t)cout * V) : nullptr;
  f.rbn_h = res ? cv.take((size_t)cout * V) : nullptr;
  f.astat_s = cv.take((size_t)2 * V * V);
  f.astat_t = cv.take((size_t)T * T);
  auto img = [&](int n) { return reinterpret_cast<uint4*>(cv.take((size_t)4 * n)); };
  f.hl_ws[0] = img(kHLConvImg);
  f.hl_ws[1] = img(kHLConvImg);
  f.hl_ws[2] = img(kHLConvImg);
  f.hl_pqs = img(kHLPQImg);
  f.hl_wt = img(kHLConvImg);
  f.hl_pqt = img(kHLPQImg);
  f.hl_rms[0] = img(hl_rm_img(T, 2 * T));
  f.hl_rms[1] = img(hl_rm_img(T, 2 * T));
  f.hl_rmt = img(hl_rm_img(V, 2 * V));
  f.hl_scale = cv.take(9 * kHLSlot);
  f.hl_rbias = cv.take((size_t)2 * T + V);
}

// adjacency scratch: the larger of the fp32 rows and the split-f16 planes
size_t adj_s_floats(int B, int T, int V) {
  const size_t row = std::max((size_t)adj_ld_spatial(V), (size_t)V * hl_sl_spatial(V));
  return (size_t)B * 2 * T * row;
}
size_t adj_t_floats(int B, int T, int V) {
  const size_t row = std::max((size_t)adj_ld_temporal(T), (size_t)T * hl_sl_temporal(T));
  return (size_t)B * V * row;
}

void carve_scratch(Carver& cv, BlockScratch& s, int B, int T, int V) {
  s.adj_s = cv.take(adj_s_floats(B, T, V));
  s.adj_t = cv.take(adj_t_floats(B, T, V));
  s.pq_s = cv.take((size_t)B * 8 * T * V);
  s.pq_t = cv.take((size_t)B * 4 * T * V);
}

using FoldList = std::vector<FoldJob>;

void add_bn_job(FoldList& fa, const dstd_bn& bn, int C, int V, float* s, float* h) {
  fa.emplace_back();
  FoldJob& j = fa.back();
  j.kind = FOLD_BN;
  j.n = C * V;
  j.C = C;
  j.V = V;
  j.p0 = bn.weight;
  j.p1 = bn.bias;
  j.p2 = bn.running_mean;
  j.p3 = bn.running_var;
  j.eps = bn.eps;
  j.o0 = s;
  j.o1 = h;
}

void add_block_jobs(FoldList& fa, const dstd_block_params* p, const BlockFold& f, int T, int V) {
  add_bn_job(fa, p->bn, p->cout, V, f.bn_s, f.bn_h);
  if (p->cin != p->cout) add_bn_job(fa, p->res_bn, p->cout, V, f.rbn_s, f.rbn_h);
  fa.emplace_back();
  FoldJob& a = fa.back();
  a.kind = FOLD_AWR;  // A_s*W_s + R_s for both graphs (model/dstdgcn.py:146-149)
  a.n = 2 * V * V;
  a.p0 = p->A_s;
  a.p1 = p->W_s;
  a.p2 = p->R_s;
  a.o0 = f.astat_s;
  fa.emplace_back();
  FoldJob& t = fa.back();
  t.kind = FOLD_AR;  // A_t + R_t (:158-160)
  t.n = T * T;
  t.p0 = p->A_t;
  t.p1 = p->R_t;
  t.o0 = f.astat_t;
}

hipError_t run_fold(const FoldList& jobs, hipStream_t s) {
  for (size_t i = 0; i < jobs.size(); i += kMaxFoldJobs) {
    FoldArgs fa{};
    for (size_t j = i; j < jobs.size() && j < i + kMaxFoldJobs; ++j) fa.jobs[fa.njobs++] = jobs[j];
    hipError_t e = launch_fold(fa, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

using HLList = std::vector<HLJob>;

hipError_t run_hl_prep(const HLList& jobs, hipStream_t s) {
  for (size_t i = 0; i < jobs.size(); i += kMaxHLJobs) {
    HLPrepArgs ha{};
    for (size_t j = i; j < jobs.size() && j < i + kMaxHLJobs; ++j) ha.jobs[ha.njobs++] = jobs[j];
    hipError_t e = launch_hl_prep(ha, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

void add_hl_conv(HLList& l, const float* w, const float* b, int rows, int cols, uint4* img, float* sc) {
  HLJob j{};
  j.kind = HLJ_CONV;
  j.w[0] = w;
  j.bias = b;
  j.nblk = 1;
  j.rows = rows;
  j.cols = cols;
  j.img = img;
  j.inv_scale = sc;
  l.push_back(j);
}
void add_hl_rm(HLList& l, const float* w, const float* b, int rows, int cols, uint4* img, float* sc, float* bout,
               const float* alpha, const float* astat, int nastat) {
  HLJob j{};
  j.kind = HLJ_RM;
  j.w[0] = w;
  j.alpha = alpha;
  j.astat = astat;
  j.nastat = nastat;
  j.bias = b;
  j.bias_out = bout;
  j.nblk = 1;
  j.rows = rows;
  j.cols = cols;
  j.img = img;
  j.inv_scale = sc;
  l.push_back(j);
}
void add_hl_pq(HLList& l, const float* const* w, int nblk, int cols, uint4* img, float* sc) {
  HLJob j{};
  j.kind = HLJ_PQ;
  for (int i = 0; i < nblk; ++i) j.w[i] = w[i];
  j.nblk = nblk;
  j.cols = cols;
  j.img = img;
  j.inv_scale = sc;
  l.push_back(j);
}

// What the temporal kernel does after the block (see TemporalEpi).
struct BlockTail {
  int epi;
  const float* xres;
  const float* bn_s;
  const float* bn_h;
  const float* prelu;
  const dstd_block_params* next;  // next block: its spatial P/Q are produced here
  // the next block's spatial adjacency planes are built here too (k_temporal_fused phase 3)
  const BlockFold* next_f = nullptr;
  bool next_adj = false;
};

// Split-f16 GC kernels (dstd_hilo.hip) where the shape has them, unless the
// call asks for exact fp32 (DSTD_FWD_EXACT_FP32).
BlockHL block_hl(const dstd_block_params* p, const BlockTail& tail, int B, int T, int V, unsigned flags) {
  const bool exact = (flags & DSTD_FWD_EXACT_FP32) != 0;
  BlockHL r{false, false, false, false};
  if (exact) return r;
  r.s = spatial_hl_supported(T, V) &&
        ((p->cin == 64 && p->cout == 64) || (p->cin == 6 && p->cout == 64) || (p->cin == 64 && p->cout == 3));
  r.t = temporal_hl_supported(T, V) &&
        ((p->cout == 64 && (tail.epi == TEPI_ENC || tail.epi == TEPI_IN || tail.epi == TEPI_RAW) &&
          (!tail.next || tail.next->cin == 64)) ||
         (p->cout == 3 && (tail.epi == TEPI_OUT || tail.epi == TEPI_RAW) && !tail.next));
#ifndef DSTD_NO_TFUSED
  // one workgroup per sample: below one sample per CU the fused kernel leaves
  // CUs idle and the unit-parallel pair (k_adj_hl<1> + k_temporal_hl) wins
  // (B = 16..128: 25-30% faster forward; B = 256: 8% slower, profiles/r03m_small_batch_ab.txt)
  r.tf = r.t && temporal_fused_supported(T, V) &&
         ((B >= hl_device_cus() && temporal_fused_default(T, V)) || (flags & DSTD_FWD_FUSED_TEMPORAL));
#endif
  // the whole block as one launch wherever both GCs run split and the
  // temporal one fused (one workgroup per sample either way)
  r.bf = r.s && r.tf && !(flags & DSTD_FWD_SEPARATE_BLOCK) && block_fused_supported(T, V, p->cin, p->cout, tail.epi);
  return r;
}

// scale slot i of a block's weight images (BlockFold::hl_scale)
float* hls(const BlockFold& f, int i) { return f.hl_scale + kHLSlot * i; }

// Weight images of the block's split-f16 launches.
void add_block_hl_jobs(HLList& l, const dstd_block_params* p, const BlockFold& f, const BlockTail& tail,
                       const BlockHL& hl, int T, int V) {
  if (hl.s) {
    add_hl_rm(l, p->conv_s[0].wrm, p->conv_s[0].brm, T, 2 * T, f.hl_rms[0], hls(f, 5), f.hl_rbias, p->alpha_sm,
              f.astat_s, V * V);
    add_hl_rm(l, p->conv_s[1].wrm, p->conv_s[1].brm, T, 2 * T, f.hl_rms[1], hls(f, 6), f.hl_rbias + T, p->alpha_sm,
              f.astat_s + V * V, V * V);
    add_hl_conv(l, p->conv_s[0].wf, p->conv_s[0].bf, p->cout, p->cin, f.hl_ws[0], hls(f, 0));
    add_hl_conv(l, p->conv_s[1].wf, p->conv_s[1].bf, p->cout, p->cin, f.hl_ws[1], hls(f, 1));
    if (p->cin != p->cout) add_hl_conv(l, p->res_w, p->res_b, p->cout, p->cin, f.hl_ws[2], hls(f, 8));
    const float* w[2] = {p->conv_t.wm1, p->conv_t.wm2};
    add_hl_pq(l, w, 2, p->cout, f.hl_pqs, hls(f, 2));
  }
  if (hl.t) {
    add_hl_rm(l, p->conv_t.wrm, p->conv_t.brm, V, 2 * V, f.hl_rmt, hls(f, 7), f.hl_rbias + 2 * T, p->alpha_tm,
              f.astat_t, T * T);
    add_hl_conv(l, p->conv_t.wf, p->conv_t.bf, p->cout, p->cout, f.hl_wt, hls(f, 3));
    if (tail.next) {
      const dstd_block_params* q = tail.next;
      const float* w[4] = {q->conv_s[0].wm1, q->conv_s[0].wm2, q->conv_s[1].wm1, q->conv_s[1].wm2};
      add_hl_pq(l, w, 4, 64, f.hl_pqt, hls(f, 4));
    }
  }
}

// One DSTDGCB on NTVC activations.  pq_s must already hold P/Q of x for the
// block's two spatial DSTDGCs; the block's weight images (add_block_hl_jobs)
// must be prepared when hl says so.
// xmodel (conv_st_in of the model, split spatial only): the model input
// [B][T][V][3]; the kernels build x6 and block-0's spatial P/Q from it, x is
// not read.
hipError_t run_block(const dstd_block_params* p, const BlockFold& f, const BlockScratch& sc, int B, int T, int V,
                     const float* x, float* h, float* y, const BlockTail& tail, hipStream_t s, Prof& pf,
                     const BlockHL& hl, const float* xmodel = nullptr) {
  const bool res = p->cin != p->cout;
  const bool from_model = xmodel && hl.s && p->cin == 6;
  // (1) spatial adjacency for both graphs
  AdjArgs aa{};
  aa.pq = sc.pq_s;
  aa.pql = pq_layout_vt(8, T, V);
  for (int g = 0; g < 2; ++g) {
    aa.p_ch[g] = 4 * g;
    aa.q_ch[g] = 4 * g + 2;
    aa.W[g] = p->conv_s[g].wrm;
    aa.bias[g] = p->conv_s[g].brm;
    aa.astat[g] = f.astat_s + g * V * V;
  }
  aa.mode = 0;
  aa.B = B;
  aa.T = T;
  aa.V = V;
  aa.nrow = T;
  aa.K = 2 * T;
  aa.NA = V;
  aa.ncol = V * V;
  aa.ngroups = 2;
  aa.alpha = p->alpha_sm;
  aa.out = sc.adj_s;
  if (hl.s) {  // split-f16 planes [B][2][T][2][V][SL]
    aa.hl = 1;
    aa.ncol = V * hl_sl_spatial(V);
    aa.ldo = 2 * aa.ncol;
    aa.out_sG = (long)T * aa.ncol;
    aa.out_sN = 2 * aa.out_sG;
  } else {
    aa.ldo = adj_ld_spatial(V);
    aa.out_sN = 2L * T * aa.ldo;
    aa.out_sG = (long)T * aa.ldo;
  }
  hipError_t e = hipSuccess;
  AdjHLArgs ah{};
  const bool adj_launch = !hl.s_pre && !(hl.adj0 && from_model);
  if (adj_launch) pf.begin(DSTD_KIND_ADJ_S, s);
  if (hl.s) {
    ah.pq = aa.pq;
    ah.pql = aa.pql;
    ah.B = B;
    ah.ngroups = 2;
    for (int g = 0; g < 2; ++g) {
      ah.p_ch[g] = aa.p_ch[g];
      ah.wimg[g] = f.hl_rms[g];
      ah.wscale[g] = hls(f, 5 + g);
      ah.bias[g] = f.hl_rbias + g * T;
      ah.astat[g] = aa.astat[g];
    }
    ah.alpha = aa.alpha;
    ah.out = reinterpret_cast<uint16_t*>(aa.out);
    ah.out_sN = 2 * aa.out_sN;  // halves
    ah.out_sG = 2 * aa.out_sG;
    if (from_model) {
      ah.xin = xmodel;
      for (int g = 0; g < 2; ++g) {
        ah.mw[g][0] = p->conv_s[g].wm1;
        ah.mw[g][1] = p->conv_s[g].wm2;
        ah.mb[g][0] = p->conv_s[g].bm1;
        ah.mb[g][1] = p->conv_s[g].bm2;
      }
    }
    // (s_pre: already in sc.adj_s, built by the previous block's temporal launch)
    if (adj_launch) e = launch_adj_hl(ah, 0, T, V, s);
#ifdef DSTD_SPRE_CHECK
    if (hl.s_pre) {
      const size_t n = (size_t)2 * adj_s_floats(B, T, V);  // halves
      uint16_t* ref = nullptr;
      unsigned* cnt = nullptr;
      (void)hipMalloc(&ref, n * 2);
      (void)hipMalloc(&cnt, 8);
      const unsigned init[2] = {0u, 0xffffffffu};
      (void)hipMemcpy(cnt, init, 8, hipMemcpyHostToDevice);
      AdjHLArgs ac = ah;
      ac.out = ref;
      (void)hipStreamSynchronize(s);
      (void)launch_adj_hl(ac, 0, T, V, s);
      hipLaunchKernelGGL(k_cmp_u16, dim3(1024), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(sc.adj_s), ref,
                         (size_t)B * ah.out_sN, cnt);
      unsigned h[2];
      (void)hipMemcpy(h, cnt, 8, hipMemcpyDeviceToHost);
      uint16_t va = 0, vb = 0;
      if (h[0]) {
        (void)hipMemcpy(&va, reinterpret_cast<const uint16_t*>(sc.adj_s) + h[1], 2, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&vb, ref + h[1], 2, hipMemcpyDeviceToHost);
      }
      const long i = h[1], per_n = ah.out_sN, per_g = ah.out_sG, ncol = V * hl_sl_spatial(V);
      fprintf(stderr, "spre check cin %d cout %d: %u of %ld halves differ; first %ld (n %ld g %ld t %ld plane %ld col %ld) %04x vs %04x\n",
              p->cin, p->cout, h[0], (long)B * per_n, h[0] ? i : -1L, h[0] ? i / per_n : -1L,
              h[0] ? i % per_n / per_g : -1L, h[0] ? i % per_g / (2 * ncol) : -1L,
              h[0] ? i % (2 * ncol) / ncol : -1L, h[0] ? i % ncol : -1L, va, vb);
      (void)hipFree(ref);
      (void)hipFree(cnt);
    }
#endif
  } else {
    e = launch_adj(aa, s);
  }
  if (adj_launch) pf.end(s);
  if (e != hipSuccess) return e;

  // (2) spatial GC + bn + residual + prelu, P_t/Q_t of h
  SpatialHLArgs ha{};
  if (hl.s) {
    ha.x = from_model ? xmodel : x;
    ha.xmodel = from_model ? 1 : 0;
    ha.B = B;
    ha.T = T;
    ha.V = V;
    ha.Cin = p->cin;
    ha.Cout = p->cout;
    ha.adj = reinterpret_cast<const uint16_t*>(sc.adj_s);
    for (int g = 0; g < 2; ++g) {
      ha.wimg[g] = f.hl_ws[g];
      ha.wscale[g] = hls(f, g);
      ha.adjb[g] = hls(f, 5 + g);
      ha.bf[g] = p->conv_s[g].bf;
    }
    if (res) {
      ha.wimg[2] = f.hl_ws[2];
      ha.wscale[2] = hls(f, 8);
      ha.bf[2] = p->res_b;
      ha.rbn_s = f.rbn_s;
      ha.rbn_h = f.rbn_h;
    }
    ha.bn_s = f.bn_s;
    ha.bn_h = f.bn_h;
    ha.prelu = p->prelu;
    ha.y = h;
    ha.pqimg = f.hl_pqs;
    ha.pqscale = hls(f, 2);
    ha.pqb[0] = p->conv_t.bm1;
    ha.pqb[1] = p->conv_t.bm2;
    ha.pq = sc.pq_t;
    if (!hl.bf) {  // (k_block_fused runs it with the temporal GC, step 4)
      pf.begin(DSTD_KIND_SPATIAL, s);
      e = launch_spatial_hl(ha, s);
      pf.end(s);
      if (e != hipSuccess) return e;
    }
  } else {
  SpatialArgs sa{};
  sa.x = x;
  sa.B = B;
  sa.T = T;
  sa.V = V;
  sa.Cin = p->cin;
  sa.Cout = p->cout;
  sa.NI = 2;
  sa.G = res ? 3 : 2;
  sa.adj = sc.adj_s;
  sa.adj_ld = adj_ld_spatial(V);
  for (int g = 0; g < 2; ++g) {
    sa.wf[g] = p->conv_s[g].wf;
    sa.bf[g] = p->conv_s[g].bf;
  }
  sa.wf[2] = res ? p->res_w : nullptr;
  sa.bf[2] = res ? p->res_b : nullptr;
  sa.epi = 1;
  sa.bn_s = f.bn_s;
  sa.bn_h = f.bn_h;
  sa.rbn_s = f.rbn_s;
  sa.rbn_h = f.rbn_h;
  sa.prelu = p->prelu;
  sa.y = h;
  sa.pqw[0] = p->conv_t.wm1;
  sa.pqw[1] = p->conv_t.wm2;
  sa.pqb[0] = p->conv_t.bm1;
  sa.pqb[1] = p->conv_t.bm2;
  sa.npqw = 2;
  sa.pq = sc.pq_t;
  sa.pql = pq_layout_tv(4, T, V);
  sa.Tt = 0;
  pf.begin(DSTD_KIND_SPATIAL, s);
  e = launch_spatial(sa, s);
  pf.end(s);
  if (e != hipSuccess) return e;
  }

  // (3) temporal adjacency
  AdjArgs ta{};
  ta.pq = sc.pq_t;
  ta.pql = pq_layout_tv(4, T, V);
  ta.p_ch[0] = 0;
  ta.q_ch[0] = 2;
  ta.W[0] = p->conv_t.wrm;
  ta.bias[0] = p->conv_t.brm;
  ta.astat[0] = f.astat_t;
  ta.mode = 1;
  ta.B = B;
  ta.T = T;
  ta.V = V;
  ta.nrow = V;
  ta.K = 2 * V;
  ta.NA = T;
  ta.ncol = T * T;
  ta.ngroups = 1;
  ta.alpha = p->alpha_tm;
  ta.out = sc.adj_t;
  ta.out_sG = 0;
  if (hl.t) {  // split-f16 planes [B][V][2][T][SL]
    ta.hl = 1;
    ta.ncol = T * hl_sl_temporal(T);
    ta.ldo = 2 * ta.ncol;
    ta.out_sN = (long)V * ta.ncol;
  } else {
    ta.ldo = adj_ld_temporal(T);
    ta.out_sN = (long)V * ta.ldo;
  }
  AdjHLArgs aht{};
  if (hl.t) {
    aht.pq = ta.pq;
    aht.pql = ta.pql;
    aht.B = B;
    aht.ngroups = 1;
    aht.p_ch[0] = ta.p_ch[0];
    aht.wimg[0] = f.hl_rmt;
    aht.wscale[0] = hls(f, 7);
    aht.bias[0] = f.hl_rbias + 2 * T;
    aht.astat[0] = ta.astat[0];
    aht.alpha = ta.alpha;
    aht.out = reinterpret_cast<uint16_t*>(ta.out);
    aht.out_sN = 2 * ta.out_sN;
    aht.out_sG = 0;
  }
  if (!hl.tf) {  // the fused temporal kernel builds its adjacency itself
    pf.begin(DSTD_KIND_ADJ_T, s);
    e = hl.t ? launch_adj_hl(aht, 1, T, V, s) : launch_adj(ta, s);
    pf.end(s);
    if (e != hipSuccess) return e;
  }

  // (4) temporal GC + tail epilogue (+ next block's spatial P/Q)
  if (hl.t) {
    TemporalHLArgs ht{};
    ht.h = h;
    ht.B = B;
    ht.T = T;
    ht.V = V;
    ht.C = p->cout;
    ht.adj = reinterpret_cast<const uint16_t*>(sc.adj_t);
    ht.wimg = f.hl_wt;
    ht.wscale = hls(f, 3);
    ht.adjb = hls(f, 7);
    ht.bf = p->conv_t.bf;
    ht.epi = tail.epi;
    ht.xres = tail.xres;
    ht.bn_s = tail.bn_s;
    ht.bn_h = tail.bn_h;
    ht.prelu = tail.prelu;
    ht.y = y;
    if (tail.next) {
      const dstd_block_params* q = tail.next;
      ht.pqimg = f.hl_pqt;
      ht.pqscale = hls(f, 4);
      ht.pqb[0] = q->conv_s[0].bm1;
      ht.pqb[1] = q->conv_s[0].bm2;
      ht.pqb[2] = q->conv_s[1].bm1;
      ht.pqb[3] = q->conv_s[1].bm2;
      ht.pq = sc.pq_s;
    }
    // the next block's spatial adjacency (its launch_adj_hl mode 0 arguments)
    AdjHLArgs sn{};
    if (tail.next_adj) {
      const dstd_block_params* q = tail.next;
      const BlockFold& nf = *tail.next_f;
      const int ncol = V * hl_sl_spatial(V);
      sn.pq = sc.pq_s;
      sn.pql = pq_layout_vt(8, T, V);
      sn.B = B;
      sn.ngroups = 2;
      for (int g = 0; g < 2; ++g) {
        sn.p_ch[g] = 4 * g;
        sn.wimg[g] = nf.hl_rms[g];
        sn.wscale[g] = hls(nf, 5 + g);
        sn.bias[g] = nf.hl_rbias + g * T;
        sn.astat[g] = nf.astat_s + g * V * V;
      }
      sn.alpha = q->alpha_sm;
      sn.out = reinterpret_cast<uint16_t*>(sc.adj_s);
      sn.out_sG = 2L * T * ncol;  // halves
      sn.out_sN = 2 * sn.out_sG;
    }
    if (hl.bf) {
      pf.begin(DSTD_KIND_BLOCK, s);
      e = launch_block_fused(ha, ht, aht, tail.next_adj ? &sn : nullptr, s, hl.adj0 && from_model ? &ah : nullptr);
      pf.end(s);
      return e;
    }
    pf.begin(DSTD_KIND_TEMPORAL, s);
    e = hl.tf ? launch_temporal_fused(ht, aht, tail.next_adj ? &sn : nullptr, s) : launch_temporal_hl(ht, s);
    pf.end(s);
    return e;
  }
  TemporalArgs tt{};
  tt.h = h;
  tt.B = B;
  tt.T = T;
  tt.V = V;
  tt.Cin = p->cout;
  tt.Cout = p->cout;
  tt.adj = sc.adj_t;
  tt.adj_ld = adj_ld_temporal(T);
  tt.wf = p->conv_t.wf;
  tt.bf = p->conv_t.bf;
  tt.epi = tail.epi;
  tt.xres = tail.xres;
  tt.bn_s = tail.bn_s;
  tt.bn_h = tail.bn_h;
  tt.prelu = tail.prelu;
  tt.y = y;
  if (tail.next) {
    const dstd_block_params* q = tail.next;
    tt.pqw[0] = q->conv_s[0].wm1;
    tt.pqw[1] = q->conv_s[0].wm2;
    tt.pqw[2] = q->conv_s[1].wm1;
    tt.pqw[3] = q->conv_s[1].wm2;
    tt.pqb[0] = q->conv_s[0].bm1;
    tt.pqb[1] = q->conv_s[0].bm2;
    tt.pqb[2] = q->conv_s[1].bm1;
    tt.pqb[3] = q->conv_s[1].bm2;
    tt.npqw = 4;
    tt.pq = sc.pq_s;
    tt.pql = pq_layout_vt(8, T, V);
  }
  tt.Vt = 0;
  pf.begin(DSTD_KIND_TEMPORAL, s);
  e = launch_temporal(tt, s);
  pf.end(s);
  return e;
}

hipError_t spatial_pq(const dstd_block_params* p, const float* x_ntvc, int B, int T, int V, float* pq_s,
                      hipStream_t s) {
  PQArgs pa{};
  pa.x = x_ntvc;
  pa.B = B;
  pa.T = T;
  pa.V = V;
  pa.Cin = p->cin;
  pa.w[0] = p->conv_s[0].wm1;
  pa.w[1] = p->conv_s[0].wm2;
  pa.w[2] = p->conv_s[1].wm1;
  pa.w[3] = p->conv_s[1].wm2;
  pa.b[0] = p->conv_s[0].bm1;
  pa.b[1] = p->conv_s[0].bm2;
  pa.b[2] = p->conv_s[1].bm1;
  pa.b[3] = p->conv_s[1].bm2;
  pa.nw = 4;
  pa.pq = pq_s;
  pa.pql = pq_layout_vt(8, T, V);
  return launch_pq(pa, s);
}

// ---- layouts ---------------------------------------------------------------
struct OpLayout {
  float* xin;
  float* yout;
  float* pq;
  float* adj;
};
void carve_op(Carver& cv, OpLayout& L, int mode, int B, int cin, int cout, int T, int V) {
  L.xin = cv.take((size_t)B * T * V * cin);
  L.yout = cv.take((size_t)B * T * V * cout);
  L.pq = cv.take((size_t)B * 4 * T * V);
  L.adj = cv.take(mode == DSTD_MODE_SPATIAL ? (size_t)B * T * adj_ld_spatial(V) : (size_t)B * V * adj_ld_temporal(T));
}

struct BlockLayout {
  float* xin;
  float* h;
  float* yout;
  BlockFold f;
  BlockScratch sc;
};
void carve_block(Carver& cv, BlockLayout& L, int B, int cin, int cout, int T, int V) {
  L.xin = cv.take((size_t)B * T * V * cin);
  L.h = cv.take((size_t)B * T * V * cout);
  L.yout = cv.take((size_t)B * T * V * cout);
  carve_fold(cv, L.f, T, V, cout, cin != cout);
  carve_scratch(cv, L.sc, B, T, V);
}

struct ModelLayout {
  float* act[3];
  BlockFold f_in, f_out, f_enc[DSTD_MAX_LAYERS];
  float* bnin_s;
  float* bnin_h;
  float* ebn_s[DSTD_MAX_LAYERS];
  float* ebn_h[DSTD_MAX_LAYERS];
  BlockScratch sc;
};
void carve_model(Carver& cv, ModelLayout& L, int B, int T, int V, int C, int layers, int cin_model,
                 int cout_model) {
  for (int i = 0; i < 3; ++i) L.act[i] = cv.take((size_t)B * T * V * C);
  carve_fold(cv, L.f_in, T, V, C, cin_model != C);
  carve_fold(cv, L.f_out, T, V, cout_model, C != cout_model);
  for (int i = 0; i < layers; ++i) {
    carve_fold(cv, L.f_enc[i], T, V, C, false);
    L.ebn_s[i] = cv.take((size_t)C * V);
    L.ebn_h[i] = cv.take((size_t)C * V);
  }
  L.bnin_s = cv.take((size_t)C * V);
  L.bnin_h = cv.take((size_t)C * V);
  carve_scratch(cv, L.sc, B, T, V);
}

hipError_t to_layout(const float* src, float* dst, int B, int C, int TV, int to_ntvc, hipStream_t s) {
  TransposeArgs t{src, dst, B, C, TV, to_ntvc};
  return launch_transpose(t, s);
}

}  // namespace

extern "C" {

const char* dstd_version(void) { return "dstd-gcn-mi355x 0.2 (gfx950; forward: split-f16 MFMA 16x16x32, fp32 storage / accumulate; training: fp32 MFMA 16x16x4)"; }

const char* dstd_error_string(int code) {
  switch (code) {
    case DSTD_OK: return "ok";
    case DSTD_EINVAL: return "invalid argument (null pointer or bad shape)";
    case DSTD_EWORKSPACE: return "workspace too small";
    case DSTD_ELIMIT: return "shape outside the supported envelope (T<=128, V<=32, C<=64)";
    case DSTD_ECOLLECTIVE: return "the dstd_bn_sync collective returned an error (SyncBN)";
    default: return code > 0 ? hipGetErrorString((hipError_t)code) : "unknown error";
  }
}

size_t dstd_dstdgc_workspace_bytes(int mode, int B, int cin, int cout, int T, int V) {
  Carver cv{nullptr};
  OpLayout L;
  carve_op(cv, L, mode, B, cin, cout, T, V);
  return cv.off + 256;
}

size_t dstd_block_workspace_bytes(int B, int cin, int cout, int T, int V) {
  Carver cv{nullptr};
  BlockLayout L;
  carve_block(cv, L, B, cin, cout, T, V);
  return cv.off + 256;
}

size_t dstd_model_workspace_bytes(int B, int T, int V, int num_feature, int num_layers) {
  Carver cv{nullptr};
  ModelLayout L;
  carve_model(cv, L, B, T, V, num_feature, num_layers, 6, 3);
  return cv.off + 256;
}

int dstd_dstdgc_fwd(int mode, const float* x, int B, int cin, int cout, int T, int V, const dstd_gc_weights* w,
                    const float* A, const float* alpha, float* y, void* workspace, size_t workspace_bytes,
                    void* stream) {
  StreamDeviceGuard dev_guard_(stream, x);
  if (!x || !y || !A || !alpha || !gc_ok(w) || !workspace || !shape_ok(B, T, V)) return DSTD_EINVAL;
  if (mode != DSTD_MODE_SPATIAL && mode != DSTD_MODE_TEMPORAL) return DSTD_EINVAL;
  if (!limits_ok(T, V, cin, cout)) return DSTD_ELIMIT;
  if (workspace_bytes < dstd_dstdgc_workspace_bytes(mode, B, cin, cout, T, V)) return DSTD_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  Carver cv{(char*)workspace};
  OpLayout L;
  carve_op(cv, L, mode, B, cin, cout, T, V);
  const int TV = T * V;
  DSTD_TRY(to_layout(x, L.xin, B, cin, TV, 1, s));
  PQArgs pa{};
  pa.x = L.xin;
  pa.B = B;
  pa.T = T;
  pa.V = V;
  pa.Cin = cin;
  pa.w[0] = w->wm1;
  pa.w[1] = w->wm2;
  pa.b[0] = w->bm1;
  pa.b[1] = w->bm2;
  pa.nw = 2;
  pa.pq = L.pq;
  pa.pql = pq_layout_tv(4, T, V);
  DSTD_TRY(launch_pq(pa, s));
  AdjArgs aa{};
  aa.pq = L.pq;
  aa.pql = pa.pql;
  aa.p_ch[0] = 0;
  aa.q_ch[0] = 2;
  aa.W[0] = w->wrm;
  aa.bias[0] = w->brm;
  aa.astat[0] = A;  // the caller's combined adjacency is row independent
  aa.mode = mode;
  aa.B = B;
  aa.T = T;
  aa.V = V;
  aa.ngroups = 1;
  aa.alpha = alpha;
  aa.out = L.adj;
  aa.out_sG = 0;
  if (mode == DSTD_MODE_SPATIAL) {
    aa.nrow = T;
    aa.K = 2 * T;
    aa.NA = V;
    aa.ncol = V * V;
    aa.ldo = adj_ld_spatial(V);
    aa.out_sN = (long)T * aa.ldo;
  } else {
    aa.nrow = V;
    aa.K = 2 * V;
    aa.NA = T;
    aa.ncol = T * T;
    aa.ldo = adj_ld_temporal(T);
    aa.out_sN = (long)V * aa.ldo;
  }
  DSTD_TRY(launch_adj(aa, s));
  if (mode == DSTD_MODE_SPATIAL) {
    SpatialArgs sa{};
    sa.x = L.xin;
    sa.B = B;
    sa.T = T;
    sa.V = V;
    sa.Cin = cin;
    sa.Cout = cout;
    sa.NI = 1;
    sa.G = 1;
    sa.adj = L.adj;
    sa.adj_ld = adj_ld_spatial(V);
    sa.wf[0] = w->wf;
    sa.bf[0] = w->bf;
    sa.epi = 0;
    sa.y = L.yout;
    DSTD_TRY(launch_spatial(sa, s));
  } else {
    TemporalArgs ta{};
    ta.h = L.xin;
    ta.B = B;
    ta.T = T;
    ta.V = V;
    ta.Cin = cin;
    ta.Cout = cout;
    ta.adj = L.adj;
    ta.adj_ld = adj_ld_temporal(T);
    ta.wf = w->wf;
    ta.bf = w->bf;
    ta.epi = TEPI_RAW;
    ta.y = L.yout;
    DSTD_TRY(launch_temporal(ta, s));
  }
  DSTD_TRY(to_layout(L.yout, y, B, cout, TV, 0, s));
  return DSTD_OK;
}

int dstd_block_fwd(const dstd_block_params* p, const float* x, int B, int T, int V, float* y, void* workspace,
                   size_t workspace_bytes, void* stream) {
  return dstd_block_fwd_ex(p, x, B, T, V, y, workspace, workspace_bytes, stream, 0u);
}

int dstd_block_fwd_ex(const dstd_block_params* p, const float* x, int B, int T, int V, float* y, void* workspace,
                      size_t workspace_bytes, void* stream, unsigned flags) {
  StreamDeviceGuard dev_guard_(stream, x);
  if (flags & ~(DSTD_FWD_EXACT_FP32 | DSTD_FWD_FUSED_TEMPORAL | DSTD_FWD_SEPARATE_BLOCK)) return DSTD_EINVAL;
  if (!x || !y || !workspace || !block_ok(p) || !shape_ok(B, T, V)) return DSTD_EINVAL;
  if (!limits_ok(T, V, p->cin, p->cout)) return DSTD_ELIMIT;
  if (workspace_bytes < dstd_block_workspace_bytes(B, p->cin, p->cout, T, V)) return DSTD_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  Carver cv{(char*)workspace};
  BlockLayout L;
  carve_block(cv, L, B, p->cin, p->cout, T, V);
  FoldList fa;
  add_block_jobs(fa, p, L.f, T, V);
  DSTD_TRY(run_fold(fa, s));
  DSTD_TRY(to_layout(x, L.xin, B, p->cin, T * V, 1, s));
  DSTD_TRY(spatial_pq(p, L.xin, B, T, V, L.sc.pq_s, s));
  BlockTail tail{TEPI_RAW, nullptr, nullptr, nullptr, nullptr, nullptr};
  const BlockHL hl = block_hl(p, tail, B, T, V, flags);
  HLList hj;
  add_block_hl_jobs(hj, p, L.f, tail, hl, T, V);
  DSTD_TRY(run_hl_prep(hj, s));
  Prof pf;
  DSTD_TRY(run_block(p, L.f, L.sc, B, T, V, L.xin, L.h, L.yout, tail, s, pf, hl));
  DSTD_TRY(to_layout(L.yout, y, B, p->cout, T * V, 0, s));
  return DSTD_OK;
}

int dstd_model_fwd(const dstd_model_params* p, const float* x, int B, float* y, void* workspace,
                   size_t workspace_bytes, void* stream) {
  return dstd_model_fwd_ex(p, x, B, y, workspace, workspace_bytes, stream, 0u, nullptr);
}

int dstd_model_fwd_profiled(const dstd_model_params* p, const float* x, int B, float* y, void* workspace,
                            size_t workspace_bytes, void* stream, dstd_profile* prof) {
  return dstd_model_fwd_ex(p, x, B, y, workspace, workspace_bytes, stream, 0u, prof);
}

int dstd_model_fwd_ex(const dstd_model_params* p, const float* x, int B, float* y, void* workspace,
                      size_t workspace_bytes, void* stream, unsigned flags, dstd_profile* prof) {
  StreamDeviceGuard dev_guard_(stream, x);
  const bool reuse = (flags & DSTD_FWD_REUSE_CONSTANTS) != 0;
  if (flags & ~(DSTD_FWD_REUSE_CONSTANTS | DSTD_FWD_EXACT_FP32 | DSTD_FWD_SEPARATE_ADJ | DSTD_FWD_FUSED_TEMPORAL |
                DSTD_FWD_SEPARATE_BLOCK))
    return DSTD_EINVAL;
  if (!p || !x || !y || !workspace) return DSTD_EINVAL;
  if (prof && (prof->capacity < 0 || (prof->capacity > 0 && (!prof->events || !prof->kinds)))) return DSTD_EINVAL;
  Prof pf;
  pf.p = prof;
  const int T = p->T, V = p->V, C = p->num_feature, L_ = p->num_layers;
  if (!shape_ok(B, T, V) || L_ < 0 || L_ > DSTD_MAX_LAYERS || p->in_channels != 6) return DSTD_EINVAL;
  if (!limits_ok(T, V, p->in_channels, C)) return DSTD_ELIMIT;
  if (!block_ok(&p->st_in) || !block_ok(&p->st_out) || !bn_ok(p->bn_in) || !p->prelu) return DSTD_EINVAL;
  if (p->st_in.cin != 6 || p->st_in.cout != C || p->st_out.cin != C || p->st_out.cout != 3) return DSTD_EINVAL;
  for (int i = 0; i < L_; ++i) {
    if (!block_ok(&p->enc[i]) || !bn_ok(p->enc_bn[i]) || !p->enc_prelu[i]) return DSTD_EINVAL;
    if (p->enc[i].cin != C || p->enc[i].cout != C) return DSTD_EINVAL;
  }
  if (workspace_bytes < dstd_model_workspace_bytes(B, T, V, C, L_)) return DSTD_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  Carver cv{(char*)workspace};
  ModelLayout L;
  carve_model(cv, L, B, T, V, C, L_, 6, 3);

  FoldList fa;
  add_block_jobs(fa, &p->st_in, L.f_in, T, V);
  add_block_jobs(fa, &p->st_out, L.f_out, T, V);
  add_bn_job(fa, p->bn_in, C, V, L.bnin_s, L.bnin_h);
  for (int i = 0; i < L_; ++i) {
    add_block_jobs(fa, &p->enc[i], L.f_enc[i], T, V);
    add_bn_job(fa, p->enc_bn[i], C, V, L.ebn_s[i], L.ebn_h[i]);
  }
  if (!reuse) {
    pf.begin(DSTD_KIND_FOLD, s);
    DSTD_TRY(run_fold(fa, s));
    pf.end(s);
  }

  // conv_st_in -> bn_in -> prelu (dropout is identity in eval); encoders
  // x = prelu_e(bn_e(DSTDGCB(x) + x)); conv_st_out + output residual written
  // straight into y [B][T][V][3].  Buffers rotate over act[0..2].
  const int NB = L_ + 2;
  const dstd_block_params* blk[DSTD_MAX_LAYERS + 2];
  const BlockFold* fold[DSTD_MAX_LAYERS + 2];
  BlockTail tails[DSTD_MAX_LAYERS + 2];
  BlockHL hls[DSTD_MAX_LAYERS + 2];
  const float* xin[DSTD_MAX_LAYERS + 2];
  float* hbuf[DSTD_MAX_LAYERS + 2];
  float* ybuf[DSTD_MAX_LAYERS + 2];
  {
    float* cur = L.act[0];
    float* h = L.act[1];
    float* out = L.act[2];
    blk[0] = &p->st_in;
    fold[0] = &L.f_in;
    tails[0] = BlockTail{TEPI_IN, nullptr, L.bnin_s, L.bnin_h, p->prelu, L_ > 0 ? &p->enc[0] : &p->st_out};
    xin[0] = cur;
    hbuf[0] = h;
    ybuf[0] = out;
    for (int i = 0; i < L_; ++i) {
      float* xi = out;
      float* hh = cur;
      float* yy = h;
      blk[1 + i] = &p->enc[i];
      fold[1 + i] = &L.f_enc[i];
      tails[1 + i] = BlockTail{TEPI_ENC, xi, L.ebn_s[i], L.ebn_h[i], p->enc_prelu[i], i + 1 < L_ ? &p->enc[i + 1] : &p->st_out};
      xin[1 + i] = xi;
      hbuf[1 + i] = hh;
      ybuf[1 + i] = yy;
      cur = xi;
      h = hh;
      out = yy;
    }
    blk[NB - 1] = &p->st_out;
    fold[NB - 1] = &L.f_out;
    tails[NB - 1] = BlockTail{TEPI_OUT, x, nullptr, nullptr, nullptr, nullptr};
    xin[NB - 1] = out;
    hbuf[NB - 1] = h;
    ybuf[NB - 1] = y;
  }
  HLList hj;
  for (int b = 0; b < NB; ++b) {
    hls[b] = block_hl(blk[b], tails[b], B, T, V, flags);
    add_block_hl_jobs(hj, blk[b], *fold[b], tails[b], hls[b], T, V);
  }
#ifndef DSTD_NO_SPRE
  // a block's spatial adjacency from the previous block's fused temporal
  // launch (phase 3), which writes the P/Q it is built from
  for (int b = 1; b < NB && !(flags & DSTD_FWD_SEPARATE_ADJ); ++b)
    if (hls[b].s && hls[b - 1].tf && blk[b - 1]->cout == 64 && temporal_fused_phase3(T, V)) {
      hls[b].s_pre = true;
      tails[b - 1].next_f = fold[b];
      tails[b - 1].next_adj = true;
    }
#endif
  // block 0's spatial planes (from the model input) inside its block launch
  // rather than a k_adj_hl<0> launch of their own
  if (hls[0].bf && !(flags & DSTD_FWD_SEPARATE_ADJ) && blk[0]->cin == 6 && block_fused_adj0_supported(T, V))
    hls[0].adj0 = true;

  // input prep: x6 = cat(x, x - x[:, -1]) and block-0 spatial P/Q (:298-305)
  PQArgs pa{};
  pa.x = x;
  pa.B = B;
  pa.T = T;
  pa.V = V;
  pa.Cin = 6;
  pa.make_x6 = 1;
  pa.x6 = L.act[0];
  const dstd_block_params* b0 = &p->st_in;
  pa.w[0] = b0->conv_s[0].wm1;
  pa.w[1] = b0->conv_s[0].wm2;
  pa.w[2] = b0->conv_s[1].wm1;
  pa.w[3] = b0->conv_s[1].wm2;
  pa.b[0] = b0->conv_s[0].bm1;
  pa.b[1] = b0->conv_s[0].bm2;
  pa.b[2] = b0->conv_s[1].bm1;
  pa.b[3] = b0->conv_s[1].bm2;
  pa.nw = 4;
  pa.pq = L.sc.pq_s;
  pa.pql = pq_layout_vt(8, T, V);
  if (!hls[0].s) {  // the split kernels build x6 and these P/Q from x themselves
    pf.begin(DSTD_KIND_PREP, s);
    DSTD_TRY(launch_pq(pa, s));
    pf.end(s);
  }

  if (!reuse) {
    pf.begin(DSTD_KIND_FOLD, s);
    DSTD_TRY(run_hl_prep(hj, s));
    pf.end(s);
  }
  for (int b = 0; b < NB; ++b) {
    pf.block = b;
    DSTD_TRY(run_block(blk[b], *fold[b], L.sc, B, T, V, xin[b], hbuf[b], ybuf[b], tails[b], s, pf, hls[b],
                       b == 0 ? x : nullptr));
  }
  return DSTD_OK;
}


int dstd_events_create(int n, void** events) {
  if (n < 0 || (n > 0 && !events)) return DSTD_EINVAL;
  for (int i = 0; i < n; ++i) {
    hipEvent_t e;
    DSTD_TRY(hipEventCreate(&e));
    events[i] = (void*)e;
  }
  return DSTD_OK;
}

int dstd_events_destroy(int n, void** events) {
  if (n < 0 || (n > 0 && !events)) return DSTD_EINVAL;
  for (int i = 0; i < n; ++i)
    if (events[i]) DSTD_TRY(hipEventDestroy((hipEvent_t)events[i]));
  return DSTD_OK;
}

int dstd_event_elapsed_ms(void* start, void* stop, float* ms) {
  if (!start || !stop || !ms) return DSTD_EINVAL;
  return (int)hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop);
}

}  // extern "C"
