// The reference's non-refine ST_GCNN_layer branch (include/dstd_gcn_aux.h):
// ConvTemporalGraphical as strided GEMMs on the training GEMM kernel, and a
// k_t x k_v Conv2d (1x1 / stride 1 / no padding goes to the GEMM; anything else
// to direct kernels).  Dead code in every shipped config, so the
// kernels favour simplicity.
#include <algorithm>

#include "../../include/dstd_gcn.h"
#include "../../include/dstd_gcn_aux.h"
#include "dstd_common.h"
#include "dstd_train.h"

using namespace dstd::train;

namespace {

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

struct CtgWs {
  float *x1, *dx1, *gs;
};
void carve_ctg(Carver& cv, CtgWs& w, int B, int C, int T, int V) {
  w.x1 = cv.take((size_t)B * C * T * V);
  w.dx1 = cv.take((size_t)B * C * T * V);
  w.gs = cv.take(gemm_scratch_floats(std::max(T, V), std::max(T, V)));
}

// x1[n,c,q,v] = sum_t x[n,c,t,v] Tm[v,t,q]      (model/dstdgcn.py:186)
Gemm ctg_time(const float* x, const float* Tm, float* x1, int B, int C, int T, int V) {
  const long long TV = (long long)T * V;
  Gemm g;
  g.M = C, g.N = T, g.K = T, g.nb1 = B, g.nb2 = V;
  g.A = x, g.a_b1 = C * TV, g.a_b2 = 1, g.a_m = TV, g.a_k = V;
  g.B = Tm, g.b_b1 = 0, g.b_b2 = (long long)T * T, g.b_k = T, g.b_n = 1;
  g.C = x1, g.c_b1 = C * TV, g.c_b2 = 1, g.c_m = TV, g.c_n = V;
  return g;
}

// y[n,c,t,w] (+)= sum_v x1[n,c,t,v] S[t,v,w] with S batch stride sS (0: A_fixed broadcast)   (:187)
Gemm ctg_space(const float* x1, const float* S, long long sS, float* y, int B, int C, int T, int V, float beta) {
  const long long TV = (long long)T * V;
  Gemm g;
  g.M = C, g.N = V, g.K = V, g.nb1 = B, g.nb2 = T;
  g.A = x1, g.a_b1 = C * TV, g.a_b2 = V, g.a_m = TV, g.a_k = 1;
  g.B = S, g.b_b1 = 0, g.b_b2 = sS, g.b_k = V, g.b_n = 1;
  g.C = y, g.c_b1 = C * TV, g.c_b2 = V, g.c_m = TV, g.c_n = 1;
  g.beta = beta;
  return g;
}

// ---- direct KxK convolution -------------------------------------------------
struct ConvGeom {
  int B, cin, H, W, cout, kh, kw, sh, sw, ph, pw, Ho, Wo;
};

__global__ void k_conv2d_fwd(const float* x, const float* w, const float* bias, ConvGeom g, float* y) {
  const size_t tot = (size_t)g.B * g.cout * g.Ho * g.Wo;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    size_t r = e;
    const int wo = r % g.Wo; r /= g.Wo;
    const int ho = r % g.Ho; r /= g.Ho;
    const int o = r % g.cout;
    const int n = r / g.cout;
    float s = bias ? bias[o] : 0.f;
    for (int i = 0; i < g.cin; ++i)
      for (int dh = 0; dh < g.kh; ++dh) {
        const int h = ho * g.sh + dh - g.ph;
        if (h < 0 || h >= g.H) continue;
        for (int dw = 0; dw < g.kw; ++dw) {
          const int wi = wo * g.sw + dw - g.pw;
          if (wi < 0 || wi >= g.W) continue;
          s = fmaf(w[((o * g.cin + i) * g.kh + dh) * g.kw + dw], x[(((size_t)n * g.cin + i) * g.H + h) * g.W + wi], s);
        }
      }
    y[e] = s;
  }
}

__global__ void k_conv2d_bwd_data(const float* dy, const float* w, ConvGeom g, float* dx) {
  const size_t tot = (size_t)g.B * g.cin * g.H * g.W;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    size_t r = e;
    const int wi = r % g.W; r /= g.W;
    const int h = r % g.H; r /= g.H;
    const int i = r % g.cin;
    const int n = r / g.cin;
    float s = 0.f;
    for (int dh = 0; dh < g.kh; ++dh) {
      const int hn = h + g.ph - dh;
      if (hn < 0 || hn % g.sh) continue;
      const int ho = hn / g.sh;
      if (ho >= g.Ho) continue;
      for (int dw = 0; dw < g.kw; ++dw) {
        const int wn = wi + g.pw - dw;
        if (wn < 0 || wn % g.sw) continue;
        const int wo = wn / g.sw;
        if (wo >= g.Wo) continue;
        for (int o = 0; o < g.cout; ++o)
          s = fmaf(w[((o * g.cin + i) * g.kh + dh) * g.kw + dw],
                   dy[(((size_t)n * g.cout + o) * g.Ho + ho) * g.Wo + wo], s);
      }
    }
    dx[e] += s;
  }
}

// one workgroup per weight element (o, i, dh, dw), fixed-order block sum
__global__ __launch_bounds__(256) void k_conv2d_bwd_weight(const float* x, const float* dy, ConvGeom g, float* dwt) {
  __shared__ float red[4];
  const int widx = blockIdx.x;
  int r = widx;
  const int dw = r % g.kw; r /= g.kw;
  const int dh = r % g.kh; r /= g.kh;
  const int i = r % g.cin;
  const int o = r / g.cin;
  const size_t tot = (size_t)g.B * g.Ho * g.Wo;
  float s = 0.f;
  for (size_t e = threadIdx.x; e < tot; e += blockDim.x) {
    size_t q = e;
    const int wo = q % g.Wo; q /= g.Wo;
    const int ho = q % g.Ho;
    const int n = q / g.Ho;
    const int h = ho * g.sh + dh - g.ph, wi = wo * g.sw + dw - g.pw;
    if (h < 0 || h >= g.H || wi < 0 || wi >= g.W) continue;
    s = fmaf(x[(((size_t)n * g.cin + i) * g.H + h) * g.W + wi], dy[(((size_t)n * g.cout + o) * g.Ho + ho) * g.Wo + wo],
             s);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) dwt[widx] += red[0] + red[1] + red[2] + red[3];
}

int grid_of(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 8192); }

bool conv_geom(ConvGeom& g, int B, int cin, int H, int W, int cout, int kh, int kw, int sh, int sw, int ph, int pw) {
  if (B <= 0 || cin <= 0 || H <= 0 || W <= 0 || cout <= 0 || kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0 || ph < 0 ||
      pw < 0)
    return false;
  g = ConvGeom{B, cin, H, W, cout, kh, kw, sh, sw, ph, pw, (H + 2 * ph - kh) / sh + 1, (W + 2 * pw - kw) / sw + 1};
  return g.Ho > 0 && g.Wo > 0;
}

bool is_pointwise(const ConvGeom& g) { return g.kh == 1 && g.kw == 1 && g.sh == 1 && g.sw == 1 && !g.ph && !g.pw; }

}  // namespace

extern "C" {

size_t dstd_ctg_workspace_bytes(int B, int C, int T, int V) {
  Carver cv{nullptr};
  CtgWs w;
  carve_ctg(cv, w, B, C, T, V);
  return cv.off + 256;
}

int dstd_ctg_fwd(const float* x, int B, int C, int T, int V, const float* Tm, const float* A, const float* A_fixed,
                 float* y, void* workspace, size_t workspace_bytes, void* stream) {
  StreamDeviceGuard dev_guard_(stream, x);
  if (!x || !Tm || !A || !A_fixed || !y || !workspace || B <= 0 || C <= 0 || T <= 0 || V <= 0) return DSTD_EINVAL;
  if (workspace_bytes < dstd_ctg_workspace_bytes(B, C, T, V)) return DSTD_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  Carver cv{(char*)workspace};
  CtgWs w;
  carve_ctg(cv, w, B, C, T, V);
  DSTD_TRY(gemm(ctg_time(x, Tm, w.x1, B, C, T, V), nullptr, s));
  DSTD_TRY(gemm(ctg_space(w.x1, A, (long long)V * V, y, B, C, T, V, 0.f), nullptr, s));
  DSTD_TRY(gemm(ctg_space(w.x1, A_fixed, 0, y, B, C, T, V, 1.f), nullptr, s));
  return DSTD_OK;
}

int dstd_ctg_bwd(const float* x, int B, int C, int T, int V, const float* Tm, const float* A, const float* A_fixed,
                 const float* dy, float* dx, float* dTm, float* dA, void* workspace, size_t workspace_bytes,
                 void* stream) {
  StreamDeviceGuard dev_guard_(stream, x);
  if (!x || !Tm || !A || !A_fixed || !dy || !dTm || !dA || !workspace || B <= 0 || C <= 0 || T <= 0 || V <= 0)
    return DSTD_EINVAL;
  if (workspace_bytes < dstd_ctg_workspace_bytes(B, C, T, V)) return DSTD_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  Carver cv{(char*)workspace};
  CtgWs w;
  carve_ctg(cv, w, B, C, T, V);
  const long long TV = (long long)T * V;
  DSTD_TRY(gemm(ctg_time(x, Tm, w.x1, B, C, T, V), nullptr, s));  // recompute x1
  // dx1[n,c,t,v] = sum_w dy[n,c,t,w] S[t,v,w]
  for (int part = 0; part < 2; ++part) {
    Gemm g;
    g.M = C, g.N = V, g.K = V, g.nb1 = B, g.nb2 = T;
    g.A = dy, g.a_b1 = C * TV, g.a_b2 = V, g.a_m = TV, g.a_k = 1;
    g.B = part ? A_fixed : A, g.b_b1 = 0, g.b_b2 = part ? 0 : (long long)V * V, g.b_k = 1, g.b_n = V;
    g.C = w.dx1, g.c_b1 = C * TV, g.c_b2 = V, g.c_m = TV, g.c_n = 1;
    g.beta = part ? 1.f : 0.f;
    DSTD_TRY(gemm(g, nullptr, s));
  }
  // dA[t] += x1_t^T dy_t, contracting (n, c) (uniform stride T*V)
  Gemm ga;
  ga.M = V, ga.N = V, ga.K = B * C, ga.nb1 = T;
  ga.A = w.x1, ga.a_b1 = V, ga.a_m = 1, ga.a_k = TV;
  ga.B = dy, ga.b_b1 = V, ga.b_k = TV, ga.b_n = 1;
  ga.C = dA, ga.c_b1 = (long long)V * V, ga.c_m = V, ga.c_n = 1;
  ga.beta = 1.f;
  DSTD_TRY(gemm(ga, nullptr, s));
  // dTm[v] += x_v^T dx1_v, contracting (n, c)
  Gemm gt;
  gt.M = T, gt.N = T, gt.K = B * C, gt.nb1 = V;
  gt.A = x, gt.a_b1 = 1, gt.a_m = V, gt.a_k = TV;
  gt.B = w.dx1, gt.b_b1 = 1, gt.b_k = TV, gt.b_n = V;
  gt.C = dTm, gt.c_b1 = (long long)T * T, gt.c_m = T, gt.c_n = 1;
  gt.beta = 1.f;
  DSTD_TRY(gemm(gt, nullptr, s));
  if (dx) {  // dx[n,c,t,v] += sum_q dx1[n,c,q,v] Tm[v,t,q]
    Gemm g;
    g.M = C, g.N = T, g.K = T, g.nb1 = B, g.nb2 = V;
    g.A = w.dx1, g.a_b1 = C * TV, g.a_b2 = 1, g.a_m = TV, g.a_k = V;
    g.B = Tm, g.b_b1 = 0, g.b_b2 = (long long)T * T, g.b_k = 1, g.b_n = T;
    g.C = dx, g.c_b1 = C * TV, g.c_b2 = 1, g.c_m = TV, g.c_n = V;
    g.beta = 1.f;
    DSTD_TRY(gemm(g, nullptr, s));
  }
  return DSTD_OK;
}

size_t dstd_conv2d_workspace_bytes(int B, int cin, int cout, int H, int W, int kh, int kw, int sh, int sw, int ph,
                                   int pw) {
  (void)B, (void)H, (void)W, (void)kh, (void)kw, (void)sh, (void)sw, (void)ph, (void)pw;
  return (gemm_scratch_floats(cout, cin) + reduce_scratch_floats(cout)) * sizeof(float) + 512;
}

int dstd_conv2d_fwd(const float* x, int B, int cin, int H, int W, const float* w, const float* bias, int cout,
                    int kh, int kw, int sh, int sw, int ph, int pw, float* y, void* workspace,
                    size_t workspace_bytes, void* stream) {
  StreamDeviceGuard dev_guard_(stream, x);
  ConvGeom g;
  if (!x || !w || !y || !conv_geom(g, B, cin, H, W, cout, kh, kw, sh, sw, ph, pw)) return DSTD_EINVAL;
  (void)workspace, (void)workspace_bytes;
  hipStream_t s = (hipStream_t)stream;
  if (is_pointwise(g)) {
    const long long HW = (long long)H * W;
    Gemm m;
    m.M = cout, m.N = (int)HW, m.K = cin, m.nb1 = B;
    m.A = w, m.a_m = cin, m.a_k = 1;
    m.B = x, m.b_b1 = cin * HW, m.b_k = HW, m.b_n = 1;
    m.C = y, m.c_b1 = cout * HW, m.c_m = HW, m.c_n = 1;
    m.bias_m = bias;
    DSTD_TRY(gemm(m, nullptr, s));
    return DSTD_OK;
  }
  k_conv2d_fwd<<<grid_of((size_t)B * cout * g.Ho * g.Wo), 256, 0, s>>>(x, w, bias, g, y);
  DSTD_TRY(hipGetLastError());
  return DSTD_OK;
}

int dstd_conv2d_bwd(const float* x, int B, int cin, int H, int W, const float* w, int cout, int kh, int kw, int sh,
                    int sw, int ph, int pw, const float* dy, float* dx, float* dw, float* db, void* workspace,
                    size_t workspace_bytes, void* stream) {
  StreamDeviceGuard dev_guard_(stream, x);
  ConvGeom g;
  if (!x || !w || !dy || !dw || !workspace || !conv_geom(g, B, cin, H, W, cout, kh, kw, sh, sw, ph, pw))
    return DSTD_EINVAL;
  if (workspace_bytes < dstd_conv2d_workspace_bytes(B, cin, cout, H, W, kh, kw, sh, sw, ph, pw))
    return DSTD_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  Carver cv{(char*)workspace};
  float* gs = cv.take(gemm_scratch_floats(cout, cin));
  float* red = cv.take(reduce_scratch_floats(cout));
  const long long HWo = (long long)g.Ho * g.Wo;
  if (db) DSTD_TRY(reduce_rows(dy, cout, B, (int)HWo, cout * HWo, HWo, 1, db, 1.f, red, s));
  if (is_pointwise(g)) {
    const long long HW = (long long)H * W;
    if (dx) {
      Gemm m;
      m.M = cin, m.N = (int)HW, m.K = cout, m.nb1 = B;
      m.A = w, m.a_m = 1, m.a_k = cin;
      m.B = dy, m.b_b1 = cout * HW, m.b_k = HW, m.b_n = 1;
      m.C = dx, m.c_b1 = cin * HW, m.c_m = HW, m.c_n = 1;
      m.beta = 1.f;
      DSTD_TRY(gemm(m, gs, s));
    }
    Gemm m;
    m.M = cout, m.N = cin, m.K = (int)HW, m.nb1 = B, m.reduce = 1;
    m.A = dy, m.a_b1 = cout * HW, m.a_m = HW, m.a_k = 1;
    m.B = x, m.b_b1 = cin * HW, m.b_k = 1, m.b_n = HW;
    m.C = dw, m.c_m = cin, m.c_n = 1;
    m.beta = 1.f;
    DSTD_TRY(gemm(m, gs, s));
    return DSTD_OK;
  }
  if (dx) k_conv2d_bwd_data<<<grid_of((size_t)B * cin * H * W), 256, 0, s>>>(dy, w, g, dx);
  k_conv2d_bwd_weight<<<cout * cin * kh * kw, 256, 0, s>>>(x, dy, g, dw);
  DSTD_TRY(hipGetLastError());
  return DSTD_OK;
}

}  // extern "C"
