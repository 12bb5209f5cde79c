// Microbenchmark of the training step's skinny GEMM shapes (config-5 B = 64
// forward-pair batch, C = 64, T = 40, V = 23): gemm() as dispatched
// (DSTD_GEMM_GENERIC=1 for k_gemm), plus a D2D copy of the panel for scale.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
#include <stdlib.h>
#include <vector>

#include "../../dstd-gcn_amd/csrc/dstd_train.h"

using namespace dstd::train;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

static float* dev_rand(size_t n) {
  std::vector<float> h(n);
  for (auto& v : h) v = (float)rand() / (float)RAND_MAX - 0.5f;
  float* d;
  CK(hipMalloc(&d, n * sizeof(float)));
  CK(hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return d;
}
template <class F>
static double time_us(F f, int iters = 50) {
  for (int i = 0; i < 5; ++i) CK(f());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i) (void)f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3 / iters;
}

int main() {
  const int B = 64, C = 64, CG = 68, T = 40, V = 23, TV = T * V;
  float* W = dev_rand(80 * 80);
  float* bias = dev_rand(80);
  float* X = dev_rand((size_t)B * C * TV);
  float* G = dev_rand((size_t)B * CG * TV);
  float* Y = dev_rand((size_t)B * CG * TV);
  float* Mt = dev_rand((size_t)B * 80 * 529);
  float* Et = dev_rand((size_t)B * 40 * 529);
  float* out = dev_rand(80 * 81);
  float* scratch;
  CK(hipMalloc(&scratch, gemm_scratch_floats(80, 81) * 4));
  // conv fwd: G = Wp . x + b
  Gemm f;
  f.M = CG, f.N = TV, f.K = C, f.nb1 = B;
  f.A = W, f.a_m = C, f.a_k = 1;
  f.B = X, f.b_b1 = (long long)C * TV, f.b_k = TV, f.b_n = 1;
  f.C = Y, f.c_b1 = (long long)CG * TV, f.c_m = TV, f.c_n = 1;
  f.bias_m = bias;
  // conv dx: dx = Wp^T dG (+)
  Gemm x;
  x.M = C, x.N = TV, x.K = CG, x.nb1 = B;
  x.A = W, x.a_m = 1, x.a_k = C;
  x.B = G, x.b_b1 = (long long)CG * TV, x.b_k = TV, x.b_n = 1;
  x.C = Y, x.c_b1 = (long long)C * TV, x.c_m = TV, x.c_n = 1;
  x.beta = 1.f;
  // conv dw (reduce, ones column)
  Gemm w;
  w.M = CG, w.N = C + 1, w.K = TV, w.nb1 = B, w.reduce = 1;
  w.A = G, w.a_b1 = (long long)CG * TV, w.a_m = TV, w.a_k = 1;
  w.B = X, w.b_b1 = (long long)C * TV, w.b_k = 1, w.b_n = TV;
  w.b_ones_last = 1;
  w.C = out, w.c_m = C + 1, w.c_n = 1;
  w.beta = 1.f;
  // wr spatial (reduce): dWrm[a][k] = sum dE[n][a][ij] M[n][k][ij], A = 40, NN2 = 529
  Gemm r;
  r.M = 40, r.N = 80, r.K = 529, r.nb1 = B, r.reduce = 1;
  r.A = Et, r.a_b1 = 40 * 529, r.a_m = 529, r.a_k = 1;
  r.B = Mt, r.b_b1 = 80 * 529, r.b_k = 1, r.b_n = 529;
  r.C = out, r.c_m = 80, r.c_n = 1;
  r.beta = 1.f;
  // E spatial (panel, odd row stride): E = Wrm . M
  Gemm e;
  e.M = 40, e.N = 529, e.K = 80, e.nb1 = B;
  e.A = W, e.a_m = 80, e.a_k = 1;
  e.B = Mt, e.b_b1 = 80 * 529, e.b_k = 529, e.b_n = 1;
  e.C = Et, e.c_b1 = 40 * 529, e.c_m = 529, e.c_n = 1;
  // correctness of the dispatched kernels against a double host reference
  // (batches 0, 17, 63; C restored before each check run)
  auto check = [&](const char* name, const Gemm& g, int nbat) {
    const size_t na = (size_t)(g.M - 1) * g.a_m + (size_t)(g.K - 1) * g.a_k + 1;
    const size_t nbb = (size_t)(nbat - 1) * g.b_b1 + (size_t)(g.K - 1) * g.b_k + (size_t)(g.N - 1) * g.b_n + 1;
    const size_t nc = (size_t)(nbat - 1) * g.c_b1 + (size_t)(g.M - 1) * g.c_m + (size_t)(g.N - 1) * g.c_n + 1;
    std::vector<float> ha(na), hb(nbb), hc0(nc), hc(nc), hbias(g.M, 0.f);
    CK(hipMemcpy(ha.data(), g.A, na * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), g.B, nbb * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hc0.data(), g.C, nc * 4, hipMemcpyDeviceToHost));
    if (g.bias_m) CK(hipMemcpy(hbias.data(), g.bias_m, g.M * 4, hipMemcpyDeviceToHost));
    CK(gemm(g, nullptr, 0));
    CK(hipMemcpy(hc.data(), g.C, nc * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(g.C, hc0.data(), nc * 4, hipMemcpyHostToDevice));
    double worst = 0;
    const int bs[3] = {0, 17, nbat - 1};
    for (int bi = 0; bi < 3; ++bi)
      for (int m = 0; m < g.M; ++m)
        for (int n = 0; n < g.N; ++n) {
          double acc = 0, mag = 0;
          for (int k = 0; k < g.K; ++k) {
            const double t = (double)ha[m * g.a_m + k * g.a_k] * hb[bs[bi] * g.b_b1 + k * g.b_k + n * g.b_n];
            acc += t;
            mag += fabs(t);
          }
          const size_t ci = bs[bi] * g.c_b1 + m * g.c_m + n * g.c_n;
          double ref = g.alpha * acc + hbias[m];
          if (g.beta != 0.f) ref += g.beta * (double)hc0[ci];
          const double err = fabs(hc[ci] - ref) / (mag + fabs(hbias[m]) + fabs(g.beta * hc0[ci]) + 1e-30);
          if (err > worst) worst = err;
        }
    printf("%s: max |err| / sum|terms| = %.3g%s\n", name, worst, worst < 1e-6 ? "" : "  <-- FAIL");
    return worst < 1e-6;
  };
  bool ok = check("conv fwd", f, B) & check("conv dx", x, B) & check("E", e, B);
  const double tf = time_us([&] { return gemm(f, nullptr, 0); });
  const double tx = time_us([&] { return gemm(x, nullptr, 0); });
  const double tw = time_us([&] { return gemm(w, scratch, 0); });
  const double tr = time_us([&] { return gemm(r, scratch, 0); });
  const double te = time_us([&] { return gemm(e, nullptr, 0); });
  const size_t xb = (size_t)B * C * TV * 4;
  const double tc = time_us([&] { return hipMemcpyAsync(Y, X, xb, hipMemcpyDeviceToDevice, 0); });
  printf("conv fwd %.1f us  conv dx %.1f us  conv dw %.1f us  wr %.1f us  E %.1f us | D2D copy of x (%.1f MB) %.1f us\n", tf,
         tx, tw, tr, te, xb / 1e6, tc);
  return ok ? 0 : 1;
}
