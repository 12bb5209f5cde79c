// Microbenchmark of the training-path aggregation products at the config-5
// training shapes (B = 64 = forward pair of 32, C = 64, T = 40, V = 23):
// slab kernels (agg_fwd / agg_bwd) vs the strided GEMMs, plus a max-abs
// comparison of the two.  Build: scripts/micro/build.sh; run on the GPU box.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
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

static float* dev_rand(size_t n, unsigned seed) {
  std::vector<float> h(n);
  srand(seed);
  for (auto& v : h) v = (float)rand() / (float)RAND_MAX - 0.5f;
  float* d;
  CK(hipMalloc(&d, n * sizeof(float)));
  CK(hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return d;
}
static double maxdiff(const float* a, const float* b, size_t n) {
  std::vector<float> x(n), y(n);
  CK(hipMemcpy(x.data(), a, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), b, n * 4, hipMemcpyDeviceToHost));
  double m = 0, r = 0;
  for (size_t i = 0; i < n; ++i) m = fmax(m, fabs((double)x[i] - y[i])), r = fmax(r, fabs((double)y[i]));
  return m / (r > 0 ? r : 1);
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

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 64, C = argc > 2 ? atoi(argv[2]) : 64;
  const int T = 40, V = 23, TV = T * V, CG = C + 4;
  for (int temporal = 0; temporal < 2; ++temporal) {
    const int A = temporal ? V : T, NN = temporal ? T : V, NN2 = NN * NN;
    const long long ps_a = temporal ? 1 : V, ps_i = temporal ? V : 1;
    float* G = dev_rand((size_t)B * CG * TV, 1);
    float* D = dev_rand((size_t)B * A * NN2, 2);
    float* dy = dev_rand((size_t)B * C * TV, 3);
    float *y1, *y2, *dG1, *dG2, *dD1, *dD2;
    CK(hipMalloc(&y1, (size_t)B * C * TV * 4));
    CK(hipMalloc(&y2, (size_t)B * C * TV * 4));
    CK(hipMalloc(&dG1, (size_t)B * CG * TV * 4));
    CK(hipMalloc(&dG2, (size_t)B * CG * TV * 4));
    CK(hipMalloc(&dD1, (size_t)B * A * NN2 * 4));
    CK(hipMalloc(&dD2, (size_t)B * A * NN2 * 4));
    const long long ldG = (long long)CG * TV;
    Gemm a;
    a.M = C, a.N = NN, a.K = NN, a.nb1 = B, a.nb2 = A;
    a.A = G, a.a_b1 = ldG, a.a_b2 = ps_a, a.a_m = TV, a.a_k = ps_i;
    a.B = D, a.b_b1 = (long long)A * NN2, a.b_b2 = NN2, a.b_k = NN, a.b_n = 1;
    a.C = y2, a.c_b1 = (long long)C * TV, a.c_b2 = ps_a, a.c_m = TV, a.c_n = ps_i;
    Gemm f;
    f.M = C, f.N = NN, f.K = NN, f.nb1 = B, f.nb2 = A;
    f.A = dy, f.a_b1 = (long long)C * TV, f.a_b2 = ps_a, f.a_m = TV, f.a_k = ps_i;
    f.B = D, f.b_b1 = (long long)A * NN2, f.b_b2 = NN2, f.b_k = 1, f.b_n = NN;
    f.C = dG2, f.c_b1 = ldG, f.c_b2 = ps_a, f.c_m = TV, f.c_n = ps_i;
    Gemm d;
    d.M = NN, d.N = NN, d.K = C, d.nb1 = B, d.nb2 = A;
    d.A = G, d.a_b1 = ldG, d.a_b2 = ps_a, d.a_m = ps_i, d.a_k = TV;
    d.B = dy, d.b_b1 = (long long)C * TV, d.b_b2 = ps_a, d.b_k = TV, d.b_n = ps_i;
    d.C = dD2, d.c_b1 = (long long)A * NN2, d.c_b2 = NN2, d.c_m = NN, d.c_n = 1;
    CK(agg_fwd(G, ldG, D, y1, (long long)C * TV, 0.f, B, C, T, V, temporal, 0));
    CK(gemm(a, nullptr, 0));
    float* dDp;
    CK(hipMalloc(&dDp, (size_t)agg_parts(C) * B * A * NN2 * 4));
    int np = 0;
    CK(agg_bwd(G, ldG, dy, (long long)C * TV, D, dG1, ldG, dD1, B, C, T, V, temporal, 0, dDp, &np));
    if (np > 1) {  // sum the partials on the host side of the check
      std::vector<float> h((size_t)np * B * A * NN2), o((size_t)B * A * NN2, 0.f);
      CK(hipMemcpy(h.data(), dDp, h.size() * 4, hipMemcpyDeviceToHost));
      for (int q = 0; q < np; ++q)
        for (size_t i = 0; i < o.size(); ++i) o[i] += h[q * o.size() + i];
      CK(hipMemcpy(dD1, o.data(), o.size() * 4, hipMemcpyHostToDevice));
    }
    CK(gemm(f, nullptr, 0));
    CK(gemm(d, nullptr, 0));
    CK(hipDeviceSynchronize());
    printf("%s B=%d C=%d: fwd rel diff %.2e  dF %.2e  dD %.2e\n", temporal ? "temporal" : "spatial", B, C,
           maxdiff(y1, y2, (size_t)B * C * TV), maxdiff(dG1, dG2, (size_t)B * CG * TV),
           maxdiff(dD1, dD2, (size_t)B * A * NN2));
    const double t_af = time_us([&] { return agg_fwd(G, ldG, D, y1, (long long)C * TV, 0.f, B, C, T, V, temporal, 0); });
    const double t_af1 = time_us([&] { return agg_fwd(G, ldG, D, y1, (long long)C * TV, 1.f, B, C, T, V, temporal, 0); });
    const double t_ab = time_us(
        [&] { return agg_bwd(G, ldG, dy, (long long)C * TV, D, dG1, ldG, dD1, B, C, T, V, temporal, 0, dDp, &np); });
    const double t_ga = time_us([&] { return gemm(a, nullptr, 0); });
    const double t_gf = time_us([&] { return gemm(f, nullptr, 0); });
    const double t_gd = time_us([&] { return gemm(d, nullptr, 0); });
    printf("  slab fwd %.1f us (beta 1: %.1f)  bwd %.1f us (dD parts %d) | gemm fwd %.1f  dF %.1f  dD %.1f us\n",
           t_af, t_af1, t_ab, np, t_ga, t_gf, t_gd);
    for (float* p : {G, D, dy, y1, y2, dG1, dG2, dD1, dD2, dDp}) CK(hipFree(p));
  }
  return 0;
}
