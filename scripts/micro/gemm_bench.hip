// Micro-benchmark of the training GEMM (dstd::train::gemm) on the 1x1-conv
// shapes of the 3DPW step, against a device-to-device copy of the same bytes.
//   make -C dstd-gcn_amd && hipcc --offload-arch=gfx950 -O3 -c scripts/micro/gemm_bench.hip -o /tmp/gb.o &&
//   hipcc --offload-arch=gfx950 /tmp/gb.o dstd-gcn_amd/build/dstd_train.o -o /tmp/gemm_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <functional>
#include <vector>
#include "../../dstd-gcn_amd/csrc/dstd_train.h"

using dstd::train::Gemm;

static float time_us(hipStream_t s, int reps, const std::function<void()>& f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) f();
  hipEventRecord(a, s);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  hipStream_t s;
  hipStreamCreate(&s);
  const int TV = 920;
  for (int B : {32, 128}) {
    for (int M : {68, 64, 16}) {
      const int K = 64;
      float *X, *W, *C, *bias, *scr;
      hipMalloc(&X, sizeof(float) * B * K * TV);
      hipMalloc(&W, sizeof(float) * M * K);
      hipMalloc(&bias, sizeof(float) * M);
      hipMalloc(&C, sizeof(float) * B * M * TV);
      hipMalloc(&scr, sizeof(float) * 128 * 128 * 128);
      hipMemset(X, 0, sizeof(float) * B * K * TV);
      hipMemset(W, 0, sizeof(float) * M * K);
      hipMemset(bias, 0, sizeof(float) * M);
      Gemm g;
      g.M = M, g.N = TV, g.K = K, g.nb1 = B;
      g.A = W, g.a_m = K, g.a_k = 1;
      g.B = X, g.b_b1 = (long long)K * TV, g.b_k = TV, g.b_n = 1;
      g.C = C, g.c_b1 = (long long)M * TV, g.c_m = TV, g.c_n = 1;
      g.bias_m = bias;
      float t = time_us(s, 200, [&] { dstd::train::gemm(g, scr, s); });
      float tc = time_us(s, 200, [&] { hipMemcpyAsync(C, X, sizeof(float) * B * std::min(K, M) * TV, hipMemcpyDeviceToDevice, s); });
      printf("B=%d M=%d K=%d N=%d: gemm %.2f us  copy %.2f us\n", B, M, K, TV, t, tc);
      hipFree(X); hipFree(W); hipFree(C); hipFree(bias); hipFree(scr);
    }
  }
  return 0;
}
