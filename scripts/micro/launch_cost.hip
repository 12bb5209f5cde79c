// Host cost per kernel launch on this stack: the same empty kernel (256
// threads x 64 workgroups, one pointer argument) issued N times on one
// stream by <<<>>> (hipLaunchKernel), hipModuleLaunchKernel on the
// hipFunction_t of the symbol, and hipExtLaunchKernel; host time of the
// issue loop only (the device runs far behind), median of 5 repeats.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

struct Args {
  float* p;
  int n;
};
__global__ void k_empty(Args a) {
  if (a.n < 0 && threadIdx.x == 0) a.p[blockIdx.x] = 1.f;
}

int main() {
  const int N = 2000;
  float* d = nullptr;
  (void)hipMalloc(&d, 4096);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  Args a{d, 1};
  hipFunction_t f = nullptr;
  if (hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(k_empty)) != hipSuccess) printf("hipGetFuncBySymbol failed\n");
  auto run = [&](int mode) {
    std::vector<double> reps;
    for (int r = 0; r < 6; ++r) {
      (void)hipStreamSynchronize(s);
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; ++i) {
        if (mode == 0) {
          k_empty<<<64, 256, 0, s>>>(a);
        } else if (mode == 1) {
          void* args[] = {&a};
          (void)hipModuleLaunchKernel(f, 64, 1, 1, 256, 1, 1, 0, s, args, nullptr);
        } else {
          void* args[] = {&a};
          (void)hipExtLaunchKernel(reinterpret_cast<const void*>(k_empty), dim3(64), dim3(256), args, 0, s, nullptr, nullptr, 0);
        }
      }
      const auto t1 = std::chrono::steady_clock::now();
      (void)hipStreamSynchronize(s);
      if (r) reps.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
    }
    std::sort(reps.begin(), reps.end());
    return reps[reps.size() / 2];
  };
  printf("host us per launch: <<<>>> %.2f  hipModuleLaunchKernel %.2f  hipExtLaunchKernel %.2f\n", run(0), run(1), run(2));
  printf("again:              <<<>>> %.2f  hipModuleLaunchKernel %.2f  hipExtLaunchKernel %.2f\n", run(0), run(1), run(2));
  return 0;
}
