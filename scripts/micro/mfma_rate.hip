// Back-to-back MFMA issue rate on one SIMD (one wave per SIMD, 8 independent
// accumulators), cycles per instruction from s_memtime.  hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int N = 4096;

template <int K>
__global__ void kmfma(float* out, unsigned long long* cyc, float seed) {
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{seed, 0, 0, 0};
  const float a = seed + threadIdx.x;
  f16x4 h4 = {(_Float16)a, (_Float16)1, (_Float16)2, (_Float16)3};
  f16x8 h8 = {(_Float16)a, (_Float16)1, (_Float16)2, (_Float16)3, (_Float16)a, (_Float16)1, (_Float16)2, (_Float16)3};
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < N / 8; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (K == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, acc[i], 0, 0, 0);
      if constexpr (K == 1) acc[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(h4, h4, acc[i], 0, 0, 0);
      if constexpr (K == 2) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(h8, h8, acc[i], 0, 0, 0);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
void run(const char* name) {
  float* o; unsigned long long* c;
  hipMalloc(&o, 1024 * 256 * 4); hipMalloc(&c, 1024 * 8);
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kmfma<K>, dim3(256), dim3(256), 0, 0, o, c, 1.0f);
  hipDeviceSynchronize();
  unsigned long long h[1024];
  hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
  double s = 0; for (int i = 0; i < 256; ++i) s += h[i];
  printf("%-22s %.2f cycles per MFMA (per SIMD, 1 wave)\n", name, s / 256 / N);
  hipFree(o); hipFree(c);
}
int main() {
  run<0>("16x16x4 f32");
  run<1>("16x16x16 f16");
  run<2>("16x16x32 f16");
  return 0;
}
