// Bisects the 1x1-conv GEMM time (C[b][m][p] = W[m][:] . X[b][:][p] + bias):
// stage 0 = tile loads only, 1 = + MFMA loop, 2 = + LDS-staged stores.
//   hipcc --offload-arch=gfx950 -O3 scripts/micro/conv_bisect.hip -o scripts/micro/conv_bisect
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <functional>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int RT, int STAGE, int NC>
__global__ __launch_bounds__(256) void k_conv(const float* __restrict__ W, const float* __restrict__ X,
                                              const float* __restrict__ bias, float* __restrict__ C, int M,
                                              int K, int N) {
  constexpr int SX = NC + 16, MP = RT * 16, SM = MP + ((16 - (MP % 32)) + 32) % 32;
  __shared__ float Wl[64 * SM];
  __shared__ float Xl[(MP > 64 ? MP : 64) * SX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * NC, b = blockIdx.y;
  const float* Xb = X + (size_t)b * K * N;
  // W: row-major [M][K], K == 64
  for (int i = tid; i < MP * 64; i += 256) {
    const int m = i >> 6, k = i & 63;
    Wl[k * SM + m] = m < M ? W[m * 64 + k] : 0.f;
  }
  constexpr int L = NC / 4;  // lanes per row
  const int c4 = (tid % L) * 4;
  float4 r[64 * L / 256];
#pragma unroll
  for (int u = 0; u < 64 * L / 256; ++u) {
    const int k = tid / L + u * (256 / L);
    r[u] = *reinterpret_cast<const float4*>(Xb + (size_t)k * N + n0 + c4);
  }
#pragma unroll
  for (int u = 0; u < 64 * L / 256; ++u) {
    const int k = tid / L + u * (256 / L);
    *reinterpret_cast<float4*>(Xl + k * SX + c4) = r[u];
  }
  __syncthreads();
  const int kl = lane >> 4, cl = lane & 15;
  f32x4 acc[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (STAGE >= 1) {
    constexpr int CT = NC / 16;  // column tiles, split over waves
    for (int ct = wave; ct < CT; ct += 4) {
      for (int ks = 0; ks < 16; ++ks) {
        const int k = ks * 4 + kl;
        const float bv = Xl[k * SX + ct * 16 + cl];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(Wl[k * SM + rt * 16 + cl], bv, acc[rt], 0, 0, 0);
      }
    }
  }
  if (STAGE == 0) {
    if (tid == 0 && Xl[5] == 12345.f) C[0] = Wl[3];
    return;
  }
  __syncthreads();
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 4; ++j) Xl[(rt * 16 + kl * 4 + j) * SX + wave * 16 + cl] = acc[rt][j];
  __syncthreads();
  if (STAGE == 1) {
    if (tid == 0 && Xl[5] == 12345.f) C[0] = Wl[3];
    return;
  }
  float* Cb = C + (size_t)b * M * N;
  for (int m = tid / L; m < M; m += 256 / L) {
    const float* o = Xl + m * SX + c4;
    const float bm = bias[m];
    *reinterpret_cast<float4*>(Cb + (size_t)m * N + n0 + c4) = make_float4(o[0] + bm, o[1] + bm, o[2] + bm, o[3] + bm);
  }
}

static float time_us(hipStream_t s, int reps, const std::function<void()>& f) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) f();
  (void)hipEventRecord(a, s);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b, s);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

template <int STAGE, int NC>
void run(hipStream_t s, const float* W, const float* X, const float* bias, float* C, int B, int M, int N) {
  const float t = time_us(s, 200, [&] {
    k_conv<4, STAGE, NC><<<dim3(N / NC, B), 256, 0, s>>>(W, X, bias, C, M, 64, N);
  });
  printf("B=%d M=%d N=%d NC=%d stage %d: %.2f us\n", B, M, N, NC, STAGE, t);
}

int main() {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  const int B = 32, M = 64, K = 64;
  for (int N : {920, 1024}) {
    const int Np = 1024;
    float *X, *W, *C, *bias;
    (void)hipMalloc(&X, sizeof(float) * B * K * Np);
    (void)hipMalloc(&W, sizeof(float) * M * K);
    (void)hipMalloc(&bias, sizeof(float) * M);
    (void)hipMalloc(&C, sizeof(float) * B * M * Np);
    (void)hipMemset(X, 0, sizeof(float) * B * K * Np);
    (void)hipMemset(W, 0, sizeof(float) * M * K);
    (void)hipMemset(bias, 0, sizeof(float) * M);
    const int Nr = N / 64 * 64;  // whole tiles only
    run<0, 64>(s, W, X, bias, C, B, M, Nr);
    run<1, 64>(s, W, X, bias, C, B, M, Nr);
    run<2, 64>(s, W, X, bias, C, B, M, Nr);
    run<0, 32>(s, W, X, bias, C, B, M, Nr);
    run<2, 32>(s, W, X, bias, C, B, M, Nr);
    run<2, 128>(s, W, X, bias, C, B, M, Nr);
    (void)hipFree(X); (void)hipFree(W); (void)hipFree(C); (void)hipFree(bias);
  }
  return 0;
}
