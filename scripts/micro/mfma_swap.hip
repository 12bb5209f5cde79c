// Checks the operand lane maps of v_mfma_f32_16x16x32_f16 that dstd_hilo.h
// documents, by computing D = A B and D^T = B^T A^T with swapped operands.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
__global__ void k16(const float* A, const float* B, float* D, float* DT) {  // 16x16x16: A 16x16, B 16x16
  const int lane = threadIdx.x, i = lane & 15, kg = lane >> 4;
  f16x4 a, b;
  for (int e = 0; e < 4; ++e) {
    const int kk = 4 * kg + e;
    a[e] = (_Float16)A[i * 32 + kk];
    b[e] = (_Float16)B[kk * 16 + i];
  }
  f32x4 c = {0, 0, 0, 0}, ct = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
  ct = __builtin_amdgcn_mfma_f32_16x16x16f16(b, a, ct, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    D[(4 * kg + r) * 16 + i] = c[r];
    DT[(4 * kg + r) * 16 + i] = ct[r];
  }
}
__global__ void k(const float* A, const float* B, float* D, float* DT) {
  const int lane = threadIdx.x, i = lane & 15, kg = lane >> 4;
  f16x8 a, b, at, bt;
  for (int e = 0; e < 8; ++e) {
    const int kk = 8 * kg + e;
    a[e] = (_Float16)A[i * 32 + kk];   // A[i][k]
    b[e] = (_Float16)B[kk * 16 + i];   // B[k][j = i]
  }
  f32x4 c = {0, 0, 0, 0}, ct = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);   // D = A B
  ct = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, ct, 0, 0, 0); // B^T-fragments as A: D^T
  for (int r = 0; r < 4; ++r) {
    D[(4 * kg + r) * 16 + i] = c[r];
    DT[(4 * kg + r) * 16 + i] = ct[r];
  }
}
int main() {
  float hA[16 * 32], hB[32 * 16], hD[256], hDT[256];
  for (int x = 0; x < 512; ++x) { hA[x] = (x * 37 % 17) - 8; hB[x] = (x * 11 % 13) - 6; }
  float *A, *B, *D, *DT;
  hipMalloc(&A, sizeof hA); hipMalloc(&B, sizeof hB); hipMalloc(&D, 1024); hipMalloc(&DT, 1024);
  hipMemcpy(A, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(B, hB, sizeof hB, hipMemcpyHostToDevice);
  k<<<1, 64>>>(A, B, D, DT);
  hipMemcpy(hD, D, 1024, hipMemcpyDeviceToHost); hipMemcpy(hDT, DT, 1024, hipMemcpyDeviceToHost);
  double e1 = 0, e2 = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double ref = 0;
      for (int kk = 0; kk < 32; ++kk) ref += hA[i * 32 + kk] * hB[kk * 16 + j];
      e1 = fmax(e1, fabs(hD[i * 16 + j] - ref));
      e2 = fmax(e2, fabs(hDT[j * 16 + i] - ref));
    }
  printf("D = AB max err %g, swapped (D^T) max err %g\n", e1, e2);
  k16<<<1, 64>>>(A, B, D, DT);
  hipMemcpy(hD, D, 1024, hipMemcpyDeviceToHost); hipMemcpy(hDT, DT, 1024, hipMemcpyDeviceToHost);
  e1 = e2 = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double ref = 0;
      for (int kk = 0; kk < 16; ++kk) ref += hA[i * 32 + kk] * hB[kk * 16 + j];
      e1 = fmax(e1, fabs(hD[i * 16 + j] - ref));
      e2 = fmax(e2, fabs(hDT[j * 16 + i] - ref));
    }
  printf("16x16x16: D = AB max err %g, swapped max err %g\n", e1, e2);
  return 0;
}
