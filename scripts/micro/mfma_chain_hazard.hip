// Which dependent-MFMA register patterns does gfx950 execute correctly with
// the wait states hipcc's hazard recognizer inserts (none, for all of these)?
//
// Found in round 3: k_temporal_fused with the conv_rm W fragments hoisted out
// of its tile loop (dstd_hilo.hip, DSTD_TF_HOISTW) computed wrong planes for
// its second row tile only.  The compiler had emitted that tile's chain as
//   v_mfma_f32_16x16x32_f16 v[48:51], v[16:19], v[12:15], 0
//   v_mfma_f32_16x16x32_f16 v[20:23], v[20:23], v[8:11], v[48:51]   (C = previous D, new D = own A)
//   v_mfma_f32_16x16x32_f16 v[16:19], v[16:19], v[8:11], v[20:23]
// while every correct build accumulated in place (D == C throughout).
// Each test below runs one pattern back to back (no s_nop between the MFMAs,
// as hipcc emitted it) and the same arithmetic with the MFMAs padded and the
// registers disjoint; bitwise comparison over 64 K of random operands.
//   P1  C = previous D, new D != C (different accumulator register)
//   P2  D == own A (in place over the A operand), C separate
//   P3  D == own B
//   P4  the compiler's chain above: P1 + P2 + a third MFMA, 16x16x32 f16
// hipcc --offload-arch=gfx950 -O3 mfma_chain_hazard.hip -o mfma_chain_hazard && ./mfma_chain_hazard
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define PAD "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"

template <int P, int SAFE>
__global__ void k(f32x4* out, const f16x8* in, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const f16x8 a1 = in[4 * i], b1 = in[4 * i + 1], a2 = in[4 * i + 2], b2 = in[4 * i + 3];
  f32x4 r;
  if constexpr (P == 1) {
    f32x4 t;
    if (SAFE)
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %2, %3, 0\n\t" PAD
                   "v_mfma_f32_16x16x32_f16 %1, %4, %5, %0\n\t" PAD
                   : "=&v"(t), "=&v"(r) : "v"(a1), "v"(b1), "v"(a2), "v"(b2));
    else
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %2, %3, 0\n\t"
                   "v_mfma_f32_16x16x32_f16 %1, %4, %5, %0\n\t" PAD
                   : "=&v"(t), "=&v"(r) : "v"(a1), "v"(b1), "v"(a2), "v"(b2));
  } else if constexpr (P == 2 || P == 3) {
    f32x4 c;
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0\n\t" PAD : "=&v"(c) : "v"(a2), "v"(b2));
    if (SAFE) {
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %3\n\t" PAD : "=&v"(r) : "v"(a1), "v"(b1), "v"(c));
    } else if (P == 2) {
      r = __builtin_bit_cast(f32x4, a1);
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %0, %1, %2\n\t" PAD : "+v"(r) : "v"(b1), "v"(c));
    } else {
      r = __builtin_bit_cast(f32x4, b1);
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %0, %2\n\t" PAD : "+v"(r) : "v"(a1), "v"(c));
    }
  } else if constexpr (P >= 5) {
    // P1 (P5-P7) / P4 (P8) with one instruction between MFMA 1 and MFMA 2, as
    // hipcc scheduled it (an SALU), an s_nop 0, or a VALU
    f32x4 t;
    uint32_t dummy = 0;
    if (SAFE) {
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %2, %3, 0\n\t" PAD
                   "v_mfma_f32_16x16x32_f16 %1, %4, %5, %0\n\t" PAD
                   : "=&v"(t), "=&v"(r) : "v"(a1), "v"(b1), "v"(a2), "v"(b2));
    } else if (P == 5) {
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %2, %3, 0\n\t"
                   "s_and_b64 s[20:21], exec, vcc\n\t"
                   "v_mfma_f32_16x16x32_f16 %1, %4, %5, %0\n\t" PAD
                   : "=&v"(t), "=&v"(r) : "v"(a1), "v"(b1), "v"(a2), "v"(b2) : "s20", "s21");
    } else if (P == 6) {
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %2, %3, 0\n\t"
                   "s_nop 0\n\t"
                   "v_mfma_f32_16x16x32_f16 %1, %4, %5, %0\n\t" PAD
                   : "=&v"(t), "=&v"(r) : "v"(a1), "v"(b1), "v"(a2), "v"(b2));
    } else if (P == 7) {
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %3, %4, 0\n\t"
                   "v_mov_b32 %2, 7\n\t"
                   "v_mfma_f32_16x16x32_f16 %1, %5, %6, %0\n\t" PAD
                   : "=&v"(t), "=&v"(r), "=&v"(dummy) : "v"(a1), "v"(b1), "v"(a2), "v"(b2));
    }
    (void)dummy;
  } else {  // P == 4
    f32x4 t, u = __builtin_bit_cast(f32x4, a2), w = __builtin_bit_cast(f32x4, a1);
    if (SAFE) {
      f32x4 u2, w2;
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %3, %4, 0\n\t" PAD
                   "v_mfma_f32_16x16x32_f16 %1, %5, %6, %0\n\t" PAD
                   "v_mfma_f32_16x16x32_f16 %2, %3, %6, %1\n\t" PAD
                   : "=&v"(t), "=&v"(u2), "=&v"(w2) : "v"(a1), "v"(b1), "v"(a2), "v"(b2));
      r = w2;
    } else {
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %3, 0\n\t"
                   "v_mfma_f32_16x16x32_f16 %2, %2, %4, %0\n\t"
                   "v_mfma_f32_16x16x32_f16 %1, %1, %4, %2\n\t" PAD
                   : "=&v"(t), "+v"(w), "+v"(u) : "v"(b1), "v"(b2));
      r = w;
    }
  }
  out[i] = r;
}

// P9: the chain of the failing build with the hazard hipcc padded to its
// minimum: MFMA 3 reads u as C, one more MFMA and s_nop 5 (7 wait states,
// SMFMA16x16ReadVgprVALUWarWaitStates), then an LDS read overwrites u.  Waves
// of the 1024-thread workgroup alternate with MFMA-only partner waves, so a
// wave's MFMAs can wait behind the partner's in the SIMD's matrix pipe.
template <int SAFE>
__global__ __launch_bounds__(1024) void k_war(f32x4* out, const f16x8* in, int n) {
  __shared__ f32x4 lds[1024];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  lds[threadIdx.x] = f32x4{1e6f, 2e6f, 3e6f, 4e6f};
  __syncthreads();
  const f16x8 a1 = in[4 * i], b1 = in[4 * i + 1], a2 = in[4 * i + 2], b2 = in[4 * i + 3];
  const uint32_t addr = (uint32_t)(uintptr_t)(lds + threadIdx.x);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  f32x4 w = {0.f, 0.f, 0.f, 0.f};
  if (wave & 1) {  // partner: a long run of MFMAs on its own registers
    f32x4 z = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < 64; ++r) z = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, z, 0, 0, 0);
    out[i] = z;
    return;
  }
  for (int r = 0; r < 16; ++r) {
    f32x4 t, u, ww;
    if (SAFE)
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %3, %4, 0\n\t"
                   "v_mfma_f32_16x16x32_f16 %1, %5, %6, %0\n\t"
                   "v_mfma_f32_16x16x32_f16 %2, %3, %6, %1\n\t"
                   "v_mfma_f32_16x16x32_f16 %2, %5, %4, %2\n\t" PAD PAD PAD
                   "ds_read_b128 %1, %7\n\t"
                   "s_waitcnt lgkmcnt(0)\n\t" PAD
                   : "=&v"(t), "=&v"(u), "=&v"(ww) : "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(addr));
    else
      asm volatile("v_mfma_f32_16x16x32_f16 %0, %3, %4, 0\n\t"
                   "v_mfma_f32_16x16x32_f16 %1, %5, %6, %0\n\t"
                   "v_mfma_f32_16x16x32_f16 %2, %3, %6, %1\n\t"
                   "v_mfma_f32_16x16x32_f16 %2, %5, %4, %2\n\t"
                   "s_nop 5\n\t"
                   "ds_read_b128 %1, %7\n\t"
                   "s_waitcnt lgkmcnt(0)\n\t" PAD
                   : "=&v"(t), "=&v"(u), "=&v"(ww) : "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(addr));
    w += ww;
  }
  out[i] = w;
}

long run_war(const f16x8* d_in, f32x4* d_o, f32x4* h_a, f32x4* h_b, int n) {
  hipLaunchKernelGGL(k_war<1>, dim3(n / 1024), dim3(1024), 0, 0, d_o, d_in, n);
  hipMemcpy(h_a, d_o, 16 * (size_t)n, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(k_war<0>, dim3(n / 1024), dim3(1024), 0, 0, d_o, d_in, n);
  hipMemcpy(h_b, d_o, 16 * (size_t)n, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int i = 0; i < n; ++i) bad += memcmp(&h_a[i], &h_b[i], 16) != 0;
  return bad;
}

template <int P>
long run(const f16x8* d_in, f32x4* d_o, f32x4* h_a, f32x4* h_b, int n) {
  hipLaunchKernelGGL((k<P, 1>), dim3(n / 256), dim3(256), 0, 0, d_o, d_in, n);
  hipMemcpy(h_a, d_o, 16 * (size_t)n, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL((k<P, 0>), dim3(n / 256), dim3(256), 0, 0, d_o, d_in, n);
  hipMemcpy(h_b, d_o, 16 * (size_t)n, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int i = 0; i < n; ++i) bad += memcmp(&h_a[i], &h_b[i], 16) != 0;
  return bad;
}

int main() {
  const int n = 1 << 16;
  _Float16* h_in = (_Float16*)malloc(64 * (size_t)n);
  uint32_t s = 777;
  for (size_t i = 0; i < 32 * (size_t)n; ++i) {
    s = s * 1664525u + 1013904223u;
    h_in[i] = (_Float16)(((int)(s >> 9) - (1 << 22)) * (1.f / (1 << 21)));
  }
  f16x8* d_in;
  f32x4* d_o;
  hipMalloc(&d_in, 64 * (size_t)n);
  hipMalloc(&d_o, 16 * (size_t)n);
  hipMemcpy(d_in, h_in, 64 * (size_t)n, hipMemcpyHostToDevice);
  f32x4* h_a = (f32x4*)malloc(16 * (size_t)n);
  f32x4* h_b = (f32x4*)malloc(16 * (size_t)n);
  printf("P1 C = previous D, new D != C       : %ld of %d lanes differ\n", run<1>(d_in, d_o, h_a, h_b, n), n);
  printf("P2 D == own A                        : %ld of %d lanes differ\n", run<2>(d_in, d_o, h_a, h_b, n), n);
  printf("P3 D == own B                        : %ld of %d lanes differ\n", run<3>(d_in, d_o, h_a, h_b, n), n);
  printf("P5 P1 with an SALU between          : %ld of %d lanes differ\n", run<5>(d_in, d_o, h_a, h_b, n), n);
  printf("P6 P1 with s_nop 0 between           : %ld of %d lanes differ\n", run<6>(d_in, d_o, h_a, h_b, n), n);
  printf("P7 P1 with a VALU between            : %ld of %d lanes differ\n", run<7>(d_in, d_o, h_a, h_b, n), n);
  printf("P4 hipcc's chain (P1 + P2, 3 MFMAs)  : %ld of %d lanes differ\n", run<4>(d_in, d_o, h_a, h_b, n), n);
  printf("P9 C read, then a ds_read over C after 7 wait states, MFMA partner waves: %ld of %d lanes differ\n",
         run_war(d_in, d_o, h_a, h_b, n), n);
  return 0;
}
