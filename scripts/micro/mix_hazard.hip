// Does a v_fma_mixhi_f16 that follows a v_fma_mixlo_f16 writing the SAME VGPR
// see the low half just written?  (gfx940+ "dst-sel forwarding" hazard: a VALU
// that writes part of a VGPR, followed by a VALU that reads it -- including
// the implicit read of a preserve-the-other-half write -- needs one wait
// state.  hipcc pads that for its own code, never inside inline asm.)
// The destination register starts as 0xBEEFBEEF; a stale read leaves 0xBEEF
// in the low half.  Variants: as split8 (dstd_hilo.h) wrote it until round 3
// (no pad), and with s_nop 0 between the two halves.
// hipcc --offload-arch=gfx950 -O3 mix_hazard.hip -o mix_hazard && ./mix_hazard
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

template <int PAD>
__global__ void k(uint32_t* out, const float* in, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = in[2 * i], b = in[2 * i + 1];
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
  const uint32_t hi = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, f16x2_t));
  uint32_t lo = 0xBEEFBEEFu;
  if (PAD)
    asm volatile("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
                 "s_nop 0\n\t"
                 "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
                 "s_nop 1"
                 : "+v"(lo) : "v"(a), "v"(b), "v"(hi));
  else
    asm volatile("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
                 "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
                 "s_nop 1"
                 : "+v"(lo) : "v"(a), "v"(b), "v"(hi));
  out[i] = lo;
}

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t u; memcpy(&u, &h, 2); return u; }

int main() {
  const int n = 1 << 20;
  float* h_in = (float*)malloc(8 * (size_t)n);
  uint32_t s = 12345;
  for (int i = 0; i < 2 * n; ++i) {
    s = s * 1664525u + 1013904223u;
    h_in[i] = ((int)(s >> 8) - (1 << 23)) * (1.f / (1 << 20));
  }
  float* d_in;
  uint32_t* d_out;
  hipMalloc(&d_in, 8 * (size_t)n);
  hipMalloc(&d_out, 4 * (size_t)n);
  hipMemcpy(d_in, h_in, 8 * (size_t)n, hipMemcpyHostToDevice);
  uint32_t* h_out = (uint32_t*)malloc(4 * (size_t)n);
  for (int pad = 0; pad < 2; ++pad) {
    if (pad) hipLaunchKernelGGL(k<1>, dim3(n / 256), dim3(256), 0, 0, d_out, d_in, n);
    else hipLaunchKernelGGL(k<0>, dim3(n / 256), dim3(256), 0, 0, d_out, d_in, n);
    hipMemcpy(h_out, d_out, 4 * (size_t)n, hipMemcpyDeviceToHost);
    long bad_lo = 0, bad_hi = 0, stale = 0;
    for (int i = 0; i < n; ++i) {
      const float a = h_in[2 * i], b = h_in[2 * i + 1];
      const _Float16 ha = (_Float16)a, hb = (_Float16)b;
      const uint16_t el = f2h(a - (float)ha), eh = f2h(b - (float)hb);
      const uint16_t gl = h_out[i] & 0xffff, gh = h_out[i] >> 16;
      bad_lo += gl != el;
      bad_hi += gh != eh;
      stale += gl == 0xBEEF;
    }
    printf("pad=%d: %d values, low half wrong %ld (stale 0xBEEF %ld), high half wrong %ld\n", pad, n, bad_lo, stale,
           bad_hi);
  }
  return 0;
}
