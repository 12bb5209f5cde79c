// Shared device helpers for the DSTDGC kernels (gfx950 / CDNA4, wave64).
//
// Matrix work uses the exact-fp32 MFMA v_mfma_f32_16x16x4_f32
// (__builtin_amdgcn_mfma_f32_16x16x4f32).  Lane maps (MI355X guide §3):
//   A[i = lane&15][k = lane>>4]        one f32 per lane
//   B[k = lane>>4][j = lane&15]        one f32 per lane
//   C/D[row = (lane>>4)*4 + r][col = lane&15], r = 0..3 (f32x4 per lane)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define DSTD_WAVE 64
#define DSTD_THREADS 256
#define DSTD_WAVES (DSTD_THREADS / DSTD_WAVE)

// The C entry points launch on the device of the caller's stream: a module
// on cuda:1 called while cuda:0 is current switches for the call and back.
// The null stream (torch's default stream) names no device -- it is the
// CURRENT device's -- so there the device comes from the call's first
// device pointer (hipPointerGetAttributes; skipped on a single-GPU process).
inline int dstd_device_count() {
  static const int n = [] {
    int c = 0;
    return hipGetDeviceCount(&c) == hipSuccess ? c : 0;
  }();
  return n;
}
struct StreamDeviceGuard {
  int prev = -1;
  explicit StreamDeviceGuard(void* stream, const void* devptr = nullptr) {
    int cur = 0, sd = -1;
    if (hipGetDevice(&cur) != hipSuccess) return;
    if (stream) {
      hipDevice_t d = 0;
      if (hipStreamGetDevice((hipStream_t)stream, &d) != hipSuccess) return;
      sd = (int)d;
    } else if (devptr && dstd_device_count() > 1) {
      hipPointerAttribute_t at{};
      if (hipPointerGetAttributes(&at, devptr) != hipSuccess) {
        (void)hipGetLastError();
        return;
      }
      if (at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeManaged) return;
      sd = at.device;
    }
    if (sd >= 0 && sd != cur && hipSetDevice(sd) == hipSuccess) prev = cur;
  }
  ~StreamDeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  StreamDeviceGuard(const StreamDeviceGuard&) = delete;
  StreamDeviceGuard& operator=(const StreamDeviceGuard&) = delete;
};

__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// tanh(x) = 1 - 2 / (exp(2x) + 1).  v_exp_f32 + v_rcp_f32; saturates to +-1
// for large |x| (exp -> inf gives rcp -> 0; exp -> 0 gives -1).  Absolute
// error ~1 ulp(1.0) ~ 1.2e-7, far inside the 1e-4 parity bar.
__device__ __forceinline__ float fast_tanh(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // 2*log2(e)
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
}

// PReLU: x for x >= 0, w*x otherwise -- as max(x,0) + w*min(x,0) (one of the
// two terms is an exact zero), which needs no compare / VCC select.
__device__ __forceinline__ float prelu_f(float x, float w) { return fmaf(w, fminf(x, 0.f), fmaxf(x, 0.f)); }

__host__ __device__ constexpr inline int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ constexpr inline int rup(int a, int b) { return cdiv(a, b) * b; }

// Smallest stride >= n with stride % 32 == want (bank placement for LDS tiles
// read with ds_read_b32 by 16-lane row groups).
__host__ __device__ constexpr inline int stride_mod32(int n, int want) {
  int s = n;
  while ((s & 31) != want) ++s;
  return s;
}

// Smallest stride >= n with stride % 4 == 2.  A [row][stride] fp32 tile read
// as an MFMA operand (lanes 0-15: 16 rows at column k, lanes 16-31: the same
// rows at column k+1) then hits 32 distinct banks: 16 rows * (stride/2 odd)
// cover the 16 even residues mod 32 and k+1 the odd ones.
__host__ __device__ constexpr inline int stride_2mod4(int n) {
  int s = n;
  while ((s & 3) != 2) ++s;
  return s;
}

// K steps (4 input channels each) of a 1x1-conv GEMM, rounded up to a power
// of two so the GEMM body is one of a few template instantiations.  Tiles are
// zero-padded to 4*ks_for(Cin) channels.
__host__ __device__ constexpr inline int ks_for(int cin) {
  const int ks = cdiv(cin, 4);
  int p = 1;
  while (p < ks) p <<= 1;
  return p;
}
