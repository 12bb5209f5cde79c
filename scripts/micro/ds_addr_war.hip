// Is an LDS read's address VGPR consumed when the ds_read issues, or may a
// VALU that overwrites it right afterwards change the address?  (Round-3
// bisection of the DSTD_TF_HOISTW build of k_temporal_fused: its second row
// tile's W fragments were read by
//   ds_read_b64 v[36:37], v16 ; ds_read_b64 v[38:39], v17 ; v_cndmask_b32 v16, 0, 1, s[8:9]
// and only that row tile came out wrong.)
//   D1  ds_read_b64 then the address register overwritten by the next VALU
//   D3  two ds_read_b64, the first's address overwritten after the second
// Each pattern against the same reads with s_waitcnt lgkmcnt(0) before the
// overwrite; 1 M lanes, bitwise.
// hipcc --offload-arch=gfx950 -O3 ds_addr_war.hip -o ds_addr_war && ./ds_addr_war
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

template <int P, int SAFE>
__global__ __launch_bounds__(256) void k(uint4* out, const uint32_t* in) {
  __shared__ uint32_t lds[4096];
  const int t = threadIdx.x;
  for (int i = t; i < 4096; i += 256) lds[i] = in[blockIdx.x * 4096 + i];
  __syncthreads();
  uint32_t addr = (uint32_t)(uintptr_t)(lds + 8 * ((t * 7) & 255));  // 32-byte aligned, per lane
  uint32_t bad = (uint32_t)(uintptr_t)(lds + 8 * ((t * 13 + 5) & 255));
  uint4 r = make_uint4(0, 0, 0, 0);
  if constexpr (P == 1) {
    uint2 v;
    uint32_t a = addr;
    if (SAFE)
      asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)\n\tv_mov_b32 %1, %2\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(v), "+v"(a) : "v"(bad));
    else
      asm volatile("ds_read_b64 %0, %1\n\tv_mov_b32 %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v), "+v"(a) : "v"(bad));
    r = make_uint4(v.x, v.y, a, 0);
  } else {
    uint2 v, w;
    uint32_t a = addr, b = addr + 16;
    if (SAFE)
      asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %3\n\ts_waitcnt lgkmcnt(0)\n\tv_mov_b32 %2, %4\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(v), "=&v"(w), "+v"(a), "+v"(b) : "v"(bad));
    else
      asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %3\n\tv_mov_b32 %2, %4\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(v), "=&v"(w), "+v"(a), "+v"(b) : "v"(bad));
    r = make_uint4(v.x, v.y, w.x, w.y);
  }
  out[blockIdx.x * 256 + t] = r;
}

template <int P>
long run(const uint32_t* d_in, uint4* d_o, uint4* h_a, uint4* h_b, int nb) {
  hipLaunchKernelGGL((k<P, 1>), dim3(nb), dim3(256), 0, 0, d_o, d_in);
  hipMemcpy(h_a, d_o, 16 * (size_t)nb * 256, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL((k<P, 0>), dim3(nb), dim3(256), 0, 0, d_o, d_in);
  hipMemcpy(h_b, d_o, 16 * (size_t)nb * 256, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int i = 0; i < nb * 256; ++i) bad += memcmp(&h_a[i], &h_b[i], 16) != 0;
  return bad;
}

int main() {
  const int nb = 4096;
  uint32_t* h_in = (uint32_t*)malloc(4 * 4096 * (size_t)nb);
  uint32_t s = 99;
  for (size_t i = 0; i < 4096 * (size_t)nb; ++i) h_in[i] = (s = s * 1664525u + 1013904223u);
  uint32_t* d_in;
  uint4* d_o;
  hipMalloc(&d_in, 4 * 4096 * (size_t)nb);
  hipMalloc(&d_o, 16 * 256 * (size_t)nb);
  hipMemcpy(d_in, h_in, 4 * 4096 * (size_t)nb, hipMemcpyHostToDevice);
  uint4* h_a = (uint4*)malloc(16 * 256 * (size_t)nb);
  uint4* h_b = (uint4*)malloc(16 * 256 * (size_t)nb);
  printf("D1 ds_read_b64, address overwritten by the next VALU : %ld of %d lanes differ\n",
         run<1>(d_in, d_o, h_a, h_b, nb), nb * 256);
  printf("D3 two ds_read_b64, first address overwritten after : %ld of %d lanes differ\n",
         run<3>(d_in, d_o, h_a, h_b, nb), nb * 256);
  return 0;
}
