// Store-data WAR: may a VALU that overwrites an LDS store's data VGPR right
// after the ds_write issues change the bytes written?
//
// Round-3 bisection of k_temporal_fused with the conv_rm W fragments hoisted
// (dstd_hilo.hip, DSTD_TF_HOISTW): only the second row tile's planes were
// wrong, and the only code difference at their stores was
//   v_add_u32_e32 v20, 0x15f00, v60
//   ds_write_b64 v20, v[18:19]            (hi plane)
//   v_add_u32_e32 v18, 0x169f0, v60       (overwrites the data register just stored)
//   ds_write_b64 v18, v[16:17]            (lo plane)
// hipcc pads the store-data hazard only for stores wider than 64 bits.
//   S1  ds_write_b64, first data VGPR overwritten by the next VALU
//   S2  ds_write_b64, second data VGPR overwritten
//   S3  ds_write_b32, data VGPR overwritten
//   S4  ds_write_b64 with s_nop 0 before the overwrite
//   S5  ds_write_b128 with s_nop 1 (hipcc's pad for wide stores)
// Each against the same store with s_waitcnt lgkmcnt(0) before the
// overwrite; 1 M lanes, bitwise on the LDS contents.
// hipcc --offload-arch=gfx950 -O3 ds_store_war.hip -o ds_store_war && ./ds_store_war
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

template <int P, int SAFE>
__global__ __launch_bounds__(256) void k(uint4* out, const uint4* in) {
  __shared__ uint4 lds[256];
  const int t = threadIdx.x;
  lds[t] = make_uint4(0xAAAAAAAAu, 0xAAAAAAAAu, 0xAAAAAAAAu, 0xAAAAAAAAu);
  __syncthreads();
  const uint4 d = in[blockIdx.x * 256 + t];
  const uint32_t addr = (uint32_t)(uintptr_t)(lds + t);
  const uint32_t x = d.x, y = d.y, z = d.z, w = d.w;
  // the data goes through fixed registers v[200:203] so that one half of a
  // pair can be named
#define LD4 "v_mov_b32 v200, %0\n\tv_mov_b32 v201, %1\n\tv_mov_b32 v202, %2\n\tv_mov_b32 v203, %3\n\ts_nop 4\n\t"
#define CLOB "v200", "v201", "v202", "v203", "memory"
  if constexpr (P == 1) {
    if (SAFE) asm volatile(LD4 "ds_write_b64 %4, v[200:201]\n\ts_waitcnt lgkmcnt(0)\n\tv_add_u32 v200, 0x15f00, %4" :: "v"(x), "v"(y), "v"(z), "v"(w), "v"(addr) : CLOB);
    else asm volatile(LD4 "ds_write_b64 %4, v[200:201]\n\tv_add_u32 v200, 0x15f00, %4" :: "v"(x), "v"(y), "v"(z), "v"(w), "v"(addr) : CLOB);
  } else if constexpr (P == 2) {
    if (SAFE) asm volatile(LD4 "ds_write_b64 %4, v[200:201]\n\ts_waitcnt lgkmcnt(0)\n\tv_add_u32 v201, 0x15f00, %4" :: "v"(x), "v"(y), "v"(z), "v"(w), "v"(addr) : CLOB);
    else asm volatile(LD4 "ds_write_b64 %4, v[200:201]\n\tv_add_u32 v201, 0x15f00, %4" :: "v"(x), "v"(y), "v"(z), "v"(w), "v"(addr) : CLOB);
  } else if constexpr (P == 3) {
    if (SAFE) asm volatile(LD4 "ds_write_b32 %4, v200\n\ts_waitcnt lgkmcnt(0)\n\tv_add_u32 v200, 0x15f00, %4" :: "v"(x), "v"(y), "v"(z), "v"(w), "v"(addr) : CLOB);
    else asm volatile(LD4 "ds_write_b32 %4, v200\n\tv_add_u32 v200, 0x15f00, %4" :: "v"(x), "v"(y), "v"(z), "v"(w), "v"(addr) : CLOB);
  } else if constexpr (P == 4) {
    if (SAFE) asm volatile(LD4 "ds_write_b64 %4, v[200:201]\n\ts_waitcnt lgkmcnt(0)\n\tv_add_u32 v200, 0x15f00, %4" :: "v"(x), "v"(y), "v"(z), "v"(w), "v"(addr) : CLOB);
    else asm volatile(LD4 "ds_write_b64 %4, v[200:201]\n\ts_nop 0\n\tv_add_u32 v200, 0x15f00, %4" :: "v"(x), "v"(y), "v"(z), "v"(w), "v"(addr) : CLOB);
  } else {
    if (SAFE) asm volatile(LD4 "ds_write_b128 %4, v[200:203]\n\ts_waitcnt lgkmcnt(0)\n\tv_mov_b32 v200, 0" :: "v"(x), "v"(y), "v"(z), "v"(w), "v"(addr) : CLOB);
    else asm volatile(LD4 "ds_write_b128 %4, v[200:203]\n\ts_nop 1\n\tv_mov_b32 v200, 0" :: "v"(x), "v"(y), "v"(z), "v"(w), "v"(addr) : CLOB);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  out[blockIdx.x * 256 + t] = lds[t];
}

template <int P>
long run(const uint4* d_in, uint4* d_o, uint4* h_a, uint4* h_b, int nb) {
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
  uint4* h_in = (uint4*)malloc(16 * 256 * (size_t)nb);
  uint32_t s = 4242;
  uint32_t* p = (uint32_t*)h_in;
  for (size_t i = 0; i < 4 * 256 * (size_t)nb; ++i) p[i] = (s = s * 1664525u + 1013904223u);
  uint4 *d_in, *d_o;
  hipMalloc(&d_in, 16 * 256 * (size_t)nb);
  hipMalloc(&d_o, 16 * 256 * (size_t)nb);
  hipMemcpy(d_in, h_in, 16 * 256 * (size_t)nb, hipMemcpyHostToDevice);
  uint4* h_a = (uint4*)malloc(16 * 256 * (size_t)nb);
  uint4* h_b = (uint4*)malloc(16 * 256 * (size_t)nb);
  const int n = nb * 256;
  printf("S1 ds_write_b64, data[0] overwritten next        : %ld of %d lanes differ\n", run<1>(d_in, d_o, h_a, h_b, nb), n);
  printf("S2 ds_write_b64, data[1] overwritten next        : %ld of %d lanes differ\n", run<2>(d_in, d_o, h_a, h_b, nb), n);
  printf("S3 ds_write_b32, data overwritten next           : %ld of %d lanes differ\n", run<3>(d_in, d_o, h_a, h_b, nb), n);
  printf("S4 ds_write_b64, s_nop 0, data[0] overwritten    : %ld of %d lanes differ\n", run<4>(d_in, d_o, h_a, h_b, nb), n);
  printf("S5 ds_write_b128, s_nop 1, data overwritten      : %ld of %d lanes differ\n", run<5>(d_in, d_o, h_a, h_b, nb), n);
  return 0;
}
