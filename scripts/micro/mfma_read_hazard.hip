// MFMA result -> VALU read: how many wait states does gfx950 need after the
// LAST MFMA of a dependent accumulate chain before a VALU may read the
// accumulator, against what hipcc inserts?
//
// Round-3 bisection of k_temporal_fused built with the conv_rm W fragments
// hoisted out of its tile loop (dstd_hilo.hip, DSTD_TF_HOISTW, -> wrong
// planes for its second row tile): a plane dump showed that exactly the first
// two of each lane's four accumulator values (acc[0], acc[1]) were wrong.
// hipcc had emitted that row tile's conv_rm as a back-to-back chain
//   v_mfma_f32_16x16x32_f16 x3 (dependent), v_mfma_f32_16x16x16_f16,
//   s_nop 5, ds_read_b32, v_mfma_f32_16x16x16_f16 x2,
//   s_waitcnt lgkmcnt(0), s_nop 6, v_fma_f32 v16, v16 ...; v_fma_f32 v17, v17 ...
// i.e. 8 wait states between the last MFMA and the first VALU read, while in
// the correct row tile the same MFMAs were interleaved with VALU work.
// Each pattern below: the chain in fixed registers v[200:203], then N wait
// states, then four v_mov_b32 reading the accumulator one element at a time;
// against the same chain with 3 x s_nop 7 before the reads.
// hipcc --offload-arch=gfx950 -O3 mfma_read_hazard.hip -o mfma_read_hazard && ./mfma_read_hazard
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define PAD "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"
#define READ "v_mov_b32 %0, v200\n\tv_mov_b32 %1, v201\n\tv_mov_b32 %2, v202\n\tv_mov_b32 %3, v203\n\t"
#define INIT "v_mov_b32 v200, 0\n\tv_mov_b32 v201, 0\n\tv_mov_b32 v202, 0\n\tv_mov_b32 v203, 0\n\ts_nop 4\n\t"
#define C32 "v_mfma_f32_16x16x32_f16 v[200:203], %4, %5, v[200:203]\n\t"
#define C16 "v_mfma_f32_16x16x16_f16 v[200:203], %6, %7, v[200:203]\n\t"
#define OPS : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3) : "v"(a), "v"(b), "v"(a4), "v"(b4) : "v200", "v201", "v202", "v203"

#define CHAIN1 INIT C32 C32 C32
#define CHAIN2 INIT C16 C16 C16
#define CHAIN3 INIT C16
#define CHAIN4 INIT C32 C32 C32 C16 "s_nop 5\n\t" C16 C16
#define CHAIN5 INIT C32 C32 C32 C32 C32 C32
#define CHAIN6 INIT C32
#define NOPS(g) "s_nop " #g "\n\t"
// pairs with a gap: 10 + 8*pair + gap, pair 0: 16->16, 1: 32->32, 2: 32->16, 3: 16->32
#define W0 "s_nop 7\n\t"
#define W1 "s_nop 7\n\ts_nop 3\n\t"
#define W2 PAD
#define EMIT(CH)                                          \
  if constexpr (W == 0) asm volatile(CH W0 READ PAD OPS); \
  else if constexpr (W == 1) asm volatile(CH W1 READ PAD OPS); \
  else asm volatile(CH W2 READ PAD OPS);

// P: the chain (CHAINp); W: wait states between its last MFMA and the first
// read: 0 = 8 (s_nop 7, what hipcc inserted), 1 = 12, 2 = 24 (reference)
template <int P, int W>
__global__ void k(f32x4* out, const f16x8* in, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const f16x8 a = in[2 * i], b = in[2 * i + 1];
  const f16x4 a4 = {a[0], a[2], a[4], a[6]}, b4 = {b[1], b[3], b[5], b[7]};
  float r0, r1, r2, r3;
  if constexpr (P == 1) { EMIT(CHAIN1) }
  else if constexpr (P == 2) { EMIT(CHAIN2) }
  else if constexpr (P == 3) { EMIT(CHAIN3) }
  else if constexpr (P == 4) { EMIT(CHAIN4) }
  else if constexpr (P == 5) { EMIT(CHAIN5) }
  else if constexpr (P == 6) { EMIT(CHAIN6) }
#define PAIR(X, Y, G) else if constexpr (P == 10 + 8 * (X) + (G)) { EMIT(INIT Y NOPS(G) Y) }
#define PAIRXY(X, A, B, G) else if constexpr (P == 10 + 8 * (X) + (G)) { EMIT(INIT A NOPS(G) B) }
  PAIRXY(0, C16, C16, 0) PAIRXY(0, C16, C16, 1) PAIRXY(0, C16, C16, 2) PAIRXY(0, C16, C16, 3)
  PAIRXY(0, C16, C16, 4) PAIRXY(0, C16, C16, 5) PAIRXY(0, C16, C16, 6) PAIRXY(0, C16, C16, 7)
  PAIRXY(1, C32, C32, 0) PAIRXY(1, C32, C32, 1) PAIRXY(1, C32, C32, 2) PAIRXY(1, C32, C32, 3)
  PAIRXY(1, C32, C32, 4) PAIRXY(1, C32, C32, 5) PAIRXY(1, C32, C32, 6) PAIRXY(1, C32, C32, 7)
  PAIRXY(2, C32, C16, 0) PAIRXY(2, C32, C16, 1) PAIRXY(2, C32, C16, 2) PAIRXY(2, C32, C16, 3)
  PAIRXY(2, C32, C16, 4) PAIRXY(2, C32, C16, 5) PAIRXY(2, C32, C16, 6) PAIRXY(2, C32, C16, 7)
  PAIRXY(3, C16, C32, 0) PAIRXY(3, C16, C32, 1) PAIRXY(3, C16, C32, 2) PAIRXY(3, C16, C32, 3)
  PAIRXY(3, C16, C32, 4) PAIRXY(3, C16, C32, 5) PAIRXY(3, C16, C32, 6) PAIRXY(3, C16, C32, 7)
  // references: the pair with 24 wait states between
  else if constexpr (P == 50) { EMIT(INIT C16 PAD C16) }
  else if constexpr (P == 51) { EMIT(INIT C32 PAD C32) }
  else if constexpr (P == 52) { EMIT(INIT C32 PAD C16) }
  else if constexpr (P == 53) { EMIT(INIT C16 PAD C32) }
  else if constexpr (P == 54) { EMIT(INIT C32 C32 C32 C16 PAD C16 C16) }
  out[i] = f32x4{r0, r1, r2, r3};
}

template <int P, int W>
long run(const f16x8* d_in, f32x4* d_o, f32x4* h_a, f32x4* h_b, int n, long* per_elem) {
  hipLaunchKernelGGL((k<P, 2>), dim3(n / 256), dim3(256), 0, 0, d_o, d_in, n);
  hipMemcpy(h_a, d_o, 16 * (size_t)n, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL((k<P, W>), dim3(n / 256), dim3(256), 0, 0, d_o, d_in, n);
  hipMemcpy(h_b, d_o, 16 * (size_t)n, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int e = 0; e < 4; ++e) per_elem[e] = 0;
  for (int i = 0; i < n; ++i) {
    bad += memcmp(&h_a[i], &h_b[i], 16) != 0;
    for (int e = 0; e < 4; ++e) {
      const float x = h_a[i][e], y = h_b[i][e];
      per_elem[e] += memcmp(&x, &y, 4) != 0;
    }
  }
  return bad;
}

// k<P, W> against the reference k<R, 2>
template <int P, int W, int R>
long cmp(const f16x8* d_in, f32x4* d_o, f32x4* h_a, f32x4* h_b, int n) {
  hipLaunchKernelGGL((k<R, 2>), dim3(n / 256), dim3(256), 0, 0, d_o, d_in, n);
  hipMemcpy(h_a, d_o, 16 * (size_t)n, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL((k<P, W>), dim3(n / 256), dim3(256), 0, 0, d_o, d_in, n);
  hipMemcpy(h_b, d_o, 16 * (size_t)n, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int i = 0; i < n; ++i) bad += memcmp(&h_a[i], &h_b[i], 16) != 0;
  return bad;
}

template <int P>
void row(const char* name, const f16x8* d_in, f32x4* d_o, f32x4* h_a, f32x4* h_b, int n) {
  long e8[4], e12[4];
  const long b8 = run<P, 0>(d_in, d_o, h_a, h_b, n, e8), b12 = run<P, 1>(d_in, d_o, h_a, h_b, n, e12);
  printf("%-52s 8 states: %6ld lanes wrong (acc[0..3] %ld %ld %ld %ld) | 12 states: %6ld\n", name, b8, e8[0], e8[1],
         e8[2], e8[3], b12);
}

int main() {
  const int n = 1 << 16;
  _Float16* h_in = (_Float16*)malloc(32 * (size_t)n);
  uint32_t s = 31337;
  for (size_t i = 0; i < 16 * (size_t)n; ++i) {
    s = s * 1664525u + 1013904223u;
    h_in[i] = (_Float16)(((int)(s >> 9) - (1 << 22)) * (1.f / (1 << 21)));
  }
  f16x8* d_in;
  f32x4* d_o;
  hipMalloc(&d_in, 32 * (size_t)n);
  hipMalloc(&d_o, 16 * (size_t)n);
  hipMemcpy(d_in, h_in, 32 * (size_t)n, hipMemcpyHostToDevice);
  f32x4* h_a = (f32x4*)malloc(16 * (size_t)n);
  f32x4* h_b = (f32x4*)malloc(16 * (size_t)n);
  row<6>("one 16x16x32 f16", d_in, d_o, h_a, h_b, n);
  row<3>("one 16x16x16 f16", d_in, d_o, h_a, h_b, n);
  row<1>("3 x 16x16x32 f16, dependent, back to back", d_in, d_o, h_a, h_b, n);
  row<5>("6 x 16x16x32 f16, dependent, back to back", d_in, d_o, h_a, h_b, n);
  row<2>("3 x 16x16x16 f16, dependent, back to back", d_in, d_o, h_a, h_b, n);
  row<4>("hipcc's: 3 x 16x16x32, 16x16x16, s_nop 5, 2 x 16x16x16", d_in, d_o, h_a, h_b, n);
  printf("hipcc's chain vs the chain with 24 states in its gap: 8 / 12 / 24 read states: %ld / %ld / %ld lanes\n",
         cmp<4, 0, 54>(d_in, d_o, h_a, h_b, n), cmp<4, 1, 54>(d_in, d_o, h_a, h_b, n), cmp<4, 2, 54>(d_in, d_o, h_a, h_b, n));
  // two dependent MFMAs (C = previous D, same register) with s_nop g between,
  // read after 8 / 12 / 24 states, against the pair with 24 states between
  const char* nm[4] = {"16x16x16 -> 16x16x16", "16x16x32 -> 16x16x32", "16x16x32 -> 16x16x16", "16x16x16 -> 16x16x32"};
  for (int pr = 0; pr < 4; ++pr) {
    printf("%s, s_nop g between (g = 0..7), lanes wrong read after 8|12|24 states:", nm[pr]);
#define GAP(X, G) if (pr == X) printf(" g%d: %ld|%ld|%ld", G, cmp<10 + 8 * X + G, 0, 50 + X>(d_in, d_o, h_a, h_b, n), \
                                     cmp<10 + 8 * X + G, 1, 50 + X>(d_in, d_o, h_a, h_b, n), cmp<10 + 8 * X + G, 2, 50 + X>(d_in, d_o, h_a, h_b, n));
#define GAPS(X) GAP(X, 0) GAP(X, 1) GAP(X, 2) GAP(X, 3) GAP(X, 4) GAP(X, 5) GAP(X, 6) GAP(X, 7)
    GAPS(0) GAPS(1) GAPS(2) GAPS(3)
    printf("\n");
  }
  return 0;
}
