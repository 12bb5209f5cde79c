// Split-f16 GC kernels for the 64 -> 64 DSTDGC launches of the forward (the
// five encoder spatial GCs and the six 64-channel temporal GCs of H36M /
// CMU / 3DPW), plus the per-forward weight-image preparation.  Operand
// format, slot maps and the precision argument: dstd_hilo.h.
//
// Design (vs the exact-fp32 wave kernels of dstd_wave.hip, which spend ~55%
// of their time in v_mfma_f32_16x16x4_f32):
//  * every contraction runs as three v_mfma_f32_16x16x32_f16 (hi*hi, hi*lo,
//    lo*hi): a 16x16x32 block costs 48 MFMA cycles instead of 256;
//  * units are small -- (sample, frame) spatial, (sample, joint) temporal --
//    so a wave holds one unit in ~200 registers and two waves share a SIMD:
//    one wave's hi/lo splitting, epilogue and stores overlap the other's
//    MFMAs;
//  * the 1x1 conv is computed transposed (positions = MFMA rows) and its
//    accumulators of tiles 2s, 2s+1 are split into the A operand of the
//    aggregation K-step s; the adjacency arrives as ready-made hi/lo B
//    fragments (one 16-byte load per lane and plane, no LDS image);
//  * the output accumulators are again the B operand of the next DSTDGC's
//    P/Q conv; everything else (BatchNorm, residual, PReLU) is register
//    epilogue, stores are 16 bytes per lane.
// Weights come as fragment images (k_hl_prep) copied into LDS with 16-byte
// loads.  Units are contiguous ranges per wave, no barrier after the prologue.
#include <type_traits>

#include "dstd_common.h"
#include "dstd_hilo.h"
#include "dstd_kernels.h"

// Workgroup timeline of the split adjacency kernel (debug builds,
// -DDSTD_STAMPS; scripts/timeline.py --hl): s_memrealtime at entry, prologue
// done, tiles done, exit.
#ifdef DSTD_TF_DUMPP
__device__ unsigned g_dbg_planes[64 * 1024];
extern "C" int dstd_debug_planes(unsigned* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dbg_planes), sizeof(g_dbg_planes), 0);
}
#endif
#ifdef DSTD_TF_DEBUGW
__device__ unsigned g_dbg_w[2 * 512 * 24];
extern "C" int dstd_debug_w(unsigned* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dbg_w), sizeof(g_dbg_w), 0);
}
#endif
#ifdef DSTD_STAMPS
// modes: 0 k_adj_hl<0>, 1 k_adj_hl<1>, 2 k_temporal_fused phase 3 (start,
// E/F ready, tiles issued, stores drained), 3 k_temporal_fused C = 64 (entry,
// chunk 0 phase 1 done, units done, exit), 5 k_block_fused 64 -> 64 (entry,
// spatial units done, after the barrier, exit)
__device__ unsigned long long g_tl_hl[6][2048][4];
#define TLH(m, i) \
  if (threadIdx.x == 0 && blockIdx.x < 2048) g_tl_hl[m][blockIdx.x][i] = __builtin_amdgcn_s_memrealtime();
#else
#define TLH(m, i)
#endif

namespace dstd {

namespace {


__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ f16x8 as_h8(const uint4& v) { return __builtin_bit_cast(f16x8, v); }
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma32(const f16x8& a, const f16x8& b, f32x4 c) {
#ifdef DSTD_ABL_MFMA
  c[0] += (float)a[0] * (float)b[0];
  return c;
#else
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#endif
}

// hi/lo pair of an f32x4 quartet from two accumulator tiles (slots e = 0..3
// from the first, 4..7 from the second)
__device__ __forceinline__ void split_acc(const f32x4& a, const f32x4& b, f16x8& hi, f16x8& lo) {
  split8(make_float4(a[0], a[1], a[2], a[3]), make_float4(b[0], b[1], b[2], b[3]), hi, lo);
}
// the same with no second tile (slots 4..7 zero)
__device__ __forceinline__ void split_acc(const f32x4& a, f16x8& hi, f16x8& lo) {
  uint2 h, l;
  split4(make_float4(a[0], a[1], a[2], a[3]), h, l);
  hi = __builtin_bit_cast(f16x8, make_uint4(h.x, h.y, 0u, 0u));
  lo = __builtin_bit_cast(f16x8, make_uint4(l.x, l.y, 0u, 0u));
}

// A zero the compiler cannot see through: added to LDS fragment addresses
// inside the unit loop it stops hipcc from hoisting the (loop-invariant)
// weight-fragment reads out of the loop into ~150 live registers.
__device__ __forceinline__ int opaque_zero() {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}

__device__ __forceinline__ int unit_range(int nunits, int& uend) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hw = blockDim.x >> 6;  // waves per workgroup (per kernel: spatial_nt / temporal_nt)
  const int gw = blockIdx.x * hw + wave;
  const long nw = (long)gridDim.x * hw;
  uend = (int)(((long)(gw + 1) * nunits) / nw);
  return (int)(((long)gw * nunits) / nw);
}

// Raw buffer access: every global load / store of the unit loop goes through
// a buffer resource over the unit's own rows, and a lane with nothing to
// load / store gets an out-of-range offset (loads return 0, stores are
// dropped).  No exec-mask branches in the loop, so hipcc's vmcnt bookkeeping
// stays exact across the loop back-edge (with branchy loads / stores it
// waited for the previous unit's stores at the top of every unit).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
template <int AUX = 0>
__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
#ifdef DSTD_ABL_LOAD
  const float f = (float)(off & 255) * 1e-3f;
  return make_float4(f, f, f, f);
#endif
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
}
__device__ __forceinline__ uint4 bldu4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
#ifdef DSTD_ABL_LOAD
  return make_uint4(off & 0x3c003c00u, off, off, off);
#endif
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
// cache policy of the activation / P-Q stores (GC kernels) and of the
// adjacency plane stores (buffer aux bits: 1 sc0, 2 nt, 16 sc1).  GC
// outputs go write-through (sc1): the next launch reads them from other
// XCDs anyway, and no dirty L2 lines are left for the kernel boundary to
// write back (forward 2% faster; sc1 on the adjacency planes measured 3%
// slower, nt 30% slower -- scripts/ab_kernels.py)
#ifndef DSTD_GC_ST_AUX
#define DSTD_GC_ST_AUX 16
#endif
#ifndef DSTD_ADJ_ST_AUX
#define DSTD_ADJ_ST_AUX 0
#endif
// (experiments: cache policy of the temporal units' h-row loads and of the
// encoder residual loads -- both the last read of those rows)
#ifndef DSTD_TF_H_LD_AUX
#define DSTD_TF_H_LD_AUX 0
#endif
#ifndef DSTD_TF_R_LD_AUX
#define DSTD_TF_R_LD_AUX 0
#endif
template <int AUX = DSTD_GC_ST_AUX>
__device__ __forceinline__ void bst4(__amdgpu_buffer_rsrc_t r, uint32_t off, float4 v) {
#ifdef DSTD_ABL_STORE
  if (v.x == 12345.f) off = 0;  // keep the value alive; store only lanes with nothing to store
  else off = OOB;
#endif
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, AUX);
}

// ---- range scaling helpers (dstd_hilo.h "range scaling") ----
// 2^e as a float, e in [-126, 127]
__device__ __forceinline__ float pow2f(int e) { return __uint_as_float((uint32_t)(127 + e) << 23); }
// e with v < 2^e for the bits of a non-negative float v (frexp's exponent;
// zero and denormals -> -126)
__device__ __forceinline__ int fexp_bits(uint32_t b) { return (int)(b >> 23) - 126; }
// max over the wave of non-negative floats, as bits (the bit patterns of
// non-negative floats order like the values): DPP within rows of 16, then
// the four row maxima through SGPRs -- a wave-uniform result
__device__ __forceinline__ uint32_t wave_max_bits(float v) {
  uint32_t b = __float_as_uint(v);
  b = max(b, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  b = max(b, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  b = max(b, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0x141, 0xF, 0xF, false));  // row_half_mirror
  b = max(b, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0x140, 0xF, 0xF, false));  // row_mirror
  const uint32_t r0 = __builtin_amdgcn_readlane(b, 0), r1 = __builtin_amdgcn_readlane(b, 16);
  const uint32_t r2 = __builtin_amdgcn_readlane(b, 32), r3 = __builtin_amdgcn_readlane(b, 48);
  return max(max(r0, r1), max(r2, r3));
}
// (accumulators that may come straight from an MFMA: plain fmaxf, which the
// hazard recognizer pads; see amax2)
__device__ __forceinline__ float amax4_mfma(float m, const f32x4& v) {
  return fmaxf(fmaxf(m, fmaxf(fabsf(v[0]), fabsf(v[1]))), fmaxf(fabsf(v[2]), fabsf(v[3])));
}
// max |x| over many values on four independent v_max3 chains: one chain
// puts an inline-asm max right behind the one it depends on, and hipcc pads
// every such pair with an s_nop (it cannot see the asm is not a
// transcendental); four chains leave independent work between them
struct AmaxAcc {
  float m[4] = {0.f, 0.f, 0.f, 0.f};
  int j = 0;  // (compile-time once the caller's loops are unrolled)
  __device__ __forceinline__ void add(float a, float b) {
    m[j] = amax2(m[j], a, b);
    j = (j + 1) & 3;
  }
  __device__ __forceinline__ void add(const float4& v) { add(v.x, v.y), add(v.z, v.w); }
  __device__ __forceinline__ void add(const f32x4& v) { add(v[0], v[1]), add(v[2], v[3]); }
  __device__ __forceinline__ float get() const { return amax2(amax2(m[0], m[1], m[2]), m[3], m[3]); }
};
__device__ __forceinline__ float4 mul4(const float4& v, float s) { return make_float4(v.x * s, v.y * s, v.z * s, v.w * s); }
// input shift of a GC unit: the smallest sx >= 0 with max|x| * max(1, |W|_inf)
// < 2^(14 + sx) and max|b| < 2^(14 + sx); efb / eb: fexp of max(1, |W|_inf) / max|b|
__device__ __forceinline__ int input_shift(uint32_t xmax_bits, int efb, int eb) {
  return hl_range_shift(max(fexp_bits(xmax_bits) + efb, eb));
}

}  // namespace

// ===========================================================================
// weight images: one workgroup per job
// ===========================================================================
__global__ __launch_bounds__(256) void k_hl_prep(HLPrepArgs a) {
  const HLJob& j = a.jobs[blockIdx.x];
  const int tid = threadIdx.x;
  __shared__ float red[4];
  auto block_max = [&](float m) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    __syncthreads();  // red[] is reused
    if ((tid & 63) == 0) red[tid >> 6] = m;
    __syncthreads();
    return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  };
  // HLJ_CONV / HLJ_RM: w[0] is rows x cols; HLJ_PQ: nblk blocks of 2 x cols
  const int n = j.kind != HLJ_PQ ? j.rows * j.cols : 2 * j.cols * j.nblk;
  float m = 0.f;
  for (int i = tid; i < n; i += 256)
    m = fmaxf(m, fabsf(j.kind != HLJ_PQ ? j.w[0][i] : j.w[i / (2 * j.cols)][i % (2 * j.cols)]));
  m = block_max(m);
  // 2^s with max|w| * 2^s < 2^14: low halves of the scaled weights stay normal
  int e = 0;
  float scale = 1.f;
  if (m > 0.f && isfinite(m)) {
    frexpf(m, &e);  // m = f * 2^e, f in [0.5, 1)
    scale = ldexpf(1.f, 14 - e);
  }
  if (tid == 0) j.inv_scale[HLS_INV] = 1.f / scale;
  // range bounds of the split operands (dstd_hilo.h "range scaling")
  if (j.kind == HLJ_CONV) {  // |W|_inf and max|b|
    float nrm = 0.f, bm = 0.f;
    for (int r = tid; r < j.rows; r += 256) {
      float acc = 0.f;
      for (int k = 0; k < j.cols; ++k) acc += fabsf(j.w[0][r * j.cols + k]);
      nrm = fmaxf(nrm, acc);
      if (j.bias) bm = fmaxf(bm, fabsf(j.bias[r]));
    }
    nrm = block_max(nrm);
    bm = block_max(bm);
    if (tid == 0) {
      j.inv_scale[HLS_BOUND] = nrm;
      j.inv_scale[HLS_BMAX] = bm;
    }
  } else if (j.kind == HLJ_RM) {  // |alpha| max_r (sum_k |W[r][k]| + |b[r]|) + max|Astat|
    float rb = 0.f, am = 0.f;
    for (int r = tid; r < j.rows; r += 256) {
      float acc = fabsf(j.bias[r]);
      for (int k = 0; k < j.cols; ++k) acc += fabsf(j.w[0][r * j.cols + k]);
      rb = fmaxf(rb, acc);
    }
    for (int i = tid; i < j.nastat; i += 256) am = fmaxf(am, fabsf(j.astat[i]));
    rb = block_max(rb);
    am = block_max(am);
    if (tid == 0) j.inv_scale[HLS_BOUND] = fabsf(*j.alpha) * rb + am;
  }
  if (j.kind == HLJ_RM)  // the conv_rm bias as the adjacency kernel reads it (LDS-staged per workgroup)
    for (int r = tid; r < j.rows; r += 256) j.bias_out[r] = j.bias[r];
  if (j.kind == HLJ_CONV) {
    const int NCT = cdiv(j.rows, 16), KSI = cdiv(j.cols, 32);
    for (int i = tid; i < NCT * KSI * 64; i += 256) {
      const int lane = i & 63, ks = (i >> 6) % KSI, ct = (i >> 6) / KSI;
      const int c = 16 * ct + (lane & 15), k0 = 32 * ks + 8 * (lane >> 4);
      float v[8];
#pragma unroll
      for (int e8 = 0; e8 < 8; ++e8) v[e8] = c < j.rows && k0 + e8 < j.cols ? j.w[0][c * j.cols + k0 + e8] * scale : 0.f;
      uint4 hi, lo;
      split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), hi, lo);
      j.img[((ct * KSI + ks) * 2 + 0) * 64 + lane] = hi;
      j.img[((ct * KSI + ks) * 2 + 1) * 64 + lane] = lo;
    }
  } else if (j.kind == HLJ_RM) {
    const int NSF = hl_rm_nsf(j.cols), RT = cdiv(j.rows, 16);
    for (int i = tid; i < RT * NSF * 64; i += 256) {
      const int lane = i & 63, s = (i >> 6) % NSF, rt = (i >> 6) / NSF;
      const int r = 16 * rt + (lane & 15), k0 = 32 * s + 8 * (lane >> 4);
      float v[8];
#pragma unroll
      for (int e8 = 0; e8 < 8; ++e8) v[e8] = r < j.rows && k0 + e8 < j.cols ? j.w[0][r * j.cols + k0 + e8] * scale : 0.f;
      uint4 hi, lo;
      split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), hi, lo);
      j.img[((rt * NSF + s) * 2 + 0) * 64 + lane] = hi;
      j.img[((rt * NSF + s) * 2 + 1) * 64 + lane] = lo;
    }
    if (hl_rm_tail(j.cols)) {  // 16x16x16 tail step: 4 halves per lane and plane
      uint2* img16 = reinterpret_cast<uint2*>(j.img + RT * NSF * 2 * 64);
      for (int i = tid; i < RT * 64; i += 256) {
        const int lane = i & 63, rt = i >> 6;
        const int r = 16 * rt + (lane & 15), k0 = 32 * NSF + 4 * (lane >> 4);
        float v[4];
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) v[e4] = r < j.rows && k0 + e4 < j.cols ? j.w[0][r * j.cols + k0 + e4] * scale : 0.f;
        uint4 hi, lo;
        split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(0.f, 0.f, 0.f, 0.f), hi, lo);
        img16[(rt * 2 + 0) * 64 + lane] = make_uint2(hi.x, hi.y);
        img16[(rt * 2 + 1) * 64 + lane] = make_uint2(lo.x, lo.y);
      }
    }
  } else {
    const int KSO = cdiv(cdiv(j.cols, 16), 2);
    for (int i = tid; i < KSO * 64; i += 256) {
      const int lane = i & 63, ks = i >> 6;
      const int ch = lane & 15, kg = lane >> 4;
      float v[8];
#pragma unroll
      for (int e8 = 0; e8 < 8; ++e8) {
        const int c = 16 * (2 * ks + (e8 >> 2)) + 4 * kg + (e8 & 3);
        v[e8] = ch < 2 * j.nblk && c < j.cols ? j.w[ch >> 1][(ch & 1) * j.cols + c] * scale : 0.f;
      }
      uint4 hi, lo;
      split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), hi, lo);
      j.img[(ks * 2 + 0) * 64 + lane] = hi;
      j.img[(ks * 2 + 1) * 64 + lane] = lo;
    }
  }
}

// ===========================================================================
// Spatial GC, two graphs (DSTDGCB.forward model/dstdgcn.py:141-154 with
// DSTDGC.forward spatial :80-87), unit = (sample n, frame t):
//   y[c][w] = sum_g sum_v (W_g x + b_g)[v][c] Adj_g[t][v][w]
//   h = prelu(bn(y) + r)  ->  NTVC, and P_t/Q_t of h ([B][T][V][4]);
//   r = x (64 -> 64) or bn_r(W_r x + b_r) (the residual conv of conv_st_in
//   6 -> 64 and conv_st_out 64 -> 3, :117-121), computed in output layout
//   (A = W_r fragments, B = x rows of the output joints).
// ===========================================================================
#ifndef DSTD_HL_WPE
#define DSTD_HL_WPE 2
#endif
// threads per workgroup: one workgroup of 4 x (waves per SIMD) waves per CU,
// so a CU stages one copy of the weight images (A/B against two 4-wave
// workgroups: forward -2.3%)
constexpr int spatial_nt() { return 64 * 4 * DSTD_HL_WPE; }
// identity residual loaded after the aggregations (see spatial_units)
#ifndef DSTD_SP_LATE_RES
#define DSTD_SP_LATE_RES (DSTD_HL_WPE > 2)
#endif
constexpr bool kSpLateRes = DSTD_SP_LATE_RES;

// 8 consecutive channels k0 .. k0+7 of row `row` of a unit (C channels per
// row, zero past C; C % 8 == 0 or C == 6 / 3)
template <int C>
__device__ __forceinline__ void load_row8(__amdgpu_buffer_rsrc_t r, int row, int k0, float4& lo4, float4& hi4) {
  if constexpr (C % 8 == 0) {
    const uint32_t off = (uint32_t)(row * C + k0) * 4;
    lo4 = bld4(r, off);
    hi4 = bld4(r, off + 16);
  } else {
    // C < 8: only k0 == 0 has data; rows are 4-byte aligned (dword loads)
    const uint32_t off = k0 == 0 ? (uint32_t)(row * C) * 4 : OOB;
    float e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = 0.f;
#pragma unroll
    for (int i = 0; i < C; ++i)
      e[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off + 4 * i, 0, 0));
    lo4 = make_float4(e[0], e[1], e[2], e[3]);
    hi4 = make_float4(e[4], e[5], e[6], e[7]);
  }
}

// conv_st_in's 6-channel input row built on the fly from the model input
// (model/dstdgcn.py:298-303): x6 = (x[t][v], x[t][v] - x[T-1][v]); rf / rl:
// the unit's frame and the last frame ([V][3] each); only k0 == 0 has data
__device__ __forceinline__ void load_x6row(__amdgpu_buffer_rsrc_t rf, __amdgpu_buffer_rsrc_t rl, int row, int k0,
                                           float4& lo4, float4& hi4) {
  const uint32_t off = k0 == 0 ? (uint32_t)row * 12 : OOB;
  float c[3], l[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    c[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rf, off + 4 * i, 0, 0));
    l[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rl, off + 4 * i, 0, 0));
  }
  lo4 = make_float4(c[0], c[1], c[2], c[0] - l[0]);
  hi4 = make_float4(c[1] - l[1], c[2] - l[2], 0.f, 0.f);
}

// folded BN vectors [V][C] -> LDS [c/4][v] for NCT*4 channel quads (zero past C)
template <int C, int NCT>
__device__ __forceinline__ void stage_bnC(float4* dst, const float* src, int V, int tid) {
  for (int i = tid; i < V * 4 * NCT; i += (int)blockDim.x) {
    const int v = i / (4 * NCT), c4 = i % (4 * NCT);
    float e[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) e[q] = 4 * c4 + q < C ? src[v * C + 4 * c4 + q] : 0.f;
    dst[c4 * V + v] = make_float4(e[0], e[1], e[2], e[3]);
  }
}

// The stage (LDS images) and the unit loop of the spatial GC (k_spatial_hl;
// factored out in round 3 for the fused-spatial experiments of DESIGN.md §4,
// whose kernels read the adjacency B fragments from LDS through load_adj_g).
template <int V, int CIN, int COUT>
struct SpatialStage {
  static constexpr bool RES = CIN != COUT;
  static constexpr int KSI = cdiv(CIN, 32), NCT = cdiv(COUT, 16), KSO = cdiv(NCT, 2);
  static constexpr int WIMG = NCT * KSI * 2 * 64, PIMG = KSO * 2 * 64;
  uint4 wl[RES ? 3 : 2][WIMG];  // conv (graphs 0, 1), residual conv
  uint4 pql[PIMG];
  float4 bnl[RES ? 4 : 2][4 * NCT * V];
  float bfl[3][16 * NCT];
  float bql[4];
  float scl[4];
  int rng[3];
};

// every global load before the first LDS write (one memory round trip)
template <int V, int CIN, int COUT, int NTH>
__device__ __forceinline__ void stage_spatial(const SpatialHLArgs& a, SpatialStage<V, CIN, COUT>& st, int tid) {
  using S = SpatialStage<V, CIN, COUT>;
  constexpr bool RES = S::RES;
  constexpr int NCT = S::NCT, WIMG = S::WIMG, PIMG = S::PIMG, NIMG = (RES ? 3 : 2) * WIMG;
  constexpr int NW = cdiv(NIMG, NTH), NP = cdiv(PIMG, NTH), NBN = cdiv(V * 4 * NCT, NTH);
  constexpr int NBV = RES ? 4 : 2;
  uint4 wv[NW], pv[NP];
  float4 bv[NBV][NBN];
#pragma unroll
  for (int it = 0; it < NW; ++it) {
    const int i = min(tid + it * NTH, NIMG - 1);
    wv[it] = a.wimg[i / WIMG][i % WIMG];
  }
#pragma unroll
  for (int it = 0; it < NP; ++it) pv[it] = a.pqimg[min(tid + it * NTH, PIMG - 1)];
  const float* bsrc[4] = {a.bn_s, a.bn_h, a.rbn_s, a.rbn_h};
#pragma unroll
  for (int q = 0; q < NBV; ++q)
#pragma unroll
    for (int it = 0; it < NBN; ++it) {
      const int i = min(tid + it * NTH, V * 4 * NCT - 1);
      const int v = i / (4 * NCT), c4 = i % (4 * NCT);
      if constexpr (COUT % 4 == 0) {
        bv[q][it] = ld4(bsrc[q] + v * COUT + 4 * c4);
      } else {  // thin output (3 channels): element loads, zero past COUT
        float e[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) e[r] = 4 * c4 + r < COUT ? bsrc[q][v * COUT + 4 * c4 + r] : 0.f;
        bv[q][it] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
  const int nbf = (RES ? 3 : 2) * 16 * NCT;
  static_assert((RES ? 3 : 2) * 16 * NCT <= NTH, "one conv bias per thread");
  const float bf = tid < nbf && tid % (16 * NCT) < COUT ? a.bf[tid / (16 * NCT)][tid % (16 * NCT)] : 0.f;
#pragma unroll
  for (int it = 0; it < NW; ++it) {
    const int i = tid + it * NTH;
    if (i < NIMG) st.wl[i / WIMG][i % WIMG] = wv[it];
  }
#pragma unroll
  for (int it = 0; it < NP; ++it)
    if (tid + it * NTH < PIMG) st.pql[tid + it * NTH] = pv[it];
#pragma unroll
  for (int q = 0; q < NBV; ++q)
#pragma unroll
    for (int it = 0; it < NBN; ++it) {
      const int i = tid + it * NTH;
      if (i < V * 4 * NCT) {
        const int v = i / (4 * NCT), c4 = i % (4 * NCT);
        st.bnl[q][c4 * V + v] = bv[q][it];
      }
    }
  if (tid < nbf) st.bfl[tid / (16 * NCT)][tid % (16 * NCT)] = bf;
  if (tid < 4) st.bql[tid] = a.pqb[tid >> 1][tid & 1];
  if (tid == 0) {
    st.scl[0] = *a.wscale[0];
    st.scl[1] = *a.wscale[1];
    st.scl[2] = *a.pqscale;
    st.scl[3] = RES ? *a.wscale[2] : 0.f;
    // range: |W_f|_inf and max|b_f| over both graphs, the planes' shared shift
    st.rng[0] = fexp_bits(__float_as_uint(fmaxf(1.f, fmaxf(a.wscale[0][HLS_BOUND], a.wscale[1][HLS_BOUND]))));
    st.rng[1] = fexp_bits(__float_as_uint(fmaxf(a.wscale[0][HLS_BMAX], a.wscale[1][HLS_BMAX])));
    st.rng[2] = hl_range_shift(fexp_bits(__float_as_uint(fmaxf(a.adjb[0][HLS_BOUND], a.adjb[1][HLS_BOUND]))));
  }
}

// The spatial GC units u, u + ustep, ... < uend (unit = (sample, frame) =
// n * T + t); load_adj_g(u, g, ab[NWT][2]) fetches the unit's graph-g
// adjacency B fragments (hi, lo planes) for its two w tiles.
// (k_block_fused: a sink that also receives every unit's temporal P/Q -- the
// values it stores -- and returns the range flag of phase 1's prologue)
struct NoPQSink {
  __device__ int operator()(int, int, float, float, float, float) const { return 0; }
};
template <int V, int CIN, int COUT, typename AdjLoad, bool LATE_RES = kSpLateRes, int ST_AUX = DSTD_GC_ST_AUX,
          typename PQSink = NoPQSink>
__device__ __forceinline__ int spatial_units(const SpatialHLArgs& a, const SpatialStage<V, CIN, COUT>& st, int u,
                                             int uend, int ustep, AdjLoad load_adj_g, PQSink pq_sink = {}) {
  int bad = 0;
  using SM = SlotMap<V, true>;
  constexpr bool RES = CIN != COUT;
  constexpr int NWT = cdiv(V, 16);
  constexpr int KSI = cdiv(CIN, 32);   // conv k-steps
  constexpr int NCT = cdiv(COUT, 16);  // output channel tiles
  constexpr int KSO = cdiv(NCT, 2);    // P/Q k-steps
  static_assert(SM::MT == 2 && SM::NS == 1, "one K-step of two tiles per frame");
  const int lane = threadIdx.x & 63;
  const int kl = lane >> 4, cl = lane & 15;
  const int T = a.T;
  const int efb = __builtin_amdgcn_readfirstlane(st.rng[0]), eb = __builtin_amdgcn_readfirstlane(st.rng[1]);
  const int sa = __builtin_amdgcn_readfirstlane(st.rng[2]);
  const float pw = *a.prelu, pc = prelu_cap(pw);
  // conv rows: joint of tile m, row cl
  // (padding slots read past the unit's range: zero rows, no memory traffic)
  const int jr0 = SM::row_idx(0, cl) < V ? SM::row_idx(0, cl) : 1 << 20;
  const int jr1 = SM::row_idx(1, cl) < V ? SM::row_idx(1, cl) : 1 << 20;
  constexpr uint32_t xunit = V * CIN * 4;         // one frame of x
  constexpr uint32_t yunit = V * COUT * 4;        // one frame of y
  // this lane's output joint w = 16wt + cl: joints past V fall outside the
  // unit's buffer range by themselves; P/Q lanes other than kl == 0 get an
  // explicit out-of-range offset
  const uint32_t wpq0 = kl == 0 ? (uint32_t)cl * 16 : OOB;                  // + wt * 256

  // xmodel (CIN == 6 only): x is the model input [B][T][V][3] and the rows
  // are x6 = cat(x, x - x[:, -1]) built on the fly (no x6 tensor, no prep launch)
  const bool x6 = CIN == 6 && a.xmodel;
  auto frame_rsrc = [&](int uu) { return x6 ? rsrc(a.x + (size_t)uu * V * 3, V * 12) : rsrc(a.x + (size_t)uu * V * CIN, xunit); };
  auto last_rsrc = [&](int uu) { return rsrc(a.x + ((size_t)(uu / T) * T + T - 1) * V * 3, V * 12); };
  auto row8 = [&](__amdgpu_buffer_rsrc_t rf, __amdgpu_buffer_rsrc_t rl, int row, int k0, float4& lo4, float4& hi4) {
    if (x6) load_x6row(rf, rl, row, k0, lo4, hi4);
    else load_row8<CIN>(rf, row, k0, lo4, hi4);
  };
  float4 xr[2][KSI][2];  // [tile][k-step][half]: channels 32ks + 8kl .. +7 of the tile row
  auto load_x = [&](int uu) {
    const auto r = frame_rsrc(uu), rl = last_rsrc(uu);
#pragma unroll
    for (int ks = 0; ks < KSI; ++ks) {
      row8(r, rl, jr0, 32 * ks + 8 * kl, xr[0][ks][0], xr[0][ks][1]);
      row8(r, rl, jr1, 32 * ks + 8 * kl, xr[1][ks][0], xr[1][ks][1]);
    }
  };
  uint4 ab[2][NWT][2];  // adjacency B fragments [graph][w tile][plane]
  if (u < uend) load_x(u);
  while (u < uend) {
    const int un = u + ustep;
    const int lz = lane + opaque_zero();
    const auto rx = frame_rsrc(u), rxl = last_rsrc(u);
    // residual: identity -> x at the output positions (w, channels 16ct + 4kl ..);
    // residual conv -> x rows of the output joints as B fragments
    float4 R[RES ? 1 : 4][RES ? 1 : NWT];
    float4 xw[RES ? NWT : 1][RES ? KSI : 1][2];
    auto load_res = [&]() {
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) R[ct][wt] = bld4(rx, (uint32_t)((16 * wt + cl) * 64 + 4 * kl) * 4 + 64 * ct);
    };
    if constexpr (RES) {
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt)
#pragma unroll
        for (int ks = 0; ks < KSI; ++ks) row8(rx, rxl, 16 * wt + cl, 32 * ks + 8 * kl, xw[wt][ks][0], xw[wt][ks][1]);
    } else if constexpr (!LATE_RES) {
      load_res();
    }
    // this unit's graph-0 adjacency now, graph 1 after the first conv (a
    // whole-unit-ahead prefetch of both measured 6% slower: registers)
    load_adj_g(u, 0, ab[0]);
    __builtin_amdgcn_sched_barrier(0);
    // range shift of the unit's rows (0 unless a half could overflow)
    AmaxAcc xa;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int ks = 0; ks < KSI; ++ks) xa.add(xr[m][ks][0]), xa.add(xr[m][ks][1]);
    const float xm = xa.get();
    const int sx = input_shift(wave_max_bits(xm), efb, eb);
    const float dnx = pow2f(-sx);
    if (sx) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int ks = 0; ks < KSI; ++ks) {
          xr[m][ks][0] = mul4(xr[m][ks][0], dnx);
          xr[m][ks][1] = mul4(xr[m][ks][1], dnx);
        }
    }
    f16x8 xh[2][KSI], xo[2][KSI];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int ks = 0; ks < KSI; ++ks) split8(xr[m][ks][0], xr[m][ks][1], xh[m][ks], xo[m][ks]);

    f32x4 O[NCT][NWT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) O[ct][wt] = zero4();
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      // ---- conv (transposed): D[p][c] = sum_k x[p][k] W'[c][k] ----
      f32x4 D[2][NCT];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) D[m][ct] = zero4();
#pragma unroll
      for (int ks = 0; ks < KSI; ++ks)
#pragma unroll
        for (int c2 = 0; c2 < NCT; c2 += 2) {
          constexpr int Q2 = NCT < 2 ? NCT : 2;
          f16x8 wh[Q2], wo[Q2];
#pragma unroll
          for (int q = 0; q < Q2; ++q) {
            wh[q] = as_h8(st.wl[g][(((c2 + q) * KSI + ks) * 2 + 0) * 64 + lz]);
            wo[q] = as_h8(st.wl[g][(((c2 + q) * KSI + ks) * 2 + 1) * 64 + lz]);
          }
#pragma unroll
          for (int q = 0; q < Q2; ++q)
#pragma unroll
            for (int m = 0; m < 2; ++m) D[m][c2 + q] = mfma32(xo[m][ks], wh[q], D[m][c2 + q]);
#pragma unroll
          for (int q = 0; q < Q2; ++q)
#pragma unroll
            for (int m = 0; m < 2; ++m) D[m][c2 + q] = mfma32(xh[m][ks], wo[q], D[m][c2 + q]);
#pragma unroll
          for (int q = 0; q < Q2; ++q)
#pragma unroll
            for (int m = 0; m < 2; ++m) D[m][c2 + q] = mfma32(xh[m][ks], wh[q], D[m][c2 + q]);
        }
      if (g == 0) {
        __builtin_amdgcn_sched_barrier(0);
        load_adj_g(u, 1, ab[1]);
        __builtin_amdgcn_sched_barrier(0);
      }
      // x is dead after the second conv: prefetch the next unit's rows
      // (unconditionally -- the last unit reloads itself -- so that no
      // branch hides the loads from hipcc's vmcnt bookkeeping)
      if (g == 1) {
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch here: its registers free up only now
        load_x(un < uend ? un : u);
        __builtin_amdgcn_sched_barrier(0);
      }
      // ---- aggregation: O[c][w] += sum_v D[v][c] Adj[v][w] ----
      const float s = st.scl[g];
      f16x8 dh[NCT], dl[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const float b = st.bfl[g][16 * ct + cl] * dnx;  // F_s = 2^-sx F
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) D[m][ct][r] = fmaf(D[m][ct][r], s, b);
        split_acc(D[0][ct], D[1][ct], dh[ct], dl[ct]);
      }
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) O[ct][wt] = mfma32(dl[ct], as_h8(ab[g][wt][0]), O[ct][wt]);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) O[ct][wt] = mfma32(dh[ct], as_h8(ab[g][wt][1]), O[ct][wt]);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) O[ct][wt] = mfma32(dh[ct], as_h8(ab[g][wt][0]), O[ct][wt]);
    }

    // the identity residual after the aggregations (kSpLateRes: its 32
    // registers are not live through the convs; the frame was just read, so
    // the rows come from the cache)
    if constexpr (!RES && LATE_RES) {
      __builtin_amdgcn_sched_barrier(0);
      load_res();
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- residual conv in output layout: rc[c][w] = sum_k W_r[c][k] x[w][k] ----
    f32x4 rc[RES ? NCT : 1][RES ? NWT : 1];
    if constexpr (RES) {
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) rc[ct][wt] = zero4();
#pragma unroll
      for (int ks = 0; ks < KSI; ++ks) {
        f16x8 bh[NWT], bo[NWT];
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) {
          if (sx) {
            xw[wt][ks][0] = mul4(xw[wt][ks][0], dnx);
            xw[wt][ks][1] = mul4(xw[wt][ks][1], dnx);
          }
          split8(xw[wt][ks][0], xw[wt][ks][1], bh[wt], bo[wt]);
        }
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
          const f16x8 ah = as_h8(st.wl[2][((ct * KSI + ks) * 2 + 0) * 64 + lz]);
          const f16x8 ao = as_h8(st.wl[2][((ct * KSI + ks) * 2 + 1) * 64 + lz]);
#pragma unroll
          for (int wt = 0; wt < NWT; ++wt) rc[ct][wt] = mfma32(ao, bh[wt], rc[ct][wt]);
#pragma unroll
          for (int wt = 0; wt < NWT; ++wt) rc[ct][wt] = mfma32(ah, bo[wt], rc[ct][wt]);
#pragma unroll
          for (int wt = 0; wt < NWT; ++wt) rc[ct][wt] = mfma32(ah, bh[wt], rc[ct][wt]);
        }
      }
    }

    // ---- epilogue: h = prelu(bn(y) + r) -> NTVC ----
    // y = 2^(sx + sa) O (the aggregation ran on 2^-sx F and 2^-sa Adj)
    if (const int su = min(sx + sa, 127)) {
      const float up = pow2f(su);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) O[ct][wt] *= up;
    }
    const auto ry = rsrc(a.y + (size_t)u * V * COUT, yunit);
#pragma unroll
    for (int wt = 0; wt < NWT; ++wt) {
      const int wc = min(16 * wt + cl, V - 1);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        f32x4& o = O[ct][wt];
        const int c4 = (4 * ct + kl) * V + wc;
        const float4 sc = st.bnl[0][c4], sh = st.bnl[1][c4];
        float r[4];
        if constexpr (RES) {
          const float4 rs = st.bnl[2][c4], rh = st.bnl[3][c4];
          const float s3 = st.scl[3] * pow2f(sx);  // the residual conv ran on 2^-sx x
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float b = st.bfl[2][16 * ct + 4 * kl + q];
            const float rv = fmaf(rc[ct][wt][q], s3, b);
            r[q] = fmaf(rv, q == 0 ? rs.x : q == 1 ? rs.y : q == 2 ? rs.z : rs.w,
                        q == 0 ? rh.x : q == 1 ? rh.y : q == 2 ? rh.z : rh.w);
          }
        } else {
          r[0] = R[ct][wt].x;
          r[1] = R[ct][wt].y;
          r[2] = R[ct][wt].z;
          r[3] = R[ct][wt].w;
        }
        o[0] = prelu_m(fmaf(o[0], sc.x, sh.x) + r[0], pw, pc);
        o[1] = prelu_m(fmaf(o[1], sc.y, sh.y) + r[1], pw, pc);
        o[2] = prelu_m(fmaf(o[2], sc.z, sh.z) + r[2], pw, pc);
        o[3] = prelu_m(fmaf(o[3], sc.w, sh.w) + r[3], pw, pc);
        if constexpr (COUT % 4 == 0) {
          bst4<ST_AUX>(ry, (uint32_t)((16 * wt + cl) * COUT + 16 * ct + 4 * kl) * 4, make_float4(o[0], o[1], o[2], o[3]));
        } else {
          static_assert(COUT == 3, "thin output: 3 channels");
          const uint32_t off = kl == 0 ? (uint32_t)(16 * wt + cl) * 12 : OOB;
          // (a whole f32x3 bit_cast: hipcc 7.2 folds __builtin_bit_cast of
          // single vector elements o[1], o[2] to o[0]'s bits -- measured)
          typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
          typedef float f32x3 __attribute__((ext_vector_type(3)));
          const f32x3 o3 = {o[0], o[1], o[2]};
          __builtin_amdgcn_raw_buffer_store_b96(__builtin_bit_cast(u32x3, o3), ry, off, 0, DSTD_GC_ST_AUX);
        }
      }
    }
    // ---- P_t/Q_t of h: out[ch][w] = sum_c wq[ch][c] h[c][w] + b ----
    // on h_s = 2^-sh h (range shift of the unit's output)
    AmaxAcc ha;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) ha.add(O[ct][wt]);
    const float hm = ha.get();
    const int sh = hl_range_shift(fexp_bits(wave_max_bits(hm)));
    if (sh) {
      const float dn = pow2f(-sh);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) O[ct][wt] *= dn;
    }
    f32x4 acc[NWT];
#pragma unroll
    for (int wt = 0; wt < NWT; ++wt) acc[wt] = zero4();
#pragma unroll
    for (int ks = 0; ks < KSO; ++ks) {
      const f16x8 qh = as_h8(st.pql[(ks * 2 + 0) * 64 + lz]), qo = as_h8(st.pql[(ks * 2 + 1) * 64 + lz]);
      f16x8 hh[NWT], hl[NWT];
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) {
        if (2 * ks + 1 < NCT) split_acc(O[2 * ks][wt], O[2 * ks + 1 < NCT ? 2 * ks + 1 : 0][wt], hh[wt], hl[wt]);
        else split_acc(O[2 * ks][wt], hh[wt], hl[wt]);
      }
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) acc[wt] = mfma32(qo, hh[wt], acc[wt]);
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) acc[wt] = mfma32(qh, hl[wt], acc[wt]);
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) acc[wt] = mfma32(qh, hh[wt], acc[wt]);
    }
    {
      const float s = st.scl[2] * pow2f(sh);
      const auto rp = rsrc(a.pq + (size_t)u * V * 4, V * 16);
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) {
        const float4 pq4 = make_float4(fmaf(acc[wt][0], s, st.bql[0]), fmaf(acc[wt][1], s, st.bql[1]),
                                       fmaf(acc[wt][2], s, st.bql[2]), fmaf(acc[wt][3], s, st.bql[3]));
        bst4<ST_AUX>(rp, wpq0 + wt * 256, pq4);
        if constexpr (!std::is_same<PQSink, NoPQSink>::value) {
          if (kl == 0 && 16 * wt + cl < V) bad |= pq_sink(u, 16 * wt + cl, pq4.x, pq4.y, pq4.z, pq4.w);
        }
      }
    }
    u = un;
  }
  return bad;
}

template <int V, int CIN, int COUT>
__global__ __launch_bounds__(spatial_nt()) __attribute__((amdgpu_waves_per_eu(DSTD_HL_WPE, DSTD_HL_WPE))) void k_spatial_hl(
    SpatialHLArgs a) {
  using SM = SlotMap<V, true>;
  constexpr int SL = SM::SL, NG = SM::NG, NWT = cdiv(V, 16);
  __shared__ SpatialStage<V, CIN, COUT> st;
  stage_spatial<V, CIN, COUT, spatial_nt()>(a, st, threadIdx.x);
  __syncthreads();
  // static VALU-arbitration priority 1 for the younger half (waves 4-7: the
  // arbitration losers at equal priority; MI355X guide "two waves per SIMD"
  // item 4, T5 static form): spatial GC -1.8%, forward -0.8% at H36M and
  // -0.9% at 3DPW, B=32 neutral, bit-identical (profiles/r05o_setprio_ab.txt)
#ifndef DSTD_SETPRIO_SP  // (0: off)
#define DSTD_SETPRIO_SP 256
#endif
  if (DSTD_SETPRIO_SP > 0 && __builtin_amdgcn_readfirstlane(threadIdx.x) >= DSTD_SETPRIO_SP)
    __builtin_amdgcn_s_setprio(1);
  const int lane = threadIdx.x & 63, kl = lane >> 4, cl = lane & 15;
  const int T = a.T;
  constexpr uint32_t adj_bytes = 2 * V * SL * 2;  // one (n, g, t) adjacency: 2 planes of V x SL halves
  // adjacency lane groups past NG get an out-of-range offset (zero fragments)
  const uint32_t wadj0 = kl < NG ? (uint32_t)(cl * SL + 8 * kl) * 2 : OOB;  // + wt * 32 * SL
  auto load_adj_g = [&](int uu, int g, uint4 (&ab)[NWT][2]) {
    const int n = uu / T, t = uu - n * T;
    const uint16_t* base = a.adj + ((size_t)(n * 2 + g) * T + t) * (adj_bytes / 2);
    const auto rh = rsrc(base, adj_bytes / 2), rl = rsrc(base + V * SL, adj_bytes / 2);  // one plane each
#pragma unroll
    for (int wt = 0; wt < NWT; ++wt) {
      ab[wt][0] = bldu4(rh, wadj0 + wt * 32 * SL);
      ab[wt][1] = bldu4(rl, wadj0 + wt * 32 * SL);
    }
  };
  int uend;
  const int u = unit_range(a.B * T, uend);
  spatial_units<V, CIN, COUT>(a, st, u, uend, 1, load_adj_g);
}

// ===========================================================================
// Temporal GC, C -> C, C = 64 (every encoder and conv_st_in) or 3 (the
// conv_st_out tail) (DSTDGC.forward temporal, model/dstdgcn.py:88-93) with the
// DSTDGCB tail epilogues (:161-163, DSTDGCN.forward :306-315), unit =
// (sample n, joint v):
//   y[c][u] = sum_t (W h + b)[t][c] Adj[v][t][u]
//   ENC: prelu(bn(y + xres));  IN: prelu(bn(y));  RAW: y;
//   OUT: y + x_model[n][T-1][v][c] (the model output, C = 3)
//   + P_s/Q_s (8 channels, [B][V][T][8]) of the output for the next block
// ===========================================================================
// waves per SIMD: 64 channels two up to 48 frames (one at 75); the 3-channel
// tail is light enough for twice as many
template <int T, int C>
constexpr int temporal_hl_wpe() {
#ifdef DSTD_T_WPE
  return DSTD_T_WPE * (C == 3 ? 2 : 1);
#endif
  return (T <= 48 || C == 64 ? 2 : 1) * (C == 3 ? 2 : 1);
}
// one workgroup per CU at the kernel's waves per SIMD (4 waves at one per
// SIMD: an 8-wave workgroup would force two per SIMD and spill), at most 8
template <int T, int C>
constexpr int temporal_nt() {
  return 64 * (4 * temporal_hl_wpe<T, C>() < 8 ? 4 * temporal_hl_wpe<T, C>() : 8);
}

// 8 channels k0 .. k0+7 of the row at byte offset `row_off` (C per row; zero
// past C, and an out-of-range row_off reads zeros)
template <int C, int AUX = 0>
__device__ __forceinline__ void load_row8_at(__amdgpu_buffer_rsrc_t r, uint32_t row_off, int k0, float4& lo4, float4& hi4) {
  if constexpr (C % 8 == 0) {
    lo4 = bld4<AUX>(r, row_off + 4 * k0);
    hi4 = bld4<AUX>(r, row_off + 4 * k0 + 16);
  } else {
    const uint32_t off = k0 == 0 ? row_off : OOB;
    float e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = 0.f;
#pragma unroll
    for (int i = 0; i < C; ++i)
      e[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off + 4 * i, 0, 0));
    lo4 = make_float4(e[0], e[1], e[2], e[3]);
    hi4 = make_float4(e[4], e[5], e[6], e[7]);
  }
}

// LDS images of one temporal GC launch: conv_f fragments, the next block's
// P/Q conv fragments, folded BN [c/4][v] for VB joints, biases and scalars
template <int T, int EPI, int C, int VB>
struct TemporalStage {
  static constexpr int KSI = cdiv(C, 32), NCT = cdiv(C, 16), KSO = cdiv(NCT, 2);
  static constexpr int WIMG = NCT * KSI * 2 * 64, PIMG = KSO * 2 * 64;
  static constexpr bool use_bn = EPI == TEPI_ENC || EPI == TEPI_IN;
  uint4 wl[WIMG];
  uint4 pql[PIMG];
  float4 bnl[2][use_bn ? 4 * NCT * VB : 1];
  float bfl[16 * NCT];
  float bql[8];
  float scl[2];
  int rng[3];
};

// The stage's global loads (load) and its LDS writes (store) as two steps:
// the fused temporal body issues the loads before the barrier that ends
// phase 1 (the tile registers are dead by then) and writes once the phase-1
// scratch is free, so the load latency hides in the barrier wait.
#ifndef DSTD_TF_STAGE_EARLY
#define DSTD_TF_STAGE_EARLY 1
#endif
template <int T, int EPI, int C, int VB, int NTH>
struct TemporalStageLoad {
  using S = TemporalStage<T, EPI, C, VB>;
  static constexpr int NW = cdiv(S::WIMG, NTH), NP = cdiv(S::PIMG, NTH);
  static constexpr int NB = S::use_bn ? cdiv(VB * 4 * S::NCT, NTH) : 0;
  // (native vectors: a uint4 array copied from global memory is a memcpy
  // that keeps the array in scratch)
  u32x4 wv[NW], pv[NP];
  float4 bs[NB > 0 ? NB : 1], bh[NB > 0 ? NB : 1];
  float bf, bq;
  // (oz: an opaque zero from a caller that stages once per loop trip, so
  // that these loop-invariant loads are not hoisted out of its loop)
  __device__ __forceinline__ void load(const TemporalHLArgs& a, int tid, int oz = 0) {
    const bool has_pq = a.pq != nullptr;
#pragma unroll
    for (int it = 0; it < NW; ++it)
      wv[it] = *reinterpret_cast<const u32x4*>(a.wimg + min(tid + it * NTH + oz, S::WIMG - 1));
#pragma unroll
    for (int it = 0; it < NP; ++it)
      pv[it] = has_pq ? *reinterpret_cast<const u32x4*>(a.pqimg + min(tid + it * NTH + oz, S::PIMG - 1)) : u32x4{0, 0, 0, 0};
    const int nbn = a.V * 4 * S::NCT;
    if constexpr (S::use_bn) {
      static_assert(C % 4 == 0, "folded BN rows load as float4");
      // folded BN vectors [V][C] -> [c/4][v]
#pragma unroll
      for (int it = 0; it < NB; ++it) {
        const int i = min(tid + it * NTH + oz, nbn - 1);
        const int v = i / (4 * S::NCT), c4 = i - v * (4 * S::NCT);
        bs[it] = ld4(a.bn_s + v * C + 4 * c4);
        bh[it] = ld4(a.bn_h + v * C + 4 * c4);
      }
    }
    bf = tid < 16 * S::NCT && tid < C ? a.bf[tid] : 0.f;
    // (the pointer by selects, not an indexed kernel-argument load: that load
    // is dependent and its wait would hold wave 0 on every load above)
    const float* p4[4] = {a.pqb[0], a.pqb[1], a.pqb[2], a.pqb[3]};
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+s"(p4[i]));
    const int g = (tid >> 1) & 3;
    const float* pb = g == 0 ? p4[0] : g == 1 ? p4[1] : g == 2 ? p4[2] : p4[3];
    typedef __attribute__((address_space(1))) const float gfloat;
    bq = tid < 8 && has_pq ? ((gfloat*)pb)[tid & 1] : 0.f;
  }
  __device__ __forceinline__ void store(const TemporalHLArgs& a, S& st, int tid) const {
    const bool has_pq = a.pq != nullptr;
    const int nbn = a.V * 4 * S::NCT;
#pragma unroll
    for (int it = 0; it < NW; ++it)
      if (tid + it * NTH < S::WIMG) *reinterpret_cast<u32x4*>(st.wl + tid + it * NTH) = wv[it];
    if (has_pq) {
#pragma unroll
      for (int it = 0; it < NP; ++it)
        if (tid + it * NTH < S::PIMG) *reinterpret_cast<u32x4*>(st.pql + tid + it * NTH) = pv[it];
    }
    if constexpr (S::use_bn) {
#pragma unroll
      for (int it = 0; it < NB; ++it) {
        const int i = tid + it * NTH;
        if (i < nbn) {
          const int v = i / (4 * S::NCT), c4 = i - v * (4 * S::NCT);
          st.bnl[0][c4 * a.V + v] = bs[it];
          st.bnl[1][c4 * a.V + v] = bh[it];
        }
      }
    }
    if (tid < 16 * S::NCT) st.bfl[tid] = bf;
    if (tid < 8) st.bql[tid] = bq;
    if (tid == 0) {
      st.scl[0] = *a.wscale;
      st.scl[1] = has_pq ? *a.pqscale : 0.f;
      // range: |W_f|_inf, max|b_f| and the planes' shift
      st.rng[0] = fexp_bits(__float_as_uint(fmaxf(1.f, a.wscale[HLS_BOUND])));
      st.rng[1] = fexp_bits(__float_as_uint(a.wscale[HLS_BMAX]));
      st.rng[2] = hl_range_shift(fexp_bits(__float_as_uint(a.adjb[HLS_BOUND])));
    }
  }
};

// every global load is issued before the first LDS write (one memory round
// trip instead of one per loop trip)
template <int T, int EPI, int C, int VB, int NTH>
__device__ __forceinline__ void stage_temporal(const TemporalHLArgs& a, TemporalStage<T, EPI, C, VB>& st, int tid,
                                               int oz = 0) {
  TemporalStageLoad<T, EPI, C, VB, NTH> sl;
  sl.load(a, tid, oz);
  sl.store(a, st, tid);
}

// The unit loop of the temporal GC over units u, u + ustep, ... < uend
// (unit = (sample, joint) = n * V + v).  The unit's adjacency B fragments
// [K-step][u tile] (hi, lo planes) come from load_adj: LAZY = false,
// load_adj(u, bh[NS][NUT], bo[NS][NUT]) at the top of the unit (the planes in
// HBM, k_temporal_hl: the loads fly during the conv); LAZY = true,
// load_adj(u, s, bh[NUT], bo[NUT]) per aggregation K-step (the planes in LDS,
// k_temporal_fused: 24 fewer live VGPRs).
#ifndef DSTD_TF_LATE_RES
#define DSTD_TF_LATE_RES 1
#endif
#ifndef DSTD_TF_RES_ACC
#define DSTD_TF_RES_ACC 1
#endif
// shapes whose ENC units take the residual as the accumulator's initial
// value: CMU (T 35, V 25; -2.8% per forward) and 3DPW (T 40, V 23; -2.3%, and
// its 8-wave fused kernel fits 256 VGPRs without its 4 spills); not H36M
// (the 12-wave fused kernel spills 3 VGPRs at 168: +1.1%) nor T = 75
// (k_temporal_hl would spill 40); profiles/r04m_res_acc_ab.txt, r04n_res_acc35_ab.txt
__host__ __device__ constexpr bool tf_res_acc(int T, int V) { return (T == 35 && V == 25) || (T == 40 && V == 23); }
// PF: the next unit's h rows are loaded during this one (48 VGPRs); without,
// each unit loads its own rows first (for more waves per SIMD instead)
template <int T, int EPI, int C, int VB, bool LAZY, typename AdjLoad, bool PF = true, bool RA = false,
          int NUTC = cdiv(T, 16)>
__device__ __forceinline__ void temporal_units(const TemporalHLArgs& a, const TemporalStage<T, EPI, C, VB>& st, int u,
                                               int uend, int ustep, AdjLoad load_adj, int ut0 = 0) {
  // NUTC / ut0: the u tiles ut0 .. ut0 + NUTC - 1 of each unit (a u chunk of
  // k_temporal_fused at T = 75; every tile otherwise); load_adj fills
  // [NUTC] fragments for them
  using SM = SlotMap<T, false>;
  using S = TemporalStage<T, EPI, C, VB>;
  constexpr int MT = SM::MT, NS = SM::NS;
  constexpr int KSI = S::KSI, NCT = S::NCT, KSO = S::KSO;
  constexpr bool use_bn = S::use_bn;
  constexpr bool use_res = EPI == TEPI_ENC || EPI == TEPI_OUT;
  const uint4* wl = st.wl;
  const uint4* pql = st.pql;
  const float* bfl = st.bfl;
  const float* bql = st.bql;
  const float* scl = st.scl;
  const int lane = threadIdx.x & 63;
  const int kl = lane >> 4, cl = lane & 15;
  const int V = a.V;
  const bool has_pq = a.pq != nullptr;
  const int efb = __builtin_amdgcn_readfirstlane(st.rng[0]), eb = __builtin_amdgcn_readfirstlane(st.rng[1]);
  const int sa = __builtin_amdgcn_readfirstlane(st.rng[2]);
  const float pw = use_bn ? *a.prelu : 0.f, pc = prelu_cap(pw);
  // a unit's rows: frame t of joint v at t * V * C floats from the unit base
  const uint32_t col_bytes = (uint32_t)((T - 1) * V + 1) * C * 4;
  const uint32_t frame_bytes = (uint32_t)V * C * 4;
  uint32_t xoff[MT];  // conv rows: frame 16m + cl (OOB past T)
#pragma unroll
  for (int m = 0; m < MT; ++m) xoff[m] = 16 * m + cl < T ? (uint32_t)(16 * m + cl) * frame_bytes : OOB;
  // output frame uo = 16ut + cl (OOB past T), channels 4kl .. (C = 64) or the
  // 3 channels on lanes kl == 0 (C = 3)
  uint32_t uoff[NUTC], upq[NUTC];
#pragma unroll
  for (int ut = 0; ut < NUTC; ++ut) {
    const int uo = 16 * (ut0 + ut) + cl;
    uoff[ut] = uo < T && (C % 4 == 0 || kl == 0) ? (uint32_t)uo * frame_bytes + (C % 4 == 0 ? 16 * kl : 0) : OOB;
    upq[ut] = uo < T && kl < 2 ? (uint32_t)(uo * 8 + 4 * kl) * 4 : OOB;
  }

  float4 xr[MT][KSI][2];  // tile m row cl = frame 16m + cl
  auto load_x = [&](int uu) {
    const int n = uu / V, v = uu - n * V;
    const auto r = rsrc(a.h + ((size_t)n * T * V + v) * C, col_bytes);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int ks = 0; ks < KSI; ++ks)
        load_row8_at<C, DSTD_TF_H_LD_AUX>(r, xoff[m], 32 * ks + 8 * kl, xr[m][ks][0], xr[m][ks][1]);
  };
  if (PF && u < uend) load_x(u);
  while (u < uend) {
    if constexpr (!PF) load_x(u);
    const int n = u / V, v = u - n * V;
    const int un = u + ustep;
    const int lz = lane + opaque_zero();
    const size_t cbase = ((size_t)n * T * V + v) * C;
    // Issue order matters: vmcnt retires in order, so every load this unit
    // waits for (adjacency, residual) is issued before the next unit's h-row
    // prefetch, which lands behind them.
    uint4 bh[LAZY ? 1 : NS][NUTC], bo[LAZY ? 1 : NS][NUTC];  // adjacency B fragments [K-step][u tile]
    if constexpr (!LAZY) load_adj(u, bh, bo);
    __builtin_amdgcn_sched_barrier(0);
    // range shift of the unit's rows (0 unless a half could overflow)
    AmaxAcc xa;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int ks = 0; ks < KSI; ++ks) xa.add(xr[m][ks][0]), xa.add(xr[m][ks][1]);
    const float xm = xa.get();
    const int sx = input_shift(wave_max_bits(xm), efb, eb);
    const float dnx = pow2f(-sx);
    if (sx) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int ks = 0; ks < KSI; ++ks) {
          xr[m][ks][0] = mul4(xr[m][ks][0], dnx);
          xr[m][ks][1] = mul4(xr[m][ks][1], dnx);
        }
    }
    f16x8 xh[MT][KSI], xo[MT][KSI];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int ks = 0; ks < KSI; ++ks) split8(xr[m][ks][0], xr[m][ks][1], xh[m][ks], xo[m][ks]);

    // ---- conv (transposed): D[t][c] = sum_k h[t][k] W'[c][k] ----
    // CTO (a u chunk of one tile at T = 75): conv and aggregation run per
    // output channel tile (below), so only that tile's MT accumulators are
    // live -- the same MFMA sequence on every accumulator, bit-identical
    constexpr bool CTO = LAZY && NUTC < cdiv(T, 16);
    f32x4 D[CTO ? 1 : MT][NCT];
    if constexpr (!CTO) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) D[m][ct] = zero4();
#pragma unroll
    for (int ks = 0; ks < KSI; ++ks) {
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const f16x8 wh = as_h8(wl[((ct * KSI + ks) * 2 + 0) * 64 + lz]);
        const f16x8 wo = as_h8(wl[((ct * KSI + ks) * 2 + 1) * 64 + lz]);
#pragma unroll
        for (int m = 0; m < MT; ++m) D[m][ct] = mfma32(xo[m][ks], wh, D[m][ct]);
#pragma unroll
        for (int m = 0; m < MT; ++m) D[m][ct] = mfma32(xh[m][ks], wo, D[m][ct]);
#pragma unroll
        for (int m = 0; m < MT; ++m) D[m][ct] = mfma32(xh[m][ks], wh, D[m][ct]);
      }
    }
    {
      const float s = scl[0];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const float b = bfl[16 * ct + cl] * dnx;  // F_s = 2^-sx F
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) D[m][ct][r] = fmaf(D[m][ct][r], s, b);
      }
    }
    }  // !CTO
    // residual of the epilogue: the encoder input (ENC) or the model input's
    // last observed frame (OUT); LAZY (LDS adjacency, no HBM loads to wait
    // for in the aggregation) defers the ENC residual past the aggregation
    // so its 48 registers are not live across it
    float4 R[use_res ? NCT : 1][use_res ? NUTC : 1];
    auto load_res_enc = [&]() {
      const auto rr = rsrc(a.xres + cbase, col_bytes);
#pragma unroll
      for (int ut = 0; ut < NUTC; ++ut)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) R[ct][ut] = bld4<DSTD_TF_R_LD_AUX>(rr, uoff[ut] + 64 * ct);
    };
    constexpr bool late_res = LAZY && DSTD_TF_LATE_RES;
    // RES_ACC: the ENC residual is the aggregation accumulator's initial
    // value (scaled like the sum, 2^-(sx+sa)) -- the MFMAs add it, the
    // epilogue does not (48 VALU adds per unit), and it needs no registers of
    // its own across the aggregation.  Chosen per shape by the kernels
    // (tf_res_acc, the same for the fused and unfused schedules of a shape so
    // they stay bit-identical)
    constexpr bool res_acc = EPI == TEPI_ENC && DSTD_TF_RES_ACC && RA;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (EPI == TEPI_ENC && !late_res && !res_acc) {
      load_res_enc();
    } else if constexpr (EPI == TEPI_ENC) {
    } else if constexpr (EPI == TEPI_OUT) {
      // x_model [B][T][V][C]: frame T-1 of joint v, 3 channels on lanes kl == 0
      const auto rr = rsrc(a.xres + (((size_t)n * T + T - 1) * V + v) * C, C * 4);
      float e[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < C && i < 4; ++i)
        e[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, kl == 0 ? 4 * i : OOB, 0, 0));
#pragma unroll
      for (int ut = 0; ut < NUTC; ++ut) R[0][ut] = make_float4(e[0], e[1], e[2], e[3]);
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- aggregation: O[c][u] = sum_t D[t][c] Adj[v][t][u] ----
    f32x4 O[NCT][NUTC];
    if constexpr (res_acc) {
      const auto rr = rsrc(a.xres + cbase, col_bytes);
#pragma unroll
      for (int ut = 0; ut < NUTC; ++ut)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
          const float4 r4 = bld4<DSTD_TF_R_LD_AUX>(rr, uoff[ut] + 64 * ct);
          O[ct][ut] = f32x4{r4.x, r4.y, r4.z, r4.w};
        }
      if (const int su0 = min(sx + sa, 127)) {
        const float dn = pow2f(-su0);
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
          for (int ut = 0; ut < NUTC; ++ut) O[ct][ut] *= dn;
      }
    } else {
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int ut = 0; ut < NUTC; ++ut) O[ct][ut] = zero4();
    }
    if constexpr (CTO) {
      uint4 bhs[NS][NUTC], bos[NS][NUTC];  // every K-step's fragments (one u tile)
#pragma unroll
      for (int s = 0; s < NS; ++s) load_adj(u, s, bhs[s], bos[s]);
      const float sc0 = scl[0];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        f32x4 Dc[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) Dc[m] = zero4();
#pragma unroll
        for (int ks = 0; ks < KSI; ++ks) {
          const f16x8 wh = as_h8(wl[((ct * KSI + ks) * 2 + 0) * 64 + lz]);
          const f16x8 wo = as_h8(wl[((ct * KSI + ks) * 2 + 1) * 64 + lz]);
#pragma unroll
          for (int m = 0; m < MT; ++m) Dc[m] = mfma32(xo[m][ks], wh, Dc[m]);
#pragma unroll
          for (int m = 0; m < MT; ++m) Dc[m] = mfma32(xh[m][ks], wo, Dc[m]);
#pragma unroll
          for (int m = 0; m < MT; ++m) Dc[m] = mfma32(xh[m][ks], wh, Dc[m]);
        }
        const float b = bfl[16 * ct + cl] * dnx;
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) Dc[m][r] = fmaf(Dc[m][r], sc0, b);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          f16x8 dh, dl;
          if (2 * s + 1 < MT) split_acc(Dc[2 * s], Dc[2 * s + 1 < MT ? 2 * s + 1 : 0], dh, dl);
          else split_acc(Dc[2 * s], dh, dl);
#pragma unroll
          for (int ut = 0; ut < NUTC; ++ut) O[ct][ut] = mfma32(dl, as_h8(bhs[s][ut]), O[ct][ut]);
#pragma unroll
          for (int ut = 0; ut < NUTC; ++ut) O[ct][ut] = mfma32(dh, as_h8(bos[s][ut]), O[ct][ut]);
#pragma unroll
          for (int ut = 0; ut < NUTC; ++ut) O[ct][ut] = mfma32(dh, as_h8(bhs[s][ut]), O[ct][ut]);
        }
      }
    }
#pragma unroll
    for (int s = 0; s < (CTO ? 0 : NS); ++s) {
      const int sb = LAZY ? 0 : s;
      if constexpr (LAZY) load_adj(u, s, bh[0], bo[0]);
      f16x8 dh[NCT], dl[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        if (2 * s + 1 < MT) split_acc(D[2 * s][ct], D[2 * s + 1 < MT ? 2 * s + 1 : 0][ct], dh[ct], dl[ct]);
        else split_acc(D[2 * s][ct], dh[ct], dl[ct]);
      }
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int ut = 0; ut < NUTC; ++ut) O[ct][ut] = mfma32(dl[ct], as_h8(bh[sb][ut]), O[ct][ut]);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int ut = 0; ut < NUTC; ++ut) O[ct][ut] = mfma32(dh[ct], as_h8(bo[sb][ut]), O[ct][ut]);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int ut = 0; ut < NUTC; ++ut) O[ct][ut] = mfma32(dh[ct], as_h8(bh[sb][ut]), O[ct][ut]);
    }
    // next unit's h rows (unconditional -- the last unit reloads itself -- so
    // that no branch hides the loads from hipcc's vmcnt bookkeeping)
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (EPI == TEPI_ENC && late_res && !res_acc) load_res_enc();
    // (long sequences: the next unit's rows after the epilogue, so that they,
    // the output accumulators and the residual are not live at once)
    constexpr bool late_x = LAZY && T > 48;
    if constexpr (PF && !late_x) load_x(un < uend ? un : u);
    __builtin_amdgcn_sched_barrier(0);

    // ---- epilogue ----
    // y = 2^(sx + sa) O (the aggregation ran on 2^-sx F and 2^-sa Adj)
    if (const int su = min(sx + sa, 127)) {
      const float up = pow2f(su);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int ut = 0; ut < NUTC; ++ut) O[ct][ut] *= up;
    }
    const auto ry = rsrc(a.y + cbase, col_bytes);
#pragma unroll
    for (int ut = 0; ut < NUTC; ++ut) {
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        f32x4& o = O[ct][ut];
        if constexpr (use_res && !res_acc) {
          o[0] += R[ct][ut].x;
          o[1] += R[ct][ut].y;
          o[2] += R[ct][ut].z;
          o[3] += R[ct][ut].w;
        }
        if constexpr (use_bn) {
          const float4 sc = st.bnl[0][(4 * ct + kl) * V + v], sh = st.bnl[1][(4 * ct + kl) * V + v];
          o[0] = prelu_m(fmaf(o[0], sc.x, sh.x), pw, pc);
          o[1] = prelu_m(fmaf(o[1], sc.y, sh.y), pw, pc);
          o[2] = prelu_m(fmaf(o[2], sc.z, sh.z), pw, pc);
          o[3] = prelu_m(fmaf(o[3], sc.w, sh.w), pw, pc);
        }
        if constexpr (C % 4 == 0) {
          bst4(ry, uoff[ut] + 64 * ct, make_float4(o[0], o[1], o[2], o[3]));
        } else {
          // (a whole f32x3 bit_cast: hipcc 7.2 folds __builtin_bit_cast of
          // single vector elements to element 0's bits -- measured)
          typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
          typedef float f32x3 __attribute__((ext_vector_type(3)));
          const f32x3 o3 = {o[0], o[1], o[2]};
          __builtin_amdgcn_raw_buffer_store_b96(__builtin_bit_cast(u32x3, o3), ry, uoff[ut], 0, DSTD_GC_ST_AUX);
        }
      }
    }
    // ---- next block's P_s/Q_s (8 channels) of the output ----
    if (has_pq) {
      // on h_s = 2^-sh h (range shift of the unit's output)
      // (long sequences: one shift per u tile, so that a u chunk of the fused
      // kernel, which holds one tile, shifts exactly as the whole unit does)
      constexpr bool PTS = T > 48;
      constexpr int NSH = PTS ? NUTC : 1;
      int sh[NSH];
#pragma unroll
      for (int k = 0; k < NSH; ++k) {
        float hm = 0.f;
        if constexpr (use_bn || use_res) {
          AmaxAcc ha;
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
            for (int ut = 0; ut < NUTC; ++ut)
              if (!PTS || ut == k) ha.add(O[ct][ut]);
          hm = ha.get();
        } else {
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
            for (int ut = 0; ut < NUTC; ++ut)
              if (!PTS || ut == k) hm = amax4_mfma(hm, O[ct][ut]);
        }
        sh[k] = hl_range_shift(fexp_bits(wave_max_bits(hm)));
        if (sh[k]) {
          const float dn = pow2f(-sh[k]);
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
            for (int ut = 0; ut < NUTC; ++ut)
              if (!PTS || ut == k) O[ct][ut] *= dn;
        }
      }
      f32x4 acc[NUTC];
#pragma unroll
      for (int ut = 0; ut < NUTC; ++ut) acc[ut] = zero4();
#pragma unroll
      for (int ks = 0; ks < KSO; ++ks) {
        const f16x8 qh = as_h8(pql[(ks * 2 + 0) * 64 + lz]), qo = as_h8(pql[(ks * 2 + 1) * 64 + lz]);
        f16x8 hh[NUTC], hl[NUTC];
#pragma unroll
        for (int ut = 0; ut < NUTC; ++ut) {
          if (2 * ks + 1 < NCT) split_acc(O[2 * ks][ut], O[2 * ks + 1 < NCT ? 2 * ks + 1 : 0][ut], hh[ut], hl[ut]);
          else split_acc(O[2 * ks][ut], hh[ut], hl[ut]);
        }
#pragma unroll
        for (int ut = 0; ut < NUTC; ++ut) acc[ut] = mfma32(qo, hh[ut], acc[ut]);
#pragma unroll
        for (int ut = 0; ut < NUTC; ++ut) acc[ut] = mfma32(qh, hl[ut], acc[ut]);
#pragma unroll
        for (int ut = 0; ut < NUTC; ++ut) acc[ut] = mfma32(qh, hh[ut], acc[ut]);
      }
      const auto rp = rsrc(a.pq + (size_t)u * T * 8, T * 32);
#pragma unroll
      for (int ut = 0; ut < NUTC; ++ut) {
        const float s = scl[1] * pow2f(sh[PTS ? ut : 0]);
        const int b4 = 4 * (kl & 1);
        bst4(rp, upq[ut],
             make_float4(fmaf(acc[ut][0], s, bql[b4]), fmaf(acc[ut][1], s, bql[b4 + 1]), fmaf(acc[ut][2], s, bql[b4 + 2]),
                         fmaf(acc[ut][3], s, bql[b4 + 3])));
      }
    }
    if constexpr (PF && late_x) {
      __builtin_amdgcn_sched_barrier(0);
      load_x(un < uend ? un : u);
    }
    u = un;
  }
}


template <int T, int EPI, int C, bool RA = false>
__global__ __launch_bounds__((temporal_nt<T, C>())) __attribute__((amdgpu_waves_per_eu(temporal_hl_wpe<T, C>(), temporal_hl_wpe<T, C>()))) void k_temporal_hl(
    TemporalHLArgs a) {
  static_assert(C == 64 || (C == 3 && (EPI == TEPI_OUT || EPI == TEPI_RAW)), "shapes of the forward");
  using SM = SlotMap<T, false>;
  constexpr int SL = SM::SL, NS = SM::NS, NUT = cdiv(T, 16);
  __shared__ TemporalStage<T, EPI, C, 32> st;
  stage_temporal<T, EPI, C, 32, temporal_nt<T, C>()>(a, st, threadIdx.x);
  __syncthreads();
#ifdef DSTD_SETPRIO_TH  // (experiment: the younger waves' static priority, as k_spatial_hl)
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= DSTD_SETPRIO_TH) __builtin_amdgcn_s_setprio(1);
#endif
  int uend;
  const int u0 = unit_range(a.B * a.V, uend);
  const int cl = threadIdx.x & 15, kl = (threadIdx.x & 63) >> 4;
  constexpr uint32_t adj_bytes = 2 * T * SL * 2;  // one (n, v): 2 planes of T x SL halves
  // the unit's planes in HBM ([B][V][2 planes][T][SL], k_adj_hl), one 16-byte load per fragment
  auto load_adj = [&](int u, uint4 (&bh)[NS][NUT], uint4 (&bo)[NS][NUT]) {
    const auto rh = rsrc(a.adj + (size_t)u * (adj_bytes / 2), adj_bytes / 2);  // hi plane
    const auto rl = rsrc(a.adj + (size_t)u * (adj_bytes / 2) + T * SL, adj_bytes / 2);
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int ut = 0; ut < NUT; ++ut) {
        const int uo = 16 * ut + cl;
        const uint32_t off = uo < T && kl < SM::ng(s) ? (uint32_t)(uo * SL + 8 * (SM::goff(s) + kl)) * 2 : OOB;
        bh[s][ut] = bldu4(rh, off);
        bo[s][ut] = bldu4(rl, off);
      }
  };
  if constexpr (T > 48) {
    // long sequences (T = 75): the unit's NS x NUT fragment pairs held through
    // the conv took 120 VGPRs and left one wave per SIMD (256 VGPRs + 184
    // AGPRs); fetched per aggregation K-step instead (LAZY), the kernel runs
    // two waves per SIMD
    auto load_adj_s = [&](int u, int s, uint4 (&bh)[NUT], uint4 (&bo)[NUT]) {
      const auto rh = rsrc(a.adj + (size_t)u * (adj_bytes / 2), adj_bytes / 2);  // hi plane
      const auto rl = rsrc(a.adj + (size_t)u * (adj_bytes / 2) + T * SL, adj_bytes / 2);
#pragma unroll
      for (int ut = 0; ut < NUT; ++ut) {
        const int uo = 16 * ut + cl;
        const uint32_t off = uo < T && kl < SM::ng(s) ? (uint32_t)(uo * SL + 8 * (SM::goff(s) + kl)) * 2 : OOB;
        bh[ut] = bldu4(rh, off);
        bo[ut] = bldu4(rl, off);
      }
    };
    temporal_units<T, EPI, C, 32, true, decltype(load_adj_s), true, RA>(a, st, u0, uend, 1, load_adj_s);
  } else {
    temporal_units<T, EPI, C, 32, false, decltype(load_adj), true, RA>(a, st, u0, uend, 1, load_adj);
  }
}

// ===========================================================================
// Dynamic adjacency in split-f16 planes (DSTDGC.forward model/dstdgcn.py:
// 83-87 spatial, 88-93 temporal: tanh(P - Q), conv_rm, * alpha + A):
//   out[row][q][slot] = alpha * (sum_k W[row][k] tanh(P[k][p] - Q[k][q]) + b[row]) + Astat[p][q]
// with p = slot_idx(slot).  MODE 0 (spatial): row = t, (p, q) = joints,
// k = r*T + t'.  MODE 1 (temporal): row = v, (p, q) = frames, k = r*V + v'.
// tanh separably, as in dstd_adj.hip: E = 2^(c P), F = 2^(-c Q) once per
// workgroup in LDS ([p][k] rows, k contiguous so a lane's 8 k of a K-step are
// two 16-byte reads), tanh = 1 - 2 / (E F + 1); a sample with |cP| or |cQ|
// above 120 takes the direct tanh(P - Q) path.  The B fragments (tanh
// values) are split into hi/lo in registers and meet the conv_rm A
// fragments (HLJ_RM image in LDS) in three 16x16x32 f16 MFMAs.
// Workgroup = (sample, graph, column chunk), 8 waves over 16-column tiles.
// ===========================================================================

// ---- pieces of the tanh GEMM shared by k_adj_hl and k_temporal_fused ----
// N (8 or 4) consecutive tanh(P[k][p] - Q[k][q]) from the E / F rows: SEP:
// E = 2^(cP), F = 2^(-cQ) and tanh = 1 - 2 / (E F + 1); else P, Q themselves
template <bool SEP, int N>
__device__ __forceinline__ void tanh_run(const float* ep, const float* fq, float (&tv)[8]) {
  float ev[8], fv[8];
#pragma unroll
  for (int h = 0; h < N; h += 4) {
    const float4 e = ld4(ep + h), f = ld4(fq + h);
    ev[h] = e.x, ev[h + 1] = e.y, ev[h + 2] = e.z, ev[h + 3] = e.w;
    fv[h] = f.x, fv[h + 1] = f.y, fv[h + 2] = f.z, fv[h + 3] = f.w;
  }
#ifdef DSTD_TANH_SCALAR
  if constexpr (SEP) {
#pragma unroll
    for (int e = 0; e < N; ++e) tv[e] = fmaf(__builtin_amdgcn_rcpf(fmaf(ev[e], fv[e], 1.f)), -2.f, 1.f);
  } else
#endif
  if constexpr (SEP) {
#pragma unroll
    for (int e2 = 0; e2 < N; e2 += 2) {  // E F + 1 and 1 - 2 r as packed fp32 (v_pk_fma_f32)
      const f32x2_t d = __builtin_elementwise_fma(f32x2_t{ev[e2], ev[e2 + 1]}, f32x2_t{fv[e2], fv[e2 + 1]}, f32x2_t{1.f, 1.f});
      const f32x2_t t = __builtin_elementwise_fma(f32x2_t{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)},
                                                  f32x2_t{-2.f, -2.f}, f32x2_t{1.f, 1.f});
      tv[e2] = t.x;
      tv[e2 + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int e = 0; e < N; ++e) tv[e] = fast_tanh(ev[e] - fv[e]);
  }
#pragma unroll
  for (int e = N; e < 8; ++e) tv[e] = 0.f;
}

// B fragments of one 16-column tile: tanh(P[k][p] - Q[k][q]) for
// k = 32s + 8kg + e (NS full 16x16x32 K-steps) and, with TAIL, k = 32 NS + 4kg
// + e (one 16x16x16 step), split into hi / lo.  El / Fl: the [p][k] rows of
// tanh_run; pr / qr: this lane's rows.
template <bool SEP, int NS, int TAIL>
__device__ __forceinline__ void tanh_frags(const float* El, const float* Fl, int pb, int qb, int kg, f16x8 (&bh)[NS],
                                           f16x8 (&bo)[NS], f16x4& th, f16x4& to) {
  // pb / qb: the lane's E / F row starts (EfRows::row of its rows)
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    float tv[8];
    tanh_run<SEP, 8>(El + pb + 32 * s + 8 * kg, Fl + qb + 32 * s + 8 * kg, tv);
    split8(make_float4(tv[0], tv[1], tv[2], tv[3]), make_float4(tv[4], tv[5], tv[6], tv[7]), bh[s], bo[s]);
  }
  if constexpr (TAIL) {
    float tv[8];
    tanh_run<SEP, 4>(El + pb + 32 * NS + 4 * kg, Fl + qb + 32 * NS + 4 * kg, tv);
    uint2 hi, lo;
    split4(make_float4(tv[0], tv[1], tv[2], tv[3]), hi, lo);
    th = __builtin_bit_cast(f16x4, hi);
    to = __builtin_bit_cast(f16x4, lo);
  }
}

// conv_rm on one column tile: acc[rt][row][col] = sum_k W'[16 rt + row][k] B[k][col]
// (W' = 2^s W, the HLJ_RM image of RT row tiles in LDS)
template <int RT, int NS, int TAIL>
__device__ __forceinline__ void rm_mfma(const uint4* wl, int lane, const f16x8 (&bh)[NS], const f16x8 (&bo)[NS],
                                        const f16x4& th, const f16x4& to, f32x4 (&acc)[RT]) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) acc[rt] = zero4();
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    f16x8 ah[RT], ao[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      ah[rt] = as_h8(wl[((rt * NS + s) * 2 + 0) * 64 + lane]);
      ao[rt] = as_h8(wl[((rt * NS + s) * 2 + 1) * 64 + lane]);
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma32(ao[rt], bh[s], acc[rt]);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma32(ah[rt], bo[s], acc[rt]);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma32(ah[rt], bh[s], acc[rt]);
  }
  if constexpr (TAIL) {
    const uint2* w16 = reinterpret_cast<const uint2*>(wl + RT * NS * 2 * 64);
    f16x4 ah[RT], ao[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      ah[rt] = __builtin_bit_cast(f16x4, w16[(rt * 2 + 0) * 64 + lane]);
      ao[rt] = __builtin_bit_cast(f16x4, w16[(rt * 2 + 1) * 64 + lane]);
    }
    // the tail runs on an accumulator of its own (dstd_hilo.h: mixed-shape MFMA chains)
    f32x4 tac[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) tac[rt] = __builtin_amdgcn_mfma_f32_16x16x16f16(ao[rt], th, zero4(), 0, 0, 0);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) tac[rt] = __builtin_amdgcn_mfma_f32_16x16x16f16(ah[rt], to, tac[rt], 0, 0, 0);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) tac[rt] = __builtin_amdgcn_mfma_f32_16x16x16f16(ah[rt], th, tac[rt], 0, 0, 0);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] += tac[rt];
  }
}

template <int MODE, int NROW, int K, int NA>
struct AdjHLGeom {
  // K-steps: NS full 16x16x32 steps, then (TAIL) one 16x16x16 step when the
  // remainder fits 16 -- K = 70 -> 64 + 16 instead of 96 (17% fewer tanh),
  // K = 44 -> 32 + 16 instead of 64 (25% fewer)
  static constexpr int NS = hl_rm_nsf(K), TAIL = hl_rm_tail(K), KP = 32 * NS + 16 * TAIL;
  static constexpr int RT = cdiv(NROW, 16), KH = K / 2;
  static constexpr int WIMG = RT * (NS * 2 * 64 + TAIL * 64);  // uint4 of the HLJ_RM image
  using EF = typename EfPick<MODE == 1, NA, K>::type;  // E / F row placement
  static constexpr int SE = EF::SE;
  using SM = SlotMap<NA, MODE == 0>;
  static constexpr int SL = SM::SL, NCOL = NA * SL, NCT = cdiv(NCOL, 16);
  // column chunks (one workgroup each) per (sample, graph) at full batch;
  // the launcher raises the count when B * ngroups * NCHUNK leaves CUs idle
#ifndef DSTD_ADJ_T_NCHUNK  // (experiments: column chunks of the temporal adjacency per sample)
#define DSTD_ADJ_T_NCHUNK 2
#endif
  static constexpr int NCHUNK = MODE == 0 ? 1 : DSTD_ADJ_T_NCHUNK;
  static constexpr int CPC = cdiv(NCT, NCHUNK);
  static constexpr int OS = 20;  // staging row stride (floats)
  static constexpr int T = MODE == 0 ? NROW : NA, V = MODE == 0 ? NA : NROW;
  static_assert(2 * KH == K, "K = 2 * (T or V)");
  // waves per workgroup: every wave gets the same number of column tiles
  // (33 spatial tiles at V = 22 -> 11 waves x 3; the old 8 waves left a
  // 5-vs-4 tail in every workgroup)
  static constexpr int ROUNDS = cdiv(CPC, 12);
  static constexpr int AW = cdiv(CPC, ROUNDS);
  static constexpr int AT = AW * 64;
};

template <int MODE, int NROW, int K, int NA>
__global__ __launch_bounds__((AdjHLGeom<MODE, NROW, K, NA>::AT)) void k_adj_hl(AdjHLArgs a) {
  using Gm = AdjHLGeom<MODE, NROW, K, NA>;
  using SM = typename Gm::SM;
  constexpr int RT = Gm::RT, NS = Gm::NS, KP = Gm::KP, KH = Gm::KH, SL = Gm::SL, NCOL = Gm::NCOL;
  constexpr int AW = Gm::AW, AT = Gm::AT, TAIL = Gm::TAIL, WIMG = Gm::WIMG;
  constexpr int OS = Gm::OS, T = Gm::T, V = Gm::V;
  constexpr float C2 = 2.8853900817779268f;  // 2*log2(e)
  using EF = typename Gm::EF;
  __shared__ float El[EF::floats(NA + 1)];
  __shared__ float Fl[EF::floats(NA + 1)];
  __shared__ uint4 wl[WIMG];
  __shared__ float asl[NA * NA + 1];
  __shared__ float bsl[RT * 16];
  __shared__ float stg[AW][32 * OS];  // two row tiles at a time

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kg = lane >> 4, cl = lane & 15;
  const int nch = a.nchunk, cpc = cdiv(Gm::NCT, nch);
  const int chunk = blockIdx.x % nch;
  const int g = (blockIdx.x / nch) % a.ngroups;
  const int n = blockIdx.x / (nch * a.ngroups);
  if (n >= a.B) return;
  TLH(MODE, 0)
#ifdef DSTD_SETPRIO_ADJ  // (experiment: the younger waves' static priority, as k_spatial_hl)
  if (__builtin_amdgcn_readfirstlane(tid) >= DSTD_SETPRIO_ADJ) __builtin_amdgcn_s_setprio(1);
#endif

  // ---- prologue: P/Q -> E/F rows, conv_rm fragments, A-stat, bias.  Every
  // global load is issued before the first LDS write (one memory round
  // trip instead of one per loop iteration) ----
  const PQLayout L = a.pql;
  const float* pqb = a.pq + (size_t)n * L.sn + a.p_ch[g];
  constexpr int NPQ = cdiv(T * V, AT), NW = cdiv(WIMG, AT), NAS = cdiv(NA * NA, AT);
  float4 q4[NPQ];
  uint4 wv[NW];
  float av[NAS];
  if (MODE == 0 && a.xin) {
    // conv_st_in (model/dstdgcn.py:298-305): P/Q of x6 = cat(x, x - x[:, -1])
    // straight from the model input [B][T][V][3]; this graph's conv_m1/m2 rows
    float wm[4][6], bm[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int c = 0; c < 6; ++c) wm[r][c] = a.mw[g][r >> 1][(r & 1) * 6 + c];
      bm[r] = a.mb[g][r >> 1][r & 1];
    }
    const float* xn = a.xin + (size_t)n * T * V * 3;
#pragma unroll
    for (int it = 0; it < NPQ; ++it) {
      const int i = min(tid + it * AT, T * V - 1);
      const int t = MODE == 0 ? i % T : i / V, v = MODE == 0 ? i / T : i % V;
      const float* xc = xn + (t * V + v) * 3;
      const float* xl = xn + ((T - 1) * V + v) * 3;
      const float x6v[6] = {xc[0], xc[1], xc[2], xc[0] - xl[0], xc[1] - xl[1], xc[2] - xl[2]};
      float pq[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float acc = bm[r];
#pragma unroll
        for (int c = 0; c < 6; ++c) acc = fmaf(wm[r][c], x6v[c], acc);
        pq[r] = acc;
      }
      q4[it] = make_float4(pq[0], pq[1], pq[2], pq[3]);
    }
  } else {
#pragma unroll
    for (int it = 0; it < NPQ; ++it) {
      const int i = min(tid + it * AT, T * V - 1);                              // clamped: no branch
      const int t = MODE == 0 ? i % T : i / V, v = MODE == 0 ? i / T : i % V;  // memory order
      q4[it] = ld4(pqb + t * L.st + v * L.sv);                                  // (P_0, P_1, Q_0, Q_1)
    }
  }
#pragma unroll
  for (int it = 0; it < NW; ++it) wv[it] = a.wimg[g][min(tid + it * AT, WIMG - 1)];
#pragma unroll
  for (int it = 0; it < NAS; ++it) av[it] = a.astat[g][min(tid + it * AT, NA * NA - 1)];
  const float bv = tid < NROW ? a.bias[g][tid] : 0.f;
  // padding: k in [K, KP) and the row p = q = NA: E = F = 1 (tanh 0)
  for (int i = tid; i < (NA + 1) * (KP - K); i += AT) {
    const int r = i / (KP > K ? KP - K : 1), k = K + i % (KP > K ? KP - K : 1);
    El[EF::row(r) + k] = 1.f;
    Fl[EF::row(r) + k] = 1.f;
  }
  for (int i = tid; i < K; i += AT) {
    El[EF::row(NA) + i] = 1.f;
    Fl[EF::row(NA) + i] = 1.f;
  }
  int bad = 0;
#pragma unroll
  for (int it = 0; it < NPQ; ++it) {
    const int i = tid + it * AT;
    if (i < T * V) {
      const int t = MODE == 0 ? i % T : i / V, v = MODE == 0 ? i / T : i % V;
      const int pr = MODE == 0 ? v : t, ki = MODE == 0 ? t : v;
      const float ep0 = C2 * q4[it].x, ep1 = C2 * q4[it].y, eq0 = -C2 * q4[it].z, eq1 = -C2 * q4[it].w;
      bad |= !(fabsf(ep0) <= 120.f && fabsf(ep1) <= 120.f && fabsf(eq0) <= 120.f && fabsf(eq1) <= 120.f);
      El[EF::row(pr) + ki] = __builtin_amdgcn_exp2f(ep0);
      El[EF::row(pr) + KH + ki] = __builtin_amdgcn_exp2f(ep1);
      Fl[EF::row(pr) + ki] = __builtin_amdgcn_exp2f(eq0);
      Fl[EF::row(pr) + KH + ki] = __builtin_amdgcn_exp2f(eq1);
    }
  }
#pragma unroll
  for (int it = 0; it < NW; ++it)
    if (tid + it * AT < WIMG) wl[tid + it * AT] = wv[it];
#pragma unroll
  for (int it = 0; it < NAS; ++it)
    if (tid + it * AT < NA * NA) asl[tid + it * AT] = av[it];
  if (tid == 0) asl[NA * NA] = 0.f;
  if (tid < RT * 16) bsl[tid] = bv;
  const bool sep = __syncthreads_or(bad) == 0;
  if (!sep) {  // direct path: E / F hold P / Q themselves (padding 0)
    __syncthreads();
#pragma unroll
    for (int it = 0; it < NPQ; ++it) {
      const int i = tid + it * AT;
      if (i < T * V) {
        const int t = MODE == 0 ? i % T : i / V, v = MODE == 0 ? i / T : i % V;
        const int pr = MODE == 0 ? v : t, ki = MODE == 0 ? t : v;
        El[EF::row(pr) + ki] = q4[it].x;
        El[EF::row(pr) + KH + ki] = q4[it].y;
        Fl[EF::row(pr) + ki] = q4[it].z;
        Fl[EF::row(pr) + KH + ki] = q4[it].w;
      }
    }
    for (int i = tid; i < (NA + 1) * (KP - K); i += AT) {
      const int r = i / (KP > K ? KP - K : 1), k = K + i % (KP > K ? KP - K : 1);
      El[EF::row(r) + k] = 0.f;
      Fl[EF::row(r) + k] = 0.f;
    }
    for (int i = tid; i < K; i += AT) {
      El[EF::row(NA) + i] = 0.f;
      Fl[EF::row(NA) + i] = 0.f;
    }
    __syncthreads();
  }
  // tanh(P - Q) = 1 - 2 / (E F + 1) formed per element (contracting W with
  // r = 1 / (E F + 1) and folding b + sum_k W into the bias saves one packed
  // FMA per element but cancels in the accumulator: the whole-model error
  // tail measured 1.7x the reference's fp32 error at the 90th percentile
  // against 1.2x this way -- scripts/parity_stats.py)
  // planes stored as 2^-sa Adj (dstd_hilo.h "range scaling"; one sa for both
  // spatial graphs, the GC kernel scales its aggregation back)
  const float bnd = a.ngroups == 2 ? fmaxf(a.wscale[0][HLS_BOUND], a.wscale[1][HLS_BOUND]) : a.wscale[0][HLS_BOUND];
  const float dna = pow2f(-hl_range_shift(fexp_bits(__float_as_uint(bnd))));
  const float alpha = *a.alpha * dna, inv = *a.wscale[g];
  TLH(MODE, 1)

  float* so = stg[wave];
  uint16_t* out = a.out + (size_t)n * a.out_sN + (size_t)g * a.out_sG;
  const auto ro = rsrc(out, 2u * NROW * 2 * NCOL);
  const int ct_end = min(Gm::NCT, (chunk + 1) * cpc);
  auto tiles = [&](auto sep_c) {
    constexpr bool SEP = decltype(sep_c)::value;
    for (int ct = chunk * cpc + wave; ct < ct_end; ct += AW) {
      // this lane's column (B operand column j = cl)
      const int col = ct * 16 + cl;
      const int q = col / SL, pi = SM::slot_idx(col - q * SL);
      const bool valid = col < NCOL && pi < NA;
      const int pr = valid ? pi : NA, qr = col < NCOL ? q : NA;
      f16x8 bh[NS], bo[NS];
      f16x4 th, to;
      tanh_frags<SEP, NS, TAIL>(El, Fl, EF::row(pr), EF::row(qr), kg, bh, bo, th, to);
      f32x4 acc[RT];
      rm_mfma<RT, NS, TAIL>(wl, lane, bh, bo, th, to, acc);
      // ---- epilogue: alpha * (acc + b) + Astat, 0 on padding slots; staged
      // through this wave's LDS slot so a lane stores 8 consecutive slots ----
      // padding slots: alpha -> 0 and Astat[NA*NA] = 0, so the value is 0 without a select
      const float as = asl[valid ? pr * NA + qr : NA * NA] * dna, al = valid ? alpha : 0.f;
  #pragma unroll
      for (int r2 = 0; r2 < RT; r2 += 2) {
  #pragma unroll
        for (int dr = 0; dr < 2; ++dr) {
          if (r2 + dr >= RT) continue;
  #pragma unroll
          for (int r = 0; r < 4; r += 2) {  // row pairs as packed fp32
            const int row = (r2 + dr) * 16 + 4 * kg + r;
            const f32x2_t v = __builtin_elementwise_fma(
                f32x2_t{al, al},
                __builtin_elementwise_fma(f32x2_t{acc[r2 + dr][r], acc[r2 + dr][r + 1]}, f32x2_t{inv, inv},
                                          f32x2_t{bsl[row], bsl[row + 1]}),
                f32x2_t{as, as});
            so[(dr * 16 + 4 * kg + r) * OS + cl] = v.x;
            so[(dr * 16 + 4 * kg + r + 1) * OS + cl] = v.y;
          }
        }
        // lane -> (row of the pair, 8-column half); rows on consecutive lanes
        // (lane & 31), halves on the wave halves: with OS = 20 every 16-lane
        // group of the ds_read_b128 hits 16 distinct 4-bank chunks (the
        // (lane >> 1, lane & 1) map was 2-way conflicted; -0.6% per launch)
        const int rl = lane & 31, h = lane >> 5, row = r2 * 16 + rl, c8 = ct * 16 + 8 * h;
        const float4 v0 = ld4(so + rl * OS + 8 * h), v1 = ld4(so + rl * OS + 8 * h + 4);
        uint4 hi, lo;
        split8(v0, v1, hi, lo);
        // rows / columns past the plane: out-of-range offset, the store is dropped
        const uint32_t off = row < NROW && c8 < NCOL ? 2u * (uint32_t)(row * (2 * NCOL) + c8) : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi), ro, off, 0, DSTD_ADJ_ST_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo), ro, off + 2u * NCOL, 0, DSTD_ADJ_ST_AUX);
      }
    }
  };
  // separable-exp path or the direct tanh fallback, chosen once per workgroup
  if (sep) tiles(std::true_type{});
  else tiles(std::false_type{});
  TLH(MODE, 2)
#ifdef DSTD_STAMPS
  // slot 3: HW_ID (cu / se) and XCC_ID of the workgroup's placement
  if (threadIdx.x == 0 && blockIdx.x < 2048)
    g_tl_hl[MODE][blockIdx.x][3] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                                   (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
#endif
}

// ===========================================================================
// Temporal DSTDGC with its dynamic adjacency built in LDS (DSTDGC.forward
// temporal, model/dstdgcn.py:88-93, and the DSTDGCB tail epilogues of
// k_temporal_hl).  One workgroup per sample, persistent over samples; per
// chunk of RC joints:
//  phase 1: Adj[v][t][u] = alpha (sum_k W_rm[v][k] tanh(P[k][t] - Q[k][u]) +
//           b[v]) + Astat[t][u] for the chunk's joints -- the tanh GEMM of
//           k_adj_hl (rows = joints, K = 2V, columns (u, slot)) -- written as
//           split-f16 planes [v][2][T][SL] into LDS;
//  phase 2: the temporal GC units (sample, joint) of the chunk, their B
//           fragments read from those planes (temporal_units).
// The planes never reach HBM (k_adj_hl<1> + k_temporal_hl wrote and re-read
// 2 V T SL halves x 2 bytes per sample: 123 KB each way at H36M).  Phase 1 is
// VALU-bound (the tanh), phase 2 MFMA / memory; the one workgroup per CU the
// LDS allows runs them back to back.  Grid = B (a persistent sample loop kept
// its loop-carried state live through phase 2 and spilled).
// Round 3 tried the phases overlapped (k_temporal_pipe: 4 waves building the
// next chunk's planes while 4 run the GC units of this one; all variants
// bit-exact): 38% slower at H36M, 24% at CMU, 34% at 3DPW -- the units are
// latency-bound streaming and lost half their loads in flight
// (profiles/r03f_pipe_ab.txt).  Retired.
// ===========================================================================
constexpr int kLdsBudget = 160 * 1024;

template <int T, int V, int EPI, int C>
struct TFusedGeom {
  using SM = SlotMap<T, false>;
  static constexpr int K = 2 * V, NS = hl_rm_nsf(K), TAIL = hl_rm_tail(K), KP = 32 * NS + 16 * TAIL;
  using EF = typename EfPick<true, T, K>::type;  // E / F row placement
  static constexpr int SE = EF::SE, EFE = EF::floats(T + 1);  // floats of the E array (every input frame + pad row)
  static constexpr int SL = SM::SL, NUT = cdiv(T, 16);
  static constexpr int RTG = cdiv(V, 16);  // row tiles of the whole HLJ_RM image
  static constexpr size_t stage_bytes = sizeof(TemporalStage<T, EPI, C, V>);
  static constexpr size_t al16(size_t b) { return (b + 15) & ~size_t(15); }
  static constexpr int jn(int rc) { return rc < V ? rc : V; }  // joints stored per chunk
  // a chunk's planes hold uf output frames (T: all of them; 16: one u tile)
  // halves per joint: two planes + 8 (a joint 4 rows down lands on other
  // banks), the 8 kept zero: the B fragment of a padding slot
  static constexpr int pj(int uf) { return 2 * uf * SL + 8; }
  // F rows: the chunk's output frames + the pad row
  static constexpr int eff(int uf) { return EF::floats((uf == T ? T : uf) + 1); }
  static constexpr int asq(int uf) { return cdiv(uf * SL, 16) * 16; }
  // phase-1 scratch: E / F rows, the chunk's conv_rm rows, the epilogue's
  // per-column tables (Astat and alpha in plane slot order), conv_rm bias
  static constexpr size_t p1_bytes(int rtc, int uf) {
    return (size_t)(EFE + eff(uf)) * 4 + (size_t)rtc * (NS * 2 * 64 + TAIL * 64) * 16 + (size_t)2 * asq(uf) * 4 +
           (size_t)rtc * 16 * 4;
  }
  static constexpr size_t total(int rc, int uf) {
    return al16((size_t)jn(rc) * pj(uf) * 2) +
           al16(p1_bytes(rc / 16, uf) > stage_bytes ? p1_bytes(rc / 16, uf) : stage_bytes);
  }
  // chunking: none when every joint's planes fit (H36M); else chunks of one
  // row tile of joints (CMU, 3DPW: each chunk regenerates the tanh operand,
  // shared by every joint row); else (T = 75: 528 KB of planes per sample)
  // every joint but one u tile of 16 output frames per chunk -- the tanh
  // operand's columns split with no regeneration, each chunk re-running the
  // units' conv (their K is every input frame) for its u tile's aggregation
  static constexpr bool FIT = total(16 * RTG, T) <= kLdsBudget;
  static constexpr bool JCH = !FIT && total(16, T) <= kLdsBudget;
  static constexpr bool UCH = !FIT && !JCH;
  static constexpr int UF = UCH ? 16 : T, NUTC = UCH ? 1 : NUT;  // output frames / u tiles per chunk
  static constexpr int RC = JCH ? 16 : 16 * RTG;
  static constexpr int RTC = RC / 16, NJCH = cdiv(V, RC), NUCH = UCH ? NUT : 1, NCHUNK = NJCH * NUCH;
  static constexpr int EFF = eff(UF), NFR = (UCH ? UF : T) + 1;  // F array floats / rows (pad row NFR - 1)
  static constexpr int NCOL = UF * SL, NCTC = cdiv(NCOL, 16), ASQ = asq(UF);
  static constexpr int PJ = pj(UF), ZPAD = 2 * UF * SL;
  static constexpr int WIMG = RTC * (NS * 2 * 64 + TAIL * 64);  // uint4 of the chunk's HLJ_RM rows
  static constexpr size_t PLANES = al16((size_t)jn(RC) * PJ * 2), LDS = total(RC, UF);
  static_assert(LDS <= kLdsBudget, "planes of one chunk must fit");
};

// ---- phase 3 of k_temporal_fused: the NEXT block's spatial adjacency planes
// of sample n (k_adj_hl<0>'s GEMM and epilogue, transposed as in phase 1:
// A = tanh columns, B = conv_rm rows).  The workgroup has just written every
// (t, v) P/Q of the sample in its units' epilogues, so the planes follow in
// the same launch: no k_adj_hl<0> launch (its prologue round trip and tail),
// the P/Q read back from L2 by the CU that wrote them.  LDS: both graphs' E/F
// rows and Astat (the planes and the stage of phases 1-2 are dead by then).
template <int T, int V>
struct SAdjGeom {
  using SM = SlotMap<V, true>;
  static constexpr int K = 2 * T, NS = hl_rm_nsf(K), TAIL = hl_rm_tail(K), KP = 32 * NS + 16 * TAIL;
  using EF = typename EfPick<false, V, K>::type;  // E / F row placement
  static constexpr int SE = EF::SE, EFN = EF::floats(V + 1);  // floats per E (F) array
  static constexpr int SL = SM::SL, NCOL = V * SL, NCTC = cdiv(NCOL, 16), RT = cdiv(T, 16), FULL = NS * 2 * 64;
  static constexpr int WIMG = RT * (FULL + TAIL * 64);  // uint4 of one graph's HLJ_RM image
  static constexpr size_t al16(size_t b) { return (b + 15) & ~size_t(15); }
  static constexpr size_t EFB = al16(2 * (size_t)EFN * 4);  // one graph's E rows then F rows
  // one graph's epilogue tables in plane slot order (as phase 1's asq / alq):
  // 2^-sa Astat[pi][q] then 2^-sa alpha per column, 0 on padding slots
  static constexpr int ASQ = NCTC * 16;
  static constexpr size_t AS = al16((size_t)2 * ASQ * 4);
  static constexpr size_t WB = (size_t)WIMG * 16;                   // one graph's image
  static constexpr size_t BB = al16((size_t)16 * RT * 4);           // one graph's conv_rm bias (rows padded)
  static constexpr size_t LDS = 2 * (EFB + AS + WB + BB);
};

// The P/Q-independent global loads of spatial_adj_sample's prologue (both
// conv_rm images, the Astat table entries, the conv_rm bias): issued by
// phase 3's caller before the barrier that ends phase 2, so their latency
// hides in the wait for the last joint units (the unit registers are dead)
template <int T, int V, int NT>
struct SAdjStatic {
  using Gm = SAdjGeom<T, V>;
  static constexpr int NWI = cdiv(2 * Gm::WIMG, NT), NAS = cdiv(2 * Gm::ASQ, NT);
  u32x4 wv[NWI];
  float av[NAS];
  int aok;  // bit it: the table entry of iteration it is a valid (pi, q)
  float bv;
  __device__ __forceinline__ void load(const AdjHLArgs& j, int tid) {
    using SM = typename Gm::SM;
    constexpr int WIMG = Gm::WIMG, SL = Gm::SL, NCOL = Gm::NCOL, RT = Gm::RT;
#pragma unroll
    for (int it = 0; it < NWI; ++it) {
      const int i = min(tid + it * NT, 2 * WIMG - 1);
      wv[it] = *reinterpret_cast<const u32x4*>((i >= WIMG ? j.wimg[1] : j.wimg[0]) + (i >= WIMG ? i - WIMG : i));
    }
    aok = 0;
#pragma unroll
    for (int it = 0; it < NAS; ++it) {
      const int i = tid + it * NT, g = i >= Gm::ASQ, col = i - g * Gm::ASQ, q = col / SL;
      const int pi = col < NCOL ? SM::slot_idx(col - q * SL) : V;
      const bool ok = pi < V && i < 2 * Gm::ASQ;
      if (ok) aok |= 1 << it;
      av[it] = (g ? j.astat[1] : j.astat[0])[ok ? pi * V + q : 0];
    }
    const int bg = tid >= 16 * RT, br = tid - bg * 16 * RT;
    bv = tid < 2 * 16 * RT && br < T ? (bg ? j.bias[1] : j.bias[0])[br] : 0.f;
  }
};

// XIN: the P/Q from the model input (j.xin, conv_st_in's conv_m1/m2 rows
// j.mw / j.mb, as k_adj_hl<0> forms them) instead of j.pq.  pre: the
// prologue's static loads, already issued (SAdjStatic::load), or null
template <int T, int V, int NT, bool XIN = false>
__device__ __forceinline__ void spatial_adj_sample(const AdjHLArgs& j, int n, unsigned char* dsm,
                                                   const SAdjStatic<T, V, NT>* pre = nullptr) {
  using Gm = SAdjGeom<T, V>;
  using SM = typename Gm::SM;
  using EF = typename Gm::EF;
  constexpr int NS = Gm::NS, TAIL = Gm::TAIL, KP = Gm::KP, K = Gm::K, EFN = Gm::EFN, SL = Gm::SL, NCOL = Gm::NCOL;
  constexpr int RT = Gm::RT, FULL = Gm::FULL, WIMG = Gm::WIMG, NW = NT / 64, NCTC = Gm::NCTC;
  constexpr float C2 = 2.8853900817779268f;  // 2*log2(e)
  // LDS: [E/F g0][E/F g1][Astat g0][Astat g1][image g0][image g1][bias g0][bias g1]
  auto Elg = [&](int g) { return reinterpret_cast<float*>(dsm + g * Gm::EFB); };  // F rows at + EFN
  auto asg = [&](int g) { return reinterpret_cast<float*>(dsm + 2 * Gm::EFB + g * Gm::AS); };  // alq: + ASQ
  uint4* wl = reinterpret_cast<uint4*>(dsm + 2 * (Gm::EFB + Gm::AS));  // both images, graph-major
  float* bl = reinterpret_cast<float*>(dsm + 2 * (Gm::EFB + Gm::AS + Gm::WB));  // [g][16 RT]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = lane >> 4, cl = lane & 15;

  // ---- prologue: both graphs' P/Q -> E/F rows, conv_rm images, Astat, bias;
  // every global load before the first LDS write ----
  const PQLayout L = j.pql;
  constexpr int NPQ = cdiv(T * V, NT), NWI = cdiv(2 * WIMG, NT), NAS = cdiv(2 * Gm::ASQ, NT);
  auto pq_at = [&](int g, int i) __attribute__((always_inline)) -> float4 {  // (P_0, P_1, Q_0, Q_1) of element i (joint-major)
    const int t = i % T, v = i / T;
    return ld4(j.pq + (size_t)n * L.sn + j.p_ch[g] + t * L.st + v * L.sv);
  };
  float4 q4[2][NPQ];
  if constexpr (XIN) {
    // conv_st_in (model/dstdgcn.py:298-305): P/Q of x6 = cat(x, x - x[:, -1]),
    // the same fmaf chain as k_adj_hl<0>'s prologue (bit-identical planes)
    const float* xn = j.xin + (size_t)n * T * V * 3;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      float wm[4][6], bm[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int c = 0; c < 6; ++c) wm[r][c] = j.mw[g][r >> 1][(r & 1) * 6 + c];
        bm[r] = j.mb[g][r >> 1][r & 1];
      }
#pragma unroll
      for (int it = 0; it < NPQ; ++it) {
        const int i = min(tid + it * NT, T * V - 1);
        const int t = i % T, v = i / T;
        const float* xc = xn + (t * V + v) * 3;
        const float* xl = xn + ((T - 1) * V + v) * 3;
        const float x6v[6] = {xc[0], xc[1], xc[2], xc[0] - xl[0], xc[1] - xl[1], xc[2] - xl[2]};
        float pq[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float acc = bm[r];
#pragma unroll
          for (int c = 0; c < 6; ++c) acc = fmaf(wm[r][c], x6v[c], acc);
          pq[r] = acc;
        }
        q4[g][it] = make_float4(pq[0], pq[1], pq[2], pq[3]);
      }
    }
  } else {
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int it = 0; it < NPQ; ++it) q4[g][it] = pq_at(g, min(tid + it * NT, T * V - 1));
  }
  static_assert(SAdjStatic<T, V, NT>::NWI == NWI && SAdjStatic<T, V, NT>::NAS == NAS, "prologue split");
  SAdjStatic<T, V, NT> sl;
  if (pre) sl = *pre;
  else sl.load(j, tid);
  // planes stored as 2^-sa Adj, one sa for both graphs (dstd_hilo.h "range scaling")
  const float dna = pow2f(-hl_range_shift(
      fexp_bits(__float_as_uint(fmaxf(j.wscale[0][HLS_BOUND], j.wscale[1][HLS_BOUND])))));
  const float alpha = *j.alpha * dna;
#pragma unroll
  for (int it = 0; it < NWI; ++it)
    if (tid + it * NT < 2 * WIMG) *reinterpret_cast<u32x4*>(wl + tid + it * NT) = sl.wv[it];
#pragma unroll
  for (int it = 0; it < NAS; ++it) {
    const int i = tid + it * NT, g = i >= Gm::ASQ;
    if (i < 2 * Gm::ASQ) {
      const bool ok = (sl.aok >> it) & 1;
      float* t = asg(g) + (i - g * Gm::ASQ);
      t[0] = ok ? sl.av[it] * dna : 0.f;
      t[Gm::ASQ] = ok ? alpha : 0.f;
    }
  }
  if (tid < 2 * 16 * RT) bl[tid] = sl.bv;
  auto ef_pad = [&](int g, float val) __attribute__((always_inline)) {  // padding k and the row p = q = V: tanh 0
    float* El = Elg(g);
    float* Fl = El + EFN;
    for (int i = tid; i < (V + 1) * (KP - K); i += NT) {
      const int r = i / (KP > K ? KP - K : 1), k = K + i % (KP > K ? KP - K : 1);
      El[EF::row(r) + k] = val;
      Fl[EF::row(r) + k] = val;
    }
    for (int i = tid; i < K; i += NT) {
      El[EF::row(V) + i] = val;
      Fl[EF::row(V) + i] = val;
    }
  };
  ef_pad(0, 1.f);
  ef_pad(1, 1.f);
  int bad[2] = {0, 0};
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    float* El = Elg(g);
    float* Fl = El + EFN;
#pragma unroll
    for (int it = 0; it < NPQ; ++it) {
      const int i = tid + it * NT;
      if (i < T * V) {
        const int t = i % T, v = i / T;
        const float ep0 = C2 * q4[g][it].x, ep1 = C2 * q4[g][it].y, eq0 = -C2 * q4[g][it].z, eq1 = -C2 * q4[g][it].w;
        bad[g] |= !(fabsf(ep0) <= 120.f && fabsf(ep1) <= 120.f && fabsf(eq0) <= 120.f && fabsf(eq1) <= 120.f);
        El[EF::row(v) + t] = __builtin_amdgcn_exp2f(ep0);
        El[EF::row(v) + T + t] = __builtin_amdgcn_exp2f(ep1);
        Fl[EF::row(v) + t] = __builtin_amdgcn_exp2f(eq0);
        Fl[EF::row(v) + T + t] = __builtin_amdgcn_exp2f(eq1);
      }
    }
  }
  // separable or direct tanh per graph, as k_adj_hl<0> decides per (sample, graph) workgroup
  // (one reduction for both graphs in the common case; __syncthreads_or
  // returns a boolean, not the OR of the bits, so a sample with a flag set
  // asks per graph)
  bool sep0 = true, sep1 = true;
  if (__syncthreads_or(bad[0] | bad[1])) {
    sep0 = __syncthreads_or(bad[0]) == 0;
    sep1 = __syncthreads_or(bad[1]) == 0;
  }
  if (!sep0 || !sep1) {  // direct path: E / F hold P / Q themselves (padding 0)
    __syncthreads();
    for (int g = 0; g < 2; ++g) {
      if (g ? sep1 : sep0) continue;
      ef_pad(g, 0.f);
      float* El = Elg(g);
      float* Fl = El + EFN;
      if constexpr (XIN) {  // (no P/Q in memory: the prologue's values)
#pragma unroll
        for (int it = 0; it < NPQ; ++it) {
          const int i = tid + it * NT;
          if (i < T * V) {
            const int t = i % T, v = i / T;
            const float4 p4 = g ? q4[1][it] : q4[0][it];
            El[EF::row(v) + t] = p4.x;
            El[EF::row(v) + T + t] = p4.y;
            Fl[EF::row(v) + t] = p4.z;
            Fl[EF::row(v) + T + t] = p4.w;
          }
        }
      } else {
        for (int i = tid; i < T * V; i += NT) {
          const int t = i % T, v = i / T;
          const float4 p4 = pq_at(g, i);
          El[EF::row(v) + t] = p4.x;
          El[EF::row(v) + T + t] = p4.y;
          Fl[EF::row(v) + t] = p4.z;
          Fl[EF::row(v) + T + t] = p4.w;
        }
      }
    }
    __syncthreads();
  }
  const float inv0 = *j.wscale[0], inv1 = *j.wscale[1];
  TLH(2, 1)

#ifndef DSTD_P3_TPI
#define DSTD_P3_TPI 1
#endif
#ifndef DSTD_P3_NOSTORE  // (timing experiments only: the plane stores dropped, wrong output)
#define DSTD_P3_NOSTORE 0
#endif
  constexpr int TPI = DSTD_P3_TPI;  // column tiles per iteration (independent dependency chains)
  if constexpr (TPI == 1) {
    // one tile space over both graphs (2 NCTC column tiles): the waves split
    // it evenly instead of rounding up twice
    f16x8 wh[RT][NS], wo[RT][NS];  // the current graph's conv_rm rows as B fragments
    f16x4 wth[RT], wto[RT];        // (lane = row 16 rt + cl, k group kg)
    float b[RT];
    int gcur = -1;
#pragma unroll 1
    for (int ti = wave; ti < 2 * NCTC; ti += NW) {
      const int g = ti >= NCTC ? 1 : 0, ct = ti - g * NCTC;
      if (g != gcur) {  // (wave-uniform: at most once per wave)
        gcur = g;
        const uint4* wg = wl + g * WIMG;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            wh[rt][s] = as_h8(wg[((rt * NS + s) * 2 + 0) * 64 + lane]);
            wo[rt][s] = as_h8(wg[((rt * NS + s) * 2 + 1) * 64 + lane]);
          }
          if constexpr (TAIL) {
            const uint2* w16 = reinterpret_cast<const uint2*>(wg + RT * FULL);
            wth[rt] = __builtin_bit_cast(f16x4, w16[(rt * 2 + 0) * 64 + lane]);
            wto[rt] = __builtin_bit_cast(f16x4, w16[(rt * 2 + 1) * 64 + lane]);
          }
          b[rt] = bl[g * 16 * RT + 16 * rt + cl];
        }
      }
      const float inv = g ? inv1 : inv0;
      const float* El = Elg(g);
      const float* Fl = El + EFN;
      const float* as = asg(g);
      const auto ro = rsrc(j.out + (size_t)n * j.out_sN + (size_t)g * j.out_sG, 2u * T * 2 * NCOL);
      // this lane's A-operand row = column ct * 16 + cl of the planes
      const int col = ct * 16 + cl;
      const int qa = col / SL, pa = SM::slot_idx(col - qa * SL);
      const bool va = col < NCOL && pa < V;
      f16x8 bh[NS], bo[NS];
      f16x4 th, to;
      const int pb = EF::row(va ? pa : V), qb = EF::row(col < NCOL ? qa : V);
      if (g ? sep1 : sep0) tanh_frags<true, NS, TAIL>(El, Fl, pb, qb, kg, bh, bo, th, to);
      else tanh_frags<false, NS, TAIL>(El, Fl, pb, qb, kg, bh, bo, th, to);
      // the accumulator's 4 columns colb .. colb + 3 (one joint q, slots slot0 ..)
      const int colb = ct * 16 + 4 * kg;
      const float4 as4 = ld4(as + colb), al4 = ld4(as + Gm::ASQ + colb);
      const float asv[4] = {as4.x, as4.y, as4.z, as4.w}, al[4] = {al4.x, al4.y, al4.z, al4.w};
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        f32x4 acc = zero4();
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          acc = mfma32(bh[s], wo[rt][s], acc);
          acc = mfma32(bo[s], wh[rt][s], acc);
          acc = mfma32(bh[s], wh[rt][s], acc);
        }
        if constexpr (TAIL) {  // on an accumulator of its own (dstd_hilo.h: mixed-shape MFMA chains)
          f32x4 tac = __builtin_amdgcn_mfma_f32_16x16x16f16(th, wto[rt], zero4(), 0, 0, 0);
          tac = __builtin_amdgcn_mfma_f32_16x16x16f16(to, wth[rt], tac, 0, 0, 0);
          tac = __builtin_amdgcn_mfma_f32_16x16x16f16(th, wth[rt], tac, 0, 0, 0);
          acc += tac;
        }
        float vv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) vv[r] = fmaf(al[r], fmaf(acc[r], inv, b[rt]), asv[r]);
        uint2 hi, lo;
        split4(make_float4(vv[0], vv[1], vv[2], vv[3]), hi, lo);
        // frame t = 16 rt + cl: the hi plane at [t][0][col], lo at [t][1][col]
        const int t = 16 * rt + cl;
        const uint32_t off = t < T && colb < NCOL && !DSTD_P3_NOSTORE ? 2u * (uint32_t)(t * 2 * NCOL + colb) : OOB;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, hi), ro, off, 0, DSTD_ADJ_ST_AUX);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, lo), ro, off + 2u * NCOL, 0, DSTD_ADJ_ST_AUX);
      }
    }
  } else {
    // TPI column tiles of ONE graph per task (the W fragments stay per
    // graph): tasks = (graph, tile group), the waves split them evenly; a
    // wave interleaves its tiles' tanh -> split -> MFMA chains (round 6:
    // phase 3 ran ~3x over its issue bound at one chain per wave)
    constexpr int NGRP = cdiv(NCTC, TPI);
    f16x8 wh[RT][NS], wo[RT][NS];
    f16x4 wth[RT], wto[RT];
    float b[RT];
    int gcur = -1;
#pragma unroll 1
    for (int ti = wave; ti < 2 * NGRP; ti += NW) {
      const int g = ti >= NGRP ? 1 : 0, ct0 = (ti - g * NGRP) * TPI;
      if (g != gcur) {  // (wave-uniform: at most once per wave)
        gcur = g;
        const uint4* wg = wl + g * WIMG;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            wh[rt][s] = as_h8(wg[((rt * NS + s) * 2 + 0) * 64 + lane]);
            wo[rt][s] = as_h8(wg[((rt * NS + s) * 2 + 1) * 64 + lane]);
          }
          if constexpr (TAIL) {
            const uint2* w16 = reinterpret_cast<const uint2*>(wg + RT * FULL);
            wth[rt] = __builtin_bit_cast(f16x4, w16[(rt * 2 + 0) * 64 + lane]);
            wto[rt] = __builtin_bit_cast(f16x4, w16[(rt * 2 + 1) * 64 + lane]);
          }
          b[rt] = bl[g * 16 * RT + 16 * rt + cl];
        }
      }
      const float inv = g ? inv1 : inv0;
      const float* El = Elg(g);
      const float* Fl = El + EFN;
      const float* as = asg(g);
      const auto ro = rsrc(j.out + (size_t)n * j.out_sN + (size_t)g * j.out_sG, 2u * T * 2 * NCOL);
      const bool sepg = g ? sep1 : sep0;
      f16x8 bh[TPI][NS], bo[TPI][NS];
      f16x4 th[TPI], to[TPI];
      float asv[TPI][4], al[TPI][4];
      int colb[TPI];
#pragma unroll
      for (int i = 0; i < TPI; ++i) {
        const int ct = ct0 + i;  // (past NCTC: padding columns, their stores dropped)
        const int col = ct * 16 + cl;
        const int qa = col / SL, pa = SM::slot_idx(col - qa * SL);
        const bool va = col < NCOL && pa < V;
        const int pb = EF::row(va ? pa : V), qb = EF::row(col < NCOL ? qa : V);
        if (sepg) tanh_frags<true, NS, TAIL>(El, Fl, pb, qb, kg, bh[i], bo[i], th[i], to[i]);
        else tanh_frags<false, NS, TAIL>(El, Fl, pb, qb, kg, bh[i], bo[i], th[i], to[i]);
        colb[i] = ct * 16 + 4 * kg;
        const int cb = min(colb[i], Gm::ASQ - 4);  // (padding tiles: any in-range table entry)
        const float4 as4 = ld4(as + cb), al4 = ld4(as + Gm::ASQ + cb);
        asv[i][0] = as4.x, asv[i][1] = as4.y, asv[i][2] = as4.z, asv[i][3] = as4.w;
        al[i][0] = al4.x, al[i][1] = al4.y, al[i][2] = al4.z, al[i][3] = al4.w;
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        f32x4 acc[TPI];
#pragma unroll
        for (int i = 0; i < TPI; ++i) acc[i] = zero4();
#pragma unroll
        for (int s = 0; s < NS; ++s) {
#pragma unroll
          for (int i = 0; i < TPI; ++i) acc[i] = mfma32(bh[i][s], wo[rt][s], acc[i]);
#pragma unroll
          for (int i = 0; i < TPI; ++i) acc[i] = mfma32(bo[i][s], wh[rt][s], acc[i]);
#pragma unroll
          for (int i = 0; i < TPI; ++i) acc[i] = mfma32(bh[i][s], wh[rt][s], acc[i]);
        }
        if constexpr (TAIL) {  // on accumulators of their own (dstd_hilo.h: mixed-shape MFMA chains)
          f32x4 tac[TPI];
#pragma unroll
          for (int i = 0; i < TPI; ++i) tac[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(th[i], wto[rt], zero4(), 0, 0, 0);
#pragma unroll
          for (int i = 0; i < TPI; ++i) tac[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(to[i], wth[rt], tac[i], 0, 0, 0);
#pragma unroll
          for (int i = 0; i < TPI; ++i) tac[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(th[i], wth[rt], tac[i], 0, 0, 0);
#pragma unroll
          for (int i = 0; i < TPI; ++i) acc[i] += tac[i];
        }
        const int t = 16 * rt + cl;
#pragma unroll
        for (int i = 0; i < TPI; ++i) {
          float vv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) vv[r] = fmaf(al[i][r], fmaf(acc[i][r], inv, b[rt]), asv[i][r]);
          uint2 hi, lo;
          split4(make_float4(vv[0], vv[1], vv[2], vv[3]), hi, lo);
          const uint32_t off = t < T && colb[i] < NCOL ? 2u * (uint32_t)(t * 2 * NCOL + colb[i]) : OOB;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, hi), ro, off, 0, DSTD_ADJ_ST_AUX);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, lo), ro, off + 2u * NCOL, 0, DSTD_ADJ_ST_AUX);
        }
      }
    }
  }
#ifdef DSTD_STAMPS
  TLH(2, 2)
  __builtin_amdgcn_s_waitcnt(0);
  TLH(2, 3)
#endif
}

// phase 3 of k_temporal_fused reuses the launch's LDS for the next block's
// spatial adjacency scratch: only where that fits
template <int T, int V>
constexpr bool tf_phase3() {
  return SAdjGeom<T, V>::LDS <= TFusedGeom<T, V, TEPI_ENC, 64>::LDS && SAdjGeom<T, V>::LDS <= TFusedGeom<T, V, TEPI_IN, 64>::LDS &&
         SAdjGeom<T, V>::LDS <= TFusedGeom<T, V, TEPI_RAW, 64>::LDS;
}

// waves per workgroup (one workgroup per CU): 8 = two per SIMD with the
// next-unit prefetch; 12 = three per SIMD without it (<= 168 VGPRs), which
// also runs a sample's 22 GC units in two rounds instead of three
// (H36M; CMU / 3DPW, whose joints run in two chunks, spill at 168 VGPRs and
// keep 8)
#ifndef DSTD_TF_NW_H36M
#define DSTD_TF_NW_H36M 12
#endif
template <int T, int V>
constexpr int tf_waves() { return T == 35 && V == 22 ? DSTD_TF_NW_H36M : 8; }

// The body of k_temporal_fused for sample n on the workgroup's dynamic LDS
// dsm (TFusedGeom::LDS bytes): the kernel below runs it once, k_block_fused
// after the sample's spatial GC.
// k_block_fused, before the barrier that ends the spatial GC: the part of
// chunk 0's phase-1 prologue that does not depend on the spatial GC's output
// -- E / F pads, the chunk's conv_rm rows, the Astat / alpha tables, the bias
// -- into the phase-1 scratch (past the planes region, where the spatial
// stage lives), each wave right after its last spatial unit.  The same values
// and places as tfused_body's own prologue writes.
template <int T, int V, int EPI, int C>
__device__ __forceinline__ void tfused_pre(const TemporalFusedArgs& fa, unsigned char* dsm) {
  using Gm = TFusedGeom<T, V, EPI, C>;
  using SM = typename Gm::SM;
  using EF = typename Gm::EF;
  constexpr int NS = Gm::NS, TAIL = Gm::TAIL, KP = Gm::KP, K = Gm::K, SL = Gm::SL, NCOL = Gm::NCOL;
  constexpr int RTC = Gm::RTC, WIMG = Gm::WIMG, NT = 64 * tf_waves<T, V>(), NFR = Gm::NFR;
  const AdjHLArgs& j = fa.j;
  float* El = reinterpret_cast<float*>(dsm + Gm::PLANES);
  float* Fl = El + Gm::EFE;
  uint4* wl = reinterpret_cast<uint4*>(Fl + Gm::EFF);
  float* asq = reinterpret_cast<float*>(wl + WIMG);
  float* alq = asq + Gm::ASQ;
  float* bsl = alq + Gm::ASQ;
  const int tid = threadIdx.x;
  constexpr int FULL = NS * 2 * 64;
  constexpr int NWF = cdiv(RTC * FULL, NT), NWT = TAIL ? cdiv(RTC * 64, NT) : 0, NAS = cdiv(Gm::ASQ, NT);
  uint4 wf[NWF], wt[NWT > 0 ? NWT : 1];
  float av[NAS];
  int aok = 0;
#pragma unroll
  for (int it = 0; it < NWF; ++it) wf[it] = j.wimg[0][min(tid + it * NT, RTC * FULL - 1)];
#pragma unroll
  for (int it = 0; it < NWT; ++it) wt[it] = j.wimg[0][Gm::RTG * FULL + min(tid + it * NT, RTC * 64 - 1)];
#pragma unroll
  for (int it = 0; it < NAS; ++it) {
    const int i = tid + it * NT, q = i / SL, pi = i < NCOL ? SM::slot_idx(i - q * SL) : T;
    const bool ok = pi < T && q < T;
    if (ok) aok |= 1 << it;
    av[it] = j.astat[0][ok ? pi * T + q : 0];
  }
  const float dna = pow2f(-hl_range_shift(fexp_bits(__float_as_uint(j.wscale[0][HLS_BOUND]))));
  const float alpha = *j.alpha * dna;
  const float bv = tid < 16 * RTC && tid < V ? j.bias[0][tid] : 0.f;
  for (int i = tid; i < (T + 1) * (KP - K); i += NT) {
    const int r = i / (KP > K ? KP - K : 1), k = K + i % (KP > K ? KP - K : 1);
    El[EF::row(r) + k] = 1.f;
    if (r < NFR) Fl[EF::row(r) + k] = 1.f;
  }
  for (int i = tid; i < K; i += NT) {
    El[EF::row(T) + i] = 1.f;
    Fl[EF::row(NFR - 1) + i] = 1.f;
  }
#pragma unroll
  for (int it = 0; it < NWF; ++it)
    if (tid + it * NT < RTC * FULL) wl[tid + it * NT] = wf[it];
#pragma unroll
  for (int it = 0; it < NWT; ++it)
    if (tid + it * NT < RTC * 64) wl[RTC * FULL + tid + it * NT] = wt[it];
#pragma unroll
  for (int it = 0; it < NAS; ++it)
    if (tid + it * NT < Gm::ASQ) {
      const bool ok = (aok >> it) & 1;
      asq[tid + it * NT] = ok ? av[it] * dna : 0.f;
      alq[tid + it * NT] = ok ? alpha : 0.f;
    }
  if (tid < 16 * RTC) bsl[tid] = bv;
}

// PRE (k_block_fused): chunk 0's phase-1 prologue is done already -- the E /
// F rows by the spatial units (pq_sink), the pads, conv_rm rows, tables and
// bias by tfused_pre before the workgroup barrier whose OR of the range flags
// is sep_pre -- so phase 1 starts with its tiles
template <int T, int V, int EPI, int C, bool PRE = false>
__device__ __forceinline__ void tfused_body(const TemporalFusedArgs& fa, const int n, unsigned char* dsm,
                                            const bool sep_pre = true) {
  using Gm = TFusedGeom<T, V, EPI, C>;
  using SM = typename Gm::SM;
  using EF = typename Gm::EF;
  constexpr int NS = Gm::NS, TAIL = Gm::TAIL, KP = Gm::KP, K = Gm::K, SL = Gm::SL, NCOL = Gm::NCOL;
  constexpr int RC = Gm::RC, RTC = Gm::RTC, PJ = Gm::PJ, WIMG = Gm::WIMG, NW = tf_waves<T, V>(), NT = 64 * NW;
  constexpr int UF = Gm::UF, NUTC = Gm::NUTC, NFR = Gm::NFR;  // frames / u tiles per chunk, F rows
  constexpr float C2 = 2.8853900817779268f;       // 2*log2(e)
  const TemporalHLArgs& a = fa.g;
  const AdjHLArgs& j = fa.j;
  _Float16* planes = reinterpret_cast<_Float16*>(dsm);
  unsigned char* un = dsm + Gm::PLANES;  // phase-1 scratch / phase-2 stage (union)
  float* El = reinterpret_cast<float*>(un);
  float* Fl = El + Gm::EFE;
  uint4* wl = reinterpret_cast<uint4*>(Fl + Gm::EFF);
  // plane column col = q * SL + slot (q the output frame, slot <-> input
  // frame pi = slot_idx(slot)): asq[col] = 2^-sa Astat[pi][q], alq[col] =
  // 2^-sa alpha -- both 0 on padding slots and past the planes
  float* asq = reinterpret_cast<float*>(wl + WIMG);
  float* alq = asq + Gm::ASQ;
  float* bsl = alq + Gm::ASQ;
  auto& st = *reinterpret_cast<TemporalStage<T, EPI, C, V>*>(un);

  // wave index through readfirstlane: wave-uniform to the compiler, so the
  // unit indices derived from it live in SGPRs (as tid >> 6 they took ~24
  // VGPRs more and spilled)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = lane >> 4, cl = lane & 15;
  if constexpr (C == 64) { TLH(3, 0) TLH(4, 0) }
#ifdef DSTD_SETPRIO_TF  // (experiment, r05o: waves 4-11 +0.6%, 8-11 neutral at H36M -- off)
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= DSTD_SETPRIO_TF) __builtin_amdgcn_s_setprio(1);
#endif

  {
    for (int ch = 0; ch < Gm::NCHUNK; ++ch) {
      // joint chunk jc (v0 .. v0 + nv - 1), u chunk uc (output frames u0 .. u0 + UF - 1)
      const int jc = ch % Gm::NJCH, uc = ch / Gm::NJCH;
      const int v0 = jc * RC, nv = min(RC, V - v0), rt0 = jc * RTC, u0 = uc * UF;
      if (ch) __syncthreads();  // the previous chunk's phase 2 is done with the planes and the stage
      // ---- phase 1 prologue: P/Q -> E/F rows, the chunk's conv_rm rows, Astat, bias ----
      const PQLayout L = j.pql;
      const float* pqb = j.pq + (size_t)n * L.sn + j.p_ch[0];
      // padding k and the pad rows (E: t = T, F: NFR - 1): E = F = 1 (tanh 0)
      auto ef_pad = [&](float val) __attribute__((always_inline)) {
        for (int i = tid; i < (T + 1) * (KP - K); i += NT) {
          const int r = i / (KP > K ? KP - K : 1), k = K + i % (KP > K ? KP - K : 1);
          El[EF::row(r) + k] = val;
          if (r < NFR) Fl[EF::row(r) + k] = val;
        }
        for (int i = tid; i < K; i += NT) {
          El[EF::row(T) + i] = val;
          Fl[EF::row(NFR - 1) + i] = val;
        }
      };
      const float inv = j.wscale[0][HLS_INV];
      bool sep;
      if (PRE && ch == 0) {
        // (the planes region held the spatial stage until the barrier: the pads now)
        if (tid < Gm::jn(RC)) *reinterpret_cast<uint4*>(planes + tid * PJ + Gm::ZPAD) = make_uint4(0u, 0u, 0u, 0u);
        sep = sep_pre;
      } else {
      ef_pad(1.f);
      // every global load of the prologue is issued before the first LDS
      // write that needs one (one memory round trip, not one per loop trip)
      constexpr int FULL = NS * 2 * 64;  // uint4 per row tile (full K-steps)
      constexpr int NPQ = cdiv(T * V, NT), NWF = cdiv(RTC * FULL, NT), NWT = TAIL ? cdiv(RTC * 64, NT) : 0;
      constexpr int NAS = cdiv(Gm::ASQ, NT);
      float4 q4[NPQ];
      uint4 wf[NWF], wt[NWT > 0 ? NWT : 1];
      float av[NAS];
      int aok = 0;  // bit it: the table entry of iteration it is a valid (pi, q)
      // (the P/Q and Astat loads do not depend on the chunk: an opaque zero
      // in their index keeps hipcc from hoisting them out of the chunk loop,
      // where they would stay live through phase 2 and spill)
      const int oz = Gm::NCHUNK > 1 ? opaque_zero() : 0;
#pragma unroll
      for (int it = 0; it < NPQ; ++it) {
        const int i = min(tid + it * NT + oz, T * V - 1);  // clamped: no branch around the load
        const int t = i / V, v = i - t * V;
        q4[it] = ld4(pqb + t * L.st + v * L.sv);  // (P_0, P_1, Q_0, Q_1)
      }
      {
        const uint4* wg = j.wimg[0];
#pragma unroll
        for (int it = 0; it < NWF; ++it) wf[it] = wg[rt0 * FULL + min(tid + it * NT, RTC * FULL - 1)];
#pragma unroll
        for (int it = 0; it < NWT; ++it) wt[it] = wg[Gm::RTG * FULL + rt0 * 64 + min(tid + it * NT, RTC * 64 - 1)];
      }
#pragma unroll
      for (int it = 0; it < NAS; ++it) {
        // column i of the chunk: output frame u0 + q, slot <-> input frame pi
        const int i = tid + it * NT + oz, q = i / SL, pi = i < NCOL ? SM::slot_idx(i - q * SL) : T;
        const bool ok = pi < T && u0 + q < T;
        if (ok) aok |= 1 << it;
        av[it] = j.astat[0][ok ? pi * T + u0 + q : 0];
      }
      // planes stored as 2^-sa Adj (dstd_hilo.h "range scaling")
      const float dna = pow2f(-hl_range_shift(fexp_bits(__float_as_uint(j.wscale[0][HLS_BOUND]))));
      const float alpha = *j.alpha * dna;
      const float bv = tid < 16 * RTC && 16 * rt0 + tid < V ? j.bias[0][16 * rt0 + tid] : 0.f;
      int bad = 0;
#pragma unroll
      for (int it = 0; it < NPQ; ++it) {
        const int i = tid + it * NT;
        if (i < T * V) {
          const int t = i / V, v = i - t * V;
          const float ep0 = C2 * q4[it].x, ep1 = C2 * q4[it].y, eq0 = -C2 * q4[it].z, eq1 = -C2 * q4[it].w;
          bad |= !(fabsf(ep0) <= 120.f && fabsf(ep1) <= 120.f && fabsf(eq0) <= 120.f && fabsf(eq1) <= 120.f);
          El[EF::row(t) + v] = __builtin_amdgcn_exp2f(ep0);
          El[EF::row(t) + V + v] = __builtin_amdgcn_exp2f(ep1);
          // (F rows: the chunk's output frames; the separable / direct choice
          // above still looks at every frame, as k_adj_hl<1> does)
          const int tq = t - u0;
          if (tq >= 0 && tq < UF) {
            Fl[EF::row(tq) + v] = __builtin_amdgcn_exp2f(eq0);
            Fl[EF::row(tq) + V + v] = __builtin_amdgcn_exp2f(eq1);
          }
        }
      }
#pragma unroll
      for (int it = 0; it < NWF; ++it)
        if (tid + it * NT < RTC * FULL) wl[tid + it * NT] = wf[it];
#pragma unroll
      for (int it = 0; it < NWT; ++it)
        if (tid + it * NT < RTC * 64) wl[RTC * FULL + tid + it * NT] = wt[it];
#pragma unroll
      for (int it = 0; it < NAS; ++it)
        if (tid + it * NT < Gm::ASQ) {
          const bool ok = (aok >> it) & 1;
          asq[tid + it * NT] = ok ? av[it] * dna : 0.f;
          alq[tid + it * NT] = ok ? alpha : 0.f;
        }
      if (tid < 16 * RTC) bsl[tid] = bv;
      if (tid < Gm::jn(RC)) *reinterpret_cast<uint4*>(planes + tid * PJ + Gm::ZPAD) = make_uint4(0u, 0u, 0u, 0u);
      sep = __syncthreads_or(bad) == 0;
      // (__syncthreads_or already orders the LDS writes above: __ockl_wgred_or_i32
      // waits lgkmcnt(0) before its first barrier, checked in the ISA; round
      // 2's "did not order" was the mixed-shape MFMA hazard)
      __syncthreads();
      }  // (!PRE || ch)
      if (!sep) {  // direct path: E / F hold P / Q themselves (padding 0)
        for (int i = tid; i < T * V; i += NT) {
          const int t = i / V, v = i % V;
          const float4 q4 = ld4(pqb + t * L.st + v * L.sv);
          El[EF::row(t) + v] = q4.x;
          El[EF::row(t) + V + v] = q4.y;
          const int tq = t - u0;
          if (tq >= 0 && tq < UF) {
            Fl[EF::row(tq) + v] = q4.z;
            Fl[EF::row(tq) + V + v] = q4.w;
          }
        }
        ef_pad(0.f);
        __syncthreads();
      }
      if constexpr (C == 64) {
        if (ch == 0) { TLH(4, 1) }
      }
      // ---- phase 1: the chunk's planes ----
      // The GEMM runs transposed -- the tanh fragments as the A operand,
      // W_rm as B (the same register layouts) -- so a lane's accumulator holds
      // 4 consecutive slots (columns 16 ct + 4 kg + r) of one joint (16 rt +
      // cl): one 8-byte LDS write per plane instead of eight 2-byte ones.
      // (Round 2 saw wrong planes with the W fragments held in registers
      // across tiles.  Cause, found in round 3: hipcc had scheduled a
      // 16x16x16 tail MFMA right behind a 16x16x32 one on the same
      // accumulator -- dstd_hilo.h, mixed-shape MFMA chains.  With the tail on its
      // own accumulator, TPI 1/2 and HOISTW 0/1 are all bit-exact.)
#ifndef DSTD_TF_TPI
#define DSTD_TF_TPI 1
#endif
#ifndef DSTD_TF_HOISTW
#define DSTD_TF_HOISTW 1  // (A/B r03a: -1..2% per launch at H36M / 3DPW, tie at CMU)
#endif
      constexpr int TPI = DSTD_TF_TPI;  // column tiles per iteration (independent chains)
      // (u chunks: the W fragments re-read per tile -- hoisted, their 24
      // registers are live through the whole chunk loop and phase 2 spills)
      constexpr bool HW = DSTD_TF_HOISTW && !Gm::UCH;
      // W_rm fragments of the chunk's row tiles (HOISTW: read once, held across tiles)
      f16x8 wfh[HW ? RTC : 1][NS], wfo[HW ? RTC : 1][NS];
      f16x4 wth[HW ? RTC : 1], wto[HW ? RTC : 1];
      auto load_w = [&](int rt, f16x8 (&h)[NS], f16x8 (&o)[NS], f16x4& th4, f16x4& to4) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          h[s] = as_h8(wl[((rt * NS + s) * 2 + 0) * 64 + lane]);
          o[s] = as_h8(wl[((rt * NS + s) * 2 + 1) * 64 + lane]);
        }
        if constexpr (TAIL) {
          const uint2* w16 = reinterpret_cast<const uint2*>(wl + RTC * NS * 2 * 64);
          th4 = __builtin_bit_cast(f16x4, w16[(rt * 2 + 0) * 64 + lane]);
          to4 = __builtin_bit_cast(f16x4, w16[(rt * 2 + 1) * 64 + lane]);
        }
      };
      if constexpr (HW) {
#pragma unroll
        for (int rt = 0; rt < RTC; ++rt) load_w(rt, wfh[rt], wfo[rt], wth[rt], wto[rt]);
      }
      auto tiles = [&](auto sep_c) {
        constexpr bool SEP = decltype(sep_c)::value;
        for (int ct0 = wave; ct0 < Gm::NCTC; ct0 += TPI * NW) {
          // TPI column tiles ct0, ct0 + NW, ...; a tile past the planes
          // computes padding (its stores are dropped)
          f16x8 bh[TPI][NS], bo[TPI][NS];
          f16x4 th[TPI], to[TPI];
          float4 as[TPI], al[TPI];
          int colb[TPI], q[TPI], slot0[TPI];
#pragma unroll
          for (int i = 0; i < TPI; ++i) {
            const int ct = ct0 + i * NW;
            // this lane's A-operand row = column ct * 16 + cl of the planes
            const int col = ct * 16 + cl;
            const int qa = col / SL, pa = SM::slot_idx(col - qa * SL);
            const bool va = col < NCOL && pa < T;
            const bool vq = col < NCOL && u0 + qa < T;  // (F rows are chunk-local)
            tanh_frags<SEP, NS, TAIL>(El, Fl, EF::row(va ? pa : T), EF::row(vq ? qa : NFR - 1), kg, bh[i], bo[i], th[i],
                                      to[i]);
            // columns colb .. colb+3 (one frame q, slots slot0 ..): alpha (acc + b) + Astat,
            // 0 on padding slots (both tables hold 0 there)
            colb[i] = ct * 16 + 4 * kg;
            q[i] = colb[i] / SL;
            slot0[i] = colb[i] - q[i] * SL;
            as[i] = ld4(asq + colb[i]);
            al[i] = ld4(alq + colb[i]);
          }
#pragma unroll
          for (int rt = 0; rt < RTC; ++rt) {
            f16x8 wh_[NS], wo_[NS];
            f16x4 wth_, wto_;
            if constexpr (HW) {
#pragma unroll
              for (int s = 0; s < NS; ++s) {
                wh_[s] = wfh[rt][s];
                wo_[s] = wfo[rt][s];
              }
              wth_ = wth[rt];
              wto_ = wto[rt];
            } else {
              load_w(rt, wh_, wo_, wth_, wto_);
            }
            f32x4 acc[TPI];
#pragma unroll
            for (int i = 0; i < TPI; ++i) acc[i] = zero4();
#pragma unroll
            for (int s = 0; s < NS; ++s) {
#pragma unroll
              for (int i = 0; i < TPI; ++i) acc[i] = mfma32(bh[i][s], wo_[s], acc[i]);
#pragma unroll
              for (int i = 0; i < TPI; ++i) acc[i] = mfma32(bo[i][s], wh_[s], acc[i]);
#pragma unroll
              for (int i = 0; i < TPI; ++i) acc[i] = mfma32(bh[i][s], wh_[s], acc[i]);
            }
            if constexpr (TAIL) {  // on an accumulator of its own (dstd_hilo.h: mixed-shape MFMA chains)
              f32x4 tac[TPI];
#pragma unroll
              for (int i = 0; i < TPI; ++i) tac[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(th[i], wto_, zero4(), 0, 0, 0);
#pragma unroll
              for (int i = 0; i < TPI; ++i) tac[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(to[i], wth_, tac[i], 0, 0, 0);
#pragma unroll
              for (int i = 0; i < TPI; ++i) tac[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(th[i], wth_, tac[i], 0, 0, 0);
#pragma unroll
              for (int i = 0; i < TPI; ++i) acc[i] += tac[i];
            }
            const float b = bsl[16 * rt + cl];
            const int jv = 16 * rt + cl;
#pragma unroll
            for (int i = 0; i < TPI; ++i) {
              const float4 vv = make_float4(fmaf(al[i].x, fmaf(acc[i][0], inv, b), as[i].x),
                                            fmaf(al[i].y, fmaf(acc[i][1], inv, b), as[i].y),
                                            fmaf(al[i].z, fmaf(acc[i][2], inv, b), as[i].z),
                                            fmaf(al[i].w, fmaf(acc[i][3], inv, b), as[i].w));
              uint2 hi, lo;
              split4(vv, hi, lo);
#ifdef DSTD_TF_ST128  // (off: 0.7-1.1% slower forward, profiles/r05h_lds_layout_ab.txt)
              // lanes kg and kg ^ 1 hold the 8 consecutive slots 8 (kg >> 1) ..
              // + 7 of one joint: v_permlane16_swap trades the even row's lo
              // quad for the odd row's hi quad, so the even lane stores the hi
              // plane's 16 bytes and the odd lane the lo plane's -- one
              // ds_write_b128 per lane (8-lane groups over 32 banks: the joint
              // stride PJ puts 8 joints on 8 distinct bank quads) instead of two
              // ds_write_b64 whose 16-lane groups can reach only 16 of the 32
              // banks from 16-byte-aligned rows (2-way)
              const auto sx = __builtin_amdgcn_permlane16_swap(hi.x, lo.x, false, false);
              const auto sy = __builtin_amdgcn_permlane16_swap(hi.y, lo.y, false, false);
              const bool odd = kg & 1;
              const uint4 w4 = odd ? make_uint4(sx[0], sy[0], lo.x, lo.y) : make_uint4(hi.x, hi.y, sx[1], sy[1]);
              if (jv < nv && colb[i] < NCOL) {
                _Float16* dst = planes + jv * PJ + q[i] * SL + slot0[i] - (odd ? 4 : 0) + (odd ? UF * SL : 0);
                *reinterpret_cast<uint4*>(dst) = w4;
              }
#else  // two 8-byte stores per lane (2-way bank conflicted, cheaper in VALU)
              if (jv < nv && colb[i] < NCOL) {
                _Float16* dst = planes + jv * PJ + q[i] * SL + slot0[i];
                *reinterpret_cast<uint2*>(dst) = hi;
                *reinterpret_cast<uint2*>(dst + UF * SL) = lo;
              }
#endif
            }
          }
        }
      };
#ifndef DSTD_TF_SKIP_P1  // (timing experiments: phase 2 alone)
      if (sep) tiles(std::true_type{});
      else tiles(std::false_type{});
#endif
#if defined(DSTD_TF_DEBUGW) && DSTD_TF_HOISTW
      // (bisection build: the hoisted W registers after the tile loop against
      // a fresh read of the same LDS words, workgroup 0, every lane)
      if (blockIdx.x == 0 && ch == 0) {
#pragma unroll
        for (int rt = 0; rt < RTC; ++rt) {
          f16x8 h2[NS], o2[NS];
          f16x4 th2, to2;
          load_w(rt, h2, o2, th2, to2);
          const uint4 a0 = __builtin_bit_cast(uint4, wfh[rt][0]), a1 = __builtin_bit_cast(uint4, wfo[rt][0]);
          const uint4 b0 = __builtin_bit_cast(uint4, h2[0]), b1 = __builtin_bit_cast(uint4, o2[0]);
          const uint2 a2 = __builtin_bit_cast(uint2, wth[rt]), a3 = __builtin_bit_cast(uint2, wto[rt]);
          const uint2 b2 = __builtin_bit_cast(uint2, th2), b3 = __builtin_bit_cast(uint2, to2);
          unsigned* d = g_dbg_w + ((rt * NT + tid) * 24);
          const unsigned v[24] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w, a2.x, a2.y, a3.x, a3.y,
                                  b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w, b2.x, b2.y, b3.x, b3.y};
          for (int i = 0; i < 24; ++i) d[i] = v[i];
        }
      }
#endif
      if constexpr (C == 64) {
        if (ch == 0) { TLH(4, 2) }
      }
      // the phase-2 stage's loads now, its LDS writes after the barrier
      // (-DDSTD_TF_STAGE_EARLY=0: both after it, as before round 6)
      TemporalStageLoad<T, EPI, C, V, NT> stl;
      if constexpr (DSTD_TF_STAGE_EARLY) stl.load(a, tid, Gm::NCHUNK > 1 ? opaque_zero() : 0);
      __syncthreads();  // planes complete; the phase-1 scratch is free
      if constexpr (!DSTD_TF_STAGE_EARLY) stl.load(a, tid, Gm::NCHUNK > 1 ? opaque_zero() : 0);
      if constexpr (C == 64) {
        if (ch == 0) { TLH(3, 1) }
      }
#ifdef DSTD_TF_DUMPP
      // (bisection build: workgroup 0's planes of chunk 0 to g_dbg_planes)
      if (blockIdx.x == 0 && ch == 0) {
        const unsigned* src = reinterpret_cast<const unsigned*>(planes);
        for (int i = tid; i < (int)(Gm::PLANES / 4) && i < 64 * 1024; i += NT) g_dbg_planes[i] = src[i];
      }
#endif
      // ---- phase 2: the stage, then the chunk's GC units ----
      stl.store(a, st, tid);
      __syncthreads();
      if constexpr (C == 64) {
        if (ch == 0) { TLH(4, 3) }
      }
      const int ub = n * V + v0;
      // (a lane outside the planes -- frame past T, slot group past ng(s) --
      // reads the joint block's zeroed 16-byte pad instead: no exec-masked
      // read, no select)
      auto load_adj = [&](int u, int s, uint4 (&bh)[NUTC], uint4 (&bo)[NUTC]) {
        const _Float16* base = planes + (u - ub) * PJ;
        // (the offsets are lane constants: recomputed per call from an opaque
        // lane index instead of 12 registers held through the unit loop)
        const int clz = cl + opaque_zero();
#pragma unroll
        for (int ut = 0; ut < NUTC; ++ut) {
          const int uo = 16 * ut + clz;  // chunk-local output frame
          const bool ok = u0 + uo < T && uo < UF && kg < SM::ng(s);
          const int off = uo * SL + 8 * (SM::goff(s) + kg);
          bh[ut] = *reinterpret_cast<const uint4*>(base + (ok ? off : Gm::ZPAD));
          bo[ut] = *reinterpret_cast<const uint4*>(base + (ok ? UF * SL + off : Gm::ZPAD));
        }
      };
#ifndef DSTD_TF_P2PRIO  // (experiments: the younger waves' static priority in the joint units)
#define DSTD_TF_P2PRIO 0
#endif
      if constexpr (DSTD_TF_P2PRIO) { if (wave >= 4) __builtin_amdgcn_s_setprio(1); }
#ifndef DSTD_TF_SKIP_P2  // (timing experiments: phase 1 alone)
      temporal_units<T, EPI, C, V, true, decltype(load_adj), (NW <= 8 && !Gm::UCH), tf_res_acc(T, V), NUTC>(
          a, st, ub + wave, ub + nv, NW, load_adj, u0 / 16);
#endif
      if constexpr (DSTD_TF_P2PRIO) __builtin_amdgcn_s_setprio(0);
    }
  }
  // ---- phase 3: the next block's spatial adjacency planes of this sample
  // (where its scratch fits the launch's LDS: not at T = 75) ----
  if constexpr (C == 64 && tf_phase3<T, V>()) {
    TLH(3, 2)
    if (fa.sn.out) {
#ifndef DSTD_P3_PRELOAD  // (1: the static loads before the barrier -- r06q: 0.0% / -0.1% / +1.7%, off)
#define DSTD_P3_PRELOAD 0
#endif
      SAdjStatic<T, V, NT> p3s;
      if constexpr (DSTD_P3_PRELOAD) p3s.load(fa.sn, tid);
      __syncthreads();  // every unit's P/Q written (one CU: the workgroup-scope fences of the barrier suffice)
      TLH(2, 0)
#ifndef DSTD_TF_P3PRIO  // (experiments: the same in phase 3)
#define DSTD_TF_P3PRIO 0
#endif
      if constexpr (DSTD_TF_P3PRIO) { if (wave >= 4) __builtin_amdgcn_s_setprio(1); }
      spatial_adj_sample<T, V, NT>(fa.sn, n, dsm, DSTD_P3_PRELOAD ? &p3s : nullptr);
      if constexpr (DSTD_TF_P3PRIO) __builtin_amdgcn_s_setprio(0);
    }
    TLH(3, 3)
  }
}

template <int T, int V, int EPI, int C>
__global__ __launch_bounds__((64 * tf_waves<T, V>())) __attribute__((amdgpu_waves_per_eu((tf_waves<T, V>() / 4), (tf_waves<T, V>() / 4)))) void k_temporal_fused(TemporalFusedArgs fa) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  tfused_body<T, V, EPI, C>(fa, blockIdx.x, dsm);  // one sample per workgroup
}

// ===========================================================================
// One whole DSTDGCB per sample (model/dstdgcn.py:141-163): the workgroup of
// k_temporal_fused first runs the sample's spatial GC units (the T (sample,
// frame) units of k_spatial_hl, its waves striding the frames), then, after a
// barrier, the fused temporal GC of the same sample (tfused_body: temporal
// adjacency in LDS, the joint units, the next block's spatial planes).  h and
// the temporal P/Q of the sample pass between the phases through the CU's own
// L1 / L2 (same workgroup: the barrier's workgroup-scope fence orders them, as
// phase 3's P/Q reads); the spatial launch, its kernel boundary and its
// grid-wide unit imbalance (T B units over the chip's waves) are gone.
// ===========================================================================
template <int T, int V, int CIN, int COUT, int EPI>
struct BlockFusedGeom {
  static constexpr size_t SP = sizeof(SpatialStage<V, CIN, COUT>);
  static constexpr size_t TF = TFusedGeom<T, V, EPI, COUT>::LDS;
  static constexpr size_t LDS = SP > TF ? SP : TF;
  static_assert(LDS <= kLdsBudget, "LDS");
};

template <int T, int V, int CIN, int COUT, int EPI>
__device__ __forceinline__ void block_fused_body(const SpatialHLArgs& sa, const TemporalFusedArgs& ta, const AdjHLArgs& s0,
                                                 const int n, unsigned char* dsm) {
  constexpr int NW = tf_waves<T, V>(), NT = 64 * NW;
  if constexpr (CIN == 64 && COUT == 64) { TLH(5, 0) }
  if constexpr (CIN == 6 && tf_phase3<T, V>()) {
    // conv_st_in: this block's own spatial planes from the model input (the
    // k_adj_hl<0> launch of block 0), stored to HBM like phase 3's and read
    // back by the units below on this CU; every wave's plane stores complete
    // before the barrier (vmcnt 0), the units' loads come after it
    if (s0.out) {
      spatial_adj_sample<T, V, NT, true>(s0, n, dsm);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
  }
  int bad = 0;
  {
    using SM = SlotMap<V, true>;
    constexpr int SL = SM::SL, NG = SM::NG, NWT = cdiv(V, 16);
    auto& st = *reinterpret_cast<SpatialStage<V, CIN, COUT>*>(dsm);
    static_assert(sizeof(SpatialStage<V, CIN, COUT>) <= TFusedGeom<T, V, EPI, COUT>::PLANES,
                  "the spatial stage must lie within the planes region (tfused_pre writes past it)");
    stage_spatial<V, CIN, COUT, NT>(sa, st, threadIdx.x);
    __syncthreads();
    const int lane = threadIdx.x & 63, kl = lane >> 4, cl = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const SpatialHLArgs& a = sa;
    constexpr uint32_t adj_bytes = 2 * V * SL * 2;  // one (n, g, t) adjacency: 2 planes of V x SL halves
    const uint32_t wadj0 = kl < NG ? (uint32_t)(cl * SL + 8 * kl) * 2 : OOB;
    auto load_adj_g = [&](int uu, int g, uint4 (&ab)[NWT][2]) {
      const int t = uu - n * T;
      const uint16_t* base = a.adj + ((size_t)(n * 2 + g) * T + t) * (adj_bytes / 2);
      const auto rh = rsrc(base, adj_bytes / 2), rl = rsrc(base + V * SL, adj_bytes / 2);
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) {
        ab[wt][0] = bldu4(rh, wadj0 + wt * 32 * SL);
        ab[wt][1] = bldu4(rl, wadj0 + wt * 32 * SL);
      }
    };
    // (three waves per SIMD: the identity residual loaded after the
    // aggregations, as DSTD_HL_WPE=3 builds of k_spatial_hl do, or it spills)
    // (h and the temporal P/Q: DSTD_BF_ST_AUX, the cache policy of their
    // stores -- the same CU reads them back right after the barrier)
#ifndef DSTD_BF_ST_AUX
#define DSTD_BF_ST_AUX DSTD_GC_ST_AUX
#endif
    // every unit also writes its frame's E / F rows of phase 1 (the tanh
    // GEMM's exp2 of its temporal P / Q -- the values it stores, the same
    // float operations as phase 1's prologue) straight into the phase-1
    // scratch, which lies past the planes region and so past the stage
    using TG = TFusedGeom<T, V, EPI, COUT>;
    using TEF = typename TG::EF;
    float* El = reinterpret_cast<float*>(dsm + TG::PLANES);
    float* Fl = El + TG::EFE;
    auto pq_sink = [&](int uu, int w, float p0, float p1, float q0, float q1) -> int {
      constexpr float C2 = 2.8853900817779268f;  // 2*log2(e)
      const int t = uu - n * T;
      const float ep0 = C2 * p0, ep1 = C2 * p1, eq0 = -C2 * q0, eq1 = -C2 * q1;
      El[TEF::row(t) + w] = __builtin_amdgcn_exp2f(ep0);
      El[TEF::row(t) + V + w] = __builtin_amdgcn_exp2f(ep1);
      Fl[TEF::row(t) + w] = __builtin_amdgcn_exp2f(eq0);
      Fl[TEF::row(t) + V + w] = __builtin_amdgcn_exp2f(eq1);
      return !(fabsf(ep0) <= 120.f && fabsf(ep1) <= 120.f && fabsf(eq0) <= 120.f && fabsf(eq1) <= 120.f);
    };
    // (experiments: static VALU priority for the younger waves during the
    // spatial units -- 1: waves 4-11 at 1, 2: 4-7 at 1 and 8-11 at 2, 3:
    // 8-11 at 1; back to 0 for the temporal phases)
#ifndef DSTD_BF_SETPRIO
#define DSTD_BF_SETPRIO 1
#endif
    if constexpr (DSTD_BF_SETPRIO == 1) { if (wave >= 4) __builtin_amdgcn_s_setprio(1); }
    if constexpr (DSTD_BF_SETPRIO == 2) {
      if (wave >= 8) __builtin_amdgcn_s_setprio(2);
      else if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    if constexpr (DSTD_BF_SETPRIO == 3) { if (wave >= 8) __builtin_amdgcn_s_setprio(1); }
    bad = spatial_units<V, CIN, COUT, decltype(load_adj_g), (NW > 8), DSTD_BF_ST_AUX, decltype(pq_sink)>(
        a, st, n * T + wave, (n + 1) * T, NW, load_adj_g, pq_sink);
    if constexpr (DSTD_BF_SETPRIO != 0) __builtin_amdgcn_s_setprio(0);
  }
  if constexpr (CIN == 64 && COUT == 64) { TLH(5, 1) }
  tfused_pre<T, V, EPI, COUT>(ta, dsm);
  // h and the temporal P/Q of sample n written, chunk 0's E / F rows and
  // tables in LDS, the range flags OR-ed; the spatial stage is dead
  const bool sep = __syncthreads_or(bad) == 0;
  if constexpr (CIN == 64 && COUT == 64) { TLH(5, 2) }
  tfused_body<T, V, EPI, COUT, true>(ta, n, dsm, sep);
  if constexpr (CIN == 64 && COUT == 64) { TLH(5, 3) }
}

template <int T, int V, int CIN, int COUT, int EPI>
__global__ __launch_bounds__((64 * tf_waves<T, V>())) __attribute__((amdgpu_waves_per_eu((tf_waves<T, V>() / 4), (tf_waves<T, V>() / 4)))) void k_block_fused(BlockFusedArgs ba) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  block_fused_body<T, V, CIN, COUT, EPI>(ba.s, ba.t, ba.s0, blockIdx.x, dsm);  // one sample per workgroup
}

// ===========================================================================
// dispatch
// ===========================================================================
namespace {

int hl_num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

template <typename K>
int hl_occupancy(K k, int nt) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k, nt, 0) != hipSuccess || nb < 1) nb = 1;
  (void)hipGetLastError();
  return nb;
}

template <auto K, int NT, typename A>
hipError_t launch_units(int units, const A& a, hipStream_t s) {
  static const int occ = hl_occupancy(K, NT);  // one per kernel instantiation
  int grid = hl_num_cus() * occ;
  grid = min(grid, cdiv(units, NT / 64));
  hipLaunchKernelGGL(K, dim3(grid), dim3(NT), 0, s, a);
  return hipGetLastError();
}

template <int T>
hipError_t temporal_hl_t(const TemporalHLArgs& a, hipStream_t s) {
  if (a.C == 3) {
    if (a.pq) return hipErrorNotSupported;
    switch (a.epi) {
      case TEPI_OUT: return launch_units<k_temporal_hl<T, TEPI_OUT, 3>, temporal_nt<T, 3>()>(a.B * a.V, a, s);
      case TEPI_RAW: return launch_units<k_temporal_hl<T, TEPI_RAW, 3>, temporal_nt<T, 3>()>(a.B * a.V, a, s);
      default: return hipErrorNotSupported;
    }
  }
  if (a.C != 64) return hipErrorNotSupported;
  switch (a.epi) {
    case TEPI_ENC:
      if constexpr (tf_res_acc(T, 25)) {
        if (a.V == 25) return launch_units<k_temporal_hl<T, TEPI_ENC, 64, true>, temporal_nt<T, 64>()>(a.B * a.V, a, s);
      }
      if constexpr (tf_res_acc(T, 23)) {
        if (a.V == 23) return launch_units<k_temporal_hl<T, TEPI_ENC, 64, true>, temporal_nt<T, 64>()>(a.B * a.V, a, s);
      }
      return launch_units<k_temporal_hl<T, TEPI_ENC, 64>, temporal_nt<T, 64>()>(a.B * a.V, a, s);
    case TEPI_IN: return launch_units<k_temporal_hl<T, TEPI_IN, 64>, temporal_nt<T, 64>()>(a.B * a.V, a, s);
    case TEPI_RAW: return launch_units<k_temporal_hl<T, TEPI_RAW, 64>, temporal_nt<T, 64>()>(a.B * a.V, a, s);
    default: return hipErrorNotSupported;
  }
}

}  // namespace

int hl_device_cus() { return hl_num_cus(); }

hipError_t launch_hl_prep(const HLPrepArgs& a, hipStream_t s) {
  if (a.njobs <= 0) return hipSuccess;
  if (a.njobs > kMaxHLJobs) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_hl_prep, dim3(a.njobs), dim3(256), 0, s, a);
  return hipGetLastError();
}

// the shapes whose adjacency kernels (dstd_adj.hip) have a split-f16 writer
static bool hl_shape(int T, int V) {
  return (T == 35 && (V == 22 || V == 25)) || (T == 40 && V == 23) || (T == 75 && V == 22);
}
bool spatial_hl_supported(int T, int V) { return hl_shape(T, V); }

template <int MODE, int NROW, int K, int NA>
hipError_t adj_hl_run(const AdjHLArgs& a, hipStream_t s) {
  using Gm = AdjHLGeom<MODE, NROW, K, NA>;
  AdjHLArgs b = a;
  if (b.nchunk <= 0) {
    // below one workgroup per CU (small batches) split each (sample, graph)'s
    // column tiles over more workgroups -- each repeats the prologue, but the
    // launch is its prologue plus 1/nch of the tiles -- keeping at least half
    // the waves of a workgroup busy
#ifndef DSTD_ADJ_CHUNK_PCT  // (experiments: workgroups aimed at, % of the CUs / the busy-wave floor's divisor)
#define DSTD_ADJ_CHUNK_PCT 100
#define DSTD_ADJ_CHUNK_DIV 2
#endif
    const int sets = a.B * a.ngroups, cus = hl_num_cus();
    b.nchunk = Gm::NCHUNK;
    if (sets * Gm::NCHUNK < cus)
      b.nchunk = max(Gm::NCHUNK, min(cdiv(DSTD_ADJ_CHUNK_PCT * cus, 100 * sets), cdiv(Gm::NCT, cdiv(Gm::AW, DSTD_ADJ_CHUNK_DIV))));
  }
  const int grid = a.B * a.ngroups * b.nchunk;
  hipLaunchKernelGGL((k_adj_hl<MODE, NROW, K, NA>), dim3(grid), dim3(Gm::AT), 0, s, b);
  return hipGetLastError();
}

hipError_t launch_adj_hl(const AdjHLArgs& a, int mode, int T, int V, hipStream_t s) {
  if (a.pql.sch != 1 || ((uintptr_t)a.pq & 15) || (a.pql.st & 3) || (a.pql.sv & 3) || (a.pql.sn & 3))
    return hipErrorNotSupported;
  for (int g = 0; g < a.ngroups; ++g)
    if (a.p_ch[g] & 3) return hipErrorNotSupported;
  if (mode == 0) {
    if (T == 35 && V == 22) return adj_hl_run<0, 35, 70, 22>(a, s);
    if (T == 35 && V == 25) return adj_hl_run<0, 35, 70, 25>(a, s);
    if (T == 40 && V == 23) return adj_hl_run<0, 40, 80, 23>(a, s);
    if (T == 75 && V == 22) return adj_hl_run<0, 75, 150, 22>(a, s);
  } else {
    if (T == 35 && V == 22) return adj_hl_run<1, 22, 44, 35>(a, s);
    if (T == 35 && V == 25) return adj_hl_run<1, 25, 50, 35>(a, s);
    if (T == 40 && V == 23) return adj_hl_run<1, 23, 46, 40>(a, s);
    if (T == 75 && V == 22) return adj_hl_run<1, 22, 44, 75>(a, s);
  }
  return hipErrorNotSupported;
}
bool temporal_hl_supported(int T, int V) { return hl_shape(T, V); }

template <int V>
hipError_t spatial_hl_v(const SpatialHLArgs& a, hipStream_t s) {
  if (a.Cin == 64 && a.Cout == 64) return launch_units<k_spatial_hl<V, 64, 64>, spatial_nt()>(a.B * a.T, a, s);
  if (a.Cin == 6 && a.Cout == 64) return launch_units<k_spatial_hl<V, 6, 64>, spatial_nt()>(a.B * a.T, a, s);
  if (a.Cin == 64 && a.Cout == 3) return launch_units<k_spatial_hl<V, 64, 3>, spatial_nt()>(a.B * a.T, a, s);
  return hipErrorNotSupported;
}

hipError_t launch_spatial_hl(const SpatialHLArgs& a, hipStream_t s) {
  if (!spatial_hl_supported(a.T, a.V)) return hipErrorNotSupported;
  switch (a.V) {
    case 22: return spatial_hl_v<22>(a, s);
    case 23: return spatial_hl_v<23>(a, s);
    case 25: return spatial_hl_v<25>(a, s);
    default: return hipErrorNotSupported;
  }
}

template <int T, int V, int EPI, int C>
hipError_t tfused_run(const TemporalFusedArgs& a, hipStream_t s) {
  using Gm = TFusedGeom<T, V, EPI, C>;
  static const hipError_t attr = hipFuncSetAttribute((const void*)k_temporal_fused<T, V, EPI, C>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)Gm::LDS);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_temporal_fused<T, V, EPI, C>), dim3(a.g.B), dim3(64 * tf_waves<T, V>()), Gm::LDS, s, a);
  return hipGetLastError();
}

template <int T, int V>
hipError_t tfused_tv(const TemporalFusedArgs& a, hipStream_t s) {
  if (a.g.C == 3) {
    if (a.g.pq) return hipErrorNotSupported;
    switch (a.g.epi) {
      case TEPI_OUT: return tfused_run<T, V, TEPI_OUT, 3>(a, s);
      case TEPI_RAW: return tfused_run<T, V, TEPI_RAW, 3>(a, s);
      default: return hipErrorNotSupported;
    }
  }
  if (a.g.C != 64) return hipErrorNotSupported;
  switch (a.g.epi) {
    case TEPI_ENC: return tfused_run<T, V, TEPI_ENC, 64>(a, s);
    case TEPI_IN: return tfused_run<T, V, TEPI_IN, 64>(a, s);
    case TEPI_RAW: return tfused_run<T, V, TEPI_RAW, 64>(a, s);
    default: return hipErrorNotSupported;
  }
}

template <int T, int V, int CIN, int COUT, int EPI>
hipError_t bfused_run(const BlockFusedArgs& a, hipStream_t s) {
  using Gm = BlockFusedGeom<T, V, CIN, COUT, EPI>;
  static const hipError_t attr = hipFuncSetAttribute((const void*)k_block_fused<T, V, CIN, COUT, EPI>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)Gm::LDS);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_block_fused<T, V, CIN, COUT, EPI>), dim3(a.t.g.B), dim3(64 * tf_waves<T, V>()), Gm::LDS, s, a);
  return hipGetLastError();
}

// the model's three block kinds: conv_st_in (6 -> 64, IN tail), encoders
// (64 -> 64, ENC tail), conv_st_out (64 -> 3, OUT tail)
template <int T, int V>
hipError_t bfused_tv(const BlockFusedArgs& a, hipStream_t s) {
  const int cin = a.s.Cin, cout = a.s.Cout, epi = a.t.g.epi;
  if (cin == 64 && cout == 64 && epi == TEPI_ENC) return bfused_run<T, V, 64, 64, TEPI_ENC>(a, s);
  if (cin == 6 && cout == 64 && epi == TEPI_IN) return bfused_run<T, V, 6, 64, TEPI_IN>(a, s);
  if (cin == 64 && cout == 3 && epi == TEPI_OUT) return bfused_run<T, V, 64, 3, TEPI_OUT>(a, s);
  return hipErrorNotSupported;
}

bool block_fused_supported(int T, int V, int cin, int cout, int epi) {
#ifdef DSTD_NO_BFUSED
  return false;
#endif
  const bool shape = (T == 35 && (V == 22 || V == 25)) || (T == 40 && V == 23);
  return shape && ((cin == 64 && cout == 64 && epi == TEPI_ENC) || (cin == 6 && cout == 64 && epi == TEPI_IN) ||
                   (cin == 64 && cout == 3 && epi == TEPI_OUT));
}

bool block_fused_adj0_supported(int T, int V) {
#ifdef DSTD_NO_BF_ADJ0
  return false;
#endif
  return block_fused_supported(T, V, 6, 64, TEPI_IN) && temporal_fused_phase3(T, V);
}

hipError_t block_fused_args(const SpatialHLArgs& sa, const TemporalHLArgs& g, const AdjHLArgs& j, const AdjHLArgs* sn,
                            BlockFusedArgs* out, const AdjHLArgs* s0) {
  if (!block_fused_supported(g.T, g.V, sa.Cin, sa.Cout, g.epi) || sa.T != g.T || sa.V != g.V || sa.B != g.B ||
      sa.Cout != g.C || sa.y != g.h || sa.pq != j.pq || g.V != (int)(j.pql.st / 4) || j.pql.sch != 1 || j.pql.sv != 4 ||
      ((uintptr_t)j.pq & 15))
    return hipErrorNotSupported;
  if (sn && (!temporal_fused_phase3(g.T, g.V) || g.C != 64 || !g.pq || sn->pq != g.pq || sn->ngroups != 2 || sn->xin ||
             sn->pql.sch != 1 || (sn->pql.st & 3) || (sn->pql.sv & 3) || (sn->pql.sn & 3) || (sn->p_ch[0] & 3) ||
             (sn->p_ch[1] & 3) || !sn->out))
    return hipErrorNotSupported;
  if (s0 && (sa.Cin != 6 || !block_fused_adj0_supported(g.T, g.V) || !s0->xin || s0->ngroups != 2 || !s0->out ||
             s0->B != g.B || !sa.xmodel || sa.adj != s0->out))
    return hipErrorNotSupported;
  *out = BlockFusedArgs{sa, TemporalFusedArgs{g, j, sn ? *sn : AdjHLArgs{}}, s0 ? *s0 : AdjHLArgs{}};
  return hipSuccess;
}

hipError_t launch_block_fused(const SpatialHLArgs& sa, const TemporalHLArgs& g, const AdjHLArgs& j, const AdjHLArgs* sn,
                              hipStream_t s, const AdjHLArgs* s0) {
  BlockFusedArgs a;
  const hipError_t e = block_fused_args(sa, g, j, sn, &a, s0);
  if (e != hipSuccess) return e;
  if (g.T == 35 && g.V == 22) return bfused_tv<35, 22>(a, s);
  if (g.T == 35 && g.V == 25) return bfused_tv<35, 25>(a, s);
  if (g.T == 40 && g.V == 23) return bfused_tv<40, 23>(a, s);
  return hipErrorNotSupported;
}

bool temporal_fused_supported(int T, int V) {
  return (T == 35 && (V == 22 || V == 25)) || (T == 40 && V == 23) || (T == 75 && V == 22);
}
// the schedule's default at full batch: T = 75 runs its u chunks only when
// asked (DSTD_FWD_FUSED_TEMPORAL) -- measured 8.8% slower per forward than the
// unfused pair (profiles/r05h_t75_fused_ab.txt)
bool temporal_fused_default(int T, int V) {
#ifdef DSTD_TF75_DEFAULT
  return temporal_fused_supported(T, V);
#else
  return temporal_fused_supported(T, V) && T != 75;
#endif
}
bool temporal_fused_phase3(int T, int V) {
  if (T == 35 && V == 22) return tf_phase3<35, 22>();
  if (T == 35 && V == 25) return tf_phase3<35, 25>();
  if (T == 40 && V == 23) return tf_phase3<40, 23>();
  if (T == 75 && V == 22) return tf_phase3<75, 22>();
  return false;
}

hipError_t launch_temporal_fused(const TemporalHLArgs& g, const AdjHLArgs& j, const AdjHLArgs* sn, hipStream_t s) {
  if (!temporal_fused_supported(g.T, g.V) || g.V != (int)(j.pql.st / 4) || j.pql.sch != 1 || j.pql.sv != 4 ||
      ((uintptr_t)j.pq & 15))
    return hipErrorNotSupported;
  if (sn && (!temporal_fused_phase3(g.T, g.V) || g.C != 64 || !g.pq || sn->pq != g.pq || sn->ngroups != 2 || sn->xin || sn->pql.sch != 1 ||
             (sn->pql.st & 3) || (sn->pql.sv & 3) || (sn->pql.sn & 3) || (sn->p_ch[0] & 3) || (sn->p_ch[1] & 3) ||
             !sn->out))
    return hipErrorNotSupported;
  const TemporalFusedArgs a{g, j, sn ? *sn : AdjHLArgs{}};
  if (g.T == 35 && g.V == 22) return tfused_tv<35, 22>(a, s);
  if (g.T == 35 && g.V == 25) return tfused_tv<35, 25>(a, s);
  if (g.T == 40 && g.V == 23) return tfused_tv<40, 23>(a, s);
  if (g.T == 75 && g.V == 22) return tfused_tv<75, 22>(a, s);
  return hipErrorNotSupported;
}

hipError_t launch_temporal_hl(const TemporalHLArgs& a, hipStream_t s) {
  if (!temporal_hl_supported(a.T, a.V)) return hipErrorNotSupported;
  switch (a.T) {
    case 35: return temporal_hl_t<35>(a, s);
    case 40: return temporal_hl_t<40>(a, s);
    case 75: return temporal_hl_t<75>(a, s);
    default: return hipErrorNotSupported;
  }
}

}  // namespace dstd

#ifdef DSTD_STAMPS
extern "C" int dstd_debug_timeline_hl(int mode, unsigned long long* host, int n) {
  if (mode < 0 || mode > 5 || n > 2048 * 4) return 1;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tl_hl), n * sizeof(unsigned long long),
                                  mode * 2048 * 4 * sizeof(unsigned long long));
}
#endif

