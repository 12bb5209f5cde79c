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
#include "dstd_common.h"
#include "dstd_hilo.h"
#include "dstd_kernels.h"

namespace dstd {

namespace {

constexpr int HW = 4;        // waves per workgroup
constexpr int HT = HW * 64;  // threads per workgroup

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ f16x8 as_h8(const uint4& v) { return __builtin_bit_cast(f16x8, v); }

__device__ __forceinline__ f32x4 mfma32(const f16x8& a, const f16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// hi/lo pair of an f32x4 quartet from two accumulator tiles (slots e = 0..3
// from the first, 4..7 from the second)
__device__ __forceinline__ void split_acc(const f32x4& a, const f32x4& b, f16x8& hi, f16x8& lo) {
  split8(make_float4(a[0], a[1], a[2], a[3]), make_float4(b[0], b[1], b[2], b[3]), hi, lo);
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
  const int gw = blockIdx.x * HW + wave;
  const long nw = (long)gridDim.x * HW;
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
constexpr uint32_t OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ uint4 bldu4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ void bst4(__amdgpu_buffer_rsrc_t r, uint32_t off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 0);
}

// folded BN vectors [V][64] -> LDS [c/4][v]
__device__ __forceinline__ void stage_bn64(float4* dst, const float* src, int V, int tid) {
  for (int i = tid; i < V * 16; i += HT) {
    const int v = i >> 4, c4 = i & 15;
    dst[c4 * V + v] = ld4(src + v * 64 + 4 * c4);
  }
}

}  // namespace

// ===========================================================================
// weight images: one workgroup per job
// ===========================================================================
__global__ __launch_bounds__(256) void k_hl_prep(HLPrepArgs a) {
  const HLJob& j = a.jobs[blockIdx.x];
  const int tid = threadIdx.x;
  const int n = j.kind == HLJ_CONV ? 64 * 64 : 128 * j.nblk;
  float m = 0.f;
  for (int i = tid; i < n; i += 256) m = fmaxf(m, fabsf(j.kind == HLJ_CONV ? j.w[0][i] : j.w[i >> 7][i & 127]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float red[4];
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  // 2^s with max|w| * 2^s < 2^14: low halves of the scaled weights stay normal
  int e = 0;
  float scale = 1.f;
  if (m > 0.f && isfinite(m)) {
    frexpf(m, &e);  // m = f * 2^e, f in [0.5, 1)
    scale = ldexpf(1.f, 14 - e);
  }
  if (tid == 0) *j.inv_scale = 1.f / scale;
  if (j.kind == HLJ_CONV) {
    for (int i = tid; i < 4 * 2 * 64; i += 256) {
      const int lane = i & 63, ks = (i >> 6) & 1, ct = i >> 7;
      const int c = 16 * ct + (lane & 15), k0 = 32 * ks + 8 * (lane >> 4);
      const float* w = j.w[0] + c * 64 + k0;
      uint4 hi, lo;
      split8(make_float4(w[0] * scale, w[1] * scale, w[2] * scale, w[3] * scale),
             make_float4(w[4] * scale, w[5] * scale, w[6] * scale, w[7] * scale), hi, lo);
      j.img[((ct * 2 + ks) * 2 + 0) * 64 + lane] = hi;
      j.img[((ct * 2 + ks) * 2 + 1) * 64 + lane] = lo;
    }
  } else {
    for (int i = tid; i < 2 * 64; i += 256) {
      const int lane = i & 63, ks = i >> 6;
      const int ch = lane & 15, kg = lane >> 4;
      float v[8];
#pragma unroll
      for (int e8 = 0; e8 < 8; ++e8) {
        const int c = 16 * (2 * ks + (e8 >> 2)) + 4 * kg + (e8 & 3);
        v[e8] = ch < 2 * j.nblk ? j.w[ch >> 1][(ch & 1) * 64 + c] * scale : 0.f;
      }
      uint4 hi, lo;
      split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), hi, lo);
      j.img[(ks * 2 + 0) * 64 + lane] = hi;
      j.img[(ks * 2 + 1) * 64 + lane] = lo;
    }
  }
}

// ===========================================================================
// Spatial GC, 64 -> 64, two graphs (DSTDGCB.forward model/dstdgcn.py:141-154
// with DSTDGC.forward spatial :80-87), unit = (sample n, frame t):
//   y[c][w] = sum_g sum_v (W_g x + b_g)[v][c] Adj_g[t][v][w]
//   h = prelu(bn(y) + x)  ->  NTVC, and P_t/Q_t of h ([B][T][V][4])
// ===========================================================================
template <int V>
__global__ __launch_bounds__(HT) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_spatial_hl(SpatialHLArgs a) {
  using SM = SlotMap<V, true>;
  constexpr int SL = SM::SL, NG = SM::NG, NWT = cdiv(V, 16);
  static_assert(SM::MT == 2 && SM::NS == 1, "one K-step of two tiles per frame");
  __shared__ uint4 wl[2][kHLConvImg];
  __shared__ uint4 pql[kHLPQImg];
  __shared__ float4 bnl[2][16 * V];
  __shared__ float bfl[2][64];
  __shared__ float bql[4];
  __shared__ float scl[3];

  const int tid = threadIdx.x, lane = tid & 63;
  const int kl = lane >> 4, cl = lane & 15;
  const int T = a.T;
  for (int i = tid; i < 2 * kHLConvImg; i += HT) wl[i / kHLConvImg][i % kHLConvImg] = a.wimg[i / kHLConvImg][i % kHLConvImg];
  for (int i = tid; i < kHLPQImg; i += HT) pql[i] = a.pqimg[i];
  stage_bn64(bnl[0], a.bn_s, V, tid);
  stage_bn64(bnl[1], a.bn_h, V, tid);
  if (tid < 128) bfl[tid >> 6][tid & 63] = a.bf[tid >> 6][tid & 63];
  if (tid < 4) bql[tid] = a.pqb[tid >> 1][tid & 1];
  if (tid == 0) {
    scl[0] = *a.wscale[0];
    scl[1] = *a.wscale[1];
    scl[2] = *a.pqscale;
  }
  __syncthreads();

  int uend;
  int u = unit_range(a.B * T, uend);
  const float pw = *a.prelu;
  // x rows of the two conv tiles: joint of tile m, row cl; k-step ks, lane group kl
  const uint32_t xo0 = (uint32_t)(min(SM::row_idx(0, cl), V - 1) * 64 + 8 * kl) * 4;
  const uint32_t xo1 = (uint32_t)(min(SM::row_idx(1, cl), V - 1) * 64 + 8 * kl) * 4;
  constexpr uint32_t unit_bytes = V * 64 * 4;     // one frame of x / y
  constexpr uint32_t adj_bytes = 2 * V * SL * 2;  // one (n, g, t) adjacency: 2 planes of V x SL halves
  // per output tile wt: this lane's joint w = 16wt + cl (OOB past V)
  uint32_t wro[NWT], wadj[NWT], wpq[NWT];
#pragma unroll
  for (int wt = 0; wt < NWT; ++wt) {
    const int w = 16 * wt + cl;
    wro[wt] = w < V ? (uint32_t)(w * 64 + 4 * kl) * 4 : OOB;
    wadj[wt] = w < V && kl < NG ? (uint32_t)(w * SL + 8 * kl) * 2 : OOB;
    wpq[wt] = w < V && kl == 0 ? (uint32_t)w * 16 : OOB;
  }

  float4 xr[2][2][2];  // [tile][k-step][half]: channels 32ks + 8kl .. +7 of the tile row
  auto load_x = [&](int uu) {
    const auto r = rsrc(a.x + (size_t)uu * V * 64, unit_bytes);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      xr[0][ks][0] = bld4(r, xo0 + 128 * ks);
      xr[0][ks][1] = bld4(r, xo0 + 128 * ks + 16);
      xr[1][ks][0] = bld4(r, xo1 + 128 * ks);
      xr[1][ks][1] = bld4(r, xo1 + 128 * ks + 16);
    }
  };
  uint4 ab[2][NWT][2];  // adjacency B fragments [graph][w tile][plane]
  auto load_adj = [&](int uu) {
    const int n = uu / T, t = uu - n * T;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const auto r = rsrc(a.adj + ((size_t)(n * 2 + g) * T + t) * (adj_bytes / 2), adj_bytes);
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) {
        ab[g][wt][0] = bldu4(r, wadj[wt]);
        ab[g][wt][1] = bldu4(r, wadj[wt] + V * SL * 2);
      }
    }
  };
  if (u < uend) {
    load_x(u);
    load_adj(u);
  }
  while (u < uend) {
    const int un = u + 1;
    const int lz = lane + opaque_zero();
    const auto rx = rsrc(a.x + (size_t)u * V * 64, unit_bytes);
    // identity residual at the output positions (w = 16wt + cl, channels 16ct + 4kl ..)
    float4 R[4][NWT];
#pragma unroll
    for (int wt = 0; wt < NWT; ++wt)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) R[ct][wt] = bld4(rx, wro[wt] + 64 * ct);
    f16x8 xh[2][2], xo[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) split8(xr[m][ks][0], xr[m][ks][1], xh[m][ks], xo[m][ks]);

    f32x4 O[4][NWT];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) O[ct][wt] = zero4();
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      // ---- conv (transposed): D[p][c] = sum_k x[p][k] W'[c][k] ----
      f32x4 D[2][4];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) D[m][ct] = zero4();
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int c2 = 0; c2 < 4; c2 += 2) {
          f16x8 wh[2], wo[2];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            wh[q] = as_h8(wl[g][(((c2 + q) * 2 + ks) * 2 + 0) * 64 + lz]);
            wo[q] = as_h8(wl[g][(((c2 + q) * 2 + ks) * 2 + 1) * 64 + lz]);
          }
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int m = 0; m < 2; ++m) D[m][c2 + q] = mfma32(xo[m][ks], wh[q], D[m][c2 + q]);
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int m = 0; m < 2; ++m) D[m][c2 + q] = mfma32(xh[m][ks], wo[q], D[m][c2 + q]);
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int m = 0; m < 2; ++m) D[m][c2 + q] = mfma32(xh[m][ks], wh[q], D[m][c2 + q]);
        }
      // x is dead after the second conv: prefetch the next unit's rows
      if (g == 1 && un < uend) load_x(un);
      // ---- aggregation: O[c][w] += sum_v D[v][c] Adj[v][w] ----
      const float s = scl[g];
      f16x8 dh[4], dl[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const float b = bfl[g][16 * ct + cl];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) D[m][ct][r] = fmaf(D[m][ct][r], s, b);
        split_acc(D[0][ct], D[1][ct], dh[ct], dl[ct]);
      }
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) O[ct][wt] = mfma32(dl[ct], as_h8(ab[g][wt][0]), O[ct][wt]);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) O[ct][wt] = mfma32(dh[ct], as_h8(ab[g][wt][1]), O[ct][wt]);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int wt = 0; wt < NWT; ++wt) O[ct][wt] = mfma32(dh[ct], as_h8(ab[g][wt][0]), O[ct][wt]);
    }
    if (un < uend) load_adj(un);

    // ---- epilogue: h = prelu(bn(y) + x) -> NTVC ----
    const auto ry = rsrc(a.y + (size_t)u * V * 64, unit_bytes);
#pragma unroll
    for (int wt = 0; wt < NWT; ++wt) {
      const int wc = min(16 * wt + cl, V - 1);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        f32x4& o = O[ct][wt];
        const float4 sc = bnl[0][(4 * ct + kl) * V + wc], sh = bnl[1][(4 * ct + kl) * V + wc];
        o[0] = prelu_f(fmaf(o[0], sc.x, sh.x) + R[ct][wt].x, pw);
        o[1] = prelu_f(fmaf(o[1], sc.y, sh.y) + R[ct][wt].y, pw);
        o[2] = prelu_f(fmaf(o[2], sc.z, sh.z) + R[ct][wt].z, pw);
        o[3] = prelu_f(fmaf(o[3], sc.w, sh.w) + R[ct][wt].w, pw);
        bst4(ry, wro[wt] + 64 * ct, make_float4(o[0], o[1], o[2], o[3]));
      }
    }
    // ---- P_t/Q_t of h: out[ch][w] = sum_c wq[ch][c] h[c][w] + b ----
    f32x4 acc[NWT];
#pragma unroll
    for (int wt = 0; wt < NWT; ++wt) acc[wt] = zero4();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const f16x8 qh = as_h8(pql[(ks * 2 + 0) * 64 + lz]), qo = as_h8(pql[(ks * 2 + 1) * 64 + lz]);
      f16x8 hh[NWT], hl[NWT];
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) split_acc(O[2 * ks][wt], O[2 * ks + 1][wt], hh[wt], hl[wt]);
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) acc[wt] = mfma32(qo, hh[wt], acc[wt]);
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) acc[wt] = mfma32(qh, hl[wt], acc[wt]);
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt) acc[wt] = mfma32(qh, hh[wt], acc[wt]);
    }
    {
      const float s = scl[2];
      const auto rp = rsrc(a.pq + (size_t)u * V * 4, V * 16);
#pragma unroll
      for (int wt = 0; wt < NWT; ++wt)
        bst4(rp, wpq[wt],
             make_float4(fmaf(acc[wt][0], s, bql[0]), fmaf(acc[wt][1], s, bql[1]), fmaf(acc[wt][2], s, bql[2]),
                         fmaf(acc[wt][3], s, bql[3])));
    }
    u = un;
  }
}

// ===========================================================================
// Temporal GC, 64 -> 64 (DSTDGC.forward temporal, model/dstdgcn.py:88-93) with
// the DSTDGCB tail epilogues (:161-163, DSTDGCN.forward :306-311), unit =
// (sample n, joint v):
//   y[c][u] = sum_t (W h + b)[t][c] Adj[v][t][u]
//   ENC: prelu(bn(y + xres));  IN: prelu(bn(y));  RAW: y
//   + P_s/Q_s (8 channels, [B][V][T][8]) of the output for the next block
// ===========================================================================
// two waves per SIMD up to 48 frames; the 75-frame units need one SIMD each
template <int T>
constexpr int temporal_hl_wpe() {
  return T <= 48 ? 2 : 1;
}
template <int T, int EPI>
__global__ __launch_bounds__(HT) __attribute__((amdgpu_waves_per_eu(temporal_hl_wpe<T>(), temporal_hl_wpe<T>()))) void k_temporal_hl(
    TemporalHLArgs a) {
  using SM = SlotMap<T, false>;
  constexpr int SL = SM::SL, MT = SM::MT, NS = SM::NS, NUT = cdiv(T, 16);
  constexpr int VMAX = 32;
  constexpr bool use_bn = EPI == TEPI_ENC || EPI == TEPI_IN;
  constexpr bool use_res = EPI == TEPI_ENC;
  __shared__ uint4 wl[kHLConvImg];
  __shared__ uint4 pql[kHLPQImg];
  __shared__ float4 bnl[2][use_bn ? 16 * VMAX : 1];
  __shared__ float bfl[64];
  __shared__ float bql[8];
  __shared__ float scl[2];

  const int tid = threadIdx.x, lane = tid & 63;
  const int kl = lane >> 4, cl = lane & 15;
  const int V = a.V;
  const bool has_pq = a.pq != nullptr;
  for (int i = tid; i < kHLConvImg; i += HT) wl[i] = a.wimg[i];
  if (has_pq)
    for (int i = tid; i < kHLPQImg; i += HT) pql[i] = a.pqimg[i];
  if constexpr (use_bn) {
    stage_bn64(bnl[0], a.bn_s, V, tid);
    stage_bn64(bnl[1], a.bn_h, V, tid);
  }
  if (tid < 64) bfl[tid] = a.bf[tid];
  if (tid < 8) bql[tid] = has_pq ? a.pqb[tid >> 1][tid & 1] : 0.f;
  if (tid == 0) {
    scl[0] = *a.wscale;
    scl[1] = has_pq ? *a.pqscale : 0.f;
  }
  __syncthreads();

  int uend;
  int u = unit_range(a.B * V, uend);
  const float pw = use_bn ? *a.prelu : 0.f;
  // a unit's rows: frame t of joint v at t * V * 64 floats from the unit base
  const uint32_t col_bytes = (uint32_t)((T - 1) * V + 1) * 64 * 4;
  const uint32_t frame_bytes = (uint32_t)V * 64 * 4;
  constexpr uint32_t adj_bytes = 2 * T * SL * 2;  // one (n, v): 2 planes of T x SL halves
  uint32_t xoff[MT];  // conv rows: frame 16m + cl, channels 8kl ..
#pragma unroll
  for (int m = 0; m < MT; ++m) xoff[m] = (uint32_t)min(16 * m + cl, T - 1) * frame_bytes + 32 * kl;
  uint32_t uoff[NUT], upq[NUT];  // output frame uo = 16ut + cl (OOB past T), channels 4kl ..
#pragma unroll
  for (int ut = 0; ut < NUT; ++ut) {
    const int uo = 16 * ut + cl;
    uoff[ut] = uo < T ? (uint32_t)uo * frame_bytes + 16 * kl : OOB;
    upq[ut] = uo < T && kl < 2 ? (uint32_t)(uo * 8 + 4 * kl) * 4 : OOB;
  }

  float4 xr[MT][2][2];  // tile m row cl = frame 16m + cl
  auto load_x = [&](int uu) {
    const int n = uu / V, v = uu - n * V;
    const auto r = rsrc(a.h + ((size_t)n * T * V + v) * 64, col_bytes);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        xr[m][ks][0] = bld4(r, xoff[m] + 128 * ks);
        xr[m][ks][1] = bld4(r, xoff[m] + 128 * ks + 16);
      }
  };
  if (u < uend) load_x(u);
  while (u < uend) {
    const int n = u / V, v = u - n * V;
    const int un = u + 1;
    const int lz = lane + opaque_zero();
    const size_t cbase = ((size_t)n * T * V + v) * 64;
    f16x8 xh[MT][2], xo[MT][2];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) split8(xr[m][ks][0], xr[m][ks][1], xh[m][ks], xo[m][ks]);

    // ---- conv (transposed): D[t][c] = sum_k h[t][k] W'[c][k] ----
    f32x4 D[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) D[m][ct] = zero4();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const f16x8 wh = as_h8(wl[((ct * 2 + ks) * 2 + 0) * 64 + lz]);
        const f16x8 wo = as_h8(wl[((ct * 2 + ks) * 2 + 1) * 64 + lz]);
#pragma unroll
        for (int m = 0; m < MT; ++m) D[m][ct] = mfma32(xo[m][ks], wh, D[m][ct]);
#pragma unroll
        for (int m = 0; m < MT; ++m) D[m][ct] = mfma32(xh[m][ks], wo, D[m][ct]);
#pragma unroll
        for (int m = 0; m < MT; ++m) D[m][ct] = mfma32(xh[m][ks], wh, D[m][ct]);
      }
    }
    if (un < uend) load_x(un);  // h rows are dead after the conv
    {
      const float s = scl[0];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const float b = bfl[16 * ct + cl];
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) D[m][ct][r] = fmaf(D[m][ct][r], s, b);
      }
    }
    // ---- aggregation: O[c][u] = sum_t D[t][c] Adj[v][t][u] ----
    f32x4 O[4][NUT];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int ut = 0; ut < NUT; ++ut) O[ct][ut] = zero4();
    const auto radj = rsrc(a.adj + (size_t)u * (adj_bytes / 2), adj_bytes);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint4 bh[NUT], bo[NUT];
#pragma unroll
      for (int ut = 0; ut < NUT; ++ut) {
        const int uo = 16 * ut + cl;
        const uint32_t off = uo < T && kl < SM::ng(s) ? (uint32_t)(uo * SL + 8 * (SM::goff(s) + kl)) * 2 : OOB;
        bh[ut] = bldu4(radj, off);
        bo[ut] = bldu4(radj, off + T * SL * 2);
      }
      f16x8 dh[4], dl[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) split_acc(D[2 * s][ct], 2 * s + 1 < MT ? D[2 * s + 1][ct] : zero4(), dh[ct], dl[ct]);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int ut = 0; ut < NUT; ++ut) O[ct][ut] = mfma32(dl[ct], as_h8(bh[ut]), O[ct][ut]);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int ut = 0; ut < NUT; ++ut) O[ct][ut] = mfma32(dh[ct], as_h8(bo[ut]), O[ct][ut]);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int ut = 0; ut < NUT; ++ut) O[ct][ut] = mfma32(dh[ct], as_h8(bh[ut]), O[ct][ut]);
    }
    // residual of the encoder epilogue, loaded after the aggregation (register pressure)
    float4 R[use_res ? 4 : 1][use_res ? NUT : 1];
    if constexpr (use_res) {
      const auto rr = rsrc(a.xres + cbase, col_bytes);
#pragma unroll
      for (int ut = 0; ut < NUT; ++ut)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) R[ct][ut] = bld4(rr, uoff[ut] + 64 * ct);
    }

    // ---- epilogue ----
    const auto ry = rsrc(a.y + cbase, col_bytes);
#pragma unroll
    for (int ut = 0; ut < NUT; ++ut) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        f32x4& o = O[ct][ut];
        if constexpr (use_res) {
          o[0] += R[ct][ut].x;
          o[1] += R[ct][ut].y;
          o[2] += R[ct][ut].z;
          o[3] += R[ct][ut].w;
        }
        if constexpr (use_bn) {
          const float4 sc = bnl[0][(4 * ct + kl) * V + v], sh = bnl[1][(4 * ct + kl) * V + v];
          o[0] = prelu_f(fmaf(o[0], sc.x, sh.x), pw);
          o[1] = prelu_f(fmaf(o[1], sc.y, sh.y), pw);
          o[2] = prelu_f(fmaf(o[2], sc.z, sh.z), pw);
          o[3] = prelu_f(fmaf(o[3], sc.w, sh.w), pw);
        }
        bst4(ry, uoff[ut] + 64 * ct, make_float4(o[0], o[1], o[2], o[3]));
      }
    }
    // ---- next block's P_s/Q_s (8 channels) of the output ----
    if (has_pq) {
      f32x4 acc[NUT];
#pragma unroll
      for (int ut = 0; ut < NUT; ++ut) acc[ut] = zero4();
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const f16x8 qh = as_h8(pql[(ks * 2 + 0) * 64 + lz]), qo = as_h8(pql[(ks * 2 + 1) * 64 + lz]);
        f16x8 hh[NUT], hl[NUT];
#pragma unroll
        for (int ut = 0; ut < NUT; ++ut) split_acc(O[2 * ks][ut], O[2 * ks + 1][ut], hh[ut], hl[ut]);
#pragma unroll
        for (int ut = 0; ut < NUT; ++ut) acc[ut] = mfma32(qo, hh[ut], acc[ut]);
#pragma unroll
        for (int ut = 0; ut < NUT; ++ut) acc[ut] = mfma32(qh, hl[ut], acc[ut]);
#pragma unroll
        for (int ut = 0; ut < NUT; ++ut) acc[ut] = mfma32(qh, hh[ut], acc[ut]);
      }
      const float s = scl[1];
      const auto rp = rsrc(a.pq + (size_t)u * T * 8, T * 32);
#pragma unroll
      for (int ut = 0; ut < NUT; ++ut) {
        const int b4 = 4 * (kl & 1);
        bst4(rp, upq[ut],
             make_float4(fmaf(acc[ut][0], s, bql[b4]), fmaf(acc[ut][1], s, bql[b4 + 1]), fmaf(acc[ut][2], s, bql[b4 + 2]),
                         fmaf(acc[ut][3], s, bql[b4 + 3])));
      }
    }
    u = un;
  }
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
int hl_occupancy(K k) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k, HT, 0) != hipSuccess || nb < 1) nb = 1;
  (void)hipGetLastError();
  return nb;
}

template <auto K, typename A>
hipError_t launch_units(int units, const A& a, hipStream_t s) {
  static const int occ = hl_occupancy(K);  // one per kernel instantiation
  int grid = hl_num_cus() * occ;
  grid = min(grid, cdiv(units, HW));
  hipLaunchKernelGGL(K, dim3(grid), dim3(HT), 0, s, a);
  return hipGetLastError();
}

template <int T>
hipError_t temporal_hl_t(const TemporalHLArgs& a, hipStream_t s) {
  switch (a.epi) {
    case TEPI_ENC: return launch_units<k_temporal_hl<T, TEPI_ENC>>(a.B * a.V, a, s);
    case TEPI_IN: return launch_units<k_temporal_hl<T, TEPI_IN>>(a.B * a.V, a, s);
    case TEPI_RAW: return launch_units<k_temporal_hl<T, TEPI_RAW>>(a.B * a.V, a, s);
    default: return hipErrorNotSupported;
  }
}

}  // namespace

hipError_t launch_hl_prep(const HLPrepArgs& a, hipStream_t s) {
  if (a.njobs <= 0) return hipSuccess;
  if (a.njobs > kMaxHLJobs) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_hl_prep, dim3(a.njobs), dim3(256), 0, s, a);
  return hipGetLastError();
}

// the shapes whose adjacency kernels (dstd_fast.hip) have a split-f16 writer
static bool hl_shape(int T, int V) {
  return (T == 35 && (V == 22 || V == 25)) || (T == 40 && V == 23) || (T == 75 && V == 22);
}
bool spatial_hl_supported(int T, int V) { return hl_shape(T, V); }
bool temporal_hl_supported(int T, int V) { return hl_shape(T, V); }

hipError_t launch_spatial_hl(const SpatialHLArgs& a, hipStream_t s) {
  if (!spatial_hl_supported(a.T, a.V)) return hipErrorNotSupported;
  switch (a.V) {
    case 22: return launch_units<k_spatial_hl<22>>(a.B * a.T, a, s);
    case 23: return launch_units<k_spatial_hl<23>>(a.B * a.T, a, s);
    case 25: return launch_units<k_spatial_hl<25>>(a.B * a.T, a, s);
    default: return hipErrorNotSupported;
  }
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
