// Split-f16 ("hi/lo") operand format of the 64 -> 64 GC kernels (dstd_hilo.hip).
//
// gfx950 runs v_mfma_f32_16x16x32_f16 at 16 cycles for 16x16x32 MACs; the
// exact-fp32 v_mfma_f32_16x16x4_f32 needs 8 x 32 cycles for the same work.  An
// fp32 operand a is carried as a pair of f16 values, a_hi = f16(a) and
// a_lo = f16(a - a_hi) (22 significant bits), and a product as
//   a*b ~= a_hi*b_hi + a_hi*b_lo + a_lo*b_hi     (three MFMAs, fp32 accumulate)
// -- 5.3x fewer MFMA cycles than fp32.  Weights are pre-scaled by a power of
// two (max|w| * 2^s < 2^14) so that their low halves stay normal f16 numbers;
// the accumulator is scaled back by 2^-s (exact).  Activations and adjacency
// entries are split under a power-of-two RANGE SCALE (below) so that no half
// can overflow f16 whatever the fp32 magnitudes; tanh values are in [0, 1].
// Emulated on the
// fixtures (scripts/split_precision.py) the whole-model error against the
// fp64 reference stays at the level of an fp32 run (0.6-1.1x the reference's
// own fp32 error), per op 0.5-0.9x.
//
// MFMA 16x16x32 f16 lane maps: A[i = lane&15][k = 8*(lane>>4) + e],
// B[k = 8*(lane>>4) + e][j = lane&15], e = 0..7; C/D as for every 16x16 MFMA,
// D[4*(lane>>4) + r][lane&15].
//
// The contraction of an aggregation (joint v of the spatial GC, frame t of
// the temporal GC) runs in K-steps of 32 slots.  Slot e = 4*mm + r of lane
// group kg in K-step s is row 4*kg + r of conv tile 2*s + mm -- so the conv
// accumulators of tiles 2s and 2s+1 ARE the A operand of K-step s (after the
// hi/lo split) -- and stands for index
//   interleaved (IL): 32*s + 8*kg + 4*mm + r     (spatial: 22 joints in 3 groups)
//   sequential      : 32*s + 16*mm + 4*kg + r    (temporal: tile m = frames 16m..16m+15)
// The adjacency writer stores, per output column (w / u) and per plane
// (hi, lo), the slot groups (s, kg) that hold a valid index, 8 halves each,
// in slot order: one 16-byte load per lane gives a B fragment.
#pragma once
#include "dstd_common.h"
#include "dstd_kernels.h"

namespace dstd {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

// 8 fp32 values -> packed hi = f16(v) (v_cvt_pk_f16_f32, round to nearest
// even) and packed lo = f16(v - hi) (v_fma_mixlo/hi_f16: the difference is
// formed exactly inside the fma and rounded once) -- 1.5 VALU per value
// instead of 2.5 for convert / convert back / subtract / convert.
// The trailing s_nop 1 covers the VALU-write -> MFMA-read hazard (2 wait
// states): hipcc's hazard recognizer does not see inside inline asm, and an
// MFMA reading lo right after the block read stale values (measured).
__device__ __forceinline__ void split8(const float4& a, const float4& b, uint4& hi, uint4& lo) {
  hi.x = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a.x, a.y}, f16x2_t));
  hi.y = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a.z, a.w}, f16x2_t));
  hi.z = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){b.x, b.y}, f16x2_t));
  hi.w = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){b.z, b.w}, f16x2_t));
#ifdef DSTD_SPLIT_CVT
  const f16x2_t h0 = __builtin_bit_cast(f16x2_t, hi.x), h1 = __builtin_bit_cast(f16x2_t, hi.y);
  const f16x2_t h2 = __builtin_bit_cast(f16x2_t, hi.z), h3 = __builtin_bit_cast(f16x2_t, hi.w);
  lo.x = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a.x - (float)h0[0], a.y - (float)h0[1]}, f16x2_t));
  lo.y = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a.z - (float)h1[0], a.w - (float)h1[1]}, f16x2_t));
  lo.z = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){b.x - (float)h2[0], b.y - (float)h2[1]}, f16x2_t));
  lo.w = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){b.z - (float)h3[0], b.w - (float)h3[1]}, f16x2_t));
#else
  asm("v_fma_mixlo_f16 %0, %4, 1.0, -%12 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %5, 1.0, -%12 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %1, %6, 1.0, -%13 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %7, 1.0, -%13 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %2, %8, 1.0, -%14 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %2, %9, 1.0, -%14 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %3, %10, 1.0, -%15 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %3, %11, 1.0, -%15 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "s_nop 1"
      : "=&v"(lo.x), "=&v"(lo.y), "=&v"(lo.z), "=&v"(lo.w)
      : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w), "v"(hi.x), "v"(hi.y),
        "v"(hi.z), "v"(hi.w));
#endif
}
__device__ __forceinline__ void split8(const float4& a, const float4& b, f16x8& hi, f16x8& lo) {
  uint4 h, l;
  split8(a, b, h, l);
  hi = __builtin_bit_cast(f16x8, h);
  lo = __builtin_bit_cast(f16x8, l);
}
// 4 values (the other four halves of an 8-half fragment are zero): split8
// without the four fma_mix on zeros, which the asm block hides from hipcc
__device__ __forceinline__ void split4(const float4& a, uint2& hi, uint2& lo) {
  hi.x = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a.x, a.y}, f16x2_t));
  hi.y = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a.z, a.w}, f16x2_t));
  asm("v_fma_mixlo_f16 %0, %2, 1.0, -%6 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %3, 1.0, -%6 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %1, %4, 1.0, -%7 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %5, 1.0, -%7 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "s_nop 1"
      : "=&v"(lo.x), "=&v"(lo.y)
      : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(hi.x), "v"(hi.y));
}

// max(m, |a|, |b|) as ONE v_max3_f32 with abs source modifiers.  fmaxf on
// loaded values costs three instructions per two values here: in IEEE mode
// hipcc first canonicalises each operand (v_max_f32 x, |x|, |x|).  Operands
// must be loads or VALU results, never an MFMA accumulator read directly: the
// hazard recognizer does not look into inline asm, so it would not pad the
// MFMA -> VALU read.
__device__ __forceinline__ float amax2(float m, float a, float b) {
  float r;
  asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}

// PReLU as one median: w <= 1 gives max(x, w x), w > 1 gives min(x, w x),
// i.e. med3(x, w x, c) with the wave-uniform c = +inf / -inf (prelu_cap).
// Equal to prelu_f bit for bit up to the sign of a zero; two VALU per value
// instead of three (max, min, fma).
__device__ __forceinline__ float prelu_cap(float w) { return w <= 1.f ? __builtin_inff() : -__builtin_inff(); }
__device__ __forceinline__ float prelu_m(float x, float w, float c) { return __builtin_amdgcn_fmed3f(x, w * x, c); }

template <int N, bool IL>
struct SlotMap {
  static constexpr int NS = cdiv(N, 32);  // K-steps
  __host__ __device__ static constexpr int idx(int s, int kg, int e) {
    return IL ? 32 * s + 8 * kg + e : 32 * s + 16 * (e >> 2) + 4 * kg + (e & 3);
  }
  // conv tile m, row i -> index
  __host__ __device__ static constexpr int row_idx(int m, int i) { return idx(m >> 1, i >> 2, 4 * (m & 1) + (i & 3)); }
  // lane groups of K-step s that hold a valid index (always a prefix kg < ng)
  __host__ __device__ static constexpr int ng(int s) {
    int g = 0;
    for (int kg = 0; kg < 4; ++kg)
      for (int e = 0; e < 8; ++e)
        if (idx(s, kg, e) < N) g = kg + 1;
    return g;
  }
  __host__ __device__ static constexpr int goff(int s) {
    int o = 0;
    for (int q = 0; q < s; ++q) o += ng(q);
    return o;
  }
  static constexpr int NG = goff(NS);  // stored groups per row
  static constexpr int SL = 8 * NG;    // halves per row and plane
  __host__ __device__ static constexpr bool tile_used(int m) {
    for (int i = 0; i < 16; ++i)
      if (row_idx(m, i) < N) return true;
    return false;
  }
  __host__ __device__ static constexpr int ntiles() {
    int t = 0;
    for (int m = 0; m < 2 * NS; ++m)
      if (tile_used(m)) t = m + 1;
    return t;
  }
  static constexpr int MT = ntiles();  // conv row tiles
  // stored slot (0 .. SL-1) -> index (>= N: padding, stored as zero)
  __host__ __device__ static constexpr int slot_idx(int sl) {
    const int G = sl >> 3, e = sl & 7;
    int s = 0;
    while (s + 1 < NS && goff(s + 1) <= G) ++s;
    return idx(s, G - goff(s), e);
  }
};

// ---- a gfx950 MFMA hazard hipcc (ROCm 7.2) does not pad -----------------
// Mixed-shape MFMA chains: an MFMA that takes the previous MFMA's result whole as
// its C operand (an accumulate chain) computes with a stale accumulator when
// the two MFMAs have DIFFERENT shapes (v_mfma_f32_16x16x32_f16 followed by
// v_mfma_f32_16x16x16_f16 or the reverse) and fewer than 5 wait states lie
// between them; same-shape chains are exact back to back and at any gap.
// Measured with scripts/micro/mfma_read_hazard.hip (64 K lanes, gaps 0..7:
// ~90% of lanes wrong at gaps 0-3 for both mixed orders, 0 at gap >= 4 and
// for every same-shape pair).  hipcc's hazard recognizer asks 0 wait states
// for any XDL -> XDL "full SrcC" dependency, so mixed-shape chains are wrong
// or right depending on how the scheduler interleaves them (round 2's
// "wrong results, not understood": DESIGN.md §4).  Rule in this tree: a
// chain never changes MFMA shape on one accumulator -- the 16x16x16 tail
// steps of the conv_rm GEMMs accumulate from zero into an accumulator of
// their own, added with four VALU adds; scripts/mfma_hazard_audit.py checks
// the built library's ISA for the pattern (tests/test_capi_host.py).

// Halves per adjacency row (one output column, one plane) on the host.
inline int hl_sl_spatial(int V) { return 8 * cdiv(V, 8); }
inline int hl_sl_temporal(int T) {
  int g = 0;
  for (int s = 0; s < cdiv(T, 32); ++s) {
    int n = 0;
    for (int kg = 0; kg < 4; ++kg)
      for (int e = 0; e < 8; ++e)
        if (32 * s + 16 * (e >> 2) + 4 * kg + (e & 3) < T) n = kg + 1;
    g += n;
  }
  return 8 * g;
}

// ---- range scaling (the split path over the whole fp32 range) -------------
// An f16 half holds at most 65504, so an fp32 activation above that would split
// into inf.  Every split operand is therefore brought below 2^14 by an exact
// power of two, chosen where it is split and undone on the fp32 accumulator:
//  * a GC unit's input rows x (spatial (sample, frame), temporal (sample,
//    joint)): x_s = 2^-sx x with the smallest sx >= 0 such that
//    max|x| * max(1, |W_f|_inf) < 2^(14 + sx) and max|b_f| < 2^(14 + sx), so
//    both x_s and the conv output F_s = W_f x_s + 2^-sx b_f (split again as
//    the aggregation operand) stay below 2^15; the aggregation result is
//    scaled back by 2^sx.  |W_f|_inf (max row L1 norm) and max|b_f| come from
//    k_hl_prep, max|x| is a wave reduction over the unit;
//  * the unit's output h before the next P/Q conv: h_s = 2^-sh h, max|h_s| < 2^14;
//  * the adjacency planes: 2^-sa Adj with |Adj| <= |alpha| max_r(sum_k |W_rm| +
//    |b_rm|) + max|Astat| < 2^(14 + sa) (a bound from the weights alone,
//    computed by k_hl_prep; both graphs of a spatial launch share one sa).
// sx = sh = sa = 0 whenever the values are in range, which leaves the
// arithmetic bit-identical to an unscaled split; every scale is exact, so the
// only cost of a shift is the dynamic range of the low halves (relative to
// the unit's largest value, 2^-24).
constexpr int kHLSlot = 4;  // floats per weight-image scale slot:
enum HLSlotField {
  HLS_INV = 0,    // 2^-s of the image
  HLS_BOUND = 1,  // HLJ_CONV: |W|_inf (max row L1 norm, unscaled); HLJ_RM: the adjacency bound
  HLS_BMAX = 2,   // HLJ_CONV: max|bias| (0 without a bias)
};
__host__ __device__ constexpr inline int hl_range_shift(int e) { return e - 14 < 0 ? 0 : e - 14 > 120 ? 120 : e - 14; }

// ---- weight images (one k_hl_prep launch per forward) --------------------
// HLJ_CONV: fragments of a 1x1 conv W[c][k] (rows = c out, cols = k in):
//   img[((ct*KSI + ks)*2 + plane)*64 + lane] = 8 halves of 2^s * W[16ct + j][32ks + 8kg + e]
//   (j = lane&15, kg = lane>>4, KSI = cdiv(cols, 32), zero outside) -- the B
//   operand of the transposed conv and the A operand of a conv in output
//   layout alike; <= 16 KiB.
// HLJ_PQ: A fragments of the P/Q conv of the next DSTDGC(s) over cols input
//   channels: row ch = 2*blk + rr of w[blk][rr*cols + c], slot (kg, e = 4mm + r)
//   of K-step ks <-> c = 16*(2ks+mm) + 4kg + r: img[(ks*2 + plane)*64 + lane], <= 4 KiB.
// HLJ_RM: A fragments of conv_rm, W[row][k] (rows x cols = T x 2T spatial,
//   V x 2V temporal), K-steps as hl_rm_ksteps(): NSF full steps of 32 for the
//   16x16x32 MFMA, img[((rt*NSF + s)*2 + plane)*64 + lane] = 8 halves of
//   2^s * W[16rt + i][32s + 8kg + e], then (when the remainder fits 16) one
//   16x16x16 tail step, img16[(rt*2 + plane)*64 + lane] = 4 halves of
//   W[16rt + i][32 NSF + 4kg + e] as uint2 after the full steps
//   (i = lane&15, kg = lane>>4, zero outside).
__host__ __device__ constexpr inline int hl_rm_nsf(int K) { return K % 32 > 16 ? K / 32 + 1 : K / 32; }
__host__ __device__ constexpr inline int hl_rm_tail(int K) { return K % 32 != 0 && K % 32 <= 16 ? 1 : 0; }
__host__ __device__ constexpr inline int hl_rm_kp(int K) { return 32 * hl_rm_nsf(K) + 16 * hl_rm_tail(K); }

// Row placement of the E / F arrays of the tanh GEMMs (k_adj_hl, phases 1 and
// 3 of k_temporal_fused): row r starts at float r * SE + 4 * (((r >> SH) & MSK)
// * MUL).  A lane of the tanh fragments reads 16 bytes of row pr (E) and qr
// (F) at k = 32 s + 8 kg (+ 4); in the slot order of the planes the 16 lanes
// of one ds_read_b128 bank group read rows whose plain-stride starts collide
// on the 64 banks (2-3 extra LDS cycles per read).  -DDSTD_EF_SWIZZLE places
// the rows by offsets chosen per shape with a bank model of the access (the
// guide's ds_read_b128 lane groups; rows disjoint and 16-byte aligned): the
// fused temporal kernel's bank-conflict cycles fell 1.041e6 -> 6.37e5 per
// launch, bit-identical, but the forward got 0.7% slower at H36M (the row
// offsets cost VALU in a kernel that is issue-bound, not LDS-bound:
// profiles/r05h_lds_layout_ab.txt), so the plain stride stays the default.
template <int SE_, int SH = 0, int MSK = 0, int MUL = 0>
struct EfRows {
  static constexpr int SE = SE_;
  __host__ __device__ static constexpr int row(int r) { return r * SE + 4 * (((r >> SH) & MSK) * MUL); }
  __host__ __device__ static constexpr int floats(int nrows) { return row(nrows - 1) + SE; }
};
// TEMPORAL: rows = frames (NA = T slots, K = 2V); spatial: rows = joints (NA =
// V, K = 2T).  Modelled extra LDS cycles per tile set (E and F reads) in the
// comments: plain KP + 4 stride -> this placement.
#ifdef DSTD_EF_SWIZZLE  // (off: measured slower, DESIGN.md section 4 "LDS bank conflicts")
template <bool TEMPORAL, int NA, int K>
struct EfPick {
  using type = EfRows<hl_rm_kp(K) + 4>;
};
template <> struct EfPick<true, 35, 44> { using type = EfRows<72, 0, 1, 5>; };    // H36M temporal: 1044 -> 484
template <> struct EfPick<false, 22, 70> { using type = EfRows<88, 0, 1, 1>; };   // H36M spatial: 660 -> 132
template <> struct EfPick<true, 40, 46> { using type = EfRows<56, 0, 1, 1>; };    // 3DPW temporal: 1200 -> 800
template <> struct EfPick<false, 23, 80> { using type = EfRows<88, 0, 1, 1>; };   // 3DPW spatial: 692 -> 140
template <> struct EfPick<true, 35, 50> { using type = EfRows<72, 0, 1, 1>; };    // CMU temporal: 1808 -> 272
template <> struct EfPick<false, 25, 70> { using type = EfRows<112, 3, 1, 1>; };  // CMU spatial: 800 -> 200
#else  // the plain KP + 4 stride
template <bool TEMPORAL, int NA, int K>
struct EfPick {
  using type = EfRows<hl_rm_kp(K) + 4>;
};
#endif
enum HLJobKind { HLJ_CONV = 0, HLJ_PQ = 1, HLJ_RM = 2 };
struct HLJob {
  int kind;
  const float* w[4];  // HLJ_CONV / HLJ_RM: w[0] = [rows][cols]; HLJ_PQ: nblk two-row blocks [2][cols]
  int nblk;
  int rows, cols;
  uint4* img;
  float* inv_scale;   // scale slot (kHLSlot floats, HLSlotField)
  const float* bias;  // HLJ_RM: conv_rm bias, copied to bias_out; HLJ_CONV: the conv bias or null (HLS_BMAX)
  float* bias_out;
  const float* alpha; // HLJ_RM: alpha and the static adjacency [nastat] of the bound
  const float* astat;
  int nastat;
};
inline int hl_rm_img(int rows, int cols) {  // uint4
  return cdiv(rows, 16) * (hl_rm_nsf(cols) * 2 * 64 + hl_rm_tail(cols) * 64);
}
constexpr int kMaxHLJobs = 48;
struct HLPrepArgs {
  HLJob jobs[kMaxHLJobs];
  int njobs;
};
constexpr int kHLConvImg = 4 * 2 * 2 * 64;  // uint4 per HLJ_CONV image
constexpr int kHLPQImg = 2 * 2 * 64;        // uint4 per HLJ_PQ image

// ---- GC kernel arguments --------------------------------------------------
struct SpatialHLArgs {
  const float* x;            // NTVC [B][T][V][Cin]; xmodel: the model input [B][T][V][3]
  int xmodel;                // Cin == 6 only: build x6 = cat(x, x - x[:, -1]) rows on the fly
  int B, T, V, Cin, Cout;    // (Cin, Cout) in {(64, 64), (6, 64), (64, 3)}
  const uint16_t* adj;       // [B][2][T][2 planes][V][SL] halves
  const uint4* wimg[3];      // HLJ_CONV images of conv_s[g].conv_f, [2]: residual conv (Cin != Cout)
  const float* wscale[3];
  const float* bf[3];        // conv_f biases, [2]: residual conv bias
  const float* bn_s;         // folded BN [V][Cout]
  const float* bn_h;
  const float* rbn_s;        // folded residual BN [V][Cout] (Cin != Cout)
  const float* rbn_h;
  const float* prelu;
  const float* adjb[2];      // scale slots of the two spatial conv_rm images (HLS_BOUND: range of the planes)
  float* y;                  // NTVC [B][T][V][Cout]
  const uint4* pqimg;        // HLJ_PQ image of conv_t.conv_m1/m2 (4 channels)
  const float* pqscale;
  const float* pqb[2];
  float* pq;                 // [B][T][V][4]
};

struct TemporalHLArgs {
  const float* h;            // NTVC [B][T][V][C]
  int B, T, V, C;            // C = 64, or 3 (conv_st_out: OUT / RAW epilogue, no P/Q)
  const uint16_t* adj;       // [B][V][2 planes][T][SL] halves
  const uint4* wimg;
  const float* wscale;
  const float* bf;
  const float* adjb;         // scale slot of the temporal conv_rm image (HLS_BOUND)
  int epi;                   // TemporalEpi: ENC, IN, RAW (C = 64); OUT, RAW (C = 3)
  const float* xres;         // ENC: block input; OUT: model input [B][T][V][3]
  const float* bn_s;
  const float* bn_h;
  const float* prelu;
  float* y;
  const uint4* pqimg;        // HLJ_PQ image of the next block's spatial conv_m1/m2 (8 channels) or null
  const float* pqscale;
  const float* pqb[4];
  float* pq;                 // [B][V][T][8]
};

// ---- dynamic adjacency in split-f16 planes ---------------------------------
// Adj = alpha * (W_rm . tanh(P - Q) + b_rm) + Astat as a GEMM on
// v_mfma_f32_16x16x32_f16 (three products): rows t (spatial) / v (temporal),
// K = 2T / 2V, columns (q, slot) in the slot order above; output planes as
// AdjArgs.hl documents.  Shapes: hl_shape() of dstd_hilo.hip.
struct AdjHLArgs {
  const float* xin;         // spatial, conv_st_in of the model: the model input [B][T][V][3]; P/Q
                            // of x6 = cat(x, x - x[:, -1]) are formed in the prologue from mw/mb
                            // (no prep launch); null: read pq
  const float* mw[2][2];    // [graph][conv_m1, conv_m2] weights [2][6]
  const float* mb[2][2];
  const float* pq;          // channel-innermost P/Q planes (PQLayout sch == 1)
  PQLayout pql;
  int p_ch[2];              // first channel (P_0, P_1, Q_0, Q_1) of each graph
  int B, ngroups;
  const uint4* wimg[2];     // HLJ_RM images of conv_rm
  const float* wscale[2];
  const float* bias[2];     // HLJob::bias_out of the conv_rm image (the conv_rm bias)
  const float* alpha;
  const float* astat[2];    // [NA][NA]
  uint16_t* out;
  long out_sN, out_sG;      // halves
  int nchunk;               // column chunks per (sample, graph) workgroup set; 0: the launcher picks
                            // (more below one workgroup per CU: small batches)
};

struct TemporalFusedArgs {
  TemporalHLArgs g;  // the GC launch (adj unused)
  AdjHLArgs j;       // P/Q (pq, pql), HLJ_RM image (wimg[0], wscale[0]), bias[0], alpha, astat[0]
  AdjHLArgs sn;      // out != null: the next block's spatial adjacency planes (launch_adj_hl mode 0 args;
                     // pq = g.pq, the P/Q this launch writes), built after the units (phase 3)
};
// one DSTDGCB of k_block_fused: the spatial GC (launch_spatial_hl
// arguments) and the fused temporal GC (launch_temporal_fused arguments)
struct BlockFusedArgs {
  SpatialHLArgs s;
  TemporalFusedArgs t;
  AdjHLArgs s0;  // out != null (conv_st_in only): this block's own spatial planes from the model
                 // input (launch_adj_hl mode 0 args with xin), built before the spatial units
};

hipError_t launch_hl_prep(const HLPrepArgs& a, hipStream_t s);
int hl_device_cus();  // compute units of the current device
// mode 0 spatial, 1 temporal
hipError_t launch_adj_hl(const AdjHLArgs& a, int mode, int T, int V, hipStream_t s);
// hipErrorNotSupported when the shape has no instantiation
hipError_t launch_spatial_hl(const SpatialHLArgs& a, hipStream_t s);
hipError_t launch_temporal_hl(const TemporalHLArgs& a, hipStream_t s);
bool spatial_hl_supported(int T, int V);
bool temporal_hl_supported(int T, int V);
// the temporal GC with its adjacency built in LDS (k_temporal_fused): g as for
// launch_temporal_hl (g.adj unused), j the adjacency's inputs as for
// launch_adj_hl mode 1 (j.out unused); sn (optional, C = 64 with g.pq): the
// next block's spatial adjacency as for launch_adj_hl mode 0 with sn->pq ==
// g.pq, built by the same launch after the units (no launch_adj_hl of it);
// hipErrorNotSupported off its shapes
hipError_t launch_temporal_fused(const TemporalHLArgs& g, const AdjHLArgs& j, const AdjHLArgs* sn, hipStream_t s);
bool temporal_fused_supported(int T, int V);
bool temporal_fused_phase3(int T, int V);  // the next block's spatial adjacency in the same launch
bool temporal_fused_default(int T, int V);  // fused at full batch without DSTD_FWD_FUSED_TEMPORAL
// a whole DSTDGCB per sample (k_block_fused): the spatial GC of launch_spatial_hl
// (sa) then the fused temporal GC of launch_temporal_fused (g, j, sn) in one
// launch, one workgroup per sample; sa.y must be g.h and sa.pq j.pq.  The
// block kinds of the model (6 -> 64 IN, 64 -> 64 ENC, 64 -> 3 OUT) at the
// fused temporal kernel's shapes (not T = 75); hipErrorNotSupported elsewhere.
// s0 (conv_st_in, block_fused_adj0_supported): the block's own spatial planes
// from the model input in the same launch instead of a k_adj_hl<0> launch
bool block_fused_supported(int T, int V, int cin, int cout, int epi);
bool block_fused_adj0_supported(int T, int V);
hipError_t launch_block_fused(const SpatialHLArgs& sa, const TemporalHLArgs& g, const AdjHLArgs& j, const AdjHLArgs* sn,
                              hipStream_t s, const AdjHLArgs* s0 = nullptr);
// validates one block's k_block_fused arguments and fills *out (no launch)
hipError_t block_fused_args(const SpatialHLArgs& sa, const TemporalHLArgs& g, const AdjHLArgs& j, const AdjHLArgs* sn,
                            BlockFusedArgs* out, const AdjHLArgs* s0 = nullptr);


}  // namespace dstd
