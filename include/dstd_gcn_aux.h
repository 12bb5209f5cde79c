/*
 * dstd_gcn_aux.h -- C ABI of the reference's non-refine ST_GCNN_layer branch
 * (SURVEY §8(f) row 4): ConvTemporalGraphical followed by a k_t x k_v Conv2d,
 * model/dstdgcn.py:166-188 and :218-223.  No shipped config builds it
 * (every ST_GCNN_layer is refine=True), it is here so the module API is whole.
 *
 *   dstd_ctg_fwd / _bwd     <- ConvTemporalGraphical.forward + autograd  :185-188
 *   dstd_conv2d_fwd / _bwd  <- nn.Conv2d(cin, cout, (kh, kw), stride, padding) (groups 1, dilation 1)
 *
 * Conventions as in dstd_gcn.h / dstd_gcn_train.h: device pointers to
 * contiguous fp32, NCTV activations, caller-owned workspace, enqueue on
 * `stream`, backward calls ACCUMULATE (+=) into dx / parameter gradients
 * (dx may be NULL).
 */
#ifndef DSTD_GCN_AUX_H
#define DSTD_GCN_AUX_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ConvTemporalGraphical: x1[n,c,q,v] = sum_t x[n,c,t,v] Tm[v,t,q];
 * y[n,c,t,w] = sum_v x1[n,c,t,v] (A[t,v,w] + A_fixed[v,w]).
 * Tm [V][T][T], A [T][V][V], A_fixed [V][V] (the reference's [1][V][V]). */
size_t dstd_ctg_workspace_bytes(int B, int C, int T, int V);
int dstd_ctg_fwd(const float* x, int B, int C, int T, int V, const float* Tm, const float* A, const float* A_fixed,
                 float* y, void* workspace, size_t workspace_bytes, void* stream);
/* dx (nullable), dTm, dA accumulate; A_fixed is a constant (requires_grad=False). */
int dstd_ctg_bwd(const float* x, int B, int C, int T, int V, const float* Tm, const float* A, const float* A_fixed,
                 const float* dy, float* dx, float* dTm, float* dA, void* workspace, size_t workspace_bytes,
                 void* stream);

/* y [B][cout][Ho][Wo] = conv2d(x [B][cin][H][W], w [cout][cin][kh][kw], bias [cout] or NULL),
 * Ho = (H + 2 ph - kh) / sh + 1, Wo likewise. */
size_t dstd_conv2d_workspace_bytes(int B, int cin, int cout, int H, int W, int kh, int kw, int sh, int sw, int ph,
                                   int pw);
int dstd_conv2d_fwd(const float* x, int B, int cin, int H, int W, const float* w, const float* bias, int cout,
                    int kh, int kw, int sh, int sw, int ph, int pw, float* y, void* workspace,
                    size_t workspace_bytes, void* stream);
/* dx (nullable), dw, db (nullable) accumulate. */
int dstd_conv2d_bwd(const float* x, int B, int cin, int H, int W, const float* w, int cout, int kh, int kw, int sh,
                    int sw, int ph, int pw, const float* dy, float* dx, float* dw, float* db, void* workspace,
                    size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DSTD_GCN_AUX_H */
