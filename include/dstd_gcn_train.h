/*
 * dstd_gcn_train.h -- C ABI of the MI355X training path.
 *
 * The reference trains through ATen autograd; these entry points replace the
 * train-mode forward and the backward of the same modules, plus the engine's
 * loss and test metric:
 *
 *   dstd_dstdgc_train_fwd/bwd  <- DSTDGC.forward + autograd   model/dstdgcn.py:80-94
 *   dstd_block_train_fwd/bwd   <- DSTDGCB.forward (train BN)  model/dstdgcn.py:141-163
 *   dstd_model_train_fwd/bwd   <- DSTDGCN.forward (train)     model/dstdgcn.py:293-317
 *   *_train_*_ex(RUNNING_STATS) <- the same under .eval() with autograd (BN on running stats)
 *   dstd_mpjpe_fwd/bwd         <- mpjpe_error_3d              engine/utils/loss.py:52-65
 *   dstd_frame_mpjpe           <- PredictionEngine.test       engine/prediction.py:366-404
 *
 * Conventions (in addition to dstd_gcn.h):
 *   - A train forward fills a caller-owned `saved` buffer (size from
 *     dstd_*_train_saved_bytes) that the matching backward reads; nothing else
 *     is kept between the two calls.
 *   - Train-mode forwards normalise with batch statistics and update every
 *     BatchNorm's running_mean / running_var in place with `momentum`
 *     (nn.BatchNorm1d semantics, unbiased running variance).  The pointers in
 *     dstd_bn are written despite their const qualifier.  num_batches_tracked
 *     is the caller's.
 *   - Backward calls ACCUMULATE (+=) into dx and into every gradient pointer;
 *     the caller zeroes them.  dx may be NULL (no input gradient).
 *   - Gradient semantics follow autograd on the reference: A_s and A_t are
 *     constants (requires_grad=False), so for the block adjacency
 *     A_s*W_s + R_s:  dW_s = dA * A_s,  dR_s = dA;  and A_t + R_t: dR_t = dA.
 */
#ifndef DSTD_GCN_TRAIN_H
#define DSTD_GCN_TRAIN_H

#include "dstd_gcn.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Gradient pointers mirror dstd_gc_weights / dstd_block_params / dstd_model_params. */
typedef struct dstd_gc_grads {
  float* wf;
  float* bf;
  float* wm1;
  float* bm1;
  float* wm2;
  float* bm2;
  float* wrm;
  float* brm;
} dstd_gc_grads;

typedef struct dstd_bn_grads {
  float* weight;
  float* bias;
} dstd_bn_grads;

typedef struct dstd_block_grads {
  float* W_s;      /* [2][V][V] */
  float* R_s;      /* [2][V][V] */
  float* R_t;      /* [1][T][T] */
  float* alpha_sm; /* [1] */
  float* alpha_tm; /* [1] */
  dstd_gc_grads conv_s[2];
  dstd_gc_grads conv_t;
  dstd_bn_grads bn;
  float* prelu;    /* [1] */
  float* res_w;    /* [cout][cin] (cin != cout only) */
  float* res_b;
  dstd_bn_grads res_bn;
} dstd_block_grads;

typedef struct dstd_model_grads {
  dstd_block_grads st_in;
  dstd_bn_grads bn_in;
  float* prelu;
  dstd_block_grads enc[DSTD_MAX_LAYERS];
  dstd_bn_grads enc_bn[DSTD_MAX_LAYERS];
  float* enc_prelu[DSTD_MAX_LAYERS];
  dstd_block_grads st_out;
} dstd_model_grads;

/* ---- one DSTDGC ---------------------------------------------------------- */
size_t dstd_dstdgc_train_saved_bytes(int mode, int B, int cin, int cout, int T, int V);
size_t dstd_dstdgc_train_workspace_bytes(int mode, int B, int cin, int cout, int T, int V);
/* y (=) DSTDGC(x, A, alpha); fills saved. */
int dstd_dstdgc_train_fwd(int mode, const float* x, int B, int cin, int cout, int T, int V,
                          const dstd_gc_weights* w, const float* A, const float* alpha, float* y, void* saved,
                          size_t saved_bytes, void* stream);
/* dx, g->*, dA ([V][V] or [T][T]) and dalpha ([1]) accumulate. */
int dstd_dstdgc_train_bwd(int mode, const float* x, int B, int cin, int cout, int T, int V,
                          const dstd_gc_weights* w, const float* alpha, const void* saved, size_t saved_bytes,
                          const float* dy, float* dx, const dstd_gc_grads* g, float* dA, float* dalpha,
                          void* workspace, size_t workspace_bytes, void* stream);

/* The same for any red_channels (the reference's DSTDGC(..., red_channels=R),
 * model/dstdgcn.py:55-68: conv_m1 / conv_m2 have R output channels and conv_rm
 * R*ref input channels; w->wm1/bm1/wm2/bm2/wrm sized accordingly).  The four
 * entries above are these with red = 2.  Limits: 1 <= red <= 8. */
size_t dstd_dstdgc_train_saved_bytes_r(int mode, int B, int cin, int cout, int T, int V, int red);
size_t dstd_dstdgc_train_workspace_bytes_r(int mode, int B, int cin, int cout, int T, int V, int red);
int dstd_dstdgc_train_fwd_r(int mode, const float* x, int B, int cin, int cout, int T, int V, int red,
                            const dstd_gc_weights* w, const float* A, const float* alpha, float* y, void* saved,
                            size_t saved_bytes, void* stream);
int dstd_dstdgc_train_bwd_r(int mode, const float* x, int B, int cin, int cout, int T, int V, int red,
                            const dstd_gc_weights* w, const float* alpha, const void* saved, size_t saved_bytes,
                            const float* dy, float* dx, const dstd_gc_grads* g, float* dA, float* dalpha,
                            void* workspace, size_t workspace_bytes, void* stream);

/* ---- one DSTDGCB --------------------------------------------------------- */
size_t dstd_block_train_saved_bytes(int B, int cin, int cout, int T, int V);
size_t dstd_block_train_workspace_bytes(int B, int cin, int cout, int T, int V);
int dstd_block_train_fwd(const dstd_block_params* p, const float* x, int B, int T, int V, float momentum, float* y,
                         void* saved, size_t saved_bytes, void* stream);
int dstd_block_train_bwd(const dstd_block_params* p, const float* x, int B, int T, int V, const void* saved,
                         size_t saved_bytes, const float* dy, float* dx, const dstd_block_grads* g,
                         void* workspace, size_t workspace_bytes, void* stream);

/* _ex variants: flags DSTD_TRAIN_RUNNING_STATS runs every BatchNorm on its
 * running statistics without updating them (eval-mode BN: the forward of an
 * eval-mode DSTDGCB / DSTDGCN whose output needs a gradient, and its
 * backward -- pass the same flags to both).  flags = 0 is the plain entry
 * point (batch statistics, running stats updated with momentum). */
#define DSTD_TRAIN_RUNNING_STATS 1u
/* DSTD_TRAIN_PAIRED: the batch is two independent BatchNorm batches of B/2
 * samples each (B even): statistics per half, running statistics updated by
 * the first half then the second -- exactly two train-mode forwards of B/2
 * (the engine's batch and its time reversal, engine/prediction.py:231-287)
 * in one launch sequence.  Pass the same flags to the backward. */
#define DSTD_TRAIN_PAIRED 2u
/* DSTD_TRAIN_SEED_DEVICE (model train fwd / bwd only): `seed` is the address
 * of a device uint64 that holds the dropout seed, read by the kernels -- a
 * seed drawn on the device (no host synchronisation, and a captured HIP graph
 * draws a fresh one per replay).  Pass the same flags and address to the
 * backward before the value changes. */
#define DSTD_TRAIN_SEED_DEVICE 4u
/* DSTD_TRAIN_ONE_STREAM (model train fwd / bwd only): every launch on the
 * caller's stream.  By default the backward runs each DSTDGC's weight-gradient
 * reductions (and its adjacency-gradient finish) on a second stream of the
 * device, and the forward builds each block's second spatial adjacency there
 * while the first spatial op runs, forked from and joined back into the
 * caller's stream by events (also inside a HIP graph capture); both orders
 * give bit-identical results. */
#define DSTD_TRAIN_ONE_STREAM 8u
int dstd_block_train_fwd_ex(const dstd_block_params* p, const float* x, int B, int T, int V, float momentum,
                            float* y, void* saved, size_t saved_bytes, void* stream, unsigned flags);
int dstd_block_train_bwd_ex(const dstd_block_params* p, const float* x, int B, int T, int V, const void* saved,
                            size_t saved_bytes, const float* dy, float* dx, const dstd_block_grads* g,
                            void* workspace, size_t workspace_bytes, void* stream, unsigned flags);

/* ---- whole DSTDGCN ------------------------------------------------------- */
/* x, y [B][T][V][in_channels/2].  dropout_p is the model's do_in rate
 * (st_gcnn_dropout); the mask is a counter-based hash of (seed, element) so
 * the backward regenerates it. */
size_t dstd_model_train_saved_bytes(int B, int T, int V, int num_feature, int num_layers);
size_t dstd_model_train_workspace_bytes(int B, int T, int V, int num_feature, int num_layers);
int dstd_model_train_fwd(const dstd_model_params* p, const float* x, int B, float momentum, float dropout_p,
                         unsigned long long seed, float* y, void* saved, size_t saved_bytes, void* stream);
int dstd_model_train_bwd(const dstd_model_params* p, const float* x, int B, float dropout_p,
                         unsigned long long seed, const void* saved, size_t saved_bytes, const float* dy,
                         const dstd_model_grads* g, void* workspace, size_t workspace_bytes, void* stream);

int dstd_model_train_fwd_ex(const dstd_model_params* p, const float* x, int B, float momentum, float dropout_p,
                            unsigned long long seed, float* y, void* saved, size_t saved_bytes, void* stream,
                            unsigned flags);
/* dx (may be NULL): the input gradient [B][T][V][in_channels/2] (=). */
int dstd_model_train_bwd_ex(const dstd_model_params* p, const float* x, int B, float dropout_p,
                            unsigned long long seed, const void* saved, size_t saved_bytes, const float* dy,
                            const dstd_model_grads* g, float* dx, void* workspace, size_t workspace_bytes,
                            void* stream, unsigned flags);

/* ---- cross-rank BatchNorm (SyncBN) for data-parallel training ------------
 * The reference trains with per-process BatchNorm (DDP's default); SURVEY
 * §8(e) names SyncBN for an 8-GPU step equal to the single-GPU one.  With a
 * dstd_bn_sync every train-mode BatchNorm of the model forward normalises with
 * the statistics of ALL ranks' batches (torch.nn.SyncBatchNorm semantics:
 * global mean and biased variance, running statistics from the global
 * unbiased variance), and its backward uses the all-reduced sum(dz) and
 * sum(dz * xhat) for the input gradient while gamma / beta / PReLU slope
 * gradients stay the rank's own (the data-parallel gradient average makes
 * them global).  The library issues no collective itself: at each
 * BatchNorm it calls `fn` on the stream of the call --
 *   op DSTD_COLL_ALLGATHER:     buf holds world x count floats, this rank's
 *                               count at offset rank * count; gather in place;
 *   op DSTD_COLL_ALLREDUCE_SUM: sum count floats in place over the ranks --
 * ordered after the kernels already issued on `stream` and before the ones
 * issued after it returns (RCCL on that stream, or anything synchronous).
 * `fn` returns 0 on success.  buf: device memory of at least
 * dstd_bn_sync_buffer_floats(world, num_feature, V) floats.  DSTD_TRAIN_PAIRED
 * syncs each half's statistics separately.  Pass the same sync to the
 * backward.  NULL sync: per-rank BatchNorm (the _ex entry points). */
#define DSTD_COLL_ALLGATHER 0
#define DSTD_COLL_ALLREDUCE_SUM 1
typedef int (*dstd_collective_fn)(void* ctx, int op, float* buf, long long count, void* stream);
typedef struct dstd_bn_sync {
  int world;
  int rank;
  dstd_collective_fn fn;
  void* ctx;
  float* buf;
  long long buf_floats;
} dstd_bn_sync;
size_t dstd_bn_sync_buffer_floats(int world, int num_feature, int V);
int dstd_model_train_fwd_sync(const dstd_model_params* p, const float* x, int B, float momentum, float dropout_p,
                              unsigned long long seed, float* y, void* saved, size_t saved_bytes, void* stream,
                              unsigned flags, const dstd_bn_sync* sync);
int dstd_model_train_bwd_sync(const dstd_model_params* p, const float* x, int B, float dropout_p,
                              unsigned long long seed, const void* saved, size_t saved_bytes, const float* dy,
                              const dstd_model_grads* g, float* dx, void* workspace, size_t workspace_bytes,
                              void* stream, unsigned flags, const dstd_bn_sync* sync);

/* ---- engine: loss and test metric --------------------------------------- */
size_t dstd_loss_workspace_bytes(void);
/* loss[0] = mean over n_points of ||pred_k - targ_k||_2 (points are xyz triples). */
int dstd_mpjpe_fwd(const float* pred, const float* targ, size_t n_points, float* loss, void* workspace,
                   size_t workspace_bytes, void* stream);
/* dpred (=) (*grad_loss) * scale * d loss / d pred; grad_loss may be NULL (1). */
int dstd_mpjpe_bwd(const float* pred, const float* targ, size_t n_points, const float* grad_loss, float scale,
                   float* dpred, void* stream);
/* PredictionEngine.test metric for one batch: sums[k] += (1/J) sum_{n,j} ||targ - pred||
 * at frame frames[k]; all_seqs [B][T][D], outputs [B][T - t_out0][n_used].
 * used_pos [D] (position of dim d in outputs or -1), joint_src [D/3], frames
 * [n_frames] are device int arrays. */
int dstd_frame_mpjpe(const float* all_seqs, const float* outputs, int B, int T, int D, int t_out0,
                     const int* used_pos, int n_used, const int* joint_src, const int* frames, int n_frames,
                     float* sums, void* stream);

/* Diagnostics: which kernel the last spatial/temporal aggregation backward of
 * this process dispatched -- the channel-chunk kernel's chunk width (16, 32 or
 * 64 channels per workgroup) or 0 for the two-launch path (dF kernel + dD
 * a-chunk kernel); -1 before the first.  Host-side record for tests. */
int dstd_debug_aggb_last(void);

#ifdef __cplusplus
}
#endif
#endif /* DSTD_GCN_TRAIN_H */
