/*
 * ctn.h — C ABI of libctn_hip.so, the MI355X (gfx950) Conv-TasNet hot path.
 *
 * Plain C: device pointers, sizes, a HIP stream passed as void*.  No torch
 * types.  The library never allocates: every scratch buffer is a caller-owned
 * workspace sized by the matching *_workspace_bytes() query, and every output
 * buffer is caller-owned.  Functions are reentrant (no global mutable state
 * except the opt-in kernel timer) and run on the caller's current device.
 * Return value: CTN_OK (0) or a ctn_status error code; ctn_last_error()
 * returns a static description of the last error on the calling thread.
 *
 * Layout convention: frame-major row tensors [M*Kp][C] with
 * channels contiguous, Kp = frames padded to a multiple of 128 per utterance
 * (ctn_padded_frames()); padded rows are zero.  Parameters are fp32 in the
 * reference's own shapes ([out,in,1] conv weights etc.); gradients are
 * written (not accumulated) as fp32 in the same shapes.
 *
 * Each entry names the reference interface it replaces (jwr1995/Conv-TasNet,
 * src/ paths).  The reference binds no FFI: its boundary is the torch.nn.Module
 * API of src/conv_tasnet.py (imported as `from conv_tasnet import ConvTasNet`,
 * src/train.py:12) plus `from pit_criterion import cal_loss`
 * (src/solver.py:9).  The Python drop-in in conv-tasnet_amd/ binds these
 * entries through ctypes.
 */
#ifndef CTN_H
#define CTN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CTN_ABI_VERSION 12

typedef enum { CTN_DTYPE_F32 = 0, CTN_DTYPE_BF16 = 1 } ctn_dtype;
/* CTN_NORM_BN: torch.nn.BatchNorm1d, chose_norm's fallback branch (conv_tasnet.py:302-303) */
typedef enum { CTN_NORM_GLN = 0, CTN_NORM_CLN = 1, CTN_NORM_BN = 2 } ctn_norm_type;
typedef enum { CTN_MASK_RELU = 0, CTN_MASK_SOFTMAX = 1 } ctn_mask_type;
typedef enum {
  CTN_OK = 0,
  CTN_ERR_ARG = 1,          /* invalid argument / shape */
  CTN_ERR_UNSUPPORTED = 2,  /* valid for the reference, not implemented here */
  CTN_ERR_WORKSPACE = 3,    /* workspace smaller than *_workspace_bytes() */
  CTN_ERR_HIP = 4           /* a HIP runtime call failed */
} ctn_status;

int ctn_abi_version(void);
const char* ctn_last_error(void);
/* frames padded to the row-tile multiple used by every kernel (128) */
int ctn_padded_frames(int K);

/* -------------------------------------------------------------------------
 * TemporalBlock: x + DSConv(norm(PReLU(Conv1x1_{B->H}(x))))
 * replaces TemporalBlock.forward, src/conv_tasnet.py:212-238, with
 * DepthwiseSeparableConv :241-272, Chomp1d :275-289, chose_norm :292-303,
 * ChannelwiseLayerNorm :307-329, GlobalLayerNorm :332-355, nn.PReLU :218,253.
 * ------------------------------------------------------------------------- */
typedef struct {
  int32_t M, K, Kp;         /* utterances, frames, padded frames */
  int32_t B, H, P;          /* bottleneck ch., block ch., depthwise kernel size */
  int32_t dilation;         /* 2**x, conv_tasnet.py:175 */
  int32_t causal;           /* 0/1, conv_tasnet.py:176 */
  int32_t norm_type;        /* ctn_norm_type */
  int32_t dtype;            /* ctn_dtype of activations (and MFMA inputs) */
} ctn_tblock_desc;

typedef struct {            /* fp32 device pointers, reference shapes */
  const float* w1;          /* [H,B,1] net.0.weight */
  const float* alpha1;      /* [1]     net.1.weight */
  const float* gamma1;      /* [1,H,1] net.2.gamma */
  const float* beta1;       /* [1,H,1] net.2.beta */
  const float* wd;          /* [H,1,P] net.3.net.0.weight */
  const float* alpha2;      /* [1]     net.3.net.{1|2}.weight */
  const float* gamma2;      /* [1,H,1] net.3.net.{2|3}.gamma */
  const float* beta2;       /* [1,H,1] net.3.net.{2|3}.beta */
  const float* w2;          /* [B,H,1] net.3.net.{3|4}.weight */
  /* optional bf16 compute copies made by ctn_pack_weights (dtype BF16 only; NULL:
   * the call converts w1/w2 itself): W1 [H][B], W2 [B][H] and their transposes */
  const void* w1_bf16;
  const void* w2_bf16;
  const void* w1t_bf16;     /* [B][H] */
  const void* w2t_bf16;     /* [H][B] */
  /* norm_type CTN_NORM_BN only (gamma/beta above = BatchNorm1d weight/bias, [H]):
   * running statistics of net.2 and net.3.net.{2|3} (NULL: none, batch statistics
   * always), updated in place by a training-mode forward with the unbiased batch
   * variance; `bn_momentum` is torch's exponential factor (momentum, or
   * 1/num_batches_tracked when momentum is None) */
  float* bn_mean1;
  float* bn_var1;
  float* bn_mean2;
  float* bn_var2;
  int32_t bn_training;      /* 1: batch statistics (train mode), 0: running statistics */
  float bn_momentum1, bn_momentum2;
  float bn_eps1, bn_eps2;
  /* optional (ABI v6, dtype BF16, B and H multiples of 32): the same four bf16 copies in
   * MFMA fragment order (ctn_weight_pack dst_frag / dst_t_frag), from which the
   * weight-stationary kernels load their resident weight 1 KiB contiguous per wave;
   * NULL: they read the row-major copies above */
  const void* w1_frag;
  const void* w2_frag;
  const void* w1t_frag;
  const void* w2t_frag;
} ctn_tblock_params;

/* One fp32 weight [rows][cols] -> bf16 copy (dst, same layout) and/or bf16
 * transpose (dst_t, [cols][rows]), and (ABI v6) the same two in MFMA fragment order
 * (dst_frag, dst_t_frag; rows and cols multiples of 32): element (n, k) of a [O][I]
 * matrix at ((g*2 + nb)*(I/32) + kb)*512 + lane*8 + e for n = g*32 + ((lane&15)>>2)*8
 * + nb*4 + (lane&3), k = kb*32 + (lane>>4)*8 + e.  Any destination may be NULL. */
typedef struct {
  const float* src;
  int32_t rows, cols;
  void* dst;
  void* dst_t;
  void* dst_frag;
  void* dst_t_frag;
} ctn_weight_pack;
/* Converts n weights in ceil(n / 64) launches (a training step's bf16 weight
 * copies for all TemporalBlocks at once, instead of per block call). */
int ctn_pack_weights(const ctn_weight_pack* packs, int n, void* stream);

typedef struct {            /* fp32 outputs, same shapes as ctn_tblock_params */
  float *w1, *alpha1, *gamma1, *beta1, *wd, *alpha2, *gamma2, *beta2, *w2;
} ctn_tblock_grads;

typedef struct {            /* forward results kept for backward */
  void* h1;                 /* [M*Kp, H] pre-PReLU output of the first 1x1 conv */
  void* d;                  /* [M*Kp, H] pre-PReLU output of the depthwise conv */
  float* stats;             /* [4*G]: (mean,rstd) of norm1 then norm2; G = M (gLN), M*Kp (cLN) or H (BN) */
} ctn_tblock_saved;

int ctn_tblock_stats_floats(const ctn_tblock_desc* d);
size_t ctn_tblock_workspace_bytes(const ctn_tblock_desc* d, int backward);
int ctn_tblock_forward(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x, void* y,
                       const ctn_tblock_saved* saved, void* ws, size_t ws_bytes, void* stream);
int ctn_tblock_backward(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x,
                        const ctn_tblock_saved* saved, const void* gy, void* gx,
                        const ctn_tblock_grads* g, void* ws, size_t ws_bytes, void* stream);
/* ABI v6: the same backward with its parameter-gradient tail on a second stream.  The
 * data-gradient chain (gx) is queued on `stream`; the first 1x1 conv's weight-gradient
 * GEMM and all parameter-gradient reductions wait for an event recorded on `stream`
 * once their inputs exist and run on `wgrad_stream`, so they overlap the previous
 * block's backward on `stream`.  The caller keeps x, ws and the gradient outputs alive
 * and unmodified until `wgrad_stream` has finished this call's work, and orders the
 * consumers of g after it (norm_type BN: everything on `stream`). */
int ctn_tblock_backward_split(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x,
                              const ctn_tblock_saved* saved, const void* gy, void* gx,
                              const ctn_tblock_grads* g, void* ws, size_t ws_bytes, void* stream,
                              void* wgrad_stream);

/* ABI v8: the same backward with every parameter-gradient reduction left for later, so
 * that one call can reduce all blocks of a backward pass (a few launches instead of two
 * per block).  The fixed-order partial sums go to `part` (ctn_tblock_partials_bytes(d)
 * bytes; ws then needs only ctn_tblock_deferred_workspace_bytes(d)); the gradients in
 * `g` are NOT written by this call.  gLN / cLN blocks only (BN: CTN_ERR_UNSUPPORTED).
 * Replaces, for a whole backward pass, the per-block gradient writes of the reference's
 * TemporalBlock backward (src/conv_tasnet.py:217-263, autograd).                       */
size_t ctn_tblock_partials_bytes(const ctn_tblock_desc* d);
size_t ctn_tblock_deferred_workspace_bytes(const ctn_tblock_desc* d);
int ctn_tblock_backward_deferred(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x,
                                 const ctn_tblock_saved* saved, const void* gy, void* gx,
                                 const ctn_tblock_grads* g, void* ws, size_t ws_bytes, void* part,
                                 size_t part_bytes, void* stream);
/* Write the gradients g[i] of n deferred block backwards from their partials parts[i]
 * (each part[i] unmodified since its ctn_tblock_backward_deferred call; descs[i] the same
 * descriptor).  Bit-identical to the per-block reductions of ctn_tblock_backward.       */
int ctn_tblock_reduce_grads(const ctn_tblock_desc* descs, const ctn_tblock_grads* g, void* const* parts, int n,
                            void* stream);

/* -------------------------------------------------------------------------
 * Front of the network: Encoder (src/conv_tasnet.py:97-117: ReLU(Conv1d(1,N,L,
 * stride L/2))) + the TemporalConvNet input cLN (:167, :307-329) + bottleneck
 * 1x1 conv N->B (:169).  wb == NULL: encoder only (standalone Encoder).
 * Back of the network: mask 1x1 conv B->C*N (:185), mask nonlinearity
 * (:202-208), Decoder (:120-142), overlap_and_add (src/utils.py:9-46) and the
 * F.pad to T (:56-59).  wm == NULL: standalone Decoder, `x_last` then holds
 * the mask rows [M*Kp, C*N] and mask_type must be CTN_MASK_IDENTITY.
 * ------------------------------------------------------------------------- */
#define CTN_MASK_IDENTITY 2
typedef struct {
  int32_t M, T, K, Kp;      /* utterances, samples, frames = (T-L)/(L/2)+1, padded frames */
  int32_t N, L, B, C;       /* encoder filters, filter length, bottleneck ch., speakers */
  int32_t mask_type;        /* ctn_mask_type or CTN_MASK_IDENTITY */
  int32_t dtype;            /* ctn_dtype of activations */
} ctn_codec_desc;

size_t ctn_encoder_workspace_bytes(const ctn_codec_desc* d, int backward);
int ctn_encoder_forward(const ctn_codec_desc* d, const float* mixture, const float* U, const float* gamma0,
                        const float* beta0, const float* wb, void* w_rows, float* cln_stats, void* x0,
                        void* ws, size_t ws_bytes, void* stream);
int ctn_encoder_backward(const ctn_codec_desc* d, const float* mixture, const float* U, const float* gamma0,
                         const float* beta0, const float* wb, const void* w_rows, const float* cln_stats,
                         const void* g_w_rows, const void* g_x0, float* gU, float* ggamma0, float* gbeta0,
                         float* gwb, void* ws, size_t ws_bytes, void* stream);

size_t ctn_decoder_workspace_bytes(const ctn_codec_desc* d, int backward);
int ctn_decoder_forward(const ctn_codec_desc* d, const void* x_last, const void* w_rows, const float* wm,
                        const float* V, void* score, float* est, void* ws, size_t ws_bytes, void* stream);
int ctn_decoder_backward(const ctn_codec_desc* d, const void* x_last, const void* w_rows, const float* wm,
                         const float* V, const void* score, const float* g_est, void* g_x_last, void* g_w_rows,
                         float* gwm, float* gV, void* ws, size_t ws_bytes, void* stream);

/* -------------------------------------------------------------------------
 * PIT SI-SNR loss: replaces cal_loss / cal_si_snr_with_pit / reorder_source /
 * get_mask, src/pit_criterion.py:12-113.  `est` is masked in place beyond
 * each length (:37-38); `reordered` (nullable) keeps the reference's
 * perm-not-inverse indexing (:91-97).  `coef` [M*C*4] is saved for backward.
 * 1 <= C <= 16 (0 workspace bytes / CTN_ERR_UNSUPPORTED beyond): C <= 10 searches all C!
 * permutations (:66) and keeps the first maximum (torch.argmax); 11 <= C <= 16, past what
 * the reference's C!-row one-hot table can hold, solves the same maximum as a linear
 * assignment (Hungarian, fp64) and reports its lexicographic rank in best_perm (exact ties
 * may pick another optimal permutation).  The encoder/decoder descriptors accept 1..16
 * (streaming: 1..8).
 * ------------------------------------------------------------------------- */
typedef struct { int32_t M, C, T; } ctn_pit_desc;
size_t ctn_pit_workspace_bytes(const ctn_pit_desc* d);
int ctn_pit_forward(const ctn_pit_desc* d, const float* source, float* est, const int64_t* lengths, float* loss,
                    float* max_snr, int64_t* best_perm, float* reordered, float* coef, void* ws, size_t ws_bytes,
                    void* stream);
int ctn_pit_backward(const ctn_pit_desc* d, const float* source, const float* est, const int64_t* lengths,
                     const float* coef, const float* g_loss, const float* g_max_snr, float* g_est, void* stream);

/* -------------------------------------------------------------------------
 * Parameter update: replaces torch.nn.utils.clip_grad_norm_(params, max_norm)
 * (src/solver.py:184-185) and torch.optim.Adam(params, lr, weight_decay=l2)
 * (src/train.py:129-133, stepped at src/solver.py:186) with one launch each
 * over ALL parameter tensors.  A segment describes one parameter tensor (fp32
 * device pointers; exp_avg/exp_avg_sq may be NULL for clipping); the chunk
 * table (ctn_opt_plan, host memory, copied to the device by the caller) cuts
 * the segments into workgroup pieces.  Rebuild the plan whenever a pointer or
 * size changes.
 * ------------------------------------------------------------------------- */
typedef struct {
  float* param;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
} ctn_opt_segment;
typedef struct { int32_t seg; uint32_t len; int64_t off; } ctn_opt_chunk;
typedef struct {
  float lr, beta1, beta2, eps, weight_decay;
  int32_t step;   /* 1-based step count after the increment (bias correction) */
} ctn_adam_hparams;

/* segs: host copy of the segment table.  Returns the number of chunks (writes
 * up to max_chunks entries when chunks != NULL), or a negative ctn_status. */
int ctn_opt_plan(const ctn_opt_segment* segs, int nseg, ctn_opt_chunk* chunks, int max_chunks);
/* grads *= min(1, max_norm / (||grads||_2 + 1e-6)); *total_norm = ||grads||_2 (device).
 * segs/chunks: device tables; partial: device scratch of nchunks floats. */
int ctn_grad_clip_norm(const ctn_opt_segment* segs, const ctn_opt_chunk* chunks, int nchunks, float max_norm,
                       float* total_norm, float* partial, void* stream);
/* one Adam step of every segment (param, exp_avg, exp_avg_sq updated in place); the bias
 * corrections of step hp->step are computed on the device in fp64 (ABI v12) */
int ctn_adam_step(const ctn_opt_segment* segs, const ctn_opt_chunk* chunks, int nchunks, const ctn_adam_hparams* hp,
                  void* stream);

/* Graph capture (ABI v10; torch.optim.Adam(capturable=True) semantics, hipGraph / torch
 * CUDA-graph capture of a whole training step).  No call below reads host memory at
 * launch time from the device, so a captured launch replays correctly:
 *  - ctn_opt_write_segments: writes n segment entries to the device table `dst` with
 *    kernels whose arguments carry the entries (no host staging buffer);
 *  - ctn_adam_step_dev (ABI v12): Adam with the step count in device memory: step
 *    t = *counter + 1, then a second kernel increments *counter; lr = *lr_dev when lr_dev
 *    is not NULL (a schedule writes it between replays), else hp->lr.  The bias
 *    corrections lr / (1 - beta1^t) and sqrt(1 - beta2^t) are computed on the device in
 *    fp64 by the same code as ctn_adam_step's (same bits for the same t and lr), with no
 *    step limit (ABI v10-11 read them from a host-built table of 2^20 steps).
 * hp->step is not read by ctn_adam_step_dev. */
int ctn_opt_write_segments(ctn_opt_segment* dst, const ctn_opt_segment* src, int n, void* stream);
int ctn_adam_step_dev(const ctn_opt_segment* segs, const ctn_opt_chunk* chunks, int nchunks,
                      const ctn_adam_hparams* hp, const float* lr_dev, int32_t* counter, void* stream);

/* -------------------------------------------------------------------------
 * Stand-alone separator layers on frame rows [M*Kp][C] (ABI v4): what the fused
 * calls above run inside themselves, exposed for the reference's module
 * forwards called on their own — TemporalConvNet.forward (src/conv_tasnet.py:
 * 192-209), DepthwiseSeparableConv.forward (:265-272), ChannelwiseLayerNorm.
 * forward (:319-329), GlobalLayerNorm.forward (:344-355) — each with its
 * backward.  Gradients are written, not accumulated.
 * ------------------------------------------------------------------------- */
typedef struct {
  int32_t M, K, Kp;         /* utterances, frames, padded frames */
  int32_t C;                /* channels of the input rows */
  int32_t dtype;            /* ctn_dtype of activations */
} ctn_rows_desc;

/* gLN / cLN (norm_type CTN_NORM_GLN / CTN_NORM_CLN; EPS 1e-8 inside the sqrt,
 * biased variance, conv_tasnet.py:10,327,353); gamma/beta [1,C,1]; stats
 * [G][2] (mean, rstd), G = M (gLN) or M*Kp (cLN), written by forward */
size_t ctn_layernorm_workspace_bytes(const ctn_rows_desc* d, int norm_type, int backward);
int ctn_layernorm_forward(const ctn_rows_desc* d, int norm_type, const void* x, const float* gamma,
                          const float* beta, void* y, float* stats, void* ws, size_t ws_bytes, void* stream);
int ctn_layernorm_backward(const ctn_rows_desc* d, int norm_type, const void* x, const float* gamma,
                           const float* stats, const void* gy, void* gx, float* ggamma, float* gbeta, void* ws,
                           size_t ws_bytes, void* stream);

/* nn.PReLU() with one shared alpha (conv_tasnet.py:218,253); alpha [1] */
size_t ctn_prelu_workspace_bytes(const ctn_rows_desc* d);
int ctn_prelu_forward(const ctn_rows_desc* d, const void* x, const float* alpha, void* y, void* stream);
int ctn_prelu_backward(const ctn_rows_desc* d, const void* x, const float* alpha, const void* gy, void* gx,
                       float* galpha, void* ws, size_t ws_bytes, void* stream);

/* depthwise Conv1d(C, C, P, dilation, groups=C, bias=False) with the reference's
 * padding (conv_tasnet.py:188,262-265) and, causal, its Chomp1d (:275-289);
 * w [C,1,P]; non-causal needs (P-1)*dilation even (output length K) */
size_t ctn_depthwise_workspace_bytes(const ctn_rows_desc* d, int P);
int ctn_depthwise_forward(const ctn_rows_desc* d, int P, int dilation, int causal, const void* x, const float* w,
                          void* y, void* stream);
int ctn_depthwise_backward(const ctn_rows_desc* d, int P, int dilation, int causal, const void* x, const float* w,
                           const void* gy, void* gx, float* gw, void* ws, size_t ws_bytes, void* stream);

/* Conv1d(C, cout, 1, bias=False) (conv_tasnet.py:169,185,215,270); w [cout,C,1];
 * C and cout multiples of 8 */
size_t ctn_conv1x1_workspace_bytes(const ctn_rows_desc* d, int cout, int backward);
int ctn_conv1x1_forward(const ctn_rows_desc* d, int cout, const void* x, const float* w, void* y, void* ws,
                        size_t ws_bytes, void* stream);
int ctn_conv1x1_backward(const ctn_rows_desc* d, int cout, const void* x, const float* w, const void* gy, void* gx,
                         float* gw, void* ws, size_t ws_bytes, void* stream);

/* mask nonlinearity (conv_tasnet.py:202-208) over nspk speakers of score rows
 * [M*Kp][nspk*N] (d->C = nspk*N, channel s*N + n as score.view(M, C, N, K)) */
int ctn_mask_forward(const ctn_rows_desc* d, int nspk, int mask_type, const void* score, void* mask, void* stream);
int ctn_mask_backward(const ctn_rows_desc* d, int nspk, int mask_type, const void* score, const void* gmask,
                      void* gscore, void* stream);

/* -------------------------------------------------------------------------
 * Streaming causal separation: replaces running src/separate.py:35-79 on a
 * causal model (conv_tasnet.py:176 Chomp1d, :289) whole-signal, with chunked
 * calls that carry state instead of re-running history.  fp32.
 * Frame k of a stream covers samples [k*L/2, k*L/2 + L).  State per
 * TemporalBlock: `ring` [M][ring_frames][H], the block's depthwise-conv input
 * frames (after conv1x1, PReLU and norm 1), frame g at slot g % ring_frames;
 * ring_frames a power of two >= (P-1)*dilation + K.  `pos` = frames of this
 * stream processed before the call (taps before frame 0 read as zero: the
 * reference's causal zero padding).  1x1 weights are passed TRANSPOSED,
 * [in][out]: wb_t [N][B], w1_t [B][H], w2_t [H][B], wm_t [B][C*N]; wd [H][P];
 * U [N][L]; V [L][N] (Linear(N, L).weight).  norm CTN_NORM_CLN takes
 * gamma/beta, CTN_NORM_BN an eval-mode BatchNorm folded to scale/shift.
 * encode: samples [M][ld] (the call's (K-1)*L/2 + L samples at offset 0)
 *         -> w_out [M][K][N] (ReLU(U*frame)), x_out [M][K][B] (cLN, bottleneck)
 * block : x_in [M][K][B] -> ring (new frames), x_out [M][K][B]
 * decode: x_last, w -> out [M][C][K*L/2]: the K frames overlap-added with
 *         tail_in [M][C][L/2] (zeros at the stream start); tail_out gets the
 *         last frame's second half.  frames_ws: [M][C][K][L] scratch.
 * ------------------------------------------------------------------------- */
typedef struct {
  int32_t M, K;
  int32_t N, L, B, H, P, C;
  int32_t norm;      /* CTN_NORM_CLN or CTN_NORM_BN (eval, affine) */
  int32_t mask_type; /* ctn_mask_type or CTN_MASK_IDENTITY */
} ctn_stream_desc;
int ctn_stream_encode(const ctn_stream_desc* d, const float* samples, int64_t ld_samples, const float* U,
                      const float* gamma0, const float* beta0, const float* wb_t, float* w_out, float* x_out,
                      void* stream);
int ctn_stream_block(const ctn_stream_desc* d, int dilation, int64_t pos, int ring_frames, const float* x_in,
                     const float* w1_t, const float* alpha1, const float* norm1_a, const float* norm1_b,
                     const float* wd, const float* alpha2, const float* norm2_a, const float* norm2_b,
                     const float* w2_t, float* ring, float* x_out, void* stream);
int ctn_stream_decode(const ctn_stream_desc* d, const float* x_last, const float* w, const float* wm_t,
                      const float* V, const float* tail_in, float* tail_out, float* frames_ws, float* out,
                      void* stream);

/* ABI v7: one whole call (encode, every TemporalBlock, decode) in one entry, its 1x1
 * convs split over 32-output column chunks so that a call with few new frames spreads
 * over many CUs (the v5 entries give each (stream, 8 frames) one workgroup that streams
 * every 1x1 weight through one CU).  Same state and layouts as the v5 entries; `blocks`
 * is a HOST array of nblocks per-block parameter sets (separator order), each with its
 * own ring.  `pos` as above; `tail_in` / `tail_out` [M][C][L/2] must not alias.
 * `ws` >= ctn_stream_workspace_bytes(d).  Same arithmetic as the v5 path (the 1x1 sums
 * are added in another order: results agree to fp32 rounding). */
typedef struct {
  int32_t dilation, ring_frames;
  const float* w1_t;     /* [B][H] */
  const float* alpha1;
  const float* norm1_a;
  const float* norm1_b;
  const float* wd;       /* [H][P] */
  const float* alpha2;
  const float* norm2_a;
  const float* norm2_b;
  const float* w2_t;     /* [H][B] */
  float* ring;           /* [M][ring_frames][H] */
} ctn_stream_block_params;
typedef struct {
  const float* U;        /* [N][L] */
  const float* gamma0;   /* separator cLN */
  const float* beta0;
  const float* wb_t;     /* [N][B] */
  const float* wm_t;     /* [B][C*N] */
  const float* V;        /* [L][N] */
  const ctn_stream_block_params* blocks;
  int32_t nblocks;
} ctn_stream_model;
size_t ctn_stream_workspace_bytes(const ctn_stream_desc* d);
int ctn_stream_call(const ctn_stream_desc* d, const ctn_stream_model* model, int64_t pos, const float* samples,
                    int64_t ld_samples, const float* tail_in, float* tail_out, float* out, void* ws,
                    size_t ws_bytes, void* stream);

/* Kernel plan of one TemporalBlock launch (no device work): writes a NUL-terminated list
 * "step=kernel,..." of the kernels ctn_tblock_forward (backward = 0) or the backward entries
 * (backward = 1) would choose for d, e.g. "pairA=dual_ws,dw_bwd=wave,gx=ws_n1bwd,dW1=cols".
 * Shapes outside a kernel's limits (tensors of 2^31 bytes or more for the persistent
 * kernels' 32-bit offsets) fall back to the tiled kernels; this is how a caller sees it. */
int ctn_tblock_plan(const ctn_tblock_desc* d, int backward, char* out, size_t cap);

/* -------------------------------------------------------------------------
 * Opt-in kernel timer (bench.py roofline; the reference has no counterpart — its
 * solver prints epoch wall time only, src/solver.py:178-188): when enabled, every
 * launch of a selected kernel family is bracketed by hipEvents on its stream.
 * Kinds of the TemporalBlock (conv_tasnet.py:212-272):
 * ------------------------------------------------------------------------- */
enum {
  CTN_TIMER_GEMM1 = 1,     /* forward first 1x1 (B -> H, PReLU-statistics epilogue)       */
  CTN_TIMER_DW_FWD = 2,    /* depthwise forward (norm 1 applied, PReLU-2 statistics)      */
  CTN_TIMER_GEMM_A = 3,    /* backward pair A: g_n2 = gy.W2 (+ dW2 on the dual kernel)     */
  CTN_TIMER_DW_BWD = 4,    /* depthwise backward (norm-2 / PReLU-2 backward, dW_dw, sums)  */
  CTN_TIMER_GEMM_GX = 5,   /* backward gx = n1bwd(g).W1 + gy (stores dL/dh1)              */
  CTN_TIMER_COLS_W1 = 6,   /* backward dW1 = (dL/dh1)^T . x column GEMM                   */
  CTN_TIMER_GEMM2 = 7      /* forward second 1x1 (H -> B, norm 2 applied, residual)       */
};
/* one kind (0 = off), or a set of kinds (bit k = kind k; max_launches per kind) */
int ctn_timer_enable(int kind, int max_launches);
int ctn_timer_enable_mask(uint32_t mask, int max_launches);
int ctn_timer_read(double* total_ms, int* launches);              /* all kinds */
int ctn_timer_read_kind(int kind, double* total_ms, int* launches);
/* ABI v11: bracket only every stride-th launch of each enabled kind (stride >= 1,
 * default 1; counted from the last enable).  Each bracketing event pair leaves the GPU
 * idle for a few microseconds around the launch, so a sampled timer perturbs the
 * measured run less; read_kind then reports the sampled launches. */
int ctn_timer_set_stride(int stride);
/* ABI v11: a streaming device-to-device copy (16 B per lane, `workgroups` x 256 threads,
 * grid-stride), bench.py's measured bandwidth ceiling beside the datasheet peak.  bytes,
 * dst and src must be multiples of 16.  flags: bit 0 nontemporal loads and stores, bit 1
 * eight loads in flight per lane instead of four. */
#define CTN_COPY_NT 1
#define CTN_COPY_DEEP 2
int ctn_copy_bytes(void* dst, const void* src, size_t bytes, int workgroups, int flags, void* stream);
/* ABI v12: an MFMA throughput microbenchmark (bench.py's measured matrix peak beside the
 * 2.5 PF/s datasheet value): `workgroups` x 4 waves, each issuing `iters` rounds of
 * independent back-to-back bf16 MFMAs on random register operands — shape 0
 * v_mfma_f32_16x16x32_bf16 (8 accumulators), 1 v_mfma_f32_32x32x16_bf16 (4) — writing
 * workgroups*256 floats to `out`; *flops (may be NULL) = the FLOP of the launch. */
int ctn_mfma_peak(int shape, int workgroups, int iters, float* out, double* flops, void* stream);

/* -------------------------------------------------------------------------
 * Device error word (ABI v9).  Kernels whose waves hand tiles to each other through
 * LDS generation words (the wave-specialised dual GEMM of ctn_tblock_backward*, the
 * ring variant of the weight-stationary GEMM) bound every wait; a wait that runs out
 * sets bit CTN_DEVERR_SPIN and the launch's outputs are invalid.  The word is copied
 * to the host asynchronously at the end of every ctn_tblock_reduce_grads, which fails
 * with CTN_ERR_HIP at its next call once a bit is set.  ctn_device_status
 * synchronises `stream`, returns the word in *word (may be NULL) and CTN_ERR_HIP when
 * it is non-zero; clear != 0 resets it.
 * ------------------------------------------------------------------------- */
#define CTN_DEVERR_SPIN 1u
int ctn_device_status(void* stream, uint32_t* word, int clear);

#ifdef __cplusplus
}
#endif
#endif /* CTN_H */
