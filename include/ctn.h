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

#define CTN_ABI_VERSION 1

typedef enum { CTN_DTYPE_F32 = 0, CTN_DTYPE_BF16 = 1 } ctn_dtype;
typedef enum { CTN_NORM_GLN = 0, CTN_NORM_CLN = 1 } ctn_norm_type;
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
} ctn_tblock_params;

typedef struct {            /* fp32 outputs, same shapes as ctn_tblock_params */
  float *w1, *alpha1, *gamma1, *beta1, *wd, *alpha2, *gamma2, *beta2, *w2;
} ctn_tblock_grads;

typedef struct {            /* forward results kept for backward */
  void* h1;                 /* [M*Kp, H] pre-PReLU output of the first 1x1 conv */
  void* d;                  /* [M*Kp, H] pre-PReLU output of the depthwise conv */
  float* stats;             /* [4*G]: (mean,rstd) of norm1 then norm2; G = M (gLN) or M*Kp (cLN) */
} ctn_tblock_saved;

int ctn_tblock_stats_floats(const ctn_tblock_desc* d);
size_t ctn_tblock_workspace_bytes(const ctn_tblock_desc* d, int backward);
int ctn_tblock_forward(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x, void* y,
                       const ctn_tblock_saved* saved, void* ws, size_t ws_bytes, void* stream);
int ctn_tblock_backward(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x,
                        const ctn_tblock_saved* saved, const void* gy, void* gx,
                        const ctn_tblock_grads* g, void* ws, size_t ws_bytes, void* stream);

/* -------------------------------------------------------------------------
 * Opt-in kernel timer (bench.py roofline): when enabled, every launch of the
 * selected kernel family is bracketed by hipEvents on its stream.
 * kind: 0 off, 1 block-forward first 1x1 GEMM, 2 depthwise forward,
 *       3 block-backward data GEMM (norm-backward epilogue)
 * ------------------------------------------------------------------------- */
int ctn_timer_enable(int kind, int max_launches);
int ctn_timer_read(double* total_ms, int* launches);

#ifdef __cplusplus
}
#endif
#endif /* CTN_H */
