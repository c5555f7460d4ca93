// Internal launcher interface for the encoder/decoder/OLA and PIT kernels.
#pragma once
#include "ctn_kernels.h"

namespace ctn {

struct CodecArgs {
  int M, T, K, Kp, N, L, S, C;
  int mask_type;                 // 0 relu, 1 softmax over speakers, 2 identity (standalone Decoder)
  const float* mixture;          // [M][T]
  const float* U;                // encoder basis [N][L]
  const float* V;                // decoder basis [L][N]
  void* w_rows;                  // encoder output [M*Kp][N]
  float2* cln_stats;             // per-frame (mean, rstd) of w
  const float* gamma0;           // separator cLN gamma (backward)
  const void* gcln;              // dL/d cLN(w) rows (backward)
  const void* gwdec;             // dL/dw from the decoder rows (backward)
  float* gpre;                   // dL/d(pre-ReLU) rows fp32 (backward)
  float* col_slab;               // per-workgroup partials
  const void* score;             // mask-conv output rows [M*Kp][C*N] (pre-nonlinearity)
  float* frames;                 // [M][C][Kp][L]
  float* est;                    // [M][C][T]
  const float* gest;             // dL/dest [M][C][T]
  void* gscore;                  // dL/dscore rows (backward)
  void* gwdec_out;               // dL/dw from the decoder rows (backward)
  // bf16 MFMA decoder backward only: the masked sources w * act(score_c) [rows][C][N]
  // and the frame gradients [rows][C][Lp] (Lp = L rounded up to 8), the two operands
  // of the decoder basis gradient dV = sum_{r,c} gframes^T src (launch_gemm_cols)
  void* src_out = nullptr;
  void* gfr_out = nullptr;
  int Lp = 0;
  // bf16 encoder backward on the column GEMM: dL/d(pre-ReLU) rows in bf16 (instead of
  // the fp32 gpre), the operand of dU = gpre^T . mixture frames
  void* gpre_bf = nullptr;
};
bool codec_dec_mfma(DType dt, const CodecArgs& a);   // the bf16 MFMA decoder applies
hipError_t launch_dec_gframes(const CodecArgs& a, hipStream_t s);   // gfr_out from gest
// bf16 frames [M*Kp*C][Lp] of a signal [M][C][T] (frame k = samples k*S .. k*S+L-1,
// zero past K, T and L): dec_gframes on gest, and the mixture frames of the encoder
hipError_t launch_frames_bf16(const CodecArgs& a, const float* sig, int C, void* out, hipStream_t s);
// out[n][l] = tmp[n][l] for l < L, tmp [N][Lp]
hipError_t launch_unpad_cols(const float* tmp, int N, int Lp, int L, float* out, hipStream_t s);

hipError_t launch_enc_fwd(DType dt, const CodecArgs& a, hipStream_t s);
hipError_t launch_enc_bwd_rows(DType dt, const CodecArgs& a, hipStream_t s);
int frame_outer_chunks(const CodecArgs& a, int C);   // C: rows of sources per frame (encoder 1)
hipError_t launch_frame_outer(DType dt, int mode, const CodecArgs& a, hipStream_t s);
hipError_t launch_dec_fwd(DType dt, const CodecArgs& a, hipStream_t s);
hipError_t launch_dec_bwd(DType dt, const CodecArgs& a, hipStream_t s);

// ---- PIT SI-SNR (pit_criterion.py) ----------------------------------------
struct PitArgs {
  int M, C, T;
  const float* src;              // [M][C][T]
  const float* est;              // [M][C][T]
  const int64_t* lengths;        // [M]
  double* slab;                  // [M][chunks][NV]
  int chunks;
  float* max_snr;                // [M]
  int64_t* best;                 // [M] argmax permutation index
  float* coef;                   // [M][C][4]: alpha, beta, offset, target index
  float* loss;                   // [1]
  const float* g_loss;           // upstream dL/d loss [1] (backward)
  const float* g_maxsnr;         // upstream dL/d max_snr [M] or null (backward)
  float* gest;                   // [M][C][T] (backward)
  float* est_inplace;            // est to mask in place (forward)
  float* reordered;              // [M][C][T]
  double* msd;                   // [M] max_snr in fp64 (C > 4: pit_final_wide -> pit_loss)
  int nperm;
  int perms[24][4];              // lexicographic permutations of range(C) (C <= 4)
};
int pit_nv(int C);
hipError_t launch_pit_forward(const PitArgs& a, hipStream_t s);
hipError_t launch_pit_backward(const PitArgs& a, hipStream_t s);

}  // namespace ctn
