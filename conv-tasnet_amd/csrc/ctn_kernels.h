// Internal (C++) launcher interface between the kernel files and the C-ABI
// layer (ctn_capi.hip).  Not part of the public ABI: see include/ctn.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ctn_common.h"

namespace ctn {

enum DType { F32 = 0, BF16 = 1 };

// The current device's error word (ctn_capi.hip: allocated and zeroed on first use, read by
// ctn_device_status / ctn_tblock_reduce_grads).  Kernels whose waves hand tiles to each
// other through LDS generation words set CTN_DEVERR_SPIN in it when a wait runs out.
uint32_t* device_error_word();
// OP_NORM1_BWD (bf16, gLN; WS kernel, the first 1x1's data gradient): the operand
// is g = dL/d(hat a1) and becomes dL/dh1 = PReLU'(h1) * rstd * (g - mean g - hat a1 *
// mean(g hat a1)) on the way into LDS (conv_tasnet.py:217-219 backward), with
// h1 = `aux`, (mean, rstd) = `stats`, the two means = `sums` or `fold`; dL/dh1 is
// also stored (`aout`) for the weight-gradient kernel.
enum RowOpKind { OP_PLAIN = 0, OP_NORM = 1, OP_PRELU_NORM = 2, OP_NORM1_BWD = 3 };
enum EpiKind { EPI_STORE = 0, EPI_PRELU_STATS = 1, EPI_RESID = 2, EPI_NORM_BWD = 3 };

// element-wise transform applied to an operand row while it is staged into LDS
struct RowOp {
  int kind = OP_PLAIN;       // RowOpKind
  int norm = 0;              // NormKind of `stats` (0 gLN per utterance, 1 cLN per row)
  const float2* stats = nullptr;   // (mean, rstd)
  const float* gamma = nullptr;
  const float* beta = nullptr;
  const float* alpha = nullptr;    // PReLU alpha (device pointer, 1 element)
  StatFold fold;                   // gLN: finalize `stats` (OP_NORM1_BWD: `sums`) in the consumer (WS kernel only)
  // OP_NORM1_BWD only
  const void* aux = nullptr;       // h1, same layout as the operand
  const float2* sums = nullptr;    // (mean g, mean g*hat a1) per utterance, when not folded
  void* aout = nullptr;            // WS kernel: the transformed operand dL/dh1 is stored here too
  float* apart = nullptr;          // WS kernel: one PReLU-alpha gradient partial per workgroup
};

// Geometry of a frame-row tensor set: rows = M * Kp, valid frames K per utterance.
struct Rows {
  int M, K, Kp;
  __host__ __device__ long rows() const { return (long)M * Kp; }
};

// ---- row GEMM:  C[r][n] = sum_k op(A[r][k]) * W[n][k]  (+ epilogue) ---------
struct GemmRows {
  Rows g;
  int Kred, Nout;
  const void* A; int lda;
  const void* W; int ldw;      // [Nout][Kred], storage type
  const void* Wf;              // optional bf16 copy of W in MFMA fragment order (frag_offset)
  RowOp aop;
  int epi = EPI_STORE;
  void* C; int ldc;
  const void* R = nullptr; int ldr = 0;   // residual (EPI_RESID) or pre-activation (EPI_NORM_BWD)
  // EPI_NORM_BWD: C = gn = A.W^T (the gradient w.r.t. the norm output, padded rows 0);
  // group sums of (gn*gamma, gn*gamma*hat a) with hat a = (PReLU(R) - mean) * rstd.
  // The gamma/beta gradients are accumulated by the depthwise backward kernel.
  const float* alpha = nullptr;           // PReLU alpha for the epilogue
  const float2* stats = nullptr;          // EPI_NORM_BWD forward stats
  const float* gamma = nullptr;           // EPI_NORM_BWD gamma
  int norm = 0;                           // NormKind for the epilogue statistics
  double2* grp_slab = nullptr;            // group partials
  // EPI_PRELU_STATS, cLN, WS kernel (gemm_ws_final_cln): per-row (mean, rstd) of the
  // output written here directly (the workgroup holds every channel of its rows)
  float2* stats_out = nullptr;
  float eps = 0.f;
  uint32_t* err = nullptr;                // device error word (ring hand-off timeouts), set by the launcher
};
// Slab sizing must be queried with the same GemmRows (shape, operand op, epilogue,
// strides) that is later launched: the kernel choice decides the part counts.
int gemm_rows_tiles_per_group(DType dt, const GemmRows& p);   // grp_slab parts per group
hipError_t launch_gemm_rows(DType dt, const GemmRows& p, hipStream_t s);
// weight-stationary persistent kernel (ctn_gemm_ws.hip), chosen by launch_gemm_rows
bool gemm_ws_eligible(DType dt, const GemmRows& p);
int gemm_ws_grid(const GemmRows& p);
int gemm_ws_group_parts(const GemmRows& p);
WsRuns gemm_ws_runs(const GemmRows& p);
// StatFold for the group partials p's epilogue writes (WS run layout or dense)
StatFold gemm_rows_stat_fold(DType dt, const GemmRows& p, const double2* slab, double cnt, float eps, int mode,
                             float2* out);
bool gemm_ws_can_fold(DType dt, const GemmRows& p);   // WS kernel and its operand stats fit the fold
bool gemm_ws_final_cln(DType dt, const GemmRows& p);  // WS kernel writes final cLN stats (stats_out)
hipError_t launch_gemm_ws(const GemmRows& p, hipStream_t s);

// ---- column GEMM (weight gradient): Cpart[chunk][p][q] = sum_r opA(A[r][p]) * opB(B[r][q])
struct GemmCols {
  Rows g;
  int P, Q;
  const void* A; int lda; RowOp aop;
  const void* B; int ldb; RowOp bop;
  float* Cpart;                // [nchunks][P][Q]
  int nchunks;
};
int gemm_cols_default_chunks(const GemmCols& p);
hipError_t launch_gemm_cols(DType dt, const GemmCols& p, hipStream_t s);

// ---- dual GEMM (ctn_gemm_dual.hip): a row GEMM and the weight gradient that shares
// its A stream, in one pass:  C[r][n] = sum_k A[r][k] W[n][k] (+ EPI_RESID / EPI_NORM_BWD
// epilogue, fields as GemmRows) and Dpart[range][k][n] = sum_{r in range} A[r][k] op(Bm[r][n]).
struct GemmDual {
  Rows g;
  int Kred, Nout;
  const void* A; int lda;
  const void* W; int ldw;
  const void* Wf;              // optional fragment-ordered bf16 copy of W (frag_offset)
  int epi = EPI_RESID;
  void* C; int ldc;
  const void* R = nullptr; int ldr = 0;
  const float* alpha = nullptr;
  const float2* stats = nullptr;
  const float* gamma = nullptr;
  int norm = 0;
  double2* grp_slab = nullptr;
  const void* Bm; int ldb;
  RowOp bop;                   // OP_PLAIN or OP_PRELU_NORM with final statistics
  float* Dpart;                // [gemm_dual_ranges][Kred][Nout]
  uint32_t* err = nullptr;     // device error word (generation-word timeouts), set by the launcher
};
bool gemm_dual_eligible(DType dt, const GemmDual& p);
int gemm_dual_ranges(const GemmDual& p);
int gemm_dual_group_parts(const GemmDual& p);
int dual_ws_cln_parts_per_slice();   // ctn_dual_ws.hip: cLN statistics entries per (row, slice)
int dual_ws_row_waves(const GemmDual& p);   // ctn_dual_ws.hip: row waves per slice (gLN partials)
StatFold gemm_dual_stat_fold(const GemmDual& p, const double2* slab, double cnt, float eps, int mode,
                             float2* out);
hipError_t launch_gemm_dual(const GemmDual& p, hipStream_t s);
// wave-specialised pair-A kernel (ctn_dual_ws.hip), chosen by launch_gemm_dual
bool gemm_dual_ws_enabled();
bool gemm_dual_ws_eligible(const GemmDual& p);
int gemm_dual_ws_ranges(const GemmDual& p);
hipError_t launch_gemm_dual_ws(const GemmDual& p, hipStream_t s);
// the same kernel's column part alone for plain bf16 column GEMMs (dW1 = gh1^T . x):
// chosen by launch_gemm_cols when nchunks == gemm_cols_ws_ranges (gemm_cols_chunks)
bool gemm_cols_ws_eligible(DType dt, const GemmCols& c);
int gemm_cols_ws_ranges(const GemmCols& c);
hipError_t launch_gemm_cols_ws(const GemmCols& c, hipStream_t s);
int gemm_cols_chunks(DType dt, const GemmCols& c);   // partial count the launch will use

// ---- statistics ------------------------------------------------------------
// slab: [G][nparts] double2 partials -> out[G] float2
//   mode 0: (mean, rstd) with biased variance, eps inside the sqrt
//   mode 1: (S1 / cnt, S2 / cnt)
hipError_t launch_stats_finalize(const double2* slab, int G, int nparts, double cnt, int mode,
                                 float eps, float2* out, hipStream_t s);

struct SlabDesc {
  const float* src;   // parts laid out with stride `pstride` floats
  float* dst;
  int nparts, n, pstride;
};
struct SlabBatch {
  SlabDesc d[12];
  int nd;
};
size_t slab_reduce_tmp_floats(const SlabBatch& b);
hipError_t launch_slab_reduce(const SlabBatch& b, float* tmp, hipStream_t s);   // tmp may be null (1 pass)
void slab_reduce_assign_tmp(const SlabDesc* d, int n, float* tmp, float** out);
// any number of descriptors, tmps[i] = descriptor i's scratch (null: one pass)
hipError_t launch_slab_reduce_list(const SlabDesc* d, float* const* tmps, int n, hipStream_t s);
hipError_t launch_copy_stream(void* dst, const void* src, size_t bytes, int wgs, int flags, hipStream_t s);   // 16-B aligned
// MFMA throughput microbenchmark (ctn_mfma_peak): *flops = the FLOP the launch performs
hipError_t launch_mfma_peak(int shape, int wgs, int iters, float* out, double* flops, hipStream_t s);

// fp32 weight [O][I] -> storage-type copy (Ws, [O][I]) and/or transpose (Wt, [I][O])
hipError_t launch_prep_weight(DType dt, const float* W, int O, int I, void* Ws, void* Wt,
                              hipStream_t s);
struct PrepDesc {
  const float* W;
  int O, I;
  void* Ws;
  void* Wt;
  void* Wf;    // W in fragment order (O, I multiples of 32), or null
  void* Wtf;   // the transpose [I][O] in fragment order, or null
};
// Fragment order of a bf16 weight W [O][I] (O, I multiples of 32): the 16-byte piece
// that lane L of output group g (32 rows) holds as MFMA A-fragment (nb, kb) of the
// weight-stationary kernels (2 fragments of 16 rows per group: rows g*32 + ((L&15)>>2)*8
// + nb*4 + (L&3), columns kb*32 + (L>>4)*8 .. +8) sits at element offset
// ((g*2 + nb)*(I/32) + kb)*512 + L*8, so every wave's fragment load is 1 KiB contiguous.
__host__ __device__ inline long frag_offset(int g, int nb, int kb, int lane, int I) {
  return (((long)g * 2 + nb) * (I / 32) + kb) * 512 + lane * 8;
}
constexpr int PREP_MAX = 64;   // descriptors per launch (kernel-argument budget)
struct PrepBatch {
  PrepDesc d[PREP_MAX];
  int nd;
};
hipError_t launch_prep_weights(DType dt, const PrepBatch& pb, hipStream_t s);   // one launch

// ---- depthwise + norm element-wise kernels ---------------------------------
struct DwArgs {
  Rows g;
  int H, P, dil, pad;
  int norm;                              // NormKind of both block norms
  int seg;                               // comb steps per work item (dw_seg)
  const void* h1;                        // pre-PReLU output of the block's first 1x1 conv
  const void* d;                         // pre-PReLU output of the depthwise conv (bwd)
  const float2* st1; const float2* st2;  // forward (mean, rstd)
  const float* alpha1; const float* gamma1; const float* beta1;
  const float* alpha2; const float* gamma2;
  const float* wd;                       // [H][P]
  // fwd
  void* d_out;
  double2* slab2;                        // stats partial of prelu(d)
  // bwd
  const void* ga2;                       // bwd: g_n2 = dL/d(norm2 output); dL/d(hat a2) = g_n2 * gamma2
  const float2* sm2;                     // (mean ga2, mean ga2*hat a2)
  void* ga1_out;                         // dL/d(hat a1)
  double2* slab1;                        // partial (S1, S2) of layer-1 norm backward
  float* col_slab;                       // [blocks][dw_col_stride]: ggamma1, gbeta1, gwd, ggamma2, gbeta2, galpha2
  const float2* sm1;                     // (ew) layer-1 sums
  void* gh1_out;                         // (ew) dL/dh1
  float* alpha_slab;                     // (ew) [blocks] galpha1 partials
  // gLN folds (StatFold): dw_fwd finalizes st1, dw_bwd sm2, norm1_bwd sm1
  StatFold f_st1, f_sm2, f_sm1;
  // cLN: a lane group holds all H channels of a row, so the per-row statistics are
  // final in-kernel: dw_fwd writes norm-2 (mean, rstd) to st2_out, dw_bwd the norm-1
  // backward means to sm1_out (instead of slab partials + a finalize launch)
  float eps = 0.f;
  float2* st2_out = nullptr;
  float2* sm1_out = nullptr;
};
int dw_seg(const DwArgs& a, bool bwd);   // comb segment length sizing one resident round
int dw_blocks(const DwArgs& a);        // depthwise (comb) kernels (a.seg set)
int ew_blocks(const DwArgs& a);        // norm1_bwd (128-row blocks)
int dw_parts_per_group(const DwArgs& a);   // slab parts per utterance (gLN) or per row (cLN)
// col_slab part layout: [ggamma1 H][gbeta1 H][gwd H*P][ggamma2 H][gbeta2 H][galpha2 1], padded to 4
__host__ __device__ inline int dw_col_stride(const DwArgs& a) { return ((4 + a.P) * a.H + 1 + 3) & ~3; }
hipError_t launch_dw_fwd(DType dt, const DwArgs& a, hipStream_t s);
hipError_t launch_dw_bwd(DType dt, const DwArgs& a, hipStream_t s);
hipError_t launch_norm1_bwd(DType dt, const DwArgs& a, hipStream_t s);
// wave-item forms (ctn_dw_wave.hip: bf16, H = 512, P = 3), chosen by launch_dw_fwd / _bwd;
// CTN_DW_WAVE=0 keeps the lane-group kernels
bool dw_wave_eligible(DType dt, const DwArgs& a);
hipError_t launch_dw_fwd_wave(const DwArgs& a, hipStream_t s);
hipError_t launch_dw_bwd_wave(const DwArgs& a, hipStream_t s);

// ---- stand-alone separator layers on frame rows (ctn_layers.hip) ------------
enum LayerOp {
  LAYER_NORM_FWD, LAYER_NORM_BWD, LAYER_PRELU_FWD, LAYER_PRELU_BWD,
  LAYER_DW_FWD, LAYER_DW_BWD, LAYER_MASK_FWD, LAYER_MASK_BWD
};
struct LayerArgs {
  Rows g;
  int C;                        // channels of x (mask: S*N)
  const void* x; void* y;       // forward input / output (mask backward: x = score)
  const void* gy; void* gx;     // backward
  // norms
  int norm = 0; float eps = 0.f;
  const float* gamma = nullptr; const float* beta = nullptr;
  float2* stats = nullptr;      // (mean, rstd): [M] gLN, [M*Kp] cLN (forward out, backward in)
  float2* sums = nullptr;       // backward scratch: (mean g*gamma, mean g*gamma*xhat) per group
  double2* slab = nullptr;      // gLN scratch [M * layer_norm_groups_nb]
  float* ggamma = nullptr; float* gbeta = nullptr;
  // PReLU
  const float* alpha = nullptr; float* galpha = nullptr;
  // depthwise
  int P = 0, dil = 1, pad = 0;
  const float* w = nullptr; float* gw = nullptr;
  // mask
  int S = 1, mask_type = 0;
  // column / alpha partials [layer_blocks][...] and the slab-reduce scratch
  float* part = nullptr; float* tmp = nullptr;
};
int layer_blocks(const Rows& g);            // row blocks of the partial reductions
int layer_norm_groups_nb(const Rows& g);    // gLN partials per utterance
hipError_t launch_layer(DType dt, LayerOp op, const LayerArgs& a, hipStream_t s);

// ---- BatchNorm1d column statistics (ctn_bn.hip) -----------------------------
struct BnArgs {
  Rows g;
  int H;
  const void* a;          // pre-PReLU activation [rows][H] (h1 or d)
  const void* gin;        // gradient [rows][H]
  void* gout;             // bn_apply output (may equal gin)
  const float* alpha;     // PReLU alpha (1 element)
  const float2* stats;    // (mean, rstd) per channel
  const float2* sums;     // (mean g, mean g*xhat) per channel (bn_apply)
  double2* part;          // [bn_blocks][H] partials (bn_partials)
  float* apart;           // [bn_blocks] alpha-gradient partials (bn_apply with PReLU)
};
struct BnFinal {
  int H, M, nparts;
  long count;             // valid frame rows M*K
  const double2* part;
  int training;
  float momentum, eps;
  float* run_mean; float* run_var;            // may be null (no running statistics)
  const float* gamma; const float* beta;
  float2* stats;                              // mode 0 out / mode 2 in
  float* gamma_eff; float* beta_eff;          // modes 0, 2
  float2* sums;                               // mode 1
  float* dgamma; float* dbeta;                // mode 1, optional
  float2* ident; float2* zero;                // per-utterance (0,1) / (0,0) tables, optional
};
int bn_blocks(const Rows& g);
hipError_t launch_bn_partials(DType dt, const BnArgs& p, int mode, hipStream_t s);
hipError_t launch_bn_finalize(const BnFinal& p, int mode, hipStream_t s);
hipError_t launch_bn_apply(DType dt, const BnArgs& p, bool prelu_bwd, hipStream_t s);
hipError_t launch_bn_gamma_fix(float* dgamma, const float* dbeta, const float2* stats, int H, hipStream_t s);

// ---------------------------------------------------------------------------
// parameter update (ctn_optim.hip); layouts identical to ctn_opt_segment /
// ctn_opt_chunk of include/ctn.h
// ---------------------------------------------------------------------------
struct OptSegment { float* p; float* g; float* m; float* v; int64_t n; };
struct OptChunk { int32_t seg; uint32_t len; int64_t off; };
constexpr int OPT_CHUNK = 8192;                 // elements per workgroup
constexpr uint32_t OPT_UNALIGNED = 0x80000000u;  // len flag: scalar path
constexpr uint32_t OPT_LEN_MASK = 0x7fffffffu;
// Bias corrections on the device in fp64 from the step count (ABI v12): step t = *counter + 1
// when counter is set (graph capture), else `step`; lr from *lr_dev when set, else `lr`
struct AdamArgs {
  float b1, b2, eps, wd, lr;
  int step;
  const float* lr_dev;
  const int* counter;
};
hipError_t launch_grad_sqnorm(const OptSegment* segs, const OptChunk* chunks, int nchunks, float* partial,
                              hipStream_t s);
hipError_t launch_grad_clip(const OptSegment* segs, const OptChunk* chunks, int nchunks, const float* partial,
                            float max_norm, float* total_norm, hipStream_t s);
hipError_t launch_adam(const OptSegment* segs, const OptChunk* chunks, int nchunks, const AdamArgs& a,
                       hipStream_t s);
// the same update with a.counter set, then a one-lane kernel increments *counter
hipError_t launch_adam_dev(const OptSegment* segs, const OptChunk* chunks, int nchunks, const AdamArgs& a,
                           int* counter, hipStream_t s);
hipError_t launch_write_segments(OptSegment* dst, const OptSegment* src, int n, hipStream_t s);

// ---- streaming causal separation (ctn_stream.hip) ----------------------------------
struct StreamArgs {
  int M, K, N, L, B, H, P, C, norm, mask_type, dil, R;
  long pos, ld_samples;
  const float* samples;          // encode: [M][ld_samples]
  const float* U;                // encode: [N][L]
  const float* na;               // norm: cLN gamma or affine scale [channels]
  const float* nb;               // norm: cLN beta or affine shift
  const float* W;                // transposed 1x1 weight [in][out]
  const float* alpha1;           // PReLU 1 (block_in)
  const float* alpha2;           // PReLU 2 (block_out)
  const float* wd;               // depthwise [H][P]
  const float* x_in;             // [M][K][B]
  const float* w_in;             // decode: encoder output [M][K][N]
  const float* V;                // decode: basis [L][N]
  const float* tail_in;          // decode: [M][C][L/2]
  float* w_out;                  // encode: [M][K][N]
  float* x_out;                  // [M][K][B]
  float* ring;                   // [M][R][H]
  float* frames;                 // decode scratch [M][C][K][L]
  float* tail_out;               // [M][C][L/2]
  float* out;                    // [M][C][K*L/2]
  // ABI v7 call path (launch_stream_call_stage): norm-2 parameters and W2 of a block
  const float* na2 = nullptr;
  const float* nb2 = nullptr;
  const float* W2 = nullptr;
  // ABI v7 graph replay: the call's first frame index read from device memory (written
  // by launch_stream_set_pos before each replay) instead of `pos`
  const long* pos_dev = nullptr;
};
// which: 0 encode, 1 block in (1x1, PReLU, norm 1 -> ring), 2 block out (depthwise, PReLU,
// norm 2, 1x1, residual), 3 decode (mask, sources, frames, overlap-add)
hipError_t launch_stream(int which, const StreamArgs& a, hipStream_t s);
// ABI v7 (ctn_stream_call): 0 encode, 1 block in (W1 chunks -> h1 scratch in `frames`),
// 2 block out (taps, depthwise, norms, W2 chunks, residual, ring), 3 decode mask
// (-> sources in `frames`), 4 decoder basis + overlap-add
hipError_t launch_stream_call_stage(int which, const StreamArgs& a, hipStream_t s);
hipError_t launch_stream_set_pos(long* pos_dev, long pos, hipStream_t s);

}  // namespace ctn
