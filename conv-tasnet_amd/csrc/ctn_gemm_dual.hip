// Dual GEMM (bf16, gfx950): one pass over the frame rows computes BOTH a 1x1
// convolution's data gradient (row GEMM, C[r][n] = sum_k A[r][k] W[n][k] + fused
// epilogue) AND its weight gradient (column GEMM, D[k][n] = sum_r A[r][k] op(Bm[r][n])),
// sharing the A stream.  On the TemporalBlock backward (conv_tasnet.py:217,256):
//   second 1x1 (H->B):  A = gy,  W = W2^T, C = g_n2 (norm-2 backward epilogue),
//                       Bm = d, op = gLN/cLN(PReLU(.)) -> D = dW2 [B][H]
//   first 1x1 (B->H):   A = gh1, W = W1^T, C = gx = gh1.W1 + gy (residual),
//                       Bm = x (plain)                     -> D = dW1 [H][B]
// Without the fusion these are four kernels, and A (and Bm) stream from HBM twice.
//
// Decomposition: the output channels are cut into S slices of NS = Nout/S channels;
// workgroup (row range, slice) keeps its slice of W resident in VGPRs (MFMA
// A-fragments, as the weight-stationary kernel ctn_gemm_ws.hip) and its D slice
// [Kred][NS] as fp32 MFMA accumulators (64 VGPRs per lane), and streams the 32-row
// tiles of its range.  The S workgroups of one row range sit on the same XCD
// (hardware workgroup ids are dealt round-robin over the 8 XCDs), so each A tile
// is fetched from HBM once and re-read by the other slices from that XCD's L2.
// Per tile:  A (all Kred channels) -> LDS in WS fragment order; op(Bm) slice ->
// LDS (4-row x 16-column blocks, conflict-free transposed reads);
//   row part : v_mfma_f32_16x16x32_bf16 against the resident W slice, epilogue
//              straight from the accumulators;
//   col part : D += A_tile^T . op(Bm)_tile, both operands read with
//              ds_read_b64_tr_b16 (the reduction runs over frame rows).
// D partials are stored once per workgroup ([range][Kred][Nout]) and summed by
// slab_reduce in a fixed order: bitwise reproducible, no atomics.
#include <stdlib.h>

#include <type_traits>

#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int DU_WV = 8, DU_NT = 512, DU_TM = 32, DU_GRID = 256;

// Bound-finding experiments only (tools/microbench/dual_bench.hip): bit 0 drops the
// row-part stores, 1 the A loads, 2 the row-part MFMAs, 3 the column part (reads and
// MFMAs), 4 the Bm loads, 5 fences the epilogue off the MFMAs, 6 drops the LDS staging.
#ifndef CTN_DU_EXP
#define CTN_DU_EXP 0
#endif

// LDS images (byte offsets), all checked conflict-free (bank model of
// MI355X_MICROARCH.md §LDS) for the staging stores, the row part's ds_read_b128
// and the column part's ds_read_b64_tr_b16, and chosen so that every read
// address is a lane base + a compile-time offset (no per-tile address math):
//   A  : 16-row block mb, k-block kb (32 channels) of 1 KiB, 16-byte chunk lg (of 4)
//        at 256*lg, frame row r at 16*(r ^ (lg odd ? 12 : 0))
//   Bm : 16-column block of 1 KiB, 4-row group rg at 128*pos(rg), pos(rg) = rg ^ ((rg>>1)&1),
//        row-in-group at 32*(r&3)
template <int KB> CTN_DEV int du_apiece(int row, int kc) {   // 16-byte chunk kc (8 channels) of row
  const int lg = kc & 3;
  return (row >> 4) * KB * 1024 + (kc >> 2) * 1024 + lg * 256 + (((row & 15) ^ ((lg & 1) * 12)) << 4);
}
CTN_DEV int du_boff(int row, int col) {
  const int rg = row >> 2;
  return (col >> 4) * 1024 + ((rg ^ ((rg >> 1) & 1)) << 7) + (row & 3) * 32 + (col & 15) * 2;
}

CTN_DEV void du_ready(const v4u& v) { asm volatile("" ::"v"(v)); }

CTN_DEV s16x4_t du_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}

typedef __amdgpu_buffer_rsrc_t rsrc_t;
CTN_DEV rsrc_t du_rsrc(const void* p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                           0x00020000);
}
constexpr uint32_t DU_OOB = 0x80000000u;   // voffset past every buffer: loads return 0

// NV consecutive bf16 (NV = 4: 8-byte access, NV = 8: 16-byte access) through a buffer resource
template <int NV> struct DuVec { uint32_t w[NV / 2]; };
template <int NV> CTN_DEV DuVec<NV> du_bload(rsrc_t r, uint32_t voff, int soff) {
  DuVec<NV> v;
  if constexpr (NV == 8) {
    const v4u a = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
    v.w[0] = a[0]; v.w[1] = a[1]; v.w[2] = a[2]; v.w[3] = a[3];
  } else {
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    const v2u a = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
    v.w[0] = a[0]; v.w[1] = a[1];
  }
  return v;
}
// Stores take their whole offset in the VGPR (soffset = 0): LLVM only guards the
// hazard of a VALU overwriting the data VGPRs of an in-flight >8-byte buffer store
// when soffset is not a register, and gfx950 does corrupt such stores (measured:
// single dwords of some lanes replaced by the next value written to the register).
template <int NV> CTN_DEV void du_bstore(rsrc_t r, uint32_t voff, int soff, const f32x2_t v[NV / 2]) {
  if constexpr (NV == 8) {
    const v4u o = {pk_bf16(v[0][0], v[0][1]), pk_bf16(v[1][0], v[1][1]), pk_bf16(v[2][0], v[2][1]),
                   pk_bf16(v[3][0], v[3][1])};
    __builtin_amdgcn_raw_buffer_store_b128(o, r, voff + (uint32_t)soff, 0, 0);
  } else {
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    const v2u o = {pk_bf16(v[0][0], v[0][1]), pk_bf16(v[1][0], v[1][1])};
    __builtin_amdgcn_raw_buffer_store_b64(o, r, voff, soff, 0);
  }
}

// KB: Kred / 32; NSB: slice width / 16; NBW: 16-channel output blocks per wave (row part)
template <int KB, int NSB, int NBW, int EPI, int OPB, int NK>
__global__ __launch_bounds__(DU_NT) void gemm_dual_kernel(GemmDual p) {
  constexpr int TM = DU_TM, WV = DU_WV, NT = DU_NT;
  constexpr int KR = KB * 32;          // reduction length of the row part (= D rows)
  constexpr int CPR = KR / 8;          // 16-byte chunks per A row
  constexpr int NA = TM * CPR / NT;    // A chunks per thread per tile
  constexpr int NS = NSB * 16;         // slice width
  constexpr int EB = NS * TM / NT;     // Bm elements per thread per tile (8 or 4)
  constexpr int WNB = NSB / NBW;       // row-part waves per 16-row block
  constexpr int NV = NBW * 4;          // output channels per lane (row part)
  constexpr int WN = NSB / 4;          // col-part waves along n (4 n-blocks each)
  static_assert(NA * NT == TM * CPR && NA * 16 == CPR, "A staging: 4 rows x 16 chunks per wave-instruction");
  static_assert(EB == 8 || EB == 4, "Bm staging: 4 rows per wave");
  static_assert(2 * WNB == WV, "row part: 2 row blocks x WNB waves");
  static_assert(WN >= 1 && (WV / WN) * 4 * 16 == KR, "col part: 4x4 blocks per wave cover D");
  static_assert(NV == 4 || NV == 8, "epilogue vector width");

  __shared__ __attribute__((aligned(16))) char sA[2][TM * KR * 2];
  __shared__ __attribute__((aligned(16))) char sB[2][TM * NS * 2];
  // slice constants: column-operand gamma/beta, epilogue gamma
  __shared__ __attribute__((aligned(16))) float sgb[3][NS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int S = p.Nout / NS;
  const int nr = (int)gridDim.x / S;   // row ranges
  int rr, sl;
  {
    const int b = (int)blockIdx.x;
    if ((int)gridDim.x % (8 * S) == 0) {   // the S slices of a range on one XCD
      const int l = b / 8;
      sl = l % S;
      rr = (b % 8) * (nr / 8) + l / S;
    } else {
      sl = b % S;
      rr = b / S;
    }
  }
  const long rows = p.g.rows();
  const int ntile = (int)(rows / TM);
  const int t0 = (int)((long)ntile * rr / nr), t1 = (int)((long)ntile * (rr + 1) / nr);
  const int n0 = sl * NS;
  const int Kp = p.g.Kp, Kv = p.g.K;
  const rsrc_t rA = du_rsrc(p.A, rows * p.lda * 2), rB = du_rsrc(p.Bm, rows * p.ldb * 2);
  const rsrc_t rR = du_rsrc(p.R, rows * p.ldr * 2), rC = du_rsrc(p.C, rows * p.ldc * 2);
  const bf16raw* W = reinterpret_cast<const bf16raw*>(p.W);

  // ---- row part: wave (mbw, nbg) owns rows mbw*16.. of each tile, channels
  //      n0 + nbg*16*NBW .. ; resident W fragments (permuted rows: lane groups get
  //      NV contiguous output channels)
  const int mbw = wid / WNB, nbg = wid % WNB;
  const int colbase = n0 + nbg * 16 * NBW + lg * NV;
  v4u wf[NBW][KB];
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb) {
    const int n = n0 + nbg * 16 * NBW + (lr >> 2) * NV + nb * 4 + (lr & 3);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) wf[nb][kb] = ldg16(W + (size_t)n * p.ldw + kb * 32 + lg * 8);
  }
  const float eal = EPI == EPI_NORM_BWD ? p.alpha[0] : 0.f;
  const float bal = OPB == OP_PRELU_NORM ? p.bop.alpha[0] : 0.f;
  for (int c = tid; c < NS; c += NT) {
    sgb[0][c] = OPB != OP_PLAIN ? p.bop.gamma[n0 + c] : 0.f;
    sgb[1][c] = OPB != OP_PLAIN ? p.bop.beta[n0 + c] : 0.f;
    sgb[2][c] = EPI == EPI_NORM_BWD ? p.gamma[n0 + c] : 0.f;
  }
  __syncthreads();

  // ---- col part: wave (wp, wn) owns D blocks p in [wp*64, +64), n in [n0 + wn*64, +64)
  const int wp = wid / WN, wn = wid % WN;
  f32x4_t dacc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) dacc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ---- lane-constant addresses
  // A staging: wave w stages rows 4w..4w+3; lane: row 4w + ((l>>1)&3), chunks skc + 16j
  const int srow = 4 * wid + ((lane >> 1) & 3), skc = 2 * ((lane >> 3) & 7) + (lane & 1);
  const uint32_t avoff = (uint32_t)(srow * p.lda * 2 + skc * 16);
  const int aw = du_apiece<KB>(srow, skc);                 // + j * 4096
  // Bm staging: wave w stages rows 4w..4w+3; lane: row 4w + (l&3), EB columns at bcol
  const int brow = 4 * wid + (lane & 3);
  const int bcol = EB == 8 ? 16 * (lane >> 3) + 8 * ((lane >> 2) & 1) : 16 * (lane >> 4) + 4 * ((lane >> 2) & 3);
  const uint32_t bvoff = (uint32_t)(brow * p.ldb * 2 + (n0 + bcol) * 2);
  const int bw = du_boff(brow, bcol);
  // row-part fragment reads: + kb * 1024
  const int rbase = mbw * KB * 1024 + lg * 256 + ((lr ^ ((lg & 1) * 12)) << 4);
  // col-part transposed reads, h = 0/1 (rows 8lg+4h+q): A + (i>>1)*1024 + (i&1)*512, B + j*1024
  const int q = lr >> 2, pp = lr & 3;
  int abase[2], bbase[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * lg + 4 * h + q;
    abase[h] = (lg >> 1) * KB * 1024 + 2 * wp * 1024 + (pp >> 1) * 256 + (((row & 15) ^ ((pp >> 1) * 12)) << 4) +
               (pp & 1) * 8;
    bbase[h] = wn * 4 * 1024 + du_boff(row, 4 * pp);
  }
  // epilogue rows: mbw*16 + lr of each tile
  const int erow = mbw * 16 + lr;
  const uint32_t rvoff = (uint32_t)(erow * p.ldr * 2 + colbase * 2);
  const uint32_t cvoff = (uint32_t)(erow * p.ldc * 2 + colbase * 2);

  // ---- per-tile operand registers (loaded one tile ahead of their use)
  v4u ra[NA];
  DuVec<EB> rb;
  float2 bst = make_float2(0.f, 0.f);
  bool bvalid = true;
  auto load_ab = [&](int t) __attribute__((always_inline)) {
    const int tk = (t * TM) % Kp;   // frame of the tile's first row (tiles never straddle utterances)
    // rows of padded frames load as zeros (out-of-range buffer offset)
    const uint32_t vo = tk + srow < Kv ? avoff : DU_OOB;
    const int so = t * TM * p.lda * 2;
#pragma unroll
    for (int j = 0; j < NA; ++j)
      if constexpr (CTN_DU_EXP & 2) ra[j] = v4u{vo, (uint32_t)so, 0u, 0u};
      else ra[j] = __builtin_amdgcn_raw_buffer_load_b128(rA, vo + j * 256, so, 0);
    if constexpr (CTN_DU_EXP & 16) { for (int e = 0; e < EB / 2; ++e) rb.w[e] = bvoff + t; }
    else rb = du_bload<EB>(rB, bvoff, t * TM * p.ldb * 2);
    if constexpr (OPB != OP_PLAIN) bst = p.bop.stats[stat_index<NK>(t * TM + brow, Kp)];
    if constexpr (OPB != OP_PLAIN && NK == NORM_CLN) bvalid = tk + brow < Kv;
  };
  // Bm transform: padded frames are zeroed only under cLN (their per-row statistics are
  // not finite); otherwise A is zero there and the D products vanish
  auto stage = [&](auto le1, int buf) __attribute__((always_inline)) {
    constexpr bool LE1 = decltype(le1)::value;
#pragma unroll
    for (int j = 0; j < NA; ++j)
      if constexpr (!(CTN_DU_EXP & 64)) stg16(sA[buf] + aw + j * 4096, ra[j]);
    uint32_t w[EB / 2];
#pragma unroll
    for (int e = 0; e < EB / 2; ++e) w[e] = rb.w[e];
    if constexpr (OPB != OP_PLAIN) {
      const f32x2_t m2 = {bst.x, bst.x};
#pragma unroll
      for (int e = 0; e < EB / 2; ++e) {
        const float2 g = *reinterpret_cast<const float2*>(&sgb[0][bcol + 2 * e]);
        const float2 bt = *reinterpret_cast<const float2*>(&sgb[1][bcol + 2 * e]);
        f32x2_t x = {__uint_as_float(w[e] << 16), __uint_as_float(w[e] & 0xffff0000u)};
        if constexpr (OPB == OP_PRELU_NORM) x = prelu2<LE1>(x, bal);
        x = pfma(x - m2, f32x2_t{bst.y * g.x, bst.y * g.y}, f32x2_t{bt.x, bt.y});
        w[e] = pk_bf16(x[0], x[1]);
        if constexpr (NK == NORM_CLN) w[e] = bvalid ? w[e] : 0u;
      }
    }
    if constexpr (CTN_DU_EXP & 64) { asm volatile("" ::"v"(w[0]), "v"(w[1])); }
    else if constexpr (EB == 8) stg16(sB[buf] + bw, v4u{w[0], w[1], w[2], w[3]});
    else *reinterpret_cast<uint2*>(sB[buf] + bw) = make_uint2(w[0], w[1]);
  };

  // ---- row epilogue operand (residual or pre-activation), one tile ahead
  DuVec<NV> rn;
  float2 est = make_float2(0.f, 0.f);
  auto load_r = [&](int t) __attribute__((always_inline)) {
    rn = du_bload<NV>(rR, rvoff, t * TM * p.ldr * 2);
    if constexpr (EPI == EPI_NORM_BWD) est = p.stats[stat_index<NK>(t * TM + erow, Kp)];
  };

  // gLN run partials (WsRuns layout with waves = S * WV: slot (sl*WV + wid)); the running
  // sum of the current utterance is stored every tile (the last store of a run is its total)
  double run_s = 0.0, run_q = 0.0;
  const int tpu = Kp / TM, m0 = t0 / tpu;
  int run_m = m0;
  const int kmax = ws_runs_kmax(ntile, nr, tpu);
  double2* run_slab = p.grp_slab + (((size_t)rr * S + sl) * WV + wid) * kmax;

  auto compute = [&](int buf, f32x4_t (&acc)[NBW]) __attribute__((always_inline)) {
    const char* a = sA[buf];
    const char* bsl = sB[buf];
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) acc[nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const v4u b = *reinterpret_cast<const v4u*>(a + rbase + kb * 1024);
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb)
        if constexpr (CTN_DU_EXP & 4) acc[nb][kb & 3] += __uint_as_float(b[0] ^ wf[nb][kb][1]);
        else acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[nb][kb]),
                                                          __builtin_bit_cast(bf16x8_t, b), acc[nb], 0, 0, 0);
    }
    if constexpr (CTN_DU_EXP & 8) return;
    bf16x8_t af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = (i >> 1) * 1024 + (i & 1) * 512;
      const s16x4_t lo = du_tr(a + abase[0] + o), hi = du_tr(a + abase[1] + o);
      af[i] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const s16x4_t lo = du_tr(bsl + bbase[0] + j * 1024), hi = du_tr(bsl + bbase[1] + j * 1024);
      bfr[j] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        dacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], dacc[i][j], 0, 0, 0);
  };

  // row epilogue of tile t: lane holds row t*TM + erow, channels colbase..+NV
  auto epilogue = [&](auto le1, int t, const f32x4_t (&acc)[NBW]) __attribute__((always_inline)) {
    constexpr bool LE1 = decltype(le1)::value;
    f32x2_t v2[NV / 2];
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      v2[2 * nb] = f32x2_t{acc[nb][0], acc[nb][1]};
      v2[2 * nb + 1] = f32x2_t{acc[nb][2], acc[nb][3]};
    }
    f32x2_t s2 = {0.f, 0.f}, q2 = {0.f, 0.f};
    if constexpr (EPI == EPI_RESID) {
#pragma unroll
      for (int c = 0; c < NV / 2; ++c)
        v2[c] += f32x2_t{__uint_as_float(rn.w[c] << 16), __uint_as_float(rn.w[c] & 0xffff0000u)};
    } else {
      const f32x2_t rs = {est.y, est.y}, ms = {-est.x * est.y, -est.x * est.y};
#pragma unroll
      for (int c = 0; c < NV / 2; ++c) {
        const float2 g = *reinterpret_cast<const float2*>(&sgb[2][colbase - n0 + 2 * c]);
        const f32x2_t x = {__uint_as_float(rn.w[c] << 16), __uint_as_float(rn.w[c] & 0xffff0000u)};
        const f32x2_t ah = pfma(prelu2<LE1>(x, eal), rs, ms);   // hat a
        const f32x2_t ga = v2[c] * f32x2_t{g.x, g.y};
        s2 += ga;
        q2 = pfma(ga, ah, q2);
      }
    }
    if constexpr (!(CTN_DU_EXP & 1)) du_bstore<NV>(rC, cvoff, t * TM * p.ldc * 2, v2);
    else asm volatile("" ::"v"(v2[0]));
    if constexpr (EPI == EPI_NORM_BWD) {
      if constexpr (NK == NORM_GLN) {
        const float s = wave_sum_dpp(s2[0] + s2[1]), ss = wave_sum_dpp(q2[0] + q2[1]);
        const int m = (t * TM) / Kp;
        const bool same = m == run_m;
        run_s = (same ? run_s : 0.0) + (double)s;
        run_q = (same ? run_q : 0.0) + (double)ss;
        run_m = m;
        run_slab[m - m0] = make_double2(run_s, run_q);
      } else {
        // per-row partial over the wave's channels: reduce across the 4 lane groups
        float s = s2[0] + s2[1], ss = q2[0] + q2[1];
        s += __shfl_xor(s, 16, 64); ss += __shfl_xor(ss, 16, 64);
        s += __shfl_xor(s, 32, 64); ss += __shfl_xor(ss, 32, 64);
        p.grp_slab[(size_t)(t * TM + erow) * (S * WNB) + sl * WNB + nbg] = make_double2((double)s, (double)ss);
      }
    }
  };

#pragma unroll
  for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) du_ready(wf[nb][kb]);
  asm volatile("" ::"v"(eal), "v"(bal));

  // Pipeline (unrolled by two: static LDS buffer parity): after one LDS-only barrier,
  // the MFMAs of tile t, its epilogue, the staging of tile t+1 (registers loaded one
  // iteration earlier) and the loads of tile t+2.  No scheduling fence: the epilogue
  // and staging VALU work interleaves with the column part's MFMAs.
  auto clampt = [&](int t) __attribute__((always_inline)) { return t < t1 ? t : t1 - 1; };
  auto run = [&](auto le1) __attribute__((always_inline)) {
    f32x4_t acc[NBW];
    load_ab(t0);
    load_r(t0);
    stage(le1, 0);
    load_ab(clampt(t0 + 1));
    auto step = [&](int t, auto par) __attribute__((always_inline)) {
      constexpr int P = decltype(par)::value;
      lds_barrier();
      compute(P, acc);
      if constexpr (CTN_DU_EXP & 32) __builtin_amdgcn_sched_barrier(0);
      epilogue(le1, t, acc);
      load_r(clampt(t + 1));
      stage(le1, 1 - P);
      load_ab(clampt(t + 2));
    };
    int t = t0;
    for (; t + 1 < t1; t += 2) {
      step(t, std::integral_constant<int, 0>{});
      step(t + 1, std::integral_constant<int, 1>{});
    }
    if (t < t1) step(t, std::integral_constant<int, 0>{});
  };
  if (t0 < t1) {
    constexpr bool PR = OPB == OP_PRELU_NORM || EPI == EPI_NORM_BWD;
    const float al = OPB == OP_PRELU_NORM ? bal : eal;
    if (!PR || al <= 1.f) run(std::true_type{});
    else run(std::false_type{});
  }

  // D partial of this workgroup: lane holds D[p = (wp*4+i)*16 + 4lg + e][n = n0 + (wn*4+j)*16 + lr]
  float* Dp = p.Dpart + (size_t)rr * KR * p.Nout;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + (wn * 4 + j) * 16 + lr;
#pragma unroll
      for (int e = 0; e < 4; ++e) Dp[(size_t)((wp * 4 + i) * 16 + 4 * lg + e) * p.Nout + n] = dacc[i][j][e];
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// CTN_GEMM_DUAL=1 selects the dual kernels, 0 the four-kernel path (row GEMM + column
// GEMM twice); read on every query so a process can compare both (tests/test_gpu_tblock.py).
// Default: off until it measures faster than the four kernels.
static bool dual_enabled() {
  const char* e = getenv("CTN_GEMM_DUAL");
  return e && atoi(e) == 1;
}

// (Kred, Nout) -> (KB, NSB, NBW); S = 4 slices
static bool dual_shape(int Kred, int Nout, int* kb, int* nsb, int* nbw) {
  if (Kred == 256 && Nout == 512) { *kb = 8; *nsb = 8; *nbw = 2; return true; }   // gy.W2, dW2
  if (Kred == 512 && Nout == 256) { *kb = 16; *nsb = 4; *nbw = 1; return true; }  // gh1.W1, dW1
  return false;
}

bool gemm_dual_eligible(DType dt, const GemmDual& p) {
  int kb, nsb, nbw;
  if (dt != BF16 || !dual_enabled() || !dual_shape(p.Kred, p.Nout, &kb, &nsb, &nbw)) return false;
  const bool pairA = p.Kred == 256 && p.epi == EPI_NORM_BWD && p.bop.kind == OP_PRELU_NORM;
  const bool pairB = p.Kred == 512 && p.epi == EPI_RESID && p.bop.kind == OP_PLAIN;
  if (!pairA && !pairB) return false;
  if (p.bop.kind != OP_PLAIN && p.bop.fold.slab) return false;   // needs final statistics
  if (p.g.Kp % DU_TM || p.lda % 8 || p.ldw % 8 || p.ldc % 8 || p.ldr % 8 || p.ldb % 8) return false;
  if (p.g.rows() / DU_TM < 1 || p.g.rows() >= (1L << 31)) return false;
  return true;
}

static int dual_slices(const GemmDual& p) {
  int kb, nsb, nbw;
  dual_shape(p.Kred, p.Nout, &kb, &nsb, &nbw);
  return p.Nout / (nsb * 16);
}

int gemm_dual_ranges(const GemmDual& p) {
  const long nt = p.g.rows() / DU_TM;
  const int want = DU_GRID / dual_slices(p);
  return (int)(nt < want ? nt : want);
}

WsRuns gemm_dual_runs(const GemmDual& p) {
  WsRuns w;
  w.ntile = (int)(p.g.rows() / DU_TM);
  w.grid = gemm_dual_ranges(p);
  w.tpu = p.g.Kp / DU_TM;
  w.waves = dual_slices(p) * DU_WV;
  w.kmax = ws_runs_kmax(w.ntile, w.grid, w.tpu);
  return w;
}

int gemm_dual_group_parts(const GemmDual& p) {
  int kb, nsb, nbw;
  dual_shape(p.Kred, p.Nout, &kb, &nsb, &nbw);
  if (p.norm != NORM_GLN) return dual_slices(p) * (nsb / nbw);
  const WsRuns w = gemm_dual_runs(p);
  const long entries = (long)w.grid * w.waves * w.kmax;
  return (int)((entries + p.g.M - 1) / p.g.M);
}

StatFold gemm_dual_stat_fold(const GemmDual& p, const double2* slab, double cnt, float eps, int mode, float2* out) {
  StatFold f;
  f.slab = slab;
  f.parts = gemm_dual_group_parts(p);
  f.cnt = cnt;
  f.eps = eps;
  f.mode = mode;
  f.out = out;
  if (p.norm == NORM_GLN) f.ws = gemm_dual_runs(p);
  return f;
}

// instantiated pairs: (256 -> 512, norm-2 backward epilogue, PReLU+norm column operand)
// and (512 -> 256, residual epilogue, plain column operand); other pairings fall back
template <int NK>
static hipError_t dual_launch_nk(const GemmDual& p, hipStream_t s) {
  const dim3 grid(gemm_dual_ranges(p) * dual_slices(p));
  if (p.Kred == 256 && p.epi == EPI_NORM_BWD && p.bop.kind == OP_PRELU_NORM)
    hipLaunchKernelGGL((gemm_dual_kernel<8, 8, 2, EPI_NORM_BWD, OP_PRELU_NORM, NK>), grid, dim3(DU_NT), 0, s, p);
  else if (p.Kred == 512 && p.epi == EPI_RESID && p.bop.kind == OP_PLAIN)
    hipLaunchKernelGGL((gemm_dual_kernel<16, 4, 1, EPI_RESID, OP_PLAIN, NORM_GLN>), grid, dim3(DU_NT), 0, s, p);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_gemm_dual(const GemmDual& p, hipStream_t s) {
  if (!gemm_dual_eligible(BF16, p)) return hipErrorInvalidValue;
  const int nk = p.bop.kind != OP_PLAIN ? p.bop.norm : p.norm;
  return nk == NORM_GLN ? dual_launch_nk<NORM_GLN>(p, s) : dual_launch_nk<NORM_CLN>(p, s);
}

}  // namespace ctn
