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
constexpr int DU_MMAX = 512;   // utterances whose gLN statistics a workgroup holds in LDS

// Bound-finding experiments only (tools/microbench/dual_bench.hip): bit 0 drops the
// row-part stores, 1 the A loads, 2 the row-part MFMAs, 3 the column part (reads and
// MFMAs), 4 the Bm loads, 5 fences the epilogue off the MFMAs, 6 drops the LDS staging.
#ifndef CTN_DU_EXP
#define CTN_DU_EXP 0
#endif
#ifndef CTN_DU_DA
#define CTN_DU_DA 4   // LDS ring depth of the (256 -> 512, norm-backward) pair
#endif
// cLN per-row statistics: 1 = a 4-byte LDS-DMA per wave and tile into a per-wave ring,
// with no LDS-DMA in flight while the epilogue runs (vmcnt(0) before it); 0 = plain
// loads from L2 at the point of use (their compiler-counted waits drain the ring
// before every use).  Both reproducible run to run; 1 is faster.
#ifndef CTN_DU_CST_DMA
#define CTN_DU_CST_DMA 1
#endif
// cLN per-row sums across the four lane rows: 1 = v_permlane16/32_swap (VALU),
// 0 = ds_bpermute (wrong sums in every launch while LDS-DMA is in flight, §10)
#ifndef CTN_DU_PERMLANE
#define CTN_DU_PERMLANE 1
#endif
// Reproducibility experiments (tools/microbench/dual_det.hip), all off:
//   CTN_DU_DBG bit 0 vmcnt(0) before each epilogue, bit 1 vmcnt(0) at the loop top,
//     bit 2 lgkmcnt(0) after each cross-lane step of the cLN row sums, bit 3
//     lgkmcnt(0) after the epilogue's statistics and raw-row LDS reads, bit 4
//     vmcnt(0) right after the cLN statistics store;
//   CTN_DU_LATE 1: each iteration issues its DMA group after the epilogue;
//   CTN_DU_NOCLAMP 1: the last D-1 iterations issue no DMA (default: they re-issue
//     the range's last tile into its own slot, same bytes).
#ifndef CTN_DU_DBG
#define CTN_DU_DBG 0
#endif
// experiment: 1 raises the wave priority (s_setprio 1) while it issues a tile's MFMAs
#ifndef CTN_DU_PRIO
#define CTN_DU_PRIO 0
#endif
// 1: the resident weight and constants are loaded and waited for before the first DMA
// groups are issued (round-2 order); 0 (experiment): the first D-1 DMA groups go out
// first, so their latency overlaps the weight's.  0 makes the cLN epilogue statistics
// of the first tiles irreproducible in every launch and gains nothing.
#ifndef CTN_DU_EARLY
#define CTN_DU_EARLY 1
#endif
#ifndef CTN_DU_LATE
#define CTN_DU_LATE 0
#endif
#ifndef CTN_DU_NOCLAMP
#define CTN_DU_NOCLAMP 0
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

// KB: Kred / 32; NSB: slice width / 16; NBW: 16-channel output blocks per wave (row
// part); D: LDS ring depth (tiles in flight + 1).
//
// Every streamed operand arrives by LDS-DMA into a D-slot ring, issued D-1 tiles
// ahead, with no VGPR-destination loads in the loop, so every wait is an explicit
// counted vmcnt and ~(D-1) tiles (40-100 KiB) stay in flight per CU across the
// barriers.  Per tile t (one LDS-only barrier):
//   wait for the DMA group the iteration reads -> barrier -> store C(t-1) from LDS
//   (whole 128-byte lines) -> DMA group t+D-1 -> [Bm transform of tile t+1 into the
//   B image] -> MFMAs of tile t -> epilogue of tile t into the C image.
// Operands: A ring (WS fragment image), Bm ring (plain: the B image itself; with a
// transform: raw rows, XOR-swizzled), R ring (plain case: residual rows), per-row
// statistics (cLN: one 256-byte copy per wave), C image (2 parities).
template <int KB, int NSB, int NBW, int EPI, int OPB, int NK, int D>
__global__ __launch_bounds__(DU_NT) void gemm_dual_kernel(GemmDual p) {
  constexpr int TM = DU_TM, WV = DU_WV, NT = DU_NT;
  constexpr int KR = KB * 32;          // reduction length of the row part (= D rows)
  constexpr int NS = NSB * 16;         // slice width
  constexpr int WNB = NSB / NBW;       // row-part waves per 16-row block
  constexpr int NV = NBW * 4;          // output channels per lane (row part)
  constexpr int WN = NSB / 4;          // col-part waves along n (4 n-blocks each)
  constexpr bool BXF = OPB != OP_PLAIN;                 // Bm transformed in LDS
  constexpr bool GST = NK == NORM_GLN && (BXF || EPI == EPI_NORM_BWD);   // per-utterance stats table
  constexpr bool CST = NK == NORM_CLN && (BXF || EPI == EPI_NORM_BWD) && CTN_DU_CST_DMA;   // per-row stats by DMA
  constexpr bool CSG = NK == NORM_CLN && (BXF || EPI == EPI_NORM_BWD) && !CTN_DU_CST_DMA;  // per-row stats from L2
  constexpr int A_SZ = TM * KR * 2, B_SZ = TM * NS * 2;
  constexpr int GA = A_SZ / 1024 / WV;                 // A blocks per wave per tile
  constexpr int G = GA + 1 + (CST ? 1 : 0);            // DMA instructions per wave per tile
  constexpr int SST = EPI == EPI_NORM_BWD ? 1 : 0;     // statistics stores per wave per tile
  constexpr int OFF_A = 0;                             // A ring
  constexpr int OFF_B = OFF_A + D * A_SZ;              // Bm ring (raw rows or B image)
  constexpr int OFF_R = OFF_B + D * B_SZ;              // residual ring (plain case)
  constexpr int OFF_BI = OFF_R + (BXF ? 0 : D * B_SZ); // B image, 2 parities (transform case)
  constexpr int OFF_C = OFF_BI + (BXF ? 2 * B_SZ : 0); // C image, 2 parities
  constexpr int OFF_ST = OFF_C + 2 * B_SZ;             // cLN row statistics ring
  constexpr int LDS = OFF_ST + (CST ? D * WV * 256 : 0);
  static_assert(GA * WV * 1024 == A_SZ, "A blocks split evenly over the waves");
  static_assert(BXF ? B_SZ == WV * 1024 : 2 * B_SZ == WV * 1024, "Bm/R blocks: one per wave");
  static_assert(2 * WNB == WV, "row part: 2 row blocks x WNB waves");
  static_assert(WN >= 1 && (WV / WN) * 4 * 16 == KR, "col part: 4x4 blocks per wave cover D");
  static_assert(NV == 4 || NV == 8, "epilogue vector width");
  static_assert(!BXF || NS == 128, "transform pass: 16 chunks per row");
  static_assert(LDS <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[LDS];   // DMA rings and images
  // Separate arrays for what no DMA writes: the compiler then proves their reads
  // independent of the in-flight LDS-DMA (a read it cannot separate from one gets a
  // vmcnt(0) in front of it, draining the ring).
  __shared__ __attribute__((aligned(16))) float sg[3 * NS];                 // gamma/beta/epilogue gamma
  __shared__ __attribute__((aligned(16))) float2 su[GST ? DU_MMAX : 1];     // gLN utterance statistics

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
  const rsrc_t rS = du_rsrc(p.stats, rows * 8);
  const bf16raw* W = reinterpret_cast<const bf16raw*>(p.W);

  // ---- row part: wave (mbw, nbg) owns rows mbw*16.. of each tile, channels
  //      n0 + nbg*16*NBW .. ; resident W fragments (permuted rows: lane groups get
  //      NV contiguous output channels)
  const int mbw = wid / WNB, nbg = wid % WNB;
  const int colbase = n0 + nbg * 16 * NBW + lg * NV;
  // ---- col part: wave (wp, wn) owns D blocks p in [wp*64, +64), n in [n0 + wn*64, +64)
  const int wp = wid / WN, wn = wid % WN;
  f32x4_t dacc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) dacc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ---- DMA sources (lane-constant; + tile offset in soffset)
  // A block f = wid*GA + u = (mb, kb): lane L -> row 16mb + ((L&15) ^ 12*((L>>4)&1)), chunk 4kb + (L>>4)
  uint32_t avo[GA];
  int arow[GA];
#pragma unroll
  for (int u = 0; u < GA; ++u) {
    const int f = wid * GA + u, mb = f / KB, kb = f % KB;
    arow[u] = 16 * mb + ((lane & 15) ^ (((lane >> 4) & 1) * 12));
    avo[u] = (uint32_t)(arow[u] * p.lda * 2 + (4 * kb + (lane >> 4)) * 16);
  }
  // Bm / R block of this wave
  int brow;
  uint32_t bvo;
  bool is_r = false;
  if constexpr (BXF) {   // raw rows: wave w -> rows 4w..4w+3, lane L -> physical chunk L&15
    brow = 4 * wid + (lane >> 4);
    bvo = (uint32_t)(brow * p.ldb * 2 + (n0 + 8 * ((lane & 15) ^ (brow & 15))) * 2);
  } else if (wid < 4) {  // B image block cb = wid (du_boff is lane-linear per block)
    const int q8 = lane >> 3;
    brow = 4 * (q8 ^ ((q8 >> 1) & 1)) + ((lane >> 1) & 3);
    bvo = (uint32_t)(brow * p.ldb * 2 + (n0 + 16 * wid + 8 * (lane & 1)) * 2);
  } else {               // residual rows: block q -> rows 8q.., physical chunk L&7
    is_r = true;
    brow = 8 * (wid - 4) + (lane >> 3);
    bvo = (uint32_t)(brow * p.ldr * 2 + (n0 + 8 * ((lane & 7) ^ (brow & 7))) * 2);
  }
  auto clampt = [&](int t) __attribute__((always_inline)) { return t < t1 ? t : t1 - 1; };
  auto dma = [&](int t) __attribute__((always_inline)) {   // group of tile t -> slot t % D
    if constexpr (CTN_DU_EXP & 2) return;
    const int slot = t % D, tk = (t * TM) % Kp;
#pragma unroll
    for (int u = 0; u < GA; ++u) {
      // rows of padded frames arrive as zeros (out-of-range offset)
      const uint32_t vo = tk + arow[u] < Kv ? avo[u] : DU_OOB;
      du_dma16(rA, smem + OFF_A + slot * A_SZ + (wid * GA + u) * 1024, vo, t * TM * p.lda * 2);
    }
    if constexpr (BXF) {
      du_dma16(rB, smem + OFF_B + slot * B_SZ + wid * 1024, bvo, t * TM * p.ldb * 2);
    } else {
      if (!is_r) du_dma16(rB, smem + OFF_B + slot * B_SZ + wid * 1024, bvo, t * TM * p.ldb * 2);
      else du_dma16(rR, smem + OFF_R + slot * B_SZ + (wid - 4) * 1024, bvo, t * TM * p.ldr * 2);
    }
    if constexpr (CST) du_dma4(rS, smem + OFF_ST + (slot * WV + wid) * 256, (uint32_t)(lane * 4), t * TM * 8);
  };
  // vmcnt that retires DMA group tq at the top of iteration t (k = t - t0): the
  // operations issued after it, by the fixed per-iteration order
  // [C store (k >= 1), DMA group (G, only for tiles < t1), statistics store (SST)]
  auto ops_after = [&](int tq, int t) __attribute__((always_inline)) {
    const int nt = t1 - t0;
    const int j = (CTN_DU_NOCLAMP && tq > t1 - 1 ? t1 - 1 : tq) - t0, k = t - t0;
    auto grp = [&](int jj) { return CTN_DU_NOCLAMP && jj >= nt ? 0 : G; };
    int n = 0, kfrom;
    if (j <= D - 2) {
      for (int jj = j + 1; jj <= D - 2; ++jj) n += grp(jj);
      kfrom = 0;
    } else {
      n = CTN_DU_LATE ? 0 : SST;   // ops of group j's own iteration issued after it
      kfrom = j - D + 2;
    }
    for (int kk = kfrom; kk < k; ++kk) n += (kk >= 1 ? 1 : 0) + grp(kk + D - 1) + SST;
    return n;
  };

  // CTN_DU_EARLY 0 (experiment): the first D-1 DMA groups go out before the resident
  // weight and the constants are loaded
  if (!CTN_DU_EARLY && t0 < t1)
    for (int i = 0; i < D - 1; ++i)
      if (!CTN_DU_NOCLAMP) dma(clampt(t0 + i));
      else if (t0 + i < t1) dma(t0 + i);
  v4u wf[NBW][KB];
  // from the fragment-ordered copy when there is one (1 KiB contiguous per wave and
  // fragment, as in gemm_ws)
  const bf16raw* WF = NBW == 2 ? reinterpret_cast<const bf16raw*>(p.Wf) : nullptr;
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb) {
    const int n = n0 + nbg * 16 * NBW + (lr >> 2) * NV + nb * 4 + (lr & 3);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
      if constexpr (CTN_DU_EXP & 256) wf[nb][kb] = v4u{(uint32_t)n, (uint32_t)kb, 0u, 0u};   // no weight loads
      else if (WF) wf[nb][kb] = ldg16(WF + frag_offset(sl * WNB + nbg, nb, kb, lane, KR));
      else wf[nb][kb] = ldg16(W + (size_t)n * p.ldw + kb * 32 + lg * 8);
  }
  const float eal = EPI == EPI_NORM_BWD ? p.alpha[0] : 0.f;
  const float bal = OPB == OP_PRELU_NORM ? p.bop.alpha[0] : 0.f;
  for (int c = tid; c < NS; c += NT) {
    sg[c] = BXF ? p.bop.gamma[n0 + c] : 0.f;
    sg[NS + c] = BXF ? p.bop.beta[n0 + c] : 0.f;
    sg[2 * NS + c] = EPI == EPI_NORM_BWD ? p.gamma[n0 + c] : 0.f;
  }
  if constexpr (GST)
    for (int m = tid; m < p.g.M; m += NT) su[m] = (BXF ? p.bop.stats : p.stats)[m];
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) du_ready(wf[nb][kb]);
  asm volatile("" ::"v"(eal), "v"(bal));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // nothing but the ring in flight from here
  __syncthreads();

  // ---- lane-constant LDS read addresses
  const int rbase = mbw * KB * 1024 + lg * 256 + ((lr ^ ((lg & 1) * 12)) << 4);   // + kb * 1024
  const int q = lr >> 2, pp = lr & 3;
  int abase[2], bbase[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * lg + 4 * h + q;
    abase[h] = (lg >> 1) * KB * 1024 + 2 * wp * 1024 + (pp >> 1) * 256 + (((row & 15) ^ ((pp >> 1) * 12)) << 4) +
               (pp & 1) * 8;
    bbase[h] = wn * 4 * 1024 + du_boff(row, 4 * pp);
  }
  const int erow = mbw * 16 + lr;                 // epilogue row of each tile
  const int ecol = colbase - n0;                  // epilogue column inside the slice
  // C image: row-major NS*2 bytes per row, NV-element granules XOR (row & 15)
  const int cw = erow * NS * 2 + (((ecol / NV) ^ (erow & 15)) * NV * 2);
  // C store pass: thread -> row tid/16, granule tid%16 (NS/16 elements)
  constexpr int CG = NS / 16;                     // elements per store granule (8 or 4)
  const int crow = tid >> 4, cgr = tid & 15;
  const int cr = crow * NS * 2 + ((cgr ^ (crow & 15)) * CG * 2);
  const uint32_t cvo = (uint32_t)(crow * p.ldc * 2 + (n0 + cgr * CG) * 2);
  // epilogue residual / pre-activation read
  int rdo;
  if constexpr (BXF) rdo = erow * 256 + (((ecol >> 3) ^ (erow & 15)) << 4);                       // raw rows
  else rdo = erow * 128 + ((((ecol >> 3) ^ (erow & 7)) << 4)) + ((ecol >> 2) & 1) * 8;          // R ring
  // transform pass (BXF): lane -> row 4w + (l&3), physical chunk ((l>>2) + 4(l&3)) & 15
  const int xrow = 4 * wid + (lane & 3), xp = ((lane >> 2) + 4 * (lane & 3)) & 15;
  const int xg = xp ^ (xrow & 15);                // global chunk (channels n0 + 8xg ..)
  const int xrd = xrow * 256 + xp * 16, xwr = du_boff(xrow, 8 * xg);

  double run_s = 0.0, run_q = 0.0;
  const int tpu = Kp / TM, m0 = t0 / tpu;
  int run_m = m0;
  const int kmax = ws_runs_kmax(ntile, nr, tpu);
  double2* run_slab = p.grp_slab + (((size_t)rr * S + sl) * WV + wid) * kmax;

  // statistics of frame row r (tile-relative rt) of tile t whose ring slot is `slot`
  auto row_stat = [&](int t, int slot, int rt) __attribute__((always_inline)) {
    if constexpr (GST) return su[(t * TM) / Kp];
    else if constexpr (CSG) return p.stats[t * TM + rt];
    else return *reinterpret_cast<const float2*>(smem + OFF_ST + (slot * WV + wid) * 256 + rt * 8);
  };

  auto transform = [&](auto le1, int t) __attribute__((always_inline)) {   // raw Bm(t) -> B image (t & 1)
    constexpr bool LE1 = decltype(le1)::value;
    if constexpr (CTN_DU_EXP & 16) return;
    const int slot = t % D;
    v4u v = *reinterpret_cast<const v4u*>(smem + OFF_B + slot * B_SZ + xrd);
    const float2 st = row_stat(t, slot, xrow);
    const float4 g0 = *reinterpret_cast<const float4*>(&sg[8 * xg]), g1 = *reinterpret_cast<const float4*>(&sg[8 * xg + 4]);
    const float4 b0 = *reinterpret_cast<const float4*>(&sg[NS + 8 * xg]), b1 = *reinterpret_cast<const float4*>(&sg[NS + 8 * xg + 4]);
    const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    const f32x2_t m2 = {st.x, st.x};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      f32x2_t x = {__uint_as_float(v[e] << 16), __uint_as_float(v[e] & 0xffff0000u)};
      if constexpr (OPB == OP_PRELU_NORM) x = prelu2<LE1>(x, bal);
      x = pfma(x - m2, f32x2_t{st.y * gv[2 * e], st.y * gv[2 * e + 1]}, f32x2_t{bv[2 * e], bv[2 * e + 1]});
      v[e] = pk_bf16(x[0], x[1]);
    }
    // cLN: padded frames' row statistics are not finite; gLN: A is zero there
    if constexpr (NK == NORM_CLN) {
      if ((t * TM) % Kp + xrow >= Kv) v = v4u{0u, 0u, 0u, 0u};
    }
    stg16(smem + OFF_BI + (t & 1) * B_SZ + xwr, v);
  };

  auto compute = [&](int t, f32x4_t (&acc)[NBW]) __attribute__((always_inline)) {
    if constexpr (CTN_DU_PRIO) __builtin_amdgcn_s_setprio(1);
    const char* a = smem + OFF_A + (t % D) * A_SZ;
    const char* bsl = BXF ? smem + OFF_BI + (t & 1) * B_SZ : smem + OFF_B + (t % D) * B_SZ;
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
    if constexpr (CTN_DU_PRIO) __builtin_amdgcn_s_setprio(0);
  };

  // row epilogue of tile t: lane holds row t*TM + erow, channels colbase..+NV -> C image (t & 1)
  auto epilogue = [&](auto le1, int t, const f32x4_t (&acc)[NBW]) __attribute__((always_inline)) {
    constexpr bool LE1 = decltype(le1)::value;
    if constexpr (CTN_DU_EXP & 64) {
      *reinterpret_cast<float*>(smem + OFF_C + (t & 1) * B_SZ + cw) = acc[0][0];
      return;
    }
    const int slot = t % D;
    f32x2_t v2[NV / 2];
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      v2[2 * nb] = f32x2_t{acc[nb][0], acc[nb][1]};
      v2[2 * nb + 1] = f32x2_t{acc[nb][2], acc[nb][3]};
    }
    uint32_t rw[NV / 2];
    if constexpr (NV == 8) {
      const v4u r4 = *reinterpret_cast<const v4u*>(smem + (BXF ? OFF_B : OFF_R) + slot * B_SZ + rdo);
      if constexpr (CTN_DU_DBG & 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      rw[0] = r4[0]; rw[1] = r4[1]; rw[2] = r4[2]; rw[3] = r4[3];
    } else {
      const uint2 r2 = *reinterpret_cast<const uint2*>(smem + (BXF ? OFF_B : OFF_R) + slot * B_SZ + rdo);
      rw[0] = r2.x; rw[1] = r2.y;
    }
    f32x2_t s2 = {0.f, 0.f}, q2 = {0.f, 0.f};
    if constexpr (EPI == EPI_RESID) {
#pragma unroll
      for (int c = 0; c < NV / 2; ++c) v2[c] += f32x2_t{__uint_as_float(rw[c] << 16), __uint_as_float(rw[c] & 0xffff0000u)};
    } else {
      const float2 est = row_stat(t, slot, erow);
      if constexpr (CTN_DU_DBG & 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const f32x2_t rs = {est.y, est.y}, ms = {-est.x * est.y, -est.x * est.y};
#pragma unroll
      for (int c = 0; c < NV / 2; ++c) {
        const float2 g = *reinterpret_cast<const float2*>(&sg[2 * NS + ecol + 2 * c]);
        const f32x2_t x = {__uint_as_float(rw[c] << 16), __uint_as_float(rw[c] & 0xffff0000u)};
        const f32x2_t ah = pfma(prelu2<LE1>(x, eal), rs, ms);   // hat a
        const f32x2_t ga = v2[c] * f32x2_t{g.x, g.y};
        s2 += ga;
        q2 = pfma(ga, ah, q2);
      }
    }
    char* cdst = smem + OFF_C + (t & 1) * B_SZ + cw;
    if constexpr (NV == 8)
      stg16(cdst, v4u{pk_bf16(v2[0][0], v2[0][1]), pk_bf16(v2[1][0], v2[1][1]), pk_bf16(v2[2][0], v2[2][1]),
                      pk_bf16(v2[3][0], v2[3][1])});
    else
      *reinterpret_cast<uint2*>(cdst) = make_uint2(pk_bf16(v2[0][0], v2[0][1]), pk_bf16(v2[1][0], v2[1][1]));
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
        float s = s2[0] + s2[1], ss = q2[0] + q2[1];
#if CTN_DU_PERMLANE
        s = xsum_rows(s);
        ss = xsum_rows(ss);
#else
        s += __shfl_xor(s, 16, 64); ss += __shfl_xor(ss, 16, 64);
        if constexpr (CTN_DU_DBG & 4) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        s += __shfl_xor(s, 32, 64); ss += __shfl_xor(ss, 32, 64);
        if constexpr (CTN_DU_DBG & 4) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
        p.grp_slab[(size_t)(t * TM + erow) * (S * WNB) + sl * WNB + nbg] = make_double2((double)s, (double)ss);
        if constexpr (CTN_DU_DBG & 16) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
  };

  // C(t) from its LDS image to global memory: every wave stores whole rows
  auto store_c = [&](int t) __attribute__((always_inline)) {
    const char* src = smem + OFF_C + (t & 1) * B_SZ + cr;
    const uint32_t vo = cvo + (uint32_t)(t * TM * p.ldc * 2);   // soffset 0: see du_bstore
    if constexpr (CG == 8) {
      const v4u v = *reinterpret_cast<const v4u*>(src);
      if constexpr (!(CTN_DU_EXP & 1)) __builtin_amdgcn_raw_buffer_store_b128(v, rC, vo, 0, 0);
      else asm volatile("" ::"v"(v));
    } else {
      typedef uint32_t v2u __attribute__((ext_vector_type(2)));
      const v2u v = *reinterpret_cast<const v2u*>(src);
      if constexpr (!(CTN_DU_EXP & 1)) __builtin_amdgcn_raw_buffer_store_b64(v, rC, vo, 0, 0);
      else asm volatile("" ::"v"(v));
    }
  };

  auto run = [&](auto le1) __attribute__((always_inline)) {
    f32x4_t acc[NBW];
    if (CTN_DU_EARLY)
      for (int i = 0; i < D - 1; ++i)
        if (!CTN_DU_NOCLAMP) dma(clampt(t0 + i));
        else if (t0 + i < t1) dma(t0 + i);
    for (int t = t0; t < t1; ++t) {
      // BXF: the transform reads raw Bm of tile t+1 this iteration, so wait for its group
      const int tq = BXF ? t + 1 : t;
      if constexpr (CTN_DU_DBG & 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if constexpr (!(CTN_DU_EXP & 128)) du_vmwait(ops_after(tq, t));
      if (BXF && t == t0) {   // the first tile's raw rows: transform them before everything
        lds_barrier();
        transform(le1, t0);
      }
      lds_barrier();
      if (t > t0) store_c(t - 1);
      if (!CTN_DU_LATE) {
        if (!CTN_DU_NOCLAMP) dma(clampt(t + D - 1));
        else if (t + D - 1 < t1) dma(t + D - 1);
      }
      if constexpr (BXF) transform(le1, clampt(t + 1));
      compute(t, acc);
      if constexpr (CTN_DU_EXP & 32) __builtin_amdgcn_sched_barrier(0);
      // cLN with DMA'd row statistics: no LDS-DMA in flight while the epilogue reads
      // its LDS operands (the one configuration measured reproducible)
      if constexpr (CST || (CTN_DU_DBG & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      epilogue(le1, t, acc);
      if (CTN_DU_LATE) {   // after the epilogue: its slot (t-1)%D was last read before this phase's barrier
        if (!CTN_DU_NOCLAMP) dma(clampt(t + D - 1));
        else if (t + D - 1 < t1) dma(t + D - 1);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the workgroup ends
    lds_barrier();
    store_c(t1 - 1);
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
      for (int e = 0; e < 4; ++e)
        if constexpr (CTN_DU_EXP & 512) asm volatile("" ::"v"(dacc[i][j][e]));   // timing: no D partial stores
        else Dp[(size_t)((wp * 4 + i) * 16 + 4 * lg + e) * p.Nout + n] = dacc[i][j][e];
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// CTN_GEMM_DUAL=<mask> selects the dual kernels per pair: bit 0 the (256 -> 512,
// norm-backward) pair "A" (gy.W2 + dW2), bit 1 the (512 -> 256, residual) pair "B"
// (gh1.W1 + dW1); cleared bits run the row GEMM + column GEMM kernels.  Read on every
// query so a process can compare both paths (tests/test_gpu_tblock.py).  Default 1:
// pair A measures 109 us against 62 + 60 us for its two kernels; pair B 103 us against
// 49 + 45 us (tools/microbench/dual_bench.hip), so B stays on the two kernels.
static int dual_mask() {
  const char* e = getenv("CTN_GEMM_DUAL");
  return e ? atoi(e) : 1;
}

// (Kred, Nout) -> (KB, NSB, NBW); S = 4 slices
static bool dual_shape(int Kred, int Nout, int* kb, int* nsb, int* nbw) {
  if (Kred == 256 && Nout == 512) { *kb = 8; *nsb = 8; *nbw = 2; return true; }   // gy.W2, dW2
  if (Kred == 512 && Nout == 256) { *kb = 16; *nsb = 4; *nbw = 1; return true; }  // gh1.W1, dW1
  return false;
}

bool gemm_dual_eligible(DType dt, const GemmDual& p) {
  int kb, nsb, nbw;
  if (dt != BF16 || !dual_shape(p.Kred, p.Nout, &kb, &nsb, &nbw)) return false;
  const bool pairA = p.Kred == 256 && p.epi == EPI_NORM_BWD && p.bop.kind == OP_PRELU_NORM;
  const bool pairB = p.Kred == 512 && p.epi == EPI_RESID && p.bop.kind == OP_PLAIN;
  const int mask = dual_mask();
  if (!(pairA && (mask & 1)) && !(pairB && (mask & 2))) return false;
  if (pairA && gemm_dual_ws_eligible(p)) return true;            // wave-specialised kernel (ctn_dual_ws.hip)
  if (p.bop.kind != OP_PLAIN && p.bop.fold.slab) return false;   // needs final statistics
  if (p.g.Kp % DU_TM || p.lda % 8 || p.ldw % 8 || p.ldc % 8 || p.ldr % 8 || p.ldb % 8) return false;
  if (p.g.rows() / DU_TM < 1 || p.g.rows() * (p.Kred > p.Nout ? p.Kred : p.Nout) * 2 >= (1L << 31)) return false;
  if (p.norm == NORM_GLN && p.g.M > DU_MMAX) return false;
  if (pairA && p.stats != p.bop.stats) return false;   // one statistics table serves both
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
  w.waves = dual_slices(p) * (gemm_dual_ws_eligible(p) ? dual_ws_row_waves(p) : DU_WV);   // ctn_dual_ws.hip
  w.kmax = ws_runs_kmax(w.ntile, w.grid, w.tpu);
  return w;
}

int gemm_dual_group_parts(const GemmDual& p) {
  int kb, nsb, nbw;
  dual_shape(p.Kred, p.Nout, &kb, &nsb, &nbw);
  if (p.norm != NORM_GLN)   // per (slice, row wave), or per slice (ctn_dual_ws.hip, CTN_DV_CLNC)
    return dual_slices(p) * (gemm_dual_ws_eligible(p) ? dual_ws_cln_parts_per_slice() : nsb / nbw);
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
    hipLaunchKernelGGL((gemm_dual_kernel<8, 8, 2, EPI_NORM_BWD, OP_PRELU_NORM, NK, CTN_DU_DA>), grid, dim3(DU_NT), 0, s, p);
  else if (p.Kred == 512 && p.epi == EPI_RESID && p.bop.kind == OP_PLAIN)
    hipLaunchKernelGGL((gemm_dual_kernel<16, 4, 1, EPI_RESID, OP_PLAIN, NORM_GLN, 3>), grid, dim3(DU_NT), 0, s, p);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_gemm_dual(const GemmDual& p, hipStream_t s) {
  if (!gemm_dual_eligible(BF16, p)) return hipErrorInvalidValue;
  if (gemm_dual_ws_eligible(p)) return launch_gemm_dual_ws(p, s);
  const int nk = p.bop.kind != OP_PLAIN ? p.bop.norm : p.norm;
  return nk == NORM_GLN ? dual_launch_nk<NORM_GLN>(p, s) : dual_launch_nk<NORM_CLN>(p, s);
}

}  // namespace ctn
