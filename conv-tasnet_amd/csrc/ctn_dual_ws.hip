// Wave-specialised dual GEMM, bf16, gfx950: the TemporalBlock backward's second 1x1
// conv ("pair A", conv_tasnet.py:256-263 backward) in one pass over gy and d:
//   C        = g_n2 = gy . W2                    (dL/d norm-2 output, stored bf16)
//   grp_slab : norm-2 backward sums of (g_n2*gamma2, g_n2*gamma2*hat a2)
//   Dpart    = gy^T . (gamma2 * hat a2 + beta2)  (dW2 partial per row range)
// with hat a2 = (PReLU(d) - mean) * rstd (gLN per utterance or cLN per frame row).
// Operands, outputs and partial layouts are those of gemm_dual_kernel's pair A
// (ctn_gemm_dual.hip); C and Dpart are bit-identical to it (same MFMA sequences, same
// operand transform), the statistics differ only by summation order.
//
// Schedule.  gemm_dual_kernel runs every wave through one barrier per tile: wait for
// the tile's LDS-DMA, then staging, MFMA and epilogue in lockstep, so the phases add
// up.  Here the roles are split inside the workgroup (16 waves,
// 4 per SIMD):
//   * 4 memory waves LDS-DMA the tiles PF tiles ahead into an LDS ring of NSL slots
//     (A = gy in MFMA fragment order, R = raw d of the slice, the tile's statistics),
//     wait for their own DMA with a counted vmcnt, write B = op(d) (PReLU + norm + affine,
//     bf16) from R, and publish FULL;
//   * 4 row waves (32 output channels each, resident W2 fragments) run the row GEMM of
//     both 16-row blocks and the norm-2 backward epilogue (hat a from R in fp32), store
//     C straight to memory and publish DONE;
//   * 8 column waves accumulate the dW2 slice (64 x 64 each) as MFMA accumulators from
//     A and B and publish DONE.
// FULL / DONE are one generation word per wave per slot in LDS (a memory wave waits
// for every DONE of tile t-NSL before refilling its slot), so the MFMAs of one tile
// overlap the DMA and transforms of the next ones, and no wave ever waits on another
// wave's memory operations.  Every LDS read of another wave's data happens after that
// wave's `s_waitcnt lgkmcnt(0)` + generation-word store and this wave's matching
// generation-word load.
#include <stdlib.h>

#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int DV_TM = 32;                        // frame rows per tile
// column waves: 8 (64 dW2 accumulators each, 4 waves per SIMD, 128 VGPRs per wave) or 4
// (128 accumulators each, 3 waves per SIMD, 168 VGPRs per wave; measured slower: 86-91 us
// at CJ=2 against 84 at 8 waves, CJ=1)
#ifndef CTN_DV_NC
#define CTN_DV_NC 8
#endif
constexpr int DV_NR = 4, DV_NC = CTN_DV_NC, DV_NMW = 4;  // row / column / memory waves
static_assert(DV_NC == 4 || DV_NC == 8, "column waves");
constexpr int DV_ND = DV_NR + DV_NC;             // waves that publish DONE
constexpr int DV_NT = (DV_ND + DV_NMW) * 64;     // 1024 threads
constexpr int DV_KB = 8, DV_KR = 256;            // reduction of the row part (gy channels)
constexpr int DV_NS = 128;                       // output channels per slice
constexpr int DV_GRID = 256;
// Slot layout.  CTN_DV_RAWB=1 (default): the B image holds the raw d slice exactly as the
// LDS-DMA lands it (row-major, 16-byte granules swizzled per row); the column waves apply
// PReLU + norm + affine to their B fragments (each fragment by the CJ waves that share
// it), the row waves read raw d from it, a slot is 24.8 KB and the ring holds 6 tiles.
// CTN_DV_RAWB=0: the memory waves write op(d) into a B image from a raw-d image R (33 KB
// slots, ring of 4) — op(d) once per element, but in the producer's critical path:
// 99.5 us against 79.5 us (RAWB=1, CJ=1) at the bench shape.
#ifndef CTN_DV_RAWB
#define CTN_DV_RAWB 1
#endif
constexpr bool DV_RB = CTN_DV_RAWB;
#ifndef CTN_DV_NSL
#define CTN_DV_NSL (CTN_DV_RAWB ? 6 : 4)
#endif
constexpr int DV_NSL = CTN_DV_NSL;               // LDS ring slots
// tiles a memory wave keeps in flight ahead of the one being consumed (<= NSL - 1: the
// slot refilled is the one the consumers released last)
#ifndef CTN_DV_PF
#define CTN_DV_PF (CTN_DV_NSL - 1)
#endif
constexpr int DV_PF = CTN_DV_PF;
static_assert(DV_PF >= 1 && DV_PF <= DV_NSL - 1, "ring look-ahead");
// the cLN form (c4's causal blocks) may take its own look-ahead
#ifndef CTN_DV_PF_CLN
#define CTN_DV_PF_CLN CTN_DV_PF
#endif
constexpr int DV_PF_CLN = CTN_DV_PF_CLN;
static_assert(DV_PF_CLN >= 1 && DV_PF_CLN <= DV_NSL - 1, "ring look-ahead (cLN)");
// Column-wave split of the 256 x 128 dW2 slice: each of the 8 waves owns CJ 16-column
// blocks x (16 / CJ) 16-row blocks (64 accumulator registers either way).  Fewer column
// blocks per wave means fewer waves share (and, RAWB=1, transform) each B fragment, at
// the price of more A fragment reads per wave: CJ=1 79.5 us, CJ=2 85.0 (bench shape).
#ifndef CTN_DV_CJ
#define CTN_DV_CJ 1
#endif
constexpr int DV_CJ = CTN_DV_CJ;
static_assert(DV_CJ == 1 || DV_CJ == 2 || DV_CJ == 4, "column blocks per column wave");
// N image (CTN_DV_NIMG=1, experiment, off; RAWB=1 only): the row waves, which already apply PReLU +
// norm to the raw d of their 16-byte granules in the epilogue, also write op(d) =
// gamma2 * hat a2 + beta2 (bf16) over that raw d in the B image, and the column waves wait
// for the four row waves' DONE of the tile instead of FULL and read op(d) fragments without
// any transform: op(d) is computed once per element instead of twice, the column waves lose
// their transform chain and the B statistics, and their split is free to read the fewest
// fragments (CTN_DV_CJN column blocks per wave).  op(d) is rounded from fmaf(hat a, gamma,
// beta) instead of fmaf(a - mean, rstd * gamma, beta): dW2 differs from the NIMG=0 kernel
// in the last bits of some bf16 operands; C and the statistics are unchanged.  Measured
// slower (microbenchmark, bench shape: 113-115 us at 8 column waves, 85-91 at 4, against
// 83-84 us without): the column waves then wait for the row waves' whole
// tile, and the row waves, which set the pace, carry the extra work.
#ifndef CTN_DV_NIMG
#define CTN_DV_NIMG 0
#endif
constexpr bool DV_NI = CTN_DV_NIMG && CTN_DV_RAWB;
#ifndef CTN_DV_CJN
#define CTN_DV_CJN 4
#endif
static_assert(CTN_DV_CJN == 1 || CTN_DV_CJN == 2 || CTN_DV_CJN == 4 || CTN_DV_CJN == 8, "column blocks per column wave (NIMG)");
// COLS mode (no operand transform to share): the split that reads the fewest fragments
#ifndef CTN_DV_CJC
#define CTN_DV_CJC 4
#endif
constexpr int DV_CJC = CTN_DV_CJC;
static_assert(DV_CJC == 1 || DV_CJC == 2 || DV_CJC == 4, "column blocks per column wave (COLS)");

// cLN: combine the four row waves' per-row statistics partials in LDS before storing
// (S entries per row instead of 4 S)
#ifndef CTN_DV_CLNC
#define CTN_DV_CLNC 1
#endif

// Column waves: two tiles per loop iteration (experiment, off): measured slower, 106.5
// against 81.3-82.8 us at the bench shape and 590 against 533-553 us at c4's
// (microbenchmark, one box) — a wave holding two slots releases the older
// one a tile later, which shortens the memory waves' look-ahead
#ifndef CTN_DV_C2
#define CTN_DV_C2 0
#endif

// Static wave priority per role (s_setprio once at the role's start): bits 0-1 row waves,
// 2-3 column waves, 4-5 memory waves (each a priority 0..3).  The SIMD's issue arbiter
// serves the higher priority first, so the memory wave sharing a SIMD with three
// consumers issues each tile's LDS-DMA as soon as its slot is free instead of behind the
// consumers' MFMA/VALU streams, and the row waves (whose stores feed the next kernel) go
// before the column waves.  Measured (microbenchmark, bench shape, three alternations on
// one box): gLN 81-89 us with none, 75-78 us with memory 3 + row 1
// (CTN_DV_PRIO=49) or memory 2 + row 1 (33); higher column priority slower (89-92 us); the
// c5 shape 84 -> 76 us; the cLN form (c4) flat to slightly slower, so it keeps none.
#ifndef CTN_DV_PRIO
#define CTN_DV_PRIO 49
#endif
#ifndef CTN_DV_PRIO_CLN
#define CTN_DV_PRIO_CLN 0
#endif
template <int SHIFT, int NK> CTN_DEV void dv_prio() {
  constexpr int pr = ((NK == NORM_CLN ? CTN_DV_PRIO_CLN : CTN_DV_PRIO) >> SHIFT) & 3;
  if constexpr (pr != 0) __builtin_amdgcn_s_setprio(pr);
}

// Row waves: A fragments read LA k-steps ahead of their MFMAs
#ifndef CTN_DV_LA
#define CTN_DV_LA 1
#endif
constexpr int DV_LA = CTN_DV_LA;

// Bound-finding builds only (tools/microbench/dual_ws_bench.hip -DCTN_DV_EXP=<bits>):
// bit 0 consumers skip all arithmetic (wait FULL, publish DONE), bit 1 no column part,
// bit 2 no epilogue math, bit 3 no C stores, bit 4 row waves store zeros and nothing else,
// bit 5 the memory waves issue no DMA (consumers read whatever the ring holds), bit 6 the
// row waves skip all arithmetic.
// 1: the row waves' output (dL/dn2) stores carry the nontemporal hint
#ifndef CTN_DV_NT
#define CTN_DV_NT 0
#endif
#ifndef CTN_DV_EXP
#define CTN_DV_EXP 0
#endif
// Diagnostic builds (tools/microbench/dual_ws_bench.hip): bit 4 the row waves store the
// raw d values they read from the ring in place of C (checked against d on the host);
// bit 3 is the bench's own (per-launch statistics dump).
#ifndef CTN_DV_DBG
#define CTN_DV_DBG 0
#endif

// Diagnostic build only (tools/microbench/dual_ws_bench.hip -DCTN_DV_STAMP=1): per wave,
// s_memtime cycles spent in each wait (row/column: FULL polls; memory: own-DMA vmcnt
// waits and DONE polls) and in the whole tile loop, summed into dv_stamps[wg][wave][4]
#ifndef CTN_DV_STAMP
#define CTN_DV_STAMP 0
#endif
#if CTN_DV_STAMP
__device__ unsigned long long dv_stamps[1024 * 16 * 4];
#define DV_TS(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define DV_ACC(i, t0v) st_acc[i] += __builtin_amdgcn_s_memtime() - (t0v)
#define DV_STAMP_DECL unsigned long long st_acc[4] = {0, 0, 0, 0}
#define DV_STAMP_STORE                                                                    \
  do {                                                                                    \
    if (lane == 0)                                                                        \
      for (int i_ = 0; i_ < 4; ++i_) dv_stamps[((size_t)blockIdx.x * 16 + wid) * 4 + i_] = st_acc[i_]; \
  } while (0)
#else
#define DV_TS(v) \
  do {           \
  } while (0)
#define DV_ACC(i, t0v) \
  do {                 \
  } while (0)
#define DV_STAMP_DECL \
  do {                \
  } while (0)
#define DV_STAMP_STORE \
  do {                 \
  } while (0)
#endif

// slot layout (bytes)
constexpr int DV_A = DV_TM * DV_KR * 2;          // 16384: gy tile, WS fragment image (du_apiece)
constexpr int DV_BST = 1024 + 32;                // (RAWB=0) B block stride: 16 columns x 32 rows + 32 B
constexpr int DV_B = DV_RB ? DV_TM * DV_NS * 2   // raw d slice, 256-byte rows (dv_rbgr)
                           : 8 * DV_BST;         // op(d) slice in 4-row x 16-column blocks (du_boff)
constexpr int DV_R = DV_RB ? 0 : DV_TM * DV_NS * 2;   // (RAWB=0) raw d rows, 16-byte granules XOR row
constexpr int DV_ST = DV_RB ? 256 : DV_NMW * 256;     // statistics (RAWB=0: 256 B per memory wave)
constexpr int OFF_A = 0, OFF_B = OFF_A + DV_A, OFF_R = OFF_B + DV_B, OFF_ST = OFF_R + DV_R;
constexpr int DV_SLOT = OFF_ST + DV_ST;

// 16-byte piece kc (8 channels) of frame row `row` in the A image (as ctn_gemm_dual.hip's du_apiece)
CTN_DEV int dv_apiece(int row, int kc) {
  const int lg = kc & 3;
  return (row >> 4) * DV_KB * 1024 + (kc >> 2) * 1024 + lg * 256 + (((row & 15) ^ ((lg & 1) * 12)) << 4);
}
// byte offset of (row, col) inside one 16-column block of the B image
CTN_DEV int dv_boff(int row, int col) {
  const int rg = row >> 2;
  return ((rg ^ ((rg >> 1) & 1)) << 7) + (row & 3) * 32 + (col & 15) * 2;
}
// 16-byte granule g (channels 8g..8g+7) of row r in the R image (RAWB=0)
CTN_DEV int dv_roff(int r, int g) { return r * 256 + ((g ^ (r & 15)) << 4); }
// RAWB=1 B image: granule g of row r at r * 256 + 16 * position, position = g's low bit
// and (g/2) XOR a 3-bit row hash.  The hash differs between the 8 rows a column wave's
// transposed 8-byte reads touch in one half-wave ({q, 8+q} or {4+q, 12+q}, q < 4, and the
// same + 16), so those 32 reads hit 32 distinct 8-byte bank pairs; a row wave's 16-byte
// reads of 16 rows see at most 2-way conflicts.
CTN_DEV int dv_rbhash(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }
CTN_DEV int dv_rbpos(int r, int g) { return (g & 1) | ((((g >> 1) ^ dv_rbhash(r)) & 7) << 1); }
CTN_DEV int dv_rbgr(int r, int g) { return r * 256 + (dv_rbpos(r, g) << 4); }
// counted wait for the RAWB=1 ring depth (up to 5 tiles x 7 DMA instructions in flight)
CTN_DEV void dv_vmwait(int n) {
#define CTN_VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n < 0 ? 0 : n) {
    CTN_VMW(0) CTN_VMW(1) CTN_VMW(2) CTN_VMW(3) CTN_VMW(4) CTN_VMW(5) CTN_VMW(6) CTN_VMW(7)
    CTN_VMW(8) CTN_VMW(9) CTN_VMW(10) CTN_VMW(11) CTN_VMW(12) CTN_VMW(13) CTN_VMW(14) CTN_VMW(15)
    CTN_VMW(16) CTN_VMW(17) CTN_VMW(18) CTN_VMW(19) CTN_VMW(20) CTN_VMW(21) CTN_VMW(22) CTN_VMW(23)
    CTN_VMW(24) CTN_VMW(25) CTN_VMW(26) CTN_VMW(27) CTN_VMW(28) CTN_VMW(29) CTN_VMW(30) CTN_VMW(31)
    CTN_VMW(32) CTN_VMW(33) CTN_VMW(34)
    default: asm volatile("s_waitcnt vmcnt(35)" ::: "memory"); break;
  }
#undef CTN_VMW
}

// counted wait with a compile-time count (the steady state of the ring: a runtime switch
// over the count compiles to ~300 scalar instructions per tile)
template <int N> CTN_DEV void dv_vmwait_c() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <bool LE1> CTN_DEV float dv_prelu(float x, float al) { return prelu_nq<LE1>(x, al); }

CTN_DEV s16x4_t dv_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}

// Generation words.  Every lane reads the same word (wave-uniform by readfirstlane);
// the poll is followed by a compiler barrier so no LDS read of the published data is
// issued before the word that publishes it has been seen (LDS executes one wave's
// DS instructions in order).
// The spin is bounded (CTN_SPIN_LIMIT polls, about 0.2 s): a protocol error sets
// CTN_DEVERR_SPIN in the device error word (p.err, ctn_device_status) and the launch
// ends, reported as failed by the host, instead of a wave that never finishes.
// (Volatile accesses keep their address space only through an explicitly LDS-typed
// pointer: through a generic one they become FLAT operations, whose waits drain every
// outstanding global load of the wave.)
typedef __attribute__((address_space(3))) volatile v4u lds_v4u;
typedef __attribute__((address_space(3))) volatile uint32_t lds_u32;
template <int N> CTN_DEV void dv_wait(const uint32_t* f, uint32_t gen, uint32_t* err) {
  static_assert(N % 4 == 0, "generation words per slot: whole 16-byte reads");
  const lds_v4u* fl = (const lds_v4u*)(f);
  uint32_t it = 0;
  for (; it < CTN_SPIN_LIMIT; ++it) {
    uint32_t mn = 0xffffffffu;
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
      const v4u a = fl[i];
      mn = min(mn, min(min(a[0], a[1]), min(a[2], a[3])));
    }
    if (__builtin_amdgcn_readfirstlane(mn) >= gen) break;
    __builtin_amdgcn_s_sleep(1);
  }
  if (it == CTN_SPIN_LIMIT) spin_timeout(err);
  asm volatile("" ::: "memory");
}
// publish: this wave's LDS writes (and reads) complete, then the generation word
CTN_DEV void dv_signal(uint32_t* f, uint32_t gen) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  *(lds_u32*)(f) = gen;
  asm volatile("" ::: "memory");
}

// COLS: the column GEMM alone (ctn_gemm.hip's GemmCols dW = A^T B with plain operands,
// e.g. dW1 = gh1^T . x): no row waves, op = identity, and the partial stored transposed
// (Dpart[range][n][k], the GemmCols layout [chunk][P][Q] with P = Nout, Q = Kred) through
// LDS at the end.  12 waves: column waves 0-7, memory waves 8-11.
template <int NK, int NSL, int PF, bool COLS = false>
__global__ __launch_bounds__(COLS ? (DV_NC + DV_NMW) * 64 : DV_NT) void gemm_dual_ws_kernel(GemmDual p) {
  constexpr int NR = COLS ? 0 : DV_NR;      // row waves
  constexpr int ND = NR + DV_NC;            // waves that publish DONE
  constexpr int TM = DV_TM, KB = DV_KB, KR = DV_KR, NS = DV_NS;
  constexpr int SLOT = DV_SLOT;
  static_assert(NSL * SLOT <= 160 * 1024 - 2048, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[NSL * SLOT];
  __shared__ __attribute__((aligned(16))) uint32_t fl_full[NSL][4];   // per memory wave
  __shared__ __attribute__((aligned(16))) uint32_t fl_done[NSL][ND];   // per row / column wave
  __shared__ __attribute__((aligned(16))) float sgb[2][NS];            // gamma2 / beta2 of the slice
  // cLN (CTN_DV_CLNC): the four row waves' per-row partials of a tile, two tiles deep, and
  // one generation word per (buffer, row wave)
  constexpr bool CLNC = NK == NORM_CLN && !COLS && CTN_DV_CLNC;
  __shared__ __attribute__((aligned(16))) double2 cln_scr[CLNC ? 2 : 1][CLNC ? DV_NR * DV_TM : 1];
  __shared__ __attribute__((aligned(16))) uint32_t fl_rows[2][4];

  // wave id through readfirstlane: wave-uniform to the compiler, so per-role pointers and
  // offsets live in SGPRs (the row waves are at the 128-VGPR limit of 4 waves per SIMD)
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int S = p.Nout / NS;
  const int nr = (int)gridDim.x / S;   // row ranges
  int rr, sl;
  {
    const int b = (int)blockIdx.x;
    if ((int)gridDim.x % (8 * S) == 0) {   // the S slices of a range on one XCD (L2 shares gy)
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
  const int Kp = p.g.Kp, Kv = p.g.K, tpu = Kp / TM;

  if (tid < NSL * 4) (&fl_full[0][0])[tid] = 0u;
  else if (tid < NSL * (4 + ND)) (&fl_done[0][0])[tid - NSL * 4] = 0u;
  else if (tid < NSL * (4 + ND) + 8) (&fl_rows[0][0])[tid - NSL * (4 + ND)] = 0u;
  if constexpr (!COLS)
    if (tid < 2 * NS) sgb[tid / NS][tid % NS] = (tid < NS ? p.bop.gamma : p.bop.beta)[n0 + tid % NS];
  __syncthreads();

  const float eal = COLS ? 0.f : p.alpha[0];
  const int kmax = ws_runs_kmax(ntile, nr, tpu);
  // COLS: the workgroup's transposed partial [n - n0][k] from the LDS image (COLS_LDT
  // floats per row) as whole 1-KiB rows of Dpart[range][n][k], by every wave
  constexpr int COLS_LDT = KR + 4;
  static_assert(!COLS || NS * COLS_LDT * 4 <= NSL * DV_SLOT, "transpose image fits the ring");
  static_assert(!COLS || DV_RB, "COLS takes the raw-B slot layout (no operand transform)");
  auto store_tr = [&](float* Dp) __attribute__((always_inline)) {
    const float* img = reinterpret_cast<const float*>(smem);
    for (int idx = tid; idx < NS * (KR / 4); idx += (DV_NC + DV_NMW) * 64) {
      const int nl = idx / (KR / 4), k4 = idx % (KR / 4);
      *reinterpret_cast<float4*>(Dp + (size_t)(n0 + nl) * KR + 4 * k4) =
          *reinterpret_cast<const float4*>(img + nl * COLS_LDT + 4 * k4);
    }
  };
  if (wid < NR) {
    // ======================= row waves =======================
    dv_prio<0, NK>();
    // wave r: output channels n0 + 32r .. +31 of both 16-row blocks of every tile, against
    // the resident W fragments (group 4*sl + r of the fragment-ordered copy, nb = 0, 1):
    // lane (lg, lr) holds channels 32r + 8lg .. +7 (slice-local) of frame rows lr, 16 + lr.
    const int r = wid;
    v4u wf[2][KB];
    const bf16raw* WF = reinterpret_cast<const bf16raw*>(p.Wf);
    const bf16raw* W = reinterpret_cast<const bf16raw*>(p.W);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int n = n0 + 32 * r + (lr >> 2) * 8 + nb * 4 + (lr & 3);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
        wf[nb][kb] = WF ? ldg16(WF + frag_offset(4 * sl + r, nb, kb, lane, KR))
                        : ldg16(W + (size_t)n * p.ldw + kb * 32 + lg * 8);
    }
    const int cl = 32 * r + 8 * lg;
    bf16raw* Cg = reinterpret_cast<bf16raw*>(p.C);
    // gamma2 (and, NIMG, beta2) of the lane's 8 channels: registers, or (NIMG, where the
    // registers are short) read per tile from the slice's LDS copy (p.bop.gamma == p.gamma:
    // gemm_dual_ws_eligible)
    float gamr[8];
    if constexpr (!DV_NI) {
      *reinterpret_cast<float4*>(gamr) = *reinterpret_cast<const float4*>(p.gamma + n0 + cl);
      *reinterpret_cast<float4*>(gamr + 4) = *reinterpret_cast<const float4*>(p.gamma + n0 + cl + 4);
    }
    const int rbase = lg * 256 + ((lr ^ ((lg & 1) * 12)) << 4);   // + rb * KB * 1024 + kb * 1024
    const int ro = DV_RB ? OFF_B + dv_rbgr(lr, 4 * r + lg)          // row lr; row 16 + lr at + 4096
                         : OFF_R + dv_roff(lr, 4 * r + lg);

    DV_STAMP_DECL;
    double run_s = 0.0, run_q = 0.0;
    const int m0 = t0 / tpu;
    int run_m = m0;
    double2* run_slab = p.grp_slab + (((size_t)rr * S + sl) * DV_NR + r) * kmax;
    auto flush = [&]() __attribute__((always_inline)) {
      const double s = wave_sum_dpp_d(run_s), ss = wave_sum_dpp_d(run_q);
      run_slab[run_m - m0] = make_double2(s, ss);
    };
    auto run = [&](auto le1) __attribute__((always_inline)) {
      constexpr bool LE1 = decltype(le1)::value;
      int slot = 0;
      uint32_t gen = 1;
      DV_TS(tl0);
      for (int t = t0; t < t1; ++t) {
        DV_TS(tw0);
        dv_wait<4>(fl_full[slot], gen, p.err);
        DV_ACC(0, tw0);
        char* base = smem + slot * SLOT;
        if constexpr (CTN_DV_EXP & 16) {   // C stores only (zeros)
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) stg16(Cg + ((size_t)t * TM + 16 * rb + lr) * p.ldc + n0 + cl, v4u{0u, 0u, 0u, 0u});
        } else if constexpr (!(CTN_DV_EXP & 65)) {
          f32x4_t acc[2][2];
#pragma unroll
          for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) acc[rb][nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          // the A fragments of k-step kb + LA are read while the MFMAs of kb run (the
          // interleave pinned below: the register-pressure scheduler would otherwise pull
          // each read down to its MFMAs and expose every read's latency)
          constexpr int LA = DV_LA;
          v4u bw[LA + 1][2];
          auto rd = [&](int kb) __attribute__((always_inline)) {
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
              bw[kb % (LA + 1)][rb] = *reinterpret_cast<const v4u*>(base + OFF_A + rb * KB * 1024 + rbase + kb * 1024);
          };
#pragma unroll
          for (int kb = 0; kb < LA && kb < KB; ++kb) rd(kb);
#pragma unroll
          for (int kb = 0; kb < KB; ++kb) {
            if (kb + LA < KB) rd(kb + LA);
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
              const v4u b = bw[kb % (LA + 1)][rb];
#pragma unroll
              for (int nb = 0; nb < 2; ++nb)
                acc[rb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[nb][kb]),
                                                                      __builtin_bit_cast(bf16x8_t, b), acc[rb][nb], 0, 0, 0);
            }
          }
          if constexpr (LA > 0) {
            __builtin_amdgcn_sched_group_barrier(0x100, 2 * (LA < KB ? LA : KB), 0);
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
              if (kb + LA < KB) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
              __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            }
          }
          // ---- epilogue: norm-2 backward sums, C image (16 bytes per lane and row).
          // (Summing ga * a and scaling by rstd once per row saves one FMA per element but
          // cancels when |mean| >> the spread of a: not used.)
          float s1[2] = {0.f, 0.f}, q1[2] = {0.f, 0.f};
          float gam[8], bet[8];
          if constexpr (DV_NI) {
            int co = cl >> 2;
            asm volatile("" : "+v"(co));   // re-read per tile: hoisted, they would hold 16 VGPRs
            const float4* g4 = reinterpret_cast<const float4*>(&sgb[0][0]);
            *reinterpret_cast<float4*>(gam) = g4[co];
            *reinterpret_cast<float4*>(gam + 4) = g4[co + 1];
            *reinterpret_cast<float4*>(bet) = g4[NS / 4 + co];
            *reinterpret_cast<float4*>(bet + 4) = g4[NS / 4 + co + 1];
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) gam[e] = gamr[e], bet[e] = 0.f;
          }
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            const v4u rw = *reinterpret_cast<const v4u*>(base + ro + rb * 4096);
            float2 est;
            if constexpr (NK == NORM_GLN) est = *reinterpret_cast<const float2*>(base + OFF_ST);   // the tile's utterance
            else if constexpr (DV_RB) est = *reinterpret_cast<const float2*>(base + OFF_ST + (16 * rb + lr) * 8);
            else est = *reinterpret_cast<const float2*>(base + OFF_ST + (2 * rb + (lr >> 3)) * 256 + (lr & 7) * 8);
            const float rs = est.y, ms = -est.x * est.y;
            const bool ok = NK == NORM_GLN || (t * TM) % Kp + 16 * rb + lr < Kv;   // cLN padded frames: stats not finite
            float f[8];
            unpack_bf16x8(rw, f);
            if constexpr (!(CTN_DV_EXP & 4)) {
              float nv[8];
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float a = dv_prelu<LE1>(f[e], eal);
                const float ah = ok ? fmaf(a, rs, ms) : 0.f;   // hat a
                const float ga = acc[rb][e >> 2][e & 3] * gam[e];
                s1[rb] += ga;
                q1[rb] = fmaf(ga, ah, q1[rb]);
                if constexpr (DV_NI) nv[e] = ok ? fmaf(ah, gam[e], bet[e]) : 0.f;   // op(d); padded cLN frames 0
              }
              if constexpr (DV_NI)   // over this lane's own raw granule (read above, by this wave only)
                *reinterpret_cast<v4u*>(base + ro + rb * 4096) =
                    v4u{pk_bf16(nv[0], nv[1]), pk_bf16(nv[2], nv[3]), pk_bf16(nv[4], nv[5]), pk_bf16(nv[6], nv[7])};
            }
            const v4u cv = {pk_bf16(acc[rb][0][0], acc[rb][0][1]), pk_bf16(acc[rb][0][2], acc[rb][0][3]),
                            pk_bf16(acc[rb][1][0], acc[rb][1][1]), pk_bf16(acc[rb][1][2], acc[rb][1][3])};
            // whole 16-byte lanes straight to memory (a wave covers 16 rows x 64 B)
            if constexpr (!(CTN_DV_EXP & 8))
              // wave-uniform 64-bit tile base + 32-bit lane offset (SGPR base, one VGPR)
              stg16h<CTN_DV_NT != 0>(Cg + (size_t)t * TM * p.ldc + n0 + (uint32_t)((16 * rb + lr) * p.ldc + cl),
                                     (CTN_DV_DBG & 16) ? rw : cv);
          }
          if constexpr (NK == NORM_GLN) {
            const int m = t / tpu;
            if (m != run_m) {
              flush();
              run_s = run_q = 0.0;
              run_m = m;
            }
            run_s += (double)(s1[0] + s1[1]);
            run_q += (double)(q1[0] + q1[1]);
          } else if constexpr (CLNC) {
            // per-row partial over this wave's 32 channels into LDS; once all four row
            // waves have written theirs, wave r sums rows 8r .. 8r+7 over the waves in
            // order 0..3 and stores one entry per (row, slice): a quarter of the
            // statistics bytes the finalize reads
            const int k = t - t0, bsel = k & 1;
            const uint32_t rgen = (uint32_t)(k >> 1) + 1u;
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
              const float s = xsum_rows(s1[rb]), ss = xsum_rows(q1[rb]);
              if (lg == 0) cln_scr[bsel][r * TM + 16 * rb + lr] = make_double2((double)s, (double)ss);
            }
            dv_signal(&fl_rows[bsel][r], rgen);
            dv_wait<4>(fl_rows[bsel], rgen, p.err);
            if (lane < 8) {
              const int row = 8 * r + lane;
              double s = 0.0, ss = 0.0;
#pragma unroll
              for (int w = 0; w < DV_NR; ++w) {
                const double2 v = cln_scr[bsel][w * TM + row];
                s += v.x;
                ss += v.y;
              }
              p.grp_slab[((size_t)t * TM + row) * S + sl] = make_double2(s, ss);
            }
          } else {
            // per-row partial over this wave's 32 channels (the four lane groups): one
            // entry per (row, slice, row wave), summed in that order by the finalize
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
              const float s = xsum_rows(s1[rb]), ss = xsum_rows(q1[rb]);
              if (lg == 0)
                p.grp_slab[((size_t)t * TM + 16 * rb + lr) * (S * DV_NR) + sl * DV_NR + r] = make_double2((double)s, (double)ss);
            }
          }
        }
        dv_signal(&fl_done[slot][r], gen);
        if (++slot == NSL) {
          slot = 0;
          ++gen;
        }
      }
      DV_ACC(3, tl0);
    };
    if (t0 < t1) {
      if (eal <= 1.f) run(std::true_type{});
      else run(std::false_type{});
      if constexpr (NK == NORM_GLN) flush();
    }
    DV_STAMP_STORE;
    return;
  }
  if (wid < ND) {
    // ======================= column waves =======================
    dv_prio<2, NK>();
    // wave c = (wp, wn) owns dW2 blocks p in [16 CI wp, +16 CI), n in [n0 + 16 CJ wn, +16 CJ):
    // dW2 += gy_tile^T . op(d)_tile, the reduction over the tile's 32 frame rows
    // the slice's 16 x 8 blocks of 16 x 16: waves in a (NC / (8 / CJ)) x (8 / CJ) grid,
    // each CI x CJ blocks
    constexpr int CJ = COLS ? DV_CJC : (DV_NI ? CTN_DV_CJN : DV_CJ), CI = 16 * (8 / CJ) / DV_NC;
    static_assert(CI >= 2 && CI <= 16 && CI % 2 == 0, "column split");
    const int c = wid - NR, wp = c / (8 / CJ), wn = c % (8 / CJ);
    DV_STAMP_DECL;
    f32x4_t dacc[CI][CJ];
#pragma unroll
    for (int i = 0; i < CI; ++i)
#pragma unroll
      for (int j = 0; j < CJ; ++j) dacc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // lane-constant LDS addresses (ctn_gemm_dual.hip's A addressing; B: RAWB=1 row-major
    // granules, block j at bbase ^ (j << 5); RAWB=0 blocks at stride DV_BST)
    const int q = lr >> 2, pp = lr & 3;
    int abase[2], bbase[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 8 * lg + 4 * h + q;
      abase[h] = (lg >> 1) * KB * 1024 + (CI / 2) * wp * 1024 + (pp >> 1) * 256 + (((row & 15) ^ ((pp >> 1) * 12)) << 4) +
                 (pp & 1) * 8;
      bbase[h] = DV_RB ? dv_rbgr(row, 2 * CJ * wn + (pp >> 1)) + 8 * (pp & 1) : wn * CJ * DV_BST + dv_boff(row, 4 * pp);
    }
    // RAWB=1: the B fragment of block j holds raw d of column 16 (CJ wn + j) + lr (slice-local)
    // at frame rows 8 lg .. 8 lg + 7; op(d) is applied here with the memory-side transform's
    // exact float operations (so C, Dpart and the statistics match RAWB=0 bit for bit)
    float cg[CJ], cb[CJ];
#pragma unroll
    for (int j = 0; j < CJ; ++j) {
      cg[j] = COLS ? 0.f : sgb[0][16 * (CJ * wn + j) + lr];
      cb[j] = COLS ? 0.f : sgb[1][16 * (CJ * wn + j) + lr];
    }
    const float bal = COLS ? 0.f : p.bop.alpha[0];
    // one tile's B fragments (raw d -> op(d) for RAWB=1), read from the ring slot at `base`
    auto load_b = [&](auto le1, int t, const char* base, bf16x8_t* bfr) __attribute__((always_inline)) {
      constexpr bool LE1 = decltype(le1)::value;
      const char* bb = base + OFF_B;
#pragma unroll
      for (int j = 0; j < CJ; ++j) {
        const s16x4_t lo = dv_tr(bb + (DV_RB ? bbase[0] ^ (j << 5) : bbase[0] + j * DV_BST));
        const s16x4_t hi = dv_tr(bb + (DV_RB ? bbase[1] ^ (j << 5) : bbase[1] + j * DV_BST));
        bfr[j] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      if constexpr (DV_RB && !COLS && !DV_NI) {
        float mu[8], rs[8];
        if constexpr (NK == NORM_GLN) {
          const float2 st = *reinterpret_cast<const float2*>(base + OFF_ST);
#pragma unroll
          for (int e = 0; e < 8; ++e) mu[e] = st.x, rs[e] = st.y;
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float4 st = *reinterpret_cast<const float4*>(base + OFF_ST + 64 * lg + 16 * k);
            mu[2 * k] = st.x, rs[2 * k] = st.y, mu[2 * k + 1] = st.z, rs[2 * k + 1] = st.w;
          }
        }
        const int tk = (t * TM) % Kp;
#pragma unroll
        for (int j = 0; j < CJ; ++j) {
          v4u v = __builtin_bit_cast(v4u, bfr[j]);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float x0 = __uint_as_float(v[k] << 16), x1 = __uint_as_float(v[k] & 0xffff0000u);
            x0 = dv_prelu<LE1>(x0, bal);
            x1 = dv_prelu<LE1>(x1, bal);
            x0 = fmaf(x0 - mu[2 * k], rs[2 * k] * cg[j], cb[j]);
            x1 = fmaf(x1 - mu[2 * k + 1], rs[2 * k + 1] * cg[j], cb[j]);
            if constexpr (NK == NORM_CLN) {   // padded frames: statistics not finite
              if (tk + 8 * lg + 2 * k >= Kv) x0 = 0.f;
              if (tk + 8 * lg + 2 * k + 1 >= Kv) x1 = 0.f;
            }
            v[k] = pk_bf16(x0, x1);
          }
          bfr[j] = __builtin_bit_cast(bf16x8_t, v);
        }
      }
    };
    auto a_frag = [&](const char* base, int i) __attribute__((always_inline)) {
      const int o = (i >> 1) * 1024 + (i & 1) * 512;
      const s16x4_t lo = dv_tr(base + OFF_A + abase[0] + o), hi = dv_tr(base + OFF_A + abase[1] + o);
      return bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    // NIMG: the row waves' DONE of the tile (they waited for FULL and wrote op(d))
    auto full_word = [&](int slot) __attribute__((always_inline)) {
      return (DV_NI && !COLS) ? fl_done[slot] : fl_full[slot];
    };
    auto run = [&](auto le1) __attribute__((always_inline)) {
      int slot = 0;
      uint32_t gen = 1;
      int t = t0;
      // CTN_DV_C2: two tiles per iteration (two independent wait / transform / read chains
      // in flight per wave); each accumulator still takes tile t before tile t + 1, so the
      // partial sums keep their order
      if constexpr (CTN_DV_C2 && !(CTN_DV_EXP & 3)) {
        for (; t + 1 < t1; t += 2) {
          const int s0 = slot;
          const uint32_t g0 = gen;
          if (++slot == NSL) slot = 0, ++gen;
          const int s1 = slot;
          const uint32_t g1 = gen;
          if (++slot == NSL) slot = 0, ++gen;
          const char* b0 = smem + s0 * SLOT;
          const char* b1 = smem + s1 * SLOT;
          bf16x8_t bf0[CJ], bf1[CJ];
          dv_wait<4>(full_word(s0), g0, p.err);
          load_b(le1, t, b0, bf0);
          dv_wait<4>(full_word(s1), g1, p.err);
          load_b(le1, t + 1, b1, bf1);
#pragma unroll
          for (int i = 0; i < CI; ++i) {
            const bf16x8_t a0 = a_frag(b0, i), a1 = a_frag(b1, i);
#pragma unroll
            for (int j = 0; j < CJ; ++j) dacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf0[j], dacc[i][j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < CJ; ++j) dacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bf1[j], dacc[i][j], 0, 0, 0);
          }
          dv_signal(&fl_done[s0][NR + c], g0);
          dv_signal(&fl_done[s1][NR + c], g1);
        }
      }
      DV_TS(tl0);
      for (; t < t1; ++t) {
        DV_TS(tw0);
        dv_wait<4>(full_word(slot), gen, p.err);
        DV_ACC(0, tw0);
        const char* base = smem + slot * SLOT;
        if constexpr (!(CTN_DV_EXP & 3)) {
          bf16x8_t bfr[CJ];
          load_b(le1, t, base, bfr);
#pragma unroll
          for (int i = 0; i < CI; ++i) {
            const bf16x8_t af = a_frag(base, i);
#pragma unroll
            for (int j = 0; j < CJ; ++j) dacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], dacc[i][j], 0, 0, 0);
          }
        }
        dv_signal(&fl_done[slot][NR + c], gen);
        if (++slot == NSL) {
          slot = 0;
          ++gen;
        }
      }
      DV_ACC(3, tl0);
    };
    if (COLS || bal <= 1.f) run(std::true_type{});
    else run(std::false_type{});
    DV_STAMP_STORE;
    // dW2 partial of this workgroup: lane holds D[(wp*CI+i)*16 + 4lg + e][n0 + (wn*CJ+j)*16 + lr]
    float* Dp = p.Dpart + (size_t)rr * KR * p.Nout;
    if constexpr (COLS) {
      // transposed through LDS (the ring is idle once every wave is past the barrier):
      // image [n - n0][k] fp32, rows padded by 4 floats against bank conflicts
      float* img = reinterpret_cast<float*>(smem);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < CI; ++i)
#pragma unroll
        for (int j = 0; j < CJ; ++j) {
          const int nl = (wn * CJ + j) * 16 + lr;
#pragma unroll
          for (int e = 0; e < 4; ++e) img[nl * COLS_LDT + (wp * CI + i) * 16 + 4 * lg + e] = dacc[i][j][e];
        }
      __syncthreads();
      store_tr(Dp);
      return;
    }
#pragma unroll
    for (int i = 0; i < CI; ++i)
#pragma unroll
      for (int j = 0; j < CJ; ++j) {
        if constexpr (CTN_PART_NT == 2) {   // lane (lg, 4q + t): row 4lg + t, channels 4q .. 4q+3
          float v[4] = {dacc[i][j][0], dacc[i][j][1], dacc[i][j][2], dacc[i][j][3]};
          quad_transpose4(v);
          const int n = n0 + (wn * CJ + j) * 16 + (lr & ~3);
          stg16h<true>(&Dp[(size_t)((wp * CI + i) * 16 + 4 * lg + (lr & 3)) * p.Nout + n], f4bits(v));
        } else {
          const int n = n0 + (wn * CJ + j) * 16 + lr;
#pragma unroll
          // nontemporal for gLN (c2, c5: keeps the activations of the next kernels in the
          // Infinity Cache); plain for cLN: at c4 every tensor is larger than the cache and
          // the hinted dword stores measured 10 us slower per launch (547.7 / 533.6 against
          // 555.3 / 544.7 us, microbenchmark, round 6) — the c4 regression of round 5
          for (int e = 0; e < 4; ++e)
            st_part<CTN_PART_NT != 0 && NK == NORM_GLN>(&Dp[(size_t)((wp * CI + i) * 16 + 4 * lg + e) * p.Nout + n],
                                                        dacc[i][j][e]);
        }
      }
    return;
  }

  // ======================= memory waves =======================
  dv_prio<4, NK>();
  // Memory wave m moves, per tile, A blocks 4m..4m+3 (16 rows x 32 channels of gy each),
  // raw-d pieces 2m, 2m+1 (4 rows x the slice's 128 channels each) and its statistics
  // piece by LDS-DMA (buffer_load ... lds: no registers, PF tiles ahead), waits for its
  // own DMA group with a counted vmcnt (no other memory operations are issued by these
  // waves), (RAWB=0 only) reads back its own raw-d pieces to write op(d) into the B image,
  // and publishes FULL.  A slot is refilled only after every row / column wave's DONE for
  // the tile that used it last.  RAWB=1: the raw-d pieces land in the B image itself and
  // wave 0 alone fetches the tile's statistics (all 32 rows).
  const int mw = wid - ND;
  DV_STAMP_DECL;
  const rsrc_t rA = du_rsrc(p.A, rows * p.lda * 2), rD = du_rsrc(p.Bm, rows * p.ldb * 2);
  const rsrc_t rS = du_rsrc(p.bop.stats, (NK == NORM_GLN ? (long)p.g.M : rows) * 8);
  int arow[4];
  uint32_t aoff[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {   // lane L lands at block + 16 L: the fragment-order image
    const int f = 4 * mw + u, mb = f / KB, kb = f % KB;
    arow[u] = 16 * mb + ((lane & 15) ^ (((lane >> 4) & 1) * 12));
    aoff[u] = (uint32_t)(arow[u] * p.lda + (4 * kb + (lane >> 4)) * 8) * 2u;
  }
  // raw-d piece i = 2*mw + h: row 4i + L/16, granule position L%16 holds channels
  // 8g .. 8g+7 with g = (L%16) ^ (row%16) (RAWB=0: the R image's swizzle) or g the granule
  // at B position L%16 (RAWB=1: dv_rbpos inverted), the swizzle applied on the source
  int drow[2], dgr[2], boff[2];
  uint32_t doff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    drow[h] = 4 * (2 * mw + h) + (lane >> 4);
    const int ps = lane & 15;
    dgr[h] = DV_RB ? (ps & 1) | ((((ps >> 1) ^ dv_rbhash(drow[h])) & 7) << 1) : ps ^ (drow[h] & 15);
    doff[h] = (uint32_t)(drow[h] * p.ldb + n0 + 8 * dgr[h]) * 2u;
    boff[h] = (dgr[h] >> 1) * DV_BST + dv_boff(drow[h], 8 * (dgr[h] & 1));
  }
  // statistics: RAWB=1 wave 0 fetches the tile's (cLN: 32 rows, one dword per lane; gLN:
  // the utterance pair, lanes 0..1).  RAWB=0 every wave fetches into its own 256 bytes (a
  // wave's vmcnt covers only its own DMA, and each reads statistics it fetched itself):
  // cLN rows 8m .. 8m+7 (lanes 0..15), gLN the pair.  Other lanes read out of range (zeros).
  const bool st_lane = NK == NORM_CLN ? (DV_RB ? true : lane < 16) : lane < 2;
  const uint32_t soff = st_lane ? (uint32_t)((NK == NORM_CLN && !DV_RB ? 8 * mw * 8 : 0) + lane * 4) : DU_OOB;
  const bool st_wave = !COLS && (!DV_RB || mw == 0);
  const float bal = COLS ? 0.f : p.bop.alpha[0];
  // DMA instructions per wave and tile: 7 (st_wave), else 6 (RAWB=1 waves 1..3)

  auto dma = [&](int t) __attribute__((always_inline)) {
    if constexpr (CTN_DV_EXP & 32) return;
    char* base = smem + ((t - t0) % NSL) * SLOT;
    const int tk = (t * TM) % Kp;
#pragma unroll
    for (int u = 0; u < 4; ++u)   // rows of padded frames arrive as zeros (out-of-range offset)
      du_dma16(rA, base + OFF_A + (4 * mw + u) * 1024, tk + arow[u] < Kv ? aoff[u] : DU_OOB, t * TM * p.lda * 2);
#pragma unroll
    for (int h = 0; h < 2; ++h) du_dma16(rD, base + (DV_RB ? OFF_B : OFF_R) + (2 * mw + h) * 1024, doff[h], t * TM * p.ldb * 2);
    if (st_wave) du_dma4(rS, base + OFF_ST + (DV_RB ? 0 : mw * 256), soff, NK == NORM_GLN ? (t / tpu) * 8 : t * TM * 8);
  };
  // the lane's gamma2 / beta2 (its granule's 8 channels, per piece) stay in registers
  float tgam[2][8], tbet[2][8];
  if constexpr (!DV_RB) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        tgam[h][e] = p.bop.gamma[n0 + 8 * dgr[h] + e];
        tbet[h][e] = p.bop.beta[n0 + 8 * dgr[h] + e];
      }
  }
  auto transform = [&](auto le1, int t, char* base) __attribute__((always_inline)) {
    constexpr bool LE1 = decltype(le1)::value;
    const int tk = (t * TM) % Kp;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = drow[h];
      v4u v = *reinterpret_cast<const v4u*>(base + OFF_R + (2 * mw + h) * 1024 + lane * 16);
      const float2 st = *reinterpret_cast<const float2*>(base + OFF_ST + mw * 256 + (NK == NORM_GLN ? 0 : (row & 7) * 8));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x0 = __uint_as_float(v[e] << 16), x1 = __uint_as_float(v[e] & 0xffff0000u);
        x0 = dv_prelu<LE1>(x0, bal);
        x1 = dv_prelu<LE1>(x1, bal);
        x0 = fmaf(x0 - st.x, st.y * tgam[h][2 * e], tbet[h][2 * e]);
        x1 = fmaf(x1 - st.x, st.y * tgam[h][2 * e + 1], tbet[h][2 * e + 1]);
        v[e] = pk_bf16(x0, x1);
      }
      if constexpr (NK == NORM_CLN)   // padded frames: statistics not finite
        if (tk + row >= Kv) v = v4u{0u, 0u, 0u, 0u};
      stg16(base + OFF_B + boff[h], v);
    }
  };
  auto run = [&](auto le1) __attribute__((always_inline)) {
    for (int i = 0; i < PF; ++i)
      if (t0 + i < t1) dma(t0 + i);
    int slot = 0;
    uint32_t gen = 1;
    DV_TS(tl0);
    for (int t = t0; t < t1; ++t) {
      const int later = t1 - 1 - t < PF - 1 ? t1 - 1 - t : PF - 1;   // DMA groups issued after tile t's
      char* base = smem + slot * SLOT;
      // tile t's DMA group done: every group issued after it may stay in flight (steady
      // state: PF - 1 of them, a compile-time count; the tail waits for all)
      DV_TS(tv0);
      if (later == PF - 1) {
        if (!DV_RB || st_wave) dv_vmwait_c<7 * (PF - 1)>();
        else dv_vmwait_c<6 * (PF - 1)>();
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      DV_ACC(1, tv0);
      if constexpr (!DV_RB) transform(le1, t, base);
      dv_signal(&fl_full[slot][mw], gen);
      const int tn = t + PF;
      if (tn < t1) {
        const int kn = tn - t0;   // its slot was last used by tile tn - NSL: wait for every DONE of it
        DV_TS(td0);
        dv_wait<ND>(fl_done[kn % NSL], (uint32_t)(kn / NSL), p.err);
        DV_ACC(2, td0);
        dma(tn);
      }
      if (++slot == NSL) {
        slot = 0;
        ++gen;
      }
    }
    DV_ACC(3, tl0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the wave ends
  };
  if (t0 < t1) {
    if (COLS || bal <= 1.f) run(std::true_type{});
    else run(std::false_type{});
  }
  DV_STAMP_STORE;
  if constexpr (COLS) {   // the column waves' two barriers, then a share of the stores
    __syncthreads();
    __syncthreads();
    store_tr(p.Dpart + (size_t)rr * KR * p.Nout);
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// CTN_DUAL_WS=0 runs pair A on gemm_dual_kernel (ctn_gemm_dual.hip) instead; read on
// every query, so one process can compare both.
bool gemm_dual_ws_enabled() {
  const char* e = getenv("CTN_DUAL_WS");
  return e ? atoi(e) != 0 : true;
}

// cLN statistics entries per (row, slice) the kernel stores (gemm_dual_group_parts)
int dual_ws_cln_parts_per_slice() { return CTN_DV_CLNC ? 1 : DV_NR; }

// row waves per slice of the wave-specialised kernel (its gLN statistics partials are per
// (range, slice, row wave): gemm_dual_runs).  Round 6 measured two other gLN forms, both
// bit-identical and slower, and removed them: eight row waves with the
// tile DMA in the column waves (commit 9656623) and the row epilogue in the memory waves
// (commit 9d56d29).
int dual_ws_row_waves(const GemmDual&) { return DV_NR; }

bool gemm_dual_ws_eligible(const GemmDual& p) {
  if (!gemm_dual_ws_enabled()) return false;
  if (!(p.Kred == DV_KR && p.Nout % DV_NS == 0 && p.epi == EPI_NORM_BWD && p.bop.kind == OP_PRELU_NORM)) return false;
  if (p.norm != NORM_GLN && p.norm != NORM_CLN) return false;
  if (p.bop.norm != p.norm || p.stats != p.bop.stats || p.bop.fold.slab) return false;
  if (DV_NI && p.gamma != p.bop.gamma) return false;   // the row waves' gamma serves op(d)
  if (p.g.Kp % DV_TM || p.lda % 8 || p.ldb % 8 || p.ldc % 8 || p.ldw % 8) return false;
  if (p.g.rows() / DV_TM < 1) return false;
  // 32-bit tile offsets and buffer sizes (du_rsrc clamps at 2^31 bytes): larger tensors
  // take the tiled kernels
  if (p.g.rows() * (p.Kred > p.Nout ? p.Kred : p.Nout) * 2 >= (1L << 31)) return false;
  const int S = p.Nout / DV_NS;
  return DV_GRID % S == 0;
}

int gemm_dual_ws_ranges(const GemmDual& p) {
  const long nt = p.g.rows() / DV_TM;
  const int want = DV_GRID / (p.Nout / DV_NS);
  return (int)(nt < want ? nt : want);
}

// The column GEMM alone (GemmCols, plain bf16 operands): dW[P][Q] partials per row range
// = A^T B with A [rows][P] (P = Nout, sliced by 128 per workgroup) and B [rows][Q]
// (Q = Kred = 256, whole rows), i.e. the dual's column part with the roles of its
// operands swapped: its "A" tile is B and its raw-B slice is A.
// Off by default (CTN_COLS_WS=1 to enable): 47.8 us against the tiled kernel's 49.4 in the
// step, but twice the partial bytes (64 row ranges instead of 32 chunks) cost the slab
// reduction more than that: bench 2129 vs 2142 utt/s.
bool gemm_cols_ws_eligible(DType dt, const GemmCols& c) {
  const char* e = getenv("CTN_COLS_WS");
  if (!e || atoi(e) == 0) return false;
  if (dt != BF16 || c.aop.kind != OP_PLAIN || c.bop.kind != OP_PLAIN) return false;
  if (c.Q != DV_KR || c.P % DV_NS || DV_GRID % (c.P / DV_NS)) return false;
  if (c.g.Kp % DV_TM || c.lda % 8 || c.ldb % 8 || c.g.rows() / DV_TM < 1) return false;
  if (c.g.rows() * (c.P > c.Q ? c.P : c.Q) * 2 >= (1L << 31)) return false;   // 32-bit offsets
  if (((uintptr_t)c.A | (uintptr_t)c.B | (uintptr_t)c.Cpart) & 15) return false;
  return true;
}

int gemm_cols_ws_ranges(const GemmCols& c) {
  const long nt = c.g.rows() / DV_TM;
  const int want = DV_GRID / (c.P / DV_NS);
  return (int)(nt < want ? nt : want);
}

hipError_t launch_gemm_cols_ws(const GemmCols& c, hipStream_t s) {
  GemmDual p{};
  p.err = device_error_word();
  p.g = c.g;
  p.Kred = c.Q;
  p.Nout = c.P;
  p.A = c.B; p.lda = c.ldb;     // whole 256-channel rows: the fragment-order tile
  p.Bm = c.A; p.ldb = c.lda;    // the 128-channel slice: raw B
  p.Dpart = c.Cpart;            // [range][P][Q]
  const dim3 grid(gemm_cols_ws_ranges(c) * (c.P / DV_NS));
  hipLaunchKernelGGL((gemm_dual_ws_kernel<NORM_GLN, DV_NSL, DV_PF, true>), grid, dim3((DV_NC + DV_NMW) * 64), 0,
                     s, p);
  return hipGetLastError();
}

hipError_t launch_gemm_dual_ws(const GemmDual& pa, hipStream_t s) {
  if (!gemm_dual_ws_eligible(pa)) return hipErrorInvalidValue;
  GemmDual p = pa;
  p.err = device_error_word();
  const dim3 grid(gemm_dual_ws_ranges(p) * (p.Nout / DV_NS));
  if (p.norm == NORM_GLN)
    hipLaunchKernelGGL((gemm_dual_ws_kernel<NORM_GLN, DV_NSL, DV_PF>), grid, dim3(DV_NT), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_dual_ws_kernel<NORM_CLN, DV_NSL, DV_PF_CLN>), grid, dim3(DV_NT), 0, s, p);
  return hipGetLastError();
}

}  // namespace ctn
