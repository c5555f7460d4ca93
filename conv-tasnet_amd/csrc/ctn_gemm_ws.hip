// Weight-stationary persistent row GEMM (bf16, gfx950): the 1x1 convolutions
// of the TemporalBlocks (conv_tasnet.py:217,256) and their data gradients at
// the model's shapes (Nout x Kred = 512x256, 256x512, 256x256).
//
// One workgroup per CU (8 waves, 512 threads) holds the WHOLE bf16 weight in
// registers (wave w owns output channels [w*16*NB, (w+1)*16*NB): NB x KB MFMA
// A-fragments = 128 VGPRs at these shapes) and streams a contiguous range of
// 16-row frame tiles: each A tile is read from HBM exactly once, the weight is
// read once per workgroup, and every output element is written once.  Per tile:
//   registers (prefetched one tile ahead) -> operand transform -> LDS image in
//   MFMA fragment order (XOR-swizzled, conflict-free writes and reads) ->
//   v_mfma_f32_16x16x32_bf16 against the resident weight -> fused epilogue
//   straight from the accumulators.
// The weight rows are loaded in a permuted order so that each lane's four
// accumulators hold NB*4 CONTIGUOUS output channels of one frame row, which
// makes the epilogue loads/stores 16-byte vectors without an LDS round trip.
//
// Statistics: gLN partials are per (workgroup, wave, utterance run): a wave
// accumulates its consecutive tiles of one utterance (WsRuns, ctn_common.h);
// cLN partials are per (row, wave).  All reductions are fixed-order: results
// are bitwise reproducible.
#include <stdlib.h>

#include <type_traits>

#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

#ifndef CTN_WS_GRID
#define CTN_WS_GRID 256
#endif
constexpr int WS_WAVES = 8, WS_TM = 16, WS_GRID = CTN_WS_GRID;
// Plain-operand configurations without a residual stream (the forward 1x1 conv, the
// mask conv) take their tiles by LDS-DMA into a WS_DR-deep ring (CTN_WS_DMA=0: the
// register-staged pipeline, for A/B builds)
#ifndef CTN_WS_DMA
#define CTN_WS_DMA 1
#endif
#ifndef CTN_WS_DR
#define CTN_WS_DR 6   // 4: 41.9/42.0 us, 6: 40.8/41.2 (forward B -> H, profiles/r05/nt_exp/r5s512_*)
#endif
constexpr int WS_DR = CTN_WS_DR;
// The LDS-DMA ring's hand-offs (gLN, no in-kernel cLN finalize): 1 = generation words per
// slot and wave instead of one workgroup barrier per tile — a wave starts tile t's MFMAs
// once every wave's DMA of tile t has landed and refills a slot once every wave has read
// it, so the waves may drift within the ring.  Measured slower (forward 1x1 35.4 ->
// 40.6 / 41.7 / 43.0 us at rings of 4 / 6 / 8 tiles): 0 (default) keeps the
// barrier.
#ifndef CTN_WS_FLAGS
#define CTN_WS_FLAGS 0
#endif
constexpr int WS_FOLD_MAX = 512;   // utterances whose gLN operand stats a workgroup holds in LDS

// Bound-finding experiments only (tools/microbench): bit 0 drops the output
// stores, bit 1 the A-tile loads, bit 2 the MFMAs, bit 3 the epilogue math, bit 7 the
// resident weight's loads, bit 10 the dL/dh1 stores of the norm-1-backward form; bit 6
// (experiment, not bound-finding) lets the scheduler move epilogue math into the MFMAs.
#ifndef CTN_WS_EXP
#define CTN_WS_EXP 0
#endif
// A-tile register ring depth (tiles whose loads are in flight while one is staged)
// of the 16-wave and 8-wave non-interleaved configurations
#ifndef CTN_WS_PF16
#define CTN_WS_PF16 1
#endif
#ifndef CTN_WS_PF8
#define CTN_WS_PF8 1
#endif
// Issue order inside a tile iteration of the non-interleaved configurations.
// gfx9 retires loads and stores in one in-order vmcnt queue, so a load issued
// behind a tile's output stores cannot be consumed before those stores are
// acknowledged.  1: stage(t+1) and the loads of the next tiles go BEFORE the output
// stores of tile t (which are written last); 0: the original order (stores, then
// the next loads).
// Output-channel slices of the Nout = 512 forward GEMM: 2 = two independent
// 8-wave workgroups per CU, each holding half the weight (the A tile is read by
// both from the XCD's L2), instead of one 16-wave workgroup.
#ifndef CTN_WS_S512
#define CTN_WS_S512 1
#endif
// LDS fragment look-ahead of the MFMA loop, in k-steps
// (16 waves: plain-operand configurations only; 1 = one k-step ahead, 124 VGPRs without
// spills for the forward B -> H GEMM: 36.1 -> 34.5 us, microbenchmark, round 6; the
// transformed-operand 16-wave configurations spill more with it)
#ifndef CTN_WS_LA16
#define CTN_WS_LA16 1
#endif
#ifndef CTN_WS_LA8
#define CTN_WS_LA8 3
#endif
// experiment: 1 raises the wave priority (s_setprio 1) while it issues a tile's MFMAs
// Nontemporal hints per configuration (bits): 1 = the resident-weight loads of the
// forward B -> H GEMM (plain operand, PReLU-statistics epilogue), 2 = the output stores
// of the forward H -> B GEMM (norm-2 operand, residual epilogue), 4 = the output (h1)
// stores of the forward B -> H GEMM, 8 = the dL/dh1 stores of the data-gradient GEMM
// (norm-1-backward operand), 16 = that GEMM's output (gx) stores, 32 = that GEMM's
// dL/da1 operand loads, 64 = its h1 loads (both their last use), 128 = the H -> B GEMM's d
// loads, 256 = the residual loads (x in the H -> B GEMM, gy in the gx GEMM).  Bit 32 measured
// -1.7 us, bit 64 -2 us in the column GEMM after it; the others slower or flat
// (profiles/r05/nt_exp/)
#ifndef CTN_WS_NT
#define CTN_WS_NT 96
#endif
#ifndef CTN_WS_PRIO
#define CTN_WS_PRIO 0
#endif
// Ping-pong (LDS-DMA ring configurations of 16 waves): waves 8-15 run each tile half a
// tile behind waves 0-7 — two barriers per tile, and between them one half runs its MFMAs
// while the other runs the previous tile's epilogue and stores, so on every SIMD (two
// waves of each half) the matrix pipe and the vector/store issue overlap instead of all
// 16 waves meeting at one barrier and then running the same phase.  Same arithmetic,
// same results bit for bit.
#ifndef CTN_WS_PP
#define CTN_WS_PP 0
#endif
#ifndef CTN_WS_HPRIO
#define CTN_WS_HPRIO 0
#endif
#ifndef CTN_WS_STAMP
#define CTN_WS_STAMP 0
#endif
#if CTN_WS_STAMP
__device__ unsigned long long ws_stamps[256 * 16 * 8];
#endif
// 1: wait for the resident weight before the first tiles' loads are issued; 0
// (experiment): after them.  Measured the same.
// cLN statistics of 64 tiles per lane, broadcast by v_readlane (see load_a)
#ifndef CTN_WS_CLN_BATCH
#define CTN_WS_CLN_BATCH 1
#endif
#ifndef CTN_WS_EARLY
#define CTN_WS_EARLY 1
#endif
#ifndef CTN_WS_ORDER
#define CTN_WS_ORDER 1
#endif

// LDS byte offset of the 16-byte piece (frame row lr, k-chunk lg) of k-block kb
// in fragment order: ds_read_b128 groups and ds_write_b128 groups both hit
// distinct banks.
CTN_DEV int ws_slot(int lr, int lg, int kb) { return (kb * 64 + lg * 16 + (lr ^ (lg + 4 * (kb & 3)))) << 4; }

// Force a register's load to complete here (an inline-asm use makes the compiler
// wait for it once, so no counted wait for it is left inside the tile loop,
// where it would also drain the prefetch issued behind it).
CTN_DEV void ready(const v4u& v) { asm volatile("" ::"v"(v)); }
CTN_DEV void ready(float v) { asm volatile("" ::"v"(v)); }


// S: output-channel slices; workgroup b -> (row range rr, slice sl), the S slices of
// a range on one XCD (hardware ids are dealt round-robin over the 8 XCDs) so the A
// tile comes from HBM once.  Each slice-workgroup holds NS = WV*16*NB channels.
// (S = 2: two 8-wave slice workgroups share a CU, CTN_WS_S512; S = 3: the three 512-channel
// slices of a 1536-channel output (c5's mask conv, C*N = 3*512) on three CUs of one XCD.)
template <int OPK, int NK, int EPI, int NB, int KB, int WV, int MB, int S = 1>
__global__ __launch_bounds__(64 * WV, (S == 2 ? 2 : 1) * WV / 4) void gemm_ws_kernel(GemmRows p) {
  constexpr int NT = 64 * WV;                  // threads
  constexpr int TM = 16 * MB;                  // frame rows per tile
  constexpr int KR = KB * 32;                  // reduction length
  constexpr int CPR = KR / 8;                  // 16-byte chunks per A row
  constexpr int NA = TM * CPR / NT;            // A chunks per thread per tile
  constexpr int RSTEP = NT / CPR;              // rows between a thread's chunks
  constexpr int NV = NB * 4;                   // output channels per lane
  constexpr int Q = NV / 8;                    // 16-byte chunks per lane and row
  static_assert(NA >= 1 && NA * NT == TM * CPR, "tile/thread mismatch");
  static_assert(Q >= 1, "at least 8 channels per lane");
  // one-tile register prefetch + two accumulator sets only where registers allow
  constexpr bool N1B = OPK == OP_NORM1_BWD;    // norm-1/PReLU-1 backward on the operand
  constexpr bool SWP = OPK == OP_PLAIN && WV == 8;
  constexpr int PF = SWP ? 1 : (WV == 16 ? CTN_WS_PF16 : CTN_WS_PF8);
  // cLN PReLU statistics finalized in the kernel: per-row partials of the WV waves of
  // one tile meet in LDS and are summed after the next barrier (tile parity buffers)
  constexpr bool CLN_FIN = EPI == EPI_PRELU_STATS && NK == NORM_CLN && !SWP && S == 1;
  __shared__ double2 scln[CLN_FIN ? 2 * TM * WV : 1];
  constexpr bool WDMA = CTN_WS_DMA && OPK == OP_PLAIN && !SWP && EPI != EPI_RESID && EPI != EPI_NORM_BWD;
  __shared__ __attribute__((aligned(16))) char sA[WDMA ? WS_DR : 2][TM * KR * 2];
  constexpr bool WFL = WDMA && CTN_WS_FLAGS && !CLN_FIN && WV % 4 == 0;   // flag-ring hand-offs
  __shared__ __attribute__((aligned(16))) uint32_t fl_full[WFL ? WS_DR : 1][WFL ? WV : 4];
  __shared__ __attribute__((aligned(16))) uint32_t fl_done[WFL ? WS_DR : 1][WFL ? WV : 4];
  __shared__ float sgam[EPI == EPI_NORM_BWD ? NB * 16 * WV : 1];
  // gLN operand statistics, one pair per utterance, finalized here (StatFold)
  constexpr bool FOLDS = NK == NORM_GLN && OPK != OP_PLAIN;
  __shared__ float2 sst[FOLDS ? WS_FOLD_MAX : 1];
  __shared__ float2 sst1[N1B ? WS_FOLD_MAX : 1];   // N1B: forward norm-1 (mean, rstd); sst holds the sums
  __shared__ float salpha[N1B ? WV : 1];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  // static priority for the second half of the waves (experiment; the younger half loses
  // every issue arbitration otherwise, MI355X_MICROARCH.md "Two waves per SIMD" item 4)
  if constexpr (CTN_WS_HPRIO != 0) { if (wid >= WV / 2) __builtin_amdgcn_s_setprio(CTN_WS_HPRIO); }
  const int ntile = (int)(p.g.rows() / TM);
  constexpr int NS = WV * 16 * NB;             // output channels per slice
  const int nr = (int)gridDim.x / S;           // row ranges
  int rr = (int)blockIdx.x, sl = 0;
  if constexpr (S > 1) {
    const int b = (int)blockIdx.x;
    if (nr % 8 == 0) {
      const int l = b / 8;
      sl = l % S;
      rr = (b % 8) * (nr / 8) + l / S;
    } else {
      sl = b % S;
      rr = b / S;
    }
  }
  const int t0 = (int)((long)ntile * rr / nr), t1 = (int)((long)ntile * (rr + 1) / nr);
  const int Kp = p.g.Kp, Kv = p.g.K;
  const bf16raw* A = reinterpret_cast<const bf16raw*>(p.A);
  const bf16raw* W = reinterpret_cast<const bf16raw*>(p.W) + (size_t)sl * NS * p.ldw;
  const int n0 = sl * NS;
  const int colbase = n0 + wid * 16 * NB + lg * NV;  // this lane's NV contiguous output channels
  const int wslot = sl * WV + wid;                    // partial-statistics column of this wave

  // ---- resident weight: fragment (nb, kb), MFMA row lr -> output channel.  From the
  // fragment-ordered copy when the caller made one (1 KiB contiguous per wave and
  // fragment: half the L2 lines of the row-major reads, whose 64-byte row pieces fill
  // only half of each line; every CU reads the whole weight, so this read is a fixed
  // cost of the launch, 12.9 -> 7.8 us at one tile per workgroup)
  constexpr bool NTW = (CTN_WS_NT & 1) && OPK == OP_PLAIN && EPI == EPI_PRELU_STATS;
  constexpr bool NTO = ((CTN_WS_NT & 2) && OPK == OP_PRELU_NORM) ||
                      ((CTN_WS_NT & 4) && OPK == OP_PLAIN && EPI == EPI_PRELU_STATS) ||
                      ((CTN_WS_NT & 16) && OPK == OP_NORM1_BWD);
  constexpr bool NTG = (CTN_WS_NT & 8) != 0;
  v4u wf[NB][KB];
  const bf16raw* WF = NB == 2 ? reinterpret_cast<const bf16raw*>(p.Wf) : nullptr;
  if (WF) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) wf[nb][kb] = ldg16h<NTW>(WF + frag_offset(sl * WV + wid, nb, kb, lane, KR));
  } else {
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = wid * 16 * NB + (lr >> 2) * NV + nb * 4 + (lr & 3);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
      if constexpr (CTN_WS_EXP & 128) wf[nb][kb] = v4u{(uint32_t)n, (uint32_t)kb, 0u, 0u};   // no weight loads
      else if constexpr (CTN_WS_EXP & 768) {   // timing only (wrong values): contiguous / rotated
        const int kr = (CTN_WS_EXP & 512) ? (kb + (int)blockIdx.x) % KB : kb;
        if constexpr (CTN_WS_EXP & 256) wf[nb][kb] = ldg16(W + ((size_t)((wid * NB + nb) * KB + kr) * 64 + lane) * 8);
        else wf[nb][kb] = ldg16(W + (size_t)n * p.ldw + kr * 32 + lg * 8);
      } else wf[nb][kb] = ldg16h<NTW>(W + (size_t)n * p.ldw + kb * 32 + lg * 8);
  }
  }

  // operand statistics into LDS (FOLDS); called after the first tiles' loads are
  // issued where the pipeline allows, so the fold's round trip overlaps them
  auto fold_stats = [&]() __attribute__((always_inline)) {
  if constexpr (FOLDS) {
    const StatFold& f = p.aop.fold;
    if (f.slab) {
      // only the utterances of this workgroup's rows (one per wave, in parallel); the
      // workgroup holding an utterance's first row stores its pair for backward
      const int mlo = (int)((long)t0 * TM / Kp), mhi = t1 > t0 ? (int)(((long)t1 * TM - 1) / Kp) : mlo - 1;
      for (int gi = mlo + wid; gi <= mhi; gi += WV) {
        const float2 v = fold_stat(f, gi);
        if (lane == 0) {
          sst[gi] = v;
          if (f.out && (long)gi * Kp >= (long)t0 * TM) f.out[gi] = v;   // saved for backward
        }
      }
    } else {
      const float2* tab = N1B ? p.aop.sums : p.aop.stats;
      for (int gi = tid; gi < p.g.M; gi += NT) sst[gi] = tab[gi];
    }
    if constexpr (N1B)
      for (int gi = tid; gi < p.g.M; gi += NT) sst1[gi] = p.aop.stats[gi];
    __syncthreads();
  }
  };

  // ---- A staging: thread owns k-chunk kc (fixed) of rows rl0 + j*RSTEP
  const int kc = tid % CPR, rl0 = tid / CPR;
  float og[8], ob[8];
  constexpr bool AFF = OPK == OP_NORM || OPK == OP_PRELU_NORM;   // operand op with gamma/beta
  if constexpr (AFF) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      og[e] = p.aop.gamma[kc * 8 + e];
      ob[e] = p.aop.beta[kc * 8 + e];
    }
  }
  const float oal = (OPK == OP_PRELU_NORM || N1B) ? p.aop.alpha[0] : 0.f;
  const bf16raw* H1 = reinterpret_cast<const bf16raw*>(p.aop.aux);
  bf16raw* GH = reinterpret_cast<bf16raw*>(p.aop.aout);
  v4u rh[PF][N1B ? NA : 1];   // N1B: h1 chunks beside the gradient chunks
  v4u ghv[N1B ? NA : 1];      // N1B: dL/dh1 chunks of the staged tile, stored after the loads
  float calpha = 0.f;     // N1B: this thread's PReLU-1 alpha gradient over its valid rows
  // Loads are issued one tile ahead together with the statistics they need, so
  // that no wait inside an iteration has to drain the next tile's prefetch
  // (vmcnt retires loads in issue order).
  // Ring of PF register tiles: tile t lives in slot (t - t0) % PF (static indices:
  // the tile loop is unrolled by PF).
  v4u ra[PF][NA];
  float2 ast[PF][NA];
  float2 asm1[PF][N1B && NK == NORM_CLN ? NA : 1];   // N1B, cLN: per-row norm-1 backward means
  // cLN with wave-uniform rows (a row's 16-byte chunks span whole waves): the per-row
  // statistics (and N1B means) of 64 consecutive tiles are loaded one tile per lane and
  // broadcast with v_readlane, instead of a load per row and tile in the prefetch
  constexpr bool CB = CTN_WS_CLN_BATCH && NK == NORM_CLN && OPK != OP_PLAIN && !FOLDS && CPR % 64 == 0;
  float2 bst[CB ? NA : 1], bsm[CB && N1B ? NA : 1];
  int bbase = -(1 << 29);
  auto batch_load = [&](int tb) __attribute__((always_inline)) {
    if constexpr (CB) {
      bbase = tb;
      const int tt = tb + lane < t1 ? tb + lane : t1 - 1;
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const int r = tt * TM + rl0 + j * RSTEP;
        bst[j] = p.aop.stats[r];
        if constexpr (N1B) bsm[j] = p.aop.sums[r];
      }
    }
  };
  auto bcast = [&](float2 v, int t) __attribute__((always_inline)) {
    const int l = __builtin_amdgcn_readfirstlane(t - bbase);
    return make_float2(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), l)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), l)));
  };
  auto load_a = [&](int t, auto slot) __attribute__((always_inline)) {
    constexpr int s = decltype(slot)::value;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int r = t * TM + rl0 + j * RSTEP;
      if constexpr (CTN_WS_EXP & 2) ra[s][j] = v4u{(uint32_t)r, 0u, 0u, 0u};
      else ra[s][j] = ldg16h<((CTN_WS_NT & 32) != 0 && N1B) || ((CTN_WS_NT & 128) != 0 && OPK == OP_PRELU_NORM)>(
               A + (size_t)r * p.lda + kc * 8);
      if constexpr (N1B) rh[s][j] = ldg16h<(CTN_WS_NT & 64) != 0>(H1 + (size_t)r * p.lda + kc * 8);
      if constexpr (CB) {
      } else if constexpr (OPK != OP_PLAIN && !FOLDS && (CTN_WS_EXP & 2048)) {
        ast[s][j] = make_float2(0.1f, 1.3f);   // timing only: no statistics loads
      } else if constexpr (OPK != OP_PLAIN && !FOLDS) {
        ast[s][j] = p.aop.stats[stat_index<NK>(r, Kp)];
      }
      if constexpr (N1B && NK == NORM_CLN && !CB) asm1[s][j] = p.aop.sums[r];
    }
  };
  // ra -> LDS image of tile t (fragment (mb, kb) at (mb*KB + kb) KiB).  Rows of padded
  // frames are staged as zeros, so every output row of a padded frame is exactly 0
  // (+ the residual's zero row) and contributes nothing to any statistic.
  // tu may run past the range: such tiles are clamped to the last one (staged again,
  // never stored, and not counted in the alpha gradient).
  auto stage = [&](auto le1, int tu, char* buf, auto slot) __attribute__((always_inline)) {
    constexpr bool LE1 = decltype(le1)::value;
    constexpr int s = decltype(slot)::value;
    const int t = tu < t1 ? tu : t1 - 1;
    const int tk = (t * TM) % Kp;   // frame index of the tile's first row (wave-uniform)
    if constexpr (CB) {
      if (t - bbase >= 64) batch_load(t);
    }
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      v4u v = ra[s][j];
      const int r = rl0 + j * RSTEP;
      if constexpr (N1B) {
        // same arithmetic as norm1_bwd_kernel (ctn_tcn.hip), element by element
        float2 sm, st;
        if constexpr (NK == NORM_GLN) {
          const int m = (t * TM) / Kp;
          sm = sst[m];
          st = sst1[m];
        } else if constexpr (CB) {   // cLN: per-row statistics and means of this tile
          sm = bcast(bsm[j], t);
          st = bcast(bst[j], t);
        } else {   // cLN: per-row statistics and means, loaded with the row
          sm = asm1[s][j];
          st = ast[s][j];
        }
        float g[8], h[8];
        unpack_bf16x8(v, g);
        unpack_bf16x8(rh[s][j], h);
        float ca = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float o[2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const float hv = h[2 * e + u];
            const float ah = (prelu(hv, oal) - st.x) * st.y;
            const float ga = st.y * (g[2 * e + u] - sm.x - ah * sm.y);
            o[u] = ga * prelu_dx(hv, oal);
            ca += ga * prelu_da(hv);
          }
          v[e] = pk_bf16(o[0], o[1]);
        }
        calpha += (tu < t1 && tk + r < Kv) ? ca : 0.f;
      } else if constexpr (OPK != OP_PLAIN) {
        float2 st;
        if constexpr (FOLDS) st = sst[(t * TM) / Kp];
        else if constexpr (CB) st = bcast(bst[j], t);
        else st = ast[s][j];
        float f[8];
        unpack_bf16x8(v, f);
        const f32x2_t m2 = {st.x, st.x};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f32x2_t x = {f[2 * e], f[2 * e + 1]};
          if constexpr (OPK == OP_PRELU_NORM) x = prelu2<LE1>(x, oal);
          x = pfma(x - m2, f32x2_t{st.y * og[2 * e], st.y * og[2 * e + 1]}, f32x2_t{ob[2 * e], ob[2 * e + 1]});
          v[e] = pk_bf16(x[0], x[1]);
        }
      }
      const v4u z = v4u{0u, 0u, 0u, 0u};
      v = tk + r < Kv ? v : z;   // tiles never straddle utterances (Kp % TM == 0)
      if constexpr (N1B) ghv[j] = v;   // dL/dh1 for the weight-gradient kernel (padded rows 0)
      stg16(buf + (r >> 4) * KB * 1024 + ws_slot(r & 15, kc & 3, kc >> 2), v);
    }
  };
  // global store of the dL/dh1 chunks staged by stage(tu)
  auto store_gh = [&](int tu) __attribute__((always_inline)) {
    if constexpr (N1B && !(CTN_WS_EXP & 1024)) {   // bit 10 (timing only): no dL/dh1 stores
      if (tu < t1) {
#pragma unroll
        for (int j = 0; j < NA; ++j) stg16h<NTG>(GH + (size_t)(tu * TM + rl0 + j * RSTEP) * p.lda + kc * 8, ghv[j]);
      }
    }
  };

  // ---- epilogue constants
  constexpr bool HAS_R = EPI == EPI_RESID || EPI == EPI_NORM_BWD;
  constexpr bool HAS_STATS = EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD;
  const float eal = (EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD) ? p.alpha[0] : 0.f;
  if constexpr (EPI == EPI_NORM_BWD)
    for (int c = tid; c < NS; c += NT) sgam[c] = p.gamma[n0 + c];
  const bf16raw* Rp = reinterpret_cast<const bf16raw*>(p.R);
  bf16raw* Cp = reinterpret_cast<bf16raw*>(p.C);
  v4u rn[MB][Q];   // epilogue operand of the current tile (loaded one tile ahead)
  float2 est[MB];  // EPI_NORM_BWD forward statistics of the lane's rows
  auto load_r = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int r = t * TM + mb * 16 + lr;
      if constexpr (HAS_R) {
        const size_t off = (size_t)r * p.ldr + colbase;
#pragma unroll
        for (int q = 0; q < Q; ++q) rn[mb][q] = ldg16h<(CTN_WS_NT & 256) != 0>(Rp + off + q * 8);
      }
      if constexpr (EPI == EPI_NORM_BWD) est[mb] = p.stats[stat_index<NK>(r, Kp)];
    }
  };

  // LDS fragment reads run LA k-steps ahead of the MFMAs that consume them (a
  // register window of LA+1 steps), so a k-step's MFMAs never wait on a read issued
  // just before them (one read in flight per step exposed the LDS latency 16x/tile).
  constexpr int LA = SWP ? 0 : WV == 16 ? (OPK == OP_PLAIN ? CTN_WS_LA16 : 0) : CTN_WS_LA8;
  auto mfma_tile = [&](const char* buf, f32x4_t (&acc)[MB][NB]) __attribute__((always_inline)) {
    if constexpr (CTN_WS_PRIO) __builtin_amdgcn_s_setprio(1);   // experiment: MFMA issue first
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    v4u bw[LA + 1][MB];
    auto rd = [&](int kb) __attribute__((always_inline)) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) bw[kb % (LA + 1)][mb] = ldg16(buf + mb * KB * 1024 + ws_slot(lr, lg, kb));
    };
#pragma unroll
    for (int kb = 0; kb < LA && kb < KB; ++kb) rd(kb);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      if (kb + LA < KB) rd(kb + LA);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const v4u b = bw[kb % (LA + 1)][mb];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          if constexpr (CTN_WS_EXP & 4) acc[mb][nb][kb & 3] += __uint_as_float(b[0] ^ wf[nb][kb][1]);
          else acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[nb][kb]),
                                                                     __builtin_bit_cast(bf16x8_t, b), acc[mb][nb], 0, 0, 0);
      }
    }
    if constexpr (LA > 0 && !(CTN_WS_EXP & 4)) {
      // pin the interleave (the register-pressure scheduler would otherwise pull each
      // read down to its MFMAs): prologue reads, then per k-step its look-ahead reads
      // followed by its MFMAs
      __builtin_amdgcn_sched_group_barrier(0x100, MB * (LA < KB ? LA : KB), 0);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        if (kb + LA < KB) __builtin_amdgcn_sched_group_barrier(0x100, MB, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, MB * NB, 0);
      }
    }
    if constexpr (CTN_WS_PRIO) __builtin_amdgcn_s_setprio(0);
  };

  // gLN run partial of this wave (WsRuns layout); every lane stores the same value
  double run_s = 0.0, run_q = 0.0;
  const int tpu = Kp / TM, m0 = t0 / tpu;
  int run_m = m0;
  const int kmax = ws_runs_kmax(ntile, nr, tpu);
  // per-lane fp64 partials of the current utterance run, reduced over the wave and
  // stored once per run
  auto flush_run = [&]() __attribute__((always_inline)) {
    // DPP, not ds_bpermute: no LDS-unit cross-lane traffic while LDS-DMA is in flight
    // (dual-GEMM reproducibility)
    const double s = wave_sum_dpp_d(run_s), q = wave_sum_dpp_d(run_q);
    if (lane == 0) p.grp_slab[((size_t)rr * (S * WV) + wslot) * kmax + (run_m - m0)] = make_double2(s, q);
  };

  // epilogue of tile t from its accumulators: lane holds rows t*TM + mb*16 + lr,
  // channels colbase .. colbase+NV-1.  Branch-free (packed fp32 math).  The math
  // leaves the packed outputs in ov; store_out(t) writes them.
  v4u ov[MB][Q];
  auto store_out = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      bf16raw* dst = Cp + (size_t)(t * TM + mb * 16 + lr) * p.ldc + colbase;
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if constexpr (!(CTN_WS_EXP & 1)) stg16h<NTO>(dst + q * 8, ov[mb][q]);
    }
  };
  auto epilogue_math = [&](auto le1, int t, const f32x4_t (&acc)[MB][NB]) __attribute__((always_inline)) {
    constexpr bool LE1 = decltype(le1)::value;
    f32x2_t gs2 = {0.f, 0.f}, gq2 = {0.f, 0.f};   // gLN partials over the tile
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int r = t * TM + mb * 16 + lr;
      f32x2_t v2[NV / 2];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        v2[2 * nb] = f32x2_t{acc[mb][nb][0], acc[mb][nb][1]};
        v2[2 * nb + 1] = f32x2_t{acc[mb][nb][2], acc[mb][nb][3]};
      }
      f32x2_t s2 = {0.f, 0.f}, q2 = {0.f, 0.f};
      if constexpr (CTN_WS_EXP & 8) {
      } else if constexpr (EPI == EPI_PRELU_STATS) {
#pragma unroll
        for (int c = 0; c < NV / 2; ++c) {
          const f32x2_t a2 = prelu2<LE1>(v2[c], eal);
          s2 += a2;
          q2 = pfma(a2, a2, q2);
        }
      } else if constexpr (EPI == EPI_RESID) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          float f[8];
          unpack_bf16x8(rn[mb][q], f);
#pragma unroll
          for (int e = 0; e < 4; ++e) v2[q * 4 + e] += f32x2_t{f[2 * e], f[2 * e + 1]};
        }
      } else if constexpr (EPI == EPI_NORM_BWD) {
        const f32x2_t rs = {est[mb].y, est[mb].y}, ms = {-est[mb].x * est[mb].y, -est[mb].x * est[mb].y};
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          float f[8];
          unpack_bf16x8(rn[mb][q], f);
          const float4 g0 = *reinterpret_cast<const float4*>(&sgam[colbase - n0 + q * 8]);
          const float4 g1 = *reinterpret_cast<const float4*>(&sgam[colbase - n0 + q * 8 + 4]);
          const f32x2_t gq[4] = {{g0.x, g0.y}, {g0.z, g0.w}, {g1.x, g1.y}, {g1.z, g1.w}};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f32x2_t ah = pfma(prelu2<LE1>(f32x2_t{f[2 * e], f[2 * e + 1]}, eal), rs, ms);   // hat a
            const f32x2_t ga = v2[q * 4 + e] * gq[e];
            s2 += ga;
            q2 = pfma(ga, ah, q2);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < Q; ++q)
        ov[mb][q] = v4u{pk_bf16(v2[q * 4][0], v2[q * 4][1]), pk_bf16(v2[q * 4 + 1][0], v2[q * 4 + 1][1]),
                        pk_bf16(v2[q * 4 + 2][0], v2[q * 4 + 2][1]), pk_bf16(v2[q * 4 + 3][0], v2[q * 4 + 3][1])};
      if constexpr (HAS_STATS) {
        if constexpr (NK == NORM_GLN) {
          if constexpr (MB == 1) {
            gs2 = s2;
            gq2 = q2;
          } else {
            gs2 += s2;
            gq2 += q2;
          }
        } else {
          // per-row partial over this wave's 16*NB channels: reduce across the 4 lane
          // groups; all four groups store the same value (no divergent store)
          const float s = xsum_rows(s2[0] + s2[1]), ss = xsum_rows(q2[0] + q2[1]);   // VALU swaps
          if (CLN_FIN && p.stats_out) {
            if (lg == 0) scln[((t & 1) * TM + mb * 16 + lr) * WV + wid] = make_double2((double)s, (double)ss);
          } else {
            p.grp_slab[(size_t)r * (S * WV) + wslot] = make_double2((double)s, (double)ss);
          }
        }
      }
    }
    if constexpr (HAS_STATS && NK == NORM_GLN) {
      // the wave's tiles of one utterance accumulate into one run partial (WsRuns)
      const int m = (t * TM) / Kp;
      if (m != run_m) {
        flush_run();
        run_m = m;
        run_s = run_q = 0.0;
      }
      run_s += (double)(gs2[0] + gs2[1]);
      run_q += (double)(gq2[0] + gq2[1]);
    }
  };
  auto epilogue = [&](auto le1, int t, const f32x4_t (&acc)[MB][NB]) __attribute__((always_inline)) {
    epilogue_math(le1, t, acc);
    store_out(t);
  };
  // cLN: final (mean, rstd) of tile t's rows from the WV wave partials, summed in wave
  // order in fp64 (the arithmetic of stats_finalize over this layout's parts)
  auto cln_final = [&](int t) __attribute__((always_inline)) {
    if constexpr (CLN_FIN) {
      if (p.stats_out && tid < TM) {
        double sm = 0.0, sq = 0.0;
#pragma unroll 1
        for (int w = 0; w < WV; ++w) {
          const double2 v = scln[((t & 1) * TM + tid) * WV + w];
          sm += v.x;
          sq += v.y;
        }
        const double mean = sm / p.Nout;
        double var = sq / p.Nout - mean * mean;
        if (var < 0.0) var = 0.0;
        p.stats_out[(size_t)t * TM + tid] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)p.eps)));
      }
    }
  };

  // wait for the resident weight and the epilogue/operand constants once, before the
  // tile loop (CTN_WS_EARLY)
  auto ready_all = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) ready(wf[nb][kb]);
    if constexpr (AFF) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { ready(og[e]); ready(ob[e]); }
    }
    ready(oal);
    ready(eal);
  };
  if constexpr (CTN_WS_EARLY) ready_all();
  if (t0 >= t1) {
    fold_stats();   // a workgroup without tiles still stores its utterances' pairs
    return;
  }

  // Pipeline, one LDS-only barrier per tile; tile t+1 is staged into the other LDS
  // buffer (its last reader finished before this barrier) from registers loaded an
  // iteration earlier.  Every counted wait has the same memory operations behind it
  // on every iteration, so none drains the prefetch; out-of-range tiles are clamped
  // to the last one (never stored).  With SWP the MFMAs of tile t interleave with
  // the epilogue of tile t-1 (two accumulator sets).
  auto clampt = [&](int t) __attribute__((always_inline)) { return t < t1 ? t : t1 - 1; };
  // Diagnostic build only (tools/microbench/ws_bench.hip -DCTN_WS_STAMP=1): s_memtime
  // stamps between the loop's phases, per-wave cycle sums in ws_stamps[] (shares only:
  // the stamps' lgkmcnt(0) forbid overlaps the real kernel has)
#if CTN_WS_STAMP
  unsigned long long st_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_last = 0;
#define WS_STAMP(i)                                                                            \
  do {                                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    unsigned long long t_;                                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                 \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    if (st_last) st_sum[i] += t_ - st_last;                                                    \
    st_last = t_;                                                                              \
  } while (0)
#else
#define WS_STAMP(i) \
  do {              \
  } while (0)
#endif
  // LE1 = (alpha <= 1) selects the exact two-instruction PReLU form once per kernel
  auto run = [&](auto le1) __attribute__((always_inline)) {
    if constexpr (WDMA) {
      // The tile's image arrives by LDS-DMA WS_DR-1 tiles ahead, with no registers and
      // no staging pass (the rows of padded frames are zero in a plain operand already).
      // Fragment f = wid + WV*i of every tile is this wave's: lane (lg, x) of the 1-KiB
      // fragment image holds row mb*16 + (x ^ (lg + 4(kb&3))), k-chunk 4kb + lg, the
      // ws_slot layout.  Per tile: wait for this wave's DMA of tile t (counted: the DMA
      // instructions of the later tiles and the output stores issued since may stay in
      // flight), barrier, DMA of tile
      // t+WS_DR-1 into the slot tile t-1 was read from, MFMAs, epilogue, stores.
      // The count assumes exactly SPT output stores per tile after each tile's DMA:
      // more (cln_final) only make the wait stricter, fewer would make it too loose,
      // so the store-free bound-finding build (CTN_WS_EXP bit 0) counts none.
      constexpr int NF = MB * KB, NFW = NF / WV, SPT = (CTN_WS_EXP & 1) ? 0 : MB * Q;
      static_assert(NF % WV == 0, "whole fragments per wave");
      static_assert(NFW * (WS_DR - 2) + SPT * (WS_DR - 1) <= 23, "vmcnt range of vmwait23");
      uint32_t voff[NFW];
#pragma unroll
      for (int i = 0; i < NFW; ++i) {
        const int f = wid + WV * i, mb = f / KB, kb = f % KB, lq = lane >> 4;
        const int row = mb * 16 + ((lane & 15) ^ (lq + 4 * (kb & 3)));
        voff[i] = (uint32_t)(row * p.lda + (kb * 4 + lq) * 8) * 2u;
      }
      auto dma = [&](int t) __attribute__((always_inline)) {
        if (t >= t1) return;
        const rsrc_t rs = du_rsrc(A + (size_t)t * TM * p.lda, (long)TM * p.lda * 2);
#pragma unroll
        for (int i = 0; i < NFW; ++i) du_dma16(rs, sA[t % WS_DR] + (wid + WV * i) * 1024, voff[i], 0);
      };
      auto mn = [](int a, int b) { return a < b ? a : b; };
      f32x4_t acc[MB][NB];
      fold_stats();
      if constexpr (WFL) {
        if (tid < WS_DR * WV) {
          (&fl_full[0][0])[tid] = 0u;
          (&fl_done[0][0])[tid] = 0u;
        }
        __syncthreads();
      }
      for (int i = 0; i < WS_DR - 1; ++i) dma(t0 + i);
      if constexpr (!CTN_WS_EARLY) ready_all();
      if constexpr (WFL) {
        // tile t in slot t % WS_DR, generation (t - t0) / WS_DR + 1 of that slot
        for (int t = t0; t < t1; ++t) {
          {
            constexpr int NST = NFW * (WS_DR - 2) + SPT * (WS_DR - 1);   // steady state
            const int n = NFW * mn(WS_DR - 2, t1 - 1 - t) + SPT * mn(WS_DR - 1, t - t0);
            if (n == NST) vmwait_c<NST>();
            else vmwait23(n);
          }
          const int slot = t % WS_DR;
          const uint32_t gen = (uint32_t)((t - t0) / WS_DR + 1);
          flag_signal(&fl_full[slot][wid], gen);   // this wave's DMA of tile t landed
          flag_wait<WV>(fl_full[slot], gen, p.err);       // every wave's
          mfma_tile(sA[slot], acc);
          if constexpr (!(CTN_WS_EXP & 64)) __builtin_amdgcn_sched_barrier(0);
          flag_signal(&fl_done[slot][wid], gen);   // this wave's reads of the slot done
          const int tn = t + WS_DR - 1;            // into the slot of tile t - 1
          if (tn < t1) {
            if (t > t0) flag_wait<WV>(fl_done[(t - 1) % WS_DR], (uint32_t)((t - 1 - t0) / WS_DR + 1), p.err);
            dma(tn);
          }
          epilogue_math(le1, t, acc);
          store_out(t);
        }
      } else if constexpr (CTN_WS_PP && WV == 16) {
        // ping-pong: half 0 (waves 0-7) MFMA(t) | epilogue(t); half 1 (waves 8-15)
        // epilogue(t-1) | MFMA(t), the two phases of tile t separated by a barrier.  The
        // slot refilled at iteration t (tile t-1's) was last read by half 1 in phase 2
        // of iteration t-1, before this iteration's first barrier.
        const bool late = wid >= WV / 2;
        for (int t = t0; t < t1; ++t) {
          {
            // half 1 has stored nothing in iteration t0 (no tile t0 - 1): one store group
            // fewer behind the DMA of tile t, so its count is one group stricter
            constexpr int NST = NFW * (WS_DR - 2) + SPT * (WS_DR - 1);   // steady state
            const int ds = t - t0 - (late ? 1 : 0);
            const int n = NFW * mn(WS_DR - 2, t1 - 1 - t) + SPT * mn(WS_DR - 1, ds < 0 ? 0 : ds);
            if (n == NST) vmwait_c<NST>();
            else vmwait23(n);
          }
          lds_barrier();
          dma(t + WS_DR - 1);
          if (!late) {
            mfma_tile(sA[t % WS_DR], acc);
          } else if (t > t0) {
            epilogue_math(le1, t - 1, acc);
            store_out(t - 1);
          }
          __builtin_amdgcn_sched_barrier(0);
          lds_barrier();
          if (t > t0) cln_final(t - 1);   // both halves' partials of tile t - 1 are in LDS
          if (!late) {
            epilogue_math(le1, t, acc);
            store_out(t);
          } else {
            mfma_tile(sA[t % WS_DR], acc);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        if (late) {
          epilogue_math(le1, t1 - 1, acc);
          store_out(t1 - 1);
        }
      } else
      for (int t = t0; t < t1; ++t) {
        {
          constexpr int NST = NFW * (WS_DR - 2) + SPT * (WS_DR - 1);   // steady state
          const int n = NFW * mn(WS_DR - 2, t1 - 1 - t) + SPT * mn(WS_DR - 1, t - t0);
          if (n == NST) vmwait_c<NST>();
          else vmwait23(n);
        }
        lds_barrier();
        if (t > t0) cln_final(t - 1);
        dma(t + WS_DR - 1);
        mfma_tile(sA[t % WS_DR], acc);
        if constexpr (!(CTN_WS_EXP & 64)) __builtin_amdgcn_sched_barrier(0);
        epilogue_math(le1, t, acc);
        store_out(t);
      }
    } else if constexpr (!SWP) {
      f32x4_t acc[MB][NB];
      // prologue: tiles t0 .. t0+PF-1 into slots 0 .. PF-1; t0 staged; t0+PF into slot 0
      static_for<PF>([&](auto i) { load_a(clampt(t0 + decltype(i)::value), i); });
      load_r(t0);
      fold_stats();
      stage(le1, t0, sA[t0 & 1], std::integral_constant<int, 0>{});
      store_gh(t0);
      load_a(clampt(t0 + PF), std::integral_constant<int, 0>{});
      if constexpr (!CTN_WS_EARLY) ready_all();
      for (int tb = t0; tb < t1; tb += PF) {
        static_for<PF>([&](auto u) {
          constexpr int nx = (decltype(u)::value + 1) % PF;   // slot of tile t+1
          const int t = tb + decltype(u)::value;
          if (PF == 1 || t < t1) {
            WS_STAMP(7);
            lds_barrier();
            if (t > t0) cln_final(t - 1);
            WS_STAMP(0);
            mfma_tile(sA[t & 1], acc);
            if constexpr (!(CTN_WS_EXP & 64)) __builtin_amdgcn_sched_barrier(0);
            WS_STAMP(1);
            if constexpr (CTN_WS_ORDER == 1) {
              // next tile's operand (its buffer's last reader finished before the barrier)
              stage(le1, t + 1, sA[(t + 1) & 1], std::integral_constant<int, nx>{});
              WS_STAMP(2);
              load_a(clampt(t + 1 + PF), std::integral_constant<int, nx>{});
              WS_STAMP(3);
              epilogue_math(le1, t, acc);
              WS_STAMP(4);
              load_r(clampt(t + 1));   // rn(t) consumed above
              WS_STAMP(5);
              store_out(t);
              store_gh(t + 1);
              WS_STAMP(6);
            } else {
              epilogue(le1, t, acc);
              load_r(clampt(t + 1));
              stage(le1, t + 1, sA[(t + 1) & 1], std::integral_constant<int, nx>{});
              store_gh(t + 1);
              load_a(clampt(t + 1 + PF), std::integral_constant<int, nx>{});
            }
          }
        });
      }
    } else {
      f32x4_t accP[MB][NB], accC[MB][NB];
      load_a(t0, std::integral_constant<int, 0>{});
      fold_stats();
      stage(le1, t0, sA[t0 & 1], std::integral_constant<int, 0>{});
      load_a(clampt(t0 + 1), std::integral_constant<int, 0>{});
      lds_barrier();
      mfma_tile(sA[t0 & 1], accP);
      load_r(t0);
      stage(le1, t0 + 1, sA[(t0 + 1) & 1], std::integral_constant<int, 0>{});
      load_a(clampt(t0 + 2), std::integral_constant<int, 0>{});
      if constexpr (!CTN_WS_EARLY) ready_all();
      // unrolled by two so the two accumulator sets swap roles without copies
      auto step = [&](int t, f32x4_t (&cur)[MB][NB], f32x4_t (&prev)[MB][NB]) __attribute__((always_inline)) {
        lds_barrier();
        mfma_tile(sA[t & 1], cur);
        epilogue(le1, t - 1, prev);
        load_r(t);
        stage(le1, t + 1, sA[(t + 1) & 1], std::integral_constant<int, 0>{});
        load_a(clampt(t + 2), std::integral_constant<int, 0>{});
      };
      int t = t0 + 1;
      for (; t + 1 < t1; t += 2) {
        step(t, accC, accP);
        step(t + 1, accP, accC);
      }
      if (t < t1) {
        step(t, accC, accP);
        epilogue(le1, t1 - 1, accC);
      } else {
        epilogue(le1, t1 - 1, accP);
      }
    }
  };
  const float al_any = (OPK == OP_PRELU_NORM || N1B) ? oal : eal;
  if constexpr (OPK == OP_PRELU_NORM || N1B || HAS_STATS) {
    if (al_any <= 1.f) run(std::true_type{});
    else run(std::false_type{});
  } else {
    run(std::true_type{});
  }
  if constexpr (HAS_STATS && NK == NORM_GLN) flush_run();
  if constexpr (CLN_FIN) {
    lds_barrier();
    cln_final(t1 - 1);
  }
#if CTN_WS_STAMP
  if (lane == 0)
    for (int i = 0; i < 8; ++i) ws_stamps[((size_t)blockIdx.x * 16 + wid) * 8 + i] = st_sum[i];
#endif
  if constexpr (N1B) {   // fixed-order workgroup sum of the alpha-gradient partials
    const float w = wave_sum_dpp(calpha);
    if (lane == 0) salpha[wid] = w;
    __syncthreads();
    if (tid == 0) {
      double a = 0.0;
      for (int i = 0; i < WV; ++i) a += (double)salpha[i];
      p.aop.apart[blockIdx.x] = (float)a;
    }
  }
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
// CTN_WS_1536=0: c5's 1536-channel mask conv on the tiled gemm_rows kernel instead (A/B)
static bool ws1536_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("CTN_WS_1536");
    on = (e && atoi(e) == 0) ? 0 : 1;
  }
  return on == 1;
}

static bool ws_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("CTN_GEMM_WS");
    on = (e && atoi(e) == 0) ? 0 : 1;
  }
  return on == 1;
}

// (Nout, Kred) shapes with a resident-weight instantiation
static bool ws_shape(int Nout, int Kred, int* nb, int* kb) {
  if ((Nout == 512 || Nout == 1536) && Kred == 256) { *nb = 4; *kb = 8; return true; }
  if (Nout == 256 && Kred == 512) { *nb = 2; *kb = 16; return true; }
  if (Nout == 256 && Kred == 256) { *nb = 2; *kb = 8; return true; }
  return false;
}

static bool ws_pair(int opk, int epi) {   // (operand op, epilogue) pairs used on the path
  return (opk == OP_PLAIN && (epi == EPI_PRELU_STATS || epi == EPI_NORM_BWD || epi == EPI_RESID || epi == EPI_STORE)) ||
         (opk == OP_PRELU_NORM && epi == EPI_RESID) || (opk == OP_NORM && epi == EPI_STORE) ||
         (opk == OP_NORM1_BWD && epi == EPI_RESID);
}

bool gemm_ws_eligible(DType dt, const GemmRows& p) {
  int nb, kb;
  if (dt != BF16 || !ws_enabled() || !ws_shape(p.Nout, p.Kred, &nb, &kb) || !ws_pair(p.aop.kind, p.epi)) return false;
  // 1536 outputs (c5's mask conv): the plain-operand store form only, as three slices
  if (p.Nout == 1536 && (p.aop.kind != OP_PLAIN || p.epi != EPI_STORE || !ws1536_enabled())) return false;
  if (p.g.Kp % WS_TM || p.lda % 8 || p.ldw % 8 || p.ldc % 8) return false;
  // 32-bit tile offsets and buffer sizes (the LDS-DMA ring's du_rsrc clamps at 2^31 bytes)
  if (p.g.rows() * (p.Kred > p.Nout ? p.Kred : p.Nout) * 2 >= (1L << 31)) return false;
  if ((p.epi == EPI_RESID || p.epi == EPI_NORM_BWD) && p.ldr % 8) return false;
  if (p.aop.kind != OP_PLAIN && p.aop.norm == NORM_GLN && p.g.M > WS_FOLD_MAX) return false;
  if (p.aop.kind == OP_NORM1_BWD && (!p.aop.aux || !p.aop.aout || !p.aop.apart || !p.aop.stats ||
                                     (!p.aop.fold.slab && !p.aop.sums) ||
                                     (p.aop.norm == NORM_CLN && !p.aop.sums)))
    return false;
  return true;
}

static int ws_slices(const GemmRows& p);
static int ws_waves(const GemmRows& p);
bool gemm_ws_final_cln(DType dt, const GemmRows& p) {
  // the 16-wave (non-interleaved, one slice) configuration of Nout = 512 or the 8-wave
  // Nout = 512 norm-backward one: every wave's partial meets in one workgroup
  return gemm_ws_eligible(dt, p) && p.epi == EPI_PRELU_STATS && p.norm == NORM_CLN && p.aop.kind == OP_PLAIN &&
         p.Nout == 512 && p.Kred == 256 && ws_slices(p) == 1;
}

bool gemm_ws_can_fold(DType dt, const GemmRows& p) {
  return gemm_ws_eligible(dt, p) && p.aop.kind != OP_PLAIN && p.aop.norm == NORM_GLN;
}

// frame rows per tile (16, or 32 for the wide configuration)
static int ws_tile_rows(const GemmRows& p);
static int ws_waves(const GemmRows& p);     // waves per row range (all slices)
static int ws_slices(const GemmRows& p);

static int ws_ranges(const GemmRows& p) {
  const long nt = p.g.rows() / ws_tile_rows(p);
  // three 16-wave slice workgroups per range fill the CUs once: 80 ranges (a multiple of
  // 8, so a range's slices share an XCD and its L2 copy of the A tile)
  const int cap = ws_slices(p) == 3 ? (WS_GRID / 3) / 8 * 8 : WS_GRID;
  return (int)(nt < cap ? nt : cap);
}
int gemm_ws_grid(const GemmRows& p) { return ws_ranges(p) * ws_slices(p); }

// gLN partials use the run layout (WsRuns): ranges*waves*kmax entries in all,
// sized here as G groups of ceil(entries / G) parts; cLN: waves parts per row
WsRuns gemm_ws_runs(const GemmRows& p) {
  WsRuns w;
  const int tm = ws_tile_rows(p);
  w.ntile = (int)(p.g.rows() / tm);
  w.grid = ws_ranges(p);
  w.tpu = p.g.Kp / tm;
  w.waves = ws_waves(p);
  w.kmax = ws_runs_kmax(w.ntile, w.grid, w.tpu);
  return w;
}

int gemm_ws_group_parts(const GemmRows& p) {
  if (p.norm != NORM_GLN) return ws_waves(p);
  const WsRuns w = gemm_ws_runs(p);
  const long entries = (long)w.grid * w.waves * w.kmax;
  return (int)((entries + p.g.M - 1) / p.g.M);
}

static bool ws_wide(const GemmRows& p) {   // Nout = 512 (or 3 x 512) on 32-row tiles (16 waves per range)
  return (p.Nout == 512 || p.Nout == 1536) && p.Kred == 256 && p.epi != EPI_NORM_BWD;
}
static int ws_waves(const GemmRows& p) { return ws_wide(p) ? 16 * (p.Nout / 512) : 8; }
static int ws_tile_rows(const GemmRows& p) { return ws_wide(p) ? 32 : WS_TM; }
static int ws_slices(const GemmRows& p) { return p.Nout == 1536 ? 3 : ws_wide(p) ? CTN_WS_S512 : 1; }

// Register-staged kernel configurations: (NB, KB, waves, m-blocks, slices).  Nout = 512
// runs 16 waves of 32 channels per 32-row range (64 weight VGPRs per lane: 4 waves
// per SIMD, so one wave's latency hides behind another's work), as one 16-wave
// workgroup or as two 8-wave slice workgroups (CTN_WS_S512); Nout = 256 runs 8 waves
// of 32 channels with a 128-register weight slice on 16-row tiles.
template <int OPK, int NK, int EPI>
static hipError_t ws_launch_shape(const GemmRows& p, hipStream_t s) {
  int nb = 0, kb = 0;
  ws_shape(p.Nout, p.Kred, &nb, &kb);
  const dim3 grid(gemm_ws_grid(p));
  if (nb == 4 && kb == 8) {
    if constexpr (EPI == EPI_NORM_BWD)   // its epilogue needs more than the 128 registers of 16 waves
      hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 4, 8, 8, 1>), grid, dim3(512), 0, s, p);
    else if (ws_slices(p) == 3) {
      if constexpr (OPK == OP_PLAIN && EPI == EPI_STORE)
        hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 2, 8, 16, 2, 3>), grid, dim3(1024), 0, s, p);
    } else if (ws_slices(p) == 2)
      hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 2, 8, 8, 2, 2>), grid, dim3(512), 0, s, p);
    else
      hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 2, 8, 16, 2>), grid, dim3(1024), 0, s, p);
  }
  else if (nb == 2 && kb == 16)
    hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 2, 16, 8, 1>), grid, dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 2, 8, 8, 1>), grid, dim3(512), 0, s, p);
  return hipGetLastError();
}

template <int NK>
static hipError_t ws_launch_nk(const GemmRows& p, hipStream_t s) {
  if (p.aop.kind == OP_PRELU_NORM) return ws_launch_shape<OP_PRELU_NORM, NK, EPI_RESID>(p, s);
  if (p.aop.kind == OP_NORM1_BWD) return ws_launch_shape<OP_NORM1_BWD, NK, EPI_RESID>(p, s);
  if (p.aop.kind == OP_NORM) return ws_launch_shape<OP_NORM, NK, EPI_STORE>(p, s);
  switch (p.epi) {
    case EPI_PRELU_STATS: return ws_launch_shape<OP_PLAIN, NK, EPI_PRELU_STATS>(p, s);
    case EPI_NORM_BWD: return ws_launch_shape<OP_PLAIN, NK, EPI_NORM_BWD>(p, s);
    case EPI_RESID: return ws_launch_shape<OP_PLAIN, NORM_GLN, EPI_RESID>(p, s);
    default: return ws_launch_shape<OP_PLAIN, NORM_GLN, EPI_STORE>(p, s);
  }
}

hipError_t launch_gemm_ws(const GemmRows& pa, hipStream_t s) {
  GemmRows p = pa;
  p.err = device_error_word();   // the generation-word ring (CTN_WS_FLAGS) reports timeouts here
  const int nk = p.aop.kind != OP_PLAIN ? p.aop.norm : p.norm;
  return nk == NORM_GLN ? ws_launch_nk<NORM_GLN>(p, s) : ws_launch_nk<NORM_CLN>(p, s);
}

}  // namespace ctn
