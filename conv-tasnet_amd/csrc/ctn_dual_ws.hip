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
// up.  Here the roles are split inside the workgroup (12 waves,
// 3 per SIMD):
//   * 4 memory waves load the tiles into registers PF tiles ahead (plain global
//     loads, no LDS-DMA), apply the column operand's PReLU + norm on the way, write
//     the tile's images (A = gy in MFMA fragment order, B = op(d), R = raw d, row
//     statistics) into an LDS ring of NSL slots, publish FULL, and store the C image
//     consumers left in the slot NSL tiles earlier (whole 16-byte lanes, full rows);
//   * 8 consumer waves wait for FULL, run the row GEMM (resident W2 fragments, both
//     16-row blocks of the tile), the column GEMM (dW2 slice as MFMA accumulators),
//     the norm-2 backward epilogue into the slot's C image, and publish DONE.
// FULL / DONE are one generation word per wave per slot in LDS (the memory waves wait
// for the consumers' DONE of tile t-NSL before refilling its slot), so the MFMAs of
// one tile overlap the loads, transforms and stores of the next ones, and no wave
// ever waits on another wave's memory operations.  Every LDS read of another wave's
// data happens after that wave's `s_waitcnt lgkmcnt(0)` + generation-word store and
// this wave's matching generation-word load.
#include <stdlib.h>

#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int DV_TM = 32;                        // frame rows per tile
constexpr int DV_NC = 8, DV_NMW = 4;             // consumer / memory waves
constexpr int DV_NT = (DV_NC + DV_NMW) * 64;     // 768 threads
constexpr int DV_KB = 8, DV_KR = 256;            // reduction of the row part (gy channels)
constexpr int DV_NS = 128;                       // output channels per slice
constexpr int DV_GRID = 256;

// Bound-finding builds only (tools/microbench/dual_bench.hip -DCTN_DV_EXP=<bits>):
// bit 0 consumers skip all arithmetic (wait FULL, publish DONE), bit 1 no column part,
// bit 2 no epilogue math.
#ifndef CTN_DV_EXP
#define CTN_DV_EXP 0
#endif
// Diagnostic builds (tools/microbench/dual_ws_bench.hip): bit 0 lgkmcnt(0) after the
// memory waves' R-image writes, bit 1 R image written after the B image, bit 2
// lgkmcnt(0) after the consumers' C-image writes, bit 4 consumers store the raw d
// values they read from the R image in place of C (checked against d on the host).
#ifndef CTN_DV_DBG
#define CTN_DV_DBG 0
#endif

// slot layout (bytes)
constexpr int DV_A = DV_TM * DV_KR * 2;          // 16384: gy tile, WS fragment image (du_apiece)
constexpr int DV_BST = 1024 + 32;                // B image block stride: 16 columns x 32 rows + 32 B
constexpr int DV_B = 8 * DV_BST;                 // op(d) slice in 4-row x 16-column blocks (du_boff)
constexpr int DV_R = DV_TM * DV_NS * 2;          // 8192: raw d rows, 16-byte granules XOR row
constexpr int DV_C = DV_R;                       // C image, same addressing as R
constexpr int DV_ST = DV_TM * 8;                 // (mean, rstd): per row (cLN) or the tile's utterance (gLN)
constexpr int DV_PT = DV_TM * DV_NC * 8;         // cLN: per-row (sum ga, sum ga*hat a) of each consumer
constexpr int OFF_A = 0, OFF_B = OFF_A + DV_A, OFF_R = OFF_B + DV_B, OFF_C = OFF_R + DV_R;
constexpr int OFF_ST = OFF_C + DV_C, OFF_PT = OFF_ST + DV_ST;
template <int NK> constexpr int dv_slot() { return NK == NORM_CLN ? OFF_PT + DV_PT : OFF_ST + 16; }

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
// 16-byte granule g (channels 8g..8g+7) of row r in the R / C images
CTN_DEV int dv_roff(int r, int g) { return r * 256 + ((g ^ (r & 15)) << 4); }

CTN_DEV s16x4_t dv_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}

// Generation words.  Every lane reads the same word (wave-uniform by readfirstlane);
// the poll is followed by a compiler barrier so no LDS read of the published data is
// issued before the word that publishes it has been seen (LDS executes one wave's
// DS instructions in order).
// The spin is bounded (about 0.2 s): a protocol error ends the launch with wrong
// results instead of a wave that never finishes.
// (Volatile accesses keep their address space only through an explicitly LDS-typed
// pointer: through a generic one they become FLAT operations, whose waits drain every
// outstanding global load of the wave.)
typedef __attribute__((address_space(3))) volatile v4u lds_v4u;
typedef __attribute__((address_space(3))) volatile uint32_t lds_u32;
template <int N> CTN_DEV void dv_wait(const uint32_t* f, uint32_t gen) {
  static_assert(N == 4 || N == 8, "generation words per slot");
  const lds_v4u* fl = (const lds_v4u*)(f);
  for (uint32_t it = 0; it < (1u << 22); ++it) {
    const v4u a = fl[0];
    uint32_t mn = min(min(a[0], a[1]), min(a[2], a[3]));
    if constexpr (N == 8) {
      const v4u b = fl[1];
      mn = min(mn, min(min(b[0], b[1]), min(b[2], b[3])));
    }
    if (__builtin_amdgcn_readfirstlane(mn) >= gen) break;
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
}
// publish: this wave's LDS writes (and reads) complete, then the generation word
CTN_DEV void dv_signal(uint32_t* f, uint32_t gen) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  *(lds_u32*)(f) = gen;
  asm volatile("" ::: "memory");
}

template <int NK, int NSL, int PF>
__global__ __launch_bounds__(DV_NT) void gemm_dual_ws_kernel(GemmDual p) {
  constexpr int TM = DV_TM, KB = DV_KB, KR = DV_KR, NS = DV_NS;
  constexpr int SLOT = dv_slot<NK>();
  static_assert(NSL * SLOT <= 160 * 1024 - 512, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[NSL * SLOT];
  __shared__ __attribute__((aligned(16))) uint32_t fl_full[NSL][4];   // per memory wave
  __shared__ __attribute__((aligned(16))) uint32_t fl_done[NSL][8];   // per consumer wave
  __shared__ __attribute__((aligned(16))) float sgb[2][NS];            // gamma2 / beta2 of the slice

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
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
  else if (tid < NSL * 12) (&fl_done[0][0])[tid - NSL * 4] = 0u;
  if (tid < 2 * NS) sgb[tid / NS][tid % NS] = (tid < NS ? p.bop.gamma : p.bop.beta)[n0 + tid % NS];
  __syncthreads();

  if (wid < DV_NC) {
    // ======================= consumer waves =======================
    const int w = wid;
    // resident W fragments: fragment (group 4*sl + w/2, nb = w&1) of W (rows = output
    // channels): lane (lg, lr) of the MFMA result then holds output channels
    // cl .. cl+3 of frame row lr, cl = 32*(w/2) + 8*lg + 4*(w&1) (slice-local)
    v4u wf[KB];
    const bf16raw* WF = reinterpret_cast<const bf16raw*>(p.Wf);
    const bf16raw* W = reinterpret_cast<const bf16raw*>(p.W);
    {
      const int n = n0 + 32 * (w >> 1) + (lr >> 2) * 8 + (w & 1) * 4 + (lr & 3);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
        wf[kb] = WF ? ldg16(WF + frag_offset(4 * sl + (w >> 1), w & 1, kb, lane, KR))
                    : ldg16(W + (size_t)n * p.ldw + kb * 32 + lg * 8);
    }
    const int cl = 32 * (w >> 1) + 8 * lg + 4 * (w & 1);
    const float4 g4 = *reinterpret_cast<const float4*>(p.gamma + n0 + cl);
    const float eal = p.alpha[0];
    // column part: wave (wp, wn) owns dW2 blocks p in [64 wp, +64), n in [n0 + 64 wn, +64)
    const int wp = w >> 1, wn = w & 1;
    f32x4_t dacc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) dacc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // lane-constant LDS addresses (ctn_gemm_dual.hip's, B blocks at stride DV_BST)
    const int rbase = lg * 256 + ((lr ^ ((lg & 1) * 12)) << 4);   // + rb * KB * 1024 + kb * 1024
    const int q = lr >> 2, pp = lr & 3;
    int abase[2], bbase[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 8 * lg + 4 * h + q;
      abase[h] = (lg >> 1) * KB * 1024 + 2 * wp * 1024 + (pp >> 1) * 256 + (((row & 15) ^ ((pp >> 1) * 12)) << 4) +
                 (pp & 1) * 8;
      bbase[h] = wn * 4 * DV_BST + dv_boff(row, 4 * pp);
    }
    const int ro = dv_roff(lr, 4 * (w >> 1) + lg) + (w & 1) * 8;   // row lr; row 16 + lr at + 4096

    double run_s = 0.0, run_q = 0.0;
    const int m0 = t0 / tpu;
    int run_m = m0;
    const int kmax = ws_runs_kmax(ntile, nr, tpu);
    double2* run_slab = p.grp_slab + (((size_t)rr * S + sl) * DV_NC + w) * kmax;
    auto flush = [&]() __attribute__((always_inline)) {
      const double s = wave_sum_dpp_d(run_s), ss = wave_sum_dpp_d(run_q);
      run_slab[run_m - m0] = make_double2(s, ss);
    };

    auto run = [&](auto le1) __attribute__((always_inline)) {
      constexpr bool LE1 = decltype(le1)::value;
      int slot = 0;
      uint32_t gen = 1;
      for (int t = t0; t < t1; ++t) {
        dv_wait<4>(fl_full[slot], gen);
        char* base = smem + slot * SLOT;
        if constexpr (!(CTN_DV_EXP & 1)) {
          // ---- column part first (its fragments die before the row part's accumulators
          //      live): dW2 += gy_tile^T . op(d)_tile (reduction over the 32 rows)
          if constexpr (!(CTN_DV_EXP & 2)) {
            const char* a = base + OFF_A;
            const char* bb = base + OFF_B;
            bf16x8_t bfr[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const s16x4_t lo = dv_tr(bb + bbase[0] + j * DV_BST), hi = dv_tr(bb + bbase[1] + j * DV_BST);
              bfr[j] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int o = (i >> 1) * 1024 + (i & 1) * 512;
              const s16x4_t lo = dv_tr(a + abase[0] + o), hi = dv_tr(a + abase[1] + o);
              const bf16x8_t af = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
              for (int j = 0; j < 4; ++j) dacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], dacc[i][j], 0, 0, 0);
            }
          }
          // ---- row part: both 16-row blocks against the resident W fragments
          f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kb = 0; kb < KB; ++kb) {
            const v4u b0 = *reinterpret_cast<const v4u*>(base + OFF_A + rbase + kb * 1024);
            const v4u b1 = *reinterpret_cast<const v4u*>(base + OFF_A + KB * 1024 + rbase + kb * 1024);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[kb]),
                                                           __builtin_bit_cast(bf16x8_t, b0), acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[kb]),
                                                           __builtin_bit_cast(bf16x8_t, b1), acc1, 0, 0, 0);
          }
          // ---- epilogue: norm-2 backward sums, C image
          const uint2 r0 = *reinterpret_cast<const uint2*>(base + OFF_R + ro);
          const uint2 r1 = *reinterpret_cast<const uint2*>(base + OFF_R + ro + 4096);
          float2 e0, e1;
          if constexpr (NK == NORM_GLN) {   // the tile's utterance statistics, staged by the memory waves
            e0 = e1 = *reinterpret_cast<const float2*>(base + OFF_ST);
          } else {
            e0 = *reinterpret_cast<const float2*>(base + OFF_ST + lr * 8);
            e1 = *reinterpret_cast<const float2*>(base + OFF_ST + (16 + lr) * 8);
          }
          f32x2_t s2[2] = {{0.f, 0.f}, {0.f, 0.f}}, q2[2] = {{0.f, 0.f}, {0.f, 0.f}};
          if constexpr (!(CTN_DV_EXP & 4)) {
            const f32x2_t gq[2] = {{g4.x, g4.y}, {g4.z, g4.w}};
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const uint2 rw = j ? r1 : r0;
              const f32x4_t& ac = j ? acc1 : acc0;
              const float2 est = j ? e1 : e0;
              const f32x2_t rs = {est.y, est.y}, ms = {-est.x * est.y, -est.x * est.y};
              const uint32_t rwv[2] = {rw.x, rw.y};
#pragma unroll
              for (int c = 0; c < 2; ++c) {
                const f32x2_t x = {__uint_as_float(rwv[c] << 16), __uint_as_float(rwv[c] & 0xffff0000u)};
                f32x2_t ah = pfma(prelu2<LE1>(x, eal), rs, ms);   // hat a
                if constexpr (NK == NORM_CLN) {   // padded frames: statistics not finite
                  const bool ok = (t * TM) % Kp + 16 * j + lr < Kv;
                  ah = ok ? ah : f32x2_t{0.f, 0.f};
                }
                const f32x2_t ga = f32x2_t{ac[2 * c], ac[2 * c + 1]} * gq[c];
                s2[j] += ga;
                q2[j] = pfma(ga, ah, q2[j]);
              }
            }
          }
          if constexpr (CTN_DV_DBG & 16) {
            *reinterpret_cast<uint2*>(base + OFF_C + ro) = r0;
            *reinterpret_cast<uint2*>(base + OFF_C + ro + 4096) = r1;
          } else {
            *reinterpret_cast<uint2*>(base + OFF_C + ro) = make_uint2(pk_bf16(acc0[0], acc0[1]), pk_bf16(acc0[2], acc0[3]));
            *reinterpret_cast<uint2*>(base + OFF_C + ro + 4096) =
                make_uint2(pk_bf16(acc1[0], acc1[1]), pk_bf16(acc1[2], acc1[3]));
          }
          if constexpr (CTN_DV_DBG & 4) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if constexpr (CTN_DV_DBG & 8) {   // per-tile, per-lane sums and their inputs (debug: p.R)
            v4u* dbg = reinterpret_cast<v4u*>(const_cast<void*>(p.R)) + ((((size_t)t * S + sl) * DV_NC + w) * 64 + lane) * 3;
            dbg[0] = v4u{__float_as_uint((s2[0][0] + s2[0][1]) + (s2[1][0] + s2[1][1])),
                         __float_as_uint((q2[0][0] + q2[0][1]) + (q2[1][0] + q2[1][1])), __float_as_uint(eal), 0u};
            dbg[1] = v4u{r0.x, r0.y, r1.x, r1.y};
            dbg[2] = v4u{__float_as_uint(e0.x), __float_as_uint(e0.y), __float_as_uint(e1.x), __float_as_uint(e1.y)};
          }
          if constexpr (NK == NORM_GLN) {
            const int m = t / tpu;
            if (m != run_m) {
              flush();
              run_s = run_q = 0.0;
              run_m = m;
            }
            run_s += (double)((s2[0][0] + s2[0][1]) + (s2[1][0] + s2[1][1]));
            run_q += (double)((q2[0][0] + q2[0][1]) + (q2[1][0] + q2[1][1]));
          } else {
            // per-row partial over this wave's 16 channels (the four lane groups), one
            // entry per row and wave; the memory waves add the 8 waves in order
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const float s = xsum_rows(s2[j][0] + s2[j][1]), ss = xsum_rows(q2[j][0] + q2[j][1]);
              if (lg == 0) *reinterpret_cast<float2*>(base + OFF_PT + ((16 * j + lr) * DV_NC + w) * 8) = make_float2(s, ss);
            }
          }
        }
        dv_signal(&fl_done[slot][w], gen);
        if (++slot == NSL) {
          slot = 0;
          ++gen;
        }
      }
    };
    if (t0 < t1) {
      if (eal <= 1.f) run(std::true_type{});
      else run(std::false_type{});
      if constexpr (NK == NORM_GLN) flush();
    }
    // dW2 partial of this workgroup: lane holds D[(wp*4+i)*16 + 4lg + e][n0 + (wn*4+j)*16 + lr]
    float* Dp = p.Dpart + (size_t)rr * KR * p.Nout;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + (wn * 4 + j) * 16 + lr;
#pragma unroll
        for (int e = 0; e < 4; ++e) Dp[(size_t)((wp * 4 + i) * 16 + 4 * lg + e) * p.Nout + n] = dacc[i][j][e];
      }
    return;
  }

  // ======================= memory waves =======================
  const int mw = wid - DV_NC;
  bf16raw* C = reinterpret_cast<bf16raw*>(p.C);
  // A: blocks f = 4*mw + u of the tile (row block f/8, k-block f%8): lane -> row, chunk
  //    such that the wave's 64 x 16 bytes fill the 1-KiB block contiguously
  // buffer loads: per-lane 32-bit byte offsets, the tile's row offset in an SGPR
  const rsrc_t rA = du_rsrc(p.A, rows * p.lda * 2), rD = du_rsrc(p.Bm, rows * p.ldb * 2);
  int arow[4];
  uint32_t aoff[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int f = 4 * mw + u, mb = f / KB, kb = f % KB;
    arow[u] = 16 * mb + ((lane & 15) ^ (((lane >> 4) & 1) * 12));
    aoff[u] = (uint32_t)(arow[u] * p.lda + (4 * kb + (lane >> 4)) * 8) * 2u;
  }
  // d / C: row dr = 8*mw + lane/8, chunks c = 8h + lane%8 (each 8 lanes: one 128-byte run)
  const int dr = 8 * mw + (lane >> 3);
  int cch[2], roff[2], boff[2];
  uint32_t doff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    cch[h] = 8 * h + (lane & 7);
    roff[h] = dv_roff(dr, cch[h]);
    boff[h] = (cch[h] >> 1) * DV_BST + dv_boff(dr, 8 * (cch[h] & 1));
    doff[h] = (uint32_t)(dr * p.ldb + n0 + 8 * cch[h]) * 2u;
  }
  const float bal = p.bop.alpha[0];

  v4u ra[PF][4], rd[PF][2];
  float2 rst[PF];
  // (the padded-frame zeroing of gy waits until write(): a select here would wait for
  // the load just issued)
  auto load = [&](int t, auto s) __attribute__((always_inline)) {
    constexpr int si = decltype(s)::value;
    const size_t r0 = (size_t)t * TM;
    const int sa = t * TM * p.lda * 2, sd = t * TM * p.ldb * 2;
#pragma unroll
    for (int u = 0; u < 4; ++u) ra[si][u] = __builtin_amdgcn_raw_buffer_load_b128(rA, aoff[u], sa, 0);
#pragma unroll
    for (int h = 0; h < 2; ++h) rd[si][h] = __builtin_amdgcn_raw_buffer_load_b128(rD, doff[h], sd, 0);
    // statistics with the tile's operands (a load issued at its point of use would be the
    // youngest in the wave's in-order vmcnt queue and drain the prefetch)
    rst[si] = p.bop.stats[NK == NORM_GLN ? (size_t)(t / tpu) : r0 + dr];
  };
  // store the C image (and the cLN per-row sums) of tile tc from slot `base`
  auto store_c = [&](int tc, const char* base) __attribute__((always_inline)) {
    const size_t r0 = (size_t)tc * TM;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const v4u v = *reinterpret_cast<const v4u*>(base + OFF_C + roff[h]);
      stg16(C + (r0 + dr) * p.ldc + n0 + 8 * cch[h], v);
    }
    if constexpr (NK == NORM_CLN) {
      if ((lane & 7) == 0) {
        double s = 0.0, ss = 0.0;
#pragma unroll
        for (int i = 0; i < DV_NC; ++i) {
          const float2 v = *reinterpret_cast<const float2*>(base + OFF_PT + (dr * DV_NC + i) * 8);
          s += (double)v.x;
          ss += (double)v.y;
        }
        p.grp_slab[(r0 + dr) * S + sl] = make_double2(s, ss);
      }
    }
  };
  auto write = [&](auto le1, int t, char* base, auto s) __attribute__((always_inline)) {
    constexpr bool LE1 = decltype(le1)::value;
    constexpr int si = decltype(s)::value;
    const int tk = (t * TM) % Kp;
#pragma unroll
    for (int u = 0; u < 4; ++u)   // padded frames: zero gy rows
      stg16(base + OFF_A + (4 * mw + u) * 1024 + lane * 16, tk + arow[u] < Kv ? ra[si][u] : v4u{0u, 0u, 0u, 0u});
    const float2 st = rst[si];
    const bool ok = NK == NORM_GLN || (t * TM) % Kp + dr < Kv;
    const f32x2_t m2 = {st.x, st.x};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      v4u v = rd[si][h];
      if constexpr (!(CTN_DV_DBG & 2)) stg16(base + OFF_R + roff[h], v);
      if constexpr (CTN_DV_DBG & 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      float gam[8], bet[8];
      *reinterpret_cast<float4*>(gam) = *reinterpret_cast<const float4*>(&sgb[0][8 * cch[h]]);
      *reinterpret_cast<float4*>(gam + 4) = *reinterpret_cast<const float4*>(&sgb[0][8 * cch[h] + 4]);
      *reinterpret_cast<float4*>(bet) = *reinterpret_cast<const float4*>(&sgb[1][8 * cch[h]]);
      *reinterpret_cast<float4*>(bet + 4) = *reinterpret_cast<const float4*>(&sgb[1][8 * cch[h] + 4]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f32x2_t x = {__uint_as_float(v[e] << 16), __uint_as_float(v[e] & 0xffff0000u)};
        x = prelu2<LE1>(x, bal);
        x = pfma(x - m2, f32x2_t{st.y * gam[2 * e], st.y * gam[2 * e + 1]}, f32x2_t{bet[2 * e], bet[2 * e + 1]});
        v[e] = pk_bf16(x[0], x[1]);
      }
      if constexpr (NK == NORM_CLN) v = ok ? v : v4u{0u, 0u, 0u, 0u};
      stg16(base + OFF_B + boff[h], v);
    }
    if constexpr (CTN_DV_DBG & 2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        v4u v = rd[si][h];
        asm volatile("" : "+v"(v));
        stg16(base + OFF_R + roff[h], v);
        if constexpr (CTN_DV_DBG & 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
    if constexpr (NK == NORM_CLN) {
      if ((lane & 7) == 0) *reinterpret_cast<float2*>(base + OFF_ST + dr * 8) = st;
    } else {
      if (mw == 0 && lane == 0) *reinterpret_cast<float2*>(base + OFF_ST) = st;
    }
  };

  auto run = [&](auto le1) __attribute__((always_inline)) {
    // Loads are issued unconditionally (tiles past the range clamped to its last one,
    // loaded and never used): the compiler's vmcnt bookkeeping then sees the same queue
    // on every path, and each wait leaves the later tiles' loads in flight.
    auto clampt = [&](int t) __attribute__((always_inline)) { return t < t1 ? t : t1 - 1; };
    static_for<PF>([&](auto s) { load(clampt(t0 + decltype(s)::value), s); });
    for (int tb = t0; tb < t1; tb += PF) {
      static_for<PF>([&](auto s) {
        const int t = tb + decltype(s)::value;
        if (t < t1) {
          const int k = t - t0, slot = k % NSL;
          const uint32_t gen = (uint32_t)(k / NSL) + 1;
          char* base = smem + slot * SLOT;
          if (k >= NSL) {   // the consumers are done with tile t - NSL: store its C image
            dv_wait<8>(fl_done[slot], gen - 1);
            store_c(t - NSL, base);
          }
          write(le1, t, base, s);
          dv_signal(&fl_full[slot][mw], gen);
        }
        load(clampt(t + PF), s);
      });
    }
    // the last NSL tiles' C images
    for (int t = (t1 - NSL > t0 ? t1 - NSL : t0); t < t1; ++t) {
      const int k = t - t0, slot = k % NSL;
      dv_wait<8>(fl_done[slot], (uint32_t)(k / NSL) + 1);
      store_c(t, smem + slot * SLOT);
    }
  };
  if (t0 < t1) {
    if (bal <= 1.f) run(std::true_type{});
    else run(std::false_type{});
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

bool gemm_dual_ws_eligible(const GemmDual& p) {
  if (!gemm_dual_ws_enabled()) return false;
  if (!(p.Kred == DV_KR && p.Nout % DV_NS == 0 && p.epi == EPI_NORM_BWD && p.bop.kind == OP_PRELU_NORM)) return false;
  if (p.norm != NORM_GLN && p.norm != NORM_CLN) return false;
  if (p.bop.norm != p.norm || p.stats != p.bop.stats || p.bop.fold.slab) return false;
  if (p.g.Kp % DV_TM || p.lda % 8 || p.ldb % 8 || p.ldc % 8 || p.ldw % 8) return false;
  if (p.g.rows() / DV_TM < 1) return false;
  const int S = p.Nout / DV_NS;
  return DV_GRID % S == 0;
}

int gemm_dual_ws_ranges(const GemmDual& p) {
  const long nt = p.g.rows() / DV_TM;
  const int want = DV_GRID / (p.Nout / DV_NS);
  return (int)(nt < want ? nt : want);
}

hipError_t launch_gemm_dual_ws(const GemmDual& p, hipStream_t s) {
  if (!gemm_dual_ws_eligible(p)) return hipErrorInvalidValue;
  const dim3 grid(gemm_dual_ws_ranges(p) * (p.Nout / DV_NS));
  if (p.norm == NORM_GLN)
    hipLaunchKernelGGL((gemm_dual_ws_kernel<NORM_GLN, 3, 3>), grid, dim3(DV_NT), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_dual_ws_kernel<NORM_CLN, 3, 3>), grid, dim3(DV_NT), 0, s, p);
  return hipGetLastError();
}

}  // namespace ctn
