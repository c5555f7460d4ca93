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
// Statistics: gLN partials are per (16-row tile, wave) -> Kp/16*8 parts per
// utterance; cLN partials are per (row, wave) -> 8 parts per row.  All
// reductions are fixed-order: results are bitwise reproducible.
#include <stdlib.h>

#include <type_traits>

#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int WS_WAVES = 8, WS_TM = 16, WS_GRID = 256;
constexpr int WSD_MB = 2;   // 16-row m-blocks per tile of the DMA-fed kernel

// Bound-finding experiments only (tools/microbench): bit 0 drops the output
// stores, bit 1 the A-tile loads, bit 2 the MFMAs, bit 3 the epilogue math.
#ifndef CTN_WS_EXP
#define CTN_WS_EXP 0
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


template <int OPK, int NK, int EPI, int NB, int KB, int WV, int MB>
__global__ __launch_bounds__(64 * WV) void gemm_ws_kernel(GemmRows p) {
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
  constexpr bool SWP = OPK == OP_PLAIN && WV == 8;
  __shared__ __attribute__((aligned(16))) char sA[2][TM * KR * 2];
  __shared__ float sgam[EPI == EPI_NORM_BWD ? NB * 16 * WV : 1];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int ntile = (int)(p.g.rows() / TM);
  const int t0 = (int)((long)ntile * blockIdx.x / gridDim.x), t1 = (int)((long)ntile * (blockIdx.x + 1) / gridDim.x);
  const int Kp = p.g.Kp, Kv = p.g.K;
  const bf16raw* A = reinterpret_cast<const bf16raw*>(p.A);
  const bf16raw* W = reinterpret_cast<const bf16raw*>(p.W);
  const int colbase = wid * 16 * NB + lg * NV;  // this lane's NV contiguous output channels

  // ---- resident weight: fragment (nb, kb), MFMA row lr -> output channel
  v4u wf[NB][KB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = wid * 16 * NB + (lr >> 2) * NV + nb * 4 + (lr & 3);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
      wf[nb][kb] = ldg16(W + (size_t)n * p.ldw + kb * 32 + lg * 8);
  }

  // ---- A staging: thread owns k-chunk kc (fixed) of rows rl0 + j*RSTEP
  const int kc = tid % CPR, rl0 = tid / CPR;
  float og[8], ob[8];
  if constexpr (OPK != OP_PLAIN) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      og[e] = p.aop.gamma[kc * 8 + e];
      ob[e] = p.aop.beta[kc * 8 + e];
    }
  }
  const float oal = (OPK == OP_PRELU_NORM) ? p.aop.alpha[0] : 0.f;
  // Loads are issued one tile ahead together with the statistics they need, so
  // that no wait inside an iteration has to drain the next tile's prefetch
  // (vmcnt retires loads in issue order).
  v4u ra[NA];
  float2 ast[NA];
  auto load_a = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int r = t * TM + rl0 + j * RSTEP;
      if constexpr (CTN_WS_EXP & 2) ra[j] = v4u{(uint32_t)r, 0u, 0u, 0u};
      else ra[j] = ldg16(A + (size_t)r * p.lda + kc * 8);
      if constexpr (OPK != OP_PLAIN) ast[j] = p.aop.stats[stat_index<NK>(r, Kp)];
    }
  };
  // ra -> LDS image of tile t (fragment (mb, kb) at (mb*KB + kb) KiB).  Rows of padded
  // frames are staged as zeros, so every output row of a padded frame is exactly 0
  // (+ the residual's zero row) and contributes nothing to any statistic.
  auto stage = [&](auto le1, int t, char* buf) __attribute__((always_inline)) {
    constexpr bool LE1 = decltype(le1)::value;
    const int tk = (t * TM) % Kp;   // frame index of the tile's first row (wave-uniform)
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      v4u v = ra[j];
      const int r = rl0 + j * RSTEP;
      if constexpr (OPK != OP_PLAIN) {
        const float2 st = ast[j];
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
      stg16(buf + (r >> 4) * KB * 1024 + ws_slot(r & 15, kc & 3, kc >> 2), v);
    }
  };

  // ---- epilogue constants
  constexpr bool HAS_R = EPI == EPI_RESID || EPI == EPI_NORM_BWD;
  constexpr bool HAS_STATS = EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD;
  const float eal = (EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD) ? p.alpha[0] : 0.f;
  if constexpr (EPI == EPI_NORM_BWD)
    for (int c = tid; c < NB * 16 * WV; c += NT) sgam[c] = p.gamma[c];
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
        for (int q = 0; q < Q; ++q) rn[mb][q] = ldg16(Rp + off + q * 8);
      }
      if constexpr (EPI == EPI_NORM_BWD) est[mb] = p.stats[stat_index<NK>(r, Kp)];
    }
  };

  auto mfma_tile = [&](const char* buf, f32x4_t (&acc)[MB][NB]) __attribute__((always_inline)) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const v4u b = ldg16(buf + mb * KB * 1024 + ws_slot(lr, lg, kb));
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          if constexpr (CTN_WS_EXP & 4) acc[mb][nb][kb & 3] += __uint_as_float(b[0] ^ wf[nb][kb][1]);
          else acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[nb][kb]),
                                                                     __builtin_bit_cast(bf16x8_t, b), acc[mb][nb], 0, 0, 0);
      }
    }
  };

  // epilogue of tile t from its accumulators: lane holds rows t*TM + mb*16 + lr,
  // channels colbase .. colbase+NV-1.  Branch-free (packed fp32 math).
  auto epilogue = [&](auto le1, int t, const f32x4_t (&acc)[MB][NB]) __attribute__((always_inline)) {
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
          const float4 g0 = *reinterpret_cast<const float4*>(&sgam[colbase + q * 8]);
          const float4 g1 = *reinterpret_cast<const float4*>(&sgam[colbase + q * 8 + 4]);
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
      {
        bf16raw* dst = Cp + (size_t)r * p.ldc + colbase;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const v4u o = {pk_bf16(v2[q * 4][0], v2[q * 4][1]), pk_bf16(v2[q * 4 + 1][0], v2[q * 4 + 1][1]),
                         pk_bf16(v2[q * 4 + 2][0], v2[q * 4 + 2][1]), pk_bf16(v2[q * 4 + 3][0], v2[q * 4 + 3][1])};
          if constexpr (!(CTN_WS_EXP & 1)) stg16(dst + q * 8, o);
        }
      }
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
          float s = s2[0] + s2[1], ss = q2[0] + q2[1];
          s += __shfl_xor(s, 16, 64); ss += __shfl_xor(ss, 16, 64);
          s += __shfl_xor(s, 32, 64); ss += __shfl_xor(ss, 32, 64);
          p.grp_slab[(size_t)r * WV + wid] = make_double2((double)s, (double)ss);
        }
      }
    }
    if constexpr (HAS_STATS && NK == NORM_GLN) {
      // one part per (tile, wave): slab index t*WV + wave = utterance-major
      // [M][Kp/TM*WV]; every lane stores the same value (no divergent store)
      const float s = wave_sum_dpp(gs2[0] + gs2[1]), ss = wave_sum_dpp(gq2[0] + gq2[1]);
      p.grp_slab[(size_t)t * WV + wid] = make_double2((double)s, (double)ss);
    }
  };

#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) ready(wf[nb][kb]);
  if constexpr (OPK != OP_PLAIN) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { ready(og[e]); ready(ob[e]); }
  }
  ready(oal);
  ready(eal);
  if (t0 >= t1) return;

  // Pipeline, one LDS-only barrier per tile; tile t+1 is staged into the other LDS
  // buffer (its last reader finished before this barrier) from registers loaded an
  // iteration earlier.  Every counted wait has the same memory operations behind it
  // on every iteration, so none drains the prefetch; out-of-range tiles are clamped
  // to the last one (never stored).  With SWP the MFMAs of tile t interleave with
  // the epilogue of tile t-1 (two accumulator sets).
  auto clampt = [&](int t) __attribute__((always_inline)) { return t < t1 ? t : t1 - 1; };
  // LE1 = (alpha <= 1) selects the exact two-instruction PReLU form once per kernel
  auto run = [&](auto le1) __attribute__((always_inline)) {
    if constexpr (!SWP) {
      f32x4_t acc[MB][NB];
      load_a(t0);
      load_r(t0);
      stage(le1, t0, sA[t0 & 1]);
      load_a(clampt(t0 + 1));
      for (int t = t0; t < t1; ++t) {
        lds_barrier();
        mfma_tile(sA[t & 1], acc);
        __builtin_amdgcn_sched_barrier(0);
        epilogue(le1, t, acc);
        load_r(clampt(t + 1));
        stage(le1, clampt(t + 1), sA[(t + 1) & 1]);
        load_a(clampt(t + 2));
      }
    } else {
      f32x4_t accP[MB][NB], accC[MB][NB];
      load_a(t0);
      stage(le1, t0, sA[t0 & 1]);
      load_a(clampt(t0 + 1));
      lds_barrier();
      mfma_tile(sA[t0 & 1], accP);
      load_r(t0);
      stage(le1, clampt(t0 + 1), sA[(t0 + 1) & 1]);
      load_a(clampt(t0 + 2));
      // unrolled by two so the two accumulator sets swap roles without copies
      auto step = [&](int t, f32x4_t (&cur)[MB][NB], f32x4_t (&prev)[MB][NB]) __attribute__((always_inline)) {
        lds_barrier();
        mfma_tile(sA[t & 1], cur);
        epilogue(le1, t - 1, prev);
        load_r(t);
        stage(le1, clampt(t + 1), sA[(t + 1) & 1]);
        load_a(clampt(t + 2));
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
  const float al_any = OPK == OP_PRELU_NORM ? oal : eal;
  if constexpr (OPK == OP_PRELU_NORM || HAS_STATS) {
    if (al_any <= 1.f) run(std::true_type{});
    else run(std::false_type{});
  } else {
    run(std::true_type{});
  }
}

// ===========================================================================
// Plain-operand variant fed entirely by LDS-DMA (global_load_lds_dwordx4):
// the A tile of every 16-row tile and the epilogue operands (R rows, forward
// statistics) are loaded D-1 tiles ahead straight into an LDS ring, so ~64 KB
// per CU are in flight (one tile of register prefetch is only 8-16 KB, far
// below the bytes x latency a CU needs to stream at HBM rate).  No VGPR-
// destination loads in the loop: every wait is an explicit counted vmcnt.
//   A ring slot : the MFMA fragment image of ws_slot (source-address swizzle;
//                 one 1-KB wave instruction = one k-block of 16 rows)
//   R ring slot : per wave, Q x 1 KB in epilogue-lane order (wave-private)
//   stat slot   : per wave, 64 dwords (wave-private)
// Rows of padded frames are zero in every plain operand on this path (the
// producers write them so), so their outputs are exactly 0 and contribute
// nothing to any statistic.
// The output channel order is permuted so that lane group g of store q owns
// channels q*32 + g*8 .. +7: each store instruction writes 64 contiguous bytes
// per frame row.
// ===========================================================================
CTN_DEV void glds16(const void* src, char* dst) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}
CTN_DEV void glds4(const void* src, char* dst) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)dst, 4, 0, 0);
}

// vmcnt wait for tile i of a workgroup's range: in steady state (i >= D-1)
// S + (D-2)(G+S) operations were issued after that tile's G loads; during the
// first D-1 tiles fewer (no stores yet).
template <int II, int D, int G, int S> CTN_DEV void wsd_wait(int i) {
  if constexpr (II >= D - 1) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S + (D - 2) * (G + S)) : "memory");
  } else {
    if (i == II) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2 - II) * G + II * (G + S)) : "memory");
    else wsd_wait<II + 1, D, G, S>(i);
  }
}

// Two workgroups of 4 waves per CU, each owning half of the output channels of
// the same tile range (the pair sits on one XCD, so the second A read hits L2):
// the two workgroups drift in phase, so one's epilogue VALU overlaps the
// other's MFMAs, which lock-step waves of a single 8-wave workgroup cannot do.
constexpr int WSD_WAVES = 4, WSD_THREADS = 64 * WSD_WAVES;

template <int NK, int EPI, int NB, int KB, int MB, int D>
__global__ __launch_bounds__(WSD_THREADS) void gemm_wsd_kernel(GemmRows p) {
  constexpr int WW = WSD_WAVES;
  constexpr int TMR = 16 * MB;                            // frame rows per tile
  constexpr int KR = KB * 32, NV = NB * 4, Q = NV / 8;
  constexpr int A_TILE = TMR * KR * 2;
  constexpr int GA = MB * KB / WW;                        // A fragments per wave per tile
  constexpr bool HAS_R = EPI == EPI_RESID || EPI == EPI_NORM_BWD;
  constexpr bool HAS_STATS = EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD;
  constexpr int GR = HAS_R ? MB * Q : 0, GS = EPI == EPI_NORM_BWD ? 1 : 0;
  constexpr int G = GA + GR + GS;                         // DMA instructions per wave per tile
  constexpr int S = MB * Q + (HAS_STATS ? (NK == NORM_GLN ? 1 : MB) : 0);   // stores per wave per tile
  constexpr int R_WAVE = MB * Q * 1024, ST_WAVE = 256;
  constexpr int OFF_R = D * A_TILE;
  constexpr int OFF_S = OFF_R + (HAS_R ? D * WW * R_WAVE : 0);
  constexpr int OFF_G = OFF_S + (GS ? D * WW * ST_WAVE : 0);
  constexpr int LDS = OFF_G + (EPI == EPI_NORM_BWD ? 2 * NB * 16 * WW * 4 : 0);
  static_assert(GA * WW == MB * KB, "fragments must split evenly over the waves");
  static_assert(MB <= 2, "stat slot holds 32 rows");
  static_assert(S + (D - 2) * (G + S) <= 63, "vmcnt range");
  static_assert(LDS <= 80 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(16))) char smem[LDS];   // one array: see §5.4 trap 4(a)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  // workgroup -> (tile range, channel half); pairs b, b+8 share an XCD
  const int nwg = gridDim.x, nrange = nwg / 2;
  int range, half;
  if (nrange % 8 == 0) {
    range = (blockIdx.x / 16) * 8 + blockIdx.x % 8;
    half = (blockIdx.x / 8) & 1;
  } else {
    range = blockIdx.x >> 1;
    half = blockIdx.x & 1;
  }
  const int ntile = (int)(p.g.rows() / TMR);
  const int t0 = (int)((long)ntile * range / nrange), t1 = (int)((long)ntile * (range + 1) / nrange);
  if (t0 >= t1) return;
  const int Kp = p.g.Kp;
  const bf16raw* A = reinterpret_cast<const bf16raw*>(p.A);
  const bf16raw* W = reinterpret_cast<const bf16raw*>(p.W);
  const bf16raw* Rp = reinterpret_cast<const bf16raw*>(p.R);
  bf16raw* Cp = reinterpret_cast<bf16raw*>(p.C);
  const float* stf = reinterpret_cast<const float*>(p.stats);
  const int wcol = (half * WW + wid) * 16 * NB;   // this wave's first output channel
  const int part = half * WW + wid;                // statistics part of this wave (of 8)
  auto colq = [&](int q) __attribute__((always_inline)) { return wcol + q * 32 + lg * 8; };

  // ---- resident weight: fragment (nb, kb); MFMA row lr -> permuted output channel
  v4u wf[NB][KB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = wcol + (nb >> 1) * 32 + (lr >> 2) * 8 + (nb & 1) * 4 + (lr & 3);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) wf[nb][kb] = ldg16(W + (size_t)n * p.ldw + kb * 32 + lg * 8);
  }
  const float eal = HAS_STATS ? p.alpha[0] : 0.f;
  if constexpr (EPI == EPI_NORM_BWD) {
    float* sg = reinterpret_cast<float*>(smem + OFF_G);
    for (int c = tid; c < 2 * NB * 16 * WW; c += WSD_THREADS) sg[c] = p.gamma[c];
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) ready(wf[nb][kb]);
  ready(eal);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // everything above has landed

  // ---- DMA issue of tile t into ring slot t % D (G instructions per wave)
  auto issue = [&](int t) __attribute__((always_inline)) {
    const int sl = t % D, row0 = t * TMR;
#pragma unroll
    for (int u = 0; u < GA; ++u) {
      const int f = wid * GA + u, mb = f / KB, kb = f % KB, h = (lg + 4 * (kb & 3)) & 15, r = lr ^ h;
      glds16(A + (size_t)(row0 + mb * 16 + r) * p.lda + kb * 32 + lg * 8, smem + sl * A_TILE + f * 1024);
    }
    if constexpr (HAS_R) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int q = 0; q < Q; ++q)
          glds16(Rp + (size_t)(row0 + mb * 16 + lr) * p.ldr + colq(q),
                 smem + OFF_R + (sl * WW + wid) * R_WAVE + (mb * Q + q) * 1024);
    }
    if constexpr (GS) {
      const int w = NK == NORM_GLN ? (row0 / Kp) * 2 + (lane & 1) : row0 * 2 + (lane & (2 * TMR - 1));
      glds4(stf + w, smem + OFF_S + (sl * WW + wid) * ST_WAVE);
    }
  };
  auto clampt = [&](int t) __attribute__((always_inline)) { return t < t1 ? t : t1 - 1; };

#pragma unroll
  for (int k = 0; k < D - 1; ++k) issue(clampt(t0 + k));

  // main loop; LE1 = (alpha <= 1) picks the exact two-instruction PReLU form once
  auto tile_loop = [&](auto le1) __attribute__((always_inline)) {
    constexpr bool LE1 = decltype(le1)::value;
    for (int t = t0; t < t1; ++t) {
      wsd_wait<0, D, G, S>(t - t0);
      lds_barrier();   // tile t's A image complete; slot (t-1)%D free for reuse
      issue(clampt(t + D - 1));
      const int sl = t % D;
      const char* abuf = smem + sl * A_TILE;
      f32x4_t acc[MB][NB];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
          const v4u b = ldg16(abuf + mb * KB * 1024 + ws_slot(lr, lg, kb));
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[nb][kb]),
                                                                  __builtin_bit_cast(bf16x8_t, b), acc[mb][nb], 0, 0, 0);
        }
      }
      // ---- epilogue (packed fp32): lane holds rows t*TMR + mb*16 + lr; value q*8+j of
      //      m-block mb is channel colq(q)+j
      const char* rbuf = smem + OFF_R + (sl * WW + wid) * R_WAVE;
      const float* sst = reinterpret_cast<const float*>(smem + OFF_S + (sl * WW + wid) * ST_WAVE);
      float sg_s = 0.f, sg_ss = 0.f;   // gLN: this wave's partial over the whole tile
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const int r = t * TMR + mb * 16 + lr;
        f32x2_t v2[NV / 2];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          v2[2 * nb] = f32x2_t{acc[mb][nb][0], acc[mb][nb][1]};
          v2[2 * nb + 1] = f32x2_t{acc[mb][nb][2], acc[mb][nb][3]};
        }
        f32x2_t s2 = {0.f, 0.f}, q2 = {0.f, 0.f};
        if constexpr (EPI == EPI_PRELU_STATS) {
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
            unpack_bf16x8(ldg16(rbuf + (mb * Q + q) * 1024 + lane * 16), f);
#pragma unroll
            for (int e = 0; e < 4; ++e) v2[q * 4 + e] += f32x2_t{f[2 * e], f[2 * e + 1]};
          }
        } else if constexpr (EPI == EPI_NORM_BWD) {
          const float2 st = NK == NORM_GLN ? make_float2(sst[0], sst[1])
                                           : make_float2(sst[2 * (mb * 16 + lr)], sst[2 * (mb * 16 + lr) + 1]);
          const f32x2_t rs = {st.y, st.y}, ms = {-st.x * st.y, -st.x * st.y};   // hat a = a*r - mean*r
          const float* sg = reinterpret_cast<const float*>(smem + OFF_G);
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            float f[8];
            unpack_bf16x8(ldg16(rbuf + (mb * Q + q) * 1024 + lane * 16), f);
            const float4 g0 = *reinterpret_cast<const float4*>(sg + colq(q));
            const float4 g1 = *reinterpret_cast<const float4*>(sg + colq(q) + 4);
            const f32x2_t gq[4] = {{g0.x, g0.y}, {g0.z, g0.w}, {g1.x, g1.y}, {g1.z, g1.w}};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const f32x2_t ah = pfma(prelu2<LE1>(f32x2_t{f[2 * e], f[2 * e + 1]}, eal), rs, ms);
              const f32x2_t ga = v2[q * 4 + e] * gq[e];
              s2 += ga;
              q2 = pfma(ga, ah, q2);
            }
          }
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const v4u o = {pk_bf16(v2[q * 4][0], v2[q * 4][1]), pk_bf16(v2[q * 4 + 1][0], v2[q * 4 + 1][1]),
                         pk_bf16(v2[q * 4 + 2][0], v2[q * 4 + 2][1]), pk_bf16(v2[q * 4 + 3][0], v2[q * 4 + 3][1])};
          stg16(Cp + (size_t)r * p.ldc + colq(q), o);
        }
        if constexpr (HAS_STATS) {
          float s = s2[0] + s2[1], ss = q2[0] + q2[1];
          if constexpr (NK == NORM_GLN) {
            sg_s += s;
            sg_ss += ss;
          } else {
            s += __shfl_xor(s, 16, 64); ss += __shfl_xor(ss, 16, 64);
            s += __shfl_xor(s, 32, 64); ss += __shfl_xor(ss, 32, 64);
            p.grp_slab[(size_t)r * WS_WAVES + part] = make_double2((double)s, (double)ss);
          }
        }
      }
      if constexpr (HAS_STATS && NK == NORM_GLN) {
        // one part per (tile, wave of 8); every lane stores the same value
        const float s = wave_sum_dpp(sg_s), ss = wave_sum_dpp(sg_ss);
        p.grp_slab[(size_t)t * WS_WAVES + part] = make_double2((double)s, (double)ss);
      }
    }
  };
  if constexpr (HAS_STATS) {
    if (eal <= 1.f) tile_loop(std::true_type{});
    else tile_loop(std::false_type{});
  } else {
    tile_loop(std::true_type{});
  }
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
// The LDS-DMA-fed split kernel is kept for experiments (CTN_WSD=1): at these
// shapes it measured no faster than the register-staged kernel.
static bool wsd_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("CTN_WSD");
    on = (e && atoi(e) == 1) ? 1 : 0;
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
  if (Nout == 512 && Kred == 256) { *nb = 4; *kb = 8; return true; }
  if (Nout == 256 && Kred == 512) { *nb = 2; *kb = 16; return true; }
  if (Nout == 256 && Kred == 256) { *nb = 2; *kb = 8; return true; }
  return false;
}

static bool ws_pair(int opk, int epi) {   // (operand op, epilogue) pairs used on the path
  return (opk == OP_PLAIN && (epi == EPI_PRELU_STATS || epi == EPI_NORM_BWD || epi == EPI_RESID || epi == EPI_STORE)) ||
         (opk == OP_PRELU_NORM && epi == EPI_RESID) || (opk == OP_NORM && epi == EPI_STORE);
}

bool gemm_ws_eligible(DType dt, const GemmRows& p) {
  int nb, kb;
  if (dt != BF16 || !ws_enabled() || !ws_shape(p.Nout, p.Kred, &nb, &kb) || !ws_pair(p.aop.kind, p.epi)) return false;
  if (p.g.Kp % WS_TM || p.lda % 8 || p.ldw % 8 || p.ldc % 8) return false;
  if ((p.epi == EPI_RESID || p.epi == EPI_NORM_BWD) && p.ldr % 8) return false;
  return true;
}

// frame rows per tile: the register-staged kernel (transformed operands) uses
// 16, the DMA-fed kernel (plain operands) 16*WSD_MB
static int ws_tile_rows(const GemmRows& p);
static int ws_waves(const GemmRows& p);

int gemm_ws_grid(const GemmRows& p) {
  const long nt = p.g.rows() / ws_tile_rows(p);
  return (int)(nt < WS_GRID ? nt : WS_GRID);
}

int gemm_ws_group_parts(const GemmRows& p) {
  return p.norm == NORM_GLN ? p.g.Kp / ws_tile_rows(p) * ws_waves(p) : ws_waves(p);
}

// Register-staged kernel configurations: (NB, KB, waves, m-blocks).  Nout = 512
// runs 16 waves of 32 channels (64 weight VGPRs per lane: 4 waves per SIMD, so one
// wave's latency hides behind another's work) on 32-row tiles; Nout = 256 runs
// 8 waves of 32 channels with a 128-register weight slice on 16-row tiles.
template <int OPK, int NK, int EPI>
static hipError_t ws_launch_shape(const GemmRows& p, hipStream_t s) {
  int nb = 0, kb = 0;
  ws_shape(p.Nout, p.Kred, &nb, &kb);
  const dim3 grid(gemm_ws_grid(p));
  if (nb == 4 && kb == 8) {
    if constexpr (EPI == EPI_NORM_BWD)   // its epilogue needs more than the 128 registers of 16 waves
      hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 4, 8, 8, 1>), grid, dim3(512), 0, s, p);
    else
      hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 2, 8, 16, 2>), grid, dim3(1024), 0, s, p);
  }
  else if (nb == 2 && kb == 16)
    hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 2, 16, 8, 1>), grid, dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 2, 8, 8, 1>), grid, dim3(512), 0, s, p);
  return hipGetLastError();
}

// DMA ring depth per workgroup: about 48 KB in flight (96 KB per CU), within
// the 80 KB LDS of one of the CU's two workgroups
template <int EPI, int NB, int KB> constexpr int wsd_depth() {
  constexpr bool HAS_R = EPI == EPI_RESID || EPI == EPI_NORM_BWD;
  constexpr int a = 16 * WSD_MB * KB * 32 * 2;
  constexpr int r = HAS_R ? 16 * WSD_MB * NB * 64 * 2 + (EPI == EPI_NORM_BWD ? 1024 : 0) : 0;
  constexpr int fixed = EPI == EPI_NORM_BWD ? 2 * NB * 64 * 4 : 0;
  constexpr int want = 1 + (48 * 1024 + a + r - 1) / (a + r);
  constexpr int fit = (80 * 1024 - fixed) / (a + r);
  constexpr int d = want < fit ? want : fit;
  return d > 8 ? 8 : d;
}

// per-wave shape of the split kernel: NB n-blocks of half of the channels
static bool wsd_shape(int Nout, int Kred, int* nb, int* kb) {
  if (Nout == 512 && Kred == 256) { *nb = 4; *kb = 8; return true; }
  if (Nout == 256 && Kred == 512) { *nb = 2; *kb = 16; return true; }
  if (Nout == 256 && Kred == 256) { *nb = 2; *kb = 8; return true; }
  return false;
}

template <int EPI> static int wsd_depth_rt(int nb, int kb) {
  return nb == 4 && kb == 8 ? wsd_depth<EPI, 4, 8>() : nb == 2 && kb == 16 ? wsd_depth<EPI, 2, 16>() : wsd_depth<EPI, 2, 8>();
}
static bool ws_wide(const GemmRows& p) {   // the 16-wave, 32-row configuration
  return p.Nout == 512 && p.Kred == 256 && p.epi != EPI_NORM_BWD && !(wsd_enabled() && p.aop.kind == OP_PLAIN);
}
static int ws_waves(const GemmRows& p) { return ws_wide(p) ? 16 : 8; }
static int ws_tile_rows(const GemmRows& p) {
  int nb = 0, kb = 0;
  if (!wsd_enabled() || p.aop.kind != OP_PLAIN || !wsd_shape(p.Nout, p.Kred, &nb, &kb))
    return ws_wide(p) ? 32 : WS_TM;
  int d = 0;
  switch (p.epi) {
    case EPI_PRELU_STATS: d = wsd_depth_rt<EPI_PRELU_STATS>(nb, kb); break;
    case EPI_NORM_BWD: d = wsd_depth_rt<EPI_NORM_BWD>(nb, kb); break;
    case EPI_RESID: d = wsd_depth_rt<EPI_RESID>(nb, kb); break;
    default: d = wsd_depth_rt<EPI_STORE>(nb, kb); break;
  }
  return d >= 2 ? 16 * WSD_MB : WS_TM;
}

template <int NK, int EPI>
static hipError_t wsd_launch_shape(const GemmRows& p, hipStream_t s) {
  int nb = 0, kb = 0;
  wsd_shape(p.Nout, p.Kred, &nb, &kb);
  const dim3 grid(2 * gemm_ws_grid(p)), block(WSD_THREADS);
  // shapes whose ring would not fit two workgroups per CU use the register-staged kernel
#define CTN_WSD_CASE(NB_, KB_)                                                                      \
  if constexpr (wsd_depth<EPI, NB_, KB_>() >= 2)                                                   \
    hipLaunchKernelGGL((gemm_wsd_kernel<NK, EPI, NB_, KB_, WSD_MB, wsd_depth<EPI, NB_, KB_>()>), grid, \
                       block, 0, s, p);                                                           \
  else                                                                                             \
    return ws_launch_shape<OP_PLAIN, NK, EPI>(p, s);
  if (nb == 4 && kb == 8) {
    CTN_WSD_CASE(4, 8)
  } else if (nb == 2 && kb == 16) {
    CTN_WSD_CASE(2, 16)
  } else {
    CTN_WSD_CASE(2, 8)
  }
#undef CTN_WSD_CASE
  return hipGetLastError();
}

template <int NK>
static hipError_t ws_launch_nk(const GemmRows& p, hipStream_t s) {
  if (p.aop.kind == OP_PRELU_NORM) return ws_launch_shape<OP_PRELU_NORM, NK, EPI_RESID>(p, s);
  if (p.aop.kind == OP_NORM) return ws_launch_shape<OP_NORM, NK, EPI_STORE>(p, s);
  if (wsd_enabled()) {
    switch (p.epi) {
      case EPI_PRELU_STATS: return wsd_launch_shape<NK, EPI_PRELU_STATS>(p, s);
      case EPI_NORM_BWD: return wsd_launch_shape<NK, EPI_NORM_BWD>(p, s);
      case EPI_RESID: return wsd_launch_shape<NORM_GLN, EPI_RESID>(p, s);
      default: return wsd_launch_shape<NORM_GLN, EPI_STORE>(p, s);
    }
  }
  switch (p.epi) {
    case EPI_PRELU_STATS: return ws_launch_shape<OP_PLAIN, NK, EPI_PRELU_STATS>(p, s);
    case EPI_NORM_BWD: return ws_launch_shape<OP_PLAIN, NK, EPI_NORM_BWD>(p, s);
    case EPI_RESID: return ws_launch_shape<OP_PLAIN, NORM_GLN, EPI_RESID>(p, s);
    default: return ws_launch_shape<OP_PLAIN, NORM_GLN, EPI_STORE>(p, s);
  }
}

hipError_t launch_gemm_ws(const GemmRows& p, hipStream_t s) {
  const int nk = p.aop.kind != OP_PLAIN ? p.aop.norm : p.norm;
  return nk == NORM_GLN ? ws_launch_nk<NORM_GLN>(p, s) : ws_launch_nk<NORM_CLN>(p, s);
}

}  // namespace ctn
