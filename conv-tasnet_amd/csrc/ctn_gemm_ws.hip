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

#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int WS_WAVES = 8, WS_THREADS = 64 * WS_WAVES, WS_TM = 16, WS_GRID = 256;

// LDS byte offset of the 16-byte piece (frame row lr, k-chunk lg) of k-block kb
// in fragment order: ds_read_b128 groups and ds_write_b128 groups both hit
// distinct banks.
CTN_DEV int ws_slot(int lr, int lg, int kb) { return (kb * 64 + lg * 16 + (lr ^ (lg + 4 * (kb & 3)))) << 4; }

// Force a register's load to complete here (an inline-asm use makes the compiler
// wait for it once, so no counted wait for it is left inside the tile loop,
// where it would also drain the prefetch issued behind it).
CTN_DEV void ready(const v4u& v) { asm volatile("" ::"v"(v)); }
CTN_DEV void ready(float v) { asm volatile("" ::"v"(v)); }


template <int OPK, int NK, int EPI, int NB, int KB>
__global__ __launch_bounds__(WS_THREADS) void gemm_ws_kernel(GemmRows p) {
  constexpr int KR = KB * 32;                  // reduction length
  constexpr int CPR = KR / 8;                  // 16-byte chunks per A row
  constexpr int NA = WS_TM * CPR / WS_THREADS; // A chunks per thread per tile
  constexpr int RSTEP = WS_THREADS / CPR;      // rows between a thread's chunks
  constexpr int NV = NB * 4;                   // output channels per lane
  static_assert(NA >= 1 && NA * WS_THREADS == WS_TM * CPR, "tile/thread mismatch");
  __shared__ __attribute__((aligned(16))) char sA[2][WS_TM * KR * 2];
  __shared__ float sgam[EPI == EPI_NORM_BWD ? NB * 16 * WS_WAVES : 1];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int ntile = (int)(p.g.rows() / WS_TM);
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
      const int r = t * WS_TM + rl0 + j * RSTEP;
      ra[j] = ldg16(A + (size_t)r * p.lda + kc * 8);
      if constexpr (OPK != OP_PLAIN) ast[j] = p.aop.stats[stat_index<NK>(r, Kp)];
    }
  };
  auto stage = [&](char* buf) __attribute__((always_inline)) {   // ra -> LDS image
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      v4u v = ra[j];
      if constexpr (OPK != OP_PLAIN) {
        const float2 st = ast[j];
        float f[8];
        unpack_bf16x8(v, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = f[e];
          if constexpr (OPK == OP_PRELU_NORM) x = prelu(x, oal);
          f[e] = (x - st.x) * (st.y * og[e]) + ob[e];
        }
        v = pack_bf16x8v(f);
      }
      const int r = rl0 + j * RSTEP;
      stg16(buf + ws_slot(r, kc & 3, kc >> 2), v);
    }
  };

  // ---- epilogue constants
  constexpr bool HAS_R = EPI == EPI_RESID || EPI == EPI_NORM_BWD;
  constexpr bool HAS_STATS = EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD;
  const float eal = (EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD) ? p.alpha[0] : 0.f;
  if constexpr (EPI == EPI_NORM_BWD)
    for (int c = tid; c < NB * 16 * WS_WAVES; c += WS_THREADS) sgam[c] = p.gamma[c];
  const bf16raw* Rp = reinterpret_cast<const bf16raw*>(p.R);
  bf16raw* Cp = reinterpret_cast<bf16raw*>(p.C);
  v4u rn[NV / 8];   // epilogue operand of the current tile (loaded one tile ahead)
  float2 est = make_float2(0.f, 0.f);   // EPI_NORM_BWD forward statistics of the lane's row
  auto load_r = [&](int t) __attribute__((always_inline)) {
    const int r = t * WS_TM + lr;
    if constexpr (HAS_R) {
      const size_t off = (size_t)r * p.ldr + colbase;
#pragma unroll
      for (int q = 0; q < NV / 8; ++q) rn[q] = ldg16(Rp + off + q * 8);
    }
    if constexpr (EPI == EPI_NORM_BWD) est = p.stats[stat_index<NK>(r, Kp)];
  };

  // Pipeline (one barrier per tile): tile t+1 is staged into the other LDS
  // buffer right after tile t's epilogue, from registers loaded one tile
  // earlier; every wait therefore has the same VMEM operations behind it on the
  // first and on later iterations, so the compiler's counted waits never drain
  // the prefetch.  The last tile re-reads itself: unconditional loads keep the
  // staging registers out of scratch.
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
  if (t0 < t1) {
    load_a(t0);
    load_r(t0);
    stage(sA[t0 & 1]);
    load_a(t0 + 1 < t1 ? t0 + 1 : t0);
  }
  for (int t = t0; t < t1; ++t) {
    const int tn = t + 1 < t1 ? t + 1 : t;
    const char* buf = sA[t & 1];
    lds_barrier();

    f32x4_t acc[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const v4u b = ldg16(buf + ws_slot(lr, lg, kb));
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[nb][kb]),
                                                          __builtin_bit_cast(bf16x8_t, b), acc[nb], 0, 0, 0);
    }

    // keep the epilogue (and its waits on the prefetched operand) after the MFMAs
    __builtin_amdgcn_sched_barrier(0);
    // ---- epilogue: lane holds row t*16+lr, channels colbase .. colbase+NV-1
    const int r = t * WS_TM + lr;
    const bool valid = (r % Kp) < Kv;
    float v[NV];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[nb * 4 + e] = acc[nb][e];
    float s = 0.f, ss = 0.f;
    if constexpr (EPI == EPI_STORE) {
#pragma unroll
      for (int c = 0; c < NV; ++c) v[c] = valid ? v[c] : 0.f;
    } else if constexpr (EPI == EPI_PRELU_STATS) {
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        const float a2 = valid ? prelu(v[c], eal) : 0.f;
        s += a2;
        ss += a2 * a2;
        v[c] = valid ? v[c] : 0.f;
      }
    } else if constexpr (EPI == EPI_RESID) {
#pragma unroll
      for (int q = 0; q < NV / 8; ++q) {
        float f[8];
        unpack_bf16x8(rn[q], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[q * 8 + e] = valid ? v[q * 8 + e] + f[e] : 0.f;
      }
    } else if constexpr (EPI == EPI_NORM_BWD) {
      const float2 st = est;
#pragma unroll
      for (int q = 0; q < NV / 8; ++q) {
        float f[8];
        unpack_bf16x8(rn[q], f);
        const float4 g0 = *reinterpret_cast<const float4*>(&sgam[colbase + q * 8]);
        const float4 g1 = *reinterpret_cast<const float4*>(&sgam[colbase + q * 8 + 4]);
        const float gq[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int c = q * 8 + e;
          const float ah = valid ? (prelu(f[e], eal) - st.x) * st.y : 0.f;
          const float gn = valid ? v[c] : 0.f;
          const float ga = gn * gq[e];
          s += ga;
          ss += ga * ah;
          v[c] = gn;
        }
      }
    }
    {
      bf16raw* dst = Cp + (size_t)r * p.ldc + colbase;
#pragma unroll
      for (int q = 0; q < NV / 8; ++q) stg16(dst + q * 8, pack_bf16x8v(v + q * 8));
    }
    if constexpr (HAS_STATS) {
      if constexpr (NK == NORM_GLN) {
        // one part per (16-row tile, wave): slab index t*8 + wave = utterance-major
        // [M][Kp/16*8]; every lane stores the same value (no divergent store)
        s = wave_sum(s);
        ss = wave_sum(ss);
        p.grp_slab[(size_t)t * WS_WAVES + wid] = make_double2((double)s, (double)ss);
      } else {
        // per-row partial over this wave's 16*NB channels: reduce across the 4 lane
        // groups; all four groups store the same value (no divergent store)
        s += __shfl_xor(s, 16, 64); ss += __shfl_xor(ss, 16, 64);
        s += __shfl_xor(s, 32, 64); ss += __shfl_xor(ss, 32, 64);
        p.grp_slab[(size_t)r * WS_WAVES + wid] = make_double2((double)s, (double)ss);
      }
    }
    load_r(tn);
    stage(sA[(t + 1) & 1]);
    load_a(tn + 1 < t1 ? tn + 1 : tn);
  }
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
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

int gemm_ws_grid(const GemmRows& p) {
  const long nt = p.g.rows() / WS_TM;
  return (int)(nt < WS_GRID ? nt : WS_GRID);
}

int gemm_ws_group_parts(const GemmRows& p) {
  return p.norm == NORM_GLN ? p.g.Kp / WS_TM * WS_WAVES : WS_WAVES;
}

template <int OPK, int NK, int EPI>
static hipError_t ws_launch_shape(const GemmRows& p, hipStream_t s) {
  int nb = 0, kb = 0;
  ws_shape(p.Nout, p.Kred, &nb, &kb);
  const dim3 grid(gemm_ws_grid(p)), block(WS_THREADS);
  if (nb == 4 && kb == 8) hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 4, 8>), grid, block, 0, s, p);
  else if (nb == 2 && kb == 16) hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 2, 16>), grid, block, 0, s, p);
  else hipLaunchKernelGGL((gemm_ws_kernel<OPK, NK, EPI, 2, 8>), grid, block, 0, s, p);
  return hipGetLastError();
}

template <int NK>
static hipError_t ws_launch_nk(const GemmRows& p, hipStream_t s) {
  if (p.aop.kind == OP_PRELU_NORM) return ws_launch_shape<OP_PRELU_NORM, NK, EPI_RESID>(p, s);
  if (p.aop.kind == OP_NORM) return ws_launch_shape<OP_NORM, NK, EPI_STORE>(p, s);
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
