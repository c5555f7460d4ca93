// MFMA GEMMs of the Conv-TasNet path (gfx950).
//
// gemm_rows : the 1x1 convolutions (conv_tasnet.py:169,185,217,256) and their
//             data gradients.  C[r][n] = sum_k op(A[r][k]) * W[n][k] over frame
//             rows r of all utterances at once (weights are shared), fused
//             with the ops around each 1x1 conv: norm-apply / PReLU on the A
//             operand while it is staged into LDS, PReLU-statistics,
//             residual add or norm-backward in the epilogue.
// gemm_cols : weight gradients dW[p][q] = sum_r op(A[r][p]) * op(B[r][q]); the
//             reduction runs over frame rows, split in chunks whose fp32
//             partial tiles are summed by slab_reduce (deterministic order).
//
// MFMA: bf16 storage -> v_mfma_f32_16x16x32_bf16; fp32 storage (parity mode)
// -> v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulate).
#include <stdlib.h>

#include <type_traits>

#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// operand transform (applied per 16-byte chunk while staging)
// ---------------------------------------------------------------------------
template <typename T> struct Chunk;
template <> struct Chunk<float> {
  static constexpr int E = 4;
  static CTN_DEV void unpack(const u128& v, float* f) {
    f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y);
    f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
  }
  static CTN_DEV u128 pack(const float* f) {
    u128 v; v.x = __float_as_uint(f[0]); v.y = __float_as_uint(f[1]);
    v.z = __float_as_uint(f[2]); v.w = __float_as_uint(f[3]); return v;
  }
};
template <> struct Chunk<bf16raw> {
  static constexpr int E = 8;
  static CTN_DEV void unpack(const u128& v, float* f) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static CTN_DEV u128 pack(const float* f) { return pack_bf16x8(f); }
};

CTN_DEV u128 zero128() { u128 z; z.x = z.y = z.z = z.w = 0u; return z; }

// XCD-aware bijective remap (cdna_hip_programming.md §5 T1): workgroups are
// dealt round-robin over the 8 XCDs, so hardware id b runs on XCD b % 8; give
// each XCD a contiguous range of logical tile ids so neighbouring tiles (which
// share an operand panel) hit the same L2.  Speed only — correctness never
// depends on placement.
CTN_DEV int xcd_remap(int b, int n) {
  const int x = b % 8, q = n / 8, r = n % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// op(v) for E consecutive channels starting at c0 of frame row `row`
template <typename T, int OPK, int NK>
CTN_DEV u128 apply_op(u128 v, int row, int c0, int Kp, const RowOp& op) {
  if constexpr (OPK == OP_PLAIN) {
    return v;
  } else {
    constexpr int E = Chunk<T>::E;
    float f[E];
    Chunk<T>::unpack(v, f);
    const float2 st = op.stats[stat_index<NK>(row, Kp)];
    const float al = (OPK == OP_PRELU_NORM) ? op.alpha[0] : 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float x = f[e];
      if constexpr (OPK == OP_PRELU_NORM) x = prelu(x, al);
      f[e] = (x - st.x) * st.y * op.gamma[c0 + e] + op.beta[c0 + e];
    }
    return Chunk<T>::pack(f);
  }
}

// op(v) on a 16-byte register vector (bf16 x8 or f32 x4)
template <typename T, int OPK>
CTN_DEV v4u apply_op_v(v4u v, float2 st, const float* g, const float* b, float al) {
  constexpr int E = Chunk<T>::E;
  float f[E];
  if constexpr (E == 8) {
    unpack_bf16x8(v, f);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = __uint_as_float(v[e]);
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float x = f[e];
    if constexpr (OPK == OP_PRELU_NORM) x = prelu(x, al);
    f[e] = (x - st.x) * (st.y * g[e]) + b[e];
  }
  if constexpr (E == 8) {
    return pack_bf16x8v(f);
  } else {
    v4u r;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = __float_as_uint(f[e]);
    return r;
  }
}

// ===========================================================================
// gemm_rows
// ===========================================================================
constexpr int RBN = 128, RPITCH = 128;   // bytes per LDS row; 16-B slots XOR-swizzled by (row & 7)

// LDS byte offset of 16-byte slot `kc` (0..7) of tile row `r`: conflict-free for the
// ds_read_b128 fragment reads (16 rows x one slot) and the row-wise staging writes
CTN_DEV int rslot(int r, int kc) { return r * RPITCH + ((kc ^ (r & 7)) << 4); }

// Tile RBM frame rows x RBN output channels, 4 waves (2 x 2), each wave
// (RBM/2) x 64 of 16x16 MFMA tiles; k-steps of 128 bytes, register-staged with
// the A-operand transform applied on the way into LDS.
constexpr int CPITCH = RBN + 4;   // floats per row of the fp32 C staging tile (epilogue)

template <int RBM> struct RowsLds {
  static constexpr int tiles = (RBM + RBN) * RPITCH;
  static constexpr int ctile = RBM * CPITCH * 4;
  static constexpr int bytes = (tiles > ctile ? tiles : ctile) + 4096;
};

template <typename T, int OPK, int NK, int EPI, int RBM>
__global__ __launch_bounds__(256) void gemm_rows_kernel(GemmRows p) {
  __shared__ __attribute__((aligned(16))) char smem[RowsLds<RBM>::bytes];
  constexpr int JT = RBM / 32;   // 16-row MFMA tiles per wave
  constexpr int E = Chunk<T>::E;              // elements per 16 B
  constexpr int BK = 128 / sizeof(T);         // elements per k-step (128 B per row)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int lr = lane & 15, lg = lane >> 4;

  const int ncol = (p.Nout + RBN - 1) / RBN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int coltile = bid % ncol, rowtile = bid / ncol;
  const int row0 = rowtile * RBM, col0 = coltile * RBN;

  const T* A = reinterpret_cast<const T*>(p.A);
  const T* W = reinterpret_cast<const T*>(p.W);
  char* sA = smem;
  char* sW = smem + RBM * RPITCH;
  constexpr int NA = RBM / 32;   // A chunks (16 B) per thread per k-step

  u128 ra[NA], rw[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int c = tid + 256 * i, r = c >> 3, kc = c & 7;
      const int k = k0 + kc * E;
      ra[i] = zero128();
      if (k < p.Kred) ra[i] = *reinterpret_cast<const u128*>(A + (size_t)(row0 + r) * p.lda + k);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i, r = c >> 3, kc = c & 7;
      const int k = k0 + kc * E;
      rw[i] = zero128();
      if (k < p.Kred && col0 + r < p.Nout) rw[i] = *reinterpret_cast<const u128*>(W + (size_t)(col0 + r) * p.ldw + k);
    }
  };
  auto swrite = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int c = tid + 256 * i, r = c >> 3, kc = c & 7;
      const int k = k0 + kc * E;
      u128 va = ra[i];
      if constexpr (OPK != OP_PLAIN)
        if (k < p.Kred) va = apply_op<T, OPK, NK>(va, row0 + r, k, p.g.Kp, p.aop);
      *reinterpret_cast<u128*>(sA + rslot(r, kc)) = va;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i, r = c >> 3, kc = c & 7;
      *reinterpret_cast<u128*>(sW + rslot(r, kc)) = rw[i];
    }
  };

  f32x4_t acc[4][JT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // epilogue operand (residual / pre-activation) prefetched now, consumed after the k loop:
  // thread owns output chunks c = tid + 256*i -> row c/16, 8 columns (c%16)*8
  constexpr int NC = RBM * RBN / 8 / 256;
  const T* Rp = reinterpret_cast<const T*>(p.R);
  Raw8<T> rpre[NC];
  if constexpr (EPI == EPI_RESID || EPI == EPI_NORM_BWD) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = tid + 256 * i, r = c >> 4, n = col0 + (c & 15) * 8;
      if (n < p.Nout) rpre[i].load(Rp + (size_t)(row0 + r) * p.ldr + n);
    }
  }

  const int nk = (p.Kred + BK - 1) / BK;
  gload(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();
    swrite(kt * BK);
    __syncthreads();
    if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u128 wf[4], af[JT];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        wf[i] = *reinterpret_cast<const u128*>(sW + rslot(wc * 64 + i * 16 + lr, kk * 4 + lg));
#pragma unroll
      for (int j = 0; j < JT; ++j)
        af[j] = *reinterpret_cast<const u128*>(sA + rslot(wr * (RBM / 2) + j * 16 + lr, kk * 4 + lg));
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < JT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8_t, wf[i]), __builtin_bit_cast(bf16x8_t, af[j]), acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t wv = s == 0 ? wf[i].x : s == 1 ? wf[i].y : s == 2 ? wf[i].z : wf[i].w;
#pragma unroll
            for (int j = 0; j < JT; ++j) {
              const uint32_t av = s == 0 ? af[j].x : s == 1 ? af[j].y : s == 2 ? af[j].z : af[j].w;
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(wv), __uint_as_float(av),
                                                               acc[i][j], 0, 0, 0);
            }
          }
        }
      }
    }
  }

  // ------------------------------------------------------------------ epilogue
  // 1) accumulators -> fp32 C tile in LDS (lane holds rows wr*(RBM/2)+j*16+lr, cols wc*64+i*16+lg*4..+3)
  __syncthreads();
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int j = 0; j < JT; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wr * (RBM / 2) + j * 16 + lr, n = wc * 64 + i * 16 + lg * 4;
      *reinterpret_cast<f32x4_t*>(Cs + r * CPITCH + n) = acc[i][j];
    }
  __syncthreads();
  // 2) row-contiguous processing: 16 threads x 8 columns cover one 128-column tile row
  T* Cp = reinterpret_cast<T*>(p.C);
  const int K = p.g.K, Kp = p.g.Kp;
  const float al = (EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD) ? p.alpha[0] : 0.f;
  const int cgi = tid & 15;                  // this thread's 8-column group (same for all its chunks)
  float ts = 0.f, tss = 0.f;
  float gam[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    gam[e] = 0.f;
    if constexpr (EPI == EPI_NORM_BWD)
      if (col0 + cgi * 8 + e < p.Nout) gam[e] = p.gamma[col0 + cgi * 8 + e];
  }
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = tid + 256 * i, rl = c >> 4, r = row0 + rl, n = col0 + cgi * 8;
    const bool valid = (r % Kp) < K && n < p.Nout;   // columns past Nout: no output, no statistics
    float v[8];
    {
      const f32x4_t lo = *reinterpret_cast<const f32x4_t*>(Cs + rl * CPITCH + cgi * 8);
      const f32x4_t hi = *reinterpret_cast<const f32x4_t*>(Cs + rl * CPITCH + cgi * 8 + 4);
      v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
      v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    }
    float s = 0.f, ss = 0.f;
    if constexpr (EPI == EPI_STORE) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = valid ? v[e] : 0.f;
    } else if constexpr (EPI == EPI_PRELU_STATS) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float a2 = valid ? prelu(v[e], al) : 0.f;
        s += a2;
        ss += a2 * a2;
        v[e] = valid ? v[e] : 0.f;
      }
    } else if constexpr (EPI == EPI_RESID) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = valid ? v[e] + rpre[i][e] : 0.f;   // select: garbage never propagates
    } else if constexpr (EPI == EPI_NORM_BWD) {
      const float2 st = p.stats[stat_index<NK>(r, Kp)];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float ah = valid ? (prelu(rpre[i][e], al) - st.x) * st.y : 0.f;
        const float gn = valid ? v[e] : 0.f;
        const float ga = gn * gam[e];
        s += ga;
        ss += ga * ah;
        v[e] = gn;
      }
    }
    if (n < p.Nout) Vec8<T>::store(Cp + (size_t)r * p.ldc + n, v);
    if constexpr (EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD) {
      if constexpr (NK == NORM_GLN) {
        ts += s;
        tss += ss;
      } else {
        // per-row partial over this tile's 128 columns: the 16 lanes of one row
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) { s += __shfl_xor(s, o, 64); ss += __shfl_xor(ss, o, 64); }
        if (cgi == 0) p.grp_slab[(size_t)r * ncol + coltile] = make_double2((double)s, (double)ss);
      }
    }
  }
  if constexpr (EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD) {
    if constexpr (NK == NORM_GLN) {
      __syncthreads();
      double v2[2] = {(double)ts, (double)tss};
      double* red = reinterpret_cast<double*>(smem + RowsLds<RBM>::bytes - 4096);
      block_sum_d<2>(v2, red);
      if (tid == 0) {
        const int tpu = (Kp / RBM) * ncol;    // tiles per utterance
        const int m = row0 / Kp;
        const int tiu = ((row0 % Kp) / RBM) * ncol + coltile;
        p.grp_slab[(size_t)m * tpu + tiu] = make_double2(v2[0], v2[1]);
      }
    }
  }
}

// rows per tile: 64 (more workgroups per CU to hide load latency on the short
// k loops of this model) unless CTN_GEMM_BM=128 is set (A/B experiments)
static int rows_bm() {
  static int bm = 0;
  if (!bm) {
    const char* e = getenv("CTN_GEMM_BM");
    bm = (e && atoi(e) == 128) ? 128 : 64;
  }
  return bm;
}

int gemm_rows_tiles_per_group(DType dt, const GemmRows& p) {
  if (gemm_ws_eligible(dt, p)) return gemm_ws_group_parts(p);
  const int ncol = (p.Nout + RBN - 1) / RBN;
  return p.norm == NORM_GLN ? (p.g.Kp / rows_bm()) * ncol : ncol;
}

StatFold gemm_rows_stat_fold(DType dt, const GemmRows& p, const double2* slab, double cnt, float eps, int mode,
                             float2* out) {
  StatFold f;
  f.slab = slab;
  f.parts = gemm_rows_tiles_per_group(dt, p);
  f.cnt = cnt;
  f.eps = eps;
  f.mode = mode;
  f.out = out;
  if (gemm_ws_eligible(dt, p) && p.norm == NORM_GLN) f.ws = gemm_ws_runs(p);
  return f;
}

template <typename T, int OPK, int NK, int EPI>
static hipError_t launch_rows_t(const GemmRows& p, hipStream_t s) {
  const int ncol = (p.Nout + RBN - 1) / RBN;
  const int bm = rows_bm();
  const int nrow = (int)(p.g.rows() / bm);
  if (bm == 128) hipLaunchKernelGGL((gemm_rows_kernel<T, OPK, NK, EPI, 128>), dim3(nrow * ncol), dim3(256), 0, s, p);
  else hipLaunchKernelGGL((gemm_rows_kernel<T, OPK, NK, EPI, 64>), dim3(nrow * ncol), dim3(256), 0, s, p);
  return hipGetLastError();
}

template <typename T, int OPK, int NK>
static hipError_t dispatch_epi(const GemmRows& p, hipStream_t s) {
  switch (p.epi) {
    case EPI_STORE: return launch_rows_t<T, OPK, NK, EPI_STORE>(p, s);
    case EPI_PRELU_STATS: return launch_rows_t<T, OPK, NK, EPI_PRELU_STATS>(p, s);
    case EPI_RESID: return launch_rows_t<T, OPK, NK, EPI_RESID>(p, s);
    case EPI_NORM_BWD: return launch_rows_t<T, OPK, NK, EPI_NORM_BWD>(p, s);
  }
  return hipErrorInvalidValue;
}

template <typename T>
static hipError_t dispatch_rows(const GemmRows& p, hipStream_t s) {
  // NK governs both the A-operand statistics and the epilogue statistics; the
  // two always agree on this path (one norm_type per model).
  const int nk = p.aop.kind != OP_PLAIN ? p.aop.norm : p.norm;
  if (p.aop.kind != OP_PLAIN && p.epi != EPI_STORE && p.epi != EPI_RESID && p.aop.norm != p.norm)
    return hipErrorInvalidValue;
#define CTN_ROWS_NK(OPK)                                                     \
  return nk == NORM_GLN ? dispatch_epi<T, OPK, NORM_GLN>(p, s)               \
                        : dispatch_epi<T, OPK, NORM_CLN>(p, s);
  switch (p.aop.kind) {
    case OP_PLAIN: CTN_ROWS_NK(OP_PLAIN)
    case OP_NORM: CTN_ROWS_NK(OP_NORM)
    case OP_PRELU_NORM: CTN_ROWS_NK(OP_PRELU_NORM)
  }
#undef CTN_ROWS_NK
  return hipErrorInvalidValue;
}

hipError_t launch_gemm_rows(DType dt, const GemmRows& p, hipStream_t s) {
  if (p.g.Kp % 128 != 0 || p.Kred % 8 != 0 || p.Nout % 8 != 0) return hipErrorInvalidValue;
  if (gemm_ws_eligible(dt, p)) return launch_gemm_ws(p, s);
  return dt == BF16 ? dispatch_rows<bf16raw>(p, s) : dispatch_rows<float>(p, s);
}

// ===========================================================================
// gemm_cols (weight gradients)
// ===========================================================================
constexpr int CBP = 128, CBQ = 128, CKR = 32;   // tile p x q, rows per k-step

// LDS byte offset of element (row, col) of a [CKR][128] staging tile.  bf16: the
// 288-B pitch puts the 4 rows of one transposed read 8 banks apart, and rows
// with bit 3 set are XOR-shifted by 64 columns (32 banks) so the two 16-lane
// groups of a 32-lane half never collide.
template <typename T> CTN_DEV int cswz(int row, int col);

template <typename T> struct ColsPitch;
template <> struct ColsPitch<bf16raw> { static constexpr int v = 288; };   // 256 B row + 32 pad
template <> struct ColsPitch<float> { static constexpr int v = 576; };     // 512 B row + 64 pad
template <> CTN_DEV int cswz<bf16raw>(int row, int col) {
  return row * ColsPitch<bf16raw>::v + ((col ^ (((row >> 3) & 1) << 6)) << 1);
}
template <> CTN_DEV int cswz<float>(int row, int col) { return row * ColsPitch<float>::v + (col << 2); }

// Two 4-wave groups per workgroup split a chunk's rows in halves, each with its
// own LDS stages, and add their 128x128 accumulators through LDS at the end: one
// partial per chunk from 8 waves halves the partial-sum traffic (write here, read
// by the slab reduction) of 4-wave workgroups at the same occupancy.
#ifndef CTN_COLS_CKS
#define CTN_COLS_CKS 2   // bf16 k-split groups per workgroup (experiment switch)
#endif
template <typename T> struct ColsCks { static constexpr int v = sizeof(T) == 2 ? CTN_COLS_CKS : 2; };
// 1 (experiment switch): the B-operand loads carry the nontemporal hint
#ifndef CTN_COLS_NTA
#define CTN_COLS_NTA 0   // 1 (experiment switch): the A-operand loads carry the nontemporal hint
#endif
#ifndef CTN_COLS_NTB
#define CTN_COLS_NTB 0
#endif
#ifndef CTN_COLS_XLM
#define CTN_COLS_XLM 0
#endif
#ifndef CTN_COLS_CKR
#define CTN_COLS_CKR 32  // bf16 frame rows per k-step (experiment switch: 32 or 64)
#endif
template <typename T> struct ColsCkr { static constexpr int v = sizeof(T) == 2 ? CTN_COLS_CKR : CKR; };
constexpr int CKS = 2;                           // k-split groups per workgroup (host-side sizing)

#ifndef CTN_COLS_PRIO
#define CTN_COLS_PRIO 0
#endif
template <typename T, int OPA, int OPB, int NK>
__global__ __launch_bounds__(256 * ColsCks<T>::v) void gemm_cols_kernel(GemmCols p) {
  constexpr int CKS = ColsCks<T>::v;
  constexpr int CKR = ColsCkr<T>::v;
  static_assert(CKR % 32 == 0, "k-steps are whole 32-row MFMA steps");
  constexpr int PITCH = ColsPitch<T>::v;
  constexpr int STAGE = 2 * CKR * PITCH;         // one k-step: A tile then B tile
  static_assert(CKS * 2 * STAGE >= CBP * CBQ * 4, "accumulator exchange (one group at a time) fits the stages");
  __shared__ __attribute__((aligned(16))) char smem_all[CKS * 2 * STAGE];
  constexpr int E = Chunk<T>::E;
  constexpr int CPR = CBP * sizeof(T) / 16;      // 16-byte chunks per LDS row
  constexpr int NCH = CKR * CPR / 256;           // chunks per thread per operand
  const int grp = threadIdx.x >> 8;              // k-split group
  char* smem = smem_all + grp * 2 * STAGE;
  // static priority of one k-split group (experiment): 1 = group 1, 2 = group 0
  if constexpr (CTN_COLS_PRIO == 1) { if (grp == 1) __builtin_amdgcn_s_setprio(1); }
  if constexpr (CTN_COLS_PRIO == 2) { if (grp == 0) __builtin_amdgcn_s_setprio(1); }
  const int tid = threadIdx.x & 255, lane = tid & 63, wid = tid >> 6;
  const int wp = wid >> 1, wq = wid & 1;
  const int lr = lane & 15, lg = lane >> 4;

  const int ntq = (p.Q + CBQ - 1) / CBQ, ntp = (p.P + CBP - 1) / CBP;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % (ntp * ntq), chunk = bid / (ntp * ntq);
  const int p0 = (tile / ntq) * CBP, q0 = (tile % ntq) * CBQ;

  // 32-bit row arithmetic (M*Kp < 2^31; checked by the launcher): no 64-bit divisions
  const int rows = (int)p.g.rows();
  const int rpc = (((rows + p.nchunks - 1) / p.nchunks + CKS * CKR - 1) / (CKS * CKR)) * (CKS * CKR);
  const int half = rpc / CKS;                               // rows per group, multiple of CKR
  const int cbeg = chunk * rpc;
  const int steps_of = [&](int g) {
    const int b = cbeg + g * half, e = b + half < rows ? b + half : rows;
    return e > b ? (e - b) / CKR : 0;                       // rows is a multiple of CKR
  }(0);
  const int rbeg = cbeg + grp * half;
  const int rend = rbeg + half < rows ? rbeg + half : rows;
  const int nks = rend > rbeg ? (rend - rbeg) / CKR : 0;    // this group's k-steps (may be 0)
  const int nks_all = steps_of;                             // group 0 holds the most steps

  const T* A = reinterpret_cast<const T*>(p.A);
  const T* B = reinterpret_cast<const T*>(p.B);
  const int K = p.g.K, Kp = p.g.Kp;

  // per-thread operand-transform constants: a thread's 16-byte column chunk cc0 is the
  // same for all its chunks and k-steps, so gamma/beta are loaded once
  const int cc0 = tid % CPR;
  float ga_[E], ba_[E], gb_[E], bb_[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    ga_[e] = ba_[e] = gb_[e] = bb_[e] = 0.f;
    if constexpr (OPA != OP_PLAIN)
      if (p0 + cc0 * E + e < p.P) { ga_[e] = p.aop.gamma[p0 + cc0 * E + e]; ba_[e] = p.aop.beta[p0 + cc0 * E + e]; }
    if constexpr (OPB != OP_PLAIN)
      if (q0 + cc0 * E + e < p.Q) { gb_[e] = p.bop.gamma[q0 + cc0 * E + e]; bb_[e] = p.bop.beta[q0 + cc0 * E + e]; }
  }
  const float ala = OPA == OP_PRELU_NORM ? p.aop.alpha[0] : 0.f;
  const float alb = OPB == OP_PRELU_NORM ? p.bop.alpha[0] : 0.f;
  const bool pin = p0 + cc0 * E < p.P, qin = q0 + cc0 * E < p.Q;

  // Two register sets, each one k-step of both operands, loaded two steps ahead;
  // rows past the chunk end are clamped to its last step (never stored).  A k-step
  // never straddles utterances (Kp % CKR == 0): one gLN statistic per step.
  constexpr int NST = NK == NORM_GLN ? 1 : NCH;
  struct Set { v4u a[NCH], b[NCH]; f32x2_t sa[NST], sb[NST]; };
  const int last_r0 = nks > 0 ? rbeg + (nks - 1) * CKR : rows - CKR;   // clamp target (valid rows)
  auto gload = [&](Set& R, int ks) __attribute__((always_inline)) {
    const int r0 = ks < nks ? rbeg + ks * CKR : last_r0;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + 256 * i, rl = c / CPR;
      const int r = r0 + rl;
      // unconditional loads (clamped column; zeroed in swrite) keep the loop branch-free
      R.a[i] = ldg16h<CTN_COLS_NTA != 0>(A + (size_t)r * p.lda + (pin ? p0 + cc0 * E : 0));
      R.b[i] = ldg16h<CTN_COLS_NTB != 0>(B + (size_t)r * p.ldb + (qin ? q0 + cc0 * E : 0));
      if constexpr (NK == NORM_CLN) {
        if constexpr (OPA != OP_PLAIN) R.sa[i] = *reinterpret_cast<const f32x2_t*>(p.aop.stats + r);
        if constexpr (OPB != OP_PLAIN) R.sb[i] = *reinterpret_cast<const f32x2_t*>(p.bop.stats + r);
      }
    }
    if constexpr (NK == NORM_GLN) {
      // indexed through the lane's own row so the load stays a (prefetched) vector
      // load: a uniform index becomes an s_load the compiler sinks to its use
      const int m = (r0 + tid / CPR) / Kp;
      if constexpr (OPA != OP_PLAIN) R.sa[0] = *reinterpret_cast<const f32x2_t*>(p.aop.stats + m);
      if constexpr (OPB != OP_PLAIN) R.sb[0] = *reinterpret_cast<const f32x2_t*>(p.bop.stats + m);
    }
  };
  // op(v) = PReLU?(v) * (rstd*gamma) + (beta - mean*rstd*gamma), packed
  auto xform = [&](auto le1, v4u v, f32x2_t st, const float* g, const float* bt, float al, bool pr)
      __attribute__((always_inline)) {
    constexpr bool LE1 = decltype(le1)::value;
    if constexpr (E == 8) {
      float f[8];
      unpack_bf16x8(v, f);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f32x2_t x = {f[2 * e], f[2 * e + 1]};
        if (pr) x = prelu2<LE1>(x, al);
        const f32x2_t sc = f32x2_t{g[2 * e], g[2 * e + 1]} * st[1];
        x = pfma(x, sc, pfma(sc, f32x2_t{-st[0], -st[0]}, f32x2_t{bt[2 * e], bt[2 * e + 1]}));
        v[e] = pk_bf16(x[0], x[1]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = __uint_as_float(v[e]);
        if (pr) x = LE1 ? fmaxf(x, al * x) : fminf(x, al * x);
        v[e] = __float_as_uint((x - st[0]) * (st[1] * g[e]) + bt[e]);
      }
    }
    return v;
  };
  auto swrite = [&](auto le1, const Set& R, int ks, char* st) __attribute__((always_inline)) {
    const int r0 = rbeg + ks * CKR;
    const int k0 = r0 % Kp;   // frame of the step's first row (wave-uniform)
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + 256 * i, rl = c / CPR;
      v4u va = R.a[i], vb = R.b[i];
      const v4u z = v4u{0u, 0u, 0u, 0u};
      // Transformed operands of padded frames would be beta, not 0: zero those rows,
      // unless the other operand is plain (zero there) and the statistic is the
      // utterance's (finite), so the product already vanishes.  Columns past P/Q hold
      // clamped real data and only reach outputs the epilogue does not store.
      if constexpr (OPA != OP_PLAIN) {
        va = xform(le1, va, R.sa[NST == 1 ? 0 : i], ga_, ba_, ala, OPA == OP_PRELU_NORM);
        if constexpr (!(OPB == OP_PLAIN && NK == NORM_GLN)) va = k0 + rl < K ? va : z;
      }
      if constexpr (OPB != OP_PLAIN) {
        vb = xform(le1, vb, R.sb[NST == 1 ? 0 : i], gb_, bb_, alb, OPB == OP_PRELU_NORM);
        if constexpr (!(OPA == OP_PLAIN && NK == NORM_GLN)) vb = k0 + rl < K ? vb : z;
      }
      stg16(st + cswz<T>(rl, cc0 * E), va);
      stg16(st + CKR * PITCH + cswz<T>(rl, cc0 * E), vb);
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const char* st) __attribute__((always_inline)) {
    const char* sA = st;
    const char* sB = st + CKR * PITCH;
    if constexpr (sizeof(T) == 2) {
      // transposed LDS reads: lane (g, 4q+pp) addresses row 8g+4h+q, columns 4pp..4pp+3
      const int q = lr >> 2, pp = lr & 3;
#pragma unroll
      for (int k32 = 0; k32 < CKR; k32 += 32) {
        bf16x8_t af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int col = wp * 64 + i * 16 + 4 * pp;
          s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4_t*)(sA + cswz<T>(k32 + 8 * lg + q, col)));
          s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4_t*)(sA + cswz<T>(k32 + 8 * lg + 4 + q, col)));
          af[i] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = wq * 64 + j * 16 + 4 * pp;
          s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4_t*)(sB + cswz<T>(k32 + 8 * lg + q, col)));
          s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4_t*)(sB + cswz<T>(k32 + 8 * lg + 4 + q, col)));
          bfr[j] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int k4 = 0; k4 < CKR; k4 += 4) {
        float af[4], bfv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = *reinterpret_cast<const float*>(sA + (k4 + lg) * PITCH + (wp * 64 + i * 16 + lr) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          bfv[j] = *reinterpret_cast<const float*>(sB + (k4 + lg) * PITCH + (wq * 64 + j * 16 + lr) * 4);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfv[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  // Pipeline: a ring of NSET register sets, each one k-step of both operands loaded
  // NSET steps ahead; step ks is written into LDS buffer ks&1, its set reloads step
  // ks+NSET, then one LDS-only barrier (the other buffer was last read before the
  // previous barrier).  The loop is unrolled by NSET so every set index is static.
  // Rows of padded frames are zero in the plain operands of this path, so they add
  // nothing; transformed operands are zeroed there explicitly.
#ifndef CTN_COLS_NSET
#define CTN_COLS_NSET 2
#endif
  constexpr int NSET = CTN_COLS_NSET;   // register sets in flight (experiment switch)
  // Both groups run nks_all rounds in lock step (the barriers are workgroup-wide);
  // a group with fewer steps keeps staging its clamped last step but skips the
  // MFMAs of the surplus rounds (a wave-uniform branch after the barrier).
  auto run = [&](auto le1) __attribute__((always_inline)) {
    Set R[NSET];
#pragma unroll
    for (int u = 0; u < NSET; ++u) gload(R[u], u);
    int ks = 0;
    for (; ks + NSET - 1 < nks_all; ks += NSET) {   // full rounds: the same loads trail every wait
#pragma unroll
      for (int u = 0; u < NSET; ++u) {
        char* st = smem + ((ks + u) & 1) * STAGE;
        swrite(le1, R[u], ks + u, st);
        gload(R[u], ks + u + NSET);
        lds_barrier();
        if (ks + u < nks) compute(st);
      }
    }
#pragma unroll
    for (int u = 0; u < NSET; ++u) {   // tail
      if (ks + u < nks_all) {
        char* st = smem + ((ks + u) & 1) * STAGE;
        swrite(le1, R[u], ks + u, st);
        lds_barrier();
        if (ks + u < nks) compute(st);
      }
    }
  };
  if (nks_all > 0) {
    constexpr bool PR = OPA == OP_PRELU_NORM || OPB == OP_PRELU_NORM;
    if (!PR || (OPB == OP_PRELU_NORM ? alb : ala) <= 1.f) run(std::true_type{});
    else run(std::false_type{});
  }
  // groups 1.. hand their accumulators to group 0 through LDS (the stages are free
  // after this barrier), in group order: a fixed summation order
  __syncthreads();
  // accumulator-major image: for accumulator a, the group's 256 lanes store 16 B each,
  // consecutively (a lane-major image put every lane of a wave on the same four banks)
  float* xch = reinterpret_cast<float*>(smem_all);
  static_assert(16 * 256 * 4 * sizeof(float) <= sizeof(smem_all), "exchange image fits the stages");
  // (CTN_COLS_XLM=1: the old lane-major image, for A/B runs)
  auto xi = [&](int a) { return CTN_COLS_XLM ? (tid * 16 + a) * 4 : (a * 256 + tid) * 4; };
  for (int g = 1; g < CKS; ++g) {
    if (grp == g) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<f32x4_t*>(&xch[xi(i * 4 + j)]) = acc[i][j];
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += *reinterpret_cast<const f32x4_t*>(&xch[xi(i * 4 + j)]);
    }
    __syncthreads();
  }
  if (grp != 0) return;
  // lane holds D[p = p0 + wp*64 + i*16 + lg*4 + q][q = q0 + wq*64 + j*16 + lr]
  float* Cp = p.Cpart + (size_t)chunk * p.P * p.Q;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (CTN_PART_NT == 2) {   // lane (lg, 4q + t): row lg*4 + t, columns 4q .. 4q+3
        const int qq = q0 + wq * 64 + j * 16 + (lr & ~3);
        if (qq >= p.Q) continue;          // whole quads (Q % 8 == 0)
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        quad_transpose4(v);
        const int pr = p0 + wp * 64 + i * 16 + lg * 4 + (lr & 3);
        if (pr < p.P) stg16h<true>(&Cp[(size_t)pr * p.Q + qq], f4bits(v));
      } else {
        const int qq = q0 + wq * 64 + j * 16 + lr;
        if (qq >= p.Q) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int pr = p0 + wp * 64 + i * 16 + lg * 4 + e;
          if (pr < p.P) st_part(&Cp[(size_t)pr * p.Q + qq], acc[i][j][e]);
        }
      }
    }
}

// target workgroup count of a column GEMM (CTN_COLS_WG overrides it for A/B experiments)
static int cols_wg_target() {
  static int t = 0;
  if (!t) {
    const char* e = getenv("CTN_COLS_WG");
    const int v = e ? atoi(e) : 0;
    t = v >= 64 && v <= 4096 ? v : 256;
  }
  return t;
}

int gemm_cols_default_chunks(const GemmCols& p) {
  const int tiles = ((p.P + CBP - 1) / CBP) * ((p.Q + CBQ - 1) / CBQ);
  const long rows = p.g.rows();
  int ch = (cols_wg_target() + tiles - 1) / tiles;   // ~256 workgroups of CKS x 4 waves
  const long maxch = (rows + CKS * CKR * 4 - 1) / (CKS * CKR * 4);   // >= 4 k-steps per group
  if (ch > maxch) ch = (int)maxch;
  return ch < 1 ? 1 : ch;
}

template <typename T, int OPA, int OPB, int NK>
static hipError_t launch_cols_t(const GemmCols& p, hipStream_t s) {
  const int tiles = ((p.P + CBP - 1) / CBP) * ((p.Q + CBQ - 1) / CBQ);
  hipLaunchKernelGGL((gemm_cols_kernel<T, OPA, OPB, NK>), dim3(tiles * p.nchunks), dim3(256 * ColsCks<T>::v), 0, s, p);
  return hipGetLastError();
}

template <typename T, int NK>
static hipError_t dispatch_cols_nk(const GemmCols& p, hipStream_t s) {
  const int a = p.aop.kind, b = p.bop.kind;
  if (a == OP_PLAIN && b == OP_PLAIN) return launch_cols_t<T, OP_PLAIN, OP_PLAIN, NK>(p, s);
  if (a == OP_PLAIN && b == OP_NORM) return launch_cols_t<T, OP_PLAIN, OP_NORM, NK>(p, s);
  if (a == OP_PLAIN && b == OP_PRELU_NORM) return launch_cols_t<T, OP_PLAIN, OP_PRELU_NORM, NK>(p, s);
  return hipErrorInvalidValue;
}

// Partial count of a column GEMM as launch_gemm_cols will run it: the wave-specialised
// kernel's row ranges where it applies (ctn_dual_ws.hip), else the tiled kernel's chunks.
int gemm_cols_chunks(DType dt, const GemmCols& p) {
  return gemm_cols_ws_eligible(dt, p) ? gemm_cols_ws_ranges(p) : gemm_cols_default_chunks(p);
}

hipError_t launch_gemm_cols(DType dt, const GemmCols& p, hipStream_t s) {
  if (gemm_cols_ws_eligible(dt, p) && p.nchunks == gemm_cols_ws_ranges(p)) return launch_gemm_cols_ws(p, s);
  if (p.g.Kp % (dt == BF16 ? ColsCkr<bf16raw>::v : CKR) != 0 || p.P % 8 != 0 || p.Q % 8 != 0 || p.nchunks < 1 || p.g.rows() >= (1L << 31))
    return hipErrorInvalidValue;
  const int nk = p.bop.kind != OP_PLAIN ? p.bop.norm : 0;
  if (dt == BF16)
    return nk == NORM_GLN ? dispatch_cols_nk<bf16raw, NORM_GLN>(p, s) : dispatch_cols_nk<bf16raw, NORM_CLN>(p, s);
  return nk == NORM_GLN ? dispatch_cols_nk<float, NORM_GLN>(p, s) : dispatch_cols_nk<float, NORM_CLN>(p, s);
}

}  // namespace ctn
