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
  static CTN_DEV u128 pack(const float* f) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
    u128 v; v.x = w[0]; v.y = w[1]; v.z = w[2]; v.w = w[3]; return v;
  }
};

CTN_DEV u128 zero128() { u128 z; z.x = z.y = z.z = z.w = 0u; return z; }

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

// ===========================================================================
// gemm_rows
// ===========================================================================
constexpr int RBM = 128, RBN = 128, RPITCH = 144;   // bytes per LDS row (128 + 16 pad)

template <typename T, int OPK, int NK, int EPI>
__global__ __launch_bounds__(256) void gemm_rows_kernel(GemmRows p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * RBM * RPITCH];
  constexpr int E = Chunk<T>::E;              // elements per 16 B
  constexpr int BK = 128 / sizeof(T);         // elements per k-step (128 B per row)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int lr = lane & 15, lg = lane >> 4;

  const int ncol = (p.Nout + RBN - 1) / RBN;
  const int bid = blockIdx.x;
  const int coltile = bid % ncol, rowtile = bid / ncol;
  const int row0 = rowtile * RBM, col0 = coltile * RBN;

  const T* A = reinterpret_cast<const T*>(p.A);
  const T* W = reinterpret_cast<const T*>(p.W);
  char* sA = smem;
  char* sW = smem + RBM * RPITCH;

  u128 ra[4], rw[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i, r = c >> 3, kc = c & 7;
      const int k = k0 + kc * E;
      ra[i] = zero128();
      rw[i] = zero128();
      if (k < p.Kred) {
        ra[i] = *reinterpret_cast<const u128*>(A + (size_t)(row0 + r) * p.lda + k);
        if (col0 + r < p.Nout)
          rw[i] = *reinterpret_cast<const u128*>(W + (size_t)(col0 + r) * p.ldw + k);
      }
    }
  };
  auto swrite = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i, r = c >> 3, kc = c & 7;
      const int k = k0 + kc * E;
      u128 va = ra[i];
      if constexpr (OPK != OP_PLAIN)
        if (k < p.Kred) va = apply_op<T, OPK, NK>(va, row0 + r, k, p.g.Kp, p.aop);
      *reinterpret_cast<u128*>(sA + r * RPITCH + kc * 16) = va;
      *reinterpret_cast<u128*>(sW + r * RPITCH + kc * 16) = rw[i];
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.Kred + BK - 1) / BK;
  gload(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();
    swrite(kt * BK);
    __syncthreads();
    if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u128 wf[4], af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        wf[i] = *reinterpret_cast<const u128*>(sW + (wc * 64 + i * 16 + lr) * RPITCH + kk * 64 + lg * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        af[j] = *reinterpret_cast<const u128*>(sA + (wr * 64 + j * 16 + lr) * RPITCH + kk * 64 + lg * 16);
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8_t, wf[i]), __builtin_bit_cast(bf16x8_t, af[j]), acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t wv = s == 0 ? wf[i].x : s == 1 ? wf[i].y : s == 2 ? wf[i].z : wf[i].w;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
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
  // lane holds C[row0 + wr*64 + j*16 + lr][col0 + wc*64 + i*16 + lg*4 + 0..3]
  T* Cp = reinterpret_cast<T*>(p.C);
  const T* Rp = reinterpret_cast<const T*>(p.R);
  const int K = p.g.K, Kp = p.g.Kp;
  float ts = 0.f, tss = 0.f;                 // gLN group partials (this thread)
  float rs[4] = {0, 0, 0, 0}, rss[4] = {0, 0, 0, 0};   // cLN per-row partials
  float cg[4][4], cb[4][4];                  // NORM_BWD column partials
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) { cg[i][q] = 0.f; cb[i][q] = 0.f; }
  const float al = (EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD) ? p.alpha[0] : 0.f;

#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = row0 + wr * 64 + j * 16 + lr;
    const bool valid = (r % Kp) < K;
    float2 st = make_float2(0.f, 0.f);
    if constexpr (EPI == EPI_NORM_BWD) st = p.stats[stat_index<NK>(r, Kp)];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = col0 + wc * 64 + i * 16 + lg * 4;
      if (n >= p.Nout) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if constexpr (EPI == EPI_STORE) {
        if (!valid) v[0] = v[1] = v[2] = v[3] = 0.f;
      } else if constexpr (EPI == EPI_PRELU_STATS) {
        if (valid) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float a = prelu(v[q], al);
            if constexpr (NK == NORM_GLN) { ts += a; tss += a * a; }
            else { rs[j] += a; rss[j] += a * a; }
          }
        } else {
          v[0] = v[1] = v[2] = v[3] = 0.f;
        }
      } else if constexpr (EPI == EPI_RESID) {
        float x[4];
        load4<T>(Rp + (size_t)r * p.ldr + n, x);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = valid ? v[q] + x[q] : 0.f;
      } else if constexpr (EPI == EPI_NORM_BWD) {
        if (valid) {
          float dv[4];
          load4<T>(Rp + (size_t)r * p.ldr + n, dv);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float ah = (prelu(dv[q], al) - st.x) * st.y;
            const float gn = v[q];
            const float ga = gn * p.gamma[n + q];
            cg[i][q] += gn * ah;
            cb[i][q] += gn;
            if constexpr (NK == NORM_GLN) { ts += ga; tss += ga * ah; }
            else { rs[j] += ga; rss[j] += ga * ah; }
            v[q] = ga;
          }
        } else {
          v[0] = v[1] = v[2] = v[3] = 0.f;
        }
      }
      store4<T>(Cp + (size_t)r * p.ldc + n, v);
    }
  }

  if constexpr (EPI == EPI_PRELU_STATS || EPI == EPI_NORM_BWD) {
    __syncthreads();   // LDS tiles are free now
    double* red = reinterpret_cast<double*>(smem);
    if constexpr (NK == NORM_GLN) {
      double v2[2] = {(double)ts, (double)tss};
      block_sum_d<2>(v2, red);
      if (tid == 0) {
        const int tpu = (Kp / RBM) * ncol;    // tiles per utterance
        const int m = row0 / Kp;
        const int tiu = ((row0 % Kp) / RBM) * ncol + coltile;
        p.grp_slab[(size_t)m * tpu + tiu] = make_double2(v2[0], v2[1]);
      }
    } else {
      // per-row partial over this block's columns: reduce lanes with equal lr, then the two wc waves
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        rs[j] += __shfl_xor(rs[j], 16, 64); rs[j] += __shfl_xor(rs[j], 32, 64);
        rss[j] += __shfl_xor(rss[j], 16, 64); rss[j] += __shfl_xor(rss[j], 32, 64);
      }
      float* fr = reinterpret_cast<float*>(smem);   // [2 wc][128 rows][2]
      if (lg == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int rl = wr * 64 + j * 16 + lr;
          fr[(wc * RBM + rl) * 2 + 0] = rs[j];
          fr[(wc * RBM + rl) * 2 + 1] = rss[j];
        }
      }
      __syncthreads();
      if (tid < RBM) {
        const double a = (double)fr[tid * 2] + (double)fr[(RBM + tid) * 2];
        const double b = (double)fr[tid * 2 + 1] + (double)fr[(RBM + tid) * 2 + 1];
        p.grp_slab[(size_t)(row0 + tid) * ncol + coltile] = make_double2(a, b);
      }
    }
  }
  if constexpr (EPI == EPI_NORM_BWD) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float a = cg[i][q], b = cb[i][q];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) { a += __shfl_xor(a, o, 64); b += __shfl_xor(b, o, 64); }
        cg[i][q] = a; cb[i][q] = b;
      }
    float* fc = reinterpret_cast<float*>(smem) + 4 * RBM;   // [2 wr][128 cols][2], after the row scratch
    if (lr == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cl = wc * 64 + i * 16 + lg * 4 + q;
          fc[(wr * RBN + cl) * 2 + 0] = cg[i][q];
          fc[(wr * RBN + cl) * 2 + 1] = cb[i][q];
        }
    }
    __syncthreads();
    if (tid < RBN && col0 + tid < p.Nout) {
      const float a = fc[tid * 2] + fc[(RBN + tid) * 2];
      const float b = fc[tid * 2 + 1] + fc[(RBN + tid) * 2 + 1];
      p.col_slab[((size_t)rowtile * 2 + 0) * p.Nout + col0 + tid] = a;
      p.col_slab[((size_t)rowtile * 2 + 1) * p.Nout + col0 + tid] = b;
    }
  }
}

int gemm_rows_tiles_per_group(const GemmRows& p) {
  const int ncol = (p.Nout + RBN - 1) / RBN;
  return p.norm == NORM_GLN ? (p.g.Kp / RBM) * ncol : ncol;
}
int gemm_rows_rowtiles(const GemmRows& p) { return (int)(p.g.rows() / RBM); }

template <typename T, int OPK, int NK, int EPI>
static hipError_t launch_rows_t(const GemmRows& p, hipStream_t s) {
  const int ncol = (p.Nout + RBN - 1) / RBN;
  const int nrow = (int)(p.g.rows() / RBM);
  hipLaunchKernelGGL((gemm_rows_kernel<T, OPK, NK, EPI>), dim3(nrow * ncol), dim3(256), 0, s, p);
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
  if (p.g.Kp % RBM != 0 || p.Kred % 8 != 0 || p.Nout % 8 != 0) return hipErrorInvalidValue;
  return dt == BF16 ? dispatch_rows<bf16raw>(p, s) : dispatch_rows<float>(p, s);
}

// ===========================================================================
// gemm_cols (weight gradients)
// ===========================================================================
constexpr int CBP = 128, CBQ = 128, CKR = 32;   // tile p x q, rows per k-step

template <typename T> struct ColsPitch;
template <> struct ColsPitch<bf16raw> { static constexpr int v = 288; };   // 256 B row + 32 pad
template <> struct ColsPitch<float> { static constexpr int v = 576; };     // 512 B row + 64 pad

template <typename T, int OPA, int OPB, int NK>
__global__ __launch_bounds__(256) void gemm_cols_kernel(GemmCols p) {
  constexpr int PITCH = ColsPitch<T>::v;
  __shared__ __attribute__((aligned(16))) char smem[2 * CKR * PITCH];
  constexpr int E = Chunk<T>::E;
  constexpr int CPR = CBP * sizeof(T) / 16;      // 16-byte chunks per LDS row
  constexpr int NCH = CKR * CPR / 256;           // chunks per thread per operand
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wp = wid >> 1, wq = wid & 1;
  const int lr = lane & 15, lg = lane >> 4;

  const int ntq = (p.Q + CBQ - 1) / CBQ, ntp = (p.P + CBP - 1) / CBP;
  const int tile = blockIdx.x % (ntp * ntq), chunk = blockIdx.x / (ntp * ntq);
  const int p0 = (tile / ntq) * CBP, q0 = (tile % ntq) * CBQ;

  const long rows = p.g.rows();
  const long rpc = (((rows + p.nchunks - 1) / p.nchunks + CKR - 1) / CKR) * CKR;   // rows per chunk, multiple of CKR
  const long rbeg = chunk * rpc;
  const long rend = rbeg + rpc < rows ? rbeg + rpc : rows;   // may be <= rbeg: empty chunk writes zeros

  const T* A = reinterpret_cast<const T*>(p.A);
  const T* B = reinterpret_cast<const T*>(p.B);
  char* sA = smem;
  char* sB = smem + CKR * PITCH;
  const int K = p.g.K, Kp = p.g.Kp;

  u128 ra[NCH], rb[NCH];
  auto gload = [&](long r0) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + 256 * i, rl = c / CPR, cc = c % CPR;
      const long r = r0 + rl;
      ra[i] = zero128();
      rb[i] = zero128();
      if (r < rend && (int)(r % Kp) < K) {
        const int pc = p0 + cc * E, qc = q0 + cc * E;
        if (pc < p.P) ra[i] = *reinterpret_cast<const u128*>(A + (size_t)r * p.lda + pc);
        if (qc < p.Q) rb[i] = *reinterpret_cast<const u128*>(B + (size_t)r * p.ldb + qc);
      }
    }
  };
  auto swrite = [&](long r0) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + 256 * i, rl = c / CPR, cc = c % CPR;
      const long r = r0 + rl;
      u128 va = ra[i], vb = rb[i];
      const bool ok = r < rend && (int)(r % Kp) < K;
      if constexpr (OPA != OP_PLAIN)
        if (ok && p0 + cc * E < p.P) va = apply_op<T, OPA, NK>(va, (int)r, p0 + cc * E, Kp, p.aop);
      if constexpr (OPB != OP_PLAIN)
        if (ok && q0 + cc * E < p.Q) vb = apply_op<T, OPB, NK>(vb, (int)r, q0 + cc * E, Kp, p.bop);
      *reinterpret_cast<u128*>(sA + rl * PITCH + cc * 16) = va;
      *reinterpret_cast<u128*>(sB + rl * PITCH + cc * 16) = vb;
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (rbeg < rend) gload(rbeg);
  for (long r0 = rbeg; r0 < rend; r0 += CKR) {
    __syncthreads();
    swrite(r0);
    __syncthreads();
    if (r0 + CKR < rend) gload(r0 + CKR);
    if constexpr (sizeof(T) == 2) {
      // transposed LDS reads: lane (g, 4q+pp) addresses row 8g+4h+q, columns 4pp..4pp+3
      const int q = lr >> 2, pp = lr & 3;
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = wp * 64 + i * 16 + 4 * pp;
        s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(sA + (8 * lg + q) * PITCH + col * 2));
        s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(sA + (8 * lg + 4 + q) * PITCH + col * 2));
        af[i] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wq * 64 + j * 16 + 4 * pp;
        s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(sB + (8 * lg + q) * PITCH + col * 2));
        s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(sB + (8 * lg + 4 + q) * PITCH + col * 2));
        bfr[j] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
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
  }
  // lane holds D[p = p0 + wp*64 + i*16 + lg*4 + q][q = q0 + wq*64 + j*16 + lr]
  float* Cp = p.Cpart + (size_t)chunk * p.P * p.Q;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int qq = q0 + wq * 64 + j * 16 + lr;
      if (qq >= p.Q) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int pr = p0 + wp * 64 + i * 16 + lg * 4 + e;
        if (pr < p.P) Cp[(size_t)pr * p.Q + qq] = acc[i][j][e];
      }
    }
}

int gemm_cols_default_chunks(const GemmCols& p) {
  const int tiles = ((p.P + CBP - 1) / CBP) * ((p.Q + CBQ - 1) / CBQ);
  const long rows = p.g.rows();
  int ch = (512 + tiles - 1) / tiles;            // ~512 workgroups
  const long maxch = (rows + CKR * 4 - 1) / (CKR * 4);   // >= 4 k-steps per chunk
  if (ch > maxch) ch = (int)maxch;
  return ch < 1 ? 1 : ch;
}

template <typename T, int OPA, int OPB, int NK>
static hipError_t launch_cols_t(const GemmCols& p, hipStream_t s) {
  const int tiles = ((p.P + CBP - 1) / CBP) * ((p.Q + CBQ - 1) / CBQ);
  hipLaunchKernelGGL((gemm_cols_kernel<T, OPA, OPB, NK>), dim3(tiles * p.nchunks), dim3(256), 0, s, p);
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

hipError_t launch_gemm_cols(DType dt, const GemmCols& p, hipStream_t s) {
  if (p.g.Kp % CKR != 0 || p.P % 8 != 0 || p.Q % 8 != 0 || p.nchunks < 1) return hipErrorInvalidValue;
  const int nk = p.bop.kind != OP_PLAIN ? p.bop.norm : 0;
  if (dt == BF16)
    return nk == NORM_GLN ? dispatch_cols_nk<bf16raw, NORM_GLN>(p, s) : dispatch_cols_nk<bf16raw, NORM_CLN>(p, s);
  return nk == NORM_GLN ? dispatch_cols_nk<float, NORM_GLN>(p, s) : dispatch_cols_nk<float, NORM_CLN>(p, s);
}

}  // namespace ctn
