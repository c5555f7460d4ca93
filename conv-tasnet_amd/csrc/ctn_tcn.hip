// Element-wise / depthwise kernels of the TemporalBlock (conv_tasnet.py:212-272)
// and the statistics plumbing shared by all kernels (gfx950).
//
// dw_fwd    : n1 = norm1(PReLU(h1)) recomputed on the fly, depthwise dilated
//             conv (causal = left pad only, identical to pad + Chomp1d,
//             conv_tasnet.py:176,247-260,289), stores d (pre-PReLU) and the
//             partial statistics of PReLU(d) for norm2.
// dw_bwd    : norm2 backward (element part) -> PReLU2 backward -> transposed
//             depthwise conv -> norm1 backward partial sums; column partials
//             for gamma1/beta1/dw weight/alpha2.
// norm1_bwd : norm1 backward finish -> PReLU1 backward -> dL/dh1.
//
// Thread layout (all three): a workgroup owns 128 frame rows of one utterance
// (Kp % 128 == 0) and all H channels; a thread owns 8 consecutive channels
// (one 16-byte bf16 vector) of every (256 / (H/8))-th row.
#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

constexpr int DW_RPB = 128;   // rows per workgroup
constexpr int DW_MAXP = 8;

int dw_blocks(const DwArgs& a) { return (int)(a.g.rows() / DW_RPB); }
int dw_parts_per_group(const DwArgs& a) { return a.norm == NORM_GLN ? a.g.Kp / DW_RPB : 1; }
__host__ __device__ int dw_col_stride(const DwArgs& a) { return ((2 + a.P) * a.H + 4 + 3) & ~3; }

template <int NK> CTN_DEV float2 ld_stat(const float2* s, int m, int row) {
  return NK == NORM_GLN ? s[m] : s[row];
}

// column-partial reduction: sum val[8] over row lanes, write H floats to dst.
CTN_DEV void col_reduce8(float* buf, const float v[8], int rl, int c, int nrl, int cg, bool act, float* dst) {
  const int H = cg * 8;
  if (act)
#pragma unroll
    for (int e = 0; e < 8; ++e) buf[rl * H + c * 8 + e] = v[e];
  __syncthreads();
  for (int ch = threadIdx.x; ch < H; ch += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < nrl; ++q) s += buf[q * H + ch];
    dst[ch] = s;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Per-row work is written "loads first": every tap row is addressed with a
// clamped (always valid) index, all tap loads are issued before any use, and
// out-of-range taps are zeroed afterwards — no branch between the loads, so a
// row costs one memory latency instead of one per tap.
// ---------------------------------------------------------------------------
// dw_fwd: one row = P raw tap loads (issued together) + the conv; two rows per
// iteration keep 2P loads in flight per thread.
// ---------------------------------------------------------------------------
template <typename T, int NK, int P>
__global__ __launch_bounds__(256) void dw_fwd_kernel(DwArgs a) {
  __shared__ double red[16];
  const int H = a.H, cg = H / 8;
  int nrl = 256 / cg;
  if (nrl > DW_RPB) nrl = DW_RPB;
  const int tid = threadIdx.x, c = tid % cg, rl = tid / cg;
  const bool act = rl < nrl;
  const int K = a.g.K, Kp = a.g.Kp;
  const int row0 = blockIdx.x * DW_RPB, m = row0 / Kp, base = m * Kp;
  const T* h1 = reinterpret_cast<const T*>(a.h1);
  T* dout = reinterpret_cast<T*>(a.d_out);
  const float al1 = a.alpha1[0], al2 = a.alpha2[0];
  const float2 st1u = NK == NORM_GLN ? a.st1[m] : make_float2(0.f, 0.f);

  float w[P][8], g1[8], b1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int ch = c * 8 + e;
    g1[e] = a.gamma1[ch];
    b1[e] = a.beta1[ch];
#pragma unroll
    for (int p = 0; p < P; ++p) w[p][e] = a.wd[ch * P + p];
  }
  float ts = 0.f, tss = 0.f;
  if (act) {
    for (int rr0 = rl; rr0 < DW_RPB; rr0 += 2 * nrl) {
      Raw8<T> v[2][P];
      bool ok[2][P];
      int rk[2][P];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = row0 + rr0 + u * nrl - base;
        const int kc = k < K ? k : K - 1;
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const int kk = k - a.pad + p * a.dil;
          ok[u][p] = k < K && rr0 + u * nrl < DW_RPB && kk >= 0 && kk < K;
          rk[u][p] = base + (ok[u][p] ? kk : kc);
          v[u][p].load(h1 + (size_t)rk[u][p] * H + c * 8);
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int rr = rr0 + u * nrl;
        if (rr >= DW_RPB) break;
        const int r = row0 + rr, k = r - base;
        float out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        float s = 0.f, ss = 0.f;
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const float2 st = NK == NORM_GLN ? st1u : a.st1[rk[u][p]];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float n1 = (prelu(v[u][p][e], al1) - st.x) * st.y * g1[e] + b1[e];
            out[e] += ok[u][p] ? w[p][e] * n1 : 0.f;
          }
        }
        if (k < K) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float a2 = prelu(out[e], al2);
            s += a2;
            ss += a2 * a2;
          }
        }
        Vec8<T>::store(dout + (size_t)r * H + c * 8, out);
        if constexpr (NK == NORM_GLN) {
          ts += s;
          tss += ss;
        } else {
          s = wave_sum_group(s, cg);
          ss = wave_sum_group(ss, cg);
          if (c == 0) a.slab2[r] = make_double2((double)s, (double)ss);
        }
      }
    }
  }
  if constexpr (NK == NORM_GLN) {
    double v2[2] = {(double)ts, (double)tss};
    block_sum_d<2>(v2, red);
    if (tid == 0) a.slab2[(size_t)m * (Kp / DW_RPB) + (row0 - base) / DW_RPB] = make_double2(v2[0], v2[1]);
  }
}

// ---------------------------------------------------------------------------
// dw_bwd: per row 3P raw loads (d and dL/d hat a2 at the P rows whose taps read
// this row, h1 at this row's P input taps), issued before any use.
// ---------------------------------------------------------------------------
template <typename T, int NK, int P>
__global__ __launch_bounds__(256) void dw_bwd_kernel(DwArgs a) {
  __shared__ double red[16];
  __shared__ float buf[256 * 8];
  __shared__ __attribute__((aligned(16))) float sw[(P + 2) * 2048];   // [P+2][H]: taps, gamma1, beta1
  const int H = a.H, cg = H / 8;
  int nrl = 256 / cg;
  if (nrl > DW_RPB) nrl = DW_RPB;
  const int tid = threadIdx.x, c = tid % cg, rl = tid / cg;
  const bool act = rl < nrl;
  const int K = a.g.K, Kp = a.g.Kp;
  const int row0 = blockIdx.x * DW_RPB, m = row0 / Kp, base = m * Kp;
  const T* h1 = reinterpret_cast<const T*>(a.h1);
  const T* dd = reinterpret_cast<const T*>(a.d);
  const T* ga2 = reinterpret_cast<const T*>(a.ga2);
  T* ga1o = reinterpret_cast<T*>(a.ga1_out);
  const float al1 = a.alpha1[0], al2 = a.alpha2[0];
  const int pown = a.pad / a.dil;   // the tap that reads the output row itself
  float2 st1u = make_float2(0.f, 0.f), st2u = st1u, sm2u = st1u;
  if constexpr (NK == NORM_GLN) { st1u = a.st1[m]; st2u = a.st2[m]; sm2u = a.sm2[m]; }

  // per-channel constants live in LDS, not in registers (this kernel is VGPR-bound)
  for (int i = tid; i < H; i += 256) {
#pragma unroll
    for (int p = 0; p < P; ++p) sw[p * H + i] = a.wd[i * P + p];
    sw[P * H + i] = a.gamma1[i];
    sw[(P + 1) * H + i] = a.beta1[i];
  }
  __syncthreads();
  auto cst = [&](int q, int e) -> float { return sw[q * H + c * 8 + e]; };
  float cgam[8], cbet[8], cwd[P][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    cgam[e] = cbet[e] = 0.f;
#pragma unroll
    for (int p = 0; p < P; ++p) cwd[p][e] = 0.f;
  }
  float calpha = 0.f, ts = 0.f, tss = 0.f;

  if (act) {
    for (int rr = rl; rr < DW_RPB; rr += nrl) {
      const int r = row0 + rr, k = r - base;
      float ga1[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      float s = 0.f, ss = 0.f;
      if (k < K) {
        Raw8<T> dv[P], gv[P], hv[P];
        bool okq[P], okk[P];
        int rq[P], rk[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const int kq = k + a.pad - p * a.dil;   // output row whose tap p reads row k
          const int kk = k - a.pad + p * a.dil;   // input row read by tap p of row k
          okq[p] = kq >= 0 && kq < K;
          okk[p] = kk >= 0 && kk < K;
          rq[p] = base + (okq[p] ? kq : k);
          rk[p] = base + (okk[p] ? kk : k);
          dv[p].load(dd + (size_t)rq[p] * H + c * 8);
          gv[p].load(ga2 + (size_t)rq[p] * H + c * 8);
          hv[p].load(h1 + (size_t)rk[p] * H + c * 8);
        }
        float gn1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, gdo[8];
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const float2 st = NK == NORM_GLN ? st2u : a.st2[rq[p]];
          const float2 sm = NK == NORM_GLN ? sm2u : a.sm2[rq[p]];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = dv[p][e];
            const float ah = (prelu(x, al2) - st.x) * st.y;
            const float ga = st.y * (gv[p][e] - sm.x - ah * sm.y);      // dL/da2
            const float gd = ga * prelu_dx(x, al2);
            gn1[e] += okq[p] ? cst(p, e) * gd : 0.f;
            if (p == pown) {
              gdo[e] = gd;
              calpha += ga * prelu_da(x);
            }
          }
        }
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const float2 st = NK == NORM_GLN ? st1u : a.st1[rk[p]];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float ah = (prelu(hv[p][e], al1) - st.x) * st.y;
            cwd[p][e] += okk[p] ? gdo[e] * (ah * cst(P, e) + cst(P + 1, e)) : 0.f;
            if (p == pown) {
              cgam[e] += gn1[e] * ah;
              cbet[e] += gn1[e];
              ga1[e] = gn1[e] * cst(P, e);
              s += ga1[e];
              ss += ga1[e] * ah;
            }
          }
        }
      }
      Vec8<T>::store(ga1o + (size_t)r * H + c * 8, ga1);
      if constexpr (NK == NORM_GLN) {
        ts += s;
        tss += ss;
      } else {
        s = wave_sum_group(s, cg);
        ss = wave_sum_group(ss, cg);
        if (c == 0) a.slab1[r] = make_double2((double)s, (double)ss);
      }
    }
  }
  // ---- block reductions
  float* cs = a.col_slab + (size_t)blockIdx.x * dw_col_stride(a);
  col_reduce8(buf, cgam, rl, c, nrl, cg, act, cs);
  col_reduce8(buf, cbet, rl, c, nrl, cg, act, cs + H);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    // stored [H][P] to match the parameter layout [H,1,P]
    if (act)
#pragma unroll
      for (int e = 0; e < 8; ++e) buf[rl * H + c * 8 + e] = cwd[p][e];
    __syncthreads();
    for (int ch = tid; ch < H; ch += blockDim.x) {
      float sacc = 0.f;
      for (int q = 0; q < nrl; ++q) sacc += buf[q * H + ch];
      cs[2 * H + ch * P + p] = sacc;
    }
    __syncthreads();
  }
  {
    double v3[3] = {(double)calpha, (double)ts, (double)tss};
    block_sum_d<3>(v3, red);
    if (tid == 0) {
      cs[(2 + P) * H] = (float)v3[0];
      if constexpr (NK == NORM_GLN)
        a.slab1[(size_t)m * (Kp / DW_RPB) + (row0 - base) / DW_RPB] = make_double2(v3[1], v3[2]);
    }
  }
}

// ---------------------------------------------------------------------------
template <typename T, int NK>
__global__ __launch_bounds__(256) void norm1_bwd_kernel(DwArgs a) {
  __shared__ double red[8];
  const int H = a.H, cg = H / 8;
  int nrl = 256 / cg;
  if (nrl > DW_RPB) nrl = DW_RPB;
  const int tid = threadIdx.x, c = tid % cg, rl = tid / cg;
  const bool act = rl < nrl;
  const int K = a.g.K, Kp = a.g.Kp;
  const int row0 = blockIdx.x * DW_RPB, m = row0 / Kp, base = m * Kp;
  const T* h1 = reinterpret_cast<const T*>(a.h1);
  const T* ga1 = reinterpret_cast<const T*>(a.ga2);   // input: dL/d(hat a1)
  T* gh = reinterpret_cast<T*>(a.gh1_out);
  const float al1 = a.alpha1[0];
  float calpha = 0.f;
  if (act) {
    for (int rr = rl; rr < DW_RPB; rr += nrl) {
      const int r = row0 + rr, k = r - base;
      float out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (k < K) {
        float v[8], g[8];
        Vec8<T>::load(h1 + (size_t)r * H + c * 8, v);
        Vec8<T>::load(ga1 + (size_t)r * H + c * 8, g);
        const float2 st = ld_stat<NK>(a.st1, m, r);
        const float2 sm = ld_stat<NK>(a.sm1, m, r);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float ah = (prelu(v[e], al1) - st.x) * st.y;
          const float ga = st.y * (g[e] - sm.x - ah * sm.y);
          out[e] = ga * prelu_dx(v[e], al1);
          calpha += ga * prelu_da(v[e]);
        }
      }
      Vec8<T>::store(gh + (size_t)r * H + c * 8, out);
    }
  }
  double v1[1] = {(double)calpha};
  block_sum_d<1>(v1, red);
  if (tid == 0) a.alpha_slab[blockIdx.x] = (float)v1[0];
}


static hipError_t dw_check(const DwArgs& a) {
  if (a.H % 8 != 0 || a.H / 8 > 256 || a.P < 1 || a.P > DW_MAXP || a.g.Kp % DW_RPB != 0) return hipErrorInvalidValue;
  if (a.norm == NORM_CLN) {
    const int cg = a.H / 8;
    if (cg > 64 || (cg & (cg - 1))) return hipErrorInvalidValue;
  }
  return hipSuccess;
}

#define CTN_DW_P_KERNEL(NAME)                                                                \
  template <typename T, int NK, int P>                                                     \
  static void NAME##_launch(const DwArgs& a, hipStream_t s) {                              \
    hipLaunchKernelGGL((NAME##_kernel<T, NK, P>), dim3(dw_blocks(a)), dim3(256), 0, s, a); \
  }                                                                                        \
  template <typename T, int NK>                                                            \
  static hipError_t NAME##_dispatch_p(const DwArgs& a, hipStream_t s) {                    \
    switch (a.P) {                                                                         \
      case 1: NAME##_launch<T, NK, 1>(a, s); break;                                        \
      case 2: NAME##_launch<T, NK, 2>(a, s); break;                                        \
      case 3: NAME##_launch<T, NK, 3>(a, s); break;                                        \
      case 4: NAME##_launch<T, NK, 4>(a, s); break;                                        \
      case 5: NAME##_launch<T, NK, 5>(a, s); break;                                        \
      case 6: NAME##_launch<T, NK, 6>(a, s); break;                                        \
      case 7: NAME##_launch<T, NK, 7>(a, s); break;                                        \
      case 8: NAME##_launch<T, NK, 8>(a, s); break;                                        \
      default: return hipErrorInvalidValue;                                                \
    }                                                                                      \
    return hipGetLastError();                                                              \
  }                                                                                        \
  hipError_t launch_##NAME(DType dt, const DwArgs& a, hipStream_t s) {                     \
    hipError_t e = dw_check(a);                                                            \
    if (e != hipSuccess) return e;                                                         \
    if (dt == BF16)                                                                        \
      return a.norm == NORM_GLN ? NAME##_dispatch_p<bf16raw, NORM_GLN>(a, s)               \
                                : NAME##_dispatch_p<bf16raw, NORM_CLN>(a, s);              \
    return a.norm == NORM_GLN ? NAME##_dispatch_p<float, NORM_GLN>(a, s)                   \
                              : NAME##_dispatch_p<float, NORM_CLN>(a, s);                  \
  }

CTN_DW_P_KERNEL(dw_fwd)
CTN_DW_P_KERNEL(dw_bwd)

hipError_t launch_norm1_bwd(DType dt, const DwArgs& a, hipStream_t s) {
  hipError_t e = dw_check(a);
  if (e != hipSuccess) return e;
  const dim3 grid(dw_blocks(a)), blk(256);
  if (dt == BF16) {
    if (a.norm == NORM_GLN) hipLaunchKernelGGL((norm1_bwd_kernel<bf16raw, NORM_GLN>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((norm1_bwd_kernel<bf16raw, NORM_CLN>), grid, blk, 0, s, a);
  } else {
    if (a.norm == NORM_GLN) hipLaunchKernelGGL((norm1_bwd_kernel<float, NORM_GLN>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((norm1_bwd_kernel<float, NORM_CLN>), grid, blk, 0, s, a);
  }
  return hipGetLastError();
}

// ===========================================================================
// statistics finalize / slab reduce / weight prep
// ===========================================================================
// one thread per group (few parts, e.g. cLN rows) ...
__global__ __launch_bounds__(256) void stats_finalize_thread_kernel(const double2* slab, int G, int nparts, double cnt,
                                                                    int mode, float eps, float2* out) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= G) return;
  double s = 0.0, ss = 0.0;
  for (int i = 0; i < nparts; ++i) {
    const double2 v = slab[(size_t)g * nparts + i];
    s += v.x;
    ss += v.y;
  }
  if (mode == 0) {
    const double mean = s / cnt;
    double var = ss / cnt - mean * mean;
    if (var < 0.0) var = 0.0;
    out[g] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
  } else {
    out[g] = make_float2((float)(s / cnt), (float)(ss / cnt));
  }
}

// ... or one workgroup per group (many parts, e.g. gLN utterances)
__global__ __launch_bounds__(256) void stats_finalize_block_kernel(const double2* slab, int nparts, double cnt,
                                                                   int mode, float eps, float2* out) {
  __shared__ double red[8];
  const int g = blockIdx.x;
  double v[2] = {0.0, 0.0};
  for (int i = threadIdx.x; i < nparts; i += 256) {
    const double2 x = slab[(size_t)g * nparts + i];
    v[0] += x.x;
    v[1] += x.y;
  }
  block_sum_d<2>(v, red);
  if (threadIdx.x == 0) {
    if (mode == 0) {
      const double mean = v[0] / cnt;
      double var = v[1] / cnt - mean * mean;
      if (var < 0.0) var = 0.0;
      out[g] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
    } else {
      out[g] = make_float2((float)(v[0] / cnt), (float)(v[1] / cnt));
    }
  }
}

hipError_t launch_stats_finalize(const double2* slab, int G, int nparts, double cnt, int mode, float eps,
                                 float2* out, hipStream_t s) {
  if (nparts >= 8)
    hipLaunchKernelGGL(stats_finalize_block_kernel, dim3(G), dim3(256), 0, s, slab, nparts, cnt, mode, eps, out);
  else
    hipLaunchKernelGGL(stats_finalize_thread_kernel, dim3((G + 255) / 256), dim3(256), 0, s, slab, G, nparts, cnt,
                       mode, eps, out);
  return hipGetLastError();
}

// out[i] = sum_q src[q * pstride + i]: workgroup = 16 consecutive outputs x 16 part lanes,
// fixed summation order (deterministic), fp64 accumulation
constexpr int SR_E = 16, SR_Q = 16;
__global__ __launch_bounds__(256) void slab_reduce_kernel(SlabBatch b) {
  __shared__ double part[SR_Q][SR_E];
  const SlabDesc d = b.d[blockIdx.y];
  const int e = threadIdx.x % SR_E, q0 = threadIdx.x / SR_E;
  for (int i0 = blockIdx.x * SR_E; i0 < d.n; i0 += gridDim.x * SR_E) {
    const int i = i0 + e;
    double sacc = 0.0;
    if (i < d.n)
      for (int q = q0; q < d.nparts; q += SR_Q) sacc += (double)d.src[(size_t)q * d.pstride + i];
    part[q0][e] = sacc;
    __syncthreads();
    if (q0 == 0 && i < d.n) {
      double t = 0.0;
#pragma unroll
      for (int qq = 0; qq < SR_Q; ++qq) t += part[qq][e];
      d.dst[i] = (float)t;
    }
    __syncthreads();
  }
}

hipError_t launch_slab_reduce(const SlabBatch& b, hipStream_t s) {
  if (b.nd <= 0) return hipSuccess;
  int mx = 1;
  for (int i = 0; i < b.nd; ++i) mx = b.d[i].n > mx ? b.d[i].n : mx;
  int gx = (mx + SR_E - 1) / SR_E;
  if (gx > 2048) gx = 2048;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(gx, b.nd), dim3(256), 0, s, b);
  return hipGetLastError();
}

template <typename T>
__global__ __launch_bounds__(256) void prep_weight_kernel(const float* W, int O, int I, T* Ws, T* Wt) {
  const long n = (long)O * I;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int o = (int)(i / I), j = (int)(i % I);
    const float v = W[i];
    if (Ws) st1<T>(Ws + i, v);
    if (Wt) st1<T>(Wt + (size_t)j * O + o, v);
  }
}

hipError_t launch_prep_weight(DType dt, const float* W, int O, int I, void* Ws, void* Wt, hipStream_t s) {
  const long n = (long)O * I;
  int g = (int)((n + 255) / 256);
  if (g > 1024) g = 1024;
  if (dt == BF16)
    hipLaunchKernelGGL(prep_weight_kernel<bf16raw>, dim3(g), dim3(256), 0, s, W, O, I, (bf16raw*)Ws, (bf16raw*)Wt);
  else
    hipLaunchKernelGGL(prep_weight_kernel<float>, dim3(g), dim3(256), 0, s, W, O, I, (float*)Ws, (float*)Wt);
  return hipGetLastError();
}

}  // namespace ctn
