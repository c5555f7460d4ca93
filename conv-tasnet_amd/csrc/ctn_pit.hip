// PIT SI-SNR loss (pit_criterion.py:12-113) as batched reductions (gfx950).
//
// pit_stats : per utterance and T-chunk, fp64 partial sums of e_i, s_j, e_i^2,
//             s_j^2, e_i*s_j (t < length) and s_j (all t); masking by length
//             is folded in (pit_criterion.py:37-38, :101-113).
// pit_final : one workgroup: zero-mean corrections (:41-48), pairwise SI-SNR
//             (:52-62), C! permutation sums (:66-71), max/argmax (:72-75),
//             loss = -mean (:22); plus per-(utterance, estimate) gradient
//             coefficients so that backward is one element-wise pass.
// pit_reorder: masked estimate in place + reorder by the winning permutation,
//             keeping the reference's perm-not-inverse indexing (:91-97).
// pit_bwd   : dL/dest[m][i][t] = scale_m (alpha s_j[t] + beta e_i[t] + offset), t < length.
//
// C <= 4: pit_final is one workgroup, one thread per utterance, the C! <= 24
// permutations from a table in the kernel arguments.  5 <= C <= 10 (C! up to 3,628,800):
// pit_final_wide runs one workgroup per utterance whose threads split the
// permutation indices (each decoded from its lexicographic rank, the order of
// itertools.permutations), then pit_loss sums the utterances' maxima.
// 11 <= C <= 16: C! (up to 2.1e13) is past what the reference itself can enumerate (its
// one-hot table, pit_criterion.py:66-69, needs C!*C*C floats); the maximum of
// sum_i snr[i][perm[i]] over permutations is a linear assignment, solved exactly by the
// Hungarian algorithm in fp64 (pit_assign_max), and best_perm is that permutation's
// lexicographic rank.  Exact ties between permutations may resolve to a different optimum
// than the reference's first-in-order argmax.  C > 8 takes its statistics from
// pit_stats_wide (runtime C, the chunk staged in LDS, one accumulator per value).
#include "ctn_codec.h"
#include "ctn_common.h"

namespace ctn {

constexpr double PIT_EPS = 1e-8;   // pit_criterion.py:9

int pit_nv(int C) { return 5 * C + C * C; }

template <int C>
__global__ __launch_bounds__(256) void pit_stats_kernel(PitArgs a) {
  constexpr int NV = 5 * C + C * C;
  __shared__ double red[NV * 4];
  const int m = blockIdx.y, chunk = blockIdx.x;
  const int T = a.T;
  const long len = a.lengths[m];
  const int span = (T + a.chunks - 1) / a.chunks;
  const int t0 = chunk * span, t1 = t0 + span < T ? t0 + span : T;
  double v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = 0.0;
  for (int t = t0 + threadIdx.x; t < t1; t += 256) {
    double e[C], s[C];
    const bool in = t < len;
#pragma unroll
    for (int i = 0; i < C; ++i) {
      e[i] = in ? (double)a.est[((size_t)m * C + i) * T + t] : 0.0;
      s[i] = (double)a.src[((size_t)m * C + i) * T + t];
    }
#pragma unroll
    for (int i = 0; i < C; ++i) {
      v[i] += e[i];                       // SE
      v[C + i] += in ? s[i] : 0.0;        // SSv
      v[2 * C + i] += s[i];               // SSa (all t: pit_criterion.py:42)
      v[3 * C + i] += e[i] * e[i];        // EE
      v[4 * C + i] += in ? s[i] * s[i] : 0.0;   // TT
#pragma unroll
      for (int j = 0; j < C; ++j) v[5 * C + i * C + j] += e[i] * (in ? s[j] : 0.0);   // ES
    }
  }
  block_sum_d<NV>(v, red);
  if (threadIdx.x == 0) {
    double* o = a.slab + ((size_t)m * a.chunks + chunk) * NV;
#pragma unroll
    for (int i = 0; i < NV; ++i) o[i] = v[i];
  }
}

template <int C>
__global__ __launch_bounds__(256) void pit_final_kernel(PitArgs a) {
  constexpr int NV = 5 * C + C * C;
  __shared__ double red[4];
  double lsum = 0.0;
  for (int m = threadIdx.x; m < a.M; m += 256) {
    double v[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = 0.0;
    for (int ch = 0; ch < a.chunks; ++ch) {
      const double* p = a.slab + ((size_t)m * a.chunks + ch) * NV;
#pragma unroll
      for (int i = 0; i < NV; ++i) v[i] += p[i];
    }
    const double n = (double)a.lengths[m];
    double eb[C], sb[C], Ee[C], Et[C], D[C][C];
#pragma unroll
    for (int i = 0; i < C; ++i) {
      eb[i] = v[i] / n;
      sb[i] = v[2 * C + i] / n;
    }
#pragma unroll
    for (int i = 0; i < C; ++i) {
      Ee[i] = v[3 * C + i] - 2.0 * eb[i] * v[i] + n * eb[i] * eb[i];
      Et[i] = v[4 * C + i] - 2.0 * sb[i] * v[C + i] + n * sb[i] * sb[i];
#pragma unroll
      for (int j = 0; j < C; ++j)
        D[i][j] = v[5 * C + i * C + j] - eb[i] * v[C + j] - sb[j] * v[i] + n * eb[i] * sb[j];
    }
    double snr[C][C], ratio[C][C], Pp[C][C], Ne[C][C];
#pragma unroll
    for (int i = 0; i < C; ++i)
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const double E = Et[j] + PIT_EPS;
        Pp[i][j] = D[i][j] * D[i][j] * Et[j] / (E * E);
        Ne[i][j] = Ee[i] - 2.0 * D[i][j] * D[i][j] / E + D[i][j] * D[i][j] * Et[j] / (E * E);
        ratio[i][j] = Pp[i][j] / (Ne[i][j] + PIT_EPS);
        snr[i][j] = 10.0 * log10(ratio[i][j] + PIT_EPS);
      }
    int best = 0;
    double bestv = -1e300;
    for (int p = 0; p < a.nperm; ++p) {
      double sv = 0.0;
#pragma unroll
      for (int i = 0; i < C; ++i) sv += snr[i][a.perms[p][i]];
      if (sv > bestv) { bestv = sv; best = p; }    // first maximum, like torch.argmax
    }
    const double ms = bestv / C;
    a.max_snr[m] = (float)ms;
    a.best[m] = best;
    lsum += ms;
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const int j = a.perms[best][i];
      const double E = Et[j] + PIT_EPS, Nd = Ne[i][j] + PIT_EPS;
      const double dsnr = 10.0 / (log(10.0) * (ratio[i][j] + PIT_EPS));
      const double dPp = 2.0 * D[i][j] * Et[j] / (E * E);
      const double dNe = -4.0 * D[i][j] / E + 2.0 * D[i][j] * Et[j] / (E * E);
      const double dr_dD = (dPp * Nd - Pp[i][j] * dNe) / (Nd * Nd);
      const double dr_dEe = -Pp[i][j] / (Nd * Nd);
      const double al = dsnr * dr_dD / C, be = 2.0 * dsnr * dr_dEe / C;
      const double off = -al * v[C + j] / n - be * eb[i];
      float* cf = a.coef + ((size_t)m * C + i) * 4;
      cf[0] = (float)al;
      cf[1] = (float)be;
      cf[2] = (float)off;
      cf[3] = (float)j;
    }
  }
  double l1[1] = {lsum};
  block_sum_d<1>(l1, red);
  if (threadIdx.x == 0) a.loss[0] = (float)(-l1[0] / a.M);
}

// C > 8: the same per-(utterance, chunk) sums as pit_stats_kernel for a runtime C <= CW,
// with C*(C+5) values: the chunk is staged through LDS 256 samples at a time and each
// thread owns one or two of the values, summed in sample order (fp64)
template <int CW>
__global__ __launch_bounds__(256) void pit_stats_wide_kernel(PitArgs a) {
  constexpr int SUB = 256;
  __shared__ float se[CW][SUB], sv[CW][SUB];
  const int C = a.C, NV = 5 * C + C * C;
  const int m = blockIdx.y, chunk = blockIdx.x, tid = threadIdx.x;
  const int T = a.T;
  const long len = a.lengths[m];
  const int span = (T + a.chunks - 1) / a.chunks;
  const int t0 = chunk * span, t1 = t0 + span < T ? t0 + span : T;
  // value v: kind (0 SE, 1 SSv, 2 SSa, 3 EE, 4 TT, 5 ES), estimate i, source j
  int kind[2], vi[2], vj[2];
  double acc[2] = {0.0, 0.0};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int v = tid + 256 * u;
    kind[u] = v < 5 * C ? v / C : (v < NV ? 5 : -1);
    vi[u] = v < 5 * C ? v % C : (v - 5 * C) / C;
    vj[u] = v < 5 * C ? v % C : (v - 5 * C) % C;
  }
  for (int tb = t0; tb < t1; tb += SUB) {
    __syncthreads();
    for (int idx = tid; idx < C * SUB; idx += 256) {
      const int i = idx / SUB, tt = idx % SUB, t = tb + tt;
      const bool inT = t < t1;
      se[i][tt] = inT && t < len ? a.est[((size_t)m * C + i) * T + t] : 0.f;
      sv[i][tt] = inT ? a.src[((size_t)m * C + i) * T + t] : 0.f;
    }
    __syncthreads();
    const int n = t1 - tb < SUB ? t1 - tb : SUB;
    const int nin = len - tb <= 0 ? 0 : (len - tb < n ? (int)(len - tb) : n);   // samples with t < len
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = vi[u], j = vj[u];
      double x = acc[u];
      switch (kind[u]) {
        case 0: for (int tt = 0; tt < n; ++tt) x += (double)se[i][tt]; break;                        // SE
        case 1: for (int tt = 0; tt < nin; ++tt) x += (double)sv[i][tt]; break;                      // SSv
        case 2: for (int tt = 0; tt < n; ++tt) x += (double)sv[i][tt]; break;                        // SSa
        case 3: for (int tt = 0; tt < n; ++tt) x += (double)se[i][tt] * (double)se[i][tt]; break;    // EE
        case 4: for (int tt = 0; tt < nin; ++tt) x += (double)sv[i][tt] * (double)sv[i][tt]; break;  // TT
        case 5: for (int tt = 0; tt < nin; ++tt) x += (double)se[i][tt] * (double)sv[j][tt]; break;  // ES
        default: break;
      }
      acc[u] = x;
    }
  }
  double* o = a.slab + ((size_t)m * a.chunks + chunk) * NV;
#pragma unroll
  for (int u = 0; u < 2; ++u)
    if (kind[u] >= 0) o[tid + 256 * u] = acc[u];
}

// maximum-weight perfect matching of estimates (rows) to sources (columns) of w, in fp64:
// the Hungarian algorithm with potentials (minimising -w), O(C^3); perm[i] = source of i
template <int C>
CTN_DEV void pit_assign_max(const double (*w)[C], int* perm) {
  double u[C + 1], v[C + 1], minv[C + 1];
  int p[C + 1], way[C + 1];
  bool used[C + 1];
  for (int j = 0; j <= C; ++j) u[j] = v[j] = 0.0, p[j] = way[j] = 0;
  for (int i = 1; i <= C; ++i) {
    p[0] = i;
    int j0 = 0;
    for (int j = 0; j <= C; ++j) minv[j] = 1e300, used[j] = false;
    do {
      used[j0] = true;
      const int i0 = p[j0];
      double delta = 1e300;
      int j1 = 0;
      for (int j = 1; j <= C; ++j)
        if (!used[j]) {
          const double cur = -w[i0 - 1][j - 1] - u[i0] - v[j];
          if (cur < minv[j]) minv[j] = cur, way[j] = j0;
          if (minv[j] < delta) delta = minv[j], j1 = j;
        }
      for (int j = 0; j <= C; ++j) {
        if (used[j]) u[p[j]] += delta, v[j] -= delta;
        else minv[j] -= delta;
      }
      j0 = j1;
    } while (p[j0] != 0);
    do {
      const int j1 = way[j0];
      p[j0] = p[j1];
      j0 = j1;
    } while (j0);
  }
  for (int j = 1; j <= C; ++j) perm[p[j] - 1] = j - 1;
}

// lexicographic rank of a permutation of range(C) (itertools.permutations order)
CTN_DEV long pit_rank(const int* perm, int C) {
  long r = 0, f = 1;
  for (int i = 2; i < C; ++i) f *= i;   // (C-1)!
  unsigned used = 0;
  for (int i = 0; i < C; ++i) {
    int smaller = 0;
    for (int v = 0; v < perm[i]; ++v) smaller += !((used >> v) & 1u);
    used |= 1u << perm[i];
    r += smaller * f;
    if (C - 1 - i > 0) f /= C - 1 - i;
  }
  return r;
}

// permutation of range(C) with lexicographic rank p (itertools.permutations order)
CTN_DEV void pit_decode(long p, int C, int* out) {
  long f = 1;
  for (int i = 2; i < C; ++i) f *= i;   // (C-1)!
  unsigned used = 0;
  for (int i = 0; i < C; ++i) {
    const int d = (int)(p / f);
    p %= f;
    if (C - 1 - i > 0) f /= C - 1 - i;
    int v = 0;
    for (int cnt = -1; v < C; ++v)
      if (!((used >> v) & 1u) && ++cnt == d) break;
    used |= 1u << v;
    out[i] = v;
  }
}

// 5 <= C <= 16: one workgroup per utterance (pit_criterion.py:41-75 for one row)
template <int C>
__global__ __launch_bounds__(256) void pit_final_wide_kernel(PitArgs a) {
  constexpr int NV = 5 * C + C * C;
  __shared__ double v[NV], snr[C][C], ratio[C][C], Pp[C][C], Ne[C][C], Dm[C][C], Et[C], eb[C];
  __shared__ double bv[256];
  __shared__ long bp[256];
  const int m = blockIdx.x, tid = threadIdx.x;
  for (int i = tid; i < NV; i += 256) {   // chunk partials in chunk order, as pit_final
    double s = 0.0;
    for (int ch = 0; ch < a.chunks; ++ch) s += a.slab[((size_t)m * a.chunks + ch) * NV + i];
    v[i] = s;
  }
  __syncthreads();
  const double n = (double)a.lengths[m];
  if (tid < C * C) {
    const int i = tid / C, j = tid % C;
    const double ebi = v[i] / n, sbj = v[2 * C + j] / n;
    const double Ee = v[3 * C + i] - 2.0 * ebi * v[i] + n * ebi * ebi;
    const double Etj = v[4 * C + j] - 2.0 * sbj * v[C + j] + n * sbj * sbj;
    const double D = v[5 * C + i * C + j] - ebi * v[C + j] - sbj * v[i] + n * ebi * sbj;
    const double E = Etj + PIT_EPS;
    Pp[i][j] = D * D * Etj / (E * E);
    Ne[i][j] = Ee - 2.0 * D * D / E + D * D * Etj / (E * E);
    ratio[i][j] = Pp[i][j] / (Ne[i][j] + PIT_EPS);
    snr[i][j] = 10.0 * log10(ratio[i][j] + PIT_EPS);
    Dm[i][j] = D;
    if (i == 0) Et[j] = Etj;
    if (j == 0) eb[i] = ebi;
  }
  __syncthreads();
  double best = -1e300;
  long bi = 0;
  if constexpr (C <= 10) {
    long nperm = 1;
    for (int i = 2; i <= C; ++i) nperm *= i;
    bi = nperm;
    for (long p = tid; p < nperm; p += 256) {
      int pm[C];
      pit_decode(p, C, pm);
      double sv = 0.0;
#pragma unroll
      for (int i = 0; i < C; ++i) sv += snr[i][pm[i]];
      if (sv > best) { best = sv; bi = p; }   // ascending p: first maximum of this thread
    }
    bv[tid] = best;
    bp[tid] = bi;
    __syncthreads();
  }
  if (tid == 0) {
    if constexpr (C <= 10) {
      for (int t = 1; t < 256; ++t)   // first maximum over all ranks, like torch.argmax
        if (bv[t] > best || (bv[t] == best && bp[t] < bi)) { best = bv[t]; bi = bp[t]; }
    } else {   // the same maximum as a linear assignment
      int pm[C];
      pit_assign_max<C>(snr, pm);
      best = 0.0;
      for (int i = 0; i < C; ++i) best += snr[i][pm[i]];
      bi = pit_rank(pm, C);
    }
    const double ms = best / C;
    a.max_snr[m] = (float)ms;
    a.best[m] = bi;
    a.msd[m] = ms;
    int pm[C];
    pit_decode(bi, C, pm);
    for (int i = 0; i < C; ++i) {
      const int j = pm[i];
      const double E = Et[j] + PIT_EPS, Nd = Ne[i][j] + PIT_EPS, D = Dm[i][j];
      const double dsnr = 10.0 / (log(10.0) * (ratio[i][j] + PIT_EPS));
      const double dPp = 2.0 * D * Et[j] / (E * E);
      const double dNe = -4.0 * D / E + 2.0 * D * Et[j] / (E * E);
      const double dr_dD = (dPp * Nd - Pp[i][j] * dNe) / (Nd * Nd);
      const double dr_dEe = -Pp[i][j] / (Nd * Nd);
      const double al = dsnr * dr_dD / C, be = 2.0 * dsnr * dr_dEe / C;
      const double off = -al * v[C + j] / n - be * eb[i];
      float* cf = a.coef + ((size_t)m * C + i) * 4;
      cf[0] = (float)al;
      cf[1] = (float)be;
      cf[2] = (float)off;
      cf[3] = (float)j;
    }
  }
}

// loss = -mean over utterances of max_snr (pit_criterion.py:22), the summation order of pit_final
__global__ __launch_bounds__(256) void pit_loss_kernel(PitArgs a) {
  __shared__ double red[4];
  double l1[1] = {0.0};
  for (int m = threadIdx.x; m < a.M; m += 256) l1[0] += a.msd[m];
  block_sum_d<1>(l1, red);
  if (threadIdx.x == 0) a.loss[0] = (float)(-l1[0] / a.M);
}

template <int C>
__global__ __launch_bounds__(256) void pit_reorder_kernel(PitArgs a) {
  const long total = (long)a.M * a.T;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int m = (int)(i / a.T), t = (int)(i % a.T);
    const bool in = t < a.lengths[m];
    float e[C];
#pragma unroll
    for (int c = 0; c < C; ++c) e[c] = in ? a.est[((size_t)m * C + c) * a.T + t] : 0.f;
    if (a.reordered) {
      const int b = (int)a.best[m];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        // reorder_source[b, c] = source[b, perm[c]] (pit_criterion.py:97)
        const int pc = C <= 4 ? a.perms[b][c] : (int)a.coef[((size_t)m * C + c) * 4 + 3];
        float val = e[0];
#pragma unroll
        for (int q = 1; q < C; ++q) val = pc == q ? e[q] : val;
        a.reordered[((size_t)m * C + c) * a.T + t] = val;
      }
    }
    if (a.est_inplace && !in)
#pragma unroll
      for (int c = 0; c < C; ++c) a.est_inplace[((size_t)m * C + c) * a.T + t] = 0.f;
  }
}

template <int C>
__global__ __launch_bounds__(256) void pit_bwd_kernel(PitArgs a) {
  const long total = (long)a.M * C * a.T;
  const float gl = a.g_loss ? a.g_loss[0] : 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int t = (int)(i % a.T);
    const int mi = (int)(i / a.T), m = mi / C;
    float g = 0.f;
    if (t < a.lengths[m]) {
      const float scale = (a.g_maxsnr ? a.g_maxsnr[m] : 0.f) - gl / (float)a.M;
      const float* cf = a.coef + (size_t)mi * 4;
      const int j = (int)cf[3];
      const float s = a.src[((size_t)m * C + j) * a.T + t];
      const float e = a.est[i];
      g = scale * (cf[0] * s + cf[1] * e + cf[2]);
    }
    a.gest[i] = g;
  }
}

constexpr int PIT_CW = 16;   // largest C (pit_stats_wide_kernel's staging arrays)

template <int C>
static hipError_t pit_fwd_c(const PitArgs& a, hipStream_t s) {
  if constexpr (C <= 8) hipLaunchKernelGGL(pit_stats_kernel<C>, dim3(a.chunks, a.M), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(pit_stats_wide_kernel<PIT_CW>, dim3(a.chunks, a.M), dim3(256), 0, s, a);
  if constexpr (C <= 4) {
    hipLaunchKernelGGL(pit_final_kernel<C>, dim3(1), dim3(256), 0, s, a);
  } else {
    if (!a.msd) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pit_final_wide_kernel<C>, dim3(a.M), dim3(256), 0, s, a);
    hipLaunchKernelGGL(pit_loss_kernel, dim3(1), dim3(256), 0, s, a);
  }
  long total = (long)a.M * a.T;
  int g = (int)((total + 255) / 256);
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(pit_reorder_kernel<C>, dim3(g), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int C>
static hipError_t pit_bwd_c(const PitArgs& a, hipStream_t s) {
  long total = (long)a.M * C * a.T;
  int g = (int)((total + 255) / 256);
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(pit_bwd_kernel<C>, dim3(g), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_pit_forward(const PitArgs& a, hipStream_t s) {
  switch (a.C) {
    case 1: return pit_fwd_c<1>(a, s);
    case 2: return pit_fwd_c<2>(a, s);
    case 3: return pit_fwd_c<3>(a, s);
    case 4: return pit_fwd_c<4>(a, s);
    case 5: return pit_fwd_c<5>(a, s);
    case 6: return pit_fwd_c<6>(a, s);
    case 7: return pit_fwd_c<7>(a, s);
    case 8: return pit_fwd_c<8>(a, s);
    case 9: return pit_fwd_c<9>(a, s);
    case 10: return pit_fwd_c<10>(a, s);
    case 11: return pit_fwd_c<11>(a, s);
    case 12: return pit_fwd_c<12>(a, s);
    case 13: return pit_fwd_c<13>(a, s);
    case 14: return pit_fwd_c<14>(a, s);
    case 15: return pit_fwd_c<15>(a, s);
    case 16: return pit_fwd_c<16>(a, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_pit_backward(const PitArgs& a, hipStream_t s) {
  switch (a.C) {
    case 1: return pit_bwd_c<1>(a, s);
    case 2: return pit_bwd_c<2>(a, s);
    case 3: return pit_bwd_c<3>(a, s);
    case 4: return pit_bwd_c<4>(a, s);
    case 5: return pit_bwd_c<5>(a, s);
    case 6: return pit_bwd_c<6>(a, s);
    case 7: return pit_bwd_c<7>(a, s);
    case 8: return pit_bwd_c<8>(a, s);
    case 9: return pit_bwd_c<9>(a, s);
    case 10: return pit_bwd_c<10>(a, s);
    case 11: return pit_bwd_c<11>(a, s);
    case 12: return pit_bwd_c<12>(a, s);
    case 13: return pit_bwd_c<13>(a, s);
    case 14: return pit_bwd_c<14>(a, s);
    case 15: return pit_bwd_c<15>(a, s);
    case 16: return pit_bwd_c<16>(a, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace ctn
