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
        const int pc = a.perms[b][c];   // reorder_source[b, c] = source[b, perm[c]] (pit_criterion.py:97)
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

template <int C>
static hipError_t pit_fwd_c(const PitArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(pit_stats_kernel<C>, dim3(a.chunks, a.M), dim3(256), 0, s, a);
  hipLaunchKernelGGL(pit_final_kernel<C>, dim3(1), dim3(256), 0, s, a);
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
  }
  return hipErrorInvalidValue;
}

hipError_t launch_pit_backward(const PitArgs& a, hipStream_t s) {
  switch (a.C) {
    case 1: return pit_bwd_c<1>(a, s);
    case 2: return pit_bwd_c<2>(a, s);
    case 3: return pit_bwd_c<3>(a, s);
    case 4: return pit_bwd_c<4>(a, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace ctn
