// BatchNorm1d for the TemporalBlock norms (norm_type "BN": conv_tasnet.py:290,
// chose_norm's fallback branch -> torch.nn.BatchNorm1d(H)).  Statistics are per
// CHANNEL over every valid frame row of the batch (M*K values), so on the frame-row
// layout [M*Kp][H] they are column reductions: each workgroup reduces a block of
// BN_RPB rows to one fp64 (sum, sum of squares) pair per channel, and one thread
// per channel adds the block partials in a fixed order (bitwise reproducible).
//
// The block's fused kernels then run in "identity" gLN mode: per-utterance
// statistics (0, 1) and per-channel gamma' = gamma*rstd, beta' = beta - gamma*mean*rstd
// make their norm-apply exactly BN's affine map.  BN's backward subtracts
// per-CHANNEL means, which the gLN backward cannot express, so it is applied to the
// incoming gradient here (bn_apply) and the fused backward runs with zero sums.
#include <math.h>

#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

constexpr int BN_RPB = 256;   // frame rows per partial block
constexpr int BN_NT = 256;

int bn_blocks(const Rows& g) { return (int)((g.rows() + BN_RPB - 1) / BN_RPB); }

// MODE 0: (sum x, sum x^2), x = PReLU(a)                       forward statistics
// MODE 1: (sum g, sum g*xhat), xhat = (PReLU(a) - mean) * rstd  backward sums
template <typename T, int MODE>
__global__ __launch_bounds__(BN_NT) void bn_partials_kernel(BnArgs p) {
  __shared__ double2 red[BN_NT * 8];
  const int H = p.H, cg = H / 8, nrl = BN_NT / cg;
  const int tid = threadIdx.x, c = tid % cg, rl = tid / cg;
  const int K = p.g.K, Kp = p.g.Kp;
  const long rows = p.g.rows(), r0 = (long)blockIdx.x * BN_RPB;
  const T* A = reinterpret_cast<const T*>(p.a);
  const T* G = reinterpret_cast<const T*>(p.gin);
  const float al = p.alpha[0];
  float m[8], rs[8];
  if constexpr (MODE == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float2 st = p.stats[c * 8 + e];
      m[e] = st.x;
      rs[e] = st.y;
    }
  }
  float s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = q[e] = 0.f;
  if (rl < nrl) {
    for (int i = rl; i < BN_RPB; i += nrl) {
      const long r = r0 + i;
      if (r >= rows || (int)(r % Kp) >= K) continue;
      float a[8];
      Vec8<T>::load(A + r * H + c * 8, a);
      if constexpr (MODE == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = prelu(a[e], al);
          s[e] += x;
          q[e] += x * x;
        }
      } else {
        float g[8];
        Vec8<T>::load(G + r * H + c * 8, g);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = (prelu(a[e], al) - m[e]) * rs[e];
          s[e] += g[e];
          q[e] += g[e] * xh;
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[tid * 8 + e] = make_double2((double)s[e], (double)q[e]);
  __syncthreads();
  for (int ch = tid; ch < H; ch += BN_NT) {   // channel ch = c'*8 + e', lanes rl' = 0..nrl-1 in order
    const int cc = ch / 8, e = ch % 8;
    double a = 0.0, b = 0.0;
    for (int j = 0; j < nrl; ++j) {
      const double2 v = red[(j * cg + cc) * 8 + e];
      a += v.x;
      b += v.y;
    }
    p.part[(size_t)blockIdx.x * H + ch] = make_double2(a, b);
  }
}

// One thread per channel: the block partials in a fixed order, then
//   MODE 0 (forward): batch mean / biased variance (training) or the running
//     statistics (eval) -> stats (mean, rstd); running-statistics update with the
//     unbiased variance (torch.nn.BatchNorm1d); gamma' / beta'.
//   MODE 1 (backward): sums = (mean g, mean g*xhat) (zeros in eval mode, where the
//     statistics are constants); optional dbeta = sum g, dgamma = sum g*xhat.
//   MODE 2 (backward prep): gamma' / beta' from saved stats.
// Every mode also writes the per-utterance identity (0, 1) and zero (0, 0) tables.
__global__ __launch_bounds__(BN_NT) void bn_finalize_kernel(BnFinal p, int mode) {
  const int gt = blockIdx.x * BN_NT + threadIdx.x;
  for (int m = gt; m < p.M; m += gridDim.x * BN_NT) {
    if (p.ident) p.ident[m] = make_float2(0.f, 1.f);
    if (p.zero) p.zero[m] = make_float2(0.f, 0.f);
  }
  const int c = gt;
  if (c >= p.H) return;
  double s = 0.0, q = 0.0;
  if (mode != 2 && (mode == 1 || p.training))
    for (int i = 0; i < p.nparts; ++i) {
      const double2 v = p.part[(size_t)i * p.H + c];
      s += v.x;
      q += v.y;
    }
  const double n = (double)p.count;
  if (mode == 0) {
    double mean, var;
    if (p.training) {
      mean = s / n;
      var = q / n - mean * mean;
      if (var < 0.0) var = 0.0;
      if (p.run_mean) {
        const double mo = p.momentum;
        p.run_mean[c] = (float)((1.0 - mo) * p.run_mean[c] + mo * mean);
        p.run_var[c] = (float)((1.0 - mo) * p.run_var[c] + mo * var * (n > 1.0 ? n / (n - 1.0) : 1.0));
      }
    } else {
      mean = p.run_mean[c];
      var = p.run_var[c];
    }
    const float rstd = (float)(1.0 / sqrt(var + (double)p.eps));
    p.stats[c] = make_float2((float)mean, rstd);
    p.gamma_eff[c] = p.gamma[c] * rstd;
    p.beta_eff[c] = p.beta[c] - p.gamma[c] * (float)mean * rstd;
  } else if (mode == 1) {
    p.sums[c] = p.training ? make_float2((float)(s / n), (float)(q / n)) : make_float2(0.f, 0.f);
    if (p.dbeta) p.dbeta[c] = (float)s;
    if (p.dgamma) p.dgamma[c] = (float)q;
  } else {
    const float2 st = p.stats[c];
    p.gamma_eff[c] = p.gamma[c] * st.y;
    p.beta_eff[c] = p.beta[c] - p.gamma[c] * st.x * st.y;
  }
}

// out = g - mean_c(g) - xhat * mean_c(g xhat)   [ * PReLU'(a), alpha partial ]
// Padded frame rows are written as 0.  In place (out == g) is allowed.
template <typename T, bool PR>
__global__ __launch_bounds__(BN_NT) void bn_apply_kernel(BnArgs p) {
  __shared__ double red[BN_NT / 64];
  const int H = p.H, cg = H / 8, nrl = BN_NT / cg;
  const int tid = threadIdx.x, c = tid % cg, rl = tid / cg;
  const int K = p.g.K, Kp = p.g.Kp;
  const long rows = p.g.rows(), r0 = (long)blockIdx.x * BN_RPB;
  const T* A = reinterpret_cast<const T*>(p.a);
  const T* G = reinterpret_cast<const T*>(p.gin);
  T* O = reinterpret_cast<T*>(p.gout);
  const float al = p.alpha[0];
  float m[8], rs[8], s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float2 st = p.stats[c * 8 + e], sm = p.sums[c * 8 + e];
    m[e] = st.x; rs[e] = st.y; s1[e] = sm.x; s2[e] = sm.y;
  }
  float ca = 0.f;
  if (rl < nrl) {
    for (int i = rl; i < BN_RPB; i += nrl) {
      const long r = r0 + i;
      if (r >= rows) break;
      float out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if ((int)(r % Kp) < K) {
        float a[8], g[8];
        Vec8<T>::load(A + r * H + c * 8, a);
        Vec8<T>::load(G + r * H + c * 8, g);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = (prelu(a[e], al) - m[e]) * rs[e];
          const float v = g[e] - s1[e] - xh * s2[e];
          if constexpr (PR) {
            out[e] = v * prelu_dx(a[e], al);
            ca += v * prelu_da(a[e]);
          } else {
            out[e] = v;
          }
        }
      }
      Vec8<T>::store(O + r * H + c * 8, out);
    }
  }
  if constexpr (PR) {
    double v1[1] = {(double)ca};
    block_sum_d<1>(v1, red);
    if (tid == 0) p.apart[blockIdx.x] = (float)v1[0];
  }
}

// dgamma = (dgamma' - mean * dbeta') * rstd: the gradient of BN's gamma from the
// fused kernels' identity-mode gamma' = gamma * rstd, beta' = beta - gamma*mean*rstd
__global__ __launch_bounds__(BN_NT) void bn_gamma_fix_kernel(float* dgamma, const float* dbeta, const float2* stats,
                                                             int H) {
  const int c = blockIdx.x * BN_NT + threadIdx.x;
  if (c >= H) return;
  const float2 st = stats[c];
  dgamma[c] = (dgamma[c] - st.x * dbeta[c]) * st.y;
}

static bool bn_ok(const BnArgs& p) { return p.H % 8 == 0 && p.H / 8 <= BN_NT && (BN_NT % (p.H / 8)) == 0; }

hipError_t launch_bn_partials(DType dt, const BnArgs& p, int mode, hipStream_t s) {
  if (!bn_ok(p)) return hipErrorInvalidValue;
  const dim3 grid(bn_blocks(p.g)), blk(BN_NT);
  if (dt == BF16) {
    if (mode == 0) hipLaunchKernelGGL((bn_partials_kernel<bf16raw, 0>), grid, blk, 0, s, p);
    else hipLaunchKernelGGL((bn_partials_kernel<bf16raw, 1>), grid, blk, 0, s, p);
  } else {
    if (mode == 0) hipLaunchKernelGGL((bn_partials_kernel<float, 0>), grid, blk, 0, s, p);
    else hipLaunchKernelGGL((bn_partials_kernel<float, 1>), grid, blk, 0, s, p);
  }
  return hipGetLastError();
}

hipError_t launch_bn_finalize(const BnFinal& p, int mode, hipStream_t s) {
  const int n = p.H > p.M ? p.H : p.M;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((n + BN_NT - 1) / BN_NT), dim3(BN_NT), 0, s, p, mode);
  return hipGetLastError();
}

hipError_t launch_bn_apply(DType dt, const BnArgs& p, bool prelu_bwd, hipStream_t s) {
  if (!bn_ok(p)) return hipErrorInvalidValue;
  const dim3 grid(bn_blocks(p.g)), blk(BN_NT);
  if (dt == BF16) {
    if (prelu_bwd) hipLaunchKernelGGL((bn_apply_kernel<bf16raw, true>), grid, blk, 0, s, p);
    else hipLaunchKernelGGL((bn_apply_kernel<bf16raw, false>), grid, blk, 0, s, p);
  } else {
    if (prelu_bwd) hipLaunchKernelGGL((bn_apply_kernel<float, true>), grid, blk, 0, s, p);
    else hipLaunchKernelGGL((bn_apply_kernel<float, false>), grid, blk, 0, s, p);
  }
  return hipGetLastError();
}

hipError_t launch_bn_gamma_fix(float* dgamma, const float* dbeta, const float2* stats, int H, hipStream_t s) {
  hipLaunchKernelGGL(bn_gamma_fix_kernel, dim3((H + BN_NT - 1) / BN_NT), dim3(BN_NT), 0, s, dgamma, dbeta, stats, H);
  return hipGetLastError();
}

}  // namespace ctn
