// Stand-alone layers of the separator on frame rows (gfx950): the public module
// forwards that the fused TemporalBlock / codec kernels otherwise run inside
// themselves — GlobalLayerNorm / ChannelwiseLayerNorm (conv_tasnet.py:307-355),
// nn.PReLU with one shared alpha (:218,253), the dilated depthwise conv with its
// Chomp1d (:262-265, :275-289), bias-free 1x1 convs (:169, :185, :215, :270; on the
// GEMM kernels of ctn_gemm.hip) and the mask nonlinearity (:202-208) — each with
// its backward.  Used by TemporalConvNet.forward, DepthwiseSeparableConv.forward and
// the norm modules' forward when they are called on their own.
//
// Layout as everywhere: rows [M*Kp][C], padded rows zero in every
// output.  Statistics and reductions in fp64/fp32 with fixed-order partials (no
// atomics): results are bitwise reproducible.
#include <math.h>

#include "../../include/ctn.h"
#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {
namespace {

constexpr int LY_RB = 64;     // rows per block of the column / group partial reductions
constexpr int LY_NT = 256;

template <typename T> struct Io {
  static CTN_DEV float ld(const T* p) { return ld1<T>(p); }
  static CTN_DEV void st(T* p, float v) { st1<T>(p, v); }
};

CTN_DEV long ly_rows(const Rows& g) { return (long)g.M * g.Kp; }

// ---------------------------------------------------------------------------
// layer norms
// ---------------------------------------------------------------------------
// cLN: one wave per frame row -> (mean, rstd) over the C channels
template <typename T>
__global__ __launch_bounds__(LY_NT) void ln_row_stats_kernel(const T* x, int C, Rows g, float eps, float2* stats) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * (LY_NT / 64) + (threadIdx.x >> 6);
  if (row >= ly_rows(g)) return;
  double s = 0.0, ss = 0.0;
  for (int c = lane; c < C; c += 64) {
    const double v = Io<T>::ld(x + row * C + c);
    s += v;
    ss += v * v;
  }
  s = wave_sum(s);
  ss = wave_sum(ss);
  if (lane == 0) {
    const double mean = s / C;
    double var = ss / C - mean * mean;
    if (var < 0.0) var = 0.0;
    stats[row] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
  }
}

// gLN: block (m, b) sums rows [b*LY_RB, +LY_RB) of utterance m (valid frames only)
template <typename T>
__global__ __launch_bounds__(LY_NT) void ln_utt_partials_kernel(const T* x, int C, Rows g, int nb, double2* slab) {
  __shared__ double red[2 * (LY_NT / 64)];
  const int m = blockIdx.x / nb, b = blockIdx.x % nb;
  const int k0 = b * LY_RB, k1 = min(g.K, k0 + LY_RB);
  double v[2] = {0.0, 0.0};
  const long base = (long)m * g.Kp;
  for (long i = (long)k0 * C + threadIdx.x; i < (long)k1 * C; i += LY_NT) {
    const double a = Io<T>::ld(x + base * C + i);
    v[0] += a;
    v[1] += a * a;
  }
  block_sum_d<2>(v, red);
  if (threadIdx.x == 0) slab[blockIdx.x] = make_double2(v[0], v[1]);
}

// y = gamma (x - mean) rstd + beta; padded rows 0
template <typename T, int NK>
__global__ __launch_bounds__(LY_NT) void ln_apply_kernel(const T* x, int C, Rows g, const float2* stats,
                                                         const float* gamma, const float* beta, T* y) {
  const long n = ly_rows(g) * C;
  for (long i = (long)blockIdx.x * LY_NT + threadIdx.x; i < n; i += (long)gridDim.x * LY_NT) {
    const long row = i / C;
    const int c = (int)(i - row * C);
    const int k = (int)(row % g.Kp);
    float o = 0.f;
    if (k < g.K) {
      const float2 st = stats[NK == NORM_GLN ? row / g.Kp : row];
      o = (Io<T>::ld(x + i) - st.x) * st.y * gamma[c] + beta[c];
    }
    Io<T>::st(y + i, o);
  }
}

// backward group sums of (g*gamma, g*gamma*xhat): cLN per row (means written
// directly), gLN per (utterance, row block) partials
template <typename T>
__global__ __launch_bounds__(LY_NT) void ln_row_gsums_kernel(const T* x, const T* gy, int C, Rows g,
                                                             const float2* stats, const float* gamma, float2* sums) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * (LY_NT / 64) + (threadIdx.x >> 6);
  if (row >= ly_rows(g)) return;
  const float2 st = stats[row];
  double s1 = 0.0, s2 = 0.0;
  if (row % g.Kp < g.K)
    for (int c = lane; c < C; c += 64) {
      const double gg = (double)Io<T>::ld(gy + row * C + c) * gamma[c];
      const double xh = ((double)Io<T>::ld(x + row * C + c) - st.x) * st.y;
      s1 += gg;
      s2 += gg * xh;
    }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) sums[row] = make_float2((float)(s1 / C), (float)(s2 / C));
}

template <typename T>
__global__ __launch_bounds__(LY_NT) void ln_utt_gpartials_kernel(const T* x, const T* gy, int C, Rows g, int nb,
                                                                 const float2* stats, const float* gamma,
                                                                 double2* slab) {
  __shared__ double red[2 * (LY_NT / 64)];
  const int m = blockIdx.x / nb, b = blockIdx.x % nb;
  const int k0 = b * LY_RB, k1 = min(g.K, k0 + LY_RB);
  const float2 st = stats[m];
  double v[2] = {0.0, 0.0};
  const long base = (long)m * g.Kp * C;
  for (long i = (long)k0 * C + threadIdx.x; i < (long)k1 * C; i += LY_NT) {
    const int c = (int)(i % C);
    const double gg = (double)Io<T>::ld(gy + base + i) * gamma[c];
    v[0] += gg;
    v[1] += gg * (((double)Io<T>::ld(x + base + i) - st.x) * st.y);
  }
  block_sum_d<2>(v, red);
  if (threadIdx.x == 0) slab[blockIdx.x] = make_double2(v[0], v[1]);
}

// dx = rstd (g gamma - mean(g gamma) - xhat mean(g gamma xhat)); padded rows 0
template <typename T, int NK>
__global__ __launch_bounds__(LY_NT) void ln_dx_kernel(const T* x, const T* gy, int C, Rows g, const float2* stats,
                                                      const float2* sums, const float* gamma, T* gx) {
  const long n = ly_rows(g) * C;
  for (long i = (long)blockIdx.x * LY_NT + threadIdx.x; i < n; i += (long)gridDim.x * LY_NT) {
    const long row = i / C;
    const int c = (int)(i - row * C);
    float o = 0.f;
    if (row % g.Kp < g.K) {
      const long gi = NK == NORM_GLN ? row / g.Kp : row;
      const float2 st = stats[gi], sm = sums[gi];
      const float xh = (Io<T>::ld(x + i) - st.x) * st.y;
      o = st.y * (Io<T>::ld(gy + i) * gamma[c] - sm.x - xh * sm.y);
    }
    Io<T>::st(gx + i, o);
  }
}

// column partials over LY_RB-row blocks: part[blk][c] = sum g*xhat, part[blk][C+c] = sum g
template <typename T, int NK>
__global__ __launch_bounds__(LY_NT) void ln_col_partials_kernel(const T* x, const T* gy, int C, Rows g,
                                                                const float2* stats, float* part) {
  const long r0 = (long)blockIdx.x * LY_RB;
  for (int c = threadIdx.x; c < C; c += LY_NT) {
    float pg = 0.f, pb = 0.f;
    for (int r = 0; r < LY_RB; ++r) {
      const long row = r0 + r;
      if (row % g.Kp >= g.K) continue;
      const float2 st = stats[NK == NORM_GLN ? row / g.Kp : row];
      const float gv = Io<T>::ld(gy + row * C + c);
      pg += gv * ((Io<T>::ld(x + row * C + c) - st.x) * st.y);
      pb += gv;
    }
    part[(size_t)blockIdx.x * 2 * C + c] = pg;
    part[(size_t)blockIdx.x * 2 * C + C + c] = pb;
  }
}

// ---------------------------------------------------------------------------
// PReLU (shared alpha)
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(LY_NT) void prelu_fwd_kernel(const T* x, long n, const float* alpha, T* y) {
  const float a = alpha[0];
  for (long i = (long)blockIdx.x * LY_NT + threadIdx.x; i < n; i += (long)gridDim.x * LY_NT)
    Io<T>::st(y + i, prelu(Io<T>::ld(x + i), a));
}

// gx = g * PReLU'(x); part[blk] = sum g * d PReLU / d alpha over the block's LY_RB rows
template <typename T>
__global__ __launch_bounds__(LY_NT) void prelu_bwd_kernel(const T* x, const T* gy, int C, const float* alpha, T* gx,
                                                          float* part) {
  __shared__ double red[LY_NT / 64];
  const float a = alpha[0];
  const long i0 = (long)blockIdx.x * LY_RB * C;
  double acc[1] = {0.0};
  for (long i = i0 + threadIdx.x; i < i0 + (long)LY_RB * C; i += LY_NT) {
    const float xv = Io<T>::ld(x + i), gv = Io<T>::ld(gy + i);
    Io<T>::st(gx + i, gv * prelu_dx(xv, a));
    acc[0] += (double)(gv * prelu_da(xv));
  }
  block_sum_d<1>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = (float)acc[0];
}

// ---------------------------------------------------------------------------
// depthwise dilated conv: y[k][c] = sum_p w[c][p] x[k - pad + p*dil][c] (0 outside
// [0,K)); pad = (P-1)*dil (causal: symmetric pad + Chomp1d) or (P-1)*dil/2
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(LY_NT) void dwc_fwd_kernel(const T* x, int C, Rows g, int P, int dil, int pad,
                                                        const float* w, T* y) {
  const long n = ly_rows(g) * C;
  for (long i = (long)blockIdx.x * LY_NT + threadIdx.x; i < n; i += (long)gridDim.x * LY_NT) {
    const long row = i / C;
    const int c = (int)(i - row * C);
    const int k = (int)(row % g.Kp);
    const long base = row - k;
    float o = 0.f;
    if (k < g.K)
      for (int p = 0; p < P; ++p) {
        const int kk = k - pad + p * dil;
        if (kk >= 0 && kk < g.K) o += w[c * P + p] * Io<T>::ld(x + (base + kk) * C + c);
      }
    Io<T>::st(y + i, o);
  }
}

template <typename T>
__global__ __launch_bounds__(LY_NT) void dwc_bwd_x_kernel(const T* gy, int C, Rows g, int P, int dil, int pad,
                                                          const float* w, T* gx) {
  const long n = ly_rows(g) * C;
  for (long i = (long)blockIdx.x * LY_NT + threadIdx.x; i < n; i += (long)gridDim.x * LY_NT) {
    const long row = i / C;
    const int c = (int)(i - row * C);
    const int k = (int)(row % g.Kp);
    const long base = row - k;
    float o = 0.f;
    if (k < g.K)
      for (int p = 0; p < P; ++p) {
        const int ko = k + pad - p * dil;   // output frame whose tap p reads frame k
        if (ko >= 0 && ko < g.K) o += w[c * P + p] * Io<T>::ld(gy + (base + ko) * C + c);
      }
    Io<T>::st(gx + i, o);
  }
}

// part[blk][c*P + p] = sum over the block's rows of gy[k][c] * x[k - pad + p*dil][c]
template <typename T>
__global__ __launch_bounds__(LY_NT) void dwc_bwd_w_kernel(const T* x, const T* gy, int C, Rows g, int P, int dil,
                                                          int pad, float* part) {
  const long r0 = (long)blockIdx.x * LY_RB;
  for (int cp = threadIdx.x; cp < C * P; cp += LY_NT) {
    const int c = cp / P, p = cp % P;
    float acc = 0.f;
    for (int r = 0; r < LY_RB; ++r) {
      const long row = r0 + r;
      const int k = (int)(row % g.Kp);
      if (k >= g.K) continue;
      const int kk = k - pad + p * dil;
      if (kk < 0 || kk >= g.K) continue;
      acc += Io<T>::ld(gy + row * C + c) * Io<T>::ld(x + (row - k + kk) * C + c);
    }
    part[(size_t)blockIdx.x * C * P + cp] = acc;
  }
}

// ---------------------------------------------------------------------------
// mask nonlinearity over S speakers: score rows [rows][S*N], channel s*N + n
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(LY_NT) void mask_fwd_kernel(const T* score, int S, int N, Rows g, int type, T* mask) {
  const long n = ly_rows(g) * N;
  for (long i = (long)blockIdx.x * LY_NT + threadIdx.x; i < n; i += (long)gridDim.x * LY_NT) {
    const long row = i / N;
    const int j = (int)(i - row * N);
    const bool valid = row % g.Kp < g.K;
    const T* s = score + row * S * N + j;
    T* o = mask + row * S * N + j;
    if (type == CTN_MASK_RELU || !valid) {
      for (int c = 0; c < S; ++c) Io<T>::st(o + c * N, valid ? fmaxf(Io<T>::ld(s + c * N), 0.f) : 0.f);
    } else {
      float mx = -INFINITY;
      for (int c = 0; c < S; ++c) mx = fmaxf(mx, Io<T>::ld(s + c * N));
      float z = 0.f;
      for (int c = 0; c < S; ++c) z += expf(Io<T>::ld(s + c * N) - mx);
      for (int c = 0; c < S; ++c) Io<T>::st(o + c * N, expf(Io<T>::ld(s + c * N) - mx) / z);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(LY_NT) void mask_bwd_kernel(const T* score, const T* gmask, int S, int N, Rows g,
                                                         int type, T* gscore) {
  const long n = ly_rows(g) * N;
  for (long i = (long)blockIdx.x * LY_NT + threadIdx.x; i < n; i += (long)gridDim.x * LY_NT) {
    const long row = i / N;
    const int j = (int)(i - row * N);
    const bool valid = row % g.Kp < g.K;
    const T* s = score + row * S * N + j;
    const T* gm = gmask + row * S * N + j;
    T* o = gscore + row * S * N + j;
    if (!valid) {
      for (int c = 0; c < S; ++c) Io<T>::st(o + c * N, 0.f);
    } else if (type == CTN_MASK_RELU) {
      for (int c = 0; c < S; ++c) Io<T>::st(o + c * N, Io<T>::ld(s + c * N) > 0.f ? Io<T>::ld(gm + c * N) : 0.f);
    } else {
      float mx = -INFINITY;
      for (int c = 0; c < S; ++c) mx = fmaxf(mx, Io<T>::ld(s + c * N));
      float z = 0.f;
      for (int c = 0; c < S; ++c) z += expf(Io<T>::ld(s + c * N) - mx);
      float dot = 0.f;
      for (int c = 0; c < S; ++c) dot += Io<T>::ld(gm + c * N) * (expf(Io<T>::ld(s + c * N) - mx) / z);
      for (int c = 0; c < S; ++c) {
        const float m = expf(Io<T>::ld(s + c * N) - mx) / z;
        Io<T>::st(o + c * N, m * (Io<T>::ld(gm + c * N) - dot));
      }
    }
  }
}

int ew_grid(long n) {
  long b = (n + LY_NT - 1) / LY_NT;
  if (b > 4096) b = 4096;
  return b < 1 ? 1 : (int)b;
}

template <typename T>
hipError_t norm_fwd_t(const LayerArgs& a, hipStream_t s) {
  const T* x = reinterpret_cast<const T*>(a.x);
  if (a.norm == NORM_CLN) {
    hipLaunchKernelGGL((ln_row_stats_kernel<T>), dim3(ceil_div(a.g.rows(), LY_NT / 64)), dim3(LY_NT), 0, s, x, a.C, a.g,
                       a.eps, a.stats);
  } else {
    const int nb = ceil_div(a.g.K, LY_RB);
    hipLaunchKernelGGL((ln_utt_partials_kernel<T>), dim3(a.g.M * nb), dim3(LY_NT), 0, s, x, a.C, a.g, nb, a.slab);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = launch_stats_finalize(a.slab, a.g.M, nb, (double)a.g.K * a.C, 0, a.eps, a.stats, s);
    if (e != hipSuccess) return e;
  }
  const int gb = ew_grid(a.g.rows() * a.C);
  if (a.norm == NORM_CLN)
    hipLaunchKernelGGL((ln_apply_kernel<T, NORM_CLN>), dim3(gb), dim3(LY_NT), 0, s, x, a.C, a.g, a.stats, a.gamma,
                       a.beta, reinterpret_cast<T*>(a.y));
  else
    hipLaunchKernelGGL((ln_apply_kernel<T, NORM_GLN>), dim3(gb), dim3(LY_NT), 0, s, x, a.C, a.g, a.stats, a.gamma,
                       a.beta, reinterpret_cast<T*>(a.y));
  return hipGetLastError();
}

template <typename T>
hipError_t norm_bwd_t(const LayerArgs& a, hipStream_t s) {
  const T* x = reinterpret_cast<const T*>(a.x);
  const T* gy = reinterpret_cast<const T*>(a.gy);
  T* gx = reinterpret_cast<T*>(a.gx);
  hipError_t e;
  if (a.norm == NORM_CLN) {
    hipLaunchKernelGGL((ln_row_gsums_kernel<T>), dim3(ceil_div(a.g.rows(), LY_NT / 64)), dim3(LY_NT), 0, s, x, gy,
                       a.C, a.g, a.stats, a.gamma, a.sums);
  } else {
    const int nb = ceil_div(a.g.K, LY_RB);
    hipLaunchKernelGGL((ln_utt_gpartials_kernel<T>), dim3(a.g.M * nb), dim3(LY_NT), 0, s, x, gy, a.C, a.g, nb,
                       a.stats, a.gamma, a.slab);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = launch_stats_finalize(a.slab, a.g.M, nb, (double)a.g.K * a.C, 1, 0.f, a.sums, s)) != hipSuccess) return e;
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int gb = ew_grid(a.g.rows() * a.C);
  const int nblk = (int)(a.g.rows() / LY_RB);
  if (a.norm == NORM_CLN) {
    hipLaunchKernelGGL((ln_dx_kernel<T, NORM_CLN>), dim3(gb), dim3(LY_NT), 0, s, x, gy, a.C, a.g, a.stats, a.sums,
                       a.gamma, gx);
    hipLaunchKernelGGL((ln_col_partials_kernel<T, NORM_CLN>), dim3(nblk), dim3(LY_NT), 0, s, x, gy, a.C, a.g, a.stats,
                       a.part);
  } else {
    hipLaunchKernelGGL((ln_dx_kernel<T, NORM_GLN>), dim3(gb), dim3(LY_NT), 0, s, x, gy, a.C, a.g, a.stats, a.sums,
                       a.gamma, gx);
    hipLaunchKernelGGL((ln_col_partials_kernel<T, NORM_GLN>), dim3(nblk), dim3(LY_NT), 0, s, x, gy, a.C, a.g, a.stats,
                       a.part);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  SlabBatch sb{};
  sb.d[sb.nd++] = SlabDesc{a.part, a.ggamma, nblk, a.C, 2 * a.C};
  sb.d[sb.nd++] = SlabDesc{a.part + a.C, a.gbeta, nblk, a.C, 2 * a.C};
  return launch_slab_reduce(sb, a.tmp, s);
}

template <typename T>
hipError_t prelu_t(const LayerArgs& a, bool bwd, hipStream_t s) {
  const long n = a.g.rows() * a.C;
  if (!bwd) {
    hipLaunchKernelGGL((prelu_fwd_kernel<T>), dim3(ew_grid(n)), dim3(LY_NT), 0, s, reinterpret_cast<const T*>(a.x), n,
                       a.alpha, reinterpret_cast<T*>(a.y));
    return hipGetLastError();
  }
  const int nblk = (int)(a.g.rows() / LY_RB);
  hipLaunchKernelGGL((prelu_bwd_kernel<T>), dim3(nblk), dim3(LY_NT), 0, s, reinterpret_cast<const T*>(a.x),
                     reinterpret_cast<const T*>(a.gy), a.C, a.alpha, reinterpret_cast<T*>(a.gx), a.part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  SlabBatch sb{};
  sb.d[sb.nd++] = SlabDesc{a.part, a.galpha, nblk, 1, 1};
  return launch_slab_reduce(sb, a.tmp, s);
}

template <typename T>
hipError_t dwc_t(const LayerArgs& a, bool bwd, hipStream_t s) {
  const int gb = ew_grid(a.g.rows() * a.C);
  if (!bwd) {
    hipLaunchKernelGGL((dwc_fwd_kernel<T>), dim3(gb), dim3(LY_NT), 0, s, reinterpret_cast<const T*>(a.x), a.C, a.g, a.P,
                       a.dil, a.pad, a.w, reinterpret_cast<T*>(a.y));
    return hipGetLastError();
  }
  const int nblk = (int)(a.g.rows() / LY_RB);
  hipLaunchKernelGGL((dwc_bwd_x_kernel<T>), dim3(gb), dim3(LY_NT), 0, s, reinterpret_cast<const T*>(a.gy), a.C, a.g,
                     a.P, a.dil, a.pad, a.w, reinterpret_cast<T*>(a.gx));
  hipLaunchKernelGGL((dwc_bwd_w_kernel<T>), dim3(nblk), dim3(LY_NT), 0, s, reinterpret_cast<const T*>(a.x),
                     reinterpret_cast<const T*>(a.gy), a.C, a.g, a.P, a.dil, a.pad, a.part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  SlabBatch sb{};
  sb.d[sb.nd++] = SlabDesc{a.part, a.gw, nblk, a.C * a.P, a.C * a.P};
  return launch_slab_reduce(sb, a.tmp, s);
}

template <typename T>
hipError_t mask_t(const LayerArgs& a, bool bwd, hipStream_t s) {
  const int N = a.C / a.S;
  const int gb = ew_grid(a.g.rows() * N);
  if (!bwd)
    hipLaunchKernelGGL((mask_fwd_kernel<T>), dim3(gb), dim3(LY_NT), 0, s, reinterpret_cast<const T*>(a.x), a.S, N, a.g,
                       a.mask_type, reinterpret_cast<T*>(a.y));
  else
    hipLaunchKernelGGL((mask_bwd_kernel<T>), dim3(gb), dim3(LY_NT), 0, s, reinterpret_cast<const T*>(a.x),
                       reinterpret_cast<const T*>(a.gy), a.S, N, a.g, a.mask_type, reinterpret_cast<T*>(a.gx));
  return hipGetLastError();
}

}  // namespace

int layer_blocks(const Rows& g) { return (int)(g.rows() / LY_RB); }
int layer_norm_groups_nb(const Rows& g) { return ceil_div(g.K, LY_RB); }

hipError_t launch_layer(DType dt, LayerOp op, const LayerArgs& a, hipStream_t s) {
  if (a.g.Kp % LY_RB) return hipErrorInvalidValue;
  const bool f = dt == F32;
  switch (op) {
    case LAYER_NORM_FWD: return f ? norm_fwd_t<float>(a, s) : norm_fwd_t<bf16raw>(a, s);
    case LAYER_NORM_BWD: return f ? norm_bwd_t<float>(a, s) : norm_bwd_t<bf16raw>(a, s);
    case LAYER_PRELU_FWD: return f ? prelu_t<float>(a, false, s) : prelu_t<bf16raw>(a, false, s);
    case LAYER_PRELU_BWD: return f ? prelu_t<float>(a, true, s) : prelu_t<bf16raw>(a, true, s);
    case LAYER_DW_FWD: return f ? dwc_t<float>(a, false, s) : dwc_t<bf16raw>(a, false, s);
    case LAYER_DW_BWD: return f ? dwc_t<float>(a, true, s) : dwc_t<bf16raw>(a, true, s);
    case LAYER_MASK_FWD: return f ? mask_t<float>(a, false, s) : mask_t<bf16raw>(a, false, s);
    case LAYER_MASK_BWD: return f ? mask_t<float>(a, true, s) : mask_t<bf16raw>(a, true, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace ctn
