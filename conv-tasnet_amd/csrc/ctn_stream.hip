#include <stdlib.h>
// Streaming causal separation (gfx950): a causal cLN (or eval-mode BatchNorm)
// Conv-TasNet run frame group by frame group with per-block state, no history
// re-run (src/separate.py:35-79 with a causal model; conv_tasnet.py:176, 289).
//
// State per TemporalBlock: a ring of its depthwise-conv INPUT frames (the output of
// conv1x1 -> PReLU -> norm 1, H channels), R frames (a power of two >= (P-1)*d + the
// frames of one call), frame g at slot g & (R-1).  A call with K new frames runs
//   stream_encode : samples -> w = ReLU(U * frame) [N], cLN, bottleneck 1x1 -> x [B]
//   per block     : stream_block_in  x -> h1 = W1 x, PReLU, norm 1 -> ring
//                   stream_block_out ring taps (g - (P-1-p) d, zero before the stream
//                                    start) -> depthwise, PReLU, norm 2, W2 ., + x
//   stream_decode : mask 1x1 + ReLU/softmax, sources = w * mask, frames = sources . V^T
//   stream_ola    : overlap-add of the K frames with the previous call's tail
// Every operation of a causal model is per frame or looks back, so the concatenated
// output equals the whole-signal forward.  fp32 arithmetic and state; the 1x1 weights
// are passed TRANSPOSED ([in][out]) so that thread j reads output column j coalesced.
#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

constexpr int ST_NT = 256;        // threads per workgroup
constexpr int ST_FPB = 8;         // frames per workgroup (encode, block)
constexpr int ST_FPB_DEC = 4;     // frames per workgroup (decode: C*N scores per frame in LDS)
constexpr float ST_LN_EPS = 1e-8f;  // conv_tasnet.py:10 (cLN: inside the sqrt)

// Per-frame mean over n values held in LDS rows v[f][0..n): sums of each thread's
// strided slice, then a fixed-order tree over the 256 threads (reproducible).
template <int F>
CTN_DEV void st_row_sums(const float* v, int ld, int nf, int n, float (&out)[F], float* red) {
  const int tid = threadIdx.x;
  float s[F];
#pragma unroll
  for (int f = 0; f < F; ++f) {
    s[f] = 0.f;
    if (f < nf)
      for (int j = tid; j < n; j += ST_NT) s[f] += v[f * ld + j];
  }
#pragma unroll
  for (int f = 0; f < F; ++f) red[f * ST_NT + tid] = s[f];
  __syncthreads();
  for (int w = ST_NT / 2; w > 0; w >>= 1) {
    if (tid < w)
#pragma unroll
      for (int f = 0; f < F; ++f) red[f * ST_NT + tid] += red[f * ST_NT + tid + w];
    __syncthreads();
  }
#pragma unroll
  for (int f = 0; f < F; ++f) out[f] = red[f * ST_NT];
  __syncthreads();
}

// norm of rows v[f][0..n) in place: cLN (mean, biased variance two-pass, EPS inside the
// sqrt, then gamma/beta: conv_tasnet.py:327-329) or an affine map (eval BatchNorm folded
// into scale/shift on the host)
template <int F>
CTN_DEV void st_norm_rows(float* v, int ld, int nf, int n, int norm, const float* a, const float* b, float* red) {
  const int tid = threadIdx.x;
  if (norm == 1) {
    float mean[F], var[F];
    st_row_sums<F>(v, ld, nf, n, mean, red);
#pragma unroll
    for (int f = 0; f < F; ++f) mean[f] /= (float)n;
    // squared deviations in a scratch pass: v holds the values, red the partial sums
    float s[F];
#pragma unroll
    for (int f = 0; f < F; ++f) {
      s[f] = 0.f;
      if (f < nf)
        for (int j = tid; j < n; j += ST_NT) {
          const float dlt = v[f * ld + j] - mean[f];
          s[f] += dlt * dlt;
        }
    }
#pragma unroll
    for (int f = 0; f < F; ++f) red[f * ST_NT + tid] = s[f];
    __syncthreads();
    for (int w = ST_NT / 2; w > 0; w >>= 1) {
      if (tid < w)
#pragma unroll
        for (int f = 0; f < F; ++f) red[f * ST_NT + tid] += red[f * ST_NT + tid + w];
      __syncthreads();
    }
#pragma unroll
    for (int f = 0; f < F; ++f) var[f] = red[f * ST_NT] / (float)n;
    __syncthreads();
#pragma unroll
    for (int f = 0; f < F; ++f) {
      if (f >= nf) break;
      const float r = 1.f / sqrtf(var[f] + ST_LN_EPS);
      for (int j = tid; j < n; j += ST_NT) v[f * ld + j] = a[j] * ((v[f * ld + j] - mean[f]) * r) + b[j];
    }
  } else {
#pragma unroll
    for (int f = 0; f < F; ++f) {
      if (f >= nf) break;
      for (int j = tid; j < n; j += ST_NT) v[f * ld + j] = v[f * ld + j] * a[j] + b[j];
    }
  }
  __syncthreads();
}

// out[f][j] = sum_i Wt[i][j] * in[f][i] for j < n_out (Wt [n_in][n_out], fp32)
template <int F>
CTN_DEV void st_matvec(const float* __restrict__ Wt, int n_in, int n_out, const float* in, int ld_in, int nf,
                       float* out, int ld_out) {
  for (int j = threadIdx.x; j < n_out; j += ST_NT) {
    float acc[F];
#pragma unroll
    for (int f = 0; f < F; ++f) acc[f] = 0.f;
    // 16 weight loads in flight per thread: one load per iteration would leave the loop
    // bound by L2 latency (the weights stream from L2/MALL once per call)
    int i = 0;
    for (; i + 16 <= n_in; i += 16) {
      float w[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) w[u] = Wt[(size_t)(i + u) * n_out + j];
#pragma unroll
      for (int u = 0; u < 16; ++u)
#pragma unroll
        for (int f = 0; f < F; ++f) acc[f] = fmaf(w[u], in[f * ld_in + i + u], acc[f]);
    }
    for (; i < n_in; ++i) {
      const float w = Wt[(size_t)i * n_out + j];
#pragma unroll
      for (int f = 0; f < F; ++f) acc[f] = fmaf(w, in[f * ld_in + i], acc[f]);
    }
#pragma unroll
    for (int f = 0; f < F; ++f)
      if (f < nf) out[f * ld_out + j] = acc[f];
  }
}

__global__ __launch_bounds__(ST_NT) void stream_encode_kernel(StreamArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int N = a.N, L = a.L, S = a.L / 2, Bc = a.B;
  const int m = blockIdx.x, f0 = blockIdx.y * ST_FPB, nf = min(ST_FPB, a.K - f0);
  float* smp = sm;                                   // (FPB-1)*S + L samples
  float* y = smp + ((ST_FPB - 1) * S + L + 3) / 4 * 4;   // [FPB][N]
  float* red = y + ST_FPB * N;                       // [FPB][256]
  const int ns = (nf - 1) * S + L;
  for (int i = threadIdx.x; i < ns; i += ST_NT) smp[i] = a.samples[(size_t)m * a.ld_samples + (size_t)f0 * S + i];
  __syncthreads();
  for (int n = threadIdx.x; n < N; n += ST_NT) {
    for (int f = 0; f < nf; ++f) {
      float acc = 0.f;
      for (int l = 0; l < L; ++l) acc = fmaf(a.U[(size_t)n * L + l], smp[f * S + l], acc);
      acc = acc > 0.f ? acc : 0.f;                   // ReLU (conv_tasnet.py:117)
      y[f * N + n] = acc;
      a.w_out[((size_t)m * a.K + f0 + f) * N + n] = acc;
    }
  }
  __syncthreads();
  st_norm_rows<ST_FPB>(y, N, nf, N, 1, a.na, a.nb, red);   // separator cLN (always channel-wise)
  float* x = a.x_out + ((size_t)m * a.K + f0) * Bc;
  st_matvec<ST_FPB>(a.W, N, Bc, y, N, nf, x, Bc);
}

__global__ __launch_bounds__(ST_NT) void stream_block_in_kernel(StreamArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Bc = a.B, H = a.H;
  const int m = blockIdx.x, f0 = blockIdx.y * ST_FPB, nf = min(ST_FPB, a.K - f0);
  float* xs = sm;                      // [FPB][B]
  float* h = xs + ST_FPB * Bc;         // [FPB][H]
  float* red = h + ST_FPB * H;
  for (int i = threadIdx.x; i < nf * Bc; i += ST_NT) xs[i] = a.x_in[((size_t)m * a.K + f0) * Bc + i];
  __syncthreads();
  st_matvec<ST_FPB>(a.W, Bc, H, xs, Bc, nf, h, H);
  __syncthreads();                     // h[f][j] was written by thread j % 256
  const float al = a.alpha1[0];
  for (int i = threadIdx.x; i < nf * H; i += ST_NT) h[i] = h[i] > 0.f ? h[i] : al * h[i];   // PReLU
  __syncthreads();
  st_norm_rows<ST_FPB>(h, H, nf, H, a.norm, a.na, a.nb, red);
  const unsigned mask = (unsigned)a.R - 1u;
  for (int f = 0; f < nf; ++f) {
    float* dst = a.ring + ((size_t)m * a.R + ((unsigned)(a.pos + f0 + f) & mask)) * H;
    for (int j = threadIdx.x; j < H; j += ST_NT) dst[j] = h[f * H + j];
  }
}

__global__ __launch_bounds__(ST_NT) void stream_block_out_kernel(StreamArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Bc = a.B, H = a.H, P = a.P, dil = a.dil;
  const int m = blockIdx.x, f0 = blockIdx.y * ST_FPB, nf = min(ST_FPB, a.K - f0);
  float* d = sm;                       // [FPB][H]
  float* red = d + ST_FPB * H;
  const unsigned mask = (unsigned)a.R - 1u;
  const float al = a.alpha2[0];
  for (int j = threadIdx.x; j < H; j += ST_NT) {
    for (int f = 0; f < nf; ++f) {
      const long g = a.pos + f0 + f;
      float s = 0.f;
      for (int p = 0; p < P; ++p) {
        const long src = g - (long)(P - 1 - p) * dil;     // causal taps (conv_tasnet.py:176, Chomp1d)
        if (src >= 0) s = fmaf(a.wd[(size_t)j * P + p], a.ring[((size_t)m * a.R + ((unsigned)src & mask)) * H + j], s);
      }
      d[f * H + j] = s > 0.f ? s : al * s;                // PReLU 2
    }
  }
  __syncthreads();
  st_norm_rows<ST_FPB>(d, H, nf, H, a.norm, a.na, a.nb, red);
  const float* xr = a.x_in + ((size_t)m * a.K + f0) * Bc;
  float* xo = a.x_out + ((size_t)m * a.K + f0) * Bc;
  for (int b = threadIdx.x; b < Bc; b += ST_NT) {
    float acc[ST_FPB];
#pragma unroll
    for (int f = 0; f < ST_FPB; ++f) acc[f] = 0.f;
    int j = 0;
    for (; j + 16 <= H; j += 16) {
      float w[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) w[u] = a.W[(size_t)(j + u) * Bc + b];
#pragma unroll
      for (int u = 0; u < 16; ++u)
#pragma unroll
        for (int f = 0; f < ST_FPB; ++f) acc[f] = fmaf(w[u], d[f * H + j + u], acc[f]);
    }
    for (; j < H; ++j) {
      const float w = a.W[(size_t)j * Bc + b];
#pragma unroll
      for (int f = 0; f < ST_FPB; ++f) acc[f] = fmaf(w, d[f * H + j], acc[f]);
    }
#pragma unroll
    for (int f = 0; f < ST_FPB; ++f)
      if (f < nf) xo[(size_t)f * Bc + b] = acc[f] + xr[(size_t)f * Bc + b];   // + residual
  }
}

__global__ __launch_bounds__(ST_NT) void stream_decode_kernel(StreamArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Bc = a.B, N = a.N, C = a.C, L = a.L, CN = C * N;
  const int m = blockIdx.x, f0 = blockIdx.y * ST_FPB_DEC, nf = min(ST_FPB_DEC, a.K - f0);
  float* xs = sm;                      // [FPB][B]
  float* sc = xs + ST_FPB_DEC * Bc;    // [FPB][C*N]
  for (int i = threadIdx.x; i < nf * Bc; i += ST_NT) xs[i] = a.x_in[((size_t)m * a.K + f0) * Bc + i];
  __syncthreads();
  st_matvec<ST_FPB_DEC>(a.W, Bc, CN, xs, Bc, nf, sc, CN);   // mask 1x1 (conv_tasnet.py:193)
  __syncthreads();
  // mask nonlinearity across speakers (conv_tasnet.py:202-207), sources = w * mask (:137)
  for (int n = threadIdx.x; n < N; n += ST_NT) {
    for (int f = 0; f < nf; ++f) {
      float* s = sc + f * CN + n;
      const float wv = a.w_in[((size_t)m * a.K + f0 + f) * N + n];
      if (a.mask_type == 1) {
        float mx = -3.4e38f, den = 0.f;
        for (int c = 0; c < C; ++c) mx = fmaxf(mx, s[c * N]);
        for (int c = 0; c < C; ++c) { s[c * N] = expf(s[c * N] - mx); den += s[c * N]; }
        for (int c = 0; c < C; ++c) s[c * N] = wv * (s[c * N] / den);
      } else if (a.mask_type == 0) {
        for (int c = 0; c < C; ++c) s[c * N] = wv * (s[c * N] > 0.f ? s[c * N] : 0.f);
      } else {
        for (int c = 0; c < C; ++c) s[c * N] = wv * s[c * N];
      }
    }
  }
  __syncthreads();
  // frames[m][c][k][l] = sum_n src_c[n] V[l][n] (decoder basis, conv_tasnet.py:138-140)
  for (int o = threadIdx.x; o < C * L; o += ST_NT) {
    const int c = o / L, l = o % L;
    for (int f = 0; f < nf; ++f) {
      float acc = 0.f;
      for (int n = 0; n < N; ++n) acc = fmaf(sc[f * CN + c * N + n], a.V[(size_t)l * N + n], acc);
      a.frames[(((size_t)m * C + c) * a.K + f0 + f) * L + l] = acc;
    }
  }
}

// out[m][c][k*S + i] = frame_k[i] + frame_{k-1}[S + i] (frame_{-1} = the previous call's
// tail); the new tail is frame_{K-1}[S ..] (utils.py:9-46 with L = 2S)
__global__ __launch_bounds__(ST_NT) void stream_ola_kernel(StreamArgs a) {
  const int S = a.L / 2, L = a.L, K = a.K;
  const long total = (long)a.M * a.C * K * S;
  for (long i = blockIdx.x * (long)ST_NT + threadIdx.x; i < total; i += (long)gridDim.x * ST_NT) {
    const int s = (int)(i % S);
    const long mck = i / S;
    const int k = (int)(mck % K);
    const long mc = mck / K;
    const float* fr = a.frames + (size_t)mc * K * L;
    const float prev = k > 0 ? fr[(size_t)(k - 1) * L + S + s] : a.tail_in[mc * S + s];
    a.out[mc * (size_t)K * S + (size_t)k * S + s] = fr[(size_t)k * L + s] + prev;
    if (k == K - 1) a.tail_out[mc * S + s] = fr[(size_t)k * L + S + s];
  }
}

// ===========================================================================
// ABI v7 call path (ctn_stream_call): the same arithmetic cut over many workgroups.
// The v5 kernels above give each (stream, 8 frames) ONE workgroup, which streams a
// whole 1x1 weight (0.5 MiB fp32) through one CU: ~50 us per launch whatever the
// chunk size.  Here every 1x1 conv is split over 32-output column chunks (each
// workgroup reads a 32-column slice of the weight), and the per-frame norms that need
// a whole row are recomputed by every chunk workgroup of that frame (same arithmetic,
// same order: every copy is bit-identical).
//   SE  encode + cLN + bottleneck chunk              grid (M, frame groups, B/32)
//   SA  block: W1 chunk -> h1 (pre-PReLU) scratch     grid (M, frame groups, H/32)
//   SB  block: taps (ring for frames of earlier calls, PReLU + norm 1 of h1 rows of
//       this call), depthwise, PReLU, norm 2, W2 chunk + residual; chunk 0 writes the
//       frame's norm-1 row to the ring                 grid (M, K, B/32)
//   SD1 mask 1x1 chunk (all speakers of 32 channels), nonlinearity, * w -> sources
//   SD2 sources . V^T -> frames, overlap-add with the carried tail
// ===========================================================================
// outputs per chunk workgroup: SC_W = 32 (8 input slices per output) for calls with many
// frames x streams, 8 (32 slices) for small calls, where a kernel's few workgroups each
// streaming a 32-column weight slice left the call latency-bound (14.5 us per block
// kernel at 1 stream x 1 frame); chosen per launch (sc_width)
constexpr int SC_FPB = 8;                // frames per workgroup (SE, SA, SD1)

// res[f] (valid in threads t < SC_W) = sum_i Wt[i][j0 + t] * in[f][i]; thread (o, s) sums
// the inputs i = s, s + 8, ... (a 128-byte weight row segment per 32 threads), then the
// 8 slices are added in order.  red: SC_FPB * ST_NT floats.
template <int F, int SC_W>
CTN_DEV void sc_matvec(const float* __restrict__ Wt, int n_in, int n_out, int j0, const float* in, int ld_in, int nf,
                       float (&res)[F], float* red) {
  constexpr int SC_SL = ST_NT / SC_W;   // input slices per output
  const int t = threadIdx.x, o = t % SC_W, sl = t / SC_W, j = j0 + o;
  float acc[F];
#pragma unroll
  for (int f = 0; f < F; ++f) acc[f] = 0.f;
  if (j < n_out) {
#pragma unroll 4
    for (int i = sl; i < n_in; i += SC_SL) {
      const float w = Wt[(size_t)i * n_out + j];
#pragma unroll
      for (int f = 0; f < F; ++f)
        if (f < nf) acc[f] = fmaf(w, in[f * ld_in + i], acc[f]);
    }
  }
#pragma unroll
  for (int f = 0; f < F; ++f) red[(f * SC_SL + sl) * SC_W + o] = acc[f];
  __syncthreads();
  if (t < SC_W) {
#pragma unroll
    for (int f = 0; f < F; ++f) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < SC_SL; ++q) v += red[(f * SC_SL + q) * SC_W + t];
      res[f] = v;
    }
  }
  __syncthreads();
}

template <int SC_W>
__global__ __launch_bounds__(ST_NT) void sc_encode_kernel(StreamArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int N = a.N, L = a.L, S = a.L / 2, Bc = a.B;
  const int m = blockIdx.x, f0 = blockIdx.y * SC_FPB, nf = min(SC_FPB, a.K - f0), j0 = blockIdx.z * SC_W;
  float* smp = sm;                                          // (FPB-1)*S + L samples
  float* y = smp + ((SC_FPB - 1) * S + L + 3) / 4 * 4;      // [FPB][N]
  float* red = y + SC_FPB * N;                              // [FPB][256]
  const int ns = (nf - 1) * S + L;
  for (int i = threadIdx.x; i < ns; i += ST_NT) smp[i] = a.samples[(size_t)m * a.ld_samples + (size_t)f0 * S + i];
  __syncthreads();
  for (int n = threadIdx.x; n < N; n += ST_NT)
    for (int f = 0; f < nf; ++f) {
      float acc = 0.f;
      for (int l = 0; l < L; ++l) acc = fmaf(a.U[(size_t)n * L + l], smp[f * S + l], acc);
      acc = acc > 0.f ? acc : 0.f;                          // ReLU (conv_tasnet.py:117)
      y[f * N + n] = acc;
      if (blockIdx.z == 0) a.w_out[((size_t)m * a.K + f0 + f) * N + n] = acc;
    }
  __syncthreads();
  st_norm_rows<SC_FPB>(y, N, nf, N, 1, a.na, a.nb, red);   // separator cLN (always channel-wise)
  float res[SC_FPB];
  sc_matvec<SC_FPB, SC_W>(a.W, N, Bc, j0, y, N, nf, res, red);
  if (threadIdx.x < SC_W && j0 + (int)threadIdx.x < Bc)
    for (int f = 0; f < nf; ++f) a.x_out[((size_t)m * a.K + f0 + f) * Bc + j0 + threadIdx.x] = res[f];
}

template <int SC_W>
__global__ __launch_bounds__(ST_NT) void sc_block_in_kernel(StreamArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Bc = a.B, H = a.H;
  const int m = blockIdx.x, f0 = blockIdx.y * SC_FPB, nf = min(SC_FPB, a.K - f0), j0 = blockIdx.z * SC_W;
  float* xs = sm;                      // [FPB][B]
  float* red = xs + SC_FPB * Bc;
  for (int i = threadIdx.x; i < nf * Bc; i += ST_NT) xs[i] = a.x_in[((size_t)m * a.K + f0) * Bc + i];
  __syncthreads();
  float res[SC_FPB];
  sc_matvec<SC_FPB, SC_W>(a.W, Bc, H, j0, xs, Bc, nf, res, red);
  if (threadIdx.x < SC_W && j0 + (int)threadIdx.x < H)
    for (int f = 0; f < nf; ++f) a.frames[((size_t)m * a.K + f0 + f) * H + j0 + threadIdx.x] = res[f];   // h1 scratch
}

template <int SC_W>
__global__ __launch_bounds__(ST_NT) void sc_block_out_kernel(StreamArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Bc = a.B, H = a.H, P = a.P, dil = a.dil;
  const int m = blockIdx.x, f = blockIdx.y, j0 = blockIdx.z * SC_W;
  float* taps = sm;                    // [P][H]: norm-1 output rows of the P taps
  float* d = taps + P * H;             // [H]
  float* red = d + H;                  // [ST_NT * SC_FPB]
  const unsigned mask = (unsigned)a.R - 1u;
  const long pos = a.pos_dev ? *a.pos_dev : a.pos;
  const long g = pos + f;
  const float al1 = a.alpha1[0], al2 = a.alpha2[0];
  for (int p = 0; p < P; ++p) {
    const long src = g - (long)(P - 1 - p) * dil;           // causal taps (conv_tasnet.py:176, Chomp1d)
    float* row = taps + p * H;
    if (src < pos) {                                         // an earlier call's frame (ring) or before the start
      for (int j = threadIdx.x; j < H; j += ST_NT)
        row[j] = src >= 0 ? a.ring[((size_t)m * a.R + ((unsigned)src & mask)) * H + j] : 0.f;
      __syncthreads();
    } else {                                                 // this call's frame: PReLU 1 + norm 1 of its h1 row
      const float* h = a.frames + ((size_t)m * a.K + (src - pos)) * H;
      for (int j = threadIdx.x; j < H; j += ST_NT) {
        const float v = h[j];
        row[j] = v > 0.f ? v : al1 * v;
      }
      __syncthreads();
      st_norm_rows<1>(row, H, 1, H, a.norm, a.na, a.nb, red);
    }
  }
  if (blockIdx.z == 0) {                                     // the frame's own norm-1 row -> its ring slot
    float* dst = a.ring + ((size_t)m * a.R + ((unsigned)g & mask)) * H;
    for (int j = threadIdx.x; j < H; j += ST_NT) dst[j] = taps[(P - 1) * H + j];
  }
  for (int j = threadIdx.x; j < H; j += ST_NT) {
    float s = 0.f;
    for (int p = 0; p < P; ++p) s = fmaf(a.wd[(size_t)j * P + p], taps[p * H + j], s);
    d[j] = s > 0.f ? s : al2 * s;                            // PReLU 2
  }
  __syncthreads();
  st_norm_rows<1>(d, H, 1, H, a.norm, a.na2, a.nb2, red);
  float res[1];
  sc_matvec<1, SC_W>(a.W2, H, Bc, j0, d, H, 1, res, red);
  if (threadIdx.x < SC_W && j0 + (int)threadIdx.x < Bc) {
    const size_t o = ((size_t)m * a.K + f) * Bc + j0 + threadIdx.x;
    a.x_out[o] = res[0] + a.x_in[o];                         // + residual
  }
}

// sources[m][c][k][n] = w * mask: the mask 1x1 for all speakers of 32 channels n, then
// the nonlinearity across speakers (conv_tasnet.py:185, 202-207, 137)
template <int SC_W>
__global__ __launch_bounds__(ST_NT) void sc_decode_mask_kernel(StreamArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Bc = a.B, N = a.N, C = a.C, CN = C * N;
  const int m = blockIdx.x, f0 = blockIdx.y * SC_FPB, nf = min(SC_FPB, a.K - f0), n0 = blockIdx.z * SC_W;
  float* xs = sm;                      // [FPB][B]
  float* sc = xs + SC_FPB * Bc;        // [C][FPB][32]
  float* red = sc + C * SC_FPB * SC_W;
  for (int i = threadIdx.x; i < nf * Bc; i += ST_NT) xs[i] = a.x_in[((size_t)m * a.K + f0) * Bc + i];
  __syncthreads();
  for (int c = 0; c < C; ++c) {
    float res[SC_FPB];
    sc_matvec<SC_FPB, SC_W>(a.W, Bc, CN, c * N + n0, xs, Bc, nf, res, red);
    if (threadIdx.x < SC_W)
      for (int f = 0; f < SC_FPB; ++f) sc[(c * SC_FPB + f) * SC_W + threadIdx.x] = res[f];
  }
  __syncthreads();
  const int t = threadIdx.x, n = n0 + t;
  if (t < SC_W && n < N)
    for (int f = 0; f < nf; ++f) {
      const float wv = a.w_in[((size_t)m * a.K + f0 + f) * N + n];
      float v[8];
      for (int c = 0; c < C; ++c) v[c] = sc[(c * SC_FPB + f) * SC_W + t];
      if (a.mask_type == 1) {
        float mx = -3.4e38f, den = 0.f;
        for (int c = 0; c < C; ++c) mx = fmaxf(mx, v[c]);
        for (int c = 0; c < C; ++c) { v[c] = expf(v[c] - mx); den += v[c]; }
        for (int c = 0; c < C; ++c) v[c] = wv * (v[c] / den);
      } else if (a.mask_type == 0) {
        for (int c = 0; c < C; ++c) v[c] = wv * (v[c] > 0.f ? v[c] : 0.f);
      } else {
        for (int c = 0; c < C; ++c) v[c] = wv * v[c];
      }
      for (int c = 0; c < C; ++c) a.frames[(((size_t)m * C + c) * a.K + f0 + f) * N + n] = v[c];
    }
}

// frames = sources . V^T (decoder basis, conv_tasnet.py:138-140), then the overlap-add with
// the previous call's tail (utils.py:9-46, L = 2S): one workgroup per (stream, speaker)
__global__ __launch_bounds__(ST_NT) void sc_decode_ola_kernel(StreamArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int N = a.N, L = a.L, S = a.L / 2, K = a.K;
  const int mc = blockIdx.x;
  float* fr = sm;                      // [K][L]
  const float* src = a.frames + (size_t)mc * K * N;
  for (int o = threadIdx.x; o < K * L; o += ST_NT) {
    const int k = o / L, l = o % L;
    float acc = 0.f;
    for (int n = 0; n < N; ++n) acc = fmaf(src[(size_t)k * N + n], a.V[(size_t)l * N + n], acc);
    fr[o] = acc;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < K * S; i += ST_NT) {
    const int k = i / S, s2 = i % S;
    const float prev = k > 0 ? fr[(k - 1) * L + S + s2] : a.tail_in[(size_t)mc * S + s2];
    a.out[(size_t)mc * K * S + i] = fr[k * L + s2] + prev;
  }
  for (int s2 = threadIdx.x; s2 < S; s2 += ST_NT) a.tail_out[(size_t)mc * S + s2] = fr[(K - 1) * L + S + s2];
}

size_t stream_call_smem(int which, const StreamArgs& a) {
  const int S = a.L / 2;
  switch (which) {
    case 0: return (size_t)(((SC_FPB - 1) * S + a.L + 3) / 4 * 4 + SC_FPB * a.N + SC_FPB * ST_NT) * 4;
    case 1: return (size_t)(SC_FPB * a.B + SC_FPB * ST_NT) * 4;
    case 2: return (size_t)(a.P * a.H + a.H + SC_FPB * ST_NT) * 4;
    case 3: return (size_t)(SC_FPB * a.B + a.C * SC_FPB * 32 + SC_FPB * ST_NT) * 4;   // SC_W <= 32
    default: return (size_t)a.K * a.L * 4;
  }
}

__global__ void sc_set_pos_kernel(long* p, long v) {
  if (threadIdx.x == 0) *p = v;
}

hipError_t launch_stream_set_pos(long* pos_dev, long pos, hipStream_t s) {
  hipLaunchKernelGGL(sc_set_pos_kernel, dim3(1), dim3(64), 0, s, pos_dev, pos);
  return hipGetLastError();
}

template <int SC_W>
static hipError_t sc_launch(int which, const StreamArgs& a, size_t lds, hipStream_t s) {
  const unsigned fg = (unsigned)((a.K + SC_FPB - 1) / SC_FPB);
  const dim3 b(ST_NT);
  switch (which) {
    case 0: hipLaunchKernelGGL(sc_encode_kernel<SC_W>, dim3(a.M, fg, (a.B + SC_W - 1) / SC_W), b, lds, s, a); break;
    case 1: hipLaunchKernelGGL(sc_block_in_kernel<SC_W>, dim3(a.M, fg, (a.H + SC_W - 1) / SC_W), b, lds, s, a); break;
    case 2: hipLaunchKernelGGL(sc_block_out_kernel<SC_W>, dim3(a.M, a.K, (a.B + SC_W - 1) / SC_W), b, lds, s, a); break;
    case 3: hipLaunchKernelGGL(sc_decode_mask_kernel<SC_W>, dim3(a.M, fg, (a.N + SC_W - 1) / SC_W), b, lds, s, a); break;
    case 4: hipLaunchKernelGGL(sc_decode_ola_kernel, dim3(a.M * a.C), b, lds, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// narrow chunks while the (stream, frame) work units of a call are few (<= 128; CTN_SC_W=8|32
// forces one width)
static int sc_width(const StreamArgs& a) {
  const char* e = getenv("CTN_SC_W");
  if (e) return atoi(e) == 8 ? 8 : 32;
  return (long)a.M * a.K <= 128 ? 8 : 32;
}

hipError_t launch_stream_call_stage(int which, const StreamArgs& a, hipStream_t s) {
  const size_t lds = stream_call_smem(which, a);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  return sc_width(a) == 8 ? sc_launch<8>(which, a, lds, s) : sc_launch<32>(which, a, lds, s);
}

size_t stream_smem(int which, const StreamArgs& a) {
  const int S = a.L / 2;
  switch (which) {
    case 0: return (size_t)(((ST_FPB - 1) * S + a.L + 3) / 4 * 4 + ST_FPB * a.N + ST_FPB * ST_NT) * 4;
    case 1: return (size_t)(ST_FPB * a.B + ST_FPB * a.H + ST_FPB * ST_NT) * 4;
    case 2: return (size_t)(ST_FPB * a.H + ST_FPB * ST_NT) * 4;
    default: return (size_t)(ST_FPB_DEC * a.B + ST_FPB_DEC * a.C * a.N) * 4;
  }
}

hipError_t launch_stream(int which, const StreamArgs& a, hipStream_t s) {
  const size_t lds = stream_smem(which, a);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int fpb = which == 3 ? ST_FPB_DEC : ST_FPB;
  const dim3 g((unsigned)a.M, (unsigned)((a.K + fpb - 1) / fpb)), b(ST_NT);
  switch (which) {
    case 0: hipLaunchKernelGGL(stream_encode_kernel, g, b, lds, s, a); break;
    case 1: hipLaunchKernelGGL(stream_block_in_kernel, g, b, lds, s, a); break;
    case 2: hipLaunchKernelGGL(stream_block_out_kernel, g, b, lds, s, a); break;
    case 3: {
      hipLaunchKernelGGL(stream_decode_kernel, g, b, lds, s, a);
      const long total = (long)a.M * a.C * a.K * (a.L / 2);
      const long gb = (total + ST_NT - 1) / ST_NT;
      hipLaunchKernelGGL(stream_ola_kernel, dim3((unsigned)(gb < 1024 ? gb : 1024)), b, 0, s, a);
      break;
    }
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace ctn
