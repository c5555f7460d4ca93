// Encoder / decoder / overlap-add kernels (gfx950).
//
// enc_fwd     : w[r][n] = ReLU(sum_l U[n][l] x[m, k*S + l])          conv_tasnet.py:106,116
//               + per-frame cLN statistics of w (two-pass, fp32)     conv_tasnet.py:167,319-329
// enc_bwd_rows: cLN backward per frame, + decoder's dL/dw, ReLU mask -> dL/d(pre-ReLU)
// frame_outer : dU[n][l] = sum_r g[r][n] x[kS+l]  (encoder weight grad) and
//               dV[l][n] = sum_{r,c} src_c[r][n] gest_c[kS+l] (decoder basis grad)
// dec_fwd     : frames[m][c][k][l] = sum_n (w[r][n] * act(score)[r][c][n]) V[l][n]   :128-140
// ola_fwd     : est[m][c][t] = sum_{k: kS<=t<kS+L} frames[m][c][k][t-kS], zero to T  utils.py:9-46, :56-59
// dec_bwd     : dL/dscore and dL/dw from dL/dest (frames gradient gathered from est)
#include <stdlib.h>

#include "ctn_common.h"
#include "ctn_codec.h"

namespace ctn {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int EN_RPB = 128;   // frame rows per workgroup (matches the row padding)

// ===========================================================================
// encoder forward
// ===========================================================================
template <typename T>
__global__ __launch_bounds__(256) void enc_fwd_kernel(CodecArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int N = a.N, L = a.L, S = a.S, cg = N / 8;
  int nrl = 256 / cg;
  if (nrl > EN_RPB) nrl = EN_RPB;
  const int tid = threadIdx.x, c = tid % cg, rl = tid / cg;
  const bool act = rl < nrl;
  const int K = a.K, Kp = a.Kp;
  const int row0 = blockIdx.x * EN_RPB, m = row0 / Kp, k0 = row0 - m * Kp;
  float* Ut = sm;                           // [L][N]
  float* xs = sm + L * N;                   // samples [k0*S, k0*S + (EN_RPB-1)*S + L)
  const int nsamp = (EN_RPB - 1) * S + L;
  for (int i = tid; i < L * N; i += 256) {
    const int l = i / N, n = i % N;
    Ut[i] = a.U[n * L + l];
  }
  for (int i = tid; i < nsamp; i += 256) {
    const long t = (long)k0 * S + i;
    xs[i] = t < a.T ? a.mixture[(size_t)m * a.T + t] : 0.f;
  }
  __syncthreads();
  T* w = reinterpret_cast<T*>(a.w_rows);
  if (!act) return;
  for (int rr = rl; rr < EN_RPB; rr += nrl) {
    const int k = k0 + rr;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (k < K) {
      for (int l = 0; l < L; ++l) {
        const float x = xs[rr * S + l];
        const float4 u0 = *reinterpret_cast<const float4*>(Ut + l * N + c * 8);
        const float4 u1 = *reinterpret_cast<const float4*>(Ut + l * N + c * 8 + 4);
        v[0] += u0.x * x; v[1] += u0.y * x; v[2] += u0.z * x; v[3] += u0.w * x;
        v[4] += u1.x * x; v[5] += u1.y * x; v[6] += u1.z * x; v[7] += u1.w * x;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
    }
    Vec8<T>::store(w + (size_t)(row0 + rr) * N + c * 8, v);
    if (a.cln_stats) {
      // two-pass per-frame statistics over the N channels (cg lanes of one wave)
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[e];
      s = wave_sum_group(s, cg);
      const float mean = s / (float)N;
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) q += (v[e] - mean) * (v[e] - mean);
      q = wave_sum_group(q, cg);
      if (c == 0) {
        const float rstd = 1.0f / sqrtf(q / (float)N + 1e-8f);
        a.cln_stats[row0 + rr] = k < K ? make_float2(mean, rstd) : make_float2(0.f, 1.f);
      }
    }
  }
}

// ===========================================================================
// encoder backward (rows): cLN backward + decoder grad + ReLU mask
//   gcln : dL/d cLN(w)  [rows][N] storage type (bottleneck data gradient)
//   gwdec: dL/dw from the decoder [rows][N] storage type (may be null)
//   out  : gpre [rows][N] fp32 = dL/d(pre-ReLU encoder output)
//   col partials per block: ggamma0[N], gbeta0[N]
// ===========================================================================
template <typename T>
__global__ __launch_bounds__(256) void enc_bwd_rows_kernel(CodecArgs a) {
  __shared__ float buf[256 * 8];
  const int N = a.N, cg = N / 8;
  int nrl = 256 / cg;
  if (nrl > EN_RPB) nrl = EN_RPB;
  const int tid = threadIdx.x, c = tid % cg, rl = tid / cg;
  const bool act = rl < nrl;
  const int K = a.K, Kp = a.Kp;
  const int row0 = blockIdx.x * EN_RPB, m = row0 / Kp, k0 = row0 - m * Kp;
  const T* w = reinterpret_cast<const T*>(a.w_rows);
  const T* gcln = reinterpret_cast<const T*>(a.gcln);
  const T* gwdec = reinterpret_cast<const T*>(a.gwdec);
  float g0[8], cgam[8], cbet[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    g0[e] = a.gamma0 ? a.gamma0[c * 8 + e] : 0.f;
    cgam[e] = cbet[e] = 0.f;
  }
  if (act) {
    for (int rr = rl; rr < EN_RPB; rr += nrl) {
      const int r = row0 + rr, k = k0 + rr;
      float out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (k < K) {   // uniform across the cg lanes of this frame
        float wv[8], gd[8];
        Vec8<T>::load(w + (size_t)r * N + c * 8, wv);
        if (gwdec) Vec8<T>::load(gwdec + (size_t)r * N + c * 8, gd);
        else
#pragma unroll
          for (int e = 0; e < 8; ++e) gd[e] = 0.f;
        if (gcln) {
          float gv[8];
          Vec8<T>::load(gcln + (size_t)r * N + c * 8, gv);
          const float2 st = a.cln_stats[r];
          float s1 = 0.f, s2 = 0.f, wh[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            wh[e] = (wv[e] - st.x) * st.y;
            const float gh = gv[e] * g0[e];
            s1 += gh;
            s2 += gh * wh[e];
            cgam[e] += gv[e] * wh[e];
            cbet[e] += gv[e];
          }
          s1 = wave_sum_group(s1, cg) / (float)N;
          s2 = wave_sum_group(s2, cg) / (float)N;
#pragma unroll
          for (int e = 0; e < 8; ++e) gd[e] += st.y * (gv[e] * g0[e] - s1 - wh[e] * s2);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) out[e] = wv[e] > 0.f ? gd[e] : 0.f;   // ReLU backward
      }
      if (a.gpre_bf) Vec8<bf16raw>::store(reinterpret_cast<bf16raw*>(a.gpre_bf) + (size_t)r * N + c * 8, out);
      else Vec8<float>::store(a.gpre + (size_t)r * N + c * 8, out);
    }
  }
  if (a.col_slab) {
    float* cs = a.col_slab + (size_t)blockIdx.x * 2 * N;
    for (int q = 0; q < 2; ++q) {
      if (act)
#pragma unroll
        for (int e = 0; e < 8; ++e) buf[rl * N + c * 8 + e] = q == 0 ? cgam[e] : cbet[e];
      __syncthreads();
      for (int ch = tid; ch < N; ch += 256) {
        float s = 0.f;
        for (int i = 0; i < nrl; ++i) s += buf[i * N + ch];
        cs[q * N + ch] = s;
      }
      __syncthreads();
    }
  }
}

// ===========================================================================
// frame_outer: weight gradients of the two framing convolutions
//   mode 0 (encoder dU [N][L]):  sum_r gpre[r][n] * x[m][kS + l]
//   mode 1 (decoder dV [L][N]):  sum_r sum_c (w[r][n] act_c(score[r][c][n])) * gest[m][c][kS + l]
// Persistent: FO_WGS workgroups each sweep a contiguous run of FO_R-row chunks
// (chunks never straddle utterances).  Per chunk the rows are staged into LDS
// with 16-byte loads by all threads (mode 1 forms src = w * act(score) on the
// way), together with the chunk's signal span; thread n then accumulates its
// channel's L outputs from LDS across all of its chunks.  Padded frames stage
// as zeros.  One fp32 partial per workgroup -> slab [FO_WGS][N*L].
// ===========================================================================
constexpr int FO_R = 16, FO_WGS = 512, FO_LMAX = 32;

// LT: compile-time L (0: generic, <= FO_LMAX); CM: speakers held per row (4, 8 for
// 5 <= C <= 8 with FO_R / 2 rows per chunk, or 16 for 9 <= C <= 16 with FO_R / 4, so the
// staged rows stay within LDS)
constexpr int fo_rows(int C) { return C > 8 ? FO_R / 4 : (C > 4 ? FO_R / 2 : FO_R); }
template <typename T, int MODE, int LT, int CM = 4>
__global__ __launch_bounds__(256) void frame_outer_kernel(CodecArgs a) {
  constexpr int FO_R = fo_rows(CM);
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int LL = LT ? LT : FO_LMAX;
  const int N = a.N, L = LT ? LT : a.L, S = a.S, C = MODE == 0 ? 1 : a.C, K = a.K, Kp = a.Kp;
  const int cg = N / 8;                               // 8-channel groups per row
  const int span = FO_R * S + L;                      // signal samples of one chunk
  float* srcs = sm;                                   // [FO_R][C][N]
  float* sig = sm + FO_R * C * N;                     // [C][span]
  const int nchunk = a.M * (Kp / FO_R);
  const int c0 = (int)((long)nchunk * blockIdx.x / gridDim.x), c1 = (int)((long)nchunk * (blockIdx.x + 1) / gridDim.x);
  const T* w = reinterpret_cast<const T*>(a.w_rows);
  const T* sc = reinterpret_cast<const T*>(a.score);
  constexpr int NPT = 2;                              // channels per thread (N <= 512)
  float acc[NPT][LL];
#pragma unroll
  for (int j = 0; j < NPT; ++j)
#pragma unroll
    for (int l = 0; l < LL; ++l) acc[j][l] = 0.f;

  for (int ch = c0; ch < c1; ++ch) {
    const int m = ch / (Kp / FO_R), kb = (ch % (Kp / FO_R)) * FO_R;
    __syncthreads();   // previous chunk fully consumed
    // ---- stage source rows
    for (int i = threadIdx.x; i < FO_R * cg; i += 256) {
      const int rr = i / cg, c8 = i % cg, k = kb + rr;
      const size_t r = (size_t)m * Kp + k;
      float v[CM][8];
      if (k < K) {
        if constexpr (MODE == 0) {
          const float4 g0 = *reinterpret_cast<const float4*>(a.gpre + r * N + c8 * 8);
          const float4 g1 = *reinterpret_cast<const float4*>(a.gpre + r * N + c8 * 8 + 4);
          v[0][0] = g0.x; v[0][1] = g0.y; v[0][2] = g0.z; v[0][3] = g0.w;
          v[0][4] = g1.x; v[0][5] = g1.y; v[0][6] = g1.z; v[0][7] = g1.w;
        } else {
          float wv[8];
          Vec8<T>::load(w + r * N + c8 * 8, wv);
          for (int cc = 0; cc < C; ++cc) Vec8<T>::load(sc + r * (size_t)(C * N) + (size_t)cc * N + c8 * 8, v[cc]);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            if (a.mask_type == 1) {
              float mx = -3.4e38f, den = 0.f;
              for (int cc = 0; cc < C; ++cc) mx = fmaxf(mx, v[cc][e]);
              for (int cc = 0; cc < C; ++cc) { v[cc][e] = __expf(v[cc][e] - mx); den += v[cc][e]; }
              for (int cc = 0; cc < C; ++cc) v[cc][e] = wv[e] * v[cc][e] / den;
            } else if (a.mask_type == 0) {
              for (int cc = 0; cc < C; ++cc) v[cc][e] = wv[e] * (v[cc][e] > 0.f ? v[cc][e] : 0.f);
            } else {
              for (int cc = 0; cc < C; ++cc) v[cc][e] = wv[e] * v[cc][e];
            }
          }
        }
      } else {
        for (int cc = 0; cc < C; ++cc)
#pragma unroll
          for (int e = 0; e < 8; ++e) v[cc][e] = 0.f;
      }
      for (int cc = 0; cc < C; ++cc) {
        float* d = srcs + (rr * C + cc) * N + c8 * 8;
        *reinterpret_cast<float4*>(d) = make_float4(v[cc][0], v[cc][1], v[cc][2], v[cc][3]);
        *reinterpret_cast<float4*>(d + 4) = make_float4(v[cc][4], v[cc][5], v[cc][6], v[cc][7]);
      }
    }
    // ---- stage the signal span of every speaker
    for (int i = threadIdx.x; i < C * span; i += 256) {
      const int cc = i / span, j = i % span;
      const long t = (long)kb * S + j;
      float v = 0.f;
      if (MODE == 0) v = t < a.T ? a.mixture[(size_t)m * a.T + t] : 0.f;
      else v = t < a.T ? a.gest[((size_t)m * a.C + cc) * a.T + t] : 0.f;
      sig[i] = v;
    }
    __syncthreads();
    // ---- accumulate: thread owns channels n = tid + 256*j
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int n = threadIdx.x + 256 * j;
      if (n >= N) break;
      for (int rr = 0; rr < FO_R; ++rr)
        for (int cc = 0; cc < C; ++cc) {
          const float sv = srcs[(rr * C + cc) * N + n];
          const float* gs = sig + cc * span + rr * S;
#pragma unroll
          for (int l = 0; l < LL; ++l)
            if (LT || l < L) acc[j][l] += sv * gs[l];
        }
    }
  }
  // mode 0 -> [N][L] (encoder weight [N,1,L]); mode 1 -> [L][N] (Linear(N, L) weight)
  float* out = a.col_slab + (size_t)blockIdx.x * N * L;
#pragma unroll
  for (int j = 0; j < NPT; ++j) {
    const int n = threadIdx.x + 256 * j;
    if (n >= N) break;
#pragma unroll
    for (int l = 0; l < LL; ++l)
      if (LT || l < L) out[MODE == 0 ? (size_t)n * L + l : (size_t)l * N + n] = acc[j][l];
  }
}

// ===========================================================================
// decoder forward: frames[m][c][k][l]  (fp32)
// workgroup = DEC_RPB frame rows; src = w * act(score) staged in LDS [rows][C][N]
// ===========================================================================
template <typename T, int CM = 4>   // CM: speakers held per row (4, 8 or 16)
__global__ __launch_bounds__(256) void dec_fwd_kernel(CodecArgs a, int rpb) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int N = a.N, L = a.L, C = a.C, K = a.K, Kp = a.Kp;
  float* Vt = sm;                       // [N][L]
  float* src = sm + ((N * L + 3) & ~3); // [rpb][C][N]
  const int row0 = blockIdx.x * rpb, m = row0 / Kp, k0 = row0 - m * Kp;
  for (int i = threadIdx.x; i < N * L; i += 256) {
    const int n = i / L, l = i % L;
    Vt[i] = a.V[l * N + n];
  }
  const T* w = reinterpret_cast<const T*>(a.w_rows);
  const T* sc = reinterpret_cast<const T*>(a.score);
  const int cg = N / 8;
  for (int i = threadIdx.x; i < rpb * cg; i += 256) {
    const int rr = i / cg, c8 = i % cg;
    const size_t r = (size_t)row0 + rr;
    float wv[8], s[CM][8];
    Vec8<T>::load(w + r * N + c8 * 8, wv);
    for (int cc = 0; cc < C; ++cc) Vec8<T>::load(sc + r * (size_t)(C * N) + (size_t)cc * N + c8 * 8, s[cc]);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (a.mask_type == 1) {
        float mx = -3.4e38f, den = 0.f;
        for (int cc = 0; cc < C; ++cc) mx = fmaxf(mx, s[cc][e]);
        for (int cc = 0; cc < C; ++cc) { s[cc][e] = __expf(s[cc][e] - mx); den += s[cc][e]; }
        for (int cc = 0; cc < C; ++cc) s[cc][e] /= den;
      } else if (a.mask_type == 0) {
        for (int cc = 0; cc < C; ++cc) s[cc][e] = s[cc][e] > 0.f ? s[cc][e] : 0.f;
      }
    }
    for (int cc = 0; cc < C; ++cc)
#pragma unroll
      for (int e = 0; e < 8; ++e) src[(rr * C + cc) * N + c8 * 8 + e] = wv[e] * s[cc][e];
  }
  __syncthreads();
  const int nout = rpb * C * L;
  for (int o = threadIdx.x; o < nout; o += 256) {
    const int l = o % L, cc = (o / L) % C, rr = o / (L * C);
    const int k = k0 + rr;
    if (k >= K) continue;
    const float* sp = src + (rr * C + cc) * N;
    float acc = 0.f;
    for (int n = 0; n < N; ++n) acc += sp[n] * Vt[n * L + l];
    a.frames[(((size_t)m * C + cc) * Kp + k) * L + l] = acc;
  }
}

// est[m][c][t] = sum over frames covering t; zero for t >= (K-1)S + L (F.pad, conv_tasnet.py:59)
__global__ __launch_bounds__(256) void ola_fwd_kernel(CodecArgs a) {
  const long total = (long)a.M * a.C * a.T;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int t = (int)(i % a.T);
    const long mc = i / a.T;
    const int K = a.K, S = a.S, L = a.L;
    int khi = t / S;
    if (khi > K - 1) khi = K - 1;
    int klo = t - L + 1 <= 0 ? 0 : (t - L + 1 + S - 1) / S;
    float s = 0.f;
    const float* f = a.frames + (size_t)mc * a.Kp * L;
    for (int k = klo; k <= khi; ++k) s += f[(size_t)k * L + (t - k * S)];
    a.est[i] = s;
  }
}

// ===========================================================================
// decoder backward (rows): gsrc = gframes . V ; gw = sum_c gsrc_c act_c ; gscore
// ===========================================================================
template <typename T, int CM = 4>   // CM: speakers held per row (4, 8 or 16)
__global__ __launch_bounds__(256) void dec_bwd_kernel(CodecArgs a, int rpb) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int N = a.N, L = a.L, C = a.C, S = a.S, K = a.K, Kp = a.Kp;
  float* Vs = sm;                          // [L][N]
  float* gf = sm + ((L * N + 3) & ~3);     // [rpb][C][L]
  const int row0 = blockIdx.x * rpb, m = row0 / Kp, k0 = row0 - m * Kp;
  for (int i = threadIdx.x; i < L * N; i += 256) Vs[i] = a.V[i];
  for (int i = threadIdx.x; i < rpb * C * L; i += 256) {
    const int l = i % L, cc = (i / L) % C, rr = i / (L * C);
    const int k = k0 + rr;
    const long t = (long)k * S + l;
    gf[i] = (k < K && t < a.T) ? a.gest[((size_t)m * C + cc) * a.T + t] : 0.f;
  }
  __syncthreads();
  const T* w = reinterpret_cast<const T*>(a.w_rows);
  const T* sc = reinterpret_cast<const T*>(a.score);
  T* gsc = reinterpret_cast<T*>(a.gscore);
  T* gw = reinterpret_cast<T*>(a.gwdec_out);
  const int cg = N / 8;
  for (int i = threadIdx.x; i < rpb * cg; i += 256) {
    const int rr = i / cg, c8 = i % cg;
    const size_t r = (size_t)row0 + rr;
    const int k = k0 + rr;
    float gwv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (k >= K) {
      for (int cc = 0; cc < C; ++cc) Vec8<T>::store(gsc + r * (size_t)(C * N) + (size_t)cc * N + c8 * 8, gwv);
      Vec8<T>::store(gw + r * N + c8 * 8, gwv);
      continue;
    }
    float wv[8], s[CM][8], ga[CM][8];
    Vec8<T>::load(w + r * N + c8 * 8, wv);
    for (int cc = 0; cc < C; ++cc) Vec8<T>::load(sc + r * (size_t)(C * N) + (size_t)cc * N + c8 * 8, s[cc]);
    // gsrc[cc][e] = sum_l gf[rr][cc][l] * V[l][n]
    for (int cc = 0; cc < C; ++cc) {
      float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      const float* gfp = gf + (rr * C + cc) * L;
      for (int l = 0; l < L; ++l) {
        const float gl = gfp[l];
        const float4 v0 = *reinterpret_cast<const float4*>(Vs + l * N + c8 * 8);
        const float4 v1 = *reinterpret_cast<const float4*>(Vs + l * N + c8 * 8 + 4);
        g[0] += gl * v0.x; g[1] += gl * v0.y; g[2] += gl * v0.z; g[3] += gl * v0.w;
        g[4] += gl * v1.x; g[5] += gl * v1.y; g[6] += gl * v1.z; g[7] += gl * v1.w;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) ga[cc][e] = g[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float act[CM];
      if (a.mask_type == 1) {
        float mx = -3.4e38f, den = 0.f;
        for (int cc = 0; cc < C; ++cc) mx = fmaxf(mx, s[cc][e]);
        for (int cc = 0; cc < C; ++cc) { act[cc] = __expf(s[cc][e] - mx); den += act[cc]; }
        for (int cc = 0; cc < C; ++cc) act[cc] /= den;
      } else if (a.mask_type == 0) {
        for (int cc = 0; cc < C; ++cc) act[cc] = s[cc][e] > 0.f ? s[cc][e] : 0.f;
      } else {
        for (int cc = 0; cc < C; ++cc) act[cc] = s[cc][e];
      }
      float gw_e = 0.f, dot = 0.f;
      for (int cc = 0; cc < C; ++cc) {
        gw_e += ga[cc][e] * act[cc];
        ga[cc][e] *= wv[e];                 // dL/d act_c
        dot += ga[cc][e] * act[cc];
      }
      gwv[e] = gw_e;
      for (int cc = 0; cc < C; ++cc) {
        float g;
        if (a.mask_type == 1) g = act[cc] * (ga[cc][e] - dot);
        else if (a.mask_type == 0) g = s[cc][e] > 0.f ? ga[cc][e] : 0.f;
        else g = ga[cc][e];
        s[cc][e] = g;
      }
    }
    for (int cc = 0; cc < C; ++cc) Vec8<T>::store(gsc + r * (size_t)(C * N) + (size_t)cc * N + c8 * 8, s[cc]);
    Vec8<T>::store(gw + r * N + c8 * 8, gwv);
  }
}

// ===========================================================================
// bf16 decoder on the matrix cores (N = 32*KBN, L <= 32, C <= 4)
//
// Both directions are GEMMs with a short side (L, the basis length): the forward
// frames[r,c,:] = src_c[r,:] . V^T with src_c = w * act(score_c), the backward
// gsrc_c[r,:] = gframes_c[r,:] . V with gframes gathered from dL/dest.  The VALU
// kernels above re-read V from LDS per output (LDS-bound, about 0.6 TB/s of the rows
// they stream); here each workgroup converts the basis once into bf16 MFMA fragments
// in LDS (lane-linear, one 16-byte read per fragment) and its waves stream 16-row
// blocks of w and score straight from HBM into v_mfma_f32_16x16x32_bf16 operands
// (the element-wise mask nonlinearity and product formed in fp32 on the way).  Waves are persistent and
// walk blocks blk, blk + (all waves), ...; blocks never straddle utterances (Kp is a
// multiple of 128).  Padded frames hold zero rows, so their outputs are zero and are
// not stored (forward) or stored as the zeros they compute (backward).
// ===========================================================================
constexpr int DM_WAVES = 4;   // waves per workgroup

// mask nonlinearity of C scores of one (row, channel), in place: relu / softmax / identity
template <int CM> CTN_DEV void dm_act(int mask_type, int C, float (&x)[CM]) {
  if (mask_type == 1) {
    float mx = -3.4e38f, den = 0.f;
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) mx = fmaxf(mx, x[c]);
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) {
        x[c] = __expf(x[c] - mx);
        den += x[c];
      }
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) x[c] /= den;
  } else if (mask_type == 0) {
#pragma unroll
    for (int c = 0; c < CM; ++c) x[c] = x[c] > 0.f ? x[c] : 0.f;
  }
}

template <int KBN, int CM>   // N / 32, speakers
__global__ __launch_bounds__(256) void dec_fwd_mfma_kernel(CodecArgs a) {
  constexpr int N = KBN * 32;
  __shared__ v4u bfrag[2 * KBN * 64];
  const int lane = threadIdx.x & 63, lg = lane >> 4, wv = threadIdx.x >> 6;
  const int L = a.L, C = a.C, K = a.K, Kp = a.Kp;
  // basis fragments (B operand) [nb][kb][lane]: column l = nb*16 + (lane & 15),
  // channels kb*32 + 8*(lane >> 4) .. +8
  for (int i = threadIdx.x; i < 2 * KBN * 64; i += 256) {
    const int ln = i & 63, kb = (i >> 6) % KBN, nb = i / (64 * KBN), l = nb * 16 + (ln & 15);
    float f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (l < L) Vec8<float>::load(a.V + (size_t)l * N + kb * 32 + 8 * (ln >> 4), f);
    bfrag[i] = pack_bf16x8v(f);
  }
  __syncthreads();
  const int lr = lane & 15;
  const bf16raw* w = reinterpret_cast<const bf16raw*>(a.w_rows);
  const bf16raw* sc = reinterpret_cast<const bf16raw*>(a.score);
  const long nblk = (long)a.M * Kp / 16;
  for (long blk = (long)blockIdx.x * DM_WAVES + wv; blk < nblk; blk += (long)gridDim.x * DM_WAVES) {
    const long r0 = blk * 16;
    const int m = (int)(r0 / Kp), k0 = (int)(r0 - (long)m * Kp);
    if (k0 >= K) continue;   // a block of padded frames (wave-uniform)
    const long r = r0 + lr;
    f32x4_t acc[CM][2];
#pragma unroll
    for (int c = 0; c < CM; ++c) acc[c][0] = acc[c][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KBN; ++kb) {
      const int ch = kb * 32 + 8 * lg;
      float wf[8], sf[CM][8];
      unpack_bf16x8(ldg16(w + r * N + ch), wf);
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c < C) unpack_bf16x8(ldg16(sc + r * (long)(C * N) + (long)c * N + ch), sf[c]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c) x[c] = c < C ? sf[c][e] : 0.f;
        dm_act<CM>(a.mask_type, C, x);
#pragma unroll
        for (int c = 0; c < CM; ++c) sf[c][e] = wf[e] * x[c];
      }
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c < C) {
          const bf16x8_t af = __builtin_bit_cast(bf16x8_t, pack_bf16x8v(sf[c]));
          const v4u b0 = bfrag[kb * 64 + lane], b1 = bfrag[(KBN + kb) * 64 + lane];
          acc[c][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8_t, b0), acc[c][0], 0, 0, 0);
          acc[c][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8_t, b1), acc[c][1], 0, 0, 0);
        }
    }
    // lane holds frames (row 4lg + i, l = nb*16 + lr)
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          const int l = nb * 16 + lr;
          if (l >= L) continue;
          float* f = a.frames + (((size_t)m * C + c) * Kp + k0) * L + l;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (k0 + 4 * lg + i < K) f[(size_t)(4 * lg + i) * L] = acc[c][nb][i];
        }
  }
}

template <int NBN, int CM>   // N / 16, speakers (compile time: per-speaker arrays stay in registers)
__global__ __launch_bounds__(256) void dec_bwd_mfma_kernel(CodecArgs a) {
  constexpr int N = NBN * 16;
  static_assert(NBN % 2 == 0, "two channel blocks per round");
  __shared__ v4u afrag[NBN * 64];
  constexpr int TS = 36;   // tile row stride (floats): 32 channels + 4 of padding against bank conflicts
  __shared__ __attribute__((aligned(16))) float gtile[DM_WAVES * CM * 16 * TS];   // per-wave transpose tiles
  const int lane = threadIdx.x & 63, lr = lane & 15, lg = lane >> 4, wv = threadIdx.x >> 6;
  const int L = a.L, C = a.C, S = a.S, K = a.K, Kp = a.Kp;
  // basis fragments (A operand) [nb][lane]: row n = nb*16 + (lane & 15), k = l =
  // 8*(lane >> 4) .. +8 (zero past L)
  for (int i = threadIdx.x; i < NBN * 64; i += 256) {
    const int ln = i & 63, nb = i >> 6;
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int l = 8 * (ln >> 4) + j;
      f[j] = l < L ? a.V[(size_t)l * N + nb * 16 + (ln & 15)] : 0.f;
    }
    afrag[i] = pack_bf16x8v(f);
  }
  __syncthreads();
  const bf16raw* w = reinterpret_cast<const bf16raw*>(a.w_rows);
  const bf16raw* sc = reinterpret_cast<const bf16raw*>(a.score);
  bf16raw* gsc = reinterpret_cast<bf16raw*>(a.gscore);
  bf16raw* gw = reinterpret_cast<bf16raw*>(a.gwdec_out);
  const long nblk = (long)a.M * Kp / 16;
  typedef uint32_t v2u __attribute__((ext_vector_type(2)));
  for (long blk = (long)blockIdx.x * DM_WAVES + wv; blk < nblk; blk += (long)gridDim.x * DM_WAVES) {
    const long r0 = blk * 16;
    const int m = (int)(r0 / Kp), k0 = (int)(r0 - (long)m * Kp);
    // frames gradient (B operand): row r = lr (column of the product), l = 8lg .. +8
    v4u gb[CM];
    {
      const int k = k0 + lr;
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        float f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (c < C && k < K) {
          const float* g = a.gest + ((size_t)m * C + c) * a.T + (long)k * S;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int l = 8 * lg + j;
            if (l < L && (long)k * S + l < a.T) f[j] = g[l];
          }
        }
        gb[c] = pack_bf16x8v(f);
      }
    }
    // Two 16-channel blocks per round: the MFMA leaves lane (n = 4lg + i, r = lr); the
    // products go through this wave's LDS tile [16 rows][32 channels (+4 pad)] so that each lane
    // then owns 8 consecutive channels of one row (r = lane / 4, n = 8 * (lane % 4)) and
    // every load and store below is 16 bytes (64-byte row segments).
    float* tile = gtile + wv * (CM * 16 * TS);
    const int er = lane >> 2, en = 8 * (lane & 3);   // element-wise row / first channel in the round
#pragma unroll 1
    for (int nb = 0; nb < NBN; nb += 2) {
      const long r = r0 + er;
      const int n0 = nb * 16 + en;
      // the round's mixture-weight and score rows are loaded before its MFMAs and tile
      // stage (which end in a compiler barrier): their latency overlaps that work
      const v4u wraw = ldg16(w + r * N + n0);
      v4u sraw[CM];
#pragma unroll
      for (int c = 0; c < CM; ++c) sraw[c] = c < C ? ldg16(sc + r * (long)(C * N) + (long)c * N + n0) : v4u{0u, 0u, 0u, 0u};
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (c < C) {
            const f32x4_t g = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8_t, afrag[(nb + h) * 64 + lane]), __builtin_bit_cast(bf16x8_t, gb[c]),
                f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            *reinterpret_cast<float4*>(tile + (c * 16 + lr) * TS + h * 16 + 4 * lg) = float4{g[0], g[1], g[2], g[3]};
          }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's own tile: no barrier needed
      float wf[8], sv[CM][8], gs[CM][8];
      unpack_bf16x8(wraw, wf);
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c < C) {
          unpack_bf16x8(sraw[c], sv[c]);
          const float4 g0 = *reinterpret_cast<const float4*>(tile + (c * 16 + er) * TS + en);
          const float4 g1 = *reinterpret_cast<const float4*>(tile + (c * 16 + er) * TS + en + 4);
          gs[c][0] = g0.x; gs[c][1] = g0.y; gs[c][2] = g0.z; gs[c][3] = g0.w;
          gs[c][4] = g1.x; gs[c][5] = g1.y; gs[c][6] = g1.z; gs[c][7] = g1.w;
        }
      float gwv[8], go[CM][8], srcv[CM][8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float s[CM], act[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c) {
          s[c] = c < C ? sv[c][i] : 0.f;
          act[c] = s[c];
        }
        dm_act<CM>(a.mask_type, C, act);
#pragma unroll
        for (int c = 0; c < CM; ++c) srcv[c][i] = wf[i] * act[c];
        float gwe = 0.f, dot = 0.f, ga[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (c < C) {
            gwe += gs[c][i] * act[c];
            ga[c] = gs[c][i] * wf[i];   // dL/d act_c
            dot += ga[c] * act[c];
          }
        gwv[i] = gwe;
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (c < C) go[c][i] = a.mask_type == 1 ? act[c] * (ga[c] - dot) : a.mask_type == 0 ? (s[c] > 0.f ? ga[c] : 0.f) : ga[c];
      }
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c < C) stg16(gsc + r * (long)(C * N) + (long)c * N + n0, pack_bf16x8v(go[c]));
      stg16(gw + r * N + n0, pack_bf16x8v(gwv));
      if (a.src_out) {
        bf16raw* so = reinterpret_cast<bf16raw*>(a.src_out);
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (c < C) stg16(so + r * (long)(C * N) + (long)c * N + n0, pack_bf16x8v(srcv[c]));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // tile reads done before the next round's writes
    }
  }
}

// frames of a signal sig [M][C][T] as bf16 rows fr[(r, c)][l] = sig[m][c][k*S + l] (0 past
// K, T or L): the frame gradients of the decoder basis gradient (sig = dL/dest) and the
// mixture frames of the encoder's (C = 1); one thread per (row, channel)
__global__ __launch_bounds__(256) void frames_bf16_kernel(CodecArgs a, const float* sig, int C, bf16raw* out) {
  const long n = (long)a.M * a.Kp * C;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long r = i / C;
    const int m = (int)(r / a.Kp), k = (int)(r % a.Kp);
    const float* g = sig + ((size_t)m * C + c) * a.T + (long)k * a.S;
    bf16raw* o = out + i * a.Lp;
    for (int l0 = 0; l0 < a.Lp; l0 += 8) {
      float f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int l = l0 + j;
        f[j] = (k < a.K && l < a.L && (long)k * a.S + l < a.T) ? g[l] : 0.f;
      }
      stg16(o + l0, pack_bf16x8v(f));
    }
  }
}

// bf16-storage encoder forward on the fp32 matrix cores (N = 16*NBN, L <= 32):
// w^T[n][r] = ReLU(sum_l U[n][l] x[kS+l]) with v_mfma_f32_16x16x4_f32 (exact fp32 operands,
// as the VALU kernel), U as A operands in LDS and the mixture frames as B operands (one
// sample per lane and k-step); the products go through a per-wave LDS tile as in
// dec_bwd_mfma so each lane stores 8 consecutive channels of one frame (16 bytes) and
// keeps them for the frame's cLN statistics (two-pass over the values the four lanes of
// the frame hold, reduced with DPP quad permutes): enc_fwd_kernel's arithmetic, fp32.
template <int NBN>
__global__ __launch_bounds__(256) void enc_fwd_mfma_kernel(CodecArgs a) {
  constexpr int N = NBN * 16, NR = NBN / 2;   // rounds of 32 channels
  constexpr int TS = 36, KKM = 8;              // k-steps of 4 samples: L <= 32
  __shared__ float afr[NBN * KKM * 64];         // [nb][kk][lane] = U[nb*16 + lane%16][4kk + lane/16]
  __shared__ __attribute__((aligned(16))) float tiles[DM_WAVES * 16 * TS];
  const int lane = threadIdx.x & 63, lr = lane & 15, lg = lane >> 4, wv = threadIdx.x >> 6;
  const int L = a.L, S = a.S, K = a.K, Kp = a.Kp, KK = (L + 3) / 4;
  for (int i = threadIdx.x; i < NBN * KKM * 64; i += 256) {
    const int ln = i & 63, kk = (i >> 6) % KKM, nb = i / (64 * KKM), l = 4 * kk + (ln >> 4);
    afr[i] = l < L ? a.U[(size_t)(nb * 16 + (ln & 15)) * L + l] : 0.f;
  }
  __syncthreads();
  bf16raw* w = reinterpret_cast<bf16raw*>(a.w_rows);
  float* tile = tiles + wv * 16 * TS;
  const int er = lane >> 2, en = 8 * (lane & 3);
  const long nblk = (long)a.M * Kp / 16;
  for (long blk = (long)blockIdx.x * DM_WAVES + wv; blk < nblk; blk += (long)gridDim.x * DM_WAVES) {
    const long r0 = blk * 16;
    const int m = (int)(r0 / Kp), k0 = (int)(r0 - (long)m * Kp);
    float fb[KKM];   // frames (B operand): column r = lr, sample l = 4kk + lg
    {
      const int k = k0 + lr;
      const float* x = a.mixture + (size_t)m * a.T + (long)k * S;
#pragma unroll
      for (int kk = 0; kk < KKM; ++kk) {
        const int l = 4 * kk + lg;
        fb[kk] = (kk < KK && k < K && l < L && (long)k * S + l < a.T) ? x[l] : 0.f;
      }
    }
    const int k = k0 + er;
    const bool valid = k < K;
    float v[NR][8];
#pragma unroll
    for (int rd = 0; rd < NR; ++rd) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4_t g = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KKM; ++kk)
          if (kk < KK) g = __builtin_amdgcn_mfma_f32_16x16x4f32(afr[((2 * rd + h) * KKM + kk) * 64 + lane], fb[kk], g, 0, 0, 0);
        *reinterpret_cast<float4*>(tile + lr * TS + h * 16 + 4 * lg) = float4{g[0], g[1], g[2], g[3]};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const float4 g0 = *reinterpret_cast<const float4*>(tile + er * TS + en);
      const float4 g1 = *reinterpret_cast<const float4*>(tile + er * TS + en + 4);
      const float t[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[rd][e] = valid ? (t[e] > 0.f ? t[e] : 0.f) : 0.f;
      stg16(w + (size_t)(r0 + er) * N + rd * 32 + en, pack_bf16x8v(v[rd]));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (a.cln_stats) {
      // the frame's 256 values are spread over its 4 lanes (quad): quad sums by DPP
      float sm = 0.f;
#pragma unroll
      for (int rd = 0; rd < NR; ++rd)
#pragma unroll
        for (int e = 0; e < 8; ++e) sm += v[rd][e];
      sm += dpp_f<0xB1, 0xF>(sm);   // quad_perm [1,0,3,2]
      sm += dpp_f<0x4E, 0xF>(sm);   // quad_perm [2,3,0,1]
      const float mean = sm / (float)N;
      float q = 0.f;
#pragma unroll
      for (int rd = 0; rd < NR; ++rd)
#pragma unroll
        for (int e = 0; e < 8; ++e) q += (v[rd][e] - mean) * (v[rd][e] - mean);
      q += dpp_f<0xB1, 0xF>(q);
      q += dpp_f<0x4E, 0xF>(q);
      if ((lane & 3) == 0) {
        const float rstd = 1.0f / sqrtf(q / (float)N + 1e-8f);
        a.cln_stats[r0 + er] = valid ? make_float2(mean, rstd) : make_float2(0.f, 1.f);
      }
    }
  }
}

// CTN_DEC_MFMA=0 keeps the VALU decoder kernels for bf16 too (read per launch: A/B)
bool codec_dec_mfma(DType dt, const CodecArgs& a);
static bool dec_mfma(DType dt, const CodecArgs& a) { return codec_dec_mfma(dt, a); }
bool codec_dec_mfma(DType dt, const CodecArgs& a) {
  const char* e = getenv("CTN_DEC_MFMA");
  if (e && atoi(e) == 0) return false;
  return dt == BF16 && (a.N == 256 || a.N == 512) && a.L <= 32 && a.C <= 4;
}
static unsigned dm_grid(const CodecArgs& a) {
  const long waves = (long)a.M * a.Kp / 16;
  long wgs = (waves + DM_WAVES - 1) / DM_WAVES;
  return (unsigned)(wgs < 1024 ? wgs : 1024);
}

// ===========================================================================
// launchers
// ===========================================================================
static bool codec_ok(const CodecArgs& a) {
  return a.N % 8 == 0 && a.N / 8 <= 64 && ((a.N / 8) & (a.N / 8 - 1)) == 0 && a.L >= 1 && a.L <= 32 &&
         a.S >= 1 && a.C >= 1 && a.C <= 16 && a.Kp % EN_RPB == 0;
}

hipError_t launch_enc_fwd(DType dt, const CodecArgs& a, hipStream_t s) {
  if (!codec_ok(a)) return hipErrorInvalidValue;
  const size_t lds = ((size_t)a.L * a.N + (EN_RPB - 1) * a.S + a.L) * sizeof(float);
  const dim3 g((unsigned)((long)a.M * a.Kp / EN_RPB)), b(256);
  const char* e = getenv("CTN_ENC_MFMA");
  const bool mf = dt == BF16 && (!e || atoi(e) != 0) && (a.N == 256 || a.N == 512) && a.L <= 32;
  if (mf && a.N == 256) hipLaunchKernelGGL(enc_fwd_mfma_kernel<16>, dim3(dm_grid(a)), b, 0, s, a);
  else if (mf) hipLaunchKernelGGL(enc_fwd_mfma_kernel<32>, dim3(dm_grid(a)), b, 0, s, a);
  else if (dt == BF16) hipLaunchKernelGGL(enc_fwd_kernel<bf16raw>, g, b, lds, s, a);
  else hipLaunchKernelGGL(enc_fwd_kernel<float>, g, b, lds, s, a);
  return hipGetLastError();
}

hipError_t launch_enc_bwd_rows(DType dt, const CodecArgs& a, hipStream_t s) {
  if (!codec_ok(a)) return hipErrorInvalidValue;
  const dim3 g((unsigned)((long)a.M * a.Kp / EN_RPB)), b(256);
  if (dt == BF16) hipLaunchKernelGGL(enc_bwd_rows_kernel<bf16raw>, g, b, 0, s, a);
  else hipLaunchKernelGGL(enc_bwd_rows_kernel<float>, g, b, 0, s, a);
  return hipGetLastError();
}

int frame_outer_chunks(const CodecArgs& a, int C) {
  const int n = a.M * (a.Kp / fo_rows(C));
  return n < FO_WGS ? n : FO_WGS;
}

hipError_t launch_frame_outer(DType dt, int mode, const CodecArgs& a, hipStream_t s) {
  if (!codec_ok(a) || a.Kp % FO_R || a.N > 512 || a.L > FO_LMAX) return hipErrorInvalidValue;
  const int C = mode == 0 ? 1 : a.C;
  const int fr = fo_rows(C);
  const size_t lds = ((size_t)fr * C * a.N + (size_t)C * (fr * a.S + a.L)) * sizeof(float);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const dim3 g(frame_outer_chunks(a, C)), b(256);
#define CTN_FO(T_, M_)                                                                                          \
  if (C > 8) hipLaunchKernelGGL((frame_outer_kernel<T_, M_, 0, 16>), g, b, lds, s, a);                       \
  else if (C > 4) hipLaunchKernelGGL((frame_outer_kernel<T_, M_, 0, 8>), g, b, lds, s, a);                   \
  else if (a.L == 20) hipLaunchKernelGGL((frame_outer_kernel<T_, M_, 20>), g, b, lds, s, a);                  \
  else if (a.L == 16) hipLaunchKernelGGL((frame_outer_kernel<T_, M_, 16>), g, b, lds, s, a);                  \
  else hipLaunchKernelGGL((frame_outer_kernel<T_, M_, 0>), g, b, lds, s, a);
  if (mode == 0) {
    if (dt == BF16) { CTN_FO(bf16raw, 0) } else { CTN_FO(float, 0) }
  } else {
    if (dt == BF16) { CTN_FO(bf16raw, 1) } else { CTN_FO(float, 1) }
  }
#undef CTN_FO
  return hipGetLastError();
}

static int dec_rpb(const CodecArgs& a) {
  // 64 KB of LDS: the [N][L] basis plus rpb frame rows of src; rpb divides 128
  const size_t budget = 64 * 1024 - (((size_t)a.N * a.L + 3) & ~(size_t)3) * 4;
  int rpb = 32;
  while (rpb > 1 && (size_t)rpb * a.C * a.N * 4 > budget) rpb >>= 1;
  return rpb;
}

hipError_t launch_dec_fwd(DType dt, const CodecArgs& a, hipStream_t s) {
  if (!codec_ok(a)) return hipErrorInvalidValue;
  const int rpb = dec_rpb(a);
  const size_t lds = (((size_t)a.N * a.L + 3) & ~(size_t)3) * 4 + (size_t)rpb * a.C * a.N * 4;
  const dim3 g((unsigned)((long)a.M * a.Kp / rpb)), b(256);
  if (dec_mfma(dt, a)) {
#define CTN_DFM(KBN_)                                                                                    \
    switch (a.C) {                                                                                     \
      case 1: hipLaunchKernelGGL((dec_fwd_mfma_kernel<KBN_, 1>), dim3(dm_grid(a)), b, 0, s, a); break; \
      case 2: hipLaunchKernelGGL((dec_fwd_mfma_kernel<KBN_, 2>), dim3(dm_grid(a)), b, 0, s, a); break; \
      case 3: hipLaunchKernelGGL((dec_fwd_mfma_kernel<KBN_, 3>), dim3(dm_grid(a)), b, 0, s, a); break; \
      default: hipLaunchKernelGGL((dec_fwd_mfma_kernel<KBN_, 4>), dim3(dm_grid(a)), b, 0, s, a); break; \
    }
    if (a.N == 256) { CTN_DFM(8) } else { CTN_DFM(16) }
#undef CTN_DFM
  } else if (a.C > 8) {
    if (dt == BF16) hipLaunchKernelGGL((dec_fwd_kernel<bf16raw, 16>), g, b, lds, s, a, rpb);
    else hipLaunchKernelGGL((dec_fwd_kernel<float, 16>), g, b, lds, s, a, rpb);
  } else if (a.C > 4) {
    if (dt == BF16) hipLaunchKernelGGL((dec_fwd_kernel<bf16raw, 8>), g, b, lds, s, a, rpb);
    else hipLaunchKernelGGL((dec_fwd_kernel<float, 8>), g, b, lds, s, a, rpb);
  } else if (dt == BF16) hipLaunchKernelGGL(dec_fwd_kernel<bf16raw>, g, b, lds, s, a, rpb);
  else hipLaunchKernelGGL(dec_fwd_kernel<float>, g, b, lds, s, a, rpb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  long total = (long)a.M * a.C * a.T;
  int gb = (int)((total + 255) / 256);
  if (gb > 4096) gb = 4096;
  hipLaunchKernelGGL(ola_fwd_kernel, dim3(gb), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_frames_bf16(const CodecArgs& a, const float* sig, int C, void* out, hipStream_t s) {
  if (!out || !sig || a.Lp < a.L || a.Lp % 8 || C < 1) return hipErrorInvalidValue;
  const long n = (long)a.M * a.Kp * C;
  long g = (n + 255) / 256;
  hipLaunchKernelGGL(frames_bf16_kernel, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, s, a, sig, C,
                     reinterpret_cast<bf16raw*>(out));
  return hipGetLastError();
}
hipError_t launch_dec_gframes(const CodecArgs& a, hipStream_t s) {
  return launch_frames_bf16(a, a.gest, a.C, a.gfr_out, s);
}

__global__ __launch_bounds__(256) void unpad_cols_kernel(const float* tmp, int N, int Lp, int L, float* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < N * L) out[i] = tmp[(i / L) * Lp + i % L];
}
hipError_t launch_unpad_cols(const float* tmp, int N, int Lp, int L, float* out, hipStream_t s) {
  hipLaunchKernelGGL(unpad_cols_kernel, dim3((N * L + 255) / 256), dim3(256), 0, s, tmp, N, Lp, L, out);
  return hipGetLastError();
}

hipError_t launch_dec_bwd(DType dt, const CodecArgs& a, hipStream_t s) {
  if (!codec_ok(a)) return hipErrorInvalidValue;
  const int rpb = 32;
  const size_t lds = (((size_t)a.N * a.L + 3) & ~(size_t)3) * 4 + (size_t)rpb * a.C * a.L * 4;
  const dim3 g((unsigned)((long)a.M * a.Kp / rpb)), b(256);
  if (dec_mfma(dt, a)) {
#define CTN_DBM(NBN_)                                                                                     \
    switch (a.C) {                                                                                      \
      case 1: hipLaunchKernelGGL((dec_bwd_mfma_kernel<NBN_, 1>), dim3(dm_grid(a)), b, 0, s, a); break;  \
      case 2: hipLaunchKernelGGL((dec_bwd_mfma_kernel<NBN_, 2>), dim3(dm_grid(a)), b, 0, s, a); break;  \
      case 3: hipLaunchKernelGGL((dec_bwd_mfma_kernel<NBN_, 3>), dim3(dm_grid(a)), b, 0, s, a); break;  \
      default: hipLaunchKernelGGL((dec_bwd_mfma_kernel<NBN_, 4>), dim3(dm_grid(a)), b, 0, s, a); break; \
    }
    if (a.N == 256) { CTN_DBM(16) } else { CTN_DBM(32) }
#undef CTN_DBM
  } else if (a.C > 8) {
    if (dt == BF16) hipLaunchKernelGGL((dec_bwd_kernel<bf16raw, 16>), g, b, lds, s, a, rpb);
    else hipLaunchKernelGGL((dec_bwd_kernel<float, 16>), g, b, lds, s, a, rpb);
  } else if (a.C > 4) {
    if (dt == BF16) hipLaunchKernelGGL((dec_bwd_kernel<bf16raw, 8>), g, b, lds, s, a, rpb);
    else hipLaunchKernelGGL((dec_bwd_kernel<float, 8>), g, b, lds, s, a, rpb);
  } else if (dt == BF16) hipLaunchKernelGGL(dec_bwd_kernel<bf16raw>, g, b, lds, s, a, rpb);
  else hipLaunchKernelGGL(dec_bwd_kernel<float>, g, b, lds, s, a, rpb);
  return hipGetLastError();
}

}  // namespace ctn
