// Parameter-update kernels of the training step (gfx950):
//   grad_sqnorm + grad_clip : torch.nn.utils.clip_grad_norm_(params, max_norm)
//                             as called by src/solver.py:184-185 (2-norm)
//   adam                    : torch.optim.Adam(params, lr, weight_decay=l2)
//                             built at src/train.py:129-133, stepped at solver.py:186
//
// All parameters of a model are one launch: a segment table names every tensor
// (param, grad, exp_avg, exp_avg_sq, numel) and a chunk table cuts the tensors
// into OPT_CHUNK-element pieces, one workgroup each.  Both tables live in device
// memory and are built once per set of pointers (ctn_opt_plan).  Pure streaming:
// HBM-bound at 4 B/element (norm), 8 B (clip), 28 B (Adam).
#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

constexpr int OPT_THREADS = 256;

// chunk c covers elements [off, off + len) of segment seg; vec = all four
// pointers of the segment are 16-byte aligned (and off is a multiple of 4)
CTN_DEV void opt_chunk(const OptChunk* ch, int& seg, long& off, int& len, bool& vec) {
  const OptChunk c = ch[blockIdx.x];
  seg = c.seg;
  off = c.off;
  len = (int)(c.len & OPT_LEN_MASK);
  vec = (c.len & OPT_UNALIGNED) == 0;
}

__global__ __launch_bounds__(OPT_THREADS) void grad_sqnorm_kernel(const OptSegment* segs, const OptChunk* chunks,
                                                                  float* partial) {
  __shared__ double red[8];
  int si, len; long off; bool vec;
  opt_chunk(chunks, si, off, len, vec);
  const float* g = segs[si].g + off;
  float s = 0.f;
  if (vec) {
    const int n4 = len >> 2;
    for (int i = threadIdx.x; i < n4; i += OPT_THREADS) {
      const float4 v = reinterpret_cast<const float4*>(g)[i];
      s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    for (int i = (n4 << 2) + threadIdx.x; i < len; i += OPT_THREADS) s += g[i] * g[i];
  } else {
    for (int i = threadIdx.x; i < len; i += OPT_THREADS) s += g[i] * g[i];
  }
  double v[1] = {(double)s};
  block_sum_d<1>(v, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = (float)v[0];
}

// every workgroup reduces the chunk partials itself (same order everywhere, so
// every workgroup derives the same coefficient); workgroup 0 reports the norm
__global__ __launch_bounds__(OPT_THREADS) void grad_clip_kernel(const OptSegment* segs, const OptChunk* chunks,
                                                                const float* partial, int nchunks, float max_norm,
                                                                float* total_norm) {
  __shared__ double red[8];
  __shared__ float coef_s;
  double acc = 0.0;
  for (int c = threadIdx.x; c < nchunks; c += OPT_THREADS) acc += (double)partial[c];
  double v[1] = {acc};
  block_sum_d<1>(v, red);
  if (threadIdx.x == 0) {
    const float tn = (float)sqrt(v[0]);
    float coef = max_norm / (tn + 1e-6f);   // torch: clip_coef = max_norm / (total_norm + 1e-6)
    coef = coef < 1.f ? coef : 1.f;         //        clamped to 1.0, always multiplied
    coef_s = coef;
    if (blockIdx.x == 0 && total_norm) *total_norm = tn;
  }
  __syncthreads();
  const float coef = coef_s;
  int si, len; long off; bool vec;
  opt_chunk(chunks, si, off, len, vec);
  float* g = segs[si].g + off;
  if (vec) {
    const int n4 = len >> 2;
    for (int i = threadIdx.x; i < n4; i += OPT_THREADS) {
      float4 x = reinterpret_cast<float4*>(g)[i];
      x.x *= coef; x.y *= coef; x.z *= coef; x.w *= coef;
      reinterpret_cast<float4*>(g)[i] = x;
    }
    for (int i = (n4 << 2) + threadIdx.x; i < len; i += OPT_THREADS) g[i] *= coef;
  } else {
    for (int i = threadIdx.x; i < len; i += OPT_THREADS) g[i] *= coef;
  }
}

// torch.optim.Adam (amsgrad=False, maximize=False), per element:
//   g += wd * p;  m = lerp(m, g, 1-b1);  v = b2 v + (1-b2) g^2
//   p -= step_size * m / (sqrt(v) / bc2_sqrt + eps),  step_size = lr / (1 - b1^t)
struct AdamStep { float step_size, bc2_sqrt; };
CTN_DEV void adam_elem(float& p, float g, float& m, float& v, const AdamArgs& a, const AdamStep& k) {
  g = a.wd != 0.f ? fmaf(a.wd, p, g) : g;
  m = fmaf(1.f - a.b1, g - m, m);   // exp_avg.lerp_(grad, 1 - beta1)
  v = fmaf(a.b2, v, (1.f - a.b2) * g * g);
  const float den = sqrtf(v) / k.bc2_sqrt + a.eps;
  p = p - k.step_size * (m / den);
}

// torch's bias corrections (torch.optim.Adam, non-capturable: Python doubles) for step t:
// step_size = lr / (1 - b1^t), bc2_sqrt = sqrt(1 - b2^t), in fp64 on the device, for the
// eager and the capturable launch alike (so both give the same bits at every step, and the
// capturable one has no step limit: t is the device counter + 1)
CTN_DEV AdamStep adam_bias(const AdamArgs& a) {
  const int t = a.counter ? *a.counter + 1 : a.step;
  const double lr = a.lr_dev ? (double)*a.lr_dev : (double)a.lr;
  const double bc1 = 1.0 - pow((double)a.b1, (double)t);
  const double bc2 = 1.0 - pow((double)a.b2, (double)t);
  return AdamStep{(float)(lr / bc1), (float)sqrt(bc2)};
}

__global__ __launch_bounds__(OPT_THREADS) void adam_kernel(const OptSegment* segs, const OptChunk* chunks,
                                                           AdamArgs a) {
  const AdamStep k = adam_bias(a);
  int si, len; long off; bool vec;
  opt_chunk(chunks, si, off, len, vec);
  const OptSegment s = segs[si];
  float* p = s.p + off;
  const float* g = s.g + off;
  float* m = s.m + off;
  float* v = s.v + off;
  int done = 0;
  if (vec) {
    const int n4 = len >> 2;
    for (int i = threadIdx.x; i < n4; i += OPT_THREADS) {
      float4 P = reinterpret_cast<float4*>(p)[i];
      const float4 G = reinterpret_cast<const float4*>(g)[i];
      float4 Mv = reinterpret_cast<float4*>(m)[i];
      float4 V = reinterpret_cast<float4*>(v)[i];
      adam_elem(P.x, G.x, Mv.x, V.x, a, k);
      adam_elem(P.y, G.y, Mv.y, V.y, a, k);
      adam_elem(P.z, G.z, Mv.z, V.z, a, k);
      adam_elem(P.w, G.w, Mv.w, V.w, a, k);
      reinterpret_cast<float4*>(p)[i] = P;
      reinterpret_cast<float4*>(m)[i] = Mv;
      reinterpret_cast<float4*>(v)[i] = V;
    }
    done = n4 << 2;
  }
  for (int i = done + threadIdx.x; i < len; i += OPT_THREADS) adam_elem(p[i], g[i], m[i], v[i], a, k);
}

__global__ void adam_bump_kernel(int* counter) {
  if (threadIdx.x == 0) *counter += 1;   // vector store: one lane of one wave
}

// Segment tables written by kernels whose arguments carry the entries (captured into a
// graph with the values of the capture, no host staging buffer): OPT_SEG_BATCH per launch
constexpr int OPT_SEG_BATCH = 64;
struct SegBatch { OptSegment e[OPT_SEG_BATCH]; int n; };
__global__ void write_segments_kernel(OptSegment* dst, SegBatch b) {
  const int i = threadIdx.x;
  if (i < b.n) dst[i] = b.e[i];
}

hipError_t launch_write_segments(OptSegment* dst, const OptSegment* src, int n, hipStream_t s) {
  if (!dst || (n > 0 && !src) || n < 0) return hipErrorInvalidValue;
  for (int i0 = 0; i0 < n; i0 += OPT_SEG_BATCH) {
    SegBatch b{};
    b.n = n - i0 < OPT_SEG_BATCH ? n - i0 : OPT_SEG_BATCH;
    for (int i = 0; i < b.n; ++i) b.e[i] = src[i0 + i];
    hipLaunchKernelGGL(write_segments_kernel, dim3(1), dim3(OPT_SEG_BATCH), 0, s, dst + i0, b);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_adam_dev(const OptSegment* segs, const OptChunk* chunks, int nchunks, const AdamArgs& a,
                           int* counter, hipStream_t s) {
  if (!segs || !chunks || nchunks < 0 || !counter) return hipErrorInvalidValue;
  AdamArgs ac = a;
  ac.counter = counter;
  if (nchunks > 0) hipLaunchKernelGGL(adam_kernel, dim3(nchunks), dim3(OPT_THREADS), 0, s, segs, chunks, ac);
  hipLaunchKernelGGL(adam_bump_kernel, dim3(1), dim3(64), 0, s, counter);
  return hipGetLastError();
}

static hipError_t opt_check(const OptSegment* segs, const OptChunk* chunks, int nchunks) {
  if (!segs || !chunks || nchunks < 0) return hipErrorInvalidValue;
  return hipSuccess;
}

hipError_t launch_grad_sqnorm(const OptSegment* segs, const OptChunk* chunks, int nchunks, float* partial,
                              hipStream_t s) {
  if (opt_check(segs, chunks, nchunks) != hipSuccess || !partial) return hipErrorInvalidValue;
  if (nchunks == 0) return hipSuccess;
  hipLaunchKernelGGL(grad_sqnorm_kernel, dim3(nchunks), dim3(OPT_THREADS), 0, s, segs, chunks, partial);
  return hipGetLastError();
}

hipError_t launch_grad_clip(const OptSegment* segs, const OptChunk* chunks, int nchunks, const float* partial,
                            float max_norm, float* total_norm, hipStream_t s) {
  if (opt_check(segs, chunks, nchunks) != hipSuccess || !partial) return hipErrorInvalidValue;
  if (nchunks == 0) return hipSuccess;
  hipLaunchKernelGGL(grad_clip_kernel, dim3(nchunks), dim3(OPT_THREADS), 0, s, segs, chunks, partial, nchunks,
                     max_norm, total_norm);
  return hipGetLastError();
}

hipError_t launch_adam(const OptSegment* segs, const OptChunk* chunks, int nchunks, const AdamArgs& a,
                       hipStream_t s) {
  if (opt_check(segs, chunks, nchunks) != hipSuccess) return hipErrorInvalidValue;
  if (nchunks == 0) return hipSuccess;
  hipLaunchKernelGGL(adam_kernel, dim3(nchunks), dim3(OPT_THREADS), 0, s, segs, chunks, a);
  return hipGetLastError();
}

}  // namespace ctn
