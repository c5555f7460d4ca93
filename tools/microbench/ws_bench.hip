// Standalone timing of the weight-stationary row GEMM at the paper shapes
// (M=32 utterances, K=3199 frames, Kp=3200), for bound-finding experiments:
// build with -DCTN_WS_EXP=<bits> (see ctn_gemm_ws.hip).  Not part of the library.
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#include "../../conv-tasnet_amd/csrc/ctn_gemm_ws.hip"

using namespace ctn;

// the library's device error word (ctn_capi.hip), here one word of this process
uint32_t* ctn::device_error_word() {
  static uint32_t* w = nullptr;
  if (!w && hipMalloc(&w, 4) == hipSuccess) (void)hipMemset(w, 0, 4);
  return w;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static void* dev_fill(size_t bytes, unsigned seed) {
  std::vector<uint16_t> h(bytes / 2);
  unsigned x = seed;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (uint16_t)(0x3c00 + ((x >> 16) & 0x3ff)) ^ ((x >> 8) & 0x8000); }
  void* d; CK(hipMalloc(&d, bytes)); CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
  return d;
}

// streaming calibration: out[i] = f(in[i % nin]) with nin/nout row counts like the GEMM
// operands (reads rows*kin, writes rows*kout bf16), 8 waves per CU or more
__global__ __launch_bounds__(256) void stream_kernel(const v4u* a, v4u* c, long na, long nc) {
  const long n = na > nc ? na : nc;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    v4u v = {0u, 0u, 0u, 0u};
    if (i < na) v = a[i];
    if (i < nc) c[i] = v + v4u{1u, 1u, 1u, 1u};
  }
}

int main() {
  // WSB_M: utterances (default 32; the fixed per-launch cost is the intercept over M)
  const int M = getenv("WSB_M") ? atoi(getenv("WSB_M")) : 32, K = 3199, Kp = 3200, B = 256, H = 512;
  const long rows = (long)M * Kp;
  void* x = dev_fill(rows * B * 2, 1);
  void* d = dev_fill(rows * H * 2, 2);
  void* out = dev_fill(rows * H * 2, 3);
  void* w = dev_fill((size_t)B * H * 2, 4);
  std::vector<float> hs(2 * rows), hg(H, 1.0f), hb(H, 0.1f);
  for (long i = 0; i < rows; ++i) { hs[2 * i] = 0.1f; hs[2 * i + 1] = 1.3f; }
  float *st, *gm, *bt, *al; double2* slab;
  CK(hipMalloc(&st, hs.size() * 4)); CK(hipMemcpy(st, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&gm, H * 4)); CK(hipMemcpy(gm, hg.data(), H * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&bt, H * 4)); CK(hipMemcpy(bt, hb.data(), H * 4, hipMemcpyHostToDevice));
  float a0 = 0.25f; CK(hipMalloc(&al, 4)); CK(hipMemcpy(al, &a0, 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&slab, rows * 8 * sizeof(double2)));

  struct Case { const char* name; GemmRows g; double bytes; };
  std::vector<Case> cs;
  auto base = [&](int Kred, int Nout) { GemmRows g{}; g.g = Rows{M, K, Kp}; g.Kred = Kred; g.Nout = Nout; g.norm = NORM_GLN;
    g.lda = Kred; g.ldw = Kred; g.ldc = Nout; g.alpha = al; g.grp_slab = slab; g.W = w;
    if (getenv("WSB_FRAG")) g.Wf = w;   // timing: the fragment-order load pattern (values not meaningful)
    return g; };
  { GemmRows g = base(B, H); g.A = x; g.C = out; g.epi = EPI_PRELU_STATS; cs.push_back({"fwd1 x.W1 prelu-stats", g, rows * (B + H) * 2.0}); }
  { GemmRows g = base(H, B); g.A = d; g.C = out; g.epi = EPI_RESID; g.R = x; g.ldr = B;
    g.aop.kind = OP_PRELU_NORM; g.aop.norm = NORM_GLN; g.aop.stats = (const float2*)st; g.aop.gamma = gm; g.aop.beta = bt; g.aop.alpha = al;
    cs.push_back({"fwd2 n2.W2 + x", g, rows * (H + 2 * B) * 2.0}); }
  {   // cLN operand (per-row statistics loaded with the rows) and cLN residual form (c4's output GEMM)
    GemmRows g = base(H, B); g.A = d; g.C = out; g.epi = EPI_RESID; g.R = x; g.ldr = B; g.norm = NORM_CLN;
    g.aop.kind = OP_PRELU_NORM; g.aop.norm = NORM_CLN; g.aop.stats = (const float2*)st; g.aop.gamma = gm; g.aop.beta = bt; g.aop.alpha = al;
    cs.push_back({"fwd2 n2.W2 + x (cLN)", g, rows * (H + 2 * B) * 2.0}); }
  {   // the same with the gLN operand statistics folded from producer partials in every
      // workgroup's prologue (the library's consumer-finalized form: 144 partials per utterance)
    GemmRows g = base(H, B); g.A = d; g.C = out; g.epi = EPI_RESID; g.R = x; g.ldr = B;
    g.aop.kind = OP_PRELU_NORM; g.aop.norm = NORM_GLN; g.aop.gamma = gm; g.aop.beta = bt; g.aop.alpha = al;
    static double2* fslab = nullptr;
    if (!fslab) {
      std::vector<double2> hf((size_t)M * 144);
      for (auto& v : hf) { v.x = 0.01; v.y = 0.02; }
      CK(hipMalloc(&fslab, hf.size() * sizeof(double2)));
      CK(hipMemcpy(fslab, hf.data(), hf.size() * sizeof(double2), hipMemcpyHostToDevice));
    }
    g.aop.fold.slab = fslab; g.aop.fold.parts = 144; g.aop.fold.cnt = 144.0 * 0.5; g.aop.fold.eps = 1e-8f;
    cs.push_back({"fwd2 n2.W2 + x (fold)", g, rows * (H + 2 * B) * 2.0}); }
  { GemmRows g = base(B, H); g.A = x; g.C = out; g.epi = EPI_NORM_BWD; g.R = d; g.ldr = H; g.stats = (const float2*)st; g.gamma = gm;
    cs.push_back({"bwd gy.W2t norm-bwd", g, rows * (B + 2 * H) * 2.0}); }
  { GemmRows g = base(H, B); g.A = d; g.C = out; g.epi = EPI_RESID; g.R = x; g.ldr = B; cs.push_back({"bwd gh1.W1t + gy", g, rows * (H + 2 * B) * 2.0}); }

  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  {
    struct SC { const char* name; long rd, wr; };
    const SC sc[] = {{"stream r52MB w105MB", rows * B * 2, rows * H * 2}, {"stream r105MB w52MB", rows * H * 2, rows * B * 2},
                     {"stream r105MB w0", rows * H * 2, 0}, {"stream r0 w105MB", 0, rows * H * 2}};
    for (const auto& c : sc) {
      for (int grid : {1024, 4096}) {
      if (getenv("WSB_NOSTREAM")) break;
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(stream_kernel, dim3(grid), dim3(256), 0, 0, (const v4u*)d, (v4u*)out, c.rd / 16, c.wr / 16);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(stream_kernel, dim3(grid), dim3(256), 0, 0, (const v4u*)d, (v4u*)out, c.rd / 16, c.wr / 16);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / 20;
        printf("%-24s grid %5d %8.1f us  %7.0f GB/s\n", c.name, grid, us, (c.rd + c.wr) / (us * 1e-6) / 1e9);
      }
    }
  }
  for (auto& c : cs) {
    if (hipError_t e = launch_gemm_ws(c.g, 0); e != hipSuccess) {   // a case this build does not take
      printf("EXP=%d  %-24s skipped: %s\n", CTN_WS_EXP, c.name, hipGetErrorString(e));
      continue;
    }
    for (int i = 0; i < 3; ++i) CK(launch_gemm_ws(c.g, 0));
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) CK(launch_gemm_ws(c.g, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    printf("EXP=%d M=%d  %-24s %8.1f us  %7.0f GB/s (alg)\n", CTN_WS_EXP, M, c.name, us, c.bytes / (us * 1e-6) / 1e9);
#if CTN_WS_STAMP
    {   // per-phase shares of the loop (diagnostic build: read shares, not lengths)
      std::vector<unsigned long long> h(256 * 16 * 8, 0ull);
      CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(ws_stamps), h.size() * 8));
      const char* nm[8] = {"barrier", "mfma", "stage", "load_a", "epi_math", "load_r", "stores", "loop"};
      double sum[8] = {0}, tot = 0;
      for (size_t w = 0; w < h.size() / 8; ++w)
        for (int i = 0; i < 8; ++i) sum[i] += (double)h[w * 8 + i];
      for (int i = 0; i < 8; ++i) tot += sum[i];
      for (int i = 0; i < 8; ++i) printf("   %-9s %5.1f %%\n", nm[i], 100.0 * sum[i] / tot);
      std::fill(h.begin(), h.end(), 0ull);
      CK(hipMemcpyToSymbol(HIP_SYMBOL(ws_stamps), h.data(), h.size() * 8));
    }
#endif
  }
  return 0;
}
