// Standalone timing of the dual GEMM (ctn_gemm_dual.hip) at the paper shapes
// (M=32 utterances, K=3199 frames, Kp=3200), for bound-finding experiments:
// build with -DCTN_DU_EXP=<bits>.  Not part of the library.
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "../../conv-tasnet_amd/csrc/ctn_gemm_dual.hip"

using namespace ctn;
#ifndef DB_CLN
#define DB_CLN 0   // 1: pair A with per-row (cLN) statistics
#endif

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static void* dev_fill(size_t bytes, unsigned seed) {
  std::vector<uint16_t> h(bytes / 2);
  unsigned x = seed;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (uint16_t)(0x3c00 + ((x >> 16) & 0x3ff)) ^ ((x >> 8) & 0x8000); }
  void* d; CK(hipMalloc(&d, bytes)); CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
  return d;
}

__global__ __launch_bounds__(256) void stream_kernel(const v4u* a, v4u* c, long na, long nc) {
  const long n = na > nc ? na : nc;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    v4u v = {0u, 0u, 0u, 0u};
    if (i < na) v = a[i];
    if (i < nc) c[i] = v + v4u{1u, 1u, 1u, 1u};
  }
}

int main() {
  // DB_M: utterances (default 32; the fixed per-launch cost is the intercept over M)
  const int M = getenv("DB_M") ? atoi(getenv("DB_M")) : 32, K = 3199, Kp = 3200, B = 256, H = 512;
  const long rows = (long)M * Kp;
  void* x = dev_fill(rows * B * 2, 1);
  void* gy = dev_fill(rows * B * 2, 5);
  void* d = dev_fill(rows * H * 2, 2);
  void* out = dev_fill(rows * H * 2, 3);
  void* w = dev_fill((size_t)B * H * 2, 4);
  std::vector<float> hs(2 * rows), hg(H, 1.0f), hb(H, 0.1f);
  for (long i = 0; i < rows; ++i) { hs[2 * i] = 0.1f; hs[2 * i + 1] = 1.3f; }
  float *st, *gm, *bt, *al, *dpart; double2* slab;
  CK(hipMalloc(&st, hs.size() * 4)); CK(hipMemcpy(st, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&gm, H * 4)); CK(hipMemcpy(gm, hg.data(), H * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&bt, H * 4)); CK(hipMemcpy(bt, hb.data(), H * 4, hipMemcpyHostToDevice));
  float a0 = 0.25f; CK(hipMalloc(&al, 4)); CK(hipMemcpy(al, &a0, 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&slab, rows * 16 * sizeof(double2)));
  CK(hipMalloc(&dpart, 64L * B * H * 4));

  struct Case { const char* name; GemmDual g; double bytes; };
  std::vector<Case> cs;
  {
    GemmDual g{}; g.g = Rows{M, K, Kp}; g.Kred = B; g.Nout = H; g.norm = DB_CLN ? NORM_CLN : NORM_GLN;
    g.A = gy; g.lda = B; g.W = w; g.ldw = B; g.C = out; g.ldc = H; g.epi = EPI_NORM_BWD; g.R = d; g.ldr = H;
    g.alpha = al; g.stats = (const float2*)st; g.gamma = gm; g.grp_slab = slab;
    g.Bm = d; g.ldb = H; g.bop.kind = OP_PRELU_NORM; g.bop.norm = g.norm; g.bop.stats = (const float2*)st;
    g.bop.gamma = gm; g.bop.beta = bt; g.bop.alpha = al; g.Dpart = dpart;
    if (getenv("DB_FRAG")) g.Wf = w;   // timing: the fragment-order load pattern
    cs.push_back({"A: gy.W2t norm-bwd + dW2", g, rows * (B + 2 * H) * 2.0});
  }
  {
    GemmDual g{}; g.g = Rows{M, K, Kp}; g.Kred = H; g.Nout = B; g.norm = NORM_GLN;
    g.A = d; g.lda = H; g.W = w; g.ldw = H; g.C = out; g.ldc = B; g.epi = EPI_RESID; g.R = gy; g.ldr = B;
    g.Bm = x; g.ldb = B; g.Dpart = dpart;
    if (getenv("DB_FRAG")) g.Wf = w;
    cs.push_back({"B: gh1.W1t + gy + dW1", g, rows * (H + 3 * B) * 2.0});
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int NIT = 20;
  for (auto& c : cs) {
    for (int i = 0; i < 3; ++i) CK(launch_gemm_dual(c.g, 0));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < NIT; ++i) CK(launch_gemm_dual(c.g, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / NIT;
    printf("EXP %3d M=%d  %-30s %8.1f us  %7.0f GB/s\n", CTN_DU_EXP, M, c.name, us, c.bytes / us * 1e-3);
#if CTN_DU_STAMP
    {   // per-phase shares of the loop (diagnostic build: read shares, not lengths)
      std::vector<unsigned long long> h(DU_GRID * DU_WV * 8);
      CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(du_stamps), h.size() * 8));
      const char* nm[8] = {"vmwait", "barrier", "store_c", "dma", "transform", "compute", "epilogue", "prologue"};
      double sum[8] = {0}, tot = 0;
      for (size_t w = 0; w < h.size() / 8; ++w)
        for (int i = 0; i < 8; ++i) sum[i] += (double)h[w * 8 + i];
      for (int i = 0; i < 7; ++i) tot += sum[i];
      const int tiles = (int)(rows / DU_TM) / (DU_GRID / (c.g.Nout / (c.g.Kred == 256 ? 128 : 64)));
      for (int i = 0; i < 8; ++i)
        printf("   %-10s %5.1f %%  %8.0f cyc/tile/wave\n", nm[i], 100.0 * sum[i] / tot, sum[i] / (h.size() / 8) / tiles);
    }
#endif
  }
  if (CTN_DU_EXP == 0) {   // streaming calibration: copy d -> out (both rows x H bf16)
    const long n = rows * H * 2 / 16;
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(stream_kernel, dim3(4096), dim3(256), 0, 0, (const v4u*)d, (v4u*)out, n, n);
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < NIT; ++i) hipLaunchKernelGGL(stream_kernel, dim3(4096), dim3(256), 0, 0, (const v4u*)d, (v4u*)out, n, n);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / NIT;
    printf("M=%d stream copy (%ld MB read, %ld MB written) %8.1f us %7.0f GB/s\n", M, n * 16 >> 20, n * 16 >> 20, us,
           2.0 * n * 16 / us * 1e-3);
  }
  return 0;
}
