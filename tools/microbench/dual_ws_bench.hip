// Pair-A dual GEMM at the paper shapes: the wave-specialised kernel (ctn_dual_ws.hip)
// against gemm_dual_kernel (ctn_gemm_dual.hip) on the same inputs.
//   * C and the dW2 partials bit for bit, the norm-2 statistics per group (sum of
//     each kernel's partials) to 1e-9 relative;
//   * run-to-run reproducibility of the wave-specialised kernel (every output byte);
//   * time per launch (hipEvents over NIT launches).
// Build with -DCTN_DV_EXP=<bits> for the bound-finding variants (timing only).
// Usage: dual_ws_bench [M] [K] [g|c] [runs].  Not part of the library.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../conv-tasnet_amd/csrc/ctn_dual_ws.hip"
#include "../../conv-tasnet_amd/csrc/ctn_gemm_dual.hip"

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
template <typename T> static std::vector<T> get(const void* d, size_t n) {
  std::vector<T> h(n);
  CK(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
  return h;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 32, K = argc > 2 ? atoi(argv[2]) : 3199;
  const int NK = argc > 3 && argv[3][0] == 'c' ? NORM_CLN : NORM_GLN;
  const int NRUN = argc > 4 ? atoi(argv[4]) : 10;
  const int Kp = (K + 127) / 128 * 128, B = 256, H = 512;
  const long rows = (long)M * Kp;
  void* gy = dev_fill(rows * B * 2, 5);
  void* d = dev_fill(rows * H * 2, 2);
  void* out = dev_fill(rows * H * 2, 3);
  void* w = dev_fill((size_t)B * H * 2, 4);
  // statistics: gLN per utterance, cLN per row (padded rows: not finite, as the forward leaves them)
  const long G = NK == NORM_GLN ? M : rows;
  std::vector<float> hs(2 * G), hg(H), hb(H);
  for (long i = 0; i < G; ++i) {
    const bool pad = NK == NORM_CLN && i % Kp >= K;
    hs[2 * i] = pad ? NAN : 0.1f + 0.01f * (i % 7);
    hs[2 * i + 1] = pad ? INFINITY : 1.3f - 0.02f * (i % 5);
  }
  for (int i = 0; i < H; ++i) { hg[i] = 0.8f + 0.001f * i; hb[i] = 0.1f - 0.0003f * i; }
  float *st, *gm, *bt, *al, *dpart; double2* slab;
  CK(hipMalloc(&st, hs.size() * 4)); CK(hipMemcpy(st, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&gm, H * 4)); CK(hipMemcpy(gm, hg.data(), H * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&bt, H * 4)); CK(hipMemcpy(bt, hb.data(), H * 4, hipMemcpyHostToDevice));
  float a0 = 0.25f; CK(hipMalloc(&al, 4)); CK(hipMemcpy(al, &a0, 4, hipMemcpyHostToDevice));
  const size_t nslab = (size_t)rows * 16 + 65536;
  CK(hipMalloc(&slab, nslab * sizeof(double2)));
  CK(hipMalloc(&dpart, 64L * B * H * 4));

  GemmDual g{}; g.g = Rows{M, K, Kp}; g.Kred = B; g.Nout = H; g.norm = NK;
  g.A = gy; g.lda = B; g.W = w; g.ldw = B; g.C = out; g.ldc = H; g.epi = EPI_NORM_BWD; g.R = d; g.ldr = H;
  g.alpha = al; g.stats = (const float2*)st; g.gamma = gm; g.grp_slab = slab;
  g.Bm = d; g.ldb = H; g.bop.kind = OP_PRELU_NORM; g.bop.norm = NK; g.bop.stats = (const float2*)st;
  g.bop.gamma = gm; g.bop.beta = bt; g.bop.alpha = al; g.Dpart = dpart;
  if (getenv("DB_FRAG")) g.Wf = w;   // timing: the fragment-order load pattern
  const long cn = rows * H;
  const size_t nd = (size_t)gemm_dual_ranges(g) * B * H;

  struct Out { std::vector<uint16_t> c; std::vector<float> dp; std::vector<double> grp_s, grp_q; };
  auto launch_once = [&](bool ws, Out* o) {
    setenv("CTN_DUAL_WS", ws ? "1" : "0", 1);
    CK(hipMemset(out, 0, cn * 2));
    CK(hipMemset(dpart, 0, nd * 4));
    CK(hipMemset(slab, 0, nslab * sizeof(double2)));
    CK(launch_gemm_dual(g, 0));
    CK(hipDeviceSynchronize());
    if (!o) return;
    o->c = get<uint16_t>(out, cn);
    o->dp = get<float>(dpart, nd);
    // per-group totals of the statistics partials, by each kernel's layout
    const int parts = gemm_dual_group_parts(g);
    const auto sl = get<double2>(slab, nslab);
    o->grp_s.assign(G, 0.0);
    o->grp_q.assign(G, 0.0);
    if (NK == NORM_GLN) {
      const WsRuns wr = gemm_dual_runs(g);
      for (int m = 0; m < M; ++m) {
        const int blo = ws_block_of_tile(wr, m * wr.tpu), bhi = ws_block_of_tile(wr, (m + 1) * wr.tpu - 1);
        for (int b = blo; b <= bhi; ++b) {
          const int t0 = ws_t0(wr, b);
          if (t0 >= ws_t0(wr, b + 1)) continue;
          for (int wv = 0; wv < wr.waves; ++wv) {
            const double2 v = sl[((size_t)b * wr.waves + wv) * wr.kmax + (m - t0 / wr.tpu)];
            o->grp_s[m] += v.x;
            o->grp_q[m] += v.y;
          }
        }
      }
    } else {
      for (long r = 0; r < rows; ++r)
        for (int i = 0; i < parts; ++i) { o->grp_s[r] += sl[r * parts + i].x; o->grp_q[r] += sl[r * parts + i].y; }
    }
  };

#if CTN_DV_DBG & 8
  {   // per-tile, per-lane epilogue sums and their inputs (stored to g.R by the kernel), run to run
    const size_t nrec = (size_t)(rows / 32) * (H / 128) * 8 * 64;   // records of 12 words
    void* dbg; CK(hipMalloc(&dbg, nrec * 48));
    g.R = dbg;
    const auto hd = get<uint16_t>(d, cn);
    std::vector<uint32_t> first;
    const char* fld[12] = {"s", "q", "alpha", "-", "r0.x", "r0.y", "r1.x", "r1.y", "e0.m", "e0.r", "e1.m", "e1.r"};
    for (int r = 0; r < NRUN; ++r) {
      CK(hipMemset(dbg, 0, nrec * 48));
      launch_once(true, nullptr);
      auto v = get<uint32_t>(dbg, nrec * 12);
      if (r == 0) { first = v; continue; }
      long nf[12] = {0};
      long shown = 0;
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i] != first[i]) {
          ++nf[i % 12];
          const size_t rec = i / 12;
          const long lane = rec % 64, w = rec / 64 % 8, sl = rec / 512 % 4, t = rec / 2048;
          if (shown++ < 4)
            printf("   tile %ld slice %ld wave %ld lane %ld field %s: 0x%08x vs 0x%08x\n", t, sl, w, lane, fld[i % 12],
                   v[i], first[i]);
        }
      printf("run %d differing fields:", r);
      for (int f = 0; f < 12; ++f) printf(" %s=%ld", fld[f], nf[f]);
      printf("\n");
      // the r values against d itself: lane (lg, lr) of wave w reads row lr / 16+lr, channels
      // n0 + 32*(w/2) + 8*lg + 4*(w&1) .. +3
      long bad = 0;
      for (size_t rec = 0; rec < nrec; ++rec) {
        const long lane = rec % 64, w = rec / 64 % 8, sl = rec / 512 % 4, t = rec / 2048;
        const long ch = sl * 128 + 32 * (w / 2) + 8 * (lane >> 4) + 4 * (w & 1);
        for (int j = 0; j < 2; ++j) {
          const long row = t * 32 + 16 * j + (lane & 15);
          const uint32_t lo = hd[row * H + ch] | ((uint32_t)hd[row * H + ch + 1] << 16);
          const uint32_t hi = hd[row * H + ch + 2] | ((uint32_t)hd[row * H + ch + 3] << 16);
          bad += v[rec * 12 + 4 + 2 * j] != lo;
          bad += v[rec * 12 + 5 + 2 * j] != hi;
        }
      }
      printf("   r values off d: %ld\n", bad);
    }
    return 0;
  }
#endif
#if CTN_DV_DBG & 16
  {   // the consumers' R-image reads, stored in place of C: every value must be d's
    const auto hd = get<uint16_t>(d, cn);
    for (int r = 0; r < NRUN; ++r) {
      Out o;
      launch_once(true, &o);
      long n = 0, first = -1;
      for (long i = 0; i < cn; ++i)
        if (o.c[i] != hd[i]) { if (first < 0) first = i; ++n; }
      printf("R-image readback run %d: %ld of %ld values differ from d (first row %ld col %ld)\n", r, n, cn,
             first < 0 ? -1 : first / H, first < 0 ? -1 : first % H);
    }
    return 0;
  }
#endif
  Out ref, cur;
  launch_once(false, &ref);
  launch_once(true, &cur);
  long dc = 0, ddp = 0, dst = 0;
  for (long i = 0; i < cn; ++i) dc += cur.c[i] != ref.c[i];
  for (size_t i = 0; i < nd; ++i) ddp += memcmp(&cur.dp[i], &ref.dp[i], 4) != 0;
  double worst = 0.0;
  for (long i = 0; i < G; ++i) {
    if (NK == NORM_CLN && i % Kp >= K) continue;
    const double es = fabs(cur.grp_s[i] - ref.grp_s[i]) / (fabs(ref.grp_s[i]) + 1e-3);
    const double eq = fabs(cur.grp_q[i] - ref.grp_q[i]) / (fabs(ref.grp_q[i]) + 1e-3);
    const double e = es > eq ? es : eq;
    if (e > 1e-6) ++dst;
    if (e > worst) worst = e;
  }
  printf("M=%d K=%d %s  ws vs old: C %ld diffs, Dpart %ld diffs, stats %ld groups > 1e-6 (worst %.3g)\n", M, K,
         NK == NORM_GLN ? "gLN" : "cLN", dc, ddp, dst, worst);

  // run-to-run reproducibility of the wave-specialised kernel
  int bad = 0;
  for (int r = 0; r < NRUN; ++r) {
    Out o;
    launch_once(true, &o);
    long n = 0;
    for (long i = 0; i < cn; ++i) n += o.c[i] != cur.c[i];
    for (size_t i = 0; i < nd; ++i) n += memcmp(&o.dp[i], &cur.dp[i], 4) != 0;
    for (long i = 0; i < G; ++i) n += memcmp(&o.grp_s[i], &cur.grp_s[i], 8) != 0 || memcmp(&o.grp_q[i], &cur.grp_q[i], 8) != 0;
    if (n) { ++bad; printf("   run %d: %ld differing outputs\n", r, n); }
  }
  printf("reproducibility: %d of %d launches differ from the first\n", bad, NRUN);

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int NIT = 20;
  const double bytes = rows * (B + 2 * H) * 2.0;
  for (int ws = 1; ws >= 0; --ws) {
    setenv("CTN_DUAL_WS", ws ? "1" : "0", 1);
    for (int i = 0; i < 3; ++i) CK(launch_gemm_dual(g, 0));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < NIT; ++i) CK(launch_gemm_dual(g, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / NIT;
    printf("EXP %d %-4s M=%d K=%d %s %8.1f us  %7.0f GB/s (alg. bytes)\n", CTN_DV_EXP, ws ? "ws" : "old", M, K,
           NK == NORM_GLN ? "gLN" : "cLN", us, bytes / us * 1e-3);
  }
#if CTN_DV_STAMP
  {   // per-role wait shares of the wave-specialised kernel (one more launch, stamps zeroed)
    std::vector<unsigned long long> h(1024 * 16 * 4, 0ull);
    CK(hipMemcpyToSymbol(HIP_SYMBOL(dv_stamps), h.data(), h.size() * 8));
    setenv("CTN_DUAL_WS", "1", 1);
    CK(launch_gemm_dual(g, 0));
    CK(hipDeviceSynchronize());
    CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(dv_stamps), h.size() * 8));
    const int nwg = gemm_dual_ws_ranges(g) * (H / 128);
    const char* role[3] = {"row", "column", "memory"};
    for (int r = 0; r < 3; ++r) {
      double acc[4] = {0, 0, 0, 0};
      int n = 0;
      for (int b = 0; b < nwg; ++b)
        for (int w = 0; w < 16; ++w) {
          const int rr = w < 4 ? 0 : w < 12 ? 1 : 2;
          if (rr != r) continue;
          ++n;
          for (int i = 0; i < 4; ++i) acc[i] += (double)h[((size_t)b * 16 + w) * 4 + i];
        }
      printf("STAMP %-6s loop %8.0f cyc  full-wait %5.1f%%  dma-vmcnt %5.1f%%  done-wait %5.1f%%\n", role[r],
             acc[3] / n, 100 * acc[0] / acc[3], 100 * acc[1] / acc[3], 100 * acc[2] / acc[3]);
    }
  }
#endif
  // the same kernel's COLS mode (dW1 = gh1^T . x shape: A = d [rows][H], B = gy [rows][B])
  {
    GemmCols c{};
    c.g = g.g; c.P = H; c.Q = B;
    c.A = d; c.lda = H; c.B = gy; c.ldb = B;
    c.nchunks = gemm_cols_ws_ranges(c);
    float* cp; CK(hipMalloc(&cp, (size_t)c.nchunks * H * B * 4));
    c.Cpart = cp;
    if (gemm_cols_ws_eligible(BF16, c)) {
      for (int i = 0; i < 3; ++i) CK(launch_gemm_cols_ws(c, 0));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < NIT; ++i) CK(launch_gemm_cols_ws(c, 0));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / NIT, cb = rows * (B + H) * 2.0;
      printf("COLS CJC=%d M=%d K=%d %8.1f us  %7.0f GB/s (alg. bytes, %d ranges)\n", CTN_DV_CJC, M, K, us, cb / us * 1e-3,
             c.nchunks);
    }
  }
  return 0;
}
