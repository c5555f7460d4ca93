// Run-to-run reproducibility of the dual GEMM (ctn_gemm_dual.hip): launches each pair
// repeatedly on fixed inputs and reports where outputs (C rows, D partials, statistics
// slab) differ from the first launch.  Diagnostic only; not part of the library.
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "../../conv-tasnet_amd/csrc/ctn_gemm_dual.hip"

using namespace ctn;

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
  const int M = argc > 1 ? atoi(argv[1]) : 3, K = argc > 2 ? atoi(argv[2]) : 1000;
  const int NRUN = argc > 3 ? atoi(argv[3]) : 20;
  const int NK = argc > 4 && argv[4][0] == 'c' ? NORM_CLN : NORM_GLN;
  const int Kp = (K + 127) / 128 * 128, B = 256, H = 512;
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
  const size_t nslab = rows * 16 + 4096;
  CK(hipMalloc(&slab, nslab * sizeof(double2)));
  const size_t ndp = 64L * B * H;
  CK(hipMalloc(&dpart, ndp * 4));

  for (int pair = 0; pair < 2; ++pair) {
    GemmDual g{};
    g.g = Rows{M, K, Kp};
    long cn;
    if (pair == 0) {
      g.Kred = B; g.Nout = H; g.norm = NK;
      g.A = gy; g.lda = B; g.W = w; g.ldw = B; g.C = out; g.ldc = H; g.epi = EPI_NORM_BWD; g.R = d; g.ldr = H;
      g.alpha = al; g.stats = (const float2*)st; g.gamma = gm; g.grp_slab = slab;
      g.Bm = d; g.ldb = H; g.bop.kind = OP_PRELU_NORM; g.bop.norm = NK; g.bop.stats = (const float2*)st;
      g.bop.gamma = gm; g.bop.beta = bt; g.bop.alpha = al; g.Dpart = dpart;
      cn = rows * H;
    } else {
      g.Kred = H; g.Nout = B; g.norm = NORM_GLN;
      g.A = d; g.lda = H; g.W = w; g.ldw = H; g.C = out; g.ldc = B; g.epi = EPI_RESID; g.R = gy; g.ldr = B;
      g.Bm = x; g.ldb = B; g.Dpart = dpart;
      cn = rows * B;
    }
    const int ranges = gemm_dual_ranges(g);
    const int E = pair == 0 && NK == NORM_CLN ? gemm_dual_group_parts(g) : 16;   // cLN entries per row
    const size_t nd = (size_t)ranges * g.Kred * g.Nout;
    std::vector<uint16_t> c0;
    std::vector<float> d0;
    std::vector<double2> s0;
    int bad = 0;
    for (int r = 0; r < NRUN; ++r) {
      CK(hipMemset(out, 0, cn * 2));
      CK(hipMemset(dpart, 0, nd * 4));
      CK(hipMemset(slab, 0, nslab * sizeof(double2)));
      CK(launch_gemm_dual(g, 0));
      CK(hipDeviceSynchronize());
      auto c = get<uint16_t>(out, cn);
      auto dd = get<float>(dpart, nd);
      auto ss = get<double2>(slab, nslab);
      if (pair == 0 && NK == NORM_CLN) {   // the per-row (sum ga, sum ga*ahat) entries against a host
        // recomputation from the bf16 C rows (approximate: the kernel sums fp32 accumulators)
        static std::vector<uint16_t> hd;
        if (hd.empty()) hd = get<uint16_t>(d, rows * H);
        auto bf = [](uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; };
        long nbad = 0, shown = 0;
        for (long row = 0; row < rows; ++row) {
          if (row % Kp >= K) continue;
          for (int e = 0; e < E; ++e) {
            double hs = 0, hq = 0;
            for (int ch = e * (H / E); ch < (e + 1) * (H / E); ++ch) {
              const float ga = bf(c[row * H + ch]);
              float x = bf(hd[row * H + ch]);
              x = x > 0.f ? x : 0.25f * x;
              hs += ga;
              hq += (double)ga * ((x - 0.1f) * 1.3f);
            }
            const double2 v = ss[row * E + e];
            const double tol = 0.02 * (fabs(hq) + fabs(hs)) + 0.05;
            if (fabs(v.x - hs) > tol || fabs(v.y - hq) > tol) {
              ++nbad;
              if (shown++ < 3) printf("   host check row %ld entry %d: kernel (%.6g, %.6g) host (%.6g, %.6g)\n", row, e, v.x, v.y, hs, hq);
            }
          }
        }
        printf("   run %d: %ld statistics entries off the host recomputation\n", r, nbad);
      }
      if (r == 0) { c0 = c; d0 = dd; s0 = ss; continue; }
      long nc = 0, ndd = 0, ns = 0, first_c = -1, first_d = -1, first_s = -1;
      std::vector<int> rowhist(32, 0), colhist(16, 0);
      for (long i = 0; i < cn; ++i)
        if (c[i] != c0[i]) {
          if (first_c < 0) first_c = i;
          ++nc;
          const long row = i / g.Nout, col = i % g.Nout;
          rowhist[row % 32]++;
          colhist[(col / 8) % 16]++;
        }
      for (size_t i = 0; i < nd; ++i)
        if (memcmp(&dd[i], &d0[i], 4)) { if (first_d < 0) first_d = i; ++ndd; }
      for (size_t i = 0; i < nslab; ++i)
        if (memcmp(&ss[i], &s0[i], sizeof(double2))) { if (first_s < 0) first_s = i; ++ns; }
      if (ns && pair == 0 && NK == NORM_CLN) {   // per-row slab: where in its range is each differing row
        const int ntile = (int)(rows / DU_TM), nr = ranges;
        std::vector<int> pos_from_end(8, 0), pos_from_start(8, 0);
        std::vector<int> lanegrp(4, 0), sl_nbg(16, 0);
        for (size_t i = 0; i < (size_t)rows * E; ++i)
          if (memcmp(&ss[i], &s0[i], sizeof(double2))) {
            const long row = i / E;
            const int t = (int)(row / DU_TM);
            int rr = 0;
            while ((long)ntile * (rr + 1) / nr <= t) ++rr;
            const int t0 = (int)((long)ntile * rr / nr), t1 = (int)((long)ntile * (rr + 1) / nr);
            pos_from_end[std::min(7, t1 - 1 - t)]++;
            pos_from_start[std::min(7, t - t0)]++;
            lanegrp[(row % DU_TM) / 8]++;
            sl_nbg[(i % E) * (16 / E)]++;
          }
        printf("   cLN slab diffs by tile position from range end:");
        for (int v : pos_from_end) printf(" %d", v);
        printf("\n   ... from range start:");
        for (int v : pos_from_start) printf(" %d", v);
        printf("\n   ... by row/8 within tile:");
        for (int v : lanegrp) printf(" %d", v);
        printf("\n   ... by (slice, wave column) entry:");
        for (int v : sl_nbg) printf(" %d", v);
        printf("\n");
      }
      if (ns && getenv("DET_VALUES")) {   // the first differing statistics entries, both runs
        int shown = 0;
        for (size_t i = 0; i < nslab && shown < 6; ++i)
          if (memcmp(&ss[i], &s0[i], sizeof(double2))) {
            printf("   slab[%zu] (row %zu, entry %zu): run0 (%.9g, %.9g) now (%.9g, %.9g)\n", i, i / E, i % E,
                   s0[i].x, s0[i].y, ss[i].x, ss[i].y);
            ++shown;
          }
      }
      if (nc || ndd || ns) {
        ++bad;
        printf("pair %c run %d: C %ld diffs (first row %ld col %ld)  Dpart %ld diffs (first range %ld)  slab %ld diffs (first %ld)\n",
               pair ? 'B' : 'A', r, nc, first_c < 0 ? -1 : first_c / g.Nout, first_c < 0 ? -1 : first_c % g.Nout, ndd,
               first_d < 0 ? -1 : first_d / ((long)g.Kred * g.Nout), ns, first_s);
        if (nc) {
          printf("   C diff rows mod 32:");
          for (int i = 0; i < 32; ++i) printf(" %d", rowhist[i]);
          printf("\n   C diff col/8 mod 16:");
          for (int i = 0; i < 16; ++i) printf(" %d", colhist[i]);
          printf("\n");
        }
      }
    }
    printf("pair %c (M=%d K=%d %s): %d of %d runs differ from the first\n", pair ? 'B' : 'A', M, K,
           NK == NORM_CLN ? "cLN" : "gLN", bad, NRUN - 1);
  }
  return 0;
}
