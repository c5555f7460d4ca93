// extern "C" entry points of libctn_hip.so (include/ctn.h) and the native
// launch sequences behind them.  Each entry validates its descriptor, carves
// the caller's workspace, and enqueues its kernels on the caller's stream.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "../../include/ctn.h"
#include "ctn_common.h"
#include "ctn_kernels.h"

using namespace ctn;

static thread_local char g_err[512] = "";

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

#define CTN_HIP(expr)                                                               \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) return fail(CTN_ERR_HIP, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

static constexpr double kEps = 1e-8;   // conv_tasnet.py:10

// ---------------------------------------------------------------------------
// kernel timer (bench.py roofline measurement)
// ---------------------------------------------------------------------------
namespace {
struct Timer {
  std::mutex mu;
  int kind = 0, cap = 0, used = 0;
  std::vector<hipEvent_t> ev;   // pairs
};
Timer g_timer;

struct TimedScope {
  hipStream_t s;
  int idx = -1;
  TimedScope(int kind, hipStream_t st) : s(st) {
    if (g_timer.kind != kind) return;
    std::lock_guard<std::mutex> lk(g_timer.mu);
    if (g_timer.used >= g_timer.cap) return;
    idx = g_timer.used++;
    (void)hipEventRecord(g_timer.ev[2 * idx], s);
  }
  ~TimedScope() {
    if (idx >= 0) (void)hipEventRecord(g_timer.ev[2 * idx + 1], s);
  }
};
}  // namespace

extern "C" int ctn_timer_enable(int kind, int max_launches) {
  std::lock_guard<std::mutex> lk(g_timer.mu);
  for (auto e : g_timer.ev) (void)hipEventDestroy(e);
  g_timer.ev.clear();
  g_timer.kind = kind;
  g_timer.cap = kind ? max_launches : 0;
  g_timer.used = 0;
  g_timer.ev.resize(2 * (size_t)g_timer.cap);
  for (auto& e : g_timer.ev) CTN_HIP(hipEventCreate(&e));
  return CTN_OK;
}

extern "C" int ctn_timer_read(double* total_ms, int* launches) {
  std::lock_guard<std::mutex> lk(g_timer.mu);
  double t = 0.0;
  for (int i = 0; i < g_timer.used; ++i) {
    CTN_HIP(hipEventSynchronize(g_timer.ev[2 * i + 1]));
    float ms = 0.f;
    CTN_HIP(hipEventElapsedTime(&ms, g_timer.ev[2 * i], g_timer.ev[2 * i + 1]));
    t += ms;
  }
  if (total_ms) *total_ms = t;
  if (launches) *launches = g_timer.used;
  return CTN_OK;
}

// ---------------------------------------------------------------------------
// workspace carving
// ---------------------------------------------------------------------------
namespace {
struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base((char*)b) {}
  template <typename P> P* take(size_t bytes) {
    off = (off + 255) & ~(size_t)255;
    P* p = base ? reinterpret_cast<P*>(base + off) : nullptr;
    off += bytes;
    return p;
  }
};
size_t esize(int dt) { return dt == CTN_DTYPE_BF16 ? 2 : 4; }
}  // namespace

extern "C" int ctn_abi_version(void) { return CTN_ABI_VERSION; }
extern "C" const char* ctn_last_error(void) { return g_err; }
extern "C" int ctn_padded_frames(int K) { return ((K + 127) / 128) * 128; }

// ===========================================================================
// TemporalBlock
// ===========================================================================
static int tb_check(const ctn_tblock_desc* d) {
  if (!d) return fail(CTN_ERR_ARG, "null descriptor");
  if (d->M < 1 || d->K < 1 || d->Kp < d->K || d->Kp % 128)
    return fail(CTN_ERR_ARG, "bad frame geometry M=%d K=%d Kp=%d (Kp must be a multiple of 128 >= K)", d->M,
                d->K, d->Kp);
  if (d->B % 8 || d->H % 8 || d->B < 8 || d->H < 8)
    return fail(CTN_ERR_UNSUPPORTED, "B=%d H=%d must be multiples of 8", d->B, d->H);
  if (d->H / 8 > 256) return fail(CTN_ERR_UNSUPPORTED, "H=%d > 2048", d->H);
  if (d->P < 1 || d->P > 8) return fail(CTN_ERR_UNSUPPORTED, "P=%d outside 1..8", d->P);
  if (!d->causal && d->P % 2 == 0)
    return fail(CTN_ERR_ARG, "non-causal padding (P-1)*d//2 needs odd P (conv_tasnet.py:236)");
  if (d->norm_type != CTN_NORM_GLN && d->norm_type != CTN_NORM_CLN)
    return fail(CTN_ERR_UNSUPPORTED, "norm_type %d (BN) not implemented on the HIP path", d->norm_type);
  if (d->norm_type == CTN_NORM_CLN) {
    const int cg = d->H / 8;
    if (cg > 64 || (cg & (cg - 1))) return fail(CTN_ERR_UNSUPPORTED, "cLN needs H/8 a power of two <= 64");
  }
  if (d->dtype != CTN_DTYPE_F32 && d->dtype != CTN_DTYPE_BF16) return fail(CTN_ERR_ARG, "dtype %d", d->dtype);
  if (d->dilation < 1) return fail(CTN_ERR_ARG, "dilation %d", d->dilation);
  return CTN_OK;
}

static int tb_groups(const ctn_tblock_desc* d) { return d->norm_type == CTN_NORM_GLN ? d->M : d->M * d->Kp; }

extern "C" int ctn_tblock_stats_floats(const ctn_tblock_desc* d) { return 4 * tb_groups(d); }

namespace {
struct TbLayout {
  // forward
  void *w1s, *w2s;
  double2 *slab1, *slab2;
  // backward
  void *w1t, *w2t, *G1, *G2;
  double2 *slabA, *slabD;
  float *colA, *colD, *alphaSlab, *cpart1, *cpart2;
  float2 *sums1, *sums2;
  int parts1, parts2, partsA, partsD, chunks1, chunks2, rowtiles;
  size_t bytes;
};

GemmRows tb_gemm1(const ctn_tblock_desc* d) {   // x[.,B] -> h1[.,H]
  GemmRows g{};
  g.g = Rows{d->M, d->K, d->Kp};
  g.Kred = d->B;
  g.Nout = d->H;
  g.norm = d->norm_type;
  return g;
}

TbLayout tb_layout(const ctn_tblock_desc* d, int backward, void* ws) {
  TbLayout L{};
  Carver c(ws);
  const Rows rg{d->M, d->K, d->Kp};
  const long rows = rg.rows();
  const size_t es = esize(d->dtype);
  const int G = tb_groups(d);
  GemmRows g1 = tb_gemm1(d);
  L.parts1 = gemm_rows_tiles_per_group(g1);
  DwArgs da{};
  da.g = rg; da.H = d->H; da.P = d->P; da.norm = d->norm_type;
  L.parts2 = dw_parts_per_group(da);
  if (!backward) {
    if (d->dtype == CTN_DTYPE_BF16) {
      L.w1s = c.take<void>((size_t)d->H * d->B * es);
      L.w2s = c.take<void>((size_t)d->H * d->B * es);
    }
    L.slab1 = c.take<double2>((size_t)G * L.parts1 * sizeof(double2));
    L.slab2 = c.take<double2>((size_t)G * L.parts2 * sizeof(double2));
  } else {
    L.w1t = c.take<void>((size_t)d->H * d->B * es);
    L.w2t = c.take<void>((size_t)d->H * d->B * es);
    L.G1 = c.take<void>((size_t)rows * d->H * es);
    L.G2 = c.take<void>((size_t)rows * d->H * es);
    GemmRows ga = tb_gemm1(d);   // same geometry as gemm1 (Nout = H)
    L.partsA = gemm_rows_tiles_per_group(ga);
    L.rowtiles = gemm_rows_rowtiles(ga);
    L.slabA = c.take<double2>((size_t)G * L.partsA * sizeof(double2));
    L.colA = c.take<float>((size_t)L.rowtiles * 2 * d->H * sizeof(float));
    L.partsD = L.parts2;
    L.slabD = c.take<double2>((size_t)G * L.partsD * sizeof(double2));
    L.colD = c.take<float>((size_t)dw_blocks(da) * dw_col_stride(da) * sizeof(float));
    L.alphaSlab = c.take<float>((size_t)dw_blocks(da) * sizeof(float));
    L.sums1 = c.take<float2>((size_t)G * sizeof(float2));
    L.sums2 = c.take<float2>((size_t)G * sizeof(float2));
    GemmCols gc{};
    gc.g = rg; gc.P = d->B; gc.Q = d->H;
    L.chunks2 = gemm_cols_default_chunks(gc);
    L.cpart2 = c.take<float>((size_t)L.chunks2 * d->B * d->H * sizeof(float));
    gc.P = d->H; gc.Q = d->B;
    L.chunks1 = gemm_cols_default_chunks(gc);
    L.cpart1 = c.take<float>((size_t)L.chunks1 * d->B * d->H * sizeof(float));
  }
  L.bytes = c.off + 256;
  return L;
}

int tb_pad(const ctn_tblock_desc* d) {
  return d->causal ? (d->P - 1) * d->dilation : (d->P - 1) * d->dilation / 2;
}
}  // namespace

extern "C" size_t ctn_tblock_workspace_bytes(const ctn_tblock_desc* d, int backward) {
  if (tb_check(d) != CTN_OK) return 0;
  return tb_layout(d, backward, nullptr).bytes;
}

extern "C" int ctn_tblock_forward(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x, void* y,
                                  const ctn_tblock_saved* sv, void* ws, size_t ws_bytes, void* stream) {
  int rc = tb_check(d);
  if (rc) return rc;
  if (!p || !x || !y || !sv || !sv->h1 || !sv->d || !sv->stats) return fail(CTN_ERR_ARG, "null pointer");
  const TbLayout L = tb_layout(d, 0, ws);
  if (!ws || ws_bytes < L.bytes) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, L.bytes);
  hipStream_t s = (hipStream_t)stream;
  const DType dt = d->dtype == CTN_DTYPE_BF16 ? BF16 : F32;
  const Rows rg{d->M, d->K, d->Kp};
  const int G = tb_groups(d);
  float2* st1 = reinterpret_cast<float2*>(sv->stats);
  float2* st2 = st1 + G;
  const double cnt = d->norm_type == CTN_NORM_GLN ? (double)d->K * d->H : (double)d->H;

  const void* w1 = p->w1;
  const void* w2 = p->w2;
  if (dt == BF16) {
    CTN_HIP(launch_prep_weight(dt, p->w1, d->H, d->B, L.w1s, nullptr, s));
    CTN_HIP(launch_prep_weight(dt, p->w2, d->B, d->H, L.w2s, nullptr, s));
    w1 = L.w1s;
    w2 = L.w2s;
  }
  // 1x1 conv B->H, PReLU statistics for norm1
  GemmRows g1 = tb_gemm1(d);
  g1.A = x; g1.lda = d->B;
  g1.W = w1; g1.ldw = d->B;
  g1.epi = EPI_PRELU_STATS;
  g1.alpha = p->alpha1;
  g1.C = sv->h1; g1.ldc = d->H;
  g1.grp_slab = L.slab1;
  {
    TimedScope ts(1, s);
    CTN_HIP(launch_gemm_rows(dt, g1, s));
  }
  CTN_HIP(launch_stats_finalize(L.slab1, G, L.parts1, cnt, 0, (float)kEps, st1, s));
  // norm1 apply + depthwise dilated conv, PReLU statistics for norm2
  DwArgs da{};
  da.g = rg; da.H = d->H; da.P = d->P; da.dil = d->dilation; da.pad = tb_pad(d); da.norm = d->norm_type;
  da.h1 = sv->h1; da.st1 = st1;
  da.alpha1 = p->alpha1; da.gamma1 = p->gamma1; da.beta1 = p->beta1; da.alpha2 = p->alpha2;
  da.wd = p->wd; da.d_out = sv->d; da.slab2 = L.slab2;
  {
    TimedScope ts(2, s);
    CTN_HIP(launch_dw_fwd(dt, da, s));
  }
  CTN_HIP(launch_stats_finalize(L.slab2, G, L.parts2, cnt, 0, (float)kEps, st2, s));
  // norm2 apply (+PReLU) on the operand, 1x1 conv H->B, residual add
  GemmRows g2{};
  g2.g = rg; g2.Kred = d->H; g2.Nout = d->B; g2.norm = d->norm_type;
  g2.A = sv->d; g2.lda = d->H;
  g2.aop.kind = OP_PRELU_NORM; g2.aop.norm = d->norm_type; g2.aop.stats = st2;
  g2.aop.gamma = p->gamma2; g2.aop.beta = p->beta2; g2.aop.alpha = p->alpha2;
  g2.W = w2; g2.ldw = d->H;
  g2.epi = EPI_RESID; g2.R = x; g2.ldr = d->B;
  g2.C = y; g2.ldc = d->B;
  CTN_HIP(launch_gemm_rows(dt, g2, s));
  return CTN_OK;
}

extern "C" int ctn_tblock_backward(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x,
                                   const ctn_tblock_saved* sv, const void* gy, void* gx, const ctn_tblock_grads* gr,
                                   void* ws, size_t ws_bytes, void* stream) {
  int rc = tb_check(d);
  if (rc) return rc;
  if (!p || !x || !sv || !gy || !gx || !gr) return fail(CTN_ERR_ARG, "null pointer");
  const TbLayout L = tb_layout(d, 1, ws);
  if (!ws || ws_bytes < L.bytes) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, L.bytes);
  hipStream_t s = (hipStream_t)stream;
  const DType dt = d->dtype == CTN_DTYPE_BF16 ? BF16 : F32;
  const Rows rg{d->M, d->K, d->Kp};
  const int G = tb_groups(d);
  const float2* st1 = reinterpret_cast<const float2*>(sv->stats);
  const float2* st2 = st1 + G;
  const double cnt = d->norm_type == CTN_NORM_GLN ? (double)d->K * d->H : (double)d->H;

  CTN_HIP(launch_prep_weight(dt, p->w2, d->B, d->H, nullptr, L.w2t, s));   // [H][B]
  CTN_HIP(launch_prep_weight(dt, p->w1, d->H, d->B, nullptr, L.w1t, s));   // [B][H]

  // (a) g_n2 = gy . W2 ; epilogue: norm2 backward element part -> G1 = g_n2*gamma2, sums, gamma2/beta2 partials
  GemmRows ga = tb_gemm1(d);
  ga.A = gy; ga.lda = d->B;
  ga.W = L.w2t; ga.ldw = d->B;
  ga.epi = EPI_NORM_BWD; ga.R = sv->d; ga.ldr = d->H;
  ga.alpha = p->alpha2; ga.stats = st2; ga.gamma = p->gamma2;
  ga.C = L.G1; ga.ldc = d->H;
  ga.grp_slab = L.slabA; ga.col_slab = L.colA;
  {
    TimedScope ts(3, s);
    CTN_HIP(launch_gemm_rows(dt, ga, s));
  }
  CTN_HIP(launch_stats_finalize(L.slabA, G, L.partsA, cnt, 1, 0.f, L.sums2, s));
  // (b) dW2 = gy^T . norm2(PReLU(d))
  GemmCols c2{};
  c2.g = rg; c2.P = d->B; c2.Q = d->H;
  c2.A = gy; c2.lda = d->B;
  c2.B = sv->d; c2.ldb = d->H;
  c2.bop.kind = OP_PRELU_NORM; c2.bop.norm = d->norm_type; c2.bop.stats = st2;
  c2.bop.gamma = p->gamma2; c2.bop.beta = p->beta2; c2.bop.alpha = p->alpha2;
  c2.Cpart = L.cpart2; c2.nchunks = L.chunks2;
  CTN_HIP(launch_gemm_cols(dt, c2, s));
  // (c) depthwise backward -> G2 = dL/d(hat a1), norm1 sums, column partials
  DwArgs da{};
  da.g = rg; da.H = d->H; da.P = d->P; da.dil = d->dilation; da.pad = tb_pad(d); da.norm = d->norm_type;
  da.h1 = sv->h1; da.d = sv->d; da.st1 = st1; da.st2 = st2;
  da.alpha1 = p->alpha1; da.gamma1 = p->gamma1; da.beta1 = p->beta1; da.alpha2 = p->alpha2; da.gamma2 = p->gamma2;
  da.wd = p->wd;
  da.ga2 = L.G1; da.sm2 = L.sums2; da.ga1_out = L.G2; da.slab1 = L.slabD; da.col_slab = L.colD;
  CTN_HIP(launch_dw_bwd(dt, da, s));
  CTN_HIP(launch_stats_finalize(L.slabD, G, L.partsD, cnt, 1, 0.f, L.sums1, s));
  // (d) norm1 backward finish + PReLU1 backward -> G1 = dL/dh1
  DwArgs de = da;
  de.ga2 = L.G2; de.sm1 = L.sums1; de.gh1_out = L.G1; de.alpha_slab = L.alphaSlab;
  CTN_HIP(launch_norm1_bwd(dt, de, s));
  // (e) gx = gh1 . W1 + gy
  GemmRows gb{};
  gb.g = rg; gb.Kred = d->H; gb.Nout = d->B; gb.norm = d->norm_type;
  gb.A = L.G1; gb.lda = d->H;
  gb.W = L.w1t; gb.ldw = d->H;
  gb.epi = EPI_RESID; gb.R = gy; gb.ldr = d->B;
  gb.C = gx; gb.ldc = d->B;
  CTN_HIP(launch_gemm_rows(dt, gb, s));
  // (f) dW1 = gh1^T . x
  GemmCols c1{};
  c1.g = rg; c1.P = d->H; c1.Q = d->B;
  c1.A = L.G1; c1.lda = d->H;
  c1.B = x; c1.ldb = d->B;
  c1.Cpart = L.cpart1; c1.nchunks = L.chunks1;
  CTN_HIP(launch_gemm_cols(dt, c1, s));
  // (g) all parameter-gradient partial sums
  const int dwb = dw_blocks(da), dws = dw_col_stride(da);
  const int HB = d->H * d->B, H = d->H;
  SlabBatch sb{};
  sb.d[0] = SlabDesc{L.cpart2, gr->w2, L.chunks2, HB, HB};
  sb.d[1] = SlabDesc{L.cpart1, gr->w1, L.chunks1, HB, HB};
  sb.d[2] = SlabDesc{L.colA, gr->gamma2, L.rowtiles, H, 2 * H};
  sb.d[3] = SlabDesc{L.colA + H, gr->beta2, L.rowtiles, H, 2 * H};
  sb.d[4] = SlabDesc{L.colD, gr->gamma1, dwb, H, dws};
  sb.d[5] = SlabDesc{L.colD + H, gr->beta1, dwb, H, dws};
  sb.d[6] = SlabDesc{L.colD + 2 * H, gr->wd, dwb, H * d->P, dws};
  sb.d[7] = SlabDesc{L.colD + (2 + d->P) * H, gr->alpha2, dwb, 1, dws};
  sb.d[8] = SlabDesc{L.alphaSlab, gr->alpha1, dwb, 1, 1};
  sb.nd = 9;
  CTN_HIP(launch_slab_reduce(sb, s));
  return CTN_OK;
}
