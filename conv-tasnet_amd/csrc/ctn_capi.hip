#include <stdlib.h>
// extern "C" entry points of libctn_hip.so (include/ctn.h) and the native
// launch sequences behind them.  Each entry validates its descriptor, carves
// the caller's workspace, and enqueues its kernels on the caller's stream.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <string>
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
// kernel timer (bench.py roofline measurement): a set of kernel kinds (CTN_TIMER_*), each
// launch of a selected kind bracketed by a pair of hipEvents on the launch's stream
// ---------------------------------------------------------------------------
namespace {
struct Timer {
  std::mutex mu;
  uint32_t mask = 0;
  int cap = 0;                              // launches per kind
  int stride = 1;                           // bracket every stride-th launch of a kind
  int used[32] = {};
  long seen[32] = {};                       // launches of a kind since enable
  std::vector<hipEvent_t> ev[32];           // pairs
};
Timer g_timer;

struct TimedScope {
  hipStream_t s;
  int kind = 0, idx = -1;
  TimedScope(int k, hipStream_t st) : s(st), kind(k) {
    if (k <= 0 || k >= 32 || !((g_timer.mask >> k) & 1u)) return;
    std::lock_guard<std::mutex> lk(g_timer.mu);
    if (g_timer.seen[k]++ % g_timer.stride != 0 || g_timer.used[k] >= g_timer.cap) return;
    idx = g_timer.used[k]++;
    (void)hipEventRecord(g_timer.ev[k][2 * idx], s);
  }
  ~TimedScope() {
    if (idx >= 0) (void)hipEventRecord(g_timer.ev[kind][2 * idx + 1], s);
  }
};
}  // namespace

extern "C" int ctn_timer_enable_mask(uint32_t mask, int max_launches) {
  if (max_launches < 0 || (mask & 1u)) return fail(CTN_ERR_ARG, "timer mask 0x%x / launches %d", mask, max_launches);
  std::lock_guard<std::mutex> lk(g_timer.mu);
  for (int k = 0; k < 32; ++k) {
    for (auto e : g_timer.ev[k]) (void)hipEventDestroy(e);
    g_timer.ev[k].clear();
    g_timer.used[k] = 0;
    g_timer.seen[k] = 0;
  }
  g_timer.mask = max_launches ? mask : 0u;
  g_timer.cap = max_launches;
  for (int k = 1; k < 32; ++k) {
    if (!((g_timer.mask >> k) & 1u)) continue;
    g_timer.ev[k].resize(2 * (size_t)g_timer.cap);
    for (auto& e : g_timer.ev[k]) CTN_HIP(hipEventCreate(&e));
  }
  return CTN_OK;
}

extern "C" int ctn_timer_set_stride(int stride) {
  if (stride < 1) return fail(CTN_ERR_ARG, "timer stride %d", stride);
  std::lock_guard<std::mutex> lk(g_timer.mu);
  g_timer.stride = stride;
  return CTN_OK;
}

extern "C" int ctn_copy_bytes(void* dst, const void* src, size_t bytes, int workgroups, int flags, void* stream) {
  if (!dst || !src || bytes % 16 || ((uintptr_t)dst | (uintptr_t)src) % 16 || workgroups < 1 ||
      workgroups > 65536 || (flags & ~3))
    return fail(CTN_ERR_ARG, "copy: %zu bytes, %d workgroups, flags %d (16-byte multiples and alignment, 1..65536, "
                "flags 0..3)", bytes, workgroups, flags);
  CTN_HIP(ctn::launch_copy_stream(dst, src, bytes, workgroups, flags, (hipStream_t)stream));
  return CTN_OK;
}

extern "C" int ctn_mfma_peak(int shape, int workgroups, int iters, float* out, double* flops, void* stream) {
  if (!out || workgroups < 1 || workgroups > 65536 || iters < 1 || (shape != 0 && shape != 1))
    return fail(CTN_ERR_ARG, "mfma_peak: shape %d, %d workgroups, %d iterations (shape 0|1, 1..65536, >= 1)", shape,
                workgroups, iters);
  CTN_HIP(ctn::launch_mfma_peak(shape, workgroups, iters, out, flops, (hipStream_t)stream));
  return CTN_OK;
}

extern "C" int ctn_timer_enable(int kind, int max_launches) {
  if (kind < 0 || kind >= 32) return fail(CTN_ERR_ARG, "timer kind %d", kind);
  return ctn_timer_enable_mask(kind ? 1u << kind : 0u, kind ? max_launches : 0);
}

extern "C" int ctn_timer_read_kind(int kind, double* total_ms, int* launches) {
  if (kind <= 0 || kind >= 32) return fail(CTN_ERR_ARG, "timer kind %d", kind);
  std::lock_guard<std::mutex> lk(g_timer.mu);
  double t = 0.0;
  for (int i = 0; i < g_timer.used[kind]; ++i) {
    CTN_HIP(hipEventSynchronize(g_timer.ev[kind][2 * i + 1]));
    float ms = 0.f;
    CTN_HIP(hipEventElapsedTime(&ms, g_timer.ev[kind][2 * i], g_timer.ev[kind][2 * i + 1]));
    t += ms;
  }
  if (total_ms) *total_ms = t;
  if (launches) *launches = g_timer.used[kind];
  return CTN_OK;
}

extern "C" int ctn_timer_read(double* total_ms, int* launches) {
  double t = 0.0;
  int n = 0;
  for (int k = 1; k < 32; ++k) {
    double tk = 0.0;
    int nk = 0;
    const int rc = ctn_timer_read_kind(k, &tk, &nk);
    if (rc) return rc;
    t += tk;
    n += nk;
  }
  if (total_ms) *total_ms = t;
  if (launches) *launches = n;
  return CTN_OK;
}

// ---------------------------------------------------------------------------
// device error word (ctn_common.h CTN_DEVERR_*): one per device, a zero-initialised
// __device__ variable of this code object (each device loads its own copy), so getting it
// needs no allocation and no memset: safe on the first launch even inside a stream or
// graph capture.  The pointer is cached per device in an atomic, so launches take no lock.
// A pinned host mirror is refreshed asynchronously at the end of every backward pass
// (ctn_tblock_reduce_grads) and checked at the next one, so a kernel that hit an error
// fails the call within a step without a device synchronisation on the fast path.
// ---------------------------------------------------------------------------
__device__ uint32_t ctn_err_words[64];   // [0] is the word; the rest pads it to its own line

namespace {
constexpr int MAX_DEV = 64;
struct DevErr {
  std::mutex mu;
  std::atomic<uint32_t*> word[MAX_DEV] = {};
  std::atomic<uint32_t*> mirror[MAX_DEV] = {};
};
DevErr g_deverr;

uint32_t* dev_err_word(int* dev) {
  if (hipGetDevice(dev) != hipSuccess || *dev < 0 || *dev >= MAX_DEV) return nullptr;
  uint32_t* w = g_deverr.word[*dev].load(std::memory_order_acquire);
  if (w) return w;
  void* a = nullptr;
  if (hipGetSymbolAddress(&a, HIP_SYMBOL(ctn_err_words)) != hipSuccess) return nullptr;
  g_deverr.word[*dev].store((uint32_t*)a, std::memory_order_release);
  return (uint32_t*)a;
}

// the pinned host mirror of a device's word (allocated on the first refresh or status
// call, never on a kernel launch)
volatile uint32_t* dev_err_mirror(int dev) {
  uint32_t* h = g_deverr.mirror[dev].load(std::memory_order_acquire);
  if (h) return h;
  std::lock_guard<std::mutex> lk(g_deverr.mu);
  h = g_deverr.mirror[dev].load(std::memory_order_relaxed);
  if (!h) {
    void* p = nullptr;
    if (hipHostMalloc(&p, 256, hipHostMallocDefault) != hipSuccess) return nullptr;
    *(volatile uint32_t*)p = 0u;
    h = (uint32_t*)p;
    g_deverr.mirror[dev].store(h, std::memory_order_release);
  }
  return h;
}

const char* dev_err_text(uint32_t w) {
  if (w & CTN_DEVERR_SPIN)
    return "a generation-word wait of a wave-specialised kernel ran out of polls (CTN_DEVERR_SPIN): that launch's "
           "outputs are invalid";
  return "unknown device error bit";
}

// the mirror of earlier copies (no synchronisation): non-zero once an error has been seen
int dev_err_check_async() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV) return CTN_OK;
  const uint32_t* h = g_deverr.mirror[dev].load(std::memory_order_acquire);
  if (!h) return CTN_OK;
  const uint32_t w = *(const volatile uint32_t*)h;
  if (w) return fail(CTN_ERR_HIP, "device error word 0x%x: %s", w, dev_err_text(w));
  return CTN_OK;
}

hipError_t dev_err_refresh(hipStream_t s) {
  int dev = 0;
  uint32_t* w = dev_err_word(&dev);
  volatile uint32_t* h = w ? dev_err_mirror(dev) : nullptr;
  if (!h) return hipErrorOutOfMemory;
  return hipMemcpyAsync((void*)h, w, 4, hipMemcpyDeviceToHost, s);
}
}  // namespace

uint32_t* ctn::device_error_word() {
  int dev = 0;
  return dev_err_word(&dev);
}

extern "C" int ctn_device_status(void* stream, uint32_t* word, int clear) {
  int dev = 0;
  uint32_t* dw = dev_err_word(&dev);
  volatile uint32_t* mirror = dw ? dev_err_mirror(dev) : nullptr;
  if (!mirror) return fail(CTN_ERR_HIP, "device error word: unavailable");
  hipStream_t s = (hipStream_t)stream;
  uint32_t w = 0;
  CTN_HIP(hipStreamSynchronize(s));
  CTN_HIP(hipMemcpy(&w, dw, 4, hipMemcpyDeviceToHost));
  if (clear && w) {
    CTN_HIP(hipMemset(dw, 0, 4));
    *mirror = 0u;
  }
  if (word) *word = w;
  if (w) return fail(CTN_ERR_HIP, "device error word 0x%x: %s", w, dev_err_text(w));
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
// scratch floats of the two-level slab reduction for one (nparts, n) descriptor
size_t sr_tmp(long nparts, long n) {
  const long ns = (nparts + 63) / 64;
  return ns > 1 ? (size_t)(ns * n) : 0;
}
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
  if (d->P < 1 || d->P > 8) return fail(CTN_ERR_UNSUPPORTED, "P=%d outside 1..8", d->P);
  if (!d->causal && d->P % 2 == 0)
    return fail(CTN_ERR_ARG, "non-causal padding (P-1)*d//2 needs odd P (conv_tasnet.py:236)");
  if (d->norm_type != CTN_NORM_GLN && d->norm_type != CTN_NORM_CLN && d->norm_type != CTN_NORM_BN)
    return fail(CTN_ERR_ARG, "norm_type %d", d->norm_type);
  {
    const int cg = d->H / 8;
    if (cg > 64 || (cg & (cg - 1))) return fail(CTN_ERR_UNSUPPORTED, "H=%d: need H/8 a power of two <= 64", d->H);
  }
  if (d->dtype != CTN_DTYPE_F32 && d->dtype != CTN_DTYPE_BF16) return fail(CTN_ERR_ARG, "dtype %d", d->dtype);
  if (d->dilation < 1) return fail(CTN_ERR_ARG, "dilation %d", d->dilation);
  return CTN_OK;
}

static int tb_groups(const ctn_tblock_desc* d) {
  if (d->norm_type == CTN_NORM_BN) return d->H;   // per-channel statistics
  return d->norm_type == CTN_NORM_GLN ? d->M : d->M * d->Kp;
}

extern "C" int ctn_tblock_stats_floats(const ctn_tblock_desc* d) { return 4 * tb_groups(d); }

namespace {
struct TbLayout {
  // forward
  void *w1s, *w2s;
  double2 *slab1, *slab2;
  // backward
  void *w1t, *w2t, *G1, *G2;
  double2 *slabA, *slabD;
  float *colD, *alphaSlab, *cpart1, *cpart2, *srtmp;
  float2 *sums1, *sums2;
  int parts1, parts2, partsA, partsD, chunks1, chunks2;
  size_t bytes;
  size_t part_bytes;   // split_parts: the parameter-gradient partials' own buffer
};

int tb_pad(const ctn_tblock_desc* d) {
  return d->causal ? (d->P - 1) * d->dilation : (d->P - 1) * d->dilation / 2;
}

// The two H-output GEMMs of a block, with everything but the data pointers
// filled in: the slab sizing in tb_layout queries exactly what is launched.
GemmRows tb_gemm1(const ctn_tblock_desc* d) {   // forward x[.,B] -> h1[.,H], PReLU statistics
  GemmRows g{};
  g.g = Rows{d->M, d->K, d->Kp};
  g.Kred = d->B;
  g.Nout = d->H;
  g.norm = d->norm_type;
  g.lda = d->B; g.ldw = d->B; g.ldc = d->H;
  g.epi = EPI_PRELU_STATS;
  return g;
}
GemmRows tb_gemmA(const ctn_tblock_desc* d) {   // backward g_n2 = gy . W2, norm-2 backward epilogue
  GemmRows g = tb_gemm1(d);
  g.epi = EPI_NORM_BWD;
  g.ldr = d->H;
  return g;
}

// The backward's two dual GEMMs (ctn_gemm_dual.hip), shapes and operand ops only:
//   A: g_n2 = gy . W2 (norm-2 backward epilogue) + dW2 = gy^T . norm2(PReLU(d))
//   B: gx = gh1 . W1 + gy                        + dW1 = gh1^T . x
GemmDual tb_dualA(const ctn_tblock_desc* d) {
  GemmDual g{};
  g.g = Rows{d->M, d->K, d->Kp};
  g.Kred = d->B; g.Nout = d->H; g.norm = d->norm_type;
  g.lda = d->B; g.ldw = d->B; g.ldc = d->H; g.ldr = d->H; g.ldb = d->H;
  g.epi = EPI_NORM_BWD;
  g.bop.kind = OP_PRELU_NORM; g.bop.norm = d->norm_type;
  return g;
}
GemmDual tb_dualB(const ctn_tblock_desc* d) {
  GemmDual g{};
  g.g = Rows{d->M, d->K, d->Kp};
  g.Kred = d->H; g.Nout = d->B; g.norm = d->norm_type;
  g.lda = d->H; g.ldw = d->H; g.ldc = d->B; g.ldr = d->B; g.ldb = d->B;
  g.epi = EPI_RESID;
  return g;
}
// backward gx = op(g) . W1 + gy; op = norm-1/PReLU-1 backward (fused path) or plain
GemmRows tb_gemmB(const ctn_tblock_desc* d, bool fused) {
  GemmRows g{};
  g.g = Rows{d->M, d->K, d->Kp};
  g.Kred = d->H; g.Nout = d->B; g.norm = d->norm_type;
  g.lda = d->H; g.ldw = d->H; g.epi = EPI_RESID; g.ldr = d->B; g.ldc = d->B;
  if (fused) {
    g.aop.kind = OP_NORM1_BWD; g.aop.norm = d->norm_type;
  }
  return g;
}
// The norm-1/PReLU-1 backward runs inside the first 1x1's two gradient GEMMs (bf16,
// gLN or cLN, weight-stationary data-gradient kernel, dual pair B off); else
// norm1_bwd_kernel.
// CTN_FUSE_N1=0 keeps the separate kernel (read on every query, so a process can
// compare both paths: tests/test_gpu_tblock.py).
// gLN statistics of the weight-stationary GEMMs' operands: folded from the producer's
// partials in every workgroup's prologue (default) or finalized by a separate launch
// before them (A/B; read on every call).  bit 0: the output 1x1 GEMM (norm 2 from dw_fwd),
// bit 1: the gx GEMM (norm-1 backward sums from dw_bwd).
static int ws_fold_mask() {
  const char* e = getenv("CTN_WS_FOLD");
  return e ? atoi(e) : 3;
}

bool tb_fused_n1(const ctn_tblock_desc* d) {
  const char* e = getenv("CTN_FUSE_N1");
  if (e && atoi(e) == 0) return false;
  if (d->dtype != CTN_DTYPE_BF16 || (d->norm_type != CTN_NORM_GLN && d->norm_type != CTN_NORM_CLN)) return false;
  if (gemm_dual_eligible(BF16, tb_dualB(d))) return false;
  GemmRows g = tb_gemmB(d, true);
  static const float dummy[2] = {0.f, 0.f};   // eligibility only checks presence
  g.aop.aux = dummy; g.aop.apart = const_cast<float*>(dummy); g.aop.aout = const_cast<float*>(dummy);
  g.aop.stats = reinterpret_cast<const float2*>(dummy); g.aop.sums = reinterpret_cast<const float2*>(dummy);
  return gemm_ws_eligible(BF16, g);
}
DType tb_dt(const ctn_tblock_desc* d) { return d->dtype == CTN_DTYPE_BF16 ? BF16 : F32; }

// backward, split_parts: the parameter-gradient partials (colD, alphaSlab, cpart1/2) and
// their reduction scratch (srtmp) come from `part` (part_bytes), everything else from ws
// (bytes) — the deferred backward (ctn_tblock_backward_deferred) keeps only `part` alive
// until ctn_tblock_reduce_grads.
TbLayout tb_layout(const ctn_tblock_desc* d, int backward, void* ws, void* part = nullptr, bool split_parts = false) {
  TbLayout L{};
  Carver c(ws), cpt(part);
  Carver& cp = split_parts ? cpt : c;
  const Rows rg{d->M, d->K, d->Kp};
  const long rows = rg.rows();
  const size_t es = esize(d->dtype);
  const int G = tb_groups(d);
  GemmRows g1 = tb_gemm1(d);
  const DType dtl = d->dtype == CTN_DTYPE_BF16 ? BF16 : F32;
  L.parts1 = gemm_rows_tiles_per_group(dtl, g1);
  DwArgs da{};
  da.g = rg; da.H = d->H; da.P = d->P; da.norm = d->norm_type; da.dil = d->dilation; da.pad = tb_pad(d);
  da.seg = dw_seg(da, false);
  L.parts2 = dw_parts_per_group(da);   // forward comb geometry (norm-2 statistics)
  da.seg = dw_seg(da, true);            // backward comb geometry from here on
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
    GemmRows ga = tb_gemmA(d);
    const GemmDual duA = tb_dualA(d), duB = tb_dualB(d);
    const bool dualA = gemm_dual_eligible(dtl, duA), dualB = gemm_dual_eligible(dtl, duB);
    L.partsA = dualA ? gemm_dual_group_parts(duA) : gemm_rows_tiles_per_group(dtl, ga);
    L.slabA = c.take<double2>((size_t)G * L.partsA * sizeof(double2));
    L.partsD = dw_parts_per_group(da);
    L.slabD = c.take<double2>((size_t)G * L.partsD * sizeof(double2));
    L.colD = cp.take<float>((size_t)dw_blocks(da) * dw_col_stride(da) * sizeof(float));
    const int na = tb_fused_n1(d) ? gemm_ws_grid(tb_gemmB(d, true)) : ew_blocks(da);
    L.alphaSlab = cp.take<float>((size_t)(na > ew_blocks(da) ? na : ew_blocks(da)) * sizeof(float));
    L.sums1 = c.take<float2>((size_t)G * sizeof(float2));
    L.sums2 = c.take<float2>((size_t)G * sizeof(float2));
    GemmCols gc{};
    gc.g = rg; gc.P = d->B; gc.Q = d->H;
    L.chunks2 = dualA ? gemm_dual_ranges(duA) : gemm_cols_default_chunks(gc);
    L.cpart2 = cp.take<float>((size_t)L.chunks2 * d->B * d->H * sizeof(float));
    gc.P = d->H; gc.Q = d->B;
    L.chunks1 = dualB ? gemm_dual_ranges(duB) : gemm_cols_chunks(dtl, gc);
    L.cpart1 = cp.take<float>((size_t)L.chunks1 * d->B * d->H * sizeof(float));
    const long HB = (long)d->H * d->B, dwb = dw_blocks(da);
    const size_t ntmp = sr_tmp(L.chunks2, HB) + sr_tmp(L.chunks1, HB) + 4 * sr_tmp(dwb, d->H) +
                        sr_tmp(dwb, (long)d->H * d->P) + sr_tmp(dwb, 1) +
                        sr_tmp(ew_blocks(da), 1);
    L.srtmp = cp.take<float>(ntmp * sizeof(float));
  }
  L.bytes = c.off + 256;
  L.part_bytes = split_parts ? cpt.off + 256 : 0;
  return L;
}

}  // namespace

// ===========================================================================
// TemporalBlock with BatchNorm1d norms (norm_type "BN", conv_tasnet.py:302-303)
// ===========================================================================
// The block's kernels run in identity gLN mode (per-utterance stats (0, 1),
// gamma' = gamma*rstd, beta' = beta - gamma*mean*rstd per channel, ctn_bn.hip);
// BN's per-channel statistics and the per-channel mean subtractions of its
// backward run in the column kernels of ctn_bn.hip.
namespace {
struct BnLayout {
  void *w1s, *w2s, *w1t, *w2t, *G1, *G2;
  double2 *part, *slab2, *slabD;
  float2 *ident, *zero, *sums1, *sums2;
  float *ge1, *be1, *ge2, *be2, *colD, *alphaSlab, *cpart1, *cpart2, *srtmp;
  int chunks1, chunks2;
  size_t bytes;
};
DwArgs bn_dw(const ctn_tblock_desc* d, bool bwd) {
  DwArgs da{};
  da.g = Rows{d->M, d->K, d->Kp};
  da.H = d->H; da.P = d->P; da.dil = d->dilation; da.pad = tb_pad(d); da.norm = NORM_GLN;
  da.seg = dw_seg(da, bwd);
  return da;
}
BnLayout bn_layout(const ctn_tblock_desc* d, int backward, void* ws) {
  BnLayout L{};
  Carver c(ws);
  const Rows rg{d->M, d->K, d->Kp};
  const long rows = rg.rows();
  const size_t es = esize(d->dtype);
  const int H = d->H, B = d->B, M = d->M, nb = bn_blocks(rg);
  L.part = c.take<double2>((size_t)nb * H * sizeof(double2));
  L.ident = c.take<float2>((size_t)M * sizeof(float2));
  L.zero = c.take<float2>((size_t)M * sizeof(float2));
  L.ge1 = c.take<float>((size_t)H * sizeof(float));
  L.be1 = c.take<float>((size_t)H * sizeof(float));
  L.ge2 = c.take<float>((size_t)H * sizeof(float));
  L.be2 = c.take<float>((size_t)H * sizeof(float));
  if (!backward) {
    if (d->dtype == CTN_DTYPE_BF16) {
      L.w1s = c.take<void>((size_t)H * B * es);
      L.w2s = c.take<void>((size_t)H * B * es);
    }
    const DwArgs da = bn_dw(d, false);
    L.slab2 = c.take<double2>((size_t)M * dw_parts_per_group(da) * sizeof(double2));
  } else {
    L.w1t = c.take<void>((size_t)H * B * es);
    L.w2t = c.take<void>((size_t)H * B * es);
    L.G1 = c.take<void>((size_t)rows * H * es);
    L.G2 = c.take<void>((size_t)rows * H * es);
    L.sums1 = c.take<float2>((size_t)H * sizeof(float2));
    L.sums2 = c.take<float2>((size_t)H * sizeof(float2));
    const DwArgs da = bn_dw(d, true);
    L.slabD = c.take<double2>((size_t)M * dw_parts_per_group(da) * sizeof(double2));
    L.colD = c.take<float>((size_t)dw_blocks(da) * dw_col_stride(da) * sizeof(float));
    L.alphaSlab = c.take<float>((size_t)nb * sizeof(float));
    GemmCols gc{};
    gc.g = rg; gc.P = B; gc.Q = H;
    L.chunks2 = gemm_cols_default_chunks(gc);
    L.cpart2 = c.take<float>((size_t)L.chunks2 * B * H * sizeof(float));
    gc.P = H; gc.Q = B;
    L.chunks1 = gemm_cols_default_chunks(gc);
    L.cpart1 = c.take<float>((size_t)L.chunks1 * B * H * sizeof(float));
    const long HB = (long)H * B, dwb = dw_blocks(da);
    const size_t ntmp = sr_tmp(L.chunks2, HB) + sr_tmp(L.chunks1, HB) + 2 * sr_tmp(dwb, H) +
                        sr_tmp(dwb, (long)H * d->P) + sr_tmp(dwb, 1) + sr_tmp(nb, 1);
    L.srtmp = c.take<float>(ntmp * sizeof(float));
  }
  L.bytes = c.off + 256;
  return L;
}

// forward statistics of PReLU(a) -> stats, gamma', beta', running statistics
int bn_forward_stats(DType dt, const ctn_tblock_desc* d, const BnLayout& L, const void* a, const float* alpha,
                     const float* gamma, const float* beta, float* rmean, float* rvar, int training, float mom,
                     float eps, float2* stats, float* ge, float* be, hipStream_t s) {
  const Rows rg{d->M, d->K, d->Kp};
  const bool batch = training || !rmean;
  if (!batch && !rvar) return fail(CTN_ERR_ARG, "BN eval mode needs running_var");
  if (batch) {
    BnArgs ba{};
    ba.g = rg; ba.H = d->H; ba.a = a; ba.alpha = alpha; ba.part = L.part;
    CTN_HIP(launch_bn_partials(dt, ba, 0, s));
  }
  BnFinal bf{};
  bf.H = d->H; bf.M = d->M; bf.nparts = bn_blocks(rg); bf.count = (long)d->M * d->K; bf.part = L.part;
  bf.training = batch; bf.momentum = mom; bf.eps = eps;
  bf.run_mean = training ? rmean : (batch ? nullptr : rmean);
  bf.run_var = training ? rvar : (batch ? nullptr : rvar);
  bf.gamma = gamma; bf.beta = beta; bf.stats = stats; bf.gamma_eff = ge; bf.beta_eff = be;
  bf.ident = L.ident; bf.zero = L.zero;
  CTN_HIP(launch_bn_finalize(bf, 0, s));
  return CTN_OK;
}
}  // namespace

static int tb_forward_bn(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x, void* y,
                         const ctn_tblock_saved* sv, void* ws, size_t ws_bytes, hipStream_t s) {
  const BnLayout L = bn_layout(d, 0, ws);
  if (!ws || ws_bytes < L.bytes) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, L.bytes);
  const DType dt = tb_dt(d);
  const Rows rg{d->M, d->K, d->Kp};
  float2* st1 = reinterpret_cast<float2*>(sv->stats);
  float2* st2 = st1 + d->H;
  const void* w1 = p->w1;
  const void* w2 = p->w2;
  if (dt == BF16 && p->w1_bf16 && p->w2_bf16) {
    w1 = p->w1_bf16;
    w2 = p->w2_bf16;
  } else if (dt == BF16) {
    PrepBatch pb{};
    pb.d[0] = PrepDesc{p->w1, d->H, d->B, L.w1s, nullptr};
    pb.d[1] = PrepDesc{p->w2, d->B, d->H, L.w2s, nullptr};
    pb.nd = 2;
    CTN_HIP(launch_prep_weights(dt, pb, s));
    w1 = L.w1s;
    w2 = L.w2s;
  }
  // 1x1 conv B->H (pre-PReLU h1)
  GemmRows g1{};
  g1.g = rg; g1.Kred = d->B; g1.Nout = d->H; g1.norm = NORM_GLN;
  g1.A = x; g1.lda = d->B; g1.W = w1; g1.ldw = d->B; g1.epi = EPI_STORE; g1.C = sv->h1; g1.ldc = d->H;
  CTN_HIP(launch_gemm_rows(dt, g1, s));
  // BN-1 statistics of PReLU(h1)
  int rc = bn_forward_stats(dt, d, L, sv->h1, p->alpha1, p->gamma1, p->beta1, p->bn_mean1, p->bn_var1,
                            p->bn_training, p->bn_momentum1, p->bn_eps1, st1, L.ge1, L.be1, s);
  if (rc) return rc;
  // BN-1 apply (identity gLN) + dilated depthwise conv
  DwArgs da = bn_dw(d, false);
  da.h1 = sv->h1; da.st1 = L.ident;
  da.alpha1 = p->alpha1; da.gamma1 = L.ge1; da.beta1 = L.be1; da.alpha2 = p->alpha2;
  da.wd = p->wd; da.d_out = sv->d; da.slab2 = L.slab2;
  CTN_HIP(launch_dw_fwd(dt, da, s));
  // BN-2 statistics of PReLU(d)
  rc = bn_forward_stats(dt, d, L, sv->d, p->alpha2, p->gamma2, p->beta2, p->bn_mean2, p->bn_var2,
                        p->bn_training, p->bn_momentum2, p->bn_eps2, st2, L.ge2, L.be2, s);
  if (rc) return rc;
  // BN-2 apply (identity gLN, with PReLU) on the operand, 1x1 conv H->B, residual
  GemmRows g2{};
  g2.g = rg; g2.Kred = d->H; g2.Nout = d->B; g2.norm = NORM_GLN;
  g2.A = sv->d; g2.lda = d->H;
  g2.aop.kind = OP_PRELU_NORM; g2.aop.norm = NORM_GLN; g2.aop.stats = L.ident;
  g2.aop.gamma = L.ge2; g2.aop.beta = L.be2; g2.aop.alpha = p->alpha2;
  g2.W = w2; g2.ldw = d->H;
  g2.epi = EPI_RESID; g2.R = x; g2.ldr = d->B;
  g2.C = y; g2.ldc = d->B;
  CTN_HIP(launch_gemm_rows(dt, g2, s));
  return CTN_OK;
}

static int tb_backward_bn(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x,
                          const ctn_tblock_saved* sv, const void* gy, void* gx, const ctn_tblock_grads* gr, void* ws,
                          size_t ws_bytes, hipStream_t s) {
  const BnLayout L = bn_layout(d, 1, ws);
  if (!ws || ws_bytes < L.bytes) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, L.bytes);
  const DType dt = tb_dt(d);
  const Rows rg{d->M, d->K, d->Kp};
  const int H = d->H, nb = bn_blocks(rg);
  const float2* st1 = reinterpret_cast<const float2*>(sv->stats);
  const float2* st2 = st1 + H;
  const int train1 = p->bn_training || !p->bn_mean1, train2 = p->bn_training || !p->bn_mean2;

  const void* w1t = L.w1t;
  const void* w2t = L.w2t;
  if (dt == BF16 && p->w1t_bf16 && p->w2t_bf16) {
    w1t = p->w1t_bf16;
    w2t = p->w2t_bf16;
  } else {
    PrepBatch pb{};
    pb.d[0] = PrepDesc{p->w2, d->B, H, nullptr, L.w2t};
    pb.d[1] = PrepDesc{p->w1, H, d->B, nullptr, L.w1t};
    pb.nd = 2;
    CTN_HIP(launch_prep_weights(dt, pb, s));
  }
  // gamma' / beta' from the saved statistics; identity and zero tables
  {
    BnFinal pf{};
    pf.H = H; pf.M = d->M; pf.gamma = p->gamma1; pf.beta = p->beta1; pf.stats = const_cast<float2*>(st1);
    pf.gamma_eff = L.ge1; pf.beta_eff = L.be1; pf.ident = L.ident; pf.zero = L.zero;
    CTN_HIP(launch_bn_finalize(pf, 2, s));
    pf.gamma = p->gamma2; pf.beta = p->beta2; pf.stats = const_cast<float2*>(st2);
    pf.gamma_eff = L.ge2; pf.beta_eff = L.be2; pf.ident = nullptr; pf.zero = nullptr;
    CTN_HIP(launch_bn_finalize(pf, 2, s));
  }
  // (a) G1 = dL/dn2 = gy . W2
  GemmRows ga{};
  ga.g = rg; ga.Kred = d->B; ga.Nout = H; ga.norm = NORM_GLN;
  ga.A = gy; ga.lda = d->B; ga.W = w2t; ga.ldw = d->B; ga.epi = EPI_STORE; ga.C = L.G1; ga.ldc = H;
  CTN_HIP(launch_gemm_rows(dt, ga, s));
  // (b) dW2 partials = gy^T . BN2(PReLU(d))
  GemmCols c2{};
  c2.g = rg; c2.P = d->B; c2.Q = H;
  c2.A = gy; c2.lda = d->B;
  c2.B = sv->d; c2.ldb = H;
  c2.bop.kind = OP_PRELU_NORM; c2.bop.norm = NORM_GLN; c2.bop.stats = L.ident;
  c2.bop.gamma = L.ge2; c2.bop.beta = L.be2; c2.bop.alpha = p->alpha2;
  c2.Cpart = L.cpart2; c2.nchunks = L.chunks2;
  CTN_HIP(launch_gemm_cols(dt, c2, s));
  // (c) BN-2 backward sums (= beta2 / gamma2 gradients) and (d) G1 -= per-channel means
  BnArgs ba{};
  ba.g = rg; ba.H = H; ba.part = L.part;
  ba.a = sv->d; ba.gin = L.G1; ba.gout = L.G1; ba.alpha = p->alpha2; ba.stats = st2; ba.sums = L.sums2;
  CTN_HIP(launch_bn_partials(dt, ba, 1, s));
  BnFinal bf{};
  bf.H = H; bf.M = d->M; bf.nparts = nb; bf.count = (long)d->M * d->K; bf.part = L.part;
  bf.training = train2; bf.sums = L.sums2; bf.dgamma = gr->gamma2; bf.dbeta = gr->beta2;
  CTN_HIP(launch_bn_finalize(bf, 1, s));
  CTN_HIP(launch_bn_apply(dt, ba, false, s));
  // (e) depthwise backward in identity mode -> G2 = dL/dn1 * gamma1' ; wd, alpha2 and
  //     (gamma1', beta1') column partials
  DwArgs da = bn_dw(d, true);
  da.h1 = sv->h1; da.d = sv->d; da.st1 = L.ident; da.st2 = L.ident;
  da.alpha1 = p->alpha1; da.gamma1 = L.ge1; da.beta1 = L.be1; da.alpha2 = p->alpha2; da.gamma2 = L.ge2;
  da.wd = p->wd;
  da.ga2 = L.G1; da.sm2 = L.zero; da.ga1_out = L.G2; da.slab1 = L.slabD; da.col_slab = L.colD;
  CTN_HIP(launch_dw_bwd(dt, da, s));
  // (f) BN-1 backward sums over (G2, h1), (g) G1 = (G2 - means) * PReLU'(h1), alpha-1 partials
  ba.a = sv->h1; ba.gin = L.G2; ba.gout = L.G1; ba.alpha = p->alpha1; ba.stats = st1; ba.sums = L.sums1;
  ba.apart = L.alphaSlab;
  CTN_HIP(launch_bn_partials(dt, ba, 1, s));
  bf.training = train1; bf.sums = L.sums1; bf.dgamma = nullptr; bf.dbeta = nullptr;
  CTN_HIP(launch_bn_finalize(bf, 1, s));
  CTN_HIP(launch_bn_apply(dt, ba, true, s));
  // (h) gx = G1 . W1 + gy ; dW1 partials = G1^T . x
  GemmRows gb{};
  gb.g = rg; gb.Kred = H; gb.Nout = d->B; gb.norm = NORM_GLN;
  gb.A = L.G1; gb.lda = H; gb.W = w1t; gb.ldw = H;
  gb.epi = EPI_RESID; gb.R = gy; gb.ldr = d->B; gb.C = gx; gb.ldc = d->B;
  CTN_HIP(launch_gemm_rows(dt, gb, s));
  GemmCols c1{};
  c1.g = rg; c1.P = H; c1.Q = d->B;
  c1.A = L.G1; c1.lda = H; c1.B = x; c1.ldb = d->B;
  c1.Cpart = L.cpart1; c1.nchunks = L.chunks1;
  CTN_HIP(launch_gemm_cols(dt, c1, s));
  // (i) parameter-gradient partial sums, (j) gamma1 from the identity-mode (gamma1', beta1')
  const int dwb = dw_blocks(da), dws = dw_col_stride(da);
  const int HB = H * d->B;
  SlabBatch sb{};
  sb.d[0] = SlabDesc{L.cpart2, gr->w2, L.chunks2, HB, HB};
  sb.d[1] = SlabDesc{L.cpart1, gr->w1, L.chunks1, HB, HB};
  sb.d[2] = SlabDesc{L.colD, gr->gamma1, dwb, H, dws};
  sb.d[3] = SlabDesc{L.colD + H, gr->beta1, dwb, H, dws};
  sb.d[4] = SlabDesc{L.colD + 2 * H, gr->wd, dwb, H * d->P, dws};
  sb.d[5] = SlabDesc{L.colD + (4 + d->P) * H, gr->alpha2, dwb, 1, dws};
  sb.d[6] = SlabDesc{L.alphaSlab, gr->alpha1, nb, 1, 1};
  sb.nd = 7;
  CTN_HIP(launch_slab_reduce(sb, L.srtmp, s));
  CTN_HIP(launch_bn_gamma_fix(gr->gamma1, gr->beta1, st1, H, s));
  return CTN_OK;
}

extern "C" size_t ctn_tblock_workspace_bytes(const ctn_tblock_desc* d, int backward) {
  if (tb_check(d) != CTN_OK) return 0;
  if (d->norm_type == CTN_NORM_BN) return bn_layout(d, backward, nullptr).bytes;
  return tb_layout(d, backward, nullptr).bytes;
}

extern "C" int ctn_tblock_forward(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x, void* y,
                                  const ctn_tblock_saved* sv, void* ws, size_t ws_bytes, void* stream) {
  int rc = tb_check(d);
  if (rc) return rc;
  if (!p || !x || !y || !sv || !sv->h1 || !sv->d || !sv->stats) return fail(CTN_ERR_ARG, "null pointer");
  if (d->norm_type == CTN_NORM_BN) return tb_forward_bn(d, p, x, y, sv, ws, ws_bytes, (hipStream_t)stream);
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
  const void *w1f = nullptr, *w2f = nullptr;   // fragment-ordered copies (caller packs only)
  if (dt == BF16 && p->w1_bf16 && p->w2_bf16) {   // packed once per step by the caller
    w1 = p->w1_bf16;
    w2 = p->w2_bf16;
    w1f = p->w1_frag;
    w2f = p->w2_frag;
  } else if (dt == BF16) {
    PrepBatch pb{};
    pb.d[0] = PrepDesc{p->w1, d->H, d->B, L.w1s, nullptr};
    pb.d[1] = PrepDesc{p->w2, d->B, d->H, L.w2s, nullptr};
    pb.nd = 2;
    CTN_HIP(launch_prep_weights(dt, pb, s));
    w1 = L.w1s;
    w2 = L.w2s;
  }
  // 1x1 conv B->H, PReLU statistics for norm1
  GemmRows g1 = tb_gemm1(d);
  g1.A = x;
  g1.W = w1;
  g1.Wf = w1f;
  g1.alpha = p->alpha1;
  g1.C = sv->h1;
  g1.grp_slab = L.slab1;
  // cLN on the WS kernel: the workgroup holds all H channels of its rows and writes
  // the final per-row statistics itself
  const bool fin1 = d->norm_type == CTN_NORM_CLN && gemm_ws_final_cln(dt, g1);
  if (fin1) {
    g1.stats_out = st1;
    g1.eps = (float)kEps;
  }
  {
    TimedScope ts(CTN_TIMER_GEMM1, s);
    CTN_HIP(launch_gemm_rows(dt, g1, s));
  }
  // gLN: the consumers finalize the statistics from the slab partials (StatFold)
  const bool fold = d->norm_type == CTN_NORM_GLN;
  if (!fold && !fin1) CTN_HIP(launch_stats_finalize(L.slab1, G, L.parts1, cnt, 0, (float)kEps, st1, s));
  // norm1 apply + depthwise dilated conv, PReLU statistics for norm2
  DwArgs da{};
  da.g = rg; da.H = d->H; da.P = d->P; da.dil = d->dilation; da.pad = tb_pad(d); da.norm = d->norm_type;
  da.seg = dw_seg(da, false);
  da.h1 = sv->h1; da.st1 = st1;
  da.alpha1 = p->alpha1; da.gamma1 = p->gamma1; da.beta1 = p->beta1; da.alpha2 = p->alpha2;
  da.wd = p->wd; da.d_out = sv->d; da.slab2 = L.slab2;
  if (fold) da.f_st1 = gemm_rows_stat_fold(dt, g1, L.slab1, cnt, (float)kEps, 0, st1);
  if (d->norm_type == CTN_NORM_CLN) {   // per-row statistics final in the depthwise kernel
    da.st2_out = st2;
    da.eps = (float)kEps;
  }
  {
    TimedScope ts(CTN_TIMER_DW_FWD, s);
    CTN_HIP(launch_dw_fwd(dt, da, s));
  }
  // norm2 apply (+PReLU) on the operand, 1x1 conv H->B, residual add
  GemmRows g2{};
  g2.g = rg; g2.Kred = d->H; g2.Nout = d->B; g2.norm = d->norm_type;
  g2.A = sv->d; g2.lda = d->H;
  g2.aop.kind = OP_PRELU_NORM; g2.aop.norm = d->norm_type; g2.aop.stats = st2;
  g2.aop.gamma = p->gamma2; g2.aop.beta = p->beta2; g2.aop.alpha = p->alpha2;
  g2.W = w2; g2.ldw = d->H; g2.Wf = w2f;
  g2.epi = EPI_RESID; g2.R = x; g2.ldr = d->B;
  g2.C = y; g2.ldc = d->B;
  if (fold && (ws_fold_mask() & 1) && gemm_ws_can_fold(dt, g2))
    g2.aop.fold = StatFold{L.slab2, L.parts2, cnt, (float)kEps, 0, st2};
  else if (!da.st2_out) CTN_HIP(launch_stats_finalize(L.slab2, G, L.parts2, cnt, 0, (float)kEps, st2, s));
  {
    TimedScope ts(CTN_TIMER_GEMM2, s);
    CTN_HIP(launch_gemm_rows(dt, g2, s));
  }
  return CTN_OK;
}

// one fork event per device (hipStreamWaitEvent takes the event's state when it is
// called, so re-recording it for the next call is safe)
static hipError_t fork_stream(hipStream_t from, hipStream_t to) {
  static hipEvent_t ev[64] = {};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  if (!ev[dev] && (e = hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming)) != hipSuccess) return e;
  if ((e = hipEventRecord(ev[dev], from)) != hipSuccess) return e;
  return hipStreamWaitEvent(to, ev[dev], 0);
}

static int tb_backward(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x,
                       const ctn_tblock_saved* sv, const void* gy, void* gx, const ctn_tblock_grads* gr,
                       void* ws, size_t ws_bytes, hipStream_t s, hipStream_t sw, void* part = nullptr,
                       size_t part_bytes = 0, bool defer = false);

extern "C" int ctn_tblock_backward(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x,
                                   const ctn_tblock_saved* sv, const void* gy, void* gx, const ctn_tblock_grads* gr,
                                   void* ws, size_t ws_bytes, void* stream) {
  return tb_backward(d, p, x, sv, gy, gx, gr, ws, ws_bytes, (hipStream_t)stream, (hipStream_t)stream);
}

extern "C" int ctn_tblock_backward_split(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x,
                                         const ctn_tblock_saved* sv, const void* gy, void* gx,
                                         const ctn_tblock_grads* gr, void* ws, size_t ws_bytes, void* stream,
                                         void* wgrad_stream) {
  return tb_backward(d, p, x, sv, gy, gx, gr, ws, ws_bytes, (hipStream_t)stream,
                     wgrad_stream ? (hipStream_t)wgrad_stream : (hipStream_t)stream);
}

// The fixed-order reductions of every parameter gradient of a block backward (step (g)):
// descriptors over the partials that layout L points at, into the gradients gr.
static int tb_grad_slabs(const ctn_tblock_desc* d, const TbLayout& L, const ctn_tblock_grads* gr, SlabDesc* out) {
  DwArgs da{};
  da.g = Rows{d->M, d->K, d->Kp}; da.H = d->H; da.P = d->P; da.dil = d->dilation; da.pad = tb_pad(d);
  da.norm = d->norm_type;
  da.seg = dw_seg(da, true);
  const int nalpha = tb_fused_n1(d) ? gemm_ws_grid(tb_gemmB(d, true)) : ew_blocks(da);
  const int dwb = dw_blocks(da), dws = dw_col_stride(da);
  const int HB = d->H * d->B, H = d->H;
  out[0] = SlabDesc{L.cpart2, gr->w2, L.chunks2, HB, HB};
  out[1] = SlabDesc{L.cpart1, gr->w1, L.chunks1, HB, HB};
  out[2] = SlabDesc{L.colD + (2 + d->P) * H, gr->gamma2, dwb, H, dws};
  out[3] = SlabDesc{L.colD + (3 + d->P) * H, gr->beta2, dwb, H, dws};
  out[4] = SlabDesc{L.colD, gr->gamma1, dwb, H, dws};
  out[5] = SlabDesc{L.colD + H, gr->beta1, dwb, H, dws};
  out[6] = SlabDesc{L.colD + 2 * H, gr->wd, dwb, H * d->P, dws};
  out[7] = SlabDesc{L.colD + (4 + d->P) * H, gr->alpha2, dwb, 1, dws};
  out[8] = SlabDesc{L.alphaSlab, gr->alpha1, nalpha, 1, 1};
  return 9;
}

// sw: the stream of the parameter-gradient tail (== s: one stream).
// defer: the parameter-gradient partials go to `part` and step (g) is left to
// ctn_tblock_reduce_grads.
static int tb_backward(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x,
                       const ctn_tblock_saved* sv, const void* gy, void* gx, const ctn_tblock_grads* gr,
                       void* ws, size_t ws_bytes, hipStream_t s, hipStream_t sw, void* part, size_t part_bytes,
                       bool defer) {
  int rc = tb_check(d);
  if (rc) return rc;
  if (!p || !x || !sv || !gy || !gx || !gr) return fail(CTN_ERR_ARG, "null pointer");
  if (d->norm_type == CTN_NORM_BN) {
    if (defer) return fail(CTN_ERR_UNSUPPORTED, "deferred gradient reductions: gLN / cLN blocks only");
    return tb_backward_bn(d, p, x, sv, gy, gx, gr, ws, ws_bytes, s);
  }
  const TbLayout L = tb_layout(d, 1, ws, part, defer);
  if (!ws || ws_bytes < L.bytes) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, L.bytes);
  if (defer && (!part || part_bytes < L.part_bytes))
    return fail(CTN_ERR_WORKSPACE, "partials buffer %zu < %zu", part_bytes, L.part_bytes);
  const DType dt = d->dtype == CTN_DTYPE_BF16 ? BF16 : F32;
  const Rows rg{d->M, d->K, d->Kp};
  const int G = tb_groups(d);
  const float2* st1 = reinterpret_cast<const float2*>(sv->stats);
  const float2* st2 = st1 + G;
  const double cnt = d->norm_type == CTN_NORM_GLN ? (double)d->K * d->H : (double)d->H;

  const void* w1t = L.w1t;
  const void* w2t = L.w2t;
  const void *w1tf = nullptr, *w2tf = nullptr;   // fragment-ordered copies (caller packs only)
  if (dt == BF16 && p->w1t_bf16 && p->w2t_bf16) {   // packed once per step by the caller
    w1t = p->w1t_bf16;
    w2t = p->w2t_bf16;
    w1tf = p->w1t_frag;
    w2tf = p->w2t_frag;
  } else {
    PrepBatch pb{};
    pb.d[0] = PrepDesc{p->w2, d->B, d->H, nullptr, L.w2t};   // [H][B]
    pb.d[1] = PrepDesc{p->w1, d->H, d->B, nullptr, L.w1t};   // [B][H]
    pb.nd = 2;
    CTN_HIP(launch_prep_weights(dt, pb, s));
  }

  // (a) G1 = g_n2 = gy . W2 ; epilogue: norm-2 backward sums of (g_n2*gamma2, g_n2*gamma2*hat a2)
  // (b) dW2 = gy^T . norm2(PReLU(d))            — one dual-GEMM pass when eligible
  GemmRows ga = tb_gemmA(d);
  ga.A = gy;
  ga.W = w2t;
  ga.Wf = w2tf;
  ga.R = sv->d;
  ga.alpha = p->alpha2; ga.stats = st2; ga.gamma = p->gamma2;
  ga.C = L.G1;
  ga.grp_slab = L.slabA;
  GemmDual duA = tb_dualA(d);
  duA.A = gy; duA.W = w2t; duA.Wf = w2tf; duA.R = sv->d; duA.C = L.G1;
  duA.alpha = p->alpha2; duA.stats = st2; duA.gamma = p->gamma2; duA.grp_slab = L.slabA;
  duA.Bm = sv->d;
  duA.bop.stats = st2; duA.bop.gamma = p->gamma2; duA.bop.beta = p->beta2; duA.bop.alpha = p->alpha2;
  duA.Dpart = L.cpart2;
  const bool dualA = gemm_dual_eligible(dt, duA);
  if (dualA) {
    TimedScope ts(CTN_TIMER_GEMM_A, s);
    CTN_HIP(launch_gemm_dual(duA, s));
  } else {
    {
      TimedScope ts(CTN_TIMER_GEMM_A, s);
      CTN_HIP(launch_gemm_rows(dt, ga, s));
    }
    GemmCols c2{};
    c2.g = rg; c2.P = d->B; c2.Q = d->H;
    c2.A = gy; c2.lda = d->B;
    c2.B = sv->d; c2.ldb = d->H;
    c2.bop.kind = OP_PRELU_NORM; c2.bop.norm = d->norm_type; c2.bop.stats = st2;
    c2.bop.gamma = p->gamma2; c2.bop.beta = p->beta2; c2.bop.alpha = p->alpha2;
    c2.Cpart = L.cpart2; c2.nchunks = L.chunks2;
    CTN_HIP(launch_gemm_cols(dt, c2, s));
  }
  const bool fold = d->norm_type == CTN_NORM_GLN;   // gLN: consumers finalize the sums (StatFold)

  // (c) depthwise backward -> G2 = dL/d(hat a1), norm1 sums, column partials (gamma1/beta1,
  //     wd, gamma2/beta2, alpha2)
  DwArgs da{};
  da.g = rg; da.H = d->H; da.P = d->P; da.dil = d->dilation; da.pad = tb_pad(d); da.norm = d->norm_type;
  da.seg = dw_seg(da, true);
  da.h1 = sv->h1; da.d = sv->d; da.st1 = st1; da.st2 = st2;
  da.alpha1 = p->alpha1; da.gamma1 = p->gamma1; da.beta1 = p->beta1; da.alpha2 = p->alpha2; da.gamma2 = p->gamma2;
  da.wd = p->wd;
  da.ga2 = L.G1; da.sm2 = L.sums2; da.ga1_out = L.G2; da.slab1 = L.slabD; da.col_slab = L.colD;
  if (fold)
    da.f_sm2 = dualA ? gemm_dual_stat_fold(duA, L.slabA, cnt, 0.f, 1, nullptr)
                     : gemm_rows_stat_fold(dt, ga, L.slabA, cnt, 0.f, 1, nullptr);
  else
    da.sm1_out = L.sums1;   // cLN: per-row norm-1 backward means final in the depthwise kernel
  // cLN: the wave-item depthwise backward folds the dual's per-row partials itself (at most
  // 4 per row: ctn_dual_ws.hip CTN_DV_CLNC) instead of a finalize launch
  if (!fold) {
    if (dualA && L.partsA <= 4 && dw_wave_eligible(dt, da))
      da.f_sm2 = gemm_dual_stat_fold(duA, L.slabA, cnt, 0.f, 1, nullptr);
    else
      CTN_HIP(launch_stats_finalize(L.slabA, G, L.partsA, cnt, 1, 0.f, L.sums2, s));
  }
  {
    TimedScope ts(CTN_TIMER_DW_BWD, s);
    CTN_HIP(launch_dw_bwd(dt, da, s));
  }
  const bool fused1 = tb_fused_n1(d);
  int nalpha = ew_blocks(da);
  if (fused1) {
    // (d+e) gx = n1bwd(G2) . W1 + gy; the operand stage applies the norm-1/PReLU-1
    //       backward (norm-1 sums folded from dw_bwd's slab), sums the alpha-1
    //       gradient and stores gh1 = dL/dh1 to G1 on the way (one pass instead of
    //       norm1_bwd's write + the GEMM's re-read)
    GemmRows gb = tb_gemmB(d, true);
    gb.A = L.G2; gb.W = w1t; gb.Wf = w1tf; gb.R = gy; gb.C = gx;
    gb.aop.stats = st1; gb.aop.alpha = p->alpha1; gb.aop.aux = sv->h1; gb.aop.apart = L.alphaSlab;
    gb.aop.aout = L.G1;
    if (fold && (ws_fold_mask() & 2)) {
      gb.aop.fold = StatFold{L.slabD, L.partsD, cnt, 0.f, 1, nullptr};
    } else {
      if (fold) CTN_HIP(launch_stats_finalize(L.slabD, G, L.partsD, cnt, 1, 0.f, L.sums1, s));
      gb.aop.sums = L.sums1;
    }
    {
      TimedScope ts(CTN_TIMER_GEMM_GX, s);
      CTN_HIP(launch_gemm_rows(dt, gb, s));
    }
    nalpha = gemm_ws_grid(gb);
    // everything below only produces parameter gradients: fork to sw
    if (sw != s) CTN_HIP(fork_stream(s, sw));
    // (f) dW1 = gh1^T . x, gh1 = G1 as stored by the kernel above
    GemmCols c1{};
    c1.g = rg; c1.P = d->H; c1.Q = d->B;
    c1.A = L.G1; c1.lda = d->H;
    c1.B = x; c1.ldb = d->B;
    c1.Cpart = L.cpart1; c1.nchunks = L.chunks1;
    {
      TimedScope ts(CTN_TIMER_COLS_W1, sw);
      CTN_HIP(launch_gemm_cols(dt, c1, sw));
    }
  } else {
    // (d) norm1 backward finish + PReLU1 backward -> G1 = dL/dh1
    DwArgs de = da;
    de.ga2 = L.G2; de.sm1 = L.sums1; de.gh1_out = L.G1; de.alpha_slab = L.alphaSlab;
    de.f_sm2 = StatFold{};
    if (fold) de.f_sm1 = StatFold{L.slabD, L.partsD, cnt, 0.f, 1, nullptr};
    CTN_HIP(launch_norm1_bwd(dt, de, s));
    // (e) gx = gh1 . W1 + gy
    // (f) dW1 = gh1^T . x                          — one dual-GEMM pass when eligible
    GemmDual duB = tb_dualB(d);
    duB.A = L.G1; duB.W = w1t; duB.Wf = w1tf; duB.R = gy; duB.C = gx;
    duB.Bm = x; duB.Dpart = L.cpart1;
    if (gemm_dual_eligible(dt, duB)) {
      CTN_HIP(launch_gemm_dual(duB, s));
    } else {
      GemmRows gb{};
      gb.g = rg; gb.Kred = d->H; gb.Nout = d->B; gb.norm = d->norm_type;
      gb.A = L.G1; gb.lda = d->H;
      gb.W = w1t; gb.ldw = d->H; gb.Wf = w1tf;
      gb.epi = EPI_RESID; gb.R = gy; gb.ldr = d->B;
      gb.C = gx; gb.ldc = d->B;
      CTN_HIP(launch_gemm_rows(dt, gb, s));
      GemmCols c1{};
      c1.g = rg; c1.P = d->H; c1.Q = d->B;
      c1.A = L.G1; c1.lda = d->H;
      c1.B = x; c1.ldb = d->B;
      c1.Cpart = L.cpart1; c1.nchunks = L.chunks1;
      CTN_HIP(launch_gemm_cols(dt, c1, s));
    }
    if (sw != s) CTN_HIP(fork_stream(s, sw));
  }
  // (g) all parameter-gradient partial sums
  (void)nalpha;   // tb_grad_slabs recomputes the alpha-1 part count from the descriptor
  if (defer) return CTN_OK;
  SlabBatch sb{};
  sb.nd = tb_grad_slabs(d, L, gr, sb.d);
  CTN_HIP(launch_slab_reduce(sb, L.srtmp, sw));
  return CTN_OK;
}

// Which kernel each step of the block would launch (ctn_tblock_plan): the eligibility
// queries the launches themselves make, on the descriptor alone
extern "C" int ctn_tblock_plan(const ctn_tblock_desc* d, int backward, char* out, size_t cap) {
  int rc = tb_check(d);
  if (rc) return rc;
  if (!out || cap < 1) return fail(CTN_ERR_ARG, "null output");
  const DType dt = tb_dt(d);
  std::string s;
  DwArgs da{};
  da.g = Rows{d->M, d->K, d->Kp}; da.H = d->H; da.P = d->P; da.dil = d->dilation; da.pad = tb_pad(d);
  da.norm = d->norm_type;
  if (d->norm_type == CTN_NORM_BN) {
    s = backward ? "bn:rows+cols" : "bn:rows";
  } else if (!backward) {
    GemmRows g2{};
    g2.g = da.g; g2.Kred = d->H; g2.Nout = d->B; g2.norm = d->norm_type; g2.lda = d->H; g2.ldw = d->H;
    g2.aop.kind = OP_PRELU_NORM; g2.aop.norm = d->norm_type; g2.epi = EPI_RESID; g2.ldr = d->B; g2.ldc = d->B;
    da.seg = dw_seg(da, false);
    s = std::string("gemm1=") + (gemm_ws_eligible(dt, tb_gemm1(d)) ? "ws" : "rows") +
        ",dw_fwd=" + (dw_wave_eligible(dt, da) ? "wave" : "lane") +
        ",gemm2=" + (gemm_ws_eligible(dt, g2) ? "ws" : "rows");
  } else {
    const GemmDual duA = tb_dualA(d), duB = tb_dualB(d);
    da.seg = dw_seg(da, true);
    const bool dualA = gemm_dual_eligible(dt, duA);
    s = std::string("pairA=") + (dualA ? (gemm_dual_ws_eligible(duA) ? "dual_ws" : "dual")
                                       : (gemm_ws_eligible(dt, tb_gemmA(d)) ? "ws+cols" : "rows+cols")) +
        ",dw_bwd=" + (dw_wave_eligible(dt, da) ? "wave" : "lane");
    if (tb_fused_n1(d)) {
      GemmCols c1{};
      c1.g = da.g; c1.P = d->H; c1.Q = d->B; c1.lda = d->H; c1.ldb = d->B;
      c1.A = c1.B = c1.Cpart = reinterpret_cast<float*>(256);   // alignment only
      s += std::string(",gx=ws_n1bwd,dW1=") + (gemm_cols_ws_eligible(dt, c1) ? "cols_ws" : "cols");
    } else {
      s += std::string(",n1bwd=ew,gx+dW1=") + (gemm_dual_eligible(dt, duB) ? "dual" : "rows+cols");
    }
  }
  if (s.size() + 1 > cap) return fail(CTN_ERR_ARG, "plan needs %zu bytes", s.size() + 1);
  memcpy(out, s.c_str(), s.size() + 1);
  return CTN_OK;
}

extern "C" size_t ctn_tblock_partials_bytes(const ctn_tblock_desc* d) {
  if (tb_check(d) != CTN_OK || d->norm_type == CTN_NORM_BN) return 0;
  return tb_layout(d, 1, nullptr, nullptr, true).part_bytes;
}

extern "C" size_t ctn_tblock_deferred_workspace_bytes(const ctn_tblock_desc* d) {
  if (tb_check(d) != CTN_OK || d->norm_type == CTN_NORM_BN) return 0;
  return tb_layout(d, 1, nullptr, nullptr, true).bytes;
}

extern "C" int ctn_tblock_backward_deferred(const ctn_tblock_desc* d, const ctn_tblock_params* p, const void* x,
                                            const ctn_tblock_saved* sv, const void* gy, void* gx,
                                            const ctn_tblock_grads* gr, void* ws, size_t ws_bytes, void* part,
                                            size_t part_bytes, void* stream) {
  return tb_backward(d, p, x, sv, gy, gx, gr, ws, ws_bytes, (hipStream_t)stream, (hipStream_t)stream, part,
                     part_bytes, true);
}

extern "C" int ctn_tblock_reduce_grads(const ctn_tblock_desc* descs, const ctn_tblock_grads* grads,
                                       void* const* parts, int n, void* stream) {
  if (n < 0 || (n > 0 && (!descs || !grads || !parts))) return fail(CTN_ERR_ARG, "null pointer");
  // an error a kernel of an earlier pass reported (device error word, copied asynchronously)
  if (int rc = dev_err_check_async()) return rc;
  std::vector<SlabDesc> sd;
  std::vector<float*> tmp;
  sd.reserve((size_t)n * 9);
  tmp.reserve((size_t)n * 9);
  for (int i = 0; i < n; ++i) {
    const ctn_tblock_desc* d = descs + i;
    int rc = tb_check(d);
    if (rc) return rc;
    if (d->norm_type == CTN_NORM_BN) return fail(CTN_ERR_UNSUPPORTED, "deferred gradient reductions: gLN / cLN only");
    if (!parts[i]) return fail(CTN_ERR_ARG, "null partials buffer (block %d)", i);
    const TbLayout L = tb_layout(d, 1, nullptr, parts[i], true);
    SlabDesc b[12];
    const int nb = tb_grad_slabs(d, L, grads + i, b);
    float* t[12];
    slab_reduce_assign_tmp(b, nb, L.srtmp, t);
    for (int k = 0; k < nb; ++k) {
      sd.push_back(b[k]);
      tmp.push_back(t[k]);
    }
  }
  CTN_HIP(launch_slab_reduce_list(sd.data(), tmp.data(), (int)sd.size(), (hipStream_t)stream));
  CTN_HIP(dev_err_refresh((hipStream_t)stream));   // checked by the next pass (or ctn_device_status)
  return CTN_OK;
}

// ===========================================================================
// Encoder front: encoder + separator cLN + bottleneck
// ===========================================================================
#include "ctn_codec.h"

static int codec_check(const ctn_codec_desc* d, bool need_b) {
  if (!d) return fail(CTN_ERR_ARG, "null descriptor");
  if (d->M < 1 || d->T < d->L || d->L < 2 || d->L > 32)
    return fail(CTN_ERR_UNSUPPORTED, "M=%d T=%d L=%d (need T >= L, 2 <= L <= 32)", d->M, d->T, d->L);
  const int S = d->L / 2;
  if (d->K != (d->T - d->L) / S + 1) return fail(CTN_ERR_ARG, "K=%d != (T-L)/(L/2)+1", d->K);
  if (d->Kp != ctn_padded_frames(d->K)) return fail(CTN_ERR_ARG, "Kp=%d != padded(K)", d->Kp);
  const int cg = d->N / 8;
  if (d->N % 8 || cg > 64 || (cg & (cg - 1)))
    return fail(CTN_ERR_UNSUPPORTED, "N=%d: need N/8 a power of two <= 64", d->N);
  if (need_b && (d->B % 8 || d->B < 8)) return fail(CTN_ERR_UNSUPPORTED, "B=%d must be a multiple of 8", d->B);
  if (d->C < 1 || d->C > 16) return fail(CTN_ERR_UNSUPPORTED, "C=%d outside 1..16", d->C);
  if (d->mask_type < 0 || d->mask_type > 2) return fail(CTN_ERR_ARG, "mask_type %d", d->mask_type);
  if (d->dtype != CTN_DTYPE_F32 && d->dtype != CTN_DTYPE_BF16) return fail(CTN_ERR_ARG, "dtype %d", d->dtype);
  return CTN_OK;
}

static CodecArgs codec_args(const ctn_codec_desc* d) {
  CodecArgs a{};
  a.M = d->M; a.T = d->T; a.K = d->K; a.Kp = d->Kp; a.N = d->N; a.L = d->L; a.S = d->L / 2; a.C = d->C;
  a.mask_type = d->mask_type;
  return a;
}

namespace {
// bf16: the encoder basis gradient dU[n][l] = sum_r gpre[r][n] x[kS + l] as a column GEMM
// (gemm_cols, P = N, Q = L padded to 8) of bf16 dL/d(pre-ReLU) rows and mixture frames,
// instead of the LDS-bound frame_outer kernel.  CTN_DU_COLS=0 keeps frame_outer (A/B).
bool du_cols(const ctn_codec_desc* d) {
  const char* e = getenv("CTN_DU_COLS");
  if (e && atoi(e) == 0) return false;
  return d->dtype == CTN_DTYPE_BF16 && d->N % 8 == 0;
}
GemmCols du_gemm(const ctn_codec_desc* d, int Lp) {
  GemmCols g{};
  g.g = Rows{d->M, d->K, d->Kp};
  g.P = d->N; g.Q = Lp;
  return g;
}
struct EncLayout {
  void *wbs, *wbt, *gcln, *gpre_bf, *xfr;
  float *gpre, *colE, *slabU, *cpartB, *cpartU, *tmpU, *srtmp;
  int chunksB, nU, rowblocks, chunksU, Lp;
  size_t bytes;
};
EncLayout enc_layout(const ctn_codec_desc* d, int backward, void* ws) {
  EncLayout L{};
  Carver c(ws);
  const size_t es = esize(d->dtype);
  const long rows = (long)d->M * d->Kp;
  if (!backward) {
    if (d->dtype == CTN_DTYPE_BF16) L.wbs = c.take<void>((size_t)d->B * d->N * es);
  } else {
    L.wbt = c.take<void>((size_t)d->B * d->N * es);
    L.gcln = c.take<void>((size_t)rows * d->N * es);
    L.rowblocks = (int)(rows / 128);
    L.colE = c.take<float>((size_t)L.rowblocks * 2 * d->N * sizeof(float));
    CodecArgs a = codec_args(d);
    if (du_cols(d)) {
      L.Lp = (d->L + 7) & ~7;
      L.gpre_bf = c.take<void>((size_t)rows * d->N * 2);
      L.xfr = c.take<void>((size_t)rows * L.Lp * 2);
      L.chunksU = gemm_cols_default_chunks(du_gemm(d, L.Lp));
      L.cpartU = c.take<float>((size_t)L.chunksU * d->N * L.Lp * sizeof(float));
      L.tmpU = c.take<float>((size_t)d->N * L.Lp * sizeof(float));
    } else {
      L.gpre = c.take<float>((size_t)rows * d->N * sizeof(float));
      L.nU = frame_outer_chunks(a, 1);
      L.slabU = c.take<float>((size_t)L.nU * d->N * d->L * sizeof(float));
    }
    GemmCols gc{};
    gc.g = Rows{d->M, d->K, d->Kp}; gc.P = d->B; gc.Q = d->N;
    L.chunksB = gemm_cols_default_chunks(gc);
    L.cpartB = c.take<float>((size_t)L.chunksB * d->B * d->N * sizeof(float));
    const size_t ntmp = sr_tmp(L.chunksB, (long)d->B * d->N) + 2 * sr_tmp(L.rowblocks, d->N) +
                        sr_tmp(L.nU, (long)d->N * d->L) + sr_tmp(L.chunksU, (long)d->N * L.Lp);
    L.srtmp = c.take<float>(ntmp * sizeof(float));
  }
  L.bytes = c.off + 256;
  return L;
}
}  // namespace

extern "C" size_t ctn_encoder_workspace_bytes(const ctn_codec_desc* d, int backward) {
  if (codec_check(d, true) != CTN_OK) return 0;
  return enc_layout(d, backward, nullptr).bytes;
}

extern "C" int ctn_encoder_forward(const ctn_codec_desc* d, const float* mixture, const float* U,
                                   const float* gamma0, const float* beta0, const float* wb, void* w_rows,
                                   float* cln_stats, void* x0, void* ws, size_t ws_bytes, void* stream) {
  int rc = codec_check(d, wb != nullptr);
  if (rc) return rc;
  if (!mixture || !U || !w_rows) return fail(CTN_ERR_ARG, "null pointer");
  if (wb && (!gamma0 || !beta0 || !cln_stats || !x0)) return fail(CTN_ERR_ARG, "bottleneck needs gamma0/beta0/stats/x0");
  const EncLayout Ly = enc_layout(d, 0, ws);
  if (!ws || ws_bytes < Ly.bytes) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, Ly.bytes);
  hipStream_t s = (hipStream_t)stream;
  const DType dt = d->dtype == CTN_DTYPE_BF16 ? BF16 : F32;
  CodecArgs a = codec_args(d);
  a.mixture = mixture; a.U = U; a.w_rows = w_rows; a.cln_stats = reinterpret_cast<float2*>(cln_stats);
  CTN_HIP(launch_enc_fwd(dt, a, s));
  if (!wb) return CTN_OK;
  const void* wbp = wb;
  if (dt == BF16) {
    CTN_HIP(launch_prep_weight(dt, wb, d->B, d->N, Ly.wbs, nullptr, s));
    wbp = Ly.wbs;
  }
  GemmRows g{};
  g.g = Rows{d->M, d->K, d->Kp}; g.Kred = d->N; g.Nout = d->B; g.norm = NORM_CLN;
  g.A = w_rows; g.lda = d->N;
  g.aop.kind = OP_NORM; g.aop.norm = NORM_CLN; g.aop.stats = a.cln_stats; g.aop.gamma = gamma0; g.aop.beta = beta0;
  g.W = wbp; g.ldw = d->N;
  g.epi = EPI_STORE; g.C = x0; g.ldc = d->B;
  CTN_HIP(launch_gemm_rows(dt, g, s));
  return CTN_OK;
}

extern "C" int ctn_encoder_backward(const ctn_codec_desc* d, const float* mixture, const float* U,
                                    const float* gamma0, const float* beta0, const float* wb, const void* w_rows,
                                    const float* cln_stats, const void* g_w_rows, const void* g_x0, float* gU,
                                    float* ggamma0, float* gbeta0, float* gwb, void* ws, size_t ws_bytes,
                                    void* stream) {
  int rc = codec_check(d, g_x0 != nullptr);
  if (rc) return rc;
  if (!mixture || !w_rows || !gU) return fail(CTN_ERR_ARG, "null pointer");
  if (g_x0 && (!wb || !gamma0 || !beta0 || !cln_stats || !ggamma0 || !gbeta0 || !gwb))
    return fail(CTN_ERR_ARG, "bottleneck backward needs wb/gamma0/beta0/stats and their gradient outputs");
  const EncLayout Ly = enc_layout(d, 1, ws);
  if (!ws || ws_bytes < Ly.bytes) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, Ly.bytes);
  hipStream_t s = (hipStream_t)stream;
  const DType dt = d->dtype == CTN_DTYPE_BF16 ? BF16 : F32;
  const Rows rg{d->M, d->K, d->Kp};
  CodecArgs a = codec_args(d);
  a.mixture = mixture; a.U = U; a.w_rows = const_cast<void*>(w_rows);
  a.cln_stats = const_cast<float2*>(reinterpret_cast<const float2*>(cln_stats));
  a.gamma0 = gamma0; a.gwdec = g_w_rows; a.gpre = Ly.gpre; a.gpre_bf = Ly.gpre_bf;
  SlabBatch sb{};
  if (g_x0) {
    CTN_HIP(launch_prep_weight(dt, wb, d->B, d->N, nullptr, Ly.wbt, s));   // [N][B]
    GemmRows g{};
    g.g = rg; g.Kred = d->B; g.Nout = d->N;
    g.A = g_x0; g.lda = d->B; g.W = Ly.wbt; g.ldw = d->B;
    g.epi = EPI_STORE; g.C = Ly.gcln; g.ldc = d->N;
    CTN_HIP(launch_gemm_rows(dt, g, s));
    GemmCols gc{};
    gc.g = rg; gc.P = d->B; gc.Q = d->N;
    gc.A = g_x0; gc.lda = d->B;
    gc.B = w_rows; gc.ldb = d->N;
    gc.bop.kind = OP_NORM; gc.bop.norm = NORM_CLN; gc.bop.stats = a.cln_stats; gc.bop.gamma = gamma0; gc.bop.beta = beta0;
    gc.Cpart = Ly.cpartB; gc.nchunks = Ly.chunksB;
    CTN_HIP(launch_gemm_cols(dt, gc, s));
    a.gcln = Ly.gcln;
    a.col_slab = Ly.colE;
    sb.d[sb.nd++] = SlabDesc{Ly.cpartB, gwb, Ly.chunksB, d->B * d->N, d->B * d->N};
    sb.d[sb.nd++] = SlabDesc{Ly.colE, ggamma0, Ly.rowblocks, d->N, 2 * d->N};
    sb.d[sb.nd++] = SlabDesc{Ly.colE + d->N, gbeta0, Ly.rowblocks, d->N, 2 * d->N};
  }
  CTN_HIP(launch_enc_bwd_rows(dt, a, s));
  const bool cols = Ly.gpre_bf != nullptr;
  if (cols) {
    a.Lp = Ly.Lp;
    CTN_HIP(launch_frames_bf16(a, mixture, 1, Ly.xfr, s));
    GemmCols gu = du_gemm(d, Ly.Lp);
    gu.A = Ly.gpre_bf; gu.lda = d->N; gu.B = Ly.xfr; gu.ldb = Ly.Lp;
    gu.Cpart = Ly.cpartU; gu.nchunks = Ly.chunksU;
    CTN_HIP(launch_gemm_cols(dt, gu, s));
    // [chunk][N][Lp] partials -> [N][Lp] -> dU [N][L]
    sb.d[sb.nd++] = SlabDesc{Ly.cpartU, Ly.Lp == d->L ? gU : Ly.tmpU, Ly.chunksU, d->N * Ly.Lp, d->N * Ly.Lp};
  } else {
    CodecArgs fo = a;
    fo.col_slab = Ly.slabU;
    CTN_HIP(launch_frame_outer(dt, 0, fo, s));
    sb.d[sb.nd++] = SlabDesc{Ly.slabU, gU, Ly.nU, d->N * d->L, d->N * d->L};
  }
  CTN_HIP(launch_slab_reduce(sb, Ly.srtmp, s));
  if (cols && Ly.Lp != d->L) CTN_HIP(launch_unpad_cols(Ly.tmpU, d->N, Ly.Lp, d->L, gU, s));
  return CTN_OK;
}

// ===========================================================================
// Decoder back: mask conv + nonlinearity + decoder + overlap-add + pad
// ===========================================================================
namespace {
// bf16 MFMA decoder: the basis gradient dV = sum over (frame, speaker) of gframes^T . src
// runs as a column GEMM (gemm_cols over M*Kp*C rows, P = L padded to 8, Q = N) on
// operands the decoder backward writes, instead of the LDS-bound frame_outer kernel.
// CTN_DV_COLS=0 keeps frame_outer (A/B).
bool dv_cols(const ctn_codec_desc* d) {
  const char* e = getenv("CTN_DV_COLS");
  if (e && atoi(e) == 0) return false;
  return codec_dec_mfma(d->dtype == CTN_DTYPE_BF16 ? BF16 : F32, codec_args(d));
}
GemmCols dv_gemm(const ctn_codec_desc* d, int Lp) {
  GemmCols g{};
  g.g = Rows{d->M, d->K * d->C, d->Kp * d->C};
  g.P = Lp; g.Q = d->N;
  return g;
}
struct DecLayout {
  void *wms, *wmt, *gscore, *srcb, *gfr;
  float *frames, *slabV, *cpartM, *cpartV, *srtmp;
  int nV, chunksM, chunksV, Lp;
  size_t bytes;
};
DecLayout dec_layout(const ctn_codec_desc* d, int backward, bool with_mask_conv, void* ws) {
  DecLayout L{};
  Carver c(ws);
  const size_t es = esize(d->dtype);
  const long rows = (long)d->M * d->Kp;
  const int CN = d->C * d->N;
  if (!backward) {
    if (with_mask_conv && d->dtype == CTN_DTYPE_BF16) L.wms = c.take<void>((size_t)CN * d->B * es);
    L.frames = c.take<float>((size_t)d->M * d->C * d->Kp * d->L * sizeof(float));
  } else {
    CodecArgs a = codec_args(d);
    if (dv_cols(d)) {
      L.Lp = (d->L + 7) & ~7;
      L.srcb = c.take<void>((size_t)rows * d->C * d->N * es);
      L.gfr = c.take<void>((size_t)rows * d->C * L.Lp * es);
      L.chunksV = gemm_cols_default_chunks(dv_gemm(d, L.Lp));
      L.cpartV = c.take<float>((size_t)L.chunksV * L.Lp * d->N * sizeof(float));
    } else {
      L.nV = frame_outer_chunks(a, d->C);
      L.slabV = c.take<float>((size_t)L.nV * d->N * d->L * sizeof(float));
    }
    if (with_mask_conv) {
      L.wmt = c.take<void>((size_t)CN * d->B * es);
      L.gscore = c.take<void>((size_t)rows * CN * es);
      GemmCols gc{};
      gc.g = Rows{d->M, d->K, d->Kp}; gc.P = CN; gc.Q = d->B;
      L.chunksM = gemm_cols_default_chunks(gc);
      L.cpartM = c.take<float>((size_t)L.chunksM * CN * d->B * sizeof(float));
    }
    L.srtmp = c.take<float>((sr_tmp(L.nV > L.chunksV ? L.nV : L.chunksV, (long)d->N * d->L) +
                             sr_tmp(L.chunksM, (long)CN * d->B)) * sizeof(float));
  }
  L.bytes = c.off + 256;
  return L;
}
}  // namespace

extern "C" size_t ctn_decoder_workspace_bytes(const ctn_codec_desc* d, int backward) {
  if (codec_check(d, d && d->mask_type != CTN_MASK_IDENTITY) != CTN_OK) return 0;
  return dec_layout(d, backward, d->mask_type != CTN_MASK_IDENTITY, nullptr).bytes;
}

extern "C" int ctn_decoder_forward(const ctn_codec_desc* d, const void* x_last, const void* w_rows,
                                   const float* wm, const float* V, void* score, float* est, void* ws,
                                   size_t ws_bytes, void* stream) {
  int rc = codec_check(d, wm != nullptr);
  if (rc) return rc;
  if (!x_last || !w_rows || !V || !est) return fail(CTN_ERR_ARG, "null pointer");
  if ((wm == nullptr) != (d->mask_type == CTN_MASK_IDENTITY))
    return fail(CTN_ERR_ARG, "wm == NULL exactly when mask_type == CTN_MASK_IDENTITY (standalone Decoder)");
  if (wm && !score) return fail(CTN_ERR_ARG, "score output required with the mask conv");
  const DecLayout Ly = dec_layout(d, 0, wm != nullptr, ws);
  if (!ws || ws_bytes < Ly.bytes) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, Ly.bytes);
  hipStream_t s = (hipStream_t)stream;
  const DType dt = d->dtype == CTN_DTYPE_BF16 ? BF16 : F32;
  const int CN = d->C * d->N;
  const void* sc = x_last;
  if (wm) {
    const void* wmp = wm;
    if (dt == BF16) {
      CTN_HIP(launch_prep_weight(dt, wm, CN, d->B, Ly.wms, nullptr, s));
      wmp = Ly.wms;
    }
    GemmRows g{};
    g.g = Rows{d->M, d->K, d->Kp}; g.Kred = d->B; g.Nout = CN;
    g.A = x_last; g.lda = d->B; g.W = wmp; g.ldw = d->B;
    g.epi = EPI_STORE; g.C = score; g.ldc = CN;
    CTN_HIP(launch_gemm_rows(dt, g, s));
    sc = score;
  }
  CodecArgs a = codec_args(d);
  a.w_rows = const_cast<void*>(w_rows); a.score = sc; a.V = V; a.frames = Ly.frames; a.est = est;
  CTN_HIP(launch_dec_fwd(dt, a, s));
  return CTN_OK;
}

extern "C" int ctn_decoder_backward(const ctn_codec_desc* d, const void* x_last, const void* w_rows,
                                    const float* wm, const float* V, const void* score, const float* g_est,
                                    void* g_x_last, void* g_w_rows, float* gwm, float* gV, void* ws,
                                    size_t ws_bytes, void* stream) {
  int rc = codec_check(d, wm != nullptr);
  if (rc) return rc;
  if (!x_last || !w_rows || !V || !g_est || !g_x_last || !g_w_rows || !gV) return fail(CTN_ERR_ARG, "null pointer");
  if ((wm == nullptr) != (d->mask_type == CTN_MASK_IDENTITY))
    return fail(CTN_ERR_ARG, "wm == NULL exactly when mask_type == CTN_MASK_IDENTITY (standalone Decoder)");
  if (wm && (!score || !gwm)) return fail(CTN_ERR_ARG, "score and gwm required with the mask conv");
  const DecLayout Ly = dec_layout(d, 1, wm != nullptr, ws);
  if (!ws || ws_bytes < Ly.bytes) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, Ly.bytes);
  hipStream_t s = (hipStream_t)stream;
  const DType dt = d->dtype == CTN_DTYPE_BF16 ? BF16 : F32;
  const Rows rg{d->M, d->K, d->Kp};
  const int CN = d->C * d->N;
  CodecArgs a = codec_args(d);
  a.w_rows = const_cast<void*>(w_rows); a.score = wm ? score : x_last; a.V = V; a.gest = g_est;
  a.gscore = wm ? Ly.gscore : g_x_last; a.gwdec_out = g_w_rows;
  const bool cols = Ly.srcb != nullptr;
  if (cols) { a.src_out = Ly.srcb; a.gfr_out = Ly.gfr; a.Lp = Ly.Lp; }
  CTN_HIP(launch_dec_bwd(dt, a, s));
  SlabBatch sb{};
  if (cols) {
    CTN_HIP(launch_dec_gframes(a, s));
    GemmCols gv = dv_gemm(d, Ly.Lp);
    gv.A = Ly.gfr; gv.lda = Ly.Lp; gv.B = Ly.srcb; gv.ldb = d->N;
    gv.Cpart = Ly.cpartV; gv.nchunks = Ly.chunksV;
    CTN_HIP(launch_gemm_cols(dt, gv, s));
    // [chunk][Lp][N] partials: the first L rows of each are dV [L][N]
    sb.d[sb.nd++] = SlabDesc{Ly.cpartV, gV, Ly.chunksV, d->N * d->L, Ly.Lp * d->N};
  } else {
    CodecArgs fo = a;
    fo.col_slab = Ly.slabV;
    CTN_HIP(launch_frame_outer(dt, 1, fo, s));
    sb.d[sb.nd++] = SlabDesc{Ly.slabV, gV, Ly.nV, d->N * d->L, d->N * d->L};
  }
  if (wm) {
    CTN_HIP(launch_prep_weight(dt, wm, CN, d->B, nullptr, Ly.wmt, s));   // [B][CN]
    GemmRows g{};
    g.g = rg; g.Kred = CN; g.Nout = d->B;
    g.A = Ly.gscore; g.lda = CN; g.W = Ly.wmt; g.ldw = CN;
    g.epi = EPI_STORE; g.C = g_x_last; g.ldc = d->B;
    CTN_HIP(launch_gemm_rows(dt, g, s));
    GemmCols gc{};
    gc.g = rg; gc.P = CN; gc.Q = d->B;
    gc.A = Ly.gscore; gc.lda = CN; gc.B = x_last; gc.ldb = d->B;
    gc.Cpart = Ly.cpartM; gc.nchunks = Ly.chunksM;
    CTN_HIP(launch_gemm_cols(dt, gc, s));
    sb.d[sb.nd++] = SlabDesc{Ly.cpartM, gwm, Ly.chunksM, CN * d->B, CN * d->B};
  }
  CTN_HIP(launch_slab_reduce(sb, Ly.srtmp, s));
  return CTN_OK;
}

// ===========================================================================
// PIT SI-SNR loss
// ===========================================================================
static int pit_chunks(int T) {
  int c = (T + 2047) / 2048;
  return c < 1 ? 1 : (c > 64 ? 64 : c);
}

constexpr int PIT_CMAX = 16;   // C <= 10: all C! permutations; 11..16: assignment (ctn_pit.hip)

static void pit_perms(PitArgs& a) {
  int p[4] = {0, 1, 2, 3};
  a.nperm = 0;
  if (a.C > 4) return;          // pit_final_wide decodes them on the device
  // lexicographic order == itertools.permutations(range(C)) (pit_criterion.py:66)
  do {
    for (int i = 0; i < a.C; ++i) a.perms[a.nperm][i] = p[i];
    ++a.nperm;
    int i = a.C - 2;
    while (i >= 0 && p[i] >= p[i + 1]) --i;
    if (i < 0) break;
    int j = a.C - 1;
    while (p[j] <= p[i]) --j;
    int t = p[i]; p[i] = p[j]; p[j] = t;
    for (int l = i + 1, r = a.C - 1; l < r; ++l, --r) { t = p[l]; p[l] = p[r]; p[r] = t; }
  } while (true);
}

extern "C" size_t ctn_pit_workspace_bytes(const ctn_pit_desc* d) {
  if (!d || d->M < 1 || d->C < 1 || d->C > PIT_CMAX || d->T < 1) return 0;
  return (size_t)d->M * pit_chunks(d->T) * pit_nv(d->C) * sizeof(double) + (size_t)d->M * sizeof(double) + 256;
}

extern "C" int ctn_pit_forward(const ctn_pit_desc* d, const float* source, float* est, const int64_t* lengths,
                               float* loss, float* max_snr, int64_t* best_perm, float* reordered, float* coef,
                               void* ws, size_t ws_bytes, void* stream) {
  if (!d || d->M < 1 || d->C < 1 || d->T < 1) return fail(CTN_ERR_ARG, "bad PIT descriptor");
  if (d->C > PIT_CMAX) return fail(CTN_ERR_UNSUPPORTED, "C=%d > %d speakers", d->C, PIT_CMAX);
  if (!source || !est || !lengths || !loss || !max_snr || !best_perm || !coef) return fail(CTN_ERR_ARG, "null pointer");
  if (!ws || ws_bytes < ctn_pit_workspace_bytes(d)) return fail(CTN_ERR_WORKSPACE, "PIT workspace too small");
  PitArgs a{};
  a.M = d->M; a.C = d->C; a.T = d->T;
  a.src = source; a.est = est; a.lengths = lengths;
  a.slab = reinterpret_cast<double*>(ws);
  a.chunks = pit_chunks(d->T);
  a.msd = a.slab + (size_t)d->M * a.chunks * pit_nv(d->C);
  a.max_snr = max_snr; a.best = best_perm; a.coef = coef; a.loss = loss;
  a.est_inplace = est; a.reordered = reordered;
  pit_perms(a);
  CTN_HIP(launch_pit_forward(a, (hipStream_t)stream));
  return CTN_OK;
}

extern "C" int ctn_pit_backward(const ctn_pit_desc* d, const float* source, const float* est,
                                const int64_t* lengths, const float* coef, const float* g_loss,
                                const float* g_max_snr, float* g_est, void* stream) {
  if (!d || d->M < 1 || d->C < 1 || d->T < 1) return fail(CTN_ERR_ARG, "bad PIT descriptor");
  if (d->C > PIT_CMAX) return fail(CTN_ERR_UNSUPPORTED, "C=%d > %d speakers", d->C, PIT_CMAX);
  if (!source || !est || !lengths || !coef || !g_est) return fail(CTN_ERR_ARG, "null pointer");
  PitArgs a{};
  a.M = d->M; a.C = d->C; a.T = d->T;
  a.src = source; a.est = est; a.lengths = lengths; a.coef = const_cast<float*>(coef);
  a.g_loss = g_loss; a.g_maxsnr = g_max_snr; a.gest = g_est;
  CTN_HIP(launch_pit_backward(a, (hipStream_t)stream));
  return CTN_OK;
}

// ===========================================================================
// Parameter update (clip_grad_norm_ + Adam), ctn_optim.hip
// ===========================================================================
static_assert(sizeof(ctn_opt_segment) == sizeof(OptSegment), "segment layout");
static_assert(sizeof(ctn_opt_chunk) == sizeof(OptChunk), "chunk layout");

extern "C" int ctn_opt_plan(const ctn_opt_segment* segs, int nseg, ctn_opt_chunk* chunks, int max_chunks) {
  if (!segs || nseg < 0) return -fail(CTN_ERR_ARG, "ctn_opt_plan: bad segment table");
  long total = 0;
  for (int i = 0; i < nseg; ++i) {
    const ctn_opt_segment& g = segs[i];
    if (g.numel < 0 || !g.grad) return -fail(CTN_ERR_ARG, "ctn_opt_plan: segment %d has no grad or numel < 0", i);
    const uintptr_t ptrs[4] = {(uintptr_t)g.param, (uintptr_t)g.grad, (uintptr_t)g.exp_avg, (uintptr_t)g.exp_avg_sq};
    bool aligned = true;
    for (uintptr_t q : ptrs) aligned = aligned && (q % 16 == 0);
    for (int64_t off = 0; off < g.numel; off += OPT_CHUNK) {
      const int64_t len = g.numel - off < OPT_CHUNK ? g.numel - off : OPT_CHUNK;
      if (chunks && total < max_chunks)
        chunks[total] = ctn_opt_chunk{i, (uint32_t)len | (aligned ? 0u : OPT_UNALIGNED), off};
      ++total;
    }
  }
  if (total > INT32_MAX) return -fail(CTN_ERR_ARG, "ctn_opt_plan: too many chunks");
  return (int)total;
}

extern "C" int ctn_grad_clip_norm(const ctn_opt_segment* segs, const ctn_opt_chunk* chunks, int nchunks,
                                  float max_norm, float* total_norm, float* partial, void* stream) {
  if (!segs || !chunks || !partial || nchunks < 0) return fail(CTN_ERR_ARG, "ctn_grad_clip_norm: null table");
  const hipStream_t s = (hipStream_t)stream;
  const OptSegment* sg = reinterpret_cast<const OptSegment*>(segs);
  const OptChunk* ch = reinterpret_cast<const OptChunk*>(chunks);
  CTN_HIP(launch_grad_sqnorm(sg, ch, nchunks, partial, s));
  CTN_HIP(launch_grad_clip(sg, ch, nchunks, partial, max_norm, total_norm, s));
  return CTN_OK;
}

extern "C" int ctn_adam_step(const ctn_opt_segment* segs, const ctn_opt_chunk* chunks, int nchunks,
                             const ctn_adam_hparams* hp, void* stream) {
  if (!segs || !chunks || !hp || nchunks < 0 || hp->step < 1)
    return fail(CTN_ERR_ARG, "ctn_adam_step: bad arguments");
  // bias corrections of step hp->step in fp64 on the device (adam_bias, ctn_optim.hip)
  AdamArgs a{hp->beta1, hp->beta2, hp->eps, hp->weight_decay, hp->lr, hp->step, nullptr, nullptr};
  CTN_HIP(launch_adam(reinterpret_cast<const OptSegment*>(segs), reinterpret_cast<const OptChunk*>(chunks), nchunks,
                      a, (hipStream_t)stream));
  return CTN_OK;
}

extern "C" int ctn_opt_write_segments(ctn_opt_segment* dst, const ctn_opt_segment* src, int n, void* stream) {
  if (!dst || n < 0 || (n > 0 && !src)) return fail(CTN_ERR_ARG, "ctn_opt_write_segments: bad arguments");
  CTN_HIP(launch_write_segments(reinterpret_cast<OptSegment*>(dst), reinterpret_cast<const OptSegment*>(src), n,
                                (hipStream_t)stream));
  return CTN_OK;
}

extern "C" int ctn_adam_step_dev(const ctn_opt_segment* segs, const ctn_opt_chunk* chunks, int nchunks,
                                 const ctn_adam_hparams* hp, const float* lr_dev, int32_t* counter, void* stream) {
  if (!segs || !chunks || !hp || nchunks < 0 || !counter)
    return fail(CTN_ERR_ARG, "ctn_adam_step_dev: bad arguments");
  AdamArgs a{hp->beta1, hp->beta2, hp->eps, hp->weight_decay, hp->lr, 1, lr_dev, nullptr};
  CTN_HIP(launch_adam_dev(reinterpret_cast<const OptSegment*>(segs), reinterpret_cast<const OptChunk*>(chunks),
                          nchunks, a, counter, (hipStream_t)stream));
  return CTN_OK;
}

// ===========================================================================
// Weight packing (bf16 compute copies for a whole step)
// ===========================================================================
static_assert(sizeof(ctn_weight_pack) == sizeof(PrepDesc), "pack layout");

extern "C" int ctn_pack_weights(const ctn_weight_pack* packs, int n, void* stream) {
  if (n < 0 || (n > 0 && !packs)) return fail(CTN_ERR_ARG, "ctn_pack_weights: bad table");
  for (int i = 0; i < n; ++i) {
    const ctn_weight_pack& w = packs[i];
    if (!w.src || w.rows <= 0 || w.cols <= 0 || (!w.dst && !w.dst_t && !w.dst_frag && !w.dst_t_frag))
      return fail(CTN_ERR_ARG, "ctn_pack_weights: entry %d is empty or has no destination", i);
    if ((w.dst_frag || w.dst_t_frag) && (w.rows % 32 || w.cols % 32))
      return fail(CTN_ERR_ARG, "ctn_pack_weights: entry %d: fragment order needs rows and cols in multiples of 32 "
                  "(%d x %d)", i, w.rows, w.cols);
  }
  for (int i0 = 0; i0 < n; i0 += PREP_MAX) {
    PrepBatch pb{};
    pb.nd = n - i0 < PREP_MAX ? n - i0 : PREP_MAX;
    for (int i = 0; i < pb.nd; ++i) {
      const ctn_weight_pack& w = packs[i0 + i];
      pb.d[i] = PrepDesc{w.src, w.rows, w.cols, w.dst, w.dst_t, w.dst_frag, w.dst_t_frag};
    }
    CTN_HIP(launch_prep_weights(BF16, pb, (hipStream_t)stream));
  }
  return CTN_OK;
}

// ===========================================================================
// Stand-alone separator layers (ctn_layers.hip): the module forwards of
// TemporalConvNet / DepthwiseSeparableConv / the layer norms when called on
// their own, with their backward
// ===========================================================================
namespace {
int rows_check(const ctn_rows_desc* d) {
  if (!d) return fail(CTN_ERR_ARG, "null descriptor");
  if (d->M <= 0 || d->K <= 0 || d->C <= 0) return fail(CTN_ERR_ARG, "M=%d K=%d C=%d", d->M, d->K, d->C);
  if (d->Kp != ctn_padded_frames(d->K)) return fail(CTN_ERR_ARG, "Kp=%d != padded(K)", d->Kp);
  if (d->dtype != CTN_DTYPE_F32 && d->dtype != CTN_DTYPE_BF16) return fail(CTN_ERR_ARG, "dtype %d", d->dtype);
  if ((long)d->M * d->Kp * d->C >= (1L << 31)) return fail(CTN_ERR_UNSUPPORTED, "tensor too large");
  return CTN_OK;
}
Rows rows_of(const ctn_rows_desc* d) { return Rows{d->M, d->K, d->Kp}; }
DType dtype_of(const ctn_rows_desc* d) { return d->dtype == CTN_DTYPE_BF16 ? BF16 : F32; }

struct LnLayout {
  double2* slab; float2* sums; float* part;
  size_t bytes;
};
LnLayout ln_layout(const ctn_rows_desc* d, int norm, int bwd, void* ws) {
  Carver c(ws);
  LnLayout L{};
  const Rows g = rows_of(d);
  const long G = norm == CTN_NORM_GLN ? d->M : g.rows();
  if (norm == CTN_NORM_GLN) L.slab = c.take<double2>((size_t)d->M * layer_norm_groups_nb(g) * sizeof(double2));
  if (bwd) {
    L.sums = c.take<float2>((size_t)G * sizeof(float2));
    L.part = c.take<float>((size_t)layer_blocks(g) * 2 * d->C * sizeof(float));
  }
  L.bytes = c.off + 256;
  return L;
}
int norm_check(int norm) {
  return norm == CTN_NORM_GLN || norm == CTN_NORM_CLN ? CTN_OK
                                                      : fail(CTN_ERR_UNSUPPORTED, "layer norm type %d", norm);
}
}  // namespace

extern "C" size_t ctn_layernorm_workspace_bytes(const ctn_rows_desc* d, int norm_type, int backward) {
  if (rows_check(d) || norm_check(norm_type)) return 0;
  return ln_layout(d, norm_type, backward, nullptr).bytes;
}

extern "C" int ctn_layernorm_forward(const ctn_rows_desc* d, int norm_type, const void* x, const float* gamma,
                                     const float* beta, void* y, float* stats, void* ws, size_t ws_bytes,
                                     void* stream) {
  if (int rc = rows_check(d)) return rc;
  if (int rc = norm_check(norm_type)) return rc;
  if (!x || !gamma || !beta || !y || !stats) return fail(CTN_ERR_ARG, "null pointer");
  const LnLayout L = ln_layout(d, norm_type, 0, ws);
  if (ws_bytes < L.bytes || (!ws && L.slab)) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, L.bytes);
  LayerArgs a{};
  a.g = rows_of(d); a.C = d->C; a.x = x; a.y = y;
  a.norm = norm_type == CTN_NORM_GLN ? NORM_GLN : NORM_CLN; a.eps = (float)kEps;
  a.gamma = gamma; a.beta = beta; a.stats = reinterpret_cast<float2*>(stats); a.slab = L.slab;
  CTN_HIP(launch_layer(dtype_of(d), LAYER_NORM_FWD, a, (hipStream_t)stream));
  return CTN_OK;
}

extern "C" int ctn_layernorm_backward(const ctn_rows_desc* d, int norm_type, const void* x, const float* gamma,
                                      const float* stats, const void* gy, void* gx, float* ggamma, float* gbeta,
                                      void* ws, size_t ws_bytes, void* stream) {
  if (int rc = rows_check(d)) return rc;
  if (int rc = norm_check(norm_type)) return rc;
  if (!x || !gamma || !stats || !gy || !gx || !ggamma || !gbeta) return fail(CTN_ERR_ARG, "null pointer");
  const LnLayout L = ln_layout(d, norm_type, 1, ws);
  if (!ws || ws_bytes < L.bytes) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, L.bytes);
  LayerArgs a{};
  a.g = rows_of(d); a.C = d->C; a.x = x; a.gy = gy; a.gx = gx;
  a.norm = norm_type == CTN_NORM_GLN ? NORM_GLN : NORM_CLN;
  a.gamma = gamma; a.stats = const_cast<float2*>(reinterpret_cast<const float2*>(stats));
  a.sums = L.sums; a.slab = L.slab; a.part = L.part; a.ggamma = ggamma; a.gbeta = gbeta;
  CTN_HIP(launch_layer(dtype_of(d), LAYER_NORM_BWD, a, (hipStream_t)stream));
  return CTN_OK;
}

extern "C" size_t ctn_prelu_workspace_bytes(const ctn_rows_desc* d) {
  if (rows_check(d)) return 0;
  return (size_t)layer_blocks(rows_of(d)) * sizeof(float) + 256;
}

extern "C" int ctn_prelu_forward(const ctn_rows_desc* d, const void* x, const float* alpha, void* y, void* stream) {
  if (int rc = rows_check(d)) return rc;
  if (!x || !alpha || !y) return fail(CTN_ERR_ARG, "null pointer");
  LayerArgs a{};
  a.g = rows_of(d); a.C = d->C; a.x = x; a.y = y; a.alpha = alpha;
  CTN_HIP(launch_layer(dtype_of(d), LAYER_PRELU_FWD, a, (hipStream_t)stream));
  return CTN_OK;
}

extern "C" int ctn_prelu_backward(const ctn_rows_desc* d, const void* x, const float* alpha, const void* gy, void* gx,
                                  float* galpha, void* ws, size_t ws_bytes, void* stream) {
  if (int rc = rows_check(d)) return rc;
  if (!x || !alpha || !gy || !gx || !galpha) return fail(CTN_ERR_ARG, "null pointer");
  if (!ws || ws_bytes < ctn_prelu_workspace_bytes(d)) return fail(CTN_ERR_WORKSPACE, "workspace too small");
  LayerArgs a{};
  a.g = rows_of(d); a.C = d->C; a.x = x; a.gy = gy; a.gx = gx; a.alpha = alpha; a.galpha = galpha;
  a.part = reinterpret_cast<float*>(ws);
  CTN_HIP(launch_layer(dtype_of(d), LAYER_PRELU_BWD, a, (hipStream_t)stream));
  return CTN_OK;
}

namespace {
// reference padding (conv_tasnet.py:188): (P-1)*d both sides, the causal copy chomped on
// the right (Chomp1d) -> left pad (P-1)*d; otherwise (P-1)*d//2 both sides, output length
// K only when (P-1)*d is even
int dw_check(const ctn_rows_desc* d, int P, int dil, int causal, int* pad) {
  if (P < 1 || P > 64 || dil < 1) return fail(CTN_ERR_ARG, "P=%d dilation=%d", P, dil);
  if (causal) {
    *pad = (P - 1) * dil;
  } else {
    if (((P - 1) * dil) % 2) return fail(CTN_ERR_UNSUPPORTED, "non-causal (P-1)*dilation odd: output length != K");
    *pad = (P - 1) * dil / 2;
  }
  return CTN_OK;
}
}  // namespace

extern "C" size_t ctn_depthwise_workspace_bytes(const ctn_rows_desc* d, int P) {
  if (rows_check(d) || P < 1) return 0;
  return (size_t)layer_blocks(rows_of(d)) * d->C * P * sizeof(float) + 256;
}

extern "C" int ctn_depthwise_forward(const ctn_rows_desc* d, int P, int dilation, int causal, const void* x,
                                     const float* w, void* y, void* stream) {
  if (int rc = rows_check(d)) return rc;
  int pad = 0;
  if (int rc = dw_check(d, P, dilation, causal, &pad)) return rc;
  if (!x || !w || !y) return fail(CTN_ERR_ARG, "null pointer");
  LayerArgs a{};
  a.g = rows_of(d); a.C = d->C; a.x = x; a.y = y; a.P = P; a.dil = dilation; a.pad = pad; a.w = w;
  CTN_HIP(launch_layer(dtype_of(d), LAYER_DW_FWD, a, (hipStream_t)stream));
  return CTN_OK;
}

extern "C" int ctn_depthwise_backward(const ctn_rows_desc* d, int P, int dilation, int causal, const void* x,
                                      const float* w, const void* gy, void* gx, float* gw, void* ws, size_t ws_bytes,
                                      void* stream) {
  if (int rc = rows_check(d)) return rc;
  int pad = 0;
  if (int rc = dw_check(d, P, dilation, causal, &pad)) return rc;
  if (!x || !w || !gy || !gx || !gw) return fail(CTN_ERR_ARG, "null pointer");
  if (!ws || ws_bytes < ctn_depthwise_workspace_bytes(d, P)) return fail(CTN_ERR_WORKSPACE, "workspace too small");
  LayerArgs a{};
  a.g = rows_of(d); a.C = d->C; a.x = x; a.gy = gy; a.gx = gx; a.P = P; a.dil = dilation; a.pad = pad;
  a.w = w; a.gw = gw; a.part = reinterpret_cast<float*>(ws);
  CTN_HIP(launch_layer(dtype_of(d), LAYER_DW_BWD, a, (hipStream_t)stream));
  return CTN_OK;
}

namespace {
struct C1Layout {
  void* ws_w; void* ws_wt; float* cpart;
  int chunks;
  size_t bytes;
};
GemmCols c1_cols(const ctn_rows_desc* d, int cout) {
  GemmCols gc{};
  gc.g = rows_of(d); gc.P = cout; gc.Q = d->C;
  return gc;
}
C1Layout c1_layout(const ctn_rows_desc* d, int cout, int bwd, void* ws) {
  Carver c(ws);
  C1Layout L{};
  const size_t es = esize(d->dtype);
  if (!bwd) {
    if (d->dtype == CTN_DTYPE_BF16) L.ws_w = c.take<void>((size_t)cout * d->C * es);
  } else {
    L.ws_wt = c.take<void>((size_t)cout * d->C * es);
    L.chunks = gemm_cols_chunks(d->dtype == CTN_DTYPE_BF16 ? BF16 : F32, c1_cols(d, cout));
    L.cpart = c.take<float>((size_t)L.chunks * cout * d->C * sizeof(float));
  }
  L.bytes = c.off + 256;
  return L;
}
int c1_check(const ctn_rows_desc* d, int cout) {
  if (cout <= 0 || cout % 8 || d->C % 8) return fail(CTN_ERR_UNSUPPORTED, "1x1 conv %d -> %d: channels must be multiples of 8", d->C, cout);
  return CTN_OK;
}
}  // namespace

extern "C" size_t ctn_conv1x1_workspace_bytes(const ctn_rows_desc* d, int cout, int backward) {
  if (rows_check(d) || c1_check(d, cout)) return 0;
  return c1_layout(d, cout, backward, nullptr).bytes;
}

extern "C" int ctn_conv1x1_forward(const ctn_rows_desc* d, int cout, const void* x, const float* w, void* y, void* ws,
                                   size_t ws_bytes, void* stream) {
  if (int rc = rows_check(d)) return rc;
  if (int rc = c1_check(d, cout)) return rc;
  if (!x || !w || !y) return fail(CTN_ERR_ARG, "null pointer");
  const C1Layout L = c1_layout(d, cout, 0, ws);
  if (ws_bytes < L.bytes || (!ws && L.ws_w)) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, L.bytes);
  hipStream_t s = (hipStream_t)stream;
  const DType dt = dtype_of(d);
  const void* wst = w;
  if (dt == BF16) {
    CTN_HIP(launch_prep_weight(dt, w, cout, d->C, L.ws_w, nullptr, s));
    wst = L.ws_w;
  }
  GemmRows g{};
  g.g = rows_of(d); g.Kred = d->C; g.Nout = cout;
  g.A = x; g.lda = d->C; g.W = wst; g.ldw = d->C;
  g.epi = EPI_STORE; g.C = y; g.ldc = cout;
  CTN_HIP(launch_gemm_rows(dt, g, s));
  return CTN_OK;
}

extern "C" int ctn_conv1x1_backward(const ctn_rows_desc* d, int cout, const void* x, const float* w, const void* gy,
                                    void* gx, float* gw, void* ws, size_t ws_bytes, void* stream) {
  if (int rc = rows_check(d)) return rc;
  if (int rc = c1_check(d, cout)) return rc;
  if (!x || !w || !gy || !gx || !gw) return fail(CTN_ERR_ARG, "null pointer");
  const C1Layout L = c1_layout(d, cout, 1, ws);
  if (!ws || ws_bytes < L.bytes) return fail(CTN_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, L.bytes);
  hipStream_t s = (hipStream_t)stream;
  const DType dt = dtype_of(d);
  CTN_HIP(launch_prep_weight(dt, w, cout, d->C, nullptr, L.ws_wt, s));   // [C][cout]
  GemmRows g{};
  g.g = rows_of(d); g.Kred = cout; g.Nout = d->C;
  g.A = gy; g.lda = cout; g.W = L.ws_wt; g.ldw = cout;
  g.epi = EPI_STORE; g.C = gx; g.ldc = d->C;
  CTN_HIP(launch_gemm_rows(dt, g, s));
  GemmCols gc = c1_cols(d, cout);
  gc.A = gy; gc.lda = cout; gc.B = x; gc.ldb = d->C;
  gc.Cpart = L.cpart; gc.nchunks = L.chunks;
  CTN_HIP(launch_gemm_cols(dt, gc, s));
  SlabBatch sb{};
  sb.d[sb.nd++] = SlabDesc{L.cpart, gw, L.chunks, cout * d->C, cout * d->C};
  CTN_HIP(launch_slab_reduce(sb, nullptr, s));
  return CTN_OK;
}

namespace {
int mask_check(const ctn_rows_desc* d, int nspk, int mask_type) {
  if (nspk < 1 || d->C % nspk) return fail(CTN_ERR_ARG, "C=%d not a multiple of nspk=%d", d->C, nspk);
  if (mask_type != CTN_MASK_RELU && mask_type != CTN_MASK_SOFTMAX) return fail(CTN_ERR_ARG, "mask type %d", mask_type);
  return CTN_OK;
}
}  // namespace

extern "C" int ctn_mask_forward(const ctn_rows_desc* d, int nspk, int mask_type, const void* score, void* mask,
                                void* stream) {
  if (int rc = rows_check(d)) return rc;
  if (int rc = mask_check(d, nspk, mask_type)) return rc;
  if (!score || !mask) return fail(CTN_ERR_ARG, "null pointer");
  LayerArgs a{};
  a.g = rows_of(d); a.C = d->C; a.x = score; a.y = mask; a.S = nspk; a.mask_type = mask_type;
  CTN_HIP(launch_layer(dtype_of(d), LAYER_MASK_FWD, a, (hipStream_t)stream));
  return CTN_OK;
}

extern "C" int ctn_mask_backward(const ctn_rows_desc* d, int nspk, int mask_type, const void* score, const void* gmask,
                                 void* gscore, void* stream) {
  if (int rc = rows_check(d)) return rc;
  if (int rc = mask_check(d, nspk, mask_type)) return rc;
  if (!score || !gmask || !gscore) return fail(CTN_ERR_ARG, "null pointer");
  LayerArgs a{};
  a.g = rows_of(d); a.C = d->C; a.x = score; a.gy = gmask; a.gx = gscore; a.S = nspk; a.mask_type = mask_type;
  CTN_HIP(launch_layer(dtype_of(d), LAYER_MASK_BWD, a, (hipStream_t)stream));
  return CTN_OK;
}

// ===========================================================================
// Streaming causal separation (ctn_stream.hip)
// ===========================================================================
namespace {
int stream_check(const ctn_stream_desc* d) {
  if (!d) return fail(CTN_ERR_ARG, "null descriptor");
  if (d->M < 1 || d->K < 1) return fail(CTN_ERR_ARG, "M=%d K=%d", d->M, d->K);
  if (d->L < 2 || d->L % 2 || d->L > 64) return fail(CTN_ERR_UNSUPPORTED, "L=%d (even, <= 64)", d->L);
  if (d->N < 1 || d->B < 1 || d->H < 1 || d->P < 1 || d->P > 8 || d->C < 1 || d->C > 8)
    return fail(CTN_ERR_ARG, "N=%d B=%d H=%d P=%d C=%d", d->N, d->B, d->H, d->P, d->C);
  if (d->norm != CTN_NORM_CLN && d->norm != CTN_NORM_BN)
    return fail(CTN_ERR_UNSUPPORTED, "norm %d: gLN normalizes over the whole utterance and cannot stream", d->norm);
  if (d->mask_type < 0 || d->mask_type > 2) return fail(CTN_ERR_ARG, "mask type %d", d->mask_type);
  return CTN_OK;
}
StreamArgs stream_args(const ctn_stream_desc* d) {
  StreamArgs a{};
  a.M = d->M; a.K = d->K; a.N = d->N; a.L = d->L; a.B = d->B; a.H = d->H; a.P = d->P; a.C = d->C;
  a.norm = d->norm == CTN_NORM_CLN ? 1 : 2;
  a.mask_type = d->mask_type;
  return a;
}
}  // namespace

extern "C" int ctn_stream_encode(const ctn_stream_desc* d, const float* samples, int64_t ld_samples, const float* U,
                                 const float* gamma0, const float* beta0, const float* wb_t, float* w_out,
                                 float* x_out, void* stream) {
  if (int rc = stream_check(d)) return rc;
  if (!samples || !U || !gamma0 || !beta0 || !wb_t || !w_out || !x_out) return fail(CTN_ERR_ARG, "null pointer");
  if (ld_samples < (int64_t)(d->K - 1) * (d->L / 2) + d->L) return fail(CTN_ERR_ARG, "ld_samples too small");
  StreamArgs a = stream_args(d);
  a.samples = samples; a.ld_samples = ld_samples; a.U = U; a.na = gamma0; a.nb = beta0; a.W = wb_t;
  a.w_out = w_out; a.x_out = x_out;
  CTN_HIP(launch_stream(0, a, (hipStream_t)stream));
  return CTN_OK;
}

extern "C" int ctn_stream_block(const ctn_stream_desc* d, int dilation, int64_t pos, int ring_frames,
                                const float* x_in, const float* w1_t, const float* alpha1, const float* norm1_a,
                                const float* norm1_b, const float* wd, const float* alpha2, const float* norm2_a,
                                const float* norm2_b, const float* w2_t, float* ring, float* x_out, void* stream) {
  if (int rc = stream_check(d)) return rc;
  if (dilation < 1 || pos < 0) return fail(CTN_ERR_ARG, "dilation %d, pos %lld", dilation, (long long)pos);
  if (ring_frames < 1 || (ring_frames & (ring_frames - 1)) || ring_frames < (d->P - 1) * dilation + d->K)
    return fail(CTN_ERR_ARG, "ring_frames %d: a power of two >= (P-1)*dilation + K = %d", ring_frames,
                (d->P - 1) * dilation + d->K);
  if (!x_in || !w1_t || !alpha1 || !norm1_a || !norm1_b || !wd || !alpha2 || !norm2_a || !norm2_b || !w2_t || !ring ||
      !x_out)
    return fail(CTN_ERR_ARG, "null pointer");
  if (x_in == x_out) return fail(CTN_ERR_ARG, "x_out must not alias x_in (the residual is read per frame)");
  StreamArgs a = stream_args(d);
  a.dil = dilation; a.pos = pos; a.R = ring_frames; a.x_in = x_in; a.ring = ring;
  a.W = w1_t; a.alpha1 = alpha1; a.na = norm1_a; a.nb = norm1_b;
  CTN_HIP(launch_stream(1, a, (hipStream_t)stream));
  a.W = w2_t; a.alpha2 = alpha2; a.na = norm2_a; a.nb = norm2_b; a.wd = wd; a.x_out = x_out;
  CTN_HIP(launch_stream(2, a, (hipStream_t)stream));
  return CTN_OK;
}

extern "C" int ctn_stream_decode(const ctn_stream_desc* d, const float* x_last, const float* w, const float* wm_t,
                                 const float* V, const float* tail_in, float* tail_out, float* frames_ws, float* out,
                                 void* stream) {
  if (int rc = stream_check(d)) return rc;
  if (!x_last || !w || !wm_t || !V || !tail_in || !tail_out || !frames_ws || !out) return fail(CTN_ERR_ARG, "null pointer");
  if (tail_in == tail_out) return fail(CTN_ERR_ARG, "tail_out must not alias tail_in");
  StreamArgs a = stream_args(d);
  a.x_in = x_last; a.w_in = w; a.W = wm_t; a.V = V; a.tail_in = tail_in; a.tail_out = tail_out;
  a.frames = frames_ws; a.out = out;
  CTN_HIP(launch_stream(3, a, (hipStream_t)stream));
  return CTN_OK;
}

// ABI v7: one whole streaming call (ctn_stream.hip, launch_stream_call_stage)
namespace {
size_t stream_ws_floats(const ctn_stream_desc* d) {
  const size_t M = d->M, K = d->K;
  return M * K * d->N + 2 * M * K * d->B + M * K * (size_t)(d->H > d->C * d->N ? d->H : d->C * d->N);
}
// the replayed graph's pos slot: 16-byte aligned, inside the workspace's 256-byte tail
long* stream_pos_slot(const ctn_stream_desc* d, void* ws) {
  const size_t off = (stream_ws_floats(d) * sizeof(float) + 15) / 16 * 16;
  return reinterpret_cast<long*>(reinterpret_cast<char*>(ws) + off);
}
// CTN_STREAM_GRAPH=0: launch the stages directly on every call (A/B only)
bool stream_graph_enabled() {
  const char* e = getenv("CTN_STREAM_GRAPH");
  return e ? atoi(e) != 0 : true;
}
struct StreamGraph {
  std::vector<uintptr_t> key;
  hipGraphExec_t exec;
  hipEvent_t done;   // recorded after every launch of exec (launches of one exec are ordered)
};
std::mutex g_sg_mu;
std::vector<StreamGraph> g_sg;   // most recently stored last; at most 8
// Finds (or builds with `build`) the graph of `key` and launches it on s behind a
// pos store, all under the cache lock, so no other thread can evict the graph between
// the lookup and the launch.  An evicted graph is destroyed after the lock is released,
// once its own last launch has finished (its event): no device-wide synchronisation,
// nothing that would stall other streams or invalidate another thread's capture.
template <typename Build>
hipError_t stream_graph_launch(const std::vector<uintptr_t>& key, Build build, long* pos_dev, long pos, hipStream_t s) {
  StreamGraph victim{{}, nullptr, nullptr};
  hipError_t e = hipSuccess;
  {
    std::lock_guard<std::mutex> lk(g_sg_mu);
    StreamGraph* g = nullptr;
    for (StreamGraph& x : g_sg)
      if (x.key == key) g = &x;
    if (!g) {
      hipGraphExec_t exec = nullptr;
      hipEvent_t ev = nullptr;
      e = build(&exec);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
      if (e != hipSuccess) {
        if (exec) (void)hipGraphExecDestroy(exec);
        return e;
      }
      if (g_sg.size() == 8) {
        victim = g_sg.front();
        g_sg.erase(g_sg.begin());
      }
      g_sg.push_back(StreamGraph{key, exec, ev});
      g = &g_sg.back();
    }
    e = launch_stream_set_pos(pos_dev, pos, s);
    if (e == hipSuccess) e = hipGraphLaunch(g->exec, s);
    if (e == hipSuccess) e = hipEventRecord(g->done, s);
  }
  if (victim.exec) {   // a ninth distinct argument set (rare)
    (void)hipEventSynchronize(victim.done);
    (void)hipGraphExecDestroy(victim.exec);
    (void)hipEventDestroy(victim.done);
  }
  return e;
}
}  // namespace

extern "C" size_t ctn_stream_workspace_bytes(const ctn_stream_desc* d) {
  if (stream_check(d)) return 0;
  return stream_ws_floats(d) * sizeof(float) + 256;
}

extern "C" int ctn_stream_call(const ctn_stream_desc* d, const ctn_stream_model* mdl, int64_t pos, const float* samples,
                               int64_t ld_samples, const float* tail_in, float* tail_out, float* out, void* ws,
                               size_t ws_bytes, void* stream) {
  if (int rc = stream_check(d)) return rc;
  if (!mdl || !samples || !tail_in || !tail_out || !out || !ws) return fail(CTN_ERR_ARG, "null pointer");
  if (!mdl->U || !mdl->gamma0 || !mdl->beta0 || !mdl->wb_t || !mdl->wm_t || !mdl->V || (mdl->nblocks && !mdl->blocks))
    return fail(CTN_ERR_ARG, "null model pointer");
  if (mdl->nblocks < 0) return fail(CTN_ERR_ARG, "nblocks %d", mdl->nblocks);
  if (pos < 0) return fail(CTN_ERR_ARG, "pos %lld", (long long)pos);
  if (tail_in == tail_out) return fail(CTN_ERR_ARG, "tail_out must not alias tail_in");
  if (ld_samples < (int64_t)(d->K - 1) * (d->L / 2) + d->L) return fail(CTN_ERR_ARG, "ld_samples too small");
  if (ws_bytes < ctn_stream_workspace_bytes(d)) return fail(CTN_ERR_ARG, "workspace too small");
  for (int i = 0; i < mdl->nblocks; ++i) {
    const ctn_stream_block_params& b = mdl->blocks[i];
    if (b.dilation < 1 || b.ring_frames < 1 || (b.ring_frames & (b.ring_frames - 1)) ||
        b.ring_frames < (d->P - 1) * b.dilation + d->K)
      return fail(CTN_ERR_ARG, "block %d: dilation %d, ring_frames %d (a power of two >= (P-1)*dilation + K)", i,
                  b.dilation, b.ring_frames);
    if (!b.w1_t || !b.alpha1 || !b.norm1_a || !b.norm1_b || !b.wd || !b.alpha2 || !b.norm2_a || !b.norm2_b ||
        !b.w2_t || !b.ring)
      return fail(CTN_ERR_ARG, "block %d: null pointer", i);
  }
  const hipStream_t s = (hipStream_t)stream;
  long* pos_dev = stream_pos_slot(d, ws);
  // the launch sequence, parameterised by where `pos` comes from
  auto enqueue = [&](hipStream_t q, const long* pd) -> hipError_t {
    const size_t M = d->M, K = d->K;
    float* w = reinterpret_cast<float*>(ws);
    float* xa = w + M * K * d->N;
    float* xb = xa + M * K * d->B;
    float* scratch = xb + M * K * d->B;   // h1 of a block / the sources
    StreamArgs a = stream_args(d);
    a.pos = pos; a.pos_dev = pd;
    a.samples = samples; a.ld_samples = ld_samples; a.U = mdl->U; a.na = mdl->gamma0; a.nb = mdl->beta0;
    a.W = mdl->wb_t; a.w_out = w; a.x_out = xa;
    hipError_t e = launch_stream_call_stage(0, a, q);
    float* x = xa;
    float* y = xb;
    for (int i = 0; e == hipSuccess && i < mdl->nblocks; ++i) {
      const ctn_stream_block_params& b = mdl->blocks[i];
      StreamArgs ab = stream_args(d);
      ab.pos = pos; ab.pos_dev = pd; ab.dil = b.dilation; ab.R = b.ring_frames; ab.ring = b.ring;
      ab.x_in = x; ab.x_out = y; ab.frames = scratch;
      ab.W = b.w1_t; ab.alpha1 = b.alpha1; ab.na = b.norm1_a; ab.nb = b.norm1_b;
      ab.wd = b.wd; ab.alpha2 = b.alpha2; ab.na2 = b.norm2_a; ab.nb2 = b.norm2_b; ab.W2 = b.w2_t;
      e = launch_stream_call_stage(1, ab, q);
      if (e == hipSuccess) e = launch_stream_call_stage(2, ab, q);
      float* t = x; x = y; y = t;
    }
    StreamArgs ad = stream_args(d);
    ad.x_in = x; ad.w_in = w; ad.W = mdl->wm_t; ad.V = mdl->V; ad.frames = scratch;
    ad.tail_in = tail_in; ad.tail_out = tail_out; ad.out = out;
    if (e == hipSuccess) e = launch_stream_call_stage(3, ad, q);
    if (e == hipSuccess) e = launch_stream_call_stage(4, ad, q);
    return e;
  };
  if (!stream_graph_enabled()) {
    CTN_HIP(enqueue(s, nullptr));
    return CTN_OK;
  }
  // Graph replay: the 4 + 2 X R launches of a call are captured once per argument set
  // (everything but pos, which the replay reads from the workspace) and replayed with
  // one graph launch after a one-thread kernel stores pos.
  std::vector<uintptr_t> key;
  int dev = 0;
  CTN_HIP(hipGetDevice(&dev));
  key.push_back((uintptr_t)dev);
  for (const int v : {d->M, d->K, d->N, d->L, d->B, d->H, d->P, d->C, d->norm, d->mask_type}) key.push_back((uintptr_t)(unsigned)v);
  for (const void* v : {(const void*)mdl->U, (const void*)mdl->gamma0, (const void*)mdl->beta0, (const void*)mdl->wb_t,
                        (const void*)mdl->wm_t, (const void*)mdl->V, (const void*)samples, (const void*)tail_in,
                        (const void*)tail_out, (const void*)out, (const void*)ws})
    key.push_back((uintptr_t)v);
  key.push_back((uintptr_t)ld_samples);
  for (int i = 0; i < mdl->nblocks; ++i) {
    const ctn_stream_block_params& b = mdl->blocks[i];
    key.push_back((uintptr_t)(unsigned)b.dilation);
    key.push_back((uintptr_t)(unsigned)b.ring_frames);
    for (const void* v : {(const void*)b.w1_t, (const void*)b.alpha1, (const void*)b.norm1_a, (const void*)b.norm1_b,
                          (const void*)b.wd, (const void*)b.alpha2, (const void*)b.norm2_a, (const void*)b.norm2_b,
                          (const void*)b.w2_t, (const void*)b.ring})
      key.push_back((uintptr_t)v);
  }
  auto build = [&](hipGraphExec_t* exec) -> hipError_t {
    hipStream_t cs = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
    if (e != hipSuccess) return e;
    hipGraph_t g = nullptr;
    e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
    if (e == hipSuccess) {
      const hipError_t el = enqueue(cs, pos_dev);
      e = hipStreamEndCapture(cs, &g);
      if (el != hipSuccess) e = el;
    }
    if (e == hipSuccess) e = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
    if (g) (void)hipGraphDestroy(g);
    (void)hipStreamDestroy(cs);
    return e;
  };
  CTN_HIP(stream_graph_launch(key, build, pos_dev, (long)pos, s));
  return CTN_OK;
}
