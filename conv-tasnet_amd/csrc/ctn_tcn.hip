// Element-wise / depthwise kernels of the TemporalBlock (conv_tasnet.py:212-272)
// and the statistics plumbing shared by all kernels (gfx950).
//
// dw_fwd    : n1 = norm1(PReLU(h1)) recomputed on the fly, depthwise dilated
//             conv (causal = left pad only, identical to pad + Chomp1d,
//             conv_tasnet.py:176,247-260,289), stores d (pre-PReLU) and the
//             partial statistics of PReLU(d) for norm2.
// dw_bwd    : norm2 backward (element part) -> PReLU2 backward -> transposed
//             depthwise conv -> norm1 backward partial sums; column partials
//             for gamma1/beta1/dw weight/alpha2.
// norm1_bwd : norm1 backward finish -> PReLU1 backward -> dL/dh1.
//
// Thread layout (all three): a workgroup owns 128 frame rows of one utterance
// (Kp % 128 == 0) and all H channels; a thread owns 8 consecutive channels
// (one 16-byte bf16 vector) of every (256 / (H/8))-th row.
#include <vector>

#include "ctn_common.h"
#include "ctn_dw.h"
#include "ctn_kernels.h"

namespace ctn {

#ifndef CTN_DW_PF
#define CTN_DW_PF 2
#endif
// dw_bwd, cLN: per-row statistics of 64 walk steps per lane, broadcast by v_readlane
#ifndef CTN_DW_BATCH
#define CTN_DW_BATCH 1
#endif
constexpr int DW_RPB = 128;   // rows per workgroup (element-wise kernels)
constexpr int DW_MAXP = 8;
constexpr int DW_MINSEG = 16; // shortest comb segment (halo rows cost (P-1)/seg)
constexpr int DW_WPS_FWD = 4, DW_WPS_BWD = 2;   // waves/SIMD the kernels' VGPR budgets allow
// comb rows prefetched per lane: 2 for bf16 (the loop is latency-bound at one row
// in flight: 8 waves x 48 B per lane per CU is half of what Little's law asks at
// 6 TB/s), 1 for fp32 (parity mode; two would exceed the VGPR budgets above)
template <typename T> constexpr int dw_pf() { return sizeof(T) == 2 ? CTN_DW_PF : 1; }

// Segment length such that all work items of the launch are resident at once:
// a wave owns 64/(H/8) items and walks its segment serially, so a second, partly
// filled round of waves would cost a whole segment time.  Items per utterance are
// dil * ceil(jmax/seg); when dil alone exceeds the budget the segment is the
// whole residue class (jmax steps, the shortest possible).
int dw_seg(const DwArgs& a, bool bwd) {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  const long cap = (long)cus * 4 * (bwd ? DW_WPS_BWD : DW_WPS_FWD) * (64 / (a.H / 8));
  const long per_utt = cap / (a.g.M > 0 ? a.g.M : 1);
  const int jmax = (a.g.Kp + a.dil - 1) / a.dil;
  long nseg = per_utt / a.dil;
  if (nseg < 1) nseg = 1;
  int seg = (int)((jmax + nseg - 1) / nseg);
  if (seg < DW_MINSEG) seg = DW_MINSEG;
  return seg;
}
int dw_blocks(const DwArgs& a) { return a.g.M * comb_geom(a).wgpu; }
int dw_parts_per_group(const DwArgs& a) { return a.norm == NORM_GLN ? comb_geom(a).wgpu : 1; }
int ew_blocks(const DwArgs& a) { return (int)(a.g.rows() / DW_RPB); }

template <int NK> CTN_DEV float2 ld_stat(const float2* s, int m, int row) {
  return NK == NORM_GLN ? s[m] : s[row];
}

struct CombItem {
  int m, wgi, rho, j0, j1, base, c, sub;
  bool active;
};
CTN_DEV CombItem comb_item(const DwArgs& a, const CombGeom& gm) {
  CombItem it;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  it.c = lane % gm.cg;
  it.sub = lane / gm.cg;
  it.m = blockIdx.x / gm.wgpu;
  it.wgi = blockIdx.x % gm.wgpu;
  const int id = it.wgi * gm.ipw + wv * (64 / gm.cg) + it.sub;
  it.active = id < gm.items;
  it.rho = it.active ? id / gm.nseg : 0;
  it.j0 = it.active ? (id % gm.nseg) * a.seg : 0;
  it.j1 = it.j0 + a.seg < gm.jmax ? it.j0 + a.seg : gm.jmax;
  if (!it.active) it.j1 = it.j0;
  it.base = it.m * a.g.Kp;
  return it;
}

// ---------------------------------------------------------------------------
// dw_fwd: d[k] = sum_p w[p] n1[k - pad + p*dil],  n1 = norm1(PReLU(h1)) (0 outside [0,K))
// ---------------------------------------------------------------------------
template <typename T, int NK, int P, bool CAUSAL>
__global__ __launch_bounds__(256) void dw_fwd_kernel(DwArgs a) {
  constexpr int POWN = CAUSAL ? P - 1 : (P - 1) / 2;   // tap that reads the output row itself
  __shared__ double red[16];
  const CombGeom gm = comb_geom(a);
  const CombItem it = comb_item(a, gm);
  const int H = a.H, K = a.g.K, Kp = a.g.Kp, dil = a.dil, c = it.c;
  const T* h1 = reinterpret_cast<const T*>(a.h1);
  T* dout = reinterpret_cast<T*>(a.d_out);
  const float al1 = a.alpha1[0], al2 = a.alpha2[0];
  float2 st1u = make_float2(0.f, 0.f);
  if constexpr (NK == NORM_GLN) {
    const StatFold& f = a.f_st1;
    if (f.slab) {
      st1u = fold_stat(f, it.m);
      if (f.out && it.wgi == 0 && threadIdx.x == 0) f.out[it.m] = st1u;   // saved for backward
    } else {
      st1u = a.st1[it.m];
    }
  }

  // per-element arithmetic in channel pairs (f32x2: v_pk_fma/mul/add_f32), as dw_bwd
  f32x2_t w[P][4], g1[4], b1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ch = c * 8 + 2 * i;
    g1[i] = f32x2_t{a.gamma1[ch], a.gamma1[ch + 1]};
    b1[i] = f32x2_t{a.beta1[ch], a.beta1[ch + 1]};
#pragma unroll
    for (int p = 0; p < P; ++p) w[p][i] = f32x2_t{a.wd[ch * P + p], a.wd[(ch + 1) * P + p]};
  }
  auto pr2 = [](f32x2_t x, float al) __attribute__((always_inline)) {
    const f32x2_t ax = x * al;
    return f32x2_t{x[0] > 0.f ? x[0] : ax[0], x[1] > 0.f ? x[1] : ax[1]};
  };
  // window win[i] = n1 at comb step j + (i - POWN), i in [0, P)
  f32x2_t win[P][4];
  auto row_of = [&](int j) { return it.rho + j * dil; };
  // cLN: the row's statistics are fetched with the row (not at the point of use,
  // where the dependent load would stall every comb step)
  auto fetch = [&](int j, Raw8<T>& r, bool& ok, int& row, float2& st) {
    const int k = row_of(j);
    ok = j >= 0 && k < K;
    row = it.base + (ok ? k : 0);
    r.load(h1 + (size_t)row * H + c * 8);
    st = NK == NORM_GLN ? st1u : a.st1[row];
  };
  auto finish = [&](const Raw8<T>& r, bool ok, float2 st, f32x2_t* out) {
    const f32x2_t nm = {-st.x, -st.x};
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // rows outside the utterance: exactly 0 (a select, so a
                                    // non-finite value in the row it fetched cannot leak in)
      const f32x2_t v = pfma((pr2(f32x2_t{r[2 * i], r[2 * i + 1]}, al1) + nm) * st.y, g1[i], b1[i]);
      out[i] = f32x2_t{ok ? v[0] : 0.f, ok ? v[1] : 0.f};
    }
  };
#pragma unroll
  for (int i = 0; i < P - 1; ++i) {           // prologue: steps j0-POWN .. j0+P-2-POWN
    Raw8<T> r; bool ok; int row; float2 st;
    fetch(it.j0 + i - POWN, r, ok, row, st);
    finish(r, ok, st, win[i]);
  }
  // DW_PF rows in flight per lane: slot q holds comb step j with j % DW_PF == q,
  // and the loop is unrolled by DW_PF so a slot is refilled (step j + DW_PF) as
  // soon as it is consumed, without register copies that would wait on a load.
  constexpr int D = dw_pf<T>();
  Raw8<T> pre[D]; bool pok[D]; int prow[D]; float2 pst[D];
#pragma unroll
  for (int q = 0; q < D; ++q) fetch(it.j0 + q + P - 1 - POWN, pre[q], pok[q], prow[q], pst[q]);
  float ts = 0.f, tss = 0.f;
  const bool wave_item = gm.cg == 64;   // one comb item per wave (see RowPark)
  const int lane = threadIdx.x & 63;
  RowPark pk;
  pk.j0 = it.j0;
  // final (mean, rstd) or the (sum, sum sq) slab entry of the rows parked in lanes < n
  auto park_flush = [&](int n) {
    const int k = row_of(pk.j0 + lane);
    if (lane < n && k < Kp) {
      if (a.st2_out) {   // the arithmetic of stats_finalize (mode 0)
        const double mean = (double)pk.s / H;
        double var = (double)pk.ss / H - mean * mean;
        if (var < 0.0) var = 0.0;
        a.st2_out[it.base + k] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)a.eps)));
      } else {
        a.slab2[it.base + k] = make_double2((double)pk.s, (double)pk.ss);
      }
    }
  };
  for (int jb = it.j0; jb < it.j1; jb += D)
#pragma unroll
  for (int q = 0; q < D; ++q) {
    const int j = jb + q;
    if (j >= it.j1) break;
    Raw8<T> cur = pre[q]; const bool cok = pok[q]; const float2 cst = pst[q];
    if (j + D < it.j1) fetch(j + D + P - 1 - POWN, pre[q], pok[q], prow[q], pst[q]);
    finish(cur, cok, cst, win[P - 1]);
    const int k = row_of(j);
    const f32x2_t z2 = {0.f, 0.f};
    f32x2_t o2[4] = {z2, z2, z2, z2};
    float s = 0.f, ss = 0.f;
    if (k < K) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o2[i] = w[0][i] * win[0][i];
#pragma unroll
        for (int p = 1; p < P; ++p) o2[i] = pfma(w[p][i], win[p][i], o2[i]);
        const f32x2_t a2 = pr2(o2[i], al2);
        s += a2[0];   // sums over the 8 channels in channel order
        ss = fmaf(a2[0], a2[0], ss);
        s += a2[1];
        ss = fmaf(a2[1], a2[1], ss);
      }
    }
    if (k < Kp) {
      const float out[8] = {o2[0][0], o2[0][1], o2[1][0], o2[1][1], o2[2][0], o2[2][1], o2[3][0], o2[3][1]};
      Vec8<T>::store(dout + (size_t)(it.base + k) * H + c * 8, out);
    }
    if constexpr (NK == NORM_GLN) {
      ts += s;
      tss += ss;
    } else if (wave_item) {
      s = wave_sum_dpp(s);
      ss = wave_sum_dpp(ss);
      const int pq = j - pk.j0;
      pk.s = lane == pq ? s : pk.s;
      pk.ss = lane == pq ? ss : pk.ss;
      if (pq == 63) {
        park_flush(64);
        pk.j0 = j + 1;
      }
    } else {
      s = wave_sum_group(s, gm.cg);
      ss = wave_sum_group(ss, gm.cg);
      if (c == 0 && k < Kp) {
        if (a.st2_out) {   // final (mean, rstd), the arithmetic of stats_finalize (mode 0)
          const double mean = (double)s / H;
          double var = (double)ss / H - mean * mean;
          if (var < 0.0) var = 0.0;
          a.st2_out[it.base + k] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)a.eps)));
        } else {
          a.slab2[it.base + k] = make_double2((double)s, (double)ss);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < P - 1; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) win[i][e] = win[i + 1][e];
  }
  if constexpr (NK != NORM_GLN)
    if (wave_item && it.j1 > pk.j0) park_flush(it.j1 - pk.j0);
  if constexpr (NK == NORM_GLN) {
    double v2[2] = {(double)ts, (double)tss};
    block_sum_d<2>(v2, red);
    if (threadIdx.x == 0) a.slab2[(size_t)it.m * gm.wgpu + it.wgi] = make_double2(v2[0], v2[1]);
  }
}

// ---------------------------------------------------------------------------
// dw_bwd: dL/dd (norm2 + PReLU2 backward) on a gd window, transposed depthwise
// conv, depthwise weight gradient against an n1 window, norm1 backward sums.
//   gd window  gdw[i] = dL/dd   at step j + (POWN - P + 1 + i)
//   ah window  ahw[i] = hat a1  at step j + (i - POWN)
// ---------------------------------------------------------------------------
template <typename T, int NK, int P, bool CAUSAL>
__global__ __launch_bounds__(256) void dw_bwd_kernel(DwArgs a) {
  constexpr int POWN = CAUSAL ? P - 1 : (P - 1) / 2;
  constexpr int GT = POWN, AT = P - 1 - POWN;           // newest step of each window, relative to j
  __shared__ double red[16];
  __shared__ float buf[256 * 8];
  const CombGeom gm = comb_geom(a);
  const CombItem it = comb_item(a, gm);
  const int H = a.H, K = a.g.K, Kp = a.g.Kp, dil = a.dil, c = it.c;
  const T* h1 = reinterpret_cast<const T*>(a.h1);
  const T* dd = reinterpret_cast<const T*>(a.d);
  const T* ga2 = reinterpret_cast<const T*>(a.ga2);
  T* ga1o = reinterpret_cast<T*>(a.ga1_out);
  const float al1 = a.alpha1[0], al2 = a.alpha2[0];
  float2 st1u = make_float2(0.f, 0.f), st2u = st1u, sm2u = st1u;
  if constexpr (NK == NORM_GLN) {
    st1u = a.st1[it.m];
    st2u = a.st2[it.m];
    const StatFold& f = a.f_sm2;
    sm2u = f.slab ? fold_stat(f, it.m) : a.sm2[it.m];
  }

  // Per-element arithmetic in channel pairs (f32x2: v_pk_fma/mul/add_f32, two channels
  // per instruction; this kernel is VALU-issue-bound at 2 waves per SIMD).  Pair i
  // holds channels 2i, 2i+1 of the lane's 8.
  f32x2_t w[P][4], g1[4], b1[4], g2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ch = c * 8 + 2 * i;
    g1[i] = f32x2_t{a.gamma1[ch], a.gamma1[ch + 1]};
    b1[i] = f32x2_t{a.beta1[ch], a.beta1[ch + 1]};
    g2[i] = f32x2_t{a.gamma2[ch], a.gamma2[ch + 1]};
#pragma unroll
    for (int q = 0; q < P; ++q) w[q][i] = f32x2_t{a.wd[ch * P + q], a.wd[(ch + 1) * P + q]};
  }
  // cgam/cbet: norm-1 affine gradients; cgam2/cbet2: norm-2 affine gradients
  // (sum over own rows of g_n2 * hat a2 and of g_n2)
  f32x2_t cgam[4], cbet[4], cgam2[4], cbet2[4], cwd[P][4];
  const f32x2_t z2 = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    cgam[i] = cbet[i] = cgam2[i] = cbet2[i] = z2;
#pragma unroll
    for (int q = 0; q < P; ++q) cwd[q][i] = z2;
  }
  float calpha = 0.f, ts = 0.f, tss = 0.f;
  // PReLU and its derivatives on a pair (exact selects, any alpha)
  auto pr2 = [](f32x2_t x, float al) __attribute__((always_inline)) {
    const f32x2_t ax = x * al;
    return f32x2_t{x[0] > 0.f ? x[0] : ax[0], x[1] > 0.f ? x[1] : ax[1]};
  };

  auto row_of = [&](int j) { return it.rho + j * dil; };
  // gd stream: d and dL/d(hat a2) of one comb step
  // (cLN statistics are loaded at the point of use here: fetching them with the rows,
  // as dw_fwd does, took this 256-VGPR kernel from 661 to 878 us at c4)
  auto fetch_g = [&](int j, Raw8<T>& rd, Raw8<T>& rg, bool& ok, int& row) {
    const int k = row_of(j);
    ok = j >= 0 && k < K;
    row = it.base + (ok ? k : 0);
    rd.load(dd + (size_t)row * H + c * 8);
    rg.load(ga2 + (size_t)row * H + c * 8);
  };
  // cLN with one comb item per wave: the per-row statistics of 64 consecutive walk steps
  // are loaded one step per lane and broadcast with v_readlane, instead of a dependent
  // global load in front of every row (bstep: the step being finished, -1 outside the walk)
  float2 bst2 = make_float2(0.f, 0.f), bsm2 = bst2, bst1 = bst2;
  int bbase = -(1 << 29), bstep = -1;
  auto bl = [&](int jj) { const int k = row_of(jj); return it.base + ((jj >= 0 && k < K) ? k : 0); };
  auto batch_load = [&](int jb) {
    bbase = jb;
    const int rgw = bl(jb + (threadIdx.x & 63) + GT), rhw = bl(jb + (threadIdx.x & 63) + AT);
    bst2 = a.st2[rgw];
    bsm2 = a.sm2[rgw];
    bst1 = a.st1[rhw];
  };
  auto bcast = [&](float2 v) {
    const int l = __builtin_amdgcn_readfirstlane(bstep - bbase);
    return make_float2(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), l)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), l)));
  };
  auto finish_g = [&](const Raw8<T>& rd, const Raw8<T>& rg, bool ok, int row, bool count, f32x2_t* gd) {
    const float2 st = NK == NORM_GLN ? st2u : (bstep >= 0 ? bcast(bst2) : a.st2[row]);
    const float2 sm = NK == NORM_GLN ? sm2u : (bstep >= 0 ? bcast(bsm2) : a.sm2[row]);
    const f32x2_t nm = {-st.x, -st.x}, nsx = {-sm.x, -sm.x}, nsy = {-sm.y, -sm.y};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x2_t x = {rd[2 * i], rd[2 * i + 1]};
      const f32x2_t ah = (pr2(x, al2) + nm) * st.y;                       // hat a2
      const f32x2_t gn = {rg[2 * i], rg[2 * i + 1]};                     // dL/d(norm2 output)
      const f32x2_t ga = pfma(ah, nsy, pfma(gn, g2[i], nsx)) * st.y;     // dL/da2
      const f32x2_t dx = {x[0] > 0.f ? 1.f : al2, x[1] > 0.f ? 1.f : al2};
      const f32x2_t g = ga * dx;
      gd[i] = f32x2_t{ok ? g[0] : 0.f, ok ? g[1] : 0.f};   // rows outside the utterance: exactly 0
      if (ok && count) {
        calpha = fmaf(ga[0], x[0] > 0.f ? 0.f : x[0], calpha);   // channel order
        calpha = fmaf(ga[1], x[1] > 0.f ? 0.f : x[1], calpha);
        cgam2[i] = pfma(gn, ah, cgam2[i]);
        cbet2[i] += gn;
      }
    }
  };
  // ah stream: hat a1 of one comb step
  auto fetch_h = [&](int j, Raw8<T>& rh, bool& ok, int& row) {
    const int k = row_of(j);
    ok = j >= 0 && k < K;
    row = it.base + (ok ? k : 0);
    rh.load(h1 + (size_t)row * H + c * 8);
  };
  auto finish_h = [&](const Raw8<T>& rh, int row, f32x2_t* ah) {
    const float2 st = NK == NORM_GLN ? st1u : (bstep >= 0 ? bcast(bst1) : a.st1[row]);
    const f32x2_t nm = {-st.x, -st.x};
#pragma unroll
    for (int i = 0; i < 4; ++i) ah[i] = (pr2(f32x2_t{rh[2 * i], rh[2 * i + 1]}, al1) + nm) * st.y;
  };

  // nw: the depthwise-weight gradient's operand of each window row, n1 = gamma1 * hat a1 +
  // beta1 (0 for rows outside the utterance), formed once when the row enters the window
  // instead of at each of its P uses
  f32x2_t gdw[P][4], ahw[P][4], nw[P][4];
  auto enter_n = [&](int q, bool ok) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x2_t n = pfma(ahw[q][i], g1[i], b1[i]);
      nw[q][i] = f32x2_t{ok ? n[0] : 0.f, ok ? n[1] : 0.f};
    }
  };
#pragma unroll
  for (int i = 0; i < P - 1; ++i) {
    Raw8<T> rd, rg, rh; bool ok, okh; int row, rowh;
    const int sg = it.j0 + GT - P + 1 + i;
    fetch_g(sg, rd, rg, ok, row);
    fetch_h(it.j0 + AT - P + 1 + i, rh, okh, rowh);
    finish_g(rd, rg, ok, row, sg >= it.j0 && sg < it.j1, gdw[i]);   // alpha2 term: own rows only
    finish_h(rh, rowh, ahw[i]);
    enter_n(i, okh);
  }
  constexpr int D = dw_pf<T>();   // rows in flight per lane, slots as in dw_fwd
  const bool wave_item = gm.cg == 64;   // one comb item per wave (see RowPark)
  const int lane = threadIdx.x & 63;
  RowPark pk;
  pk.j0 = it.j0;
  // final norm-1 backward means or the slab entry of the rows parked in lanes < n
  auto park_flush = [&](int n) {
    const int k = row_of(pk.j0 + lane);
    if (lane < n && k < Kp) {
      if (a.sm1_out)   // the arithmetic of stats_finalize (mode 1)
        a.sm1_out[it.base + k] = make_float2((float)((double)pk.s / H), (float)((double)pk.ss / H));
      else
        a.slab1[it.base + k] = make_double2((double)pk.s, (double)pk.ss);
    }
  };
  // one step of the walk: row j's operands (d, dL/dn2 of step j+GT; h1 of step j+AT)
  auto body = [&](int j, const Raw8<T>& cd, const Raw8<T>& cgv, const Raw8<T>& ch, bool cok, bool cokh, int crow,
                  int crowh) __attribute__((always_inline)) {
    finish_g(cd, cgv, cok, crow, j + GT < it.j1, gdw[P - 1]);   // halo rows are counted by their own segment
    finish_h(ch, crowh, ahw[P - 1]);
    enter_n(P - 1, cokh);
    const int k = row_of(j);
    f32x2_t ga1[4] = {z2, z2, z2, z2};
    float s = 0.f, ss = 0.f;
    if (k < K) {
      f32x2_t gn1[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gn1[i] = w[0][i] * gdw[P - 1][i];
#pragma unroll
        for (int q = 1; q < P; ++q) gn1[i] = pfma(w[q][i], gdw[P - 1 - q][i], gn1[i]);
      }
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) cwd[q][i] = pfma(gdw[P - 1 - POWN][i], nw[q][i], cwd[q][i]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2_t ah = ahw[POWN][i];
        cgam[i] = pfma(gn1[i], ah, cgam[i]);
        cbet[i] += gn1[i];
        ga1[i] = gn1[i] * g1[i];
        s += ga1[i][0];   // sums over the 8 channels in channel order
        ss = fmaf(ga1[i][0], ah[0], ss);
        s += ga1[i][1];
        ss = fmaf(ga1[i][1], ah[1], ss);
      }
    }
    if (k < Kp) {
      const float o[8] = {ga1[0][0], ga1[0][1], ga1[1][0], ga1[1][1], ga1[2][0], ga1[2][1], ga1[3][0], ga1[3][1]};
      Vec8<T>::store(ga1o + (size_t)(it.base + k) * H + c * 8, o);
    }
    if constexpr (NK == NORM_GLN) {
      ts += s;
      tss += ss;
    } else if (wave_item) {
      s = wave_sum_dpp(s);
      ss = wave_sum_dpp(ss);
      const int pq = j - pk.j0;
      pk.s = lane == pq ? s : pk.s;
      pk.ss = lane == pq ? ss : pk.ss;
      if (pq == 63) {
        park_flush(64);
        pk.j0 = j + 1;
      }
    } else {
      s = wave_sum_group(s, gm.cg);
      ss = wave_sum_group(ss, gm.cg);
      if (c == 0 && k < Kp) {
        if (a.sm1_out)   // final means, the arithmetic of stats_finalize (mode 1)
          a.sm1_out[it.base + k] = make_float2((float)((double)s / H), (float)((double)ss / H));
        else
          a.slab1[it.base + k] = make_double2((double)s, (double)ss);
      }
    }
#pragma unroll
    for (int i = 0; i < P - 1; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gdw[i][e] = gdw[i + 1][e];
        ahw[i][e] = ahw[i + 1][e];
        nw[i][e] = nw[i + 1][e];
      }
  };
  Raw8<T> pd[D], pg[D], ph[D]; bool pok[D], pokh[D]; int prow[D], prowh[D];
#pragma unroll
  for (int q = 0; q < D; ++q) {
    fetch_g(it.j0 + q + GT, pd[q], pg[q], pok[q], prow[q]);
    fetch_h(it.j0 + q + AT, ph[q], pokh[q], prowh[q]);
  }
  for (int jb = it.j0; jb < it.j1; jb += D)
#pragma unroll
  for (int q = 0; q < D; ++q) {
    const int j = jb + q;
    if (j >= it.j1) break;
    Raw8<T> cd = pd[q], cgv = pg[q], ch = ph[q];
    const bool cok = pok[q], cokh = pokh[q];
    const int crow = prow[q], crowh = prowh[q];
    if (j + D < it.j1) {
      fetch_g(j + D + GT, pd[q], pg[q], pok[q], prow[q]);
      fetch_h(j + D + AT, ph[q], pokh[q], prowh[q]);
    }
    if constexpr (NK != NORM_GLN && CTN_DW_BATCH) {
      if (wave_item) {
        if (j - bbase >= 64) batch_load(j);
        bstep = j;
      }
    }
    body(j, cd, cgv, ch, cok, cokh, crow, crowh);
  }
  if constexpr (NK != NORM_GLN)
    if (wave_item && it.j1 > pk.j0) park_flush(it.j1 - pk.j0);
  // ---- workgroup reductions: column partials, alpha2, norm1 sums
  const int cgn = gm.cg, nrl = 256 / cgn, rl = threadIdx.x / cgn;
  float* cs = a.col_slab + (size_t)blockIdx.x * dw_col_stride(a);
  auto unpair = [](const f32x2_t (&v)[4], float (&o)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[2 * i] = v[i][0]; o[2 * i + 1] = v[i][1]; }
  };
  {
    float o[8];
    unpair(cgam, o);
    col_reduce8(buf, o, rl, c, nrl, cgn, true, cs);
    unpair(cbet, o);
    col_reduce8(buf, o, rl, c, nrl, cgn, true, cs + H);
    unpair(cgam2, o);
    col_reduce8(buf, o, rl, c, nrl, cgn, true, cs + (2 + P) * H);
    unpair(cbet2, o);
    col_reduce8(buf, o, rl, c, nrl, cgn, true, cs + (3 + P) * H);
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    // stored [H][P] to match the parameter layout [H,1,P]
    float o[8];
    unpair(cwd[p], o);
#pragma unroll
    for (int e = 0; e < 8; ++e) buf[rl * H + c * 8 + e] = o[e];
    __syncthreads();
    for (int chn = threadIdx.x; chn < H; chn += blockDim.x) {
      float sacc = 0.f;
      for (int q = 0; q < nrl; ++q) sacc += buf[q * H + chn];
      cs[2 * H + chn * P + p] = sacc;
    }
    __syncthreads();
  }
  {
    double v3[3] = {(double)calpha, (double)ts, (double)tss};
    block_sum_d<3>(v3, red);
    if (threadIdx.x == 0) {
      cs[(4 + P) * H] = (float)v3[0];
      if constexpr (NK == NORM_GLN) a.slab1[(size_t)it.m * gm.wgpu + it.wgi] = make_double2(v3[1], v3[2]);
    }
  }
}

// ---------------------------------------------------------------------------
template <typename T, int NK>
__global__ __launch_bounds__(256) void norm1_bwd_kernel(DwArgs a) {
  __shared__ double red[8];
  const int H = a.H, cg = H / 8;
  int nrl = 256 / cg;
  if (nrl > DW_RPB) nrl = DW_RPB;
  const int tid = threadIdx.x, c = tid % cg, rl = tid / cg;
  const bool act = rl < nrl;
  const int K = a.g.K, Kp = a.g.Kp;
  const int row0 = blockIdx.x * DW_RPB, m = row0 / Kp, base = m * Kp;
  const T* h1 = reinterpret_cast<const T*>(a.h1);
  const T* ga1 = reinterpret_cast<const T*>(a.ga2);   // input: dL/d(hat a1)
  T* gh = reinterpret_cast<T*>(a.gh1_out);
  const float al1 = a.alpha1[0];
  float calpha = 0.f;
  float2 sm1u = make_float2(0.f, 0.f);
  if constexpr (NK == NORM_GLN) {
    const StatFold& f = a.f_sm1;
    sm1u = f.slab ? fold_stat(f, m) : a.sm1[m];
  }
  if (act) {
    for (int rr = rl; rr < DW_RPB; rr += nrl) {
      const int r = row0 + rr, k = r - base;
      float out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (k < K) {
        float v[8], g[8];
        Vec8<T>::load(h1 + (size_t)r * H + c * 8, v);
        Vec8<T>::load(ga1 + (size_t)r * H + c * 8, g);
        const float2 st = ld_stat<NK>(a.st1, m, r);
        const float2 sm = NK == NORM_GLN ? sm1u : a.sm1[r];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float ah = (prelu(v[e], al1) - st.x) * st.y;
          const float ga = st.y * (g[e] - sm.x - ah * sm.y);
          out[e] = ga * prelu_dx(v[e], al1);
          calpha += ga * prelu_da(v[e]);
        }
      }
      Vec8<T>::store(gh + (size_t)r * H + c * 8, out);
    }
  }
  double v1[1] = {(double)calpha};
  block_sum_d<1>(v1, red);
  if (tid == 0) a.alpha_slab[blockIdx.x] = (float)v1[0];
}


static hipError_t dw_check(const DwArgs& a) {
  const int cg = a.H / 8;
  if (a.H % 8 != 0 || cg > 64 || (cg & (cg - 1)) || a.P < 1 || a.P > DW_MAXP || a.g.Kp % DW_RPB != 0 ||
      a.dil < 1 || a.seg < 1)
    return hipErrorInvalidValue;
  const int pown = a.pad / a.dil;
  if (pown * a.dil != a.pad || (pown != a.P - 1 && pown != (a.P - 1) / 2)) return hipErrorInvalidValue;
  return hipSuccess;
}

#define CTN_DW_P_KERNEL(NAME)                                                                  \
  template <typename T, int NK, int P>                                                       \
  static void NAME##_launch(const DwArgs& a, hipStream_t s) {                                \
    const bool causal = a.pad / a.dil == P - 1 && P > 1 && (P - 1) != (P - 1) / 2;           \
    if (causal) hipLaunchKernelGGL((NAME##_kernel<T, NK, P, true>), dim3(dw_blocks(a)), dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((NAME##_kernel<T, NK, P, false>), dim3(dw_blocks(a)), dim3(256), 0, s, a); \
  }                                                                                          \
  template <typename T, int NK>                                                              \
  static hipError_t NAME##_dispatch_p(const DwArgs& a, hipStream_t s) {                      \
    switch (a.P) {                                                                           \
      case 1: NAME##_launch<T, NK, 1>(a, s); break;                                          \
      case 2: NAME##_launch<T, NK, 2>(a, s); break;                                          \
      case 3: NAME##_launch<T, NK, 3>(a, s); break;                                          \
      case 4: NAME##_launch<T, NK, 4>(a, s); break;                                          \
      case 5: NAME##_launch<T, NK, 5>(a, s); break;                                          \
      case 6: NAME##_launch<T, NK, 6>(a, s); break;                                          \
      case 7: NAME##_launch<T, NK, 7>(a, s); break;                                          \
      case 8: NAME##_launch<T, NK, 8>(a, s); break;                                          \
      default: return hipErrorInvalidValue;                                                  \
    }                                                                                        \
    return hipGetLastError();                                                                \
  }                                                                                          \
  hipError_t launch_##NAME(DType dt, const DwArgs& a, hipStream_t s) {                       \
    hipError_t e = dw_check(a);                                                              \
    if (e != hipSuccess) return e;                                                           \
    if (dw_wave_eligible(dt, a)) return launch_##NAME##_wave(a, s);                           \
    if (dt == BF16)                                                                          \
      return a.norm == NORM_GLN ? NAME##_dispatch_p<bf16raw, NORM_GLN>(a, s)                 \
                                : NAME##_dispatch_p<bf16raw, NORM_CLN>(a, s);                \
    return a.norm == NORM_GLN ? NAME##_dispatch_p<float, NORM_GLN>(a, s)                     \
                              : NAME##_dispatch_p<float, NORM_CLN>(a, s);                    \
  }

CTN_DW_P_KERNEL(dw_fwd)

template <typename T, int NK, int P>
static void dw_bwd_launch(const DwArgs& a, hipStream_t s) {
  const bool causal = a.pad / a.dil == P - 1 && P > 1 && (P - 1) != (P - 1) / 2;
  const dim3 grid(dw_blocks(a)), blk(256);
  if (causal) hipLaunchKernelGGL((dw_bwd_kernel<T, NK, P, true>), grid, blk, 0, s, a);
  else hipLaunchKernelGGL((dw_bwd_kernel<T, NK, P, false>), grid, blk, 0, s, a);
}
template <typename T, int NK>
static hipError_t dw_bwd_dispatch_p(const DwArgs& a, hipStream_t s) {
  switch (a.P) {
    case 1: dw_bwd_launch<T, NK, 1>(a, s); break;
    case 2: dw_bwd_launch<T, NK, 2>(a, s); break;
    case 3: dw_bwd_launch<T, NK, 3>(a, s); break;
    case 4: dw_bwd_launch<T, NK, 4>(a, s); break;
    case 5: dw_bwd_launch<T, NK, 5>(a, s); break;
    case 6: dw_bwd_launch<T, NK, 6>(a, s); break;
    case 7: dw_bwd_launch<T, NK, 7>(a, s); break;
    case 8: dw_bwd_launch<T, NK, 8>(a, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
hipError_t launch_dw_bwd(DType dt, const DwArgs& a, hipStream_t s) {
  hipError_t e = dw_check(a);
  if (e != hipSuccess) return e;
  if (dw_wave_eligible(dt, a)) return launch_dw_bwd_wave(a, s);
  if (dt == BF16)
    return a.norm == NORM_GLN ? dw_bwd_dispatch_p<bf16raw, NORM_GLN>(a, s) : dw_bwd_dispatch_p<bf16raw, NORM_CLN>(a, s);
  return a.norm == NORM_GLN ? dw_bwd_dispatch_p<float, NORM_GLN>(a, s) : dw_bwd_dispatch_p<float, NORM_CLN>(a, s);
}

hipError_t launch_norm1_bwd(DType dt, const DwArgs& a, hipStream_t s) {
  hipError_t e = dw_check(a);
  if (e != hipSuccess) return e;
  const dim3 grid(ew_blocks(a)), blk(256);
  if (dt == BF16) {
    if (a.norm == NORM_GLN) hipLaunchKernelGGL((norm1_bwd_kernel<bf16raw, NORM_GLN>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((norm1_bwd_kernel<bf16raw, NORM_CLN>), grid, blk, 0, s, a);
  } else {
    if (a.norm == NORM_GLN) hipLaunchKernelGGL((norm1_bwd_kernel<float, NORM_GLN>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((norm1_bwd_kernel<float, NORM_CLN>), grid, blk, 0, s, a);
  }
  return hipGetLastError();
}

// ===========================================================================
// statistics finalize / slab reduce / weight prep
// ===========================================================================
// one thread per group (few parts, e.g. cLN rows) ...
__global__ __launch_bounds__(256) void stats_finalize_thread_kernel(const double2* slab, int G, int nparts, double cnt,
                                                                    int mode, float eps, float2* out) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= G) return;
  double s = 0.0, ss = 0.0;
  for (int i = 0; i < nparts; ++i) {
    const double2 v = slab[(size_t)g * nparts + i];
    s += v.x;
    ss += v.y;
  }
  if (mode == 0) {
    const double mean = s / cnt;
    double var = ss / cnt - mean * mean;
    if (var < 0.0) var = 0.0;
    out[g] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
  } else {
    out[g] = make_float2((float)(s / cnt), (float)(ss / cnt));
  }
}

// ... or a tile of 64 groups per workgroup staged through LDS with coalesced loads
// (cLN: 516k rows x 16 parts at c4; a thread walking its own row's parts read the
// slab with a 256-byte lane stride), summed per thread in the same part order
constexpr int SF_ROWS = 64;
__global__ __launch_bounds__(256) void stats_finalize_tile_kernel(const double2* slab, int G, int nparts, double cnt,
                                                                  int mode, float eps, float2* out) {
  extern __shared__ double2 sh[];   // [SF_ROWS][nparts + 1] (padded row: 4-way banks)
  const long g0 = (long)blockIdx.x * SF_ROWS;
  const int rows = (int)(G - g0 < SF_ROWS ? G - g0 : SF_ROWS);
  const int n = rows * nparts;
  for (int i = threadIdx.x; i < n; i += 256) sh[(i / nparts) * (nparts + 1) + i % nparts] = slab[g0 * nparts + i];
  __syncthreads();
  if (threadIdx.x >= rows) return;
  double s = 0.0, ss = 0.0;
  for (int i = 0; i < nparts; ++i) {
    const double2 v = sh[threadIdx.x * (nparts + 1) + i];
    s += v.x;
    ss += v.y;
  }
  const long g = g0 + threadIdx.x;
  if (mode == 0) {
    const double mean = s / cnt;
    double var = ss / cnt - mean * mean;
    if (var < 0.0) var = 0.0;
    out[g] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
  } else {
    out[g] = make_float2((float)(s / cnt), (float)(ss / cnt));
  }
}

// ... or one workgroup per group (many parts, e.g. gLN utterances)
__global__ __launch_bounds__(256) void stats_finalize_block_kernel(const double2* slab, int nparts, double cnt,
                                                                   int mode, float eps, float2* out) {
  __shared__ double red[8];
  const int g = blockIdx.x;
  double v[2] = {0.0, 0.0};
  for (int i = threadIdx.x; i < nparts; i += 256) {
    const double2 x = slab[(size_t)g * nparts + i];
    v[0] += x.x;
    v[1] += x.y;
  }
  block_sum_d<2>(v, red);
  if (threadIdx.x == 0) {
    if (mode == 0) {
      const double mean = v[0] / cnt;
      double var = v[1] / cnt - mean * mean;
      if (var < 0.0) var = 0.0;
      out[g] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
    } else {
      out[g] = make_float2((float)(v[0] / cnt), (float)(v[1] / cnt));
    }
  }
}

hipError_t launch_stats_finalize(const double2* slab, int G, int nparts, double cnt, int mode, float eps,
                                 float2* out, hipStream_t s) {
  // one workgroup per group only when groups are few and long (gLN: one per
  // utterance); cLN has a group per frame row (G = M*Kp, 516k at c4), where a
  // workgroup per row cost 540 us per launch against a few us for a thread per row
  if (nparts >= 8 && (G < 8192 || nparts > 64))
    hipLaunchKernelGGL(stats_finalize_block_kernel, dim3(G), dim3(256), 0, s, slab, nparts, cnt, mode, eps, out);
  else if (nparts >= 2)
    hipLaunchKernelGGL(stats_finalize_tile_kernel, dim3((G + SF_ROWS - 1) / SF_ROWS), dim3(256),
                       (size_t)SF_ROWS * (nparts + 1) * sizeof(double2), s, slab, G, nparts, cnt, mode, eps, out);
  else
    hipLaunchKernelGGL(stats_finalize_thread_kernel, dim3((G + 255) / 256), dim3(256), 0, s, slab, G, nparts, cnt,
                       mode, eps, out);
  return hipGetLastError();
}

// out[i] = sum_q src[q * pstride + i], deterministic, fp64 accumulation.
// Workgroup = one 64-output tile x one slice of <= SR_SLICE parts of one
// descriptor; wave w sums parts w, w+4, ... of the slice (lanes = 64
// consecutive outputs: 256-byte rows, loads unrolled 8 deep); the 4 wave
// partials combine in a fixed order.  Descriptors with more than one slice
// write slice partials to `tmp` and a second pass sums the slices in order.
constexpr int SR_SLICE = 64;

struct SrJob {
  const float* src;
  float* dst;
  int nparts, n, pstride, nslices;
  int vec4;   // 4 consecutive outputs per lane (16-byte loads); same per-output order
};
// The grid is flat: job jb owns workgroups [wg0[jb], wg0[jb+1]), one per (slice, output
// tile) pair, so no workgroup is launched only to exit (a (tiles, slices, jobs) grid sized
// by the largest job launched ~70k workgroups per block backward for ~1.3k with work).
// Up to SR_MAXJ jobs per launch (kernel arguments: ~3 KiB): a whole backward's deferred
// reductions (ctn_tblock_reduce_grads) take a few launches instead of two per block.
constexpr int SR_MAXJ = 64;
struct SrBatch {
  SrJob j[SR_MAXJ];
  int wg0[SR_MAXJ + 1];   // prefix sums of the jobs' workgroup counts
  int ntx[SR_MAXJ];       // output tiles per slice
  int nj;
};

// Streaming copy (bench.py's measured bandwidth ceiling, ctn_copy_bytes): 16 B per lane,
// U independent loads in flight per lane before their stores, grid-stride; NT: the loads
// and stores carry the nontemporal hint.
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_stream_kernel(const v4u* __restrict__ src, v4u* __restrict__ dst,
                                                          long n16) {
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

hipError_t launch_copy_stream(void* dst, const void* src, size_t bytes, int wgs, int flags, hipStream_t s) {
  if (!dst || !src || bytes % 16 || ((uintptr_t)dst | (uintptr_t)src) % 16 || wgs < 1 || wgs > 65536 ||
      (flags & ~3))
    return hipErrorInvalidValue;
  if (!bytes) return hipSuccess;
  const v4u* a = (const v4u*)src;
  v4u* b = (v4u*)dst;
  const long n = (long)(bytes / 16);
  switch (flags) {
    case 0: hipLaunchKernelGGL((copy_stream_kernel<4, false>), dim3(wgs), dim3(256), 0, s, a, b, n); break;
    case 1: hipLaunchKernelGGL((copy_stream_kernel<4, true>), dim3(wgs), dim3(256), 0, s, a, b, n); break;
    case 2: hipLaunchKernelGGL((copy_stream_kernel<8, false>), dim3(wgs), dim3(256), 0, s, a, b, n); break;
    default: hipLaunchKernelGGL((copy_stream_kernel<8, true>), dim3(wgs), dim3(256), 0, s, a, b, n); break;
  }
  return hipGetLastError();
}

// MFMA throughput microbenchmark (bench.py's measured matrix peak beside the 2.5 PF/s
// datasheet value, ctn_mfma_peak): every wave issues `iters` rounds of NACC independent
// back-to-back bf16 MFMAs on register operands drawn from a hash of its lane (random
// data: the chip holds a lower clock on random than on zero operands), and writes its
// accumulators so nothing is dead.  SHAPE 0: v_mfma_f32_16x16x32_bf16 (16384 FLOP, the
// block kernels' instruction), 1: v_mfma_f32_32x32x16_bf16 (32768 FLOP).
typedef short mp_bf16x8 __attribute__((ext_vector_type(8)));
typedef float mp_f32x4 __attribute__((ext_vector_type(4)));
typedef float mp_f32x16 __attribute__((ext_vector_type(16)));
template <int SHAPE>
__global__ __launch_bounds__(256) void mfma_peak_kernel(int iters, float* out) {
  constexpr int NACC = SHAPE == 0 ? 8 : 4;
  const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
  uint32_t h = gid * 2654435761u + 12345u;
  short av[8], bv[8];
  for (int e = 0; e < 8; ++e) {
    h ^= h << 13; h ^= h >> 17; h ^= h << 5;
    av[e] = (short)(0x3800 | (h & 0x807f));   // bf16 of magnitude ~2^-15..2^-14, random sign and mantissa
    h ^= h << 13; h ^= h >> 17; h ^= h << 5;
    bv[e] = (short)(0x3800 | (h & 0x807f));
  }
  const mp_bf16x8 a = {av[0], av[1], av[2], av[3], av[4], av[5], av[6], av[7]};
  const mp_bf16x8 b = {bv[0], bv[1], bv[2], bv[3], bv[4], bv[5], bv[6], bv[7]};
  float sum = 0.f;
  if constexpr (SHAPE == 0) {
    mp_f32x4 acc[NACC];
    for (int j = 0; j < NACC; ++j) acc[j] = mp_f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
    for (int j = 0; j < NACC; ++j) sum += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  } else {
    mp_f32x16 acc[NACC];
    for (int j = 0; j < NACC; ++j)
      for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
    for (int j = 0; j < NACC; ++j)
      for (int e = 0; e < 16; ++e) sum += acc[j][e];
  }
  out[gid] = sum;
}

hipError_t launch_mfma_peak(int shape, int wgs, int iters, float* out, double* flops, hipStream_t s) {
  if (!out || wgs < 1 || wgs > 65536 || iters < 1 || (shape != 0 && shape != 1)) return hipErrorInvalidValue;
  // waves x iterations x independent accumulators x FLOP per instruction
  if (flops) *flops = (double)wgs * 4 * iters * (shape == 0 ? 8.0 * 16384 : 4.0 * 32768);
  if (shape == 0) hipLaunchKernelGGL((mfma_peak_kernel<0>), dim3(wgs), dim3(256), 0, s, iters, out);
  else hipLaunchKernelGGL((mfma_peak_kernel<1>), dim3(wgs), dim3(256), 0, s, iters, out);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void slab_reduce_kernel(SrBatch b) {
  __shared__ double part[4][64];
  __shared__ double part4[4][4][64];
  int jb = 0;   // the job owning this workgroup: binary search of the prefix sums
  for (int step = SR_MAXJ / 2; step > 0; step >>= 1)
    if (jb + step < b.nj && (int)blockIdx.x >= b.wg0[jb + step]) jb += step;
  const SrJob d = b.j[jb];
  const int ntx = b.ntx[jb];
  const int loc = (int)blockIdx.x - b.wg0[jb];
  const int sl = loc / ntx, tx = loc - sl * ntx;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q0 = sl * SR_SLICE;
  const int q1 = d.nslices == 1 ? d.nparts : (q0 + SR_SLICE < d.nparts ? q0 + SR_SLICE : d.nparts);
  float* out = d.nslices > 1 ? d.dst + (size_t)sl * d.n : d.dst;
  if (d.vec4) {   // lanes own 4 consecutive outputs: 1 KiB per wave load instead of 256 B
    for (int i0 = tx * 256; i0 < d.n; i0 += ntx * 256) {
      const int i = i0 + 4 * lane;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      if (i < d.n) {
        const float* src = d.src + i;
        int q = q0 + w;
        for (; q + 28 < q1; q += 32) {
          float4 v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(src + (size_t)(q + 4 * u) * d.pstride);
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            a0 += (double)v[u].x;
            a1 += (double)v[u].y;
            a2 += (double)v[u].z;
            a3 += (double)v[u].w;
          }
        }
        for (; q < q1; q += 4) {
          const float4 v = *reinterpret_cast<const float4*>(src + (size_t)q * d.pstride);
          a0 += (double)v.x;
          a1 += (double)v.y;
          a2 += (double)v.z;
          a3 += (double)v.w;
        }
      }
      part4[w][0][lane] = a0;
      part4[w][1][lane] = a1;
      part4[w][2][lane] = a2;
      part4[w][3][lane] = a3;
      __syncthreads();
      if (w == 0 && i < d.n) {
        float4 o;
        o.x = (float)(((part4[0][0][lane] + part4[1][0][lane]) + part4[2][0][lane]) + part4[3][0][lane]);
        o.y = (float)(((part4[0][1][lane] + part4[1][1][lane]) + part4[2][1][lane]) + part4[3][1][lane]);
        o.z = (float)(((part4[0][2][lane] + part4[1][2][lane]) + part4[2][2][lane]) + part4[3][2][lane]);
        o.w = (float)(((part4[0][3][lane] + part4[1][3][lane]) + part4[2][3][lane]) + part4[3][3][lane]);
        *reinterpret_cast<float4*>(out + i) = o;
      }
      __syncthreads();
    }
    return;
  }
  for (int i0 = tx * 64; i0 < d.n; i0 += ntx * 64) {
    const int i = i0 + lane;
    double acc = 0.0;
    if (i < d.n) {
      const float* src = d.src + i;
      int q = q0 + w;
      for (; q + 28 < q1; q += 32) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(q + 4 * u) * d.pstride];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += (double)v[u];
      }
      for (; q < q1; q += 4) acc += (double)src[(size_t)q * d.pstride];
    }
    part[w][lane] = acc;
    __syncthreads();
    if (w == 0 && i < d.n) out[i] = (float)(((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane]);
    __syncthreads();
  }
}

static hipError_t sr_launch(SrBatch b, hipStream_t s) {
  if (b.nj <= 0) return hipSuccess;
  long tot = 0;
  for (int i = 0; i < b.nj; ++i) {
    const int per = b.j[i].vec4 ? 256 : 64;
    int g = (b.j[i].n + per - 1) / per;
    if (g > 1024) g = 1024;   // larger outputs: grid-stride over the tiles
    if (g < 1) g = 1;
    b.ntx[i] = g;
    b.wg0[i] = (int)tot;
    tot += (long)g * b.j[i].nslices;
  }
  b.wg0[b.nj] = (int)tot;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)tot), dim3(256), 0, s, b);
  return hipGetLastError();
}

size_t slab_reduce_tmp_floats(const SlabBatch& b) {
  size_t t = 0;
  for (int i = 0; i < b.nd; ++i) {
    const int ns = (b.d[i].nparts + SR_SLICE - 1) / SR_SLICE;
    if (ns > 1) t += (size_t)ns * b.d[i].n;
  }
  return t;
}

// Scratch of each descriptor with more than one slice, carved from `tmp` in descriptor
// order (slab_reduce_tmp_floats' sizing); null where one pass suffices or tmp is null.
void slab_reduce_assign_tmp(const SlabDesc* d, int n, float* tmp, float** out) {
  size_t off = 0;
  for (int i = 0; i < n; ++i) {
    const int ns = (d[i].nparts + SR_SLICE - 1) / SR_SLICE;
    out[i] = nullptr;
    if (ns > 1 && tmp) {
      out[i] = tmp + off;
      off += (size_t)ns * d[i].n;
    }
  }
}

// Every first pass (slice partials) of the list, then every second pass, SR_MAXJ jobs per
// launch.  Each descriptor's per-output summation order is that of launch_slab_reduce.
hipError_t launch_slab_reduce_list(const SlabDesc* descs, float* const* tmps, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  std::vector<SrJob> j1, j2;
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  for (int i = 0; i < n; ++i) {
    const SlabDesc& d = descs[i];
    const int ns = (d.nparts + SR_SLICE - 1) / SR_SLICE;
    const bool v4 = d.n % 4 == 0 && d.pstride % 4 == 0 && a16(d.src) && a16(d.dst);
    float* t = tmps ? tmps[i] : nullptr;
    if (ns <= 1 || !t) {
      // single pass straight into dst (also the fallback when no scratch is given)
      j2.push_back(SrJob{d.src, d.dst, d.nparts, d.n, d.pstride, 1, v4 ? 1 : 0});
    } else {
      const bool v4t = v4 && a16(t);
      j1.push_back(SrJob{d.src, t, d.nparts, d.n, d.pstride, ns, v4t ? 1 : 0});
      j2.push_back(SrJob{t, d.dst, ns, d.n, d.n, 1, v4t ? 1 : 0});
    }
  }
  for (const std::vector<SrJob>* js : {&j1, &j2}) {
    for (size_t k = 0; k < js->size(); k += SR_MAXJ) {
      SrBatch b{};
      for (size_t i = k; i < js->size() && b.nj < SR_MAXJ; ++i) b.j[b.nj++] = (*js)[i];
      const hipError_t e = sr_launch(b, s);
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

hipError_t launch_slab_reduce(const SlabBatch& b, float* tmp, hipStream_t s) {
  float* tmps[12];
  slab_reduce_assign_tmp(b.d, b.nd, tmp, tmps);
  return launch_slab_reduce_list(b.d, tmps, b.nd, s);
}

// fp32 [O][I] weight -> storage-type copy Ws [O][I] and/or transpose Wt [I][O], one
// 64x64 tile per workgroup through LDS: both the row-major reads/writes and the
// transposed writes are coalesced.  grid = (tiles of the largest matrix, nd).
constexpr int PW_T = 64;
template <typename T>
__global__ __launch_bounds__(256) void prep_weight_kernel(PrepBatch pb) {
  __shared__ float tile[PW_T][PW_T + 1];
  const PrepDesc d = pb.d[blockIdx.y];
  const int tcol = (d.I + PW_T - 1) / PW_T, trow = (d.O + PW_T - 1) / PW_T;
  if ((int)blockIdx.x >= tcol * trow) return;
  const int r0 = (blockIdx.x / tcol) * PW_T, c0 = (blockIdx.x % tcol) * PW_T;
  T* Ws = reinterpret_cast<T*>(d.Ws);
  T* Wt = reinterpret_cast<T*>(d.Wt);
  for (int i = threadIdx.x; i < PW_T * PW_T; i += 256) {
    const int r = i / PW_T, c = i % PW_T;
    float v = 0.f;
    if (r0 + r < d.O && c0 + c < d.I) {
      v = d.W[(size_t)(r0 + r) * d.I + c0 + c];
      if (Ws) st1<T>(Ws + (size_t)(r0 + r) * d.I + c0 + c, v);
    }
    tile[r][c] = v;
  }
  if (!Wt && !d.Wf && !d.Wtf) return;
  __syncthreads();
  if (Wt) {
    for (int i = threadIdx.x; i < PW_T * PW_T; i += 256) {
      const int c = i / PW_T, r = i % PW_T;
      if (r0 + r < d.O && c0 + c < d.I) st1<T>(Wt + (size_t)(c0 + c) * d.O + r0 + r, tile[r][c]);
    }
  }
  // fragment-order copies (frag_offset; O and I are multiples of 32, checked by the
  // caller, so the tile holds whole 32x32 fragment pairs): 512 pieces of 8 per copy
  for (int pass = 0; pass < 2; ++pass) {
    T* F = reinterpret_cast<T*>(pass ? d.Wtf : d.Wf);
    if (!F) continue;
    const int Icols = pass ? d.O : d.I;     // reduction length of the copy
    const int gb = (pass ? c0 : r0) / 32, kb0 = (pass ? r0 : c0) / 32;
    for (int i = threadIdx.x; i < 512; i += 256) {
      const int lane = i & 63, nb = (i >> 6) & 1, kb = (i >> 7) & 1, g = i >> 8;
      const int n = g * 32 + ((lane & 15) >> 2) * 8 + nb * 4 + (lane & 3), k = kb * 32 + (lane >> 4) * 8;
      if ((pass ? c0 + n >= d.I || r0 + k >= d.O : r0 + n >= d.O || c0 + k >= d.I)) continue;
      T* dst = F + frag_offset(gb + g, nb, kb0 + kb, lane, Icols);
#pragma unroll
      for (int e = 0; e < 8; ++e) st1<T>(dst + e, pass ? tile[k + e][n] : tile[n][k + e]);
    }
  }
}

hipError_t launch_prep_weights(DType dt, const PrepBatch& pb, hipStream_t s) {
  if (pb.nd <= 0) return hipSuccess;
  if (pb.nd > PREP_MAX) return hipErrorInvalidValue;
  int mx = 1;
  for (int i = 0; i < pb.nd; ++i) {
    const int t = ((pb.d[i].O + PW_T - 1) / PW_T) * ((pb.d[i].I + PW_T - 1) / PW_T);
    mx = t > mx ? t : mx;
  }
  if (dt == BF16) hipLaunchKernelGGL(prep_weight_kernel<bf16raw>, dim3(mx, pb.nd), dim3(256), 0, s, pb);
  else hipLaunchKernelGGL(prep_weight_kernel<float>, dim3(mx, pb.nd), dim3(256), 0, s, pb);
  return hipGetLastError();
}

hipError_t launch_prep_weight(DType dt, const float* W, int O, int I, void* Ws, void* Wt, hipStream_t s) {
  PrepBatch pb{};
  pb.d[0] = PrepDesc{W, O, I, Ws, Wt, nullptr, nullptr};
  pb.nd = 1;
  return launch_prep_weights(dt, pb, s);
}

}  // namespace ctn
