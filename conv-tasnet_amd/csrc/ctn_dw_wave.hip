// Wave-item depthwise kernels (bf16, H = 512, P = 3: every configuration of BASELINE.json):
// the TemporalBlock's dilated depthwise conv with its norms and PReLUs, forward and
// backward (conv_tasnet.py:176,212-272,289,307-355), on the comb walk of ctn_tcn.hip's
// dw_fwd_kernel / dw_bwd_kernel with the same work items, partial layouts and per-element
// arithmetic (bit-identical outputs), scheduled for the hardware:
//
//  * With H = 512 a wave's 64 lanes hold all channels of a row, so one comb item is one
//    wave and every walk quantity (utterance, residue, step, row) is wave-uniform: the
//    walk runs on scalar registers and branches, row-validity is a scalar per step.
//  * Interior steps (every row the step touches inside the utterance, the step's
//    alpha-2 / norm-2 terms counted) run a body without the per-element validity
//    selects; the few edge steps at the utterance ends and the segment tail run the
//    masked body.
//  * Rows are loaded two steps ahead into three register buffers used round robin,
//    and the window of P = 3 taps rotates through three slots, with the walk unrolled by
//    lcm(NB, P) = 3: every buffer and window slot is a compile-time register set, so the
//    loads stay in flight across the loop back edge.  The lane-group kernels carry their
//    prefetch in a register array that the loop shifts: the back edge copies the rows
//    just loaded into the array, and the copies wait for those loads (s_waitcnt vmcnt(0)
//    at the loop head), so their prefetch never overlapped a step's arithmetic.
#include <stdlib.h>

#include "ctn_common.h"
#include "ctn_dw.h"
#include "ctn_kernels.h"

namespace ctn {

namespace {

constexpr int WV_H = 512, WV_P = 3, WV_NB = 3;

// the wave's comb item: all fields wave-uniform (readfirstlane of the wave index)
struct WItem {
  int m, wgi, rho, j0, j1, base;
};
CTN_DEV WItem witem(const DwArgs& a, const CombGeom& gm) {
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  WItem it;
  it.m = (int)blockIdx.x / gm.wgpu;
  it.wgi = (int)blockIdx.x % gm.wgpu;
  const int id = it.wgi * gm.ipw + wv;   // ipw = 4: one item per wave
  const bool active = id < gm.items;
  it.rho = active ? id / gm.nseg : 0;
  it.j0 = active ? (id % gm.nseg) * a.seg : 0;
  it.j1 = active ? min(it.j0 + a.seg, gm.jmax) : it.j0;
  it.base = it.m * a.g.Kp;
  return it;
}
// comb steps s >= 0 whose row rho + s*dil lies inside the utterance (< K)
CTN_DEV int steps_below(int K, int rho, int dil) { return K > rho ? (K - rho - 1) / dil + 1 : 0; }

CTN_DEV void unpack8(const v4u& v, float f[8]) { unpack_bf16x8(v, f); }
// One 1 KiB row (512 bf16 channels) stored by the wave, 16 bytes per lane.  A global store,
// not buffer_store_dwordx4 with the row offset in soffset: on gfx950 that store wrote stale
// data for some lanes when the compiler reused its data registers for the next step's
// buffer_load (dword 0 of lanes 12-15 of every 16, ~0.1 % of the rows, data-race-like; gone
// with 16 wait states after the store, or with a global store: tools/exp/dw_debug.py,
// DESIGN.md §15).  The compiler inserts no wait state for it: its hazard model treats a
// >64-bit MUBUF store with a register soffset as safe.
// CTN_DW_NT bits: the nontemporal hint on the forward's d rows (1) and on the backward's
// dL/da1 rows (2).  Both on: the rows stream past the Infinity Cache instead of evicting
// what the next kernels read from it (dw_fwd 44.6 -> 38.4 us, the H -> B GEMM after it
// 47.5 -> 42.5, dw_bwd 82.5 -> 80); the hint on the producers of h1, dL/dn2
// or dL/dh1 slows their consumers instead.
#ifndef CTN_DW_NT
#define CTN_DW_NT 3
#endif
// CTN_DW_NTL bits: the nontemporal hint on dw_bwd's d and dL/dn2 loads (1: their last use;
// dw_bwd -2.8 us, gx after it -1.7, the next dual +2.4), on dw_fwd's h1 loads (2: dw_fwd
// +6.4, off)
// 1: dw_bwd's per-channel constants half-major in LDS (conflict-free reads); 0: lane-major
#ifndef CTN_DW_CSTH
#define CTN_DW_CSTH 1
#endif
#ifndef CTN_DW_NTL
#define CTN_DW_NTL 1
#endif
template <bool NT = false>
CTN_DEV void row_store(void* base, v4u v, int row) {
  stg16h<NT>(reinterpret_cast<char*>(base) + (size_t)row * 1024 + (threadIdx.x & 63) * 16u, v);
}
// a wave-uniform pair into scalar registers (readfirstlane works on 32-bit integers)
CTN_DEV float2 uniform2(float2 v) {
  return make_float2(__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.x))),
                     __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.y))));
}
CTN_DEV float sel_pos(float x, float a, float b) { return x > 0.f ? a : b; }

// ===========================================================================
// forward: d[k] = sum_t w[t] n1[k - pad + t*dil], n1 = norm1(PReLU(h1)) (0 outside [0, K)),
// and the statistics of PReLU(d) for norm 2 (dw_fwd_kernel)
// ===========================================================================
template <int NK, bool CAUSAL>
__global__ __launch_bounds__(256, 4) void dw_fwd_wave_kernel(DwArgs a) {
  constexpr int P = WV_P, H = WV_H;
  constexpr int POWN = CAUSAL ? P - 1 : (P - 1) / 2;
  constexpr int HT = P - 1 - POWN;   // the newest window row runs HT steps ahead of the walk
  __shared__ double red[16];
  const CombGeom gm = comb_geom(a);
  const WItem it = witem(a, gm);
  const int lane = threadIdx.x & 63;
  const int K = a.g.K, Kp = a.g.Kp, dil = a.dil;
  const long nbytes = a.g.rows() * H * 2;
  const rsrc_t rH = du_rsrc(a.h1, nbytes);
  const uint32_t vo = lane * 16;
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
    st1u = uniform2(st1u);
  }
  float w[P][8], g1[8], b1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int ch = lane * 8 + e;
    g1[e] = a.gamma1[ch];
    b1[e] = a.beta1[ch];
#pragma unroll
    for (int t = 0; t < P; ++t) w[t][e] = a.wd[ch * P + t];
  }
  const int jK = steps_below(K, it.rho, dil);
  auto row_at = [&](int s) { return it.base + ((unsigned)s < (unsigned)jK ? it.rho + s * dil : 0); };
  auto ld = [&](int row) {
    return __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rH, vo, row * (H * 2), (CTN_DW_NTL & 2) ? 2 : 0));
  };

  // cLN statistics of the newest row, in batches of CB steps (as dw_bwd_wave_kernel)
  constexpr int CB = 63;
  float2 bst = make_float2(0.f, 0.f), nst = bst;
  int bbase = it.j0;
  auto batch_fetch = [&](int jb) { nst = a.st1[row_at(jb + lane + HT)]; };
  auto batch_next = [&]() {
    bbase += CB;
    bst = nst;
    batch_fetch(bbase + CB);
  };
  auto bcast = [&](float2 v, int j) {
    const int l = j - bbase;
    return make_float2(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), l)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), l)));
  };
  // n1 of one row (EDGE: 0 outside the utterance, a select, so a non-finite value in the
  // row it fetched cannot leak in)
  auto finish = [&](auto edge, const v4u& vh, bool ok, float2 st, float* out) __attribute__((always_inline)) {
    constexpr bool EDGE = decltype(edge)::value;
    float x[8];
    unpack8(vh, x);
    const float nm = -st.x;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float ax = x[e] * al1;
      const float v = fmaf((sel_pos(x[e], x[e], ax) + nm) * st.y, g1[e], b1[e]);
      out[e] = EDGE ? (ok ? v : 0.f) : v;
    }
  };
  // window: step s in slot (s - j0 - HT) mod 3; at walk step j (q = (j - j0) mod 3) tap t
  // (step j - POWN + t) sits in slot (q + t + 1) mod 3, the newest (t = P-1) in q
  float win[3][8];
#pragma unroll
  for (int i = 0; i < P - 1; ++i) {
    const int sh = it.j0 - POWN + i;
    const int rh = row_at(sh);
    finish(std::true_type{}, ld(rh), (unsigned)sh < (unsigned)jK, NK == NORM_GLN ? st1u : a.st1[rh], win[i + 1]);
  }

  float ts = 0.f, tss = 0.f;
  RowPark pk;
  pk.j0 = it.j0;
  auto park_flush = [&](int n) {   // final (mean, rstd) or the (sum, sum sq) slab entry
    const int k = it.rho + (pk.j0 + lane) * dil;
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
  auto step = [&](auto edge, auto qc, int j, const v4u& vh) __attribute__((always_inline)) {
    constexpr bool EDGE = decltype(edge)::value;
    constexpr int q = decltype(qc)::value;
    const float2 st = NK == NORM_GLN ? st1u : bcast(bst, j);
    finish(edge, vh, EDGE ? j + HT < jK : true, st, win[q]);
    const int k = it.rho + j * dil;
    float o[8];
    float s = 0.f, ss = 0.f;
    if (!EDGE || j < jK) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] = w[0][e] * win[(q + 1) % 3][e];
#pragma unroll
        for (int t = 1; t < P; ++t) o[e] = fmaf(w[t][e], win[(q + t + 1) % 3][e], o[e]);
        const float a2 = sel_pos(o[e], o[e], o[e] * al2);
        s += a2;   // sums over the 8 channels in channel order
        ss = fmaf(a2, a2, ss);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = 0.f;
    }
    if (!EDGE || k < Kp)
      row_store<(CTN_DW_NT & 1) != 0>(a.d_out, pack_bf16x8v(o), it.base + k);
    if constexpr (NK == NORM_GLN) {
      ts += s;
      tss += ss;
    } else {
      s = wave_sum_dpp(s);
      ss = wave_sum_dpp(ss);
      const int pq = j - pk.j0;
      pk.s = lane == pq ? s : pk.s;
      pk.ss = lane == pq ? ss : pk.ss;
    }
  };
  auto boundary = [&]() {
    park_flush(CB);
    pk.j0 = bbase + CB;
    batch_next();
  };

  const int jint = min(it.j1, jK - HT);
  v4u rb[WV_NB];
  if (it.j0 < it.j1) rb[0] = ld(row_at(it.j0 + HT));
  if (it.j0 + 1 < it.j1) rb[1] = ld(row_at(it.j0 + 1 + HT));
  if constexpr (NK != NORM_GLN) {
    batch_fetch(it.j0);
    bbase = it.j0 - CB;
    batch_next();
  }
  auto triple = [&](int jb) __attribute__((always_inline)) {
    static_for<3>([&](auto qc) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      const int j = jb + q;
      __builtin_amdgcn_sched_barrier(0);
      rb[(q + 2) % 3] = ld(row_at(j + 2 + HT));   // unconditional (clamped) refill
      step(std::false_type{}, qc, j, rb[q]);
    });
  };
  int jb = it.j0;
  if constexpr (NK == NORM_GLN) {
    for (; jb + 3 <= jint; jb += 3) triple(jb);
  } else {
    for (;;) {
      const int jend = min(jint, bbase + CB);
      for (; jb + 3 <= jend; jb += 3) triple(jb);
      if (jb != bbase + CB || jb + 3 > jint) break;
      boundary();
    }
  }
  for (; jb < it.j1; jb += 3) {
    static_for<3>([&](auto qc) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      const int j = jb + q;
      if (j < it.j1) {
        if (j + 2 < it.j1) rb[(q + 2) % 3] = ld(row_at(j + 2 + HT));
        if constexpr (NK != NORM_GLN)
          if (j == bbase + CB) boundary();
        if (j < jint) step(std::false_type{}, qc, j, rb[q]);
        else step(std::true_type{}, qc, j, rb[q]);
      }
    });
  }
  if constexpr (NK != NORM_GLN) {
    if (it.j1 > pk.j0) park_flush(it.j1 - pk.j0);
  } else {
    double v2[2] = {(double)ts, (double)tss};
    block_sum_d<2>(v2, red);
    if (threadIdx.x == 0) a.slab2[(size_t)it.m * gm.wgpu + it.wgi] = make_double2(v2[0], v2[1]);
  }
}

// ===========================================================================
// backward: dL/dd (norm-2 + PReLU-2 backward) on a gd window, transposed depthwise conv,
// depthwise-weight gradient, norm-1 backward sums (dw_bwd_kernel)
//
// The weight gradient pairs each n1 row r of the walk with the gd rows r + POWN - t of its
// P taps (dL/dw[t] = sum_r n1[r] gd[r + POWN - t], the same products as the lane-group
// kernel's sum over gd rows, grouped by the n1 row): the gd window that the transposed conv
// needs already holds them, so n1 and hat a1 of row j are used at step j and need no
// window of their own (the lane-group kernel carries two, 48 registers).
// ===========================================================================
struct BwdRow {
  v4u d, g, h;   // d and dL/dn2 of G-step j+GT, h1 of step j
};

template <int NK, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void dw_bwd_wave_kernel(DwArgs a) {
  constexpr int P = WV_P, H = WV_H;
  constexpr int POWN = CAUSAL ? P - 1 : (P - 1) / 2;
  constexpr int GT = POWN;   // G stream (d, dL/dn2) runs POWN steps ahead of the walk
  __shared__ double red[16];
  __shared__ float buf[256 * 8];
  const CombGeom gm = comb_geom(a);
  const WItem it = witem(a, gm);
  const int lane = threadIdx.x & 63;
  const int K = a.g.K, Kp = a.g.Kp, dil = a.dil;
  const long nbytes = a.g.rows() * H * 2;
  const rsrc_t rH = du_rsrc(a.h1, nbytes), rD = du_rsrc(a.d, nbytes), rG = du_rsrc(a.ga2, nbytes);
  const uint32_t vo = lane * 16;   // the lane's 8 channels in a 1 KiB row
  const float al1 = a.alpha1[0], al2 = a.alpha2[0];
  float2 st1u = make_float2(0.f, 0.f), st2u = st1u, sm2u = st1u;
  if constexpr (NK == NORM_GLN) {
    st1u = a.st1[it.m];
    st2u = a.st2[it.m];
    const StatFold& f = a.f_sm2;
    sm2u = f.slab ? fold_stat(f, it.m) : a.sm2[it.m];
    sm2u = uniform2(sm2u);
  }
  // Per-channel constants (taps, gamma1, beta1, gamma2) live in LDS, read where they are
  // used: held in registers for the whole walk (48 per lane) they pushed the kernel past
  // the 256 registers of two waves per SIMD.
  // Row r holds the two 4-channel halves of every lane's 8 channels half-major
  // ([hf][lane][4]): one ds_read_b128 of a half then takes 16 consecutive bytes per lane,
  // conflict-free in every lane group (lane-major, the lanes' 32-byte stride put two lanes
  // of each group on one 16-byte slot: a 2-way conflict on every read of the walk).
  __shared__ __attribute__((aligned(16))) float cst[P + 3][H];   // w[0..P-1], gamma1, beta1, gamma2
  for (int i = threadIdx.x; i < H; i += 256) {
    const int c = CTN_DW_CSTH ? ((i >> 2) & 1) * (H / 2) + (i >> 3) * 4 + (i & 3) : i;   // i = 8 lane + 4 hf + k
#pragma unroll
    for (int t = 0; t < P; ++t) cst[t][c] = a.wd[i * P + t];
    cst[P][c] = a.gamma1[i];
    cst[P + 1][c] = a.beta1[i];
    cst[P + 2][c] = a.gamma2[i];
  }
  __syncthreads();
  // LDS address of the lane's 8 channels; re-derived opaquely in every step so the loads
  // are not hoisted out of the walk
  // (the lane's LDS base is re-derived opaquely once per use site, cbase(), so the loads are
  // not hoisted out of the walk; the row / half offsets fold into the instructions' offsets)
  auto cbase = [&]() __attribute__((always_inline)) {
    uint32_t b = lane * (CTN_DW_CSTH ? 16u : 32u);
    asm volatile("" : "+v"(b));
    return b;
  };
  auto cvec4 = [&](uint32_t b, int r, int hf) __attribute__((always_inline)) {   // channels 8 lane + 4 hf ..
    return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(&cst[0][0]) + b + (r * H * 4 + hf * (CTN_DW_CSTH ? H * 2 : 16)));
  };
  auto f4 = [](const float4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; };
  float cgam[8], cbet[8], cgam2[8], cbet2[8], cwd[P][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    cgam[e] = cbet[e] = cgam2[e] = cbet2[e] = 0.f;
#pragma unroll
    for (int t = 0; t < P; ++t) cwd[t][e] = 0.f;
  }
  float calpha = 0.f, ts = 0.f, tss = 0.f;

  // comb step s: steps [0, jK) lie inside the utterance; outside, the utterance's first
  // row is loaded (and masked)
  const int jK = steps_below(K, it.rho, dil);
  // (one unsigned compare: a short-circuit && becomes a branch, and branches let the
  // compiler sink one step's accumulations into the next step's blocks)
  auto row_at = [&](int s) { return it.base + ((unsigned)s < (unsigned)jK ? it.rho + s * dil : 0); };
  auto ld = [&](rsrc_t r, int row) { return __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, vo, row * (H * 2), 0)); };
  // d and dL/dn2 are read here for the last time (CTN_DW_NTL bit 0: with the nontemporal hint)
  auto ld_last = [&](rsrc_t r, int row) {
    return __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, vo, row * (H * 2), (CTN_DW_NTL & 1) ? 2 : 0));
  };
  auto load_row = [&](int j, BwdRow& r) __attribute__((always_inline)) {
    const int rg = row_at(j + GT);
    r.d = ld_last(rD, rg);
    r.g = ld_last(rG, rg);
    r.h = ld(rH, row_at(j));
  };

  // cLN: per-row statistics of CB consecutive steps, one step per lane, broadcast by
  // v_readlane (walk steps), or a direct load (prologue).  The next batch is loaded into
  // n* when the current one starts, so it has arrived when the walk reaches it.  CB is a
  // multiple of the walk's unroll (3) so batch boundaries fall between triples.
  constexpr int CB = 63;
  float2 bst2 = make_float2(0.f, 0.f), bsm2 = bst2, bst1 = bst2, nst2 = bst2, nsm2 = bst2, nst1 = bst2;
  int bbase = it.j0;
  // cLN norm-2 backward means: final (a.sm2), or folded here from the dual GEMM's per-row
  // partials (a.f_sm2: dense, at most 4 per row; the finalize launch's arithmetic: parts
  // summed in order from 0, divided by cnt in fp64, bit-identical).  A batch's raw parts
  // are loaded with the batch and summed when it becomes current.
  const StatFold& fs = a.f_sm2;
  const bool fsm = NK == NORM_CLN && fs.slab != nullptr;
  double2 nsmp[4];
  auto sm_fold = [&](const double2* v) {
    double s = 0.0, ss = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < fs.parts) s += v[q].x, ss += v[q].y;
    return make_float2((float)(s / fs.cnt), (float)(ss / fs.cnt));
  };
  auto sm_load = [&](int row, double2* v) {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = q < fs.parts ? fs.slab[(size_t)row * fs.parts + q] : make_double2(0.0, 0.0);
  };
  auto sm_row = [&](int row) {   // one row, outside the batches (prologue)
    if (!fsm) return a.sm2[row];
    double2 v[4];
    sm_load(row, v);
    return sm_fold(v);
  };
  auto batch_fetch = [&](int jb) {
    const int rgw = row_at(jb + lane + GT), rhw = row_at(jb + lane);
    nst2 = a.st2[rgw];
    if (fsm) sm_load(rgw, nsmp);
    else nsm2 = a.sm2[rgw];
    nst1 = a.st1[rhw];
  };
  auto batch_next = [&]() {   // the prefetched batch becomes current; fetch the one after
    bbase += CB;
    bst2 = nst2;
    bsm2 = fsm ? sm_fold(nsmp) : nsm2;
    bst1 = nst1;
    batch_fetch(bbase + CB);
  };
  auto bcast = [&](float2 v, int j) {
    const int l = j - bbase;
    return make_float2(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), l)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), l)));
  };

  // gd window: G-step s in slot (s - j0 - GT) mod 3, so at walk step j (q = (j - j0) mod 3)
  // the gd of row j + POWN - t (tap t) sits in slot (q + 3 - t) mod 3, the newest in q
  float gdw[3][8];

  // G-step terms of one row: EDGE masks rows outside the utterance (gd = 0) and counts the
  // alpha-2 / norm-2 affine terms only for `count` rows (the segment's own)
  auto finish_g = [&](auto edge, const v4u& vd, const v4u& vg, bool ok, bool count, float2 st, float2 sm,
                      float* gd) __attribute__((always_inline)) {
    constexpr bool EDGE = decltype(edge)::value;
    float x[8], gn[8];
    unpack8(vd, x);
    unpack8(vg, gn);
    const float nm = -st.x, nsx = -sm.x, nsy = -sm.y;
    // in halves of 4 channels: the channel constants and temporaries of one half at a time
    const uint32_t cb = cbase();
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const float4 g2v = cvec4(cb, P + 2, hf);
      float ah[4], ga[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = 4 * hf + i;
        const float ax = x[e] * al2;
        ah[i] = (sel_pos(x[e], x[e], ax) + nm) * st.y;                   // hat a2
        ga[i] = fmaf(ah[i], nsy, fmaf(gn[e], f4(g2v, i), nsx)) * st.y;   // dL/da2
        const float g = ga[i] * sel_pos(x[e], 1.f, al2);
        gd[e] = EDGE ? (ok ? g : 0.f) : g;                               // rows outside: exactly 0
        if constexpr (!EDGE) {
          calpha = fmaf(ga[i], sel_pos(x[e], 0.f, x[e]), calpha);         // channel order
          cgam2[e] = fmaf(gn[e], ah[i], cgam2[e]);
          cbet2[e] += gn[e];
        }
      }
      if constexpr (EDGE) {
        if (ok && count) {   // alpha-2 / norm-2 affine terms: the segment's own rows only
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int e = 4 * hf + i;
            calpha = fmaf(ga[i], sel_pos(x[e], 0.f, x[e]), calpha);
            cgam2[e] = fmaf(gn[e], ah[i], cgam2[e]);
            cbet2[e] += gn[e];
          }
        }
      }
    }
  };
  auto gstat = [&](int row, int j, bool batch, float2& st, float2& sm) __attribute__((always_inline)) {
    if constexpr (NK == NORM_GLN) {
      st = st2u;
      sm = sm2u;
    } else if (batch) {
      st = bcast(bst2, j);
      sm = bcast(bsm2, j);
    } else {
      st = a.st2[row];
      sm = sm_row(row);
    }
  };

  // ---- prologue: the gd window's two older entries (G-steps j0+GT-2, j0+GT-1: slots 1, 2)
#pragma unroll
  for (int i = 0; i < P - 1; ++i) {
    const int sg = it.j0 + GT - P + 1 + i;
    const int rg = row_at(sg);
    float2 st, sm;
    gstat(rg, 0, false, st, sm);
    finish_g(std::true_type{}, ld(rD, rg), ld(rG, rg), sg >= 0 && sg < jK, sg >= it.j0 && sg < it.j1, st, sm,
             gdw[i + 1]);
  }

  RowPark pk;
  pk.j0 = it.j0;
  auto park_flush = [&](int n) {
    const int k = it.rho + (pk.j0 + lane) * dil;
    if (lane < n && k < Kp) {
      if (a.sm1_out)   // the arithmetic of stats_finalize (mode 1)
        a.sm1_out[it.base + k] = make_float2((float)((double)pk.s / H), (float)((double)pk.ss / H));
      else
        a.slab1[it.base + k] = make_double2((double)pk.s, (double)pk.ss);
    }
  };

  // one walk step with its operands in r; q = (j - j0) mod 3 picks the window slots
  auto step = [&](auto edge, auto qc, int j, const BwdRow& r) __attribute__((always_inline)) {
    constexpr bool EDGE = decltype(edge)::value;
    constexpr int q = decltype(qc)::value;
    const int rg = row_at(j + GT), rh = row_at(j);
    float2 st, sm;
    gstat(rg, j, NK != NORM_GLN, st, sm);
    finish_g(edge, r.d, r.g, EDGE ? j + GT < jK : true, EDGE ? j + GT < it.j1 : true, st, sm, gdw[q]);
    // phases are scheduled one after the other: the scheduler otherwise sinks finish_g's
    // alpha-2 / norm-2 accumulations past the transposed conv, keeping every temporary of
    // both alive (pressure 105 -> 265 registers inside a step)
    __builtin_amdgcn_sched_barrier(0);
    const bool kin = !EDGE || j < jK;   // row j inside the utterance
    const int k = it.rho + j * dil;
    float ga1[8];
    float s = 0.f, ss = 0.f;
    if (kin) {
      float2 s1;
      if constexpr (NK == NORM_GLN) s1 = st1u;
      else s1 = bcast(bst1, j);
      float x[8];
      unpack8(r.h, x);
      const float nm = -s1.x;
      const uint32_t cb = cbase();
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        float4 wv[P];
#pragma unroll
        for (int t = 0; t < P; ++t) wv[t] = cvec4(cb, t, hf);
        const float4 g1v = cvec4(cb, P, hf), b1v = cvec4(cb, P + 1, hf);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = 4 * hf + i;
          const float ax = x[e] * al1;
          const float ah = (sel_pos(x[e], x[e], ax) + nm) * s1.y;   // hat a1 of row j
          const float n = fmaf(ah, f4(g1v, i), f4(b1v, i));         // n1 of row j
          float gn1 = f4(wv[0], i) * gdw[q][e];                     // dL/dn1 of row j
#pragma unroll
          for (int t = 1; t < P; ++t) gn1 = fmaf(f4(wv[t], i), gdw[(q + 3 - t) % 3][e], gn1);
#pragma unroll
          for (int t = 0; t < P; ++t) cwd[t][e] = fmaf(gdw[(q + 3 - t) % 3][e], n, cwd[t][e]);
          cgam[e] = fmaf(gn1, ah, cgam[e]);
          cbet[e] += gn1;
          ga1[e] = gn1 * f4(g1v, i);
          s += ga1[e];   // sums over the 8 channels in channel order
          ss = fmaf(ga1[e], ah, ss);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) ga1[e] = 0.f;
    }
    if (!EDGE || k < Kp)
      row_store<(CTN_DW_NT & 2) != 0>(a.ga1_out, pack_bf16x8v(ga1), it.base + k);
    (void)rh;
    if constexpr (NK == NORM_GLN) {
      ts += s;
      tss += ss;
    } else {   // parked in lane j - pk.j0 (flushed at batch boundaries: pk.j0 == bbase)
      s = wave_sum_dpp(s);
      ss = wave_sum_dpp(ss);
      const int pq = j - pk.j0;
      pk.s = lane == pq ? s : pk.s;
      pk.ss = lane == pq ? ss : pk.ss;
    }
  };
  auto boundary = [&]() {   // cLN: the walk reached bbase + CB
    park_flush(CB);
    pk.j0 = bbase + CB;
    batch_next();
  };

  // Interior steps in whole triples (no per-step guards: no value of a skipped step has
  // to survive a branch), then the edge steps at the segment / utterance end.  Edge steps
  // only occur at the end of a walk (every walk step is >= 0 and GT >= 0: the rows below
  // the utterance start only enter in the prologue).
  const int jint = min(it.j1, jK) - GT;
  BwdRow rb[WV_NB];
  if (it.j0 < it.j1) load_row(it.j0, rb[0]);
  if (it.j0 + 1 < it.j1) load_row(it.j0 + 1, rb[1]);
  if constexpr (NK != NORM_GLN) {
    batch_fetch(it.j0);
    bbase = it.j0 - CB;
    batch_next();   // current = [j0, j0 + CB), next in flight
  }
  auto triple = [&](int jb) __attribute__((always_inline)) {
    static_for<3>([&](auto qc) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      const int j = jb + q;
      // steps are scheduled one by one (interleaving them multiplies the live temporaries)
      __builtin_amdgcn_sched_barrier(0);
      // unconditional (clamped) refill: a guarded one would keep the slot's old value alive
      // around the loop (a step past j1 loads a row of the utterance that is never used)
      load_row(j + 2, rb[(q + 2) % 3]);
      step(std::false_type{}, qc, j, rb[q]);
    });
  };
  int jb = it.j0;
  if constexpr (NK == NORM_GLN) {
    for (; jb + 3 <= jint; jb += 3) triple(jb);
  } else {
    for (;;) {
      const int jend = min(jint, bbase + CB);
      for (; jb + 3 <= jend; jb += 3) triple(jb);
      if (jb != bbase + CB || jb + 3 > jint) break;
      boundary();
    }
  }
  for (; jb < it.j1; jb += 3) {
    static_for<3>([&](auto qc) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      const int j = jb + q;
      if (j < it.j1) {
        if (j + 2 < it.j1) load_row(j + 2, rb[(q + 2) % 3]);
        if constexpr (NK != NORM_GLN)
          if (j == bbase + CB) boundary();
        if (j < jint) step(std::false_type{}, qc, j, rb[q]);
        else step(std::true_type{}, qc, j, rb[q]);
      }
    });
  }
  if constexpr (NK != NORM_GLN)
    if (it.j1 > pk.j0) park_flush(it.j1 - pk.j0);

  // ---- workgroup reductions: column partials, alpha2, norm1 sums (dw_bwd_kernel's order)
  constexpr int cgn = 64, nrl = 4;
  const int rl = threadIdx.x >> 6;
  float* cs = a.col_slab + (size_t)blockIdx.x * dw_col_stride(a);
  col_reduce8(buf, cgam, rl, lane, nrl, cgn, true, cs);
  col_reduce8(buf, cbet, rl, lane, nrl, cgn, true, cs + H);
  col_reduce8(buf, cgam2, rl, lane, nrl, cgn, true, cs + (2 + P) * H);
  col_reduce8(buf, cbet2, rl, lane, nrl, cgn, true, cs + (3 + P) * H);
#pragma unroll
  for (int t = 0; t < P; ++t) {   // stored [H][P] to match the parameter layout [H,1,P]
#pragma unroll
    for (int e = 0; e < 8; ++e) buf[rl * H + lane * 8 + e] = cwd[t][e];
    __syncthreads();
    for (int chn = threadIdx.x; chn < H; chn += blockDim.x) {
      float sacc = 0.f;
      for (int u = 0; u < nrl; ++u) sacc += buf[u * H + chn];
      cs[2 * H + chn * P + t] = sacc;
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

}  // namespace

// CTN_DW_WAVE=0 keeps the lane-group kernels; read on every launch so one process can
// compare both (tests/test_gpu_dw_wave.py)
bool dw_wave_enabled() {
  const char* e = getenv("CTN_DW_WAVE");
  return e ? atoi(e) != 0 : true;
}

bool dw_wave_eligible(DType dt, const DwArgs& a) {
  if (dt != BF16 || a.H != WV_H || a.P != WV_P || !dw_wave_enabled()) return false;
  if (a.g.rows() * WV_H * 2 > 0x7fffffffL) return false;   // 32-bit buffer offsets
  const int pown = a.pad / a.dil;
  return pown * a.dil == a.pad && (pown == a.P - 1 || pown == (a.P - 1) / 2);
}

hipError_t launch_dw_fwd_wave(const DwArgs& a, hipStream_t s) {
  const bool causal = a.pad / a.dil == WV_P - 1;
  const dim3 grid(dw_blocks(a)), blk(256);
  if (a.norm == NORM_GLN) {
    if (causal) hipLaunchKernelGGL((dw_fwd_wave_kernel<NORM_GLN, true>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((dw_fwd_wave_kernel<NORM_GLN, false>), grid, blk, 0, s, a);
  } else {
    if (causal) hipLaunchKernelGGL((dw_fwd_wave_kernel<NORM_CLN, true>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((dw_fwd_wave_kernel<NORM_CLN, false>), grid, blk, 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_dw_bwd_wave(const DwArgs& a, hipStream_t s) {
  const bool causal = a.pad / a.dil == WV_P - 1;
  const dim3 grid(dw_blocks(a)), blk(256);
  if (a.norm == NORM_GLN) {
    if (causal) hipLaunchKernelGGL((dw_bwd_wave_kernel<NORM_GLN, true>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((dw_bwd_wave_kernel<NORM_GLN, false>), grid, blk, 0, s, a);
  } else {
    if (causal) hipLaunchKernelGGL((dw_bwd_wave_kernel<NORM_CLN, true>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((dw_bwd_wave_kernel<NORM_CLN, false>), grid, blk, 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace ctn
