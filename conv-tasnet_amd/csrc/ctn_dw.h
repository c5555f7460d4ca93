// Comb geometry of the depthwise kernels, shared by the generic lane-group kernels
// (ctn_tcn.hip) and the wave-item kernels (ctn_dw_wave.hip).
#pragma once
#include "ctn_common.h"
#include "ctn_kernels.h"

namespace ctn {

// ---------------------------------------------------------------------------
// Comb decomposition of the dilated depthwise conv.  Rows of one utterance are
// split into residue classes rho mod d; a work item walks rows rho + j*d for
// j in one segment of a.seg steps (dw_seg).  A lane group of H/8 lanes owns one item and
// all H channels of its rows (8 per lane, 16-byte vectors); the P taps of a
// row are consecutive comb steps, so they live in a sliding register window:
// every row is loaded and transformed once (plus P-1 halo rows per segment)
// and the next row is prefetched while the current one is computed.
// ---------------------------------------------------------------------------
struct CombGeom {
  int cg, ipw, jmax, nseg, items, wgpu;
};
__host__ __device__ inline CombGeom comb_geom(const DwArgs& a) {
  CombGeom g;
  g.cg = a.H / 8;
  g.ipw = 4 * (64 / g.cg);
  g.jmax = (a.g.Kp + a.dil - 1) / a.dil;
  g.nseg = (g.jmax + a.seg - 1) / a.seg;
  g.items = a.dil * g.nseg;
  g.wgpu = (g.items + g.ipw - 1) / g.ipw;
  return g;
}

// cLN per-row sums of a comb walk.  With H = 512 one wave owns one comb item (its 64
// lanes hold all channels of each row), so a row's sums are reduced with DPP (no LDS
// round trips), parked one row per lane, and every 64 rows each lane finishes the row
// it holds: the fp64 finishing arithmetic runs once per 64 rows, not once per row.
// Narrower H (several items per wave) reduces per row over the lane group as before.
struct RowPark {
  float s = 0.f, ss = 0.f;
  int j0;   // comb step held by lane 0
};

// column-partial reduction: sum val[8] over the lanes that own channel group c, write H floats
CTN_DEV void col_reduce8(float* buf, const float v[8], int rl, int c, int nrl, int cg, bool act, float* dst) {
  const int H = cg * 8;
  if (act)
#pragma unroll
    for (int e = 0; e < 8; ++e) buf[rl * H + c * 8 + e] = v[e];
  __syncthreads();
  for (int ch = threadIdx.x; ch < H; ch += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < nrl; ++q) s += buf[q * H + ch];
    dst[ch] = s;
  }
  __syncthreads();
}

}  // namespace ctn
