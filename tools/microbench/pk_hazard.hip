// Packed-FP32 VALU hazard probe (gfx950).  Each test runs a short hand-written
// instruction sequence (inline asm, fixed registers, no compiler scheduling) in every
// lane of many waves, while other waves of the same workgroup keep the SIMDs busy
// (MFMA and VALU), and counts lanes whose result is not the value the sequence
// defines.  Not part of the library: it decides which instruction pairs need a wait
// state.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

// Each test: inputs a, b, c (per lane), output r (2 floats); `expect` computed on the host.
//   T0 WAR src0.hi : v_pk_fma_f32 D, S0, S1, 0 ; v_mov S0.hi <- c            (D = a*b, b*b? see below)
//   T1 WAR src1.hi : v_pk_mul_f32 D, S0, S1    ; v_mov S1.hi <- c
//   T2 WAR src0.lo : v_pk_mul_f32 D, S0, S1    ; v_mov S0.lo <- c
//   T3 RAW D.hi    : v_pk_mul_f32 D, S0, S1    ; v_mov r <- D.hi
//   T4 RAW chain   : v_pk_mul_f32 D, S0, S1    ; v_pk_fma_f32 E, D, S1, 0
//   T5 WAR pk->pk  : v_pk_fma_f32 D, S0, S1, 0 ; v_pk_mul_f32 S0, S1, S1       (overwrite both halves of S0)
//   T6             : as T5 with s_nop 0 between
//   T7 WAR both    : v_pk_fma_f32 D, S0, S1, 0 ; v_mov S0.hi <- c ; v_mov S0.lo <- c
template <int T>
__device__ void probe(float a, float b, float c, float& r0, float& r1) {
  float x0, x1;
  if constexpr (T == 0) {
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %3\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %3\n\ts_nop 7\n\t"
        "v_pk_fma_f32 v[204:205], v[200:201], v[202:203], 0\n\t"
        "v_mov_b32 v201, %4\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v204\n\tv_mov_b32 %1, v205\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205");
  } else if constexpr (T == 1) {
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %3\n\ts_nop 7\n\t"
        "v_pk_mul_f32 v[204:205], v[200:201], v[202:203]\n\t"
        "v_mov_b32 v203, %4\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v204\n\tv_mov_b32 %1, v205\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205");
  } else if constexpr (T == 2) {
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %3\n\ts_nop 7\n\t"
        "v_pk_mul_f32 v[204:205], v[200:201], v[202:203]\n\t"
        "v_mov_b32 v200, %4\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v204\n\tv_mov_b32 %1, v205\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205");
  } else if constexpr (T == 3) {
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %3\n\ts_nop 7\n\t"
        "v_pk_mul_f32 v[204:205], v[200:201], v[202:203]\n\t"
        "v_mov_b32 %1, v205\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v204\n\t"
        : "=v"(x0), "=&v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205");
  } else if constexpr (T == 4) {
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %3\n\ts_nop 7\n\t"
        "v_pk_mul_f32 v[204:205], v[200:201], v[202:203]\n\t"
        "v_pk_fma_f32 v[206:207], v[204:205], v[202:203], 0\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v206\n\tv_mov_b32 %1, v207\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207");
  } else if constexpr (T == 5) {
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %3\n\ts_nop 7\n\t"
        "v_pk_fma_f32 v[204:205], v[200:201], v[202:203], 0\n\t"
        "v_pk_mul_f32 v[200:201], v[202:203], v[202:203]\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v204\n\tv_mov_b32 %1, v205\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205");
  } else if constexpr (T == 6) {
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %3\n\ts_nop 7\n\t"
        "v_pk_fma_f32 v[204:205], v[200:201], v[202:203], 0\n\t"
        "s_nop 0\n\t"
        "v_pk_mul_f32 v[200:201], v[202:203], v[202:203]\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v204\n\tv_mov_b32 %1, v205\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205");
  } else if constexpr (T == 7) {
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %3\n\ts_nop 7\n\t"
        "v_pk_fma_f32 v[204:205], v[200:201], v[202:203], 0\n\t"
        "v_mov_b32 v201, %4\n\t"
        "v_mov_b32 v200, %4\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v204\n\tv_mov_b32 %1, v205\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205");
  } else if constexpr (T == 8) {   // src2 written by the previous VALU, read with op_sel_hi 0
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %4\n\ts_nop 7\n\t"
        "v_mul_f32_e64 v204, v203, -v202\n\t"
        "v_pk_fma_f32 v[206:207], v[200:201], v[202:203], v[204:205] op_sel:[0,1,0] op_sel_hi:[1,1,0]\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v206\n\tv_mov_b32 %1, v207\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207");
  } else if constexpr (T == 9) {   // src1.hi written by the previous VALU, broadcast by op_sel
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v204, %4\n\tv_mov_b32 v205, %4\n\ts_nop 7\n\t"
        "v_mul_f32_e32 v203, v202, v202\n\t"
        "v_pk_fma_f32 v[206:207], v[200:201], v[202:203], v[204:205] op_sel:[0,1,0] op_sel_hi:[1,1,0]\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v206\n\tv_mov_b32 %1, v207\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207");
  } else if constexpr (T == 12 || T == 13 || T == 14) {   // T8 with 1 / 2 wait states, or an independent VALU between
    if constexpr (T == 12)
      asm volatile(
          "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %4\n\ts_nop 7\n\t"
          "v_mul_f32_e64 v204, v203, -v202\n\ts_nop 0\n\t"
          "v_pk_fma_f32 v[206:207], v[200:201], v[202:203], v[204:205] op_sel:[0,1,0] op_sel_hi:[1,1,0]\n\t"
          "s_nop 7\n\tv_mov_b32 %0, v206\n\tv_mov_b32 %1, v207\n\t"
          : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207");
    else if constexpr (T == 13)
      asm volatile(
          "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %4\n\ts_nop 7\n\t"
          "v_mul_f32_e64 v204, v203, -v202\n\ts_nop 1\n\t"
          "v_pk_fma_f32 v[206:207], v[200:201], v[202:203], v[204:205] op_sel:[0,1,0] op_sel_hi:[1,1,0]\n\t"
          "s_nop 7\n\tv_mov_b32 %0, v206\n\tv_mov_b32 %1, v207\n\t"
          : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207");
    else
      asm volatile(
          "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %4\n\ts_nop 7\n\t"
          "v_mul_f32_e64 v204, v203, -v202\n\tv_mov_b32 v208, v200\n\t"
          "v_pk_fma_f32 v[206:207], v[200:201], v[202:203], v[204:205] op_sel:[0,1,0] op_sel_hi:[1,1,0]\n\t"
          "s_nop 7\n\tv_mov_b32 %0, v206\n\tv_mov_b32 %1, v207\n\t"
          : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208");
  } else if constexpr (T == 15) {   // T8 without op_sel: src2 pair (v204, v205) both written, plain packed read
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %4\n\tv_mov_b32 v203, %4\n\tv_mov_b32 v205, 0\n\ts_nop 7\n\t"
        "v_mul_f32_e64 v204, v203, -%3\n\tv_mul_f32_e64 v205, v203, -%3\n\t"
        "v_pk_fma_f32 v[206:207], v[200:201], v[202:203], v[204:205]\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v206\n\tv_mov_b32 %1, v207\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207");
  } else if constexpr (T == 10) {   // src0 pair written by the previous packed VALU
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %2\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %3\n\ts_nop 7\n\t"
        "v_pk_mul_f32 v[204:205], v[200:201], v[202:203]\n\t"
        "v_pk_fma_f32 v[206:207], v[204:205], v[202:203], 0 op_sel_hi:[1,1,0]\n\t"
        "v_pk_mul_f32 v[204:205], v[202:203], v[202:203]\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v206\n\tv_mov_b32 %1, v207\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c) : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207");
  } else if constexpr (T == 11) {   // the compiler's epilogue sequence (ah, ga, q)
    asm volatile(
        "v_mov_b32 v200, %2\n\tv_mov_b32 v201, %3\n\tv_mov_b32 v202, %3\n\tv_mov_b32 v203, %2\n\t"
        "v_mov_b32 v208, %2\n\tv_mov_b32 v209, %3\n\ts_nop 7\n\t"
        "v_mul_f32_e64 v204, v203, -v202\n\t"
        "v_pk_fma_f32 v[206:207], v[200:201], v[202:203], v[204:205] op_sel:[0,1,0] op_sel_hi:[1,1,0]\n\t"
        "v_pk_mul_f32 v[210:211], v[208:209], v[200:201]\n\t"
        "v_lshlrev_b32_e32 v212, 16, v201\n\t"
        "v_and_b32_e32 v213, 0xffff0000, v201\n\t"
        "v_pk_fma_f32 v[206:207], v[210:211], v[206:207], 0 op_sel_hi:[1,1,0]\n\t"
        "v_pk_mul_f32 v[210:211], v[208:209], v[212:213]\n\t"
        "s_nop 7\n\tv_mov_b32 %0, v206\n\tv_mov_b32 %1, v207\n\t"
        : "=v"(x0), "=v"(x1) : "v"(a), "v"(b), "v"(c)
        : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213");
  }
  r0 = x0;
  r1 = x1;
}

template <int T>
__global__ __launch_bounds__(512) void probe_kernel(const float* in, float* out, unsigned* bad, int iters, int busy) {
  const int tid = threadIdx.x, wid = tid >> 6;
  if (wid >= 4 && busy) {   // co-resident load on the same SIMDs: MFMA + VALU
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    bf16x8 av = {1, 2, 3, 4, 5, 6, 7, 8};
    float v = in[tid];
    for (int i = 0; i < iters * 4; ++i) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, av, acc, 0, 0, 0);
      v = v * 1.0001f + 0.5f;
    }
    out[(size_t)gridDim.x * 512 * 2 + blockIdx.x * 512 + tid] = acc[0] + v;
    return;
  }
  const size_t g = (size_t)blockIdx.x * 512 + tid;
  const float a = in[g % 4096], b = in[(g + 7) % 4096], c = in[(g + 13) % 4096] + 100.f;
  // Each iteration must reproduce the first one's result bit for bit (no compiler
  // arithmetic on the results: the expectations are checked on the host from out[]).
  unsigned nb = 0;
  float f0 = 0.f, f1 = 0.f;
  for (int i = 0; i < iters; ++i) {
    float r0, r1;
    probe<T>(a, b, c, r0, r1);
    if (i == 0) { f0 = r0; f1 = r1; }
    nb += (__float_as_uint(r0) != __float_as_uint(f0)) | (__float_as_uint(r1) != __float_as_uint(f1)) ? 1u : 0u;
  }
  if (nb) atomicAdd(bad, nb);
  out[g * 2] = f0;
  out[g * 2 + 1] = f1;
}

template <int T> void run(const float* in, float* out, unsigned* bad, int busy) {
  CK(hipMemset(bad, 0, 4));
  const int grid = 1024, iters = 2000;
  hipLaunchKernelGGL(probe_kernel<T>, dim3(grid), dim3(512), 0, 0, in, out, bad, iters, busy);
  CK(hipDeviceSynchronize());
  unsigned h;
  CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
  // first-iteration results against the sequence's definition (host arithmetic)
  static float hin[4096];
  CK(hipMemcpy(hin, in, sizeof hin, hipMemcpyDeviceToHost));
  float* ho = (float*)malloc((size_t)grid * 512 * 2 * 4);
  CK(hipMemcpy(ho, out, (size_t)grid * 512 * 2 * 4, hipMemcpyDeviceToHost));
  long wrong_first = 0;
  for (long gi = 0; gi < (long)grid * 512; ++gi) {
    if (busy && (gi % 512) >= 256) continue;
    const float a = hin[gi % 4096], b = hin[(gi + 7) % 4096];
    float e0 = a * b, e1 = a * b;
    if (T == 0) e1 = b * b;
    const float c = hin[(gi + 13) % 4096] + 100.f;
    if (T == 4) { e0 = fmaf(a * b, b, 0.f); e1 = e0; }
    if (T == 8 || T == 12 || T == 13 || T == 14 || T == 15) { e0 = e1 = fmaf(a, c, -(c * b)); }
    if (T == 9) { e0 = e1 = fmaf(a, b * b, c); }
    if (T == 10) { e0 = e1 = fmaf(a * b, b, 0.f); }
    if (T == 11) {
      const float ah0 = fmaf(a, b, -(a * b)), ah1 = fmaf(b, b, -(a * b));   // lo: v200*v203(hi=a) ...
      (void)ah0; (void)ah1;
      e0 = e1 = 0.f;   // self-consistency only (first-iteration check skipped)
    }
    if (T != 11) wrong_first += ho[gi * 2] != e0 || ho[gi * 2 + 1] != e1;
  }
  free(ho);
  const double n = (double)grid * (busy ? 256 : 512) * iters;
  printf("T%d busy=%d: %u iterations differ from the first of %.0f (%.3g); first iteration wrong in %ld lanes\n",
         T, busy, h, n, h / n, wrong_first);
}

int main() {
  float *in, *out;
  unsigned* bad;
  CK(hipMalloc(&in, 4096 * 4));
  CK(hipMalloc(&out, 1024L * 512 * 3 * 4));
  CK(hipMalloc(&bad, 4));
  float h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = 0.5f + (float)((i * 2654435761u) % 1000) / 997.f;
  CK(hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice));
  for (int busy = 1; busy < 2; ++busy) {
    run<0>(in, out, bad, busy);
    run<1>(in, out, bad, busy);
    run<2>(in, out, bad, busy);
    run<3>(in, out, bad, busy);
    run<4>(in, out, bad, busy);
    run<5>(in, out, bad, busy);
    run<6>(in, out, bad, busy);
    run<7>(in, out, bad, busy);
    run<8>(in, out, bad, busy);
    run<9>(in, out, bad, busy);
    run<10>(in, out, bad, busy);
    run<11>(in, out, bad, busy);
    run<12>(in, out, bad, busy);
    run<13>(in, out, bad, busy);
    run<14>(in, out, bad, busy);
    run<15>(in, out, bad, busy);
  }
  return 0;
}
