// Store-pattern calibration (bound-finding only, not part of the library): 102400 rows x
// 256 bf16 channels written (a) as whole rows (each wave instruction writes 1 KiB
// contiguous), (b) as the WS GEMM epilogue writes them (a wave instruction covers 16
// rows x 64 B: lane group lg -> 16 B at channel 8*lg of a 32-channel slice), and (c)
// 16 rows x 32 B (8-byte lanes).  Also with a concurrent read stream of the same size.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)
constexpr long ROWS = 102400;
constexpr int CH = 256;   // bf16 channels per row -> 512 B rows
// grid-stride over 16-row tiles; 8 waves per block, wave w owns channel slice w (32 ch = 64 B)
template <int MODE, bool RD>
__global__ __launch_bounds__(512) void st_kernel(v4u* out, const v4u* in) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long ntile = ROWS / 16;
  v4u acc = {0u, 0u, 0u, 0u};
  for (long t = blockIdx.x; t < ntile; t += gridDim.x) {
    v4u v = {(unsigned)t, (unsigned)lane, 1u, 2u};
    if (RD) { v += in[t * 16 * CH / 8 + threadIdx.x]; }
    if (MODE == 0) {          // contiguous: thread i -> 16 B at i within the 8 KiB tile
      out[t * 16 * CH / 8 + threadIdx.x] = v;
    } else if (MODE == 1) {   // WS epilogue: row lane&15, 16 B at channel w*32 + 8*(lane>>4)
      const long r = t * 16 + (lane & 15);
      out[(r * CH + w * 32 + 8 * (lane >> 4)) / 8] = v;
    } else {                  // 8-byte lanes, 16 rows x 32 B per instruction, two instructions
      const long r = t * 16 + (lane & 15);
      v2u* o2 = reinterpret_cast<v2u*>(out);
      o2[(r * CH + w * 32 + 4 * (lane >> 4)) / 4] = v2u{v[0], v[1]};
      o2[(r * CH + w * 32 + 16 + 4 * (lane >> 4)) / 4] = v2u{v[2], v[3]};
    }
  }
  if (acc[0] == 12345u) out[0] = acc;
}
template <int MODE, bool RD> void run(const char* name, v4u* out, const v4u* in) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int grid : {256, 512, 2048}) {
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((st_kernel<MODE, RD>), dim3(grid), dim3(512), 0, 0, out, in);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((st_kernel<MODE, RD>), dim3(grid), dim3(512), 0, 0, out, in);
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 20, by = ROWS * CH * 2.0 * (RD ? 2 : 1);
    printf("%-28s grid %5d %7.1f us %6.0f GB/s\n", name, grid, us, by / us / 1e3);
  }
}
int main() {
  v4u *out, *in;
  CK(hipMalloc(&out, ROWS * CH * 2)); CK(hipMalloc(&in, ROWS * CH * 2));
  CK(hipMemset(in, 0, ROWS * CH * 2));
  run<0, false>("whole rows", out, in);
  run<1, false>("16 rows x 64 B (WS)", out, in);
  run<2, false>("16 rows x 32 B (8-B lanes)", out, in);
  run<0, true>("whole rows + read", out, in);
  run<1, true>("WS pattern + read", out, in);
  return 0;
}
