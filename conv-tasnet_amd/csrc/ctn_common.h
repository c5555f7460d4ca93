// Common device helpers for the Conv-TasNet HIP kernels (gfx950 / CDNA4 only).
//
// Storage convention: every frame-major activation is a row
// matrix [M*Kp][C] — utterance-major, frame rows padded to Kp (a multiple of
// 128) so that no GEMM row tile straddles two utterances, channels contiguous.
// Padded rows (k >= K inside an utterance) are kept at zero by every kernel
// that writes a row tensor.  Storage type T is float (parity mode) or bf16
// (throughput mode); all arithmetic, statistics and accumulation are fp32
// (block/utterance reductions in fp64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#define CTN_DEV __device__ __forceinline__

typedef uint16_t bf16raw;
struct alignas(16) u128 { uint32_t x, y, z, w; };

CTN_DEV float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
CTN_DEV uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

// ---------------------------------------------------------------------------
// 8-element vector load/store in fp32 registers for either storage type.
// bf16: one 16-byte access; f32: two 16-byte accesses.
// ---------------------------------------------------------------------------
template <typename T> struct Vec8;

template <> struct Vec8<float> {
  static CTN_DEV void load(const float* p, float v[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static CTN_DEV void store(float* p, const float v[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

template <> struct Vec8<bf16raw> {
  static CTN_DEV void load(const bf16raw* p, float v[8]) {
    const u128 a = *reinterpret_cast<const u128*>(p);
    const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static CTN_DEV void store(bf16raw* p, const float v[8]);
};

// 16-byte register value as a first-class vector: copies of it never become
// memcpy's, so arrays of them stay in registers (a struct copy can keep an
// alloca alive in scratch or LDS).
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
// CTN_NT bits (experiment switch): 1 = 16-byte loads, 2 = 16-byte stores carry the
// nontemporal hint
#ifndef CTN_NT
#define CTN_NT 0
#endif
CTN_DEV v4u ldg16(const void* p) {
  if constexpr (CTN_NT & 1) return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  else return *reinterpret_cast<const v4u*>(p);
}
CTN_DEV void stg16(void* p, v4u v) {
  if constexpr (CTN_NT & 2) __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
  else *reinterpret_cast<v4u*>(p) = v;
}
// CTN_PART_NT: the fp32 split-K partial sums of the dual and column GEMMs (read back only
// by the reductions at the end of the backward pass) are stored with the nontemporal
// hint, so they do not evict the activations the next kernels read from the Infinity
// Cache (dw_bwd after the dual 85 -> 77 us, the dual itself +2.4, the column GEMM -1.5;
// DESIGN.md §15).  1: one dword per lane and row; 2 (experiment, slower): 16-byte
// stores after a quad transpose of the accumulators; 0: plain stores.
#ifndef CTN_PART_NT
#define CTN_PART_NT 1
#endif
template <bool NT = (CTN_PART_NT != 0)> CTN_DEV void st_part(float* p, float v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
// the same with the nontemporal hint when NT (per-kernel choice)
template <bool NT> CTN_DEV v4u ldg16h(const void* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  else return ldg16(p);
}
template <bool NT> CTN_DEV void stg16h(void* p, v4u v) {
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
  else stg16(p, v);
}
CTN_DEV void unpack_bf16x8(const v4u& v, float f[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
// two floats -> one dword of 2 bf16 (round to nearest even): one v_cvt_pk_bf16_f32
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
CTN_DEV uint32_t pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}
CTN_DEV v4u pack_bf16x8v(const float f[8]) {
  return v4u{pk_bf16(f[0], f[1]), pk_bf16(f[2], f[3]), pk_bf16(f[4], f[5]), pk_bf16(f[6], f[7])};
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations
// but NOT for its outstanding global loads/stores (__syncthreads()' release
// fence would emit vmcnt(0) and drain the prefetch in flight).
CTN_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Generation words in LDS (ring hand-offs between waves of one workgroup, no barrier):
// a wave publishes `gen` in its word of a slot after its own LDS operations on the slot
// completed (flag_signal), and a consumer polls the N words of a slot until all reach
// `gen` (flag_wait; wave-uniform by readfirstlane).  The poll is bounded (CTN_SPIN_LIMIT
// polls, ~0.2 s) so that a protocol error cannot leave a wave spinning forever; when the
// bound runs out the wave sets CTN_DEVERR_SPIN in the device error word `err` (one vector
// atomic by lane 0) and goes on, and the host reports the launch as failed
// (ctn_device_status, ctn_tblock_reduce_grads: CTN_ERR_HIP) instead of returning its
// wrong results silently.
// Volatile accesses keep their address space only through an LDS-typed pointer (a
// generic one becomes a FLAT access, whose wait drains every outstanding global load).
#ifndef CTN_SPIN_LIMIT
#define CTN_SPIN_LIMIT (1u << 22)
#endif
#ifndef CTN_DEVERR_SPIN
#define CTN_DEVERR_SPIN 1u   // a generation-word wait timed out (include/ctn.h)
#endif
CTN_DEV void spin_timeout(uint32_t* err) {
  if (err && (threadIdx.x & 63) == 0) atomicOr(err, CTN_DEVERR_SPIN);
}
typedef __attribute__((address_space(3))) volatile v4u flag_v4u;
typedef __attribute__((address_space(3))) volatile uint32_t flag_u32;
template <int N> CTN_DEV void flag_wait(const uint32_t* f, uint32_t gen, uint32_t* err) {
  static_assert(N % 4 == 0, "generation words per slot: whole 16-byte reads");
  const flag_v4u* fl = (const flag_v4u*)(f);
  uint32_t it = 0;
  for (; it < CTN_SPIN_LIMIT; ++it) {
    uint32_t mn = 0xffffffffu;
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
      const v4u a = fl[i];
      mn = min(mn, min(min(a[0], a[1]), min(a[2], a[3])));
    }
    if (__builtin_amdgcn_readfirstlane(mn) >= gen) break;
    __builtin_amdgcn_s_sleep(1);
  }
  if (it == CTN_SPIN_LIMIT) spin_timeout(err);
  asm volatile("" ::: "memory");
}
CTN_DEV void flag_signal(uint32_t* f, uint32_t gen) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  *(flag_u32*)(f) = gen;
  asm volatile("" ::: "memory");
}

// Buffer resources and LDS-DMA (the dual GEMM and the plain column GEMM)
typedef __amdgpu_buffer_rsrc_t rsrc_t;
CTN_DEV rsrc_t du_rsrc(const void* p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                           0x00020000);
}
// LDS-DMA (buffer_load ... lds) of one 16-byte (4-byte) piece per lane into the LDS
// block at the wave-uniform byte address `lds` (lane l lands at lds + 16 l).  Written
// as inline asm so that the compiler does not see an LDS write it cannot place: it
// would put a vmcnt(0) in front of every later LDS read it cannot prove disjoint,
// draining the ring.  The kernel counts these loads itself (du_vmwait).
CTN_DEV uint32_t du_ldsaddr(const char* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)p);
}
// CTN_DMA_TAIL: wait states after the LDS-DMA issue (diagnostic builds)
#ifndef CTN_DMA_TAIL
#define CTN_DMA_TAIL ""
#endif
#ifndef CTN_DMA_HEAD
#define CTN_DMA_HEAD "s_nop 0\n\t"
#endif
CTN_DEV void du_dma16(rsrc_t r, const char* lds, uint32_t voff, int soff) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\t" CTN_DMA_HEAD "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t" CTN_DMA_TAIL "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(r), "s"(du_ldsaddr(lds)), "s"(soff)
               : "memory");
}
CTN_DEV void du_dma4(rsrc_t r, const char* lds, uint32_t voff, int soff) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\t" CTN_DMA_HEAD "buffer_load_dword %1, %2, %4 offen lds\n\t" CTN_DMA_TAIL "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(r), "s"(du_ldsaddr(lds)), "s"(soff)
               : "memory");
}
constexpr uint32_t DU_OOB = 0x80000000u;   // voffset past every buffer: loads (and LDS-DMA) return 0
// s_waitcnt vmcnt(n) for a wave-uniform n (clamped down: waiting for more is safe)
CTN_DEV void du_vmwait(int n) {
  switch (n < 0 ? 0 : n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
  }
}
// the same up to vmcnt(23) (the WS GEMM's ring)
// counted wait with a compile-time count: the steady state of a DMA ring (the runtime
// switch below compiles to a chain of scalar compares and branches per call)
template <int N> CTN_DEV void vmwait_c() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
CTN_DEV void vmwait23(int n) {
#define CTN_VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n < 0 ? 0 : n) {
    CTN_VMW(0) CTN_VMW(1) CTN_VMW(2) CTN_VMW(3) CTN_VMW(4) CTN_VMW(5) CTN_VMW(6) CTN_VMW(7)
    CTN_VMW(8) CTN_VMW(9) CTN_VMW(10) CTN_VMW(11) CTN_VMW(12) CTN_VMW(13) CTN_VMW(14) CTN_VMW(15)
    CTN_VMW(16) CTN_VMW(17) CTN_VMW(18) CTN_VMW(19) CTN_VMW(20) CTN_VMW(21) CTN_VMW(22)
    default: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); break;
  }
#undef CTN_VMW
}

// 8 bf16 held in a 16-byte register value <-> 8 floats (no memory round trip)
CTN_DEV void unpack_bf16x8(const u128& v, float f[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
CTN_DEV u128 pack_bf16x8(const float f[8]) {
  u128 v;
  v.x = pk_bf16(f[0], f[1]);
  v.y = pk_bf16(f[2], f[3]);
  v.z = pk_bf16(f[4], f[5]);
  v.w = pk_bf16(f[6], f[7]);
  return v;
}
CTN_DEV void Vec8<bf16raw>::store(bf16raw* p, const float v[8]) { stg16(p, pack_bf16x8v(v)); }

// Raw 8-element vector: loaded as-is (bf16: 4 dwords, f32: 8 dwords) so many
// loads can be in flight in few registers; unpacked to fp32 at the point of use.
template <typename T> struct Raw8;
template <> struct Raw8<bf16raw> {
  u128 v;
  CTN_DEV void load(const bf16raw* p) { v = *reinterpret_cast<const u128*>(p); }
  CTN_DEV float operator[](int e) const {
    const uint32_t w = e < 2 ? v.x : e < 4 ? v.y : e < 6 ? v.z : v.w;
    return (e & 1) ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(w << 16);
  }
};
template <> struct Raw8<float> {
  float4 a, b;
  CTN_DEV void load(const float* p) {
    a = *reinterpret_cast<const float4*>(p);
    b = *reinterpret_cast<const float4*>(p + 4);
  }
  CTN_DEV float operator[](int e) const {
    return e == 0 ? a.x : e == 1 ? a.y : e == 2 ? a.z : e == 3 ? a.w : e == 4 ? b.x : e == 5 ? b.y : e == 6 ? b.z : b.w;
  }
};

// 4-element store (GEMM epilogue: one lane owns 4 consecutive output columns)
template <typename T> CTN_DEV void store4(T* p, const float v[4]);
template <> CTN_DEV void store4<float>(float* p, const float v[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <> CTN_DEV void store4<bf16raw>(bf16raw* p, const float v[4]) {
  uint2 a;
  a.x = pk_bf16(v[0], v[1]);
  a.y = pk_bf16(v[2], v[3]);
  *reinterpret_cast<uint2*>(p) = a;
}
template <typename T> CTN_DEV void load4(const T* p, float v[4]);
template <> CTN_DEV void load4<float>(const float* p, float v[4]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
template <> CTN_DEV void load4<bf16raw>(const bf16raw* p, float v[4]) {
  const uint2 a = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(a.x << 16); v[1] = __uint_as_float(a.x & 0xffff0000u);
  v[2] = __uint_as_float(a.y << 16); v[3] = __uint_as_float(a.y & 0xffff0000u);
}

template <typename T> CTN_DEV float ld1(const T* p);
template <> CTN_DEV float ld1<float>(const float* p) { return *p; }
template <> CTN_DEV float ld1<bf16raw>(const bf16raw* p) { return bf2f(*p); }
template <typename T> CTN_DEV void st1(T* p, float v);
template <> CTN_DEV void st1<float>(float* p, float v) { *p = v; }
template <> CTN_DEV void st1<bf16raw>(bf16raw* p, float v) { *p = f2bf(v); }

// ---------------------------------------------------------------------------
// activations
// ---------------------------------------------------------------------------
// nn.PReLU with one shared alpha: max(0,x) + a*min(0,x)  (conv_tasnet.py:218,253)
CTN_DEV float prelu(float x, float a) { return x > 0.f ? x : a * x; }
// d prelu / dx, with torch's convention at x == 0 (slope a)
CTN_DEV float prelu_dx(float x, float a) { return x > 0.f ? 1.f : a; }
// d prelu / da
CTN_DEV float prelu_da(float x) { return x > 0.f ? 0.f : x; }

// ---------------------------------------------------------------------------
// wave64 / block reductions
// ---------------------------------------------------------------------------
template <typename V> CTN_DEV V wave_sum(V v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// sum over lanes that share (lane % width) == const, i.e. reduce across lane / width groups
template <typename V> CTN_DEV V wave_sum_stride(V v, int width) {
  for (int o = 32; o >= width; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// sum over aligned lane groups of size `width` (power of two <= 64)
template <typename V> CTN_DEV V wave_sum_group(V v, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Wave64 sum with DPP row operations (no LDS traffic); the total is returned
// wave-uniform (read from lane 63).
template <int CTRL, int ROW_MASK> CTN_DEV float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, ROW_MASK, 0xF, false));
}
// 4x4 transpose within each quad of lanes (DPP quad_perm, no LDS): on entry lane t = lane & 3
// holds v[e] = M[e][t], on exit v[c] = M[t][c].  Every lane of a quad must be active.
CTN_DEV void quad_transpose4(float v[4]) {
  const int t = (int)(threadIdx.x & 3);
#pragma unroll
  for (int e = 0; e < 4; e += 2) {   // partner t ^ 1 (quad_perm [1,0,3,2])
    const float r = dpp_f<0xB1, 0xF>((t & 1) ? v[e] : v[e + 1]);
    if (t & 1) v[e] = r;
    else v[e + 1] = r;
  }
#pragma unroll
  for (int e = 0; e < 2; ++e) {      // partner t ^ 2 (quad_perm [2,3,0,1])
    const float r = dpp_f<0x4E, 0xF>((t & 2) ? v[e] : v[e + 2]);
    if (t & 2) v[e] = r;
    else v[e + 2] = r;
  }
}
CTN_DEV v4u f4bits(const float v[4]) {
  return v4u{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
}
CTN_DEV float wave_sum_dpp(float v) {
  v += dpp_f<0xB1, 0xF>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4E, 0xF>(v);    // quad_perm [2,3,0,1]
  v += dpp_f<0x141, 0xF>(v);   // row_half_mirror
  v += dpp_f<0x140, 0xF>(v);   // row_mirror: every lane holds its 16-lane row sum
  v += dpp_f<0x142, 0xA>(v);   // row_bcast:15 into rows 1 and 3
  v += dpp_f<0x143, 0xC>(v);   // row_bcast:31 into rows 2 and 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// Sum over the four 16-lane rows of a wave (the lanes l, l^16, l^32, l^48) with
// v_permlane16_swap / v_permlane32_swap: VALU lane exchanges, no LDS instruction
// (a kernel with LDS-DMA in flight keeps its cross-lane traffic off the LDS unit).
// Every lane ends with the same bits: a swap pair adds the same two values.
CTN_DEV float xsum_rows(float v) {
  auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(q[0]) + __uint_as_float(q[1]);   // v_l + v_{l^16}
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// fp64 wave64 sum with the same DPP row operations on both halves (no ds_bpermute:
// kernels with LDS-DMA in flight reduce this way; total read from lane 63)
template <int CTRL, int ROW_MASK> CTN_DEV double dpp_d(double x) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, ROW_MASK, 0xF, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, ROW_MASK, 0xF, false);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
CTN_DEV double wave_sum_dpp_d(double v) {
  v += dpp_d<0xB1, 0xF>(v);
  v += dpp_d<0x4E, 0xF>(v);
  v += dpp_d<0x141, 0xF>(v);
  v += dpp_d<0x140, 0xF>(v);
  v += dpp_d<0x142, 0xA>(v);
  v += dpp_d<0x143, 0xC>(v);
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, 63);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), 63);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// float2 (packed fp32: v_pk_add/mul/fma_f32 on gfx950) helpers
// IEEE maximum/minimum (NaN-propagating): one v_maximum3/v_minimum3_f32 per element on
// gfx950, where maxnum/minnum in IEEE mode also quiet each non-arithmetic input first
// (two more v_max_f32 per element)
// 0 (default): maxnum/minnum as before.  1 measured neutral (fwd1 51.5 -> 51.2 us); in
// round 2 it moved the dual GEMM's code placement into the epilogue/LDS-DMA
// reproducibility problem of DESIGN.md §10 (round 3: reproducible, profiles/r03/race)
#ifndef CTN_IEEE_MAX
#define CTN_IEEE_MAX 0
#endif
#if CTN_IEEE_MAX
CTN_DEV f32x2_t pmax(f32x2_t a, f32x2_t b) { return __builtin_elementwise_maximum(a, b); }
CTN_DEV f32x2_t pmin(f32x2_t a, f32x2_t b) { return __builtin_elementwise_minimum(a, b); }
#else
CTN_DEV f32x2_t pmax(f32x2_t a, f32x2_t b) { return __builtin_elementwise_max(a, b); }
CTN_DEV f32x2_t pmin(f32x2_t a, f32x2_t b) { return __builtin_elementwise_min(a, b); }
#endif
CTN_DEV f32x2_t pfma(f32x2_t a, f32x2_t b, f32x2_t c) { return __builtin_elementwise_fma(a, b, c); }
// PReLU with one shared alpha: max(x, a*x) when a <= 1, min(x, a*x) when a > 1 (both
// exact: the branch is chosen once per kernel, LE1 = (alpha <= 1)).  One v_max_f32 /
// v_min_f32 per element: fmaxf / fminf in IEEE mode first copy every operand not known to
// be canonical through another v_max_f32 (NaN quieting), a third of the PReLU's
// instructions; the operands here are finite activations, for which the results agree bit
// for bit.  (CTN_IEEE_MAX=1 keeps the round-2 builtin forms for A/B.)
template <bool LE1> CTN_DEV float prelu_nq(float x, float a) {
  const float ax = x * a;
  float r;
  if constexpr (LE1) asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(ax));
  else asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(ax));
  return r;
}
template <bool LE1> CTN_DEV f32x2_t prelu2(f32x2_t x, float a) {
#if CTN_IEEE_MAX
  const f32x2_t ax = x * a;
  return LE1 ? pmax(x, ax) : pmin(x, ax);
#else
  return f32x2_t{prelu_nq<LE1>(x.x, a), prelu_nq<LE1>(x.y, a)};
#endif
}

// Block-wide sum of NV doubles; result valid in thread 0.  `red` must hold
// NV * (blockDim.x / 64) doubles.  Contains __syncthreads().
template <int NV> CTN_DEV void block_sum_d(double (&v)[NV], double* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < NV; ++i) red[wid * NV + i] = v[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < nw; ++w)
#pragma unroll
      for (int i = 0; i < NV; ++i) v[i] += red[w * NV + i];
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Statistics finalized by their consumer ("folded", gLN only): instead of a
// separate finalize launch, every consumer workgroup reduces the producer's
// partials of the utterances it needs (fold_stat: one canonical order, so all
// workgroups agree bit for bit), and one designated workgroup stores the
// finalized pairs for the kernels that follow.
//
// Partial layouts:
//   dense   : slab[g * parts + i], i < parts
//   WS runs : the persistent weight-stationary GEMM (ctn_gemm_ws.hip) gives
//             workgroup b the tiles [t0(b), t0(b+1)), t0(b) = ntile*b/grid;
//             each wave accumulates the consecutive tiles of one utterance and
//             stores one partial per run: slab[((b*waves + w)*kmax + m - m0(b)],
//             m0(b) = t0(b) / tpu (tpu = tiles per utterance)
// ---------------------------------------------------------------------------
struct WsRuns {
  int ntile = 0, grid = 0, tpu = 1, waves = 0, kmax = 0;   // grid == 0: dense layout
};
__host__ __device__ inline int ws_t0(const WsRuns& w, int b) { return (int)((long)w.ntile * b / w.grid); }
// the workgroup whose range holds tile t (the last b with t0(b) <= t)
__host__ __device__ inline int ws_block_of_tile(const WsRuns& w, int t) {
  return (int)(((long)(t + 1) * w.grid + w.ntile - 1) / w.ntile) - 1;
}
__host__ __device__ inline int ws_runs_kmax(int ntile, int grid, int tpu) {
  const int twg = (ntile + grid - 1) / grid;
  return (twg + tpu - 1) / tpu + 1;
}

struct StatFold {
  const double2* slab = nullptr;   // producer partials; null: stats already final
  int parts = 0;                   // dense layout: parts per group
  double cnt = 1.0;                // elements per group
  float eps = 0.f;
  int mode = 0;                    // 0: (mean, rstd); 1: (S / cnt, SS / cnt)
  float2* out = nullptr;           // finalized pairs [G] (may be null)
  WsRuns ws;                       // WS run layout when ws.grid > 0
};

// Finalize group m, executed by a whole wave: lane l sums the group's partials
// l, l+64, ... in order, then an xor butterfly (every lane ends with the same
// bits, addition being commutative).
CTN_DEV float2 fold_stat(const StatFold& f, int m) {
  double s = 0.0, ss = 0.0;
  const int lane = (int)(threadIdx.x & 63);
  // Each lane sums its partials i = lane, lane+64, ... in that order; the loads of four
  // consecutive ones are issued together (a load-add chain would pay one memory latency
  // per partial, serially, at the start of every consumer workgroup).
  // Every round issues its (up to) four loads before any add, the last, partial round
  // too: as a serial load-add loop its one to three loads each paid a full memory
  // latency in the prologue of every weight-stationary GEMM (same summation order).
  if (f.ws.grid == 0) {
    const double2* sg = f.slab + (size_t)m * f.parts;
    for (int i = lane; i < f.parts; i += 256) {
      double2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i + 64 * u < f.parts ? sg[i + 64 * u] : make_double2(0.0, 0.0);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + 64 * u < f.parts) {
          s += v[u].x;
          ss += v[u].y;
        }
    }
  } else {
    const WsRuns& w = f.ws;
    const int blo = ws_block_of_tile(w, m * w.tpu), bhi = ws_block_of_tile(w, (m + 1) * w.tpu - 1);
    const int n = (bhi - blo + 1) * w.waves;
    auto get = [&](int i) {   // partial i of utterance m, or zero for a range that stored none
      const int b = blo + i / w.waves, wv = i % w.waves;
      const int t0 = ws_t0(w, b);
      return t0 < ws_t0(w, b + 1) ? f.slab[((size_t)b * w.waves + wv) * w.kmax + (m - t0 / w.tpu)]
                                  : make_double2(0.0, 0.0);
    };
    for (int i = lane; i < n; i += 256) {
      double2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i + 64 * u < n ? get(i + 64 * u) : make_double2(0.0, 0.0);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + 64 * u < n) {
          s += v[u].x;
          ss += v[u].y;
        }
    }
  }
  s = wave_sum(s);
  ss = wave_sum(ss);
  if (f.mode == 0) {
    const double mean = s / f.cnt;
    double var = ss / f.cnt - mean * mean;
    if (var < 0.0) var = 0.0;
    return make_float2((float)mean, (float)(1.0 / sqrt(var + (double)f.eps)));
  }
  return make_float2((float)(s / f.cnt), (float)(ss / f.cnt));
}

// ---------------------------------------------------------------------------
// normalisation statistics: layout shared by all kernels
//   gLN : one (mean, rstd) pair per utterance       index = m
//   cLN : one (mean, rstd) pair per padded frame row index = row
// ---------------------------------------------------------------------------
enum NormKind { NORM_GLN = 0, NORM_CLN = 1 };

template <int NK> CTN_DEV int stat_index(int row, int Kp) {
  return NK == NORM_GLN ? row / Kp : row;
}

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// Compile-time loop: f(std::integral_constant<int, i>{}) for i = 0 .. N-1, so that
// register-array indices derived from i stay static (register rings unrolled by
// their depth).
template <class F, int... I> CTN_DEV void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F> CTN_DEV void static_for(F&& f) { static_for_impl(f, std::make_integer_sequence<int, N>{}); }
