// Shared device helpers for the gfx950 (CDNA4) kernel library.
//
// Everything here is written for wave64 / MFMA hardware directly: bf16 values
// travel as raw 16-bit patterns (ushort) so loads vectorise to 16 B/lane, and
// reductions are 64-lane butterflies.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

#define LK_DEVICE __device__ __forceinline__

typedef unsigned short bf16_t;  // raw bf16 bits
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned int uint4_t __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

LK_DEVICE float bf2f(bf16_t v) { return __uint_as_float(((unsigned)v) << 16); }

// round-to-nearest-even f32 -> bf16: gfx950 has v_cvt_pk_bf16_f32, which the
// __bf16 cast lowers to (NaN stays NaN, unlike the integer rounding trick).
LK_DEVICE bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

// two f32 -> one dword of 2 x bf16 (lo in bits 0-15): a vector conversion lowers to ONE
// v_cvt_pk_bf16_f32 (two scalar casts cost two converts + a shift + an or)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float floatx2_t __attribute__((ext_vector_type(2)));
LK_DEVICE unsigned pack_bf2(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((floatx2_t){lo, hi}, bf16x2_t));
}

LK_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

LK_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x = NW*64; `red` must hold NW floats.
template <int NW>
LK_DEVICE float block_sum(float v, float* red) {
  v = wave_sum(v);
  if constexpr (NW == 1) {
    return v;
  } else {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) t += red[i];
    return t;
  }
}

// 8 x bf16 <-> 8 x f32 through one 16-byte access
LK_DEVICE void load8(const bf16_t* p, float* f) {
  short8 v = *reinterpret_cast<const short8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf2f((bf16_t)v[i]);
}
LK_DEVICE void store8(bf16_t* p, const float* f) {
  short8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (short)f2bf(f[i]);
  *reinterpret_cast<short8*>(p) = v;
}

// Activations shared by the elementwise kernels and the GEMM epilogues.
LK_DEVICE float lk_silu(float x) { return x / (1.f + __expf(-x)); }
// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below bf16's 2^-9): one
// hardware exp + one reciprocal + a 5-term Horner polynomial.  The library erff made the
// GELU kernel VALU-bound at ~3.4 TB/s (benchmarks/kernel_bench.py act).
LK_DEVICE float lk_fast_erf(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float y = 1.f - p * t * __expf(-a * a);
  return copysignf(y, x);
}
LK_DEVICE float lk_gelu_erf(float x) { return 0.5f * x * (1.f + lk_fast_erf(x * 0.70710678118654752f)); }
// The same GELU on two values: the polynomial and the products as packed fp32 ops (v_pk_fma_f32 /
// v_pk_mul_f32, two values per issue) around the two scalar transcendentals -- the epilogue of the
// encoder's bias + GELU projection was VALU-bound (+19 % over the bias epilogue at K 768:
// benchmarks/epi_cost.py)
typedef float lk_f2 __attribute__((ext_vector_type(2)));
LK_DEVICE lk_f2 lk_gelu_erf2(lk_f2 x) {
  const lk_f2 z = x * 0.70710678118654752f;
  const lk_f2 a = __builtin_elementwise_abs(z);
  const lk_f2 d = __builtin_elementwise_fma(a, (lk_f2){0.3275911f, 0.3275911f}, (lk_f2){1.f, 1.f});
  const lk_f2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  lk_f2 p = __builtin_elementwise_fma((lk_f2){1.061405429f, 1.061405429f}, t, (lk_f2){-1.453152027f, -1.453152027f});
  p = __builtin_elementwise_fma(p, t, (lk_f2){1.421413741f, 1.421413741f});
  p = __builtin_elementwise_fma(p, t, (lk_f2){-0.284496736f, -0.284496736f});
  p = __builtin_elementwise_fma(p, t, (lk_f2){0.254829592f, 0.254829592f});
  const lk_f2 na = -(a * a);
  const lk_f2 e = {__expf(na.x), __expf(na.y)};
  const lk_f2 y = 1.f - p * t * e;
  const lk_f2 erf = {copysignf(y.x, z.x), copysignf(y.y, z.y)};
  return 0.5f * x * (1.f + erf);
}

// Bijective XCD-aware remap of a flat workgroup id (8 XCDs, round-robin dispatch):
// consecutive logical tiles land on the same XCD so they share its L2.
LK_DEVICE int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Launch failures are loud: a rejected launch (bad grid / block / LDS request) returns a
// distinct code that the bindings turn into a Python exception (bindings.cpp CHECK_RC), never
// a "successful" op over an uninitialised output.
// (the codes kLkLaunchError / kLkAttrError are in kernels.h, shared with the bindings)
// first refused kernel attribute of the process (sticky: the kernel it belongs to cannot run)
inline hipError_t& lk_attr_error() {
  static hipError_t e = hipSuccess;
  return e;
}
#define LK_CHECK_LAUNCH()                                                           \
  do {                                                                              \
    const hipError_t lk_e_ = hipGetLastError();                                     \
    if (lk_attr_error() != hipSuccess) return kLkAttrError - (int)lk_attr_error(); \
    if (lk_e_ != hipSuccess) return kLkLaunchError - (int)lk_e_;                    \
  } while (0)
// One-time dynamic-LDS opt-in of a kernel, its result kept: a refusal is reported by the
// launch's LK_CHECK_LAUNCH instead of surfacing as an unexplained launch failure.
#define LK_SET_MAX_LDS(kern, bytes)                                                                     \
  do {                                                                                                  \
    static const hipError_t lk_attr_ = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),        \
                                                           hipFuncAttributeMaxDynamicSharedMemorySize, \
                                                           (int)(bytes));                              \
    if (lk_attr_ != hipSuccess) lk_attr_error() = lk_attr_;                                             \
  } while (0)

// Device-side bounds checks for debug builds (`python csrc/build.py --debug`, objects
// under build/csrc-debug): a failing check traps the wave with the kernel's file/line
// instead of silently reading or writing out of range.  Compiled out otherwise.
#ifdef LK_DEBUG
#include <cassert>
#define LK_DASSERT(cond) assert(cond)
#else
#define LK_DASSERT(cond) ((void)0)
#endif
