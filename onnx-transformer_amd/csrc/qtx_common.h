// qtx_common.h — device helpers shared by every qtx kernel (gfx950 / CDNA4, wave64).
//
// Numerics contract: the library is compiled with -ffp-contract=off and
// HIP's default correctly-rounded fp32 '/' and sqrtf, so every elementwise float step is
// one IEEE operation in a fixed order.  Reductions use the fixed trees below.  The numpy
// oracle (oracle/qtx_oracle.py) evaluates the same order, so results agree bit-for-bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define QTX_WAVE 64

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

namespace qtx {

// ---------------------------------------------------------------- wave reductions
// xor-butterfly, offsets 32,16,8,4,2,1.  Lane l adds its partner l^off; fp32 addition
// is commutative, so every lane ends with the same value as lane 0.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// ---------------------------------------------------------------- canonical exp
// qexp(): Cody-Waite reduction + degree-7 Taylor in Horner form, no FMA.  Identical to
// oracle/qtx_oracle.py:qexp.  x < -80 returns exactly 0.
__device__ __forceinline__ float qexp(float x) {
  // constants are the exact float32 values the oracle uses (hex literals: no
  // double-rounding ambiguity between the two sides)
  const float xc = fmaxf(x, -100.0f);                  // keeps (int)n in range
  const float n = rintf(xc * 0x1.715476p+0f);          // log2(e)
  float r = xc - n * 0x1.62e4p-1f;                      // ln2 hi
  r = r - n * 0x1.7f7d1cp-20f;                         // ln2 lo
  float p = 0x1.a01a02p-13f;                           // 1/5040
  p = p * r + 0x1.6c16c2p-10f;                         // 1/720
  p = p * r + 0x1.111112p-7f;                          // 1/120
  p = p * r + 0x1.555556p-5f;                          // 1/24
  p = p * r + 0x1.555556p-3f;                          // 1/6
  p = p * r + 0.5f;
  p = p * r + 1.0f;
  p = p * r + 1.0f;
  const float e = ldexpf(p, (int)n);
  return x < -80.0f ? 0.0f : e;
}

// ---------------------------------------------------------------- quantizer
// quant_linear.py:30-43 / :5-17:  s = max(absmax, 1e-5) / qmax;  q = rint(x / s).
__device__ __forceinline__ float quant_scale(float absmax, float qmax) {
  return fmaxf(absmax, 1e-5f) / qmax;
}
__device__ __forceinline__ int quant_val(float x, float s) { return (int)rintf(x / s); }

// pack 4 ints (already in [-127,127]) into one dword of int8
__device__ __forceinline__ uint32_t pack4_i8(int a, int b, int c, int d) {
  return (uint32_t)(a & 0xff) | ((uint32_t)(b & 0xff) << 8) | ((uint32_t)(c & 0xff) << 16) |
         ((uint32_t)(d & 0xff) << 24);
}

// |x| as an order-preserving uint (for atomicMax on non-negative floats)
__device__ __forceinline__ unsigned abs_bits(float x) { return __float_as_uint(fabsf(x)); }

}  // namespace qtx
