// qtx_common.h — device helpers shared by every qtx kernel (gfx950 / CDNA4, wave64).
//
// Numerics contract: the library is compiled with -ffp-contract=off and
// HIP's default correctly-rounded fp32 '/' and sqrtf, so every elementwise float step is
// one IEEE operation in a fixed order.  Reductions use the fixed trees below.  The numpy
// oracle (oracle/qtx_oracle.py) evaluates the same order, so results agree bit-for-bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#define QTX_WAVE 64

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// In-kernel phase stamps for diagnosis (tools/kernel_bench.py --stamps): compiled in only
// with -DQTX_STAMPS; thread 0 of each block records s_memtime at phase boundaries into
// qtx_stamp_buf[block][slot] (a device buffer of its own; never read by the kernels).
#ifdef QTX_STAMPS
// one buffer pointer per translation unit; each .hip that stamps exports a setter
// qtx_debug_set_stamps_<unit> (QTX_STAMP_SETTER below)
static __device__ unsigned long long* qtx_stamp_buf;
#define QTX_STAMP_SETTER(unit)                                                            \
  extern "C" int qtx_debug_set_stamps_##unit(void* buf) {                                 \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(qtx_stamp_buf), &buf, sizeof(buf));          \
  }
#define QTX_STAMP(slot)                                                                 \
  do {                                                                                    \
    if (threadIdx.x == 0 && qtx_stamp_buf)                                                \
      qtx_stamp_buf[(blockIdx.y * gridDim.x + blockIdx.x) * 16 + (slot)] =                \
          __builtin_amdgcn_s_memtime();                                                   \
  } while (0)
// accumulated phase times: QTX_NOW() reads the clock, QTX_STAMP_VAL stores a value
#define QTX_NOW() ((long long)__builtin_amdgcn_s_memtime())
// the constant 100 MHz clock: in-kernel clock = delta(QTX_NOW) / delta(QTX_RNOW) x 100 MHz
#define QTX_RNOW() ((long long)__builtin_amdgcn_s_memrealtime())
#define QTX_STAMP_VAL(slot, v)                                                          \
  do {                                                                                    \
    if (threadIdx.x == 0 && qtx_stamp_buf)                                                \
      qtx_stamp_buf[(blockIdx.y * gridDim.x + blockIdx.x) * 16 + (slot)] = (v);           \
  } while (0)
#else
#define QTX_STAMP_SETTER(unit)
#define QTX_STAMP(slot) \
  do {                  \
  } while (0)
#define QTX_NOW() 0LL
#define QTX_RNOW() 0LL
#define QTX_STAMP_VAL(slot, v) \
  do {                         \
  } while (0)
#endif

namespace qtx {

// VM_CNT_ORDER.  On gfx950 (as on every GFX9 target) loads and stores share vmcnt, and a
// store may retire before a load issued ahead of it; only loads retire in issue order
// among themselves (LLVM's SIInsertWaitcnts treats a counter with both pending as out of
// order).  So a hand-counted "s_waitcnt vmcnt(N)" that waits for an LDS-DMA is exact only
// when the N newest operations are loads; with stores behind the DMA it must be vmcnt(0).
// The weight-stationary kernels once counted the stores behind their DMA (vmcnt(3)): two
// encodes on two streams then read blocks whose DMA had not landed (wrong whole sentences
// in ~1 of 6 runs, tests/test_gpu_configs.py two_threads, tools/conc_encode_diag.py).

// ---------------------------------------------------------------- wave reductions
// Canonical sum of 64 lane values = the balanced pairwise tree over lanes in natural
// order: ((l0+l1)+(l2+l3)) ... — what an xor-butterfly computes in every lane.
// Implemented with DPP (VALU, no LDS round trip): xor1 / xor2 by quad_perm, then
// half-mirror (pairs the two quads of an 8-lane group) and mirror (the two octets of a
// 16-lane row) — once groups are uniform a mirror pairs the same two partial sums as an
// xor would — and the four row sums combined as (r0 + r1) + (r2 + r3) via readlane.
// fp32 addition is commutative, so the result is bit-identical to the oracle's
// butterfly (oracle/qtx_oracle.py:_butterfly).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_sum(float v) {
  v = v + dpp<0xB1>(v);    // quad_perm [1,0,3,2]  (xor 1)
  v = v + dpp<0x4E>(v);    // quad_perm [2,3,0,1]  (xor 2)
  v = v + dpp<0x141>(v);   // row_half_mirror      (xor 4 on uniform quads)
  v = v + dpp<0x140>(v);   // row_mirror           (xor 8 on uniform octets)
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x141>(v));
  v = fmaxf(v, dpp<0x140>(v));
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

// wave_sum / wave_max of R values at once, level by level: the R DPP chains interleave
// instead of each waiting out its own DPP and readlane latencies (the compiler kept
// per-value calls serial, with s_nop between dependent DPP adds).  Bit-identical to R calls.
template <int R>
__device__ __forceinline__ void wave_sum_n(float (&v)[R]) {
#pragma unroll
  for (int j = 0; j < R; ++j) v[j] = v[j] + dpp<0xB1>(v[j]);
#pragma unroll
  for (int j = 0; j < R; ++j) v[j] = v[j] + dpp<0x4E>(v[j]);
#pragma unroll
  for (int j = 0; j < R; ++j) v[j] = v[j] + dpp<0x141>(v[j]);
#pragma unroll
  for (int j = 0; j < R; ++j) v[j] = v[j] + dpp<0x140>(v[j]);
#pragma unroll
  for (int j = 0; j < R; ++j) v[j] = (lane_f(v[j], 0) + lane_f(v[j], 16)) + (lane_f(v[j], 32) + lane_f(v[j], 48));
}
template <int R>
__device__ __forceinline__ void wave_max_n(float (&v)[R]) {
#pragma unroll
  for (int j = 0; j < R; ++j) v[j] = fmaxf(v[j], dpp<0xB1>(v[j]));
#pragma unroll
  for (int j = 0; j < R; ++j) v[j] = fmaxf(v[j], dpp<0x4E>(v[j]));
#pragma unroll
  for (int j = 0; j < R; ++j) v[j] = fmaxf(v[j], dpp<0x141>(v[j]));
#pragma unroll
  for (int j = 0; j < R; ++j) v[j] = fmaxf(v[j], dpp<0x140>(v[j]));
#pragma unroll
  for (int j = 0; j < R; ++j)
    v[j] = fmaxf(fmaxf(lane_f(v[j], 0), lane_f(v[j], 16)), fmaxf(lane_f(v[j], 32), lane_f(v[j], 48)));
}

// The same trees restricted to each 16-lane DPP row: every lane of the row gets the row's
// canonical sum / max (the first four levels of wave_sum).
__device__ __forceinline__ float row16_sum(float v) {
  v = v + dpp<0xB1>(v);
  v = v + dpp<0x4E>(v);
  v = v + dpp<0x141>(v);
  return v + dpp<0x140>(v);
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x141>(v));
  return fmaxf(v, dpp<0x140>(v));
}

__device__ __forceinline__ int wave_min_i32(int v) {
  auto d = [](int x, auto ctrl) {
    return __builtin_amdgcn_update_dpp(0x7fffffff, x, decltype(ctrl)::value, 0xF, 0xF, false);
  };
  v = min(v, d(v, std::integral_constant<int, 0xB1>{}));
  v = min(v, d(v, std::integral_constant<int, 0x4E>{}));
  v = min(v, d(v, std::integral_constant<int, 0x141>{}));
  v = min(v, d(v, std::integral_constant<int, 0x140>{}));
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
__device__ __forceinline__ int wave_max_i32(int v) {
  auto d = [](int x, auto ctrl) {
    return __builtin_amdgcn_update_dpp(int(0x80000000), x, decltype(ctrl)::value, 0xF, 0xF, false);
  };
  v = max(v, d(v, std::integral_constant<int, 0xB1>{}));
  v = max(v, d(v, std::integral_constant<int, 0x4E>{}));
  v = max(v, d(v, std::integral_constant<int, 0x141>{}));
  v = max(v, d(v, std::integral_constant<int, 0x140>{}));
  return max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

// ---------------------------------------------------------------- canonical exp
// qexp(): Cody-Waite reduction + degree-7 Taylor in Horner form with fma (7 fused steps
// instead of 14 separate ones).  Identical to oracle/qtx_oracle.py:qexp (its fma32 is the
// correctly rounded fma).  x < -80 returns exactly 0.
__device__ __forceinline__ float qexp(float x) {
  // constants are the exact float32 values the oracle uses (hex literals: no
  // double-rounding ambiguity between the two sides)
  const float xc = fmaxf(x, -100.0f);                  // keeps (int)n in range
  const float n = rintf(xc * 0x1.715476p+0f);          // log2(e)
  // ln2 hi has a 15-bit significand and |n| <= 145, so n * ln2hi is exact and the fma is
  // bit-identical to the separate multiply and subtract (one VALU instead of two)
  float r = fmaf(-n, 0x1.62e4p-1f, xc);                 // ln2 hi
  r = r - n * 0x1.7f7d1cp-20f;                         // ln2 lo
  float p = 0x1.a01a02p-13f;                           // 1/5040
  p = fmaf(p, r, 0x1.6c16c2p-10f);                     // 1/720
  p = fmaf(p, r, 0x1.111112p-7f);                      // 1/120
  p = fmaf(p, r, 0x1.555556p-5f);                      // 1/24
  p = fmaf(p, r, 0x1.555556p-3f);                      // 1/6
  p = fmaf(p, r, 0.5f);
  p = fmaf(p, r, 1.0f);
  p = fmaf(p, r, 1.0f);
  const float e = ldexpf(p, (int)n);
  return x < -80.0f ? 0.0f : e;
}

// ---------------------------------------------------------------- shared-divisor division
// Correctly rounded a / b for many a sharing one divisor b (Markstein): with
// y = RN(1/b), q = RN(a*y), r = fma(-q, b, a) (exact), RN(q + r*y) == RN(a/b) provided
// nothing over/underflows.  div_ok() is that range guard; callers vote it over the wave
// and take the true division when any lane is outside (tools/ + DESIGN.md §3).
__device__ __forceinline__ float div_cr(float a, float b, float y) {
  const float q = a * y;
  const float r = fmaf(-q, b, a);
  return fmaf(r, y, q);
}
__device__ __forceinline__ bool div_ok(float a) {
  const float m = fabsf(a);
  return m == 0.0f || (m > 0x1p-60f && m < 0x1p60f);
}
// The same guard folded over many numerators without branches: track max(|a|) and
// min(|a| - 1) on the bit patterns (|a| = 0 wraps to UINT_MAX and drops out of the min),
// then test once.  ok() == AND of div_ok(a) over everything added.
struct DivRange {
  uint32_t mn = 0xffffffffu, mx = 0u;
  __device__ __forceinline__ void add(float a) {
    const uint32_t m = __float_as_uint(a) & 0x7fffffffu;
    mx = max(mx, m);
    mn = min(mn, m - 1u);
  }
  __device__ __forceinline__ bool ok() const {
    return mx < 0x5d800000u && mn >= 0x21800000u;   // |a| < 2^60, |a| > 2^-60
  }
};
__device__ __forceinline__ bool divisor_ok(float b) {
  const uint32_t m = __float_as_uint(b) & 0x7fffffffu;
  return m - 0x30800001u < 0x4e800000u - 0x30800001u;   // 2^-30 < |b| < 2^30
}

// RN(a / b) for a divisor known at compile time (y = RN(1/b) is folded): div_cr when a is
// in its range (any lane outside -> the true division, a wave-uniform vote), i.e. the IEEE
// quotient without the ~10-instruction division sequence on the dependent chain.
__device__ __forceinline__ float div_const(float a, float b) {
  const float y = 1.0f / b;
  if (__builtin_expect(__ballot(!div_ok(a)) == 0ull, 1)) return div_cr(a, b, y);
  return a / b;
}
// R of them in place behind ONE wave-uniform vote (the true division for all R when any
// is out of range: it equals div_cr wherever div_cr is exact, so the values are those of
// R div_const calls)
template <int R>
__device__ __forceinline__ void div_const_n(float (&a)[R], float b) {
  const float y = 1.0f / b;
  bool bad = false;
#pragma unroll
  for (int j = 0; j < R; ++j) bad |= !div_ok(a[j]);
  if (__builtin_expect(__ballot(bad) == 0ull, 1)) {
#pragma unroll
    for (int j = 0; j < R; ++j) a[j] = div_cr(a[j], b, y);
  } else {
#pragma unroll
    for (int j = 0; j < R; ++j) a[j] = a[j] / b;
  }
}

// RN(c / 127) for an integer-valued c in [0, 127] (a P code, attention.py's P grid) in two
// operations instead of div_cr's three or a true division: fma(c, RN(1/127), c * lo) with
// lo = RN(1/127 - RN(1/127)) = RN(1/127) * 2^-28.  Checked for every c against the exactly
// rounded quotient (rational arithmetic; tools/ and DESIGN.md §3).
__device__ __forceinline__ float div127(float c) {
  return fmaf(c, 0x1.020408p-7f, c * 0x1.020408p-35f);
}

// ---------------------------------------------------------------- quantizer
// quant_linear.py:30-43 / :5-17:  s = max(absmax, 1e-5) / qmax;  q = rint(x / s).
__device__ __forceinline__ float quant_scale(float absmax, float qmax) {
  return div_const(fmaxf(absmax, 1e-5f), qmax);
}
__device__ __forceinline__ int quant_val(float x, float s) { return (int)rintf(x / s); }
// Branch-free short forms of the scale chain for a >= 1e-5 (a row's clamped absmax), each
// equal to the IEEE operation on every such input — checked exhaustively on the GPU's own
// v_rcp_f32 (tools/probe_scale_exact.hip, profiles/r04_scale_exact.log):
//   scale127(a) = RN(a / 127): div_cr with the folded reciprocal, a scaled by 2^-64 when
//                 a >= 2^60 (exact power-of-two scaling), +inf passed through
//   rcp_cr(s)   = RN(1 / s) for s >= 1e-5 / 127: one Newton step with fma from v_rcp_f32,
//                 1 / +inf = 0
__device__ __forceinline__ float scale127(float a) {
  const bool big = a >= 0x1p60f;
  const float q = div_cr(big ? a * 0x1p-64f : a, 127.0f, 1.0f / 127.0f);
  return a == __builtin_inff() ? a : (big ? q * 0x1p64f : q);
}
__device__ __forceinline__ float rcp_cr(float s) {
  const float y0 = __builtin_amdgcn_rcpf(s);
  const float y = fmaf(fmaf(-s, y0, 1.0f), y0, y0);
  return s == __builtin_inff() ? 0.0f : y;
}

// pack 4 ints (already in [-127,127]) into one dword of int8
__device__ __forceinline__ uint32_t pack4_i8(int a, int b, int c, int d) {
  return (uint32_t)(a & 0xff) | ((uint32_t)(b & 0xff) << 8) | ((uint32_t)(c & 0xff) << 16) |
         ((uint32_t)(d & 0xff) << 24);
}

// K-panel-paired ("KP") int8 layout of an [R, K] matrix (R even, K % 64 == 0): rows 2p and
// 2p+1 of one 64-byte K chunk form one 128-byte line, lines ordered (p, chunk).  A DMA
// piece of 8 lines then fills a 16-row x 64-byte LDS tile with full-line reads, so the
// row GEMM can run a 4-stage ring of 64-byte K steps (qtx_gemm.hip, k_gemm_row<.., KP>).
__host__ __device__ __forceinline__ long kp_off(long r, long k, long K) {
  return (((r >> 1) * (K >> 6) + (k >> 6)) << 7) + ((r & 1) << 6) + (k & 63);
}

// *(T*)((char*)base + byte_off) with a 32-bit unsigned byte offset: for a wave-uniform base
// (a kernel argument) the compiler emits the scalar-base + vector-offset global load instead
// of 64-bit address arithmetic per load (in the latency-bound decode kernels the
// instructions before a kernel's loads are on its critical path)
template <class T>
__device__ __forceinline__ const T& ld_at(const T* base, unsigned byte_off) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}
template <class T>
__device__ __forceinline__ void st_at(T* base, unsigned byte_off, const T& v) {
  *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + byte_off) = v;
}

// rint(q) packed as int8 for |q| <= 2^22: RN(q + 1.5 * 2^23) is 1.5 * 2^23 + rint(q)
// (the add rounds to an integer, ties to even, exactly as rintf: 1.5 * 2^23 is even), so
// the low byte of its bit pattern is rint(q) in two's complement.  One add per value plus
// three byte permutes per 4 values, instead of rint + cvt + mask/shift/or.
__device__ __forceinline__ float rint_biased(float q) { return q + 12582912.0f; }
__device__ __forceinline__ uint32_t pack4_biased(float t0, float t1, float t2, float t3) {
  const uint32_t p01 = __builtin_amdgcn_perm(__float_as_uint(t1), __float_as_uint(t0), 0x0c0c0400u);
  const uint32_t p23 = __builtin_amdgcn_perm(__float_as_uint(t3), __float_as_uint(t2), 0x0c0c0400u);
  return __builtin_amdgcn_perm(p23, p01, 0x05040100u);
}
// min(max(rint(q), 0), 255) of four quotients packed as bytes: v_cvt_pk_u8_f32 rounds to
// nearest even, clamps to [0, 255] and maps NaN to 0 (probed against rintf + clamp on halves,
// near-halves, signed zeros, +-inf and NaN: tools/probe_cvt_pk_u8.hip).  For a quantized ReLU
// output (codes in [0, 127]) this is the ReLU, the rint and the packing in one op per value:
// rint(max(y, 0) / s) == max(rint(y / s), 0) for s > 0.
__device__ __forceinline__ uint32_t pack4_relu_u8(float q0, float q1, float q2, float q3) {
  uint32_t d = __builtin_amdgcn_cvt_pk_u8_f32(q0, 0u, 0u);
  d = __builtin_amdgcn_cvt_pk_u8_f32(q1, 1u, d);
  d = __builtin_amdgcn_cvt_pk_u8_f32(q2, 2u, d);
  return __builtin_amdgcn_cvt_pk_u8_f32(q3, 3u, d);
}
// the codes of four quotients y / s: rint and two's-complement bytes, or, for a ReLU output
// (RELU), pack4_relu_u8
template <bool RELU>
__device__ __forceinline__ uint32_t pack4_codes(float q0, float q1, float q2, float q3) {
  if constexpr (RELU) return pack4_relu_u8(q0, q1, q2, q3);
  else return pack4_biased(rint_biased(q0), rint_biased(q1), rint_biased(q2), rint_biased(q3));
}

// rint(x / s) with the correctly rounded quotient, computed as x * (1/s) except within
// 2^-13 of a rounding tie, where the true division is taken.  Exact: |x/s| <= ~127, so
// the reciprocal product is within 2^-16 of x/s and fl(x/s) within 2^-18; away from a
// tie both round to the same integer.
// The near-tie test is folded over all of a lane's values and voted across the wave, so
// the division runs behind ONE wave-uniform branch that is almost never taken.
// The reciprocal is v_rcp_f32 (within 1 ulp): r is then within 2^-15.5 of x/s, inside the
// 2^-13 tie window, so the rounding decision is unchanged.
template <int N>
__device__ __forceinline__ void quant_pack(const float* x, float s, uint32_t* out) {
  static_assert(N % 4 == 0, "groups of 4");
  // the tie test on the biased rint the packing needs anyway (as quant_rows512):
  // t = RN(r + 1.5 * 2^23), |r - (t - 1.5 * 2^23)| > 0.5 - 2^-13 is exactly
  // |frac(r) - 0.5| < 2^-13, folded with one max per value
  constexpr float BIAS = 12582912.0f;
  const float inv = __builtin_amdgcn_rcpf(s);
  float t[N];
  float dm = 0.0f;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float r = x[i] * inv;
    t[i] = r + BIAS;
    dm = fmaxf(dm, fabsf(r - (t[i] - BIAS)));
  }
  if (__builtin_expect(__ballot(dm > 0.5f - 0x1p-13f) != 0ull, 0)) {
#pragma unroll
    for (int i = 0; i < N; ++i) t[i] = x[i] / s + BIAS;
  }
#pragma unroll
  for (int i = 0; i < N / 4; ++i) out[i] = pack4_biased(t[4 * i], t[4 * i + 1], t[4 * i + 2], t[4 * i + 3]);
}
// single value per lane
__device__ __forceinline__ int quant_one(float x, float s) {
  float r = x * __builtin_amdgcn_rcpf(s);
  const bool near = fabsf((r - floorf(r)) - 0.5f) < 0x1p-13f;
  if (__builtin_expect(__ballot(near) != 0ull, 0)) r = x / s;
  return (int)rintf(r);
}

// The decoder's PV order (oracle attention_pv dec) for one (query row, dim):
// four chains, chain c over the keys j < Sk with (j >> 2) & 3 == c in key order, each
// from +0, term fma(ps(j), v(j), acc_c) with ps(j) = RN(P_j * s_v[j]) and v(j) = float(v_jd)
// supplied by the caller; summed (c0 + c1) + (c2 + c3).
template <class PSF, class VF>
__device__ __forceinline__ float pv_dec_chains(int Sk, PSF&& ps, VF&& v) {
  float c[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int g = 0; g < Sk; g += 16)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = g + 4 * q + e;
        if (j < Sk) c[q] = fmaf(ps(j), v(j), c[q]);
      }
  return (c[0] + c[1]) + (c[2] + c[3]);
}

// |x| as an order-preserving uint (for atomicMax on non-negative floats)
__device__ __forceinline__ unsigned abs_bits(float x) { return __float_as_uint(fabsf(x)); }

// LayerNorm (canonical order, layer_norm.py:12-15) of R rows of 512 floats, each held as
// 2 float4 per lane, in place.  The R rows are processed step by step together so their
// independent reduction chains overlap (ILP) instead of running one row after another.
template <int R>
__device__ __forceinline__ void ln_rows512(float (&v)[R][2][4], const float (&ga)[2][4],
                                           const float (&gb)[2][4]) {
  float mean[R], den[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    float s = v[j][0][0];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c | e) s = s + v[j][c][e];
    mean[j] = s;
  }
  wave_sum_n<R>(mean);
#pragma unroll
  for (int j = 0; j < R; ++j) mean[j] = mean[j] / 512.0f;
#pragma unroll
  for (int j = 0; j < R; ++j) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][c][e] = v[j][c][e] - mean[j];   // v now holds d
    float ss = v[j][0][0] * v[j][0][0];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c | e) ss = ss + v[j][c][e] * v[j][c][e];
    den[j] = ss;
  }
  wave_sum_n<R>(den);
  div_const_n<R>(den, 511.0f);
#pragma unroll
  for (int j = 0; j < R; ++j) den[j] = sqrtf(den[j]) + 1e-6f;
  // y = (a * d) / den + b, the division correctly rounded via div_cr (one true division
  // per row for the reciprocal), true division if any value is outside div_cr's range.
  // The range guard costs 2 VALU per value: max |a| on bit patterns (NaN / inf fail it) and
  // min |a| as floats (v_max3 / v_min3 pairs); a zero numerator fails the fast guard too,
  // and then DivRange's zero-exempt check (4 VALU per value) decides, off the common path.
  uint32_t mx = 0u;
  float mn = __builtin_inff();
#pragma unroll
  for (int j = 0; j < R; ++j) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[j][c][e] = ga[c][e] * v[j][c][e];     // numerator a * d
        mx = max(mx, __float_as_uint(v[j][c][e]) & 0x7fffffffu);
        mn = fminf(mn, fabsf(v[j][c][e]));
      }
  }
  bool dok = true;
#pragma unroll
  for (int j = 0; j < R; ++j) dok &= divisor_ok(den[j]);
  bool ok = dok && mx < 0x5d800000u && mn > 0x1p-60f;
  if (__builtin_expect(__ballot(!ok) != 0ull, 0)) {
    DivRange rg;
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) rg.add(v[j][c][e]);
    ok = dok && rg.ok();
  }
  if (__builtin_expect(__ballot(!ok) == 0ull, 1)) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const float y = 1.0f / den[j];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][c][e] = div_cr(v[j][c][e], den[j], y) + gb[c][e];
    }
  } else {
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][c][e] = v[j][c][e] / den[j] + gb[c][e];
  }
}

// the lane's LayerNorm parameters (canonical chunks 4*lane and 256 + 4*lane), loaded once
__device__ __forceinline__ void ln_params512(const float* a, const float* b, int lane,
                                             float (&ga)[2][4], float (&gb)[2][4]) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float4 ta = *reinterpret_cast<const float4*>(a + 4 * (lane + 64 * c));
    const float4 tb = *reinterpret_cast<const float4*>(b + 4 * (lane + 64 * c));
    ga[c][0] = ta.x; ga[c][1] = ta.y; ga[c][2] = ta.z; ga[c][3] = ta.w;
    gb[c][0] = tb.x; gb[c][1] = tb.y; gb[c][2] = tb.z; gb[c][3] = tb.w;
  }
}
template <int R>
__device__ __forceinline__ void ln_rows512(float (&v)[R][2][4], const float* a, const float* b,
                                           int lane) {
  float ga[2][4], gb[2][4];
  ln_params512(a, b, lane, ga, gb);
  ln_rows512<R>(v, ga, gb);
}

// per-token quantization of R rows (2 float4 per lane each) into int8 dwords + scales:
// rint(x / s) as quant_pack computes it, for all R rows behind ONE near-tie vote.  The tie
// test reuses the biased rint: t = RN(r + 1.5 * 2^23), d = r - (t - 1.5 * 2^23) (both
// subtractions exact for |r| < 2^22) is r's distance to the nearest integer, and
// |d| > 0.5 - 2^-13 is exactly quant_pack's |frac(r) - 0.5| < 2^-13; one v_max3 per two
// values folds it (4.5 VALU per value with the rint, against 6).
template <int R>
__device__ __forceinline__ void quant_rows512(const float (&v)[R][2][4], uint32_t (&q)[R][2],
                                              float (&sc)[R]) {
#pragma unroll
  for (int j = 0; j < R; ++j) {
    sc[j] = 0.0f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) sc[j] = fmaxf(sc[j], fabsf(v[j][c][e]));
  }
  wave_max_n<R>(sc);
#pragma unroll
  for (int j = 0; j < R; ++j) sc[j] = fmaxf(sc[j], 1e-5f);
  div_const_n<R>(sc, 127.0f);                     // quant_scale of each row
  constexpr float BIAS = 12582912.0f;
  float t[R][8];
  float dm = 0.0f;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const float inv = __builtin_amdgcn_rcpf(sc[j]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float r = v[j][i >> 2][i & 3] * inv;
      t[j][i] = r + BIAS;
      dm = fmaxf(dm, fabsf(r - (t[j][i] - BIAS)));
    }
  }
  if (__builtin_expect(__ballot(dm > 0.5f - 0x1p-13f) != 0ull, 0)) {
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) t[j][i] = v[j][i >> 2][i & 3] / sc[j] + BIAS;
  }
#pragma unroll
  for (int j = 0; j < R; ++j) {
    q[j][0] = pack4_biased(t[j][0], t[j][1], t[j][2], t[j][3]);
    q[j][1] = pack4_biased(t[j][4], t[j][5], t[j][6], t[j][7]);
  }
}

}  // namespace qtx
