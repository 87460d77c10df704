// qtx_attn.hip — encoder / decoder-module attention on the matrix cores (gfx950, wave64).
//
//   s_ij = ((float(q_i . k_j) * s_q[i]) * s_k[j]) / 8     (exact int8 dot: MFMA i8)
//   masked_fill(mask == 0, -1e9); P_ij = rint(softmax_j(s_ij) * 127) / 127
//   ctx_id = fma chain over j = 0..Sk-1 of P_ij * (float(v_jd) * s_v[j])
//            (a decoder layer's attention, a.dec: four chains over interleaved 4-key groups
//            of fma(P_ij * s_v[j], float(v_jd), .), oracle attention_pv dec)
//   attention.py:23-36 (per head, 64-wide), canonical order of oracle/qtx_oracle.py.
//
// The PV chain runs on v_mfma_f32_16x16x4f32: chained over k in order (C starts at 0) it
// is bit-for-bit the k-ordered fmaf chain (the generator relies on the same fact), so the
// canonical sequential-fma PV becomes 16x16 tiles on the matrix cores instead of one
// latency-bound VALU chain per (row, dim).
//
// k_attn_mfma: workgroup = (head h, sentence b, block of 64 query rows), 4 waves, wave w
// owns query rows 16w..16w+15 of the block.  K and V (int8, per head) and their scales
// are staged in LDS once per workgroup.  Everything after that stays in registers:
// the scores are computed TRANSPOSED (S^T = K Q^T: A = 16 keys, B = the wave's 16 query
// rows) from K rows staged in the key order perm(j) (the two 2-bit fields of j & 15
// swapped), so C row 4 fg + e of key tile kt is key 16 kt + 4 e + fg: lane (fr, fg) holds
// row i = fr at keys 4 s + fg (s = 4 kt + e) — exactly the A operand of step s of the PV
// MFMA chain (row fr, k = 4 s + fg).
// Softmax reductions: 32 values in the lane, then lanes xor 16 / xor 32 (permlane swaps).
// The canonical denominator tree (oracle row_sum_lanesplit: lane-split partial of
// position L = (0 + e[L]) + e[L+64], then a 64-position xor butterfly) maps onto this
// layout as: L = 16 kt + 4 e + fg, so bits 0-1 are the lane xor 16 / xor 32 levels, bits
// 2-3 in-lane (e), bits 4-5 in-lane (kt).  Keys <= 128.
#include <cstdlib>

#include "qtx_common.h"
#include "qtx_kernels.h"
#include "qtx_knobs.h"

QTX_STAMP_SETTER(attn)

namespace qtx {

constexpr int AM_MAXK = 128;

// 64-byte K rows, slot swizzle of qtx_gemm.hip (conflict-free ds_read_b128 fragments)
__device__ __forceinline__ int am_slot(int r, int c) { return c ^ (((r >> 3) & 1) << 1); }
// staged position of key j (an involution): bits 0-1 <-> bits 2-3
__device__ __forceinline__ int am_perm(int j) { return (j & ~15) | ((j & 3) << 2) | ((j >> 2) & 3); }

// x + (x of lane ^ 16) / (lane ^ 32): one permlane swap, the pair's sum / max
__device__ __forceinline__ float xsum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xmax16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xmax32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

template <bool DEC>
__global__ __launch_bounds__(256) void k_attn_mfma(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t Ks[AM_MAXK * 64];
  __shared__ __attribute__((aligned(16))) int8_t Vs[AM_MAXK * 64];
  __shared__ __attribute__((aligned(16))) float sks[AM_MAXK];     // staged order (am_perm)
  __shared__ __attribute__((aligned(16))) float svs[AM_MAXK];     // key order
  __shared__ __attribute__((aligned(16))) uint8_t mks[AM_MAXK];   // per-key mask, staged order
  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int Sk = a.Sk, Sq = a.Sq, hoff = h * 64;
  const int nk4 = (Sk + 3) & ~3;            // keys rounded up to the PV MFMA k step
  const int r0 = blockIdx.z * 64 + wave * 16;
  QTX_STAMP(0);

  // ---- stage K, V, scales, mask for all 128 key slots (slots >= Sk zero) ----------------
  const int8_t* kb = a.k + b * a.k_bs + hoff;
  const int8_t* vb = a.v + b * a.v_bs + hoff;
  if (tid < AM_MAXK) {    // thread j stages key j: K row at perm(j), V transposed (below)
    const int j = tid, jc = min(j, Sk - 1), pj = am_perm(j);
    const bool ok = j < Sk;
    uint4 kv[4], vv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {          // clamped, unconditional loads; zeroed if j >= Sk
      kv[c] = *reinterpret_cast<const uint4*>(kb + (long)jc * a.k_ld + 16 * c);
      vv[c] = *reinterpret_cast<const uint4*>(vb + (long)jc * a.v_ld + 16 * c);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      *reinterpret_cast<uint4*>(Ks + pj * 64 + 16 * am_slot(pj, c)) = ok ? kv[c] : make_uint4(0, 0, 0, 0);
    // Vt dword (j, f) = bytes v[j][f], v[j][16+f], v[j][32+f], v[j][48+f] (f = 0..15): the PV
    // B operand of lane (f = lane & 15) for the four 16-wide dim tiles in one ds_read_b32
    uint32_t* vt = reinterpret_cast<uint32_t*>(Vs + j * 64);
    const uint32_t* w0 = reinterpret_cast<const uint32_t*>(&vv[0]);
    const uint32_t* w1 = reinterpret_cast<const uint32_t*>(&vv[1]);
    const uint32_t* w2 = reinterpret_cast<const uint32_t*>(&vv[2]);
    const uint32_t* w3 = reinterpret_cast<const uint32_t*>(&vv[3]);
#pragma unroll
    for (int f = 0; f < 16; ++f) {
      const int q = f >> 2, pb = f & 3;
      const uint32_t sel = (uint32_t)pb | ((uint32_t)(pb + 4) << 8);   // [lo.pb, hi.pb]
      const uint32_t t01 = __builtin_amdgcn_perm(w1[q], w0[q], sel);
      const uint32_t t23 = __builtin_amdgcn_perm(w3[q], w2[q], sel);
      vt[f] = ok ? __builtin_amdgcn_perm(t23, t01, 0x05040100u) : 0u;
    }
    const float skj = a.sk[b * a.sk_bs + jc], svj = a.sv[b * a.sv_bs + jc];
    sks[pj] = ok ? skj : 0.0f;
    svs[j] = ok ? svj : 0.0f;
    const bool row_mask = a.mask && a.m_is != 0;
    mks[pj] = (a.mask && !row_mask && ok) ? a.mask[b * a.m_bs + j] : (uint8_t)1;
  }
  const bool row_mask = a.mask && a.m_is != 0;   // per-query mask rows (causal decoder)
  // this wave's query fragment (MFMA B operand: query row fr, bytes 16*fg..) and row scale
  const int qrow = min(r0 + fr, Sq - 1);
  const v4i qf = *reinterpret_cast<const v4i*>(a.q + b * a.q_bs + (long)qrow * a.q_ld + hoff + 16 * fg);
  const float sqr = a.sq[b * a.sq_bs + qrow];
  __syncthreads();
  if (r0 >= Sq) return;                    // (after the only block-wide barrier)
  QTX_STAMP(1);

  // ---- scores S^T: C[staged row 4fg + e = key 16kt + 4e + fg][query fr] ------------------
  float x[8][4];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    if (16 * kt < Sk) {
      const int krow = kt * 16 + fr;
      const v4i kf = *reinterpret_cast<const v4i*>(Ks + krow * 64 + 16 * am_slot(krow, fg));
      const v4i sc4 = __builtin_amdgcn_mfma_i32_16x16x64_i8(kf, qf, v4i{0, 0, 0, 0}, 0, 0, 0);
      const int k0 = 16 * kt + 4 * fg;         // staged rows k0..k0+3
      const float4 skv = *reinterpret_cast<const float4*>(sks + k0);
      const uint32_t mk = *reinterpret_cast<const uint32_t*>(mks + k0);
      const float skk[4] = {skv.x, skv.y, skv.z, skv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int key = 16 * kt + 4 * e + fg;
        float sc = (((float)sc4[e] * sqr) * skk[e]) * 0.125f;
        bool keep = ((mk >> (8 * e)) & 0xffu) != 0u;
        if (row_mask) keep = a.mask[b * a.m_bs + (long)qrow * a.m_is + min(key, Sk - 1)] != 0;
        if (!keep) sc = -1.0e9f;
        x[kt][e] = key < Sk ? sc : -3.0e38f;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) x[kt][e] = -3.0e38f;
    }
  }
  QTX_STAMP(2);

  // ---- softmax of row fr over its 128 key slots (32 in the lane, 4 lanes) -----------------
  float m = x[0][0];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt)
#pragma unroll
    for (int e = 0; e < 4; ++e) m = fmaxf(m, x[kt][e]);
  m = xmax16(m);
  m = xmax32(m);
#pragma unroll
  for (int kt = 0; kt < 8; ++kt)
#pragma unroll
    for (int e = 0; e < 4; ++e) x[kt][e] = (16 * kt + 4 * e + fg < Sk) ? qexp(x[kt][e] - m) : 0.0f;
  float t[4];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    float u[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)        // lane-split partial, then tree levels 1-2 (lanes)
      u[e] = xsum32(xsum16((0.0f + x[kt][e]) + x[kt + 4][e]));
    t[kt] = (u[0] + u[1]) + (u[2] + u[3]);
  }
  const float den = (t[0] + t[1]) + (t[2] + t[3]);
  // e/den correctly rounded via the shared reciprocal (div_cr) unless some e is outside
  // its range (then the true division, wave-uniform); q/127 by div127 (exact for the codes)
  DivRange rg;
#pragma unroll
  for (int kt = 0; kt < 8; ++kt)
#pragma unroll
    for (int e = 0; e < 4; ++e) rg.add(x[kt][e]);
  const bool fast = __ballot(!(rg.ok() && divisor_ok(den))) == 0ull;
  const float rden = 1.0f / den;
  if (fast) {
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) x[kt][e] = div_cr(x[kt][e], den, rden);
  } else {
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) x[kt][e] = x[kt][e] / den;
  }
#pragma unroll
  for (int kt = 0; kt < 8; ++kt)
#pragma unroll
    for (int e = 0; e < 4; ++e) {      // keys >= Sk: P = 0 (their padded PV steps add 0)
      const float pq = div127(rintf(x[kt][e] * 127.0f));
      x[kt][e] = (16 * kt + 4 * e + fg < Sk) ? pq : 0.0f;
    }
  QTX_STAMP(3);

  // ---- PV on fp32 MFMA: A = P[row fr][k] (the lane's x[s/4][s%4], k = 4s + fg),
  // B = float(v[k][d]) * s_v[k].  DEC (the decoder's PV order, oracle attention_pv dec):
  // A = RN(P * s_v[k]), B = float(v[k][d]), and step s goes to chain s & 3 — one MFMA step is
  // one chain's 4 keys in order — the four chains summed (c0 + c1) + (c2 + c3) ----------------
  constexpr int NCH = DEC ? 4 : 1;
  v4f acc[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[c][dt] = v4f{0, 0, 0, 0};
  const uint32_t* vt32 = reinterpret_cast<const uint32_t*>(Vs);
#pragma unroll
  for (int s4 = 0; s4 < 32; ++s4) {
    if (4 * s4 < nk4) {
      const int k = 4 * s4 + fg;
      const float svk = svs[k];
      const float pa = DEC ? x[s4 >> 2][s4 & 3] * svk : x[s4 >> 2][s4 & 3];
      const uint32_t vd = vt32[k * 16 + fr];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const float vb2 = DEC ? (float)(int8_t)(vd >> (8 * dt)) : (float)(int8_t)(vd >> (8 * dt)) * svk;
        acc[s4 % NCH][dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa, vb2, acc[s4 % NCH][dt], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = r0 + 4 * fg + e;
      const float cv = DEC ? (acc[0][dt][e] + acc[1 % NCH][dt][e]) + (acc[2 % NCH][dt][e] + acc[3 % NCH][dt][e])
                           : acc[0][dt][e];
      if (row < Sq) a.ctx[b * a.c_bs + (long)row * a.c_ld + hoff + dt * 16 + fr] = cv;
    }
  QTX_STAMP(4);
}

// Returns hipErrorNotSupported for shapes it does not take (caller keeps k_attention).
hipError_t launch_attention_mfma(const AttnArgs& a, hipStream_t st) {
  if (a.sk_dev || a.qpos_dev || a.H * 64 > 4096 || a.Sk <= 0 || a.Sk > AM_MAXK)
    return hipErrorNotSupported;
  if (a.dec)
    k_attn_mfma<true><<<dim3(a.H, a.B, (a.Sq + 63) / 64), dim3(256), 0, st>>>(a);
  else
    k_attn_mfma<false><<<dim3(a.H, a.B, (a.Sq + 63) / 64), dim3(256), 0, st>>>(a);
  return hipGetLastError();
}


// =====================================================================================
// k_attn_encq: encoder self-attention of ONE sentence, all heads, with the context
// quantized per token in the epilogue (attention.py:23-67 + the O-projection's input
// quantizer, quant_linear.py:30-43): no fp32 context round trip through HBM and no
// separate quantization kernel.
//
// Workgroup = sentence b, 8 waves; wave w owns query rows 16w..16w+15 and ALL 8 heads,
// so each lane ends with 4 whole-row segments (rows 4fg+e, 32 dims each) and the row
// absmax needs only the 16 lanes of its DPP row.  K and V of every head (2 x 64 KB) are
// staged once by LDS-DMA (global_load_lds_dwordx4, 2 key rows of 512 B per wave
// instruction): K rows in the staged key order am_perm with chunk swizzle
// slot = chunk ^ (row & 15) (conflict-free ds_read_b128 fragments for every head), V rows
// in key order with slot = chunk ^ 4 (row & 1) (conflict-free ds_read_b32 operands).
// Per head: S^T = K Q^T on i8 MFMA (Q fragments straight from HBM, one head ahead),
// softmax + P-quant in registers (the canonical trees of k_attn_mfma), PV on f32 MFMA
// with the output column n of dim tile dt = head dim 4n + dt, so one ds_read_b32 of a
// row-major V row feeds the four dim tiles of a k step.
// PIPE (all 128 keys, the cfg3 shape): V is not staged as int8; each head's V is
// dequantized ONCE per workgroup (every wave converts its 16 key rows) into a
// double-buffered fp32 [128][64] LDS tile, and the PV B operands are ds_read_b128s of it —
// instead of every wave re-converting all 128 rows for its own PV (3 VALU per MFMA): the
// same rounded products float(v) * s_v, so bit-identical; 93.6 -> 85.4 us per launch.
// =====================================================================================
template <int I, int N, class F>
__device__ __forceinline__ void static_for_(F& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_<I + 1, N>(f);
  }
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) { static_for_<0, N>(f); }

__device__ __forceinline__ void dma16_lds(const void* gsrc, const void* lds_dst) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
}

template <bool PIPE>
__global__ __launch_bounds__(512) void k_attn_encq(AttnArgs a, int8_t* ctx8, float* sctx, int kp) {
  __shared__ __attribute__((aligned(16))) uint8_t Ks[AM_MAXK * 512];
  // PIPE (all 128 keys): V of one head at a time, dequantized once per workgroup into fp32
  // (float(v) * s_v, double-buffered) instead of by every wave for its own PV; otherwise the
  // int8 V of all heads
  __shared__ __attribute__((aligned(16))) uint8_t Vs[PIPE ? 2 * AM_MAXK * 64 * 4 : AM_MAXK * 512];
  float* const Vf = reinterpret_cast<float*>(Vs);
  __shared__ __attribute__((aligned(16))) float sks[AM_MAXK];     // s_k / 8 (0 if masked), staged order
  __shared__ __attribute__((aligned(16))) float kadd[AM_MAXK];    // 0 kept, -1e9 masked, -3e38 absent
  __shared__ __attribute__((aligned(16))) float svs[AM_MAXK];     // s_v, key order
  const int b = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int Sk = a.Sk, Sq = a.Sq;
  const int r0 = wave * 16;
  QTX_STAMP(0);

  // ---- stage K and V of all heads: wave w moves LDS rows 16w..16w+15 of each ----------
  {
    const int rp = lane >> 5, slot = lane & 31;
    const int8_t* kb = a.k + b * a.k_bs;
    const int8_t* vb = a.v + b * a.v_bs;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int p = wave * 16 + 2 * i + rp;                 // LDS row of this lane
      const int kk = min(am_perm(p), Sk - 1), kv = min(p, Sk - 1);
      dma16_lds(kb + (long)kk * a.k_ld + 16 * (slot ^ (p & 15)), Ks + (wave * 16 + 2 * i) * 512);
      if constexpr (!PIPE)
        dma16_lds(vb + (long)kv * a.v_ld + 16 * (slot ^ (4 * (p & 1))), Vs + (wave * 16 + 2 * i) * 512);
    }
  }
  // PIPE: this lane's 16 bytes of head h's V — key row 16 wave + lane / 4, dims
  // 16 (lane % 4) .. + 15 — loaded one head ahead of their conversion
  const int vkey = wave * 16 + (lane >> 2), vd0 = 16 * (lane & 3);
  const int8_t* vsrc = a.v + b * a.v_bs + (long)vkey * a.v_ld + vd0;
  uint4 vnext = make_uint4(0, 0, 0, 0);
  if constexpr (PIPE) vnext = *reinterpret_cast<const uint4*>(vsrc);
  if (tid < AM_MAXK) {
    // score of key j = ((float(acc) * s_q) * (s_k / 8 or 0)) + kadd: the exact form of
    // ((acc * s_q) * s_k) / 8 then masked_fill(-1e9) (kept: x + 0 == x; masked:
    // x * 0 - 1e9 == -1e9; / 8 is exact and commutes with rounding for these normal
    // magnitudes); keys >= Sk get -3e38, so their e and P come out exactly 0 with no
    // per-element test
    const int j = tid, jc = min(j, Sk - 1), pj = am_perm(j);
    const bool ok = j < Sk;
    const float skj = a.sk[b * a.sk_bs + jc], svj = a.sv[b * a.sv_bs + jc];
    const bool keep = ok && (!a.mask || a.mask[b * a.m_bs + jc] != 0);
    sks[pj] = keep ? skj * 0.125f : 0.0f;
    kadd[pj] = !ok ? -3.0e38f : (keep ? 0.0f : -1.0e9f);
    svs[j] = ok ? svj : 0.0f;
  }
  const int qrow = min(r0 + fr, Sq - 1);
  const int8_t* qbase = a.q + b * a.q_bs + (long)qrow * a.q_ld + 16 * fg;
  v4i qf = *reinterpret_cast<const v4i*>(qbase);
  const float sqr = a.sq[b * a.sq_bs + qrow];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (r0 >= Sq) return;                    // (after the only block-wide barrier)
  QTX_STAMP(1);

  v4f ctx[8][4];
#pragma unroll
  for (int h = 0; h < 8; ++h)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) ctx[h][dt] = v4f{0, 0, 0, 0};

  // scores + softmax + P quantization of head h into x (the canonical trees of
  // k_attn_mfma), and PV of head h from x into ctx[h]; FULL: all 128 keys present (no
  // per-chunk tests, so the two phases of a pipelined iteration share one basic block)
  auto scores_softmax = [&](auto hc, const v4i qcur, float (&x)[8][4], auto fullc) {
    constexpr int h = decltype(hc)::value;
    constexpr bool FULL = decltype(fullc)::value;
    // ---- scores S^T: C[staged row 4fg + e = key 16kt + 4e + fg][query fr] --------------
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      if (FULL || 16 * kt < Sk) {
        const int krow = kt * 16 + fr;
        const v4i kf = *reinterpret_cast<const v4i*>(Ks + krow * 512 + 16 * ((4 * h + fg) ^ fr));
        const v4i sc4 = __builtin_amdgcn_mfma_i32_16x16x64_i8(kf, qcur, v4i{0, 0, 0, 0}, 0, 0, 0);
        const int k0 = 16 * kt + 4 * fg;         // staged rows k0..k0+3
        const float4 skv = *reinterpret_cast<const float4*>(sks + k0);
        const float4 kav = *reinterpret_cast<const float4*>(kadd + k0);
        const float skk[4] = {skv.x, skv.y, skv.z, skv.w};
        const float kak[4] = {kav.x, kav.y, kav.z, kav.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) x[kt][e] = ((float)sc4[e] * sqr) * skk[e] + kak[e];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[kt][e] = -3.0e38f;
      }
    }
    // ---- softmax of row fr over its key slots (32 in the lane, 4 lanes), the canonical
    // trees of k_attn_mfma.  Absent keys: qexp(-3e38 - m) == 0 exactly.
    float m = x[0][0];
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) m = fmaxf(m, x[kt][e]);
    m = xmax16(m);
    m = xmax32(m);
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) x[kt][e] = qexp(x[kt][e] - m);
    float t[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      float u[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) u[e] = xsum32(xsum16((0.0f + x[kt][e]) + x[kt + 4][e]));
      t[kt] = (u[0] + u[1]) + (u[2] + u[3]);
    }
    const float den = (t[0] + t[1]) + (t[2] + t[3]);
    // P = rint((e / den) * 127) / 127 with both divisions by div_cr, unguarded: den is in
    // [1, 128] (the row max contributes qexp(0) == 1), so e / den is correctly rounded for
    // every e >= 2^-60, and e < 2^-60 (or 0) gives P == 0 through either quotient
    const float rden = rcp_cr(den);       // RN(1 / den), den in [1, 128] (qtx_common.h)
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        x[kt][e] = div127(rintf(div_cr(x[kt][e], den, rden) * 127.0f));
  };
  // ---- PV: A = P[row fr][k = 4 s4 + fg], B[k][n] = float(v[k][64h + 4n + dt]) * s_v[k] --
  // in chunks of 32 keys (the V operand reads of a chunk are issued ahead of its MFMAs);
  // padded keys of a chunk have P == 0 and s_v == 0, so their steps add +0 to a
  // nonzero-or-+0 accumulator: exact
  // PIPE: V of head h (loaded in vnext) -> Vf[h & 1][key][dim] = float(v) * s_v[key]
  auto convert_v = [&](auto hc) {
    constexpr int h = decltype(hc)::value;
    const uint4 vv = vnext;
    if constexpr (h < 7) vnext = *reinterpret_cast<const uint4*>(vsrc + 64 * (h + 1));
    const float svk = svs[vkey];
    const uint32_t w[4] = {vv.x, vv.y, vv.z, vv.w};
    float* dst = Vf + (h & 1) * (AM_MAXK * 64) + vkey * 64 + vd0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float4 f;
      f.x = (float)(int8_t)(w[c] & 0xffu) * svk;
      f.y = (float)(int8_t)((w[c] >> 8) & 0xffu) * svk;
      f.z = (float)(int8_t)((w[c] >> 16) & 0xffu) * svk;
      f.w = (float)(int8_t)(w[c] >> 24) * svk;
      *reinterpret_cast<float4*>(dst + 4 * c) = f;
    }
  };
  // PIPE: PV of head h from Vf[h & 1]: one ds_read_b128 (dims 4fr .. 4fr + 3 of key
  // 4 s4 + fg) feeds the four dim tiles of a k step
  auto pv_f = [&](auto hc, const float (&x)[8][4]) {
    constexpr int h = decltype(hc)::value;
    const float* vrow = Vf + (h & 1) * (AM_MAXK * 64) + fg * 64 + 4 * fr;
#pragma unroll
    for (int s4 = 0; s4 < 32; ++s4) {
      const float pa = x[s4 >> 2][s4 & 3];
      const float4 vb = *reinterpret_cast<const float4*>(vrow + s4 * 256);
      const float vbs[4] = {vb.x, vb.y, vb.z, vb.w};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        ctx[h][dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa, vbs[dt], ctx[h][dt], 0, 0, 0);
    }
  };
  auto pv = [&](auto hc, const float (&x)[8][4], auto fullc) {
    constexpr int h = decltype(hc)::value;
    constexpr bool FULL = decltype(fullc)::value;
    const uint8_t* vrow = Vs + fg * 512 + 16 * ((4 * h + (fr >> 2)) ^ (4 * (fg & 1))) + 4 * (fr & 3);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (FULL || 32 * c < Sk) {
#pragma unroll
        for (int s4 = 8 * c; s4 < 8 * c + 8; ++s4) {
          const float pa = x[s4 >> 2][s4 & 3];
          const float svk = svs[4 * s4 + fg];
          const uint32_t vd = *reinterpret_cast<const uint32_t*>(vrow + s4 * 2048);
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            const float vb2 = (float)(int8_t)(vd >> (8 * dt)) * svk;
            ctx[h][dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa, vb2, ctx[h][dt], 0, 0, 0);
          }
        }
      }
    }
  };
  using full_t = std::integral_constant<bool, true>;
  using part_t = std::integral_constant<bool, false>;
  if constexpr (!PIPE) {
    // the head loop is unrolled by instantiation (ctx[h] must be register-resident: a
    // run-time head index would put the 128 accumulators in scratch)
    static_for<8>([&](auto hc) {
      constexpr int h = decltype(hc)::value;
      __builtin_amdgcn_sched_barrier(0);
      const v4i qcur = qf;
      if (h < 7) qf = *reinterpret_cast<const v4i*>(qbase + 64 * (h + 1));   // next head
      float x[8][4];
      scores_softmax(hc, qcur, x, part_t{});
      __builtin_amdgcn_sched_barrier(0);
      pv(hc, x, part_t{});
    });
  } else {
    // all 128 keys present: pipelined over heads — iteration h runs the PV of head h-1
    // (f32 MFMA) and then the scores and softmax of head h (VALU)
    // V of head h is converted in iteration h (into buffer h & 1, last read by the PV of
    // head h - 2 in iteration h - 1) and read by the PV of head h in iteration h + 1: one
    // barrier at the top of each iteration orders both
    float xp[8][4];
    long long st_bar = 0, st_pv = 0, st_sm = 0, st_cv = 0;   // QTX_STAMPS builds only
    static_for<9>([&](auto hc) {
      constexpr int h = decltype(hc)::value;
      const long long tb0 = QTX_NOW();
      __syncthreads();
      st_bar += QTX_NOW() - tb0;
      QTX_STAMP(4 + h);
      __builtin_amdgcn_sched_barrier(0);
      const long long tc0 = QTX_NOW();
      if constexpr (h < 8) convert_v(std::integral_constant<int, (h < 8 ? h : 0)>{});
      st_cv += QTX_NOW() - tc0;
      float xn[8][4];
      auto sm = [&]() {
        if constexpr (h < 8) {
          const v4i qcur = qf;
          if (h < 7) qf = *reinterpret_cast<const v4i*>(qbase + 64 * (h + 1));   // next head
          scores_softmax(std::integral_constant<int, (h < 8 ? h : 0)>{}, qcur, xn, full_t{});
        }
      };
      auto pvp = [&]() {
        if constexpr (h >= 1) pv_f(std::integral_constant<int, (h >= 1 ? h - 1 : 0)>{}, xp);
      };
      // the PV of head h-1 first (its P dies there), then the scores and softmax of head h,
      // as two phases: the f32 MFMA and the VALU share the SIMD's vector datapath
      // (profiles/r04_f32_split_probe.log), so interleaving them buys no overlap; in this
      // order the previous and the next P are never live together (no spill; 82.9 -> 81.6 us
      // at cfg3, A/B in gpurun_out/r04at2; waves of a SIMD in opposite phase orders: 86 us)
      {
        const long long tp0 = QTX_NOW();
        pvp();
        __builtin_amdgcn_sched_barrier(0);
        const long long tp1 = QTX_NOW();
        sm();
        __builtin_amdgcn_sched_barrier(0);
        st_pv += tp1 - tp0;
        st_sm += QTX_NOW() - tp1;
      }
      if constexpr (h < 8) {
#pragma unroll
        for (int kt = 0; kt < 8; ++kt)
#pragma unroll
          for (int e = 0; e < 4; ++e) xp[kt][e] = xn[kt][e];
      }
    });
#ifdef QTX_STAMPS
    // per wave (lane 0), summed over the head loop: barrier wait, PV, scores + softmax,
    // V conversion, at [4096 + 4 (8 block + wave) + 0..3]
    if (lane == 0 && qtx_stamp_buf) {
      unsigned long long* pw = qtx_stamp_buf + 4096 + 4 * (b * 8 + wave);
      pw[0] = st_bar; pw[1] = st_pv; pw[2] = st_sm; pw[3] = st_cv;
    }
#endif
  }
  QTX_STAMP(2);

  // ---- per-token quantization of the context rows 4fg + e (dims 64h + 4fr + dt):
  // rint(y / s) with y / s by div_cr — exact for a whole row when its absmax < 2^37 (as
  // the GEMM epilogues, qtx_gemm.hip); otherwise the true division (wave-uniform) -------
  float sc[4], inv[4];
  bool big = false;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float am = 0.0f;
#pragma unroll
    for (int h = 0; h < 8; ++h)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) am = fmaxf(am, fabsf(ctx[h][dt][e]));
    am = row16_max(am);
    sc[e] = scale127(fmaxf(am, 1e-5f));   // quant_scale(am, 127) and 1 / s, branch-free
    inv[e] = rcp_cr(sc[e]);
    big |= !(am < 0x1p37f);
  }
  auto store_rows = [&](auto quot) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = r0 + 4 * fg + e;
      if (row < Sq) {
        const long grow = (long)b * Sq + row;
        uint32_t* orow = reinterpret_cast<uint32_t*>(ctx8 + grow * a.c_ld) + fr;
#pragma unroll
        for (int h = 0; h < 8; ++h) {
          float qv[4];
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) qv[dt] = rint_biased(quot(ctx[h][dt][e], sc[e], inv[e]));
          const uint32_t pk = pack4_biased(qv[0], qv[1], qv[2], qv[3]);
          if (kp)   // the O-projection reads its A operand in the KP layout
            *reinterpret_cast<uint32_t*>(ctx8 + kp_off(grow, 64 * h + 4 * fr, 512)) = pk;
          else
            orow[16 * h] = pk;
        }
        if (fr == 0) sctx[(long)b * Sq + row] = sc[e];
      }
    }
  };
  if (__builtin_expect(__ballot(big) != 0ull, 0))
    store_rows([](float y, float s, float) { return y / s; });
  else
    store_rows([](float y, float s, float r) { return div_cr(y, s, r); });
  QTX_STAMP(3);
}

// Encoder self-attention with the per-token-quantized context (int8 [B,S,512] with row
// stride a.c_ld, scales [B*S]); H == 8, Sq == Sk <= 128, per-key mask (m_is == 0).
hipError_t launch_attention_encq(const AttnArgs& a, int8_t* ctx8, float* sctx, hipStream_t st,
                                 bool force_encq, bool kp) {
  if (a.dec || a.sk_dev || a.qpos_dev || a.H != 8 || a.Sk <= 0 || a.Sk > AM_MAXK || a.Sq != a.Sk ||
      (a.mask && a.m_is != 0) || (a.k_ld % 16) || (a.v_ld % 16) || (a.c_ld % 4))
    return hipErrorNotSupported;
  if (a.B < 128 && !force_encq) return hipErrorNotSupported;   // one workgroup per sentence:
  // below ~128 sentences the per-(head, query block) kernel spreads over more CUs
  if (kp && a.c_ld != 512) return hipErrorInvalidValue;
  // all keys present and unmasked positions only differ through kadd/sks: the pipelined
  // head loop (QTX_ENCQ_NOPIPE=1: the sequential one, A/B)
  const bool nopipe = knobs().encq_nopipe;    // QTX_DIAG build only
  if (a.Sk == AM_MAXK && !nopipe)
    k_attn_encq<true><<<dim3(a.B), dim3(512), 0, st>>>(a, ctx8, sctx, kp ? 1 : 0);
  else
    k_attn_encq<false><<<dim3(a.B), dim3(512), 0, st>>>(a, ctx8, sctx, kp ? 1 : 0);
  return hipGetLastError();
}

}  // namespace qtx

namespace qtx {

// =====================================================================================
// k_attn_fault_rows: fault injection into the attention MatMuls (QK^T "FirstMatMul", PV
// "SecondMatMul": the reference's campaign targets input/*/matmul_{8L+3,8L+4}.json etc.).
// Recomputes the context of the affected query rows of ONE (sentence, head) from the int8
// Q/K/V with the fault applied, in the canonical order (oracle attention_scores /
// softmax_quant / attention_pv), overwriting their fp32 context (the unfused path's ctx,
// quantized per token afterwards).  One wave per affected row.
//   AF_QK_INPUT   q[row i][d] bit-flipped: acc[i][j] += dq * k[j][d] for keys j in [lo, hi)
//   AF_QK_WEIGHT  k[j0][d] bit-flipped:     acc[i][j0] += q[i][d] * dk for rows i in [lo, hi)
//   AF_PV_INPUT   P*127 int at (i, j0) bit-flipped: the PV chain of row i uses the flipped P
//                 for dims d in [lo, hi)
//   AF_PV_WEIGHT  v[j0][d0] bit-flipped: the PV chain of dim d0 uses it for rows in [lo, hi)
// =====================================================================================
__global__ __launch_bounds__(64) void k_attn_fault_rows(AttnArgs a, AttnFault f) {
  __shared__ float Ps[512];
  __shared__ float Pf[512];
  const int lane = threadIdx.x;
  const int b = f.b, h = f.h, Sk = a.Sk;
  const int i = f.row0 + blockIdx.x;                 // the query row of this wave
  const int hoff = 64 * h;
  const int8_t* qrow = a.q + b * a.q_bs + (long)i * a.q_ld + hoff;
  const float sqi = a.sq[b * a.sq_bs + i];
  auto flip = [&](int8_t v) { return (int)(int8_t)(v ^ (1 << f.bit)); };
  // ---- scores of the lane's keys j = lane + 64 t -------------------------------------
  float x[8];
  float m = -3.0e38f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int j = lane + 64 * t;
    x[t] = -3.0e38f;
    if (j < Sk) {
      const int8_t* krow = a.k + b * a.k_bs + (long)j * a.k_ld + hoff;
      int acc = 0;
      for (int d = 0; d < 64; ++d) acc += (int)qrow[d] * (int)krow[d];
      if (f.kind == AF_QK_INPUT && i == f.i && j >= f.lo && j < f.hi)
        acc += (flip(qrow[f.d]) - (int)qrow[f.d]) * (int)krow[f.d];
      if (f.kind == AF_QK_WEIGHT && j == f.j && i >= f.lo && i < f.hi)
        acc += (int)qrow[f.d] * (flip(krow[f.d]) - (int)krow[f.d]);
      float sc = (((float)acc * sqi) * a.sk[b * a.sk_bs + j]) / 8.0f;
      if (f.kind == AF_QK_OUTPUT && i == f.i && j == f.j) sc = f.value / 8.0f;
      const bool keep = !a.mask || a.mask[b * a.m_bs + (long)i * a.m_is + j] != 0;
      x[t] = keep ? sc : -1.0e9f;
      m = fmaxf(m, x[t]);
    }
  }
  m = wave_max(m);
  // ---- softmax: lane-split partial sums (start 0), canonical butterfly ------------------
  float part = 0.0f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int j = lane + 64 * t;
    x[t] = j < Sk ? qexp(x[t] - m) : 0.0f;
    if (64 * t < Sk) part = part + x[t];
  }
  const float den = wave_sum(part);
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int j = lane + 64 * t;
    if (j < Sk) {
      const float n = rintf((x[t] / den) * 127.0f);
      Ps[j] = n / 127.0f;
      Pf[j] = Ps[j];
      if (f.kind == AF_PV_INPUT && i == f.i && j == f.j)
        Pf[j] = (float)flip((int8_t)(int)n) / 127.0f;
    }
  }
  __syncthreads();
  // ---- PV: lane = dim d, sequential fma chain over the keys ----------------------------
  const int d = lane;
  const bool pin = f.kind == AF_PV_INPUT && i == f.i && d >= f.lo && d < f.hi;
  const bool vw = f.kind == AF_PV_WEIGHT && d == f.d && i >= f.lo && i < f.hi;
  auto vint = [&](int j) {
    const int8_t v8 = a.v[b * a.v_bs + (long)j * a.v_ld + hoff + d];
    return (vw && j == f.j) ? flip(v8) : (int)v8;
  };
  float acc = 0.0f;
  if (a.dec) {   // the decoder's PV order (qtx_common.h pv_dec_chains)
    acc = pv_dec_chains(Sk, [&](int j) { return (pin ? Pf[j] : Ps[j]) * a.sv[b * a.sv_bs + j]; },
                        [&](int j) { return (float)vint(j); });
  } else {
    for (int j = 0; j < Sk; ++j) {
      const float vb = (float)vint(j) * a.sv[b * a.sv_bs + j];
      acc = fmaf(pin ? Pf[j] : Ps[j], vb, acc);
    }
  }
  if (f.kind == AF_PV_OUTPUT && i == f.i && d == f.d) acc = f.value;
  a.ctx[b * a.c_bs + (long)i * a.c_ld + hoff + d] = acc;
}

// =====================================================================================
// k_attn_trace: the attention MatMuls' intermediates for the traced executor (qtx/trace.py:
// the reference's node-by-node executor stores every node output by name,
// onnx_optimized_inference.py:57).  One wave per (query row i, sentence b x head h), the
// canonical order of the oracle (attention_scores / softmax_quant / attention_pv):
//   qk [B,H,Sq,Sk]  float(sum_d q[i][d] k[j][d])  (QK^T "FirstMatMul", exact integers)
//   pc [B,H,Sq,Sk]  rint(P * 127)                 (the Round of attention.py:33-35)
//   ctx             sum_j (P/127) v_j s_v[j] per head, as launch_attention writes it (a.dec:
//                   the decoder's PV order)
// Off the hot path (diagnostics / campaigns): scalar int8 loads, one row per wave.
// =====================================================================================
__global__ __launch_bounds__(64) void k_attn_trace(AttnArgs a, float* qk, float* pc) {
  __shared__ float Ps[512];
  const int lane = threadIdx.x;
  const int i = blockIdx.x, b = blockIdx.y / a.H, h = blockIdx.y % a.H, Sk = a.Sk;
  const int hoff = 64 * h;
  const long orow = ((long)blockIdx.y * a.Sq + i) * Sk;
  const int8_t* qrow = a.q + b * a.q_bs + (long)i * a.q_ld + hoff;
  const float sqi = a.sq[b * a.sq_bs + i];
  float x[8];
  float m = -3.0e38f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int j = lane + 64 * t;
    x[t] = -3.0e38f;
    if (j < Sk) {
      const int8_t* krow = a.k + b * a.k_bs + (long)j * a.k_ld + hoff;
      int acc = 0;
      for (int d = 0; d < 64; ++d) acc += (int)qrow[d] * (int)krow[d];
      if (qk) qk[orow + j] = (float)acc;
      const float sc = (((float)acc * sqi) * a.sk[b * a.sk_bs + j]) / 8.0f;
      const bool keep = !a.mask || a.mask[b * a.m_bs + (long)i * a.m_is + j] != 0;
      x[t] = keep ? sc : -1.0e9f;
      m = fmaxf(m, x[t]);
    }
  }
  m = wave_max(m);
  float part = 0.0f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int j = lane + 64 * t;
    x[t] = j < Sk ? qexp(x[t] - m) : 0.0f;
    if (64 * t < Sk) part = part + x[t];
  }
  const float den = wave_sum(part);
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int j = lane + 64 * t;
    if (j < Sk) {
      const float n = rintf((x[t] / den) * 127.0f);
      Ps[j] = n / 127.0f;
      if (pc) pc[orow + j] = n;
    }
  }
  __syncthreads();
  const int d = lane;
  float acc = 0.0f;
  if (a.dec) {   // the decoder's PV order (qtx_common.h pv_dec_chains)
    acc = pv_dec_chains(Sk, [&](int j) { return Ps[j] * a.sv[b * a.sv_bs + j]; },
                        [&](int j) { return (float)a.v[b * a.v_bs + (long)j * a.v_ld + hoff + d]; });
  } else {
    for (int j = 0; j < Sk; ++j) {
      const float vb = (float)a.v[b * a.v_bs + (long)j * a.v_ld + hoff + d] * a.sv[b * a.sv_bs + j];
      acc = fmaf(Ps[j], vb, acc);
    }
  }
  a.ctx[b * a.c_bs + (long)i * a.c_ld + hoff + d] = acc;
}

hipError_t launch_attn_trace(const AttnArgs& a, float* qk, float* pc, hipStream_t st) {
  if (a.Sk <= 0 || a.Sk > 512 || a.Sq <= 0 || a.B <= 0 || a.H <= 0) return hipErrorInvalidValue;
  k_attn_trace<<<dim3(a.Sq, a.B * a.H), dim3(64), 0, st>>>(a, qk, pc);
  return hipGetLastError();
}

hipError_t launch_attn_fault_rows(const AttnArgs& a, const AttnFault& f, hipStream_t st) {
  if (a.Sk <= 0 || a.Sk > 512 || f.nrows <= 0 || f.b < 0 || f.b >= a.B || f.h < 0 ||
      f.h >= a.H || f.row0 < 0 || f.row0 + f.nrows > a.Sq)
    return hipErrorInvalidValue;
  k_attn_fault_rows<<<dim3(f.nrows), dim3(64), 0, st>>>(a, f);
  return hipGetLastError();
}

}  // namespace qtx
