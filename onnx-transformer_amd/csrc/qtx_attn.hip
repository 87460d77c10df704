// qtx_attn.hip — encoder / decoder-module attention on the matrix cores (gfx950, wave64).
//
//   s_ij = ((float(q_i . k_j) * s_q[i]) * s_k[j]) / 8     (exact int8 dot: MFMA i8)
//   masked_fill(mask == 0, -1e9); P_ij = rint(softmax_j(s_ij) * 127) / 127
//   ctx_id = fma chain over j = 0..Sk-1 of P_ij * (float(v_jd) * s_v[j])
//   attention.py:23-36 (per head, 64-wide), canonical order of oracle/qtx_oracle.py.
//
// The PV chain runs on v_mfma_f32_16x16x4f32: chained over k in order (C starts at 0) it
// is bit-for-bit the k-ordered fmaf chain (the generator relies on the same fact), so the
// canonical sequential-fma PV becomes 16x16 tiles on the matrix cores instead of one
// latency-bound VALU chain per (row, dim).  Softmax rows use the canonical lane-split sum.
//
// k_attn_mfma: workgroup = (head h, sentence b, block of 64 query rows), 4 waves, wave w
// owns query rows 16w..16w+15 of the block.  K and V (int8, per head) and their scales
// are staged in LDS once per workgroup; the scores / P of a wave's 16 rows live in LDS.
// Keys <= 128.
#include "qtx_common.h"
#include "qtx_kernels.h"

QTX_STAMP_SETTER(attn)

namespace qtx {

constexpr int AM_MAXK = 128;
constexpr int AM_PS = AM_MAXK + 2;   // P row stride (floats): == 2 mod 32, conflict-free A reads

// 64-byte K rows, slot swizzle of qtx_gemm.hip (conflict-free ds_read_b128 fragments)
__device__ __forceinline__ int am_slot(int r, int c) { return c ^ (((r >> 3) & 1) << 1); }

__global__ __launch_bounds__(256) void k_attn_mfma(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t Ks[AM_MAXK * 64];
  __shared__ __attribute__((aligned(16))) int8_t Vs[AM_MAXK * 64];
  __shared__ float sks[AM_MAXK], svs[AM_MAXK];
  __shared__ uint8_t mks[AM_MAXK];           // key mask when it is the same for every query
  __shared__ float Pl[4][16 * AM_PS];
  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int Sk = a.Sk, Sq = a.Sq, hoff = h * 64;
  const int nk4 = (Sk + 3) & ~3;            // keys rounded up to the MFMA k step
  const int r0 = blockIdx.z * 64 + wave * 16;
  QTX_STAMP(0);

  // ---- stage K, V (rows < nk4; rows >= Sk zero) and the key scales -------------------
  const int8_t* kb = a.k + b * a.k_bs + hoff;
  const int8_t* vb = a.v + b * a.v_bs + hoff;
  if (tid < nk4) {        // thread j stages key row j: K swizzled, V transposed (below)
    const int j = tid, jc = min(j, Sk - 1);
    const bool ok = j < Sk;
    uint4 kv[4], vv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {          // clamped, unconditional loads; zeroed if j >= Sk
      kv[c] = *reinterpret_cast<const uint4*>(kb + (long)jc * a.k_ld + 16 * c);
      vv[c] = *reinterpret_cast<const uint4*>(vb + (long)jc * a.v_ld + 16 * c);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      *reinterpret_cast<uint4*>(Ks + j * 64 + 16 * am_slot(j, c)) = ok ? kv[c] : make_uint4(0, 0, 0, 0);
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
  }
  const bool row_mask = a.mask && a.m_is != 0;   // per-query mask rows (causal decoder)
  for (int j = tid; j < nk4; j += 256) {
    sks[j] = j < Sk ? a.sk[b * a.sk_bs + j] : 0.0f;
    svs[j] = j < Sk ? a.sv[b * a.sv_bs + j] : 0.0f;
    mks[j] = (a.mask && !row_mask && j < Sk) ? a.mask[b * a.m_bs + j] : (uint8_t)1;
  }
  // this wave's query fragment (MFMA A operand: row fr, bytes 16*fg..) and row scales
  const int qrow = min(r0 + fr, Sq - 1);
  const v4i qf = *reinterpret_cast<const v4i*>(a.q + b * a.q_bs + (long)qrow * a.q_ld + hoff + 16 * fg);
  float sqr[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) sqr[e] = a.sq[b * a.sq_bs + min(r0 + 4 * fg + e, Sq - 1)];
  __syncthreads();
  if (r0 >= Sq) return;                    // (after the only block-wide barrier)
  QTX_STAMP(1);

  // ---- scores: one i8 MFMA per 16 keys ---------------------------------------------------
  float* P = Pl[wave];
  for (int kt = 0; kt * 16 < Sk; ++kt) {
    const int key = kt * 16 + fr;
    const v4i kf = *reinterpret_cast<const v4i*>(Ks + key * 64 + 16 * am_slot(key, fg));
    const v4i s = __builtin_amdgcn_mfma_i32_16x16x64_i8(qf, kf, v4i{0, 0, 0, 0}, 0, 0, 0);
    const float skk = sks[key];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = 4 * fg + e;          // C layout: col = key, row = 4*(lane>>4) + e
      float sc = (((float)s[e] * sqr[e]) * skk) * 0.125f;
      bool keep = mks[min(key, AM_MAXK - 1)] != 0;
      if (row_mask) {
        const int qi = min(r0 + row, Sq - 1);
        keep = a.mask[b * a.m_bs + (long)qi * a.m_is + min(key, Sk - 1)] != 0;
      }
      if (!keep) sc = -1.0e9f;
      if (key < Sk) P[row * AM_PS + key] = sc;
    }
  }
  __builtin_amdgcn_wave_barrier();

  QTX_STAMP(2);
  // ---- softmax, 4 rows per pass: the 16-lane DPP row r of the wave holds query row rb+r,
  // lane j of it keys j + 16 i (i < 8).  Canonical order: lane-split partial of position L
  // (L < 64) = (0 + e[L]) + e[L+64]; positions j, j+16, j+32, j+48 live in lane j, so the
  // 64-position pairwise tree = a 16-lane tree per register, then (S0 + S1) + (S2 + S3).
  {
    const int sub = lane >> 4, jj = lane & 15;
    for (int rb = 0; rb < 16; rb += 4) {
      float* pr = P + (rb + sub) * AM_PS;
      float x[8], e[8];
      float m = -3.0e38f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int key = jj + 16 * i;
        x[i] = key < Sk ? pr[key] : -3.0e38f;
        m = fmaxf(m, x[i]);
      }
      m = row16_max(m);
#pragma unroll
      for (int i = 0; i < 8; ++i) e[i] = (jj + 16 * i < Sk) ? qexp(x[i] - m) : 0.0f;
      float pp[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) pp[q] = row16_sum((0.0f + e[q]) + e[q + 4]);
      const float den = (pp[0] + pp[1]) + (pp[2] + pp[3]);
      // e/den correctly rounded via the shared reciprocal (div_cr) unless some e is outside
      // its range (then the true division, wave-uniform); q/127 likewise (always in range)
      DivRange rg;
#pragma unroll
      for (int i = 0; i < 8; ++i) rg.add(e[i]);
      const bool fast = __ballot(!(rg.ok() && divisor_ok(den))) == 0ull;
      const float rden = 1.0f / den, r127 = 1.0f / 127.0f;
      float p[8];
      if (fast) {
#pragma unroll
        for (int i = 0; i < 8; ++i) p[i] = div_cr(e[i], den, rden);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) p[i] = e[i] / den;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int key = jj + 16 * i;      // keys in [Sk, nk4) get P = 0 (padded MFMA steps)
        const float pq = div_cr(rintf(p[i] * 127.0f), 127.0f, r127);
        if (key < nk4) pr[key] = key < Sk ? pq : 0.0f;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  QTX_STAMP(3);
  // ---- PV on fp32 MFMA: A = P[row fr][k], B = float(v[k][d]) * s_v[k], k = 4s + fg -------
  v4f acc[4] = {v4f{0, 0, 0, 0}, v4f{0, 0, 0, 0}, v4f{0, 0, 0, 0}, v4f{0, 0, 0, 0}};
  const uint32_t* vt32 = reinterpret_cast<const uint32_t*>(Vs);
#pragma unroll 4
  for (int s = 0; s < nk4 / 4; ++s) {
    const int k = 4 * s + fg;
    const float pa = P[fr * AM_PS + k];
    const float svk = svs[k];
    const uint32_t vd = vt32[k * 16 + fr];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const float vb2 = (float)(int8_t)(vd >> (8 * dt)) * svk;
      acc[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa, vb2, acc[dt], 0, 0, 0);
    }
  }
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = r0 + 4 * fg + e;
      if (row < Sq) a.ctx[b * a.c_bs + (long)row * a.c_ld + hoff + dt * 16 + fr] = acc[dt][e];
    }
  QTX_STAMP(4);
}

// Returns hipErrorNotSupported for shapes it does not take (caller keeps k_attention).
hipError_t launch_attention_mfma(const AttnArgs& a, hipStream_t st) {
  if (a.sk_dev || a.qpos_dev || a.H * 64 > 4096 || a.Sk <= 0 || a.Sk > AM_MAXK)
    return hipErrorNotSupported;
  k_attn_mfma<<<dim3(a.H, a.B, (a.Sq + 63) / 64), dim3(256), 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace qtx
