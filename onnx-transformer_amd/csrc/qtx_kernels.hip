// qtx_kernels.hip — hand-written gfx950 (CDNA4, wave64) kernels for the W8A8 transformer.
//
//   k_rows          per-token quantizer / LayerNorm(+quantizer)     quant_linear.py:30-43,
//                                                                   layer_norm.py:12-15
//   k_gemm          int8 x int8 -> int32 on v_mfma_i32_16x16x64_i8, LDS-staged tiles,
//                   fused dequant + bias (+ReLU) (+residual) epilogue quant_linear.py:111-119
//   k_attention     exact int8 QK^T, softmax, P-quant, PV            attention.py:23-36
//   k_embed         lut[id] * sqrt(512) + pe[pos]                    embeddings.py:12-13
//   k_generator     fp32 x.W^T + b (sequential fma chain over k)     generator.py:14-15
//   k_lsm_argmax    log_softmax + first-index argmax                 onnx_reference_inference.py:640-641
//
// Every float step follows the canonical order of qtx_common.h / oracle/qtx_oracle.py.
#include <cstdlib>

#include "qtx_common.h"
#include "qtx_kernels.h"
#include "qtx_knobs.h"

namespace qtx {

// =====================================================================================
// k_rows: one wave per row of D = 256*NCH floats; lane l owns float4 chunks l + 64*c.
// =====================================================================================
template <int NCH>
__global__ __launch_bounds__(256) void k_rows(RowArgs a) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + wave;
  if (r >= a.rows) return;
  const float* xr = a.x + (long)r * a.ldx;
  float v[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const float4 t = *reinterpret_cast<const float4*>(xr + 4 * (lane + 64 * c));
    v[c][0] = t.x; v[c][1] = t.y; v[c][2] = t.z; v[c][3] = t.w;
  }
  if (a.ln_a) {
    constexpr float D = 256.0f * NCH;
    float s = v[0][0];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c | e) s = s + v[c][e];
    const float mean = wave_sum(s) / D;
    float d[NCH][4];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) d[c][e] = v[c][e] - mean;
    float ss = d[0][0] * d[0][0];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c | e) ss = ss + d[c][e] * d[c][e];
    const float var = wave_sum(ss) / (D - 1.0f);
    const float den = sqrtf(var) + 1e-6f;
    float gb[NCH][4];
    DivRange rg;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const float4 ga = *reinterpret_cast<const float4*>(a.ln_a + 4 * (lane + 64 * c));
      const float4 tb = *reinterpret_cast<const float4*>(a.ln_b + 4 * (lane + 64 * c));
      d[c][0] = ga.x * d[c][0]; d[c][1] = ga.y * d[c][1];
      d[c][2] = ga.z * d[c][2]; d[c][3] = ga.w * d[c][3];
      gb[c][0] = tb.x; gb[c][1] = tb.y; gb[c][2] = tb.z; gb[c][3] = tb.w;
#pragma unroll
      for (int e = 0; e < 4; ++e) rg.add(d[c][e]);
    }
    const bool ok = divisor_ok(den) && rg.ok();
    // (a * d) / den: correctly rounded via div_cr unless a value is out of its range
    if (__builtin_expect(__ballot(!ok) == 0ull, 1)) {
      const float y = 1.0f / den;
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[c][e] = div_cr(d[c][e], den, y) + gb[c][e];
    } else {
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[c][e] = d[c][e] / den + gb[c][e];
    }
  }
  if (a.yout) {
    float* yr = a.yout + (long)r * a.ldy;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      *reinterpret_cast<float4*>(yr + 4 * (lane + 64 * c)) =
          make_float4(v[c][0], v[c][1], v[c][2], v[c][3]);
  }
  if (a.q) {
    float am = 0.0f;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) am = fmaxf(am, fabsf(v[c][e]));
    am = wave_max(am);
    const float sc = quant_scale(am, a.qmax);
    const int off = a.dst_off_dev ? *a.dst_off_dev + a.dst_off : a.dst_off;
    const long dst = (long)(r / a.rpb) * a.dst_bstride + off + (r % a.rpb);
    int8_t* qr = a.q + dst * a.ldq;
    uint32_t qd[NCH];
    quant_pack<4 * NCH>(&v[0][0], sc, qd);
    if (a.kp) {
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        *reinterpret_cast<uint32_t*>(a.q + kp_off(dst, 4 * (lane + 64 * c), 256 * NCH)) = qd[c];
    } else {
#pragma unroll
      for (int c = 0; c < NCH; ++c) *reinterpret_cast<uint32_t*>(qr + 4 * (lane + 64 * c)) = qd[c];
    }
    if (lane == 0) a.s[dst] = sc;
  }
}

hipError_t launch_rows(const RowArgs& a, hipStream_t st) {
  if (a.rows <= 0) return hipSuccess;
  const dim3 grid((a.rows + 3) / 4), block(256);
  switch (a.D) {
    case 256: k_rows<1><<<grid, block, 0, st>>>(a); break;
    case 512: k_rows<2><<<grid, block, 0, st>>>(a); break;
    case 1024: k_rows<4><<<grid, block, 0, st>>>(a); break;
    case 2048: k_rows<8><<<grid, block, 0, st>>>(a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// =====================================================================================
// k_gemm: block tile BM x BN, K step 64, 4 waves as WM x WN; each wave owns a
// (BM/WM) x (BN/WN) sub-tile of 16x16 MFMA fragments.  A and W tiles are staged through
// registers into double-buffered LDS (64-byte rows, 16-byte chunks XOR-swizzled so the
// ds_read_b128 fragment reads are bank-conflict free), one barrier per K step.
// MFMA operands: lane l supplies row (l & 15), bytes k = 16*(l>>4) .. +15 of its tile;
// the same k mapping on A and B keeps the dot product exact for any hardware k order.
// =====================================================================================
__device__ __forceinline__ int swz_off(int r, int c) {
  // chunk permutation per row group (r>>2)&3: {0,2,3,1} — conflict-free for the
  // 4x16-lane groups of ds_read_b128
  const int p = (0x1320 >> (((r >> 2) & 3) * 4)) & 3;
  return r * 64 + ((c ^ p) << 4);
}

__device__ __forceinline__ uint4 unpack_int4x16(uint2 h) {
  // 16 two's-complement nibbles (k = 2j low, 2j+1 high of byte j) -> 16 int8
  auto sext = [](uint32_t v) { return v | ((v & 0x08080808u) * 0x1Eu); };
  const uint32_t lo0 = sext(h.x & 0x0F0F0F0Fu), hi0 = sext((h.x >> 4) & 0x0F0F0F0Fu);
  const uint32_t lo1 = sext(h.y & 0x0F0F0F0Fu), hi1 = sext((h.y >> 4) & 0x0F0F0F0Fu);
  uint4 o;
  o.x = __builtin_amdgcn_perm(hi0, lo0, 0x05010400u);
  o.y = __builtin_amdgcn_perm(hi0, lo0, 0x07030602u);
  o.z = __builtin_amdgcn_perm(hi1, lo1, 0x05010400u);
  o.w = __builtin_amdgcn_perm(hi1, lo1, 0x07030602u);
  return o;
}

template <int BM, int BN, int WM, int WN, int WBITS>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int AP = (BM * 4 + 255) / 256, BP = (BN * 4 + 255) / 256;
  constexpr int TILE = (BM + BN) * 64;
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * TILE];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int bm0 = blockIdx.y * BM, bn0 = blockIdx.x * BN;

  uint4 ra[AP], rb[BP];
  auto gload = [&](int k0) {
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int idx = tid + 256 * p;
      if (idx < BM * 4) {
        const int r = idx >> 2, c = idx & 3;
        const int gr = min(bm0 + r, g.M - 1);
        ra[p] = *reinterpret_cast<const uint4*>(g.A + (long)gr * g.lda + k0 + c * 16);
      }
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + 256 * p;
      if (idx < BN * 4) {
        const int r = idx >> 2, c = idx & 3;
        const int gn = min(bn0 + r, g.N - 1);
        if constexpr (WBITS == 8) {
          rb[p] = *reinterpret_cast<const uint4*>(g.W + (long)gn * g.ldw + k0 + c * 16);
        } else {
          rb[p] = unpack_int4x16(
              *reinterpret_cast<const uint2*>(g.W + (long)gn * g.ldw + (k0 >> 1) + c * 8));
        }
      }
    }
  };
  auto swrite = [&](int buf) {
    uint8_t* base = lds + buf * TILE;
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int idx = tid + 256 * p;
      if (idx < BM * 4)
        *reinterpret_cast<uint4*>(base + swz_off(idx >> 2, idx & 3)) = ra[p];
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + 256 * p;
      if (idx < BN * 4)
        *reinterpret_cast<uint4*>(base + BM * 64 + swz_off(idx >> 2, idx & 3)) = rb[p];
    }
  };

  v4i acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  const int nk = g.K / 64;
  gload(0);
  swrite(0);
  __syncthreads();
  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * 64);
    const uint8_t* base = lds + cur * TILE;
    v4i af[FM], bf[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
      af[i] = *reinterpret_cast<const v4i*>(base + swz_off(wm * TM + i * 16 + fr, fg));
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bf[j] = *reinterpret_cast<const v4i*>(base + BM * 64 + swz_off(wn * TN + j * 16 + fr, fg));
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) swrite(cur ^ 1);
    __syncthreads();
  }

  // epilogue: C/D layout col = lane & 15, row = (lane >> 4) * 4 + e
  const bool relu = g.flags & EPI_RELU, resid = g.flags & EPI_RESIDUAL;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = bn0 + wn * TN + j * 16 + fr;
    if (col >= g.N) continue;
    const float swc = g.sw[col], bc = g.bias[col];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = bm0 + wm * TM + i * 16 + fg * 4 + e;
        if (row >= g.M) continue;
        float y = ((float)acc[i][j][e] * g.sa[row]) * swc + bc;
        if (relu) y = y > 0.0f ? y : 0.0f;
        if (resid) y = g.res[(long)row * g.ldr + col] + y;
        g.out[(long)row * g.ldo + col] = y;
      }
    }
  }
}

hipError_t launch_gemm(const GemmArgs& g, int wbits, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  if (g.K % 64 != 0 || (wbits != 8 && wbits != 4)) return hipErrorInvalidValue;
  const dim3 block(256);
  if (wbits == 8 && !knobs().gemm128) {       // QTX_GEMM128 (QTX_DIAG build): timing experiments
    const hipError_t e = launch_gemm256(g, st);
    if (e != hipErrorNotSupported) return e;
  }
  if (g.M >= 256) {
    const dim3 grid((g.N + 127) / 128, (g.M + 127) / 128);
    if (wbits == 8) k_gemm<128, 128, 2, 2, 8><<<grid, block, 0, st>>>(g);
    else k_gemm<128, 128, 2, 2, 4><<<grid, block, 0, st>>>(g);
  } else {
    const dim3 grid((g.N + 31) / 32, (g.M + 31) / 32);
    if (wbits == 8) k_gemm<32, 32, 2, 2, 8><<<grid, block, 0, st>>>(g);
    else k_gemm<32, 32, 2, 2, 4><<<grid, block, 0, st>>>(g);
  }
  return hipGetLastError();
}

// =====================================================================================
// k_attention: one workgroup (4 waves) per (head, batch).  K (rows padded to 68 B),
// V and the key scales are staged once in LDS; each wave walks query rows.
//   s_j  = ((float(sum_d q_d k_jd) * s_q) * s_k[j]) / 8      (exact int8 dot: v_dot4)
//   mask -> -1e9;  e_j = qexp(s_j - max);  den = lane-split sum;  P_j = rint(e_j/den*127)/127
//   ctx_d = fma chain over j of P_j * (float(v_jd) * s_v[j])  (a.dec: the decoder's order,
//           pv_dec_chains)
// =====================================================================================
constexpr int ATT_MAXK = 512;

__global__ __launch_bounds__(256) void k_attention(AttnArgs a) {
  __shared__ uint32_t Ks[ATT_MAXK * 17];
  __shared__ uint8_t Vs[ATT_MAXK * 64];
  __shared__ float sks[ATT_MAXK], svs[ATT_MAXK];
  __shared__ float Pb[4][ATT_MAXK];
  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int Sk = a.sk_dev ? (*a.sk_dev + a.sk_add) : a.Sk;
  const int hoff = h * 64;

  const int8_t* kb = a.k + b * a.k_bs + hoff;
  const int8_t* vb = a.v + b * a.v_bs + hoff;
  for (int idx = tid; idx < Sk * 16; idx += 256) {
    const int j = idx >> 4, w = idx & 15;
    Ks[j * 17 + w] = *reinterpret_cast<const uint32_t*>(kb + (long)j * a.k_ld + 4 * w);
    *reinterpret_cast<uint32_t*>(Vs + j * 64 + 4 * w) =
        *reinterpret_cast<const uint32_t*>(vb + (long)j * a.v_ld + 4 * w);
  }
  for (int j = tid; j < Sk; j += 256) {
    sks[j] = a.sk[b * a.sk_bs + j];
    svs[j] = a.sv[b * a.sv_bs + j];
  }
  __syncthreads();

  float* P = Pb[wave];
  for (int i = wave; i < a.Sq; i += 4) {
    const int8_t* qr = a.q + b * a.q_bs + (long)i * a.q_ld + hoff;
    uint32_t qd[16];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint4 t = *reinterpret_cast<const uint4*>(qr + 16 * w);
      qd[4 * w] = t.x; qd[4 * w + 1] = t.y; qd[4 * w + 2] = t.z; qd[4 * w + 3] = t.w;
    }
    const float sqi = a.sq[b * a.sq_bs + i];
    const int mrow = a.qpos_dev ? (*a.qpos_dev + i) : i;
    const uint8_t* mk = a.mask ? a.mask + b * a.m_bs + (long)mrow * a.m_is : nullptr;
    float lmax = -3.0e38f;
    for (int j = lane; j < Sk; j += 64) {
      int acc = 0;
#pragma unroll
      for (int w = 0; w < 16; ++w) acc = __builtin_amdgcn_sdot4(qd[w], Ks[j * 17 + w], acc, false);
      float s = (((float)acc * sqi) * sks[j]) * 0.125f;
      if (mk && mk[j] == 0) s = -1.0e9f;
      P[j] = s;
      lmax = fmaxf(lmax, s);
    }
    const float m = wave_max(lmax);
    float lsum = 0.0f;
    for (int j = lane; j < Sk; j += 64) {
      const float e = qexp(P[j] - m);
      P[j] = e;
      lsum = lsum + e;
    }
    const float den = wave_sum(lsum);
    for (int j = lane; j < Sk; j += 64) P[j] = rintf((P[j] / den) * 127.0f) / 127.0f;
    __builtin_amdgcn_wave_barrier();
    float acc = 0.0f;
    if (a.dec) {   // the decoder's PV order (qtx_common.h pv_dec_chains)
      acc = pv_dec_chains(Sk, [&](int j) { return P[j] * svs[j]; },
                          [&](int j) { return (float)(int8_t)Vs[j * 64 + lane]; });
    } else {
      for (int j = 0; j < Sk; ++j)
        acc = fmaf(P[j], (float)(int8_t)Vs[j * 64 + lane] * svs[j], acc);
    }
    a.ctx[b * a.c_bs + (long)i * a.c_ld + hoff + lane] = acc;
    __builtin_amdgcn_wave_barrier();
  }
}

hipError_t launch_attention(const AttnArgs& a, hipStream_t st) {
  if (a.B <= 0 || a.Sq <= 0) return hipSuccess;
  if (!a.sk_dev && (a.Sk <= 0 || a.Sk > ATT_MAXK)) return hipErrorInvalidValue;
  if (!knobs().attn_valu) {              // QTX_ATTN_VALU (QTX_DIAG build): timing experiments
    const hipError_t e = launch_attention_mfma(a, st);
    if (e != hipErrorNotSupported) return e;
  }
  k_attention<<<dim3(a.H, a.B), dim3(256), 0, st>>>(a);
  return hipGetLastError();
}

// =====================================================================================
// k_embed: out[b, t, :] = lut[id] * fp32(sqrt(512)) + pe[pos]   (embeddings.py:12-13,
// positional_encodings.py:23-26).  With pos_dev the token column and the position are
// *pos_dev + pos0 + t (the decode step).
// =====================================================================================
__global__ __launch_bounds__(128) void k_embed(const int64_t* ids, long ids_bs, int T,
                                               const int* pos_dev, int pos0, const float* lut,
                                               int vocab, const float* pe, int max_len,
                                               float* out, long out_bs) {
  const int t = blockIdx.x, b = blockIdx.y, c = threadIdx.x;  // 128 x float4 = 512
  const int base = pos_dev ? *pos_dev : 0;   // token column and position offset
  const int pos = base + pos0 + t;
  long id = ids[b * ids_bs + base + t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const int p = pos < max_len ? pos : max_len - 1;
  const float4 e = *reinterpret_cast<const float4*>(lut + id * 512 + 4 * c);
  const float4 q = *reinterpret_cast<const float4*>(pe + (long)p * 512 + 4 * c);
  const float sc = 0x1.6a09e6p+4f;  // float32(sqrt(512))
  *reinterpret_cast<float4*>(out + b * out_bs + (long)t * 512 + 4 * c) =
      make_float4(e.x * sc + q.x, e.y * sc + q.y, e.z * sc + q.z, e.w * sc + q.w);
}

hipError_t launch_embed(const int64_t* ids, long ids_bs, int B, int T, const int* pos_dev,
                        int pos0, const float* lut, int vocab, const float* pe, int max_len,
                        float* out, long out_bs, hipStream_t st) {
  if (B <= 0 || T <= 0) return hipSuccess;
  k_embed<<<dim3(T, B), dim3(128), 0, st>>>(ids, ids_bs, T, pos_dev, pos0, lut, vocab, pe,
                                             max_len, out, out_bs);
  return hipGetLastError();
}

// =====================================================================================
// k_generator: logits[m, v] = ((c0 + c1) + (c2 + c3)) + b[v], c_q = the fma chain of
// x[m,k] * W[v,k] over k in [128q, 128q + 128) from 0 (the oracle's canonical order).
// Block = 64 vocab rows x 32 token rows; W chunk transposed in LDS.
// =====================================================================================
__global__ __launch_bounds__(256) void k_generator(const float* x, long ldx, int M,
                                                   const float* W, const float* bias, int V,
                                                   float* logits) {
  __shared__ float Wt[64][65];
  __shared__ float X[32][64];
  const int tid = threadIdx.x, v = tid & 63, mg = tid >> 6;
  const int v0 = blockIdx.x * 64, m0 = blockIdx.y * 32;
  float acc[8], part[3][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.0f;
  for (int k0 = 0; k0 < 512; k0 += 64) {
    if (k0 && (k0 & 127) == 0) {            // a new k-quarter: its chain starts from 0
#pragma unroll
      for (int i = 0; i < 8; ++i) { part[(k0 >> 7) - 1][i] = acc[i]; acc[i] = 0.0f; }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int idx = tid + 256 * p, vv = idx >> 4, kq = idx & 15;
      const int gv = min(v0 + vv, V - 1);
      const float4 w = *reinterpret_cast<const float4*>(W + (long)gv * 512 + k0 + 4 * kq);
      Wt[4 * kq][vv] = w.x; Wt[4 * kq + 1][vv] = w.y; Wt[4 * kq + 2][vv] = w.z;
      Wt[4 * kq + 3][vv] = w.w;
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int idx = tid + 256 * p, mm = idx >> 4, kq = idx & 15;
      const int gm = min(m0 + mm, M - 1);
      *reinterpret_cast<float4*>(&X[mm][4 * kq]) =
          *reinterpret_cast<const float4*>(x + (long)gm * ldx + k0 + 4 * kq);
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < 64; ++kk) {
      const float w = Wt[kk][v];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(X[mg + 4 * i][kk], w, acc[i]);
    }
    __syncthreads();
  }
  const int gv = v0 + v;
  if (gv >= V) return;
  const float bv = bias[gv];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + mg + 4 * i;
    if (m < M) logits[(long)m * V + gv] = ((part[0][i] + part[1][i]) + (part[2][i] + acc[i])) + bv;
  }
}

hipError_t launch_generator(const float* x, long ldx, int M, const float* W, const float* b,
                            int V, float* logits, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  k_generator<<<dim3((V + 63) / 64, (M + 31) / 32), dim3(256), 0, st>>>(x, ldx, M, W, b, V,
                                                                       logits);
  return hipGetLastError();
}

// =====================================================================================
// k_lsm_argmax: one wave per row.  z = x - max; lse = log(lane-split sum of qexp(z));
// logp = z - lse; id = first index of the maximum logp (torch.max tie rule).  A row with a
// NaN or a +inf, or only -inf, is all-NaN under torch's log_softmax and its torch.max is
// index 0 (oracle log_softmax_argmax): logp NaN, id 0.
// =====================================================================================
__global__ __launch_bounds__(64) void k_lsm_argmax(const float* logits, int V, float* logp,
                                                   int64_t* ids, long ids_bs,
                                                   const int* col_dev, int col_add) {
  const int m = blockIdx.x, lane = threadIdx.x;
  const float* x = logits + (long)m * V;
  float lm = -3.0e38f;
  bool nonfin = false, fin = false;
  for (int v = lane; v < V; v += 64) {
    lm = fmaxf(lm, x[v]);
    nonfin |= !(x[v] < __builtin_inff());
    fin |= x[v] > -__builtin_inff();
  }
  if (__ballot(nonfin) != 0ull || __ballot(fin) == 0ull) {     // wave-uniform
    if (logp)
      for (int v = lane; v < V; v += 64) logp[(long)m * V + v] = __builtin_nanf("");
    if (lane == 0 && ids) ids[m * ids_bs + (col_dev ? *col_dev : 0) + col_add] = 0;
    return;
  }
  const float mx = wave_max(lm);
  float ls = 0.0f;
  for (int v = lane; v < V; v += 64) ls = ls + qexp(x[v] - mx);
  const float lse = logf(wave_sum(ls));
  float best = -3.0e38f;
  int bi = 0x7fffffff;
  for (int v = lane; v < V; v += 64) {
    const float lp = (x[v] - mx) - lse;
    if (logp) logp[(long)m * V + v] = lp;
    if (lp > best) { best = lp; bi = v; }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float ob = __shfl_xor(best, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane == 0 && ids) {
    const int col = (col_dev ? *col_dev : 0) + col_add;
    ids[m * ids_bs + col] = bi;
  }
}

hipError_t launch_logsoftmax_argmax(const float* logits, int M, int V, float* logp,
                                    int64_t* ids, long ids_bs, const int* col_dev,
                                    int col_add, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  k_lsm_argmax<<<dim3(M), dim3(64), 0, st>>>(logits, V, logp, ids, ids_bs, col_dev, col_add);
  return hipGetLastError();
}

// =====================================================================================
// small helpers
// =====================================================================================
__global__ void k_pack_int4(const int8_t* q, int N, int K, uint8_t* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // output byte
  if (i >= (long)N * K / 2) return;
  const int8_t lo = q[2 * i], hi = q[2 * i + 1];
  out[i] = (uint8_t)((lo & 0xF) | ((hi & 0xF) << 4));
}
hipError_t launch_pack_int4(const int8_t* q, int N, int K, uint8_t* packed, hipStream_t st) {
  const long n = (long)N * K / 2;
  k_pack_int4<<<dim3((n + 255) / 256), dim3(256), 0, st>>>(q, N, K, packed);
  return hipGetLastError();
}

__global__ void k_u8(const uint8_t* src, int eb, long n, uint8_t* dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t nz = 0;
  for (int b = 0; b < eb; ++b) nz |= src[i * eb + b];
  dst[i] = nz ? 1 : 0;
}
hipError_t launch_u8_from_any(const void* src, int elem_bytes, long n, uint8_t* dst,
                              hipStream_t st) {
  if (n <= 0) return hipSuccess;
  k_u8<<<dim3((n + 255) / 256), dim3(256), 0, st>>>((const uint8_t*)src, elem_bytes, n, dst);
  return hipGetLastError();
}

__global__ void k_step_inc(int* s) { *s += 1; }
__global__ void k_nop() {}
hipError_t launch_nop(hipStream_t st) {   // timing experiments (QTX_ABLATE)
  k_nop<<<1, 64, 0, st>>>();
  return hipGetLastError();
}
hipError_t launch_step_inc(int* step, hipStream_t st) {
  k_step_inc<<<1, 1, 0, st>>>(step);
  return hipGetLastError();
}

// zero `n16` 16-byte chunks: used instead of hipMemsetAsync inside work that is captured
// into a hipGraph (the decode prologue), where a captured memset did not re-run on replay
__global__ void k_zero16(uint4* p, long n16) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) p[i] = make_uint4(0, 0, 0, 0);
}
hipError_t launch_zero(void* p, size_t bytes, hipStream_t st) {
  if (bytes % 16 || (reinterpret_cast<uintptr_t>(p) & 15)) return hipErrorInvalidValue;
  const long n16 = (long)(bytes / 16);
  if (n16 == 0) return hipSuccess;
  k_zero16<<<dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, st>>>(reinterpret_cast<uint4*>(p), n16);
  return hipGetLastError();
}

__global__ void k_fill_col(int64_t* ids, long bs, int B, int64_t val) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) ids[b * bs] = val;
}
hipError_t launch_fill_col(int64_t* ids, long bs, int B, int64_t val, hipStream_t st) {
  k_fill_col<<<dim3((B + 255) / 256), dim3(256), 0, st>>>(ids, bs, B, val);
  return hipGetLastError();
}

}  // namespace qtx
