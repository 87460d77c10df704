// qtx_decode.hip — fused kernels of the KV-cached greedy decode step (gfx950, wave64).
//
//   k_skinny        M<=32-row int8 GEMM, 16 columns per workgroup, K split over 4 waves,
//                   A operand built in the prologue (int8 | LayerNorm+quant | rowmax-quant)
//                   quant_linear.py:111-119, layer_norm.py:12-15, position_feed_forward.py:12
//   k_dec_attn      one query per sentence, 8 heads = 8 waves; quantizes q/k/v per token,
//                   appends k/v to the cache, attention, quantizes the context row
//                   attention.py:23-67, get_quantized_model.py:160-168
//   k_generator_ln  final LayerNorm fused into the fp32 generator projection  generator.py:14-15
//   k_argmax_embed  log_softmax + first argmax + next-token embedding + step advance
//                   onnx_reference_inference.py:632,640-643
//
// All float steps follow the canonical order shared with oracle/qtx_oracle.py.
#include "qtx_common.h"
#include "qtx_kernels.h"

#ifdef QTX_STAMPS
__device__ unsigned long long* qtx_stamp_buf;
extern "C" int qtx_debug_set_stamps(void* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(qtx_stamp_buf), &buf, sizeof(buf));
}
#endif

namespace qtx {

__device__ __forceinline__ uint4 unpack_i4(uint2 h) {
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

// LayerNorm (canonical order, layer_norm.py:12-15) of R rows of 512 floats, each held as
// 2 float4 per lane, in place.  The R rows are processed step by step together so their
// independent reduction chains overlap (ILP) instead of running one row after another.
template <int R>
__device__ __forceinline__ void ln_rows512(float (&v)[R][2][4], const float* a, const float* b,
                                           int lane) {
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
#pragma unroll
  for (int j = 0; j < R; ++j) mean[j] = wave_sum(mean[j]) / 512.0f;
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
#pragma unroll
  for (int j = 0; j < R; ++j) den[j] = sqrtf(wave_sum(den[j]) / 511.0f) + 1e-6f;
  // y = (a * d) / den + b, the division correctly rounded via div_cr (one true division
  // per row for the reciprocal), true division if any value is outside div_cr's range
  float ga[2][4], gb[2][4];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float4 ta = *reinterpret_cast<const float4*>(a + 4 * (lane + 64 * c));
    const float4 tb = *reinterpret_cast<const float4*>(b + 4 * (lane + 64 * c));
    ga[c][0] = ta.x; ga[c][1] = ta.y; ga[c][2] = ta.z; ga[c][3] = ta.w;
    gb[c][0] = tb.x; gb[c][1] = tb.y; gb[c][2] = tb.z; gb[c][3] = tb.w;
  }
  DivRange rg;
#pragma unroll
  for (int j = 0; j < R; ++j) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[j][c][e] = ga[c][e] * v[j][c][e];     // numerator a * d
        rg.add(v[j][c][e]);
      }
  }
  bool ok = rg.ok();
#pragma unroll
  for (int j = 0; j < R; ++j) ok &= divisor_ok(den[j]);
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

// per-token quantization of R rows (2 float4 per lane each) into int8 dwords + scales
template <int R>
__device__ __forceinline__ void quant_rows512(const float (&v)[R][2][4], uint32_t (&q)[R][2],
                                              float (&sc)[R]) {
  float am[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    am[j] = 0.0f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) am[j] = fmaxf(am[j], fabsf(v[j][c][e]));
  }
#pragma unroll
  for (int j = 0; j < R; ++j) sc[j] = quant_scale(wave_max(am[j]), 127.0f);
#pragma unroll
  for (int j = 0; j < R; ++j) quant_pack<8>(&v[j][0][0], sc[j], q[j]);
}

// =====================================================================================
// k_skinny
// =====================================================================================
template <int MF, int K, int WBITS, int AMODE, int FLAGS>
__global__ __launch_bounds__(256) void k_skinny(SkinnyArgs g) {
  constexpr int BM = 16 * MF;
  constexpr int KW = K / 4;       // K range of one wave
  constexpr int NS = KW / 64;     // MFMA k-steps per wave
  constexpr int LDA = K + 16;     // padded LDS row (bytes)
  __shared__ __attribute__((aligned(16))) uint8_t As[BM * LDA];
  __shared__ float sas[BM];
  __shared__ v4i red[3][MF][64];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * BM;

  QTX_STAMP(0);
  if (g.zero && blockIdx.x == 0 && blockIdx.y == 0)
    for (int i = tid; i < g.zero_n; i += 256) g.zero[i] = 0u;

  // 1. this lane's W fragments for its wave's K range, issued first
  const int n = min(n0 + fr, g.N - 1);
  uint4 wf[NS];
  uint2 wp[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int k = wave * KW + 64 * s + 16 * fg;
    if constexpr (WBITS == 8)
      wf[s] = *reinterpret_cast<const uint4*>(g.W + (long)n * g.ldw + k);
    else
      wp[s] = *reinterpret_cast<const uint2*>(g.W + (long)n * g.ldw + (k >> 1));
  }
  // epilogue operands of wave 0 (it finishes the tile), also issued up front: a load
  // first issued after the reduction barrier would add a whole memory round trip
  const int col = n0 + fr;
  const bool cok = col < g.N;
  float swc = 0.0f, bc = 0.0f, rv[MF][4];
  constexpr bool resid = FLAGS & EPI_RESIDUAL;
  if (wave == 0) {
    swc = cok ? g.sw[col] : 0.0f;
    bc = cok ? g.bias[col] : 0.0f;
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + 16 * i + 4 * fg + e;
        rv[i][e] = (resid && cok && row < g.M) ? g.res[(long)row * g.ldr + col] : 0.0f;
      }
  }

  // 2. A panel (int8) and per-row scales into LDS.  Every branch issues all of its
  //    global loads before consuming any (one memory latency, not one per row).
  constexpr int RPW = BM / 4;  // rows per wave: r = wave + 4*j
  if constexpr (AMODE == A_I8) {
    constexpr int CPR = K / 16, NLD = BM * CPR / 256;
    uint4 v[NLD];
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int idx = tid + 256 * j, m = min(m0 + idx / CPR, g.M - 1);
      v[j] = *reinterpret_cast<const uint4*>(g.A + (long)m * K + 16 * (idx % CPR));
    }
    if (tid < BM) sas[tid] = (m0 + tid < g.M) ? g.sa[m0 + tid] : 0.0f;
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int idx = tid + 256 * j, r = idx / CPR;
      *reinterpret_cast<uint4*>(As + r * LDA + 16 * (idx % CPR)) =
          (m0 + r < g.M) ? v[j] : make_uint4(0, 0, 0, 0);
    }
  } else if constexpr (AMODE == A_LN) {
    float v[RPW][2][4];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int m = min(m0 + wave + 4 * j, g.M - 1);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float4 t = *reinterpret_cast<const float4*>(g.X + (long)m * g.ldx + 4 * (lane + 64 * c));
        v[j][c][0] = t.x; v[j][c][1] = t.y; v[j][c][2] = t.z; v[j][c][3] = t.w;
      }
    }
    ln_rows512<RPW>(v, g.ln_a, g.ln_b, lane);
    uint32_t q[RPW][2];
    float sc[RPW];
    quant_rows512<RPW>(v, q, sc);
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int r = wave + 4 * j;
      const bool ok = m0 + r < g.M;
      uint32_t* dst = reinterpret_cast<uint32_t*>(As + r * LDA);
      dst[lane] = ok ? q[j][0] : 0u;
      dst[lane + 64] = ok ? q[j][1] : 0u;
      if (lane == 0) sas[r] = ok ? sc[j] : 0.0f;
    }
  } else {  // A_F32Q: rows in batches of 4 (32 float4 in flight per lane at K = 2048)
    constexpr int NC = K / 256, RB = RPW < 4 ? RPW : 4;
#pragma unroll
    for (int j0 = 0; j0 < RPW; j0 += RB) {
      float4 t[RB][NC];
      float sc[RB];
#pragma unroll
      for (int jb = 0; jb < RB; ++jb) {
        const int m = min(m0 + wave + 4 * (j0 + jb), g.M - 1);
        sc[jb] = quant_scale(__uint_as_float(g.rowmax_in[m]), 127.0f);
#pragma unroll
        for (int c = 0; c < NC; ++c)
          t[jb][c] = *reinterpret_cast<const float4*>(g.X + (long)m * g.ldx + 4 * (lane + 64 * c));
      }
#pragma unroll
      for (int jb = 0; jb < RB; ++jb) {
        const int r = wave + 4 * (j0 + jb);
        const bool ok = m0 + r < g.M;
        uint32_t* dst = reinterpret_cast<uint32_t*>(As + r * LDA);
        float tf[4 * NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          tf[4 * c] = t[jb][c].x; tf[4 * c + 1] = t[jb][c].y;
          tf[4 * c + 2] = t[jb][c].z; tf[4 * c + 3] = t[jb][c].w;
        }
        uint32_t qd[NC];
        quant_pack<4 * NC>(tf, sc[jb], qd);
#pragma unroll
        for (int c = 0; c < NC; ++c) dst[lane + 64 * c] = ok ? qd[c] : 0u;
        if (lane == 0) sas[r] = ok ? sc[jb] : 0.0f;
      }
    }
  }
  __syncthreads();

  QTX_STAMP(1);
  // 3. MFMA over this wave's K range
  v4i acc[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) acc[i] = v4i{0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    v4i bfr;
    if constexpr (WBITS == 8) {
      bfr = __builtin_bit_cast(v4i, wf[s]);
    } else {
      bfr = __builtin_bit_cast(v4i, unpack_i4(wp[s]));
    }
    const int k = wave * KW + 64 * s + 16 * fg;
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const v4i afr = *reinterpret_cast<const v4i*>(As + (16 * i + fr) * LDA + k);
      acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr, bfr, acc[i], 0, 0, 0);
    }
  }

  // 4. exact int32 reduction of the 4 K ranges
  if (wave > 0)
#pragma unroll
    for (int i = 0; i < MF; ++i) red[wave - 1][i][lane] = acc[i];
  __syncthreads();
  if (wave != 0) return;
  QTX_STAMP(2);
#pragma unroll
  for (int w = 0; w < 3; ++w)
#pragma unroll
    for (int i = 0; i < MF; ++i) acc[i] += red[w][i][lane];

  // 5. epilogue (C layout: col = lane & 15, row = 4*(lane>>4) + e)
  constexpr bool relu = FLAGS & EPI_RELU, rmax = FLAGS & EPI_ROWMAX;
#pragma unroll
  for (int i = 0; i < MF; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = 16 * i + 4 * fg + e, row = m0 + r;
      const bool ok = cok && row < g.M;
      float y = ((float)acc[i][e] * sas[r]) * swc + bc;
      if constexpr (relu) y = y > 0.0f ? y : 0.0f;
      if constexpr (resid) y = rv[i][e] + y;
      if (ok) g.out[(long)row * g.ldo + col] = y;
      if constexpr (rmax) {
        float am = ok ? fabsf(y) : 0.0f;
        am = fmaxf(am, __shfl_xor(am, 8, 64));
        am = fmaxf(am, __shfl_xor(am, 4, 64));
        am = fmaxf(am, __shfl_xor(am, 2, 64));
        am = fmaxf(am, __shfl_xor(am, 1, 64));
        if (fr == 0 && row < g.M) atomicMax(g.rowmax_out + row, __float_as_uint(am));
      }
    }
  }
  QTX_STAMP(3);
}

// dispatch: the prologue mode and epilogue flags are template parameters (no runtime
// branches per output element).  Supported: K 512 with A_I8 / A_LN, K 2048 with A_I8 /
// A_F32Q; flags 0, RELU, RESIDUAL, RELU|ROWMAX.
template <int MF, int K, int WB, int AM>
hipError_t skinny_flags(const SkinnyArgs& g, dim3 grid, hipStream_t st) {
  switch (g.flags) {
    case 0: k_skinny<MF, K, WB, AM, 0><<<grid, 256, 0, st>>>(g); break;
    case EPI_RELU: k_skinny<MF, K, WB, AM, EPI_RELU><<<grid, 256, 0, st>>>(g); break;
    case EPI_RESIDUAL: k_skinny<MF, K, WB, AM, EPI_RESIDUAL><<<grid, 256, 0, st>>>(g); break;
    case EPI_RELU | EPI_ROWMAX:
      k_skinny<MF, K, WB, AM, EPI_RELU | EPI_ROWMAX><<<grid, 256, 0, st>>>(g);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
template <int MF, int WB>
hipError_t skinny_mode(const SkinnyArgs& g, dim3 grid, hipStream_t st) {
  if (g.K == 512) {
    if (g.amode == A_I8) return skinny_flags<MF, 512, WB, A_I8>(g, grid, st);
    if (g.amode == A_LN) return skinny_flags<MF, 512, WB, A_LN>(g, grid, st);
  } else if (g.K == 2048) {
    if (g.amode == A_I8) return skinny_flags<MF, 2048, WB, A_I8>(g, grid, st);
    if (g.amode == A_F32Q) return skinny_flags<MF, 2048, WB, A_F32Q>(g, grid, st);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_skinny(const SkinnyArgs& g, int wbits, hipStream_t st) {
  if (g.M <= 0) return hipSuccess;
  if (g.N % 16) return hipErrorInvalidValue;
  const int MF = g.M <= 16 ? 1 : 2;
  const dim3 grid(g.N / 16, (g.M + 16 * MF - 1) / (16 * MF));
  if (wbits == 8) return MF == 1 ? skinny_mode<1, 8>(g, grid, st) : skinny_mode<2, 8>(g, grid, st);
  if (wbits == 4) return MF == 1 ? skinny_mode<1, 4>(g, grid, st) : skinny_mode<2, 4>(g, grid, st);
  return hipErrorInvalidValue;
}

// =====================================================================================
// k_dec_attn: 512 threads = 8 waves; wave h = head h.  Keys staged in LDS (<= 128).
// =====================================================================================
constexpr int DEC_MAXK = 128;

// block-wide max of one value per thread (512 threads), result broadcast
__device__ __forceinline__ float block_max512(float v, float* scratch) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float m = scratch[0];
#pragma unroll
  for (int i = 1; i < 8; ++i) m = fmaxf(m, scratch[i]);
  return m;
}

template <bool KV_NEW>
__global__ __launch_bounds__(512) void k_dec_attn(DecAttnArgs a) {
  __shared__ uint32_t Ks[8][DEC_MAXK * 17];     // per head: key rows of 64 int8 (+4 B pad)
  __shared__ __attribute__((aligned(16))) uint8_t Vs[DEC_MAXK * 512];
  __shared__ float sks[DEC_MAXK], svs[DEC_MAXK];
  __shared__ float Pb[8][DEC_MAXK];
  __shared__ float red[3][8];
  __shared__ __attribute__((aligned(16))) int8_t qrow[512];   // read back as dwords
  const int b = blockIdx.x, t = threadIdx.x, h = t >> 6, lane = t & 63;
  QTX_STAMP(0);
  const float* yr = a.y + (long)b * a.ldy;
  const int step = KV_NEW ? *a.step : 0;
  const int Sk = KV_NEW ? step + 1 : a.S;

  // phase 0: issue the loads of the cached keys/values first (one memory latency):
  // row j = 32 uint4 of K and of V; thread t takes uint4 index t + 512*i
  const int nk = KV_NEW ? step : a.S;
  const uint4* kb4 = reinterpret_cast<const uint4*>(a.kc + (long)b * a.kv_bs * 512);
  const uint4* vb4 = reinterpret_cast<const uint4*>(a.vc + (long)b * a.kv_bs * 512);
  constexpr int NLD = DEC_MAXK * 32 / 512;
  // Loads sit behind a wave-uniform bound on the iteration and read a clamped index (row
  // 0 always exists): a load under a divergent branch makes the compiler wait for it
  // before the join, serializing them; unconditional clamped loads waste L1 bandwidth.
  const int lastk = nk * 32 > 0 ? nk * 32 - 1 : 0;
  const int nit = (nk * 32 + 511) >> 9;
  uint4 kr[NLD], vr[NLD];
#pragma unroll
  for (int i = 0; i < NLD; ++i) {
    if (i < nit) {
      const int idx = min(t + 512 * i, lastk);
      kr[i] = kb4[idx];
      vr[i] = vb4[idx];
    }
  }
  const int tj = min(t, nk > 0 ? nk - 1 : 0);
  const float skj = a.skc[(long)b * a.kv_bs + tj];
  const float svj = a.svc[(long)b * a.kv_bs + tj];

  // phase 1: per-token quantization of the new q (and k, v) rows: one block reduction
  // for the three row maxima
  const float vq = yr[t];
  const float vk = KV_NEW ? yr[512 + t] : 0.0f, vv = KV_NEW ? yr[1024 + t] : 0.0f;
  {
    const float wq = wave_max(fabsf(vq)), wk = wave_max(fabsf(vk)), wv = wave_max(fabsf(vv));
    if (lane == 0) { red[0][h] = wq; red[1][h] = wk; red[2][h] = wv; }
  }
  __syncthreads();
  float amq = red[0][0], amk = red[1][0], amv = red[2][0];
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    amq = fmaxf(amq, red[0][i]); amk = fmaxf(amk, red[1][i]); amv = fmaxf(amv, red[2][i]);
  }
  const float sq = quant_scale(amq, 127.0f);
  qrow[t] = (int8_t)quant_one(vq, sq);
  if constexpr (KV_NEW) {
    const float sk = quant_scale(amk, 127.0f), sv = quant_scale(amv, 127.0f);
    const int8_t qk = (int8_t)quant_one(vk, sk), qv = (int8_t)quant_one(vv, sv);
    const long row = (long)b * a.kv_bs + step;
    a.kc[row * 512 + t] = qk;
    a.vc[row * 512 + t] = qv;
    reinterpret_cast<int8_t*>(Ks[h])[step * 68 + lane] = qk;
    Vs[step * 512 + t] = (uint8_t)qv;
    if (t == 0) {
      a.skc[row] = sk; a.svc[row] = sv;
      sks[step] = sk; svs[step] = sv;
    }
  }
  // phase 2: cached keys 0 .. nk-1 from registers into LDS
#pragma unroll
  for (int i = 0; i < NLD; ++i) {
    const int idx = t + 512 * i;
    if (idx < nk * 32) {
      const int j = idx >> 5, q = idx & 31;      // q-th uint4 of row j = dwords 4q..4q+3
      uint32_t* kd = &Ks[q >> 2][j * 17 + 4 * (q & 3)];
      kd[0] = kr[i].x; kd[1] = kr[i].y; kd[2] = kr[i].z; kd[3] = kr[i].w;
      reinterpret_cast<uint4*>(Vs + j * 512)[q] = vr[i];
    }
  }
  if (t < nk) { sks[t] = skj; svs[t] = svj; }
  __syncthreads();
  QTX_STAMP(1);

  // phase 3: head h
  uint32_t qd[16];
#pragma unroll
  for (int w = 0; w < 16; ++w) qd[w] = reinterpret_cast<const uint32_t*>(qrow + h * 64)[w];
  float* P = Pb[h];
  const uint8_t* mk = KV_NEW ? nullptr : a.mask + (long)b * a.S;
  float lmax = -3.0e38f;
  for (int j = lane; j < Sk; j += 64) {
    int acc = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) acc = __builtin_amdgcn_sdot4(qd[w], Ks[h][j * 17 + w], acc, false);
    float s = (((float)acc * sq) * sks[j]) * 0.125f;
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
  QTX_STAMP(2);
  float acc = 0.0f;
#pragma unroll 8
  for (int j = 0; j < Sk; ++j)
    acc = fmaf(P[j], (float)(int8_t)Vs[j * 512 + t] * svs[j], acc);
  QTX_STAMP(3);

  // phase 4: quantize the context row (all heads) per token -> next GEMM's A operand
  const float sc = quant_scale(block_max512(fabsf(acc), red[0]), 127.0f);
  a.a8[(long)b * 512 + t] = (int8_t)quant_one(acc, sc);
  if (t == 0) a.sa[b] = sc;
  QTX_STAMP(4);
}

hipError_t launch_dec_attn(const DecAttnArgs& a, int B, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (!a.kv_new && (a.S <= 0 || a.S > DEC_MAXK)) return hipErrorInvalidValue;
  if (a.kv_new) k_dec_attn<true><<<dim3(B), dim3(512), 0, st>>>(a);
  else k_dec_attn<false><<<dim3(B), dim3(512), 0, st>>>(a);
  return hipGetLastError();
}

// =====================================================================================
// k_generator_ln: block = 16 vocab rows x 32 token rows (278 blocks for 4444 x 32).
// The 16 W rows (32 KB) and the 32 x rows are loaded with all loads in flight, the rows
// are LayerNormed (final norm, decoder.py:16) into LDS, then each thread runs two
// sequential fma chains over k (the canonical generator order):
//   logits[m, v] = (fma chain over k of x[m,k] * W[v,k]) + b[v]
// =====================================================================================
__global__ __launch_bounds__(256) void k_generator_ln(const float* x, long ldx, int M,
                                                      const float* ln_a, const float* ln_b,
                                                      const float* W, const float* bias, int V,
                                                      float* logits) {
  __shared__ __attribute__((aligned(16))) float X[32][516];   // +4: rows on distinct banks
  __shared__ float Wt[512][17];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int v0 = blockIdx.x * 16, m0 = blockIdx.y * 32;
  float4 wr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int idx = tid + 256 * j, gv = min(v0 + (idx >> 7), V - 1);
    wr[j] = *reinterpret_cast<const float4*>(W + (long)gv * 512 + 4 * (idx & 127));
  }
  float xv[8][2][4];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int m = min(m0 + wave + 4 * j, M - 1);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float4 t = *reinterpret_cast<const float4*>(x + (long)m * ldx + 4 * (lane + 64 * c));
      xv[j][c][0] = t.x; xv[j][c][1] = t.y; xv[j][c][2] = t.z; xv[j][c][3] = t.w;
    }
  }
  if (ln_a) ln_rows512<8>(xv, ln_a, ln_b, lane);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
      *reinterpret_cast<float4*>(&X[wave + 4 * j][4 * (lane + 64 * c)]) =
          make_float4(xv[j][c][0], xv[j][c][1], xv[j][c][2], xv[j][c][3]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int idx = tid + 256 * j, vv = idx >> 7, k = 4 * (idx & 127);
    Wt[k][vv] = wr[j].x; Wt[k + 1][vv] = wr[j].y; Wt[k + 2][vv] = wr[j].z; Wt[k + 3][vv] = wr[j].w;
  }
  __syncthreads();
  const int v = tid & 15, mi = tid >> 4;
  float a0 = 0.0f, a1 = 0.0f;
#pragma unroll 16
  for (int k = 0; k < 512; ++k) {
    const float w = Wt[k][v];
    a0 = fmaf(X[mi][k], w, a0);
    a1 = fmaf(X[mi + 16][k], w, a1);
  }
  const int gv = v0 + v;
  if (gv >= V) return;
  const float bv = bias[gv];
  if (m0 + mi < M) logits[(long)(m0 + mi) * V + gv] = a0 + bv;
  if (m0 + mi + 16 < M) logits[(long)(m0 + mi + 16) * V + gv] = a1 + bv;
}

hipError_t launch_generator_ln(const float* x, long ldx, int M, const float* ln_a,
                               const float* ln_b, const float* W, const float* b, int V,
                               float* logits, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  k_generator_ln<<<dim3((V + 15) / 16, (M + 31) / 32), dim3(256), 0, st>>>(
      x, ldx, M, ln_a, ln_b, W, b, V, logits);
  return hipGetLastError();
}

// =====================================================================================
// k_generator_mfma: the same canonical chain on the fp32 matrix cores.
// v_mfma_f32_16x16x4_f32 chained over k = 0..511 (128 instructions, C starts at 0) is
// bit-for-bit the k-ordered fmaf chain (cdna_hip_programming.md §3 "FP32-input MFMA"),
// so logits[m, v] = (fma chain of x[m,k] * W[v,k]) + b[v] exactly as the oracle.
// Block = 16 token rows x 64 vocab columns (4 waves, 16 columns each).  A operand =
// the LayerNormed rows in LDS; B operand = Wt [512][V] (the generator weight stored
// transposed at load), lane l reading Wt[4s + (l>>4)][v0 + (l&15)].
// =====================================================================================
__global__ __launch_bounds__(256) void k_generator_mfma(const float* x, long ldx, int M,
                                                        const float* ln_a, const float* ln_b,
                                                        const float* Wt, const float* bias,
                                                        int V, float* logits) {
  __shared__ __attribute__((aligned(16))) float X[16][514];   // stride 514: conflict-free reads
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int m0 = blockIdx.y * 16;
  const int vcol = blockIdx.x * 64 + 16 * wave + fr;
  const int vl = min(vcol, V - 1);
  float bq[2][32];
#pragma unroll
  for (int s = 0; s < 32; ++s) bq[0][s] = Wt[(long)(4 * s + fg) * V + vl];
  const float bv = bias[vl];
  float xv[4][2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = min(m0 + wave + 4 * j, M - 1);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float4 t = *reinterpret_cast<const float4*>(x + (long)m * ldx + 4 * (lane + 64 * c));
      xv[j][c][0] = t.x; xv[j][c][1] = t.y; xv[j][c][2] = t.z; xv[j][c][3] = t.w;
    }
  }
  if (ln_a) ln_rows512<4>(xv, ln_a, ln_b, lane);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float* d = &X[wave + 4 * j][4 * (lane + 64 * c)];
      *reinterpret_cast<float2*>(d) = make_float2(xv[j][c][0], xv[j][c][1]);
      *reinterpret_cast<float2*>(d + 2) = make_float2(xv[j][c][2], xv[j][c][3]);
    }
  __syncthreads();
  v4f acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q + 1 < 4) {
#pragma unroll
      for (int s = 0; s < 32; ++s)
        bq[(q + 1) & 1][s] = Wt[(long)(4 * (32 * (q + 1) + s) + fg) * V + vl];
    }
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      const float a = X[fr][4 * (32 * q + s) + fg];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bq[q & 1][s], acc, 0, 0, 0);
    }
  }
  if (vcol >= V) return;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int m = m0 + 4 * fg + e;
    if (m < M) logits[(long)m * V + vcol] = acc[e] + bv;
  }
}

hipError_t launch_generator_mfma(const float* x, long ldx, int M, const float* ln_a,
                                 const float* ln_b, const float* Wt, const float* b, int V,
                                 float* logits, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  k_generator_mfma<<<dim3((V + 63) / 64, (M + 15) / 16), dim3(256), 0, st>>>(
      x, ldx, M, ln_a, ln_b, Wt, b, V, logits);
  return hipGetLastError();
}

__global__ void k_transpose(const float* in, int R, int Cc, float* out) {
  __shared__ float t[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32, tx = threadIdx.x, ty = threadIdx.y;
  for (int i = ty; i < 32; i += 8)
    if (r0 + i < R && c0 + tx < Cc) t[i][tx] = in[(long)(r0 + i) * Cc + c0 + tx];
  __syncthreads();
  for (int i = ty; i < 32; i += 8)
    if (c0 + i < Cc && r0 + tx < R) out[(long)(c0 + i) * R + r0 + tx] = t[tx][i];
}
hipError_t launch_transpose(const float* in, int R, int Cc, float* out, hipStream_t st) {
  k_transpose<<<dim3((Cc + 31) / 32, (R + 31) / 32), dim3(32, 8), 0, st>>>(in, R, Cc, out);
  return hipGetLastError();
}

// =====================================================================================
// k_argmax_embed: one workgroup per row.  The row of logits is staged in LDS (all loads
// in flight), wave 0 runs the canonical reductions, then the block writes the next
// decoder input.
// =====================================================================================
constexpr int ARG_MAXV = 8192;

__global__ __launch_bounds__(256) void k_argmax_embed(const float* logits, int V, int64_t* ids,
                                                      long ids_bs, int* step, unsigned* arrive,
                                                      const float* lut, const float* pe,
                                                      int max_pos, float* xnext) {
  __shared__ float Lg[ARG_MAXV];
  __shared__ float Ev[ARG_MAXV];
  __shared__ float red[5], redv[4];
  __shared__ int redi[4], bsh;
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int s = *step;
  const float* x = logits + (long)m * V;
#pragma unroll
  for (int i = 0; i < ARG_MAXV / 256; ++i) {
    const int v = tid + 256 * i;
    if (v < V) Lg[v] = x[v];
  }
  // max: order-free, whole block
  float lm = -3.0e38f;
#pragma unroll
  for (int i = 0; i < ARG_MAXV / 256; ++i) {
    const int v = tid + 256 * i;
    if (v < V) lm = fmaxf(lm, Lg[v]);
  }
  lm = wave_max(lm);
  if (lane == 0) red[tid >> 6] = lm;
  __syncthreads();
  const float mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  // e_v = qexp(x_v - max) by the whole block, in place
#pragma unroll
  for (int i = 0; i < ARG_MAXV / 256; ++i) {
    const int v = tid + 256 * i;
    if (v < V) Ev[v] = qexp(Lg[v] - mx);
  }
  __syncthreads();
  // canonical denominator: lane l sums e[l], e[l+64], ... in order (one wave), then tree
  if (tid < 64) {
    float ls = 0.0f;
#pragma unroll 8
    for (int v = lane; v < V; v += 64) ls = ls + Ev[v];
    ls = wave_sum(ls);
    if (lane == 0) red[4] = logf(ls);
  }
  __syncthreads();
  const float lse = red[4];
  // first argmax of logp = (x - max) - lse (torch.max tie rule), block-wide
  float best = -3.0e38f;
  int bi = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < ARG_MAXV / 256; ++i) {
    const int v = tid + 256 * i;
    if (v < V) {
      const float lp = (Lg[v] - mx) - lse;
      if (lp > best) { best = lp; bi = v; }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float ob = __shfl_xor(best, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane == 0) { redv[tid >> 6] = best; redi[tid >> 6] = bi; }
  __syncthreads();
  if (tid == 0) {
    best = redv[0]; bi = redi[0];
    for (int w = 1; w < 4; ++w)
      if (redv[w] > best || (redv[w] == best && redi[w] < bi)) { best = redv[w]; bi = redi[w]; }
    bi = min(bi, V - 1);   // all-NaN row guard: keep the embedding gather in bounds
    ids[m * ids_bs + s + 1] = bi;
    bsh = bi;
  }
  __syncthreads();
  // next decoder input: tgt_embed(id) at position s + 1 (embeddings.py:12-13)
  if (tid < 128) {
    const int bi = bsh, p = min(s + 1, max_pos - 1);
    const float sc = 0x1.6a09e6p+4f;
    const float4 e = *reinterpret_cast<const float4*>(lut + (long)bi * 512 + 4 * tid);
    const float4 q = *reinterpret_cast<const float4*>(pe + (long)p * 512 + 4 * tid);
    *reinterpret_cast<float4*>(xnext + (long)m * 512 + 4 * tid) =
        make_float4(e.x * sc + q.x, e.y * sc + q.y, e.z * sc + q.z, e.w * sc + q.w);
  }
  // every workgroup has read *step above; the last one to arrive advances it
  if (tid == 0) {
    const unsigned tk = atomicAdd(arrive, 1u);
    if (tk == gridDim.x - 1) {
      *step = s + 1;
      *arrive = 0u;
    }
  }
}

hipError_t launch_argmax_embed(const float* logits, int M, int V, int64_t* ids, long ids_bs,
                               int* step, unsigned* arrive, const float* lut, const float* pe,
                               int max_pos, float* xnext, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (V > ARG_MAXV) return hipErrorInvalidValue;
  k_argmax_embed<<<dim3(M), dim3(256), 0, st>>>(logits, V, ids, ids_bs, step, arrive, lut, pe,
                                                max_pos, xnext);
  return hipGetLastError();
}

}  // namespace qtx
