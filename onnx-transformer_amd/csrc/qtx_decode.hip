// qtx_decode.hip — fused kernels of the KV-cached greedy decode step (gfx950, wave64).
//
//   k_skinny        M<=32-row int8 GEMM, 16 columns per workgroup, K split over 4 waves,
//                   A operand built in the prologue (int8 | LayerNorm+quant | rowmax-quant)
//                   quant_linear.py:111-119, layer_norm.py:12-15, position_feed_forward.py:12
//   k_dec_attn      one query per sentence, one wave per (sentence, head); quantizes q/k/v
//                   per token, appends k/v to the cache, attention; fp32 context + per-head
//                   absmax for the next GEMM's per-token quantization
//                   attention.py:23-67, get_quantized_model.py:160-168
//   k_generator_mfma final LayerNorm fused into the fp32 generator projection on fp32 MFMA
//                   generator.py:14-15, decoder.py:16
//   k_argmax_embed  log_softmax + first argmax + next-token embedding + step advance
//                   onnx_reference_inference.py:632,640-643
//
// All float steps follow the canonical order shared with oracle/qtx_oracle.py.
#include <cstdlib>

#include "qtx_common.h"
#include "qtx_kernels.h"
#include "qtx_knobs.h"

QTX_STAMP_SETTER(decode)

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

// =====================================================================================
// k_skinny
// =====================================================================================
// The A operand of a skinny GEMM workgroup (rows m0 .. m0 + RB - 1) into LDS: int8 rows
// (A_I8), LayerNorm + per-token quant of fp32 rows (A_LN), or per-token quant of fp32 rows
// from their partial maxima (A_F32Q).  Rows >= M are zero; sas = per-row scales.  Every
// branch issues all of its global loads before consuming any (one memory latency, not one
// per row).  Wave w takes rows w, w + 4, ...  issue_rest() (the weight fragments and the
// epilogue operands) is called right after the A operand's loads are issued: vmcnt retires
// in issue order, so the LayerNorm / quantization then waits for its own rows only and
// runs while the weights are in flight (measured: issuing the weights first made the two
// latencies add up, ~0.7 us per launch).
template <int RB, int K, int AMODE, class F>
__device__ __forceinline__ void skinny_prologue(const SkinnyArgs& g, uint8_t* As, float* sas,
                                                int m0, int tid, int wave, int lane,
                                                F&& issue_rest) {
  constexpr int LDA = K + 16;
  constexpr int BM = RB <= 16 ? 16 : 32;
  constexpr int RPW = RB / 4;  // rows per wave: r = wave + 4*j
  if constexpr (AMODE == A_I8) {
    // the panel is RB*K/16 uint4; the index is clamped (a duplicate load, no divergent
    // branch around the load) and only in-range indices are stored
    constexpr int CPR = K / 16, TOT = RB * CPR, NLD = (TOT + 255) / 256;
    uint4 v[NLD];
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int idx = min(tid + 256 * j, TOT - 1), m = min(m0 + idx / CPR, g.M - 1);
      v[j] = ld_at(reinterpret_cast<const uint4*>(g.A), (unsigned)(m * K + 16 * (idx % CPR)));
    }
    issue_rest();
    if (tid < BM) sas[tid] = (tid < RB && m0 + tid < g.M) ? g.sa[m0 + tid] : 0.0f;
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int idx = tid + 256 * j, r = idx / CPR;
      if (TOT % 256 == 0 || idx < TOT)
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
        const float4 t = ld_at(reinterpret_cast<const float4*>(g.X), 4u * (unsigned)(m * (int)g.ldx + 4 * (lane + 64 * c)));
        v[j][c][0] = t.x; v[j][c][1] = t.y; v[j][c][2] = t.z; v[j][c][3] = t.w;
      }
    }
    float ga[2][4], gb[2][4];
    ln_params512(g.ln_a, g.ln_b, lane, ga, gb);
    issue_rest();
    uint32_t q[RPW][2];
    float sc[RPW];
#if defined(QTX_ABL) && (QTX_ABL & 2)   // diagnostic builds only: no LayerNorm / quant chain
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      q[j][0] = __float_as_uint(v[j][0][0]); q[j][1] = __float_as_uint(v[j][1][0]); sc[j] = v[j][0][1];
    }
#else
    ln_rows512<RPW>(v, ga, gb);
    quant_rows512<RPW>(v, q, sc);
#endif
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int r = wave + 4 * j;
      const bool ok = m0 + r < g.M;
      uint32_t* dst = reinterpret_cast<uint32_t*>(As + r * LDA);
      dst[lane] = ok ? q[j][0] : 0u;
      dst[lane + 64] = ok ? q[j][1] : 0u;
      if (lane == 0) sas[r] = ok ? sc[j] : 0.0f;
    }
  } else {  // A_F32Q: each wave's rows (<= 4 at a time) with their partial maxima
            // A_F32R: the same rows, the row maximum from the row itself
    constexpr bool OWN = AMODE == A_F32R;
    constexpr int NC = K / 256, RBT = RPW < 4 ? RPW : 4;
#pragma unroll
    for (int j0 = 0; j0 < RPW; j0 += RBT) {
      float4 t[RBT][NC];
      float pm[RBT][2];
#pragma unroll
      for (int jb = 0; jb < RBT; ++jb) {
        const int m = min(m0 + wave + 4 * (j0 + jb), g.M - 1);
#pragma unroll
        for (int c = 0; c < NC; ++c)
          t[jb][c] = ld_at(reinterpret_cast<const float4*>(g.X), 4u * (unsigned)(m * (int)g.ldx + 4 * (lane + 64 * c)));
        if constexpr (!OWN)
#pragma unroll
          for (int u = 0; u < 2; ++u)   // lane takes partials lane, lane+64 (clamped: max-safe)
            pm[jb][u] = ld_at(g.pmax_in, 4u * (unsigned)(min(lane + 64 * u, g.pmax_n - 1) * g.M + m));
      }
      if (j0 == 0) issue_rest();
#pragma unroll
      for (int jb = 0; jb < RBT; ++jb) {
        const int r = wave + 4 * (j0 + jb);
        const bool ok = m0 + r < g.M;
        float lm;
        if constexpr (OWN) {   // |x| max of this lane's values (fmaxf: NaN drops out as in
          lm = 0.0f;           // the partial maxima the producer would have formed)
#pragma unroll
          for (int c = 0; c < NC; ++c)
            lm = fmaxf(lm, fmaxf(fmaxf(fabsf(t[jb][c].x), fabsf(t[jb][c].y)),
                                 fmaxf(fabsf(t[jb][c].z), fabsf(t[jb][c].w))));
        } else {
          lm = fmaxf(pm[jb][0], pm[jb][1]);
        }
        const float sc = quant_scale(wave_max(lm), 127.0f);
        uint32_t* dst = reinterpret_cast<uint32_t*>(As + r * LDA);
        float tf[4 * NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          tf[4 * c] = t[jb][c].x; tf[4 * c + 1] = t[jb][c].y;
          tf[4 * c + 2] = t[jb][c].z; tf[4 * c + 3] = t[jb][c].w;
        }
        uint32_t qd[NC];
#if defined(QTX_ABL) && (QTX_ABL & 8)   // diagnostic builds only: no per-token quantization
#pragma unroll
        for (int c = 0; c < NC; ++c) qd[c] = __float_as_uint(tf[4 * c] * sc);
#else
        quant_pack<4 * NC>(tf, sc, qd);
#endif
#pragma unroll
        for (int c = 0; c < NC; ++c) dst[lane + 64 * c] = ok ? qd[c] : 0u;
        if (lane == 0) sas[r] = ok ? sc : 0.0f;
      }
    }
  }
}

template <int MF, int RB, int K, int WBITS, int AMODE, int FLAGS>
__global__ __launch_bounds__(256) void k_skinny(SkinnyArgs g) {
  constexpr int BM = 16 * MF;     // MFMA rows (rows >= RB of the A panel are don't-care)
  static_assert(RB % 4 == 0 && RB <= BM, "rows per block");
  constexpr int KW = K / 4;       // K range of one wave
  constexpr int NS = KW / 64;     // MFMA k-steps per wave
  constexpr int LDA = K + 16;     // padded LDS row (bytes)
  __shared__ __attribute__((aligned(16))) uint8_t As[BM * LDA];
  __shared__ float sas[BM];
  __shared__ v4i red[4][MF][64];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * RB;

  QTX_STAMP(0);

  // 1. this lane's W fragments for its wave's K range, and the epilogue operands of wave 0
  //    (it finishes the tile: a load first issued after the reduction barrier would add a
  //    whole memory round trip) — issued right after the A operand's loads (prologue)
  const int n = min(n0 + fr, g.N - 1);
  uint4 wf[NS];
  uint2 wp[NS];
  const int col = n0 + fr;
  const bool cok = col < g.N;
  float swc = 0.0f, bc = 0.0f, rv[MF];
  constexpr bool resid = FLAGS & EPI_RESIDUAL;
  auto issue_rest = [&]() {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int k = wave * KW + 64 * s + 16 * fg;
#if defined(QTX_ABL) && (QTX_ABL & 1)   // diagnostic builds only: no weight loads
      wf[s] = make_uint4(n + k, k, n, 1); wp[s] = make_uint2(n, k);
#else
      if constexpr (WBITS == 8)
        wf[s] = ld_at(reinterpret_cast<const uint4*>(g.W), (unsigned)(n * (int)g.ldw + k));
      else
        wp[s] = ld_at(reinterpret_cast<const uint2*>(g.W), (unsigned)(n * (int)g.ldw + (k >> 1)));
#endif
    }
    // every wave, unconditionally, at clamped addresses (values of rows / columns outside
    // the tile are never stored): a load under a branch makes the compiler's vmcnt for the
    // prologue's own loads count the branch-free path, i.e. wait for the weights too
    const int cc = min(col, g.N - 1);
    swc = ld_at(g.sw, 4u * cc);
    bc = ld_at(g.bias, 4u * cc);
    if constexpr (resid) {   // the rows this wave finishes: 4 fg + wave of each tile
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const int row = min(m0 + 16 * i + 4 * fg + wave, g.M - 1);
        rv[i] = ld_at(g.res, 4u * (unsigned)(row * (int)g.ldr + cc));
      }
    }
  };

  // 2. A panel (int8) and per-row scales into LDS
  skinny_prologue<RB, K, AMODE>(g, As, sas, m0, tid, wave, lane, issue_rest);
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
#if defined(QTX_ABL) && (QTX_ABL & 4)   // diagnostic builds only: no matrix work
      acc[i] += afr ^ bfr;
#else
      acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr, bfr, acc[i], 0, 0, 0);
#endif
    }
  }

  // 4. exact int32 reduction of the 4 K ranges
#pragma unroll
  for (int i = 0; i < MF; ++i) red[wave][i][lane] = acc[i];
  __syncthreads();
  QTX_STAMP(2);
  // 5. epilogue, split over the waves: wave w finishes element e = w of every lane's four
  //    (C layout: col = lane & 15, row = 4*(lane>>4) + e), its int32 sum over the 4 K ranges
  //    exact in any order
  constexpr bool relu = FLAGS & EPI_RELU, rmax = FLAGS & EPI_ROWMAX;
  const int e = wave;
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    {
      int sum = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) sum += reinterpret_cast<const int*>(&red[w][i][lane])[e];
      const int r = 16 * i + 4 * fg + e, row = m0 + r;
      const bool ok = cok && r < RB && row < g.M;
      float y = ((float)sum * sas[r]) * swc + bc;
      if constexpr (relu) y = y > 0.0f ? y : 0.0f;
      if constexpr (resid) y = rv[i] + y;
      if (ok) st_at(g.out, 4u * (unsigned)(row * (int)g.ldo + col), y);
      if constexpr (rmax) {
        float am = ok ? fabsf(y) : 0.0f;   // max over the 16 lanes (columns) of this row
        am = fmaxf(am, dpp<0xB1>(am));
        am = fmaxf(am, dpp<0x4E>(am));
        am = fmaxf(am, dpp<0x141>(am));
        am = fmaxf(am, dpp<0x140>(am));
        if (fr == 0 && r < RB && row < g.M) g.pmax_out[(long)blockIdx.x * g.M + row] = am;
      }
    }
  }
  QTX_STAMP(3);
}

// =====================================================================================
// k_skinny8: the decode FFN2 (K = 2048, fp32 hidden quantized per token from its partial
// maxima, residual epilogue) on 8 waves: two waves per row quantize one half of it each
// (16 values per lane: half the dependent quantization chain of k_skinny's one row per
// wave), K split 8 ways (4 weight fragments per lane), exact int32 reduction over the 8
// waves.  Rows per workgroup 4, 16 columns.  Bit-identical to k_skinny.
// OWN (A_F32R): the row maximum from the row itself — each wave's half-row maximum, the two
// halves met through LDS — instead of FFN1's per-tile partial maxima.
// =====================================================================================
template <bool OWN>
__global__ __launch_bounds__(512) void k_skinny8_ffn2(SkinnyArgs g) {
  constexpr int K = 2048, RB = 4, KW = K / 8, NS = KW / 64, LDA = K + 16;
  __shared__ __attribute__((aligned(16))) uint8_t As[16 * LDA];
  __shared__ float sas[16];
  __shared__ v4i red[8][64];
  __shared__ float hmax[8];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * RB;
  // 1. the A operand's loads first: row r = wave / 2, half = wave & 1 (1024 values)
  const int r = wave >> 1, half = wave & 1;
  const int m = min(m0 + r, g.M - 1);
  float4 t[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
    t[c] = ld_at(reinterpret_cast<const float4*>(g.X), 4u * (unsigned)(m * (int)g.ldx + 4 * (lane + 64 * (4 * half + c))));
  float pm[2] = {0.0f, 0.0f};
  if constexpr (!OWN)
#pragma unroll
    for (int u = 0; u < 2; ++u) pm[u] = ld_at(g.pmax_in, 4u * (unsigned)(min(lane + 64 * u, g.pmax_n - 1) * g.M + m));
  // 2. then this wave's weight fragments and (wave 0) the epilogue operands
  const int n = min(n0 + fr, g.N - 1);
  uint4 wf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s)
    wf[s] = ld_at(reinterpret_cast<const uint4*>(g.W), (unsigned)(n * (int)g.ldw + wave * KW + 64 * s + 16 * fg));
  const int col = n0 + fr, cc = min(col, g.N - 1);
  const bool cok = col < g.N;
  const float swc = ld_at(g.sw, 4u * cc), bc = ld_at(g.bias, 4u * cc);
  // the epilogue's output of this lane (wave 0): row m0 + (lane >> 4), column n0 + (lane & 15)
  const float rv = ld_at(g.res, 4u * (unsigned)(min(m0 + fg, g.M - 1) * (int)g.ldr + cc));
  // 3. per-token quantization of the half row into LDS
  {
    const bool ok = m0 + r < g.M;
    float rmax;
    if constexpr (OWN) {
      float lm = 0.0f;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        lm = fmaxf(lm, fmaxf(fmaxf(fabsf(t[c].x), fabsf(t[c].y)), fmaxf(fabsf(t[c].z), fabsf(t[c].w))));
      lm = wave_max(lm);
      if (lane == 0) hmax[wave] = lm;
      __syncthreads();
      rmax = fmaxf(hmax[2 * r], hmax[2 * r + 1]);
    } else {
      rmax = wave_max(fmaxf(pm[0], pm[1]));
    }
    const float sc = quant_scale(rmax, 127.0f);
    float tf[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      tf[4 * c] = t[c].x; tf[4 * c + 1] = t[c].y; tf[4 * c + 2] = t[c].z; tf[4 * c + 3] = t[c].w;
    }
    uint32_t qd[4];
    quant_pack<16>(tf, sc, qd);
    uint32_t* dst = reinterpret_cast<uint32_t*>(As + r * LDA);
#pragma unroll
    for (int c = 0; c < 4; ++c) dst[lane + 64 * (4 * half + c)] = ok ? qd[c] : 0u;
    if (lane == 0 && half == 0) sas[r] = ok ? sc : 0.0f;
  }
  __syncthreads();
  // 4. MFMA over this wave's K range, exact int32 reduction of the 8 ranges
  v4i acc = v4i{0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const v4i afr = *reinterpret_cast<const v4i*>(As + fr * LDA + wave * KW + 64 * s + 16 * fg);
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr, __builtin_bit_cast(v4i, wf[s]), acc, 0, 0, 0);
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave != 0) return;
  // 5. epilogue: out = res + y.  The RB = 4 useful rows of the 16-row tile sit in lanes
  //    0-15 (element e = row); wave 0 takes one output per lane — lane l: row e = l >> 4,
  //    column l & 15 — summing element e of lane l & 15 over the 8 K ranges (exact int32;
  //    conflict-free LDS reads)
  {
    const int e = fg, src = fr;
    int sum = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) sum += reinterpret_cast<const int*>(&red[w][src])[e];
    const int row = m0 + e;
    const float y = ((float)sum * sas[e]) * swc + bc;
    if (cok && row < g.M) st_at(g.out, 4u * (unsigned)(row * (int)g.ldo + col), rv + y);
  }
}

// =====================================================================================
// k_skinny_wide: the K = 512 skinny GEMM with N split over the 4 waves instead of K — a
// workgroup covers 64 columns (wave w: columns n0 + 16w .. +15, all 8 K steps, 8 weight
// fragments = 128 B per lane in flight) and its RB rows; no cross-wave reduction.  The
// prologue (LayerNorm + quant of the RB rows, or their per-token quant) then serves 64
// columns instead of 16: 4x fewer redundant LayerNorms per launch.  Same int32 sums, same
// epilogue arithmetic: bit-identical to k_skinny.
// =====================================================================================
template <int RB, int WBITS, int AMODE, int FLAGS>
__global__ __launch_bounds__(256) void k_skinny_wide(SkinnyArgs g) {
  constexpr int K = 512, NS = K / 64, LDA = K + 16;
  static_assert(RB % 4 == 0 && RB <= 16, "rows per block");
  __shared__ __attribute__((aligned(16))) uint8_t As[16 * LDA];
  __shared__ float sas[16];
  // RB = 4 / 8: each wave's useful C rows (lanes 0 .. 4 RB - 1), remapped through LDS
  constexpr int RPL = RB / 4;                        // outputs per lane after the remap
  constexpr bool REMAP = RB == 4 || RB == 8;
  __shared__ v4i tail[REMAP ? 4 : 1][REMAP ? 4 * RB : 1];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int n0 = blockIdx.x * 64 + 16 * wave, m0 = blockIdx.y * RB;
  QTX_STAMP(0);
  // 1. this lane's W fragments (all of K) and the epilogue operands of the wave's 16
  //    columns — issued right after the A operand's loads (prologue)
  const int n = min(n0 + fr, g.N - 1);
  uint4 wf[NS];
  uint2 wp[NS];
  const int col = n0 + fr;
  const bool cok = col < g.N;
  constexpr bool resid = FLAGS & EPI_RESIDUAL;
  float swc, bc, rv[4];
  auto issue_rest = [&]() {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int k = 64 * s + 16 * fg;
#if defined(QTX_ABL) && (QTX_ABL & 1)   // diagnostic builds only: no weight loads
      wf[s] = make_uint4(n + k, k, n, 1); wp[s] = make_uint2(n, k);
#else
      if constexpr (WBITS == 8)
        wf[s] = ld_at(reinterpret_cast<const uint4*>(g.W), (unsigned)(n * (int)g.ldw + k));
      else
        wp[s] = ld_at(reinterpret_cast<const uint2*>(g.W), (unsigned)(n * (int)g.ldw + (k >> 1)));
#endif
    }
    swc = cok ? ld_at(g.sw, 4u * col) : 0.0f;
    bc = cok ? ld_at(g.bias, 4u * col) : 0.0f;
    if constexpr (RB == 4) {   // the epilogue's one output per lane: row m0 + fg
      rv[0] = (resid && cok && m0 + fg < g.M) ? ld_at(g.res, 4u * (unsigned)((m0 + fg) * (int)g.ldr + col)) : 0.0f;
    } else if constexpr (RB == 8) {   // its two: rows m0 + fg, m0 + fg + 4
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = m0 + fg + 4 * j;
        rv[j] = (resid && cok && row < g.M) ? ld_at(g.res, 4u * (unsigned)(row * (int)g.ldr + col)) : 0.0f;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * fg + e, row = m0 + r;
        rv[e] = (resid && cok && r < RB && row < g.M) ? ld_at(g.res, 4u * (unsigned)(row * (int)g.ldr + col)) : 0.0f;
      }
    }
  };
  // 2. A panel and per-row scales into LDS
  skinny_prologue<RB, K, AMODE>(g, As, sas, m0, tid, wave, lane, issue_rest);
  __syncthreads();
  QTX_STAMP(1);
  // 3. MFMA over all of K
  v4i acc = v4i{0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    v4i bfr;
    if constexpr (WBITS == 8) bfr = __builtin_bit_cast(v4i, wf[s]);
    else bfr = __builtin_bit_cast(v4i, unpack_i4(wp[s]));
    const v4i afr = *reinterpret_cast<const v4i*>(As + fr * LDA + 64 * s + 16 * fg);
#if defined(QTX_ABL) && (QTX_ABL & 4)   // diagnostic builds only: no matrix work
    acc += afr ^ bfr;
#else
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr, bfr, acc, 0, 0, 0);
#endif
  }
  QTX_STAMP(2);
  // 4. epilogue (C layout: col = lane & 15, row = 4*(lane>>4) + e)
  constexpr bool relu = FLAGS & EPI_RELU, rmax = FLAGS & EPI_ROWMAX;
  if constexpr (RB == 4) {
    // the 4 useful rows are elements 0-3 of lanes 0-15: through the wave's own LDS slot
    // (in-order within the wave, conflict-free) lane l takes row l >> 4 of column l & 15 —
    // one output per lane instead of four on a quarter of the lanes
    if (fg == 0) tail[wave][fr] = acc;
    // (no instruction: keeps the compiler from moving the other lanes' reads above the
    // store — the hardware keeps one wave's LDS operations in order)
    __builtin_amdgcn_wave_barrier();
    const int v = reinterpret_cast<const int*>(&tail[wave][fr])[fg];
    const int row = m0 + fg;
    const bool ok = cok && row < g.M;
    float y = ((float)v * sas[fg]) * swc + bc;
    if constexpr (relu) y = y > 0.0f ? y : 0.0f;
    if constexpr (resid) y = rv[0] + y;
    if (ok) st_at(g.out, 4u * (unsigned)(row * (int)g.ldo + col), y);
    if constexpr (rmax) {
      float am = ok ? fabsf(y) : 0.0f;   // max over the 16 lanes (columns) of this row
      am = fmaxf(am, dpp<0xB1>(am));
      am = fmaxf(am, dpp<0x4E>(am));
      am = fmaxf(am, dpp<0x141>(am));
      am = fmaxf(am, dpp<0x140>(am));
      if (fr == 0 && row < g.M) g.pmax_out[(long)(n0 >> 4) * g.M + row] = am;
    }
    QTX_STAMP(3);
    return;
  }
  if constexpr (RB == 8) {
    // the 8 useful rows are elements 0-3 of lanes 0-31 (row 4 (l >> 4) + e): the same
    // remap, lane l takes rows (l >> 4) and (l >> 4) + 4 of column l & 15 — two outputs per
    // lane instead of four on half of the lanes
    if (fg < RPL) tail[wave][16 * fg + fr] = acc;
    __builtin_amdgcn_wave_barrier();      // as at RB == 4
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      const int v = reinterpret_cast<const int*>(&tail[wave][16 * j + fr])[fg];
      const int r = fg + 4 * j, row = m0 + r;
      const bool ok = cok && row < g.M;
      float y = ((float)v * sas[r]) * swc + bc;
      if constexpr (relu) y = y > 0.0f ? y : 0.0f;
      if constexpr (resid) y = rv[j] + y;
      if (ok) st_at(g.out, 4u * (unsigned)(row * (int)g.ldo + col), y);
      if constexpr (rmax) {
        float am = ok ? fabsf(y) : 0.0f;   // max over the 16 lanes (columns) of this row
        am = fmaxf(am, dpp<0xB1>(am));
        am = fmaxf(am, dpp<0x4E>(am));
        am = fmaxf(am, dpp<0x141>(am));
        am = fmaxf(am, dpp<0x140>(am));
        if (fr == 0 && row < g.M) g.pmax_out[(long)(n0 >> 4) * g.M + row] = am;
      }
    }
    QTX_STAMP(3);
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int r = 4 * fg + e, row = m0 + r;
    const bool ok = cok && r < RB && row < g.M;
    float y = ((float)acc[e] * sas[r]) * swc + bc;
    if constexpr (relu) y = y > 0.0f ? y : 0.0f;
    if constexpr (resid) y = rv[e] + y;
    if (ok) st_at(g.out, 4u * (unsigned)(row * (int)g.ldo + col), y);
    if constexpr (rmax) {
      float am = ok ? fabsf(y) : 0.0f;   // max over the 16 lanes (columns) of this row
      am = fmaxf(am, dpp<0xB1>(am));
      am = fmaxf(am, dpp<0x4E>(am));
      am = fmaxf(am, dpp<0x141>(am));
      am = fmaxf(am, dpp<0x140>(am));
      if (fr == 0 && r < RB && row < g.M) g.pmax_out[(long)(n0 >> 4) * g.M + row] = am;
    }
  }
  QTX_STAMP(3);
}

template <int RB, int WB, int AM>
hipError_t skinny_wide_flags(const SkinnyArgs& g, hipStream_t st) {
  const dim3 grid(g.N / 64, (g.M + RB - 1) / RB);
  switch (g.flags) {
    case 0: k_skinny_wide<RB, WB, AM, 0><<<grid, 256, 0, st>>>(g); break;
    case EPI_RELU: k_skinny_wide<RB, WB, AM, EPI_RELU><<<grid, 256, 0, st>>>(g); break;
    case EPI_RESIDUAL: k_skinny_wide<RB, WB, AM, EPI_RESIDUAL><<<grid, 256, 0, st>>>(g); break;
    case EPI_RELU | EPI_ROWMAX:
      k_skinny_wide<RB, WB, AM, EPI_RELU | EPI_ROWMAX><<<grid, 256, 0, st>>>(g);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
template <int WB, int AM>
hipError_t skinny_wide_rb(const SkinnyArgs& g, int rb, hipStream_t st) {
  switch (rb) {
    case 4: return skinny_wide_flags<4, WB, AM>(g, st);
    case 8: return skinny_wide_flags<8, WB, AM>(g, st);
    case 16: return skinny_wide_flags<16, WB, AM>(g, st);
    default: return hipErrorInvalidValue;
  }
}

// dispatch: the prologue mode and epilogue flags are template parameters (no runtime
// branches per output element).  Supported: K 512 with A_I8 / A_LN, K 2048 with A_I8 /
// A_F32Q; flags 0, RELU, RESIDUAL, RELU|ROWMAX.  Rows per workgroup RB: 16*MF for an int8
// A panel; 4 (one row per wave) for the LayerNorm prologue, which re-normalizes its rows
// in every column workgroup — few rows per workgroup keeps that short and spreads the
// fp32 row reads over many CUs (measured: RB 32 -> 8 -> 4 = 11.0 -> 5.1 -> 4.6 us for
// N=1536, M=32; in the decode step the fused form beats LN kernel + GEMM).
template <int MF, int RB, int K, int WB, int AM>
hipError_t skinny_flags(const SkinnyArgs& g, hipStream_t st) {
  const dim3 grid(g.N / 16, (g.M + RB - 1) / RB);
  switch (g.flags) {
    case 0: k_skinny<MF, RB, K, WB, AM, 0><<<grid, 256, 0, st>>>(g); break;
    case EPI_RELU: k_skinny<MF, RB, K, WB, AM, EPI_RELU><<<grid, 256, 0, st>>>(g); break;
    case EPI_RESIDUAL: k_skinny<MF, RB, K, WB, AM, EPI_RESIDUAL><<<grid, 256, 0, st>>>(g); break;
    case EPI_RELU | EPI_ROWMAX:
      k_skinny<MF, RB, K, WB, AM, EPI_RELU | EPI_ROWMAX><<<grid, 256, 0, st>>>(g);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
template <int K, int WB, int AM>
hipError_t skinny_rb(const SkinnyArgs& g, int rb, hipStream_t st) {
  switch (rb) {
    case 4: return skinny_flags<1, 4, K, WB, AM>(g, st);
    case 8: return skinny_flags<1, 8, K, WB, AM>(g, st);
    case 16: return skinny_flags<1, 16, K, WB, AM>(g, st);
    case 32: return skinny_flags<2, 32, K, WB, AM>(g, st);
    default: return hipErrorInvalidValue;
  }
}
// Rows per workgroup (decode step, M = 32, measured in bench.py; tools/rb_sweep.sh: the
// K = 512 int8 / F32Q row block 8 -> 4 took the step 234.8 -> 230.3 us): small row blocks spread
// the A-panel and weight reads over more CUs — each CU sustains only a few KB in flight,
// so a latency-bound kernel is fastest when every workgroup touches ~10-40 KB.
template <int WB>
hipError_t skinny_mode(const SkinnyArgs& g, hipStream_t st) {
  // The N-split workgroup (k_skinny_wide) for the LayerNorm-prologue GEMMs with N >= 1024
  // (LN+QKV, LN+FFN1): measured in the decode graph at M = 32 (tools/kernel_chain.py)
  // 4.50 -> 3.67 and 5.26 -> 3.95 us per launch; at N = 512 the K-split one is faster
  // (64 workgroups of 32 KB each vs 256 of 8 KB: 3.09 vs 3.60 us).  QTX_SKINNY_WIDE=0: never,
  // =<rb>: every K = 512 launch (experiments).
  // From M >= 96 (the decode of >= 96 sentences per sub-batch, e.g. cfg5's 256 per GPU) the
  // small blocks re-read W once per 4 rows: there every K = 512 GEMM runs N-split with 8-row
  // blocks, and FFN2 (whose hidden the decode step then quantizes with its own kernel,
  // qtx_api.hip greedy_step_fused) takes 16-row blocks — or 8 / 16 with the fp32 prologue
  // (tools/rb_sweep256.py, profiles/r05_rb_sweep.md: B = 256 decode 35.0 -> 27.5 ms,
  // B = 128 23.1 -> 21.0 ms; at B = 32 / 64 the small blocks stay faster).
  const Knobs& kn = knobs();     // QTX_SKINNY_WIDE / QTX_RB_* / QTX_SKINNY8_MAXM: QTX_DIAG build
  const bool big = g.M >= 96;
  const int wide_env = kn.skinny_wide;
  const bool wide = wide_env < 0 ? ((g.amode == A_LN && g.N >= 1024) || big) : wide_env > 0;
  if (wide && g.K == 512 && g.N % 64 == 0) {
    const int rb = wide_env > 0 && g.M > 4 ? wide_env : (big ? 8 : 4);
    if (g.amode == A_I8) return skinny_wide_rb<WB, A_I8>(g, rb, st);
    if (g.amode == A_LN) return skinny_wide_rb<WB, A_LN>(g, rb, st);
    if (g.amode == A_F32Q) return skinny_wide_rb<WB, A_F32Q>(g, rb, st);
    if (g.amode == A_F32R) return skinny_wide_rb<WB, A_F32R>(g, rb, st);
  }
  if (g.K == 512) {
    const int rb_i8 = kn.rb_i8_512, rb_ln = kn.rb_ln;
    if (g.amode == A_I8) return skinny_rb<512, WB, A_I8>(g, g.M <= 4 ? 4 : rb_i8, st);
    if (g.amode == A_LN) return skinny_rb<512, WB, A_LN>(g, rb_ln, st);
    if (g.amode == A_F32Q) return skinny_rb<512, WB, A_F32Q>(g, g.M <= 4 ? 4 : rb_i8, st);
    if (g.amode == A_F32R) return skinny_rb<512, WB, A_F32R>(g, g.M <= 4 ? 4 : rb_i8, st);
  } else if (g.K == 2048) {
    // the decode FFN2 (fp32 hidden, residual, 8-bit weights) at M <= QTX_SKINNY8_MAXM
    // (default 32): 8 waves (measured: B = 32 decode 14.45 -> 14.40 ms; at B = 256 the
    // 4-wave kernel is faster, 35.1 vs 36.8 ms)
    const int sk8_maxm = kn.skinny8_maxm;
    if (g.M <= sk8_maxm && WB == 8 && g.flags == EPI_RESIDUAL &&
        ((g.amode == A_F32Q && g.pmax_n <= 128) || g.amode == A_F32R)) {
      if (g.amode == A_F32R)
        k_skinny8_ffn2<true><<<dim3(g.N / 16, (g.M + 3) / 4), 512, 0, st>>>(g);
      else
        k_skinny8_ffn2<false><<<dim3(g.N / 16, (g.M + 3) / 4), 512, 0, st>>>(g);
      return hipGetLastError();
    }
    const int rb_i8 = kn.rb_i8_2048 > 0 ? kn.rb_i8_2048 : (big ? 16 : 4);
    const int rb_f = kn.rb_f32q > 0 ? kn.rb_f32q : (g.M >= 192 ? 16 : big ? 8 : 4);
    if (g.amode == A_I8) return skinny_rb<2048, WB, A_I8>(g, rb_i8, st);
    if (g.amode == A_F32Q) return skinny_rb<2048, WB, A_F32Q>(g, rb_f, st);
    if (g.amode == A_F32R) return skinny_rb<2048, WB, A_F32R>(g, rb_f, st);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_skinny(const SkinnyArgs& g, int wbits, hipStream_t st) {
  if (g.M <= 0) return hipSuccess;
  if (g.N % 16) return hipErrorInvalidValue;
  // the kernels address X / res / A / W with 32-bit byte offsets (ld_at)
  const long lim = 1L << 30;
  if ((long)g.M * (g.ldx > g.K ? g.ldx : g.K) >= lim || (long)g.M * g.ldr >= lim ||
      (long)g.M * g.ldo >= lim || (long)g.N * g.ldw >= lim || (long)g.M * g.pmax_n >= lim)
    return hipErrorInvalidValue;
  if (wbits == 8) return skinny_mode<8>(g, st);
  if (wbits == 4) return skinny_mode<4>(g, st);
  return hipErrorInvalidValue;
}

// =====================================================================================
// k_dec_attn: one wave per (sentence, head) — 8*B workgroups, so the cached keys/values
// (the bulk of the bytes) are spread over many CUs instead of one CU per sentence.  Each
// wave quantizes the q (and new k/v) row itself (full-row maxima recomputed per head:
// 2-6 KB of reads), attends over its head and writes its 64 fp32 context values plus
// their absmax; the per-token quantization of the context row happens in the prologue of
// the output-projection GEMM (A_F32Q), so no cross-workgroup step is needed here.
// Keys staged in LDS (<= 128).  Grid (B, 8): the 8 heads of sentence b share blockIdx.x,
// so with B % 8 == 0 they land on one XCD (workgroups go round-robin over the 8 XCDs).
// The value cache is kept in groups of 4 keys (round 6): byte ((b * G4 + j / 4) * 512 + d) * 4
// + j % 4 holds v[b][j][d] (G4 = ceil(kv_bs / 4)), so one dword is 4 consecutive keys of one
// dim — the PV's 4-key step in one ds_read_b32 and 4 SDWA conversions instead of 4 byte
// reads.  Key rows are staged 20 dwords apart (16 B aligned: ds_read_b128 / ds_write_b128,
// conflict-free: 20 j mod 64 steps through distinct 4-bank groups over 16 lanes).
// =====================================================================================
constexpr int DEC_MAXK = 128;
constexpr int DEC_KST = 20;   // staged key row stride in dwords

template <bool KV_NEW, int NIT>
__global__ __launch_bounds__(64) void k_dec_attn(DecAttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t Ks[DEC_MAXK * DEC_KST];   // key rows of this head
  // values of this head, 4-key groups: dword g * 64 + d = keys 4g .. 4g + 3 of dim d
  __shared__ __attribute__((aligned(16))) uint8_t Vs[DEC_MAXK * 64];
  __shared__ float svs[DEC_MAXK];
  __shared__ __attribute__((aligned(16))) float PS[DEC_MAXK];   // RN(P_j * s_v[j]), 0 past Sk
  __shared__ __attribute__((aligned(16))) int8_t qs[64];
  const int b = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  QTX_STAMP(0);
  const float* yr = a.y + (long)b * a.ldy;
  // rows staged (self: rows 0 .. the position when the host passes it, else all allocated)
  const int nrows = KV_NEW ? (a.host_step1 > 0 ? a.host_step1 : (int)a.kv_bs) : a.S;
  const long kvb = (long)b * a.kv_bs;
  const long vgb = (long)b * ((a.kv_bs + 3) >> 2);     // the sentence's first value group

  // phase 0: every global load first (one memory latency): this step's q (k, v) rows
  // first — vmcnt retires in issue order, so their quantization (phase 1) then runs while
  // the cached keys and values are in flight — then the key/value rows of this head (row r
  // = 4 uint4; lane takes row 16*i + lane/4, chunk lane%4; clamped: no divergent loads)
  float4 yq[2], yk[2], yv[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    yq[c] = *reinterpret_cast<const float4*>(yr + 4 * (lane + 64 * c));
    if constexpr (KV_NEW) {
      yk[c] = *reinterpret_cast<const float4*>(yr + 512 + 4 * (lane + 64 * c));
      yv[c] = *reinterpret_cast<const float4*>(yr + 1024 + 4 * (lane + 64 * c));
    }
  }
  const float q_own = yr[h * 64 + lane];
  const float k_own = KV_NEW ? yr[512 + h * 64 + lane] : 0.0f;
  const float v_own = KV_NEW ? yr[1024 + h * 64 + lane] : 0.0f;
  // clamped: a stale position (a counter not reset) must not index past the cache
  const int step = !KV_NEW ? 0 : a.host_step1 > 0 ? a.host_step1 - 1 : min(max(*a.step, 0), (int)a.kv_bs - 1);
  const int rsub = lane >> 2, ch = lane & 3;
  // values: per 16 keys, 4 groups x this head's 64 dims x 4 B = 1 KB, lane = group
  // 4 i + lane / 16, dims 4 (lane % 16) .. + 3
  const int vg = lane >> 4, vd = 4 * (lane & 15), glast = (nrows - 1) >> 2;
  // wave-uniform bases of this head's rows and 32-bit lane offsets: the loads take the
  // scalar-base + vector-offset form instead of 64-bit address arithmetic per load
  const int8_t* const kbase = a.kc + kvb * 512 + h * 64;
  const int8_t* const vbase = a.vc + vgb * 2048 + h * 256;
  uint4 kr[NIT], vr[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const unsigned koff = (unsigned)(min(16 * i + rsub, nrows - 1) * 512 + 16 * ch);
    const unsigned voff = (unsigned)(min(4 * i + vg, glast) * 2048 + 4 * vd);
    // non-temporal: each K/V row is read once per step by one wave, so it should not push
    // the weights (re-read every step) out of the XCD's L2 (B = 256: 36.2 -> 35.1 ms; the
    // default policy re-measured in round 6: B = 32 12.87 vs 12.84, B = 256 26.25 vs 25.58 ms)
    kr[i] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const v4i*>(kbase + koff)));
    vr[i] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const v4i*>(vbase + voff)));
  }
  const int j0 = min(lane, nrows - 1), j1 = min(lane + 64, nrows - 1);
  const float* const skb = a.skc + kvb;
  const float* const svb = a.svc + kvb;
  float sk0 = skb[(unsigned)j0], sk1 = skb[(unsigned)j1];
  const float sv0 = svb[(unsigned)j0], sv1 = svb[(unsigned)j1];
  bool keep0 = true, keep1 = true;
  if constexpr (!KV_NEW) {
    const uint8_t* const mb = a.mask + (long)b * a.S;
    keep0 = mb[(unsigned)j0] != 0;
    keep1 = mb[(unsigned)j1] != 0;
  }
  // cross: keys past the sentence's last unmasked one contribute exactly nothing (score
  // -1e9 -> qexp 0 -> P 0, and fma(0, v, acc) == acc), so the key loops stop there; a
  // fully masked row keeps all S keys (the reference's uniform softmax over -1e9 scores)
  int Sk = KV_NEW ? step + 1 : a.S;
  if constexpr (!KV_NEW) {
    const int last = wave_max_i32(max(keep0 && lane < a.S ? lane + 1 : 0,
                                      keep1 && lane + 64 < a.S ? lane + 65 : 0));
    if (last > 0) Sk = last;
  }

  // phase 1: per-token scales of q (and k, v) over the full 512-wide rows
  auto amax8 = [](const float4 (&v)[2]) {
    float m = 0.0f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[c].x), fabsf(v[c].y)), fmaxf(fabsf(v[c].z), fabsf(v[c].w))));
    return wave_max(m);
  };
  const float sq = quant_scale(amax8(yq), 127.0f);
  qs[lane] = (int8_t)quant_one(q_own, sq);
  int8_t kq = 0, vq = 0;
  float sk = 0.0f, sv = 0.0f;
  if constexpr (KV_NEW) {
    sk = quant_scale(amax8(yk), 127.0f);
    sv = quant_scale(amax8(yv), 127.0f);
    kq = (int8_t)quant_one(k_own, sk);
    vq = (int8_t)quant_one(v_own, sv);
    const long row = kvb + step;
    a.kc[row * 512 + h * 64 + lane] = kq;     // cache append (attention.py: k/v of this step)
    a.vc[((vgb + (step >> 2)) * 512 + h * 64 + lane) * 4 + (step & 3)] = vq;
    if (h == 0 && lane == 0) { a.skc[row] = sk; a.svc[row] = sv; }
  }

  // phase 2: staged rows into LDS, then (self) the new row over the stale one
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int r = min(16 * i + rsub, nrows - 1);
    *reinterpret_cast<uint4*>(&Ks[r * DEC_KST + 4 * ch]) = kr[i];
    *reinterpret_cast<uint4*>(Vs + (min(4 * i + vg, glast) * 64 + vd) * 4) = vr[i];
  }
  svs[j0] = sv0; svs[j1] = sv1;
  __syncthreads();
  if constexpr (KV_NEW) {
    reinterpret_cast<int8_t*>(&Ks[step * DEC_KST])[lane] = kq;
    Vs[((step >> 2) * 64 + lane) * 4 + (step & 3)] = (uint8_t)vq;
    if (lane == 0) svs[step] = sv;
    if (lane == step) sk0 = sk;            // the key scales stay in the lane that scores
    if (lane + 64 == step) sk1 = sk;       // the key (lane + 64 u)
    __syncthreads();
  }
  QTX_STAMP(1);

  // phase 3: scores (lane owns keys lane, lane+64), softmax, P quantization
  uint32_t qd[16];
#pragma unroll
  for (int w = 0; w < 16; ++w) qd[w] = reinterpret_cast<const uint32_t*>(qs)[w];
  // (the scores and exponentials stay in registers: lane owns keys lane, lane + 64)
  float sc[2] = {0.0f, 0.0f};
  float lmax = -3.0e38f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = lane + 64 * u;
    if (j < Sk) {
      // the key row in 4 ds_read_b128; two partial int32 sums (exact in any order)
      uint32_t kw[16];
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) {
        const uint4 t = *reinterpret_cast<const uint4*>(&Ks[j * DEC_KST + 4 * w4]);
        kw[4 * w4] = t.x; kw[4 * w4 + 1] = t.y; kw[4 * w4 + 2] = t.z; kw[4 * w4 + 3] = t.w;
      }
      int a0 = 0, a1 = 0;
#pragma unroll
      for (int w = 0; w < 16; w += 2) {
        a0 = __builtin_amdgcn_sdot4(qd[w], kw[w], a0, false);
        a1 = __builtin_amdgcn_sdot4(qd[w + 1], kw[w + 1], a1, false);
      }
      const int acc = a0 + a1;
      float s = (((float)acc * sq) * (u ? sk1 : sk0)) * 0.125f;
      if (!(u ? keep1 : keep0)) s = -1.0e9f;
      sc[u] = s;
      lmax = fmaxf(lmax, s);
    }
  }
  const float m = wave_max(lmax);
  float lsum = 0.0f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = lane + 64 * u;
    if (j < Sk) {
      const float e = qexp(sc[u] - m);
      sc[u] = e;
      lsum = lsum + e;
    }
  }
  // P = rint((e / den) * 127) / 127: e / den by div_cr, unguarded (den in [1, Sk]: the
  // row max contributes qexp(0) == 1; e >= 2^-60 gives the correctly rounded quotient and
  // e < 2^-60 a P of 0 through either), / 127 by div127 — no true division per key; the PV
  // term's P * s_v once per key (the decoder's PV order, oracle attention_pv dec), and 0
  // for the padded keys Sk .. nk16 - 1 of the last 16-key group
  const float den = wave_sum(lsum);
  const float rden = 1.0f / den;
  const int nk16 = (Sk + 15) & ~15;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = lane + 64 * u;
    if (j < Sk) PS[j] = div127(rintf(div_cr(sc[u], den, rden) * 127.0f)) * svs[j];
    else if (j < nk16) PS[j] = 0.0f;
  }
  __syncthreads();
  QTX_STAMP(2);

  // phase 4: context dim h*64 + lane in the decoder's PV order: four chains, chain c over
  // the keys j with (j >> 2) & 3 == c in key order, term fma(PS[j], float(v_j), acc_c),
  // summed (c0 + c1) + (c2 + c3).  Per 16-key group the four chains' fmas are independent,
  // so the lone wave's dependent chain is a quarter of the keys (it was one fma per key,
  // 26-46 cycles each).  Padded keys: PS == 0 and a finite v, fma(0, v, acc) == acc.
  // The values of 4 keys of the lane's dim in one dword (the 4-key group layout): one
  // ds_read_b32 per chain step of 4 keys, each byte converted by one SDWA v_cvt_f32_i32.
  float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, c3 = 0.0f;
  const uint32_t* vl = reinterpret_cast<const uint32_t*>(Vs) + lane;
  // every 16-key group's operands are read first (the NIT groups that cover the staged rows;
  // those at or past nk16 are read and not used), so the chains pay the LDS latency once
  // instead of once per group (a rolled loop waited on its reads every 16 keys)
  float4 pg[NIT][4];
  uint32_t vg4[NIT][4];
#pragma unroll
  for (int g = 0; g < NIT; ++g) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pg[g][q] = *reinterpret_cast<const float4*>(PS + 16 * g + 4 * q);
      vg4[g][q] = vl[(4 * g + q) * 64];
    }
    // in group order (LDS returns in issue order: the first chains then wait for group 0
    // alone, which the scheduler would otherwise issue last)
    __builtin_amdgcn_sched_barrier(0);
  }
  // each fma an asm v_fmac_f32 (the IEEE fused multiply-add, as fmaf): left to itself the
  // compiler SLP-packs the four chains into v_pk_fma_f32 pairs — no faster on gfx950 (a
  // packed fp32 op issues at half rate) — and assembles their operand pairs with ~1 v_mov
  // per fma
  auto fmac = [](float& c, float p, float x) { asm("v_fmac_f32 %0, %1, %2" : "+v"(c) : "v"(p), "v"(x)); };
#pragma unroll
  for (int g = 0; g < NIT; ++g) {
    if (g == 0 || 16 * g < nk16) {       // (Sk >= 1: group 0 always)
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = (float)(int8_t)(vg4[g][q] >> (8 * e));
      const float4 p0 = pg[g][0], p1 = pg[g][1], p2 = pg[g][2], p3 = pg[g][3];
      fmac(c0, p0.x, v[0]);  fmac(c1, p1.x, v[4]);  fmac(c2, p2.x, v[8]);  fmac(c3, p3.x, v[12]);
      fmac(c0, p0.y, v[1]);  fmac(c1, p1.y, v[5]);  fmac(c2, p2.y, v[9]);  fmac(c3, p3.y, v[13]);
      fmac(c0, p0.z, v[2]);  fmac(c1, p1.z, v[6]);  fmac(c2, p2.z, v[10]); fmac(c3, p3.z, v[14]);
      fmac(c0, p0.w, v[3]);  fmac(c1, p1.w, v[7]);  fmac(c2, p2.w, v[11]); fmac(c3, p3.w, v[15]);
    }
  }
  const float acc = (c0 + c1) + (c2 + c3);
  QTX_STAMP(3);

  // phase 5: this head's 64 context values (and their absmax when asked for: the consumer
  // GEMM then takes the row maximum over the 8 heads, A_F32Q; the fused decode's consumer
  // forms it from the row itself, A_F32R)
  st_at(a.ctx, 4u * (unsigned)(b * 512 + h * 64 + lane), acc);
  if (a.pmax) {
    const float am = wave_max(fabsf(acc));
    if (lane == 0) a.pmax[(long)h * a.B + b] = am;
  }
  QTX_STAMP(4);
}

template <bool KV_NEW>
hipError_t dec_attn_nit(const DecAttnArgs& a, int B, int nrows, hipStream_t st) {
  const dim3 grid(B, 8), block(64);
  switch ((nrows + 15) / 16) {
    case 1: k_dec_attn<KV_NEW, 1><<<grid, block, 0, st>>>(a); break;
    case 2: k_dec_attn<KV_NEW, 2><<<grid, block, 0, st>>>(a); break;
    case 3: k_dec_attn<KV_NEW, 3><<<grid, block, 0, st>>>(a); break;
    case 4: k_dec_attn<KV_NEW, 4><<<grid, block, 0, st>>>(a); break;
    case 5: k_dec_attn<KV_NEW, 5><<<grid, block, 0, st>>>(a); break;
    case 6: k_dec_attn<KV_NEW, 6><<<grid, block, 0, st>>>(a); break;
    case 7: k_dec_attn<KV_NEW, 7><<<grid, block, 0, st>>>(a); break;
    case 8: k_dec_attn<KV_NEW, 8><<<grid, block, 0, st>>>(a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_dec_attn(const DecAttnArgs& a, int B, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (!a.ctx || a.B != B) return hipErrorInvalidValue;
  if (a.kv_new) {
    if (a.kv_bs <= 0 || a.kv_bs > DEC_MAXK || a.host_step1 < 0 || a.host_step1 > a.kv_bs)
      return hipErrorInvalidValue;
    return dec_attn_nit<true>(a, B, a.host_step1 > 0 ? a.host_step1 : (int)a.kv_bs, st);
  }
  if (a.S <= 0 || a.S > DEC_MAXK) return hipErrorInvalidValue;
  return dec_attn_nit<false>(a, B, a.S, st);
}

// k_vgroup4: a [B * S, 512] int8 value matrix (L layers, layer stride v_ls) into k_dec_attn's
// 4-key group layout (byte ((b * G4 + g) * 512 + d) * 4 + e = v[b * S + 4 g + e][d], 0 past
// S; G4 = ceil(S / 4); layer stride o_ls): the decode's cross values, once per decode.
__global__ void k_vgroup4(const int8_t* v, long v_ls, int B, int S, int8_t* out, long o_ls) {
  const int G4 = (S + 3) >> 2;
  const long n = (long)B * G4 * 512;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int d = (int)(i & 511);
  const long bg = i >> 9;
  const int g = (int)(bg % G4), b = (int)(bg / G4);
  const int8_t* src = v + (long)blockIdx.y * v_ls;
  uint32_t w = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int j = 4 * g + e;
    const uint32_t byte = j < S ? (uint8_t)src[((long)b * S + j) * 512 + d] : 0u;
    w |= byte << (8 * e);
  }
  reinterpret_cast<uint32_t*>(out + (long)blockIdx.y * o_ls)[i] = w;
}

hipError_t launch_vgroup4(const int8_t* v, long v_ls, int L, int B, int S, int8_t* out,
                          long o_ls, hipStream_t st) {
  if (B <= 0 || S <= 0 || L <= 0) return hipSuccess;
  const long n = (long)B * ((S + 3) / 4) * 512;
  k_vgroup4<<<dim3((unsigned)((n + 255) / 256), L), dim3(256), 0, st>>>(v, v_ls, B, S, out, o_ls);
  return hipGetLastError();
}

// =====================================================================================
// k_quant_h2048: per-token quantization of fp32 rows of 2048 (the decode FFN's hidden from
// B >= 96, quant_linear.py:30-43): one 4-wave workgroup per row, wave w quarter w (8 values
// per lane), the row maximum met in LDS — a quarter of k_rows' one-wave-per-row chain.  The
// same scale (quant_scale of the row absmax, order-free) and codes (quant_pack).
// =====================================================================================
__global__ __launch_bounds__(256) void k_quant_h2048(const float* X, long ldx, int M,
                                                     int8_t* q, float* s) {
  __shared__ float wm[4];
  const int m = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const float* xr = X + (long)m * ldx + 512 * wave;
  float4 t[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) t[c] = *reinterpret_cast<const float4*>(xr + 4 * (lane + 64 * c));
  float lm = 0.0f;
#pragma unroll
  for (int c = 0; c < 2; ++c)
    lm = fmaxf(lm, fmaxf(fmaxf(fabsf(t[c].x), fabsf(t[c].y)), fmaxf(fabsf(t[c].z), fabsf(t[c].w))));
  lm = wave_max(lm);
  if (lane == 0) wm[wave] = lm;
  __syncthreads();
  const float sc = quant_scale(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3])), 127.0f);
  float tf[8];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    tf[4 * c] = t[c].x; tf[4 * c + 1] = t[c].y; tf[4 * c + 2] = t[c].z; tf[4 * c + 3] = t[c].w;
  }
  uint32_t qd[2];
  quant_pack<8>(tf, sc, qd);
  uint32_t* dst = reinterpret_cast<uint32_t*>(q + (long)m * 2048 + 512 * wave);
#pragma unroll
  for (int c = 0; c < 2; ++c) dst[lane + 64 * c] = qd[c];
  if (tid == 0) s[m] = sc;
}

hipError_t launch_quant_h2048(const float* X, long ldx, int M, int8_t* q, float* s,
                              hipStream_t st) {
  if (M <= 0) return hipSuccess;
  k_quant_h2048<<<dim3(M), dim3(256), 0, st>>>(X, ldx, M, q, s);
  return hipGetLastError();
}

// =====================================================================================
// k_generator_mfma: the canonical generator order on the fp32 matrix cores.
// logits[m, v] = ((c0 + c1) + (c2 + c3)) + b[v] with c_q the k-ordered fma chain over
// k in [128q, 128q + 128) from 0 (oracle OracleModel.logits): v_mfma_f32_16x16x4_f32 chained
// over a quarter (32 instructions, C starting at 0) is bit-for-bit that chain
// (cdna_hip_programming.md §3 "FP32-input MFMA").
// Block = 16 token rows x 64 vocab columns, 16 waves: wave w takes strip w & 3 (16
// columns) and k-quarter w >> 2, so the dependent MFMA chain per wave is 32 long (a lone
// 128-long chain cost ~6,100 cycles, ~48 per dependent MFMA: tools/stamp_bench.py).  A
// operand = the LayerNormed rows in LDS (one row per wave); B operand = the weight packed at
// load in MFMA order (k_pack_gen: per strip, per group of 4 k-steps, per lane one float4),
// each wave streaming its quarter strip (8 KB) with 8 coalesced 1 KB loads issued before
// the LayerNorm.  The quarters' partial tiles meet in LDS; the waves of quarter 0 add them
// in the canonical order and store.  The two 16-row blocks of a strip group run on one XCD
// (blockIdx remap): the second reads the strips from that XCD's L2.
// =====================================================================================
constexpr int GEN_Q = 32;   // float4 groups of 4 k-steps per lane (K = 512)

__global__ __launch_bounds__(1024) void k_generator_mfma(const float* x, long ldx, int M,
                                                         const float* ln_a, const float* ln_b,
                                                         const float* Wm, const float* bias,
                                                         int V, float* logits) {
  __shared__ __attribute__((aligned(16))) float X[16][514];   // stride 514: conflict-free reads
  __shared__ __attribute__((aligned(16))) v4f part[3][4][64];  // quarters 1..3: [strip][lane]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int sw = wave & 3, qq = wave >> 2;          // strip within the group, k-quarter
  // blockIdx -> (strip group g, row block rb): hw = 8 (nrb (g / 8) + rb) + g % 8, so the
  // row blocks of group g share hw % 8 (one XCD under round-robin placement)
  const unsigned nrb = (unsigned)(M + 15) >> 4, hw = blockIdx.x;   // (unsigned: a shorter division)
  const int rb = (int)((hw >> 3) % nrb), g = (int)(((hw >> 3) / nrb) * 8 + (hw & 7));
  const int nstrip = (V + 15) / 16, strip = g * 4 + sw;
  if (g * 4 >= nstrip) return;                     // whole block (uniform)
  const int m0 = rb * 16;
  const int vcol = strip * 16 + fr;
  QTX_STAMP(0);
  // 1. the quarter strip's B operands, all in flight before anything else
  constexpr int QQ = GEN_Q / 4;
  const unsigned wo = 16u * (unsigned)((min(strip, nstrip - 1) * GEN_Q + QQ * qq) * 64 + lane);
  float4 wq[QQ];
#pragma unroll
  for (int q = 0; q < QQ; ++q) wq[q] = ld_at(reinterpret_cast<const float4*>(Wm), wo + 1024u * q);
  const float bv = ld_at(bias, 4u * min(vcol, V - 1));
  // 2. row `wave` of the block, LayerNorm in the canonical order, into LDS
  float xv[1][2][4];
  {
    const int m = min(m0 + wave, M - 1);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float4 t = ld_at(reinterpret_cast<const float4*>(x), 4u * (unsigned)(m * (int)ldx + 4 * (lane + 64 * c)));
      xv[0][c][0] = t.x; xv[0][c][1] = t.y; xv[0][c][2] = t.z; xv[0][c][3] = t.w;
    }
  }
  if (ln_a) ln_rows512<1>(xv, ln_a, ln_b, lane);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    float* d = &X[wave][4 * (lane + 64 * c)];
    *reinterpret_cast<float2*>(d) = make_float2(xv[0][c][0], xv[0][c][1]);
    *reinterpret_cast<float2*>(d + 2) = make_float2(xv[0][c][2], xv[0][c][3]);
  }
  __syncthreads();
  QTX_STAMP(1);
  // 3. the quarter's k-ordered chain: step s = 4 (QQ qq + q) + e uses A = X[fr][4s + fg],
  //    B = wq[q][e]
  v4f acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int q = 0; q < QQ; ++q) {
    const float b4[4] = {wq[q].x, wq[q].y, wq[q].z, wq[q].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = X[fr][4 * (4 * (QQ * qq + q) + e) + fg];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b4[e], acc, 0, 0, 0);
    }
  }
  if (qq) part[qq - 1][sw][lane] = acc;
  __syncthreads();
  QTX_STAMP(2);
  if (qq || vcol >= V) return;
  const v4f p1 = part[0][sw][lane], p2 = part[1][sw][lane], p3 = part[2][sw][lane];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int m = m0 + 4 * fg + e;
    if (m < M) st_at(logits, 4u * (unsigned)(m * V + vcol), ((acc[e] + p1[e]) + (p2[e] + p3[e])) + bv);
  }
  QTX_STAMP(3);
}

hipError_t launch_generator_mfma(const float* x, long ldx, int M, const float* ln_a,
                                 const float* ln_b, const float* Wm, const float* b, int V,
                                 float* logits, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if ((long)M * V >= (1L << 30) || (long)M * ldx >= (1L << 30)) return hipErrorInvalidValue;   // 32-bit offsets
  const int ngroup = (V + 63) / 64, nrb = (M + 15) / 16;
  const unsigned grid = 8u * nrb * ((ngroup + 7) / 8);
  k_generator_mfma<<<dim3(grid), dim3(1024), 0, st>>>(x, ldx, M, ln_a, ln_b, Wm, b, V, logits);
  return hipGetLastError();
}

// W [V][512] -> the MFMA-ordered strips of k_generator_mfma: out[((c * 32 + q) * 64 + l) * 4 + e]
// = W[16 c + (l & 15)][4 (4 q + e) + (l >> 4)] (0 past V).  One thread per float4.
__global__ void k_pack_gen(const float* W, int V, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nstrip = (V + 15) / 16;
  if (i >= (long)nstrip * GEN_Q * 64) return;
  const int l = (int)(i % 64), q = (int)((i / 64) % GEN_Q), c = (int)(i / (64 * GEN_Q));
  const int v = 16 * c + (l & 15);
  float4 o;
  float* op = reinterpret_cast<float*>(&o);
#pragma unroll
  for (int e = 0; e < 4; ++e) op[e] = v < V ? W[(long)v * 512 + 4 * (4 * q + e) + (l >> 4)] : 0.0f;
  reinterpret_cast<float4*>(out)[i] = o;
}
hipError_t launch_pack_gen(const float* W, int V, float* out, hipStream_t st) {
  const long n = (long)((V + 15) / 16) * GEN_Q * 64;
  k_pack_gen<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>(W, V, out);
  return hipGetLastError();
}

#ifdef QTX_STAMPS   // diagnostic builds only: the generator launched bare (tools/stamp_bench.py)
extern "C" int qtx_debug_generator(const float* x, int M, const float* lna, const float* lnb,
                                   const float* Wt, const float* b, int V, float* logits,
                                   void* st) {
  return (int)launch_generator_mfma(x, 512, M, lna, lnb, Wt, b, V, logits, (hipStream_t)st);
}
#endif

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
// k_argmax_embed: one 1024-thread workgroup per row.  The row of logits stays in
// registers (8 per thread, all loads in flight at once).  The token is the first argmax
// of logp = (x - max) - lse (generator.py:15 log_softmax, torch.max's first-index rule).
// lse only matters when another logit lies within a few ulps of the maximum: with
// lse = logf(sum) <= logf(V) < 16, (x - max) < -ARG_DELTA rounds below -lse, so only
// values above max - ARG_DELTA can tie it.  Fast path (block-uniform): exactly one such
// value — it is the maximum and the token.  Otherwise the exponentials go through LDS
// for the canonical lane-split denominator (wave 0) and the first argmax of logp decides.
// A non-finite row (any NaN or +inf, or only -inf) is all-NaN under torch's log_softmax,
// and torch.max of it is index 0: that row's token is 0 (oracle log_softmax_argmax).
// Then the block writes the next decoder input (embedding + PE of the token).
// =====================================================================================
constexpr int ARG_T = 1024, ARG_NV = 8, ARG_MAXV = ARG_T * ARG_NV;
constexpr float ARG_DELTA = 4.0e-6f;   // >= 2 ulp(16): covers every V <= ARG_MAXV

__device__ __forceinline__ int wave_sum_i32(int v) {
  auto d = [](int x, auto ctrl) {
    return __builtin_amdgcn_update_dpp(0, x, decltype(ctrl)::value, 0xF, 0xF, true);
  };
  v += d(v, std::integral_constant<int, 0xB1>{});
  v += d(v, std::integral_constant<int, 0x4E>{});
  v += d(v, std::integral_constant<int, 0x141>{});
  v += d(v, std::integral_constant<int, 0x140>{});
  return (__builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16)) +
         (__builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48));
}

// host_s1: the position + 1 when the host knows it (then no read of *step and no step
// advance: nothing of a decode whose every step knows its position reads the counter);
// 0: read *step and advance it (the last workgroup to arrive)
__global__ __launch_bounds__(1024) void k_argmax_embed(const float* logits, int V, int64_t* ids,
                                                       long ids_bs, int* step, unsigned* arrive,
                                                       const float* lut, const float* pe,
                                                       int max_pos, float* xnext, int host_s1) {
  __shared__ float Ev[ARG_MAXV];
  __shared__ float redf[16], lse_s;
  __shared__ int redi[16], redc[16], redb[16];
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  QTX_STAMP(0);
  const int s = host_s1 > 0 ? host_s1 - 1 : *step;
  const unsigned xo = 4u * (unsigned)(m * V);
  float4 pe_row = make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // position s+1 is known up front
  if (tid < 128) pe_row = ld_at(reinterpret_cast<const float4*>(pe), 16u * (unsigned)(min(s + 1, max_pos - 1) * 128 + tid));
  float t[ARG_NV];
#pragma unroll
  for (int i = 0; i < ARG_NV; ++i) t[i] = ld_at(logits, xo + 4u * min(tid + ARG_T * i, V - 1));   // clamped
  QTX_STAMP(1);
  // max: order-free; every wave reduces the 16 wave maxima itself (no second barrier);
  // with it the non-finite test: bit 0 = a NaN or +inf, bit 1 = a value above -inf
  float lm = -3.0e38f;
  bool nonfin = false, fin = false;
#pragma unroll
  for (int i = 0; i < ARG_NV; ++i)
    if (tid + ARG_T * i < V) {
      lm = fmaxf(lm, t[i]);
      nonfin |= !(t[i] < __builtin_inff());
      fin |= t[i] > -__builtin_inff();
    }
  lm = wave_max(lm);
  const int flags = (__ballot(nonfin) ? 1 : 0) | (__ballot(fin) ? 2 : 0);
  if (lane == 0) { redf[w] = lm; redb[w] = flags; }
  __syncthreads();
  const float mx = wave_max(lane < 16 ? redf[lane] : -3.0e38f);
  // candidates for the first argmax of logp, and the first index of the maximum
  int cnt = 0, bi = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < ARG_NV; ++i) {
    const int v = tid + ARG_T * i;
    if (v < V) {
      cnt += t[i] > mx - ARG_DELTA ? 1 : 0;
      if (t[i] == mx && v < bi) bi = v;
    }
  }
  cnt = wave_sum_i32(cnt);
  bi = wave_min_i32(bi);
  if (lane == 0) { redc[w] = cnt; redi[w] = bi; }
  __syncthreads();
  cnt = wave_sum_i32(lane < 16 ? redc[lane] : 0);
  int id = wave_min_i32(lane < 16 ? redi[lane] : 0x7fffffff);
  const bool bad = __ballot(lane < 16 && (redb[lane] & 1)) != 0ull ||
                   __ballot(lane < 16 && (redb[lane] & 2)) == 0ull;
  QTX_STAMP(2);
  if (bad) {
    id = 0;                                // torch.max of an all-NaN log_softmax row
  } else if (cnt != 1) {   // near-tie: the exact log-softmax decides (block-uniform)
    // e_v = qexp(x_v - max) into LDS for the ordered sum
#pragma unroll
    for (int i = 0; i < ARG_NV; ++i) {
      const int v = tid + ARG_T * i;
      if (v < V) Ev[v] = qexp(t[i] - mx);
    }
    __syncthreads();
    // canonical denominator: lane l sums e[l], e[l+64], ... in order (one wave), then tree
    if (w == 0) {
      float ls = 0.0f;
#pragma unroll 8
      for (int v = lane; v < V; v += 64) ls = ls + Ev[v];
      ls = wave_sum(ls);
      if (lane == 0) lse_s = logf(ls);
    }
    __syncthreads();
    const float lse = lse_s;
    // first argmax of logp = (x - max) - lse (torch.max tie rule)
    float best = -3.0e38f;
    int bj = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < ARG_NV; ++i) {
      const int v = tid + ARG_T * i;
      if (v < V) {
        const float lp = (t[i] - mx) - lse;
        if (lp > best) { best = lp; bj = v; }
      }
    }
    // the maximum, then the smallest index holding it: per wave, then over the 16 waves
    const float wb = wave_max(best);
    const int wi = wave_min_i32(best == wb ? bj : 0x7fffffff);
    __syncthreads();                       // (redf / redi are reused)
    if (lane == 0) { redf[w] = wb; redi[w] = wi; }
    __syncthreads();
    const float gv = lane < 16 ? redf[lane] : -3.0e38f;
    const float gb = wave_max(gv);
    id = wave_min_i32(lane < 16 && gv == gb ? redi[lane] : 0x7fffffff);
    id = min(id, V - 1);                   // keeps the embedding gather in bounds, whatever
  }
  if (tid == 0 && s >= 0 && s + 1 < ids_bs) ids[m * ids_bs + s + 1] = id;   // bounded (stale position)
  QTX_STAMP(4);
  // next decoder input: tgt_embed(id) at position s + 1 (embeddings.py:12-13)
  if (tid < 128) {
    const float sc = 0x1.6a09e6p+4f;
    const float4 e = ld_at(reinterpret_cast<const float4*>(lut), 16u * (unsigned)(id * 128 + tid));
    const float4 q = pe_row;
    st_at(reinterpret_cast<float4*>(xnext), 16u * (unsigned)(m * 128 + tid),
          make_float4(e.x * sc + q.x, e.y * sc + q.y, e.z * sc + q.z, e.w * sc + q.w));
  }
  QTX_STAMP(5);
  // every workgroup has read *step above; the last one to arrive advances it
  if (host_s1 == 0 && tid == 0) {
    const unsigned tk = atomicAdd(arrive, 1u);
    if (tk == gridDim.x - 1) {
      *step = s + 1;
      *arrive = 0u;
    }
  }
}

hipError_t launch_argmax_embed(const float* logits, int M, int V, int64_t* ids, long ids_bs,
                               int* step, unsigned* arrive, const float* lut, const float* pe,
                               int max_pos, float* xnext, hipStream_t st, int host_s1) {
  if (M <= 0) return hipSuccess;
  if (V > ARG_MAXV || host_s1 < 0 || (long)M * V >= (1L << 30)) return hipErrorInvalidValue;
  k_argmax_embed<<<dim3(M), dim3(ARG_T), 0, st>>>(logits, V, ids, ids_bs, step, arrive, lut,
                                                  pe, max_pos, xnext, host_s1);
  return hipGetLastError();
}

}  // namespace qtx
