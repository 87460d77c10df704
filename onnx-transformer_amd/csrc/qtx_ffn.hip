// qtx_ffn.hip — the encoder's FFN sublayer as ONE launch (gfx950, wave64), for a block of
// 128 token rows per workgroup:
//   h   = relu(((float(x1q . W1^T) * sa) * sw1) + b1)            position_feed_forward.py:12
//   hq  = rint(h / s_h),  s_h = max(max_n h, 1e-5) / 127         quant_linear.py:30-43
//   x2  = x1 + (((float(hq . W2^T) * s_h) * sw2) + b2)           sublayer_connection.py:15-17
//   the next sublayer's LayerNorm(x2) quantized per token (KP)   layer_norm.py:12-15
//   — or, after the last layer, the encoder's final LayerNorm in fp32 (encoder.py:17)
// replacing the one-pass FFN1 launch (k_gemm_wsy) and the FFN2 row GEMM (k_gemm_row
// RE_RES_LN): the hidden h never leaves the chip (the two launches moved 2 x 64 MB of int8 h
// through HBM at cfg3), and FFN2's main loop runs inside FFN1's weight stream.
//
// The per-token quantization of h needs the whole 2048-wide row's maximum before any value
// is rounded, and 128 rows x 2048 fp32 (1 MB) do not fit on a CU, so FFN1 runs twice: pass 1
// forms the row maxima, pass 2 recomputes each 64-column chunk of h, quantizes it and feeds
// it straight into FFN2 ("The fused FFN kernel").
//
// Geometry: 512 threads = 8 waves, wave w owns rows 16w .. 16w+15 of the block for every
// matrix, so no value crosses waves:
//   FFN1 as D1 = W1c . x1q^T (v_mfma_i32_16x16x64_i8, W1 the A operand): lane l (f = l & 15,
//     g = l >> 4) gets row f, h columns 4g .. 4g+3 of each 16-column fragment; the block's
//     x1q rows stay in registers as the B operand (8 K steps x 16 bytes).
//   FFN2 as D2 = hq . W2^T: the A operand lane l must hold row f and 16 K bytes — exactly what
//     the lane holds of h for the chunk's 4 fragments (4 columns each), so hq goes from the
//     FFN1 accumulators to the FFN2 operand in registers (W2's K order is permuted to match
//     at pack time: operand byte 4j' + e = h column 64c + 16j' + 4g + e).  Lane l then holds
//     rows 4g .. 4g+3 and 32 columns 16f .. 16f+15, 256+16f .. 256+16f+15 (W2's column order
//     permuted at pack time): exactly the canonical LayerNorm lanes L = 4f .. 4f+3 of
//     ln_rows512, so the residual + LayerNorm + quantization epilogue runs in registers, its
//     64-lane reduction tree as 2 in-lane levels + the 4 DPP levels of a 16-lane row.
// Weights: one stream per layer (k_pack_ffn), in consumption order and MFMA fragment order
// (1 KB per fragment, lane l's 16 bytes at 16 l): per 64-column chunk c a 32 KB W1 slot
// (8 K steps x 4 fragments) and a 32 KB W2 slot (32 column fragments of K step c).  Pass 1
// reads the W1 slots (1 MB), pass 2 both (2 MB), through a 4-slot LDS ring filled by LDS-DMA
// (linear 1 KB pieces, 4 per wave per slot; one barrier per slot).  Each workgroup starts
// the chunk sequence at its own rotation (int32 sums and maxima are order-free: exact), so
// the CUs of one XCD do not request the same weight lines at the same time.
#include "qtx_common.h"
#include "qtx_kernels.h"

QTX_STAMP_SETTER(ffn)

namespace qtx {

constexpr int FF_R = 128, FF_SLOT = 32768, FF_NSLOT = 4, FF_WAVES = 8;
constexpr int FF_PPW = FF_SLOT / 1024 / FF_WAVES;   // 1 KB DMA pieces per wave per slot

// the FFN2 output column of fragment j (0..31), lane column f (0..15)
__host__ __device__ __forceinline__ int ff_col2(int j, int f) {
  return j < 16 ? 16 * f + j : 256 + 16 * f + (j - 16);
}

__device__ __forceinline__ void ff_dma(const int8_t* gsrc, const uint8_t* lds_dst) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
}

__device__ __forceinline__ v4i ff_ld(const uint8_t* p) { return *reinterpret_cast<const v4i*>(p); }

// FFN1 of one 64-column chunk for the wave's 16 rows: acc[j'] (j' = 0..3) over 8 K steps.
// The fragment reads run one K step ahead; sched_barrier pins that distance (the scheduler
// would otherwise sink each read next to its MFMAs and expose the LDS latency every step).
__device__ __forceinline__ void ff_ffn1(const uint8_t* sl, const v4i (&xb)[8], v4i (&acc)[4]) {
  v4i wa[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) wa[0][j] = ff_ld(sl + j * 1024);
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    if (s < 7)
#pragma unroll
      for (int j = 0; j < 4; ++j) wa[(s + 1) & 1][j] = ff_ld(sl + ((s + 1) * 4 + j) * 1024);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wa[s & 1][j], xb[s], s == 0 ? v4i{0, 0, 0, 0} : acc[j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// the chunk's h values of the lane (row f, columns 64c + 16j' + 4g + e) from the FFN1
// accumulators: ((float(acc) * sa) * sw1) + b1, then ReLU (k_gemm_row's order)
__device__ __forceinline__ float ff_h(int a, float sar, float sw, float b) {
  const float v = ((float)a * sar) * sw + b;
  return v > 0.0f ? v : 0.0f;
}

template <bool FULL, bool LNQ>
__global__ __launch_bounds__(512) void k_ffn_fused(FfnArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[FF_NSLOT * FF_SLOT];
  __shared__ __attribute__((aligned(16))) float tsw[2048];   // FFN1 column scales
  __shared__ __attribute__((aligned(16))) float tb[2048];    // FFN1 biases
  __shared__ float shs[FF_R];                                // h row scales
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, f = l & 15, g = l >> 4;
  const int F = a.F, nch = F >> 6, P = 3 * nch;
  const long m0 = (long)blockIdx.x * FF_R;
  const int rot = (int)((((blockIdx.x >> 3) * 5u) + (blockIdx.x & 7) * 3u) % (unsigned)nch);
  QTX_STAMP(0);

  // stream position p -> slot of the weight stream: pass 1 the W1 slots (2c), pass 2 the
  // pairs (2c, 2c + 1), chunk c = (position + rot) mod nch
  auto slot_of = [&](int p) {
    if (p < nch) {
      int c = p + rot;
      if (c >= nch) c -= nch;
      return 2 * c;
    }
    const int q = p - nch;
    int c = (q >> 1) + rot;
    if (c >= nch) c -= nch;
    return 2 * c + (q & 1);
  };
  auto issue = [&](int p) {
    if (p >= P) return;
    const int8_t* src = a.wf + (long)slot_of(p) * FF_SLOT + (w * FF_PPW) * 1024 + 16 * l;
    uint8_t* dst = ring + (p & (FF_NSLOT - 1)) * FF_SLOT + (w * FF_PPW) * 1024;
#pragma unroll
    for (int k = 0; k < FF_PPW; ++k) ff_dma(src + k * 1024, dst + k * 1024);
  };
  // top of slot p: this wave's pieces of it landed (the youngest memory operations are the
  // pieces of slots p + 1, p + 2: the loop issues nothing else), every wave's too and every
  // wave is past slot p - 1 (barrier), then slot p + 3 goes into p - 1's buffer
  auto ring_wait = [&](int p) {
    const int ahead = P - 1 - p;
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issue(p + FF_NSLOT - 1);
  };

  issue(0);
  issue(1);
  issue(2);
  // FFN1 column scales and biases into LDS; the wave's x1q rows (KP layout) and row scales
  for (int i = tid; i < F / 4; i += 512) {
    reinterpret_cast<float4*>(tsw)[i] = reinterpret_cast<const float4*>(a.sw1)[i];
    reinterpret_cast<float4*>(tb)[i] = reinterpret_cast<const float4*>(a.b1)[i];
  }
  const long rx = FULL ? m0 + 16 * w + f : min(m0 + 16 * w + f, (long)a.M - 1);
  v4i xb[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) xb[s] = *reinterpret_cast<const v4i*>(a.A + kp_off(rx, 64 * s + 16 * g, 512));
  const float sar = a.sa[rx];
  __syncthreads();
  QTX_STAMP(1);

  // ---- pass 1: the row maxima of h (the lane: row f, 16 of each chunk's columns)
  float mx = 0.0f;
  for (int p = 0; p < nch; ++p) {
    ring_wait(p);
    v4i acc[4];
    ff_ffn1(ring + (p & (FF_NSLOT - 1)) * FF_SLOT + 16 * l, xb, acc);
    int c = p + rot;
    if (c >= nch) c -= nch;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 s4 = *reinterpret_cast<const float4*>(tsw + 64 * c + 16 * j + 4 * g);
      const float4 b4 = *reinterpret_cast<const float4*>(tb + 64 * c + 16 * j + 4 * g);
      mx = fmaxf(mx, ff_h(acc[j][0], sar, s4.x, b4.x));
      mx = fmaxf(mx, ff_h(acc[j][1], sar, s4.y, b4.y));
      mx = fmaxf(mx, ff_h(acc[j][2], sar, s4.z, b4.z));
      mx = fmaxf(mx, ff_h(acc[j][3], sar, s4.w, b4.w));
    }
  }
  // the row's maximum over the 4 lanes of row f (lane groups g), then its quantization scale
  mx = fmaxf(mx, __shfl_xor(mx, 16));
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  const float sh = scale127(fmaxf(mx, 1e-5f));   // quant_scale(max, 127), exhaustively equal
  const float invh = __builtin_amdgcn_rcpf(sh);
  if (g == 0) shs[16 * w + f] = sh;
  QTX_STAMP(2);

  // ---- pass 2: each chunk of h recomputed, quantized with s_h, fed to FFN2 in registers
  constexpr float BIAS = 12582912.0f;   // rint via the biased add (qtx_common.h rint_biased)
  v4i acc2[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) acc2[j] = v4i{0, 0, 0, 0};
  long long tw = 0, t1 = 0, te = 0, t2 = 0;          // accumulated phase cycles (QTX_STAMPS)
  for (int q = 0; q < nch; ++q) {
    const int p = nch + 2 * q;
    long long ts = QTX_NOW();
    ring_wait(p);
    long long tn = QTX_NOW();
    tw += tn - ts;
    v4i acc[4];
    ff_ffn1(ring + (p & (FF_NSLOT - 1)) * FF_SLOT + 16 * l, xb, acc);
    ts = QTX_NOW();
    t1 += ts - tn;
    int c = q + rot;
    if (c >= nch) c -= nch;
    // rint(h / s_h) as x * (1 / s_h) except within 2^-13 of a rounding tie, where the true
    // quotient is taken (quant_rows512's guarded form: exact)
    float t[4][4];
    float dm = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 s4 = *reinterpret_cast<const float4*>(tsw + 64 * c + 16 * j + 4 * g);
      const float4 b4 = *reinterpret_cast<const float4*>(tb + 64 * c + 16 * j + 4 * g);
      const float sw[4] = {s4.x, s4.y, s4.z, s4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float r = ff_h(acc[j][e], sar, sw[e], bb[e]) * invh;
        t[j][e] = r + BIAS;
        dm = fmaxf(dm, fabsf(r - (t[j][e] - BIAS)));
      }
    }
    if (__builtin_expect(__ballot(dm > 0.5f - 0x1p-13f) != 0ull, 0)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 s4 = *reinterpret_cast<const float4*>(tsw + 64 * c + 16 * j + 4 * g);
        const float4 b4 = *reinterpret_cast<const float4*>(tb + 64 * c + 16 * j + 4 * g);
        const float sw[4] = {s4.x, s4.y, s4.z, s4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) t[j][e] = ff_h(acc[j][e], sar, sw[e], bb[e]) / sh + BIAS;
      }
    }
    v4i hq;
#pragma unroll
    for (int j = 0; j < 4; ++j) hq[j] = (int)pack4_biased(t[j][0], t[j][1], t[j][2], t[j][3]);
    tn = QTX_NOW();
    te += tn - ts;
    ring_wait(p + 1);
    ts = QTX_NOW();
    tw += ts - tn;
    const uint8_t* s2 = ring + ((p + 1) & (FF_NSLOT - 1)) * FF_SLOT + 16 * l;
    v4i wb[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) wb[j] = ff_ld(s2 + j * 1024);
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      if (j + 4 < 32) wb[(j + 4) & 7] = ff_ld(s2 + (j + 4) * 1024);
      __builtin_amdgcn_sched_barrier(0);
      acc2[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(hq, wb[j & 7], acc2[j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    t2 += QTX_NOW() - ts;
  }
  QTX_STAMP(3);
  QTX_STAMP_VAL(8, tw);
  QTX_STAMP_VAL(9, t1);
  QTX_STAMP_VAL(10, te);
  QTX_STAMP_VAL(11, t2);
  (void)tw; (void)t1; (void)te; (void)t2;

  // ---- epilogue: y2 = ((float(acc2) * s_h) * sw2) + b2, x2 = x1 + y2, LayerNorm, quant.
  // Lane: rows 16w + 4g + e (e = 0..3), columns ff_col2(j, f) (j = 0..31): the canonical
  // lanes L = 4f + t own columns 4L .. 4L+3 (j = 4t ..) and 256 + 4L .. (j = 16 + 4t ..).
  __syncthreads();                                   // every wave is done with the ring
  float* et = reinterpret_cast<float*>(ring);        // [4][512]: sw2, b2, ln_a, ln_b
  et[tid] = a.sw2[tid];
  et[512 + tid] = a.b2[tid];
  et[1024 + tid] = a.ln_a[tid];
  et[1536 + tid] = a.ln_b[tid];
  __syncthreads();
  float shr[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) shr[e] = shs[16 * w + 4 * g + e];
  auto colv = [&](const float* tab, int run, int k) {   // 4 consecutive columns of a run
    return *reinterpret_cast<const float4*>(tab + 256 * run + 16 * f + 4 * k);
  };
  const long rbase = m0 + 16 * w + 4 * g;
  auto res_ptr = [&](int e) {
    const long r = FULL ? rbase + e : min(rbase + e, (long)a.M - 1);
    return a.x + r * 512 + 16 * f;
  };
  float4 rv[8];                                       // the next row's residual
  auto load_res = [&](int e) {
    const float* p = res_ptr(e);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      rv[k] = *reinterpret_cast<const float4*>(p + 4 * k);
      rv[4 + k] = *reinterpret_cast<const float4*>(p + 256 + 4 * k);
    }
  };
  load_res(0);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long row = rbase + e;
    const bool live = FULL || row < a.M;
    // y2 of this row from the accumulators (per row: acc2 stays int until its last row),
    // then x2 = x1 + y2
    float v[32];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int run = k >> 2, kk = k & 3;
      const float4 s4 = colv(et, run, kk), b4 = colv(et + 512, run, kk), r4 = rv[k];
      const float sw[4] = {s4.x, s4.y, s4.z, s4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
      const float rr[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
        v[4 * k + i] = rr[i] + (((float)acc2[4 * k + i][e] * shr[e]) * sw[i] + bb[i]);
    }
    if (e < 3) load_res(e + 1);
    if (live) {
      float* xp = a.x + row * 512 + 16 * f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        *reinterpret_cast<float4*>(xp + 4 * k) = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
        *reinterpret_cast<float4*>(xp + 256 + 4 * k) =
            make_float4(v[16 + 4 * k], v[17 + 4 * k], v[18 + 4 * k], v[19 + 4 * k]);
      }
    }
    // LayerNorm in ln_rows512's order: canonical lane L = 4f + t sums its chunk-0 values
    // (j = 4t ..) then its chunk-1 values (j = 16 + 4t ..) sequentially; the 64-lane tree is
    // L^1, L^2 in the lane, then L^4, L^8, L^16, L^32 = DPP xor 1, xor 2, half-mirror, mirror
    // of the 16-lane row (row16_sum)
    float ps[4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      float s = v[4 * tt];
      s = s + v[4 * tt + 1];
      s = s + v[4 * tt + 2];
      s = s + v[4 * tt + 3];
      s = s + v[16 + 4 * tt];
      s = s + v[17 + 4 * tt];
      s = s + v[18 + 4 * tt];
      s = s + v[19 + 4 * tt];
      ps[tt] = s;
    }
    const float mean = row16_sum((ps[0] + ps[1]) + (ps[2] + ps[3])) / 512.0f;
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = v[j] - mean;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      float s = v[4 * tt] * v[4 * tt];
      s = s + v[4 * tt + 1] * v[4 * tt + 1];
      s = s + v[4 * tt + 2] * v[4 * tt + 2];
      s = s + v[4 * tt + 3] * v[4 * tt + 3];
      s = s + v[16 + 4 * tt] * v[16 + 4 * tt];
      s = s + v[17 + 4 * tt] * v[17 + 4 * tt];
      s = s + v[18 + 4 * tt] * v[18 + 4 * tt];
      s = s + v[19 + 4 * tt] * v[19 + 4 * tt];
      ps[tt] = s;
    }
    const float var = div_const(row16_sum((ps[0] + ps[1]) + (ps[2] + ps[3])), 511.0f);
    const float den = sqrtf(var) + 1e-6f;
    // (a * d) / den + b, the division correctly rounded (ln_rows512's guard and div_cr)
    uint32_t mxb = 0u;
    float mn = __builtin_inff();
#pragma unroll
    for (int run = 0; run < 2; ++run)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 g4 = colv(et + 1024, run, k);
        const float ga[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int j = 16 * run + 4 * k + i;
          v[j] = ga[i] * v[j];
          mxb = max(mxb, __float_as_uint(v[j]) & 0x7fffffffu);
          mn = fminf(mn, fabsf(v[j]));
        }
      }
    const bool dok = divisor_ok(den);
    bool ok = dok && mxb < 0x5d800000u && mn > 0x1p-60f;
    if (__builtin_expect(__ballot(!ok) != 0ull, 0)) {
      DivRange rg;
#pragma unroll
      for (int j = 0; j < 32; ++j) rg.add(v[j]);
      ok = dok && rg.ok();
    }
    if (__builtin_expect(__ballot(!ok) == 0ull, 1)) {
      const float yd = 1.0f / den;
#pragma unroll
      for (int j = 0; j < 32; ++j) v[j] = div_cr(v[j], den, yd);
    } else {
#pragma unroll
      for (int j = 0; j < 32; ++j) v[j] = v[j] / den;
    }
#pragma unroll
    for (int run = 0; run < 2; ++run)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 b4 = colv(et + 1536, run, k);
        const float gb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) v[16 * run + 4 * k + i] = v[16 * run + 4 * k + i] + gb[i];
      }
    if constexpr (LNQ) {
      // per-token quantization (quant_rows512's order and guarded rint)
      float am = 0.0f;
#pragma unroll
      for (int j = 0; j < 32; ++j) am = fmaxf(am, fabsf(v[j]));
      const float sc = div_const(fmaxf(row16_max(am), 1e-5f), 127.0f);
      const float inv = __builtin_amdgcn_rcpf(sc);
      uint32_t pk[8];                                 // packed as they are formed
      float dq = 0.0f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float tq[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float r = v[4 * k + i] * inv;
          tq[i] = r + BIAS;
          dq = fmaxf(dq, fabsf(r - (tq[i] - BIAS)));
        }
        pk[k] = pack4_biased(tq[0], tq[1], tq[2], tq[3]);
      }
      if (__builtin_expect(__ballot(dq > 0.5f - 0x1p-13f) != 0ull, 0)) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          pk[k] = pack4_biased(v[4 * k] / sc + BIAS, v[4 * k + 1] / sc + BIAS, v[4 * k + 2] / sc + BIAS,
                               v[4 * k + 3] / sc + BIAS);
      }
      if (live) {
#pragma unroll
        for (int run = 0; run < 2; ++run)
          *reinterpret_cast<uint4*>(a.lnq + kp_off(row, 256 * run + 16 * f, 512)) =
              make_uint4(pk[4 * run], pk[4 * run + 1], pk[4 * run + 2], pk[4 * run + 3]);
        if (f == 0) a.lns[row] = sc;
      }
    } else if (live) {
      float* op = a.lnout + row * 512 + 16 * f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        *reinterpret_cast<float4*>(op + 4 * k) = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
        *reinterpret_cast<float4*>(op + 256 + 4 * k) =
            make_float4(v[16 + 4 * k], v[17 + 4 * k], v[18 + 4 * k], v[19 + 4 * k]);
      }
    }
  }
  QTX_STAMP(4);
}

hipError_t launch_ffn_fused(const FfnArgs& a, hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  if (a.F % 64 || a.F < 256 || a.F > 2048 || !a.wf) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((a.M + FF_R - 1) / FF_R)), block(512);
  const bool full = a.M % FF_R == 0;
  if (a.lnq) {
    if (full) k_ffn_fused<true, true><<<grid, block, 0, st>>>(a);
    else k_ffn_fused<false, true><<<grid, block, 0, st>>>(a);
  } else {
    if (full) k_ffn_fused<true, false><<<grid, block, 0, st>>>(a);
    else k_ffn_fused<false, false><<<grid, block, 0, st>>>(a);
  }
  return hipGetLastError();
}

// W1 int8 [F, 512] and W2 int8 [512, F] (row-major) -> the fused FFN weight stream
// (F / 64 chunks x 2 slots x 32 KB): one thread per 16-byte lane piece.
//   slot 2c, fragment 4s + j', lane l:  W1[64c + 16j' + (l & 15)][64s + 16(l >> 4) .. +16]
//   slot 2c+1, fragment j, lane l:      byte 4j' + e = W2[ff_col2(j, l & 15)][64c + 16j' + 4(l >> 4) + e]
__global__ void k_pack_ffn(const int8_t* W1, const int8_t* W2, int F, int8_t* out) {
  const long u = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nu = (long)F / 64 * 2 * 2048;
  if (u >= nu) return;
  const int c = (int)(u / 4096), part = (int)((u / 2048) & 1), v = (int)(u % 2048);
  const int fr = v / 64, lane = v % 64, f = lane & 15, g = lane >> 4;
  uint4 d;
  if (part == 0) {
    const int s = fr >> 2, j = fr & 3;
    d = *reinterpret_cast<const uint4*>(W1 + (long)(64 * c + 16 * j + f) * 512 + 64 * s + 16 * g);
  } else {
    const int8_t* row = W2 + (long)ff_col2(fr, f) * F + 64 * c + 4 * g;
    d = make_uint4(*reinterpret_cast<const uint32_t*>(row), *reinterpret_cast<const uint32_t*>(row + 16),
                   *reinterpret_cast<const uint32_t*>(row + 32), *reinterpret_cast<const uint32_t*>(row + 48));
  }
  *reinterpret_cast<uint4*>(out + 16 * u) = d;
}

hipError_t launch_pack_ffn(const int8_t* W1, const int8_t* W2, int F, int8_t* out, hipStream_t st) {
  if (F % 64 || F < 256 || F > 2048) return hipErrorInvalidValue;
  const long nu = (long)F / 64 * 2 * 2048;
  k_pack_ffn<<<dim3((unsigned)((nu + 255) / 256)), dim3(256), 0, st>>>(W1, W2, F, out);
  return hipGetLastError();
}

}  // namespace qtx
