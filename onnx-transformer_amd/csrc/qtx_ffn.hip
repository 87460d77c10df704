// qtx_ffn.hip — the encoder's FFN sublayer as ONE launch (gfx950, wave64), for a block of
// 128 token rows per workgroup:
//   h   = relu(((float(x1q . W1^T) * sa) * sw1) + b1)            position_feed_forward.py:12
//   hq  = rint(h / s_h),  s_h = max(max_n h, 1e-5) / 127         quant_linear.py:30-43
//   x2  = x1 + (((float(hq . W2^T) * s_h) * sw2) + b2)           sublayer_connection.py:15-17
//   the next sublayer's LayerNorm(x2) quantized per token (KP)   layer_norm.py:12-15
//   — or, after the last layer, the encoder's final LayerNorm in fp32 (encoder.py:17)
// in place of the one-pass FFN1 launch (k_gemm_wsy) and the FFN2 row GEMM (k_gemm_row
// RE_RES_LN): the hidden h never leaves the chip (the two launches move 2 x 64 MB of int8 h
// through HBM at cfg3).
//
// The per-token quantization of h needs the whole 2048-wide row's maximum before any value
// is rounded, and 128 rows x 2048 fp32 (1 MB) do not fit on a CU, so FFN1 runs twice: pass 1
// forms the row maxima, pass 2 recomputes each 64-column chunk of h, quantizes it and feeds
// it to FFN2 ("The fused FFN kernel").
//
// What bounds it is LDS read bandwidth (256 B/clk per CU): every weight fragment is read
// from LDS by each wave that multiplies it.  Geometry (8 waves, 2 per SIMD): wave w owns the
// 32 rows 32 rg .. of the block (rg = w & 3) and one column half ch = w >> 2, so each weight
// fragment is read by 4 waves and feeds 2 MFMAs per read (the first version gave each wave
// 16 rows and all columns: 8 reads per fragment, LDS-bound at twice the MFMA time).
//   FFN1, D1 = W1c . x1q^T (v_mfma_i32_16x16x64_i8, W1 the A operand): per 64-column chunk
//     the wave computes its 32 rows x 32 columns (2 x 2 fragments); lane l (f = l & 15,
//     g = l >> 4) gets row f of each row fragment, h columns 4g .. 4g+3 of each 16-column
//     fragment.  The block's x1q sits in LDS in fragment order (64 KB, read by pass 2) and
//     pass 1 holds the wave's rows in registers (64 VGPRs).
//   hq: the two waves of a row group exchange their halves through LDS (8 bytes per lane
//     and row fragment) and assemble the FFN2 A operand: lane l holds row f and operand
//     bytes 4j' + e = h column 64c + 16j' + 4g + e (W2's K order is permuted to match).
//   FFN2, D2 = hq . W2^T: the wave's 32 rows x 256 columns (2 x 16 fragments, 128 VGPRs);
//     lane l holds rows 4g + e and the 16 columns 16f + 8ch .. +8, 256 + 16f + 8ch .. +8
//     (W2's column order permuted at pack time) = the canonical LayerNorm lanes L = 4f + t,
//     t in {2ch, 2ch + 1} of ln_rows512: the residual + LayerNorm + quantization epilogue
//     runs in registers, its 64-lane reduction tree as 1 in-lane level, 1 exchange with the
//     partner wave (LDS) and the 4 DPP levels of a 16-lane row.
// Weights: one stream per layer (k_pack_ffn), in consumption order and MFMA fragment order
// (1 KB per fragment, lane l's 16 bytes at 16 l): per chunk four 16 KB slots — W1 K steps
// 0-3, W1 K steps 4-7 (fragment 4 s' + j'), W2 for ch 0, W2 for ch 1 (fragment j).  Pass 1
// reads the W1 slots (1 MB), pass 2 all of them (2 MB), through a 4-slot LDS ring filled by
// LDS-DMA (linear 1 KB pieces, 2 per wave per slot, one barrier per slot).  Each workgroup
// starts the chunk sequence at its own rotation (int32 sums and maxima are order-free:
// exact), so the CUs of one XCD do not request the same weight lines at the same time.
#include "qtx_common.h"
#include "qtx_kernels.h"

QTX_STAMP_SETTER(ffn)

namespace qtx {

constexpr int FF_R = 128, FF_SLOT = 16384, FF_NSLOT = 4, FF_WAVES = 8;
constexpr int FF_PPW = FF_SLOT / 1024 / FF_WAVES;   // 1 KB DMA pieces per wave per slot

// the FFN2 output column of column half ch, fragment j (0..15), lane column f (0..15)
__host__ __device__ __forceinline__ int ff_col2(int ch, int j, int f) {
  return j < 8 ? 16 * f + 8 * ch + j : 256 + 16 * f + 8 * ch + (j - 8);
}

__device__ __forceinline__ void ff_dma(const int8_t* gsrc, const uint8_t* lds_dst) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
}

__device__ __forceinline__ v4i ff_ld(const uint8_t* p) { return *reinterpret_cast<const v4i*>(p); }

// h of one accumulator element: ((float(acc) * sa) * sw1) + b1, then ReLU (k_gemm_row's order)
__device__ __forceinline__ float ff_h(int a, float sar, float sw, float b) {
  const float v = ((float)a * sar) * sw + b;
  return v > 0.0f ? v : 0.0f;
}

template <bool FULL, bool LNQ>
__global__ __launch_bounds__(512) void k_ffn_fused(FfnArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t xq[FF_R * 512];              // 64 KB
  __shared__ __attribute__((aligned(16))) uint8_t ring[FF_NSLOT * FF_SLOT];    // 64 KB
  __shared__ __attribute__((aligned(16))) float tsw[2048];   // FFN1 column scales
  __shared__ __attribute__((aligned(16))) float tb[2048];    // FFN1 biases
  __shared__ __attribute__((aligned(16))) uint2 hx[FF_WAVES][2][64];   // hq halves, row maxima
  __shared__ float shs[FF_R];                                          // h row scales
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, f = l & 15, g = l >> 4;
  const int rg = w & 3, ch = w >> 2;
  const int F = a.F, nch = F >> 6, P = 6 * nch;     // stream positions: 2 + 4 per chunk
  const int m0 = (int)blockIdx.x * FF_R, mlast = a.M - 1;
  const int rot = (int)((((blockIdx.x >> 3) * 5u) + (blockIdx.x & 7) * 3u) % (unsigned)nch);
  QTX_STAMP(0);

  // stream position p -> 16 KB slot of the weight stream (4 per chunk: W1a, W1b, W2 ch 0,
  // W2 ch 1): pass 1 the W1 slots, pass 2 all four; chunk c = (position + rot) mod nch
  auto slot_of = [&](int p) {
    const bool p2 = p >= 2 * nch;
    const int q = p2 ? p - 2 * nch : p;
    int c = (p2 ? q >> 2 : q >> 1) + rot;
    if (c >= nch) c -= nch;
    return 4 * c + (p2 ? (q & 3) : (q & 1));
  };
  auto issue = [&](int p) {
    if (p >= P) return;
    const int8_t* src = a.wf + (long)slot_of(p) * FF_SLOT + (w * FF_PPW) * 1024 + 16 * l;
    uint8_t* dst = ring + (p & (FF_NSLOT - 1)) * FF_SLOT + (w * FF_PPW) * 1024;
#pragma unroll
    for (int k = 0; k < FF_PPW; ++k) ff_dma(src + k * 1024, dst + k * 1024);
  };
  // top of slot p: this wave's pieces of it landed (the youngest memory operations are the
  // pieces of the slots issued after p: the loop issues nothing else), every wave's too, and
  // every wave is past what it read before this point (barrier); then the slots up to
  // `upto` are issued, position q into buffer q mod 4, which held q - 4: the caller passes
  // p + 3 when slot p - 1 is consumed, less when a slot before p is still to be read (both
  // W2 slots of a chunk are read after the W2b wait)
  int nissued = 0;                                   // positions issued so far (uniform)
  auto ring_wait = [&](int p, int upto) {
    const int younger = nissued - 1 - p;
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(2)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (; nissued <= upto && nissued < P; ++nissued) issue(nissued);
  };
  auto slot = [&](int p) { return ring + (p & (FF_NSLOT - 1)) * FF_SLOT + 16 * l; };

  // ---- prologue: the block's x1q into LDS in fragment order (fragment (rf, s) of the 8
  // 16-row fragments x 8 K steps at (8 rf + s) KB, lane l = row 16 rf + f, K bytes
  // 64 s + 16 g ..) by LDS-DMA from the KP layout, then the first three ring slots
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int fr = 8 * w + k, rf = fr >> 3, s = fr & 7;
    const int r = FULL ? m0 + 16 * rf + f : min(m0 + 16 * rf + f, mlast);
    ff_dma(a.A + kp_off(r, 64 * s + 16 * g, 512), xq + fr * 1024);
  }
  for (; nissued < 3; ++nissued) issue(nissued);
  for (int i = tid; i < F / 4; i += 512) {
    reinterpret_cast<float4*>(tsw)[i] = reinterpret_cast<const float4*>(a.sw1)[i];
    reinterpret_cast<float4*>(tb)[i] = reinterpret_cast<const float4*>(a.b1)[i];
  }
  float sar[2];                                       // x1q row scales of rows 32 rg + 16 rf + f
#pragma unroll
  for (int rf = 0; rf < 2; ++rf) {
    const int r = FULL ? m0 + 32 * rg + 16 * rf + f : min(m0 + 32 * rg + 16 * rf + f, mlast);
    sar[rf] = a.sa[r];
  }
  // the x1q pieces landed in every wave (with the first ring slots: a plain vmcnt(0), as
  // the row scales' loads sit among the youngest operations; VM_CNT_ORDER), tables written
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  QTX_STAMP(1);

  // ---- pass 1: the row maxima of h; the wave's x1q rows in registers
  v4i xr[2][8];
#pragma unroll
  for (int rf = 0; rf < 2; ++rf)
#pragma unroll
    for (int s = 0; s < 8; ++s) xr[rf][s] = ff_ld(xq + ((2 * rg + rf) * 8 + s) * 1024 + 16 * l);
  float mx[2] = {0.0f, 0.0f};
  for (int q = 0; q < nch; ++q) {
    v4i acc[2][2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {                 // W1a: K steps 0-3, W1b: 4-7
      ring_wait(2 * q + hh, 2 * q + hh + 3);
      const uint8_t* sl = slot(2 * q + hh);
      v4i wa[2][2];
#pragma unroll
      for (int cf = 0; cf < 2; ++cf) wa[0][cf] = ff_ld(sl + (2 * ch + cf) * 1024);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        if (s4 < 3)
#pragma unroll
          for (int cf = 0; cf < 2; ++cf) wa[(s4 + 1) & 1][cf] = ff_ld(sl + ((s4 + 1) * 4 + 2 * ch + cf) * 1024);
        __builtin_amdgcn_sched_barrier(0);
        const int s = 4 * hh + s4;
#pragma unroll
        for (int rf = 0; rf < 2; ++rf)
#pragma unroll
          for (int cf = 0; cf < 2; ++cf)
            acc[rf][cf] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wa[s4 & 1][cf], xr[rf][s],
                                                                 s == 0 ? v4i{0, 0, 0, 0} : acc[rf][cf], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    int c = q + rot;
    if (c >= nch) c -= nch;
#pragma unroll
    for (int cf = 0; cf < 2; ++cf) {
      const int col = 64 * c + 16 * (2 * ch + cf) + 4 * g;
      const float4 s4 = *reinterpret_cast<const float4*>(tsw + col);
      const float4 b4 = *reinterpret_cast<const float4*>(tb + col);
#pragma unroll
      for (int rf = 0; rf < 2; ++rf) {
        mx[rf] = fmaxf(mx[rf], ff_h(acc[rf][cf][0], sar[rf], s4.x, b4.x));
        mx[rf] = fmaxf(mx[rf], ff_h(acc[rf][cf][1], sar[rf], s4.y, b4.y));
        mx[rf] = fmaxf(mx[rf], ff_h(acc[rf][cf][2], sar[rf], s4.z, b4.z));
        mx[rf] = fmaxf(mx[rf], ff_h(acc[rf][cf][3], sar[rf], s4.w, b4.w));
      }
    }
  }
  // the row's maximum: the 4 lanes of row f (lane groups g), then the partner wave's half
  float* pm = reinterpret_cast<float*>(&hx[0][0][0]);   // [ch][128 rows]
#pragma unroll
  for (int rf = 0; rf < 2; ++rf) {
    mx[rf] = fmaxf(mx[rf], __shfl_xor(mx[rf], 16));
    mx[rf] = fmaxf(mx[rf], __shfl_xor(mx[rf], 32));
    if (g == 0) pm[128 * ch + 32 * rg + 16 * rf + f] = mx[rf];
  }
  __syncthreads();
  float sh[2], invh[2];                               // s_h of rows 32 rg + 16 rf + f
#pragma unroll
  for (int rf = 0; rf < 2; ++rf) {
    const int r = 32 * rg + 16 * rf + f;
    sh[rf] = scale127(fmaxf(fmaxf(pm[r], pm[128 + r]), 1e-5f));   // quant_scale(max, 127)
    invh[rf] = __builtin_amdgcn_rcpf(sh[rf]);
  }
  // the epilogue's layout needs s_h of rows 32 rg + 16 rf + 4 g + e: through LDS
  if (g == 0 && ch == 0) {
    shs[32 * rg + f] = sh[0];
    shs[32 * rg + 16 + f] = sh[1];
  }
  QTX_STAMP(2);

  // ---- pass 2: each chunk of h recomputed (x1q fragments from LDS), quantized with s_h,
  // the halves exchanged, FFN2 accumulated
  constexpr float BIAS = 12582912.0f;   // rint via the biased add (qtx_common.h rint_biased)
  v4i acc2[2][16];
#pragma unroll
  for (int rf = 0; rf < 2; ++rf)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc2[rf][j] = v4i{0, 0, 0, 0};
  long long tw = 0, t1 = 0, te = 0, t2 = 0;          // accumulated phase cycles (QTX_STAMPS)
  for (int q = 0; q < nch; ++q) {
    const int p0 = 2 * nch + 4 * q;
    v4i acc[2][2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      long long ts = QTX_NOW();
      ring_wait(p0 + hh, p0 + hh + 3);
      long long tn = QTX_NOW();
      tw += tn - ts;
      const uint8_t* sl = slot(p0 + hh);
      v4i wa[2][2], xa[2][2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        wa[0][k] = ff_ld(sl + (2 * ch + k) * 1024);
        xa[0][k] = ff_ld(xq + ((2 * rg + k) * 8 + 4 * hh) * 1024 + 16 * l);
      }
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int s = 4 * hh + s4;
        if (s4 < 3)
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            wa[(s4 + 1) & 1][k] = ff_ld(sl + ((s4 + 1) * 4 + 2 * ch + k) * 1024);
            xa[(s4 + 1) & 1][k] = ff_ld(xq + ((2 * rg + k) * 8 + s + 1) * 1024 + 16 * l);
          }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rf = 0; rf < 2; ++rf)
#pragma unroll
          for (int cf = 0; cf < 2; ++cf)
            acc[rf][cf] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wa[s4 & 1][cf], xa[s4 & 1][rf],
                                                                 s == 0 ? v4i{0, 0, 0, 0} : acc[rf][cf], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      t1 += QTX_NOW() - tn;
    }
    long long ts = QTX_NOW();
    int c = q + rot;
    if (c >= nch) c -= nch;
    // rint(h / s_h) as h * (1 / s_h) except within 2^-13 of a rounding tie, where the true
    // quotient is taken (quant_rows512's guarded form: exact)
    float t[2][2][4];
    float dm = 0.0f;
#pragma unroll
    for (int cf = 0; cf < 2; ++cf) {
      const int col = 64 * c + 16 * (2 * ch + cf) + 4 * g;
      const float4 s4 = *reinterpret_cast<const float4*>(tsw + col);
      const float4 b4 = *reinterpret_cast<const float4*>(tb + col);
      const float sw[4] = {s4.x, s4.y, s4.z, s4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int rf = 0; rf < 2; ++rf)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float r = ff_h(acc[rf][cf][e], sar[rf], sw[e], bb[e]) * invh[rf];
          t[rf][cf][e] = r + BIAS;
          dm = fmaxf(dm, fabsf(r - (t[rf][cf][e] - BIAS)));
        }
    }
    if (__builtin_expect(__ballot(dm > 0.5f - 0x1p-13f) != 0ull, 0)) {
#pragma unroll
      for (int cf = 0; cf < 2; ++cf) {
        const int col = 64 * c + 16 * (2 * ch + cf) + 4 * g;
        const float4 s4 = *reinterpret_cast<const float4*>(tsw + col);
        const float4 b4 = *reinterpret_cast<const float4*>(tb + col);
        const float sw[4] = {s4.x, s4.y, s4.z, s4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int rf = 0; rf < 2; ++rf)
#pragma unroll
          for (int e = 0; e < 4; ++e) t[rf][cf][e] = ff_h(acc[rf][cf][e], sar[rf], sw[e], bb[e]) / sh[rf] + BIAS;
      }
    }
    uint2 own[2];
#pragma unroll
    for (int rf = 0; rf < 2; ++rf) {
      own[rf] = make_uint2(pack4_biased(t[rf][0][0], t[rf][0][1], t[rf][0][2], t[rf][0][3]),
                           pack4_biased(t[rf][1][0], t[rf][1][1], t[rf][1][2], t[rf][1][3]));
      hx[w][rf][l] = own[rf];
    }
    long long tn = QTX_NOW();
    te += tn - ts;
    ring_wait(p0 + 2, p0 + 5);                       // barrier: the partner's half is in hx
    v4i hq[2];
#pragma unroll
    for (int rf = 0; rf < 2; ++rf) {
      const uint2 pt = hx[w ^ 4][rf][l];
      hq[rf] = ch == 0 ? v4i{(int)own[rf].x, (int)own[rf].y, (int)pt.x, (int)pt.y}
                       : v4i{(int)pt.x, (int)pt.y, (int)own[rf].x, (int)own[rf].y};
    }
    ring_wait(p0 + 3, p0 + 5);                       // W2a (p0 + 2) is read below: not p0 + 6
    ts = QTX_NOW();
    tw += ts - tn;
    const uint8_t* s2 = slot(p0 + 2 + ch);
    v4i wb[4];
#pragma unroll
    for (int j = 0; j < 2; ++j) wb[j] = ff_ld(s2 + j * 1024);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j + 2 < 16) wb[(j + 2) & 3] = ff_ld(s2 + (j + 2) * 1024);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rf = 0; rf < 2; ++rf)
        acc2[rf][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(hq[rf], wb[j & 3], acc2[rf][j], 0, 0, 0);
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
  // Lane: rows 32 rg + 16 rf + 4 g + e, columns ff_col2(ch, j, f): canonical lane L = 4f + t
  // (t = 2ch + tt) owns columns 4L .. (j = 4 tt ..) and 256 + 4L .. (j = 8 + 4 tt ..).
  __syncthreads();                                   // every wave is done with the ring
  float* et = reinterpret_cast<float*>(ring);        // [4][512]: sw2, b2, ln_a, ln_b
  float* ex = et + 2048;                             // [8 waves][4 rows][64 lanes] exchange
  et[tid] = a.sw2[tid];
  et[512 + tid] = a.b2[tid];
  et[1024 + tid] = a.ln_a[tid];
  et[1536 + tid] = a.ln_b[tid];
  __syncthreads();
  auto colv = [&](const float* tab, int run, int k) {   // 4 consecutive columns of a run
    return *reinterpret_cast<const float4*>(tab + 256 * run + 16 * f + 8 * ch + 4 * k);
  };
  // the partner's value of each of the 4 rows through LDS (workgroup barriers: every wave
  // of the block runs the same epilogue, so they are uniform)
  auto exchange = [&](float (&u)[4], float (&o)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) ex[(w * 4 + e) * 64 + l] = u[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = ex[((w ^ 4) * 4 + e) * 64 + l];
    __syncthreads();
  };
#pragma unroll
  for (int rf = 0; rf < 2; ++rf) {
    const int rbase = m0 + 32 * rg + 16 * rf + 4 * g;
    float v[4][16];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = FULL ? rbase + e : min(rbase + e, mlast);
      const float* rp = a.x + (long)row * 512 + 16 * f + 8 * ch;
      const float she = shs[32 * rg + 16 * rf + 4 * g + e];
      float4 rv[4];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        rv[k] = *reinterpret_cast<const float4*>(rp + 4 * k);
        rv[2 + k] = *reinterpret_cast<const float4*>(rp + 256 + 4 * k);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int run = k >> 1, kk = k & 1;
        const float4 s4 = colv(et, run, kk), b4 = colv(et + 512, run, kk);
        const float sw[4] = {s4.x, s4.y, s4.z, s4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
        const float rr[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
          v[e][4 * k + i] = rr[i] + (((float)acc2[rf][4 * k + i][e] * she) * sw[i] + bb[i]);
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = rbase + e;
      if (FULL || row < a.M) {
        float* xp = a.x + (long)row * 512 + 16 * f + 8 * ch;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          *reinterpret_cast<float4*>(xp + 4 * k) =
              make_float4(v[e][4 * k], v[e][4 * k + 1], v[e][4 * k + 2], v[e][4 * k + 3]);
          *reinterpret_cast<float4*>(xp + 256 + 4 * k) =
              make_float4(v[e][8 + 4 * k], v[e][9 + 4 * k], v[e][10 + 4 * k], v[e][11 + 4 * k]);
        }
      }
    }
    // LayerNorm in ln_rows512's order: canonical lane L sums its chunk-0 values then its
    // chunk-1 values sequentially; the 64-lane tree is L^1 in the lane, L^2 with the partner
    // wave (u_ch0 + u_ch1 — the same sum in both waves), then L^4 .. L^32 = row16_sum
    float u[4], o[4], tot[4];
    auto row_sums = [&](bool sq) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float ps[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const float* vv = v[e];
          float s = sq ? vv[4 * tt] * vv[4 * tt] : vv[4 * tt];
#pragma unroll
          for (int i = 1; i < 4; ++i) s = s + (sq ? vv[4 * tt + i] * vv[4 * tt + i] : vv[4 * tt + i]);
#pragma unroll
          for (int i = 0; i < 4; ++i) s = s + (sq ? vv[8 + 4 * tt + i] * vv[8 + 4 * tt + i] : vv[8 + 4 * tt + i]);
          ps[tt] = s;
        }
        u[e] = ps[0] + ps[1];
      }
      exchange(u, o);
#pragma unroll
      for (int e = 0; e < 4; ++e) tot[e] = row16_sum(ch == 0 ? u[e] + o[e] : o[e] + u[e]);
    };
    row_sums(false);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float mean = tot[e] / 512.0f;
#pragma unroll
      for (int j = 0; j < 16; ++j) v[e][j] = v[e][j] - mean;
    }
    row_sums(true);
    float den[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) den[e] = tot[e];
    div_const_n<4>(den, 511.0f);
#pragma unroll
    for (int e = 0; e < 4; ++e) den[e] = sqrtf(den[e]) + 1e-6f;
    // (a * d) / den + b, the division correctly rounded (ln_rows512's guard and div_cr)
    uint32_t mxb = 0u;
    float mn = __builtin_inff();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 g4 = colv(et + 1024, k >> 1, k & 1);
      const float ga[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float& x = v[e][4 * k + i];
          x = ga[i] * x;
          mxb = max(mxb, __float_as_uint(x) & 0x7fffffffu);
          mn = fminf(mn, fabsf(x));
        }
    }
    bool dok = true;
#pragma unroll
    for (int e = 0; e < 4; ++e) dok &= divisor_ok(den[e]);
    bool ok = dok && mxb < 0x5d800000u && mn > 0x1p-60f;
    if (__builtin_expect(__ballot(!ok) != 0ull, 0)) {
      DivRange rg2;
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < 16; ++j) rg2.add(v[e][j]);
      ok = dok && rg2.ok();
    }
    if (__builtin_expect(__ballot(!ok) == 0ull, 1)) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float yd = 1.0f / den[e];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[e][j] = div_cr(v[e][j], den[e], yd);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < 16; ++j) v[e][j] = v[e][j] / den[e];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 b4 = colv(et + 1536, k >> 1, k & 1);
      const float gb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 4; ++i) v[e][4 * k + i] = v[e][4 * k + i] + gb[i];
    }
    if constexpr (LNQ) {
      // per-token quantization (quant_rows512's order and guarded rint); the row's
      // maximum: own 16 values, the 16-lane row, the partner wave
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float am = 0.0f;
#pragma unroll
        for (int j = 0; j < 16; ++j) am = fmaxf(am, fabsf(v[e][j]));
        u[e] = row16_max(am);
      }
      exchange(u, o);
      float sc[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) sc[e] = fmaxf(fmaxf(u[e], o[e]), 1e-5f);
      div_const_n<4>(sc, 127.0f);
      // one near-tie vote per row (the values are those of one vote over all: the true
      // quotient is exact either way), so only a row's 4 packed dwords are live at a time
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float inv = __builtin_amdgcn_rcpf(sc[e]);
        uint32_t pk[4];
        float dq = 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float tq[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float r = v[e][4 * k + i] * inv;
            tq[i] = r + BIAS;
            dq = fmaxf(dq, fabsf(r - (tq[i] - BIAS)));
          }
          pk[k] = pack4_biased(tq[0], tq[1], tq[2], tq[3]);
        }
        if (__builtin_expect(__ballot(dq > 0.5f - 0x1p-13f) != 0ull, 0)) {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            pk[k] = pack4_biased(v[e][4 * k] / sc[e] + BIAS, v[e][4 * k + 1] / sc[e] + BIAS,
                                 v[e][4 * k + 2] / sc[e] + BIAS, v[e][4 * k + 3] / sc[e] + BIAS);
        }
        const int row = rbase + e;
        if (FULL || row < a.M) {
#pragma unroll
          for (int run = 0; run < 2; ++run)
            *reinterpret_cast<uint2*>(a.lnq + kp_off(row, 256 * run + 16 * f + 8 * ch, 512)) =
                make_uint2(pk[2 * run], pk[2 * run + 1]);
          if (f == 0 && ch == 0) a.lns[row] = sc[e];
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rbase + e;
        if (FULL || row < a.M) {
          float* op = a.lnout + (long)row * 512 + 16 * f + 8 * ch;
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            *reinterpret_cast<float4*>(op + 4 * k) =
                make_float4(v[e][4 * k], v[e][4 * k + 1], v[e][4 * k + 2], v[e][4 * k + 3]);
            *reinterpret_cast<float4*>(op + 256 + 4 * k) =
                make_float4(v[e][8 + 4 * k], v[e][9 + 4 * k], v[e][10 + 4 * k], v[e][11 + 4 * k]);
          }
        }
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

// W1 int8 [F, 512] and W2 int8 [512, F] (row-major) -> the fused FFN weight stream: per
// 64-column chunk c, four 16 KB slots of 16 fragments x 64 lanes x 16 bytes:
//   slots 4c, 4c+1 (W1, K steps 4h .. 4h+3), fragment 4s' + j', lane l:
//       W1[64c + 16j' + (l & 15)][64(4h + s') + 16(l >> 4) .. +16]
//   slots 4c+2+ch (W2, column half ch), fragment j, lane l:
//       byte 4j' + e = W2[ff_col2(ch, j, l & 15)][64c + 16j' + 4(l >> 4) + e]
// One thread per 16-byte lane piece.
__global__ void k_pack_ffn(const int8_t* W1, const int8_t* W2, int F, int8_t* out) {
  const long u = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nu = (long)F / 64 * 4 * 1024;
  if (u >= nu) return;
  const int c = (int)(u / 4096), part = (int)((u / 1024) & 3), v = (int)(u % 1024);
  const int fr = v / 64, lane = v % 64, f = lane & 15, g = lane >> 4;
  uint4 d;
  if (part < 2) {
    const int s = 4 * part + (fr >> 2), j = fr & 3;
    d = *reinterpret_cast<const uint4*>(W1 + (long)(64 * c + 16 * j + f) * 512 + 64 * s + 16 * g);
  } else {
    const int8_t* row = W2 + (long)ff_col2(part - 2, fr, f) * F + 64 * c + 4 * g;
    d = make_uint4(*reinterpret_cast<const uint32_t*>(row), *reinterpret_cast<const uint32_t*>(row + 16),
                   *reinterpret_cast<const uint32_t*>(row + 32), *reinterpret_cast<const uint32_t*>(row + 48));
  }
  *reinterpret_cast<uint4*>(out + 16 * u) = d;
}

hipError_t launch_pack_ffn(const int8_t* W1, const int8_t* W2, int F, int8_t* out, hipStream_t st) {
  if (F % 64 || F < 256 || F > 2048) return hipErrorInvalidValue;
  const long nu = (long)F / 64 * 4 * 1024;
  k_pack_ffn<<<dim3((unsigned)((nu + 255) / 256)), dim3(256), 0, st>>>(W1, W2, F, out);
  return hipGetLastError();
}

}  // namespace qtx
