// qtx_wsgemm_diag.hip — DIAGNOSTIC BUILD ONLY (compiled into libqtx_diag.so by
// qtx/_build.py build(extra=...), never into the product libqtx.so): weight-stationary
// GEMM variants that were measured and not kept, kept reproducible for A/B
// runs: k_gemm_wsz / k_gemm_wsa / k_gemm_wsa2 (round 4), k_gemm_wss and k_gemm_wsx (round 3).
// launch_gemm_ws_diag() is consulted by launch_gemm_ws / launch_gemm_wsx in QTX_DIAG builds.
#include <cstdlib>
#include <type_traits>

#include "../qtx_knobs.h"
#include "../qtx_ws.h"

namespace qtx {

// =====================================================================================
// k_gemm_wsz: the weight-stationary Q/K/V GEMM (RE_QUANT) with its WHOLE epilogue between
// the MFMAs.  k_gemm_wsq interleaves only the quantization and runs y = ((acc * sa) * sw) + b
// as a VALU-only phase after the block's MFMAs; its stamps show the matrix pipe idle during
// that phase and the younger wave of each SIMD finishing its MFMAs ~1,200 cycles after the
// older one, so a block took ~3x its 2,048-cycle MFMA floor.  Here one more
// block of lag removes the VALU-only phase:
//   iteration k:  top barrier (block k's A landed; the partial row maxima of block k-2
//                 complete in red[k & 1]); block k+1's A and row scales by LDS-DMA; the 64
//                 MFMAs of block k, with ONE output of y(k-1) (converted in place in the
//                 registers that hold block k-1's accumulators, its partial row maximum
//                 folded) pinned after every odd MFMA and ONE quantized output of block k-2
//                 after every even one; then block k-1's partial row maxima -> red[(k-1) & 1].
// Three register buffers of 32 VGPRs rotate through the roles accumulators(k) / y(k-1) /
// y(k-2), so the iteration is unrolled by three.  Per MFMA the wave then issues ~5 VALU
// (half a y output, half a quantized one) in the gaps the matrix pipe leaves, instead of
// ~2.4 beside it and ~5 per output alone afterwards.  Numerics: exactly k_gemm_wsq's (the
// same canonical operations per output; GPU == oracle bit for bit).
// Row scales: block k's 32 scales come by LDS-DMA with its A rows into sal[k % 3] (three
// slots: block k+1's DMA is issued while y(k-1) still reads its slot).
// =====================================================================================
template <int XG = 1>
__global__ __launch_bounds__(512) void k_gemm_wsz(RowGemmArgs g) {
  constexpr int SR = WS_SR, WL = 8 * (8 - SR) * 4 * 1024;
  // LDS: 2 A stages (32 KB) | W K steps 5-7 (96 KB) | sw, bias (4 KB) | red [2][8][32] (2 KB) |
  // sal [3][8 waves][64] (6 KB)
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WP_STAGE + WL + 4096 + 2 * 8 * WP_R * 4 + 3 * 8 * 64 * 4];
  uint8_t* const wl = lds + 2 * WP_STAGE;
  float* const swl = reinterpret_cast<float*>(wl + WL);
  float* const red0 = swl + 1024;                            // [2][8][32]
  float* const sal = red0 + 2 * 8 * WP_R;                    // [3][8 waves][64]: row scales
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int f = lane & 15, gq = lane >> 4;
  const int nsl = g.N >> 9;
  const int wpt = gridDim.x / nsl;
  int t = blockIdx.x % nsl, r0 = blockIdx.x / nsl;
  if (XG) {          // the slices of a row group on one XCD (speed only), as k_gemm_wsq
    const int b = blockIdx.x, A = gridDim.x / (8 * nsl), aligned = 8 * nsl * A;
    if (b < aligned) {
      const int j = b >> 3;
      t = j % nsl;
      r0 = 8 * (j / nsl) + (b & 7);
    } else {
      t = (b - aligned) % nsl;
      r0 = 8 * A + (b - aligned) / nsl;
    }
  }
  const int nb = (g.M + WP_R - 1) / WP_R;
  if (r0 >= nb) return;
  const int nblk = (nb - r0 + wpt - 1) / wpt;

  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto dma4 = [](const float* gsrc, const float* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto rbk = [&](int k) { return r0 + min(k, nblk - 1) * wpt; };
  auto issue = [&](int k) {
    uint8_t* st = lds + (k & 1) * WP_STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long row = min(rbk(k) * WP_R + 16 * i + f, g.M - 1);
      dma16(g.A + kp_off(row, 64 * wave + 16 * gq, WS_K), st + ((wave * 2 + i) << 10));
    }
    dma4(g.sa + min(rbk(k) * WP_R + (lane & 31), g.M - 1), sal + ((k % 3) * 8 + wave) * 64);
  };
  issue(0);
  v4i wr[SR][4];
  {
    const int8_t* wsrc = g.W + ((long)(t * 8 + wave) << 15);
    const v4i* ws = reinterpret_cast<const v4i*>(wsrc) + lane;
#pragma unroll
    for (int s = 0; s < SR; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) wr[s][j] = ws[(s * 4 + j) * 64];
#pragma unroll
    for (int p = 0; p < (8 - SR) * 4; ++p)
      dma16(wsrc + ((SR * 4 + p) << 10) + lane * 16, wl + ((wave * (8 - SR) * 4 + p) << 10));
    if (wave < 4) {
      const int c = 128 * wave + 2 * lane;
      *reinterpret_cast<float2*>(swl + c) = *reinterpret_cast<const float2*>(g.sw + 512 * t + c);
      *reinterpret_cast<float2*>(swl + 512 + c) = *reinterpret_cast<const float2*>(g.bias + 512 * t + c);
    }
#pragma unroll
    for (int s = 0; s < SR; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(wr[s][j]));
  }
  const int cs = 64 * wave + 16 * gq;
  const __amdgpu_buffer_rsrc_t orsrc = ws_rsrc(g.out8 + (long)t * g.o8_ts, (long)g.M * g.ldo8);
  const __amdgpu_buffer_rsrc_t srsrc = ws_rsrc(g.os + (long)t * g.os_ts, 4L * g.M);
  auto redb = [&](int k) { return red0 + (k & 1) * 8 * WP_R; };

  // block k's scale per row (lane: row lane & 31) from its complete partial maxima, stored;
  // broadcast per row fragment: divisor bq, reciprocal iq
  auto scales = [&](int k, float (&bq)[2], float (&iq)[2]) {
    const float* red = redb(k);
    float m = red[lane & 31];
#pragma unroll
    for (int w = 1; w < 8; ++w) m = fmaxf(m, red[w * WP_R + (lane & 31)]);
    const float sc = fmaxf(m, 1e-5f) / 127.0f;
    const float inv = 1.0f / sc;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sc), srsrc, 4 * (rbk(k) * WP_R + (lane & 31)), 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bq[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (16 * i + f), __float_as_int(sc)));
      iq[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (16 * i + f), __float_as_int(inv)));
    }
  };
  auto store_row = [&](int k, int i, const uint32_t (&d)[4]) {
    const long row = rbk(k) * WP_R + 16 * i + f;
    __builtin_amdgcn_raw_buffer_store_b128(v4u{d[0], d[1], d[2], d[3]}, orsrc, (int)(row * g.ldo8 + cs), 0, 0);
  };
  // the partial row maxima of block k (am: the lane's 16 columns of rows 16i + f) -> red
  auto put_max = [&](int k, const float (&am)[2]) {
    float* red = redb(k);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float a = am[i];
      a = fmaxf(a, __shfl_xor(a, 16));
      a = fmaxf(a, __shfl_xor(a, 32));
      red[wave * WP_R + 16 * i + f] = a;
    }
  };
  // one y output (y of block ky, in place): o -> column group jj, row fragment ii, element e
  auto y_one = [&](v4i (&YB)[2][4], int o, const float (&sr)[2], float4& s4, float4& b4, float (&am)[2],
                   float av) {
    const int jj = o >> 3, ii = (o >> 2) & 1, e = o & 3;
    const float swe = e == 0 ? s4.x : e == 1 ? s4.y : e == 2 ? s4.z : s4.w;
    const float be = e == 0 ? b4.x : e == 1 ? b4.y : e == 2 ? b4.z : b4.w;
    const float v = ((float)__float_as_int(av) * sr[ii]) * swe + be;
    am[ii] = fmaxf(am[ii], fabsf(v));
    YB[ii][jj][e] = __float_as_int(v);
    (void)jj;
    return v;
  };
  auto sw_group = [&](int jj, float4& s4, float4& b4) {
    s4 = *reinterpret_cast<const float4*>(swl + cs + 4 * jj);
    b4 = *reinterpret_cast<const float4*>(swl + 512 + cs + 4 * jj);
  };
  // one quantized output of block kq (y in QB): o -> row fragment ii, column group jj, e
  auto q_val = [&](float yv, int ii, const float (&bq)[2], const float (&iq)[2]) {
    return rint_biased(div_cr(yv, bq[ii], iq[ii]));
  };

  // iteration k with compile-time roles: HM = MFMAs of block k into MF, HY = y(k-1) in YB,
  // HQ = quantization of block k-2 from QB
  auto iter = [&](int k, v4i (&MF)[2][4], v4i (&YB)[2][4], v4i (&QB)[2][4], auto hm, auto hy, auto hq) {
    constexpr bool HM = decltype(hm)::value, HY = decltype(hy)::value, HQ = decltype(hq)::value;
#ifndef QTX_WSZ_NOWAIT                               // diagnostic builds only (timing)
    __builtin_amdgcn_s_waitcnt(WAIT_VM(0));     // block k's DMA and the last stores (VM_CNT_ORDER)
#endif
    __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
#ifndef QTX_WSZ_NOBAR                                // diagnostic builds only (timing)
    __builtin_amdgcn_s_barrier();
#endif
#ifndef QTX_WSZ_NODMA
    if (HM && k + 1 < nblk) issue(k + 1);
#endif
    float bq[2] = {0.0f, 0.0f}, iq[2] = {0.0f, 0.0f};
    if constexpr (HQ) scales(k - 2, bq, iq);
    float sr[2] = {0.0f, 0.0f};
    if constexpr (HY) {
#pragma unroll
      for (int i = 0; i < 2; ++i) sr[i] = sal[(((k - 1) % 3) * 8 + wave) * 64 + 16 * i + f];
    }
    float am[2] = {0.0f, 0.0f};
    float4 s4, b4;
    if constexpr (HY) sw_group(0, s4, b4);
    uint32_t d[4];
    float tq[4];
    if constexpr (HM) {
      // row fragment major (i, then K step s, then column fragment j): the accumulators of
      // row fragment 1 start only half way, while the quantization (first half, one output
      // per MFMA) has freed y(k-2) — the three buffers are never all live at once.  Each
      // step's A fragment (and W fragments from LDS) are read one step ahead, and a pinned
      // output's result gates the MFMA ZL places later (its dependent chain of 4-5 VALU then
      // runs under ZL MFMAs instead of stalling the next one).
      constexpr int ZL = 3;
      const uint8_t* cur = lds + (k & 1) * WP_STAGE;
      float qh[ZL], yh[ZL];                 // the last ZL quantized / y results (pins)
#pragma unroll
      for (int z = 0; z < ZL; ++z) qh[z] = yh[z] = 0.0f;
      auto lda = [&](int i, int s) { return *reinterpret_cast<const v4i*>(cur + ((s * 2 + i) << 10) + lane * 16); };
      auto ldw = [&](int s, int j) {
        return *reinterpret_cast<const v4i*>(wl + (((wave * (8 - SR) + s - SR) * 4 + j) << 10) + lane * 16);
      };
      v4i an = lda(0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const v4i a = an;
          v4i b[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) b[j] = s < SR ? wr[s < SR ? s : 0][j] : ldw(s, j);
#ifdef QTX_WSZ_NOWLDS                                 // diagnostic builds only (timing)
#pragma unroll
          for (int j = 0; j < 4; ++j) b[j] = wr[s % SR][j];
#endif
          if (s < 7 || i == 0) an = lda(s < 7 ? i : 1, s < 7 ? s + 1 : 0);
#ifdef QTX_WSZ_NOALDS
          an = wr[(s + i) % SR][s & 3];
#endif
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = i * 32 + s * 4 + j;
#ifdef QTX_WSZ_NOQ                                  // diagnostic builds only (timing)
            constexpr bool DQ = false;
#else
            constexpr bool DQ = true;
#endif
#ifdef QTX_WSZ_NOY
            constexpr bool DY = false;
#else
            constexpr bool DY = true;
#endif
            if (n < 32 && HQ && DQ) {
              const int o = n, ii = o >> 4, jj = (o >> 2) & 3, e = o & 3;
              float yv = __int_as_float(QB[ii][jj][e]);
              if (s == 0) mfma_pin<true>(MF[i][j], b[j], a, qh[ZL - 1], yv);
              else mfma_pin<false>(MF[i][j], b[j], a, qh[ZL - 1], yv);
              tq[e] = q_val(yv, ii, bq, iq);
#pragma unroll
              for (int z = ZL - 1; z > 0; --z) qh[z] = qh[z - 1];
              qh[0] = tq[e];
              if (e == 3) {
                d[jj] = pack4_biased(tq[0], tq[1], tq[2], tq[3]);
                if (jj == 3) store_row(k - 2, ii, d);
              }
            } else if (n >= 32 && HY && DY) {
              const int o = n - 32, jj = o >> 3, ii = (o >> 2) & 1, e = o & 3;
              if (e == 0 && ii == 0 && jj > 0) sw_group(jj, s4, b4);
              float av = __int_as_float(YB[ii][jj][e]);
              if (s == 0) mfma_pin<true>(MF[i][j], b[j], a, yh[ZL - 1], av);
              else mfma_pin<false>(MF[i][j], b[j], a, yh[ZL - 1], av);
#pragma unroll
              for (int z = ZL - 1; z > 0; --z) yh[z] = yh[z - 1];
              yh[0] = y_one(YB, o, sr, s4, b4, am, av);
            } else {
              if (s == 0) mfma_asm<true>(MF[i][j], b[j], a);
              else mfma_asm<false>(MF[i][j], b[j], a);
            }
          }
        }
      mfma_settle(MF);
    } else {
      // no MFMAs left (the last two iterations): the same outputs, plain VALU
      if constexpr (HQ) {
#pragma unroll
        for (int o = 0; o < 32; ++o) {
          const int ii = o >> 4, jj = (o >> 2) & 3, e = o & 3;
          tq[e] = q_val(__int_as_float(QB[ii][jj][e]), ii, bq, iq);
          if (e == 3) {
            d[jj] = pack4_biased(tq[0], tq[1], tq[2], tq[3]);
            if (jj == 3) store_row(k - 2, ii, d);
          }
        }
      }
      if constexpr (HY) {
#pragma unroll
        for (int o = 0; o < 32; ++o) {
          const int jj = o >> 3, ii = (o >> 2) & 1, e = o & 3;
          if (e == 0 && ii == 0 && jj > 0) sw_group(jj, s4, b4);
          y_one(YB, o, sr, s4, b4, am, __int_as_float(YB[ii][jj][e]));
        }
      }
    }
    if constexpr (HY) put_max(k - 1, am);
  };
  const std::true_type T_{};
  const std::false_type F_{};

  v4i B0[2][4], B1[2][4], B2[2][4];
  // roles in iteration k: accumulators B[k % 3], y(k-1) in B[(k-1) % 3], y(k-2) in B[(k-2) % 3].
  // The loop runs whole groups of three iterations, so every path into the remainder below
  // has the same register roles (breaking out between the three would merge three role
  // permutations and the compiler copies / spills the buffers).
  iter(0, B0, B2, B1, T_, F_, F_);
  if (nblk == 1) {
    iter(1, B1, B0, B2, F_, T_, F_);
    iter(2, B2, B1, B0, F_, F_, T_);
  } else {
    iter(1, B1, B0, B2, T_, T_, F_);
    int k = 2;
    for (; k + 3 <= nblk; k += 3) {
      iter(k, B2, B1, B0, T_, T_, T_);
      iter(k + 1, B0, B2, B1, T_, T_, T_);
      iter(k + 2, B1, B0, B2, T_, T_, T_);
    }
    // k % 3 == 2; nblk - k in {0, 1, 2} iterations with MFMAs left, then the two tails
    if (k == nblk) {
      iter(k, B2, B1, B0, F_, T_, T_);
      iter(k + 1, B0, B2, B1, F_, F_, T_);
    } else if (k + 1 == nblk) {
      iter(k, B2, B1, B0, T_, T_, T_);
      iter(k + 1, B0, B2, B1, F_, T_, T_);
      iter(k + 2, B1, B0, B2, F_, F_, T_);
    } else {
      iter(k, B2, B1, B0, T_, T_, T_);
      iter(k + 1, B0, B2, B1, T_, T_, T_);
      iter(k + 2, B1, B0, B2, F_, T_, T_);
      iter(k + 3, B2, B1, B0, F_, F_, T_);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// =====================================================================================
// k_gemm_wsa: the weight-stationary Q/K/V GEMM (RE_QUANT) with ONE wave per SIMD and the
// whole slice of W in accumulation registers.  A 256-thread workgroup (4 waves, 512
// registers per lane each) keeps its 512-column slice of W (256 KB) in the waves' AGPRs —
// wave w holds columns 128w .. 128w+127 for all of K, 256 AGPRs — so the main loop reads
// only A from LDS (16 KB per 32-row block for the whole workgroup: 64 ds_read_b128, against
// k_gemm_wsq's 224 KB of A and W fragment reads), and the VGPRs hold three 64-register
// buffers that rotate through accumulators(k) / y(k-1) / y(k-2):
//   iteration k:  wait for block k's A (LDS-DMA issued two iterations ago: a counted vmcnt
//                 whose youngest operations are only the next block's DMA, VM_CNT_ORDER);
//                 barrier; the codes of block k-3 stored; block k+2's A by LDS-DMA; the 128
//                 MFMAs of block k with one quantized output of block k-2 pinned after every
//                 even MFMA and one y output of block k-1 (in place, partial row maximum
//                 folded) after every odd one; block k-1's partial row maxima -> red.
// Numerics: exactly k_gemm_wsq's (the same canonical operations per output).
// =====================================================================================
template <bool Z, typename T>
__device__ __forceinline__ void mfma_pin_a(v4i& acc, const v4i& w, const v4i& a, float before, T& after) {
  if constexpr (Z)
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %2, %3, 0" : "=&v"(acc), "+v"(after) : "a"(w), "v"(a), "v"(before));
  else
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %2, %3, %0" : "+v"(acc), "+v"(after) : "a"(w), "v"(a), "v"(before));
}
template <bool Z>
__device__ __forceinline__ void mfma_asm_a(v4i& acc, const v4i& w, const v4i& a) {
  if constexpr (Z)
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, 0" : "=&v"(acc) : "a"(w), "v"(a));
  else
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(a));
}
__device__ __forceinline__ void mfma_settle8(v4i (&acc)[8]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4"
               : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]),
                 "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]));
}

template <int XG = 1>
__global__ __launch_bounds__(256, 1) void k_gemm_wsa(RowGemmArgs g) {
  constexpr int NS = 3;                                      // A stages (prefetch distance 2)
  constexpr int R = 16, STG = R * WS_K;                      // 16-row blocks: 8 KB A stages
  // LDS: 3 A stages (24 KB) | sw, bias (4 KB) | red [2][4][16] | sal [3][4 waves][64] (3 KB)
  __shared__ __attribute__((aligned(16))) uint8_t lds[NS * STG + 4096 + 2 * 4 * R * 4 + 3 * 4 * 64 * 4];
  float* const swl = reinterpret_cast<float*>(lds + NS * STG);
  float* const red0 = swl + 1024;                            // [2][4][16]
  float* const sal = red0 + 2 * 4 * R;                       // [3][4 waves][64]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int f = lane & 15, gq = lane >> 4;
  const int nsl = g.N >> 9;
  const int wpt = gridDim.x / nsl;
  int t = blockIdx.x % nsl, r0 = blockIdx.x / nsl;
  if (XG) {          // the slices of a row group on one XCD (speed only), as k_gemm_wsq
    const int b = blockIdx.x, A = gridDim.x / (8 * nsl), aligned = 8 * nsl * A;
    if (b < aligned) {
      const int j = b >> 3;
      t = j % nsl;
      r0 = 8 * (j / nsl) + (b & 7);
    } else {
      t = (b - aligned) % nsl;
      r0 = 8 * A + (b - aligned) / nsl;
    }
  }
  const int nb = (g.M + R - 1) / R;
  if (r0 >= nb) return;
  const int nblk = (nb - r0 + wpt - 1) / wpt;

  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto dma4 = [](const float* gsrc, const float* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto rbk = [&](int k) { return r0 + min(k, nblk - 1) * wpt; };
  // block k's A (wave w: K steps 2w, 2w+1) and row scales: 3 VM operations per wave
  constexpr int WSA_DMA_OPS = 3;
  auto issue = [&](int k) {
    uint8_t* st = lds + (k % NS) * STG;
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const int s = 2 * wave + ss;
      const long row = min(rbk(k) * R + f, g.M - 1);
      dma16(g.A + kp_off(row, 64 * s + 16 * gq, WS_K), st + (s << 10));
    }
    dma4(g.sa + min(rbk(k) * R + f, g.M - 1), sal + ((k % 3) * 4 + wave) * 64);
  };
  // W: fragment (s, jn) of this wave = WS-layout fragment (s, jn & 3) of 64-column group
  // 2w + (jn >> 2) (k_pack_w_ws); used only as the MFMAs' "a" operand: it lives in AGPRs
  v4i wa[8][8];
  {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int jn = 0; jn < 8; ++jn) {
        const int8_t* src = g.W + ((long)(t * 8 + 2 * wave + (jn >> 2)) << 15) + ((s * 4 + (jn & 3)) << 10) + lane * 16;
        wa[s][jn] = *reinterpret_cast<const v4i*>(src);
      }
    const int c = 2 * tid;
    *reinterpret_cast<float2*>(swl + c) = *reinterpret_cast<const float2*>(g.sw + 512 * t + c);
    *reinterpret_cast<float2*>(swl + 512 + c) = *reinterpret_cast<const float2*>(g.bias + 512 * t + c);
  }
  issue(0);
  if (nblk > 1) issue(1);
  // the lane's two 16-column groups h: columns cs(h) + 4jj + e within the slice
  auto csh = [&](int h) { return 64 * (2 * wave + h) + 16 * gq; };
  const __amdgpu_buffer_rsrc_t orsrc = ws_rsrc(g.out8 + (long)t * g.o8_ts, (long)g.M * g.ldo8);
  const __amdgpu_buffer_rsrc_t srsrc = ws_rsrc(g.os + (long)t * g.os_ts, 4L * g.M);
  auto redb = [&](int k) { return red0 + (k & 1) * 4 * R; };

  // block k's scale per row from its complete partial maxima; broadcast per row fragment
  // (lane: row f; lanes 16-63 repeat rows 0-15, so each lane holds its own row's scale)
  auto scales = [&](int k, float& sc, float& bq, float& iq) {
    const float* red = redb(k);
    float m = red[f];
#pragma unroll
    for (int w = 1; w < 4; ++w) m = fmaxf(m, red[w * R + f]);
    sc = fmaxf(m, 1e-5f) / 127.0f;
    bq = sc;
    iq = 1.0f / sc;
  };
  // 16 codes of block k, column group h
  auto store_row = [&](int k, int h, const uint32_t (&d)[4]) {
    const long row = rbk(k) * R + f;
    __builtin_amdgcn_raw_buffer_store_b128(v4u{d[0], d[1], d[2], d[3]}, orsrc, (int)(row * g.ldo8 + csh(h)), 0, 0);
  };
  auto put_max = [&](int k, float am) {
    float* red = redb(k);
    am = fmaxf(am, __shfl_xor(am, 16));
    am = fmaxf(am, __shfl_xor(am, 32));
    red[wave * R + f] = am;
  };
  auto sw_group = [&](int h, int jj, float4& s4, float4& b4) {
    s4 = *reinterpret_cast<const float4*>(swl + csh(h) + 4 * jj);
    b4 = *reinterpret_cast<const float4*>(swl + 512 + csh(h) + 4 * jj);
  };
  auto el = [](const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; };
  // y output o of YB (in place): group h, column group jj, row fragment ii, element e
  auto y_val = [&](int av, float sr, float swe, float be) {
#ifdef QTX_WSA_FAST
    return fmaf((float)av, sr * swe, be);
#else
    return ((float)av * sr) * swe + be;
#endif
  };
  auto q_val = [&](float yv, float bq, float iq) {
#ifdef QTX_WSA_FAST
    (void)bq;
    return fmaf(yv, iq, 12582912.0f);
#else
    return rint_biased(div_cr(yv, bq, iq));
#endif
  };

  auto iter = [&](int k, v4i (&MF)[8], v4i (&YB)[8], v4i (&QB)[8], auto hm, auto hy, auto hq) {
    constexpr bool HM = decltype(hm)::value, HY = decltype(hy)::value, HQ = decltype(hq)::value;
    // block k's DMA landed: only block k+1's (issued after every older operation of this
    // wave) may remain in flight
    if (k + 1 < nblk && k > 0) __builtin_amdgcn_s_waitcnt(WAIT_VM(WSA_DMA_OPS));   // counted: VM_CNT_ORDER holds
    else __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
    __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
    float bq = 0.0f, iq = 0.0f;
    if constexpr (HQ) {
      float sc;
      scales(k - 2, sc, bq, iq);
      if (lane < 16)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sc), srsrc, 4 * (rbk(k - 2) * R + f), 0, 0);
    }
    float sr = 0.0f;
    if constexpr (HY) sr = sal[(((k - 1) % 3) * 4 + wave) * 64 + f];
    float am = 0.0f;
    float4 s4, b4;
    if constexpr (HY) sw_group(0, 0, s4, b4);
    float tq[4];
    uint32_t d[4];
    // one quantized output o of QB (h, jj, e order: a group's 16 codes stored when complete)
    auto q_out = [&](int o, float yv) {
      const int h = o >> 4, jj = (o >> 2) & 3, e = o & 3;
      tq[e] = q_val(yv, bq, iq);
      if (e == 3) {
        d[jj] = pack4_biased(tq[0], tq[1], tq[2], tq[3]);
        if (jj == 3) store_row(k - 2, h, d);
      }
      return tq[e];
    };
    auto q_in = [&](int o) { return __int_as_float(QB[o >> 2][o & 3]); };
    // one y output o of YB (one sw / bias group per 4 outputs)
    auto y_in = [&](int o) { return __int_as_float(YB[o >> 2][o & 3]); };
    auto y_out = [&](int o, float av) {
      const int jn = o >> 2, e = o & 3;
      if (e == 0 && o > 0) sw_group(jn >> 2, jn & 3, s4, b4);
      const float v = y_val(__float_as_int(av), sr, el(s4, e), el(b4, e));
      am = fmaxf(am, fabsf(v));
      YB[jn][e] = __float_as_int(v);
      return v;
    };
    if constexpr (HM) {
      constexpr int ZL = 3;
      const uint8_t* cur = lds + (k % NS) * STG;
      float qh[ZL], yh[ZL];
#pragma unroll
      for (int z = 0; z < ZL; ++z) qh[z] = yh[z] = 0.0f;
      auto lda = [&](int s) { return *reinterpret_cast<const v4i*>(cur + (s << 10) + lane * 16); };
      v4i an = lda(0);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const v4i a = an;
        if (s < 7) an = lda(s + 1);
        // the quantization (and its stores) in the first half, then block k+2's DMA: at the
        // next top its operations are this wave's youngest (a counted wait is exact)
        if (s == 4 && k + 2 < nblk) issue(k + 2);
#pragma unroll
        for (int jn = 0; jn < 8; ++jn) {
          const int n = s * 8 + jn, o = n & 31;
          if (n < 32 && HQ) {
            float yv = q_in(o);
            if (s == 0) mfma_pin_a<true>(MF[jn], wa[s][jn], a, qh[ZL - 1], yv);
            else mfma_pin_a<false>(MF[jn], wa[s][jn], a, qh[ZL - 1], yv);
#pragma unroll
            for (int z = ZL - 1; z > 0; --z) qh[z] = qh[z - 1];
            qh[0] = q_out(o, yv);
          } else if (n >= 32 && HY) {
            float av = y_in(o);
            if (s == 0) mfma_pin_a<true>(MF[jn], wa[s][jn], a, yh[ZL - 1], av);
            else mfma_pin_a<false>(MF[jn], wa[s][jn], a, yh[ZL - 1], av);
#pragma unroll
            for (int z = ZL - 1; z > 0; --z) yh[z] = yh[z - 1];
            yh[0] = y_out(o, av);
          } else {
            if (s == 0) mfma_asm_a<true>(MF[jn], wa[s][jn], a);
            else mfma_asm_a<false>(MF[jn], wa[s][jn], a);
          }
        }
      }
      mfma_settle8(MF);
    } else {
      if constexpr (HQ) {
#pragma unroll
        for (int o = 0; o < 32; ++o) q_out(o, q_in(o));
      }
      if (k + 2 < nblk) issue(k + 2);
      if constexpr (HY) {
#pragma unroll
        for (int o = 0; o < 32; ++o) y_out(o, y_in(o));
      }
    }
    if constexpr (HY) put_max(k - 1, am);
  };
  const std::true_type T_{};
  const std::false_type F_{};

  v4i B0[8], B1[8], B2[8];
  // roles in iteration k: accumulators B[k % 3], y(k-1) in B[(k-1) % 3], y(k-2) in B[(k-2) % 3];
  // whole groups of three iterations in the loop (one register-role permutation at its exit)
  iter(0, B0, B2, B1, T_, F_, F_);
  if (nblk == 1) {
    iter(1, B1, B0, B2, F_, T_, F_);
    iter(2, B2, B1, B0, F_, F_, T_);
  } else {
    iter(1, B1, B0, B2, T_, T_, F_);
    int k = 2;
    for (; k + 3 <= nblk; k += 3) {
      iter(k, B2, B1, B0, T_, T_, T_);
      iter(k + 1, B0, B2, B1, T_, T_, T_);
      iter(k + 2, B1, B0, B2, T_, T_, T_);
    }
    if (k == nblk) {
      iter(k, B2, B1, B0, F_, T_, T_);
      iter(k + 1, B0, B2, B1, F_, F_, T_);
    } else if (k + 1 == nblk) {
      iter(k, B2, B1, B0, T_, T_, T_);
      iter(k + 1, B0, B2, B1, F_, T_, T_);
      iter(k + 2, B1, B0, B2, F_, F_, T_);
    } else {
      iter(k, B2, B1, B0, T_, T_, T_);
      iter(k + 1, B0, B2, B1, T_, T_, T_);
      iter(k + 2, B1, B0, B2, F_, T_, T_);
      iter(k + 3, B2, B1, B0, F_, F_, T_);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// =====================================================================================
// k_gemm_wsa2<EPI>: the FFN1 passes (RE_RELU_PMAX, then RE_RELU_QUANT_PMAX) on k_gemm_wsa's
// structure — one wave per SIMD, the workgroup's 512-column slice of W1 in the waves'
// AGPRs, 16-row blocks of A by LDS-DMA two blocks ahead — with two register buffers: the
// 64 MFMAs of block k carry the epilogue of block k-1, one output pinned after every
// second MFMA.
//   RE_RELU_PMAX:        y = relu(((acc * sa) * sw) + b) folded into the row's maximum over
//                        the slice (the 4 waves' partials through LDS) -> pmax_out[t][M].
//   RE_RELU_QUANT_PMAX:  the row's maximum over all slices from pmax_in (its pmax_n partials
//                        come by LDS-DMA with the block's A rows), the per-token scale by
//                        true division, y as above quantized by div_cr -> out8 (KP layout),
//                        scales -> os (slice 0).
// No in-launch exchange between workgroups: the two passes replace k_gemm_wsy's granule
// hand-off (and its timeout path) by one more pass over W1's MFMAs.
// =====================================================================================
template <int EPI, int XG = 1>
__global__ __launch_bounds__(256, 1) void k_gemm_wsa2(RowGemmArgs g) {
  static_assert(EPI == RE_RELU_PMAX || EPI == RE_RELU_QUANT_PMAX, "FFN1 passes");
  constexpr bool QP = EPI == RE_RELU_QUANT_PMAX;
  constexpr int NS = 3;
  constexpr int R = 16, STG = R * WS_K;
  constexpr int NPM = QP ? 4 : 0;                            // partial maxima per row (DMA)
  // LDS: 3 A stages (24 KB) | sw, bias (4 KB) | red [2][4][16] | sal / pm [3][1 + NPM][4 waves][64]
  __shared__ __attribute__((aligned(16))) uint8_t lds[NS * STG + 4096 + 2 * 4 * R * 4 + 3 * (1 + NPM) * 4 * 64 * 4];
  float* const swl = reinterpret_cast<float*>(lds + NS * STG);
  float* const red0 = swl + 1024;                            // [2][4][16]
  float* const sal = red0 + 2 * 4 * R;                       // [3][1 + NPM][4 waves][64]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int f = lane & 15, gq = lane >> 4;
  const int nsl = g.N >> 9;
  const int wpt = gridDim.x / nsl;
  int t = blockIdx.x % nsl, r0 = blockIdx.x / nsl;
  if (XG) {
    const int b = blockIdx.x, A = gridDim.x / (8 * nsl), aligned = 8 * nsl * A;
    if (b < aligned) {
      const int j = b >> 3;
      t = j % nsl;
      r0 = 8 * (j / nsl) + (b & 7);
    } else {
      t = (b - aligned) % nsl;
      r0 = 8 * A + (b - aligned) / nsl;
    }
  }
  const int nb = (g.M + R - 1) / R;
  if (r0 >= nb) return;
  const int nblk = (nb - r0 + wpt - 1) / wpt;

  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto dma4 = [](const float* gsrc, const float* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto rbk = [&](int k) { return r0 + min(k, nblk - 1) * wpt; };
  auto slot = [&](int k, int p) { return sal + (((k % 3) * (1 + NPM) + p) * 4 + wave) * 64; };
  constexpr int DMA_OPS = 3 + NPM;
  auto issue = [&](int k) {
    uint8_t* st = lds + (k % NS) * STG;
    const int row = min(rbk(k) * R + f, g.M - 1);
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const int s = 2 * wave + ss;
      dma16(g.A + kp_off(row, 64 * s + 16 * gq, WS_K), st + (s << 10));
    }
    dma4(g.sa + row, slot(k, 0));
#pragma unroll
    for (int p = 0; p < NPM; ++p) dma4(g.pmax_in + (long)min(p, g.pmax_n - 1) * g.M + row, slot(k, 1 + p));
  };
  v4i wa[8][8];
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int jn = 0; jn < 8; ++jn) {
      const int8_t* src = g.W + ((long)(t * 8 + 2 * wave + (jn >> 2)) << 15) + ((s * 4 + (jn & 3)) << 10) + lane * 16;
      wa[s][jn] = *reinterpret_cast<const v4i*>(src);
    }
  {
    const int c = 2 * tid;
    *reinterpret_cast<float2*>(swl + c) = *reinterpret_cast<const float2*>(g.sw + 512 * t + c);
    *reinterpret_cast<float2*>(swl + 512 + c) = *reinterpret_cast<const float2*>(g.bias + 512 * t + c);
  }
  issue(0);
  if (nblk > 1) issue(1);
  auto csh = [&](int h) { return 64 * (2 * wave + h) + 16 * gq; };
  const __amdgpu_buffer_rsrc_t orsrc = ws_rsrc(g.out8, QP ? (long)(g.M + (g.M & 1)) * g.ldo8 : 0L);
  // per-row outputs: QUANT the scales (slice 0 writes them), RELU_PMAX this slice's maxima;
  // the range check drops the rows past M of a ragged last block
  const __amdgpu_buffer_rsrc_t srsrc = QP ? ws_rsrc(g.os, t == 0 ? 4L * g.M : 0L)
                                          : ws_rsrc(g.pmax_out + (long)t * g.M, 4L * g.M);
  auto redb = [&](int k) { return red0 + (k & 1) * 4 * R; };
  auto sw_group = [&](int jn, float4& s4, float4& b4) {
    s4 = *reinterpret_cast<const float4*>(swl + csh(jn >> 2) + 4 * (jn & 3));
    b4 = *reinterpret_cast<const float4*>(swl + 512 + csh(jn >> 2) + 4 * (jn & 3));
  };
  auto el = [](const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; };

  // iteration k: MFMAs of block k (HM) with the epilogue of block k-1 (HE)
  auto iter = [&](int k, v4i (&MF)[8], v4i (&EB)[8], auto hm, auto he) {
    constexpr bool HM = decltype(hm)::value, HE = decltype(he)::value;
    if (k + 1 < nblk && k > 0) __builtin_amdgcn_s_waitcnt(WAIT_VM(DMA_OPS));   // counted: VM_CNT_ORDER holds
    else __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
    __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
    // RELU_PMAX: the slice maximum of block k-2 (its 4 partials complete since the barrier)
    if constexpr (!QP) {
      if (k >= 2 && lane < 16) {
        const float* red = redb(k - 2);
        float m = red[f];
#pragma unroll
        for (int w = 1; w < 4; ++w) m = fmaxf(m, red[w * R + f]);
        if (wave == 0)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(m), srsrc, 4 * (rbk(k - 2) * R + f), 0, 0);
      }
    }
    float sr = 0.0f, bq = 0.0f, iq = 0.0f;
    if constexpr (HE) {
      sr = slot(k - 1, 0)[f];
      if constexpr (QP) {
        float m = slot(k - 1, 1)[f];
#pragma unroll
        for (int p = 1; p < NPM; ++p) m = fmaxf(m, slot(k - 1, 1 + p)[f]);
        bq = fmaxf(m, 1e-5f) / 127.0f;
        iq = 1.0f / bq;
        if (wave == 0 && lane < 16)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bq), srsrc, 4 * (rbk(k - 1) * R + f), 0, 0);
      }
    }
    float am = 0.0f;
    float4 s4, b4;
    if constexpr (HE) sw_group(0, s4, b4);
    float tq[4];
    uint32_t d[4];
    // output o of EB: column fragment jn = o >> 2, element e (one sw / bias group per 4)
    auto e_in = [&](int o) { return __int_as_float(EB[o >> 2][o & 3]); };
    auto e_out = [&](int o, float av) {
      const int jn = o >> 2, e = o & 3;
      if (e == 0 && o > 0) sw_group(jn, s4, b4);
      const float y = fmaxf(((float)__float_as_int(av) * sr) * el(s4, e) + el(b4, e), 0.0f);
      if constexpr (!QP) {
        am = fmaxf(am, y);
        return y;
      } else {
        tq[e] = rint_biased(div_cr(y, bq, iq));
        if (e == 3) {
          d[jn & 3] = pack4_biased(tq[0], tq[1], tq[2], tq[3]);
          if ((jn & 3) == 3) {
            const long row = rbk(k - 1) * R + f;
            __builtin_amdgcn_raw_buffer_store_b128(v4u{d[0], d[1], d[2], d[3]}, orsrc,
                                                   (int)kp_off(row, 512 * t + csh(jn >> 2), g.ldo8), 0, 0);
          }
        }
        return tq[e];
      }
    };
    if constexpr (HM) {
      constexpr int ZL = 2;
      const uint8_t* cur = lds + (k % NS) * STG;
      float eh[ZL];
#pragma unroll
      for (int z = 0; z < ZL; ++z) eh[z] = 0.0f;
      auto lda = [&](int s) { return *reinterpret_cast<const v4i*>(cur + (s << 10) + lane * 16); };
      v4i an = lda(0);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const v4i a = an;
        if (s < 7) an = lda(s + 1);
#pragma unroll
        for (int jn = 0; jn < 8; ++jn) {
          const int n = s * 8 + jn;
          if (HE && (n & 1) == 1 && n < 63) {
            const int o = n >> 1;
            float av = e_in(o);
            if (s == 0) mfma_pin_a<true>(MF[jn], wa[s][jn], a, eh[ZL - 1], av);
            else mfma_pin_a<false>(MF[jn], wa[s][jn], a, eh[ZL - 1], av);
#pragma unroll
            for (int z = ZL - 1; z > 0; --z) eh[z] = eh[z - 1];
            eh[0] = e_out(o, av);
          } else {
            if (s == 0) mfma_asm_a<true>(MF[jn], wa[s][jn], a);
            else mfma_asm_a<false>(MF[jn], wa[s][jn], a);
          }
        }
      }
      mfma_settle8(MF);
      if constexpr (HE) e_out(31, e_in(31));   // the last output after the MFMAs
      // block k+2's DMA after this iteration's last store: at the next top its operations
      // are this wave's youngest, so the counted wait there is exact (VM_CNT_ORDER)
      if (k + 2 < nblk) issue(k + 2);
    } else {
      if constexpr (HE) {
#pragma unroll
        for (int o = 0; o < 32; ++o) e_out(o, e_in(o));
      }
      if (k + 2 < nblk) issue(k + 2);
    }
    if constexpr (HE && !QP) {
      float* red = redb(k - 1);
      am = fmaxf(am, __shfl_xor(am, 16));
      am = fmaxf(am, __shfl_xor(am, 32));
      red[wave * R + f] = am;
    }
  };
  const std::true_type T_{};
  const std::false_type F_{};
  v4i B0[8], B1[8];
  iter(0, B0, B1, T_, F_);
  int k = 1;
  for (; k + 2 <= nblk; k += 2) {
    iter(k, B1, B0, T_, T_);
    iter(k + 1, B0, B1, T_, T_);
  }
  // k odd; nblk - k in {0, 1}
  if (k == nblk) {
    iter(k, B1, B0, F_, T_);
    k += 1;
  } else {
    iter(k, B1, B0, T_, T_);
    iter(k + 1, B0, B1, F_, T_);
    k += 2;
  }
  if constexpr (!QP) {         // the last block's slice maximum (its partials: after a barrier)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (lane < 16 && wave == 0) {
      const float* red = redb(k - 2);
      float m = red[f];
#pragma unroll
      for (int w = 1; w < 4; ++w) m = fmaxf(m, red[w * R + f]);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(m), srsrc, 4 * (rbk(k - 2) * R + f), 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// =====================================================================================
// k_gemm_wss: k_gemm_wsq with the two waves of every SIMD in opposite phases.  Stamps of
// k_gemm_wsq (tools/wsq_stamps.py): the older wave of a SIMD pair (waves 0-3) ends its
// MFMA phase at ~2450 cycles, its y phase at ~3250, then waits ~1400 at the barrier for
// the younger one (waves 4-7), whose MFMAs were starved behind it (~3880 cycles): the
// matrix pipe is busy ~45 % of a block.  Here the groups work in opposite order, so on each
// SIMD one wave's MFMAs run beside the other wave's VALU-only phase.  Between barriers k
// and k+1 (interval k):
//   A (waves 0-3):  M(k);  wait for B's Y(k-1);  Q(k-1);  Y(k)
//   B (waves 4-7):  Y(k-1);  signal;  M(k) with Q(k-1) interleaved between its MFMAs
// M = the block's 64 MFMAs per wave, Y = y of a block from its accumulators + the wave's
// partial row maxima (-> red[j & 1]), Q = quantization of a block with its complete row
// maxima.  red[j & 1] gets A's partials in interval j and B's in interval j + 1 (before
// B signals): an LDS counter that every B wave bumps after its Y (monotonic: 4j after
// interval j's) tells A and the other B waves when block j's maxima are complete.  B keeps
// a block's accumulators across one barrier; each wave holds one y buffer.
// =====================================================================================
__global__ __launch_bounds__(512) void k_gemm_wss(RowGemmArgs g) {
  constexpr int LAG = 1;
  constexpr int SR = WS_SR, WL = 8 * (8 - SR) * 4 * 1024;
  // LDS: 2 A stages (32 KB) | W K steps 5-7 (96 KB) | sw, bias (4 KB) | red [2][8][32] (2 KB)
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WP_STAGE + WL + 4096 + 2 * 8 * WP_R * 4 + 2 * 8 * 64 * 4];
  __shared__ unsigned ydone;                                 // B waves' finished Y phases
  uint8_t* const wl = lds + 2 * WP_STAGE;
  float* const swl = reinterpret_cast<float*>(wl + WL);
  float* const red0 = swl + 1024;                            // [2][8][32]
  float* const sal = red0 + 2 * 8 * WP_R;                    // [2][8 waves][64]: row scales
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int f = lane & 15, gq = lane >> 4;
  const bool grpB = __builtin_amdgcn_readfirstlane(wave) >= 4;
  const int nsl = g.N >> 9;
  const int wpt = gridDim.x / nsl;
  const int t = blockIdx.x % nsl, r0 = blockIdx.x / nsl;
  const int nb = (g.M + WP_R - 1) / WP_R;
  if (r0 >= nb) return;
  const int nblk = (nb - r0 + wpt - 1) / wpt;
  if (tid == 0) ydone = 0u;

  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto rbk = [&](int k) { return r0 + min(k, nblk - 1) * wpt; };
  auto dma4 = [](const float* gsrc, const float* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto issue = [&](int k) {      // block k's A rows and its row scales (as k_gemm_wsq)
    uint8_t* st = lds + (k & 1) * WP_STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long row = min(rbk(k) * WP_R + 16 * i + f, g.M - 1);
      dma16(g.A + kp_off(row, 64 * wave + 16 * gq, WS_K), st + ((wave * 2 + i) << 10));
    }
    dma4(g.sa + min(rbk(k) * WP_R + (lane & 31), g.M - 1), sal + ((k & 1) * 8 + wave) * 64);
  };
  issue(0);
  v4i wr[SR][4];
  {
    const int8_t* wsrc = g.W + ((long)(t * 8 + wave) << 15);
    const v4i* ws = reinterpret_cast<const v4i*>(wsrc) + lane;
#pragma unroll
    for (int s = 0; s < SR; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) wr[s][j] = ws[(s * 4 + j) * 64];
#pragma unroll
    for (int p = 0; p < (8 - SR) * 4; ++p)
      dma16(wsrc + ((SR * 4 + p) << 10) + lane * 16, wl + ((wave * (8 - SR) * 4 + p) << 10));
    if (wave < 4) {
      const int c = 128 * wave + 2 * lane;
      *reinterpret_cast<float2*>(swl + c) = *reinterpret_cast<const float2*>(g.sw + 512 * t + c);
      *reinterpret_cast<float2*>(swl + 512 + c) = *reinterpret_cast<const float2*>(g.bias + 512 * t + c);
    }
#pragma unroll
    for (int s = 0; s < SR; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(wr[s][j]));
  }
  const int cs = 64 * wave + 16 * gq;
  const __amdgpu_buffer_rsrc_t orsrc = ws_rsrc(g.out8 + (long)t * g.o8_ts, (long)g.M * g.ldo8);
  const __amdgpu_buffer_rsrc_t srsrc = ws_rsrc(g.os + (long)t * g.os_ts, 4L * g.M);
  auto redb = [&](int k) { return red0 + (k & 1) * 8 * WP_R; };
  auto sr_of = [&](int k, float (&sr)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) sr[i] = sal[((k & 1) * 8 + wave) * 64 + 16 * i + f];
  };
  auto top_wait = [&]() {
    __builtin_amdgcn_s_waitcnt(WAIT_VM(0));      // the block's DMA and the stores after it (VM_CNT_ORDER)
    __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
  };
  auto dummy_stores = [&]() {
    const __amdgpu_buffer_rsrc_t nul = ws_rsrc(g.out8, 0L);
#pragma unroll
    for (int d2 = 0; d2 < 3; ++d2) __builtin_amdgcn_raw_buffer_store_b32(0u, nul, 0, 0, 0);
  };
  // B's Y phases of blocks < j all done and visible (bounded: never hang)
  auto wait_y = [&](int j) {
#pragma unroll 1
    for (unsigned spin = 0; spin < (1u << 20); ++spin) {
      if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&ydone, __ATOMIC_ACQUIRE,
                                                           __HIP_MEMORY_SCOPE_WORKGROUP)) >= 4u * j)
        break;
      __builtin_amdgcn_s_sleep(1);
    }
  };
  // Y: y of block k from acc (row scale sa) and the wave's partial row maxima -> red[k & 1]
  auto form_y = [&](v4i (&acc)[2][4], const float (&sr_in)[2], float (&y)[2][16], int k) {
    float sr[2];     // B: read at the top of its iteration, before the DMA reuses the stage
#pragma unroll
    for (int i = 0; i < 2; ++i) sr[i] = sr_in[i];
    float am[2] = {0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 s4 = *reinterpret_cast<const float4*>(swl + cs + 4 * j);
      const float4 b4 = *reinterpret_cast<const float4*>(swl + 512 + cs + 4 * j);
      const float swj[4] = {s4.x, s4.y, s4.z, s4.w}, bj[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          y[i][4 * j + e] = ((float)acc[i][j][e] * sr[i]) * swj[e] + bj[e];
          am[i] = fmaxf(am[i], fabsf(y[i][4 * j + e]));
        }
    }
    float* red = redb(k);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float a = am[i];
      a = fmaxf(a, __shfl_xor(a, 16));
      a = fmaxf(a, __shfl_xor(a, 32));
      red[wave * WP_R + 16 * i + f] = a;
    }
  };
  auto scales = [&](int k, float (&bq)[2], float (&iq)[2]) {
    const float* red = redb(k);
    float m = red[lane & 31];
#pragma unroll
    for (int w = 1; w < 8; ++w) m = fmaxf(m, red[w * WP_R + (lane & 31)]);
    const float sc = fmaxf(m, 1e-5f) / 127.0f;
    const float inv = 1.0f / sc;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sc), srsrc, 4 * (rbk(k) * WP_R + (lane & 31)), 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bq[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (16 * i + f), __float_as_int(sc)));
      iq[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (16 * i + f), __float_as_int(inv)));
    }
  };
  auto store_row = [&](int k, int i, const uint32_t (&d)[4]) {
    const long row = rbk(k) * WP_R + 16 * i + f;
    __builtin_amdgcn_raw_buffer_store_b128(v4u{d[0], d[1], d[2], d[3]}, orsrc, (int)(row * g.ldo8 + cs), 0, 0);
  };
  auto quant_all = [&](int k, const float (&y)[2][16]) {      // 3 stores
    float bq[2], iq[2];
    scales(k, bq, iq);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        d[j] = pack4_biased(rint_biased(div_cr(y[i][4 * j], bq[i], iq[i])),
                            rint_biased(div_cr(y[i][4 * j + 1], bq[i], iq[i])),
                            rint_biased(div_cr(y[i][4 * j + 2], bq[i], iq[i])),
                            rint_biased(div_cr(y[i][4 * j + 3], bq[i], iq[i])));
      store_row(k, i, d);
    }
  };
  // M(k) into acc; Q: with Q(kq) of y between the MFMAs (pinned), 3 stores; else plain
  auto mfma_block = [&](v4i (&acc)[2][4], int k, auto q_c, int kq, float (&y)[2][16]) {
    constexpr bool Q = decltype(q_c)::value;
    const uint8_t* cur = lds + (k & 1) * WP_STAGE;
    float bq[2] = {0.0f, 0.0f}, iq[2] = {0.0f, 0.0f};
    if constexpr (Q) scales(kq, bq, iq);
    float hist[3] = {0.0f, 0.0f, 0.0f}, tq[4];   // results of the last outputs, newest first
    uint32_t d[4];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      v4i a[2], b[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const v4i*>(cur + ((s * 2 + i) << 10) + lane * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = s < SR ? wr[s < SR ? s : 0][j]
                      : *reinterpret_cast<const v4i*>(wl + (((wave * (8 - SR) + s - SR) * 4 + j) << 10) + lane * 16);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = s * 8 + i * 4 + j;
          if (!Q || (n & 1) == 0) {
            if (s == 0) mfma_asm<true>(acc[i][j], b[j], a[i]);
            else mfma_asm<false>(acc[i][j], b[j], a[i]);
          } else {
            const int o = n >> 1, ii = o >> 4, jj = (o >> 2) & 3, e = o & 3;
            float yv = y[ii][4 * jj + e];
            if (s == 0) mfma_pin<true>(acc[i][j], b[j], a[i], hist[LAG - 1], yv);
            else mfma_pin<false>(acc[i][j], b[j], a[i], hist[LAG - 1], yv);
            tq[e] = rint_biased(div_cr(yv, bq[ii], iq[ii]));
            hist[2] = hist[1]; hist[1] = hist[0]; hist[0] = tq[e];
            if (e == 3) {
              d[jj] = pack4_biased(tq[0], tq[1], tq[2], tq[3]);
              if (jj == 3) store_row(kq, ii, d);
            }
          }
        }
    }
    mfma_settle(acc);
  };
  const std::true_type T_{};
  const std::false_type F_{};

  __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
  __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
  __builtin_amdgcn_s_barrier();
  // one loop per group (the same iterations and barriers): a loop shared by both would carry
  // the union of their loop-carried values (A: y, B: acc) and spill — and a spill reload's
  // wait is vmcnt(0), which also waits for the next block's DMA and every store
  if (!grpB) {
    v4i acc[2][4];
    float y[2][16];
    for (int k = 0; k <= nblk; ++k) {
      if (k > 0) top_wait();
      if (k + 1 < nblk) issue(k + 1);
      if (k < nblk) mfma_block(acc, k, F_, 0, y);
      if (k >= 1) {
        wait_y(k);                          // B's partial maxima of block k-1
        quant_all(k - 1, y);
      } else {
        dummy_stores();
      }
      if (k < nblk) {
        float sr[2];
        sr_of(k, sr);
        form_y(acc, sr, y, k);
      }
    }
  } else {
    v4i acc[2][4];
    float y[2][16];
    for (int k = 0; k <= nblk; ++k) {
      if (k > 0) top_wait();
      float sr[2];
      if (k >= 1) {                         // block k-1's scales, before DMA(k+1) reuses the stage
        sr_of(k - 1, sr);
        __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
      }
      if (k + 1 < nblk) issue(k + 1);
      if (k >= 1) {
        form_y(acc, sr, y, k - 1);
        if (lane == 0) __hip_atomic_fetch_add(&ydone, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        wait_y(k);                          // every B wave's partials of block k-1
      }
      if (k < nblk) {
        if (k >= 1) mfma_block(acc, k, T_, k - 1, y);
        else {
          mfma_block(acc, k, F_, 0, y);
          dummy_stores();
        }
      } else {
        quant_all(k - 1, y);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// =====================================================================================
// k_gemm_wsx: FFN1 (N = 2048, K = 512) in ONE pass — ReLU + per-token quantization of the
// hidden over all 2048 columns, without the row-max pre-pass (position_feed_forward.py:12,
// quant_linear.py:30-43).  The 4 workgroups holding the 4 512-column slices of a row group
// (one XCD under round-robin placement — speed only) exchange their partial row maxima
// inside the launch: for each 32-row block a workgroup publishes its slice's row maxima as
// data-tagged 8-byte granules {tag, value} (one write-through sc1 store each, the
// MI355X_MICROARCH.md R2 hand-off: no flag, no fence) and reads the other three slices'
// granules with sc1 loads.  The software pipeline is one block deeper than k_gemm_wsp:
// iteration k issues block k's MFMAs, forms y and the slice maxima of block k-1 (published
// at the end of the iteration) and quantizes block k-2, whose partner maxima were published
// an iteration earlier — the hand-off latency hides under a whole iteration.
// Work is assigned by arrival ticket (below), so a row group only waits for partners that
// have started or will start once other groups finish: no co-residency assumption, safe
// beside any other launch.  Every spin is still bounded (g.spin_limit polls): a wait that
// times out sets DEV_E_EXCHANGE_TIMEOUT in *g.status, which the host turns into an error
// (qtx_model_check / the next model call; qtx_linear_rows callers read the word) — a block
// quantized from a partial maximum is never silent.
// The granule array (4 x 32 x ceil(M/32) u64 + the ticket counter + the status word, in
// g.pmax_out) is zeroed before every launch.
// =====================================================================================
__global__ __launch_bounds__(512) void k_gemm_wsx(RowGemmArgs g) {
  constexpr int SR = WS_SR, WL = 8 * (8 - SR) * 4 * 1024;
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WP_STAGE + WL + 4096 + 8 * WP_R * 4];
  uint8_t* const wl = lds + 2 * WP_STAGE;
  float* const swl = reinterpret_cast<float*>(wl + WL);    // [512] sw, then [512] bias
  float* const red = swl + 1024;                            // [8][32]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int f = lane & 15, gq = lane >> 4;
  // Work by arrival ticket, not blockIdx: the started workgroups always hold the lowest
  // tickets, so groups whose 4 tickets have all started run to completion and free their
  // CUs, whatever else shares the GPU (another launch of this kernel included): no
  // co-residency assumption, no deadlock.  The ticket counter follows the granules.
  const int nb = (g.M + WP_R - 1) / WP_R;
  unsigned long long* const gran = reinterpret_cast<unsigned long long*>(g.pmax_out);
  __shared__ int ticket;
  if (tid == 0)
    ticket = (int)atomicAdd(reinterpret_cast<unsigned*>(gran + 4L * 32 * nb), 1u);
  __syncthreads();
  // slices of a row group at tickets 8 apart: workgroups start about in blockIdx order and
  // are dealt round-robin to the 8 XCDs, so the 4 partners mostly share an XCD (speed only);
  // a group is complete once its highest ticket has started (any 25 started tickets hold one)
  const int q = ticket, wpt = gridDim.x >> 2;
  const int t = (q >> 3) & 3, r0 = (q & 7) + 8 * (q >> 5);
  if (r0 >= nb) return;                         // the whole row group (all 4 slices) skips
  const int nblk = (nb - r0 + wpt - 1) / wpt;

  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto rbk = [&](int k) { return r0 + min(k, nblk - 1) * wpt; };
  auto issue = [&](int k) {
    uint8_t* st = lds + (k & 1) * WP_STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long row = min(rbk(k) * WP_R + 16 * i + f, g.M - 1);
      dma16(g.A + kp_off(row, 64 * wave + 16 * gq, WS_K), st + ((wave * 2 + i) << 10));
    }
  };
  issue(0);
  v4i wr[SR][4];
  {
    const int8_t* wsrc = g.W + ((long)(t * 8 + wave) << 15);
#pragma unroll
    for (int p = 0; p < (8 - SR) * 4; ++p)
      dma16(wsrc + ((SR * 4 + p) << 10) + lane * 16, wl + ((wave * (8 - SR) * 4 + p) << 10));
    const v4i* ws = reinterpret_cast<const v4i*>(wsrc) + lane;
#pragma unroll
    for (int s = 0; s < SR; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) wr[s][j] = ws[(s * 4 + j) * 64];
    if (wave < 4) {
      const int c = 128 * wave + 2 * lane;
      *reinterpret_cast<float2*>(swl + c) = *reinterpret_cast<const float2*>(g.sw + 512 * t + c);
      *reinterpret_cast<float2*>(swl + 512 + c) = *reinterpret_cast<const float2*>(g.bias + 512 * t + c);
    }
#pragma unroll
    for (int s = 0; s < SR; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(wr[s][j]));
  }
  const int cs = 64 * wave + 16 * gq;
  const int c0 = 512 * t + cs;
  const __amdgpu_buffer_rsrc_t orsrc = ws_rsrc(g.out8, (long)(g.M + (g.M & 1)) * g.ldo8);
  const __amdgpu_buffer_rsrc_t srsrc = ws_rsrc(g.os, t == 0 ? 4L * g.M : 0L);

  auto mfma_steps = [&](v4i (&acc)[2][4], const uint8_t* cur, int s0, int s1) {
#pragma unroll
    for (int s = s0; s < s1; ++s) {
      v4i a[2], b[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const v4i*>(cur + ((s * 2 + i) << 10) + lane * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = s < SR ? wr[s < SR ? s : 0][j]
                      : *reinterpret_cast<const v4i*>(wl + (((wave * (8 - SR) + s - SR) * 4 + j) << 10) + lane * 16);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[j], a[i], acc[i][j], 0, 0, 0);
    }
  };
  // y = relu(((acc * sa) * sw) + b) of a block, and the wave's partial row maxima into red
  auto form_y = [&](const v4i (&acc)[2][4], float sa, float (&y)[2][16]) {
    float sr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      sr[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (16 * i + f), __float_as_int(sa)));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 s4 = *reinterpret_cast<const float4*>(swl + cs + 4 * j);
      const float4 b4 = *reinterpret_cast<const float4*>(swl + 512 + cs + 4 * j);
      const float swj[4] = {s4.x, s4.y, s4.z, s4.w}, bj[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          y[i][4 * j + e] = fmaxf(((float)acc[i][j][e] * sr[i]) * swj[e] + bj[e], 0.0f);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float a = y[i][0];
#pragma unroll
      for (int c = 1; c < 16; ++c) a = fmaxf(a, y[i][c]);
      a = fmaxf(a, __shfl_xor(a, 16));
      a = fmaxf(a, __shfl_xor(a, 32));
      red[wave * WP_R + 16 * i + f] = a;
    }
  };
  // the slice's row maximum of row (lane & 31) over its 8 waves (after a barrier)
  auto slice_max = [&]() {
    float m = red[lane & 31];
#pragma unroll
    for (int w = 1; w < 8; ++w) m = fmaxf(m, red[w * WP_R + (lane & 31)]);
    return m;
  };
  auto gidx = [&](int rb, int tt) { return ((long)rb * 4 + tt) * 32 + (lane & 31); };
  auto publish = [&](int k, float m) {
    if (wave == 0 && lane < 32)
      __hip_atomic_store(gran + gidx(rbk(k), t), (1ull << 32) | __float_as_uint(m),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // the row maximum over all 4 slices: this slice's, then the partners' granules (bounded)
  const unsigned lim = (unsigned)g.spin_limit;
  auto full_max = [&](int k, float mloc) {
    const int rb = rbk(k);
    float m = mloc;
    for (unsigned spin = 0;; ++spin) {
      bool ok = true;
      float mx = mloc;
#pragma unroll
      for (int d = 1; d < 4; ++d) {
        const unsigned long long v = __hip_atomic_load(gran + gidx(rb, (t + d) & 3), __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        ok &= (v >> 32) == 1ull;
        mx = fmaxf(mx, __uint_as_float((unsigned)v));
      }
      if (__all(ok)) { m = mx; break; }
      if (spin >= lim) {                            // bounded: never hang, never silent
        if (lane == 0)
          __hip_atomic_fetch_or(g.status, DEV_E_EXCHANGE_TIMEOUT, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    return m;
  };
  auto quant_store = [&](int k, const float (&y)[2][16], float m) {
    const int m0 = rbk(k) * WP_R;
    const float sc = fmaxf(m, 1e-5f) / 127.0f;   // true division: branch-free (see k_gemm_wsp)
    const float kk = m < 0x1p37f ? 1.0f : 0x1p-64f;
    const float scs = sc * kk, invs = 1.0f / scs;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sc), srsrc, 4 * (m0 + (lane & 31)), 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int src = 4 * (16 * i + f);
      const float b = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(scs)));
      const float yi = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(invs)));
      const float k2 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(kk)));
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        d[j] = pack4_biased(rint_biased(div_cr(y[i][4 * j] * k2, b, yi)),
                            rint_biased(div_cr(y[i][4 * j + 1] * k2, b, yi)),
                            rint_biased(div_cr(y[i][4 * j + 2] * k2, b, yi)),
                            rint_biased(div_cr(y[i][4 * j + 3] * k2, b, yi)));
      const long row = m0 + 16 * i + f;
      __builtin_amdgcn_raw_buffer_store_b128(v4u{d[0], d[1], d[2], d[3]}, orsrc, (int)kp_off(row, c0, g.ldo8), 0, 0);
    }
  };
  auto zero = [](v4i (&acc)[2][4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  };
  auto sa_of = [&](int k) { return g.sa[min(rbk(k) * WP_R + (lane & 31), g.M - 1)]; };

  // ---- block 0: main loop only
  v4i accp[2][4];
  float yq[2][16];                  // y of the block waiting for its partners' maxima
  float mq = 0.0f;                  // ... and its own slice maximum
  __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
  __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
  __builtin_amdgcn_s_barrier();
  float sap = sa_of(0);
  issue(1);
  zero(accp);
  mfma_steps(accp, lds, 0, 8);
  __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
  // ---- steady state: iteration k: MFMAs of block k, y + maxima of block k-1 (published),
  // quantization of block k-2
  for (int k = 1; k <= nblk; ++k) {
    // block k's DMA retired, and the previous iteration's stores (3 per wave, plus wave 0's
    // granule store) with it: VM_CNT_ORDER (qtx_common.h) — a store issued after the DMA
    // may retire before it, so vmcnt(3) could release the barrier with the DMA in flight
    __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
    __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
    const bool more = k < nblk;     // block k exists (uniform)
    asm volatile("" ::"v"(sap));
    float sac = more ? sa_of(k) : 0.0f;
    if (more) issue(k + 1);
    const uint8_t* cur = lds + (k & 1) * WP_STAGE;
    v4i acc[2][4];
    zero(acc);
    float y[2][16];
    if (more) mfma_steps(acc, cur, 0, 4);
    form_y(accp, sap, y);           // block k-1
    __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
    const float mloc = slice_max(); // block k-1's slice maximum (red complete)
    float m2 = 0.0f;
    if (k >= 2) m2 = full_max(k - 2, mq);
    if (more) mfma_steps(acc, cur, 4, 8);
    if (k >= 2) {
      quant_store(k - 2, yq, m2);
    } else {                        // the 3 stores the next top wait counts (range 0: dropped)
      const __amdgpu_buffer_rsrc_t nul = ws_rsrc(g.out8, 0L);
#pragma unroll
      for (int d = 0; d < 3; ++d) __builtin_amdgcn_raw_buffer_store_b32(0u, nul, 0, 0, 0);
    }
    publish(k - 1, mloc);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) accp[i][j] = acc[i][j];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int c = 0; c < 16; ++c) yq[i][c] = y[i][c];
    mq = mloc;
    sap = sac;
  }
  // ---- the last block: its partners' maxima, then its quantization
  quant_store(nblk - 1, yq, full_max(nblk - 1, mq));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The same statements for v_mfma_i32_32x32x32_i8 (k_gemm_wsq32, this file): 16 accumulators per lane,
// 16 passes, so the settle pad is 24 wait states.
template <bool Z, typename T>
__device__ __forceinline__ void mfma32_pin(v16i& acc, const v4i& w, const v4i& a, float before, T& after) {
  if constexpr (Z)
    asm volatile("v_mfma_i32_32x32x32_i8 %0, %2, %3, 0" : "=&v"(acc), "+v"(after) : "v"(w), "v"(a), "v"(before));
  else
    asm volatile("v_mfma_i32_32x32x32_i8 %0, %2, %3, %0" : "+v"(acc), "+v"(after) : "v"(w), "v"(a), "v"(before));
}
template <bool Z>
__device__ __forceinline__ void mfma32_asm(v16i& acc, const v4i& w, const v4i& a) {
  if constexpr (Z)
    asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %2, 0" : "=&v"(acc) : "v"(w), "v"(a));
  else
    asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %2, %0" : "+v"(acc) : "v"(w), "v"(a));
}
__device__ __forceinline__ void mfma32_settle(v16i (&acc)[2]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(acc[0]), "+v"(acc[1]));
}

// =====================================================================================
// k_gemm_wsq32: k_gemm_wsq on v_mfma_i32_32x32x32_i8.  The round-4 fill probe
// (profiles/r04_mfma_fill_probe.log) measured ~4 VALU per 32x32x32 MFMA riding free beside
// two waves per SIMD and ~3.5 cycles per further one (16x16x64: ~2 free, ~4.3 each), so the
// same epilogue per MAC prices ~15 % lower; one output per MFMA is pinned between them.
// Tile: C^T = W . A^T per wave: 2 feature tiles of 32 (u) x 32 tokens, 16 K steps of 32 B.
// The W rows are permuted at pack time (k_pack_w_ws32) so that lane l's 16 accumulators of
// tile u are 16 CONSECUTIVE output columns 64w + 32u + 16 (l >> 5) .. + 15 of token
// l & 31: one 16-byte store per tile, one row scale per lane (no broadcast), and a token's
// partial max over the wave's 64 columns in one cross-lane step (lanes l, l ^ 32).
// Layouts (K = 512):
//   W  "WS32": slice t, wave w, K step s (32 B), tile u: 1 KB in MFMA operand order, lane l
//      = W[n][32s + 16(l >> 5) .. + 16] with n = 512t + 64w + 32u + phi(l & 31),
//      phi(r) = 16 ((r >> 2) & 1) + 4 (r >> 3) + (r & 3)  (D row r of the 32x32 result).
//   LDS A piece s (1 KB): lane l = token l & 31, bytes 32s + 16 (l >> 5) .. + 16.
// Numerics, barriers, DMA and store counts: k_gemm_wsq's.
// Measured (round 5, tools/ws32_ab.py, three alternated rounds in one process): Q/K/V
// 39.7 us against k_gemm_wsq's 39.4, with all of W in registers (SR = 16) 38.4; the
// one-pass FFN1 on k_gemm_wsy32 64.5-72.9 against 58.7-69.2 us; the cfg3 encoder the same
// within noise (1.661-1.681 vs 1.660-1.672 ms).  Diagnostic build only.
// =====================================================================================
constexpr int W32_SR = 10;                       // K steps (of 16) of W in registers
template <int XG = 1, int SR = W32_SR>   // SR: K steps of W in registers (16: all of W)
__global__ __launch_bounds__(512) void k_gemm_wsq32(RowGemmArgs g) {
  constexpr int WL = 8 * (16 - SR) * 2 * 1024 + 16;  // W's LDS part: 96 KB at SR = 10
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WP_STAGE + WL + 4096 + 2 * 8 * WP_R * 4 + 2 * 8 * 64 * 4];
  uint8_t* const wl = lds + 2 * WP_STAGE;
  float* const swl = reinterpret_cast<float*>(wl + WL);
  float* const red0 = swl + 1024;                            // [2][8][32]
  float* const sal = red0 + 2 * 8 * WP_R;                    // [2][8 waves][64]: row scales
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tok = lane & 31, hh = lane >> 5;
  const int nsl = g.N >> 9;
  const int wpt = gridDim.x / nsl;
  int t = blockIdx.x % nsl, r0 = blockIdx.x / nsl;
  if (XG) {
    const int b = blockIdx.x, A = gridDim.x / (8 * nsl), aligned = 8 * nsl * A;
    if (b < aligned) {
      const int j = b >> 3;
      t = j % nsl;
      r0 = 8 * (j / nsl) + (b & 7);
    } else {
      t = (b - aligned) % nsl;
      r0 = 8 * A + (b - aligned) / nsl;
    }
  }
  const int nb = (g.M + WP_R - 1) / WP_R;
  if (r0 >= nb) return;
  const int nblk = (nb - r0 + wpt - 1) / wpt;

  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto dma4 = [](const float* gsrc, const float* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto rbk = [&](int k) { return r0 + min(k, nblk - 1) * wpt; };
  // block k: wave w brings A pieces 2w, 2w + 1 and (as k_gemm_wsq) its copy of the 32 row scales
  auto issue = [&](int k) {
    uint8_t* st = lds + (k & 1) * WP_STAGE;
    const long row = min(rbk(k) * WP_R + tok, g.M - 1);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int s = 2 * wave + i;
      dma16(g.A + kp_off(row, 32 * s + 16 * hh, WS_K), st + (s << 10));
    }
    dma4(g.sa + min(rbk(k) * WP_R + tok, g.M - 1), sal + ((k & 1) * 8 + wave) * 64);
  };
  issue(0);
  v4i wr[SR][2];
  {
    const int8_t* wsrc = g.W + ((long)(t * 8 + wave) << 15);
    const v4i* ws = reinterpret_cast<const v4i*>(wsrc) + lane;
#pragma unroll
    for (int s = 0; s < SR; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) wr[s][u] = ws[(s * 2 + u) * 64];
#pragma unroll
    for (int p = 0; p < (16 - SR) * 2; ++p)
      dma16(wsrc + ((SR * 2 + p) << 10) + lane * 16, wl + ((wave * (16 - SR) * 2 + p) << 10));
    if (wave < 4) {
      const int c = 128 * wave + 2 * lane;
      *reinterpret_cast<float2*>(swl + c) = *reinterpret_cast<const float2*>(g.sw + 512 * t + c);
      *reinterpret_cast<float2*>(swl + 512 + c) = *reinterpret_cast<const float2*>(g.bias + 512 * t + c);
    }
#pragma unroll
    for (int s = 0; s < SR; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) asm volatile("" ::"v"(wr[s][u]));
  }
  const __amdgpu_buffer_rsrc_t orsrc = ws_rsrc(g.out8 + (long)t * g.o8_ts, (long)g.M * g.ldo8);
  const __amdgpu_buffer_rsrc_t srsrc = ws_rsrc(g.os + (long)t * g.os_ts, 4L * g.M);
  auto redb = [&](int k) { return red0 + (k & 1) * 8 * WP_R; };
  auto top_wait = [&]() {
    __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
    __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
  };
  // y of block k and the wave's partial row maxima into red[k & 1]; lane: token tok,
  // columns 64 wave + 32 u + 16 hh + r
  auto form_y = [&](v16i (&acc)[2], float (&y)[2][16], int k) {
    const float sr = sal[((k & 1) * 8 + wave) * 64 + lane];
    float am = 0.0f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 64 * wave + 32 * u + 16 * hh + 4 * q;
        const float4 s4 = *reinterpret_cast<const float4*>(swl + c);
        const float4 b4 = *reinterpret_cast<const float4*>(swl + 512 + c);
        const float swq[4] = {s4.x, s4.y, s4.z, s4.w}, bq4[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          y[u][4 * q + e] = ((float)acc[u][4 * q + e] * sr) * swq[e] + bq4[e];
          am = fmaxf(am, fabsf(y[u][4 * q + e]));
        }
      }
    am = fmaxf(am, __shfl_xor(am, 32));
    if (lane < 32) redb(k)[wave * WP_R + lane] = am;
  };
  // the scale of block k's rows: lane's token only (no broadcast needed)
  auto scales = [&](int k, float& bq, float& iq) {
    const float* red = redb(k);
    float m = red[tok];
#pragma unroll
    for (int w = 1; w < 8; ++w) m = fmaxf(m, red[w * WP_R + tok]);
    bq = scale127(fmaxf(m, 1e-5f));
    iq = rcp_cr(bq);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bq), srsrc, 4 * (rbk(k) * WP_R + tok), 0, 0);
  };
  auto store_tile = [&](int k, int u, const uint32_t (&d)[4]) {
    const long row = rbk(k) * WP_R + tok;
    __builtin_amdgcn_raw_buffer_store_b128(v4u{d[0], d[1], d[2], d[3]}, orsrc,
                                           (int)(row * g.ldo8 + 64 * wave + 32 * u + 16 * hh), 0, 0);
  };
  // the 32 MFMAs of block k into acc; with q: block k-1's 32 quantized outputs, one pinned
  // after each MFMA
  auto mfma_block = [&](v16i (&acc)[2], const uint8_t* cur, bool q, int kq, float (&y)[2][16]) {
    float bq = 0.0f, iq = 0.0f;
    if (q) scales(kq, bq, iq);
    float hist = 0.0f, tq[4];
    uint32_t d[4];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const v4i x = *reinterpret_cast<const v4i*>(cur + (s << 10) + lane * 16);
      v4i w[2];
#pragma unroll
      for (int u = 0; u < 2; ++u)
        w[u] = s < SR ? wr[s < SR ? s : 0][u]
                          : *reinterpret_cast<const v4i*>(wl + (((wave * (16 - SR) + s - SR) * 2 + u) << 10) + lane * 16);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (!q) {
          if (s == 0) mfma32_asm<true>(acc[u], w[u], x);
          else mfma32_asm<false>(acc[u], w[u], x);
        } else {
          const int o = 2 * s + u, uo = o >> 4, r = o & 15;
          float yv = y[uo][r];
          if (s == 0) mfma32_pin<true>(acc[u], w[u], x, hist, yv);
          else mfma32_pin<false>(acc[u], w[u], x, hist, yv);
          tq[r & 3] = rint_biased(div_cr(yv, bq, iq));
          hist = tq[r & 3];
          if ((r & 3) == 3) {
            d[r >> 2] = pack4_biased(tq[0], tq[1], tq[2], tq[3]);
            if (r == 15) store_tile(kq, uo, d);
          }
        }
      }
    }
    mfma32_settle(acc);
    if (!q) {           // the 3 stores per iteration of the q path (dropped)
      const __amdgpu_buffer_rsrc_t nul = ws_rsrc(g.out8, 0L);
#pragma unroll
      for (int d2 = 0; d2 < 3; ++d2) __builtin_amdgcn_raw_buffer_store_b32(0u, nul, 0, 0, 0);
    }
  };

  v16i acc[2];
  float y[2][16];
  __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
  __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
  __builtin_amdgcn_s_barrier();
  issue(1);
  mfma_block(acc, lds, false, 0, y);
  form_y(acc, y, 0);
  for (int k = 1; k < nblk; ++k) {
    top_wait();
    issue(k + 1);
    mfma_block(acc, lds + (k & 1) * WP_STAGE, true, k - 1, y);
    form_y(acc, y, k);
  }
  top_wait();
  {
    float bq, iq;
    scales(nblk - 1, bq, iq);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        d[j] = pack4_biased(rint_biased(div_cr(y[u][4 * j], bq, iq)),
                            rint_biased(div_cr(y[u][4 * j + 1], bq, iq)),
                            rint_biased(div_cr(y[u][4 * j + 2], bq, iq)),
                            rint_biased(div_cr(y[u][4 * j + 3], bq, iq)));
      store_tile(nblk - 1, u, d);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// =====================================================================================
// k_gemm_wsy32: k_gemm_wsy on v_mfma_i32_32x32x32_i8 (W in the WS32 layout, k_gemm_wsq32's
// tile: lane l = token l & 31 x 16 consecutive columns 64w + 32u + 16 (l >> 5) per tile u).
// Tickets, granules, the bounded partner waits, wave 0's gather and the two-parity y
// buffers are k_gemm_wsy's; the hidden is written KP as there.
// =====================================================================================
__global__ __launch_bounds__(512) void k_gemm_wsy32(RowGemmArgs g) {
  constexpr int WL = 8 * (16 - W32_SR) * 2 * 1024;
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WP_STAGE + WL + 4096 + 2 * 8 * WP_R * 4 + 2 * 8 * 64 * 4 +
                                                      2 * 2 * WP_R * 4];
  uint8_t* const wl = lds + 2 * WP_STAGE;
  float* const swl = reinterpret_cast<float*>(wl + WL);
  float* const red0 = swl + 1024;                            // [2][8][32]
  float* const sal = red0 + 2 * 8 * WP_R;                    // [2][8 waves][64]: row scales
  float* const gsc = sal + 2 * 8 * 64;                       // [2][2][32]: s and RN(1/s)
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tok = lane & 31, hh = lane >> 5;
  const int nb = (g.M + WP_R - 1) / WP_R;
  unsigned long long* const gran = reinterpret_cast<unsigned long long*>(g.pmax_out);
  __shared__ int ticket;
  if (tid == 0)
    ticket = (int)atomicAdd(reinterpret_cast<unsigned*>(gran + 4L * 32 * nb), 1u);
  __syncthreads();
  const int q = ticket, wpt = gridDim.x >> 2;       // tickets as in k_gemm_wsx
  const int t = (q >> 3) & 3, r0 = (q & 7) + 8 * (q >> 5);
  if (r0 >= nb) return;
  const int nblk = (nb - r0 + wpt - 1) / wpt;

  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto rbk = [&](int k) { return r0 + min(k, nblk - 1) * wpt; };
  auto dma4 = [](const float* gsrc, const float* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto issue = [&](int k) {      // block k's A pieces 2w, 2w + 1 and its row scales
    uint8_t* st = lds + (k & 1) * WP_STAGE;
    const long row = min(rbk(k) * WP_R + tok, g.M - 1);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int s = 2 * wave + i;
      dma16(g.A + kp_off(row, 32 * s + 16 * hh, WS_K), st + (s << 10));
    }
    dma4(g.sa + min(rbk(k) * WP_R + tok, g.M - 1), sal + ((k & 1) * 8 + wave) * 64);
  };
  issue(0);
  v4i wr[W32_SR][2];
  {
    const int8_t* wsrc = g.W + ((long)(t * 8 + wave) << 15);
    const v4i* ws = reinterpret_cast<const v4i*>(wsrc) + lane;
#pragma unroll
    for (int s = 0; s < W32_SR; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) wr[s][u] = ws[(s * 2 + u) * 64];
#pragma unroll
    for (int p = 0; p < (16 - W32_SR) * 2; ++p)
      dma16(wsrc + ((W32_SR * 2 + p) << 10) + lane * 16, wl + ((wave * (16 - W32_SR) * 2 + p) << 10));
    if (wave < 4) {
      const int c = 128 * wave + 2 * lane;
      *reinterpret_cast<float2*>(swl + c) = *reinterpret_cast<const float2*>(g.sw + 512 * t + c);
      *reinterpret_cast<float2*>(swl + 512 + c) = *reinterpret_cast<const float2*>(g.bias + 512 * t + c);
    }
#pragma unroll
    for (int s = 0; s < W32_SR; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) asm volatile("" ::"v"(wr[s][u]));
  }
  const int c0 = 512 * t + 64 * wave + 16 * hh;   // + 32 u: the lane's first column of tile u
  const __amdgpu_buffer_rsrc_t orsrc = ws_rsrc(g.out8, (long)(g.M + (g.M & 1)) * g.ldo8);
  const __amdgpu_buffer_rsrc_t srsrc = ws_rsrc(g.os, t == 0 ? 4L * g.M : 0L);
  auto redb = [&](int k) { return red0 + (k & 1) * 8 * WP_R; };
  auto dummy_stores = [&]() {
    const __amdgpu_buffer_rsrc_t nul = ws_rsrc(g.out8, 0L);
#pragma unroll
    for (int d2 = 0; d2 < 3; ++d2) __builtin_amdgcn_raw_buffer_store_b32(0u, nul, 0, 0, 0);
  };
  auto form_y = [&](v16i (&acc)[2], float (&y)[2][16], int k) {
    const float sr = sal[((k & 1) * 8 + wave) * 64 + lane];
    float am = 0.0f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int c = 64 * wave + 32 * u + 16 * hh + 4 * qq;
        const float4 s4 = *reinterpret_cast<const float4*>(swl + c);
        const float4 b4 = *reinterpret_cast<const float4*>(swl + 512 + c);
        const float swq[4] = {s4.x, s4.y, s4.z, s4.w}, bq4[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          y[u][4 * qq + e] = fmaxf(((float)acc[u][4 * qq + e] * sr) * swq[e] + bq4[e], 0.0f);
          am = fmaxf(am, y[u][4 * qq + e]);
        }
      }
    am = fmaxf(am, __shfl_xor(am, 32));
    if (lane < 32) redb(k)[wave * WP_R + lane] = am;
  };
  auto slice_max = [&](int k) {
    const float* red = redb(k);
    float m = red[tok];
#pragma unroll
    for (int w = 1; w < 8; ++w) m = fmaxf(m, red[w * WP_R + tok]);
    return m;
  };
  auto gidx = [&](int rb, int tt) { return ((long)rb * 4 + tt) * 32 + tok; };
  auto publish = [&](int k, float m) {
    if (wave == 0 && lane < 32 && t != g.drop_slice)
      __hip_atomic_store(gran + gidx(rbk(k), t), (1ull << 32) | __float_as_uint(m),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  const unsigned lim = (unsigned)g.spin_limit;
  auto full_max = [&](int k, float mloc) {
    const int rb = rbk(k);
    float m = mloc;
    for (unsigned spin = 0;; ++spin) {
      bool ok = true;
      float mx = mloc;
#pragma unroll
      for (int d = 1; d < 4; ++d) {
        const unsigned long long v = __hip_atomic_load(gran + gidx(rb, (t + d) & 3), __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        ok &= (v >> 32) == 1ull;
        mx = fmaxf(mx, __uint_as_float((unsigned)v));
      }
      if (__all(ok)) { m = mx; break; }
      if (spin >= lim) {                            // bounded: never hang, never silent
        if (lane == 0)
          __hip_atomic_fetch_or(g.status, DEV_E_EXCHANGE_TIMEOUT, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    return m;
  };
  auto scales = [&](int k, float& bq, float& iq) {
    const float* gs = gsc + (k & 1) * 2 * WP_R;
    bq = gs[tok];
    iq = gs[WP_R + tok];
  };
  auto store_tile = [&](int k, int u, const uint32_t (&d)[4]) {
    const long row = rbk(k) * WP_R + tok;
    __builtin_amdgcn_raw_buffer_store_b128(v4u{d[0], d[1], d[2], d[3]}, orsrc,
                                           (int)kp_off(row, c0 + 32 * u, g.ldo8), 0, 0);
  };
  auto quant_all = [&](int k, const float (&y)[2][16]) {      // 2 stores (+ wave 0's scale)
    float bq, iq;
    scales(k, bq, iq);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        d[j] = pack4_biased(rint_biased(div_cr(y[u][4 * j], bq, iq)),
                            rint_biased(div_cr(y[u][4 * j + 1], bq, iq)),
                            rint_biased(div_cr(y[u][4 * j + 2], bq, iq)),
                            rint_biased(div_cr(y[u][4 * j + 3], bq, iq)));
      store_tile(k, u, d);
    }
  };
  auto mfma_block = [&](v16i (&acc)[2], int k, auto q_c, int kq, float (&y)[2][16]) {
    constexpr bool Q = decltype(q_c)::value;
    const uint8_t* cur = lds + (k & 1) * WP_STAGE;
    float bq = 0.0f, iq = 0.0f;
    if constexpr (Q) scales(kq, bq, iq);
    float hist = 0.0f, tq[4];
    uint32_t d[4];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const v4i x = *reinterpret_cast<const v4i*>(cur + (s << 10) + lane * 16);
      v4i w[2];
#pragma unroll
      for (int u = 0; u < 2; ++u)
        w[u] = s < W32_SR ? wr[s < W32_SR ? s : 0][u]
                          : *reinterpret_cast<const v4i*>(wl + (((wave * (16 - W32_SR) + s - W32_SR) * 2 + u) << 10) + lane * 16);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if constexpr (!Q) {
          if (s == 0) mfma32_asm<true>(acc[u], w[u], x);
          else mfma32_asm<false>(acc[u], w[u], x);
        } else {
          const int o = 2 * s + u, uo = o >> 4, r = o & 15;
          float yv = y[uo][r];
          if (s == 0) mfma32_pin<true>(acc[u], w[u], x, hist, yv);
          else mfma32_pin<false>(acc[u], w[u], x, hist, yv);
          tq[r & 3] = rint_biased(div_cr(yv, bq, iq));
          hist = tq[r & 3];
          if ((r & 3) == 3) {
            d[r >> 2] = pack4_biased(tq[0], tq[1], tq[2], tq[3]);
            if (r == 15) store_tile(kq, uo, d);
          }
        }
      }
    }
    mfma32_settle(acc);
    if constexpr (!Q) dummy_stores();
  };
  const std::true_type T_{};
  const std::false_type F_{};

  v16i acc[2];
  float y0[2][16], y1[2][16];      // y of the even / odd blocks
  float mq0 = 0.0f, mq1 = 0.0f;    // their slice maxima
  __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
  __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
  __builtin_amdgcn_s_barrier();
  auto iter = [&](int k, float (&yb)[2][16], float& mb, float& mo) {
    if (k > 0) {
      __builtin_amdgcn_s_waitcnt(WAIT_VM(0));   // block k's DMA and the 3 stores after it (VM_CNT_ORDER)
      __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
      __builtin_amdgcn_s_barrier();
    }
    if (wave == 0 && k >= 1 && k <= nblk) {     // only wave 0 publishes and gathers
      mo = slice_max(k - 1);
      publish(k - 1, mo);
    }
    if (k + 1 < nblk) issue(k + 1);
    if (k < nblk) {
      if (k >= 2) mfma_block(acc, k, T_, k - 2, yb);
      else mfma_block(acc, k, F_, 0, yb);
      form_y(acc, yb, k);
    } else if (k >= 2) {
      quant_all(k - 2, yb);
    } else {
      dummy_stores();
    }
    if (wave == 0 && k >= 1 && k <= nblk) {
      const float m = full_max(k - 1, mo);
      const float sc = fmaxf(m, 1e-5f) / 127.0f;
      const float inv = 1.0f / sc;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sc), srsrc, 4 * (rbk(k - 1) * WP_R + tok), 0, 0);
      if (lane < WP_R) {
        float* gs = gsc + ((k - 1) & 1) * 2 * WP_R;
        gs[lane] = sc;
        gs[WP_R + lane] = inv;
      }
    }
  };
  for (int k = 0; k <= nblk + 1; k += 2) {
    iter(k, y0, mq0, mq1);
    if (k + 1 <= nblk + 1) iter(k + 1, y1, mq1, mq0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// W [N, 512] row-major -> the WS32 layout (k_gemm_wsq32): one thread per 16-byte chunk.
__global__ void k_pack_w_ws32(const int8_t* W, int N, int8_t* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;   // output chunk index
  if (i >= (long)N * 32) return;
  const int lane = (int)(i & 63), u = (int)((i >> 6) & 1), s = (int)((i >> 7) & 15);
  const int w = (int)((i >> 11) & 7), t = (int)(i >> 14);
  const int r = lane & 31;
  const long n = 512L * t + 64 * w + 32 * u + 16 * ((r >> 2) & 1) + 4 * (r >> 3) + (r & 3);
  *reinterpret_cast<uint4*>(out + 16 * i) =
      *reinterpret_cast<const uint4*>(W + n * WS_K + 32 * s + 16 * (lane >> 5));
}
hipError_t launch_pack_w_ws32(const int8_t* W, int N, int K, int8_t* out, hipStream_t st) {
  if (N % 512 || N <= 0 || K != WS_K) return hipErrorInvalidValue;
  const long nch = (long)N * 32;
  k_pack_w_ws32<<<dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, st>>>(W, N, out);
  return hipGetLastError();
}

hipError_t launch_gemm_ws32_diag(const RowGemmArgs& g, dim3 grid, hipStream_t st) {
  if (g.epi != RE_QUANT) return hipErrorInvalidValue;
  if (knobs().ws32 == 2) k_gemm_wsq32<1, 16><<<grid, dim3(512), 0, st>>>(g);   // all of W in VGPRs
  else k_gemm_wsq32<<<grid, dim3(512), 0, st>>>(g);
  return hipGetLastError();
}
hipError_t launch_gemm_wsy32_diag(const RowGemmArgs& a, int ng, hipStream_t st) {
  k_gemm_wsy32<<<dim3(4 * 8 * ng), dim3(512), 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_gemm_ws_diag(const RowGemmArgs& g, dim3 grid, hipStream_t st) {
  const Knobs& kn = knobs();
  if (g.epi == RE_QUANT) {
    switch (kn.wsq) {
      case 2: k_gemm_wss<<<grid, dim3(512), 0, st>>>(g); return hipGetLastError();
      case 3: k_gemm_wsz<><<<grid, dim3(512), 0, st>>>(g); return hipGetLastError();
      case 4: k_gemm_wsa<><<<grid, dim3(256), 0, st>>>(g); return hipGetLastError();
      default: return hipErrorNotSupported;
    }
  }
  if (!kn.wsa2) return hipErrorNotSupported;
  if (g.epi == RE_RELU_PMAX) k_gemm_wsa2<RE_RELU_PMAX><<<grid, dim3(256), 0, st>>>(g);
  else if (g.epi == RE_RELU_QUANT_PMAX) k_gemm_wsa2<RE_RELU_QUANT_PMAX><<<grid, dim3(256), 0, st>>>(g);
  else return hipErrorNotSupported;
  return hipGetLastError();
}

hipError_t launch_gemm_wsx_diag(const RowGemmArgs& a, int ng, hipStream_t st) {
  if (knobs().wsy != 0) return hipErrorNotSupported;
  k_gemm_wsx<<<dim3(4 * 8 * ng), dim3(512), 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace qtx

// W [N, 512] -> the WS32 layout, for tests/diag_variants.py (diagnostic library only)
extern "C" int qtx_debug_pack_w_ws32(const int8_t* W, int N, int K, int8_t* out, void* st) {
  return (int)qtx::launch_pack_w_ws32(W, N, K, out, (hipStream_t)st);
}
