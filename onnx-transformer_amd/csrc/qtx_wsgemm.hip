// qtx_wsgemm.hip — the encoder's K = 512 QuantLinear GEMMs, weight-stationary
// (quant_linear.py:111-119; Q/K/V, O-projection and FFN1 of encoder.py at large M):
//   out[m, n] = epilogue( sum_k A[m,k] * W[n,k] ),  y = ((float(acc) * sa[m]) * sw[n]) + b[n]
//
// Why: k_gemm_row streams BOTH operands through LDS (128 x 512 tile, 205 int8 ops per LDS
// byte) and is bound by the ~70 GB/s per-CU L2 -> LDS fill.  At K = 512 a whole 512-column
// slice of W is 256 KB — half of a CU's 512 KB register file.  So each workgroup keeps its
// slice of W on chip for the whole launch (wave w: columns 64w..64w+63, K steps 0-4 in 80
// VGPRs and K steps 5-7 in LDS: with 2 waves per SIMD a wave has 256 registers, and the
// accumulators and epilogues need the rest), and only A moves: 64-row blocks (32 KB) by
// LDS-DMA, read by all 8 waves — 512 ops per LDS byte filled, so the MFMA pipe, not the
// fill, paces the main loop.  The workgroup is persistent over the row blocks of its slice.
//
// The MFMA computes the transposed tile C^T = W . A^T (W fragments as the A operand): its
// output layout then gives each lane 4 token rows (16i + (lane & 15)) x 16 CONSECUTIVE
// output columns — 4 per-row scalars per lane instead of 16, one 16-byte int8 store per row,
// and a row's partial max over the wave's 64 columns in 2 cross-lane steps.
//
// Layouts (all K = 512):
//   A   KP layout (qtx_common.h kp_off), as the encoder's producers write it.
//   W   "WS" layout (k_pack_w_ws): for slice t, wave w, K step s (64 B), fragment j, 1 KB in
//       MFMA operand lane order: lane l holds W[n][64s + 16(l>>4) .. +16] with
//       n = 512t + 64w + 16((l & 15) >> 2) + 4j + (l & 3), so that C^T row 4q + e of
//       fragment j (lane group q = l >> 4, element e) is column 512t + 64w + 16q + 4j + e.
//   LDS A tile: piece (s, i) = row fragment i (16 rows), K step s: 1 KB in MFMA lane order
//       (lane l: row 16i + (l & 15), bytes 64s + 16(l>>4)) — conflict-free lane-linear
//       ds_read_b128; filled from KP lines (8 full 128-byte lines per piece).
// Epilogues (RowEpi, qtx_kernels.h): RE_QUANT (per-token quant over the 512-column slice),
// RE_RES_LN (N = 512: residual + next LayerNorm + quant), RE_RELU_PMAX, RE_RELU_QUANT_PMAX.
// Numerics: identical to k_gemm_row (the same canonical order; GPU == oracle bit for bit).
#include "qtx_ws.h"

#include "qtx_knobs.h"

QTX_STAMP_SETTER(ws)

namespace qtx {

template <int EPI>
__global__ __launch_bounds__(512) void k_gemm_ws(RowGemmArgs g) {
  // LDS (160 KB): A stages | W K steps 5-7 (96 KB) | epilogue staging.  RES_LN keeps ONE A
  // stage (the next block's DMA flies under the epilogue) and stages y a quarter block (16
  // rows, 32 KB) at a time; the others keep two A stages (the next block's DMA flies under
  // this block's MFMAs) and exchange partial row maxima in the consumed stage.
  constexpr int NST = EPI == RE_RES_LN ? 1 : 2;
  constexpr int EXTRA = EPI == RE_RES_LN ? 16 * 512 * 4 : 0;
  __shared__ __attribute__((aligned(16))) uint8_t lds[NST * WS_STAGE + WS_WL + EXTRA];
  uint8_t* const wl = lds + NST * WS_STAGE;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int f = lane & 15, gq = lane >> 4;
  const int nsl = g.N >> 9;
  const int wpt = gridDim.x / nsl;               // workgroups per slice
  const int t = blockIdx.x % nsl, r0 = blockIdx.x / nsl;
  const int nb = (g.M + WS_R - 1) / WS_R;
  if (r0 >= nb) return;
  QTX_STAMP(0);

  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  // wave w moves K step w of the four row fragments (4 pieces of 8 KP lines)
  auto issue = [&](uint8_t* st, int rb) {
    const int m0 = rb * WS_R;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long row = min(m0 + 16 * i + f, g.M - 1);
      dma16(g.A + kp_off(row, 64 * wave + 16 * gq, WS_K), st + ((wave * 4 + i) << 10));
    }
  };
  issue(lds, r0);

  // this wave's W fragments, resident for the whole launch: K steps 5-7 into LDS (12
  // pieces, DMA), 0-4 into registers (K-step order: the first MFMAs wait only for the first
  // loads)
  v4i wr[WS_SR][4];
  {
    const int8_t* wsrc = g.W + ((long)(t * 8 + wave) << 15);
#pragma unroll
    for (int p = 0; p < (8 - WS_SR) * 4; ++p)
      dma16(wsrc + ((WS_SR * 4 + p) << 10) + lane * 16, wl + ((wave * (8 - WS_SR) * 4 + p) << 10));
    const v4i* ws = reinterpret_cast<const v4i*>(wsrc) + lane;
#pragma unroll
    for (int s = 0; s < WS_SR; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) wr[s][j] = ws[(s * 4 + j) * 64];
    // consume them here: otherwise the compiler's wait for them lands at the top of the
    // block loop, where vmcnt(0) would also wait for the next block's DMA every iteration
#pragma unroll
    for (int s = 0; s < WS_SR; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(wr[s][j]));
  }
  const int cs = 64 * wave + 16 * gq;            // the lane's 16 columns within the slice
  const int c0 = 512 * t + cs;                   // ... within the whole output row

  int it = 0;
  for (int rb = r0; rb < nb; rb += wpt, ++it) {
    const int m0 = rb * WS_R;
    uint8_t* cur = lds + (NST == 2 ? (it & 1) * WS_STAGE : 0);
    // this wave's DMA of the block retired, and with it the previous epilogue's stores:
    // VM_CNT_ORDER (qtx_common.h) — a store issued after the DMA may retire before it, so a
    // count that leaves the stores in flight could release the barrier early; the barrier
    // makes every wave's part visible and frees the other stage / the epilogue areas
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (it == 0) QTX_STAMP(1);
    // per-row operands of the block, one row per lane (fetched by ds_bpermute later); issued
    // BEFORE the next block's DMA: vmcnt retires in issue order, so waiting for these loads
    // does not wait for the DMA
    const int lrow = min(m0 + lane, g.M - 1);
    const float sa_l = g.sa[lrow];
    float pmv[4] = {0.0f, 0.0f, 0.0f, 0.0f};     // reduced in the epilogue, not here
    if constexpr (EPI == RE_RELU_QUANT_PMAX) {
#pragma unroll
      for (int p = 0; p < 4; ++p) pmv[p] = g.pmax_in[(long)min(p, g.pmax_n - 1) * g.M + lrow];
    }
    if (NST == 2 && rb + wpt < nb) issue(lds + ((it + 1) & 1) * WS_STAGE, rb + wpt);

    // acc[i][j]: C^T fragment (W fragment j) x (token row fragment i)
    v4i acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};
    // sw / bias of the lane's 16 columns: issued during the last K steps (scheduling
    // barriers keep them there and keep their consumers out of the main loop: a compiler wait
    // inside the loop would also wait for the next block's DMA, vmcnt retiring in order)
    float4 sw4[4], b4[4];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (s == 6) {
        __builtin_amdgcn_sched_barrier(0);
        const float4* swp = reinterpret_cast<const float4*>(g.sw + c0);
        const float4* bp = reinterpret_cast<const float4*>(g.bias + c0);
#pragma unroll
        for (int j = 0; j < 4; ++j) { sw4[j] = swp[j]; b4[j] = bp[j]; }
        __builtin_amdgcn_sched_barrier(0);
      }
      v4i a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *reinterpret_cast<const v4i*>(cur + ((s * 4 + i) << 10) + lane * 16);
      v4i b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = s < WS_SR ? wr[s < WS_SR ? s : 0][j]
                         : *reinterpret_cast<const v4i*>(wl + (((wave * (8 - WS_SR) + s - WS_SR) * 4 + j) << 10) + lane * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[j], a[i], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (it < 5) QTX_STAMP(2 + 2 * it);
    if constexpr (NST == 1) {
      // every wave is past its fragment reads: the stage takes the next block's DMA now
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (rb + wpt < nb) issue(lds, rb + wpt);
    }

    // ---- y = ((float(acc) * sa[m]) * sw[n]) + b[n]; lane: token rows 16i + f, columns
    // cs + 4j + e (16 consecutive: y[i][4j + e])
    float y[4][16];
    {
      // opaque: keeps the compiler from hoisting the consumers of the per-row loads (and
      // with them a vmcnt wait that would include the next block's DMA) into the main loop
      float sa_e = sa_l;
      asm volatile("" : "+v"(sa_e));
      float sr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        sr[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (16 * i + f), __float_as_int(sa_e)));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float swj[4] = {sw4[j].x, sw4[j].y, sw4[j].z, sw4[j].w};
        const float bj[4] = {b4[j].x, b4[j].y, b4[j].z, b4[j].w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = ((float)acc[i][j][e] * sr[i]) * swj[e] + bj[e];
            // relu: v > 0 ? v : 0 up to the sign of a zero, which no consumer sees (the
            // row max takes |.|, the quantizer maps +-0 to the same code)
            y[i][4 * j + e] = (EPI == RE_RELU_PMAX || EPI == RE_RELU_QUANT_PMAX) ? fmaxf(v, 0.0f) : v;
          }
      }
    }

    if (it == 0) QTX_STAMP(12);
    if constexpr (EPI == RE_RES_LN) {
      // four quarters of 16 rows (row fragment qq): stage y as fp32 rows [16][512] (16-byte
      // chunk c of row r at chunk position c ^ (r & 7): conflict-free writes and reads);
      // wave w then takes rows 2w, 2w+1 of the quarter: x = res + y (residual in the
      // canonical lane layout, loaded before the staging), x out, LayerNorm (ln_rows512),
      // per-token quant (or fp32 out)
      float* stg = reinterpret_cast<float*>(wl + WS_WL);
      float ga[2][4], gb[2][4];
      ln_params512(g.ln_a, g.ln_b, lane, ga, gb);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int rowb = m0 + 16 * qq + 2 * wave;
        float4 rv[2][2];
#pragma unroll
        for (int r2 = 0; r2 < 2; ++r2) {
          const int row = min(rowb + r2, g.M - 1);
#pragma unroll
          for (int c = 0; c < 2; ++c)
            rv[r2][c] = *reinterpret_cast<const float4*>(g.res + (long)row * 512 + 4 * (lane + 64 * c));
        }
        if (qq > 0) {                             // every wave is done reading the last quarter
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<float4*>(stg + f * 512 + 4 * ((cs / 4 + j) ^ (f & 7))) =
              make_float4(y[qq][4 * j], y[qq][4 * j + 1], y[qq][4 * j + 2], y[qq][4 * j + 3]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        float v[2][2][4];
#pragma unroll
        for (int r2 = 0; r2 < 2; ++r2)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int r = 2 * wave + r2;
            const float4 t4 = *reinterpret_cast<const float4*>(stg + r * 512 + 4 * ((lane + 64 * c) ^ (r & 7)));
            v[r2][c][0] = rv[r2][c].x + t4.x; v[r2][c][1] = rv[r2][c].y + t4.y;
            v[r2][c][2] = rv[r2][c].z + t4.z; v[r2][c][3] = rv[r2][c].w + t4.w;
          }
#pragma unroll
        for (int r2 = 0; r2 < 2; ++r2)
          if (rowb + r2 < g.M)
#pragma unroll
            for (int c = 0; c < 2; ++c)
              *reinterpret_cast<float4*>(g.xout + (long)(rowb + r2) * 512 + 4 * (lane + 64 * c)) =
                  make_float4(v[r2][c][0], v[r2][c][1], v[r2][c][2], v[r2][c][3]);
        ln_rows512<2>(v, ga, gb);
        if (g.lnq) {
          uint32_t qd[2][2];
          float sc[2];
          quant_rows512<2>(v, qd, sc);
#pragma unroll
          for (int r2 = 0; r2 < 2; ++r2)
            if (rowb + r2 < g.M) {
              const long row = rowb + r2;
              *reinterpret_cast<uint32_t*>(g.lnq + kp_off(row, 4 * lane, 512)) = qd[r2][0];
              *reinterpret_cast<uint32_t*>(g.lnq + kp_off(row, 4 * (lane + 64), 512)) = qd[r2][1];
              if (lane == 0) g.lns[row] = sc[r2];
            }
        } else {
#pragma unroll
          for (int r2 = 0; r2 < 2; ++r2)
            if (rowb + r2 < g.M)
#pragma unroll
              for (int c = 0; c < 2; ++c)
                *reinterpret_cast<float4*>(g.lnout + (long)(rowb + r2) * 512 + 4 * (lane + 64 * c)) =
                    make_float4(v[r2][c][0], v[r2][c][1], v[r2][c][2], v[r2][c][3]);
        }
      }
      if (it < 5) QTX_STAMP(3 + 2 * it);
      continue;
    } else {
      // ---- the row's absmax over the 512-column slice (QUANT, RELU_PMAX: the wave's 64
      // columns in 16 values x the 4 lane groups, then the 8 waves through LDS) or over the
      // whole row from the partial maxima (RELU_QUANT_PMAX); one row per lane after that
      float m;
      if constexpr (EPI == RE_RELU_QUANT_PMAX) {
#pragma unroll
        for (int p = 0; p < 4; ++p) asm volatile("" : "+v"(pmv[p]));
        m = fmaxf(fmaxf(pmv[0], pmv[1]), fmaxf(pmv[2], pmv[3]));
        for (int p = 4; p < g.pmax_n; ++p) m = fmaxf(m, g.pmax_in[(long)p * g.M + lrow]);
      } else {
        float pm[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float a = fabsf(y[i][0]);
#pragma unroll
          for (int c = 1; c < 16; ++c) a = fmaxf(a, fabsf(y[i][c]));
          a = fmaxf(a, __shfl_xor(a, 16));
          pm[i] = fmaxf(a, __shfl_xor(a, 32));
        }
        // the block's A stage is free once every wave is past its fragment reads: it holds
        // the per-wave partial maxima [8][64]
        float* red = reinterpret_cast<float*>(cur);
        if (it == 0) QTX_STAMP(13);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (it == 0) QTX_STAMP(14);
        if (gq == 0)
#pragma unroll
          for (int i = 0; i < 4; ++i) red[wave * WS_R + 16 * i + f] = pm[i];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        m = red[lane];
#pragma unroll
        for (int w = 1; w < 8; ++w) m = fmaxf(m, red[w * WS_R + lane]);
        if (it == 0) QTX_STAMP(15);
      }
      const int orow = m0 + lane;
      if constexpr (EPI == RE_RELU_PMAX) {
        // every wave stores the (identical) row maxima: 1 store per wave (counted above)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(m), ws_rsrc(g.pmax_out + (long)t * g.M, 4L * g.M),
                                              4 * orow, 0, 0);
        if (it < 5) QTX_STAMP(3 + 2 * it);
        continue;
      } else {
        // per-token quantization rint(y / s) with the correctly rounded quotient (div_cr:
        // shared reciprocal per row), guard as in k_gemm_row: rmax < 2^37 for every row of
        // the block, else every lane takes the true division (uniform branch)
        const float sc_l = quant_scale(m, 127.0f);
        const float inv_l = 1.0f / sc_l;
        const bool big = __ballot(!(m < 0x1p37f)) != 0ull;
        // every wave stores the (identical) scales: 1 store per wave (RELU_QUANT_PMAX: in the
        // slice-0 workgroups only, so the counted wait there does not include it)
        if (EPI == RE_QUANT || t == 0)
          __builtin_amdgcn_raw_buffer_store_b32(
              __float_as_uint(sc_l), ws_rsrc(EPI == RE_QUANT ? g.os + (long)t * g.os_ts : g.os, 4L * g.M),
              4 * orow, 0, 0);
        float sc[4], inv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sc[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (16 * i + f), __float_as_int(sc_l)));
          inv[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (16 * i + f), __float_as_int(inv_l)));
        }
        // data: 4 x 16 bytes per lane, unconditional (rows >= M fall past the range; the KP
        // output's range includes the pad row of an odd M, which is scratch)
        const __amdgpu_buffer_rsrc_t orsrc =
            EPI == RE_QUANT ? ws_rsrc(g.out8 + (long)t * g.o8_ts, (long)g.M * g.ldo8)
                            : ws_rsrc(g.out8, (long)(g.M + (g.M & 1)) * g.ldo8);
        auto store = [&](auto quot) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            uint32_t d[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
              d[j] = pack4_codes<EPI == RE_RELU_QUANT_PMAX>(
                  quot(y[i][4 * j], sc[i], inv[i]), quot(y[i][4 * j + 1], sc[i], inv[i]),
                  quot(y[i][4 * j + 2], sc[i], inv[i]), quot(y[i][4 * j + 3], sc[i], inv[i]));
            const long row = m0 + 16 * i + f;
            const long off = EPI == RE_QUANT ? row * g.ldo8 + cs : kp_off(row, c0, g.ldo8);
            __builtin_amdgcn_raw_buffer_store_b128(v4u{d[0], d[1], d[2], d[3]}, orsrc, (int)off, 0, 0);
          }
        };
        if (__builtin_expect(big, 0))
          store([](float a, float b, float) { return a / b; });
        else
          store([](float a, float b, float yy) { return div_cr(a, b, yy); });
        if (it < 5) QTX_STAMP(3 + 2 * it);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // trailing DMA (never read) drained
}

// =====================================================================================
// k_gemm_wsp: the same weight-stationary GEMM, software-pipelined (RE_QUANT, RE_RELU_PMAX,
// RE_RELU_QUANT_PMAX).  Measured on k_gemm_ws: the main loop alone runs at the MFMA floor
// and the epilogue alone takes about as long again, and the two do not overlap (every wave
// reaches its epilogue together).  Here row blocks are 32 rows and iteration b issues the
// MFMAs of block b in the same basic blocks as the epilogue of block b-1 (y, row maxima,
// quantization, stores), so the VALU / LDS latency chains of one block run under the
// matrix work of the next.  Two barriers per block: the top one (block b's A landed in
// every wave's part; the other stage and the max-exchange area free) and one between the
// epilogue's two halves (the partial row maxima of block b-1 visible).
// Nothing in an iteration waits for the next block's DMA: the only vector-memory loads of
// an iteration (per-row scales / maxima of block b) are issued before it, sw / bias live in
// LDS, and the stores are unconditional buffer stores, so the top of the next iteration
// waits with a counted vmcnt.
// =====================================================================================
template <int EPI, int SR = WS_SR>   // SR: K steps of W in registers (8: all of W, no LDS part)
__global__ __launch_bounds__(512) void k_gemm_wsp(RowGemmArgs g) {
  constexpr int WL = 8 * (8 - SR) * 4 * 1024;      // W's LDS part
  // LDS: 2 A stages (32 KB) | W K steps 5-7 (96 KB) | sw, bias of the slice (4 KB) |
  // partial row maxima [8][32] (1 KB)
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WP_STAGE + WL + 4096 + 8 * WP_R * 4];
  uint8_t* const wl = lds + 2 * WP_STAGE;
  float* const swl = reinterpret_cast<float*>(wl + WL);    // [512] sw, then [512] bias
  float* const red = swl + 1024;                               // [8][32]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int f = lane & 15, gq = lane >> 4;
  const int nsl = g.N >> 9;
  const int wpt = gridDim.x / nsl;
  const int t = blockIdx.x % nsl, r0 = blockIdx.x / nsl;
  const int nb = (g.M + WP_R - 1) / WP_R;
  if (r0 >= nb) return;
  const int nblk = (nb - r0 + wpt - 1) / wpt;          // row blocks r0, r0 + wpt, ...

  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  // block k of this workgroup (clamped: past the last one the last is re-loaded, never read,
  // so every iteration issues the same DMAs); wave w moves K step w of the 2 row fragments
  auto issue = [&](int k) {
    const int rb = r0 + min(k, nblk - 1) * wpt;
    uint8_t* st = lds + (k & 1) * WP_STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long row = min(rb * WP_R + 16 * i + f, g.M - 1);
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
    // sw / bias of the slice into LDS (wave w: 128 floats)
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
  const int cs = 64 * wave + 16 * gq;            // the lane's 16 columns within the slice
  const int c0 = 512 * t + cs;
  // outputs: unconditional range-checked buffer stores (rows >= M dropped)
  const __amdgpu_buffer_rsrc_t orsrc =
      EPI == RE_QUANT ? ws_rsrc(g.out8 + (long)t * g.o8_ts, (long)g.M * g.ldo8)
                      : ws_rsrc(g.out8, EPI == RE_RELU_QUANT_PMAX ? (long)(g.M + (g.M & 1)) * g.ldo8 : 0L);
  const __amdgpu_buffer_rsrc_t srsrc =
      EPI == RE_RELU_PMAX ? ws_rsrc(g.pmax_out + (long)t * g.M, 4L * g.M)
      : EPI == RE_QUANT   ? ws_rsrc(g.os + (long)t * g.os_ts, 4L * g.M)
                          : ws_rsrc(g.os, t == 0 ? 4L * g.M : 0L);   // the slice-0 WGs store it

  // per-row operands of block k: lane l holds row (l & 31) (loaded before the block's DMA)
  auto rowops = [&](int k, float& sa, float (&pm)[4]) {
    const int row = min(r0 * WP_R + min(k, nblk - 1) * wpt * WP_R + (lane & 31), g.M - 1);
    sa = g.sa[row];
    if constexpr (EPI == RE_RELU_QUANT_PMAX) {
#pragma unroll
      for (int p = 0; p < 4; ++p) pm[p] = g.pmax_in[(long)min(p, g.pmax_n - 1) * g.M + row];
    }
  };
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
  // epilogue of block k, first half: y (lane: rows 16i + f, columns cs .. cs+15) and, for
  // QUANT / RELU_PMAX, the wave's partial row maxima into red
  auto epi1 = [&](const v4i (&acc)[2][4], float sa, float (&y)[2][16]) {
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
        for (int e = 0; e < 4; ++e) {
          const float v = ((float)acc[i][j][e] * sr[i]) * swj[e] + bj[e];
          y[i][4 * j + e] = EPI == RE_QUANT ? v : fmaxf(v, 0.0f);   // relu up to the sign of 0
        }
    }
    if constexpr (EPI != RE_RELU_QUANT_PMAX) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float a = fabsf(y[i][0]);
#pragma unroll
        for (int c = 1; c < 16; ++c) a = fmaxf(a, fabsf(y[i][c]));
        a = fmaxf(a, __shfl_xor(a, 16));
        a = fmaxf(a, __shfl_xor(a, 32));
        red[wave * WP_R + 16 * i + f] = a;      // the 4 lane groups store the same value
      }
    }
  };
  // second half: the row max (8 waves' partials, or the FFN1 partial maxima), the scale,
  // and the unconditional stores of block k
  auto epi2 = [&](int k, const float (&y)[2][16], const float (&pm)[4]) {
    const int m0 = (r0 + min(k, nblk - 1) * wpt) * WP_R;
    float m;
    if constexpr (EPI == RE_RELU_QUANT_PMAX) {
      m = fmaxf(fmaxf(pm[0], pm[1]), fmaxf(pm[2], pm[3]));   // pmax_n <= 4 (launch check)
    } else {
      m = red[lane & 31];
#pragma unroll
      for (int w = 1; w < 8; ++w) m = fmaxf(m, red[w * WP_R + (lane & 31)]);
    }
    // rows m0 + (lane & 31); lanes 32-63 duplicate 0-31 and store the same values
    if constexpr (EPI == RE_RELU_PMAX) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(m), srsrc, 4 * (m0 + (lane & 31)), 0, 0);
    } else {
      // rint(y / s) exactly: div_cr (shared reciprocal per row) on y and s both scaled by
      // 2^-64 when the row max is >= 2^37 (an exact power-of-two scaling that keeps every
      // intermediate of the Markstein step normal; |y / s| <= 127 either way) — branch-free
      // the scale by the true division (one per row and lane: cheap), not quant_scale's
      // guarded shared-reciprocal form, whose wave-uniform branch would split this basic
      // block and keep the quantization from interleaving with the MFMAs above
      const float sc = fmaxf(m, 1e-5f) / 127.0f;
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
          d[j] = pack4_codes<EPI == RE_RELU_QUANT_PMAX>(
              div_cr(y[i][4 * j] * k2, b, yi), div_cr(y[i][4 * j + 1] * k2, b, yi),
              div_cr(y[i][4 * j + 2] * k2, b, yi), div_cr(y[i][4 * j + 3] * k2, b, yi));
        const long row = m0 + 16 * i + f;
        const long off = EPI == RE_QUANT ? row * g.ldo8 + cs : kp_off(row, c0, g.ldo8);
        __builtin_amdgcn_raw_buffer_store_b128(v4u{d[0], d[1], d[2], d[3]}, orsrc, (int)off, 0, 0);
      }
    }
  };
  auto top_wait = [&]() {
    // the block's DMA retired, and the previous epilogue's stores with it (VM_CNT_ORDER,
    // qtx_common.h: stores issued after the DMA may retire before it), then every wave's
    // part visible (compiler-visible waits: its own wait insertion then knows what they
    // retired)
    __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
    __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
  };
  auto zero = [](v4i (&acc)[2][4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  };

  // ---- block 0: main loop only
  long long st_top = 0, st_mid = 0, st_h1 = 0, st_h2 = 0;   // QTX_STAMPS builds only
  const long long st_0 = QTX_NOW();
  v4i accp[2][4];
  float sap, pmp[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
  __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
  __builtin_amdgcn_s_barrier();
  rowops(0, sap, pmp);
  issue(1);
  zero(accp);
  mfma_steps(accp, lds, 0, 8);
  __builtin_amdgcn_s_waitcnt(WAIT_VM(0));   // block 1's DMA (no stores behind it yet)
  // ---- steady state: block k's MFMAs with block k-1's epilogue
  const long long st_1 = QTX_NOW();
  for (int k = 1; k < nblk; ++k) {
    const long long t0 = QTX_NOW();
    top_wait();
    const long long t1 = QTX_NOW();
    st_top += t1 - t0;
    // last iteration's per-row loads complete HERE, before this iteration's loads and DMA:
    // the compiler's wait for them at their use would otherwise count only its own younger
    // loads and also wait for the DMA issued in between
    asm volatile("" ::"v"(sap));
#pragma unroll
    for (int p = 0; p < 4; ++p) asm volatile("" ::"v"(pmp[p]));
    float sac, pmc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    rowops(k, sac, pmc);
    issue(k + 1);
    const uint8_t* cur = lds + (k & 1) * WP_STAGE;
    v4i acc[2][4];
    zero(acc);
    float y[2][16];
    mfma_steps(acc, cur, 0, 4);
    epi1(accp, sap, y);
#ifdef QTX_WSP_IGLP
    interleave<32, QTX_WSP_IGLP_V1>();
#endif
    const long long t2 = QTX_NOW();
    st_h1 += t2 - t1;
    __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
    const long long t3 = QTX_NOW();
    st_mid += t3 - t2;
    mfma_steps(acc, cur, 4, 8);
    epi2(k - 1, y, pmp);
#ifdef QTX_WSP_IGLP
    interleave<32, QTX_WSP_IGLP_V2>();
#endif
    st_h2 += QTX_NOW() - t3;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) accp[i][j] = acc[i][j];
    sap = sac;
#pragma unroll
    for (int p = 0; p < 4; ++p) pmp[p] = pmc[p];
  }
  // ---- the last block's epilogue
  {
    top_wait();
    float y[2][16];
    epi1(accp, sap, y);
    __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
    epi2(nblk - 1, y, pmp);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // phase totals for tools/wsp_stamps.py (QTX_STAMPS builds only)
  QTX_STAMP_VAL(0, st_1 - st_0);
  QTX_STAMP_VAL(1, st_top);
  QTX_STAMP_VAL(2, st_h1);
  QTX_STAMP_VAL(3, st_mid);
  QTX_STAMP_VAL(4, st_h2);
  QTX_STAMP_VAL(5, QTX_NOW() - st_0);
  QTX_STAMP_VAL(6, nblk);
}

// =====================================================================================
// k_gemm_wsq: the weight-stationary Q/K/V GEMM (RE_QUANT) with ONE barrier per 32-row block
// and the quantization one block behind, interleaved between the MFMAs in a fixed order:
//   iteration k:  the 64 MFMAs of block k with one quantized output of block k-1 after every
//                 second one (its row maxima in red[(k-1) & 1] are complete: every wave
//                 wrote them at the end of iteration k-1, before this barrier); then, as a
//                 VALU-only phase, y = ((acc * sa) * sw) + b of block k and its partial row
//                 maxima -> red[k & 1].
// Why this split (tools/probe_mfma_valu.hip, two waves per SIMD): about two VALU per i8
// MFMA issue for free beside the matrix work, each further one costs ~4 cycles there,
// while VALU with no MFMA to share the SIMD with costs ~2 cycles (the two waves
// alternate).  The quantization (~4.5 VALU per output) fills exactly the free slots; y
// (~5 per output) runs on its own.  The compiler's list scheduler puts MFMAs back to back
// and the epilogue before or after them (k_gemm_wsp), so each MFMA here is an asm statement
// (asm statements keep their order) and each quantized output is pinned between two of them
// by operands the asm text does not touch: the previous output's result is an input of the
// next MFMA, the next output's input an output of it.
// Numerics as k_gemm_wsp: div_cr with the row's reciprocal (Markstein: RN(y / s) for every
// y with |y| <= the row maximum, any magnitude), the scale by true division.
// =====================================================================================
// PRIO: s_setprio 1 for waves 4-7 (the arbitration losers), experiment.  LAG: a pinned MFMA
// waits for the quantized output LAG places back (1: the one just before it), so the
// quantization's dependent VALU chain need not finish before the next MFMA issues; 2 and 3
// measured no faster (QKV 40.5 / 40.4 vs 40.0 us, FFN1 70.9 / 70.0 vs 68.1 us).
// XG: the nsl column-slice workgroups of a row group on one XCD (blockIdx % 8 under
// round-robin placement — speed only), dispatched together, so a row block's A is fetched
// from HBM once and read from L2 by the other slices (0: slice = blockIdx % nsl)
template <int PRIO = 0, int LAG = 1, int XG = 1>
__global__ __launch_bounds__(512) void k_gemm_wsq(RowGemmArgs g) {
  constexpr int SR = WS_SR, WL = 8 * (8 - SR) * 4 * 1024;
  // LDS: 2 A stages (32 KB) | W K steps 5-7 (96 KB) | sw, bias (4 KB) | red [2][8][32] (2 KB)
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WP_STAGE + WL + 4096 + 2 * 8 * WP_R * 4 + 2 * 8 * 64 * 4];
  uint8_t* const wl = lds + 2 * WP_STAGE;
  float* const swl = reinterpret_cast<float*>(wl + WL);
  float* const red0 = swl + 1024;                            // [2][8][32]
  float* const sal = red0 + 2 * 8 * WP_R;                    // [2][8 waves][64]: row scales
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int f = lane & 15, gq = lane >> 4;
  const long long rt_entry = QTX_RNOW();          // QTX_STAMPS builds: kernel entry
  // the side job (before any early exit): this workgroup's share of the next FFN1's
  // exchange scratch, zeroed (the stores retire under the prologue's vmcnt(0))
  if (g.zero16 > 0) {
    const long per = (g.zero16 + gridDim.x - 1) / gridDim.x;
    const long z0 = per * blockIdx.x, z1 = min(z0 + per, g.zero16);
    uint4* zp = reinterpret_cast<uint4*>(g.zero);
    for (long i = z0 + tid; i < z1; i += 512) zp[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  const int nsl = g.N >> 9;
  const int wpt = gridDim.x / nsl;
  int t = blockIdx.x % nsl, r0 = blockIdx.x / nsl;
  if (XG) {
    // the first 8 * nsl * A workgroups: XCD x, slot j -> slice j % nsl of row group
    // 8 * (j / nsl) + x; the rest (fewer than 8 * nsl) in blockIdx order after them
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
  if (PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);

  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto rbk = [&](int k) { return r0 + min(k, nblk - 1) * wpt; };
  // block k's A rows and, per wave, its 32 row scales (lanes 32-63 repeat them) by LDS-DMA:
  // no global load in the loop whose wait the compiler would count past the DMA (its
  // counted vmcnt does not see the asm DMAs, so it would also wait for them)
  auto dma4 = [](const float* gsrc, const float* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto issue = [&](int k) {
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
  auto top_wait = [&]() {
    // the block's DMA retired, and the previous iteration's 3 stores per wave with it
    // (VM_CNT_ORDER, qtx_common.h: a count leaving them in flight can release early)
    __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
    __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
  };
  // y of block k (acc, row scale sa) and the wave's partial row maxima into red[k & 1]
  auto form_y = [&](v4i (&acc)[2][4], float (&y)[2][16], int k) {
    float sr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) sr[i] = sal[((k & 1) * 8 + wave) * 64 + 16 * i + f];
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
  // the scale of block k's rows (lane: row lane & 31) from red (stored), broadcast per
  // row fragment: divisor bq, reciprocal iq.  This chain sits before the block's first
  // pinned quantization (with constant scales QKV ran 38.2 vs 39.9 us): scale127 / rcp_cr
  // (the IEEE quotient and reciprocal, qtx_common.h) instead of two division sequences
  auto scales = [&](int k, float (&bq)[2], float (&iq)[2]) {
    const float* red = redb(k);
    float m = red[lane & 31];
#pragma unroll
    for (int w = 1; w < 8; ++w) m = fmaxf(m, red[w * WP_R + (lane & 31)]);
    const float sc = scale127(fmaxf(m, 1e-5f));
    const float inv = rcp_cr(sc);
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
  // MFMAs of block k into acc; with q: the quantization of block k-1 (y) between them
  auto mfma_block = [&](v4i (&acc)[2][4], const uint8_t* cur, bool q, int kq, float (&y)[2][16]) {
    float bq[2] = {0.0f, 0.0f}, iq[2] = {0.0f, 0.0f};
    if (q) scales(kq, bq, iq);
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
          const int n = s * 8 + i * 4 + j;             // MFMA slot 0..63
          if (!q || (n & 1) == 0) {
            if (s == 0) mfma_asm<true>(acc[i][j], b[j], a[i]);
            else mfma_asm<false>(acc[i][j], b[j], a[i]);
          } else {
            // quantized output o of block k-1: row fragment ii, column group jj, element e
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
    if (!q) {           // the 3 stores per iteration the next top wait counts (dropped)
      const __amdgpu_buffer_rsrc_t nul = ws_rsrc(g.out8, 0L);
#pragma unroll
      for (int d2 = 0; d2 < 3; ++d2) __builtin_amdgcn_raw_buffer_store_b32(0u, nul, 0, 0, 0);
    }
  };

  v4i acc[2][4];
  float y[2][16];
  long long st_top = 0, st_mm = 0, st_y = 0;          // QTX_STAMPS builds only
  const long long st_0 = QTX_NOW(), rt_0 = QTX_RNOW();
  // ---- block 0: MFMAs, then its y
  __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
  __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
  __builtin_amdgcn_s_barrier();
  issue(1);
  mfma_block(acc, lds, false, 0, y);
  form_y(acc, y, 0);
  const long long st_1 = QTX_NOW();
  // ---- block k: MFMAs with the quantization of block k-1, then the y of block k
  for (int k = 1; k < nblk; ++k) {
    const long long t0 = QTX_NOW();
    top_wait();
    const long long t1 = QTX_NOW();
    issue(k + 1);
    mfma_block(acc, lds + (k & 1) * WP_STAGE, true, k - 1, y);
    const long long t2 = QTX_NOW();
    form_y(acc, y, k);
    const long long t3 = QTX_NOW();
    st_top += t1 - t0;
    st_mm += t2 - t1;
    st_y += t3 - t2;
  }
  QTX_STAMP_VAL(0, st_1 - st_0);
  QTX_STAMP_VAL(1, st_top);
  QTX_STAMP_VAL(2, st_mm);
  QTX_STAMP_VAL(4, st_y);
  QTX_STAMP_VAL(6, nblk);
#ifdef QTX_STAMPS
  // per wave (lane 0 of every wave): top wait, MFMA + quantization, y — after the 16
  // per-block slots, at [256 * 16 + (block * 8 + wave) * 4 + phase]
  if (lane == 0 && qtx_stamp_buf) {
    unsigned long long* pw = qtx_stamp_buf + 256 * 16 + ((long)blockIdx.x * 8 + wave) * 4;
    pw[0] = st_top; pw[1] = st_mm; pw[2] = st_y; pw[3] = nblk;
  }
#endif
  // ---- the last block's quantization
  top_wait();
  {
    float bq[2], iq[2];
    scales(nblk - 1, bq, iq);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        d[j] = pack4_biased(rint_biased(div_cr(y[i][4 * j], bq[i], iq[i])),
                            rint_biased(div_cr(y[i][4 * j + 1], bq[i], iq[i])),
                            rint_biased(div_cr(y[i][4 * j + 2], bq[i], iq[i])),
                            rint_biased(div_cr(y[i][4 * j + 3], bq[i], iq[i])));
      store_row(nblk - 1, i, d);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  QTX_STAMP_VAL(5, QTX_NOW() - st_0);
  QTX_STAMP_VAL(7, QTX_RNOW() - rt_0);
  QTX_STAMP_VAL(8, rt_entry);
  QTX_STAMP_VAL(9, QTX_RNOW());
}

// =====================================================================================
// k_gemm_wsy: the one-pass FFN1 of k_gemm_wsx with k_gemm_wsq's schedule — ONE barrier per
// 32-row block and the quantization between the MFMAs (asm statements, pinned):
//   iteration k:  top barrier (block k-1's partial row maxima complete in red[(k-1) & 1],
//                 block k-2's row scales in LDS); wave 0 publishes block k-1's slice
//                 maxima; block k+1's A by LDS-DMA; the 64 MFMAs of block k with block
//                 k-2's quantized outputs pinned between them; y = relu(((acc * sa) * sw)
//                 + b) of block k and its partial row maxima -> red[k & 1] (VALU-only
//                 phase); then wave 0 alone gathers block k-1's maxima over all 4 slices
//                 (its partners published them an iteration ago) and forms that block's
//                 row scales for every wave — in the ~1,300 cycles by which wave 0, a SIMD
//                 arbitration winner, reaches the next barrier before the losers.
// y of blocks k-1 and k-2 are both held (one buffer per block parity): the quantization of
// block k waits two iterations for its partners' maxima, so the hand-off latency hides under
// a whole iteration as in k_gemm_wsx.  The exchange (tickets, granules, bounded waits that
// report DEV_E_EXCHANGE_TIMEOUT) is k_gemm_wsx's.  Numerics as k_gemm_wsq: RN(y / s) by
// div_cr with the row's reciprocal, s by true division.
// Wait ordering: the top of an iteration waits vmcnt(0) (VM_CNT_ORDER, qtx_common.h: a store
// may retire before a DMA issued ahead of it, so counting the stores behind the DMA is
// unsafe); wave 0's granule loads are waited for where it gathers them.
// =====================================================================================
template <int PRIO = 0, int LAG = 1>   // as k_gemm_wsq
__global__ __launch_bounds__(512) void k_gemm_wsy(RowGemmArgs g) {
  constexpr int SR = WS_SR, WL = 8 * (8 - SR) * 4 * 1024;
  // LDS: 2 A stages (32 KB) | W K steps 5-7 (96 KB) | sw, bias (4 KB) | red [2][8][32] (2 KB)
  // | row scales [2][8][64] (4 KB) | full row maxima [2][32]
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WP_STAGE + WL + 4096 + 2 * 8 * WP_R * 4 + 2 * 8 * 64 * 4 +
                                                      2 * 2 * WP_R * 4];
  uint8_t* const wl = lds + 2 * WP_STAGE;
  float* const swl = reinterpret_cast<float*>(wl + WL);
  float* const red0 = swl + 1024;                            // [2][8][32]
  float* const sal = red0 + 2 * 8 * WP_R;                    // [2][8 waves][64]: row scales
  float* const gsc = sal + 2 * 8 * 64;                       // [2][2][32]: rows' scale s and
                                                             // RN(1/s) per block parity
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int f = lane & 15, gq = lane >> 4;
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
  if (PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);

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
  const int c0 = 512 * t + cs;
  const __amdgpu_buffer_rsrc_t orsrc = ws_rsrc(g.out8, (long)(g.M + (g.M & 1)) * g.ldo8);
  const __amdgpu_buffer_rsrc_t srsrc = ws_rsrc(g.os, t == 0 ? 4L * g.M : 0L);
  auto redb = [&](int k) { return red0 + (k & 1) * 8 * WP_R; };
  auto dummy_stores = [&]() {
    const __amdgpu_buffer_rsrc_t nul = ws_rsrc(g.out8, 0L);
#pragma unroll
    for (int d2 = 0; d2 < 3; ++d2) __builtin_amdgcn_raw_buffer_store_b32(0u, nul, 0, 0, 0);
  };
  // Y: y of block k (before the ReLU) from acc and the wave's partial ReLU'd row maxima
  // -> red[k & 1]
  auto form_y = [&](v4i (&acc)[2][4], float (&y)[2][16], int k) {
    float sr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) sr[i] = sal[((k & 1) * 8 + wave) * 64 + 16 * i + f];
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
          // pre-ReLU y: the maximum from 0 is the ReLU'd row maximum, and the codes take the
          // ReLU in their conversion (pack4_relu_u8)
          y[i][4 * j + e] = ((float)acc[i][j][e] * sr[i]) * swj[e] + bj[e];
          am[i] = fmaxf(am[i], y[i][4 * j + e]);
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
  auto slice_max = [&](int k) {
    const float* red = redb(k);
    float m = red[lane & 31];
#pragma unroll
    for (int w = 1; w < 8; ++w) m = fmaxf(m, red[w * WP_R + (lane & 31)]);
    return m;
  };
  auto gidx = [&](int rb, int tt) { return ((long)rb * 4 + tt) * 32 + (lane & 31); };
  auto publish = [&](int k, float m) {
    // (g.drop_slice: the test hook that withholds one slice's maxima so its partners' waits
    // time out, QTX_WSX_DROP_SLICE; -1 in production)
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
  // block k's scale from its full row maximum m (stored; lane: row lane & 31), broadcast per
  // row fragment: divisor bq, reciprocal iq
  // block k's row scales (s and RN(1/s), written by wave 0 before this iteration's
  // barrier, gather_scales below) for the lane's rows of each row fragment
  auto scales = [&](int k, float (&bq)[2], float (&iq)[2]) {
    const float* gs = gsc + (k & 1) * 2 * WP_R;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bq[i] = gs[16 * i + f];
      iq[i] = gs[WP_R + 16 * i + f];
    }
  };
  auto store_row = [&](int k, int i, const uint32_t (&d)[4]) {
    const long row = rbk(k) * WP_R + 16 * i + f;
    __builtin_amdgcn_raw_buffer_store_b128(v4u{d[0], d[1], d[2], d[3]}, orsrc, (int)kp_off(row, c0, g.ldo8), 0, 0);
  };
  auto quant_all = [&](int k, const float (&y)[2][16]) {      // 2 stores (+ wave 0's scale)
    float bq[2], iq[2];
    scales(k, bq, iq);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        d[j] = pack4_relu_u8(div_cr(y[i][4 * j], bq[i], iq[i]), div_cr(y[i][4 * j + 1], bq[i], iq[i]),
                             div_cr(y[i][4 * j + 2], bq[i], iq[i]), div_cr(y[i][4 * j + 3], bq[i], iq[i]));
      store_row(k, i, d);
    }
  };
  // M(k) into acc; Q: block kq's quantization (y, full maximum m) pinned between the MFMAs
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
            tq[e] = div_cr(yv, bq[ii], iq[ii]);
            hist[2] = hist[1]; hist[1] = hist[0]; hist[0] = tq[e];
            if (e == 3) {
              d[jj] = pack4_relu_u8(tq[0], tq[1], tq[2], tq[3]);
              if (jj == 3) store_row(kq, ii, d);
            }
          }
        }
    }
    mfma_settle(acc);
    if constexpr (!Q) dummy_stores();
  };
  const std::true_type T_{};
  const std::false_type F_{};

  v4i acc[2][4];
  float y0[2][16], y1[2][16];      // y of the even / odd blocks
  float mq0 = 0.0f, mq1 = 0.0f;    // their slice maxima
  __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
  __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
  __builtin_amdgcn_s_barrier();
  // iteration k; yb / mb: the buffers of blocks of k's parity (block k-2 in, block k out),
  // mo: the slice maximum of block k-1 (the other parity)
  long long st_top = 0, st_fm = 0, st_mm = 0, st_y = 0;   // QTX_STAMPS builds only
  const long long st_0 = QTX_NOW();
  auto iter = [&](int k, float (&yb)[2][16], float& mb, float& mo) {
    const long long t0 = QTX_NOW();
    if (k > 0) {
      __builtin_amdgcn_s_waitcnt(WAIT_VM(0));   // block k's DMA and the 3 stores after it (VM_CNT_ORDER)
      __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
      __builtin_amdgcn_s_barrier();
    }
    const long long t1 = QTX_NOW();
    // (block k-2's row scales: gathered by wave 0 at the end of iteration k-1 from the
    // maxima its partners published an iteration before that; read after the barrier)
    const long long t2 = QTX_NOW();
    if (wave == 0 && k >= 1 && k <= nblk) {     // only wave 0 publishes and gathers
      mo = slice_max(k - 1);
      publish(k - 1, mo);
    }
    if (k + 1 < nblk) issue(k + 1);
    if (k < nblk) {
      if (k >= 2) mfma_block(acc, k, T_, k - 2, yb);
      else mfma_block(acc, k, F_, 0, yb);
      const long long t3 = QTX_NOW();
      form_y(acc, yb, k);
      if (k >= 2) {
        st_top += t1 - t0;
        st_fm += t2 - t1;
        st_mm += t3 - t2;
        st_y += QTX_NOW() - t3;
      }
    } else if (k >= 2) {
      quant_all(k - 2, yb);
    } else {
      dummy_stores();
    }
    // wave 0 (a SIMD arbitration winner: it reaches the next barrier ~1,300 cycles before
    // the losers) gathers block k-1's partner maxima now, so the load latency hides in its
    // barrier slack instead of opening every wave's next iteration
    // and turns them into the block's row scales (s = max(m, 1e-5) / 127, stored for the
    // next GEMM; RN(1/s) for div_cr) once, for every wave
    if (wave == 0 && k >= 1 && k <= nblk) {
      const long long tf0 = QTX_NOW();
      const float m = full_max(k - 1, mo);
      const float sc = fmaxf(m, 1e-5f) / 127.0f;
      const float inv = 1.0f / sc;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sc), srsrc, 4 * (rbk(k - 1) * WP_R + (lane & 31)), 0, 0);
      if (lane < WP_R) {
        float* gs = gsc + ((k - 1) & 1) * 2 * WP_R;
        gs[lane] = sc;
        gs[WP_R + lane] = inv;
      }
      st_fm += QTX_NOW() - tf0;
    }
  };
  for (int k = 0; k <= nblk + 1; k += 2) {
    iter(k, y0, mq0, mq1);
    if (k + 1 <= nblk + 1) iter(k + 1, y1, mq1, mq0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  QTX_STAMP_VAL(5, QTX_NOW() - st_0);
  QTX_STAMP_VAL(6, nblk);
#ifdef QTX_STAMPS
  // per wave (lane 0): top wait, partners' maxima, MFMA + quantization, y over blocks 2..,
  // at [256 * 16 + (block * 8 + wave) * 8 + phase]
  if (lane == 0 && qtx_stamp_buf) {
    unsigned long long* pw = qtx_stamp_buf + 256 * 16 + ((long)blockIdx.x * 8 + wave) * 8;
    pw[0] = st_top; pw[1] = st_fm; pw[2] = st_mm; pw[3] = st_y; pw[4] = nblk;
  }
#endif
}

// =====================================================================================
// k_gemm_wsr: the O-projection (RE_RES_LN, K = N = 512) weight-stationary at large M:
// x = res + y, x stored, the next LayerNorm in the canonical order and its per-token
// quantization (KP out) — sublayer_connection.py:15-17, layer_norm.py:12-15,
// quant_linear.py:30-43.  The launch is bound by HBM (per 32-row block: 64 KB of residual
// in, 64 KB of x and 16 KB of codes out, against 2,048 MFMA cycles per SIMD), so the design
// keeps HBM busy: 32-row blocks (4 per workgroup at cfg3's M), two A stages (block k+1's
// DMA under block k), block k's residual rows loaded at the top of its iteration (their
// latency hides under the MFMAs), and every store unconditional (buffer range check), so
// the next top waits with a counted vmcnt instead of draining the stores.
// Epilogue in 4 rounds of 8 rows: the lanes holding those rows stage y in the block's A
// stage (free once every wave is past its MFMAs; 16 KB = 8 rows x 512 fp32, chunk c of row
// r at c ^ (r & 7)), then wave w takes row w of the round whole (ln_rows512 / quant_rows512
// need a row's 512 values in the canonical lane layout).
// =====================================================================================
__global__ __launch_bounds__(512) void k_gemm_wsr(RowGemmArgs g) {
  constexpr int SR = WS_SR, WL = 8 * (8 - SR) * 4 * 1024;
  // LDS: 2 A stages (32 KB; the consumed one stages y) | W K steps 5-7 (96 KB) | sw, bias
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WP_STAGE + WL + 4096];
  uint8_t* const wl = lds + 2 * WP_STAGE;
  float* const swl = reinterpret_cast<float*>(wl + WL);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int f = lane & 15, gq = lane >> 4;
  const int wpt = gridDim.x;
  const int r0 = blockIdx.x;
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
    const int8_t* wsrc = g.W + ((long)wave << 15);
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
      *reinterpret_cast<float2*>(swl + c) = *reinterpret_cast<const float2*>(g.sw + c);
      *reinterpret_cast<float2*>(swl + 512 + c) = *reinterpret_cast<const float2*>(g.bias + c);
    }
#pragma unroll
    for (int s = 0; s < SR; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(wr[s][j]));
  }
  const int cs = 64 * wave + 16 * gq;
  float ga[2][4], gb[2][4];
  ln_params512(g.ln_a, g.ln_b, lane, ga, gb);
  const __amdgpu_buffer_rsrc_t xrsrc = ws_rsrc(g.xout, 4L * 512 * g.M);
  const __amdgpu_buffer_rsrc_t qrsrc = ws_rsrc(g.lnq, (long)(g.M + (g.M & 1)) * 512);
  const __amdgpu_buffer_rsrc_t srsrc = ws_rsrc(g.lns, 4L * g.M);

  __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
  __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
  __builtin_amdgcn_s_barrier();
  for (int k = 0; k < nblk; ++k) {
    if (k > 0) {
      // block k's DMA retired, and block k-1's 20 stores (4 rounds x 5) with it
      // (VM_CNT_ORDER, qtx_common.h)
      __builtin_amdgcn_s_waitcnt(WAIT_VM(0));
      __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
      __builtin_amdgcn_s_barrier();
    }
    const int m0 = rbk(k) * WP_R;
    const float sa = g.sa[min(m0 + (lane & 31), g.M - 1)];
    // this wave's 4 residual rows (row 8r + wave of round r), before the next block's DMA
    float4 rv[4][2];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long row = min(m0 + 8 * r + wave, g.M - 1);
#pragma unroll
      for (int c = 0; c < 2; ++c)
        rv[r][c] = *reinterpret_cast<const float4*>(g.res + row * 512 + 4 * (lane + 64 * c));
    }
    if (k + 1 < nblk) issue(k + 1);
    uint8_t* const cur = lds + (k & 1) * WP_STAGE;
    v4i acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};
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
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[j], a[i], acc[i][j], 0, 0, 0);
    }
    // y = ((acc * sa) * sw) + b; lane: rows 16i + f, columns cs + 4j + e
    float y[2][16];
    {
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
          for (int e = 0; e < 4; ++e) y[i][4 * j + e] = ((float)acc[i][j][e] * sr[i]) * swj[e] + bj[e];
      }
    }
    float* const stg = reinterpret_cast<float*>(cur);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // every wave is past its reads of the stage (the MFMAs' A, or the previous round)
      __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
      __builtin_amdgcn_s_barrier();
      const int i = r >> 1, h = r & 1;            // round r: rows 16i + 8h .. +7
      if ((f >> 3) == h) {
        const int rr = f & 7;                     // row within the round
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<float4*>(stg + rr * 512 + 4 * ((cs / 4 + j) ^ rr)) =
              make_float4(y[i][4 * j], y[i][4 * j + 1], y[i][4 * j + 2], y[i][4 * j + 3]);
      }
      __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
      __builtin_amdgcn_s_barrier();
      const int rr = wave;                        // this wave's row of the round
      const int row = m0 + 8 * r + rr;
      float v[1][2][4];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float4 t4 = *reinterpret_cast<const float4*>(stg + rr * 512 + 4 * ((lane + 64 * c) ^ rr));
        v[0][c][0] = rv[r][c].x + t4.x; v[0][c][1] = rv[r][c].y + t4.y;
        v[0][c][2] = rv[r][c].z + t4.z; v[0][c][3] = rv[r][c].w + t4.w;
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
        __builtin_amdgcn_raw_buffer_store_b128(
            v4u{__float_as_uint(v[0][c][0]), __float_as_uint(v[0][c][1]), __float_as_uint(v[0][c][2]),
                __float_as_uint(v[0][c][3])},
            xrsrc, (int)(((long)row * 512 + 4 * (lane + 64 * c)) * 4), 0, 0);
      ln_rows512<1>(v, ga, gb);
      uint32_t qd[1][2];
      float sc[1];
      quant_rows512<1>(v, qd, sc);
      __builtin_amdgcn_raw_buffer_store_b32(qd[0][0], qrsrc, (int)kp_off(row, 4 * lane, 512), 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(qd[0][1], qrsrc, (int)kp_off(row, 4 * (lane + 64), 512), 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sc[0]), srsrc, 4 * row, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

hipError_t launch_gemm_wsx(const RowGemmArgs& g, hipStream_t st) {
  if (g.M <= 0) return hipSuccess;
  if (g.K != WS_K || g.N != 2048 || g.epi != RE_RELU_QUANT_PMAX || g.fault.kind != FK_NONE ||
      !g.pmax_out || !g.out8 || !g.os)
    return hipErrorInvalidValue;
  const Knobs& kn = knobs();
  const int nb = (g.M + WP_R - 1) / WP_R;
  int ng = 8;                                 // row groups per XCD (4 slices each: 32 WGs)
  if (8 * ng > nb) ng = (nb + 7) / 8;
  // u64 granules + the ticket counter (padded: a memset of a multiple of 16 bytes), zeroed
  // before every launch
  const long ngran = 4L * 32 * nb + 2;
  hipError_t e = hipSuccess;
  if (!g.prezeroed) {   // (the encoder's Q/K/V launch zeroes it as a side job: prezeroed)
    e = launch_zero(g.pmax_out, (size_t)ngran * 8, st);   // (a kernel: graph-capturable)
    if (e != hipSuccess) return e;
  }
  RowGemmArgs a = g;
  if (!a.status)                              // the u32 after the ticket counter
    a.status = reinterpret_cast<unsigned*>(g.pmax_out) + 2 * (4L * 32 * nb) + 1;
  if (a.spin_limit <= 0) {
    // 2^18 polls x s_sleep 2 (~14 ms): far beyond any partner's start under load.  The
    // QTX_WSX_SPIN_LIMIT / QTX_WSX_DROP_SLICE hooks make the timeout path fire in tests.
    a.spin_limit = kn.wsx_spin_limit >= 0 ? kn.wsx_spin_limit : (1 << 18);
  }
  a.drop_slice = kn.wsx_drop_slice;
#ifdef QTX_DIAG
  if (a.kp == 3 && (e = launch_gemm_wsx_diag(a, ng, st)) != hipErrorNotSupported) return e;
  if (a.kp == 3 && kn.ws_prio) {
    k_gemm_wsy<1><<<dim3(4 * 8 * ng), dim3(512), 0, st>>>(a);
    return hipGetLastError();
  }
#endif
  if (a.kp == 5) {                            // W in WS32: the diagnostic build's k_gemm_wsy32
#ifdef QTX_DIAG
    return launch_gemm_wsy32_diag(a, ng, st);
#else
    return hipErrorInvalidValue;
#endif
  }
  k_gemm_wsy<<<dim3(4 * 8 * ng), dim3(512), 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_gemm_ws_(const RowGemmArgs& g, hipStream_t st);
// The zeroing side job (RowGemmArgs::zero) runs inside the product's Q/K/V kernel; any other
// kernel this call selects gets the zeroing kernel first.
hipError_t launch_gemm_ws(const RowGemmArgs& g, hipStream_t st) {
  if (g.zero16 <= 0) return launch_gemm_ws_(g, st);
  const Knobs& kn = knobs();
  const bool in_wsq = g.M > 0 && g.epi == RE_QUANT && g.kp == 2 && g.pmax_n <= 4 &&
                      !kn.ws_nopipe && kn.wsq == 1 && !kn.ws_prio && kn.ws_xg;
  if (in_wsq) return launch_gemm_ws_(g, st);
  if (const hipError_t e = launch_zero(g.zero, (size_t)g.zero16 * 16, st); e != hipSuccess) return e;
  RowGemmArgs a = g;
  a.zero = nullptr; a.zero16 = 0;
  return launch_gemm_ws_(a, st);
}
hipError_t launch_gemm_ws_(const RowGemmArgs& g, hipStream_t st) {
  if (g.M <= 0) return hipSuccess;
  if (g.K != WS_K || g.N % 512 || g.N <= 0 || (g.epi == RE_RES_LN && g.N != 512) ||
      g.fault.kind != FK_NONE || (g.epi == RE_RELU_QUANT_PMAX && g.pmax_n <= 0))
    return hipErrorInvalidValue;
  const Knobs& kn = knobs();
  const int nsl = g.N / 512;
  if (g.epi == RE_RES_LN && g.lnq && !g.lnout && !kn.ws_nopipe && !kn.wsr_off) {
    // k_gemm_wsr (QTX_WSR=0: k_gemm_ws<RE_RES_LN>): the decode's encoder at B = 32 (M = 2304)
    // 0.656 -> 0.616 ms; at cfg3's M = 32768 the KP row GEMM stays faster (40.3 vs 43.5 us,
    // qtx_api.hip ws_res_ok)
    const int nb = (g.M + WP_R - 1) / WP_R;
    k_gemm_wsr<<<dim3(nb < 256 ? nb : 256), dim3(512), 0, st>>>(g);
    return hipGetLastError();
  }
  if (g.epi != RE_RES_LN && g.pmax_n <= 4 && !kn.ws_nopipe) {   // pipelined
    const int nb = (g.M + WP_R - 1) / WP_R;
    int wpt = 256 / nsl;
    if (wpt > nb) wpt = nb;
    const dim3 grid(nsl * wpt), block(512);
    if (g.kp == 4) {                 // W in the WS32 layout: the diagnostic build's k_gemm_wsq32
#ifdef QTX_DIAG
      return launch_gemm_ws32_diag(g, grid, st);
#else
      return hipErrorInvalidValue;
#endif
    }
#ifdef QTX_DIAG
    // the measured-negative variants: k_gemm_wss / wsz / wsa / wsa2 in
    // qtx_wsgemm_diag.hip; here the template variants of the product kernels
    if (const hipError_t e = launch_gemm_ws_diag(g, grid, st); e != hipErrorNotSupported) return e;
    if (g.epi == RE_QUANT && (kn.wsq == 0 || kn.ws_prio || !kn.ws_xg)) {
      if (kn.wsq == 0) k_gemm_wsp<RE_QUANT><<<grid, block, 0, st>>>(g);
      else if (kn.ws_prio) k_gemm_wsq<1><<<grid, block, 0, st>>>(g);
      else k_gemm_wsq<0, 1, 0><<<grid, block, 0, st>>>(g);
      return hipGetLastError();
    }
    if (g.epi == RE_RELU_PMAX && kn.wsp_pmax_sr5) {
      k_gemm_wsp<RE_RELU_PMAX><<<grid, block, 0, st>>>(g);
      return hipGetLastError();
    }
#endif
    switch (g.epi) {
      // Q/K/V: k_gemm_wsq (39.6 us at cfg3's M = 32768; measured and not kept: k_gemm_wsp
      // 45.2, k_gemm_wss 46.5, k_gemm_wsz 56, k_gemm_wsa 47.7 us — DESIGN.md §4)
      case RE_QUANT: k_gemm_wsq<<<grid, block, 0, st>>>(g); break;
      // the row-max pass has a light epilogue: all of W fits in registers (no W reads from
      // LDS in the main loop)
      case RE_RELU_PMAX: k_gemm_wsp<RE_RELU_PMAX, 8><<<grid, block, 0, st>>>(g); break;
      default: k_gemm_wsp<RE_RELU_QUANT_PMAX><<<grid, block, 0, st>>>(g); break;
    }
    return hipGetLastError();
  }
  const int nb = (g.M + WS_R - 1) / WS_R;
  int wpt = 256 / nsl;
  if (wpt > nb) wpt = nb;
  if (wpt < 1) wpt = 1;
  const dim3 grid(nsl * wpt), block(512);
  switch (g.epi) {
    case RE_QUANT: k_gemm_ws<RE_QUANT><<<grid, block, 0, st>>>(g); break;
    case RE_RES_LN: k_gemm_ws<RE_RES_LN><<<grid, block, 0, st>>>(g); break;
    case RE_RELU_PMAX: k_gemm_ws<RE_RELU_PMAX><<<grid, block, 0, st>>>(g); break;
    case RE_RELU_QUANT_PMAX: k_gemm_ws<RE_RELU_QUANT_PMAX><<<grid, block, 0, st>>>(g); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// W [N, 512] row-major -> the WS layout (header): one thread per 16-byte chunk.
__global__ void k_pack_w_ws(const int8_t* W, int N, int8_t* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;   // output chunk index
  if (i >= (long)N * 32) return;
  const int lane = (int)(i & 63), j = (int)((i >> 6) & 3), s = (int)((i >> 8) & 7);
  const int w = (int)((i >> 11) & 7), t = (int)(i >> 14);
  const int r = lane & 15;
  const long n = 512L * t + 64 * w + 16 * (r >> 2) + 4 * j + (r & 3);
  *reinterpret_cast<uint4*>(out + 16 * i) =
      *reinterpret_cast<const uint4*>(W + n * WS_K + 64 * s + 16 * (lane >> 4));
}

hipError_t launch_pack_w_ws(const int8_t* W, int N, int K, int8_t* out, hipStream_t st) {
  if (N % 512 || N <= 0 || K != WS_K) return hipErrorInvalidValue;
  const long nch = (long)N * 32;
  k_pack_w_ws<<<dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, st>>>(W, N, out);
  return hipGetLastError();
}

}  // namespace qtx
