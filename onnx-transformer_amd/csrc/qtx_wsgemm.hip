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
#include "qtx_common.h"
#include "qtx_kernels.h"

#include <cstdlib>

QTX_STAMP_SETTER(ws)

namespace {
bool getenv_flag(const char* name) {        // experiment switches (A/B on one box)
  const char* v = getenv(name);
  return v && *v && *v != '0';
}
}  // namespace

namespace qtx {

constexpr int WS_K = 512, WS_R = 64;
constexpr int WS_STAGE = WS_R * WS_K;          // 32 KB: one A row block in fragment order
constexpr int WS_SR = 5;                        // K steps of W held in registers (rest: LDS)
constexpr int WS_WL = 8 * (8 - WS_SR) * 4 * 1024;   // W's LDS part: 96 KB

// Raw buffer stores with the hardware range check (a store at or past `bytes` is dropped):
// the epilogue's stores are then unconditional, so every wave issues the same known number
// of them and the next block's top can wait with a counted vmcnt instead of draining them.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ws_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                           0x00020000);
}
typedef unsigned v4u __attribute__((ext_vector_type(4)));

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
#ifdef QTX_WS_NOMFMA                               // diagnostic builds only
          asm volatile("" ::"v"(a[i]), "v"(b[j]));
#else
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[j], a[i], acc[i][j], 0, 0, 0);
#endif
    }
    __builtin_amdgcn_sched_barrier(0);
    if (it < 5) QTX_STAMP(2 + 2 * it);
#ifdef QTX_WS_NOEPI                                 // diagnostic builds only: main loop alone
    {
      int sum = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
      if (sum == 0x7fffffff) g.out8[0] = (int8_t)(sw4[0].x + b4[0].x);
      continue;
    }
#endif
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
              d[j] = pack4_biased(rint_biased(quot(y[i][4 * j], sc[i], inv[i])),
                                  rint_biased(quot(y[i][4 * j + 1], sc[i], inv[i])),
                                  rint_biased(quot(y[i][4 * j + 2], sc[i], inv[i])),
                                  rint_biased(quot(y[i][4 * j + 3], sc[i], inv[i])));
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
constexpr int WP_R = 32, WP_STAGE = WP_R * WS_K;    // 16 KB A stage

// Scheduling pattern for the compiler's IGroupLP: NM times {one MFMA, NV VALU} over the
// current scheduling region, so the epilogue arithmetic of the previous block is spread
// between this block's MFMAs instead of running before or after them (the matrix pipe
// and the vector issue then overlap: tools/probe_mfma_valu.hip)
template <int NM, int NV>
__device__ __forceinline__ void interleave() {
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
  }
}
// s_waitcnt immediates (gfx9 encoding: vmcnt bits 3:0 and 15:14, expcnt 6:4, lgkmcnt 11:8)
constexpr int WAIT_VM(int n) { return (n & 15) | ((n >> 4) << 14) | 0x70 | 0xF00; }
constexpr int WAIT_LGKM0 = 0xC07F;

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
          d[j] = pack4_biased(rint_biased(div_cr(y[i][4 * j] * k2, b, yi)),
                              rint_biased(div_cr(y[i][4 * j + 1] * k2, b, yi)),
                              rint_biased(div_cr(y[i][4 * j + 2] * k2, b, yi)),
                              rint_biased(div_cr(y[i][4 * j + 3] * k2, b, yi)));
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
// Z: the block's first K step, accumulator from the inline constant 0.  (Zeroing it with
// VALU instead needs wait states before the MFMA reads it, which the compiler inserts only
// for MFMAs it knows about, not for these asm statements.)
template <bool Z, typename T>
__device__ __forceinline__ void mfma_pin(v4i& acc, const v4i& w, const v4i& a, float before, T& after) {
  // operands: %0 acc, %1 after (outputs first), %2 w, %3 a, %4 before
  if constexpr (Z)
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %2, %3, 0" : "=&v"(acc), "+v"(after) : "v"(w), "v"(a), "v"(before));
  else
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %2, %3, %0" : "+v"(acc), "+v"(after) : "v"(w), "v"(a), "v"(before));
}
template <bool Z>
__device__ __forceinline__ void mfma_asm(v4i& acc, const v4i& w, const v4i& a) {
  if constexpr (Z)
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, 0" : "=&v"(acc) : "v"(w), "v"(a));
  else
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc) : "v"(w), "v"(a));
}

// After the last asm MFMA of a block: the compiler tracks no wait states for asm MFMAs, so
// pad their results before anything reads them (every acc is an operand here, so no read,
// copy or spill of one moves above the pad).
__device__ __forceinline__ void mfma_settle(v4i (&acc)[2][4]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4"
               : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[0][2]), "+v"(acc[0][3]),
                 "+v"(acc[1][0]), "+v"(acc[1][1]), "+v"(acc[1][2]), "+v"(acc[1][3]));
}

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
#ifdef QTX_EXP_FASTQ
          y[i][4 * j + e] = fmaf((float)acc[i][j][e], sr[i] * swj[e], bj[e]);
#else
          y[i][4 * j + e] = ((float)acc[i][j][e] * sr[i]) * swj[e] + bj[e];
#endif
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
  // row fragment: divisor bq, reciprocal iq
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
#ifdef QTX_EXP_FASTQ
            tq[e] = fmaf(yv, iq[ii], 12582912.0f);
#else
            tq[e] = rint_biased(div_cr(yv, bq[ii], iq[ii]));
#endif
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

// =====================================================================================
// k_gemm_wsy: the one-pass FFN1 of k_gemm_wsx with k_gemm_wsq's schedule — ONE barrier per
// 32-row block and the quantization between the MFMAs (asm statements, pinned):
//   iteration k:  top barrier (block k-1's partial row maxima complete in red[(k-1) & 1]);
//                 the row maxima of block k-2 over all 4 slices (the partners published
//                 them an iteration ago); block k-1's slice maxima published; block k+1's
//                 A by LDS-DMA; the 64 MFMAs of block k with block k-2's quantized outputs
//                 pinned between them; y = relu(((acc * sa) * sw) + b) of block k and its
//                 partial row maxima -> red[k & 1] (VALU-only phase).
// y of blocks k-1 and k-2 are both held (one buffer per block parity): the quantization of
// block k waits two iterations for its partners' maxima, so the hand-off latency hides under
// a whole iteration as in k_gemm_wsx.  The exchange (tickets, granules, bounded waits that
// report DEV_E_EXCHANGE_TIMEOUT) is k_gemm_wsx's.  Numerics as k_gemm_wsq: RN(y / s) by
// div_cr with the row's reciprocal, s by true division.
// Wait ordering: the granule loads (waited for at once) go before this iteration's DMA and
// stores; the top of an iteration waits vmcnt(0) (VM_CNT_ORDER, qtx_common.h: a store may
// retire before a DMA issued ahead of it, so counting the stores behind the DMA is unsafe).
// =====================================================================================
template <int PRIO = 0, int LAG = 1>   // as k_gemm_wsq
__global__ __launch_bounds__(512) void k_gemm_wsy(RowGemmArgs g) {
  constexpr int SR = WS_SR, WL = 8 * (8 - SR) * 4 * 1024;
  // LDS: 2 A stages (32 KB) | W K steps 5-7 (96 KB) | sw, bias (4 KB) | red [2][8][32] (2 KB)
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WP_STAGE + WL + 4096 + 2 * 8 * WP_R * 4 + 2 * 8 * 64 * 4];
  uint8_t* const wl = lds + 2 * WP_STAGE;
  float* const swl = reinterpret_cast<float*>(wl + WL);
  float* const red0 = swl + 1024;                            // [2][8][32]
  float* const sal = red0 + 2 * 8 * WP_R;                    // [2][8 waves][64]: row scales
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
  // Y: y of block k (ReLU) from acc and the wave's partial row maxima -> red[k & 1]
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
#ifdef QTX_EXP_FASTQ
          y[i][4 * j + e] = fmaxf(fmaf((float)acc[i][j][e], sr[i] * swj[e], bj[e]), 0.0f);
#else
          y[i][4 * j + e] = fmaxf(((float)acc[i][j][e] * sr[i]) * swj[e] + bj[e], 0.0f);
#endif
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
    if (wave == 0 && lane < 32)
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
  auto scales = [&](int k, float m, float (&bq)[2], float (&iq)[2]) {
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
    __builtin_amdgcn_raw_buffer_store_b128(v4u{d[0], d[1], d[2], d[3]}, orsrc, (int)kp_off(row, c0, g.ldo8), 0, 0);
  };
  auto quant_all = [&](int k, const float (&y)[2][16], float m) {      // 3 stores
    float bq[2], iq[2];
    scales(k, m, bq, iq);
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
  // M(k) into acc; Q: block kq's quantization (y, full maximum m) pinned between the MFMAs
  auto mfma_block = [&](v4i (&acc)[2][4], int k, auto q_c, int kq, float (&y)[2][16], float m) {
    constexpr bool Q = decltype(q_c)::value;
    const uint8_t* cur = lds + (k & 1) * WP_STAGE;
    float bq[2] = {0.0f, 0.0f}, iq[2] = {0.0f, 0.0f};
    if constexpr (Q) scales(kq, m, bq, iq);
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
#ifdef QTX_EXP_FASTQ
            tq[e] = fmaf(yv, iq[ii], 12582912.0f);
#else
            tq[e] = rint_biased(div_cr(yv, bq[ii], iq[ii]));
#endif
            hist[2] = hist[1]; hist[1] = hist[0]; hist[0] = tq[e];
            if (e == 3) {
              d[jj] = pack4_biased(tq[0], tq[1], tq[2], tq[3]);
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
    float m2 = 0.0f;
    if (k >= 2) m2 = full_max(k - 2, mb);       // granule loads: before this iteration's DMA
    const long long t2 = QTX_NOW();
    if (k >= 1 && k <= nblk) {
      mo = slice_max(k - 1);
      publish(k - 1, mo);
    }
    if (k + 1 < nblk) issue(k + 1);
    if (k < nblk) {
      if (k >= 2) mfma_block(acc, k, T_, k - 2, yb, m2);
      else mfma_block(acc, k, F_, 0, yb, 0.0f);
      const long long t3 = QTX_NOW();
      form_y(acc, yb, k);
      if (k >= 2) {
        st_top += t1 - t0;
        st_fm += t2 - t1;
        st_mm += t3 - t2;
        st_y += QTX_NOW() - t3;
      }
    } else if (k >= 2) {
      quant_all(k - 2, yb, m2);
    } else {
      dummy_stores();
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
  const int nb = (g.M + WP_R - 1) / WP_R;
  int ng = 8;                                 // row groups per XCD (4 slices each: 32 WGs)
  if (8 * ng > nb) ng = (nb + 7) / 8;
  // u64 granules + the ticket counter (padded: a memset of a multiple of 16 bytes), zeroed
  // before every launch
  const long ngran = 4L * 32 * nb + 2;
  hipError_t e = launch_zero(g.pmax_out, (size_t)ngran * 8, st);   // (a kernel: graph-capturable)
  if (e != hipSuccess) return e;
  RowGemmArgs a = g;
  if (!a.status)                              // the u32 after the ticket counter
    a.status = reinterpret_cast<unsigned*>(g.pmax_out) + 2 * (4L * 32 * nb) + 1;
  if (a.spin_limit <= 0) {
    // 2^18 polls x s_sleep 2 (~14 ms): far beyond any partner's start under load.  The
    // environment override exists for the test that makes the timeout path fire.
    const char* v = getenv("QTX_WSX_SPIN_LIMIT");
    a.spin_limit = v && *v ? atoi(v) : (1 << 18);
    if (a.spin_limit < 0) a.spin_limit = 0;
  }
  // k_gemm_wsy (MFMA-interleaved quantization) unless QTX_WSY=0 picks k_gemm_wsx
  if (const char* v = getenv("QTX_WSY"); v && *v == '0') k_gemm_wsx<<<dim3(4 * 8 * ng), dim3(512), 0, st>>>(a);
  else if (getenv_flag("QTX_WS_PRIO")) k_gemm_wsy<1><<<dim3(4 * 8 * ng), dim3(512), 0, st>>>(a);
  else k_gemm_wsy<<<dim3(4 * 8 * ng), dim3(512), 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_gemm_ws(const RowGemmArgs& g, hipStream_t st) {
  if (g.M <= 0) return hipSuccess;
  if (g.K != WS_K || g.N % 512 || g.N <= 0 || (g.epi == RE_RES_LN && g.N != 512) ||
      g.fault.kind != FK_NONE || (g.epi == RE_RELU_QUANT_PMAX && g.pmax_n <= 0))
    return hipErrorInvalidValue;
  const int nsl = g.N / 512;
  const char* wsr = getenv("QTX_WSR");
  if (g.epi == RE_RES_LN && g.lnq && !g.lnout && !getenv_flag("QTX_WS_NOPIPE") &&
      !(wsr && *wsr == '0')) {
    // k_gemm_wsr (QTX_WSR=0: k_gemm_ws<RE_RES_LN>): the decode's encoder at B = 32 (M = 2304)
    // 0.656 -> 0.616 ms; at cfg3's M = 32768 the KP row GEMM stays faster (40.3 vs 43.5 us,
    // qtx_api.hip ws_res_ok)
    const int nb = (g.M + WP_R - 1) / WP_R;
    k_gemm_wsr<<<dim3(nb < 256 ? nb : 256), dim3(512), 0, st>>>(g);
    return hipGetLastError();
  }
  if (g.epi != RE_RES_LN && g.pmax_n <= 4 && !getenv_flag("QTX_WS_NOPIPE")) {   // pipelined
    const int nb = (g.M + WP_R - 1) / WP_R;
    int wpt = 256 / nsl;
    if (wpt > nb) wpt = nb;
    const dim3 grid(nsl * wpt), block(512);
    switch (g.epi) {
      case RE_QUANT:
        // k_gemm_wsq (39.6 us at cfg3's M = 32768, profiles/r03b_*) unless QTX_WSQ picks
        // k_gemm_wsp (0: 45.2 us) or k_gemm_wss (2: 58.7 us, experimental)
        if (const char* v = getenv("QTX_WSQ"); v && *v == '0') k_gemm_wsp<RE_QUANT><<<grid, block, 0, st>>>(g);
        else if (v && *v == '3') k_gemm_wsz<><<<grid, block, 0, st>>>(g);
        else if (v && *v == '4') k_gemm_wsa<><<<grid, dim3(256), 0, st>>>(g);
        else if (v && *v == '2') k_gemm_wss<<<grid, block, 0, st>>>(g);
        else if (getenv_flag("QTX_WS_PRIO")) k_gemm_wsq<1><<<grid, block, 0, st>>>(g);
        else if (const char* x = getenv("QTX_WS_XG"); x && *x == '0') k_gemm_wsq<0, 1, 0><<<grid, block, 0, st>>>(g);
        else k_gemm_wsq<<<grid, block, 0, st>>>(g);
        break;
      case RE_RELU_PMAX:
        // the row-max pass has a light epilogue: all of W fits in registers (no W reads
        // from LDS in the main loop); QTX_WSP_PMAX_SR=5: the LDS-split variant (A/B)
        if (getenv_flag("QTX_WSA2")) k_gemm_wsa2<RE_RELU_PMAX><<<grid, dim3(256), 0, st>>>(g);
        else if (getenv_flag("QTX_WSP_PMAX_SR5")) k_gemm_wsp<RE_RELU_PMAX><<<grid, block, 0, st>>>(g);
        else k_gemm_wsp<RE_RELU_PMAX, 8><<<grid, block, 0, st>>>(g);
        break;
      default:
        if (getenv_flag("QTX_WSA2")) k_gemm_wsa2<RE_RELU_QUANT_PMAX><<<grid, dim3(256), 0, st>>>(g);
        else k_gemm_wsp<RE_RELU_QUANT_PMAX><<<grid, block, 0, st>>>(g);
        break;
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
