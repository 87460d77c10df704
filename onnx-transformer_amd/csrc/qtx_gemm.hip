// qtx_gemm.hip — the encoder's QuantLinear GEMM at large M (gfx950, wave64):
//   out[m, n] = epilogue( sum_k A[m,k] * W[n,k] )      quant_linear.py:111-119
// int8 x int8 -> exact int32 on v_mfma_i32_16x16x64_i8, fp32 dequant epilogue
// y = ((float(acc) * s_a[m]) * s_w[n]) + b[n]  (+ReLU) (+residual), as every qtx GEMM.
//
// k_gemm256: 256 x 256 output tile per workgroup, K step 64 bytes, 512 threads = 8 waves
// as 2 (M) x 4 (N); each wave owns 128 x 64 outputs = 8 x 4 MFMA fragments (128 int32
// accumulators per lane).  Both operands are K-contiguous ("NT"), so A and W tiles have
// the same LDS image: 256 rows x 64 B.  Global -> LDS by global_load_lds_dwordx4 (16 B
// per lane; one wave instruction fills 16 rows x 64 B = 1 KB of LDS, lane-linear); the
// bank-conflict swizzle is applied on the per-lane GLOBAL address (g_slot), so the 16
// lanes of a ds_read_b128 fragment read hit 16 distinct 4-bank groups.  Four LDS stages
// (4 x 32 KB): three K-tiles are in flight while one is multiplied (one barrier per tile).
#include "qtx_common.h"
#include "qtx_kernels.h"

QTX_STAMP_SETTER(gemm)

namespace qtx {

constexpr int G_BM = 256, G_BN = 256, G_BK = 64;
constexpr int G_STAGE = (G_BM + G_BN) * G_BK;   // bytes per LDS stage (32 KB)

// 64-byte LDS rows: slot s of row r holds chunk c = s ^ (2 * ((r >> 3) & 1)).  A fragment
// read (lane l: row l & 15, chunk l >> 4) is a ds_read_b128, serviced in the four lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, +32 (MI355X_MICROARCH.md §LDS); with this
// swizzle each group's 16 lanes hit 16 distinct 4-bank slots (found by exhaustive search
// over per-row XOR masks; the plain layout and (r>>2)&3 both conflict 2-way).
__device__ __forceinline__ int g_slot(int r, int c) { return c ^ (((r >> 3) & 1) << 1); }

template <int FLAGS>
__global__ __launch_bounds__(512) void k_gemm256(GemmArgs g) {
  // Four LDS stages as four distinct arrays: hipcc then sees that the fragment reads of
  // stage t do not alias the DMA in flight into stages t+1..t+3 and does not drain it
  // (with one array it waits vmcnt(0) before every ds_read issued after a glds).
  __shared__ __attribute__((aligned(16))) uint8_t st0[G_STAGE];
  __shared__ __attribute__((aligned(16))) uint8_t st1[G_STAGE];
  __shared__ __attribute__((aligned(16))) uint8_t st2[G_STAGE];
  __shared__ __attribute__((aligned(16))) uint8_t st3[G_STAGE];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;
  // XCD-aware tile order (workgroups are dealt round-robin to the 8 XCDs): logical tile
  // L = row-block-major, and XCD x runs the contiguous logical range x*T/8.. in order, so
  // the column tiles sharing one A row block run together on one XCD and read it from
  // HBM into that XCD's L2 once (bijective for any T: cdna_hip_programming.md T1)
  const int ncol = (g.N + G_BN - 1) / G_BN;
  const int T = gridDim.x, hw = blockIdx.x, q = T / 8, rr = T % 8, xcd = hw % 8;
  const int logical = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + hw / 8;
  const int m0 = (logical / ncol) * G_BM, n0 = (logical % ncol) * G_BN;
  const int nk = g.K / G_BK;    // multiple of 4 (launch check)

  // staging: one wave instruction = 16 rows x 64 B; wave w fills A rows 32w..32w+31 and
  // W rows 32w..32w+31 (2 + 2 instructions per tile)
  const int lrow = lane >> 2, lslot = lane & 3;
  const int8_t* asrc[2];
  const int8_t* wsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = wave * 32 + i * 16 + lrow;
    asrc[i] = g.A + (long)min(m0 + r, g.M - 1) * g.lda + 16 * g_slot(r, lslot);
    wsrc[i] = g.W + (long)min(n0 + r, g.N - 1) * g.ldw + 16 * g_slot(r, lslot);
  }
  // The DMA is issued from inline asm so that hipcc does not track it: it would otherwise
  // wait vmcnt(0) before reading any stage with a DMA in flight (draining the prefetch);
  // completion is counted by hand (vmcnt(8) per step below).  M0 = the wave-uniform LDS
  // destination, written and restored inside the statement (cdna_hip_programming.md §5.7).
  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto issue = [&](uint8_t* base, int kt) {
    // past the last tile: re-load the last one (harmless, the stage is never read
    // again) so every step issues exactly 4 DMAs and the vmcnt counts stay constant
    const int k0 = min(kt, nk - 1) * G_BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) dma16(asrc[i] + k0, base + (wave * 32 + i * 16) * G_BK);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dma16(wsrc[i] + k0, base + G_BM * G_BK + (wave * 32 + i * 16) * G_BK);
  };

  v4i acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  auto compute = [&](const uint8_t* As) {
    const uint8_t* Bs = As + G_BM * G_BK;
    v4i bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = wn * 64 + j * 16 + fr;
      bfr[j] = *reinterpret_cast<const v4i*>(Bs + r * G_BK + 16 * g_slot(r, fg));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = wm * 128 + i * 16 + fr;
      const v4i afr = *reinterpret_cast<const v4i*>(As + r * G_BK + 16 * g_slot(r, fg));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr, bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  // K-tile t lives in stage t % 4; three tiles are in flight ahead of the one multiplied.
  // Top of tile t: this wave's DMAs for t are retired by vmcnt(8) (t+1, t+2 may still be
  // outstanding: 4 instructions each), the barrier makes every wave's part visible and
  // guarantees stage (t+3) % 4 (read at t-1) is free, then t+3 is issued.
  auto step = [&](uint8_t* cur, uint8_t* nxt3, int kt) {
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    // raw barrier: __syncthreads() would add a vmcnt(0) fence draining the DMAs in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(nxt3, kt + 3);
    compute(cur);
  };
  issue(st0, 0);
  issue(st1, 1);
  issue(st2, 2);
  for (int kt = 0; kt < nk; kt += 4) {
    step(st0, st3, kt);
    step(st1, st0, kt + 1);
    step(st2, st1, kt + 2);
    step(st3, st2, kt + 3);
  }

  // epilogue (C layout: col = lane & 15, row = 4 * (lane >> 4) + e)
  constexpr bool relu = FLAGS & EPI_RELU, resid = FLAGS & EPI_RESIDUAL;
  // every operand load is unconditional (clamped index): a load under a divergent branch
  // is waited for before the branch joins, which would serialize them
  float swc[4], bc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = min(n0 + wn * 64 + j * 16 + fr, g.N - 1);
    swc[j] = g.sw[col];
    bc[j] = g.bias[col];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float sr[4], rv[4][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) sr[e] = g.sa[min(m0 + wm * 128 + i * 16 + 4 * fg + e, g.M - 1)];
    if constexpr (resid) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          rv[e][j] = g.res[(long)min(m0 + wm * 128 + i * 16 + 4 * fg + e, g.M - 1) * g.ldr +
                           min(n0 + wn * 64 + j * 16 + fr, g.N - 1)];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = m0 + wm * 128 + i * 16 + 4 * fg + e;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + j * 16 + fr;
        float y = ((float)acc[i][j][e] * sr[e]) * swc[j] + bc[j];
        if constexpr (relu) y = y > 0.0f ? y : 0.0f;
        if constexpr (resid) y = rv[e][j] + y;
        if (row < g.M && col < g.N) g.out[(long)row * g.ldo + col] = y;
      }
    }
  }
}

// Large-M int8 GEMM (M >= 256, K % 256 == 0, 8-bit weights); returns hipErrorNotSupported
// for shapes it does not take (the caller falls back to k_gemm).
hipError_t launch_gemm256(const GemmArgs& g, hipStream_t st) {
  if (g.M < G_BM || g.K % (4 * G_BK) != 0 || (g.lda % 16) || (g.ldw % 16))
    return hipErrorNotSupported;
  const dim3 grid(((g.N + G_BN - 1) / G_BN) * ((g.M + G_BM - 1) / G_BM)), block(512);
  switch (g.flags & (EPI_RELU | EPI_RESIDUAL)) {
    case 0: k_gemm256<0><<<grid, block, 0, st>>>(g); break;
    case EPI_RELU: k_gemm256<EPI_RELU><<<grid, block, 0, st>>>(g); break;
    case EPI_RESIDUAL: k_gemm256<EPI_RESIDUAL><<<grid, block, 0, st>>>(g); break;
    default: k_gemm256<EPI_RELU | EPI_RESIDUAL><<<grid, block, 0, st>>>(g); break;
  }
  return hipGetLastError();
}

// =====================================================================================
// k_gemm_row: 128 rows x 512 columns per workgroup (see RowGemmArgs), K step 128, two LDS
// stages of 80 KB (the whole 160 KB LDS; the DMA of tile k+1 flies during the MFMAs of
// tile k), 8 waves as 2 (M) x 4 (N), each wave 64 x 128 outputs = 4 x 8 fragments.  The
// epilogue works on whole 512-wide row segments.
// K step 128 makes every DMA row a full 128-byte line (8 rows x 128 B per wave-instruction):
// half-line pieces (16 rows x 64 B) cost the texture path twice the work per byte and held
// the K-step-64 version of this kernel at ~16 B/clk/CU of LDS fill.
// LDS rows are 128 B with slot swizzle c ^ ((r >> 1) & 7): conflict-free ds_read_b128
// fragments (both 64-byte halves of the K step) for every 16-row fragment base.
// Column order: LDS W row rho = 128 b + 16 j + f holds output column 128 b + 8 f + j, so
// fragment j / lane column f of a wave's block is column 8 f + j: every lane holds 8
// CONSECUTIVE columns of each of its rows (16-byte fp32 and 8-byte int8 pieces in the
// epilogue instead of 4-byte / 1-byte ones).
// =====================================================================================
constexpr int R_BM = 128, R_BN = 512, R_BK = 128;
constexpr int R_ASZ = R_BM * R_BK;                  // 16 KB
constexpr int R_STAGE = (R_BM + R_BN) * R_BK;       // 80 KB

__device__ __forceinline__ int r_slot(int r, int c) { return c ^ ((r >> 1) & 7); }

// FULL: every row of every tile is < M (M % 128 == 0): the epilogue stores carry no row
// guards, so no divergent branch sits between a load and its use (the compiler's counted
// vmcnt waits would otherwise fall back to waiting for every store in flight).
// FAULT: the fault-injection variant (RowGemmArgs::fault); the product kernels carry none
// of its code or registers.
// Measured and not kept: a persistent variant (grid = #CUs, next tile's first K step
// prefetched under the epilogue) and software-pipelined fragment reads: within noise —
// the main loop is bound by the L2 -> LDS fill (~75 GB/s per CU), not by LDS latency or
// workgroup turnover.
template <int EPI, bool FULL, bool FAULT, bool KP>
__global__ __launch_bounds__(512) void k_gemm_row(RowGemmArgs g) {
  // one 160 KB LDS array: two 80 KB stages of 128-byte K steps (row-major operands) or
  // four 40 KB stages of 64-byte K steps (KP operands); the epilogues reuse it
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * R_STAGE];
  uint8_t* const st0 = lds;
  uint8_t* const st1 = lds + R_STAGE;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;
  const int ncol = g.N / R_BN;
  const int T = gridDim.x, hw = blockIdx.x, q8 = T / 8, rr = T % 8, xcd = hw % 8;
  const int logical = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + hw / 8;
  const int m0 = (logical / ncol) * R_BM, t = logical % ncol, n0 = t * R_BN;
  QTX_STAMP(0);
  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  v4i acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  // the epilogue's per-row / per-column scales and bias, loaded before the main loop (their
  // latency hides under it instead of opening the epilogue)
  const int cl = wn * 128 + 8 * fr;              // first of the lane's 8 columns in the tile
  // (KP full-tile instances only: the others have no registers to spare, they would spill)
  constexpr bool PF = KP && FULL && !FAULT;
  float sra[4][4];
  float4 sw4[2], b4[2];
  auto epi_loads = [&]() {
    const float4* sp = reinterpret_cast<const float4*>(g.sw + n0 + cl);
    const float4* bp = reinterpret_cast<const float4*>(g.bias + n0 + cl);
    sw4[0] = sp[0]; sw4[1] = sp[1]; b4[0] = bp[0]; b4[1] = bp[1];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) sra[i][e] = g.sa[min(m0 + wm * 64 + i * 16 + 4 * fg + e, g.M - 1)];
  };
  if constexpr (PF) epi_loads();

  if constexpr (KP) {
    // ---- KP main loop: 64-byte K steps, 4 stages (three in flight while one is
    // multiplied), every DMA piece 8 full 128-byte lines = 16 rows x 64 B.  LDS rows are
    // 64 B with the conflict-free slot swizzle of k_gemm256 (g_slot).  Wave w moves A row
    // pairs 8w..8w+7 (1 piece) and W row pairs 32w..32w+31 (4 pieces) per step.
    constexpr int KB = 64, KA = R_BM * KB, KSTG = (R_BM + R_BN) * KB;   // 8 KB, 40 KB
    // split K (RE_PARTIAL): this workgroup's K range is chunks [kb0, kb0 + nk)
    const int nk = g.K / KB / (int)gridDim.y;     // multiple of 4 (launch check)
    const int kb0 = (int)blockIdx.y * nk;
    const long lpr = g.K >> 6;                    // 128-byte lines per row pair
    const int q = lane & 7, pr = lane >> 3;       // line chunk, pair within the piece
    const int rsub = 2 * pr + (q >> 2), slot = q & 3;   // LDS row within the piece, slot
    auto src_off = [&](long pair, int r) {        // this lane's source within a K chunk
      return ((pair * lpr) << 7) + ((q >> 2) << 6) + 16 * g_slot(r, slot);
    };
    const int ra = wave * 16 + rsub;              // A LDS row (0..127)
    const long aoff = src_off((min(m0 + ra, g.M - 1)) >> 1, ra);
    long woff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rw = wave * 64 + 16 * i + rsub;   // W LDS row (0..511)
      woff[i] = src_off((n0 + rw) >> 1, rw);
    }
    const int krot = (hw >> 3) % nk;
    auto issue = [&](uint8_t* base, int kt) {
      // past the last step: re-load the last one (never read) so every step issues
      // exactly 5 DMAs and the vmcnt counts stay constant
      int kk = min(kt, nk - 1) + krot;
      if (kk >= nk) kk -= nk;
      const long k0 = (long)(kk + kb0) << 7;      // line index offset of K chunk kk
#ifdef QTX_DIAG_NODMA                             // diagnostic builds only (bound decomposition)
      return;
#endif
      dma16(g.A + aoff + k0, base + wave * 16 * KB);
#pragma unroll
      for (int i = 0; i < 4; ++i) dma16(g.W + woff[i] + k0, base + KA + (wave * 64 + 16 * i) * KB);
    };
    auto compute = [&](const uint8_t* As) {
      const uint8_t* Bs = As + KA;
      v4i bfr[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = wn * 128 + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const v4i*>(Bs + r * KB + 16 * g_slot(r, fg));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + fr;
        const v4i afr = *reinterpret_cast<const v4i*>(As + r * KB + 16 * g_slot(r, fg));
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr, bfr[j], acc[i][j], 0, 0, 0);
      }
    };
    uint8_t* s0 = lds;
    uint8_t* s1 = lds + KSTG;
    uint8_t* s2 = lds + 2 * KSTG;
    uint8_t* s3 = lds + 3 * KSTG;
    // top of step kt: this wave's DMAs for kt retired (kt+1, kt+2 may still fly: 5 each),
    // the barrier makes every wave's part visible and frees stage (kt+3) % 4
    auto step = [&](uint8_t* cur, uint8_t* nxt3, int kt) {
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      issue(nxt3, kt + 3);
      compute(cur);
    };
    issue(s0, 0);
    issue(s1, 1);
    issue(s2, 2);
    for (int kt = 0; kt < nk; kt += 4) {
      step(s0, s3, kt);
      step(s1, s0, kt + 1);
      step(s2, s1, kt + 2);
      step(s3, s2, kt + 3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing re-loads
  } else {
  const int nk = g.K / R_BK;

  // DMA (asm: untracked by hipcc, counted by hand; see k_gemm256): one wave-instruction
  // fills 8 LDS rows of 128 B, lane l row l/8, slot l%8 (source chunk = slot ^ swizzle).
  // Wave w: A rows 16w..16w+15 (2 instructions), W LDS rows 64w..64w+63 (8).
  const int lrow = lane >> 3, lslot = lane & 7;
  const int8_t* asrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ra = wave * 16 + i * 8 + lrow;
    asrc[i] = g.A + (long)min(m0 + ra, g.M - 1) * g.lda + 16 * r_slot(ra, lslot);
  }
  const int8_t* wsrc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rho = wave * 64 + i * 8 + lrow;                   // LDS row
    const int n = (rho & ~127) + 8 * (rho & 15) + ((rho >> 4) & 7);   // its output column
    wsrc[i] = g.W + (long)(n0 + n) * g.ldw + 16 * r_slot(rho, lslot);
  }
  // K steps in rotated order (exact int32 sums: any order gives the same accumulators):
  // the workgroups of one XCD start at different K panels, so they do not all request the
  // same W lines (same L2 channels) at the same time
  const int krot = (hw >> 3) % nk;
  auto issue = [&](uint8_t* base, int kt) {
    int kk = kt + krot;
    if (kk >= nk) kk -= nk;
    const int k0 = kk * R_BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) dma16(asrc[i] + k0, base + (wave * 16 + i * 8) * R_BK);
#pragma unroll
    for (int i = 0; i < 8; ++i) dma16(wsrc[i] + k0, base + R_ASZ + (wave * 64 + i * 8) * R_BK);
  };
  auto compute = [&](const uint8_t* As) {
    const uint8_t* Bs = As + R_ASZ;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      v4i bfr[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = wn * 128 + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const v4i*>(Bs + r * R_BK + 16 * r_slot(r, 4 * h + fg));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + fr;
        const v4i afr = *reinterpret_cast<const v4i*>(As + r * R_BK + 16 * r_slot(r, 4 * h + fg));
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  // step kt: tile kt landed (the only DMA in flight) and every wave is past tile kt-1, so
  // the other stage is free for tile kt+1
  auto step = [&](uint8_t* cur, uint8_t* nxt, int kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 1 < nk) issue(nxt, kt + 1);
    compute(cur);
  };
  issue(st0, 0);
  for (int kt = 0; kt < nk; kt += 2) {
    step(st0, st1, kt);
    if (kt + 1 < nk) step(st1, st0, kt + 1);
  }
  }
  __syncthreads();                                 // all fragment reads done: LDS reusable
  QTX_STAMP(1);
  if constexpr (EPI == RE_PARTIAL) {
    // the raw accumulators of this K range: lane rows 4 fg + e of fragment i, 8 consecutive
    // columns n0 + wn * 128 + 8 fr .. + 7 (two 16-byte stores; 16 lanes = 512 B of a row)
    int32_t* dst = g.part + (long)blockIdx.y * g.M * 512;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long row = m0 + wm * 64 + i * 16 + 4 * fg + e;
        if (FULL || row < g.M) {
          int4* d = reinterpret_cast<int4*>(dst + row * 512 + n0 + wn * 128 + 8 * fr);
          d[0] = make_int4(acc[i][0][e], acc[i][1][e], acc[i][2][e], acc[i][3][e]);
          d[1] = make_int4(acc[i][4][e], acc[i][5][e], acc[i][6][e], acc[i][7][e]);
        }
      }
    return;
  } else {
  if (FAULT && (g.fault.kind == FK_INPUT || g.fault.kind == FK_WEIGHT)) {
    // exact integer correction of the accumulators for one bit-flipped int8 operand
    // (the perturbation the reference propagates through the MatMul, inject_utils/layers.py)
    const FaultArgs& f = g.fault;
    const bool inp = f.kind == FK_INPUT;
    const int8_t orig = inp ? g.A[f.row * g.lda + f.col] : g.W[f.row * g.ldw + f.col];
    const int delta = (int)(int8_t)(orig ^ (1 << f.bit)) - (int)orig;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long row = m0 + wm * 64 + i * 16 + 4 * fg + e;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const long col = n0 + wn * 128 + 8 * fr + j;
          if (row < g.M) {
            if (inp && row == f.row && col >= f.lo && col < f.hi)
              acc[i][j][e] += delta * (int)g.W[col * g.ldw + f.col];
            if (!inp && col == f.row && row >= f.lo && row < f.hi)
              acc[i][j][e] += delta * (int)g.A[row * g.lda + f.col];
          }
        }
      }
  }

  // ---- y = ((float(acc) * sa[m]) * sw[n]) + b[n] (relu for the FFN1 epilogues), computed
  // once in place of the accumulators; lane: rows 4*fg + e of fragment i, columns cb + j
  // (j < 8) with cb = n0 + wn*128 + 8*fr ------------------------------------------------
  float y[4][8][4];
  {
    if constexpr (!PF) epi_loads();
    float swc[8], bc[8];
    const float4 s0 = sw4[0], s1 = sw4[1], b0 = b4[0], b1 = b4[1];
    swc[0] = s0.x; swc[1] = s0.y; swc[2] = s0.z; swc[3] = s0.w;
    swc[4] = s1.x; swc[5] = s1.y; swc[6] = s1.z; swc[7] = s1.w;
    bc[0] = b0.x; bc[1] = b0.y; bc[2] = b0.z; bc[3] = b0.w;
    bc[4] = b1.x; bc[5] = b1.y; bc[6] = b1.z; bc[7] = b1.w;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float sr = sra[i][e];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = ((float)acc[i][j][e] * sr) * swc[j] + bc[j];
          y[i][j][e] = (EPI == RE_RELU_PMAX || EPI == RE_RELU_QUANT_PMAX) ? (v > 0.0f ? v : 0.0f) : v;
        }
      }
    if (FAULT && g.fault.kind == FK_OUTPUT) {   // RANDOM fault models: one MatMul output value replaced
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const long row = m0 + wm * 64 + i * 16 + 4 * fg + e;
            if (row == g.fault.row && n0 + cl + j == g.fault.col) {
              const float v = g.fault.value + bc[j];
              y[i][j][e] = (EPI == RE_RELU_PMAX || EPI == RE_RELU_QUANT_PMAX) ? (v > 0.0f ? v : 0.0f) : v;
            }
          }
    }
  }
  auto yv = [&](int i, int j, int e) { return y[i][j][e]; };
  QTX_STAMP(3);

  if constexpr (EPI == RE_RES_LN) {
    // Two halves of 64 rows (fragments 2h, 2h+1 of both row halves): every wave stages its
    // 32 x 128 block of y as fp32 rows in LDS (rows 0..31 of the half in st0, 32..63 in
    // st1), then each wave takes 8 whole rows in two groups of 4: x = res + y (the residual
    // rows loaded in the canonical lane layout, the next group's while this one works),
    // writes x, LayerNorm in the canonical order (ln_rows512) and per-token quant (or fp32
    // out).  Staging y without the residual frees its registers before the LN work.
    float ga[2][4], gb[2][4];                     // LN parameters: loaded once
    ln_params512(g.ln_a, g.ln_b, lane, ga, gb);
    auto lds_row = [&](int r) {                   // LDS row r of the staged half (0..63)
      return reinterpret_cast<float*>(r < 32 ? st0 : st1) + (r & 31) * R_BN;
    };
    // global row of LDS row r in half hh: rows wm*64 + (2hh + ii)*16 + rem
    auto grow = [&](int hh, int r) { return m0 + (r >> 5) * 64 + (2 * hh + ((r >> 4) & 1)) * 16 + (r & 15); };
    float4 rb[4][2];
    auto load_res = [&](int hh, int grp) {
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int row = min(grow(hh, 8 * wave + 4 * grp + r4), g.M - 1);
#pragma unroll
        for (int c = 0; c < 2; ++c)
          rb[r4][c] = *reinterpret_cast<const float4*>(g.res + (long)row * R_BN + 4 * (lane + 64 * c));
      }
    };
    load_res(0, 0);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 2 * hh + ii;
          float4* dp = reinterpret_cast<float4*>(lds_row(wm * 32 + ii * 16 + 4 * fg + e) + cl);
          dp[0] = make_float4(yv(i, 0, e), yv(i, 1, e), yv(i, 2, e), yv(i, 3, e));
          dp[1] = make_float4(yv(i, 4, e), yv(i, 5, e), yv(i, 6, e), yv(i, 7, e));
        }
      __syncthreads();
#pragma unroll
      for (int grp = 0; grp < 2; ++grp) {
        const bool stg = hh == 0 && grp == 0;     // diagnostic stamps (QTX_STAMPS builds)
        if (stg) QTX_STAMP(5);
        float v[4][2][4];
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const float4 t4 = *reinterpret_cast<const float4*>(lds_row(8 * wave + 4 * grp + r4) + 4 * (lane + 64 * c));
            v[r4][c][0] = rb[r4][c].x + t4.x; v[r4][c][1] = rb[r4][c].y + t4.y;
            v[r4][c][2] = rb[r4][c].z + t4.z; v[r4][c][3] = rb[r4][c].w + t4.w;
          }
        // the next group's residual, issued before this group's stores
        if (grp == 0) load_res(hh, 1);
        else if (hh == 0) load_res(1, 0);
        if (stg) QTX_STAMP(6);
        const int rowb = grow(hh, 8 * wave + 4 * grp);   // 4 consecutive global rows
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4)
          if (FULL || rowb + r4 < g.M)
#pragma unroll
            for (int c = 0; c < 2; ++c)
              *reinterpret_cast<float4*>(g.xout + (long)(rowb + r4) * R_BN + 4 * (lane + 64 * c)) =
                  make_float4(v[r4][c][0], v[r4][c][1], v[r4][c][2], v[r4][c][3]);
        if (stg) QTX_STAMP(7);
        ln_rows512<4>(v, ga, gb);
        if (stg) QTX_STAMP(8);
        if (g.lnq) {
          uint32_t qd[4][2];
          float sc[4];
          quant_rows512<4>(v, qd, sc);
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4)
            if (FULL || rowb + r4 < g.M) {
              if constexpr (KP) {      // the next GEMM's A operand in the KP layout
                const long row = rowb + r4;
                *reinterpret_cast<uint32_t*>(g.lnq + kp_off(row, 4 * lane, R_BN)) = qd[r4][0];
                *reinterpret_cast<uint32_t*>(g.lnq + kp_off(row, 4 * (lane + 64), R_BN)) = qd[r4][1];
              } else {
                uint32_t* qr = reinterpret_cast<uint32_t*>(g.lnq + (long)(rowb + r4) * R_BN);
                qr[lane] = qd[r4][0];
                qr[lane + 64] = qd[r4][1];
              }
              if (lane == 0) g.lns[rowb + r4] = sc[r4];
            }
        } else {
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4)
            if (FULL || rowb + r4 < g.M)
#pragma unroll
              for (int c = 0; c < 2; ++c)
                *reinterpret_cast<float4*>(g.lnout + (long)(rowb + r4) * R_BN + 4 * (lane + 64 * c)) =
                    make_float4(v[r4][c][0], v[r4][c][1], v[r4][c][2], v[r4][c][3]);
        }
        if (stg) QTX_STAMP(9);
      }
      __syncthreads();                            // staging free for the next half
    }
    QTX_STAMP(2);
    return;
  }

  // ---- per-row absmax over the tile: 8 columns in the lane, the 16 lanes of the DPP row
  // (one row, 16 x 8 columns), then the 4 column waves through LDS (st0, free now) -------
  float* red = reinterpret_cast<float*>(st0);       // [4][128]
  float rmax[4][4];
  if constexpr (EPI == RE_RELU_QUANT_PMAX) {
    // the scale comes from the partial maxima of the whole row (all column tiles)
    if (tid < R_BM) {
      const int row = min(m0 + tid, g.M - 1);
      float m = g.pmax_in[row];
      for (int pidx = 1; pidx < g.pmax_n; ++pidx) m = fmaxf(m, g.pmax_in[(long)pidx * g.M + row]);
      red[tid] = m;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) rmax[i][e] = red[wm * 64 + i * 16 + 4 * fg + e];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float m = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(yv(i, j, e)));
        m = row16_max(m);
        if (fr == 0) red[wn * R_BM + wm * 64 + i * 16 + 4 * fg + e] = m;
      }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rl = wm * 64 + i * 16 + 4 * fg + e;
        rmax[i][e] = fmaxf(fmaxf(red[rl], red[R_BM + rl]), fmaxf(red[2 * R_BM + rl], red[3 * R_BM + rl]));
      }
  }
  QTX_STAMP(4);
  if constexpr (EPI == RE_RELU_PMAX) {
    if (wn == 0 && fr == 0)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm * 64 + i * 16 + 4 * fg + e;
          if (FULL || row < g.M) g.pmax_out[(long)t * g.M + row] = rmax[i][e];
        }
    QTX_STAMP(2);
    return;
  } else {
    // ---- per-token quantization rint(y / s): the quotient correctly rounded by div_cr
    // (shared reciprocal per row, 3 ops).  Its guard holds for a whole row when
    // rmax < 2^37: then |y| <= rmax < 2^60 and s < 2^30, while |y| < 2^-60 gives a quotient
    // below 2^-36 that rounds to 0 either way.  Otherwise (never in practice) every lane
    // of the wave takes the true division (uniform branch).
    float sc[4][4], inv[4][4];
    bool big = false;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc[i][e] = quant_scale(rmax[i][e], 127.0f);
        inv[i][e] = 1.0f / sc[i][e];
        big |= !(rmax[i][e] < 0x1p37f);
      }
    int8_t* ob = EPI == RE_QUANT ? g.out8 + (long)t * g.o8_ts : g.out8 + n0;
    // Stores widened to 16 bytes (the tail is store-issue-bound, not HBM-bound): lanes fr,
    // fr^1 hold columns 8fr..8fr+7 and the next 8 of the same rows; for each pair of rows
    // (e, e+1) the even lane sends its row-(e+1) half and receives the odd lane's row-e
    // half (one DPP lane swap per dword), so the even lane stores row e and the odd lane
    // row e+1, 16 consecutive bytes each: 8 dwordx4 stores per lane instead of 16 dwordx2.
    const bool odd = fr & 1;
    const int cw = wn * 128 + 16 * (fr >> 1);     // the pair's 16 columns in the tile
    auto swap1 = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true); };
    auto store_rows = [&](auto quot) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ep = 0; ep < 4; ep += 2) {
          uint2 pk[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int e = ep + h;
            float qv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) qv[j] = quot(yv(i, j, e), sc[i][e], inv[i][e]);
            pk[h] = make_uint2(pack4_codes<EPI == RE_RELU_QUANT_PMAX>(qv[0], qv[1], qv[2], qv[3]),
                               pack4_codes<EPI == RE_RELU_QUANT_PMAX>(qv[4], qv[5], qv[6], qv[7]));
          }
          const uint32_t r0 = swap1(odd ? pk[0].x : pk[1].x);
          const uint32_t r1 = swap1(odd ? pk[0].y : pk[1].y);
          const uint4 v = odd ? make_uint4(r0, r1, pk[1].x, pk[1].y) : make_uint4(pk[0].x, pk[0].y, r0, r1);
          const int row = m0 + wm * 64 + i * 16 + 4 * fg + ep + (odd ? 1 : 0);
          if (FULL || row < g.M) {
            if (KP && EPI == RE_RELU_QUANT_PMAX)   // FFN2's A operand in the KP layout
              *reinterpret_cast<uint4*>(g.out8 + kp_off(row, n0 + cw, g.ldo8)) = v;
            else
              *reinterpret_cast<uint4*>(ob + (long)row * g.ldo8 + cw) = v;
          }
        }
    };
    if (__builtin_expect(__ballot(big) != 0ull, 0))
      store_rows([](float a, float b, float) { return a / b; });
    else
      store_rows([](float a, float b, float y) { return div_cr(a, b, y); });
    if (wn == 0 && fr == 0) {
      float* osp = EPI == RE_QUANT ? g.os + (long)t * g.os_ts : g.os;
      if (EPI == RE_QUANT || t == 0)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = m0 + wm * 64 + i * 16 + 4 * fg + e;
            if (FULL || row < g.M) osp[row] = sc[i][e];
          }
    }
    QTX_STAMP(2);
  }
  }  // EPI != RE_PARTIAL
}

// The split-K RE_RES_LN epilogue: one wave per row — the ksplit int32 partials summed
// (exact), y = ((float(acc) * sa) * sw) + b, x = res + y (stored), then LayerNorm and the
// per-token quantization (KP out) or the fp32 LayerNorm output: the same arithmetic, in
// the same order, as k_gemm_row<RE_RES_LN>'s epilogue.
__global__ __launch_bounds__(256) void k_res_ln_partials(RowGemmArgs g) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + wave;
  if (row >= g.M) return;                          // whole wave: no barrier below
  int4 p[2];
  float4 r4[2], s4[2], b4[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int col = 4 * (lane + 64 * c);
    p[c] = make_int4(0, 0, 0, 0);
    for (int z = 0; z < g.ksplit; ++z) {
      const int4 t = *reinterpret_cast<const int4*>(g.part + ((long)z * g.M + row) * 512 + col);
      p[c].x += t.x; p[c].y += t.y; p[c].z += t.z; p[c].w += t.w;
    }
    r4[c] = *reinterpret_cast<const float4*>(g.res + row * 512 + col);
    s4[c] = *reinterpret_cast<const float4*>(g.sw + col);
    b4[c] = *reinterpret_cast<const float4*>(g.bias + col);
  }
  const float sr = g.sa[row];
  float v[1][2][4];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int pa[4] = {p[c].x, p[c].y, p[c].z, p[c].w};
    const float sw[4] = {s4[c].x, s4[c].y, s4[c].z, s4[c].w}, bb[4] = {b4[c].x, b4[c].y, b4[c].z, b4[c].w};
    const float rr[4] = {r4[c].x, r4[c].y, r4[c].z, r4[c].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) v[0][c][e] = rr[e] + (((float)pa[e] * sr) * sw[e] + bb[e]);
    *reinterpret_cast<float4*>(g.xout + row * 512 + 4 * (lane + 64 * c)) =
        make_float4(v[0][c][0], v[0][c][1], v[0][c][2], v[0][c][3]);
  }
  float ga[2][4], gb[2][4];
  ln_params512(g.ln_a, g.ln_b, lane, ga, gb);
  ln_rows512<1>(v, ga, gb);
  if (g.lnq) {
    uint32_t qd[1][2];
    float sc[1];
    quant_rows512<1>(v, qd, sc);
    *reinterpret_cast<uint32_t*>(g.lnq + kp_off(row, 4 * lane, 512)) = qd[0][0];
    *reinterpret_cast<uint32_t*>(g.lnq + kp_off(row, 4 * (lane + 64), 512)) = qd[0][1];
    if (lane == 0) g.lns[row] = sc[0];
  } else {
#pragma unroll
    for (int c = 0; c < 2; ++c)
      *reinterpret_cast<float4*>(g.lnout + row * 512 + 4 * (lane + 64 * c)) =
          make_float4(v[0][c][0], v[0][c][1], v[0][c][2], v[0][c][3]);
  }
}

hipError_t launch_gemm_row(const RowGemmArgs& g, hipStream_t st) {
  if (g.M <= 0) return hipSuccess;
  if (g.N % R_BN || g.K % R_BK || g.K <= 0 || (g.lda % 16) || (g.ldw % 16))
    return hipErrorInvalidValue;
  if (g.epi == RE_RES_LN && g.N != R_BN) return hipErrorInvalidValue;
  if (g.kp && (g.fault.kind != FK_NONE || g.K % 256)) return hipErrorInvalidValue;
  const dim3 grid((g.N / R_BN) * ((g.M + R_BM - 1) / R_BM)), block(512);
  const bool full = g.M % R_BM == 0;
  if (g.epi == RE_RES_LN && g.kp && g.part && g.ksplit > 1 && g.fault.kind == FK_NONE) {
    // split K: ksplit x the workgroups of a small M, then the row-wise epilogue
    if ((g.K / 64) % (4 * g.ksplit)) return hipErrorInvalidValue;
    const dim3 gs(grid.x, g.ksplit);
    if (full) k_gemm_row<RE_PARTIAL, true, false, true><<<gs, block, 0, st>>>(g);
    else k_gemm_row<RE_PARTIAL, false, false, true><<<gs, block, 0, st>>>(g);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    k_res_ln_partials<<<dim3((g.M + 3) / 4), dim3(256), 0, st>>>(g);
    return hipGetLastError();
  }
#define QTX_ROW_LAUNCH(E)                                                                      \
  (g.fault.kind != FK_NONE ? (k_gemm_row<E, false, true, false><<<grid, block, 0, st>>>(g), 0)   \
   : g.kp ? (full ? (k_gemm_row<E, true, false, true><<<grid, block, 0, st>>>(g), 0)             \
                  : (k_gemm_row<E, false, false, true><<<grid, block, 0, st>>>(g), 0))            \
   : full ? (k_gemm_row<E, true, false, false><<<grid, block, 0, st>>>(g), 0)                    \
          : (k_gemm_row<E, false, false, false><<<grid, block, 0, st>>>(g), 0))
  switch (g.epi) {
    case RE_QUANT: QTX_ROW_LAUNCH(RE_QUANT); break;
    case RE_RES_LN: QTX_ROW_LAUNCH(RE_RES_LN); break;
    case RE_RELU_PMAX: QTX_ROW_LAUNCH(RE_RELU_PMAX); break;
    case RE_RELU_QUANT_PMAX: QTX_ROW_LAUNCH(RE_RELU_QUANT_PMAX); break;
    default: return hipErrorInvalidValue;
  }
#undef QTX_ROW_LAUNCH
  return hipGetLastError();
}

// W [N, K] row-major -> KP layout with the per-512-tile LDS column order of k_gemm_row:
// packed row rho of tile t holds W row t*512 + (rho & ~127) + 8 (rho & 15) + ((rho >> 4) & 7).
// One thread per 16-byte chunk.
__global__ void k_pack_w_kp(const int8_t* W, int N, int K, int8_t* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;   // chunk index
  const long nch = (long)N * (K / 16);
  if (i >= nch) return;
  const int rho_g = (int)(i / (K / 16)), kc16 = (int)(i % (K / 16));
  const int t = rho_g / 512, rho = rho_g % 512;
  const int n = t * 512 + (rho & ~127) + 8 * (rho & 15) + ((rho >> 4) & 7);
  *reinterpret_cast<uint4*>(out + kp_off(rho_g, 16L * kc16, K)) =
      *reinterpret_cast<const uint4*>(W + (long)n * K + 16L * kc16);
}

hipError_t launch_pack_w_kp(const int8_t* W, int N, int K, int8_t* out, hipStream_t st) {
  if (N % 512 || K % 64) return hipErrorInvalidValue;
  const long nch = (long)N * (K / 16);
  k_pack_w_kp<<<dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, st>>>(W, N, K, out);
  return hipGetLastError();
}

}  // namespace qtx
