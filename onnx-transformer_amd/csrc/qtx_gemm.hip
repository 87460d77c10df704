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

}  // namespace qtx
