// qtx_ws.h — shared pieces of the weight-stationary K = 512 GEMMs (qtx_wsgemm.hip and the
// diagnostic-only variants in qtx_wsgemm_diag.hip): layout constants, raw buffer resources,
// s_waitcnt immediates and the asm MFMA statements with their hazard padding.
#pragma once
#include "qtx_common.h"
#include "qtx_kernels.h"

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

#ifdef QTX_DIAG
// qtx_wsgemm_diag.hip (diagnostic build only): the measured-negative weight-stationary
// variants the knobs select (QTX_WSQ=2/3/4, QTX_WSA2, QTX_WSY=0); hipErrorNotSupported when
// they select none
hipError_t launch_gemm_ws_diag(const RowGemmArgs& g, dim3 grid, hipStream_t st);
hipError_t launch_gemm_wsx_diag(const RowGemmArgs& a, int ng, hipStream_t st);
// k_gemm_wsq32 / k_gemm_wsy32 (RowGemmArgs kp = 4 / 5: W in the WS32 layout)
hipError_t launch_gemm_ws32_diag(const RowGemmArgs& g, dim3 grid, hipStream_t st);
hipError_t launch_gemm_wsy32_diag(const RowGemmArgs& a, int ng, hipStream_t st);
hipError_t launch_pack_w_ws32(const int8_t* W, int N, int K, int8_t* out, hipStream_t st);
#endif

}  // namespace qtx
