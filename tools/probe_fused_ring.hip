// probe_fused_ring.hip — diagnostic (not shipped): the weight-stream floor of a fused
// post-attention row-block kernel (O -> FFN1 (row-max pass + recompute) -> FFN2, SURVEY §7
// "hard parts"), measured as a skeleton: the real weight stream of one
// 64-row block (Wo 256 KB, W1 twice 2 MB, W2 1 MB = 3.25 MB) through a 3-slot LDS-DMA ring
// of 32 KB slots (one 64-byte K step of 512 weight rows), consumed by the MFMAs the block
// needs (8 waves, each 64 rows x 64 columns per slot: 16 v_mfma_i32_16x16x64_i8), no
// epilogue arithmetic.  One 512-thread workgroup per CU, BLK blocks each (cfg3: M = 32768
// rows = 512 blocks of 64 -> 2 per CU).  Prefetch distance 2 (slot s+2 issued while s is
// consumed).  Reports the launch time and the per-CU fill rate.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_fused_ring tools/probe_fused_ring.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int SLOT = 32 * 1024;
constexpr int SLOTS_PER_BLOCK = 8 + 32 + 32 + 32;   // O, FFN1 pass 1, FFN1 pass 2, FFN2

__device__ __forceinline__ void dma16(const int8_t* gsrc, const uint8_t* lds_dst) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
}

template <bool MFMA, int NSLOT>
__global__ __launch_bounds__(512) void k_ring(const int8_t* W, long wbytes, int blocks, int* sink,
                                              unsigned long long* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[NSLOT * SLOT + 32 * 1024];
  uint8_t* const A = lds + NSLOT * SLOT;            // the block's A operand (64 rows x 512)
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long nsl = wbytes / SLOT;
  // slot j of the stream: 32 KB at ((j % nsl) * SLOT); wave w moves 4 x 1 KB of it
  auto issue = [&](int j) {
    const int8_t* src = W + (long)(j % nsl) * SLOT + wave * 4096 + lane * 16;
    uint8_t* dst = lds + (j % NSLOT) * SLOT + wave * 4096;
#pragma unroll
    for (int p = 0; p < 4; ++p) dma16(src + p * 1024, dst + p * 1024);
  };
  for (int i = tid; i < 32 * 1024 / 16; i += 512) reinterpret_cast<v4i*>(A)[i] = v4i{i, i ^ 5, i * 3, 7};
  const int total = blocks * SLOTS_PER_BLOCK;
  for (int j = 0; j < NSLOT - 1; ++j) issue(j);
  v4i acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int s = 0; s < total; ++s) {
    // slot s landed (this wave's part; the youngest operations are the DMAs of the next
    // NSLOT - 2 slots, 4 each)
    if (NSLOT == 3 && s + 1 < total) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (NSLOT == 4 && s + 2 < total) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (NSLOT == 4 && s + 1 < total) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (s + NSLOT - 1 < total) issue(s + NSLOT - 1);
    const uint8_t* slot = lds + (s % NSLOT) * SLOT;
    v4i b[4], a[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const v4i*>(slot + (wave * 4 + j) * 1024 + lane * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const v4i*>(A + ((s & 7) * 4 + i) * 1024 + lane * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (MFMA) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[j], a[i], acc[i][j], 0, 0, 0);
        else acc[i][j] += b[j] ^ a[i];
      }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  int sum = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) sum += acc[i][j][0] ^ acc[i][j][3];
  if (sum == 0x1234567) sink[tid] = sum;
  if (tid == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = r1 - r0; }
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const long wbytes = 3328L * 1024;                  // 3.25 MB: the block's weights
  int8_t* W; int* sink; unsigned long long* d;
  hipMalloc(&W, wbytes); hipMalloc(&sink, 4096); hipMalloc(&d, 4096 * 16);
  {
    int8_t* h = (int8_t*)malloc(wbytes);
    unsigned x = 7;
    for (long i = 0; i < wbytes; ++i) { x = x * 1664525u + 1013904223u; h[i] = (int8_t)(x >> 24); }
    hipMemcpy(W, h, wbytes, hipMemcpyHostToDevice);
    free(h);
  }
  printf("CUs %d\n", ncu);
  for (int mode = 0; mode < 4; ++mode)
    for (int blocks : {2}) {
      const int grid = ncu;
      auto launch = [&]() {
        if (mode == 0) k_ring<true, 3><<<grid, 512>>>(W, wbytes, blocks, sink, d);
        else if (mode == 1) k_ring<false, 3><<<grid, 512>>>(W, wbytes, blocks, sink, d);
        else if (mode == 2) k_ring<true, 4><<<grid, 512>>>(W, wbytes, blocks, sink, d);
        else k_ring<false, 4><<<grid, 512>>>(W, wbytes, blocks, sink, d);
      };
      for (int w = 0; w < 3; ++w) launch();
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      const int reps = 10;
      for (int w = 0; w < reps; ++w) launch();
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      unsigned long long h[2 * 512];
      hipMemcpy(h, d, grid * 16, hipMemcpyDeviceToHost);
      double ticks = 0, real = 0;
      for (int b = 0; b < grid; ++b) { ticks += h[2 * b]; real += h[2 * b + 1]; }
      ticks /= grid; real /= grid;
      const double us = ms / reps * 1e3;
      const double bytes_cu = (double)blocks * SLOTS_PER_BLOCK * SLOT;
      printf("%s ring %d slots, blocks/CU %d: %.1f us per launch (in-kernel %.1f us, clock %.0f MHz), fill %.1f GB/s per CU;"
             " scaled to cfg3 (2 blocks/CU): %.1f us\n", mode % 2 == 0 ? "MFMA   " : "no-MFMA", mode < 2 ? 3 : 4, blocks, us,
             real / 100.0, ticks / (real / 100.0), bytes_cu / (real / 100.0 * 1e-6) / 1e9, us * 2 / blocks);
    }
  return 0;
}
