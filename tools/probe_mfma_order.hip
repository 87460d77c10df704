// probe_mfma_order.hip — diagnostic (not shipped): cycles per v_mfma_i32_16x16x64_i8 and the
// shader clock for the weight-stationary GEMMs' MFMA streams, operands in registers
// (random), asm MFMAs as the kernels issue them:
//   S8:  2 waves / SIMD, K-step major, 8 accumulators (2 row x 4 column fragments), W from 20
//        resident fragments + 3 "LDS" steps (registers here), 2 A fragments per step
//   I4:  the same MFMAs row-fragment major (4 accumulators live at a time)
//   A16: 1 wave / SIMD, W (64 fragments) in AGPRs, 8 accumulators per row fragment
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma_order tools/probe_mfma_order.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));

template <bool Z>
__device__ __forceinline__ void mf(v4i& acc, const v4i& w, const v4i& a) {
  if constexpr (Z) asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, 0" : "=&v"(acc) : "v"(w), "v"(a));
  else asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc) : "v"(w), "v"(a));
}
template <bool Z>
__device__ __forceinline__ void mfa(v4i& acc, const v4i& w, const v4i& a) {
  if constexpr (Z) asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, 0" : "=&v"(acc) : "a"(w), "v"(a));
  else asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(a));
}
__device__ __forceinline__ void settle(v4i& a) { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+v"(a)); }

// MODE 0: S8, 1: I4
template <int MODE>
__global__ __launch_bounds__(512) void k_two(int blocks, unsigned long long* out, int* sink, const v4i* rnd) {
  const int tid = threadIdx.x;
  v4i w[8][4], a[2][8];
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int j = 0; j < 4; ++j) w[s][j] = rnd[((blockIdx.x * 512 + tid) * 48 + s * 4 + j) & 0xfffff];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int s = 0; s < 8; ++s) a[i][s] = rnd[((blockIdx.x * 512 + tid) * 48 + 32 + i * 8 + s) & 0xfffff];
  v4i acc[2][4];
  int sum = 0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int b = 0; b < blocks; ++b) {
    if (MODE == 0) {
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (s == 0) mf<true>(acc[i][j], w[s][j], a[i][s]);
            else mf<false>(acc[i][j], w[s][j], a[i][s]);
          }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (s == 0) mf<true>(acc[i][j], w[s][j], a[i][s]);
            else mf<false>(acc[i][j], w[s][j], a[i][s]);
          }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) settle(acc[i][j]);
    sum += acc[0][0][0] ^ acc[1][3][1];
    a[0][0] ^= sum;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (sum == 0x1234567) sink[tid] = sum;
  if (tid == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = r1 - r0; }
}

__global__ __launch_bounds__(256, 1) void k_one(int blocks, unsigned long long* out, int* sink, const v4i* rnd) {
  const int tid = threadIdx.x;
  v4i w[8][8], a[8];
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) w[s][j] = rnd[((blockIdx.x * 256 + tid) * 80 + s * 8 + j) & 0xfffff];
#pragma unroll
  for (int s = 0; s < 8; ++s) a[s] = rnd[((blockIdx.x * 256 + tid) * 80 + 64 + s) & 0xfffff];
  v4i acc[8];
  int sum = 0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int b = 0; b < blocks; ++b) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (s == 0) mfa<true>(acc[j], w[s][j], a[s]);
        else mfa<false>(acc[j], w[s][j], a[s]);
      }
#pragma unroll
    for (int j = 0; j < 8; ++j) settle(acc[j]);
    sum += acc[0][0] ^ acc[7][1];
    a[0] ^= sum;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (sum == 0x1234567) sink[tid] = sum;
  if (tid == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = r1 - r0; }
}

int main() {
  const int grid = 256, blocks = 2000;
  unsigned long long* d; int* s; v4i* rnd;
  hipMalloc(&d, grid * 16); hipMalloc(&s, 4096);
  const size_t nr = 1 << 20;
  hipMalloc(&rnd, nr * 16);
  {
    int* h = (int*)malloc(nr * 16);
    unsigned x = 12345;
    for (size_t i = 0; i < nr * 4; ++i) { x = x * 1664525u + 1013904223u; h[i] = (int)x; }
    hipMemcpy(rnd, h, nr * 16, hipMemcpyHostToDevice);
    free(h);
  }
  for (int mode = 0; mode < 3; ++mode) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto launch = [&]() {
      if (mode == 0) k_two<0><<<grid, 512>>>(blocks, d, s, rnd);
      else if (mode == 1) k_two<1><<<grid, 512>>>(blocks, d, s, rnd);
      else k_one<<<grid, 256>>>(blocks, d, s, rnd);
    };
    for (int w = 0; w < 5; ++w) launch();
    hipEventRecord(e0);
    const int reps = 10;
    for (int w = 0; w < reps; ++w) launch();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[512];
    hipMemcpy(h, d, grid * 16, hipMemcpyDeviceToHost);
    double ticks = 0, real = 0;
    for (int b = 0; b < grid; ++b) { ticks += h[2 * b]; real += h[2 * b + 1]; }
    ticks /= grid; real /= grid;
    const double mfma_per_simd = 128.0 * blocks;     // every mode: 128 MFMAs per SIMD per block
    const double ops = 2.0 * 16 * 16 * 64 * mfma_per_simd * 4 * grid;
    const char* name[3] = {"S8  (2 waves/SIMD, K-step major)", "I4  (2 waves/SIMD, row-frag major)", "A16 (1 wave/SIMD, W in AGPRs)"};
    printf("%s: clock %.0f MHz, %.1f cyc per MFMA per SIMD, %.1f TOPS (%.1f%% of 5033)\n", name[mode],
           ticks / (real / 100.0), ticks / mfma_per_simd, ops / (ms / reps * 1e-3) / 1e12,
           ops / (ms / reps * 1e-3) / 1e12 / 5033 * 100);
  }
  return 0;
}
