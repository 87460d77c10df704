// probe_mfma_valu.hip — diagnostic (not shipped): how much VALU hides beside i8 MFMAs at two
// waves per SIMD (512-thread workgroups, one per CU), for the two int8 shapes:
//   v_mfma_i32_16x16x64_i8 (16 cycles, 16K MAC)  vs  v_mfma_i32_32x32x32_i8 (32 cycles, 32K MAC)
// Per loop iteration every wave issues 128K MAC of MFMAs (8 x 16x16x64 or 4 x 32x32x32) and
// 8*NV independent v_fma_f32, interleaved in a fixed order (inline asm, not reordered).
// MFMA-bound floor: 256 shader cycles per iteration (2 waves per SIMD x 128 cycles).
// SPLIT = 1: the same work per SIMD, specialised: waves 0-3 (one per SIMD) issue all the
// MFMAs (twice as many), waves 4-7 all the VALU (twice as many), no interleaving.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma_valu tools/probe_mfma_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int NV>
__device__ __forceinline__ void fillers(float (&f)[8], float x, float y) {
#pragma unroll
  for (int i = 0; i < NV; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[i & 7]) : "v"(x), "v"(y));
}

template <int SHAPE, int NV, int SPLIT = 0>
__global__ __launch_bounds__(512) void k_probe(int iters, unsigned long long* out, const int* rnd,
                                               int* sink) {
  const int t = blockIdx.x * 512 + threadIdx.x;
  v4i a = {rnd[4 * t], rnd[4 * t + 1], rnd[4 * t + 2], rnd[4 * t + 3]};
  v4i b = {rnd[4 * t + 5], rnd[4 * t + 6], rnd[4 * t + 7], rnd[4 * t + 8]};
  float f[8];
  for (int i = 0; i < 8; ++i) f[i] = (float)(t + i) * 1e-3f;
  const float x = 0.999f, y = 1e-3f;
  v4i acc4[8];
  v16i acc16[4];
  for (int i = 0; i < 8; ++i) acc4[i] = v4i{0, 0, 0, 0};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 16; ++j) acc16[i][j] = 0;
  __syncthreads();
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const bool mfma_wave = threadIdx.x < 256;
  if (SPLIT) {
    for (int it = 0; it < iters; ++it) {
      if (mfma_wave) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc4[i & 7]) : "v"(a), "v"(b));
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) fillers<NV>(f, x, y);
      }
    }
  }
  for (int it = 0; it < (SPLIT ? 0 : iters); ++it) {
    if constexpr (SHAPE == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc4[i]) : "v"(a), "v"(b));
        fillers<NV>(f, x, y);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %2, %0" : "+v"(acc16[i]) : "v"(a), "v"(b));
        fillers<2 * NV>(f, x, y);
      }
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  int s = 0;
  for (int i = 0; i < 8; ++i) s += acc4[i][0] + (int)f[i];
  for (int i = 0; i < 4; ++i) s += acc16[i][0];
  if (s == 0x1234567) sink[threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) out[t >> 6] = t1 - t0;
}

template <int SHAPE, int NV, int SPLIT = 0>
void run(int iters, const int* rnd, unsigned long long* d, int* s) {
  const int grid = 256;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 5; ++w) k_probe<SHAPE, NV, SPLIT><<<grid, 512>>>(iters, d, rnd, s);
  hipEventRecord(e0);
  const int reps = 10;
  for (int w = 0; w < reps; ++w) k_probe<SHAPE, NV, SPLIT><<<grid, 512>>>(iters, d, rnd, s);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  static unsigned long long h[256 * 8];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  double ticks = 0;
  for (int i = 0; i < grid * 8; ++i) ticks = h[i] > ticks ? h[i] : ticks;   // slowest wave
  const double macs = 131072.0 * iters * 8 * grid;
  printf("%s%s NV=%2d (VALU per 16K MAC): %6.1f cyc/iter (floor 256), %.0f TOPS\n",
         SHAPE ? "32x32x32" : "16x16x64", SPLIT ? " split" : "", NV, ticks / iters,
         2 * macs / (ms / reps * 1e-3) / 1e12);
}

int main() {
  int* rnd;
  unsigned long long* d;
  int* s;
  const size_t n = 256 * 512 * 4 + 16;
  hipMalloc(&rnd, n * 4);
  hipMalloc(&d, 256 * 8 * 8);
  hipMalloc(&s, 4096);
  int* hr = (int*)malloc(n * 4);
  unsigned x = 12345;
  for (size_t i = 0; i < n; ++i) { x = x * 1664525u + 1013904223u; hr[i] = (int)x; }
  hipMemcpy(rnd, hr, n * 4, hipMemcpyHostToDevice);
  const int it = 2000;
  run<0, 0, 1>(it, rnd, d, s);
  run<0, 2, 1>(it, rnd, d, s);
  run<0, 4, 1>(it, rnd, d, s);
  run<0, 5, 1>(it, rnd, d, s);
  run<0, 6, 1>(it, rnd, d, s);
  run<0, 8, 1>(it, rnd, d, s);
  run<0, 10, 1>(it, rnd, d, s);
  run<0, 12, 1>(it, rnd, d, s);
  run<0, 0>(it, rnd, d, s); run<1, 0>(it, rnd, d, s);
  run<0, 2>(it, rnd, d, s); run<1, 2>(it, rnd, d, s);
  run<0, 3>(it, rnd, d, s); run<1, 3>(it, rnd, d, s);
  run<0, 4>(it, rnd, d, s); run<1, 4>(it, rnd, d, s);
  run<0, 5>(it, rnd, d, s); run<1, 5>(it, rnd, d, s);
  run<0, 6>(it, rnd, d, s); run<1, 6>(it, rnd, d, s);
  run<0, 8>(it, rnd, d, s); run<1, 8>(it, rnd, d, s);
  run<0, 10>(it, rnd, d, s); run<1, 10>(it, rnd, d, s);
  return 0;
}
