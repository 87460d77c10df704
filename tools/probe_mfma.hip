// probe_mfma.hip — diagnostic (not shipped): i8 MFMA issue rate and the shader clock under
// an MFMA-dense load (v_mfma_i32_16x16x64_i8, 32 independent accumulators per wave).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma tools/probe_mfma.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_mfma(int iters, unsigned long long* out, int* sink,
                                                     const v4i* rnd) {
  const int lane = threadIdx.x & 63;
  v4i a = rnd[(blockIdx.x * 64 * WAVES + threadIdx.x) * 2];
  v4i b = rnd[(blockIdx.x * 64 * WAVES + threadIdx.x) * 2 + 1];
  v4i acc[32];
  for (int i = 0; i < 32; ++i) acc[i] = v4i{0, 0, 0, 0};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
    a = a ^ (acc[0] * 0x9e3779b1);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  int s = 0;
  for (int i = 0; i < 32; ++i) s += acc[i][0];
  if (s == 0x1234567) sink[threadIdx.x] = s;
  if (threadIdx.x == 0) {
    out[blockIdx.x * 2] = t1 - t0;
    out[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

template <int WAVES>
void run(int grid, int iters, bool zero) {
  unsigned long long* d; int* s; v4i* rnd;
  hipMalloc(&d, grid * 16); hipMalloc(&s, 4096);
  const size_t nr = (size_t)grid * 64 * WAVES * 2;
  hipMalloc(&rnd, nr * 16);
  {
    v4i* h = (v4i*)malloc(nr * 16);
    unsigned x = 12345;
    for (size_t i = 0; i < nr * 4; ++i) { x = x * 1664525u + 1013904223u; ((int*)h)[i] = zero ? 0 : (int)x; }
    hipMemcpy(rnd, h, nr * 16, hipMemcpyHostToDevice);
    free(h);
  }
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int w = 0; w < 20; ++w) k_mfma<WAVES><<<grid, 64 * WAVES>>>(iters, d, s, rnd);
  hipEventRecord(e0);
  const int reps = 20;
  for (int w = 0; w < reps; ++w) k_mfma<WAVES><<<grid, 64 * WAVES>>>(iters, d, s, rnd);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[2048];
  hipMemcpy(h, d, grid * 16, hipMemcpyDeviceToHost);
  double ticks = 0, real = 0;
  for (int b = 0; b < grid; ++b) { ticks += h[2 * b]; real += h[2 * b + 1]; }
  ticks /= grid; real /= grid;
  const double mfma_per_wave = 32.0 * iters;
  const double ops = 2.0 * 16 * 16 * 64 * mfma_per_wave * WAVES * grid;
  printf("%s waves/WG %d grid %d: clock %.0f MHz, %.1f cyc per MFMA per SIMD, %.1f TOPS (%.1f%% of 5033)\n",
         zero ? "zero  " : "random", WAVES, grid, ticks / (real / 100.0), ticks / (mfma_per_wave * WAVES / 4.0),
         ops / (ms / reps * 1e-3) / 1e12, ops / (ms / reps * 1e-3) / 1e12 / 5033 * 100);
  hipFree(d); hipFree(s); hipFree(rnd);
}

int main() {
  run<8>(256, 4000, true);
  run<8>(256, 4000, false);
  run<8>(256, 20000, false);
  run<8>(256, 4000, true);
  return 0;
}
