// Diagnostic: in-kernel shader clock (s_memtime ticks / s_memrealtime at 100 MHz) for a
// short dependent-VALU kernel launched back to back, like the decode step's kernels.
//   hipcc --offload-arch=gfx950 -O3 -o tools/clock_probe tools/clock_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned long long* out, float* sink, int iters) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  float v = threadIdx.x;
  for (int i = 0; i < iters; ++i) v = v * 1.0000001f + 0.5f;
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[blockIdx.x * 2] = t1 - t0;
    out[blockIdx.x * 2 + 1] = r1 - r0;
  }
  if (v == 12345.0f) sink[0] = v;
}

int main() {
  unsigned long long* d;
  float* s;
  hipMalloc(&d, 256 * 16);
  hipMalloc(&s, 4);
  unsigned long long h[512];
  for (int iters : {1000, 10000, 100000}) {
    for (int grid : {32, 256}) {
      for (int rep = 0; rep < 50; ++rep) probe<<<grid, 256>>>(d, s, iters);
      hipDeviceSynchronize();
      hipMemcpy(h, d, grid * 16, hipMemcpyDeviceToHost);
      double ticks = 0, real = 0;
      for (int b = 0; b < grid; ++b) { ticks += h[2 * b]; real += h[2 * b + 1]; }
      printf("iters %6d grid %3d: %.0f ticks / %.2f us -> %.0f MHz\n", iters, grid,
             ticks / grid, real / grid / 100.0, ticks / (real / 100.0) );
    }
  }
  return 0;
}
