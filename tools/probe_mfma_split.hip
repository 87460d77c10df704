// probe_mfma_split.hip — diagnostic (not shipped): with two waves per SIMD issuing
// v_mfma_i32_16x16x64_i8 with NV independent VALU after each, does giving the arbitration
// winners (waves 0-3) more of the MFMAs than the losers (waves 4-7) shorten the SIMD's
// time for the same total?  Per SIMD 128 MFMAs per round (the weight-stationary GEMMs'
// 32-row block), split W:L between the winner and the loser; time = the slowest wave.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma_split tools/probe_mfma_split.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));

template <int NV>
__device__ __forceinline__ void step(v4i& acc, const v4i& w, const v4i& a, float (&v)[8], int m) {
  asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc) : "v"(w), "v"(a));
#pragma unroll
  for (int i = 0; i < NV; ++i)
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[(m * NV + i) & 7]) : "v"(v[(m + i + 3) & 7]), "v"(v[(i + 5) & 7]));
}

template <int NV, int WIN>
__global__ __launch_bounds__(512) void k(int rounds, const v4i* rnd, float* sink, unsigned long long* out) {
  const int tid = threadIdx.x, wave = tid >> 6;
  const v4i w = rnd[(blockIdx.x * 512 + tid) * 2], a = rnd[(blockIdx.x * 512 + tid) * 2 + 1];
  v4i acc[4] = {};
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = tid * (i + 1) * 1e-5f;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < rounds; ++r) {
    if (wave < 4) {
#pragma unroll
      for (int m = 0; m < WIN; ++m) step<NV>(acc[m & 3], w, a, v, m);
    } else {
#pragma unroll
      for (int m = 0; m < 128 - WIN; ++m) step<NV>(acc[m & 3], w, a, v, m);
    }
    __syncthreads();                     // the block boundary of the GEMMs
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += v[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) s += (float)(acc[i][0] ^ acc[i][3]);
  asm volatile("" ::"v"(s));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (s == 1234.5f) sink[tid] = s;
  if ((tid & 63) == 0) out[blockIdx.x * 8 + wave] = t1 - t0;
}

template <int NV, int WIN>
void run(int rounds, const v4i* rnd, float* sink, unsigned long long* d) {
  (void)hipMemset(d, 0, 256 * 8 * 8);
  for (int w = 0; w < 2; ++w) k<NV, WIN><<<256, 512>>>(rounds, rnd, sink, d);
  (void)hipDeviceSynchronize();
  unsigned long long h[256 * 8];
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  double c = 0;
  for (int i = 0; i < 256; ++i) {
    unsigned long long mx = 0;
    for (int q = 0; q < 8; ++q) mx = h[i * 8 + q] > mx ? h[i * 8 + q] : mx;
    c += mx;
  }
  printf("NV=%d winner %3d / loser %3d MFMAs: %.0f cycles per 128-MFMA round per SIMD\n", NV, WIN, 128 - WIN,
         c / 256 / rounds);
}

int main() {
  const int rounds = 100;
  unsigned long long* d; float* sink; v4i* rnd;
  (void)hipMalloc(&d, 256 * 8 * 8); (void)hipMalloc(&sink, 4096 * 4); (void)hipMalloc(&rnd, 256 * 512 * 2 * 16);
  {
    const size_t n = 256 * 512 * 2 * 4;
    int* h = (int*)malloc(n * 4);
    unsigned x = 5;
    for (size_t i = 0; i < n; ++i) { x = x * 1664525u + 1013904223u; h[i] = (int)x; }
    (void)hipMemcpy(rnd, h, n * 4, hipMemcpyHostToDevice);
    free(h);
  }
  run<5, 64>(rounds, rnd, sink, d);
  run<5, 72>(rounds, rnd, sink, d);
  run<5, 80>(rounds, rnd, sink, d);
  run<5, 88>(rounds, rnd, sink, d);
  run<2, 64>(rounds, rnd, sink, d);
  run<2, 80>(rounds, rnd, sink, d);
  return 0;
}
