// probe_mfma_1wave.hip — diagnostic (not shipped): is one wave per SIMD enough to keep
// v_mfma_i32_16x16x64_i8 at its full rate, and does it matter where the operands and the
// accumulators live?  (tools/probe_mfma_order.hip measured ≈ 27 cycles per MFMA for ONE
// wave per SIMD with the B operand in AGPRs, ≈ 13.8 for two waves with VGPR operands.)
// Independent accumulators, operands in registers, asm MFMAs, 256 workgroups; time = the
// workgroup's slowest wave, stamped after its accumulators are consumed:
//   V1    1 wave / SIMD: A, B in VGPRs, 8 accumulators in VGPRs
//   V1A   1 wave / SIMD: A, B in VGPRs, 8 accumulators in AGPRs
//   V1B   1 wave / SIMD: src0 (the weight fragment) in AGPRs (the k_gemm_wsa shape)
//   V1C   1 wave / SIMD: src1 in AGPRs
//   V1_16 1 wave / SIMD: as V1 with 16 accumulators
//   V2    2 waves / SIMD: as V1 (reference)
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma_1wave tools/probe_mfma_1wave.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));

template <int MODE>
__device__ __forceinline__ void mf(v4i& acc, const v4i& w, const v4i& a) {
  if constexpr (MODE == 1)        // accumulator in AGPRs
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(acc) : "v"(w), "v"(a));
  else if constexpr (MODE == 2)   // src0 (the weight fragment, as the kernels pass it) in AGPRs
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(a));
  else if constexpr (MODE == 3)   // src1 in AGPRs
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(w));
  else
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc) : "v"(w), "v"(a));
}

template <int MODE, int NACC>
__global__ void k(int rounds, const v4i* rnd, int* sink, unsigned long long* out) {
  const int tid = threadIdx.x;
  v4i w[8], a[2];
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = rnd[(blockIdx.x * blockDim.x + tid) * 16 + j];
#pragma unroll
  for (int i = 0; i < 2; ++i) a[i] = rnd[(blockIdx.x * blockDim.x + tid) * 16 + 8 + i];
  v4i acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = v4i{0, 0, 0, 0};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < rounds; ++r) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < NACC; ++i) mf<MODE>(acc[i], w[(s + i) & 7], a[i & 1]);
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory");
  int s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s ^= acc[i][0] ^ acc[i][3];
  asm volatile("" ::"v"(s));                     // the stream has retired before the stamp
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (s == 0x1234567) sink[tid] = s;
  if ((tid & 63) == 0) out[blockIdx.x * 8 + (tid >> 6)] = t1 - t0;   // every wave
}

int main() {
  const int grid = 256, rounds = 400;
  unsigned long long* d; int* sink; v4i* rnd;
  hipMalloc(&d, grid * 8 * 8); hipMalloc(&sink, 4096 * 4);
  const size_t nr = 512 * 256 * 16;
  hipMalloc(&rnd, nr * 16);
  {
    int* h = (int*)malloc(nr * 16);
    unsigned x = 99;
    for (size_t i = 0; i < nr * 4; ++i) { x = x * 1664525u + 1013904223u; h[i] = (int)x; }
    hipMemcpy(rnd, h, nr * 16, hipMemcpyHostToDevice);
    free(h);
  }
  struct M { const char* name; int threads; int nacc; void (*f)(int, const v4i*, int*, unsigned long long*); };
  M modes[] = {
      {"V1    1 wave/SIMD, VGPR operands, 8 VGPR accumulators ", 256, 8, k<0, 8>},
      {"V1A   1 wave/SIMD, VGPR operands, 8 AGPR accumulators ", 256, 8, k<1, 8>},
      {"V1B   1 wave/SIMD, B in AGPRs,    8 VGPR accumulators ", 256, 8, k<2, 8>},
      {"V1C   1 wave/SIMD, src1 in AGPRs, 8 VGPR accumulators ", 256, 8, k<3, 8>},
      {"V1_16 1 wave/SIMD, VGPR operands, 16 VGPR accumulators", 256, 16, k<0, 16>},
      {"V2    2 waves/SIMD, VGPR operands, 8 VGPR accumulators", 512, 8, k<0, 8>},
  };
  for (const M& m : modes) {
    hipMemset(d, 0, grid * 8 * 8);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(m.f, dim3(grid), dim3(m.threads), 0, 0, rounds, rnd, sink, d);
    hipDeviceSynchronize();
    unsigned long long h[256 * 8];
    hipMemcpy(h, d, grid * 8 * 8, hipMemcpyDeviceToHost);
    double c = 0;                                  // the workgroup's slowest wave
    for (int i = 0; i < grid; ++i) {
      unsigned long long mx = 0;
      for (int w = 0; w < 8; ++w) mx = h[i * 8 + w] > mx ? h[i * 8 + w] : mx;
      c += mx;
    }
    c /= grid;
    const double per_simd = (double)rounds * 8 * m.nacc * (m.threads / 256);   // MFMAs per SIMD
    printf("%s: %.1f cycles per MFMA per SIMD\n", m.name, c / per_simd);
  }
  return 0;
}
