// probe_mfma_fill.hip — diagnostic (not shipped): how many independent VALU instructions
// ride free beside the int8 MFMA stream, per multiply-accumulate, for the two int8 shapes?
// 512-thread workgroups (2 waves per SIMD, both issuing), operands in registers, asm MFMAs
// on 4 independent accumulators, N v_fma_f32 fillers (8 independent chains) after each
// MFMA.  Prints ticks (shader cycles) per MFMA per SIMD and per 1k MACs for N = 0..16; time
// = the workgroup's slowest wave, stamped after its accumulators are consumed.
//   v_mfma_i32_16x16x64_i8: 16,384 MACs;  v_mfma_i32_32x32x32_i8: 32,768 MACs
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma_fill tools/probe_mfma_fill.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int BIG, int NV>
__global__ __launch_bounds__(512) void k(int rounds, const v4i* rnd, float* sink, unsigned long long* out) {
  // blockDim.x = 512: two waves per SIMD; 256: one
  const int tid = threadIdx.x;
  const v4i w = rnd[(blockIdx.x * 512 + tid) * 2], a = rnd[(blockIdx.x * 512 + tid) * 2 + 1];
  v4i acc4[4] = {};
  v16i acc16[4] = {};
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = tid * (i + 1) * 1e-5f;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < rounds; ++r) {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if constexpr (BIG)
        asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %2, %0" : "+v"(acc16[m & 3]) : "v"(w), "v"(a));
      else
        asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc4[m & 3]) : "v"(w), "v"(a));
#pragma unroll
      for (int i = 0; i < NV; ++i)
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[(m * NV + i) & 7]) : "v"(v[(m + i + 3) & 7]), "v"(v[(i + 5) & 7]));
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += v[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) s += (float)(acc4[i][0] ^ acc16[i][5]);
  asm volatile("" ::"v"(s));                     // the streams have retired before the stamp
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (s == 1234.5f) sink[tid] = s;
  if ((tid & 63) == 0) out[blockIdx.x * 8 + (tid >> 6)] = t1 - t0;   // every wave
}

static int g_threads = 512;
template <int BIG, int NV>
double run(int rounds, const v4i* rnd, float* sink, unsigned long long* d) {
  (void)hipMemset(d, 0, 256 * 8 * 8);
  for (int w = 0; w < 2; ++w) k<BIG, NV><<<256, g_threads>>>(rounds, rnd, sink, d);
  (void)hipDeviceSynchronize();
  unsigned long long h[256 * 8];
  (void)hipMemcpy(h, d, 256 * 8 * 8, hipMemcpyDeviceToHost);
  double c = 0;                                    // the workgroup's slowest wave
  for (int i = 0; i < 256; ++i) {
    unsigned long long mx = 0;
    for (int w = 0; w < 8; ++w) mx = h[i * 8 + w] > mx ? h[i * 8 + w] : mx;
    c += mx;
  }
  return c / 256 / (rounds * 16.0 * (g_threads / 256));   // ticks per MFMA per SIMD
}

template <int BIG, int... NV>
void sweep(int rounds, const v4i* rnd, float* sink, unsigned long long* d) {
  const double macs = BIG ? 32768 : 16384;
  ((printf("%s waves/SIMD %d N=%d: %.2f ticks per MFMA, %.3f per 1k MACs\n", BIG ? "32x32x32" : "16x16x64", g_threads / 256, NV,
           run<BIG, NV>(rounds, rnd, sink, d), run<BIG, NV>(rounds, rnd, sink, d) / macs * 1000)), ...);
}

int main() {
  const int rounds = 200;
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
  for (int t : {512, 256}) {
    g_threads = t;
    sweep<0, 0, 1, 2, 3, 4, 6, 8>(rounds, rnd, sink, d);
    sweep<1, 0, 2, 4, 6, 8, 12, 16>(rounds, rnd, sink, d);
  }
  return 0;
}
