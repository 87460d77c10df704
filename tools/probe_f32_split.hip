// probe_f32_split.hip — diagnostic (not shipped): can the f32 matrix work of one wave run
// beside the VALU work of the other wave of its SIMD?  (encoder attention: PV on
// v_mfma_f32_16x16x4_f32, softmax on VALU; DESIGN.md §4 "Where the encoder attention's time
// goes").  512-thread workgroups (waves w and w + 4 share a SIMD), one per CU, operands in
// registers.  Per SIMD the same total work in every mode:
//   MIX    both waves: NM/2 MFMAs interleaved with NV/2 VALU (one basic block)
//   SPLIT  waves 0-3: NM MFMAs only; waves 4-7: NV VALU only
//   MFMA   both waves: NM/2 MFMAs, no VALU          (the matrix work alone)
//   VALU   both waves: NV/2 VALU, no MFMA           (the vector work alone)
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_f32_split tools/probe_f32_split.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int NM = 256;      // f32 MFMAs per SIMD per round (2 waves' PV of one head: 2 x 128)
constexpr int NV = 2048;     // VALU per SIMD per round (2 waves' softmax: ~2 x 1,150)

template <int MODE>
__global__ __launch_bounds__(512) void k(int rounds, float* sink, unsigned long long* out) {
  const int tid = threadIdx.x, wave = tid >> 6;
  float a = tid * 1e-3f, b = 1.0f + tid * 1e-4f;
  v4f acc[4] = {v4f{0, 0, 0, 0}, v4f{0, 0, 0, 0}, v4f{0, 0, 0, 0}, v4f{0, 0, 0, 0}};
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = tid * (i + 1) * 1e-5f;
  const bool mf = MODE == 0 || MODE == 2 || (MODE == 1 && wave < 4);
  const bool va = MODE == 0 || MODE == 3 || (MODE == 1 && wave >= 4);
  const int nm = MODE == 1 ? NM : NM / 2, nv = MODE == 1 ? NV : NV / 2;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < rounds; ++r) {
    if (mf && va) {
      // MIX: nm MFMAs, nv / nm VALU (8 independent fma chains) after each
#pragma unroll 4
      for (int m = 0; m < NM / 2; ++m) {
        acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < NV / NM; ++i) v[i & 7] = __builtin_fmaf(v[i & 7], 0.999f, 1e-3f);
      }
    } else if (mf) {
      for (int m = 0; m < nm; m += 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u) acc[u & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[u & 3], 0, 0, 0);
      }
    } else if (va) {
      for (int i = 0; i < nv; i += 64) {
#pragma unroll
        for (int u = 0; u < 64; ++u) v[u & 7] = __builtin_fmaf(v[u & 7], 0.999f, 1e-3f);
      }
    }
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += v[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][3];
  if (s == 1234.5f) sink[tid] = s;
  if (tid == 0) out[blockIdx.x] = t1 - t0;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float* sink; unsigned long long* d;
  hipMalloc(&sink, 4096 * 4); hipMalloc(&d, 4096 * 8);
  const int rounds = 200;
  const char* name[4] = {"MIX   (both waves MFMA+VALU)", "SPLIT (MFMA wave + VALU wave)", "MFMA  alone", "VALU  alone"};
  for (int mode = 0; mode < 4; ++mode) {
    auto launch = [&]() {
      if (mode == 0) k<0><<<ncu, 512>>>(rounds, sink, d);
      else if (mode == 1) k<1><<<ncu, 512>>>(rounds, sink, d);
      else if (mode == 2) k<2><<<ncu, 512>>>(rounds, sink, d);
      else k<3><<<ncu, 512>>>(rounds, sink, d);
    };
    for (int w = 0; w < 3; ++w) launch();
    hipDeviceSynchronize();
    unsigned long long h[1024];
    hipMemcpy(h, d, ncu * 8, hipMemcpyDeviceToHost);
    double c = 0;
    for (int i = 0; i < ncu; ++i) c += h[i];
    c /= ncu;
    printf("%s: %.0f cycles per round per SIMD (MFMA floor %d at 32 cyc, VALU floor %d at 4 cyc)\n",
           name[mode], c / rounds, NM * 32, NV * 4);
  }
  return 0;
}
