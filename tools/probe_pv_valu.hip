// probe_pv_valu.hip — diagnostic (not shipped): the encoder attention's PV (per wave and head:
// 16 queries x 64 dims x 128 keys, the sequential fma chain over the keys) on
//   MFMA  v_mfma_f32_16x16x4_f32 as k_attn_encq<true> runs it (32 steps x 4 dim tiles, one
//         ds_read_b128 of V per step), or on
//   DPP   the VALU: v_fmac_f32_dpp with row_newbcast:n — row r of the wave owns queries
//         4r..4r+3, lane n of the row dims 4n..4n+3; key k = 16 kt + n: P[4r + e][k] sits in
//         lane n of row r, register x[kt][e], and is broadcast to the row inside the fmac;
//         one ds_read_b128 (V row k, dims 4n..4n+3, the same 256 B for the 4 rows) per key.
//   MOV   as DPP with the broadcast as its own v_mov_b32_dpp (the compiler's form).
// 8 heads unrolled (the accumulators of every head live, as in the kernel; head h reads V
// 16 h floats further on, so the compiler cannot merge the heads), 512-thread workgroups
// (2 waves per SIMD), one per CU; time = the workgroup's slowest wave per head.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_pv_valu tools/probe_pv_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v4f __attribute__((ext_vector_type(4)));

#define FMAC_BC(N)                                                                            \
  case N:                                                                                     \
    asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:" #N " row_mask:0xf bank_mask:0xf"   \
                 : "+v"(acc) : "v"(x), "v"(v));                                                \
    break;
template <int N>
__device__ __forceinline__ void fmac_bc(float& acc, float x, float v) {
  switch (N) {
    FMAC_BC(0) FMAC_BC(1) FMAC_BC(2) FMAC_BC(3) FMAC_BC(4) FMAC_BC(5) FMAC_BC(6) FMAC_BC(7)
    FMAC_BC(8) FMAC_BC(9) FMAC_BC(10) FMAC_BC(11) FMAC_BC(12) FMAC_BC(13) FMAC_BC(14) FMAC_BC(15)
  }
}

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

template <int MODE>
__global__ __launch_bounds__(512) void k(const float* vin, float* sink, unsigned long long* out) {
  __shared__ __attribute__((aligned(16))) float Vf[128 * 64 + 8 * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  for (int i = tid; i < 128 * 64 + 8 * 16; i += 512) Vf[i] = vin[i % (128 * 64)];
  float x[8][4];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt)
#pragma unroll
    for (int e = 0; e < 4; ++e) x[kt][e] = (lane * 8 + kt * 4 + e) * (1.0f / 4096);
  v4f ctxm[8][4];     // MFMA: 8 heads x 4 dim tiles
  float ctx[8][16];   // VALU: 8 heads x (4 queries x 4 dims)
#pragma unroll
  for (int h = 0; h < 8; ++h) {
#pragma unroll
    for (int i = 0; i < 4; ++i) ctxm[h][i] = v4f{0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; ++i) ctx[h][i] = 0.0f;
  }
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  sfor<0, 8>([&](auto hc) {
    constexpr int h = decltype(hc)::value;
    if constexpr (MODE == 0) {
      const float* vrow = Vf + 16 * h + fg * 64 + 4 * fr;
#pragma unroll
      for (int s4 = 0; s4 < 32; ++s4) {
        const float pa = x[s4 >> 2][s4 & 3];
        const float4 vb = *reinterpret_cast<const float4*>(vrow + s4 * 256);
        const float vbs[4] = {vb.x, vb.y, vb.z, vb.w};
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          ctxm[h][dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa, vbs[dt], ctxm[h][dt], 0, 0, 0);
      }
    } else {
      sfor<0, 128>([&](auto kc) {
        constexpr int kk = decltype(kc)::value, kt = kk >> 4, n = kk & 15;
        const float4 vb = *reinterpret_cast<const float4*>(Vf + 16 * h + kk * 64 + 4 * fr);
        const float vv[4] = {vb.x, vb.y, vb.z, vb.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (MODE == 1) {
#pragma unroll
            for (int d = 0; d < 4; ++d) fmac_bc<n>(ctx[h][4 * e + d], x[kt][e], vv[d]);
          } else {
            const float b = __builtin_bit_cast(
                float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x[kt][e]), 0x150 + n, 0xf, 0xf, true));
#pragma unroll
            for (int d = 0; d < 4; ++d) ctx[h][4 * e + d] = __builtin_fmaf(b, vv[d], ctx[h][4 * e + d]);
          }
        }
      });
    }
  });
  float s = 0.0f;
#pragma unroll
  for (int h = 0; h < 8; ++h) {
#pragma unroll
    for (int i = 0; i < 4; ++i) s += (ctxm[h][i][0] + ctxm[h][i][1]) + (ctxm[h][i][2] + ctxm[h][i][3]);
#pragma unroll
    for (int i = 0; i < 16; ++i) s += ctx[h][i];
  }
  asm volatile("" ::"v"(s));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (s == 1234.5f) sink[tid] = s;
  if (lane == 0) out[blockIdx.x * 8 + wave] = t1 - t0;
}

int main() {
  float *vin, *sink;
  unsigned long long* d;
  (void)hipMalloc(&vin, 128 * 64 * 4);
  (void)hipMalloc(&sink, 512 * 4);
  (void)hipMalloc(&d, 256 * 8 * 8);
  {
    float h[128 * 64];
    for (int i = 0; i < 128 * 64; ++i) h[i] = ((i * 37) % 255 - 127) * 0.01f;
    (void)hipMemcpy(vin, h, sizeof h, hipMemcpyHostToDevice);
  }
  void (*fs[3])(const float*, float*, unsigned long long*) = {k<0>, k<1>, k<2>};
  const char* names[3] = {"MFMA v_mfma_f32_16x16x4_f32", "DPP  v_fmac_f32_dpp row_newbcast", "MOV  v_mov_b32_dpp + v_fmac_f32"};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int m = 0; m < 3; ++m) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(fs[m], dim3(256), dim3(512), 0, 0, vin, sink, d);
    (void)hipEventRecord(e0);
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(fs[m], dim3(256), dim3(512), 0, 0, vin, sink, d);
    (void)hipEventRecord(e1);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[256 * 8];
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    double c = 0;
    for (int i = 0; i < 256; ++i) {
      unsigned long long mx = 0;
      for (int q = 0; q < 8; ++q) mx = h[i * 8 + q] > mx ? h[i * 8 + q] : mx;
      c += mx;
    }
    printf("%s: %.0f cycles per head per SIMD (slowest wave), %.1f us per launch\n", names[m], c / 256 / 8,
           ms * 1e3 / 20);
  }
  return 0;
}
