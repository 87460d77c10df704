// probe_fma_chain.hip — diagnostic (not shipped): cycles per step of a dependent v_fmac_f32
// chain in ONE wave on an otherwise idle CU (the decode attention's PV chain, k_dec_attn),
// alone and with the chain's per-key companions (v_cvt_f32_i32 + v_mul_f32 of an
// independent value) interleaved, and with the operands coming from LDS as in the kernel.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_fma_chain tools/probe_fma_chain.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void k_chain(const float* in, float* out, long long* cyc, int n) {
  __shared__ float P[1024], S[1024];
  __shared__ signed char V[1024 * 64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) { P[i] = in[i] * 1e-3f; S[i] = in[i + 1024] * 1e-3f; }
  for (int i = lane; i < 1024 * 64; i += 64) V[i] = (signed char)(i * 7);
  __syncthreads();
  float acc = 0.0f, p = in[lane], s = in[lane + 64];
  int v = (int)in[lane + 128];
  const long long t0 = clock64();
  if (MODE == 0) {                       // bare dependent chain
#pragma unroll 16
    for (int j = 0; j < n; ++j) acc = fmaf(p, s, acc);
  } else if (MODE == 1) {                // + an independent cvt and mul per step
#pragma unroll 16
    for (int j = 0; j < n; ++j) acc = fmaf(p, (float)(v + j) * s, acc);
  } else {                               // the kernel's loop: P, S, V from LDS
#pragma unroll 8
    for (int j = 0; j < n; ++j) acc = fmaf(P[j & 1023], (float)V[(j & 1023) * 64 + lane] * S[j & 1023], acc);
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float *in, *out;
  long long* cyc;
  hipMalloc(&in, 4096 * 4); hipMalloc(&out, 256 * 64 * 4); hipMalloc(&cyc, 256 * 8);
  float h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (float)(i % 97) * 0.25f + 1.0f;
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const int n = 1024;
  const char* names[3] = {"bare fmac chain", "fmac + cvt + mul", "kernel loop (LDS operands)"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      if (mode == 0) k_chain<0><<<256, 64>>>(in, out, cyc, n);
      if (mode == 1) k_chain<1><<<256, 64>>>(in, out, cyc, n);
      if (mode == 2) k_chain<2><<<256, 64>>>(in, out, cyc, n);
    }
    hipDeviceSynchronize();
    long long c[256];
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    long long mn = c[0], mx = c[0];
    for (int i = 1; i < 256; ++i) { mn = c[i] < mn ? c[i] : mn; mx = c[i] > mx ? c[i] : mx; }
    printf("%-28s: %.1f - %.1f cycles per step (one wave per CU, %d steps)\n", names[mode],
           (double)mn / n, (double)mx / n, n);
  }
  return 0;
}
