// Diagnostic: the floor of one dependent decode-like kernel in a captured hipGraph.
// Each variant is a chain of 100 kernels replayed from a graph; every kernel reads what the
// previous one wrote (ping-pong activation buffers, 32 rows x 512 floats = 64 KB) and:
//   dep     : one dependent 16-byte load per thread, one store
//   dep+w   : + an independent 16-byte weight load per thread from a 1.5 MB buffer
//   dep+w+r : + a 4-wave LDS reduction (two __syncthreads) before the store
//   ... +ln : + a 512-float wave reduction chain (LayerNorm-like: 2 DPP sums + 2 divisions)
//   hipcc --offload-arch=gfx950 -O3 -o tools/chain_probe tools/chain_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ float wsum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <int MODE>
__global__ __launch_bounds__(256) void chain_k(const float* __restrict__ x, float* __restrict__ y,
                                               const int8_t* __restrict__ w, int nact) {
  __shared__ float red[4][64];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long gi = (long)blockIdx.x * 256 + tid;
  float4 wv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (MODE >= 1) {
    const int4 t = reinterpret_cast<const int4*>(w)[gi % (1536 * 1024 / 16)];
    wv = make_float4((float)t.x, (float)t.y, (float)t.z, (float)t.w);
  }
  const float4 a = reinterpret_cast<const float4*>(x)[gi % (nact / 4)];
  float v = a.x + a.y + a.z + a.w;
  if (MODE >= 3) {
    const float m = wsum(v) * (1.0f / 256.0f);
    const float d = v - m;
    const float var = wsum(d * d) / 255.0f;
    v = d / (sqrtf(var) + 1e-6f);
  }
  v += wv.x + wv.y + wv.z + wv.w;
  if (MODE >= 2) {
    red[wave][lane] = v;
    __syncthreads();
    if (wave == 0) v = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    __syncthreads();
    if (wave != 0) return;
  }
  y[gi % nact] = v;
}

template <class F>
double time_graph(F launch_one, int nk, hipStream_t st) {
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < nk; ++i) launch_one(st, i);
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int w = 0; w < 5; ++w) hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 20;
  hipEventRecord(e0, st);
  for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, st);
  hipEventRecord(e1, st);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return ms * 1e3 / reps / nk;
}

int main() {
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  float *x, *y;
  int8_t* w;
  hipMalloc(&x, 1 << 22);
  hipMalloc(&y, 1 << 22);
  hipMalloc(&w, 1 << 22);
  hipMemset(x, 0, 1 << 22);
  hipMemset(y, 0, 1 << 22);
  hipMemset(w, 1, 1 << 22);
  const int nact = 32 * 512;
  for (int grid : {64, 256, 768}) {
    auto run = [&](auto mode) {
      constexpr int M = decltype(mode)::value;
      return time_graph([&](hipStream_t s, int i) {
        chain_k<M><<<grid, 256, 0, s>>>(i & 1 ? y : x, i & 1 ? x : y, w, nact);
      }, 100, st);
    };
    printf("grid %4d: dep %.2f  dep+w %.2f  dep+w+r %.2f  dep+w+r+ln %.2f us/kernel\n", grid,
           run(std::integral_constant<int, 0>{}), run(std::integral_constant<int, 1>{}),
           run(std::integral_constant<int, 2>{}), run(std::integral_constant<int, 3>{}));
  }
  return 0;
}
