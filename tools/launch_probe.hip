// Diagnostic: cost per dependent kernel in a captured hipGraph (empty kernel, a kernel
// with one L2 round trip, 32 vs 256 workgroups).
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_probe tools/launch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void empty_k(int* p) {
  if (p == nullptr) return;
}
__global__ void load_k(const float* x, float* y, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float v = x[i % n];
  y[i % n] = v + 1.0f;
}

template <class F>
double time_graph(F launch_one, int nk, hipStream_t st) {
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < nk; ++i) launch_one(st);
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
  return ms * 1e3 / reps / nk;
}

int main() {
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  float *x, *y;
  hipMalloc(&x, 1 << 24);
  hipMalloc(&y, 1 << 24);
  hipMemset(x, 0, 1 << 24);
  for (int grid : {1, 32, 256, 1024}) {
    double e = time_graph([&](hipStream_t s) { empty_k<<<grid, 256, 0, s>>>(nullptr); }, 100, st);
    double l = time_graph([&](hipStream_t s) { load_k<<<grid, 256, 0, s>>>(x, y, 1 << 20); },
                          100, st);
    printf("grid %5d: empty %.2f us/kernel, one-load %.2f us/kernel\n", grid, e, l);
  }
  return 0;
}
