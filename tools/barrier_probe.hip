// barrier_probe.hip — diagnostic (not shipped): what a grid-wide hand-off costs inside one
// persistent launch on this chip, against a kernel boundary in a hipGraph chain — the
// question behind a persistent decode layer.
//   * boundary: a hipGraph of 256 dependent launches of G workgroups (empty, and each
//     reading a value its predecessor wrote), µs per node
//   * barrier: ONE launch of G workgroups (256 threads, one per CU at G <= 256, all
//     co-resident) crossing N grid barriers: a monotonic device-scope counter, one release
//     atomicAdd per workgroup, then a poll by one lane with s_sleep until every workgroup of
//     the phase has arrived (acquire); bounded polls (a timed-out run is reported, never hangs)
//   * barrier + data: each phase also reads a value another workgroup wrote in the last one
//   hipcc --offload-arch=gfx950 -O3 -o tools/barrier_probe tools/barrier_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_empty() {}
__global__ void k_dep(float* buf) {      // reads what the previous launch wrote, writes one
  const float v = buf[(blockIdx.x * 7 + 1) % gridDim.x];
  if (threadIdx.x == 0) buf[blockIdx.x] = v + 1.0f;
}

__global__ void k_barriers(unsigned* counter, float* buf, int nphase, int data, unsigned* timeouts) {
  const unsigned G = gridDim.x;
  float v = 0.0f;
  for (int p = 0; p < nphase; ++p) {
    if (data) {                          // read another workgroup's value of the last phase
      v += __hip_atomic_load(buf + ((blockIdx.x * 7 + 1) % G) + (p & 1) * 1024, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      if (threadIdx.x == 0)
        __hip_atomic_store(buf + blockIdx.x + ((p + 1) & 1) * 1024, v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(p + 1) * G;
      unsigned spins = 0;
      while (__hip_atomic_load(counter, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (++spins > (1u << 22)) { atomicAdd(timeouts, 1u); break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && v == 12345.0f) buf[2047] = v;
}

int main() {
  float* buf;
  unsigned *counter, *timeouts;
  CHK(hipMalloc(&buf, 2048 * sizeof(float)));
  CHK(hipMalloc(&counter, 64));
  CHK(hipMalloc(&timeouts, 64));
  CHK(hipMemset(buf, 0, 2048 * sizeof(float)));
  CHK(hipMemset(timeouts, 0, 64));
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int grids[] = {8, 32, 64, 128, 256};
  for (int G : grids) {
    float us[2];
    for (int kind = 0; kind < 2; ++kind) {
      hipGraph_t graph;
      CHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < 256; ++i) {
        if (kind == 0) k_empty<<<G, 256, 0, st>>>();
        else k_dep<<<G, 256, 0, st>>>(buf);
      }
      CHK(hipStreamEndCapture(st, &graph));
      hipGraphExec_t ex;
      CHK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
      for (int w = 0; w < 3; ++w) CHK(hipGraphLaunch(ex, st));
      CHK(hipEventRecord(e0, st));
      for (int r = 0; r < 10; ++r) CHK(hipGraphLaunch(ex, st));
      CHK(hipEventRecord(e1, st));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      us[kind] = ms * 1e3f / (10 * 256);
      CHK(hipGraphExecDestroy(ex));
      CHK(hipGraphDestroy(graph));
    }
    float bus[2];
    const int nph = 2000;
    for (int data = 0; data < 2; ++data) {
      for (int w = 0; w < 2; ++w) {
        CHK(hipMemsetAsync(counter, 0, 64, st));
        k_barriers<<<G, 256, 0, st>>>(counter, buf, 100, data, timeouts);
      }
      CHK(hipMemsetAsync(counter, 0, 64, st));
      CHK(hipEventRecord(e0, st));
      k_barriers<<<G, 256, 0, st>>>(counter, buf, nph, data, timeouts);
      CHK(hipEventRecord(e1, st));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      bus[data] = ms * 1e3f / nph;
    }
    unsigned to = 0;
    CHK(hipMemcpy(&to, timeouts, 4, hipMemcpyDeviceToHost));
    printf("G=%3d workgroups: graph node empty %.2f us, dependent %.2f us | in-launch grid barrier %.2f us, with a data hand-off %.2f us%s\n",
           G, us[0], us[1], bus[0], bus[1], to ? "  (TIMEOUTS!)" : "");
  }
  return 0;
}
