// phase_probe.hip — diagnostic (not shipped): the cost of one dependent phase of a
// persistent decode step partitioned by sentence groups (the alternative to 50 kernel
// launches per step).  32 workgroups = 4 groups of 8; workgroup 8g + j holds
// slice j of group g, so the 8 slices of a group sit on the 8 XCDs (round-robin placement:
// speed only).  One phase: publish this slice (512 fp32 = 2 KB), a group barrier (one
// device-scope counter per group: release add, one polling lane with s_sleep, acquire),
// read the group's 8 slices (16 KB), and (W) read this phase's weight slice (64 KB,
// L2-resident: the same 50 slices every step).  µs per phase over 50 phases x steps.
//   MODE 0: data by plain stores / loads; the barrier's release / acquire orders them
//   MODE 1: data by device-scope relaxed atomic stores / loads (sc1: coherent across the
//           XCDs' L2s), every store acknowledged (s_waitcnt) before the workgroup barrier, the
//           group barrier relaxed: no L2 writeback / invalidate
//   hipcc --offload-arch=gfx950 -O3 -o tools/phase_probe tools/phase_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int NPH = 50;

template <int MODE, bool W>
__global__ __launch_bounds__(256) void k_phases(float* xbuf, unsigned* counters, const float4* wts,
                                                int steps, unsigned* timeouts, float* sink) {
  const int g = blockIdx.x >> 3, j = blockIdx.x & 7, tid = threadIdx.x;
  float acc = 0.0f;
  unsigned* ctr = counters + g * 64;              // one counter per group, own 256-byte line
  for (int it = 0; it < steps * NPH; ++it) {
    const int p = it & 1;
    float* mine = xbuf + ((size_t)(p * 4 + g) * 8 + j) * 512;
    // 1. publish this slice (2 floats per thread)
    const float v0 = acc + (float)(it + tid), v1 = acc - (float)j;
    if (MODE == 0) { mine[2 * tid] = v0; mine[2 * tid + 1] = v1; }
    else {
      __hip_atomic_store(mine + 2 * tid, v0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(mine + 2 * tid + 1, v1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0);    // every thread's stores acknowledged before the barrier
    }
    // 2. group barrier
    __syncthreads();
    if (tid == 0) {
      if (MODE == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      else __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(it + 1) * 8;
      unsigned spins = 0;
      while ((MODE == 0 ? __hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                        : __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < target) {
        if (++spins > (1u << 22)) { atomicAdd(timeouts, 1u); break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    // 3. read the group's 8 slices (16 KB): thread t reads floats 16t .. 16t+15
    const float* grp = xbuf + (size_t)(p * 4 + g) * 8 * 512;
    float s = 0.0f;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const float* a = grp + 16 * tid + u;
      s += __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    acc = acc * 0.5f + s * 1e-6f;
    // 4. this phase's weight slice: 64 KB = 4096 float4, 16 per thread
    if (W) {
      const float4* w = wts + ((size_t)(it % NPH) * 8 + j) * 4096;
      float4 t = make_float4(0, 0, 0, 0);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float4 q = w[tid + 256 * u];
        t.x += q.x; t.y += q.y; t.z += q.z; t.w += q.w;
      }
      acc += (t.x + t.y + t.z + t.w) * 1e-9f;
    }
  }
  if (acc == 1234.5f) sink[blockIdx.x] = acc;
}

template <int MODE, bool W>
void run(float* xbuf, unsigned* ctr, const float4* wts, unsigned* to, float* sink, hipStream_t st) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int steps = 20;
  CHK(hipMemsetAsync(ctr, 0, 4 * 64 * 4, st));
  k_phases<MODE, W><<<32, 256, 0, st>>>(xbuf, ctr, wts, 2, to, sink);   // warm (and L2 warm)
  CHK(hipMemsetAsync(ctr, 0, 4 * 64 * 4, st));
  CHK(hipEventRecord(e0, st));
  k_phases<MODE, W><<<32, 256, 0, st>>>(xbuf, ctr, wts, steps, to, sink);
  CHK(hipEventRecord(e1, st));
  CHK(hipEventSynchronize(e1));
  float ms;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  unsigned t = 0;
  CHK(hipMemcpy(&t, to, 4, hipMemcpyDeviceToHost));
  printf("MODE %d (%s), weights %s: %.2f us per phase, %.1f us per 50-phase step%s\n", MODE,
         MODE ? "sc1 data, relaxed barrier" : "plain data, release/acquire barrier",
         W ? "64 KB/phase" : "none", ms * 1e3f / (steps * NPH), ms * 1e3f / steps, t ? "  TIMEOUTS" : "");
}

int main() {
  float *xbuf, *sink;
  unsigned *ctr, *to;
  float4* wts;
  CHK(hipMalloc(&xbuf, 2 * 4 * 8 * 512 * sizeof(float)));
  CHK(hipMalloc(&ctr, 4 * 64 * 4));
  CHK(hipMalloc(&to, 64));
  CHK(hipMalloc(&sink, 4096));
  CHK(hipMalloc(&wts, (size_t)NPH * 8 * 4096 * sizeof(float4)));   // 50 x 8 x 64 KB = 25.6 MB
  CHK(hipMemset(wts, 0, (size_t)NPH * 8 * 4096 * sizeof(float4)));
  CHK(hipMemset(to, 0, 64));
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  run<0, false>(xbuf, ctr, wts, to, sink, st);
  run<1, false>(xbuf, ctr, wts, to, sink, st);
  run<0, true>(xbuf, ctr, wts, to, sink, st);
  run<1, true>(xbuf, ctr, wts, to, sink, st);
  return 0;
}
