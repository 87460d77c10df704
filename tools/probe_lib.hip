// Diagnostic: per-kernel cost of a chain of empty kernels in a captured hipGraph, as a
// shared library so it can be timed inside a Python/torch process (tools/probe_lib.py).
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/libprobe.so tools/probe_lib.hip
#include <hip/hip_runtime.h>

__global__ void probe_nop() {}

extern "C" double probe_graph_us(int nk, int reps, int nonblocking) {
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, nonblocking ? hipStreamNonBlocking : hipStreamDefault))
    return -1;
  hipGraph_t g;
  hipGraphExec_t ge;
  if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal)) return -2;
  for (int i = 0; i < nk; ++i) probe_nop<<<1, 64, 0, st>>>();
  if (hipStreamEndCapture(st, &g)) return -3;
  if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0)) return -4;
  for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, st);
  (void)hipStreamSynchronize(st);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, st);
  for (int r = 0; r < reps; ++r) (void)hipGraphLaunch(ge, st);
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  (void)hipStreamDestroy(st);
  return ms * 1e3 / reps / nk;
}

// same chain, each node launched by an external launcher (e.g. libqtx's qtx::launch_nop)
typedef int (*launcher_t)(hipStream_t);
extern "C" double probe_graph_fn_us(launcher_t fn, int nk, int reps) {
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) return -1;
  hipGraph_t g;
  hipGraphExec_t ge;
  if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal)) return -2;
  for (int i = 0; i < nk; ++i) fn(st);
  if (hipStreamEndCapture(st, &g)) return -3;
  if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0)) return -4;
  for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, st);
  (void)hipStreamSynchronize(st);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, st);
  for (int r = 0; r < reps; ++r) (void)hipGraphLaunch(ge, st);
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3 / reps / nk;
}
