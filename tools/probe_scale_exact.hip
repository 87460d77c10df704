// probe_scale_exact.hip — diagnostic (not shipped): exhaustive check, on the GPU's own
// v_rcp_f32, of two short forms of the per-token scale chain against IEEE division:
//   div127(a) = RN(a / 127) as div_cr with the folded reciprocal, a scaled by 2^-64 when
//               a >= 2^60 (exact power-of-two scaling; a >= 1e-5 here)
//   rcp_nr(s) = RN(1 / s) as y0 = v_rcp_f32(s), e = fma(-s, y0, 1), y = fma(e, y0, y0)
// over every float a in [1e-5, FLT_MAX] and every s in [1e-5 / 127, FLT_MAX / 127].
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_scale_exact tools/probe_scale_exact.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__device__ __forceinline__ float div_cr(float a, float b, float y) {
  const float q = a * y;
  const float r = fmaf(-q, b, a);
  return fmaf(r, y, q);
}
__device__ __forceinline__ float div127(float a) {
  const bool big = a >= 0x1p60f;
  const float kk = big ? 0x1p-64f : 1.0f;
  const float q = div_cr(a * kk, 127.0f, 1.0f / 127.0f);
  return big ? q * 0x1p64f : q;
}
__device__ __forceinline__ float rcp_nr(float s) {
  const float y0 = __builtin_amdgcn_rcpf(s);
  const float e = fmaf(-s, y0, 1.0f);
  return fmaf(e, y0, y0);
}

__global__ void k(unsigned lo, unsigned hi, int mode, unsigned long long* bad, unsigned* first) {
  const unsigned n = hi - lo;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float x = __uint_as_float(lo + i);
    float got, want;
    if (mode == 0) {
      got = div127(x);
      want = x / 127.0f;
    } else {
      got = rcp_nr(x);
      want = 1.0f / x;
    }
    if (__float_as_uint(got) != __float_as_uint(want)) {
      atomicAdd(bad, 1ull);
      atomicMin(first, lo + i);
    }
  }
}

int main() {
  unsigned long long* bad;
  unsigned* first;
  (void)hipMalloc(&bad, 8);
  (void)hipMalloc(&first, 4);
  auto bits = [](float f) { unsigned u; memcpy(&u, &f, 4); return u; };
  struct R { const char* name; int mode; unsigned lo, hi; } rs[] = {
      {"div127 over a in [1e-5, FLT_MAX]", 0, bits(1e-5f), 0x7f800000u},
      {"rcp_nr over s in [1e-5/127, FLT_MAX/127]", 1, bits(1e-5f / 127.0f), bits(3.4028235e38f / 127.0f) + 1},
  };
  int rc = 0;
  for (const R& r : rs) {
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(first, 0xff, 4);
    hipLaunchKernelGGL(k, dim3(8192), dim3(256), 0, 0, r.lo, r.hi, r.mode, bad, first);
    (void)hipDeviceSynchronize();
    unsigned long long hb;
    unsigned hf;
    (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
    float ff;
    memcpy(&ff, &hf, 4);
    printf("%s: %u values, %llu mismatches%s", r.name, r.hi - r.lo, hb, hb ? "" : "\n");
    if (hb) printf(" (first at %a)\n", ff), rc = 1;
  }
  return rc;
}
