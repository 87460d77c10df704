// probe_cvt_pk_u8.hip — diagnostic (not shipped): does v_cvt_pk_u8_f32 round to nearest even
// and clamp to [0, 255] (so it could replace rint + byte packing for the non-negative FFN1
// hidden codes)?  Compares it with rintf + clamp on halves, near-halves, signed zeros,
// negatives, large values, inf and NaN.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_cvt_pk_u8 tools/probe_cvt_pk_u8.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_cvt(const float* x, unsigned* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned d = 0;
  asm volatile("v_cvt_pk_u8_f32 %0, %1, 0, %2" : "=v"(d) : "v"(x[i]), "v"(0u));
  out[i] = d;
}

int main() {
  std::vector<float> xs;
  for (int k = -600; k <= 600; ++k) {
    const float h = k * 0.5f;
    xs.push_back(h);
    xs.push_back(std::nextafter(h, 1e9f));
    xs.push_back(std::nextafter(h, -1e9f));
  }
  for (float v : {0.0f, -0.0f, 1e-30f, -1e-30f, 254.5f, 255.49f, 255.5f, 256.0f, 1e10f, -1e10f,
                  INFINITY, -INFINITY, NAN})
    xs.push_back(v);
  const int n = (int)xs.size();
  float* dx; unsigned* dout;
  hipMalloc(&dx, n * 4); hipMalloc(&dout, n * 4);
  hipMemcpy(dx, xs.data(), n * 4, hipMemcpyHostToDevice);
  k_cvt<<<(n + 255) / 256, 256>>>(dx, dout, n);
  std::vector<unsigned> o(n);
  if (hipMemcpy(o.data(), dout, n * 4, hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 1; }
  int bad = 0, shown = 0;
  for (int i = 0; i < n; ++i) {
    const float x = xs[i];
    const float r = std::isnan(x) ? 0.0f : std::fmin(std::fmax(std::rint(x), 0.0f), 255.0f);
    const unsigned want = (unsigned)r;
    if ((o[i] & 0xffu) != want) {
      ++bad;
      if (shown++ < 20) printf("x=%.9g (0x%08x): cvt_pk_u8 %u, rint+clamp %u\n", x, *(unsigned*)&x, o[i] & 0xffu, want);
    }
  }
  printf("v_cvt_pk_u8_f32 vs rint + clamp[0,255] (NaN -> 0): %d of %d differ\n", bad, n);
  return 0;
}
