// probe_bf16_mfma.hip — diagnostic (not shipped): how does v_mfma_f32_16x16x32_bf16 round?
// (could the encoder attention's PV — today the sequential fp32 fma chain
// over the keys on v_mfma_f32_16x16x4_f32, which shares the VALU datapath with the softmax —
// move to the bf16 matrix core with results the numpy oracle can reproduce exactly?)
// One wave computes D = A . B + C for T random trials of bf16 A [16 x 32], B [32 x 16] and
// fp32 C, with operand exponents spread over 2^-8 .. 2^8 (and a second set with cancelling
// signs); the raw operands and results go to a file that tools/probe_bf16_mfma.py compares
// against rounding models (exact sum rounded once, sequential fp32 chains, pairwise trees).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_bf16_mfma tools/probe_bf16_mfma.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef float v4f __attribute__((ext_vector_type(4)));

// lane l: A row l & 15, 8 bf16 (16 bytes) of K group l >> 4; B column l & 15, the same K
// group; D rows 4 (l >> 4) + e, column l & 15
__global__ void k_mfma(const uint16_t* A, const uint16_t* B, const float* C, float* D, int T) {
  const int l = threadIdx.x;
  for (int t = 0; t < T; ++t) {
    bf16x8 a, b;
    uint16_t ra[8], rb[8];
    for (int i = 0; i < 8; ++i) {
      ra[i] = A[(size_t)t * 512 + l * 8 + i];
      rb[i] = B[(size_t)t * 512 + l * 8 + i];
    }
    memcpy(&a, ra, 16);
    memcpy(&b, rb, 16);
    v4f c;
    for (int e = 0; e < 4; ++e) c[e] = C[(size_t)t * 256 + l * 4 + e];
    const v4f d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    for (int e = 0; e < 4; ++e) D[(size_t)t * 256 + l * 4 + e] = d[e];
  }
}

static uint16_t bf16_bits(float x) {          // x already representable in bf16
  uint32_t u;
  memcpy(&u, &x, 4);
  return (uint16_t)(u >> 16);
}

int main(int argc, char** argv) {
  const int T = 400;
  std::vector<uint16_t> A((size_t)T * 512), B((size_t)T * 512);
  std::vector<float> C((size_t)T * 256), D((size_t)T * 256);
  unsigned x = 12345;
  auto rnd = [&]() { x = x * 1664525u + 1013904223u; return x; };
  for (int t = 0; t < T; ++t) {
    const bool cancel = t >= T / 2;              // second half: mixed signs, similar magnitudes
    for (int i = 0; i < 512; ++i) {
      for (int w = 0; w < 2; ++w) {
        const int e = cancel ? (int)(rnd() % 5) - 2 : (int)(rnd() % 17) - 8;
        const float m = 1.0f + (float)(rnd() & 127) / 128.0f;      // 8 significant bits
        const float v = ldexpf(m, e) * ((rnd() & 1) ? -1.0f : 1.0f);
        (w ? B : A)[(size_t)t * 512 + i] = bf16_bits(v);
      }
    }
    for (int i = 0; i < 256; ++i) {
      const int e = cancel ? (int)(rnd() % 5) - 2 : (int)(rnd() % 17) - 8;
      const float m = 1.0f + (float)(rnd() & 0x7fffff) / 8388608.0f;
      C[(size_t)t * 256 + i] = ldexpf(m, e) * ((rnd() & 1) ? -1.0f : 1.0f);
    }
  }
  uint16_t *dA, *dB;
  float *dC, *dD;
  hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2);
  hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
  hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
  k_mfma<<<1, 64>>>(dA, dB, dC, dD, T);
  hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
  const char* out = argc > 1 ? argv[1] : "bf16_mfma.bin";
  FILE* f = fopen(out, "wb");
  fwrite(&T, 4, 1, f);
  fwrite(A.data(), 2, A.size(), f);
  fwrite(B.data(), 2, B.size(), f);
  fwrite(C.data(), 4, C.size(), f);
  fwrite(D.data(), 4, D.size(), f);
  fclose(f);
  printf("wrote %d trials to %s\n", T, out);
  return 0;
}
