// probe_mfma32_layout.hip — diagnostic (not shipped): checks the operand / result lane
// layout assumed for v_mfma_i32_32x32x32_i8 (and, as a control, v_mfma_i32_16x16x64_i8):
//   operands: lane l holds row (l % R) and K bytes 16 * (l / R) .. +16 of the step
//   result 32x32: lane l, register r -> D[8 (r / 4) + 4 (l / 32) + r % 4][l % 32]
//   result 16x16: lane l, register r -> D[4 (l / 16) + r][l % 16]
// with A[i][0] = i + 1, A[i][1] = 64, B[j][0] = 1, B[j][1] = j + 1: D[i][j] = i + 1 + 64 (j + 1).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma32_layout tools/probe_mfma32_layout.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k_layout(int* bad32, int* bad16) {
  const int l = threadIdx.x;
  {
    const int R = 32, half = l / R, row = l % R;
    unsigned char a[16] = {}, b[16] = {};
    if (half == 0) {
      a[0] = (unsigned char)(row + 1); a[1] = 64;
      b[0] = 1; b[1] = (unsigned char)(row + 1);
    }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v16i acc = {};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc, 0, 0, 0);
    int bad = 0;
    for (int r = 0; r < 16; ++r) {
      const int i = 8 * (r / 4) + 4 * (l / 32) + r % 4, j = l % 32;
      bad += acc[r] != i + 1 + 64 * (j + 1);
    }
    atomicAdd(bad32, bad);
  }
  {
    const int R = 16, q = l / R, row = l % R;
    unsigned char a[16] = {}, b[16] = {};
    if (q == 0) {
      a[0] = (unsigned char)(row + 1); a[1] = 64;
      b[0] = 1; b[1] = (unsigned char)(row + 1);
    }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v4i acc = {};
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc, 0, 0, 0);
    int bad = 0;
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * (l / 16) + r, j = l % 16;
      bad += acc[r] != i + 1 + 64 * (j + 1);
    }
    atomicAdd(bad16, bad);
  }
}

int main() {
  int* d;
  (void)hipMalloc(&d, 8);
  (void)hipMemset(d, 0, 8);
  k_layout<<<1, 64>>>(d, d + 1);
  int h[2];
  (void)hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
  printf("mfma layout check: 32x32x32 mismatches %d / 1024, 16x16x64 mismatches %d / 256\n", h[0], h[1]);
  return h[0] || h[1];
}
