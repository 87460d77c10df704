// probe_fill.hip — diagnostic (not shipped): LDS-fill rate of the k_gemm_row DMA pattern,
// with and without the MFMA work, to find what bounds the row GEMM's main loop.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/libprobe_fill.so tools/probe_fill.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int BM = 128, BN = 512, BK = 128, ASZ = BM * BK, STAGE = (BM + BN) * BK;

__device__ __forceinline__ int r_slot(int r, int c) { return c ^ ((r >> 1) & 7); }

// MODE bit 0: DMA; bit 1: MFMA; bit 2: no wait between steps (DMA throughput only);
// bit 3: W k-panel contiguous layout (Wt[kt][512 rows][128])
template <int MODE>
__global__ __launch_bounds__(512) void k_fill(const int8_t* A, const int8_t* W, int M, int N,
                                              int K, int* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t st0[STAGE];
  __shared__ __attribute__((aligned(16))) uint8_t st1[STAGE];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3, fr = lane & 15, fg = lane >> 4;
  const int ncol = N / BN, logical = blockIdx.x;
  const int m0 = (logical / ncol) * BM, t = logical % ncol, n0 = t * BN, nk = K / BK;
  const int lrow = lane >> 3, lslot = lane & 7;
  const int8_t* asrc[2];
  for (int i = 0; i < 2; ++i) {
    const int ra = wave * 16 + i * 8 + lrow;
    asrc[i] = A + (long)min(m0 + ra, M - 1) * K + 16 * r_slot(ra, lslot);
  }
  const int8_t* wsrc[8];
  for (int i = 0; i < 8; ++i) {
    const int rho = wave * 64 + i * 8 + lrow;
    const int n = (rho & ~127) + 8 * (rho & 15) + ((rho >> 4) & 7);
    wsrc[i] = (MODE & 8) ? W + (long)t * BN * K + (long)rho * BK + 16 * r_slot(rho, lslot)
                         : W + (long)(n0 + n) * K + 16 * r_slot(rho, lslot);
  }
  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto issue = [&](uint8_t* base, int kt) {
    const long k0 = (long)kt * BK;
    for (int i = 0; i < 2; ++i) dma16(asrc[i] + k0, base + (wave * 16 + i * 8) * BK);
    const long kw = (MODE & 8) ? (long)kt * BN * BK : k0;
    for (int i = 0; i < 8; ++i) dma16(wsrc[i] + kw, base + ASZ + (wave * 64 + i * 8) * BK);
  };
  v4i acc[4][8];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  auto compute = [&](const uint8_t* As) {
    const uint8_t* Bs = As + ASZ;
    if (MODE & 32) {     // register operands only: the bare MFMA rate
      v4i a0 = {fr, fg, wave, 1}, b0 = {fg, fr, lane, 3};
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0 ^ (As[0] + i), b0 ^ (j + h), acc[i][j], 0, 0, 0);
      return;
    }
    if (MODE & 16) {     // every fragment of the step loaded up front into its own registers
      v4i bf[2][8], af[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = wn * 128 + j * 16 + fr;
          bf[h][j] = *reinterpret_cast<const v4i*>(Bs + r * BK + 16 * r_slot(r, 4 * h + fg));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = wm * 64 + i * 16 + fr;
          af[h][i] = *reinterpret_cast<const v4i*>(As + r * BK + 16 * r_slot(r, 4 * h + fg));
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[h][i], bf[h][j], acc[i][j], 0, 0, 0);
      // schedule: the 12 reads of half 0, then its 32 MFMAs with the 12 reads of half 1
      // interleaved (2 MFMAs, 1 read), then the 32 MFMAs of half 1
      __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
#pragma unroll
      for (int q = 0; q < 12; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 40, 0);
      return;
    }
    for (int h = 0; h < 2; ++h) {
      v4i bfr[8];
      for (int j = 0; j < 8; ++j) {
        const int r = wn * 128 + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const v4i*>(Bs + r * BK + 16 * r_slot(r, 4 * h + fg));
      }
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + fr;
        const v4i afr = *reinterpret_cast<const v4i*>(As + r * BK + 16 * r_slot(r, 4 * h + fg));
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  auto step = [&](uint8_t* cur, uint8_t* nxt, int kt) {
    if (!(MODE & 4)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if ((MODE & 1) && kt + 1 < nk) issue(nxt, kt + 1);
    if (MODE & 2) compute(cur);
  };
  if (MODE & 1) issue(st0, 0);
  for (int kt = 0; kt < nk; kt += 2) {
    step(st0, st1, kt);
    if (kt + 1 < nk) step(st1, st0, kt + 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int s = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) s += acc[i][j][0] + acc[i][j][3];
  if (s == 0x12345678) sink[tid] = s;
}

extern "C" int probe_fill(int mode, const int8_t* A, const int8_t* W, int M, int N, int K,
                          int* sink, hipStream_t st) {
  const dim3 grid((N / BN) * (M / BM)), block(512);
  switch (mode) {
#define C(m) case m: k_fill<m><<<grid, block, 0, st>>>(A, W, M, N, K, sink); break;
    C(1) C(2) C(3) C(5) C(9) C(11) C(13) C(18) C(19) C(34)
#undef C
    default: return -1;
  }
  return (int)hipGetLastError();
}

// 4 waves x (128 rows x 128 columns) per workgroup: half the fragment reads per MAC of the
// 8-wave (64 x 128) layout; one wave per SIMD, accumulators in AGPRs
template <int MODE>
__global__ __launch_bounds__(256) void k_fill4(const int8_t* A, const int8_t* W, int M, int N,
                                               int K, int* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t st0[STAGE];
  __shared__ __attribute__((aligned(16))) uint8_t st1[STAGE];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wn = wave, fr = lane & 15, fg = lane >> 4;
  const int ncol = N / BN, logical = blockIdx.x;
  const int m0 = (logical / ncol) * BM, t = logical % ncol, n0 = t * BN, nk = K / BK;
  const int lrow = lane >> 3, lslot = lane & 7;
  const int8_t* asrc[4];
  for (int i = 0; i < 4; ++i) {
    const int ra = wave * 32 + i * 8 + lrow;
    asrc[i] = A + (long)min(m0 + ra, M - 1) * K + 16 * r_slot(ra, lslot);
  }
  // W LDS row rho = 128 wave + 8 i + lrow holds column 128 wave + 64 (i&1) + 8 lrow + (i>>1):
  // two lane bases (i even / odd) plus a wave-uniform offset per instruction
  const int8_t* wb[2];
  for (int p = 0; p < 2; ++p)
    wb[p] = W + (long)(n0 + wave * 128 + 8 * lrow) * K + 16 * (lslot ^ ((p * 4 + (lrow >> 1)) & 7));
  auto dma16 = [](const int8_t* gsrc, const uint8_t* lds_dst) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  };
  auto issue = [&](uint8_t* base, int kt) {
    const long k0 = (long)kt * BK;
    for (int i = 0; i < 4; ++i) dma16(asrc[i] + k0, base + (wave * 32 + i * 8) * BK);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      dma16(wb[i & 1] + (long)(64 * (i & 1) + (i >> 1)) * K + k0, base + ASZ + (wave * 128 + i * 8) * BK);
  };
  v4i acc[8][8];
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  auto compute = [&](const uint8_t* As) {
    const uint8_t* Bs = As + ASZ;
    v4i bf[2][8], af[2][8];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = wn * 128 + j * 16 + fr;
        bf[h][j] = *reinterpret_cast<const v4i*>(Bs + r * BK + 16 * r_slot(r, 4 * h + fg));
        const int ra = j * 16 + fr;
        af[h][j] = *reinterpret_cast<const v4i*>(As + ra * BK + 16 * r_slot(ra, 4 * h + fg));
      }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[h][i], bf[h][j], acc[i][j], 0, 0, 0);
    if (MODE & 16) {
      __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 64, 0);
    }
  };
  auto step = [&](uint8_t* cur, uint8_t* nxt, int kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if ((MODE & 1) && kt + 1 < nk) issue(nxt, kt + 1);
    if (MODE & 2) compute(cur);
  };
  if (MODE & 1) issue(st0, 0);
  for (int kt = 0; kt < nk; kt += 2) {
    step(st0, st1, kt);
    if (kt + 1 < nk) step(st1, st0, kt + 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int s = 0;
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) s += acc[i][j][0] + acc[i][j][3];
  if (s == 0x12345678) sink[tid] = s;
}

extern "C" int probe_fill4(int mode, const int8_t* A, const int8_t* W, int M, int N, int K,
                           int* sink, hipStream_t st) {
  const dim3 grid((N / BN) * (M / BM)), block(256);
  switch (mode) {
#define C(m) case m: k_fill4<m><<<grid, block, 0, st>>>(A, W, M, N, K, sink); break;
    C(1) C(2) C(3) C(18) C(19)
#undef C
    default: return -1;
  }
  return (int)hipGetLastError();
}
