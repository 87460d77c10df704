// probe_ffn_ring.hip — diagnostic (not shipped): the L2 -> LDS weight stream of the fused FFN
// row-block kernel (VERDICT r04 "next round" item 1, step 1), measured as a skeleton with the
// MFMAs the kernel issues and no epilogue arithmetic.
//
// One 128-row block per CU (cfg3: M = 32768 = 256 blocks).  The block's weights arrive as one
// linear stream of 32 KB slots in MFMA-fragment order (1 KB = one 16 x 64 fragment, lane l's
// 16 bytes at 16 l), so a slot is filled by 32 linear 1 KB LDS-DMA pieces and read by linear
// ds_read_b128 (conflict-free):
//   pass 1 (FFN1 row maxima):   32 W1 slots,                      64 MFMAs per wave each
//   pass 2 (FFN1 + FFN2):        32 x (W1 slot, W2 K-step slot),   64 MFMAs per wave each
// = 96 slots = 3 MB per CU.  Every wave reads every byte of every slot (its own rows).
// Ring: NSLOT slots, per slot each wave waits for its own pieces (counted vmcnt: the loop
// holds no other memory operation), one s_barrier, then issues slot s + NSLOT - 1 into the
// slot consumed at s - 1.
// Variants: waves per workgroup (4 = one per SIMD, the 512-register design; 8 = two per SIMD,
// rows split), ring depth, per-CU rotation of the mini-chunk order (exact in the kernel: int32
// sums and maxima are order-free; CUs of one XCD then do not request the same W lines at the
// same time), nt policy on the weight pieces, and the fill alone / the consumers alone.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_ffn_ring tools/probe_ffn_ring.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int SLOT = 32 * 1024;
constexpr int NCHUNK = 32;                 // 64-column FFN1 mini-chunks (d_ff 2048)
constexpr int NSTREAM = 3 * NCHUNK;        // slots consumed per block

// DMA issue forms: 0 global_load_lds 64-bit VGPR address; 1 global_load_lds SGPR base +
// 32-bit VGPR offset.  A third form — buffer_load_dwordx4 ... lds with ADD_TID_ENABLE in the
// V# (no VGPR address operand: lane i's 16 bytes at base + soffset + i * stride) — failed its
// data check and lost the context in round 5 (never committed) and again, re-derived from
// the MUBUF rules, in round 6 (stride 16, num_records in records, DATA_FORMAT 32; encoding
// "buffer_load_dwordx4 off, s[0:3], sN lds" with M0 = the LDS slot): dropped for good,
// DESIGN.md §4 and profiles/r06_ring_probe.log.
template <int DM>
__device__ __forceinline__ void dmax(const int8_t* base, unsigned off, unsigned voff, const uint8_t* lds_dst) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
  unsigned keep;
  if constexpr (DM == 0)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(base + off + voff), "s"(dst) : "memory");
  else if constexpr (DM == 1) {
    const unsigned long long bb = (unsigned long long)(uintptr_t)base;
    const unsigned long long sb = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(bb >> 32)) << 32) |
                                  (unsigned)__builtin_amdgcn_readfirstlane((unsigned)bb);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %3, %1\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(sb), "s"(dst), "v"(voff + off) : "memory");
  }
}

template <bool NT>
__device__ __forceinline__ void dma16(const int8_t* gsrc, const uint8_t* lds_dst) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
  unsigned keep;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
}

// MODE 0: fill + consume; 1: fill only; 2: consume only (no DMA)
template <int NW, int NSLOT, bool ROT, bool NT, int MODE, int PD = 0, bool SB = false, bool ASM = false, int SYNC = 0, int DM = -1>
__global__ __launch_bounds__(NW * 64) void k_ring(const int8_t* W, int* sink, unsigned long long* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[NSLOT * SLOT];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  constexpr int PPW = 32 / NW;               // 1 KB pieces per wave per slot
  // pass 2's stream is (W1 chunk c, W2 K-step c) interleaved: slot 2c and 2c + 1 of a 2 MB
  // region; pass 1 reads the W1 slots of it
  const int rot = ROT ? (int)((blockIdx.x >> 3) * 5 + (blockIdx.x & 7) * 3) % NCHUNK : 0;
  auto src_slot = [&](int j) {               // stream position j -> slot index in W
    const int pass2 = j >= NCHUNK;
    const int c0 = pass2 ? (j - NCHUNK) >> 1 : j;
    const int c = (c0 + rot) % NCHUNK;
    return pass2 ? 2 * c + ((j - NCHUNK) & 1) : 2 * c;
  };
  auto issue = [&](int j) {
    if (MODE == 2 || j >= NSTREAM) return;
    uint8_t* dst = lds + (j % NSLOT) * SLOT + (wave * PPW) * 1024;
    if constexpr (DM < 0) {
      const int8_t* src = W + (long)src_slot(j) * SLOT + (wave * PPW) * 1024 + lane * 16;
#pragma unroll
      for (int p = 0; p < PPW; ++p) dma16<NT>(src + p * 1024, dst + p * 1024);
    } else {
      const unsigned off = (unsigned)(src_slot(j) * SLOT + (wave * PPW) * 1024);
#pragma unroll
      for (int p = 0; p < PPW; ++p) dmax<DM>(W, off + p * 1024, lane * 16, dst + p * 1024);
    }
  };
  // operands held in registers by the kernel: the block's x1q rows (4 waves: 2 row
  // fragments x 8 K steps; 8 waves: 1 x 8) and FFN2's hq fragments
  constexpr int RF = NW == 4 ? 2 : 1;
  v4i xa[RF][8];
#pragma unroll
  for (int i = 0; i < RF; ++i)
#pragma unroll
    for (int s = 0; s < 8; ++s) xa[i][s] = v4i{tid + i, s, lane * 3, i ^ s};
  v4i acc[RF][8];
#pragma unroll
  for (int i = 0; i < RF; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  for (int j = 0; j < NSLOT - 1; ++j) issue(j);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int s = 0; s < NSTREAM; ++s) {
    if (MODE != 2 && SYNC != 2) {
      // this wave's pieces of slot s landed: the youngest are slots s+1 .. s+NSLOT-2
      const int ahead = min(NSLOT - 2, NSTREAM - 1 - s);
      if (ahead >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PPW) : "memory");
      else if (ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (SYNC != 1) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    issue(s + NSLOT - 1);
    if (MODE == 1) continue;
    const uint8_t* slot = lds + (s % NSLOT) * SLOT;
    if constexpr (PD == 0) {
      // 32 fragments per slot; each consumed by RF row fragments (2 MFMAs per fragment at
      // 4 waves: 64 per slot per wave)
#pragma unroll 4
      for (int f = 0; f < 32; f += 4) {
        v4i b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = *reinterpret_cast<const v4i*>(slot + (f + q) * 1024 + lane * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int i = 0; i < RF; ++i)
            acc[i][(f + q) & 7] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[q], xa[i][(f + q) & 7], acc[i][(f + q) & 7], 0, 0, 0);
      }
    } else {
      // software-pipelined: the fragment PD ahead is read while this one is multiplied
      v4i b[PD];
#pragma unroll
      for (int q = 0; q < PD; ++q) b[q] = *reinterpret_cast<const v4i*>(slot + q * 1024 + lane * 16);
#pragma unroll
      for (int f = 0; f < 32; ++f) {
        const v4i cur = b[f % PD];
        if (f + PD < 32) b[f % PD] = *reinterpret_cast<const v4i*>(slot + (f + PD) * 1024 + lane * 16);
        // pin the prefetch distance: the scheduler would otherwise sink each read next to
        // its MFMAs (two buffers, the LDS latency exposed every 4 MFMAs)
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < RF; ++i) {
          if constexpr (ASM)   // accumulators pinned to AGPRs, no copies between iterations
            asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(acc[i][f & 7]) : "v"(cur), "v"(xa[i][f & 7]));
          else
            acc[i][f & 7] = __builtin_amdgcn_mfma_i32_16x16x64_i8(cur, xa[i][f & 7], acc[i][f & 7], 0, 0, 0);
        }
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory");
  int sum = 0;
#pragma unroll
  for (int i = 0; i < RF; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) sum += acc[i][j][0] ^ acc[i][j][3];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (sum == 0x1234567) sink[tid] = sum;
  if (tid == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = r1 - r0; }
}

// ---- round 6: the ring the guide measures (MI355X_MICROARCH.md
// ring-gemm) — dedicated loader waves and per-slot FULL / FREE words in LDS, no s_barrier.
// NC consumer waves (each 128 / NC rows of the block: RF = 8 / NC row fragments, so every
// fragment it reads feeds RF MFMAs) + NL loader waves (no compute).  The same 3 MB per CU
// (pass 1's W1 + pass 2's W1 / W2 interleaved, per-CU rotation), in SLOTKB-KB slots.
//   loader l, stream slot j: wait until every consumer has released slot j - NSLOT (its FREE
//     word >= j - NSLOT), issue its SLOTKB / NL pieces, then publish slot j - D (its FULL
//     word = j - D) behind s_waitcnt vmcnt(D * pieces): the loop holds no memory op but
//     the DMAs, so the counted wait is exact (VM_CNT_ORDER); D slots stay in flight.
//   consumer c, slot s: poll the NL FULL words (one lane each) until all >= s, read the
//     slot's fragments into registers, s_waitcnt lgkmcnt(0), write its FREE word = s, then
//     the MFMAs (the next slot's poll and reads issue under them).
// MODE 0 fill + consume, 1 loaders only (consumers release at once, read nothing),
// 2 consumers only (the FULL words pre-set, no DMA).
template <int NC, int NL, int NSLOT, int SLOTKB, int D, int MODE, bool NT>
__global__ __launch_bounds__((NC + NL) * 64) void k_ring2(const int8_t* W, int* sink, unsigned long long* out) {
  constexpr int SL = SLOTKB * 1024;
  constexpr int NS = 3 * NCHUNK * SLOT / SL;          // stream slots per block (3 MB)
  constexpr int FR = SLOTKB;                          // 1 KB fragments per slot
  constexpr int PPL = FR / NL;                        // pieces per loader per slot
  constexpr int RF = 8 / NC;                          // row fragments per consumer
  static_assert(FR % NL == 0 && 8 % NC == 0 && D + 1 < NSLOT, "shape");
  __shared__ __attribute__((aligned(16))) uint8_t lds[NSLOT * SL];
  __shared__ int fullw[NSLOT][NL];
  __shared__ int freew[NSLOT][NC];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int rot = (int)((blockIdx.x >> 3) * 5 + (blockIdx.x & 7) * 3) % NCHUNK;
  // stream slot j -> its byte offset in the 2 MB region (32 KB units as k_ring, split)
  auto src_off = [&](int j) {
    constexpr int SUB = SLOT / SL;                    // stream slots per 32 KB unit
    const int u = j / SUB, part = j % SUB;
    const int pass2 = u >= NCHUNK;
    const int c0 = pass2 ? (u - NCHUNK) >> 1 : u;
    const int c = (c0 + rot) % NCHUNK;
    const int unit = pass2 ? 2 * c + ((u - NCHUNK) & 1) : 2 * c;
    return (long)unit * SLOT + (long)part * SL;
  };
  for (int i = tid; i < NSLOT * NL; i += (NC + NL) * 64) (&fullw[0][0])[i] = MODE == 2 ? 1 << 30 : -1;
  for (int i = tid; i < NSLOT * NC; i += (NC + NL) * 64) (&freew[0][0])[i] = -1;
  __syncthreads();
  volatile int* vfull = &fullw[0][0];
  volatile int* vfree = &freew[0][0];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  int sum = 0;
  if (wave >= NC) {
    // ---------------- loader
    const int l = wave - NC;
    if constexpr (MODE != 2) {
      for (int j = 0; j < NS; ++j) {
        const int slot = j % NSLOT;
        if (j >= NSLOT) {
          while (true) {
            const int v = lane < NC ? vfree[slot * NC + lane] : j;
            if (__builtin_amdgcn_ballot_w64(v < j - NSLOT) == 0ull) break;
            __builtin_amdgcn_s_sleep(1);
          }
        }
        const int8_t* src = W + src_off(j) + (l * PPL) * 1024 + lane * 16;
        uint8_t* dst = lds + slot * SL + (l * PPL) * 1024;
#pragma unroll
        for (int p = 0; p < PPL; ++p) dma16<NT>(src + p * 1024, dst + p * 1024);
        if (j >= D) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D * PPL) : "memory");
          if (lane == 0) vfull[((j - D) % NSLOT) * NL + l] = j - D;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0)
        for (int j = (NS > D ? NS - D : 0); j < NS; ++j) vfull[(j % NSLOT) * NL + l] = j;
    }
  } else {
    // ---------------- consumer
    const int c = wave;
    v4i xa[RF][8];
#pragma unroll
    for (int i = 0; i < RF; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) xa[i][k] = v4i{tid + i, k, lane * 3, i ^ k};
    v4i acc[RF][8];
#pragma unroll
    for (int i = 0; i < RF; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[i][k] = v4i{0, 0, 0, 0};
    for (int s = 0; s < NS; ++s) {
      const int slot = s % NSLOT;
      if constexpr (MODE != 2) {
        while (true) {
          const int v = lane < NL ? vfull[slot * NL + lane] : s;
          if (__builtin_amdgcn_ballot_w64(v < s) == 0ull) break;
          __builtin_amdgcn_s_sleep(0);
        }
      }
      if constexpr (MODE == 1) {
        if (lane == 0) vfree[slot * NC + c] = s;
        continue;
      }
      const uint8_t* sp = lds + slot * SL + lane * 16;
      v4i b[FR];
#pragma unroll
      for (int f = 0; f < FR; ++f) b[f] = *reinterpret_cast<const v4i*>(sp + f * 1024);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (MODE != 2)
        if (lane == 0) vfree[slot * NC + c] = s;
#pragma unroll
      for (int f = 0; f < FR; ++f)
#pragma unroll
        for (int i = 0; i < RF; ++i)
          acc[i][f & 7] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[f], xa[i][f & 7], acc[i][f & 7], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < RF; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) sum += acc[i][k][0] ^ acc[i][k][3];
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (sum == 0x1234567) sink[tid] = sum;
  if (tid == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = r1 - r0; }
}

typedef void (*KFn)(const int8_t*, int*, unsigned long long*);
struct Var { const char* name; KFn f; int threads; int mode; };

int main(int argc, char** argv) {
  const bool pmc = argc > 1;                 // under rocprofv3 --pmc: 1 round, 3 launches each
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const long wbytes = 2L * NCHUNK * SLOT;           // the 2 MB stream region (3 MB read per CU)
  int8_t* W; int* sink; unsigned long long* d;
  hipMalloc(&W, wbytes); hipMalloc(&sink, 4096); hipMalloc(&d, 4096 * 16);
  {
    int8_t* h = (int8_t*)malloc(wbytes);
    unsigned x = 7;
    for (long i = 0; i < wbytes; ++i) { x = x * 1664525u + 1013904223u; h[i] = (int8_t)(x >> 24); }
    hipMemcpy(W, h, wbytes, hipMemcpyHostToDevice);
    free(h);
  }
  // round 6: the round-5 best (8 waves, every wave DMAs + one s_barrier per slot) against
  // dedicated loaders with FULL / FREE words (k_ring2 <NC consumers, NL loaders, slots,
  // KB per slot, slots in flight>)
  Var vars[] = {
      {"r05 8w all-DMA+barrier 4x32K pd4  ", k_ring<8, 4, true, false, 0, 4, true, true, 0, 0>, 512, 0},
      {"r05 8w consume-only pd4           ", k_ring<8, 4, true, false, 2, 4, true, true>, 512, 2},
      {"r05 4w fill-only                  ", k_ring<4, 4, true, false, 1, 0, false, false, 0, 0>, 256, 1},
      {"ring2 4c+4l 6x16K D2              ", k_ring2<4, 4, 6, 16, 2, 0, false>, 512, 0},
      {"ring2 4c+2l 6x16K D2              ", k_ring2<4, 2, 6, 16, 2, 0, false>, 384, 0},
      {"ring2 4c+4l 8x16K D3              ", k_ring2<4, 4, 8, 16, 3, 0, false>, 512, 0},
      {"ring2 4c+4l 4x32K D1              ", k_ring2<4, 4, 4, 32, 1, 0, false>, 512, 0},
      {"ring2 8c+4l 6x16K D2              ", k_ring2<8, 4, 6, 16, 2, 0, false>, 768, 0},
      {"ring2 4c+4l 8x16K D5              ", k_ring2<4, 4, 8, 16, 5, 0, false>, 512, 0},
      {"ring2 4c+4l 9x16K D6              ", k_ring2<4, 4, 9, 16, 6, 0, false>, 512, 0},
      {"ring2 8c+4l 9x16K D6              ", k_ring2<8, 4, 9, 16, 6, 0, false>, 768, 0},
      {"ring2 4c+4l fill-only 6x16K D2    ", k_ring2<4, 4, 6, 16, 2, 1, false>, 512, 1},
      {"ring2 4c+4l fill-only 8x16K D5    ", k_ring2<4, 4, 8, 16, 5, 1, false>, 512, 1},
      {"ring2 4c+4l fill-only 9x16K D6    ", k_ring2<4, 4, 9, 16, 6, 1, false>, 512, 1},
      {"ring2 4c consume-only 6x16K       ", k_ring2<4, 4, 6, 16, 2, 2, false>, 512, 2},
      {"ring2 8c consume-only 6x16K       ", k_ring2<8, 4, 6, 16, 2, 2, false>, 768, 2},
  };
  printf("CUs %d; per CU %.2f MB streamed (96 x 32 KB slots); MFMA floor at 4 waves = 96 x 64 x 16 cycles\n",
         ncu, 3.0 * NCHUNK * SLOT / 1048576.0);
  // (the buffer ADD_TID form, DM 2, is not run: round 6 tested it once — MISMATCH, then the
  // context was lost — profiles/r06_ring_probe.log)
  for (int rep = 0; rep < (pmc ? 1 : 2); ++rep)
    for (const Var& v : vars) {
      auto launch = [&]() { v.f<<<ncu, v.threads>>>(W, sink, d); };
      for (int w = 0; w < (pmc ? 1 : 3); ++w) launch();
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      const int reps = pmc ? 2 : 20;
      for (int w = 0; w < reps; ++w) launch();
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      unsigned long long h[2 * 1024];
      hipMemcpy(h, d, ncu * 16, hipMemcpyDeviceToHost);
      double ticks = 0, real = 0;
      for (int b = 0; b < ncu; ++b) { ticks += h[2 * b]; real += h[2 * b + 1]; }
      ticks /= ncu; real /= ncu;
      const double us = ms / reps * 1e3;
      const double bytes_cu = v.mode == 2 ? 0.0 : (double)NSTREAM * SLOT;
      printf("%s: %6.1f us per launch (in-kernel %6.1f us, clock %4.0f MHz, %6.0f cycles), fill %5.1f GB/s per CU\n",
             v.name, us, real / 100.0, ticks / (real / 100.0), ticks, bytes_cu / (real / 100.0 * 1e-6) / 1e9);
      hipEventDestroy(e0); hipEventDestroy(e1);
    }
  return 0;
}
