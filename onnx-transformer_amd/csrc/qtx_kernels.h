// qtx_kernels.h — argument blocks and launcher declarations for the gfx950 kernels.
// Internal to libqtx (the public C-ABI is include/qtx.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qtx {

enum : int {
  EPI_RELU = 1,      // y = max(y, 0)                         (position_feed_forward.py:12)
  EPI_RESIDUAL = 2,  // out = res + y  (res may alias out)     (sublayer_connection.py:17)
};

// C[m, n] = A[m, :] . W[n, :]   (int8 x int8 -> int32, exact)
// y = ((float(acc) * sa[m]) * sw[n]) + bias[n]  then the EPI_* flags.
struct GemmArgs {
  const int8_t* A; long lda;      // [M, K] row-major, int8
  const float* sa;                // [M] per-token scales
  const int8_t* W; long ldw;      // [N, K] int8 (ldw in bytes; int4: [N, K/2] packed)
  const float* sw;                // [N] per-channel scales
  const float* bias;              // [N]
  float* out; long ldo;           // [M, N] fp32
  const float* res; long ldr;     // residual (EPI_RESIDUAL)
  int M, N, K;
  int flags;
};

// Row quantizer / LayerNorm+quantizer over rows of D floats (one wave per row).
//   x row r at x + r*ldx.  If ln_a: y = LN(x) (layer_norm.py:12-15) else y = x.
//   If yout: yout row r = y (fp32).   If q: quantize y per row (quant_linear.py:30-43)
//   into q row dst(r), scale s[dst(r)], dst(r) = (r / rpb) * dst_bstride + dst_off + r % rpb.
struct RowArgs {
  const float* x; long ldx;
  const float* ln_a; const float* ln_b;
  float* yout; long ldy;
  int8_t* q; long ldq; float* s;
  int rows, D;
  int rpb; long dst_bstride; const int* dst_off_dev; int dst_off;  // KV-cache scatter
  float qmax;
};

// Attention core (attention.py:23-36) for one (batch, head) per workgroup.
struct AttnArgs {
  const int8_t* q; long q_bs, q_ld; const float* sq; long sq_bs;
  const int8_t* k; long k_bs, k_ld; const float* sk; long sk_bs;
  const int8_t* v; long v_bs, v_ld; const float* sv; long sv_bs;
  const uint8_t* mask; long m_bs, m_is;     // keep[b, i, j] = mask[b*m_bs + i*m_is + j]
  float* ctx; long c_bs, c_ld;
  int B, H, Sq, Sk;                         // Sk: keys used (<= cached length)
  const int* sk_dev; int sk_add;            // if sk_dev: Sk = *sk_dev + sk_add (decode)
  const int* qpos_dev;                      // if set, query i's mask row = *qpos_dev + i
};

hipError_t launch_gemm(const GemmArgs& a, int wbits, hipStream_t st);
hipError_t launch_rows(const RowArgs& a, hipStream_t st);
hipError_t launch_attention(const AttnArgs& a, hipStream_t st);
hipError_t launch_embed(const int64_t* ids, long ids_bs, int B, int T, const int* pos_dev,
                        int pos0, const float* lut, int vocab, const float* pe, int max_len,
                        float* out, long out_bs, hipStream_t st);
hipError_t launch_generator(const float* x, long ldx, int M, const float* W, const float* b,
                            int V, float* logits, hipStream_t st);
hipError_t launch_logsoftmax_argmax(const float* logits, int M, int V, float* logp,
                                    int64_t* ids, long ids_bs, const int* col_dev,
                                    int col_add, hipStream_t st);
hipError_t launch_pack_int4(const int8_t* q, int N, int K, uint8_t* packed, hipStream_t st);
hipError_t launch_u8_from_any(const void* src, int elem_bytes, long n, uint8_t* dst,
                              hipStream_t st);
hipError_t launch_step_inc(int* step, hipStream_t st);
hipError_t launch_fill_col(int64_t* ids, long bs, int B, int64_t val, hipStream_t st);

}  // namespace qtx
