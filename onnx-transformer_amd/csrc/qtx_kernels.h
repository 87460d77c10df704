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

// Skinny (decode) GEMM: M <= 64 rows per workgroup, 16 output columns per workgroup,
// the 4 waves split K and reduce their exact int32 partials through LDS.
// The A operand is produced in the prologue according to amode:
enum : int {
  A_I8 = 0,    // int8 A [M,K] + sa[M]
  A_LN = 1,    // fp32 X [M,512]: LayerNorm(ln_a, ln_b) + per-token quant in the prologue
  A_F32Q = 2,  // fp32 X [M,K] + partial absmax: quant with s = max(max_p pmax,1e-5)/127
  A_F32R = 3,  // fp32 X [M,K] quantized per token from its own row absmax (no partials)
};
enum : int {
  EPI_ROWMAX = 4,  // pmax_out[tile][m] = max |y| over the tile's 16 columns (last)
};
struct SkinnyArgs {
  int amode;
  const int8_t* A; const float* sa;               // A_I8
  const float* X; long ldx;                       // A_LN / A_F32Q
  const float* ln_a; const float* ln_b;           // A_LN
  const float* pmax_in; int pmax_n;               // A_F32Q: [pmax_n][M] partial row absmax
  const int8_t* W; long ldw; const float* sw; const float* bias;
  float* out; long ldo; const float* res; long ldr;
  float* pmax_out;                                // EPI_ROWMAX: [N/16][M] per column tile
  int M, N, K, flags;
};

// Fused decode attention: one wave per (sentence b, head h), one query.
//   self  (kv_new != 0): q/k/v rows from y [B, 3*512] fp32 are quantized per token;
//                        k/v appended to the caches at position *step; keys 0..*step.
//   cross (kv_new == 0): q row from y [B, 512]; keys = the S cached cross K/V rows,
//                        masked by mask[b*S + j].
//   Both write the fp32 context ctx [B, 512] and the per-head partial absmax
//   pmax [8][B]; the next GEMM quantizes the row per token from them (A_F32Q).
//   Caches: kc [B][kv_bs][512]; vc in groups of 4 keys, [B][ceil(kv_bs / 4)][512][4]
//   (byte ((b * G4 + j / 4) * 512 + d) * 4 + j % 4 = v[b][j][d]; launch_vgroup4).
struct DecAttnArgs {
  const float* y; long ldy;
  int8_t* kc; int8_t* vc; float* skc; float* svc; long kv_bs;   // [B][kv_bs rows][512]
  const int* step;            // self: current position
  int S;                      // cross: number of keys
  const uint8_t* mask;        // cross: [B, S]
  float* ctx; float* pmax;    // out
  int B, kv_new;
  // self: the position + 1 when the host knows it (a decode step captured at its own
  // position): no read of *step, and only rows 0 .. position staged; 0: read *step and stage
  // all kv_bs rows (a step replayed at several positions)
  int host_step1;
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
  int kp;                     // q in the KP layout ([rows, D], qtx_common.h kp_off)
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
  int dec;                                  // a decoder layer's attention: the decoder's PV
                                            // order (oracle attention_pv dec)
};

// Fault in an attention MatMul of one (sentence b, head h) (k_attn_fault_rows): the
// affected query rows row0 .. row0+nrows-1 are recomputed with it.  i / j / d: the faulty
// element's query row, key, head dim; [lo, hi): the window (keys for AF_QK_INPUT, rows for
// the *_WEIGHT kinds, dims for AF_PV_INPUT).
//   AF_QK_OUTPUT / AF_PV_OUTPUT: the MatMul output at (i, j) / (i, d) replaced by value
enum { AF_QK_INPUT = 1, AF_QK_WEIGHT = 2, AF_PV_INPUT = 3, AF_PV_WEIGHT = 4, AF_QK_OUTPUT = 5,
       AF_PV_OUTPUT = 6 };
struct AttnFault {
  int kind, bit, b, h, i, j, d, lo, hi, row0, nrows;
  float value;
};
hipError_t launch_attn_fault_rows(const AttnArgs& a, const AttnFault& f, hipStream_t st);
// The attention MatMuls' intermediates (k_attn_trace, canonical order): QK^T accumulators
// qk [B,H,Sq,Sk] (float of the exact int), P codes pc [B,H,Sq,Sk] (rint(P*127)), and ctx as
// launch_attention; qk / pc may be null.  Sk <= 512.
hipError_t launch_attn_trace(const AttnArgs& a, float* qk, float* pc, hipStream_t st);

// Row-complete int8 GEMM (large M, 8-bit weights, N % 512 == 0, K % 64 == 0): each
// workgroup owns 128 rows x one 512-wide column tile, so epilogues that need a whole
// 512-wide row segment run in the same kernel.  y = ((float(acc) * sa[m]) * sw[n]) + b[n]:
//   RE_QUANT            per-token quant of y over the tile -> out8 + t*o8_ts [M,512] (ld
//                       ldo8) and scale os + t*os_ts [M]        (Q/K/V outputs, cross K/V)
//   RE_RES_LN           x = res + y -> xout [M,512]; LayerNorm(x) (ln_a, ln_b) quantized per
//                       token -> lnq [M,512] + lns [M], or fp32 -> lnout   (O-proj / FFN2)
//   RE_RELU_PMAX        relu(y): per-row absmax of the tile -> pmax_out [N/512][M] (no y)
//   RE_RELU_QUANT_PMAX  relu(y) quantized per token with the max over pmax_in [pmax_n][M]
//                       -> out8 [M,N] (ld ldo8) + os [M]                 (FFN1, 2nd pass)
//   RE_PARTIAL          (internal: split-K RE_RES_LN at small M) the raw int32 accumulators
//                       of K range blockIdx.y -> part + blockIdx.y * M * 512 [M,512]
enum RowEpi { RE_QUANT = 0, RE_RES_LN = 1, RE_RELU_PMAX = 2, RE_RELU_QUANT_PMAX = 3, RE_PARTIAL = 4 };
// Fault injected into one row-GEMM launch (the reference's fault models, qtx.h qtx_fault),
// in GEMM-local coordinates:
//   FK_INPUT   A[row, col] bit-flipped: acc[row, n] += (flip(a) - a) * W[n, col], n in [lo, hi)
//   FK_WEIGHT  W[row, col] bit-flipped: acc[m, row] += A[m, col] * (flip(w) - w), m in [lo, hi)
//   FK_OUTPUT  the MatMul output (before bias) at (row, col) replaced by value
enum { FK_NONE = 0, FK_INPUT = 1, FK_WEIGHT = 2, FK_OUTPUT = 3 };
struct FaultArgs {
  int kind, bit;
  long row, col, lo, hi;
  float value;
};

struct RowGemmArgs {
  const int8_t* A; long lda; const float* sa;
  const int8_t* W; long ldw; const float* sw; const float* bias;
  int M, N, K, epi;
  int8_t* out8; long ldo8, o8_ts; float* os; long os_ts;
  const float* res; float* xout; const float* ln_a; const float* ln_b;
  int8_t* lnq; float* lns; float* lnout;
  float* pmax_out; const float* pmax_in; int pmax_n;
  FaultArgs fault;                          // kind FK_NONE: no fault (the product path)
  // kp: A and W in the KP layout (W rows additionally in the per-512-tile LDS column order,
  // pack_w_kp), and the int8 lnq / RELU_QUANT out8 outputs written KP (RE_QUANT outputs
  // stay row-major: attention reads them); no fault support.  2: W in the WS layout
  // (weight-stationary, launch_gemm_ws); 3: the one-pass FFN1 (launch_gemm_wsx); 4 / 5: Q/K/V
  // / the one-pass FFN1 with W in the WS32 layout (k_gemm_wsq32 / wsy32: diagnostic build)
  int kp;
  // k_gemm_wsx (kp = 3): device status word OR-ed with DEV_E_EXCHANGE_TIMEOUT when a wait
  // for the partner slices' row maxima hit its spin bound (that block's codes were then
  // quantized from a partial maximum: the host must report the error, never use them);
  // nullptr: the u32 after the ticket counter in the exchange scratch.  spin_limit: polls
  // per wait before giving up (0: the launcher's default).
  unsigned* status;
  int spin_limit;
  int drop_slice;           // test hook (QTX_WSX_DROP_SLICE): this slice never publishes; -1
  // RE_RES_LN with kp at small M (at most 64 row tiles): split K over ksplit workgroups per
  // tile (int32 partials into part [ksplit][M][512], >= ksplit * M * 2 KB), then one wave per
  // row sums them and runs the residual + LayerNorm + quant epilogue.  0 / 1: no split.
  int32_t* part;
  int ksplit;
  // side job of the Q/K/V launch (k_gemm_wsq, encoder): zero `zero16` 16-byte chunks at
  // `zero` — the next one-pass FFN1's exchange scratch (granules, ticket) — so that launch
  // needs no zeroing kernel of its own (prezeroed).  0: none.
  void* zero;
  long zero16;
  int prezeroed;   // kp = 3: the exchange scratch is already zero (launch_gemm_wsx)
};
enum : unsigned { DEV_E_EXCHANGE_TIMEOUT = 1u };
// W [N, K] int8 row-major -> KP layout with the row GEMM's column permutation per 512-wide
// tile (LDS row rho holds column (rho & ~127) + 8 (rho & 15) + ((rho >> 4) & 7))
hipError_t launch_pack_w_kp(const int8_t* W, int N, int K, int8_t* out, hipStream_t st);
hipError_t launch_gemm_row(const RowGemmArgs& a, hipStream_t st);
// Weight-stationary variant for K == 512 (qtx_wsgemm.hip): each workgroup keeps a 512-column
// slice of W in registers and streams 64-row blocks of A (KP layout); W packed by
// launch_pack_w_ws.  Same epilogues and outputs as launch_gemm_row(kp = 1); no faults.
hipError_t launch_gemm_ws(const RowGemmArgs& a, hipStream_t st);
// FFN1 in one pass (N = 2048, K = 512, WS weights, RE_RELU_QUANT_PMAX outputs): the slices'
// row maxima exchanged in-launch through the u64 granule array in a.pmax_out (>= 32*M B)
hipError_t launch_gemm_wsx(const RowGemmArgs& a, hipStream_t st);
hipError_t launch_pack_w_ws(const int8_t* W, int N, int K, int8_t* out, hipStream_t st);

// The encoder's FFN sublayer in one launch (qtx_ffn.hip, k_ffn_fused): FFN1 (+ReLU, per-token
// quantization of the hidden over all F columns) and FFN2 (+residual, next LayerNorm + quant)
// per 128-row block, the hidden kept on chip.  A: x1q int8 [M (+1 if odd), 512] in the KP
// layout, sa [M]; wf: the weight stream (launch_pack_ffn); x [M, 512] fp32 residual in,
// x + FFN(x) out (in place); then LayerNorm(ln_a, ln_b) quantized -> lnq (KP) + lns [M], or
// fp32 -> lnout when lnq is null.  F % 64 == 0, 256 <= F <= 2048.
struct FfnArgs {
  const int8_t* A; const float* sa;
  const int8_t* wf;
  const float* sw1; const float* b1;        // [F]
  const float* sw2; const float* b2;        // [512]
  float* x;
  const float* ln_a; const float* ln_b;
  int8_t* lnq; float* lns; float* lnout;
  int M, F;
};
hipError_t launch_ffn_fused(const FfnArgs& a, hipStream_t st);
// W1 int8 [F, 512], W2 int8 [512, F] -> the stream k_ffn_fused reads (F * 1024 bytes)
hipError_t launch_pack_ffn(const int8_t* W1, const int8_t* W2, int F, int8_t* out, hipStream_t st);

hipError_t launch_gemm(const GemmArgs& a, int wbits, hipStream_t st);
hipError_t launch_skinny(const SkinnyArgs& a, int wbits, hipStream_t st);
hipError_t launch_dec_attn(const DecAttnArgs& a, int B, hipStream_t st);
// [B * S, 512] int8 values (L layers, layer stride v_ls) -> k_dec_attn's 4-key group layout
// (DecAttnArgs::vc; layer stride o_ls, B * ceil(S / 4) * 2048 bytes per layer)
hipError_t launch_vgroup4(const int8_t* v, long v_ls, int L, int B, int S, int8_t* out,
                          long o_ls, hipStream_t st);
// per-token int8 quantization of fp32 rows of 2048 (q row-major [M, 2048], s [M])
hipError_t launch_quant_h2048(const float* X, long ldx, int M, int8_t* q, float* s,
                              hipStream_t st);
// generator with the final LayerNorm fused in (ln_a may be null = no LN)
// the same on fp32 MFMA (bit-identical chain); Wt = generator weight transposed [512][V]
hipError_t launch_generator_mfma(const float* x, long ldx, int M, const float* ln_a,
                                 const float* ln_b, const float* Wt, const float* b, int V,
                                 float* logits, hipStream_t st);
hipError_t launch_transpose(const float* in, int R, int C, float* out, hipStream_t st);
hipError_t launch_pack_gen(const float* W, int V, float* out, hipStream_t st);
// log_softmax + argmax + next-token embedding + step increment (decode tail):
//   ids[m, *step + 1] = argmax;  xnext[m] = lut[id]*sqrt(512) + pe[*step + 1];
//   the last workgroup to finish advances *step (arrive is its private counter).
hipError_t launch_argmax_embed(const float* logits, int M, int V, int64_t* ids, long ids_bs,
                               int* step, unsigned* arrive, const float* lut, const float* pe,
                               int max_pos, float* xnext, hipStream_t st, int host_s1 = 0);
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
hipError_t launch_nop(hipStream_t st);
hipError_t launch_gemm256(const GemmArgs& g, hipStream_t st);
hipError_t launch_attention_mfma(const AttnArgs& a, hipStream_t st);
// encoder self-attention, all heads of a sentence per workgroup, context quantized per
// token -> ctx8 (row stride a.c_ld) + sctx; hipErrorNotSupported unless H == 8,
// Sq == Sk <= 128 and the mask is per key (m_is == 0), and (unless forced) B >= 128
hipError_t launch_attention_encq(const AttnArgs& a, int8_t* ctx8, float* sctx, hipStream_t st,
                                 bool force_encq = false, bool kp = false);
hipError_t launch_fill_col(int64_t* ids, long bs, int B, int64_t val, hipStream_t st);
// zero bytes (multiple of 16, 16-byte aligned) with a kernel (capturable into a hipGraph)
hipError_t launch_zero(void* p, size_t bytes, hipStream_t st);

}  // namespace qtx
