/* qtx.h — C-ABI of libqtx.so, the MI355X (gfx950) W8A8 transformer inference path.
 *
 * This library replaces the ONNXRuntime-CPU execution of the reference's exported
 * encoder/decoder graphs (gebegebegebe/onnx-transformer).  Each entry point names the
 * reference interface it stands in for:
 *
 *   qtx_encoder_forward  <- ort.InferenceSession('encoder_fixed.onnx').run(None,
 *                           {global_in, global_in_1})       reference/onnx_reference_inference.py:625-626
 *                           / run_module("encoder", ...)     onnx_optimized_inference.py:297-304
 *   qtx_decoder_forward  <- InferenceSession('decoder_fixed.onnx').run(None, {global_in,
 *                           global_in_1, global_in_2, global_in_3})
 *                                                            reference/onnx_reference_inference.py:633-639
 *   qtx_greedy_decode    <- greedy_decode(model, src, src_mask, max_len, start_symbol)
 *                                                            reference/onnx_reference_inference.py:622-646
 *                                                            (batched form batch_output.py:659-673)
 *   qtx_embed            <- model.get_src_embed / get_tgt_embed  encoder_decoder.py:54-58
 *   qtx_generator        <- model.generator(x) + torch.max     generator.py:14-15,
 *                                                            reference/onnx_reference_inference.py:640-641
 *   qtx_row_quant        <- quantize_activation_per_token_absmax / quantize_weight_per_channel_absmax
 *                                                            quant_linear.py:30-43 / :5-17
 *   qtx_layernorm_quant  <- LayerNorm.forward (+ the next W8A8Linear's act quant)
 *                                                            layer_norm.py:12-15
 *   qtx_linear_i8        <- W8A8Linear.forward (int8 GEMM + dequant epilogue) quant_linear.py:111-119
 *   qtx_linear_rows      <- W8A8Linear.forward + the per-token quantizer / LayerNorm that
 *                           consumes its output (fused epilogues)        quant_linear.py:111-119
 *   qtx_attention_i8     <- MultiHeadedAttention.attention     attention.py:23-36
 *
 * Conventions: every pointer is a DEVICE pointer (HIP, gfx950) unless the
 * parameter says host; buffers are caller-owned; no entry point allocates device memory
 * except qtx_model_create; `stream` is a hipStream_t (0 = default stream); every function
 * returns 0 on success or a non-zero qtx_status, with a message in qtx_last_error().
 * Thread-compatible: one stream per thread; the model handle is read-only after creation.
 */
#ifndef QTX_H_
#define QTX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  QTX_OK = 0,
  QTX_E_INVALID = 1,   /* bad argument / shape (the reference raises on shape mismatch) */
  QTX_E_HIP = 2,       /* a HIP runtime error, message in qtx_last_error() */
  QTX_E_WORKSPACE = 3, /* workspace too small: see qtx_*_workspace_size */
  QTX_E_UNSUPPORTED = 4,
  QTX_E_DEVICE = 5     /* a kernel flagged an error it cannot repair in the calling
                        * thread's device status word on the model (k_gemm_wsx: FFN1 row-max
                        * exchange timed out, outputs invalid); reported (and cleared) by
                        * qtx_model_check — no later call clears it before that */
} qtx_status;

typedef struct qtx_model qtx_model;

/* make_model hyper-parameters (model.py:15-16).  d_model must be 512, d_ff a multiple of
 * 256 up to 2048, n_heads * 64 == d_model.  weight_bits: 8 (W8A8) or 4 (packed int4). */
typedef struct {
  int32_t src_vocab, tgt_vocab, n_layers, d_model, d_ff, n_heads, max_len, weight_bits;
} qtx_config;

const char* qtx_last_error(void);
const char* qtx_version(void);

/* Number of float tensors qtx_model_create expects, and their names in order (the
 * reference state_dict keys; see qtx/weights.py:tensor_order).  names may be NULL. */
int32_t qtx_model_tensor_count(const qtx_config* cfg);

/* Build the device-resident quantized model from fp32 DEVICE tensors given in
 * tensor_order, plus the positional table pe [max_len, d_model].  Weights are quantized
 * per output channel on the device (quant_linear.py:5-17).  The inputs may be freed after
 * the call returns (it synchronizes `stream`). */
int32_t qtx_model_create(const qtx_config* cfg, const float* const* tensors,
                         int32_t n_tensors, const float* pe, void* stream, qtx_model** out);
int32_t qtx_model_destroy(qtx_model* m);
/* bytes of device memory owned by the model */
size_t qtx_model_device_bytes(const qtx_model* m);

/* Read-only views of the model's device tensors, for the op-by-op traced executor
 * (qtx/trace.py: the reference's node-by-node executor storing every intermediate by
 * name, onnx_optimized_inference.py:32-57).  module 0 = encoder, 1 = decoder; index in the
 * layer's weights.py:linear_names order (encoder 0..3 self_attn.linears, 4 w_1, 5 w_2;
 * decoder 0..3 self_attn, 4..7 src_attn, 8 w_1, 9 w_2).  q: int8 [N,K] (weight_bits 4:
 * packed [N,K/2]), s [N], b [N]: the per-channel quantized weight (quant_linear.py:5-17). */
int32_t qtx_model_linear(const qtx_model* m, int32_t module, int32_t layer, int32_t index,
                         const void** q, const float** s, const float** b, int32_t* N,
                         int32_t* K);
/* LayerNorm a_2 / b_2 [d_model]: sublayer index within the layer, or layer = -1 for the
 * stack's final norm (encoder.py:18, decoder.py:16). */
int32_t qtx_model_norm(const qtx_model* m, int32_t module, int32_t layer, int32_t sub,
                       const float** a, const float** b);

/* Workspace sizes (bytes) for the model-level calls. */
size_t qtx_encoder_workspace_size(const qtx_model* m, int32_t B, int32_t S);
size_t qtx_decoder_workspace_size(const qtx_model* m, int32_t B, int32_t T, int32_t S);
size_t qtx_greedy_workspace_size(const qtx_model* m, int32_t B, int32_t S, int32_t max_len);

/* Encoder graph: x [B,S,d] fp32 (= src_embed(src), "global_in"), src_mask [B,S] uint8
 * (nonzero = keep, "global_in_1" [B,1,S]) -> out [B,S,d] fp32 ("global_out"). */
int32_t qtx_encoder_forward(const qtx_model* m, const float* x, const uint8_t* src_mask,
                            int32_t B, int32_t S, float* out, void* ws, size_t ws_bytes,
                            void* stream);

/* Decoder graph: y [B,T,d] (= tgt_embed(ys), "global_in"), memory [B,S,d] ("global_in_1"),
 * src_mask [B,S] uint8 ("global_in_2"), tgt_mask uint8 [T,T] or [B,T,T]
 * (tgt_mask_batched = 0/1, "global_in_3") -> out [B,T,d] ("global_out"). */
int32_t qtx_decoder_forward(const qtx_model* m, const float* y, const float* memory,
                            const uint8_t* src_mask, const uint8_t* tgt_mask,
                            int32_t tgt_mask_batched, int32_t B, int32_t T, int32_t S,
                            float* out, void* ws, size_t ws_bytes, void* stream);

/* Whole greedy decode: src ids int64 [B,S], src_mask uint8 [B,S] -> ids int64 [B,max_len]
 * (ids[:,0] = start, then max_len-1 greedy steps with no EOS exit, like the reference).
 * KV-cached; results equal the reference's full-prefix recompute (causal invariance). */
int32_t qtx_greedy_decode(const qtx_model* m, const int64_t* src, const uint8_t* src_mask,
                          int32_t B, int32_t S, int32_t max_len, int64_t start, int64_t* ids,
                          void* ws, size_t ws_bytes, void* stream);

/* Synchronise `stream`, then report (and clear) the calling thread's device status word on
 * this model: QTX_OK, or QTX_E_DEVICE if a kernel of any of the thread's model-level calls on
 * it since its last check raised an error (the bits accumulate; nothing but this check clears
 * them).  Thread affinity: the word belongs to the thread that made the calls, so check from
 * that thread; a thread that made no encoder / greedy-decode call on the model gets QTX_OK.
 * A thread claims its word at its first encoder / greedy-decode call on the model and returns
 * it when it exits; at most 256 threads may hold one per model at a time — the call of a
 * further thread fails with QTX_E_UNSUPPORTED instead of sharing a word. */
int32_t qtx_model_check(const qtx_model* m, void* stream);

/* ---- fault injection (the reference's campaigns: inject_utils/layers.py:48-84,
 * onnx_optimized_inference.py:59-204, parallelized_inject_onnx_transformer.py:536-720) ----
 * One fault per run, at one QuantLinear MatMul of one module.  Targets use the reference's
 * ONNX MatMul numbering: encoder layer L MatMul_{8L+i}, i = QTX_LIN_Q/K/V/O/
 * FFN1/FFN2; decoder layer L MatMul_{12+12L+i} (self Q/K/V/O, cross Q/O, FFN) and the
 * memory K/V projections MatMul_{2L}, MatMul_{2L+1} (QTX_LIN_CK / QTX_LIN_CV).
 * Kinds (rows index the module's flattened [B*S] or [B*T] tokens; cross K/V: memory tokens):
 *   INPUT     bit `bit` of the int8 input q[row, col] flipped (every output column)
 *   WEIGHT    bit `bit` of the int8 weight q[row = out channel, col] flipped (every row)
 *   INPUT16   as INPUT, the output perturbation kept on columns win_start .. +win_len (<= 16)
 *   WEIGHT16  as WEIGHT, the perturbation kept on rows win_start .. +win_len (<= 16)
 *   OUTPUT    the MatMul output (before bias) at (row, col) replaced by `value`
 *             (RANDOM: a random float; RANDOM_BITFLIP: a bit-flipped golden value)
 * Attention MatMuls (QTX_LIN_QK / PV, decoder cross QTX_LIN_CQK / CPV; the reference's
 * "FirstMatMul" / "SecondMatMul" campaign targets) on one (sentence b, head h), Sq query
 * and Sk key rows per sentence:
 *   QK  INPUT*:  q element  row = b*Sq + i, col = h*64 + d   (INPUT16 window: keys)
 *       WEIGHT*: k element  row = b*Sk + j, col = h*64 + d   (WEIGHT16 window: query rows)
 *       OUTPUT:  QK^T value row = b*Sq + i, col = h*Sk + j   (before the / 8 and the mask)
 *   PV  INPUT*:  P*127 int  row = b*Sq + i, col = h*Sk + j   (INPUT16 window: head dims)
 *       WEIGHT*: v element  row = b*Sk + j, col = h*64 + d   (WEIGHT16 window: query rows)
 *       OUTPUT:  context    row = b*Sq + i, col = h*64 + d
 * Requires 8-bit weights. */
typedef enum {
  QTX_FAULT_NONE = 0, QTX_FAULT_INPUT = 1, QTX_FAULT_WEIGHT = 2, QTX_FAULT_INPUT16 = 3,
  QTX_FAULT_WEIGHT16 = 4, QTX_FAULT_OUTPUT = 5
} qtx_fault_kind;
typedef enum {
  QTX_LIN_Q = 0, QTX_LIN_K = 1, QTX_LIN_V = 2, QTX_LIN_QK = 3, QTX_LIN_PV = 4, QTX_LIN_O = 5,
  QTX_LIN_FFN1 = 6, QTX_LIN_FFN2 = 7, QTX_LIN_CQ = 8, QTX_LIN_CK = 9, QTX_LIN_CV = 10,
  QTX_LIN_CO = 11, QTX_LIN_CQK = 12, QTX_LIN_CPV = 13
} qtx_linear_id;
typedef struct {
  int32_t kind;      /* qtx_fault_kind */
  int32_t module;    /* 0 encoder, 1 decoder */
  int32_t layer;
  int32_t linear;    /* qtx_linear_id */
  int64_t row, col;  /* see the kinds above */
  int64_t win_start;
  int32_t win_len;
  int32_t bit;       /* 0..7 */
  float value;       /* OUTPUT */
  int32_t reserved;
} qtx_fault;

/* qtx_encoder_forward / qtx_decoder_forward / qtx_greedy_decode with one fault (host
 * pointer; NULL or kind NONE = golden run).  The greedy decode takes encoder faults. */
int32_t qtx_encoder_forward_fault(const qtx_model* m, const float* x, const uint8_t* src_mask,
                                  int32_t B, int32_t S, float* out, void* ws, size_t ws_bytes,
                                  const qtx_fault* fault, void* stream);
int32_t qtx_decoder_forward_fault(const qtx_model* m, const float* y, const float* memory,
                                  const uint8_t* src_mask, const uint8_t* tgt_mask,
                                  int32_t tgt_mask_batched, int32_t B, int32_t T, int32_t S,
                                  float* out, void* ws, size_t ws_bytes,
                                  const qtx_fault* fault, void* stream);
int32_t qtx_greedy_decode_fault(const qtx_model* m, const int64_t* src,
                                const uint8_t* src_mask, int32_t B, int32_t S, int32_t max_len,
                                int64_t start, int64_t* ids, void* ws, size_t ws_bytes,
                                const qtx_fault* fault, void* stream);

/* Embeddings + positional encoding: which = 0 (src) / 1 (tgt); ids int64 [B,T] ->
 * out [B,T,d], positions pos0 .. pos0+T-1. */
int32_t qtx_embed(const qtx_model* m, int32_t which, const int64_t* ids, int32_t B, int32_t T,
                  int32_t pos0, float* out, void* stream);

/* Generator: x [M,d] -> logp [M,tgt_vocab] (may be NULL), ids int64 [M] (first argmax).
 * ws: M * tgt_vocab floats. */
int32_t qtx_generator(const qtx_model* m, const float* x, int32_t M, float* logp,
                      int64_t* ids, void* ws, size_t ws_bytes, void* stream);

/* ---- per-op entry points (parity tests, fault-injection hooks later) ---- */

/* q[r,:] = rint(x[r,:] / s[r]), s[r] = max(max|x[r,:]|, 1e-5) / qmax.  D in {256,512,1024,2048}. */
int32_t qtx_row_quant(const float* x, int32_t rows, int32_t D, float qmax, int8_t* q,
                      float* s, void* stream);

/* y = LN(x) (unbiased std, eps on std); optional fp32 y (may be NULL), optional q/s. */
int32_t qtx_layernorm_quant(const float* x, const float* a, const float* b, int32_t rows,
                            int32_t D, float* y, int8_t* q, float* s, void* stream);

/* out[m,n] = ((float(sum_k A[m,k] W[n,k]) * sa[m]) * sw[n]) + bias[n], then
 * flags: 1 = ReLU, 2 = residual (out = res + y).  weight_bits 8: W int8 [N,K];
 * 4: W packed [N,K/2] (low nibble = even k).  K % 64 == 0. */
int32_t qtx_linear_i8(const int8_t* A, const float* sa, const void* W, const float* sw,
                      const float* bias, int32_t M, int32_t N, int32_t K, int32_t weight_bits,
                      int32_t flags, const float* res, float* out, void* stream);

/* Pack int8 values in [-8,7] [N,K] into int4 [N,K/2]. */
int32_t qtx_pack_int4(const int8_t* q, int32_t N, int32_t K, uint8_t* packed, void* stream);

/* Attention core on quantized Q/K/V laid out [B,S,H*64] with per-token scales [B,S]:
 * ctx [B,Sq,H*64] fp32.  mask uint8 [B,Sq,Sk] with strides (m_bs, m_is) in elements
 * (m_is = 0 broadcasts one row, e.g. the encoder's [B,1,S] mask); NULL = keep all.
 * dec != 0: a decoder layer's attention (decoder.py:28-33), whose PV MatMul runs in the
 * decoder's canonical order (four partial chains); 0: the encoder's. */
int32_t qtx_attention_i8(const int8_t* q, const float* sq, const int8_t* k, const float* sk,
                         const int8_t* v, const float* sv, const uint8_t* mask, int64_t m_bs,
                         int64_t m_is, int32_t B, int32_t H, int32_t Sq, int32_t Sk,
                         float* ctx, int32_t dec, void* stream);

/* qtx_attention_i8 plus the attention MatMuls' intermediates, for the traced executor
 * (run_module(expose_intermediates=...), onnx_optimized_inference.py:57 stores every node
 * output by name): qk_acc [B,H,Sq,Sk] = float(sum_d q k), the exact integer accumulators of
 * QK^T ("FirstMatMul" MatMul_{8L+3}, before the / 8 and the mask); p_codes [B,H,Sq,Sk] =
 * rint(P * 127) (the Round of attention.py:33-35); ctx as qtx_attention_i8, bit for bit.
 * qk_acc / p_codes may be NULL.  Off the hot path (one wave per query row and head). */
int32_t qtx_attention_trace(const int8_t* q, const float* sq, const int8_t* k, const float* sk,
                            const int8_t* v, const float* sv, const uint8_t* mask, int64_t m_bs,
                            int64_t m_is, int32_t B, int32_t H, int32_t Sq, int32_t Sk,
                            float* ctx, float* qk_acc, float* p_codes, int32_t dec, void* stream);

/* Encoder self-attention with the context quantized per token for the O-projection
 * (attention.py:23-67 + quant_linear.py:30-43, replacing the MatMul_{8L+3,8L+4} pair of the
 * encoder graph and the following QuantizeLinear): q/k/v int8 [B,S,512] (8 heads) +
 * per-token scales [B,S], key mask uint8 [B,S] (NULL = keep all) -> ctx8 int8 [B,S,512] +
 * sctx [B,S].  S <= 128.  One workgroup per sentence. */
int32_t qtx_attention_i8_quant(const int8_t* q, const float* sq, const int8_t* k,
                               const float* sk, const int8_t* v, const float* sv,
                               const uint8_t* key_mask, int32_t B, int32_t S, int8_t* ctx8,
                               float* sctx, void* stream);

/* ---- fused decode-step kernels (the KV-cached greedy step is built from these) ---- */

/* Row-complete int8 GEMM (8-bit weights, N % 512 == 0, K % 64 == 0) whose epilogue sees
 * whole 512-wide row segments; y = ((float(sum_k A W) * sa[m]) * sw[n]) + bias[n]:
 *   epi 0  per-token quant of y over each 512-column tile t -> out8 + t*o8_ts [M,512]
 *          (row stride ldo8) and scale os + t*os_ts [M]  (Q/K/V outputs, attention.py:53-56)
 *   epi 1  (N == 512) x = res + y -> xout; LayerNorm(x; ln_a, ln_b) quantized per token
 *          -> lnq [M,512] + lns [M], or fp32 -> lnout when lnq is NULL (sublayer_connection.py
 *          + layer_norm.py of the next sublayer)
 *   epi 2  relu(y): per-row absmax of each tile -> pmax_out [N/512][M]
 *   epi 3  relu(y) quantized per token with m = max_p pmax_in[p][M] (p < pmax_n) ->
 *          out8 [M,N] (ld ldo8) + os [M]         (FFN hidden, position_feed_forward.py:12) */
typedef struct qtx_row_gemm {
  const int8_t* A; const float* sa; const int8_t* W; const float* sw; const float* bias;
  int32_t M, N, K, epi;
  int8_t* out8; int64_t ldo8, o8_ts; float* os; int64_t os_ts;
  const float* res; float* xout; const float* ln_a; const float* ln_b;
  int8_t* lnq; float* lns; float* lnout;
  float* pmax_out; const float* pmax_in; int32_t pmax_n;
  /* kp = 1: A [M (+1 if odd), K] and W in the KP layout (row pair p, K chunk c of 64 bytes
   * = one 128-byte line at ((p * K/64 + c) * 128), rows 2p | 2p+1 at +0 | +64; W packed by
   * qtx_pack_w_kp); lnq (epi 1) and out8 (epi 3) are then written KP, epi 0's out8 row-major.
   * K % 256 == 0.
   * kp = 2: the weight-stationary kernel (K == 512 only): A in the KP layout, W packed by
   * qtx_pack_w_ws; each workgroup keeps a 512-column slice of W on chip and streams 64-row
   * blocks of A.  Outputs exactly as kp = 1, except that epi 3's out8 must hold M + (M & 1)
   * rows (the KP pad row of an odd M is written as scratch).
   * kp = 3: epi 3 in ONE pass (N == 2048, K == 512, W as for kp = 2): the per-token row
   * maximum is exchanged between the column slices' workgroups inside the launch, so
   * pmax_in / pmax_n are not read; pmax_out is the exchange scratch (>= 32 * M + 2048 bytes,
   * overwritten).  The encoder's FFN1 (qtx_encoder_forward at M >= 2048).
   * kp = 4 / 5 (diagnostic library only: QTX_UNSUPPORTED here): kp = 2 epi 0 / kp = 3 on the
   * 32x32x32-MFMA kernels, W in their WS32 layout. */
  int32_t kp;
  /* kp = 3 only: device word OR-ed with 1 when a wait for the partner slices' row maxima
   * timed out (the affected codes came from a partial maximum: the call's outputs are
   * invalid).  NULL: the flag is the u32 at byte offset 1024 * ceil(M / 32) + 4 of pmax_out,
   * zeroed by each launch; read it after the stream completes. */
  uint32_t* status;
  /* epi 1 with kp = 1 only: split K over `ksplit` workgroups per 128-row tile (ksplit in
   * {2, 4, 8}, (K / 64) % (4 * ksplit) == 0), int32 partials in `part` (>= ksplit * M * 2 KB
   * of device scratch), then a row-wise residual + LayerNorm + quant epilogue; the same
   * results.  What the encoder does for FFN2 below 64 row tiles.  0: no split. */
  int32_t* part;
  int32_t ksplit;
} qtx_row_gemm;
int32_t qtx_linear_rows(const qtx_row_gemm* args, void* stream);
/* The encoder's FFN sublayer as ONE launch (position_feed_forward.py:11-12 with its
 * sublayer_connection.py:15-17 residual and the next layer_norm.py:12-15 + quant_linear.py:30-43),
 * replacing the FFN1 (qtx_linear_rows kp = 3) and FFN2 (kp = 1, epi 1) calls:
 *   h = relu(((float(A . W1^T) * sa) * sw1) + b1) quantized per token over all F columns,
 *   x = x + (((float(hq . W2^T) * s_h) * sw2) + b2)   (in place),
 *   LayerNorm(x; ln_a, ln_b) quantized per token -> lnq (KP) + lns [M], or fp32 -> lnout when
 *   lnq is NULL.  A: int8 [M (+1 if odd), 512] in the KP layout (qtx_linear_rows kp = 1);
 *   wf: W1 / W2 packed by qtx_pack_ffn.  lnq / lns may alias A / sa (each 128-row block reads
 *   its rows before it writes them).  F % 64 == 0, 256 <= F <= 2048.  Results equal the two
 *   calls it replaces bit for bit. */
typedef struct qtx_ffn_args {
  const int8_t* A; const float* sa; const int8_t* wf;
  const float* sw1; const float* b1; const float* sw2; const float* b2;
  float* x; const float* ln_a; const float* ln_b;
  int8_t* lnq; float* lns; float* lnout;
  int32_t M, F;
} qtx_ffn_args;
int32_t qtx_ffn_rows(const qtx_ffn_args* args, void* stream);
/* W1 int8 [F, 512] and W2 int8 [512, F] row-major -> the weight stream qtx_ffn_rows reads
 * (F * 1024 bytes): per 64-column chunk c four 16 KB slots of 16 fragments x 64 lanes x 16
 * bytes — slots 4c + h (h = 0, 1; W1 K steps 4h .. 4h+3), fragment 4s' + j', lane l:
 * W1[64c + 16j' + (l & 15)][64(4h + s') + 16(l >> 4) .. +16]; slots 4c + 2 + ch (W2, column
 * half ch), fragment j, lane l: byte 4j' + e = W2[col][64c + 16j' + 4(l >> 4) + e] with
 * col = 16(l & 15) + 8ch + j for j < 8, else 256 + 16(l & 15) + 8ch + j - 8. */
int32_t qtx_pack_ffn(const int8_t* W1, const int8_t* W2, int32_t F, int8_t* out, void* stream);
/* W int8 [N, K] row-major -> out [N, K] in the KP layout with the per-512-column-tile row
 * order qtx_linear_rows(kp = 1) reads.  N % 512 == 0, K % 64 == 0. */
int32_t qtx_pack_w_kp(const int8_t* W, int32_t N, int32_t K, int8_t* out, void* stream);
/* W int8 [N, 512] row-major -> out (N*512 bytes) in the order qtx_linear_rows(kp = 2) reads:
 * for 512-column slice t, wave w (0..7), K step s (0..7), column fragment j (0..3) one 1 KB
 * block at ((t*8 + w)*8 + s)*4 + j whose 16-byte lane l (0..63) holds
 * W[512t + 64w + 16((l & 15) >> 2) + 4j + (l & 3)][64s + 16(l >> 4) .. +16].
 * N % 512 == 0, K == 512. */
int32_t qtx_pack_w_ws(const int8_t* W, int32_t N, int32_t K, int8_t* out, void* stream);

/* Skinny int8 GEMM for decode (M small): out = epilogue(A . W^T) with the A operand made
 * in the prologue: amode 0 = int8 A [M,K] + sa; 1 = LayerNorm(X [M,512]; ln_a, ln_b) then
 * per-token quant; 2 = fp32 X [M,K] quantized per token with s = max(m, 1e-5)/127 where m =
 * max over p < pmax_n of pmax_in[p*M + row] (partial row absmaxima, e.g. per head or per
 * column tile; pmax_n <= 128); 3 = fp32 X [M,K] quantized per token from its own row
 * absmax (the scale amode 2 forms from complete partials).  flags: 1 ReLU, 2 residual
 * (res), 4 partial row absmax of the output per 16-column tile into pmax_out [N/16][M].
 * N % 16 == 0, K in {512, 2048} (amode 1: K = 512); M * max(ldx, K), M * N and N * K below
 * 2^30 (the kernels address their operands with 32-bit byte offsets), else QTX_E_UNSUPPORTED.
 * quant_linear.py:111-119, layer_norm.py:12-15. */
int32_t qtx_skinny_linear(int32_t amode, const int8_t* A, const float* sa, const float* X,
                          int64_t ldx, const float* ln_a, const float* ln_b,
                          const float* pmax_in, int32_t pmax_n, const void* W, const float* sw,
                          const float* bias, int32_t M, int32_t N, int32_t K,
                          int32_t weight_bits, int32_t flags, const float* res, float* out,
                          float* pmax_out, void* stream);

/* One-query-per-sentence attention of the decode step (attention.py:23-67).
 * kv_new = 1 (self): y [B, 3*512] holds this step's q|k|v projections; they are quantized
 *   per token, k/v written to the caches at row b*kv_bs + *step_dev, keys 0..*step_dev
 *   (kv_bs <= 128).
 * kv_new = 0 (cross): y [B,512] holds q; keys = S cached rows per sentence, mask [B,S].
 * Caches: kc int8 [B][kv_bs][512]; vc int8 in groups of 4 keys, [B][ceil(kv_bs/4)][512][4]
 *   (byte ((b*G4 + j/4)*512 + d)*4 + j%4 holds v[b][j][d]: one dword = 4 keys of one dim);
 *   skc/svc [B][kv_bs].  Out: fp32 context ctx [B,512]
 * and the per-head absmax pmax [8][B] (the next GEMM's per-token quantization, amode 2 of
 * qtx_skinny_linear with pmax_n = 8).  Keys <= 128.  The PV MatMul runs in the decoder's
 * canonical order (four partial chains; qtx_attention_i8 with dec = 1). */
int32_t qtx_decode_attention(int32_t kv_new, const float* y, int64_t ldy, int8_t* kc,
                             int8_t* vc, float* skc, float* svc, int32_t kv_bs,
                             const int32_t* step_dev, int32_t S, const uint8_t* mask,
                             int32_t B, float* ctx, float* pmax, void* stream);

/* The decode step's tail (onnx_reference_inference.py:632,640-643): per row m of logits
 * [M, tgt_vocab], the first argmax of log_softmax (generator.py:15, torch.max's tie rule)
 * into ids[m * ids_bs + s + 1], and the next decoder input tgt_embed(id) at position s + 1
 * into x_next [M, d_model], with s = step_dev[0]; step_dev[1] must be 0 (arrival counter);
 * the last workgroup advances step_dev[0] by one. */
int32_t qtx_decode_argmax_embed(const qtx_model* m, const float* logits, int32_t M,
                                int64_t* ids, int64_t ids_bs, int32_t* step_dev,
                                float* x_next, void* stream);

/* An empty one-wave kernel on `stream`: the dependent-launch floor that bench.py subtracts
 * from a chain of launches to get per-kernel durations (measurement only, no reference
 * counterpart). */
int32_t qtx_debug_nop(void* stream);

/* Re-read the library's environment switches (csrc/qtx_knobs.h), which are otherwise read
 * once: the path switches the tests use to force the library's alternative code paths
 * (QTX_NO_GRAPH, QTX_UNFUSED, QTX_DECODE_GROUPS, QTX_NO_WSX, ...) and the hooks of the FFN1
 * exchange's error path (QTX_WSX_SPIN_LIMIT, QTX_WSX_DROP_SLICE).  Not for concurrent use
 * with running calls (test / measurement only, no reference counterpart). */
int32_t qtx_debug_reload_knobs(void);

#ifdef __cplusplus
}
#endif
#endif /* QTX_H_ */
