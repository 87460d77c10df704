// qtx_knobs.h — the library's environment switches, read ONCE (at the first launch that
// consults them), never per launch.  Two kinds:
//   * path switches of the product: alternative code paths the library carries for other
//     shapes (two-pass FFN1, eager decode, unfused decoder, split K, ...) that the test suite
//     forces at the shapes it tests, plus the hooks that make the FFN1 exchange's error path
//     fire deterministically;
//   * diagnostic switches (ablations, measured-negative kernels, timing aids): read only in the
//     QTX_DIAG build (libqtx_diag.so, qtx/_build.py build(extra=...)); in the product build
//     they are compile-time defaults and the variants they select are not compiled in.
// qtx_debug_reload_knobs() (include/qtx.h) re-reads the environment: the tests that switch
// paths within one process call it after changing a variable.
#pragma once

// A diagnostic switch: a field read from the environment in the QTX_DIAG build, a
// compile-time constant (its default) in the product build, so the product's branches on it
// fold away and the library carries only the paths some shape takes by default.
#ifdef QTX_DIAG
#define QTX_DKNOB(T, name, def) T name = def
#else
#define QTX_DKNOB(T, name, def) static constexpr T name = def
#endif

namespace qtx {

struct Knobs {
  // ---- product path switches
  bool no_rowgemm = false;   // QTX_NO_ROWGEMM: the generic GEMM instead of the row GEMMs
  bool no_splitk = false;    // QTX_NO_SPLITK: FFN2 at small M without the K split
  bool no_wsx = false;       // QTX_NO_WSX: FFN1 in two passes instead of the in-launch exchange
  bool no_kp = false;        // QTX_NO_KP: row GEMMs on the plain (non-KP) layout
  bool no_attn_encq = false; // QTX_NO_ATTN_ENCQ: encoder attention without k_attn_encq
  bool enc_nosplit = false;  // QTX_ENC_NOSPLIT: no two-stream encoder (two-pass FFN1 only)
  bool unfused = false;      // QTX_UNFUSED: the unfused decoder step
  bool no_graph = false;     // QTX_NO_GRAPH: eager decode launches
  bool ffn_qkernel = false;  // QTX_FFN_QKERNEL: the FFN hidden quantized by its own kernel
                             // (the default from B >= 96; forced below it by tests)
  int decode_groups = 0;     // QTX_DECODE_GROUPS: sub-batch graphs (0: by batch size)
  int graph_steps = 0;       // QTX_GRAPH_STEPS: decode steps per graph (0: all)
  long ws_min_m = 2048;      // QTX_WS_MIN_M: weight-stationary from this many rows
  long ws_res_min_m = 2048;  // QTX_WS_RES_MIN_M / _MAX_M: the O-projection's WS range
  long ws_res_max_m = 8192;
  int status_slots = 0;      // QTX_STATUS_SLOTS: device status words per model (0: all 256;
                             // tests lower it to make exhaustion happen)
  // ---- hooks of the FFN1 exchange's error path (tests/test_gpu_status.py)
  int wsx_spin_limit = -1;   // QTX_WSX_SPIN_LIMIT: polls per wait (-1: the launcher's bound)
  int wsx_drop_slice = -1;   // QTX_WSX_DROP_SLICE: this column slice never publishes its
                             // row maxima, so its partners' waits time out (-1: none)
  // ---- diagnostic switches (QTX_DIAG build only; constants in the product build)
  // measured-negative decode / GEMM alternatives (round 6, VERDICT r05 item 5: moved out of
  // the product; DESIGN.md records each A/B)
  QTX_DKNOB(bool, group_graph, false);  // QTX_GROUP_GRAPH: sub-batches as branches of one graph
  QTX_DKNOB(bool, split_ln, false);     // QTX_SPLIT_LN: separate LayerNorm kernels in the decode step
  QTX_DKNOB(bool, ws_nopipe, false);    // QTX_WS_NOPIPE: the unpipelined weight-stationary kernel
  QTX_DKNOB(bool, wsr_off, false);      // QTX_WSR=0: the O-projection's WS epilogue on k_gemm_ws
  QTX_DKNOB(bool, attn_pmax, false);    // QTX_ATTN_PMAX: decode O / Oc from the attention's per-head maxima
  QTX_DKNOB(bool, ffn_pmax, false);     // QTX_FFN_PMAX: decode FFN2 from FFN1's per-tile maxima
  QTX_DKNOB(bool, hquant_rows, false);  // QTX_HQUANT_ROWS: the decode hidden quantized by k_rows
  QTX_DKNOB(bool, device_step, false);  // QTX_DEVICE_STEP: self-attention reads its position from
                                        // the device counter even where the host knows it
  QTX_DKNOB(bool, int4_packed, false);  // QTX_INT4_PACKED: a 4-bit model's decode step on the
                                        // packed int4 kernels
  // QTX_FFN_FUSED_MIN_M: the encoder's fused FFN launch (k_ffn_fused) from this many rows
  // (default off — measured slower than the split launches at cfg3, DESIGN.md §4 "The fused
  // FFN kernel"; the product keeps it as the C-ABI entry qtx_ffn_rows only);
  // QTX_NO_FFN_FUSED: never
  QTX_DKNOB(long, ffn_fused_min_m, 1L << 40);
  QTX_DKNOB(bool, no_ffn_fused, false);
  int ablate = 0;            // QTX_ABLATE: kernel classes dropped from the decode step
  bool ablate_nop = false;   // QTX_ABLATE_NOP
  bool dbg_tail = false;     // QTX_DBG_TAIL
  bool time_graph = false;   // QTX_TIME_GRAPH
  bool gemm128 = false;      // QTX_GEMM128
  bool attn_valu = false;    // QTX_ATTN_VALU
  bool encq_nopipe = false;  // QTX_ENCQ_NOPIPE
  int wsq = 1;               // QTX_WSQ: 0 wsp, 1 wsq (product), 2 wss, 3 wsz, 4 wsa
  int wsy = 1;               // QTX_WSY: 0 wsx, 1 wsy (product)
  bool ws_prio = false;      // QTX_WS_PRIO
  bool ws_xg = true;         // QTX_WS_XG
  bool wsp_pmax_sr5 = false; // QTX_WSP_PMAX_SR5
  bool wsa2 = false;         // QTX_WSA2
  int skinny_wide = -1;      // QTX_SKINNY_WIDE
  int rb_i8_512 = 4, rb_ln = 4;   // QTX_RB_*
  int rb_i8_2048 = 0, rb_f32q = 0;  // QTX_RB_I8_2048 / _F32Q (0: by M, qtx_decode.hip skinny_mode)
  int skinny8_maxm = 32;     // QTX_SKINNY8_MAXM
  int ws32 = 0;              // QTX_WS32: Q/K/V + FFN1 on k_gemm_wsq32 / wsy32 (32x32x32 MFMA;
                             // 2: Q/K/V with all of W in registers)
};

// the switches, read from the environment on first use
const Knobs& knobs();
// re-read them (tests; not thread-safe against concurrent launches)
void knobs_reload();
// how many reloads so far: part of every cached decode graph's key, so a graph captured
// under other switches is never replayed after a reload
int knobs_generation();

}  // namespace qtx
