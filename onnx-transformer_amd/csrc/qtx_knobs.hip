// qtx_knobs.hip — reads the environment switches of qtx_knobs.h once.
#include "qtx_knobs.h"

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "../../include/qtx.h"

namespace qtx {
namespace {

bool flag(const char* name, bool def = false) {
  const char* v = getenv(name);
  if (!v || !*v) return def;
  return strcmp(v, "0") != 0;
}
long num(const char* name, long def) {
  const char* v = getenv(name);
  return v && *v ? strtol(v, nullptr, 0) : def;
}

Knobs read_env() {
  Knobs k;
  k.no_rowgemm = flag("QTX_NO_ROWGEMM");
  k.no_splitk = flag("QTX_NO_SPLITK");
  k.no_wsx = flag("QTX_NO_WSX");
  k.no_kp = flag("QTX_NO_KP");
  k.no_attn_encq = flag("QTX_NO_ATTN_ENCQ");
  k.enc_nosplit = flag("QTX_ENC_NOSPLIT");
  k.unfused = flag("QTX_UNFUSED");
  k.no_graph = flag("QTX_NO_GRAPH");
  k.ffn_qkernel = flag("QTX_FFN_QKERNEL");
  k.decode_groups = (int)num("QTX_DECODE_GROUPS", 0);
  k.graph_steps = (int)num("QTX_GRAPH_STEPS", 0);
  k.ws_min_m = num("QTX_WS_MIN_M", 2048L);
  k.ws_res_min_m = num("QTX_WS_RES_MIN_M", 2048L);
  k.ws_res_max_m = num("QTX_WS_RES_MAX_M", 8192L);
  k.status_slots = (int)num("QTX_STATUS_SLOTS", 0);
  k.wsx_spin_limit = (int)num("QTX_WSX_SPIN_LIMIT", -1);
  k.wsx_drop_slice = (int)num("QTX_WSX_DROP_SLICE", -1);
#ifdef QTX_DIAG
  k.group_graph = flag("QTX_GROUP_GRAPH");
  k.split_ln = flag("QTX_SPLIT_LN");
  k.ws_nopipe = flag("QTX_WS_NOPIPE");
  k.wsr_off = getenv("QTX_WSR") && *getenv("QTX_WSR") == '0';
  k.attn_pmax = flag("QTX_ATTN_PMAX");
  k.ffn_pmax = flag("QTX_FFN_PMAX");
  k.hquant_rows = flag("QTX_HQUANT_ROWS");
  k.device_step = flag("QTX_DEVICE_STEP");
  k.int4_packed = flag("QTX_INT4_PACKED");
  k.no_ffn_fused = flag("QTX_NO_FFN_FUSED");
  k.ffn_fused_min_m = num("QTX_FFN_FUSED_MIN_M", 1L << 40);
  k.ablate = (int)num("QTX_ABLATE", 0);
  k.ablate_nop = flag("QTX_ABLATE_NOP");
  k.dbg_tail = flag("QTX_DBG_TAIL");
  k.time_graph = flag("QTX_TIME_GRAPH");
  k.gemm128 = flag("QTX_GEMM128");
  k.attn_valu = flag("QTX_ATTN_VALU");
  k.encq_nopipe = flag("QTX_ENCQ_NOPIPE");
  k.wsq = (int)num("QTX_WSQ", 1);
  k.wsy = (int)num("QTX_WSY", 1);
  k.ws_prio = flag("QTX_WS_PRIO");
  k.ws_xg = flag("QTX_WS_XG", true);
  k.wsp_pmax_sr5 = flag("QTX_WSP_PMAX_SR5");
  k.wsa2 = flag("QTX_WSA2");
  k.skinny_wide = (int)num("QTX_SKINNY_WIDE", -1);
  k.rb_i8_512 = (int)num("QTX_RB_I8_512", 4);
  k.rb_ln = (int)num("QTX_RB_LN", 4);
  k.rb_i8_2048 = (int)num("QTX_RB_I8_2048", 0);
  k.rb_f32q = (int)num("QTX_RB_F32Q", 0);
  k.skinny8_maxm = (int)num("QTX_SKINNY8_MAXM", 32);
  k.ws32 = (int)num("QTX_WS32", 0);
#endif
  return k;
}

Knobs g_knobs;
std::once_flag g_once;
std::atomic<int> g_generation{0};

}  // namespace

const Knobs& knobs() {
  std::call_once(g_once, [] { g_knobs = read_env(); });
  return g_knobs;
}
void knobs_reload() {
  knobs();
  g_knobs = read_env();
  g_generation.fetch_add(1);
}
int knobs_generation() { return g_generation.load(); }

}  // namespace qtx

extern "C" int32_t qtx_debug_reload_knobs(void) {
  qtx::knobs_reload();
  return 0;
}
