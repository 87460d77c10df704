// qtx_api.hip — the C-ABI (include/qtx.h): model handle, per-op entry points and the
// encoder / decoder / greedy-decode drivers built from the kernels of qtx_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <string>
#include <vector>

#include "../../include/qtx.h"
#include "qtx_kernels.h"
#include "qtx_knobs.h"

using namespace qtx;

#ifdef QTX_DIAG
namespace qtx {   // csrc/diag/qtx_wsgemm_diag.hip
hipError_t launch_pack_w_ws32(const int8_t* W, int N, int K, int8_t* out, hipStream_t st);
}
#endif

namespace {

thread_local std::string g_err;

// the WS32 copies exist only in the diagnostic build (qws32 stays null in the product)
hipError_t pack_w_ws32(const int8_t* W, int N, int K, int8_t* out, hipStream_t st) {
#ifdef QTX_DIAG
  return launch_pack_w_ws32(W, N, K, out, st);
#else
  (void)W; (void)N; (void)K; (void)out; (void)st;
  return hipErrorInvalidValue;
#endif
}

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(QTX_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                  __LINE__);                                                            \
  } while (0)

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// bump allocator over a caller-provided (or model-owned) device region
struct Arena {
  uint8_t* base = nullptr;
  size_t cap = 0, used = 0;
  template <class T>
  T* take(size_t n) {
    const size_t off = align_up(used);
    used = off + n * sizeof(T);
    return base ? reinterpret_cast<T*>(base + off) : nullptr;
  }
};

}  // namespace

// One quantized linear: int8 q [N,K] (or packed int4 [N,K/2]), per-channel scale, bias.
struct QLin {
  int8_t* q = nullptr;
  float* s = nullptr;
  float* b = nullptr;
  int N = 0, K = 0;
  int8_t* qkp = nullptr;   // encoder, 8-bit: q in the row GEMM's KP layout (pack_w_kp)
  int8_t* qws = nullptr;   // encoder, 8-bit, K == 512: q in the weight-stationary order
  int8_t* qws32 = nullptr; // encoder Q/K/V, FFN1 in the WS32 order (diagnostic build: QTX_WS32)
  // 4-bit models: the int4 values (in [-7, 7]) unpacked to int8 [N, K] once at load, so the
  // int8 kernels run them — exact (integer products), and the decode is latency-bound, so
  // the packed form's half bytes bought nothing while its unpack lengthened every kernel
  // (cfg4 15.97 vs cfg2 14.45 ms per decode at r03d).  q stays packed (qtx_model_linear).
  int8_t* q8 = nullptr;
  const int8_t* w8() const { return q8 ? q8 : q; }   // the int8 form (8-bit models: q)
};

struct EncLayer {
  QLin qkv, o, w1, w2;
  const float* ln[2][2];
  int8_t* ffn = nullptr;   // W1 + W2 as k_ffn_fused's weight stream (launch_pack_ffn)
};
struct DecLayer {
  QLin qkv, o, cq, ckv, co, w1, w2;
  const float* ln[3][2];
};

// The captured decode graphs depend on the shapes and the workspace only: the caller's
// ids and src_mask are staged through workspace buffers around each replay, so callers
// that allocate fresh id/mask tensors per call still hit the cache.
struct GraphKey {
  int B, S, L, G;
  const void* ws;
  std::string variant;   // the QTX_* experiment switches the captured step depends on
  bool operator<(const GraphKey& o) const {
    return std::tie(B, S, L, G, ws, variant) < std::tie(o.B, o.S, o.L, o.G, o.ws, o.variant);
  }
};
struct GraphEntry {
  std::vector<hipGraphExec_t> execs;   // one graph per sub-batch
  hipEvent_t done = nullptr;           // recorded after the entry's last replay
};

// The fused decode runs the batch as up to QTX_MAX_GROUPS independent sub-batches, each a
// graph on its own stream (qtx_greedy_decode).
constexpr int QTX_MAX_GROUPS = 4;

struct qtx_model {
  qtx_config cfg;
  std::vector<EncLayer> enc;
  std::vector<DecLayer> dec;
  const float* enc_norm[2];
  const float* dec_norm[2];
  const float *src_lut, *tgt_lut, *pe, *gen_w, *gen_b;
  float* gen_wt = nullptr;   // generator weight in k_generator_mfma's MFMA order (pack_gen)
  // the decoder layers' cross K/V linears as ONE [n_layers * 2 * d_model, d_model] linear
  // (each dec[l].ckv is a view of rows 2 d_model l ..): the once-per-decode cross K/V of all
  // layers in one launch instead of n_layers (cross_kv)
  QLin ckv_all;
  void* mem = nullptr;
  size_t bytes = 0;
  // decode-step graphs, keyed by shape and the buffers baked into them
  std::mutex mu;
  hipStream_t gstream[QTX_MAX_GROUPS] = {};
  hipEvent_t ev_in = nullptr, ev_out[QTX_MAX_GROUPS] = {};
  std::map<GraphKey, GraphEntry> graphs;
  // encoder sub-batch pipelining: second stream + fork/lag/join events (lazily created)
  hipStream_t estream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_lag = nullptr, ev_join = nullptr;
  int device = 0;            // the device the model's memory lives on
  unsigned long long serial = 0;   // unique per created model (call status records)
  unsigned* status = nullptr;      // kStatusSlots 16-byte status words (model memory)
  std::mutex slot_mu;              // guards slot_used
  std::vector<bool> slot_used;     // a live thread holds the slot (qtx_api.hip CallStatus)
  std::vector<bool> slot_had_owner;  // a thread held the slot before (its kernels may still
                                     // be in flight on that thread's streams)
  // an exec may still be running on a caller's stream: wait for its last replay first
  void clear_graphs() {
    for (auto& kv : graphs) {
      if (kv.second.done) {
        (void)hipEventSynchronize(kv.second.done);
        (void)hipEventDestroy(kv.second.done);
      }
      for (hipGraphExec_t e : kv.second.execs) (void)hipGraphExecDestroy(e);
    }
    graphs.clear();
  }
};

namespace {
// Makes the model's device current for the lifetime of the guard (streams and events are
// created on the current device), restoring the caller's device afterwards.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
    else prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
}  // namespace

namespace {

// ---- the device status word ------------------------------------------------------------
const char* status_text(unsigned v) {
  return (v & DEV_E_EXCHANGE_TIMEOUT)
             ? "k_gemm_wsx: the in-launch exchange of FFN1 row maxima timed out (the encoder's "
               "FFN hidden was quantized from a partial row maximum): outputs invalid"
             : "device status word set";
}
// Status words live in the model's own memory: kStatusSlots 16-byte words, one per live
// calling thread.  A thread's first model-level call that can raise a device error (the
// encoder and greedy-decode entry points) claims a free slot and zeroes it (call_status_begin);
// the slot returns to the model when the thread exits.  A thread should check (or at least
// synchronise) before it exits: an error its kernels raise after it is gone is dropped when
// the next owner claims the slot.  A kernel that detects an error it
// cannot repair (k_gemm_wsy's exchange timeout) ORs a DEV_E_* bit into the word, and the bit
// stays until qtx_model_check reports it (later calls never clear it: ADVICE r04).
// qtx_model_check(m, stream) synchronises the stream and reads the calling thread's word,
// so an error is reported to the thread whose call raised it and no other thread's call can
// clear it, and no later use of a caller's workspace can overwrite it.
// No slot is ever shared: a thread that finds every slot held by a live thread gets
// QTX_E_UNSUPPORTED (VERDICT r04 hygiene; QTX_STATUS_SLOTS lowers the cap for the test).
constexpr int kStatusSlots = 256;
struct CallStatus {
  const qtx_model* m = nullptr;
  unsigned long long serial = 0;    // the model's creation serial (a new model at a freed
  int slot = -1;                    // address is a different model)
};
// live models by serial: a thread's exit returns its slots only to models still alive
std::mutex g_live_mu;
std::map<unsigned long long, qtx_model*> g_live;
void release_slot(const CallStatus& c);
struct ThreadCalls {
  std::vector<CallStatus> v;
  ~ThreadCalls() {
    for (const CallStatus& c : v) release_slot(c);
  }
};
thread_local ThreadCalls t_calls;

int status_slot_cap() {
  const int n = knobs().status_slots;
  return n > 0 && n < kStatusSlots ? n : kStatusSlots;
}

// the calling thread's word for m if it holds one (nullptr otherwise)
unsigned* held_status_word(const qtx_model* m) {
  for (const CallStatus& c : t_calls.v)
    if (c.m == m && c.serial == m->serial) return m->status + 4 * c.slot;
  return nullptr;
}

// the calling thread's word for m (nullptr: every slot is held by a live thread); *fresh is
// set when the slot was claimed by this call (its word must be zeroed), *reused when a
// thread held that slot before
unsigned* thread_status_word(qtx_model* m, bool* fresh, bool* reused) {
  *fresh = false;
  *reused = false;
  if (unsigned* w = held_status_word(m)) return w;
  int slot = -1;
  {
    std::lock_guard<std::mutex> lk(m->slot_mu);
    const int cap = status_slot_cap();
    for (int i = 0; i < cap; ++i)
      if (!m->slot_used[i]) {
        m->slot_used[i] = true;
        *reused = m->slot_had_owner[i];
        m->slot_had_owner[i] = true;
        slot = i;
        break;
      }
  }
  if (slot < 0) return nullptr;
  // drop the records of models destroyed since (their serials are gone from g_live)
  {
    std::lock_guard<std::mutex> lk(g_live_mu);
    auto& v = t_calls.v;
    v.erase(std::remove_if(v.begin(), v.end(),
                           [](const CallStatus& c) {
                             auto it = g_live.find(c.serial);
                             return it == g_live.end() || it->second != c.m;
                           }),
            v.end());
  }
  t_calls.v.push_back(CallStatus{m, m->serial, slot});
  *fresh = true;
  return m->status + 4 * slot;
}

void release_slot(const CallStatus& c) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  auto it = g_live.find(c.serial);
  if (it == g_live.end() || it->second != c.m) return;   // the model is gone
  qtx_model* m = it->second;
  std::lock_guard<std::mutex> lk2(m->slot_mu);
  m->slot_used[c.slot] = false;
}

// the calling thread's word, claimed and zeroed by its first status-carrying call on the
// model: zeroed eagerly (a synchronous hipMemset, so a claim cannot be
// captured into a graph and never run), and — when a thread held the slot before and may
// have exited with kernels still in flight that can set a bit — after the device has
// drained them, so no stale bit of the previous owner survives the zero
int call_status_begin(const qtx_model* mc, unsigned** word, hipStream_t st) {
  qtx_model* m = const_cast<qtx_model*>(mc);
  if ((*word = held_status_word(m)) != nullptr) return QTX_OK;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIPCHK(hipStreamIsCapturing(st, &cs));
  if (cs != hipStreamCaptureStatusNone)
    return fail(QTX_E_INVALID,
                "a thread's first encoder / greedy call on a model claims its device status "
                "word and cannot be stream-captured: make one uncaptured call first");
  bool fresh = false, reused = false;
  *word = thread_status_word(m, &fresh, &reused);
  if (!*word)
    return fail(QTX_E_UNSUPPORTED,
                "every device status word of this model is held by a live thread (%d): "
                "at most that many threads may call one model at a time",
                status_slot_cap());
  if (fresh) {
    if (reused) HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemset(*word, 0, 16));
  }
  return QTX_OK;
}

// ---- model layout ---------------------------------------------------------------------
// Linear order per layer follows qtx/weights.py:linear_names():
//   enc: self_attn.linears.0..3, w_1, w_2        (6 linears, 12 tensors)
//   dec: self_attn.linears.0..3, src_attn.linears.0..3, w_1, w_2   (10 linears)
int enc_tensor_base(const qtx_config& c, int L) { return 12 * L; }
int dec_tensor_base(const qtx_config& c, int L) { return 12 * c.n_layers + 20 * L; }
int norm_tensor_base(const qtx_config& c) { return 32 * c.n_layers; }

int check_cfg(const qtx_config* c) {
  if (!c) return fail(QTX_E_INVALID, "null config");
  if (c->d_model != 512 || c->n_heads * 64 != c->d_model)
    return fail(QTX_E_UNSUPPORTED, "d_model must be 512 with 64-wide heads");
  if (c->d_ff % 256 || c->d_ff > 2048 || c->d_ff < 256)
    return fail(QTX_E_UNSUPPORTED, "d_ff must be a multiple of 256 <= 2048");
  if (c->weight_bits != 8 && c->weight_bits != 4)
    return fail(QTX_E_UNSUPPORTED, "weight_bits must be 8 or 4");
  if (c->n_layers <= 0 || c->src_vocab <= 0 || c->tgt_vocab <= 0 || c->max_len <= 0)
    return fail(QTX_E_INVALID, "bad config");
  return QTX_OK;
}

size_t wbytes(const qtx_config& c, int N, int K) {
  return c.weight_bits == 8 ? (size_t)N * K : (size_t)N * K / 2;
}

// quantize rows [row0, row0+N) of lin from fp32 W [N,K] on device
int quantize_into(const qtx_config& c, QLin& L, int row0, const float* W, const float* b,
                  int N, int K, int8_t* tmp, hipStream_t st) {
  RowArgs a{};
  a.x = W; a.ldx = K; a.rows = N; a.D = K;
  a.qmax = c.weight_bits == 8 ? 127.0f : 7.0f;
  a.rpb = N; a.dst_bstride = 0; a.dst_off = 0;
  a.s = L.s + row0;
  if (c.weight_bits == 8) {
    a.q = L.q + (size_t)row0 * K; a.ldq = K;
    HIPCHK(launch_rows(a, st));
  } else {
    a.q = tmp; a.ldq = K;
    HIPCHK(launch_rows(a, st));
    HIPCHK(launch_pack_int4(tmp, N, K, reinterpret_cast<uint8_t*>(L.q) + (size_t)row0 * K / 2,
                            st));
    if (L.q8)
      HIPCHK(hipMemcpyAsync(L.q8 + (size_t)row0 * K, tmp, (size_t)N * K, hipMemcpyDeviceToDevice, st));
  }
  HIPCHK(hipMemcpyAsync(L.b + row0, b, N * sizeof(float), hipMemcpyDeviceToDevice, st));
  return QTX_OK;
}

}  // namespace

// =======================================================================================
extern "C" {

const char* qtx_last_error(void) { return g_err.c_str(); }
const char* qtx_version(void) { return "qtx 0.1 gfx950"; }

int32_t qtx_model_tensor_count(const qtx_config* cfg) {
  if (check_cfg(cfg)) return -1;
  const int L = cfg->n_layers;
  return 12 * L + 20 * L + 2 * (2 * L + 1 + 3 * L + 1) + 4;
}

int32_t qtx_model_create(const qtx_config* cfg, const float* const* t, int32_t n,
                         const float* pe, void* stream, qtx_model** out) {
  if (int e = check_cfg(cfg)) return e;
  if (!t || !pe || !out) return fail(QTX_E_INVALID, "null argument");
  if (n != qtx_model_tensor_count(cfg))
    return fail(QTX_E_INVALID, "expected %d tensors, got %d", qtx_model_tensor_count(cfg), n);
  for (int i = 0; i < n; ++i)
    if (!t[i]) return fail(QTX_E_INVALID, "tensor %d is null", i);
  hipStream_t st = (hipStream_t)stream;
  const qtx_config c = *cfg;
  const int D = c.d_model, F = c.d_ff, NL = c.n_layers;

  // ---- size the arena (two passes of the same carve) ----
  auto carve = [&](qtx_model* m, Arena& ar) {
    auto lin = [&](QLin& L, int N, int K) {
      L.N = N; L.K = K;
      L.q = ar.take<int8_t>(wbytes(c, N, K));
      if (c.weight_bits == 4) L.q8 = ar.take<int8_t>((size_t)N * K);
      L.s = ar.take<float>(N);
      L.b = ar.take<float>(N);
    };
    m->enc.resize(NL);
    m->dec.resize(NL);
    for (auto& e : m->enc) { lin(e.qkv, 3 * D, D); lin(e.o, D, D); lin(e.w1, F, D); lin(e.w2, D, F); }
    for (auto& e : m->enc)
        for (QLin* L : {&e.qkv, &e.o, &e.w1, &e.w2}) L->qkp = ar.take<int8_t>((size_t)L->N * L->K);
    if (c.d_ff % 512 == 0)   // weight-stationary copies (K = 512 GEMMs)
      for (auto& e : m->enc) {
        for (QLin* L : {&e.qkv, &e.o, &e.w1}) L->qws = ar.take<int8_t>((size_t)L->N * L->K);
#ifdef QTX_DIAG
        for (QLin* L : {&e.qkv, &e.w1}) L->qws32 = ar.take<int8_t>((size_t)L->N * L->K);
#endif
      }
#ifdef QTX_DIAG
    // the fused FFN's weight stream (F KB per layer): only where QTX_FFN_FUSED_MIN_M can turn
    // that launch on (the diagnostic build; measured slower than the split launches, DESIGN
    // §4), not 12 MB of every product model
    if (c.d_ff % 64 == 0)
      for (auto& e : m->enc) e.ffn = ar.take<int8_t>((size_t)F * 1024);
#endif
    lin(m->ckv_all, NL * 2 * D, D);
    for (int l = 0; l < NL; ++l) {   // dec[l].ckv: rows 2Dl .. 2D(l+1) of ckv_all
      QLin& v = m->dec[l].ckv;
      const QLin& a = m->ckv_all;
      v.N = 2 * D; v.K = D;
      if (a.q) {
        v.q = a.q + wbytes(c, 2 * D, D) * l;
        v.q8 = a.q8 ? a.q8 + (size_t)2 * D * D * l : nullptr;
        v.s = a.s + 2 * D * l;
        v.b = a.b + 2 * D * l;
      }
    }
    for (auto& d : m->dec) {
      lin(d.qkv, 3 * D, D); lin(d.o, D, D); lin(d.cq, D, D);
      lin(d.co, D, D); lin(d.w1, F, D); lin(d.w2, D, F);
    }
    float* norms = ar.take<float>((size_t)2 * D * (5 * NL + 2));
    float* src_lut = ar.take<float>((size_t)c.src_vocab * D);
    float* tgt_lut = ar.take<float>((size_t)c.tgt_vocab * D);
    float* pe_d = ar.take<float>((size_t)c.max_len * D);
    float* gw = ar.take<float>((size_t)c.tgt_vocab * D);
    float* gb = ar.take<float>(c.tgt_vocab);
    int8_t* tmp = ar.take<int8_t>((size_t)F * D);
    m->gen_wt = ar.take<float>((size_t)((c.tgt_vocab + 15) / 16) * 16 * D);
    m->status = ar.take<unsigned>(4 * kStatusSlots);
    return std::make_tuple(norms, src_lut, tgt_lut, pe_d, gw, gb, tmp);
  };
  qtx_model* m = new qtx_model();
  static std::atomic<unsigned long long> next_serial{1};
  m->serial = next_serial.fetch_add(1);
  m->slot_used.assign(kStatusSlots, false);
  m->slot_had_owner.assign(kStatusSlots, false);
  {
    std::lock_guard<std::mutex> lk(g_live_mu);
    g_live[m->serial] = m;
  }
  m->cfg = c;
  (void)hipGetDevice(&m->device);
  Arena sizing;
  carve(m, sizing);
  const size_t bytes = align_up(sizing.used);
  void* mem = nullptr;
  hipError_t he = hipMalloc(&mem, bytes);
  if (he != hipSuccess) {
    delete m;
    return fail(QTX_E_HIP, "hipMalloc(%zu): %s", bytes, hipGetErrorString(he));
  }
  m->mem = mem;
  m->bytes = bytes;
  Arena ar;
  ar.base = (uint8_t*)mem;
  ar.cap = bytes;
  float *norms, *src_lut, *tgt_lut, *pe_d, *gw, *gb;
  int8_t* tmp;
  std::tie(norms, src_lut, tgt_lut, pe_d, gw, gb, tmp) = carve(m, ar);
  if (hipMemset(m->status, 0, 16 * kStatusSlots) != hipSuccess) {
    qtx_model_destroy(m);
    return fail(QTX_E_HIP, "hipMemset(status words)");
  }

  int rc = QTX_OK;
  auto Q = [&](QLin& L, int row0, int ti, int N, int K) {
    if (rc == QTX_OK) rc = quantize_into(c, L, row0, t[ti], t[ti + 1], N, K, tmp, st);
  };
  for (int l = 0; l < NL; ++l) {
    const int b = enc_tensor_base(c, l);
    EncLayer& e = m->enc[l];
    for (int i = 0; i < 3; ++i) Q(e.qkv, i * D, b + 2 * i, D, D);
    Q(e.o, 0, b + 6, D, D);
    Q(e.w1, 0, b + 8, F, D);
    Q(e.w2, 0, b + 10, D, F);
  }
  for (int l = 0; l < NL; ++l) {
    const int b = dec_tensor_base(c, l);
    DecLayer& d = m->dec[l];
    for (int i = 0; i < 3; ++i) Q(d.qkv, i * D, b + 2 * i, D, D);
    Q(d.o, 0, b + 6, D, D);
    Q(d.cq, 0, b + 8, D, D);
    Q(d.ckv, 0, b + 10, D, D);
    Q(d.ckv, D, b + 12, D, D);
    Q(d.co, 0, b + 14, D, D);
    Q(d.w1, 0, b + 16, F, D);
    Q(d.w2, 0, b + 18, D, F);
  }
  if (rc) { qtx_model_destroy(m); return rc; }
  for (auto& e : m->enc)
    for (QLin* L : {&e.qkv, &e.o, &e.w1, &e.w2})
      if ((L->qkp && launch_pack_w_kp(L->w8(), L->N, L->K, L->qkp, st) != hipSuccess) ||
          (L->qws && launch_pack_w_ws(L->w8(), L->N, L->K, L->qws, st) != hipSuccess) ||
          (L->qws32 && pack_w_ws32(L->w8(), L->N, L->K, L->qws32, st) != hipSuccess)) {
        qtx_model_destroy(m);
        return fail(QTX_E_HIP, "KP / WS weight pack");
      }
  for (auto& e : m->enc)
    if (e.ffn && launch_pack_ffn(e.w1.w8(), e.w2.w8(), F, e.ffn, st) != hipSuccess) {
      qtx_model_destroy(m);
      return fail(QTX_E_HIP, "fused FFN weight pack");
    }
  // norms: order of weights.py:norm_names — enc L x 2, enc final, dec L x 3, dec final
  const int nb = norm_tensor_base(c);
  const int n_norms = 5 * NL + 2;
  for (int i = 0; i < n_norms; ++i)
    for (int j = 0; j < 2; ++j) {
      he = hipMemcpyAsync(norms + (size_t)(2 * i + j) * D, t[nb + 2 * i + j], D * sizeof(float),
                          hipMemcpyDeviceToDevice, st);
      if (he != hipSuccess) { qtx_model_destroy(m); return fail(QTX_E_HIP, "copy norms"); }
    }
  auto nrm = [&](int i, int j) -> const float* { return norms + (size_t)(2 * i + j) * D; };
  int ni = 0;
  for (int l = 0; l < NL; ++l)
    for (int s = 0; s < 2; ++s, ++ni) { m->enc[l].ln[s][0] = nrm(ni, 0); m->enc[l].ln[s][1] = nrm(ni, 1); }
  m->enc_norm[0] = nrm(ni, 0); m->enc_norm[1] = nrm(ni, 1); ++ni;
  for (int l = 0; l < NL; ++l)
    for (int s = 0; s < 3; ++s, ++ni) { m->dec[l].ln[s][0] = nrm(ni, 0); m->dec[l].ln[s][1] = nrm(ni, 1); }
  m->dec_norm[0] = nrm(ni, 0); m->dec_norm[1] = nrm(ni, 1); ++ni;
  const int eb = nb + 2 * n_norms;
  struct Cp { float* dst; const float* src; size_t n; } cps[] = {
      {src_lut, t[eb], (size_t)c.src_vocab * D}, {tgt_lut, t[eb + 1], (size_t)c.tgt_vocab * D},
      {gw, t[eb + 2], (size_t)c.tgt_vocab * D}, {gb, t[eb + 3], (size_t)c.tgt_vocab},
      {pe_d, pe, (size_t)c.max_len * D}};
  for (auto& cp : cps) {
    he = hipMemcpyAsync(cp.dst, cp.src, cp.n * sizeof(float), hipMemcpyDeviceToDevice, st);
    if (he != hipSuccess) { qtx_model_destroy(m); return fail(QTX_E_HIP, "copy tables"); }
  }
  m->src_lut = src_lut; m->tgt_lut = tgt_lut; m->pe = pe_d; m->gen_w = gw; m->gen_b = gb;
  he = launch_pack_gen(gw, c.tgt_vocab, m->gen_wt, st);
  if (he != hipSuccess) { qtx_model_destroy(m); return fail(QTX_E_HIP, "pack generator"); }
  he = hipStreamSynchronize(st);
  if (he != hipSuccess) {
    qtx_model_destroy(m);
    return fail(QTX_E_HIP, "model create: %s", hipGetErrorString(he));
  }
  *out = m;
  return QTX_OK;
}

int32_t qtx_model_destroy(qtx_model* m) {
  if (!m) return QTX_OK;
  {
    std::lock_guard<std::mutex> lk(g_live_mu);   // no thread exit returns a slot to it now
    g_live.erase(m->serial);
  }
  for (hipStream_t s : m->gstream)
    if (s) (void)hipStreamSynchronize(s);
  m->clear_graphs();
  if (m->ev_in) (void)hipEventDestroy(m->ev_in);
  for (hipEvent_t e : {m->ev_fork, m->ev_lag, m->ev_join})
    if (e) (void)hipEventDestroy(e);
  if (m->estream) (void)hipStreamDestroy(m->estream);
  for (int i = 0; i < QTX_MAX_GROUPS; ++i) {
    if (m->ev_out[i]) (void)hipEventDestroy(m->ev_out[i]);
    if (m->gstream[i]) (void)hipStreamDestroy(m->gstream[i]);
  }
  if (m->mem) (void)hipFree(m->mem);
  delete m;
  return QTX_OK;
}

size_t qtx_model_device_bytes(const qtx_model* m) { return m ? m->bytes : 0; }

int32_t qtx_model_linear(const qtx_model* m, int32_t module, int32_t layer, int32_t index,
                         const void** q, const float** s, const float** b, int32_t* N,
                         int32_t* K) {
  if (!m || !q || !s || !b || !N || !K) return fail(QTX_E_INVALID, "qtx_model_linear: null argument");
  if (layer < 0 || layer >= m->cfg.n_layers) return fail(QTX_E_INVALID, "layer %d out of range", layer);
  // a slice of `rows` output channels starting at `r0` of a stored (possibly concatenated) linear
  auto view = [&](const QLin& l, int r0, int rows) {
    const long rb = m->cfg.weight_bits == 4 ? l.K / 2 : l.K;   // bytes per weight row
    *q = l.q + (long)r0 * rb;
    *s = l.s + r0;
    *b = l.b + r0;
    *N = rows;
    *K = l.K;
    return (int32_t)QTX_OK;
  };
  const int D = m->cfg.d_model;
  if (module == 0) {
    const EncLayer& e = m->enc[layer];
    switch (index) {
      case 0: case 1: case 2: return view(e.qkv, index * D, D);
      case 3: return view(e.o, 0, e.o.N);
      case 4: return view(e.w1, 0, e.w1.N);
      case 5: return view(e.w2, 0, e.w2.N);
    }
  } else if (module == 1) {
    const DecLayer& d = m->dec[layer];
    switch (index) {
      case 0: case 1: case 2: return view(d.qkv, index * D, D);
      case 3: return view(d.o, 0, d.o.N);
      case 4: return view(d.cq, 0, d.cq.N);
      case 5: case 6: return view(d.ckv, (index - 5) * D, D);
      case 7: return view(d.co, 0, d.co.N);
      case 8: return view(d.w1, 0, d.w1.N);
      case 9: return view(d.w2, 0, d.w2.N);
    }
  }
  return fail(QTX_E_INVALID, "qtx_model_linear: no linear %d of module %d", index, module);
}

int32_t qtx_model_norm(const qtx_model* m, int32_t module, int32_t layer, int32_t sub,
                       const float** a, const float** b) {
  if (!m || !a || !b) return fail(QTX_E_INVALID, "qtx_model_norm: null argument");
  if (layer == -1 && (module == 0 || module == 1)) {
    const float* const* n = module == 0 ? m->enc_norm : m->dec_norm;
    *a = n[0];
    *b = n[1];
    return QTX_OK;
  }
  if (layer < 0 || layer >= m->cfg.n_layers) return fail(QTX_E_INVALID, "layer %d out of range", layer);
  if (module == 0 && sub >= 0 && sub < 2) {
    *a = m->enc[layer].ln[sub][0];
    *b = m->enc[layer].ln[sub][1];
    return QTX_OK;
  }
  if (module == 1 && sub >= 0 && sub < 3) {
    *a = m->dec[layer].ln[sub][0];
    *b = m->dec[layer].ln[sub][1];
    return QTX_OK;
  }
  return fail(QTX_E_INVALID, "qtx_model_norm: no norm %d of module %d layer %d", sub, module, layer);
}

}  // extern "C"

// =======================================================================================
// drivers
// =======================================================================================
namespace {

// scratch for one stack pass over M rows (fp32 residual stream + quant buffers)
struct Scratch {
  float* x;      // [M, D] residual stream
  int8_t* a8;    // [M, F] activation ints (max K)
  float* sa;     // [M]
  float* y;      // [M, max(3D, F)] GEMM output
  int8_t* q8;    // [M, D]   q8, k8, v8 contiguous ([3][M][D]) with sq, sk, sv ([3][M]):
  float* sq;     // [M]      the row GEMM writes the three quantized projections in one
  int8_t* k8;    // [M, D]   launch (tile stride M*D / M)
  float* sk;
  int8_t* v8;    // [M, D]
  float* sv;
  float* ctx;    // [M, D]
  int8_t* h8;    // [M, F]  quantized FFN hidden
  float* sh;     // [M]
  float* pmax;   // [F/512, M] FFN1 per-tile row maxima
  unsigned* status = nullptr;   // the call's status word (call_status_begin)
};

Scratch carve_scratch(Arena& ar, const qtx_config& c, long M) {
  const int D = c.d_model, F = c.d_ff;
  const int Y = 3 * D > F ? 3 * D : F;
  Scratch s;
  s.x = ar.take<float>(M * D);
  s.a8 = ar.take<int8_t>((M + 1) * F);    // + 1 row: KP row pairs of an odd M
  s.sa = ar.take<float>(M);
  s.y = ar.take<float>(M * Y);
  s.q8 = ar.take<int8_t>(3 * M * D); s.k8 = s.q8 + M * D; s.v8 = s.k8 + M * D;
  s.sq = ar.take<float>(3 * M); s.sk = s.sq + M; s.sv = s.sk + M;
  s.ctx = ar.take<float>(M * D);
  s.h8 = ar.take<int8_t>((M + 1) * F);
  s.sh = ar.take<float>(M);
  s.pmax = ar.take<float>((F / 512 + 1) * M);
  return s;
}

// ---- building blocks ------------------------------------------------------------------
RowArgs rows_quant(const float* x, long ldx, int rows, int D, int8_t* q, float* s) {
  RowArgs a{};
  a.x = x; a.ldx = ldx; a.rows = rows; a.D = D;
  a.q = q; a.ldq = D; a.s = s; a.qmax = 127.0f;
  a.rpb = rows > 0 ? rows : 1; a.dst_bstride = 0; a.dst_off = 0;
  return a;
}

int ln_quant(const float* x, int rows, const float* const* ln, int D, int8_t* q, float* s,
             hipStream_t st, bool kp = false) {
  RowArgs a = rows_quant(x, D, rows, D, q, s);
  a.ln_a = ln[0]; a.ln_b = ln[1]; a.kp = kp;
  HIPCHK(launch_rows(a, st));
  return QTX_OK;
}

int ln_out(const float* x, int rows, const float* const* ln, int D, float* y, hipStream_t st) {
  RowArgs a{};
  a.x = x; a.ldx = D; a.rows = rows; a.D = D; a.ln_a = ln[0]; a.ln_b = ln[1];
  a.yout = y; a.ldy = D; a.rpb = rows > 0 ? rows : 1;
  HIPCHK(launch_rows(a, st));
  return QTX_OK;
}

int quant(const float* x, long ldx, int rows, int D, int8_t* q, float* s, hipStream_t st,
          bool kp = false) {
  RowArgs a = rows_quant(x, ldx, rows, D, q, s);
  a.kp = kp;
  HIPCHK(launch_rows(a, st));
  return QTX_OK;
}

int linear(const qtx_config& c, const QLin& L, const int8_t* a8, const float* sa, int M,
           int flags, const float* res, float* out, long ldo, hipStream_t st) {
  GemmArgs g{};
  g.A = a8; g.lda = L.K; g.sa = sa;
  const int wb = L.q8 ? 8 : c.weight_bits;
  g.W = L.w8(); g.ldw = wb == 8 ? L.K : L.K / 2; g.sw = L.s; g.bias = L.b;
  g.out = out; g.ldo = ldo; g.res = res; g.ldr = ldo;
  g.M = M; g.N = L.N; g.K = L.K; g.flags = flags;
  HIPCHK(launch_gemm(g, wb, st));
  return QTX_OK;
}

// Row-complete GEMM (k_gemm_row) for 8-bit weights: epilogues of whole 512-wide rows.
bool row_path(const qtx_config& c) {   // (4-bit models: on the unpacked int8 weights)
  return c.d_ff % 512 == 0 && !knobs().no_rowgemm;
}
// kp: A (a8) in the KP layout and W from L.qkp; the int8 lnq / FFN-hidden outputs are
// then written KP as well (RE_QUANT's q8 stays row-major: attention reads it).
// With kp, a K = 512 GEMM over many rows runs weight-stationary (kp = 2, W from L.qws):
// each workgroup keeps a 512-column slice of W on chip (qtx_wsgemm.hip); below ws_min_m
// rows the per-workgroup W load is not amortized and the row GEMM is faster.
// Measured (tools/enc_small.py, the greedy decode's encoder): at M = 2304 (B = 32, S = 72)
// the Q/K/V and FFN1 launches on the weight-stationary kernel took the encoder 0.83 ->
// 0.73 ms (the row GEMM's 128-row tiles give 18 workgroups).  The O-projection's residual +
// LayerNorm epilogue runs weight-stationary only between ws_res_min_m and ws_res_max_m
// (above it the KP row GEMM is faster).  QTX_WS_MIN_M / QTX_WS_RES_MIN_M / _MAX_M: A/B.
long ws_min_m() { return knobs().ws_min_m; }
bool ws_res_ok(long M) { return M >= knobs().ws_res_min_m && M < knobs().ws_res_max_m; }
RowGemmArgs rowgemm(const QLin& L, const int8_t* a8, const float* sa, int M, int epi,
                    bool kp = false) {
  RowGemmArgs g{};
  const bool ws = kp && L.qws && L.K == 512 &&
                  (epi == RE_RES_LN ? ws_res_ok(M) : M >= ws_min_m());
  // Q/K/V on the 32x32x32 MFMA kernel (diagnostic build, QTX_WS32)
  const bool ws32 = ws && epi == RE_QUANT && L.qws32 && knobs().ws32;
  g.A = a8; g.lda = L.K; g.sa = sa; g.W = ws32 ? L.qws32 : ws ? L.qws : kp ? L.qkp : L.w8();
  g.ldw = L.K;
  g.sw = L.s; g.bias = L.b;
  g.M = M; g.N = L.N; g.K = L.K; g.epi = epi; g.kp = ws32 ? 4 : ws ? 2 : kp;
  return g;
}
hipError_t launch_row_gemm_any(const RowGemmArgs& g, hipStream_t st) {
  return g.kp == 2 || g.kp == 4 ? launch_gemm_ws(g, st) : launch_gemm_row(g, st);
}
// out = per-token quantized (a8 . W^T) per 512-wide tile into out8 + t*M*512, os + t*M
int row_quant(const QLin& L, const int8_t* a8, const float* sa, int M, int8_t* out8,
              float* os, hipStream_t st, const FaultArgs& fa = FaultArgs{}, bool kp = false,
              void* zero = nullptr, long zero16 = 0) {
  RowGemmArgs g = rowgemm(L, a8, sa, M, RE_QUANT, kp);
  g.fault = fa;
  g.zero = zero; g.zero16 = zero16;   // a side job (launch_gemm_ws), else a zeroing kernel
  g.out8 = out8; g.ldo8 = 512; g.o8_ts = (long)M * 512; g.os = os; g.os_ts = M;
  HIPCHK(launch_row_gemm_any(g, st));
  return QTX_OK;
}
// x += a8 . W^T, then LayerNorm(x) (ln) quantized into (lnq, lns) or fp32 into lnout
// part: scratch for split-K partials (>= 4 * M * 2 KB; the FFN2 call sites pass the fp32
// GEMM scratch, free by then).  A KP row GEMM over at most 64 row tiles (FFN2 at the decode
// encoder's M = 2304: 18 workgroups, 43.9 us) runs K split 4 ways + a row-wise epilogue.
int row_res_ln(const QLin& L, const int8_t* a8, const float* sa, int M, float* x,
               const float* const* ln, int8_t* lnq, float* lns, float* lnout, hipStream_t st,
               const FaultArgs& fa = FaultArgs{}, bool kp = false, float* part = nullptr) {
  RowGemmArgs g = rowgemm(L, a8, sa, M, RE_RES_LN, kp);
  g.fault = fa;
  g.res = x; g.xout = x; g.ln_a = ln[0]; g.ln_b = ln[1];
  g.lnq = lnq; g.lns = lns; g.lnout = lnout;
  if (part && g.kp == 1 && fa.kind == FK_NONE && (M + 127) / 128 <= 64 && L.K % 2048 == 0 &&
      !knobs().no_splitk) {
    g.part = reinterpret_cast<int32_t*>(part);
    g.ksplit = 4;
  }
  HIPCHK(launch_row_gemm_any(g, st));
  return QTX_OK;
}
// FFN1: relu(a8 . W1^T) quantized per token over all d_ff columns, two passes (row
// maxima, then recompute + quantize: cheaper than the fp32 hidden's round trip)
// FFN1 in one weight-stationary pass with the row maxima exchanged between the column
// slices' workgroups inside the launch (k_gemm_wsx); QTX_NO_WSX=1: the two passes
bool wsx_on() { return !knobs().no_wsx; }
// Whether row_ffn1 takes the one-pass FFN1 (k_gemm_wsx / wsy) with its exchange scratch in
// s.y: then the layer's Q/K/V launch can zero that scratch as a side job (encoder_run).
bool ffn1_onepass(const QLin& L, int M, bool kp, const FaultArgs& fa) {
  return rowgemm(L, nullptr, nullptr, M, RE_RELU_PMAX, kp).kp == 2 && L.N == 2048 &&
         fa.kind == FK_NONE && wsx_on();
}
long ffn1_scratch16(int M) { return (4L * 32 * ((M + 31) / 32) + 2) / 2; }   // 16-B chunks
int row_ffn1(const qtx_config& c, const QLin& L, const int8_t* a8, const float* sa, int M,
             Scratch& s, hipStream_t st,
             const FaultArgs& fa = FaultArgs{}, bool kp = false, unsigned* status = nullptr,
             bool prezeroed = false) {
  RowGemmArgs g = rowgemm(L, a8, sa, M, RE_RELU_PMAX, kp);
  if (g.kp == 2 && L.N == 2048 && fa.kind == FK_NONE && wsx_on()) {
    g.epi = RE_RELU_QUANT_PMAX;
    g.prezeroed = prezeroed;
    if (L.qws32 && knobs().ws32) { g.W = L.qws32; g.kp = 5; }   // k_gemm_wsy32
    g.pmax_out = s.y;                // granules + ticket: <= 32 * M + 2048 bytes of the (unused) fp32 GEMM scratch
    g.out8 = s.h8; g.ldo8 = c.d_ff; g.os = s.sh;
    g.status = status;               // the model's status word: a timeout becomes an error
    HIPCHK(launch_gemm_wsx(g, st));
    return QTX_OK;
  }
  g.fault = fa;
  g.pmax_out = s.pmax;
  HIPCHK(launch_row_gemm_any(g, st));
  g.epi = RE_RELU_QUANT_PMAX;
  g.pmax_in = s.pmax; g.pmax_n = c.d_ff / 512;
  g.out8 = s.h8; g.ldo8 = c.d_ff; g.os = s.sh;
  HIPCHK(launch_row_gemm_any(g, st));
  return QTX_OK;
}

AttnArgs attn_args(const Scratch& s, int B, int Sq, int Sk, long kbs_rows) {
  AttnArgs a{};
  const int D = 512;
  a.q = s.q8; a.q_bs = (long)Sq * D; a.q_ld = D; a.sq = s.sq; a.sq_bs = Sq;
  a.k = s.k8; a.k_bs = kbs_rows * D; a.k_ld = D; a.sk = s.sk; a.sk_bs = kbs_rows;
  a.v = s.v8; a.v_bs = kbs_rows * D; a.v_ld = D; a.sv = s.sv; a.sv_bs = kbs_rows;
  a.ctx = s.ctx; a.c_bs = (long)Sq * D; a.c_ld = D;
  a.B = B; a.H = 8; a.Sq = Sq; a.Sk = Sk;
  return a;
}

#define RC(expr)                       \
  do {                                 \
    int rc_ = (expr);                  \
    if (rc_ != QTX_OK) return rc_;     \
  } while (0)

// Self-attention sublayer: x += O(attn(LN(x)))   (sublayer_connection.py:15-17,
// attention.py:39-67).  Q/K/V come out of ONE N=3D GEMM and are quantized per token.
int self_attn_block(const qtx_config& c, const QLin& qkv, const QLin& o,
                    const float* const* ln, Scratch& s, int B, int S, const uint8_t* mask,
                    long m_bs, long m_is, bool dec, hipStream_t st) {
  const int D = c.d_model, M = B * S;
  RC(ln_quant(s.x, M, ln, D, s.a8, s.sa, st));
  RC(linear(c, qkv, s.a8, s.sa, M, 0, nullptr, s.y, 3 * D, st));
  RC(quant(s.y, 3 * D, M, D, s.q8, s.sq, st));
  RC(quant(s.y + D, 3 * D, M, D, s.k8, s.sk, st));
  RC(quant(s.y + 2 * D, 3 * D, M, D, s.v8, s.sv, st));
  AttnArgs a = attn_args(s, B, S, S, S);
  a.mask = mask; a.m_bs = m_bs; a.m_is = m_is;
  a.dec = dec;
  HIPCHK(launch_attention(a, st));
  RC(quant(s.ctx, D, M, D, s.a8, s.sa, st));
  RC(linear(c, o, s.a8, s.sa, M, EPI_RESIDUAL, s.x, s.x, D, st));
  return QTX_OK;
}

// FFN sublayer: x += w_2(relu(w_1(LN(x))))   (position_feed_forward.py:11-12)
int ffn_block(const qtx_config& c, const QLin& w1, const QLin& w2, const float* const* ln,
              Scratch& s, int M, hipStream_t st) {
  const int D = c.d_model, F = c.d_ff;
  RC(ln_quant(s.x, M, ln, D, s.a8, s.sa, st));
  RC(linear(c, w1, s.a8, s.sa, M, EPI_RELU, nullptr, s.y, F, st));
  RC(quant(s.y, F, M, F, s.a8, s.sa, st));
  RC(linear(c, w2, s.a8, s.sa, M, EPI_RESIDUAL, s.x, s.x, D, st));
  return QTX_OK;
}


// ---- fault injection (qtx_fault, include/qtx.h) -------------------------------------
// The GEMM that computes a given reference MatMul, and that linear's column offset in it.
enum GemmId { G_QKV, G_O, G_FFN1, G_FFN2, G_CQ, G_CKV, G_CO };
FaultArgs fault_for(const qtx_fault* f, int module, int layer, GemmId gid, int M,
                    const qtx_config& c) {
  FaultArgs fa{};
  if (!f || f->kind == QTX_FAULT_NONE || f->module != module || f->layer != layer) return fa;
  const int lin = f->linear;
  long off = 0, nlin = c.d_model;
  switch (gid) {
    case G_QKV: if (lin < QTX_LIN_Q || lin > QTX_LIN_V) return fa; off = (long)lin * c.d_model; break;
    case G_CKV: if (lin != QTX_LIN_CK && lin != QTX_LIN_CV) return fa;
                off = (long)(lin - QTX_LIN_CK) * c.d_model; break;
    case G_O: if (lin != QTX_LIN_O) return fa; break;
    case G_FFN1: if (lin != QTX_LIN_FFN1) return fa; nlin = c.d_ff; break;
    case G_FFN2: if (lin != QTX_LIN_FFN2) return fa; break;
    case G_CQ: if (lin != QTX_LIN_CQ) return fa; break;
    case G_CO: if (lin != QTX_LIN_CO) return fa; break;
  }
  fa.bit = f->bit;
  switch (f->kind) {
    case QTX_FAULT_INPUT: case QTX_FAULT_INPUT16:
      fa.kind = FK_INPUT; fa.row = f->row; fa.col = f->col;
      fa.lo = off + (f->kind == QTX_FAULT_INPUT16 ? f->win_start : 0);
      fa.hi = f->kind == QTX_FAULT_INPUT16 ? fa.lo + f->win_len : off + nlin;
      break;
    case QTX_FAULT_WEIGHT: case QTX_FAULT_WEIGHT16:
      fa.kind = FK_WEIGHT; fa.row = off + f->row; fa.col = f->col;
      fa.lo = f->kind == QTX_FAULT_WEIGHT16 ? f->win_start : 0;
      fa.hi = f->kind == QTX_FAULT_WEIGHT16 ? fa.lo + f->win_len : M;
      break;
    case QTX_FAULT_OUTPUT:
      fa.kind = FK_OUTPUT; fa.row = f->row; fa.col = off + f->col; fa.value = f->value;
      break;
  }
  return fa;
}

// The fault as an AttnFault if it targets this layer's self (cross = false) or cross
// attention MatMuls (see qtx.h for the index conventions).
bool attn_fault_for(const qtx_fault* f, int module, int layer, bool cross, int Sq, int Sk,
                    AttnFault& af) {
  if (!f || f->kind == QTX_FAULT_NONE || f->module != module || f->layer != layer) return false;
  const int lin = f->linear;
  bool qk;
  if (!cross && (lin == QTX_LIN_QK || lin == QTX_LIN_PV)) qk = lin == QTX_LIN_QK;
  else if (cross && (lin == QTX_LIN_CQK || lin == QTX_LIN_CPV)) qk = lin == QTX_LIN_CQK;
  else return false;
  const bool in = f->kind == QTX_FAULT_INPUT || f->kind == QTX_FAULT_INPUT16;
  const bool win = f->kind == QTX_FAULT_INPUT16 || f->kind == QTX_FAULT_WEIGHT16;
  af = AttnFault{};
  af.bit = f->bit;
  af.value = f->value;
  const long row = f->row, col = f->col;
  if (f->kind == QTX_FAULT_OUTPUT) {
    af.kind = qk ? AF_QK_OUTPUT : AF_PV_OUTPUT;
    af.b = row / Sq; af.i = row % Sq;
    if (qk) { af.h = col / Sk; af.j = col % Sk; } else { af.h = col / 64; af.d = col % 64; }
    af.row0 = af.i; af.nrows = 1;
    return true;
  }
  if (in) {
    af.kind = qk ? AF_QK_INPUT : AF_PV_INPUT;
    af.b = row / Sq; af.i = row % Sq;
    if (qk) { af.h = col / 64; af.d = col % 64; } else { af.h = col / Sk; af.j = col % Sk; }
    af.lo = win ? (int)f->win_start : 0;
    af.hi = win ? (int)(f->win_start + f->win_len) : (qk ? Sk : 64);
    af.row0 = af.i; af.nrows = 1;
  } else {
    af.kind = qk ? AF_QK_WEIGHT : AF_PV_WEIGHT;
    af.b = row / Sk; af.j = row % Sk; af.h = col / 64; af.d = col % 64;
    af.lo = win ? (int)f->win_start : 0;
    af.hi = win ? (int)(f->win_start + f->win_len) : Sq;
    af.row0 = af.lo; af.nrows = af.hi - af.lo;
  }
  return true;
}

// attention with an optional fault: fp32 context (+ the faulty rows recomputed), then the
// per-token quantization of the O-projection input
int attention_fault(const AttnArgs& a, const AttnFault& af, int M, int D, Scratch& s,
                    hipStream_t st) {
  HIPCHK(launch_attention(a, st));
  HIPCHK(launch_attn_fault_rows(a, af, st));
  RC(quant(s.ctx, D, M, D, s.a8, s.sa, st));
  return QTX_OK;
}

// Validates a fault against the shapes of its target MatMul (M token rows of the module,
// Ms memory rows for the decoder's cross K/V); returns QTX_OK or an error code.
int check_fault(const qtx_model* m, const qtx_fault* f, int module, long B, long Sq, long Ss) {
  if (!f || f->kind == QTX_FAULT_NONE) return QTX_OK;
  const qtx_config& c = m->cfg;
  const long M = B * Sq, Ms = B * Ss;
  if (!row_path(c) || c.weight_bits != 8)
    return fail(QTX_E_UNSUPPORTED, "fault injection needs 8-bit weights");
  if (f->kind < 0 || f->kind > QTX_FAULT_OUTPUT) return fail(QTX_E_INVALID, "fault kind %d", f->kind);
  if (f->module != module) return fail(QTX_E_INVALID, "fault module %d", f->module);
  if (f->layer < 0 || f->layer >= c.n_layers) return fail(QTX_E_INVALID, "fault layer %d", f->layer);
  const int lin = f->linear;
  const bool in_kind = f->kind == QTX_FAULT_INPUT || f->kind == QTX_FAULT_INPUT16;
  const bool w_kind = f->kind == QTX_FAULT_WEIGHT || f->kind == QTX_FAULT_WEIGHT16;
  const bool win = f->kind == QTX_FAULT_INPUT16 || f->kind == QTX_FAULT_WEIGHT16;
  if ((in_kind || w_kind) && (f->bit < 0 || f->bit > 7)) return fail(QTX_E_INVALID, "fault bit %d", f->bit);
  auto bad_idx = [&](long r, long nr, long cc, long nc) {
    return fail(QTX_E_INVALID, "fault index (%ld, %ld) outside [%ld, %ld]", r, cc, nr, nc);
  };
  const long row = f->row, col = f->col;
  const bool attn_self = lin == QTX_LIN_QK || lin == QTX_LIN_PV;
  const bool attn_cross = lin == QTX_LIN_CQK || lin == QTX_LIN_CPV;
  if (attn_self || attn_cross) {
    if (attn_cross && module != 1) return fail(QTX_E_INVALID, "fault linear %d", lin);
    const long sq = Sq, sk = attn_cross ? Ss : Sq, H = c.n_heads;
    if (sk > 512) return fail(QTX_E_UNSUPPORTED, "attention fault with %ld keys", sk);
    const bool qk = lin == QTX_LIN_QK || lin == QTX_LIN_CQK;
    long nr, nc, wmax;
    if (f->kind == QTX_FAULT_OUTPUT) { nr = B * sq; nc = qk ? H * sk : H * 64; wmax = 0; }
    else if (in_kind) { nr = B * sq; nc = qk ? H * 64 : H * sk; wmax = qk ? sk : 64; }
    else { nr = B * sk; nc = H * 64; wmax = sq; }
    if (row < 0 || row >= nr || col < 0 || col >= nc) return bad_idx(row, nr, col, nc);
    if (win && (f->win_len < 1 || f->win_len > 16 || f->win_start < 0 || f->win_start + f->win_len > wmax))
      return fail(QTX_E_INVALID, "fault window [%ld, +%d) outside %ld", (long)f->win_start, f->win_len, wmax);
    return QTX_OK;
  }
  const bool enc_ok = lin == QTX_LIN_Q || lin == QTX_LIN_K || lin == QTX_LIN_V || lin == QTX_LIN_O ||
                      lin == QTX_LIN_FFN1 || lin == QTX_LIN_FFN2;
  const bool dec_ok = enc_ok || (lin >= QTX_LIN_CQ && lin <= QTX_LIN_CO);
  if (!(module == 0 ? enc_ok : dec_ok)) return fail(QTX_E_INVALID, "fault linear %d", lin);
  const long rows = (lin == QTX_LIN_CK || lin == QTX_LIN_CV) ? Ms : M;
  const long K = lin == QTX_LIN_FFN2 ? c.d_ff : c.d_model;
  const long N = lin == QTX_LIN_FFN1 ? c.d_ff : c.d_model;
  if (in_kind && (row < 0 || row >= rows || col < 0 || col >= K)) return bad_idx(row, rows, col, K);
  if (w_kind && (row < 0 || row >= N || col < 0 || col >= K)) return bad_idx(row, N, col, K);
  if (f->kind == QTX_FAULT_OUTPUT && (row < 0 || row >= rows || col < 0 || col >= N))
    return bad_idx(row, rows, col, N);
  if (f->kind == QTX_FAULT_INPUT16 &&
      (f->win_len < 1 || f->win_len > 16 || f->win_start < 0 || f->win_start + f->win_len > N))
    return fail(QTX_E_INVALID, "INPUT16 window");
  if (f->kind == QTX_FAULT_WEIGHT16 &&
      (f->win_len < 1 || f->win_len > 16 || f->win_start < 0 || f->win_start + f->win_len > rows))
    return fail(QTX_E_INVALID, "WEIGHT16 window");
  return QTX_OK;
}

// The fused FFN launch (qtx_ffn.hip) replaces the one-pass FFN1 + the FFN2 row GEMM on the
// KP path from ffn_fused_min_m rows (QTX_FFN_FUSED_MIN_M; QTX_NO_FFN_FUSED: never): one
// workgroup per 128 rows, so below ~1 block per CU the split launches use the chip better.
bool ffn_fused_ok(const EncLayer& L, long M, bool kp) {
  return kp && L.ffn && !knobs().no_ffn_fused && M >= knobs().ffn_fused_min_m;
}

int encoder_run(const qtx_model* m, const float* x, const uint8_t* mask, int B, int S,
                float* out, Scratch& s, hipStream_t st, const qtx_fault* f = nullptr,
                hipEvent_t after_first = nullptr) {
  const qtx_config& c = m->cfg;
  const int D = c.d_model, M = B * S;
  if (x != s.x) HIPCHK(hipMemcpyAsync(s.x, x, (size_t)M * D * 4, hipMemcpyDeviceToDevice, st));
  if (!row_path(c)) {
    for (const EncLayer& L : m->enc) {
      RC(self_attn_block(c, L.qkv, L.o, L.ln[0], s, B, S, mask, S, 0, false, st));
      RC(ffn_block(c, L.w1, L.w2, L.ln[1], s, M, st));
    }
    RC(ln_out(s.x, M, m->enc_norm, D, out, st));
    return QTX_OK;
  }
  // Every LayerNorm + per-token quantization after the first is fused into the epilogue of
  // the GEMM that produces the residual it normalizes (O-proj, FFN2); Q/K/V and the FFN
  // hidden are quantized in their GEMM's epilogue; the last FFN2 applies the final norm.
  // KP: the int8 activations between the kernels (LN output, attention context, FFN
  // hidden) live in the KP layout the row GEMM's 64-byte-step DMA reads as full lines
  // (qtx_common.h kp_off); the fault variants keep the row-major layout.
  const int NL = c.n_layers;
  const bool kp = (f == nullptr || f->kind == QTX_FAULT_NONE) && m->enc[0].qkv.qkp &&
                  !knobs().no_kp;
  RC(ln_quant(s.x, M, m->enc[0].ln[0], D, s.a8, s.sa, st, kp));
  for (int l = 0; l < NL; ++l) {
    const EncLayer& L = m->enc[l];
    auto fa = [&](GemmId gid) { return fault_for(f, 0, l, gid, M, c); };
    // the FFN1 below in one pass: its exchange scratch (in s.y, which nothing between here
    // and it writes) zeroed by the Q/K/V launch instead of a kernel of its own
    const bool zero_ffn1 = kp && !ffn_fused_ok(L, M, kp) && ffn1_onepass(L.w1, M, kp, fa(G_FFN1));
    RC(row_quant(L.qkv, s.a8, s.sa, M, s.q8, s.sq, st, fa(G_QKV), kp,
                 zero_ffn1 ? s.y : nullptr, zero_ffn1 ? ffn1_scratch16(M) : 0));
    if (l == 0 && after_first) HIPCHK(hipEventRecord(after_first, st));
    AttnArgs a = attn_args(s, B, S, S, S);
    a.mask = mask; a.m_bs = S; a.m_is = 0;
    a.c_ld = D;
    AttnFault af;
    const hipError_t ea = attn_fault_for(f, 0, l, false, S, S, af)
                              ? hipErrorNotSupported
                              : (knobs().no_attn_encq ? hipErrorNotSupported
                                                            : launch_attention_encq(a, s.a8, s.sa, st,
                                                                                    false, kp));
    if (attn_fault_for(f, 0, l, false, S, S, af)) {
      RC(attention_fault(a, af, M, D, s, st));
    } else if (ea == hipErrorNotSupported) {  // other shapes: fp32 context + quantization
      HIPCHK(launch_attention(a, st));
      RC(quant(s.ctx, D, M, D, s.a8, s.sa, st, kp));
    } else {
      HIPCHK(ea);
    }
    RC(row_res_ln(L.o, s.a8, s.sa, M, s.x, L.ln[1], s.a8, s.sa, nullptr, st, fa(G_O), kp));
    if (ffn_fused_ok(L, M, kp)) {
      // the FFN sublayer in one launch (k_ffn_fused): the hidden stays on chip; each
      // workgroup reads its rows of a8 / sa before it writes them (the next LN's codes)
      FfnArgs g{};
      g.A = s.a8; g.sa = s.sa; g.wf = L.ffn;
      g.sw1 = L.w1.s; g.b1 = L.w1.b; g.sw2 = L.w2.s; g.b2 = L.w2.b;
      g.x = s.x; g.M = M; g.F = c.d_ff;
      if (l + 1 < NL) {
        g.ln_a = m->enc[l + 1].ln[0][0]; g.ln_b = m->enc[l + 1].ln[0][1];
        g.lnq = s.a8; g.lns = s.sa;
      } else {
        g.ln_a = m->enc_norm[0]; g.ln_b = m->enc_norm[1]; g.lnout = out;
      }
      HIPCHK(launch_ffn_fused(g, st));
      continue;
    }
    RC(row_ffn1(c, L.w1, s.a8, s.sa, M, s, st, fa(G_FFN1), kp, s.status, zero_ffn1));
    if (l + 1 < NL)
      RC(row_res_ln(L.w2, s.h8, s.sh, M, s.x, m->enc[l + 1].ln[0], s.a8, s.sa, nullptr, st,
                    fa(G_FFN2), kp, s.y));
    else
      RC(row_res_ln(L.w2, s.h8, s.sh, M, s.x, m->enc_norm, nullptr, nullptr, out, st,
                    fa(G_FFN2), kp, s.y));
  }
  return QTX_OK;
}

// Encoder sub-batch pipelining: a batch of >= 256 sentences runs as two halves on two
// streams, the second half one kernel behind, so the HBM-bound epilogues (residual +
// LayerNorm) of one half overlap the MFMA / VALU-bound kernels (attention, FFN) of the
// other on different CUs.  Results are identical (rows are independent).
// (not with the one-pass FFN1, which makes the layer's kernels MFMA / exchange-bound rather
// than HBM-bound: the split measured no gain before it, 2.07 vs 2.05 ms)
bool wsx_on();
bool enc_split(int B) { return B >= 256 && !knobs().enc_nosplit && !wsx_on(); }

size_t enc_ws(const qtx_config& c, int B, int S) {
  Arena ar;
  carve_scratch(ar, c, (long)B * S);
  if (enc_split(B)) {
    Arena a2;
    carve_scratch(a2, c, (long)(B / 2) * S);
    carve_scratch(a2, c, (long)(B - B / 2) * S);
    ar.used = std::max(ar.used, a2.used);
  }
  return align_up(ar.used);
}

// decoder-specific scratch: quantized memory + cross K/V for all layers
struct CrossKV {
  int8_t* am8;  // [B*S, D] quantized memory (per token, layer independent)
  float* sam;
  std::vector<int8_t*> k8, v8;
  std::vector<float*> sk, sv;
  float* y;     // [B*S, 2D]
};

CrossKV carve_cross(Arena& ar, const qtx_config& c, long Ms) {
  const int D = c.d_model;
  CrossKV x;
  x.am8 = ar.take<int8_t>(Ms * D);
  x.sam = ar.take<float>(Ms);
  x.y = ar.take<float>(Ms * 2 * D);
  // k8 / v8 of every layer contiguous (tile t = 2 l + {0: K, 1: V} at t * Ms * D), and
  // sk / sv likewise (t * Ms): the layout of one row GEMM's per-512-column-tile outputs
  int8_t* kv = ar.take<int8_t>(2L * c.n_layers * Ms * D);
  float* sc = ar.take<float>(2L * c.n_layers * Ms);
  for (int l = 0; l < c.n_layers; ++l) {
    x.k8.push_back(kv ? kv + 2L * l * Ms * D : nullptr);
    x.v8.push_back(kv ? kv + (2L * l + 1) * Ms * D : nullptr);
    x.sk.push_back(sc ? sc + 2L * l * Ms : nullptr);
    x.sv.push_back(sc ? sc + (2L * l + 1) * Ms : nullptr);
  }
  return x;
}

// memory -> per-layer cross K/V (get_quantized_model.py:160-168: K/V outputs quantized)
int cross_kv(const qtx_model* m, const float* memory, int Ms, CrossKV& x, hipStream_t st,
             const qtx_fault* f = nullptr) {
  const qtx_config& c = m->cfg;
  const int D = c.d_model;
  RC(quant(memory, D, Ms, D, x.am8, x.sam, st));
  bool ckv_fault = false;
  for (int l = 0; l < c.n_layers; ++l) ckv_fault |= fault_for(f, 1, l, G_CKV, Ms, c).kind != FK_NONE;
  if (row_path(c) && D == 512 && !ckv_fault) {
    // every layer's K and V in ONE row GEMM (N = n_layers * 2 * 512): its 512-column tiles
    // are the layers' K / V, each quantized per token in the epilogue exactly as the
    // per-layer launches below (decode prologue: 6 launches of 36 workgroups -> one of 216)
    RC(row_quant(m->ckv_all, x.am8, x.sam, Ms, x.k8[0], x.sk[0], st));
    return QTX_OK;
  }
  for (int l = 0; l < c.n_layers; ++l) {
    if (row_path(c)) {     // K and V tiles quantized in the GEMM epilogue
      RC(row_quant(m->dec[l].ckv, x.am8, x.sam, Ms, x.k8[l], x.sk[l], st,
                   fault_for(f, 1, l, G_CKV, Ms, c)));
      continue;
    }
    RC(linear(c, m->dec[l].ckv, x.am8, x.sam, Ms, 0, nullptr, x.y, 2 * D, st));
    RC(quant(x.y, 2 * D, Ms, D, x.k8[l], x.sk[l], st));
    RC(quant(x.y + D, 2 * D, Ms, D, x.v8[l], x.sv[l], st));
  }
  return QTX_OK;
}

// Cross-attention sublayer: x += O(attn(LN(x) -> Q, memory -> K/V)), decoder.py:32
int cross_attn_block(const qtx_model* m, const DecLayer& L, int l, Scratch& s,
                     const CrossKV& x, int B, int T, int S, const uint8_t* src_mask,
                     hipStream_t st) {
  const qtx_config& c = m->cfg;
  const int D = c.d_model, M = B * T;
  RC(ln_quant(s.x, M, L.ln[1], D, s.a8, s.sa, st));
  RC(linear(c, L.cq, s.a8, s.sa, M, 0, nullptr, s.y, D, st));
  RC(quant(s.y, D, M, D, s.q8, s.sq, st));
  AttnArgs a = attn_args(s, B, T, S, S);
  a.k = x.k8[l]; a.sk = x.sk[l]; a.v = x.v8[l]; a.sv = x.sv[l];
  a.mask = src_mask; a.m_bs = S; a.m_is = 0;
  a.dec = 1;
  HIPCHK(launch_attention(a, st));
  RC(quant(s.ctx, D, M, D, s.a8, s.sa, st));
  RC(linear(c, L.co, s.a8, s.sa, M, EPI_RESIDUAL, s.x, s.x, D, st));
  return QTX_OK;
}

size_t dec_ws(const qtx_config& c, int B, int T, int S) {
  Arena ar;
  carve_scratch(ar, c, (long)B * T);
  carve_cross(ar, c, (long)B * S);
  return align_up(ar.used);
}

// greedy decode workspace: encoder scratch, decoder step scratch (M=B), cross K/V,
// self K/V caches [L][B][max_len][D], memory, logits, step counter
struct GreedyWS {
  Scratch enc, dec;
  CrossKV cross;
  std::vector<int8_t*> cvg;   // the cross values in k_dec_attn's 4-key groups, per layer
  std::vector<int8_t*> kc, vc;   // self K [B][max_len][D]; V in 4-key groups (fused step) or
                                 // [B][max_len][D] (unfused step)
  std::vector<float*> skc, svc;
  float* memory;
  float* xo;
  float* logits;
  int* step;          // [0] = decode position, [1] = argmax arrival counter
  float* pmax_a;      // [8][B]    per-head absmax of the attention context (A_F32Q input)
  float* pmax_f;      // [F/16][B] per-column-tile absmax of FFN1's output
  // fused-decode sub-batches: step scratch (grp[0] = dec) and step counters, 4 ints each
  std::vector<Scratch> grp;
  int* gsteps;
  int64_t* ids;       // [B][max_len] the decode writes here; copied out to the caller's ids
  uint8_t* mask;      // [B][S] staged copy of the caller's src_mask
};

// Sub-batch split of the fused decode.  Sentences are independent (per-token quantization:
// no value depends on another sentence), and one sub-batch's step is a chain of ~50
// latency-bound kernels that each occupy a fraction of the 256 CUs.  G sub-batch graphs
// on G streams (ms per decode, profiles/r03_concurrency.md): B = 32: 14.5 / 21.0 for
// G = 1 / 2; B = 256: 34.9 / 35.8; B = 512: 59.0 / 51.9 — two chains of 256 rows overlap
// as well as two processes of 256 sentences each (50.6), two of 128 or 16 do not gain.
// Default G = 2 from B = 512, else 1; QTX_DECODE_GROUPS overrides it (experiments).
struct Groups {
  int G, Bg;   // G groups of Bg rows (the last one may be shorter)
  int b0(int i) const { return i * Bg; }
  int rows(int i, int B) const { return std::min(B, (i + 1) * Bg) - i * Bg; }
};
Groups decode_groups(int B) {
  int G = B >= 512 ? 2 : 1;
  if (knobs().decode_groups > 0) G = knobs().decode_groups;
  G = std::max(1, std::min(std::min(G, QTX_MAX_GROUPS), B));
  const int Bg = (B + G - 1) / G;
  return Groups{(B + Bg - 1) / Bg, Bg};   // no empty group
}

GreedyWS carve_greedy(Arena& ar, const qtx_config& c, int B, int S, int max_len) {
  GreedyWS g;
  const int D = c.d_model;
  g.enc = carve_scratch(ar, c, (long)B * S);
  g.dec = carve_scratch(ar, c, B);
  g.cross = carve_cross(ar, c, (long)B * S);
  // the cross values regrouped once per decode (layer stride: B * ceil(S/4) * 4 * D bytes)
  int8_t* cvg = ar.take<int8_t>((size_t)c.n_layers * B * ((S + 3) & ~3) * D);
  for (int l = 0; l < c.n_layers; ++l) {
    g.cvg.push_back(cvg ? cvg + (size_t)l * B * ((S + 3) & ~3) * D : nullptr);
    g.kc.push_back(ar.take<int8_t>((size_t)B * max_len * D));
    g.skc.push_back(ar.take<float>((size_t)B * max_len));
    g.vc.push_back(ar.take<int8_t>((size_t)B * ((max_len + 3) & ~3) * D));
    g.svc.push_back(ar.take<float>((size_t)B * max_len));
  }
  g.memory = ar.take<float>((size_t)B * S * D);
  g.xo = ar.take<float>((size_t)B * D);
  g.logits = ar.take<float>((size_t)B * c.tgt_vocab);
  g.step = ar.take<int>(4);
  g.pmax_a = ar.take<float>((size_t)8 * B);
  g.pmax_f = ar.take<float>((size_t)(c.d_ff / 16) * B);
  const Groups gr = decode_groups(B);
  g.grp.push_back(g.dec);
  for (int i = 1; i < gr.G; ++i) g.grp.push_back(carve_scratch(ar, c, gr.Bg));
  g.gsteps = ar.take<int>(4 * QTX_MAX_GROUPS);
  g.ids = ar.take<int64_t>((size_t)B * max_len);
  g.mask = ar.take<uint8_t>((size_t)B * S);
  return g;
}

// The workspace of sub-batch i (rows b0 ..): every per-sentence buffer offset by b0.
GreedyWS group_view(const GreedyWS& g, const qtx_config& c, int i, int b0, int S,
                    int max_len) {
  const long D = c.d_model;
  GreedyWS v = g;
  v.dec = g.grp[i];
  for (int l = 0; l < c.n_layers; ++l) {
    v.kc[l] += b0 * max_len * D; v.vc[l] += b0 * ((max_len + 3) & ~3) * D;
    v.skc[l] += b0 * max_len; v.svc[l] += b0 * max_len;
    v.cross.k8[l] += b0 * S * D; v.cross.v8[l] += b0 * S * D;
    v.cvg[l] += b0 * ((S + 3) & ~3) * D;
    v.cross.sk[l] += b0 * S; v.cross.sv[l] += b0 * S;
  }
  v.logits += (long)b0 * c.tgt_vocab;
  v.pmax_a += (long)8 * b0;               // each sub-batch: its own [P][rows] block
  v.pmax_f += (long)(c.d_ff / 16) * b0;
  v.step = g.gsteps + 4 * i;
  return v;
}


// ---- fused decode step (M = B rows, keys <= 128) ----------------------------------------
SkinnyArgs skinny(int wbits, const QLin& L, int M, int amode, int flags, float* out, long ldo) {
  SkinnyArgs s{};
  // wbits 8 on a 4-bit model: its unpacked int8 copy
  s.amode = amode; s.W = wbits == 8 ? L.w8() : L.q; s.ldw = wbits == 8 ? L.K : L.K / 2;
  s.sw = L.s; s.bias = L.b;
  s.out = out; s.ldo = ldo; s.M = M; s.N = L.N; s.K = L.K; s.flags = flags;
  return s;
}

// One KV-cached decoder step for every sentence, 8 kernels per layer + 2:
//   [LN+QKV] [self-attn] [O+res] [LN+Qc] [cross-attn] [Oc+res] [LN+FFN1+relu] [FFN2+res]
//   [final LN + generator] [log_softmax/argmax + next embedding + step++]
// Reads the position from g.step (device), so it can be captured once and replayed.
// t_host: the step's position when the caller knows it at launch or capture time (the
// whole decode in one graph, or eager launches), else -1
int greedy_step_fused(const qtx_model* m, GreedyWS& g, int B, int S, int max_len,
                      int64_t* ids, const uint8_t* src_mask, hipStream_t st, int t_host) {
  const qtx_config& c = m->cfg;
  const int D = c.d_model, F = c.d_ff;
  const int wb = m->dec[0].qkv.q8 && !knobs().int4_packed ? 8 : c.weight_bits;
  // the FFN hidden quantized once by its own kernel (instead of in every FFN2 workgroup's
  // prologue from FFN1's partial maxima) from 96 rows on: measured faster there despite the
  // extra launch (profiles/r05_rb_sweep.md), slower at B = 32
  const bool ffn_qkernel = knobs().ffn_qkernel || B >= 96;
  const bool fused_ln = !knobs().split_ln;
  // O / Oc form the context's per-token maximum from the rows they load (A_F32R) instead of
  // the attention's per-head maxima (QTX_ATTN_PMAX=1: the per-head maxima, A_F32Q)
  const bool own_max = !knobs().attn_pmax;
  // likewise FFN2 forms the hidden's per-token maximum itself (QTX_FFN_PMAX=1: from FFN1's
  // per-tile maxima, FFN1 with the maxima epilogue)
  const bool ffn_own = !knobs().ffn_pmax;
  // the position from the host (self-attention, argmax + embedding; the device counter then
  // neither read nor advanced) or from the device counter (QTX_DEVICE_STEP, or a step replayed
  // at several positions)
  const bool host_pos = t_host >= 0 && !knobs().device_step;
  Scratch& s = g.dec;
  // Timing experiments only (wrong results): QTX_ABLATE=<bitmask> drops kernel classes
  // from the step (replaced by an empty kernel with QTX_ABLATE_NOP=1) to measure what
  // each costs inside the real graph.  1 LN, 2 QKV/Qc, 4 self-attn, 8 cross-attn,
  // 16 O/Oc, 32 FFN1, 64 h-quant, 128 FFN2, 256 tail.
  const int abl = knobs().ablate;           // always 0 outside the QTX_DIAG build
  const bool abl_nop = knobs().ablate_nop;
#define QTX_RUN(bit, launch)                   \
  do {                                         \
    if (abl & (bit)) {                         \
      if (abl_nop) HIPCHK(launch_nop(st));     \
    } else {                                   \
      HIPCHK(launch);                          \
    }                                          \
  } while (0)
  // out = epilogue(quant(LN(x)) . W^T): the LayerNorm + per-token quant is recomputed in
  // the prologue of every GEMM workgroup (4 rows each, A_LN) — cheaper than its own kernel
  // launch; QTX_SPLIT_LN=1 restores the separate LN kernel (timing experiments).
#define QTX_RUNRC(bit, expr)                   \
  do {                                         \
    if (abl & (bit)) {                         \
      if (abl_nop) HIPCHK(launch_nop(st));     \
    } else {                                   \
      RC(expr);                                \
    }                                          \
  } while (0)
  auto ln_linear = [&](const QLin& W, const float* const* ln, int flags, float* out,
                       long ldo, int bit) -> int {
    SkinnyArgs k = skinny(wb, W, B, fused_ln ? A_LN : A_I8, flags, out, ldo);
    if (flags & EPI_ROWMAX) k.pmax_out = g.pmax_f;
    if (fused_ln) {
      k.X = s.x; k.ldx = D; k.ln_a = ln[0]; k.ln_b = ln[1];
    } else {
      QTX_RUNRC(1, ln_quant(s.x, B, ln, D, s.a8, s.sa, st));
      k.A = s.a8; k.sa = s.sa;
    }
    QTX_RUN(bit, launch_skinny(k, wb, st));
    return QTX_OK;
  };
  for (int l = 0; l < c.n_layers; ++l) {
    const DecLayer& L = m->dec[l];
    SkinnyArgs a;
    RC(ln_linear(L.qkv, L.ln[0], 0, s.y, 3 * D, 2));
    DecAttnArgs at{};
    at.y = s.y; at.ldy = 3 * D; at.kv_new = 1; at.step = g.step;
    at.kc = g.kc[l]; at.vc = g.vc[l]; at.skc = g.skc[l]; at.svc = g.svc[l]; at.kv_bs = max_len;
    at.ctx = s.ctx; at.pmax = own_max ? nullptr : g.pmax_a; at.B = B;
    at.host_step1 = host_pos ? t_host + 1 : 0;
    QTX_RUN(4, launch_dec_attn(at, B, st));
    a = skinny(wb, L.o, B, own_max ? A_F32R : A_F32Q, EPI_RESIDUAL, s.x, D);   // quantizes ctx per token
    a.X = s.ctx; a.ldx = D; a.pmax_in = g.pmax_a; a.pmax_n = 8; a.res = s.x; a.ldr = D;
    QTX_RUN(16, launch_skinny(a, wb, st));
    RC(ln_linear(L.cq, L.ln[1], 0, s.y, D, 2));
    at = DecAttnArgs{};
    at.y = s.y; at.ldy = D; at.kv_new = 0; at.S = S; at.mask = src_mask;
    at.kc = g.cross.k8[l]; at.vc = g.cvg[l]; at.skc = g.cross.sk[l];
    at.svc = g.cross.sv[l]; at.kv_bs = S;
    at.ctx = s.ctx; at.pmax = own_max ? nullptr : g.pmax_a; at.B = B;
    QTX_RUN(8, launch_dec_attn(at, B, st));
    a = skinny(wb, L.co, B, own_max ? A_F32R : A_F32Q, EPI_RESIDUAL, s.x, D);
    a.X = s.ctx; a.ldx = D; a.pmax_in = g.pmax_a; a.pmax_n = 8; a.res = s.x; a.ldr = D;
    QTX_RUN(16, launch_skinny(a, wb, st));
    if (!ffn_qkernel) {   // FFN2 quantizes h itself (from its rows, or FFN1's per-tile maxima)
      RC(ln_linear(L.w1, L.ln[2], ffn_own ? EPI_RELU : EPI_RELU | EPI_ROWMAX, s.y, F, 32));
      a = skinny(wb, L.w2, B, ffn_own ? A_F32R : A_F32Q, EPI_RESIDUAL, s.x, D);
      a.X = s.y; a.ldx = F; a.pmax_in = g.pmax_f; a.pmax_n = F / 16; a.res = s.x; a.ldr = D;
      QTX_RUN(128, launch_skinny(a, wb, st));
    } else {              // one wave per row quantizes h (quant_linear.py:30-43), then FFN2
      RC(ln_linear(L.w1, L.ln[2], EPI_RELU, s.y, F, 32));
      if (F == 2048 && !knobs().hquant_rows)   // one 4-wave workgroup per row
        QTX_RUN(64, launch_quant_h2048(s.y, F, B, s.a8, s.sa, st));
      else
        QTX_RUNRC(64, quant(s.y, F, B, F, s.a8, s.sa, st));
      a = skinny(wb, L.w2, B, A_I8, EPI_RESIDUAL, s.x, D);
      a.A = s.a8; a.sa = s.sa; a.res = s.x; a.ldr = D;
      QTX_RUN(128, launch_skinny(a, wb, st));
    }
  }
  if (knobs().dbg_tail) {   // bisection aid (QTX_DIAG build): reference-shaped tail kernels
    RC(ln_out(s.x, B, m->dec_norm, D, g.xo, st));
    HIPCHK(launch_generator(g.xo, D, B, m->gen_w, m->gen_b, c.tgt_vocab, g.logits, st));
    HIPCHK(launch_logsoftmax_argmax(g.logits, B, c.tgt_vocab, nullptr, ids, max_len, g.step,
                                    1, st));
    HIPCHK(launch_step_inc(g.step, st));
    HIPCHK(launch_embed(ids, max_len, B, 1, g.step, 0, m->tgt_lut, c.tgt_vocab, m->pe,
                        c.max_len, s.x, D, st));
    return QTX_OK;
  }
  QTX_RUN(256, launch_generator_mfma(s.x, D, B, m->dec_norm[0], m->dec_norm[1], m->gen_wt,
                                     m->gen_b, c.tgt_vocab, g.logits, st));
  QTX_RUN(256, launch_argmax_embed(g.logits, B, c.tgt_vocab, ids, max_len, g.step,
                                   reinterpret_cast<unsigned*>(g.step + 1), m->tgt_lut, m->pe,
                                   c.max_len, s.x, st, host_pos ? t_host + 1 : 0));
  return QTX_OK;
#undef QTX_RUN
#undef QTX_RUNRC
}

// The reference-shaped unfused step (any key count up to 512).
int greedy_step_unfused(const qtx_model* m, GreedyWS& g, int B, int S, int max_len,
                        int64_t* ids, const uint8_t* src_mask, hipStream_t st) {
  const qtx_config& c = m->cfg;
  const int D = c.d_model;
  Scratch& s = g.dec;
  HIPCHK(launch_embed(ids, max_len, B, 1, g.step, 0, m->tgt_lut, c.tgt_vocab, m->pe,
                      c.max_len, s.x, D, st));
  for (int l = 0; l < c.n_layers; ++l) {
    const DecLayer& L = m->dec[l];
    RC(ln_quant(s.x, B, L.ln[0], D, s.a8, s.sa, st));
    RC(linear(c, L.qkv, s.a8, s.sa, B, 0, nullptr, s.y, 3 * D, st));
    RC(quant(s.y, 3 * D, B, D, s.q8, s.sq, st));
    RowArgs kr = rows_quant(s.y + D, 3 * D, B, D, g.kc[l], g.skc[l]);
    kr.rpb = 1; kr.dst_bstride = max_len; kr.dst_off_dev = g.step;
    HIPCHK(launch_rows(kr, st));
    RowArgs vr = rows_quant(s.y + 2 * D, 3 * D, B, D, g.vc[l], g.svc[l]);
    vr.rpb = 1; vr.dst_bstride = max_len; vr.dst_off_dev = g.step;
    HIPCHK(launch_rows(vr, st));
    AttnArgs a = attn_args(s, B, 1, 0, max_len);
    a.k = g.kc[l]; a.sk = g.skc[l]; a.v = g.vc[l]; a.sv = g.svc[l];
    a.sk_dev = g.step; a.sk_add = 1;
    a.dec = 1;
    HIPCHK(launch_attention(a, st));
    RC(quant(s.ctx, D, B, D, s.a8, s.sa, st));
    RC(linear(c, L.o, s.a8, s.sa, B, EPI_RESIDUAL, s.x, s.x, D, st));
    RC(cross_attn_block(m, L, l, s, g.cross, B, 1, S, src_mask, st));
    RC(ffn_block(c, L.w1, L.w2, L.ln[2], s, B, st));
  }
  RC(ln_out(s.x, B, m->dec_norm, D, g.xo, st));
  HIPCHK(launch_generator(g.xo, D, B, m->gen_w, m->gen_b, c.tgt_vocab, g.logits, st));
  HIPCHK(launch_logsoftmax_argmax(g.logits, B, c.tgt_vocab, nullptr, ids, max_len, g.step, 1,
                                  st));
  HIPCHK(launch_step_inc(g.step, st));
  return QTX_OK;
}


int greedy_run(const qtx_model* m, GreedyWS& g, const int64_t* src, int B, int S, int max_len,
               int64_t start, const qtx_fault* f, hipStream_t st);

}  // namespace

extern "C" {

size_t qtx_encoder_workspace_size(const qtx_model* m, int32_t B, int32_t S) {
  return m ? enc_ws(m->cfg, B, S) : 0;
}
size_t qtx_decoder_workspace_size(const qtx_model* m, int32_t B, int32_t T, int32_t S) {
  return m ? dec_ws(m->cfg, B, T, S) : 0;
}
size_t qtx_greedy_workspace_size(const qtx_model* m, int32_t B, int32_t S, int32_t max_len) {
  if (!m) return 0;
  Arena ar;
  carve_greedy(ar, m->cfg, B, S, max_len);
  return align_up(ar.used);
}

int32_t qtx_encoder_forward_fault(const qtx_model* m, const float* x, const uint8_t* src_mask,
                                  int32_t B, int32_t S, float* out, void* ws, size_t ws_bytes,
                                  const qtx_fault* f, void* stream) {
  if (!m || !x || !src_mask || !out || !ws) return fail(QTX_E_INVALID, "null argument");
  if (B <= 0 || S <= 0 || S > 512) return fail(QTX_E_INVALID, "bad shape B=%d S=%d", B, S);
  if (ws_bytes < enc_ws(m->cfg, B, S)) return fail(QTX_E_WORKSPACE, "workspace too small");
  RC(check_fault(m, f, 0, B, S, 0));
  Arena ar;
  ar.base = (uint8_t*)ws; ar.cap = ws_bytes;
  hipStream_t st = (hipStream_t)stream;
  unsigned* cst = nullptr;
  RC(call_status_begin(m, &cst, st));
  if (!enc_split(B) || (f && f->kind != QTX_FAULT_NONE)) {
    Scratch s = carve_scratch(ar, m->cfg, (long)B * S);
    s.status = cst;
    return encoder_run(m, x, src_mask, B, S, out, s, st, f);
  }
  // The model's second stream and its three events are shared by every caller: the lock
  // is held across the whole record / wait sequence, so two threads' fork, lag and join
  // records cannot interleave (a wait always pairs with its own call's record).
  qtx_model* mm = const_cast<qtx_model*>(m);
  std::lock_guard<std::mutex> lk(mm->mu);
  DeviceGuard dg(mm->device);
  if (!mm->estream) {
    HIPCHK(hipStreamCreateWithFlags(&mm->estream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&mm->ev_fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&mm->ev_lag, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&mm->ev_join, hipEventDisableTiming));
  }
  const int B0 = B / 2, B1 = B - B0;
  const long D = m->cfg.d_model;
  Scratch s0 = carve_scratch(ar, m->cfg, (long)B0 * S);
  Scratch s1 = carve_scratch(ar, m->cfg, (long)B1 * S);
  s0.status = s1.status = cst;
  // half 1 starts when half 0's first layer has passed its QKV GEMM (ev_lag)
  HIPCHK(hipEventRecord(mm->ev_fork, st));
  HIPCHK(hipStreamWaitEvent(mm->estream, mm->ev_fork, 0));
  RC(encoder_run(m, x, src_mask, B0, S, out, s0, st, nullptr, mm->ev_lag));
  HIPCHK(hipStreamWaitEvent(mm->estream, mm->ev_lag, 0));
  RC(encoder_run(m, x + (long)B0 * S * D, src_mask + (long)B0 * S, B1, S, out + (long)B0 * S * D,
                 s1, mm->estream, nullptr));
  HIPCHK(hipEventRecord(mm->ev_join, mm->estream));
  HIPCHK(hipStreamWaitEvent(st, mm->ev_join, 0));
  return QTX_OK;
}

int32_t qtx_encoder_forward(const qtx_model* m, const float* x, const uint8_t* src_mask,
                            int32_t B, int32_t S, float* out, void* ws, size_t ws_bytes,
                            void* stream) {
  return qtx_encoder_forward_fault(m, x, src_mask, B, S, out, ws, ws_bytes, nullptr, stream);
}

int32_t qtx_decoder_forward_fault(const qtx_model* m, const float* y, const float* memory,
                                  const uint8_t* src_mask, const uint8_t* tgt_mask,
                                  int32_t tgt_mask_batched, int32_t B, int32_t T, int32_t S,
                                  float* out, void* ws, size_t ws_bytes, const qtx_fault* f,
                                  void* stream) {
  if (!m || !y || !memory || !src_mask || !tgt_mask || !out || !ws)
    return fail(QTX_E_INVALID, "null argument");
  if (B <= 0 || T <= 0 || S <= 0 || T > 512 || S > 512)
    return fail(QTX_E_INVALID, "bad shape B=%d T=%d S=%d", B, T, S);
  if (ws_bytes < dec_ws(m->cfg, B, T, S)) return fail(QTX_E_WORKSPACE, "workspace too small");
  RC(check_fault(m, f, 1, B, T, S));
  hipStream_t st = (hipStream_t)stream;
  const qtx_config& c = m->cfg;
  const int D = c.d_model, M = B * T;
  // no decoder kernel sets a status word (the in-launch FFN1 exchange runs on the KP
  // encoder path only), so this call neither claims nor touches the thread's word: an
  // error an earlier encode left there stays until qtx_model_check reports it
  Arena ar;
  ar.base = (uint8_t*)ws; ar.cap = ws_bytes;
  Scratch s = carve_scratch(ar, c, M);
  CrossKV x = carve_cross(ar, c, (long)B * S);
  RC(cross_kv(m, memory, B * S, x, st, f));
  HIPCHK(hipMemcpyAsync(s.x, y, (size_t)M * D * 4, hipMemcpyDeviceToDevice, st));
  const long tm_bs = tgt_mask_batched ? (long)T * T : 0;
  if (!row_path(c)) {
    for (int l = 0; l < c.n_layers; ++l) {
      const DecLayer& L = m->dec[l];
      RC(self_attn_block(c, L.qkv, L.o, L.ln[0], s, B, T, tgt_mask, tm_bs, T, true, st));
      RC(cross_attn_block(m, L, l, s, x, B, T, S, src_mask, st));
      RC(ffn_block(c, L.w1, L.w2, L.ln[2], s, M, st));
    }
    RC(ln_out(s.x, M, m->dec_norm, D, out, st));
    return QTX_OK;
  }
  // LayerNorm + quant of each sublayer's input fused into the previous residual GEMM
  // (as encoder_run); the last FFN2 applies the final decoder norm
  const int NL = c.n_layers;
  RC(ln_quant(s.x, M, m->dec[0].ln[0], D, s.a8, s.sa, st));
  for (int l = 0; l < NL; ++l) {
    const DecLayer& L = m->dec[l];
    auto fa = [&](GemmId gid) { return fault_for(f, 1, l, gid, M, c); };
    RC(row_quant(L.qkv, s.a8, s.sa, M, s.q8, s.sq, st, fa(G_QKV)));
    AttnArgs a = attn_args(s, B, T, T, T);
    a.mask = tgt_mask; a.m_bs = tm_bs; a.m_is = T;
    a.c_ld = D;
    a.dec = 1;
    AttnFault af;
    if (attn_fault_for(f, 1, l, false, T, T, af)) {
      RC(attention_fault(a, af, M, D, s, st));
    } else {
      const hipError_t ea = knobs().no_attn_encq ? hipErrorNotSupported
                                                       : launch_attention_encq(a, s.a8, s.sa, st);
      if (ea == hipErrorNotSupported) {  // other shapes: fp32 context + quantization kernel
        HIPCHK(launch_attention(a, st));
        RC(quant(s.ctx, D, M, D, s.a8, s.sa, st));
      } else {
        HIPCHK(ea);
      }
    }
    RC(row_res_ln(L.o, s.a8, s.sa, M, s.x, L.ln[1], s.a8, s.sa, nullptr, st, fa(G_O)));
    RC(row_quant(L.cq, s.a8, s.sa, M, s.q8, s.sq, st, fa(G_CQ)));
    a = attn_args(s, B, T, S, S);
    a.k = x.k8[l]; a.sk = x.sk[l]; a.v = x.v8[l]; a.sv = x.sv[l];
    a.mask = src_mask; a.m_bs = S; a.m_is = 0;
    a.dec = 1;
    if (attn_fault_for(f, 1, l, true, T, S, af)) {
      RC(attention_fault(a, af, M, D, s, st));
    } else {
      HIPCHK(launch_attention(a, st));
      RC(quant(s.ctx, D, M, D, s.a8, s.sa, st));
    }
    RC(row_res_ln(L.co, s.a8, s.sa, M, s.x, L.ln[2], s.a8, s.sa, nullptr, st, fa(G_CO)));
    RC(row_ffn1(c, L.w1, s.a8, s.sa, M, s, st, fa(G_FFN1)));
    if (l + 1 < NL)
      RC(row_res_ln(L.w2, s.h8, s.sh, M, s.x, m->dec[l + 1].ln[0], s.a8, s.sa, nullptr, st, fa(G_FFN2)));
    else
      RC(row_res_ln(L.w2, s.h8, s.sh, M, s.x, m->dec_norm, nullptr, nullptr, out, st, fa(G_FFN2)));
  }
  return QTX_OK;
}

int32_t qtx_decoder_forward(const qtx_model* m, const float* y, const float* memory,
                            const uint8_t* src_mask, const uint8_t* tgt_mask,
                            int32_t tgt_mask_batched, int32_t B, int32_t T, int32_t S,
                            float* out, void* ws, size_t ws_bytes, void* stream) {
  return qtx_decoder_forward_fault(m, y, memory, src_mask, tgt_mask, tgt_mask_batched, B, T, S,
                                   out, ws, ws_bytes, nullptr, stream);
}

int32_t qtx_embed(const qtx_model* m, int32_t which, const int64_t* ids, int32_t B, int32_t T,
                  int32_t pos0, float* out, void* stream) {
  if (!m || !ids || !out) return fail(QTX_E_INVALID, "null argument");
  if (pos0 < 0 || pos0 + T > m->cfg.max_len)
    return fail(QTX_E_INVALID, "positions exceed max_len %d", m->cfg.max_len);
  const float* lut = which ? m->tgt_lut : m->src_lut;
  const int vocab = which ? m->cfg.tgt_vocab : m->cfg.src_vocab;
  HIPCHK(launch_embed(ids, T, B, T, nullptr, pos0, lut, vocab, m->pe, m->cfg.max_len, out,
                      (long)T * m->cfg.d_model, (hipStream_t)stream));
  return QTX_OK;
}

int32_t qtx_generator(const qtx_model* m, const float* x, int32_t M, float* logp,
                      int64_t* ids, void* ws, size_t ws_bytes, void* stream) {
  if (!m || !x || !ws) return fail(QTX_E_INVALID, "null argument");
  const int V = m->cfg.tgt_vocab;
  if (ws_bytes < (size_t)M * V * sizeof(float)) return fail(QTX_E_WORKSPACE, "ws too small");
  hipStream_t st = (hipStream_t)stream;
  float* logits = (float*)ws;   // the raw logits stay in ws[0 .. M*V) for the caller
  HIPCHK(launch_generator_mfma(x, m->cfg.d_model, M, nullptr, nullptr, m->gen_wt, m->gen_b, V,
                               logits, st));
  HIPCHK(launch_logsoftmax_argmax(logits, M, V, logp, ids, 1, nullptr, 0, st));
  return QTX_OK;
}

int32_t qtx_greedy_decode_fault(const qtx_model* m, const int64_t* src,
                                const uint8_t* src_mask, int32_t B, int32_t S, int32_t max_len,
                                int64_t start, int64_t* ids, void* ws, size_t ws_bytes,
                                const qtx_fault* f, void* stream) {
  if (!m || !src || !src_mask || !ids || !ws) return fail(QTX_E_INVALID, "null argument");
  const qtx_config& c = m->cfg;
  if (B <= 0 || S <= 0 || S > 512 || max_len < 1 || max_len > 512 || max_len > c.max_len ||
      S > c.max_len)
    return fail(QTX_E_INVALID, "bad shape B=%d S=%d max_len=%d", B, S, max_len);
  if (ws_bytes < qtx_greedy_workspace_size(m, B, S, max_len))
    return fail(QTX_E_WORKSPACE, "workspace too small");
  if (f && f->kind != QTX_FAULT_NONE && f->module != 0)
    return fail(QTX_E_UNSUPPORTED, "greedy decode takes encoder faults (decoder faults: "
                                   "qtx_decoder_forward_fault on the step's prefix)");
  RC(check_fault(m, f, 0, B, S, 0));
  hipStream_t st = (hipStream_t)stream;
  Arena ar;
  ar.base = (uint8_t*)ws; ar.cap = ws_bytes;
  unsigned* cst = nullptr;
  RC(call_status_begin(m, &cst, st));
  GreedyWS g = carve_greedy(ar, c, B, S, max_len);
  g.enc.status = cst;
  // the decode reads the workspace's copy of src_mask and writes the workspace's ids
  // (the captured graphs then depend on the workspace only); ids go out at the end
  HIPCHK(hipMemcpyAsync(g.mask, src_mask, (size_t)B * S, hipMemcpyDeviceToDevice, st));
  RC(greedy_run(m, g, src, B, S, max_len, start, f, st));
  HIPCHK(hipMemcpyAsync(ids, g.ids, (size_t)B * max_len * sizeof(int64_t),
                        hipMemcpyDeviceToDevice, st));
  return QTX_OK;
}

int32_t qtx_model_check(const qtx_model* m, void* stream) {
  if (!m) return fail(QTX_E_INVALID, "null model");
  DeviceGuard dg(m->device);
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  unsigned v = 0;
  unsigned* word = nullptr;
  for (const CallStatus& cs : t_calls.v)
    if (cs.m == m && cs.serial == m->serial) word = m->status + 4 * cs.slot;
  // no word: this thread has made no call on m that can raise a device error (the word is
  // per thread: a check reports the calling thread's calls only)
  if (!word) return QTX_OK;
  HIPCHK(hipMemcpy(&v, word, sizeof v, hipMemcpyDeviceToHost));
  if (!v) return QTX_OK;
  HIPCHK(hipMemset(word, 0, sizeof(unsigned)));   // reported once (the thread's own word)
  return fail(QTX_E_DEVICE, "%s", status_text(v));
}

int32_t qtx_greedy_decode(const qtx_model* m, const int64_t* src, const uint8_t* src_mask,
                          int32_t B, int32_t S, int32_t max_len, int64_t start, int64_t* ids,
                          void* ws, size_t ws_bytes, void* stream) {
  return qtx_greedy_decode_fault(m, src, src_mask, B, S, max_len, start, ids, ws, ws_bytes,
                                 nullptr, stream);
}

}  // extern "C"

namespace {

int greedy_run(const qtx_model* m, GreedyWS& g, const int64_t* src, int B, int S, int max_len,
               int64_t start, const qtx_fault* f, hipStream_t st) {
  const qtx_config& c = m->cfg;
  const int D = c.d_model;
  const uint8_t* src_mask = g.mask;
  int64_t* ids = g.ids;
  const bool fused = S <= 128 && max_len <= 128 && !knobs().unfused;

  // encoder: memory = encode(src_embed(src), src_mask); the cross K/V of every layer
  // (captured into a hipGraph with the steps' replay — QTX_PRE_GRAPH in round 3 — it
  // measured no faster: 14.34 vs 14.31 ms per B = 32 decode; the host's enqueue of these
  // launches runs ahead of the GPU)
  HIPCHK(launch_embed(src, S, B, S, nullptr, 0, m->src_lut, c.src_vocab, m->pe, c.max_len,
                      g.enc.x, (long)S * D, st));
  RC(encoder_run(m, g.enc.x, src_mask, B, S, g.memory, g.enc, st, f));
  RC(cross_kv(m, g.memory, B * S, g.cross, st));
  if (fused) {   // the cross values of every layer in k_dec_attn's 4-key groups
    const long v_ls = g.cross.v8.size() > 1 ? (long)(g.cross.v8[1] - g.cross.v8[0]) : 0;
    HIPCHK(launch_vgroup4(g.cross.v8[0], v_ls, c.n_layers, B, S, g.cvg[0],
                          (long)B * ((S + 3) & ~3) * D, st));
  }

  // ids[:, 0] = start ; step[0] = position 0, step[1] = arrival counter
  HIPCHK(launch_fill_col(ids, max_len, B, start, st));
  HIPCHK(launch_zero(g.step, 16, st));
  if (!fused) {
    for (int t = 0; t + 1 < max_len; ++t) RC(greedy_step_unfused(m, g, B, S, max_len, ids, src_mask, st));
    return QTX_OK;
  }
  // sub-batches: each has its own step scratch and step counter; the first decoder input
  // is tgt_embed(ys[:, 0]) at position 0, later ones come from the previous step's argmax
  const Groups gr = decode_groups(B);
  std::vector<GreedyWS> gv;
  HIPCHK(hipMemsetAsync(g.gsteps, 0, sizeof(int) * 4 * QTX_MAX_GROUPS, st));
  for (int i = 0; i < gr.G; ++i) {
    gv.push_back(group_view(g, c, i, gr.b0(i), S, max_len));
    HIPCHK(launch_embed(ids + (long)gr.b0(i) * max_len, max_len, gr.rows(i, B), 1, gv[i].step,
                        0, m->tgt_lut, c.tgt_vocab, m->pe, c.max_len, gv[i].dec.x, D, st));
  }
  auto step_fn = [&](int i, hipStream_t s, int t) {
    return greedy_step_fused(m, gv[i], gr.rows(i, B), S, max_len, ids + (long)gr.b0(i) * max_len,
                             src_mask + (long)gr.b0(i) * S, s, t);
  };
  // One decode step per sub-batch captured once per (shape, buffers) as a hipGraph on its
  // own stream and replayed max_len-1 times there; the streams fork from and join back
  // into the caller's stream.
  qtx_model* mm = const_cast<qtx_model*>(m);
  std::lock_guard<std::mutex> lock(mm->mu);
  DeviceGuard dg(mm->device);
  if (!mm->ev_in) HIPCHK(hipEventCreateWithFlags(&mm->ev_in, hipEventDisableTiming));
  for (int i = 0; i < gr.G; ++i)
    if (!mm->gstream[i]) {
      HIPCHK(hipStreamCreateWithFlags(&mm->gstream[i], hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&mm->ev_out[i], hipEventDisableTiming));
    }
  if (knobs().no_graph) {     // eager launches (QTX_NO_GRAPH); sub-batches on their streams
    const bool fk = gr.G > 1;
    if (fk) {
      HIPCHK(hipEventRecord(mm->ev_in, st));
      for (int i = 0; i < gr.G; ++i) HIPCHK(hipStreamWaitEvent(mm->gstream[i], mm->ev_in, 0));
    }
    for (int t = 0; t + 1 < max_len; ++t)
      for (int i = 0; i < gr.G; ++i) RC(step_fn(i, fk ? mm->gstream[i] : st, t));
    if (fk)
      for (int i = 0; i < gr.G; ++i) {
        HIPCHK(hipEventRecord(mm->ev_out[i], mm->gstream[i]));
        HIPCHK(hipStreamWaitEvent(st, mm->ev_out[i], 0));
      }
    return QTX_OK;
  }
  // steps per graph: the whole decode in one graph by default (one graph launch); must
  // divide max_len-1 (the step position is read from device memory, so replays chain)
  int per_graph = max_len - 1;
  if (const int v = knobs().graph_steps; v > 0 && (max_len - 1) % v == 0) per_graph = v;
  if (max_len <= 1) return QTX_OK;
  // a graph of the whole decode is replayed once per decode from position 0: each captured
  // step knows its position (a shorter graph replays at several)
  const bool known = per_graph == max_len - 1;
  const bool joint = gr.G > 1 && knobs().group_graph;
  // the switches a captured step depends on are part of its key (knobs can be reloaded)
  const Knobs& kn = knobs();
  // (every switch: the key carries the knob generation, bumped by each reload — ADVICE r04:
  // QTX_SKINNY_WIDE, QTX_RB_*, ... pick launch shapes inside the captured step too)
  const std::string variant = std::to_string(knobs_generation()) + ":" + std::to_string(kn.split_ln) +
                              std::to_string(kn.ffn_qkernel) + std::to_string(kn.group_graph) +
                              std::to_string(kn.device_step);
  const GraphKey key{B, S, max_len, gr.G * 1000 + per_graph, g.gsteps, variant};
  auto it = mm->graphs.find(key);
  if (it == mm->graphs.end()) {
    if (mm->graphs.size() >= 16) mm->clear_graphs();
    std::vector<hipGraphExec_t> execs;
    auto drop = [&] {
      for (hipGraphExec_t e : execs) (void)hipGraphExecDestroy(e);
    };
    // QTX_GROUP_GRAPH (experiment): the G sub-batches as G independent branches of ONE graph
    // (forked and joined inside the capture), launched on the caller's stream
    if (joint) {
      hipGraph_t graph = nullptr;
      hipStream_t s0 = mm->gstream[0];
      HIPCHK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
      int rc = QTX_OK;
      hipError_t e = hipEventRecord(mm->ev_in, s0);
      for (int i = 1; i < gr.G && e == hipSuccess; ++i) e = hipStreamWaitEvent(mm->gstream[i], mm->ev_in, 0);
      for (int t = 0; t < per_graph && rc == QTX_OK && e == hipSuccess; ++t)
        for (int i = 0; i < gr.G && rc == QTX_OK; ++i) rc = step_fn(i, mm->gstream[i], known ? t : -1);
      for (int i = 1; i < gr.G && e == hipSuccess; ++i) {
        e = hipEventRecord(mm->ev_out[i], mm->gstream[i]);
        if (e == hipSuccess) e = hipStreamWaitEvent(s0, mm->ev_out[i], 0);
      }
      const hipError_t e2 = hipStreamEndCapture(s0, &graph);
      if (rc != QTX_OK || e != hipSuccess || e2 != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        if (rc != QTX_OK) return rc;
        HIPCHK(e != hipSuccess ? e : e2);
      }
      hipGraphExec_t exec = nullptr;
      e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      HIPCHK(e);
      execs.push_back(exec);
    }
    for (int i = 0; i < (joint ? 0 : gr.G); ++i) {
      hipGraph_t graph = nullptr;
      hipError_t e = hipStreamBeginCapture(mm->gstream[i], hipStreamCaptureModeThreadLocal);
      if (e != hipSuccess) { drop(); HIPCHK(e); }
      int rc = QTX_OK;
      for (int t = 0; t < per_graph && rc == QTX_OK; ++t) rc = step_fn(i, mm->gstream[i], known ? t : -1);
      e = hipStreamEndCapture(mm->gstream[i], &graph);
      if (rc != QTX_OK || e != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        drop();
        if (rc != QTX_OK) return rc;
        HIPCHK(e);
      }
      hipGraphExec_t exec = nullptr;
      e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      if (e != hipSuccess) { drop(); HIPCHK(e); }
      execs.push_back(exec);
    }
    GraphEntry ent;
    ent.execs = std::move(execs);
    it = mm->graphs.emplace(key, std::move(ent)).first;
  }
  // One sub-batch (or one joint graph): replay on the caller's stream itself (a graph
  // captured on one stream can be launched on any).  Several: fork to the model's streams
  // and join back.
  const bool fork = gr.G > 1 && !joint;
  hipStream_t ls[QTX_MAX_GROUPS];
  for (int i = 0; i < gr.G; ++i) ls[i] = fork ? mm->gstream[i] : st;
  if (fork) {
    HIPCHK(hipEventRecord(mm->ev_in, st));
    for (int i = 0; i < gr.G; ++i) HIPCHK(hipStreamWaitEvent(ls[i], mm->ev_in, 0));
  }
  hipEvent_t tg0 = nullptr, tg1 = nullptr;   // QTX_TIME_GRAPH: diagnostic timing to stderr
  const bool time_graph = knobs().time_graph;
  if (time_graph) {
    HIPCHK(hipEventCreate(&tg0));
    HIPCHK(hipEventCreate(&tg1));
    HIPCHK(hipEventRecord(tg0, ls[0]));
  }
  for (int t = 0; t < (max_len - 1) / per_graph; ++t)
    for (int i = 0; i < (int)it->second.execs.size(); ++i) HIPCHK(hipGraphLaunch(it->second.execs[i], ls[i]));
  if (time_graph) {
    float ms = 0.0f;
    HIPCHK(hipEventRecord(tg1, ls[0]));
    HIPCHK(hipEventSynchronize(tg1));
    HIPCHK(hipEventElapsedTime(&ms, tg0, tg1));
    fprintf(stderr, "qtx: decode graphs %.3f ms (%d steps, group 0)\n", ms, max_len - 1);
    (void)hipEventDestroy(tg0);
    (void)hipEventDestroy(tg1);
  }
  if (fork)
    for (int i = 0; i < gr.G; ++i) {
      HIPCHK(hipEventRecord(mm->ev_out[i], ls[i]));
      HIPCHK(hipStreamWaitEvent(st, mm->ev_out[i], 0));
    }
  // completion marker of this entry's replays (after the join: covers every sub-batch)
  if (!it->second.done) HIPCHK(hipEventCreateWithFlags(&it->second.done, hipEventDisableTiming));
  HIPCHK(hipEventRecord(it->second.done, st));
  return QTX_OK;
}

}  // namespace

extern "C" {

// ---- per-op entry points ---------------------------------------------------------------
int32_t qtx_row_quant(const float* x, int32_t rows, int32_t D, float qmax, int8_t* q,
                      float* s, void* stream) {
  if (!x || !q || !s) return fail(QTX_E_INVALID, "null argument");
  RowArgs a = rows_quant(x, D, rows, D, q, s);
  a.qmax = qmax;
  hipError_t e = launch_rows(a, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(QTX_E_UNSUPPORTED, "D=%d unsupported", D);
  HIPCHK(e);
  return QTX_OK;
}

int32_t qtx_layernorm_quant(const float* x, const float* a, const float* b, int32_t rows,
                            int32_t D, float* y, int8_t* q, float* s, void* stream) {
  if (!x || !a || !b || (!y && !q)) return fail(QTX_E_INVALID, "null argument");
  RowArgs r{};
  r.x = x; r.ldx = D; r.rows = rows; r.D = D; r.ln_a = a; r.ln_b = b;
  r.yout = y; r.ldy = D; r.q = q; r.ldq = D; r.s = s; r.qmax = 127.0f;
  r.rpb = rows > 0 ? rows : 1;
  hipError_t e = launch_rows(r, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(QTX_E_UNSUPPORTED, "D=%d unsupported", D);
  HIPCHK(e);
  return QTX_OK;
}

int32_t qtx_linear_i8(const int8_t* A, const float* sa, const void* W, const float* sw,
                      const float* bias, int32_t M, int32_t N, int32_t K, int32_t weight_bits,
                      int32_t flags, const float* res, float* out, void* stream) {
  if (!A || !sa || !W || !sw || !bias || !out) return fail(QTX_E_INVALID, "null argument");
  if ((flags & EPI_RESIDUAL) && !res) return fail(QTX_E_INVALID, "residual flag without res");
  if (K % 64) return fail(QTX_E_UNSUPPORTED, "K=%d not a multiple of 64", K);
  GemmArgs g{};
  g.A = A; g.lda = K; g.sa = sa; g.W = (const int8_t*)W;
  g.ldw = weight_bits == 8 ? K : K / 2; g.sw = sw; g.bias = bias;
  g.out = out; g.ldo = N; g.res = res; g.ldr = N;
  g.M = M; g.N = N; g.K = K; g.flags = flags;
  hipError_t e = launch_gemm(g, weight_bits, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(QTX_E_UNSUPPORTED, "weight_bits=%d", weight_bits);
  HIPCHK(e);
  return QTX_OK;
}

int32_t qtx_linear_rows(const qtx_row_gemm* a, void* stream) {
  if (!a || !a->A || !a->sa || !a->W || !a->sw || !a->bias) return fail(QTX_E_INVALID, "null argument");
  RowGemmArgs g{};
  g.A = a->A; g.lda = a->K; g.sa = a->sa; g.W = a->W; g.ldw = a->K; g.sw = a->sw;
  g.bias = a->bias; g.M = a->M; g.N = a->N; g.K = a->K; g.epi = a->epi;
  g.out8 = a->out8; g.ldo8 = a->ldo8; g.o8_ts = a->o8_ts; g.os = a->os; g.os_ts = a->os_ts;
  g.res = a->res; g.xout = a->xout; g.ln_a = a->ln_a; g.ln_b = a->ln_b;
  g.lnq = a->lnq; g.lns = a->lns; g.lnout = a->lnout;
  g.pmax_out = a->pmax_out; g.pmax_in = a->pmax_in; g.pmax_n = a->pmax_n; g.kp = a->kp;
  g.status = reinterpret_cast<unsigned*>(a->status);
  g.part = a->part; g.ksplit = a->ksplit;
  if (g.ksplit > 1 && (g.epi != RE_RES_LN || g.kp != 1 || !g.part || (g.ksplit & (g.ksplit - 1)) ||
                       g.ksplit > 8))
    return fail(QTX_E_INVALID, "ksplit %d: epi 1 with kp 1, a power of two <= 8, and part", g.ksplit);
  if (g.ksplit > 1 && (g.K % 64 || (g.K / 64) % (4 * g.ksplit)))   // launch_gemm_row's split
    return fail(QTX_E_INVALID, "ksplit %d needs K / 64 a multiple of 4 * ksplit (K=%d)", g.ksplit, g.K);
  const bool ok = (g.epi == RE_QUANT && g.out8 && g.os) ||
                  (g.epi == RE_RES_LN && g.res && g.xout && g.ln_a && g.ln_b &&
                   (g.lnq ? g.lns != nullptr : g.lnout != nullptr)) ||
                  (g.epi == RE_RELU_PMAX && g.pmax_out) ||
                  (g.epi == RE_RELU_QUANT_PMAX && g.out8 && g.os &&
                   (g.kp == 3 || g.kp == 5 ? g.pmax_out != nullptr : (g.pmax_in && g.pmax_n > 0)));
  if (!ok) return fail(QTX_E_INVALID, "operands missing for epi %d", g.epi);
  const hipError_t e = g.kp == 3 || g.kp == 5 ? launch_gemm_wsx(g, (hipStream_t)stream)
                       : g.kp == 2 || g.kp == 4 ? launch_gemm_ws(g, (hipStream_t)stream)
                                   : launch_gemm_row(g, (hipStream_t)stream);
  if (e == hipErrorInvalidValue)
    return fail(QTX_E_UNSUPPORTED, "rows GEMM: N=%d K=%d epi=%d kp=%d", g.N, g.K, g.epi, g.kp);
  HIPCHK(e);
  return QTX_OK;
}

int32_t qtx_pack_w_kp(const int8_t* W, int32_t N, int32_t K, int8_t* out, void* stream) {
  if (!W || !out) return fail(QTX_E_INVALID, "null argument");
  const hipError_t e = launch_pack_w_kp(W, N, K, out, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(QTX_E_UNSUPPORTED, "pack_w_kp N=%d K=%d", N, K);
  HIPCHK(e);
  return QTX_OK;
}

int32_t qtx_ffn_rows(const qtx_ffn_args* a, void* stream) {
  if (!a || !a->A || !a->sa || !a->wf || !a->sw1 || !a->b1 || !a->sw2 || !a->b2 || !a->x ||
      !a->ln_a || !a->ln_b || (a->lnq ? !a->lns : !a->lnout))
    return fail(QTX_E_INVALID, "null argument");
  FfnArgs g{};
  g.A = a->A; g.sa = a->sa; g.wf = a->wf; g.sw1 = a->sw1; g.b1 = a->b1; g.sw2 = a->sw2;
  g.b2 = a->b2; g.x = a->x; g.ln_a = a->ln_a; g.ln_b = a->ln_b; g.lnq = a->lnq;
  g.lns = a->lns; g.lnout = a->lnout; g.M = a->M; g.F = a->F;
  const hipError_t e = launch_ffn_fused(g, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(QTX_E_UNSUPPORTED, "ffn_rows: F=%d", a->F);
  HIPCHK(e);
  return QTX_OK;
}

int32_t qtx_pack_ffn(const int8_t* W1, const int8_t* W2, int32_t F, int8_t* out, void* stream) {
  if (!W1 || !W2 || !out) return fail(QTX_E_INVALID, "null argument");
  const hipError_t e = launch_pack_ffn(W1, W2, F, out, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(QTX_E_UNSUPPORTED, "pack_ffn F=%d", F);
  HIPCHK(e);
  return QTX_OK;
}

int32_t qtx_pack_w_ws(const int8_t* W, int32_t N, int32_t K, int8_t* out, void* stream) {
  if (!W || !out) return fail(QTX_E_INVALID, "null argument");
  const hipError_t e = launch_pack_w_ws(W, N, K, out, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(QTX_E_UNSUPPORTED, "pack_w_ws N=%d K=%d", N, K);
  HIPCHK(e);
  return QTX_OK;
}

int32_t qtx_skinny_linear(int32_t amode, const int8_t* A, const float* sa, const float* X,
                          int64_t ldx, const float* ln_a, const float* ln_b,
                          const float* pmax_in, int32_t pmax_n, const void* W, const float* sw,
                          const float* bias, int32_t M, int32_t N, int32_t K,
                          int32_t weight_bits, int32_t flags, const float* res, float* out,
                          float* pmax_out, void* stream) {
  if (!W || !sw || !bias || !out) return fail(QTX_E_INVALID, "null argument");
  if ((amode == A_I8 && (!A || !sa)) || (amode == A_LN && (!X || !ln_a || !ln_b)) ||
      (amode == A_F32Q && (!X || !pmax_in || pmax_n <= 0 || pmax_n > 128)) ||
      (amode == A_F32R && !X) || amode < 0 || amode > 3)
    return fail(QTX_E_INVALID, "operands missing for amode %d", amode);
  if (((flags & EPI_RESIDUAL) && !res) || ((flags & EPI_ROWMAX) && !pmax_out))
    return fail(QTX_E_INVALID, "flags need res / pmax_out");
  SkinnyArgs g{};
  g.amode = amode; g.A = A; g.sa = sa; g.X = X; g.ldx = ldx; g.ln_a = ln_a; g.ln_b = ln_b;
  g.pmax_in = pmax_in; g.pmax_n = pmax_n;
  g.W = (const int8_t*)W; g.ldw = weight_bits == 8 ? K : K / 2;
  g.sw = sw; g.bias = bias; g.out = out; g.ldo = N; g.res = res; g.ldr = N;
  g.pmax_out = pmax_out; g.M = M; g.N = N; g.K = K; g.flags = flags;
  hipError_t e = launch_skinny(g, weight_bits, (hipStream_t)stream);
  if (e == hipErrorInvalidValue)
    return fail(QTX_E_UNSUPPORTED, "skinny: N=%d K=%d amode=%d bits=%d", N, K, amode, weight_bits);
  HIPCHK(e);
  return QTX_OK;
}

int32_t qtx_decode_attention(int32_t kv_new, const float* y, int64_t ldy, int8_t* kc,
                             int8_t* vc, float* skc, float* svc, int32_t kv_bs,
                             const int32_t* step_dev, int32_t S, const uint8_t* mask,
                             int32_t B, float* ctx, float* pmax, void* stream) {
  if (!y || !kc || !vc || !skc || !svc || !ctx || !pmax)
    return fail(QTX_E_INVALID, "null argument");
  if (kv_new ? (!step_dev || kv_bs <= 0 || kv_bs > 128)
             : (!mask || S <= 0 || S > 128 || S > kv_bs))
    return fail(QTX_E_INVALID, "decode attention: bad step/mask/S/kv_bs");
  DecAttnArgs a{};
  a.y = y; a.ldy = ldy; a.kc = kc; a.vc = vc; a.skc = skc; a.svc = svc; a.kv_bs = kv_bs;
  a.step = step_dev; a.S = S; a.mask = mask; a.kv_new = kv_new;
  a.ctx = ctx; a.pmax = pmax; a.B = B;
  HIPCHK(launch_dec_attn(a, B, (hipStream_t)stream));
  return QTX_OK;
}

int32_t qtx_debug_nop(void* stream) {
  HIPCHK(launch_nop((hipStream_t)stream));
  return QTX_OK;
}

int32_t qtx_decode_argmax_embed(const qtx_model* m, const float* logits, int32_t M,
                                int64_t* ids, int64_t ids_bs, int32_t* step_dev,
                                float* x_next, void* stream) {
  if (!m || !logits || !ids || !step_dev || !x_next) return fail(QTX_E_INVALID, "null argument");
  if (M <= 0) return QTX_OK;
  const qtx_config& c = m->cfg;
  const hipError_t e = launch_argmax_embed(logits, M, c.tgt_vocab, ids, ids_bs, step_dev,
                                           reinterpret_cast<unsigned*>(step_dev + 1),
                                           m->tgt_lut, m->pe, c.max_len, x_next,
                                           (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(QTX_E_UNSUPPORTED, "tgt_vocab %d", c.tgt_vocab);
  HIPCHK(e);
  return QTX_OK;
}

int32_t qtx_pack_int4(const int8_t* q, int32_t N, int32_t K, uint8_t* packed, void* stream) {
  if (!q || !packed || K % 2) return fail(QTX_E_INVALID, "bad argument");
  HIPCHK(launch_pack_int4(q, N, K, packed, (hipStream_t)stream));
  return QTX_OK;
}

int32_t qtx_attention_trace(const int8_t* q, const float* sq, const int8_t* k, const float* sk,
                            const int8_t* v, const float* sv, const uint8_t* mask, int64_t m_bs,
                            int64_t m_is, int32_t B, int32_t H, int32_t Sq, int32_t Sk,
                            float* ctx, float* qk_acc, float* p_codes, int32_t dec, void* stream) {
  if (!q || !sq || !k || !sk || !v || !sv || !ctx) return fail(QTX_E_INVALID, "null argument");
  if (Sk <= 0 || Sk > 512 || Sq <= 0 || B <= 0 || H <= 0)
    return fail(QTX_E_UNSUPPORTED, "Sk=%d (max 512) Sq=%d B=%d H=%d", Sk, Sq, B, H);
  const long D = (long)H * 64;
  AttnArgs a{};
  a.q = q; a.q_bs = Sq * D; a.q_ld = D; a.sq = sq; a.sq_bs = Sq;
  a.k = k; a.k_bs = Sk * D; a.k_ld = D; a.sk = sk; a.sk_bs = Sk;
  a.v = v; a.v_bs = Sk * D; a.v_ld = D; a.sv = sv; a.sv_bs = Sk;
  a.mask = mask; a.m_bs = m_bs; a.m_is = m_is;
  a.ctx = ctx; a.c_bs = Sq * D; a.c_ld = D;
  a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk;
  a.dec = dec != 0;
  HIPCHK(launch_attn_trace(a, qk_acc, p_codes, (hipStream_t)stream));
  return QTX_OK;
}

int32_t qtx_attention_i8_quant(const int8_t* q, const float* sq, const int8_t* k,
                               const float* sk, const int8_t* v, const float* sv,
                               const uint8_t* key_mask, int32_t B, int32_t S, int8_t* ctx8,
                               float* sctx, void* stream) {
  if (!q || !sq || !k || !sk || !v || !sv || !ctx8 || !sctx) return fail(QTX_E_INVALID, "null argument");
  if (B <= 0 || S <= 0 || S > 128) return fail(QTX_E_UNSUPPORTED, "S=%d (1..128)", S);
  const long D = 512;
  AttnArgs a{};
  a.q = q; a.q_bs = S * D; a.q_ld = D; a.sq = sq; a.sq_bs = S;
  a.k = k; a.k_bs = S * D; a.k_ld = D; a.sk = sk; a.sk_bs = S;
  a.v = v; a.v_bs = S * D; a.v_ld = D; a.sv = sv; a.sv_bs = S;
  a.mask = key_mask; a.m_bs = S; a.m_is = 0;
  a.c_bs = S * D; a.c_ld = D;
  a.B = B; a.H = 8; a.Sq = S; a.Sk = S;
  HIPCHK(launch_attention_encq(a, ctx8, sctx, (hipStream_t)stream, true));
  return QTX_OK;
}

int32_t qtx_attention_i8(const int8_t* q, const float* sq, const int8_t* k, const float* sk,
                         const int8_t* v, const float* sv, const uint8_t* mask, int64_t m_bs,
                         int64_t m_is, int32_t B, int32_t H, int32_t Sq, int32_t Sk,
                         float* ctx, int32_t dec, void* stream) {
  if (!q || !sq || !k || !sk || !v || !sv || !ctx) return fail(QTX_E_INVALID, "null argument");
  if (Sk <= 0 || Sk > 512 || Sq <= 0) return fail(QTX_E_UNSUPPORTED, "Sk=%d (max 512)", Sk);
  const long D = (long)H * 64;
  AttnArgs a{};
  a.q = q; a.q_bs = Sq * D; a.q_ld = D; a.sq = sq; a.sq_bs = Sq;
  a.k = k; a.k_bs = Sk * D; a.k_ld = D; a.sk = sk; a.sk_bs = Sk;
  a.v = v; a.v_bs = Sk * D; a.v_ld = D; a.sv = sv; a.sv_bs = Sk;
  a.mask = mask; a.m_bs = m_bs; a.m_is = m_is;
  a.ctx = ctx; a.c_bs = Sq * D; a.c_ld = D;
  a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk;
  a.dec = dec != 0;
  HIPCHK(launch_attention(a, (hipStream_t)stream));
  return QTX_OK;
}

}  // extern "C"
