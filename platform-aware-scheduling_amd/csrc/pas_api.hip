// pas_api.hip — the C-ABI surface (include/pas.h): context, errors, timing, quantity
// parsing and the host-pointer wrappers around the device launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "pas.h"
#include "pas_internal.h"

namespace pas {

int set_error(pas_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

int check_hip(pas_ctx* ctx, hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return set_error(ctx, e == hipErrorOutOfMemory ? PAS_ENOMEM : PAS_EDEVICE, m);
}

int activate(pas_ctx* ctx) {
  PAS_HIP(ctx, hipSetDevice(ctx->device));
  return PAS_OK;
}

hipStream_t pick_stream(pas_ctx* ctx, void* s) {
  if (s == PAS_STREAM_NULL) return nullptr;  // the HIP null stream
  return s ? reinterpret_cast<hipStream_t>(s) : ctx->stream;
}

int ensure_scratch(pas_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->scratch_bytes) return PAS_OK;
  if (ctx->scratch) {
    PAS_HIP(ctx, hipStreamSynchronize(ctx->stream));
    PAS_HIP(ctx, hipFree(ctx->scratch));
    ctx->scratch = nullptr;
    ctx->scratch_bytes = 0;
  }
  size_t want = std::max(bytes, size_t(1) << 20);
  PAS_HIP(ctx, hipMalloc(&ctx->scratch, want));
  ctx->scratch_bytes = want;
  return PAS_OK;
}

// PAS_OK, or check_hip's status for a failed call
static int hip_status(pas_ctx* ctx, hipError_t e, const char* what) {
  return e == hipSuccess ? PAS_OK : check_hip(ctx, e, what);
}

AuxSlot* aux_acquire(pas_ctx* ctx, hipStream_t s, size_t bytes, int* rc) {
  AuxSlot* slot = nullptr;
  for (AuxSlot& a : ctx->aux_slot)
    if (a.used && a.stream == s) slot = &a;  // this stream's own slot: stream order
  if (!slot)
    for (AuxSlot& a : ctx->aux_slot)
      if (!a.used && !slot) slot = &a;
  if (!slot) {  // the least recently used slot, after its last call
    slot = &ctx->aux_slot[0];
    for (AuxSlot& a : ctx->aux_slot)
      if (a.last < slot->last) slot = &a;
    *rc = hip_status(ctx, hipStreamWaitEvent(s, slot->ev, 0), "aux_acquire: hipStreamWaitEvent");
    if (*rc) return nullptr;
  }
  if (!slot->ev) {
    *rc = hip_status(ctx, hipEventCreateWithFlags(&slot->ev, hipEventDisableTiming),
                    "aux_acquire: hipEventCreateWithFlags");
    if (*rc) return nullptr;
  }
  if (bytes > slot->bytes) {
    if (slot->p) {  // the slot's earlier calls are ordered before s: let them finish
      *rc = hip_status(ctx, hipStreamSynchronize(s), "aux_acquire: hipStreamSynchronize");
      if (!*rc) *rc = hip_status(ctx, hipFree(slot->p), "aux_acquire: hipFree");
      if (*rc) return nullptr;
      slot->p = nullptr;
      slot->bytes = 0;
    }
    *rc = hip_status(ctx, hipMalloc(&slot->p, bytes), "aux_acquire: hipMalloc");
    if (*rc) return nullptr;
    slot->bytes = bytes;
  }
  *rc = PAS_OK;
  return slot;
}

void* slot_buf(pas_ctx* ctx, AuxSlot* slot, int which, size_t bytes, hipStream_t s, int* rc) {
  *rc = PAS_OK;
  if (bytes <= slot->buf_bytes[which]) return slot->buf[which];
  if (slot->buf[which]) {  // the slot's earlier calls are ordered before s: let them finish
    *rc = hip_status(ctx, hipStreamSynchronize(s), "slot_buf: hipStreamSynchronize");
    if (!*rc) *rc = hip_status(ctx, hipFree(slot->buf[which]), "slot_buf: hipFree");
    if (*rc) return nullptr;
    slot->buf[which] = nullptr;
    slot->buf_bytes[which] = 0;
  }
  *rc = hip_status(ctx, hipMalloc(&slot->buf[which], bytes), "slot_buf: hipMalloc");
  if (*rc) return nullptr;
  slot->buf_bytes[which] = bytes;
  return slot->buf[which];
}

int derived_built(pas_ctx* ctx, DerivedSync& d, hipStream_t s) {
  if (!d.ev) {
    int rc = hip_status(ctx, hipEventCreateWithFlags(&d.ev, hipEventDisableTiming),
                        "derived_built: hipEventCreateWithFlags");
    if (rc) return rc;
  }
  int rc = hip_status(ctx, hipEventRecord(d.ev, s), "derived_built: hipEventRecord");
  if (rc) return rc;
  d.stream = s;
  d.valid = true;
  return PAS_OK;
}

int derived_wait(pas_ctx* ctx, const DerivedSync& d, hipStream_t s) {
  if (!d.valid || d.stream == s) return PAS_OK;  // same stream: stream order
  return hip_status(ctx, hipStreamWaitEvent(s, d.ev, 0), "derived_wait: hipStreamWaitEvent");
}

void aux_release(pas_ctx* ctx, AuxSlot* slot, hipStream_t s) {
  (void)hipEventRecord(slot->ev, s);
  slot->stream = s;
  slot->used = true;
  slot->last = ++ctx->aux_clock;
}

static hipEvent_t take_event(pas_ctx* ctx) {
  if (!ctx->event_pool.empty()) {
    hipEvent_t e = ctx->event_pool.back();
    ctx->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

void timing_begin(pas_ctx* ctx, hipStream_t s, int kernel, TimedLaunch* tl) {
  tl->kernel = -1;
  // span-level timing brackets whole paths only: events between the launches of a path
  // would add gaps to the span they measure
  if (!ctx->timing || (ctx->timing == PAS_TIMING_SPAN && kernel != PAS_K_TAS_SPAN &&
                       kernel != PAS_K_PRIO_REQUEST && kernel != PAS_K_GAS_FIT && kernel != PAS_K_TAS_VIOLATIONS &&
                       kernel != PAS_K_TAS_LABELS))
    return;
  tl->start = take_event(ctx);
  tl->stop = take_event(ctx);
  if (!tl->start || !tl->stop) return;
  tl->kernel = kernel;
  (void)hipEventRecord(tl->start, s);
}

void timing_end(pas_ctx* ctx, hipStream_t s, TimedLaunch* tl) {
  if (tl->kernel < 0) return;
  (void)hipEventRecord(tl->stop, s);
  ctx->pending.push_back(*tl);
}

static void resolve_timing(pas_ctx* ctx) {
  for (auto& tl : ctx->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(tl.stop) == hipSuccess &&
        hipEventElapsedTime(&ms, tl.start, tl.stop) == hipSuccess) {
      ctx->total_ms[tl.kernel] += ms;
      ctx->launches[tl.kernel] += 1;
    }
    ctx->event_pool.push_back(tl.start);
    ctx->event_pool.push_back(tl.stop);
  }
  ctx->pending.clear();
}

static void free_ptr(void*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

void free_tas(pas_ctx* ctx) {
  TasSnapshot& t = ctx->tas;
  free_ptr(reinterpret_cast<void*&>(t.vals));
  free_ptr(reinterpret_cast<void*&>(t.present));
  free_ptr(reinterpret_cast<void*&>(t.vals_t));
  free_ptr(reinterpret_cast<void*&>(t.pres_t));
  t.t_bytes = 0;
  t.t_epoch = 0;
  free_ptr(reinterpret_cast<void*&>(t.cnt));
  free_ptr(reinterpret_cast<void*&>(t.sorted));
  free_ptr(reinterpret_cast<void*&>(t.perm));
  free_ptr(reinterpret_cast<void*&>(t.f1k));
  free_ptr(reinterpret_cast<void*&>(t.f32));
  free_ptr(reinterpret_cast<void*&>(t.scale_tab));
  free_ptr(t.keys_a);
  free_ptr(t.keys_b);
  free_ptr(reinterpret_cast<void*&>(t.ids_a));
  free_ptr(reinterpret_cast<void*&>(t.ids_b));
  free_ptr(reinterpret_cast<void*&>(t.popc));
  free_ptr(reinterpret_cast<void*&>(t.word_scan));
  free_ptr(reinterpret_cast<void*&>(t.rows));
  free_ptr(t.sort_tmp);
  free_ptr(t.scan_tmp);
  const hipEvent_t ev = t.t_sync.ev;  // kept for the context's life (pas_destroy)
  t = TasSnapshot{};
  t.t_sync.ev = ev;
}

void free_gas(pas_ctx* ctx) {
  GasSnapshot& g = ctx->gas;
  free_ptr(reinterpret_cast<void*&>(g.n_cards));
  free_ptr(reinterpret_cast<void*&>(g.cap));
  free_ptr(reinterpret_cast<void*&>(g.used));
  free_ptr(g.derived);
  free_ptr(g.free_t);
  const hipEvent_t ev = g.derived_sync.ev;
  g = GasSnapshot{};
  g.derived_sync.ev = ev;
}

struct Carve {
  char* base;
  size_t off = 0;
  template <typename T>
  T* take(size_t count) {
    T* p = reinterpret_cast<T*>(base + off);
    off += (count * sizeof(T) + 255) & ~size_t(255);
    return p;
  }
};

static size_t carve_size(std::initializer_list<size_t> sizes) {
  size_t s = 0;
  for (size_t b : sizes) s += (b + 255) & ~size_t(255);
  return s;
}

}  // namespace pas

using namespace pas;

extern "C" {

int pas_abi_version(void) { return PAS_ABI_VERSION; }

int pas_create(const pas_config* cfg, pas_ctx** out) {
  if (!out) return PAS_EINVAL;
  *out = nullptr;
  pas_ctx* ctx = new (std::nothrow) pas_ctx();
  if (!ctx) return PAS_ENOMEM;
  int dev = cfg ? cfg->device : -1;
  if (dev < 0) {
    if (hipGetDevice(&dev) != hipSuccess) {
      delete ctx;
      return PAS_EDEVICE;
    }
  }
  ctx->device = dev;
  if (hipSetDevice(dev) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return PAS_EDEVICE;
  }
  ctx->stream = ctx->own_stream;
  int n_cu = 0;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      n_cu > 0)
    ctx->n_cu = n_cu;
  *out = ctx;
  return PAS_OK;
}

void pas_destroy(pas_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();
  resolve_timing(ctx);
  for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
  free_tas(ctx);
  free_gas(ctx);
  if (ctx->tas.t_sync.ev) (void)hipEventDestroy(ctx->tas.t_sync.ev);
  if (ctx->gas.derived_sync.ev) (void)hipEventDestroy(ctx->gas.derived_sync.ev);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->gas_sync_fault) (void)hipHostFree(ctx->gas_sync_fault);
  for (AuxSlot& a : ctx->aux_slot) {
    if (a.p) (void)hipFree(a.p);
    if (a.gas_counts) (void)hipFree(a.gas_counts);
    if (a.gas_limit) (void)hipFree(a.gas_limit);
    if (a.gas_sync) (void)hipFree(a.gas_sync);
    if (a.ev) (void)hipEventDestroy(a.ev);
    if (a.fork) (void)hipEventDestroy(a.fork);
    if (a.join) (void)hipEventDestroy(a.join);
    if (a.join2) (void)hipEventDestroy(a.join2);
    if (a.side) (void)hipStreamDestroy(a.side);
    if (a.side2) (void)hipStreamDestroy(a.side2);
    for (void* b : a.buf)
      if (b) (void)hipFree(b);
  }
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  delete ctx;
}

const char* pas_last_error(const pas_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int pas_set_stream(pas_ctx* ctx, void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  ctx->stream = hip_stream == PAS_STREAM_NULL ? nullptr
                : hip_stream                  ? reinterpret_cast<hipStream_t>(hip_stream)
                                              : ctx->own_stream;
  return PAS_OK;
}

int pas_synchronize(pas_ctx* ctx) {
  if (!ctx) return PAS_EINVAL;
  PAS_HIP(ctx, hipSetDevice(ctx->device));
  PAS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  // every stream's calls: the slots' last users and the GAS fits' side streams
  for (AuxSlot& a : ctx->aux_slot) {
    if (a.used && a.ev) PAS_HIP(ctx, hipEventSynchronize(a.ev));
    if (a.side) PAS_HIP(ctx, hipStreamSynchronize(a.side));
    if (a.side2) PAS_HIP(ctx, hipStreamSynchronize(a.side2));
  }
  // a GAS fit whose side-stream wait gave up (device flags): its results are incomplete
  return gas_fault_check(ctx);
}

int pas_parse_operator(const char* op) {
  if (!op) return PAS_EINVAL;
  if (std::strcmp(op, "LessThan") == 0) return PAS_OP_LESS_THAN;
  if (std::strcmp(op, "GreaterThan") == 0) return PAS_OP_GREATER_THAN;
  if (std::strcmp(op, "Equals") == 0) return PAS_OP_EQUALS;
  return PAS_EINVAL;
}

// pas_quantity_to_milli / pas_quantity_as_int64: quantity.cpp (host only)

// --------------------------------------------------------------------------- TAS

int pas_tas_snapshot_set(pas_ctx* ctx, uint64_t gen, int32_t n_nodes, int32_t n_metrics,
                         const int64_t* v_milli, const uint64_t* present) {
  if (!ctx) return PAS_EINVAL;
  if (n_nodes < 0 || n_metrics < 0 || (n_nodes > 0 && n_metrics > 0 && (!v_milli || !present)))
    return set_error(ctx, PAS_EINVAL, "pas_tas_snapshot_set: bad shape or null input");
  int rc = activate(ctx);
  if (rc) return rc;
  const size_t vb = sizeof(int64_t) * (size_t)n_nodes * (size_t)n_metrics;
  const size_t pb = sizeof(uint64_t) * (size_t)w64(n_nodes) * (size_t)n_metrics;
  rc = ensure_scratch(ctx, vb + pb + 256);
  if (rc) return rc;
  char* base = static_cast<char*>(ctx->scratch);
  int64_t* d_v = reinterpret_cast<int64_t*>(base);
  uint64_t* d_p = reinterpret_cast<uint64_t*>(base + ((vb + 255) & ~size_t(255)));
  if (vb) PAS_HIP(ctx, hipMemcpyAsync(d_v, v_milli, vb, hipMemcpyHostToDevice, ctx->stream));
  if (pb) PAS_HIP(ctx, hipMemcpyAsync(d_p, present, pb, hipMemcpyHostToDevice, ctx->stream));
  rc = tas_snapshot_build(ctx, gen, n_nodes, n_metrics, d_v, d_p, ctx->stream);
  if (rc) return rc;
  PAS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return PAS_OK;
}

int pas_tas_snapshot_set_device(pas_ctx* ctx, uint64_t gen, int32_t n_nodes, int32_t n_metrics,
                                const int64_t* d_v_milli, const uint64_t* d_present,
                                void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  if (n_nodes < 0 || n_metrics < 0) return set_error(ctx, PAS_EINVAL, "bad snapshot shape");
  int rc = activate(ctx);
  if (rc) return rc;
  return tas_snapshot_build(ctx, gen, n_nodes, n_metrics, d_v_milli, d_present,
                            pick_stream(ctx, hip_stream));
}

static int check_update(pas_ctx* ctx, uint64_t gen_from, int32_t n_cols, const int32_t* cols,
                        const void* vals, const void* present, const char* fn) {
  if (!ctx->tas.valid) return set_error(ctx, PAS_ENOSNAP, std::string(fn) + ": no TAS snapshot");
  if (ctx->tas.gen != gen_from)
    return set_error(ctx, PAS_ESTALE, std::string(fn) + ": resident generation " +
                                          std::to_string(ctx->tas.gen) + ", update from " +
                                          std::to_string(gen_from));
  const int32_t M = ctx->tas.n_metrics;
  if (n_cols < 0 || n_cols > M)
    return set_error(ctx, PAS_EINVAL, std::string(fn) + ": bad column count");
  if (n_cols > 0 && (!cols || (ctx->tas.n_nodes > 0 && (!vals || !present))))
    return set_error(ctx, PAS_EINVAL, std::string(fn) + ": null input");
  std::vector<char> seen((size_t)M, 0);
  for (int32_t c = 0; c < n_cols; ++c) {
    if (cols[c] < 0 || cols[c] >= M || seen[(size_t)cols[c]]++)
      return set_error(ctx, PAS_EINVAL,
                       std::string(fn) + ": columns must be distinct metric indices < n_metrics");
  }
  return PAS_OK;
}

int pas_tas_snapshot_update(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_cols,
                            const int32_t* cols, const int64_t* v_milli,
                            const uint64_t* present) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_update(ctx, gen_from, n_cols, cols, v_milli, present, "pas_tas_snapshot_update");
  if (rc) return rc;
  if ((rc = activate(ctx))) return rc;
  const int32_t N = ctx->tas.n_nodes;
  const size_t vb = sizeof(int64_t) * (size_t)n_cols * N;
  const size_t pb = sizeof(uint64_t) * (size_t)n_cols * w64(N);
  if ((rc = ensure_scratch(ctx, carve_size({vb, pb})))) return rc;
  Carve cv{static_cast<char*>(ctx->scratch)};
  int64_t* d_v = cv.take<int64_t>((size_t)n_cols * N);
  uint64_t* d_p = cv.take<uint64_t>((size_t)n_cols * w64(N));
  hipStream_t s = ctx->stream;
  if (vb) PAS_HIP(ctx, hipMemcpyAsync(d_v, v_milli, vb, hipMemcpyHostToDevice, s));
  if (pb) PAS_HIP(ctx, hipMemcpyAsync(d_p, present, pb, hipMemcpyHostToDevice, s));
  if ((rc = tas_snapshot_update(ctx, gen_to, n_cols, cols, d_v, d_p, s))) return rc;
  PAS_HIP(ctx, hipStreamSynchronize(s));
  return PAS_OK;
}

int pas_tas_snapshot_update_device(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to,
                                   int32_t n_cols, const int32_t* cols, const int64_t* d_v_milli,
                                   const uint64_t* d_present, void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_update(ctx, gen_from, n_cols, cols, d_v_milli, d_present,
                        "pas_tas_snapshot_update_device");
  if (rc) return rc;
  if ((rc = activate(ctx))) return rc;
  return tas_snapshot_update(ctx, gen_to, n_cols, cols, d_v_milli, d_present,
                             pick_stream(ctx, hip_stream));
}

int pas_tas_snapshot_info(const pas_ctx* ctx, uint64_t* gen, int32_t* n_nodes,
                          int32_t* n_metrics) {
  if (!ctx) return PAS_EINVAL;
  if (!ctx->tas.valid) return PAS_ENOSNAP;
  if (gen) *gen = ctx->tas.gen;
  if (n_nodes) *n_nodes = ctx->tas.n_nodes;
  if (n_metrics) *n_metrics = ctx->tas.n_metrics;
  return PAS_OK;
}

static int check_tas_gen(pas_ctx* ctx, uint64_t gen) {
  if (!ctx->tas.valid) return set_error(ctx, PAS_ENOSNAP, "no TAS snapshot uploaded");
  if (ctx->tas.gen != gen)
    return set_error(ctx, PAS_ESTALE, "TAS snapshot generation mismatch: resident " +
                                          std::to_string(ctx->tas.gen) + ", requested " +
                                          std::to_string(gen));
  return PAS_OK;
}

int pas_tas_snapshot_set_scale(pas_ctx* ctx, uint64_t gen, int32_t n_metrics,
                               const int32_t* col_scale, void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_tas_gen(ctx, gen);
  if (rc) return rc;
  const int32_t M = ctx->tas.n_metrics;
  if (n_metrics != M || (M > 0 && !col_scale))
    return set_error(ctx, PAS_EINVAL, "pas_tas_snapshot_set_scale: n_metrics != the snapshot's");
  std::vector<int64_t> tab(2 * (size_t)M);
  for (int32_t m = 0; m < M; ++m) {
    if (col_scale[m] < 0 || col_scale[m] > 9)
      return set_error(ctx, PAS_EINVAL, "pas_tas_snapshot_set_scale: scale outside 0..9");
    int64_t mult = 1;
    for (int32_t i = 0; i < col_scale[m]; ++i) mult *= 10;
    tab[2 * (size_t)m] = mult;
    tab[2 * (size_t)m + 1] = INT64_MAX / mult;
  }
  if (M == 0) return PAS_OK;
  if ((rc = activate(ctx))) return rc;
  hipStream_t s = pick_stream(ctx, hip_stream);
  PAS_HIP(ctx, hipMemcpyAsync(ctx->tas.scale_tab, tab.data(), sizeof(int64_t) * tab.size(),
                              hipMemcpyHostToDevice, s));
  PAS_HIP(ctx, hipStreamSynchronize(s));  // tab is this call's
  return PAS_OK;
}

// Host-side rule validation: an unknown operator string panics in core.EvaluateRule
// (operator.go:25) only when the rule is evaluated, i.e. when its metric is cached
// (dontschedule/strategy.go:28-32 skips missing metrics first).  Here: PAS_EINVAL.
// An unknown operator panics in the reference only when EvaluateRule runs, i.e. when the
// rule's metric map has at least one node (dontschedule/strategy.go:33-41, operator.go:25);
// otherwise the rule is never evaluated.  The column count is read back only in that
// (rare) case.  The *_device entry points do not validate: their callers parse operators
// with pas_parse_operator when the policy is built, and the kernels skip unknown ones.
static int validate_rules(pas_ctx* ctx, int32_t n, const pas_rule* rules) {
  for (int32_t i = 0; i < n; ++i) {
    const pas_rule& r = rules[i];
    if (r.op >= 0 && r.op <= 2) continue;
    if (r.metric < 0 || r.metric >= ctx->tas.n_metrics) continue;  // never evaluated
    int32_t c = 0;
    PAS_HIP(ctx, hipStreamSynchronize(ctx->stream));
    PAS_HIP(ctx, hipMemcpy(&c, ctx->tas.cnt + r.metric, sizeof(c), hipMemcpyDeviceToHost));
    if (c == 0) continue;  // empty metric map: no EvaluateRule call
    return set_error(ctx, PAS_EINVAL, "rule " + std::to_string(i) + ": unknown operator " +
                                          std::to_string(r.op) +
                                          " (the reference panics in EvaluateRule)");
  }
  return PAS_OK;
}

static int validate_csr(pas_ctx* ctx, int32_t n, const int32_t* off, const char* what) {
  if (off[0] != 0) return set_error(ctx, PAS_EINVAL, std::string(what) + ": offsets[0] != 0");
  for (int32_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i])
      return set_error(ctx, PAS_EINVAL, std::string(what) + ": offsets not monotone");
  return PAS_OK;
}

int pas_tas_eval(pas_ctx* ctx, uint64_t gen, int32_t n_pods, const pas_rule* rules,
                 const int32_t* rule_off, const pas_rule* prio, const uint64_t* cand,
                 uint32_t flags, uint64_t* pass_out, int32_t* order_out, int32_t* order_len) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_tas_gen(ctx, gen);
  if (rc) return rc;
  if (n_pods < 0 || (n_pods > 0 && (!rule_off || !prio)))
    return set_error(ctx, PAS_EINVAL, "pas_tas_eval: null rule_off/prio");
  if ((flags & PAS_TAS_FILTER) && n_pods > 0 && !pass_out)
    return set_error(ctx, PAS_EINVAL, "pas_tas_eval: FILTER without pass_out");
  if ((flags & PAS_TAS_PRIORITIZE) && n_pods > 0 && (!order_out || !order_len))
    return set_error(ctx, PAS_EINVAL, "pas_tas_eval: PRIORITIZE without order outputs");
  if (n_pods == 0) return PAS_OK;
  if ((rc = validate_csr(ctx, n_pods, rule_off, "rule_off"))) return rc;
  const int32_t n_rules = rule_off[n_pods];
  if (n_rules > 0 && !rules) return set_error(ctx, PAS_EINVAL, "pas_tas_eval: null rules");
  if ((rc = validate_rules(ctx, n_rules, rules))) return rc;
  if ((rc = activate(ctx))) return rc;
  const int64_t N = ctx->tas.n_nodes, W = w64(N);
  const size_t b_rules = sizeof(pas_rule) * (size_t)std::max(n_rules, 1);
  const size_t b_off = sizeof(int32_t) * (size_t)(n_pods + 1);
  const size_t b_prio = sizeof(pas_rule) * (size_t)n_pods;
  const size_t b_cand = cand ? sizeof(uint64_t) * (size_t)(W * n_pods) : 0;
  const size_t b_pass = (flags & PAS_TAS_FILTER) ? sizeof(uint64_t) * (size_t)(W * n_pods) : 0;
  const size_t b_order =
      (flags & PAS_TAS_PRIORITIZE) ? sizeof(int32_t) * (size_t)(N * n_pods) : 0;
  const size_t b_len = sizeof(int32_t) * (size_t)n_pods;
  if ((rc = ensure_scratch(ctx, carve_size({b_rules, b_off, b_prio, b_cand, b_pass, b_order,
                                            b_len}))))
    return rc;
  Carve cv{static_cast<char*>(ctx->scratch)};
  pas_rule* d_rules = cv.take<pas_rule>(std::max(n_rules, 1));
  int32_t* d_off = cv.take<int32_t>(n_pods + 1);
  pas_rule* d_prio = cv.take<pas_rule>(n_pods);
  uint64_t* d_cand = cand ? cv.take<uint64_t>(W * n_pods) : nullptr;
  uint64_t* d_pass = b_pass ? cv.take<uint64_t>(W * n_pods) : nullptr;
  int32_t* d_order = b_order ? cv.take<int32_t>(N * n_pods) : nullptr;
  int32_t* d_len = cv.take<int32_t>(n_pods);
  hipStream_t s = ctx->stream;
  if (n_rules) PAS_HIP(ctx, hipMemcpyAsync(d_rules, rules, b_rules, hipMemcpyHostToDevice, s));
  PAS_HIP(ctx, hipMemcpyAsync(d_off, rule_off, b_off, hipMemcpyHostToDevice, s));
  PAS_HIP(ctx, hipMemcpyAsync(d_prio, prio, b_prio, hipMemcpyHostToDevice, s));
  if (d_cand) PAS_HIP(ctx, hipMemcpyAsync(d_cand, cand, b_cand, hipMemcpyHostToDevice, s));
  rc = tas_eval_launch(ctx, n_pods, n_rules, d_rules, d_off, d_prio, d_cand, flags, d_pass,
                       d_order, d_len, 0, s);
  if (rc) return rc;
  if (d_pass) PAS_HIP(ctx, hipMemcpyAsync(pass_out, d_pass, b_pass, hipMemcpyDeviceToHost, s));
  if (flags & PAS_TAS_PRIORITIZE) {
    PAS_HIP(ctx, hipMemcpyAsync(order_len, d_len, b_len, hipMemcpyDeviceToHost, s));
    PAS_HIP(ctx, hipMemcpyAsync(order_out, d_order, b_order, hipMemcpyDeviceToHost, s));
  }
  PAS_HIP(ctx, hipStreamSynchronize(s));
  return PAS_OK;
}

int pas_tas_eval_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t n_rules,
                        const pas_rule* d_rules, const int32_t* d_rule_off,
                        const pas_rule* d_prio, const uint64_t* d_cand, uint32_t flags,
                        uint64_t* d_pass_out, int32_t* d_order_out, int32_t* d_order_len,
                        void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_tas_gen(ctx, gen);
  if (rc) return rc;
  if (n_pods < 0 || n_rules < 0) return set_error(ctx, PAS_EINVAL, "negative count");
  if (n_pods == 0) return PAS_OK;
  if (!d_rule_off || !d_prio || (n_rules > 0 && !d_rules))
    return set_error(ctx, PAS_EINVAL, "pas_tas_eval_device: null input");
  if ((flags & PAS_TAS_FILTER) && !d_pass_out)
    return set_error(ctx, PAS_EINVAL, "pas_tas_eval_device: FILTER without pass_out");
  if ((flags & PAS_TAS_PRIORITIZE) && (!d_order_out || !d_order_len))
    return set_error(ctx, PAS_EINVAL, "pas_tas_eval_device: PRIORITIZE without outputs");
  if ((rc = activate(ctx))) return rc;
  return tas_eval_launch(ctx, n_pods, n_rules, d_rules, d_rule_off, d_prio, d_cand, flags,
                         d_pass_out, d_order_out, d_order_len, 0, pick_stream(ctx, hip_stream));
}

static int check_prio_request(pas_ctx* ctx, const pas_rule* prio, int32_t n_req,
                              const void* req, const void* pos, const void* len) {
  if (!prio || n_req < 0 || !len || (n_req > 0 && (!req || !pos)))
    return set_error(ctx, PAS_EINVAL, "pas_tas_prioritize_request: bad argument");
  if (prio->metric >= ctx->tas.n_metrics)
    return set_error(ctx, PAS_EINVAL, "pas_tas_prioritize_request: metric out of range");
  return PAS_OK;
}

int pas_tas_prioritize_request(pas_ctx* ctx, uint64_t gen, const pas_rule* prio, int32_t n_req,
                               const int32_t* req_node, int32_t* pos_out, int32_t* len_out) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_tas_gen(ctx, gen);
  if (rc) return rc;
  if ((rc = check_prio_request(ctx, prio, n_req, req_node, pos_out, len_out))) return rc;
  if ((rc = activate(ctx))) return rc;
  size_t ws = 0;
  if ((rc = prio_request_workspace(ctx, n_req, &ws))) return rc;
  const size_t b_req = sizeof(int32_t) * (size_t)std::max(n_req, 1);
  if ((rc = ensure_scratch(ctx, carve_size({b_req, b_req, sizeof(int32_t), ws})))) return rc;
  Carve cv{static_cast<char*>(ctx->scratch)};
  int32_t* d_req = cv.take<int32_t>(std::max(n_req, 1));
  int32_t* d_pos = cv.take<int32_t>(std::max(n_req, 1));
  int32_t* d_len = cv.take<int32_t>(1);
  void* d_ws = cv.take<char>(ws);
  hipStream_t s = ctx->stream;
  if (n_req) PAS_HIP(ctx, hipMemcpyAsync(d_req, req_node, b_req, hipMemcpyHostToDevice, s));
  if ((rc = prio_request_launch(ctx, *prio, n_req, d_req, d_pos, d_len, d_ws, ws, s))) return rc;
  PAS_HIP(ctx, hipMemcpyAsync(len_out, d_len, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  if (n_req) PAS_HIP(ctx, hipMemcpyAsync(pos_out, d_pos, b_req, hipMemcpyDeviceToHost, s));
  PAS_HIP(ctx, hipStreamSynchronize(s));
  return PAS_OK;
}

int pas_tas_prioritize_request_device(pas_ctx* ctx, uint64_t gen, const pas_rule* prio,
                                      int32_t n_req, const int32_t* d_req_node,
                                      int32_t* d_pos_out, int32_t* d_len_out,
                                      void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_tas_gen(ctx, gen);
  if (rc) return rc;
  if ((rc = check_prio_request(ctx, prio, n_req, d_req_node, d_pos_out, d_len_out))) return rc;
  if ((rc = activate(ctx))) return rc;
  size_t ws = 0;
  if ((rc = prio_request_workspace(ctx, n_req, &ws))) return rc;
  // the workspace is the stream's aux slot (calls on other streams may run beside this one)
  hipStream_t s = pick_stream(ctx, hip_stream);
  SlotScope sc(ctx, s, ws, &rc);
  if (!sc.slot) return rc;
  return prio_request_launch(ctx, *prio, n_req, d_req_node, d_pos_out, d_len_out, sc.slot->p, ws,
                             s);
}

int pas_tas_violations(pas_ctx* ctx, uint64_t gen, int32_t n_strategies, const pas_rule* rules,
                       const int32_t* rule_off, uint64_t* viol_out) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_tas_gen(ctx, gen);
  if (rc) return rc;
  if (n_strategies < 0) return set_error(ctx, PAS_EINVAL, "negative strategy count");
  if (n_strategies == 0) return PAS_OK;
  if (!rule_off || !viol_out) return set_error(ctx, PAS_EINVAL, "null rule_off/viol_out");
  if ((rc = validate_csr(ctx, n_strategies, rule_off, "rule_off"))) return rc;
  const int32_t n_rules = rule_off[n_strategies];
  if (n_rules > 0 && !rules) return set_error(ctx, PAS_EINVAL, "null rules");
  if ((rc = validate_rules(ctx, n_rules, rules))) return rc;
  if ((rc = activate(ctx))) return rc;
  const int64_t W = w64(ctx->tas.n_nodes);
  const size_t b_rules = sizeof(pas_rule) * (size_t)std::max(n_rules, 1);
  const size_t b_off = sizeof(int32_t) * (size_t)(n_strategies + 1);
  const size_t b_viol = sizeof(uint64_t) * (size_t)(W * n_strategies);
  if ((rc = ensure_scratch(ctx, carve_size({b_rules, b_off, b_viol})))) return rc;
  Carve cv{static_cast<char*>(ctx->scratch)};
  pas_rule* d_rules = cv.take<pas_rule>(std::max(n_rules, 1));
  int32_t* d_off = cv.take<int32_t>(n_strategies + 1);
  uint64_t* d_viol = cv.take<uint64_t>(W * n_strategies);
  hipStream_t s = ctx->stream;
  if (n_rules) PAS_HIP(ctx, hipMemcpyAsync(d_rules, rules, b_rules, hipMemcpyHostToDevice, s));
  PAS_HIP(ctx, hipMemcpyAsync(d_off, rule_off, b_off, hipMemcpyHostToDevice, s));
  rc = tas_violations_launch(ctx, n_strategies, n_rules, d_rules, d_off, d_viol, s);
  if (rc) return rc;
  PAS_HIP(ctx, hipMemcpyAsync(viol_out, d_viol, b_viol, hipMemcpyDeviceToHost, s));
  PAS_HIP(ctx, hipStreamSynchronize(s));
  return PAS_OK;
}

int pas_tas_violations_device(pas_ctx* ctx, uint64_t gen, int32_t n_strategies,
                              int32_t n_rules, const pas_rule* d_rules,
                              const int32_t* d_rule_off, uint64_t* d_viol_out,
                              void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_tas_gen(ctx, gen);
  if (rc) return rc;
  if (n_strategies < 0 || n_rules < 0) return set_error(ctx, PAS_EINVAL, "negative count");
  if (n_strategies == 0) return PAS_OK;
  if (!d_rule_off || !d_viol_out || (n_rules > 0 && !d_rules))
    return set_error(ctx, PAS_EINVAL, "pas_tas_violations_device: null input");
  if ((rc = activate(ctx))) return rc;
  return tas_violations_launch(ctx, n_strategies, n_rules, d_rules, d_rule_off, d_viol_out,
                               pick_stream(ctx, hip_stream));
}

// --------------------------------------------------------------------------- GAS

static int gas_alloc(pas_ctx* ctx, int32_t n_nodes, int32_t max_cards, int32_t n_res) {
  GasSnapshot& g = ctx->gas;
  if (g.n_nodes != n_nodes || g.max_cards != max_cards || g.n_res != n_res || !g.n_cards) {
    PAS_HIP(ctx, hipStreamSynchronize(ctx->stream));
    free_gas(ctx);
    const size_t nn = (size_t)std::max(n_nodes, 1);
    PAS_HIP(ctx, hipMalloc(&g.n_cards, sizeof(int32_t) * nn));
    PAS_HIP(ctx, hipMalloc(&g.cap, sizeof(int64_t) * nn * (size_t)std::max(n_res, 1)));
    PAS_HIP(ctx, hipMalloc(&g.used, sizeof(int64_t) * nn * (size_t)std::max(max_cards, 1) *
                                        (size_t)std::max(n_res, 1)));
    PAS_HIP(ctx, hipMalloc(&g.derived, 64 + sizeof(int32_t) * nn));
    PAS_HIP(ctx, hipMalloc(&g.free_t, sizeof(int64_t) * PAS_GAS_PACKED *
                                          (size_t)std::max(n_res, 1) * nn));
    g.n_nodes = n_nodes;
    g.max_cards = max_cards;
    g.n_res = n_res;
  }
  return PAS_OK;
}

static int gas_shape_ok(pas_ctx* ctx, int32_t n_nodes, int32_t max_cards, int32_t n_res) {
  if (n_nodes < 0 || max_cards < 1 || n_res < 1)
    return set_error(ctx, PAS_EINVAL, "pas_gas_snapshot_set: bad shape");
  if (max_cards > PAS_GAS_MAX_CARDS || n_res > PAS_GAS_MAX_RES)
    return set_error(ctx, PAS_ECAPACITY,
                     "pas_gas_snapshot_set: max_cards <= 64 and n_res <= 4 supported");
  return PAS_OK;
}

int pas_gas_snapshot_set(pas_ctx* ctx, uint64_t gen, int32_t n_nodes, int32_t max_cards,
                         int32_t n_res, const int32_t* n_cards, const int64_t* cap_per_gpu,
                         const int64_t* used) {
  if (!ctx) return PAS_EINVAL;
  int rc = gas_shape_ok(ctx, n_nodes, max_cards, n_res);
  if (rc) return rc;
  if (n_nodes > 0 && (!n_cards || !cap_per_gpu || !used))
    return set_error(ctx, PAS_EINVAL, "pas_gas_snapshot_set: null input");
  for (int32_t n = 0; n < n_nodes; ++n)
    if (n_cards[n] > max_cards)
      return set_error(ctx, PAS_EINVAL, "pas_gas_snapshot_set: n_cards > max_cards");
  if ((rc = activate(ctx))) return rc;
  if ((rc = gas_alloc(ctx, n_nodes, max_cards, n_res))) return rc;
  GasSnapshot& g = ctx->gas;
  hipStream_t s = ctx->stream;
  if (n_nodes > 0) {
    PAS_HIP(ctx, hipMemcpyAsync(g.n_cards, n_cards, sizeof(int32_t) * n_nodes,
                                hipMemcpyHostToDevice, s));
    PAS_HIP(ctx, hipMemcpyAsync(g.cap, cap_per_gpu, sizeof(int64_t) * n_nodes * n_res,
                                hipMemcpyHostToDevice, s));
    PAS_HIP(ctx, hipMemcpyAsync(g.used, used,
                                sizeof(int64_t) * (size_t)n_nodes * max_cards * n_res,
                                hipMemcpyHostToDevice, s));
  }
  PAS_HIP(ctx, hipStreamSynchronize(s));
  g.gen = gen;
  ++g.epoch;
  g.valid = true;
  return PAS_OK;
}

// The device snapshot's card counts, which the host cannot check: a count past max_cards is
// read as max_cards (pas_gas_snapshot_set rejects it), so every node has its result written
// by the fit kernels that cover its cards.
__global__ void clamp_cards_kernel(int32_t* __restrict__ n_cards, int32_t n, int32_t max_cards) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) n_cards[i] = min(n_cards[i], max_cards);
}

int pas_gas_snapshot_set_device(pas_ctx* ctx, uint64_t gen, int32_t n_nodes, int32_t max_cards,
                                int32_t n_res, const int32_t* d_n_cards,
                                const int64_t* d_cap_per_gpu, const int64_t* d_used,
                                void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  int rc = gas_shape_ok(ctx, n_nodes, max_cards, n_res);
  if (rc) return rc;
  if (n_nodes > 0 && (!d_n_cards || !d_cap_per_gpu || !d_used))
    return set_error(ctx, PAS_EINVAL, "pas_gas_snapshot_set_device: null input");
  if ((rc = activate(ctx))) return rc;
  if ((rc = gas_alloc(ctx, n_nodes, max_cards, n_res))) return rc;
  GasSnapshot& g = ctx->gas;
  hipStream_t s = pick_stream(ctx, hip_stream);
  if (n_nodes > 0) {
    PAS_HIP(ctx, hipMemcpyAsync(g.n_cards, d_n_cards, sizeof(int32_t) * n_nodes,
                                hipMemcpyDeviceToDevice, s));
    PAS_HIP(ctx, hipMemcpyAsync(g.cap, d_cap_per_gpu, sizeof(int64_t) * n_nodes * n_res,
                                hipMemcpyDeviceToDevice, s));
    PAS_HIP(ctx, hipMemcpyAsync(g.used, d_used,
                                sizeof(int64_t) * (size_t)n_nodes * max_cards * n_res,
                                hipMemcpyDeviceToDevice, s));
    clamp_cards_kernel<<<(unsigned)((n_nodes + 255) / 256), 256, 0, s>>>(g.n_cards, n_nodes,
                                                                         max_cards);
    PAS_HIP(ctx, hipGetLastError());
  }
  g.gen = gen;
  ++g.epoch;
  g.valid = true;
  return PAS_OK;
}

static int check_gas_gen(pas_ctx* ctx, uint64_t gen) {
  if (!ctx->gas.valid) return set_error(ctx, PAS_ENOSNAP, "no GAS snapshot uploaded");
  if (ctx->gas.gen != gen) return set_error(ctx, PAS_ESTALE, "GAS snapshot generation mismatch");
  return PAS_OK;
}

// Shared host path of pas_gas_bind / pas_gas_release: validates, groups the operations by
// node (stable), uploads everything in one scratch carve and runs the commit kernel.
static int gas_commit(pas_ctx* ctx, bool release, uint64_t gen_from, uint64_t gen_to,
                      int32_t n_ops, const int32_t* op_pod, const int32_t* op_node,
                      int32_t n_pods, int32_t max_containers, int32_t i915_index,
                      const int64_t* req, const uint32_t* req_mask, const int32_t* n_containers,
                      const int32_t* cpc, const int32_t* cards, int32_t cards_stride,
                      uint32_t* res_out, int32_t* status_out, uint8_t* cards_out,
                      int32_t* nsel_out, int64_t* counts_out, const int64_t* counts,
                      const char* fn) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_gas_gen(ctx, gen_from);
  if (rc) return rc;
  const GasSnapshot& g = ctx->gas;
  const int32_t Q = g.n_res, N = g.n_nodes;
  if (n_ops < 0 || n_pods < 0 || max_containers < 0 || i915_index >= Q || i915_index < -1)
    return set_error(ctx, PAS_EINVAL, std::string(fn) + ": bad shape");
  if (n_ops > 0 && (!op_pod || !op_node || !status_out || !n_containers ||
                    (max_containers > 0 && (!req || !req_mask)) ||
                    (release ? (!counts && (!cpc || !cards)) : !res_out)))
    return set_error(ctx, PAS_EINVAL, std::string(fn) + ": null input");
  const int32_t K = g.max_cards;
  std::vector<int32_t> order((size_t)n_ops);
  for (int32_t i = 0; i < n_ops; ++i) {
    order[(size_t)i] = i;
    if (op_node[i] < 0 || op_node[i] >= N || op_pod[i] < 0 || op_pod[i] >= n_pods)
      return set_error(ctx, PAS_EINVAL, std::string(fn) + ": node or pod index out of range");
    const int32_t p = op_pod[i];
    if (n_containers[p] < 0 || n_containers[p] > max_containers)
      return set_error(ctx, PAS_EINVAL, std::string(fn) + ": n_containers out of range");
    // annotation cards of a release: within the card list (cards[i][cards_stride]), or per
    // container a count sum that fits int64 (counts form).  Binds have no selection limit.
    const int64_t limit = cards_stride;
    int64_t sel = 0;
    for (int32_t c = 0; c < n_containers[p]; ++c) {
      const int64_t b = (int64_t)p * max_containers + c;
      if ((req_mask[b] & ~PAS_REQ_UNKNOWN_KIND) >> Q) return set_error(ctx, PAS_EINVAL, std::string(fn) + ": mask bit >= n_res");
      if (!release) continue;
      if (counts) {
        int64_t kc = 0;
        for (int32_t k = 0; k < K; ++k) {
          const int64_t t = counts[((int64_t)i * max_containers + c) * K + k];
          if (t < 0 || kc > INT64_MAX - t)
            return set_error(ctx, PAS_EINVAL, std::string(fn) + ": card counts negative or "
                                                               "past int64");
          kc += t;
        }
        continue;
      }
      const int64_t v = cpc[(int64_t)i * max_containers + c];
      if (v < 0) return set_error(ctx, PAS_EINVAL, std::string(fn) + ": negative card count");
      sel = std::min(sel + std::min(v, limit + 1), limit + 1);
    }
    if (release && !counts && sel > limit)
      return set_error(ctx, PAS_EINVAL, std::string(fn) + ": more than " +
                                            std::to_string(limit) + " cards for one pod");
  }
  std::stable_sort(order.begin(), order.end(),
                   [&](int32_t a, int32_t b) { return op_node[a] < op_node[b]; });
  std::vector<int32_t> seg_off;
  for (int32_t i = 0; i < n_ops; ++i)
    if (i == 0 || op_node[order[(size_t)i]] != op_node[order[(size_t)i - 1]])
      seg_off.push_back(i);
  const int32_t n_seg = (int32_t)seg_off.size();
  seg_off.push_back(n_ops);
  if ((rc = activate(ctx))) return rc;
  const size_t C = (size_t)std::max(max_containers, 1);
  const size_t ops = (size_t)std::max(n_ops, 1);
  const size_t pods = (size_t)std::max(n_pods, 1);
  const size_t b_req = sizeof(int64_t) * pods * C * Q, b_mask = sizeof(uint32_t) * pods * C;
  const size_t b_nc = sizeof(int32_t) * pods, b_op = sizeof(int32_t) * ops;
  const size_t b_seg = sizeof(int32_t) * (size_t)(n_seg + 1);
  const size_t b_cpc = sizeof(int32_t) * ops * C;
  const size_t b_cards = sizeof(int32_t) * ops * (size_t)cards_stride;
  const size_t b_sel = cards_out ? ops * PAS_GAS_MAX_SELECTIONS : 1;
  const size_t b_cnt = (counts || counts_out) ? sizeof(int64_t) * ops * C * (size_t)K : 8;
  if ((rc = ensure_scratch(ctx, carve_size({b_req, b_mask, b_nc, b_op, b_op, b_op, b_seg, b_cpc,
                                            b_cards, b_op, b_op, b_sel, b_op, b_cnt}))))
    return rc;
  Carve cv{static_cast<char*>(ctx->scratch)};
  int64_t* d_req = cv.take<int64_t>(pods * C * Q);
  uint32_t* d_mask = cv.take<uint32_t>(pods * C);
  int32_t* d_nc = cv.take<int32_t>(pods);
  int32_t* d_pod = cv.take<int32_t>(ops);
  int32_t* d_node = cv.take<int32_t>(ops);
  int32_t* d_order = cv.take<int32_t>(ops);
  int32_t* d_seg = cv.take<int32_t>((size_t)n_seg + 1);
  int32_t* d_cpc = cv.take<int32_t>(ops * C);
  int32_t* d_cards = cv.take<int32_t>(ops * (size_t)cards_stride);
  uint32_t* d_res = cv.take<uint32_t>(ops);
  int32_t* d_status = cv.take<int32_t>(ops);
  uint8_t* d_sel = cv.take<uint8_t>(b_sel);
  int32_t* d_nsel = cv.take<int32_t>(ops);
  int64_t* d_cnt = cv.take<int64_t>(b_cnt / sizeof(int64_t));
  hipStream_t s = ctx->stream;
  if (n_ops > 0) {
    if (max_containers > 0 && n_pods > 0) {
      PAS_HIP(ctx, hipMemcpyAsync(d_req, req, sizeof(int64_t) * n_pods * max_containers * Q,
                                  hipMemcpyHostToDevice, s));
      PAS_HIP(ctx, hipMemcpyAsync(d_mask, req_mask, sizeof(uint32_t) * n_pods * max_containers,
                                  hipMemcpyHostToDevice, s));
    }
    PAS_HIP(ctx, hipMemcpyAsync(d_nc, n_containers, sizeof(int32_t) * n_pods,
                                hipMemcpyHostToDevice, s));
    PAS_HIP(ctx, hipMemcpyAsync(d_pod, op_pod, b_op, hipMemcpyHostToDevice, s));
    PAS_HIP(ctx, hipMemcpyAsync(d_node, op_node, b_op, hipMemcpyHostToDevice, s));
    PAS_HIP(ctx, hipMemcpyAsync(d_order, order.data(), b_op, hipMemcpyHostToDevice, s));
    PAS_HIP(ctx, hipMemcpyAsync(d_seg, seg_off.data(), b_seg, hipMemcpyHostToDevice, s));
    if (release && counts) {
      if (max_containers > 0 && K > 0)
        PAS_HIP(ctx, hipMemcpyAsync(d_cnt, counts, b_cnt, hipMemcpyHostToDevice, s));
    } else if (release) {
      if (max_containers > 0)
        PAS_HIP(ctx, hipMemcpyAsync(d_cpc, cpc, sizeof(int32_t) * n_ops * max_containers,
                                    hipMemcpyHostToDevice, s));
      PAS_HIP(ctx, hipMemcpyAsync(d_cards, cards, b_cards, hipMemcpyHostToDevice, s));
    }
    if ((rc = gas_commit_launch(ctx, release, n_seg, max_containers, i915_index, d_order, d_seg,
                                d_pod, d_node, d_req, d_mask, d_nc, d_cpc, d_cards,
                                cards_stride, d_res, d_status, cards_out ? d_sel : nullptr,
                                cards_out ? d_nsel : nullptr, counts_out ? d_cnt : nullptr,
                                counts ? d_cnt : nullptr, s)))
      return rc;
    if (!release)
      PAS_HIP(ctx, hipMemcpyAsync(res_out, d_res, b_op, hipMemcpyDeviceToHost, s));
    if (counts_out && max_containers > 0 && K > 0)
      PAS_HIP(ctx, hipMemcpyAsync(counts_out, d_cnt, b_cnt, hipMemcpyDeviceToHost, s));
    if (cards_out) {
      PAS_HIP(ctx, hipMemcpyAsync(cards_out, d_sel, b_sel, hipMemcpyDeviceToHost, s));
      PAS_HIP(ctx, hipMemcpyAsync(nsel_out, d_nsel, b_op, hipMemcpyDeviceToHost, s));
    }
    PAS_HIP(ctx, hipMemcpyAsync(status_out, d_status, b_op, hipMemcpyDeviceToHost, s));
  }
  PAS_HIP(ctx, hipStreamSynchronize(s));
  ctx->gas.gen = gen_to;
  ++ctx->gas.epoch;
  return PAS_OK;
}

int pas_gas_bind(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_binds,
                 const int32_t* bind_pod, const int32_t* bind_node, int32_t n_pods,
                 int32_t max_containers, int32_t i915_index, const int64_t* req,
                 const uint32_t* req_mask, const int32_t* n_containers, uint32_t* res_out,
                 int32_t* status_out) {
  return gas_commit(ctx, false, gen_from, gen_to, n_binds, bind_pod, bind_node, n_pods,
                    max_containers, i915_index, req, req_mask, n_containers, nullptr, nullptr,
                    PAS_GAS_PACKED, res_out, status_out, nullptr, nullptr, nullptr, nullptr,
                    "pas_gas_bind");
}

int pas_gas_bind_ex(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_binds,
                    const int32_t* bind_pod, const int32_t* bind_node, int32_t n_pods,
                    int32_t max_containers, int32_t i915_index, const int64_t* req,
                    const uint32_t* req_mask, const int32_t* n_containers, uint32_t* res_out,
                    int32_t* status_out, uint8_t* cards_out, int32_t* n_sel_out) {
  if (!ctx) return PAS_EINVAL;
  if (n_binds > 0 && (!cards_out || !n_sel_out))
    return set_error(ctx, PAS_EINVAL, "pas_gas_bind_ex: null input");
  return gas_commit(ctx, false, gen_from, gen_to, n_binds, bind_pod, bind_node, n_pods,
                    max_containers, i915_index, req, req_mask, n_containers, nullptr, nullptr,
                    PAS_GAS_PACKED, res_out, status_out, n_binds > 0 ? cards_out : nullptr,
                    n_sel_out, nullptr, nullptr, "pas_gas_bind_ex");
}

int pas_gas_bind_counts(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_binds,
                        const int32_t* bind_pod, const int32_t* bind_node, int32_t n_pods,
                        int32_t max_containers, int32_t i915_index, const int64_t* req,
                        const uint32_t* req_mask, const int32_t* n_containers,
                        uint32_t* res_out, int32_t* status_out, int64_t* counts_out) {
  if (!ctx) return PAS_EINVAL;
  if (n_binds > 0 && max_containers > 0 && !counts_out)
    return set_error(ctx, PAS_EINVAL, "pas_gas_bind_counts: null input");
  return gas_commit(ctx, false, gen_from, gen_to, n_binds, bind_pod, bind_node, n_pods,
                    max_containers, i915_index, req, req_mask, n_containers, nullptr, nullptr,
                    PAS_GAS_PACKED, res_out, status_out, nullptr, nullptr,
                    n_binds > 0 && max_containers > 0 ? counts_out : nullptr, nullptr,
                    "pas_gas_bind_counts");
}

int pas_gas_release(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_releases,
                    const int32_t* rel_pod, const int32_t* rel_node, int32_t n_pods,
                    int32_t max_containers, const int64_t* req, const uint32_t* req_mask,
                    const int32_t* n_containers, const int32_t* cards_per_container,
                    const int32_t* cards, int32_t* status_out) {
  return gas_commit(ctx, true, gen_from, gen_to, n_releases, rel_pod, rel_node, n_pods,
                    max_containers, -1, req, req_mask, n_containers, cards_per_container, cards,
                    PAS_GAS_PACKED, nullptr, status_out, nullptr, nullptr, nullptr, nullptr,
                    "pas_gas_release");
}

int pas_gas_release_ex(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to, int32_t n_releases,
                       const int32_t* rel_pod, const int32_t* rel_node, int32_t n_pods,
                       int32_t max_containers, const int64_t* req, const uint32_t* req_mask,
                       const int32_t* n_containers, const int32_t* cards_per_container,
                       const int32_t* cards, int32_t* status_out) {
  return gas_commit(ctx, true, gen_from, gen_to, n_releases, rel_pod, rel_node, n_pods,
                    max_containers, -1, req, req_mask, n_containers, cards_per_container, cards,
                    PAS_GAS_MAX_SELECTIONS, nullptr, status_out, nullptr, nullptr, nullptr,
                    nullptr, "pas_gas_release_ex");
}

int pas_gas_release_counts(pas_ctx* ctx, uint64_t gen_from, uint64_t gen_to,
                           int32_t n_releases, const int32_t* rel_pod, const int32_t* rel_node,
                           int32_t n_pods, int32_t max_containers, const int64_t* req,
                           const uint32_t* req_mask, const int32_t* n_containers,
                           const int64_t* counts, int32_t* status_out) {
  if (!ctx) return PAS_EINVAL;
  if (n_releases > 0 && max_containers > 0 && !counts)
    return set_error(ctx, PAS_EINVAL, "pas_gas_release_counts: null input");
  static const int64_t kNone = 0;  // no containers: nothing to read
  return gas_commit(ctx, true, gen_from, gen_to, n_releases, rel_pod, rel_node, n_pods,
                    max_containers, -1, req, req_mask, n_containers, nullptr, nullptr, 1,
                    nullptr, status_out, nullptr, nullptr, nullptr, counts ? counts : &kNone,
                    "pas_gas_release_counts");
}

int pas_gas_snapshot_get(pas_ctx* ctx, uint64_t* gen, int64_t* used_out) {
  if (!ctx) return PAS_EINVAL;
  if (!ctx->gas.valid) return set_error(ctx, PAS_ENOSNAP, "no GAS snapshot uploaded");
  const GasSnapshot& g = ctx->gas;
  const size_t b = sizeof(int64_t) * (size_t)g.n_nodes * g.max_cards * g.n_res;
  if (b && !used_out) return set_error(ctx, PAS_EINVAL, "pas_gas_snapshot_get: null output");
  int rc = activate(ctx);
  if (rc) return rc;
  if (b) PAS_HIP(ctx, hipMemcpyAsync(used_out, g.used, b, hipMemcpyDeviceToHost, ctx->stream));
  PAS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (gen) *gen = g.gen;
  return PAS_OK;
}

// Host path of pas_gas_fit / pas_gas_fit_ex: validates, uploads the batch, runs the fit and
// copies the words (and side records) back.
static int gas_fit_host(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                        int32_t i915_index, const int64_t* req, const uint32_t* req_mask,
                        const int32_t* n_containers, uint32_t* res_out,
                        pas_gas_selection* side, int64_t side_cap, int64_t* side_count,
                        const char* fn) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_gas_gen(ctx, gen);
  if (rc) return rc;
  const int32_t Q = ctx->gas.n_res;
  if (n_pods < 0 || max_containers < 0 || i915_index >= Q || i915_index < -1 || side_cap < 0)
    return set_error(ctx, PAS_EINVAL, std::string(fn) + ": bad shape");
  if (side_count) *side_count = 0;
  if (n_pods == 0) return PAS_OK;
  if (!n_containers || !res_out || (max_containers > 0 && (!req || !req_mask)) ||
      (side_cap > 0 && !side))
    return set_error(ctx, PAS_EINVAL, std::string(fn) + ": null input");
  // Validate the batch (no limit on card selections: see PAS_GAS_SEL_LIMIT)
  for (int32_t p = 0; p < n_pods; ++p) {
    if (n_containers[p] < 0 || n_containers[p] > max_containers)
      return set_error(ctx, PAS_EINVAL, std::string(fn) + ": n_containers out of range");
    for (int32_t c = 0; c < n_containers[p]; ++c) {
      const int64_t b = (int64_t)p * max_containers + c;
      if ((req_mask[b] & ~PAS_REQ_UNKNOWN_KIND) >> Q) return set_error(ctx, PAS_EINVAL, std::string(fn) + ": mask bit >= n_res");
    }
  }
  if ((rc = activate(ctx))) return rc;
  const int64_t N = ctx->gas.n_nodes;
  const size_t C = (size_t)std::max(max_containers, 1);
  const size_t b_req = sizeof(int64_t) * (size_t)n_pods * C * Q;
  const size_t b_mask = sizeof(uint32_t) * (size_t)n_pods * C;
  const size_t b_nc = sizeof(int32_t) * (size_t)n_pods;
  const size_t b_res = sizeof(uint32_t) * (size_t)n_pods * (size_t)N;
  const size_t b_side = sizeof(pas_gas_selection) * (size_t)side_cap;
  if ((rc = ensure_scratch(ctx, carve_size({b_req, b_mask, b_nc, b_res, b_side, 8})))) return rc;
  Carve cv{static_cast<char*>(ctx->scratch)};
  int64_t* d_req = cv.take<int64_t>((size_t)n_pods * C * Q);
  uint32_t* d_mask = cv.take<uint32_t>((size_t)n_pods * C);
  int32_t* d_nc = cv.take<int32_t>(n_pods);
  uint32_t* d_res = cv.take<uint32_t>((size_t)n_pods * N);
  pas_gas_selection* d_side = cv.take<pas_gas_selection>((size_t)side_cap);
  int64_t* d_count = cv.take<int64_t>(1);
  hipStream_t s = ctx->stream;
  if (max_containers > 0) {
    PAS_HIP(ctx, hipMemcpyAsync(d_req, req, b_req, hipMemcpyHostToDevice, s));
    PAS_HIP(ctx, hipMemcpyAsync(d_mask, req_mask, b_mask, hipMemcpyHostToDevice, s));
  }
  PAS_HIP(ctx, hipMemcpyAsync(d_nc, n_containers, b_nc, hipMemcpyHostToDevice, s));
  rc = gas_fit_launch(ctx, n_pods, max_containers, i915_index, d_req, d_mask, d_nc, d_res, N,
                      nullptr, side_cap > 0 ? d_side : nullptr, side_cap,
                      side_count ? d_count : nullptr, s);
  if (rc) return rc;
  if (b_res) PAS_HIP(ctx, hipMemcpyAsync(res_out, d_res, b_res, hipMemcpyDeviceToHost, s));
  int64_t count = 0;
  if (side_count)
    PAS_HIP(ctx, hipMemcpyAsync(&count, d_count, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  PAS_HIP(ctx, hipStreamSynchronize(s));
  // a side-stream wait of this fit that gave up: its words are incomplete
  if ((rc = gas_fault_check(ctx))) return rc;
  if (side_count) {
    *side_count = count;
    const int64_t got = std::min(count, side_cap);
    if (got > 0)
      PAS_HIP(ctx, hipMemcpy(side, d_side, sizeof(pas_gas_selection) * (size_t)got,
                             hipMemcpyDeviceToHost));
  }
  return PAS_OK;
}

int pas_gas_fit(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                int32_t i915_index, const int64_t* req, const uint32_t* req_mask,
                const int32_t* n_containers, uint32_t* res_out) {
  return gas_fit_host(ctx, gen, n_pods, max_containers, i915_index, req, req_mask, n_containers,
                      res_out, nullptr, 0, nullptr, "pas_gas_fit");
}

int pas_gas_fit_ex(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                   int32_t i915_index, const int64_t* req, const uint32_t* req_mask,
                   const int32_t* n_containers, uint32_t* res_out, pas_gas_selection* side,
                   int64_t side_cap, int64_t* side_count) {
  if (!ctx) return PAS_EINVAL;
  if (!side_count) return set_error(ctx, PAS_EINVAL, "pas_gas_fit_ex: null side_count");
  return gas_fit_host(ctx, gen, n_pods, max_containers, i915_index, req, req_mask, n_containers,
                      res_out, side, side_cap, side_count, "pas_gas_fit_ex");
}

static int gas_fit_device_common(pas_ctx* ctx, uint64_t gen, int32_t n_pods,
                                 int32_t max_containers, int32_t i915_index,
                                 const int64_t* d_req, const uint32_t* d_req_mask,
                                 const int32_t* d_n_containers, uint32_t* d_res_out,
                                 int64_t ld_res, uint64_t* d_fit_out, pas_gas_selection* d_side,
                                 int64_t side_cap, int64_t* d_side_count, void* hip_stream,
                                 const char* fn) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_gas_gen(ctx, gen);
  if (rc) return rc;
  if (ld_res < 0) ld_res = ctx->gas.n_nodes;  // dense rows
  if (n_pods < 0 || max_containers < 0 || i915_index >= ctx->gas.n_res || i915_index < -1 ||
      side_cap < 0 || ld_res < ctx->gas.n_nodes)
    return set_error(ctx, PAS_EINVAL, std::string(fn) + ": bad shape");
  if (n_pods > 0 && (!d_n_containers || (!d_res_out && !d_fit_out) ||
                     (max_containers > 0 && (!d_req || !d_req_mask)) || (side_cap > 0 && !d_side)))
    return set_error(ctx, PAS_EINVAL, std::string(fn) + ": null input");
  if ((rc = activate(ctx))) return rc;
  return gas_fit_launch(ctx, n_pods, max_containers, i915_index, d_req, d_req_mask,
                        d_n_containers, d_res_out, ld_res, d_fit_out,
                        side_cap > 0 ? d_side : nullptr, side_cap, d_side_count,
                        pick_stream(ctx, hip_stream));
}

int pas_gas_fit_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                       int32_t i915_index, const int64_t* d_req, const uint32_t* d_req_mask,
                       const int32_t* d_n_containers, uint32_t* d_res_out, void* hip_stream) {
  if (ctx && !d_res_out && n_pods > 0)
    return set_error(ctx, PAS_EINVAL, "pas_gas_fit_device: null input");
  return gas_fit_device_common(ctx, gen, n_pods, max_containers, i915_index, d_req, d_req_mask,
                               d_n_containers, d_res_out, -1, nullptr, nullptr, 0, nullptr,
                               hip_stream, "pas_gas_fit_device");
}

int pas_gas_fit_ex_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                          int32_t i915_index, const int64_t* d_req, const uint32_t* d_req_mask,
                          const int32_t* d_n_containers, uint32_t* d_res_out,
                          pas_gas_selection* d_side, int64_t side_cap, int64_t* d_side_count,
                          void* hip_stream) {
  if (ctx && ((!d_res_out && n_pods > 0) || !d_side_count))
    return set_error(ctx, PAS_EINVAL, "pas_gas_fit_ex_device: null input");
  return gas_fit_device_common(ctx, gen, n_pods, max_containers, i915_index, d_req, d_req_mask,
                               d_n_containers, d_res_out, -1, nullptr, d_side, side_cap,
                               d_side_count, hip_stream, "pas_gas_fit_ex_device");
}

int pas_gas_fit_ld_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                          int32_t i915_index, const int64_t* d_req, const uint32_t* d_req_mask,
                          const int32_t* d_n_containers, uint32_t* d_res_out, int64_t ld_res,
                          pas_gas_selection* d_side, int64_t side_cap, int64_t* d_side_count,
                          void* hip_stream) {
  if (ctx && !d_res_out && n_pods > 0)
    return set_error(ctx, PAS_EINVAL, "pas_gas_fit_ld_device: null input");
  if (ctx && ld_res < 0) return set_error(ctx, PAS_EINVAL, "pas_gas_fit_ld_device: ld_res < 0");
  return gas_fit_device_common(ctx, gen, n_pods, max_containers, i915_index, d_req, d_req_mask,
                               d_n_containers, d_res_out, ld_res, nullptr, d_side, side_cap,
                               d_side_count, hip_stream, "pas_gas_fit_ld_device");
}

int pas_gas_limit_count(pas_ctx* ctx, int64_t* n_pods_out) {
  if (!ctx) return PAS_EINVAL;
  if (!n_pods_out) return set_error(ctx, PAS_EINVAL, "pas_gas_limit_count: null output");
  *n_pods_out = 0;
  if (ctx->gas_last_slot < 0) return PAS_OK;  // no fit on this context yet
  const AuxSlot& a = ctx->aux_slot[ctx->gas_last_slot];
  int rc = activate(ctx);
  if (rc) return rc;
  PAS_HIP(ctx, hipEventSynchronize(a.ev));
  PAS_HIP(ctx, hipMemcpy(n_pods_out, a.gas_limit, sizeof(int64_t), hipMemcpyDeviceToHost));
  return PAS_OK;
}

int pas_gas_fit_bitmap_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t max_containers,
                              int32_t i915_index, const int64_t* d_req,
                              const uint32_t* d_req_mask, const int32_t* d_n_containers,
                              uint64_t* d_fit_out, void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_gas_gen(ctx, gen);
  if (rc) return rc;
  if (n_pods < 0 || max_containers < 0 || i915_index >= ctx->gas.n_res || i915_index < -1)
    return set_error(ctx, PAS_EINVAL, "pas_gas_fit_bitmap_device: bad shape");
  if (n_pods > 0 && !d_fit_out)
    return set_error(ctx, PAS_EINVAL, "pas_gas_fit_bitmap_device: null input");
  return gas_fit_device_common(ctx, gen, n_pods, max_containers, i915_index, d_req, d_req_mask,
                               d_n_containers, nullptr, -1, d_fit_out, nullptr, 0, nullptr,
                               hip_stream, "pas_gas_fit_bitmap_device");
}

// --------------------------------------------------------------------------- deschedule labels

static int check_label_plan(pas_ctx* ctx, int32_t n_nodes, int32_t n_strat, const void* viol,
                            const void* add, const void* rem, const void* total,
                            const char* fn) {
  if (n_nodes < 0 || n_strat < 0 || n_strat > 64)
    return set_error(ctx, PAS_EINVAL, std::string(fn) + ": bad shape (0 <= n_strat <= 64)");
  if (!total || (n_nodes > 0 && (!add || !rem || (n_strat > 0 && !viol))))
    return set_error(ctx, PAS_EINVAL, std::string(fn) + ": null argument");
  return PAS_OK;
}

int pas_tas_label_plan(pas_ctx* ctx, int32_t n_nodes, int32_t n_strat, const uint64_t* viol,
                       const int32_t* name_id, const uint64_t* labels, uint64_t* add_out,
                       uint64_t* remove_out, int64_t* total_out) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_label_plan(ctx, n_nodes, n_strat, viol, add_out, remove_out, total_out,
                            "pas_tas_label_plan");
  if (rc) return rc;
  if ((rc = activate(ctx))) return rc;
  const size_t W = ((size_t)n_nodes + 63) / 64;
  const size_t b_bits = sizeof(uint64_t) * (size_t)n_strat * W;
  const size_t b_mask = sizeof(uint64_t) * (size_t)n_nodes;
  if ((rc = ensure_scratch(ctx, carve_size({b_bits, b_bits, b_mask, b_mask, sizeof(int64_t)}))))
    return rc;
  Carve cv{static_cast<char*>(ctx->scratch)};
  uint64_t* d_viol = cv.take<uint64_t>((size_t)n_strat * W);
  uint64_t* d_labels = cv.take<uint64_t>((size_t)n_strat * W);
  uint64_t* d_add = cv.take<uint64_t>(n_nodes);
  uint64_t* d_rem = cv.take<uint64_t>(n_nodes);
  int64_t* d_total = cv.take<int64_t>(1);
  hipStream_t s = ctx->stream;
  if (b_bits) {
    PAS_HIP(ctx, hipMemcpyAsync(d_viol, viol, b_bits, hipMemcpyHostToDevice, s));
    if (labels) PAS_HIP(ctx, hipMemcpyAsync(d_labels, labels, b_bits, hipMemcpyHostToDevice, s));
  }
  rc = label_plan_launch(ctx, n_nodes, n_strat, make_name_plan(n_strat, name_id), d_viol,
                         labels ? d_labels : nullptr, d_add, d_rem, d_total, s);
  if (rc) return rc;
  if (b_mask) {
    PAS_HIP(ctx, hipMemcpyAsync(add_out, d_add, b_mask, hipMemcpyDeviceToHost, s));
    PAS_HIP(ctx, hipMemcpyAsync(remove_out, d_rem, b_mask, hipMemcpyDeviceToHost, s));
  }
  PAS_HIP(ctx, hipMemcpyAsync(total_out, d_total, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  PAS_HIP(ctx, hipStreamSynchronize(s));
  return PAS_OK;
}

int pas_tas_label_plan_device(pas_ctx* ctx, int32_t n_nodes, int32_t n_strat,
                              const uint64_t* d_viol, const int32_t* name_id,
                              const uint64_t* d_labels, uint64_t* d_add_out,
                              uint64_t* d_remove_out, int64_t* d_total_out, void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_label_plan(ctx, n_nodes, n_strat, d_viol, d_add_out, d_remove_out,
                            d_total_out, "pas_tas_label_plan_device");
  if (rc) return rc;
  if ((rc = activate(ctx))) return rc;
  return label_plan_launch(ctx, n_nodes, n_strat, make_name_plan(n_strat, name_id), d_viol,
                           d_labels, d_add_out, d_remove_out, d_total_out,
                           pick_stream(ctx, hip_stream));
}

int pas_tas_deschedule_device(pas_ctx* ctx, uint64_t gen, int32_t n_strategies,
                              int32_t n_rules, const pas_rule* d_rules,
                              const int32_t* d_rule_off, uint64_t* d_viol_out,
                              const int32_t* name_id, const uint64_t* d_labels,
                              uint64_t* d_add_out, uint64_t* d_remove_out, int64_t* d_total_out,
                              void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_tas_gen(ctx, gen);
  if (rc) return rc;
  if (n_rules < 0) return set_error(ctx, PAS_EINVAL, "negative count");
  if ((rc = check_label_plan(ctx, ctx->tas.n_nodes, n_strategies, d_viol_out, d_add_out,
                             d_remove_out, d_total_out, "pas_tas_deschedule_device")))
    return rc;
  if (n_strategies > 0 && (!d_rule_off || (n_rules > 0 && !d_rules)))
    return set_error(ctx, PAS_EINVAL, "pas_tas_deschedule_device: null input");
  if ((rc = activate(ctx))) return rc;
  return tas_deschedule_launch(ctx, n_strategies, n_rules, d_rules, d_rule_off, d_viol_out,
                               make_name_plan(n_strategies, name_id), d_labels, d_add_out,
                               d_remove_out, d_total_out, pick_stream(ctx, hip_stream));
}

// --------------------------------------------------------------------------- node shards

int pas_tas_topk_device(pas_ctx* ctx, uint64_t gen, int32_t n_pods, int32_t n_rules,
                        const pas_rule* d_rules, const int32_t* d_rule_off,
                        const pas_rule* d_prio, const uint64_t* d_cand, int32_t k,
                        int32_t node_base, int64_t* d_top_key, int32_t* d_top_node,
                        int32_t* d_top_len, void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_tas_gen(ctx, gen);
  if (rc) return rc;
  if (n_pods < 0 || n_rules < 0 || k < 1 || node_base < 0)
    return set_error(ctx, PAS_EINVAL, "pas_tas_topk_device: bad shape");
  if ((int64_t)node_base + ctx->tas.n_nodes > INT32_MAX)
    return set_error(ctx, PAS_EINVAL, "pas_tas_topk_device: node ids past int32");
  if (n_pods == 0) return PAS_OK;
  if (!d_rule_off || !d_prio || (n_rules > 0 && !d_rules) || !d_top_key || !d_top_node ||
      !d_top_len)
    return set_error(ctx, PAS_EINVAL, "pas_tas_topk_device: null argument");
  if ((rc = activate(ctx))) return rc;
  return tas_topk_launch(ctx, n_pods, n_rules, d_rules, d_rule_off, d_prio, d_cand, k,
                         node_base, d_top_key, d_top_node, d_top_len,
                         pick_stream(ctx, hip_stream));
}

int pas_tas_gas_topk_device(pas_ctx* ctx, uint64_t tas_gen, uint64_t gas_gen, int32_t n_pods,
                            int32_t n_rules, const pas_rule* d_rules, const int32_t* d_rule_off,
                            const pas_rule* d_prio, const uint64_t* d_cand,
                            int32_t max_containers, int32_t i915_index, const int64_t* d_req,
                            const uint32_t* d_req_mask, const int32_t* d_n_containers,
                            int32_t k, int32_t node_base, int64_t* d_top_key,
                            int32_t* d_top_node, int32_t* d_top_len, void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  int rc = check_tas_gen(ctx, tas_gen);
  if (rc) return rc;
  if ((rc = check_gas_gen(ctx, gas_gen))) return rc;
  if (ctx->gas.n_nodes != ctx->tas.n_nodes)
    return set_error(ctx, PAS_EINVAL, "pas_tas_gas_topk_device: TAS and GAS snapshots differ "
                                      "in node count");
  if (n_pods < 0 || n_rules < 0 || k < 1 || node_base < 0 || max_containers < 0 ||
      i915_index >= ctx->gas.n_res || i915_index < -1)
    return set_error(ctx, PAS_EINVAL, "pas_tas_gas_topk_device: bad shape");
  if ((int64_t)node_base + ctx->tas.n_nodes > INT32_MAX)
    return set_error(ctx, PAS_EINVAL, "pas_tas_gas_topk_device: node ids past int32");
  if (n_pods == 0) return PAS_OK;
  if (!d_rule_off || !d_prio || (n_rules > 0 && !d_rules) || !d_top_key || !d_top_node ||
      !d_top_len || !d_n_containers || (max_containers > 0 && (!d_req || !d_req_mask)))
    return set_error(ctx, PAS_EINVAL, "pas_tas_gas_topk_device: null argument");
  if ((rc = activate(ctx))) return rc;
  return tas_gas_topk_launch(ctx, n_pods, n_rules, d_rules, d_rule_off, d_prio, d_cand, max_containers,
                             i915_index, d_req, d_req_mask, d_n_containers, k, node_base,
                             d_top_key, d_top_node, d_top_len, pick_stream(ctx, hip_stream));
}

int pas_topk_merge_device(pas_ctx* ctx, int32_t n_pods, int32_t k, int32_t n_shards,
                          const int64_t* d_keys, const int32_t* d_nodes, int32_t* d_out_node,
                          int32_t* d_out_len, void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  if (n_pods < 0 || k < 1 || n_shards < 1)
    return set_error(ctx, PAS_EINVAL, "pas_topk_merge_device: bad shape");
  if (n_pods == 0) return PAS_OK;
  if (!d_keys || !d_nodes || !d_out_node || !d_out_len)
    return set_error(ctx, PAS_EINVAL, "pas_topk_merge_device: null argument");
  int rc = activate(ctx);
  if (rc) return rc;
  return topk_merge_launch(ctx, n_pods, k, n_shards, d_keys, d_nodes, d_out_node, d_out_len,
                           pick_stream(ctx, hip_stream));
}

int pas_list_merge_device(pas_ctx* ctx, int32_t n_pods, int32_t n_shards, int32_t width,
                          const int64_t* d_keys, const int32_t* d_nodes, int32_t* d_out_node,
                          int64_t out_ld, int32_t* d_out_len, void* hip_stream) {
  if (!ctx) return PAS_EINVAL;
  if (n_pods < 0 || n_shards < 1 || n_shards > 4096 || width < 1 ||
      out_ld < (int64_t)n_shards * width || (int64_t)n_shards * width > INT32_MAX)
    return set_error(ctx, PAS_EINVAL, "pas_list_merge_device: bad shape");
  if (n_pods == 0) return PAS_OK;
  if (!d_keys || !d_nodes || !d_out_node || !d_out_len)
    return set_error(ctx, PAS_EINVAL, "pas_list_merge_device: null argument");
  int rc = activate(ctx);
  if (rc) return rc;
  return list_merge_launch(ctx, n_pods, n_shards, width, d_keys, d_nodes, d_out_node, out_ld,
                           d_out_len, pick_stream(ctx, hip_stream));
}

// --------------------------------------------------------------------------- timing

int pas_set_timing(pas_ctx* ctx, int enable) {
  if (!ctx) return PAS_EINVAL;
  if (enable < 0 || enable > PAS_TIMING_KERNELS)
    return set_error(ctx, PAS_EINVAL, "pas_set_timing: level must be 0, 1 or 2");
  ctx->timing = enable;
  return PAS_OK;
}

int pas_kernel_time(pas_ctx* ctx, int32_t kernel_id, double* total_ms, int64_t* launches) {
  if (!ctx || kernel_id < 0 || kernel_id >= PAS_K_COUNT) return PAS_EINVAL;
  resolve_timing(ctx);
  if (total_ms) *total_ms = ctx->total_ms[kernel_id];
  if (launches) *launches = ctx->launches[kernel_id];
  return PAS_OK;
}

int pas_reset_timing(pas_ctx* ctx) {
  if (!ctx) return PAS_EINVAL;
  resolve_timing(ctx);
  for (int i = 0; i < PAS_K_COUNT; ++i) {
    ctx->total_ms[i] = 0;
    ctx->launches[i] = 0;
  }
  return PAS_OK;
}

}  // extern "C"
