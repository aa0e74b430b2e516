// pas_internal.h — context and snapshot state shared by the HIP translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "pas.h"

namespace pas {

constexpr int kOrderAsc = 0;   // LessThan   (operator.go:38-39)
constexpr int kOrderDesc = 1;  // GreaterThan (operator.go:36-37)
constexpr int kOrderIndex = 2; // any other operator: no sort
constexpr int kNumOrders = 3;

inline int64_t w64(int64_t n) { return (n + 63) / 64; }
inline int64_t w32(int64_t n) { return (n + 31) / 32; }

// Order rows are padded to whole 1024-position segments plus one more segment, filled with
// a sentinel node id (see TasSnapshot), so that a segment load never needs a bound check.
constexpr int kOrderPad = 1024;
inline int64_t order_row(int64_t n) { return (n + kOrderPad - 1) / kOrderPad * kOrderPad + kOrderPad; }

// Data a call derives from the resident snapshot on its own stream (once per snapshot
// change) and later calls read, possibly on other streams: an event recorded after the build
// orders those calls after it (derived_wait).
struct DerivedSync {
  hipEvent_t ev = nullptr;
  hipStream_t stream = nullptr;
  bool valid = false;
};

// Device-resident TAS snapshot.  Layout in HBM (M metrics, N nodes, R = order_row(N)):
//   vals     int64 [M][N]      raw v_milli (deschedule sweep reads it directly)
//   present  uint64 [M][W64]
//   cnt      int32 [M]         nodes that have metric m
//   sorted   int64 [M][R]      ascending values of the present nodes (first cnt[m])
//   perm     int32 [3][M][R]   node ids in asc / desc / index order (first cnt[m]); the
//                              rest of each row holds the sentinel W64 * 64, a node id
//                              whose bit in the evaluator's LDS pass bitmap is always 0
//   f1k, f32 int64 [M][R/1024], [M][R/32]  every 1024th / 32nd sorted value (rule ranges
//                              are found in three coalesced rounds: tas_eval.hip)
struct TasSnapshot {
  bool valid = false;
  uint64_t gen = 0;
  int32_t n_nodes = 0;
  int32_t n_metrics = 0;
  int32_t row = 0;  // R
  int64_t* vals = nullptr;
  uint64_t* present = nullptr;
  int32_t* cnt = nullptr;
  int64_t* sorted = nullptr;
  int32_t* perm = nullptr;
  int64_t* f1k = nullptr;  // [M][R / 1024] sorted[m][1024 a]: fences of the range search
  int64_t* f32 = nullptr;  // [M][R / 32]   sorted[m][32 b]
  // column m holds value * 10^scale[m]: scale_tab[m] = {10^scale, INT64_MAX / 10^scale}
  // (pas_tas_snapshot_set_scale; milli after every snapshot_set)
  int64_t* scale_tab = nullptr;
  // build scratch (kept for column updates): sort keys {value, row} and node ids, two
  // buffers each, [M][R]; per-word popcounts and their scan; the updated rows
  void* keys_a = nullptr;
  void* keys_b = nullptr;
  int32_t* ids_a = nullptr;
  int32_t* ids_b = nullptr;
  uint32_t* popc = nullptr;        // [M*W64 + 1]
  uint32_t* word_scan = nullptr;   // [M*W64 + 1]
  int32_t* rows = nullptr;         // [M]
  void* sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  void* scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;
  // node-major copies for per-node gathers (tas_gas_topk.hip), built by the first call that
  // needs them after a change: vals_t int64 [N][M], pres_t uint64 [N][ceil(M / 64)].
  // `epoch` counts snapshot changes, `t_epoch` is the epoch the copies were built at.
  uint64_t epoch = 1;
  uint64_t t_epoch = 0;
  int64_t* vals_t = nullptr;
  uint64_t* pres_t = nullptr;
  size_t t_bytes = 0;
  DerivedSync t_sync;  // the copies' build
};

// Device-resident GAS snapshot (node-major):
//   n_cards int32 [N], cap int64 [N][Q], used int64 [N][K][Q]
// core.EvaluateRule's CmpInt64 (operator.go:16-22) against column m's fixed point: the
// integer target * 10^scale[m] in *tm (0), or the saturation when that is past int64: +1 above
// every value, -1 below every value.  A column at scale 0 never saturates
// below: its values are ParseQuantity's, >= -(2^63 - 1).
__device__ __forceinline__ int target_scaled(int64_t t, const int64_t* __restrict__ scale_tab,
                                             int32_t m, int64_t* tm) {
  const int64_t mult = scale_tab[2 * m], maxq = scale_tab[2 * m + 1];
  if (t > maxq) return 1;
  if (t < -maxq) return -1;
  *tm = t * mult;
  return 0;
}

struct GasSnapshot {
  bool valid = false;
  uint64_t gen = 0;
  int32_t n_nodes = 0;
  int32_t max_cards = 0;
  int32_t n_res = 0;
  int32_t* n_cards = nullptr;
  int64_t* cap = nullptr;
  int64_t* used = nullptr;
  // per-snapshot values the fit derives (gas_fit.hip: flipped kind minima, nodes past the
  // fast kernels' card count), recomputed by the first fit after a change: `epoch` counts
  // changes of n_cards / cap / used, `derived_epoch` is the epoch they were computed at
  uint64_t epoch = 1;
  uint64_t derived_epoch = 0;
  void* derived = nullptr;  // gflip[4] u64 | n_big_nodes i32 (+pad) | big_nodes[N] i32
  // card-major free values of the first 8 cards, free_t[k][q][n] (gas_fit.hip), derived
  // with the above: the fit kernels' per-node loads are then coalesced
  void* free_t = nullptr;
  DerivedSync derived_sync;  // the derived values' build
};

// slot_buf buffers
enum SlotBuf {
  kBufGpass = 0,  // pass bitmaps of clusters past the LDS bitmap (tas_eval)
  kBufMerge = 1,  // cut list and ping-pong rows of the full-list merge (tas_list_merge.hip)
  kBufLabel = 2,  // per-workgroup partial counts of the label plan (tas_labels.hip)
  kSlotBufs = 3
};

// Per-call device scratch of the _device entry points (TAS rule ranges and pod descriptors,
// GAS lists, rank rows and list counts), one set per stream in use.  A call takes the slot of
// its stream (stream order protects it), else a free slot, else the least recently used one
// after waiting (hipStreamWaitEvent) for that slot's last call: calls on different streams
// never share scratch while they may run, and calls on two alternating streams (a pipeline
// of batches) run without waiting for each other.
struct AuxSlot {
  void* p = nullptr;  // aux: TAS ranges | desc | keys, or the GAS fit's lists and rank rows
  size_t bytes = 0;
  hipStream_t stream = nullptr;
  bool used = false;      // stream / ev are valid
  hipEvent_t ev = nullptr;  // recorded on `stream` after the slot's last call
  uint64_t last = 0;      // use clock (LRU)
  // the GAS fit's list counts, two sets: a fit uses one (zero) and its prep kernel zeroes the
  // other for the next fit on this slot (no fill launch per fit)
  int32_t* gas_counts = nullptr;
  int gas_counts_set = 0;
  int64_t* gas_limit = nullptr;  // pods of the slot's last GAS fit past PAS_GAS_MAX_SELECTIONS
  // the GAS fit's side streams (one-selection + generic kernels; sequential kernel), forked
  // from and joined to the caller's stream per fit, and their events (events mode)
  hipStream_t side = nullptr, side2 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr, join2 = nullptr;
  // device-side fork / join (gas_fit.hip): flags [prep done, side done, side2 done, abort,
  // prep started] each set to the fit's epoch (a per-slot count of fits); abort = the epoch of
  // a fit whose wait timed out (its fit kernels return at entry)
  uint32_t* gas_sync = nullptr;
  uint32_t gas_epoch = 0;
  // further per-stream buffers of the _device entry points (slot_buf), grown on demand
  void* buf[kSlotBufs] = {};
  size_t buf_bytes[kSlotBufs] = {};
};
constexpr int kAuxSlots = 4;

struct TimedLaunch {
  hipEvent_t start;
  hipEvent_t stop;
  int32_t kernel;
};

}  // namespace pas

struct pas_ctx {
  int device = 0;
  int n_cu = 256;  // compute units of the device (persistent grids)
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  pas::TasSnapshot tas;
  pas::GasSnapshot gas;
  // per-call scratch of the host-buffer entry points, which all run on ctx->stream and
  // synchronize it before they return (grown on demand; the _device entry points use the
  // per-stream AuxSlot buffers instead)
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  pas::AuxSlot aux_slot[pas::kAuxSlots];
  uint64_t aux_clock = 0;
  int gas_last_slot = -1;  // aux slot of the last GAS fit (pas_gas_limit_count)
  // the GAS fit's fork / join of its side streams: -1 unresolved, 0 events, 1 device flags
  // (gas_fit.hip gas_sync_mode), and the flags' sticky timeout report (host-pinned, written
  // by a wait kernel that gave up)
  int gas_sync_mode = -1;
  uint32_t* gas_sync_fault = nullptr;
  int gas_force_timeouts = 0;  // PAS_GAS_FORCE_TIMEOUT: the next n flag-mode fits time out
  // timing
  int timing = 0;  // 0 off, PAS_TIMING_SPAN, PAS_TIMING_KERNELS (pas_set_timing)
  std::vector<pas::TimedLaunch> pending;
  std::vector<hipEvent_t> event_pool;
  double total_ms[PAS_K_COUNT] = {};
  int64_t launches[PAS_K_COUNT] = {};
};

namespace pas {

int set_error(pas_ctx* ctx, int code, const std::string& msg);
int check_hip(pas_ctx* ctx, hipError_t e, const char* what);
#define PAS_HIP(ctx, expr)                                       \
  do {                                                           \
    hipError_t _e = (expr);                                      \
    if (_e != hipSuccess) return ::pas::check_hip(ctx, _e, #expr); \
  } while (0)

int ensure_scratch(pas_ctx* ctx, size_t bytes);
// After building snapshot-derived data on s / before reading it on s.
int derived_built(pas_ctx* ctx, DerivedSync& d, hipStream_t s);
int derived_wait(pas_ctx* ctx, const DerivedSync& d, hipStream_t s);
// The aux slot for a call on stream s with at least `bytes` of aux (ordered after the slot's
// previous user when that ran on another stream), and its release after the call's launches
// (records the slot's event on s).  nullptr on error (ctx->err set, *rc the status).
AuxSlot* aux_acquire(pas_ctx* ctx, hipStream_t s, size_t bytes, int* rc);
void aux_release(pas_ctx* ctx, AuxSlot* slot, hipStream_t s);
// Buffer `which` (SlotBuf) of an acquired slot, at least `bytes`: grown after the slot's
// earlier calls (ordered before s by aux_acquire) have finished.  nullptr on error (*rc).
void* slot_buf(pas_ctx* ctx, AuxSlot* slot, int which, size_t bytes, hipStream_t s, int* rc);
// aux_acquire + aux_release around a scope (every exit records the slot's event on s).
struct SlotScope {
  pas_ctx* ctx;
  AuxSlot* slot;
  hipStream_t s;
  SlotScope(pas_ctx* c, hipStream_t st, size_t bytes, int* rc)
      : ctx(c), slot(aux_acquire(c, st, bytes, rc)), s(st) {}
  ~SlotScope() {
    if (slot) aux_release(ctx, slot, s);
  }
  SlotScope(const SlotScope&) = delete;
  SlotScope& operator=(const SlotScope&) = delete;
};
int activate(pas_ctx* ctx);  // hipSetDevice(ctx->device)
hipStream_t pick_stream(pas_ctx* ctx, void* s);

// Bracket a launch with timing events when ctx->timing is on.
void timing_begin(pas_ctx* ctx, hipStream_t s, int kernel, TimedLaunch* tl);
void timing_end(pas_ctx* ctx, hipStream_t s, TimedLaunch* tl);

void free_tas(pas_ctx* ctx);
void free_gas(pas_ctx* ctx);

// Per-translation-unit entry points used by the C-ABI layer.
int tas_snapshot_build(pas_ctx* ctx, uint64_t gen, int32_t n_nodes, int32_t n_metrics,
                       const int64_t* d_vals, const uint64_t* d_present, hipStream_t s);
// Replace metric columns cols[0..n_cols) (host array, distinct, < n_metrics) with
// d_vals [n_cols][N] / d_present [n_cols][W64] and rebuild their orders.
int tas_snapshot_update(pas_ctx* ctx, uint64_t gen, int32_t n_cols, const int32_t* cols,
                        const int64_t* d_vals, const uint64_t* d_present, hipStream_t s);
int tas_eval_launch(pas_ctx* ctx, int32_t n_pods, int32_t n_rules, const pas_rule* d_rules,
                    const int32_t* d_rule_off, const pas_rule* d_prio, const uint64_t* d_cand,
                    uint32_t flags, uint64_t* d_pass, int32_t* d_order, int32_t* d_len,
                    int32_t topk, hipStream_t s);
// Single-request prioritize (tas_request.hip): workspace bytes for n_req positions, and the
// launch (rule is host-side; ws = that many device bytes).
int prio_request_workspace(pas_ctx* ctx, int32_t n_req, size_t* bytes);  // status
int prio_request_launch(pas_ctx* ctx, const pas_rule& rule, int32_t n_req, const int32_t* d_req,
                        int32_t* d_pos, int32_t* d_len, void* ws, size_t ws_bytes,
                        hipStream_t s);
// (n_rules bounds the device rule_off: offsets are clamped into [0, n_rules], rule_span)
int tas_violations_launch(pas_ctx* ctx, int32_t n_strat, int32_t n_rules,
                          const pas_rule* d_rules, const int32_t* d_rule_off, uint64_t* d_viol,
                          hipStream_t s);
// A GAS fit whose side-stream wait timed out (device flags) reports here: after the fit's
// stream was synchronized, PAS_EDEVICE (and the side streams drained) if a wait gave up since
// the last report, else PAS_OK.
int gas_fault_check(pas_ctx* ctx);
int gas_fit_launch(pas_ctx* ctx, int32_t n_pods, int32_t max_containers, int32_t i915_index,
                   const int64_t* d_req, const uint32_t* d_req_mask,
                   const int32_t* d_n_containers, uint32_t* d_res, int64_t ld_res,
                   uint64_t* d_fit, pas_gas_selection* d_side, int64_t side_cap,
                   int64_t* d_side_count, hipStream_t s);
int tas_topk_launch(pas_ctx* ctx, int32_t n_pods, int32_t n_rules, const pas_rule* d_rules,
                    const int32_t* d_rule_off, const pas_rule* d_prio, const uint64_t* d_cand,
                    int32_t k, int32_t node_base, int64_t* d_key, int32_t* d_node,
                    int32_t* d_len, hipStream_t s);
// The eval prep's grouping alone: pods bucketed by prioritize order row (metric x asc / desc
// / index), desc[2 pos] = {pod, order * M + metric or -1, present count, 0},
// desc[2 pos + 1] = {rule_off[pod], rule_off[pod + 1], 0, 0}; keys [P] scratch.  With
// d_ranges, also every rule's range of the metric's ascending order (EvaluateRule, a3):
// ranges[r] = {first, end} positions of the nodes the rule selects.
int tas_group_launch(pas_ctx* ctx, int32_t n_pods, const pas_rule* d_prio,
                     const int32_t* d_rule_off, int4* d_desc, int2* d_keys, int32_t n_rules,
                     const pas_rule* d_rules, int2* d_ranges, hipStream_t s);
int tas_gas_topk_launch(pas_ctx* ctx, int32_t n_pods, int32_t n_rules, const pas_rule* d_rules,
                        const int32_t* d_rule_off, const pas_rule* d_prio,
                        const uint64_t* d_cand, int32_t max_containers, int32_t i915_index,
                        const int64_t* d_req, const uint32_t* d_req_mask,
                        const int32_t* d_n_containers, int32_t k, int32_t node_base,
                        int64_t* d_key, int32_t* d_node, int32_t* d_len, hipStream_t s);
int list_merge_launch(pas_ctx* ctx, int32_t n_pods, int32_t n_shards, int32_t width,
                      const int64_t* d_keys, const int32_t* d_nodes, int32_t* d_out_node,
                      int64_t out_ld, int32_t* d_out_len, hipStream_t s);
int topk_merge_launch(pas_ctx* ctx, int32_t n_pods, int32_t k, int32_t n_shards,
                      const int64_t* d_keys, const int32_t* d_nodes, int32_t* d_out_node,
                      int32_t* d_out_len, hipStream_t s);
// Bind (fit + commit, release = false) or release of operations grouped by node: order =
// operation indices sorted by node (stable), seg_off [n_seg + 1] the node segments.
int gas_commit_launch(pas_ctx* ctx, bool release, int32_t n_seg, int32_t max_containers,
                      int32_t i915_index, const int32_t* d_order, const int32_t* d_seg_off,
                      const int32_t* d_pod, const int32_t* d_node, const int64_t* d_req,
                      const uint32_t* d_mask, const int32_t* d_ncont, const int32_t* d_cpc,
                      const int32_t* d_cards, int32_t cards_stride, uint32_t* d_res,
                      int32_t* d_status, uint8_t* d_cards_out, int32_t* d_nsel_out,
                      int64_t* d_counts_out, const int64_t* d_counts, hipStream_t s);
// Policy names of the deschedule strategies (updateNodeLabels keys its non-violated set by
// name, deschedule/enforce.go:89-134).  A name is represented by its first strategy k
// (canonical); bit k of canon marks those.  Names held by one strategy are the bits of single;
// each name held by two or more strategies is a group: its member strategies and its k.  A
// node's violated names: (add & single) | {key[g] : add & group[g] != 0}.
struct NamePlan {
  uint64_t canon = 0;
  uint64_t single = 0;
  int32_t n_groups = 0;
  uint8_t key[32] = {};
  uint64_t group[32] = {};
};
// The plan of name_id[0 .. n_strat) (NULL = all distinct); n_strat <= 64.
NamePlan make_name_plan(int32_t n_strat, const int32_t* name_id);
__device__ __forceinline__ uint64_t violated_names(const NamePlan& np, uint64_t add) {
  uint64_t vn = add & np.single;
  for (int32_t g = 0; g < np.n_groups; ++g)
    vn |= (add & np.group[g]) ? 1ull << np.key[g] : 0ull;
  return vn;
}
int label_plan_launch(pas_ctx* ctx, int32_t n_nodes, int32_t n_strat, const NamePlan& names,
                      const uint64_t* d_viol, const uint64_t* d_labels, uint64_t* d_add,
                      uint64_t* d_rem, int64_t* d_total, hipStream_t s);
// totalViolations from per-block counts of violated pairs: *d_total = pairs - sum(d_part).
int label_total_launch(pas_ctx* ctx, int32_t n_parts, int64_t pairs, const int64_t* d_part,
                       int64_t* d_total, hipStream_t s);
// The deschedule sweep with the label plan fused in (pas_tas_deschedule_device): viol as
// tas_violations_launch, add / rem / total as label_plan_launch on those bitmaps.
int tas_deschedule_launch(pas_ctx* ctx, int32_t n_strat, int32_t n_rules,
                          const pas_rule* d_rules, const int32_t* d_rule_off, uint64_t* d_viol,
                          const NamePlan& names,
                          const uint64_t* d_labels, uint64_t* d_add, uint64_t* d_rem,
                          int64_t* d_total, hipStream_t s);

}  // namespace pas
