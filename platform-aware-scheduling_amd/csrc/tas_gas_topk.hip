// tas_gas_topk.hip — combined TAS + GAS per-pod top-k, evaluated along each pod's order.
//
// BASELINE configs[4]: per pending pod, the first k entries of the
// HostPriorityList over the nodes that pass the pod's dontschedule filter
// (dontschedule.Violated + filterNodes, telemetryscheduler.go:184-225) and fit its GPU
// request (GASExtender.filterNodes -> runSchedulingLogic, gpuscheduler/scheduler.go:280-338,
// 449-482), in prioritizeNodesForRule order (telemetryscheduler.go:128-149,
// operator.go:30-42), as merge records for the node-sharded top-k of tas_topk.hip.
//
// The composed path (pas_gas_fit_bitmap_device -> pas_tas_topk_device) evaluates every
// (pod, node): a fit bit for each of the shard's nodes and the pod's whole LDS pass bitmap,
// although only the first k passing nodes of the order are kept.  Here half a wave (32
// lanes) owns a pod and walks its order row (the snapshot's per-metric order,
// tas_snapshot.hip) 32 positions at a time: each lane evaluates its position's node directly
// — candidate bit, every dontschedule rule of the pod (EvaluateRule on the node's value),
// then the GAS first fit on the node's card usage (only for lanes still passing) — and the
// pod stops once k nodes are kept.  The result is the same list: the k first positions of
// the order whose node passes both filters.  With filter and fit rates near 1 (C5: ~0.93
// and ~0.97) a pod with k = 16 needs one round, 32 node evaluations instead of the shard's N.
//
// The node values come from node-major copies of the snapshot (vals_t [N][M], pres_t
// [N][M/64], built once per snapshot change): a lane's rules read its node's own row (the
// 16 metrics of a 128-byte line together) and one presence word, instead of one line per
// rule in the metric-major columns.  A pod's dontschedule rules are compiled once into LDS
// as value ranges (LazyRule) and read back per round as broadcast LDS reads.
//
// Records: key = order key of the node's value under the pod's operator (tas_topk.hip),
// node = global id (local + node_base); past len: key INT64_MAX, node INT32_MAX.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gas_runs.h"
#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;
constexpr int kWaves = kTpb / 64;
constexpr int kRuleBatch = 8;  // rule gathers in flight per lane
constexpr int kMaxRes = PAS_GAS_MAX_RES;

struct LazyTopkParams {
  int32_t n_pods, N, M, R, W64, k, node_base;
  const pas_rule* rules;
  const int32_t* rule_off;
  int32_t n_rules;  // bounds rule_off: a pod's span is clamped into [0, n_rules]
  const pas_rule* prio;
  const uint64_t* cand;  // [P][W64] or null (every node a candidate)
  const int32_t* perm;   // [3][M][R] snapshot orders
  const int32_t* cnt;    // [M]
  const int64_t* vals;   // [M][N]
  const int64_t* vals_t;    // [N][M]
  const uint64_t* pres_t;   // [N][WM]
  int32_t WM;
  const int64_t* sorted;  // [M][R] ascending present values; fences f1k [M][R/1024], f32
  const int64_t* f1k;
  const int64_t* f32;
  const int64_t* scale_tab;  // [M][2] the columns' fixed point (target_scaled)
  // GAS snapshot (same nodes) and the pods' requests
  int32_t K, Q, C, i915;
  const int32_t* n_cards;
  const int64_t* cap;
  const int64_t* used;
  const int64_t* req;     // [P][C][Q]
  const uint32_t* mask;   // [P][C]
  const int32_t* ncont;   // [P]
  int64_t* key_out;       // [P][k]
  int32_t* node_out;      // [P][k]
  int32_t* len_out;       // [P]
};


__device__ __forceinline__ int64_t order_key(int32_t op, int64_t v) {
  return op == PAS_OP_GREATER_THAN ? ~v : op == PAS_OP_LESS_THAN ? v : 0;
}

// checkResourceCapacity for one kind (scheduler.go:341-383): need >= 0, capacity > 0,
// used >= 0, used + need without overflow and within capacity.
__device__ __forceinline__ bool kind_fits(int64_t need, int64_t cap, int64_t used) {
  if (need < 0 || cap <= 0 || used < 0) return false;
  const int64_t sum = (int64_t)((uint64_t)used + (uint64_t)need);
  return sum >= 0 && cap >= sum;
}

// runSchedulingLogic (scheduler.go:280-338) of pod p on node n, the fit verdict only: a
// working copy of the node's card usage (readNodeResources, node_resource_cache.go:474-491),
// per container getPerGPUResourceRequest (:180-190) and numI915 selections (:192-198), each
// the first card in lexicographic order passing checkResourceCapacity, whose usage then
// takes the request (addRM).  KMAX: the snapshot's cards per node fit in registers
// (fully unrolled) for KMAX <= 16; the wide case keeps the copy in scratch.  QW: the kinds
// the copy holds (the snapshot's Q for KMAX <= 8, so C5's three kinds take 8 x 3 values, not
// 8 x 4; PAS_GAS_MAX_RES otherwise).
template <int KMAX, int QW>
__device__ bool lane_fit(const LazyTopkParams& a, int32_t p, int32_t n) {
  // every load of the node at once (card count, capacities, the usage of all its card slots):
  // predicating the usage loads on the card count would wait for that load first
  const int32_t nc = a.n_cards[n];
  constexpr int kUnroll = KMAX <= 16 ? KMAX : 1;
  const int32_t Q = a.Q, K = a.K;
  int64_t cap[kMaxRes];
  int64_t w[KMAX][QW];
#pragma unroll
  for (int q = 0; q < kMaxRes; ++q) cap[q] = q < Q ? a.cap[(int64_t)n * Q + q] : 0;
  if (Q == QW && ((KMAX * QW) & 1) == 0 && ((K * Q) & 1) == 0 && K <= KMAX) {
    // the node's usage row as 16-byte loads (half the load instructions; the row starts on
    // 16 bytes: an even number of values per node)
    typedef int64_t v2i64 __attribute__((ext_vector_type(2)));
    const v2i64* row = reinterpret_cast<const v2i64*>(a.used + (int64_t)n * K * Q);
    int64_t f[KMAX * QW];
#pragma unroll
    for (int i = 0; i < KMAX * QW / 2; ++i) {
      const v2i64 x = 2 * i < K * Q ? row[i] : v2i64{0, 0};
      f[2 * i] = x.x;
      f[2 * i + 1] = x.y;
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
#pragma unroll
      for (int q = 0; q < QW; ++q) w[k][q] = f[k * QW + q];
  } else {
#pragma unroll kUnroll
    for (int k = 0; k < KMAX; ++k)
#pragma unroll
      for (int q = 0; q < QW; ++q)
        w[k][q] = (k < K && q < Q) ? a.used[((int64_t)n * K + k) * Q + q] : 0;
  }
  if (nc <= 0) return false;  // FetchNode error / no cards label (:282-298)
  const int32_t ncard = min(nc, min(K, KMAX));
#pragma unroll kUnroll
  for (int k = 0; k < KMAX; ++k)
#pragma unroll
    for (int q = 0; q < QW; ++q) w[k][q] = k < ncard ? w[k][q] : 0;
  const int32_t nct = min(max(a.ncont[p], 0), a.C);  // (as gas_prep_kernel: within the rows)
  for (int32_t c = 0; c < nct; ++c) {
    const int64_t b = (int64_t)p * a.C + c;
    const uint32_t m = a.mask[b];
    if (m == 0u) continue;  // no GPU resources: no cards (:206-208)
    int64_t r[kMaxRes];
#pragma unroll
    for (int q = 0; q < kMaxRes; ++q) r[q] = q < Q ? a.req[b * Q + q] : 0;
    int64_t num = 0;  // getNumI915
    if (a.i915 >= 0 && ((m >> a.i915) & 1u) && r[a.i915] > 0) num = r[a.i915];
    if (num > 1)
#pragma unroll
      for (int q = 0; q < kMaxRes; ++q) r[q] /= num;
    if (num > kRunsFrom) {  // card runs (gas_runs.h)
      if (!container_runs<KMAX, QW>(Q, m, r, num, cap, w, ncard, [](int, int64_t) {}))
        return false;
      continue;
    }
    for (int64_t g = 0; g < num; ++g) {
      int chosen = -1;
#pragma unroll kUnroll
      for (int k = KMAX - 1; k >= 0; --k) {  // first fit = lowest k
        bool ok = k < ncard && !(m & PAS_REQ_UNKNOWN_KIND);  // (a key no capacity has)
#pragma unroll
        for (int q = 0; q < QW; ++q)
          if (q < Q && ((m >> q) & 1u)) ok = ok && kind_fits(r[q], cap[q], w[k][q]);
        chosen = ok ? k : chosen;
      }
      if (chosen < 0) return false;  // errWontFit (:249-253)
#pragma unroll kUnroll
      for (int k = 0; k < KMAX; ++k)
#pragma unroll
        for (int q = 0; q < QW; ++q)
          if (k == chosen && q < Q && ((m >> q) & 1u)) w[k][q] += r[q];
    }
  }
  return true;
}

// Positions [lb, ub) of value t (milli) in metric m's ascending column (c present values),
// found by the pod's 32 lanes in three rounds of loads, as the eval prep's range search does
// (tas_eval.hip ranges_group): the 1024-stride fences, the 32-stride fences of one block, the
// 32 values of one 32-block.  lb = values < t, ub = values <= t.
__device__ void half_bounds(const LazyTopkParams& a, int32_t m, int32_t c, int64_t t, int sub,
                            uint64_t half_mask, int32_t* lb, int32_t* ub) {
  const int64_t* sv = a.sorted + (int64_t)m * a.R;
  const int64_t* f1 = a.f1k + (int64_t)m * (a.R >> 10);
  const int64_t* f2 = a.f32 + (int64_t)m * (a.R >> 5);
  const int32_t na = (c + 1023) >> 10, nb = (c + 31) >> 5;
  int32_t cl = 0, cu = 0;
  for (int32_t i0 = 0; i0 < na; i0 += 8 * 32) {
    int64_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = f1[min(i0 + u * 32 + sub, max(na - 1, 0))];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool in = i0 + u * 32 + sub < na;
      cl += in && v[u] < t;
      cu += in && v[u] <= t;
    }
  }
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) {  // (xor within the half)
    cl += __shfl_xor(cl, off, 64);
    cu += __shfl_xor(cu, off, 64);
  }
  const int32_t n1l = cl, n1u = cu;
  const int32_t b1l = max(n1l - 1, 0), b1u = max(n1u - 1, 0);
  const int32_t e2l = n1l ? min(32, nb - b1l * 32) : 0, e2u = n1u ? min(32, nb - b1u * 32) : 0;
  const int64_t x2l = f2[b1l * 32 + min(sub, max(e2l - 1, 0))];
  const int64_t x2u = f2[b1u * 32 + min(sub, max(e2u - 1, 0))];
  const int32_t n2l = __popcll(__ballot(sub < e2l && x2l < t) & half_mask);
  const int32_t n2u = __popcll(__ballot(sub < e2u && x2u <= t) & half_mask);
  const int32_t b2l = b1l * 32 + max(n2l - 1, 0), b2u = b1u * 32 + max(n2u - 1, 0);
  const int32_t e3l = n1l ? min(32, c - b2l * 32) : 0, e3u = n1u ? min(32, c - b2u * 32) : 0;
  const int64_t x3l = sv[b2l * 32 + min(sub, max(e3l - 1, 0))];
  const int64_t x3u = sv[b2u * 32 + min(sub, max(e3u - 1, 0))];
  const int32_t n3l = __popcll(__ballot(sub < e3l && x3l < t) & half_mask);
  const int32_t n3u = __popcll(__ballot(sub < e3u && x3u <= t) & half_mask);
  *lb = n1l ? b2l * 32 + n3l : 0;
  *ub = n1u ? b2u * 32 + n3u : 0;
}

constexpr int kPodLanes = 32;                // lanes per pod (order positions per round)
constexpr int kPodsPerWave = 64 / kPodLanes;
constexpr int kPodsPerBlock = kWaves * kPodsPerWave;
constexpr int kStageRules = kPodLanes;       // rules of a pod compiled into LDS (one per lane)

// A dontschedule rule compiled once per pod: EvaluateRule (operator.go:13-26) on the node's
// value v (milli) as the range test  (uint64)(v - lo) <= span, with the saturating target
//  folded in: LessThan t -> [INT64_MIN, t*1000 - 1], GreaterThan t ->
// [t*1000 + 1, INT64_MAX], Equals t -> [t*1000, t*1000]; a target past the int64 milli range
// selects every value or none.  metric < 0: never evaluated (not cached, unknown operator, or
// a range that selects nothing).
struct alignas(16) LazyRule {
  int64_t lo;
  uint64_t span;
};

__device__ __forceinline__ void compile_rule(const pas_rule& ru, int32_t M,
                                             const int64_t* __restrict__ scale_tab,
                                             int32_t* metric, LazyRule* out) {
  int64_t tm = 0;
  const int sat = target_scaled(ru.target, scale_tab, (ru.metric >= 0 && ru.metric < M)
                                                          ? ru.metric : 0, &tm);
  int64_t lo = 0, hi = -1;  // empty
  if (ru.metric >= 0 && ru.metric < M) {
    if (ru.op == PAS_OP_LESS_THAN) {
      if (sat > 0) lo = INT64_MIN, hi = INT64_MAX;
      else if (sat == 0 && tm > INT64_MIN) lo = INT64_MIN, hi = tm - 1;
    } else if (ru.op == PAS_OP_GREATER_THAN) {
      if (sat < 0) lo = INT64_MIN, hi = INT64_MAX;
      else if (sat == 0 && tm < INT64_MAX) lo = tm + 1, hi = INT64_MAX;
    } else if (ru.op == PAS_OP_EQUALS) {
      if (sat == 0) lo = hi = tm;
    }
  }
  const bool live = lo <= hi;
  *metric = live ? ru.metric : -1;
  out->lo = lo;
  out->span = (uint64_t)hi - (uint64_t)lo;
}

// (at least 4 waves per SIMD for the register-resident shapes: the gathers need waves in
// flight)
template <int KMAX, int QW>
constexpr int topk_waves() { return KMAX <= 8 && QW <= 3 ? 4 : 1; }
template <int KMAX, int QW>
__global__ __launch_bounds__(kTpb) __attribute__((amdgpu_waves_per_eu(topk_waves<KMAX, QW>())))
void tas_gas_topk_kernel(LazyTopkParams a) {
  // the pods' compiled rules, kStageRules per pod (pods of at most that many rules)
  __shared__ LazyRule srule[kPodsPerBlock][kStageRules];
  __shared__ int32_t smetric[kPodsPerBlock][kStageRules];
  const int lane = threadIdx.x & 63;
  const int half = lane / kPodLanes, sub = lane % kPodLanes;
  // XCD-aware: blocks b and b + 8 share an XCD; each XCD takes a contiguous run of the
  // bucketed pod list (MI355X_MICROARCH.md)
  const int32_t nb = gridDim.x, b = blockIdx.x;
  const int32_t xcd = b & 7, per = nb >> 3, rem = nb & 7;
  const int32_t slot = xcd * per + min(xcd, rem) + (b >> 3);
  const int32_t pos = slot * kPodsPerBlock + (int32_t)(threadIdx.x >> 6) * kPodsPerWave + half;
  const uint64_t half_mask = half ? ~0ull << 32 : 0xFFFFFFFFull;
  const uint64_t below = half_mask & ((1ull << lane) - 1ull);
  const bool have = pos < a.n_pods;
  // the pod's descriptor (the eval prep's form): {pod, order row or -1, present count},
  // {first rule, end rule}; pods in index order (bucketing them by order row first, as the
  // eval prep does, was measured slower here: the one-block grouping of 64k pods costs more
  // than the L2 locality gains)
  int4 d0 = make_int4(0, -1, 0, 0), d1 = make_int4(0, 0, 0, 0);
  if (have) {
    const pas_rule q = a.prio[pos];
    const int32_t cq = (q.metric >= 0 && q.metric < a.M) ? a.cnt[q.metric] : 0;
    const int oq = q.op == PAS_OP_GREATER_THAN ? kOrderDesc
                   : q.op == PAS_OP_LESS_THAN  ? kOrderAsc
                                               : kOrderIndex;
    d0 = make_int4(pos, cq > 0 ? oq * a.M + q.metric : -1, cq, 0);
    // (clamped into [0, n_rules] and non-decreasing: a device rule_off that is not a CSR
    // never indexes past the rules, as the eval prep's rule_span)
    const int32_t r0 = min(max(a.rule_off[pos], 0), a.n_rules);
    d1 = make_int4(r0, min(max(a.rule_off[pos + 1], r0), a.n_rules), 0, 0);
  }
  const int32_t p = d0.x;
  const int32_t k = a.k;
  const pas_rule pr = a.prio[p];
  // bucket -1: no scheduling rule / metric not cached / no node has it: empty list
  // (telemetryscheduler.go:92-96); d0.z = the metric's present count
  const int32_t c0 = (have && d0.y >= 0) ? d0.z : 0;
  const int32_t r0 = d1.x, r1 = d1.y;
  // Rules on the prioritize metric itself select one contiguous range of a sorted order row
  // (EvaluateRule over the ascending column, a3): a pod whose rule excludes the top of its
  // own order (e.g. GreaterThan on the metric it prioritizes by GreaterThan) would walk
  // thousands of violating positions.  Such ranges (asc positions from the prep's search,
  // mirrored for the descending row) are jumped over at the start of each round; the rule
  // check per node still runs, so the skip only saves rounds.
  constexpr int kSkip = 4;
  int32_t slo[kSkip], shi[kSkip], ns = 0;
#pragma unroll
  for (int i = 0; i < kSkip; ++i) slo[i] = shi[i] = 0;
  const int ord = d0.y >= 0 ? d0.y / a.M : kOrderIndex;
  const bool sorted_row = c0 > 0 && ord != kOrderIndex;
  // The pod's rules are loaded one per lane (32 at a time, a single round trip) and only the
  // ones on the prioritize metric are walked, one per half at a time (a rule by rule scan
  // waited for a load per rule).
  for (int32_t rc = r0; __ballot(sorted_row && rc < r1); rc += kPodLanes) {
   const bool in_l = sorted_row && rc + sub < r1;
   const pas_rule ru_l = a.rules[in_l ? rc + sub : 0];
   const bool same_l = in_l && ru_l.metric == pr.metric && ru_l.op >= 0 && ru_l.op <= 2;
   const uint64_t sm = __ballot(same_l);
   uint32_t todo = (uint32_t)sm | (uint32_t)(sm >> 32);  // rule slots some half walks
   while (todo) {
    const int u = __builtin_ctz(todo);
    todo &= todo - 1;
    const int src = half * kPodLanes + u;  // this half's rule in slot u
    pas_rule ru;
    ru.metric = __shfl(ru_l.metric, src, 64);
    ru.op = __shfl(ru_l.op, src, 64);
    ru.target = __shfl(ru_l.target, src, 64);
    const bool same = (sm >> src) & 1ull;
    int64_t tm = 0;
    const int sat = target_scaled(ru.target, a.scale_tab, same ? pr.metric : 0, &tm);
    int32_t lb = 0, ub = 0;
    half_bounds(a, same ? pr.metric : 0, same ? c0 : 0, tm, sub, half_mask, &lb, &ub);
    if (sat != 0) lb = ub = sat > 0 ? c0 : 0;
    if (same) {
      // the rule's nodes in ascending positions, mirrored for the descending row
      const int32_t gx = ru.op == PAS_OP_LESS_THAN ? 0 : ru.op == PAS_OP_GREATER_THAN ? ub : lb;
      const int32_t gy = ru.op == PAS_OP_LESS_THAN ? lb : ru.op == PAS_OP_GREATER_THAN ? c0 : ub;
      const int32_t lo = ord == kOrderDesc ? c0 - gy : gx;
      const int32_t hi = ord == kOrderDesc ? c0 - gx : gy;
      if (hi > lo) {
#pragma unroll
        for (int i = 0; i < kSkip; ++i)
          if (i == ns) {
            slo[i] = lo;
            shi[i] = hi;
          }
        ns = min(ns + 1, kSkip);
      }
    }
   }
  }
  // Pods of at most kStageRules rules (every pod of the wave): each lane compiles one rule
  // of its pod into LDS, read back per round as broadcast LDS reads instead of a global load
  // per lane, rule and round.
  const int pslot = (int)(threadIdx.x >> 6) * kPodsPerWave + half;
  const bool staged = !__ballot(have && r1 - r0 > kStageRules);
  if (staged) {
    LazyRule cr{0, 0};
    int32_t cm = -1;
    if (have && r0 + sub < r1) compile_rule(a.rules[r0 + sub], a.M, a.scale_tab, &cm, &cr);
    srule[pslot][sub] = cr;
    smetric[pslot][sub] = cm;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  }
  const int32_t nr = have ? r1 - r0 : 0;
  const int32_t* row = a.perm + (int64_t)(d0.y >= 0 ? d0.y : 0) * a.R;
  const int64_t* mcol = a.vals + (int64_t)(d0.y >= 0 ? pr.metric : 0) * a.N;
  int64_t* keys = a.key_out + (int64_t)p * k;
  int32_t* nodes = a.node_out + (int64_t)p * k;
  int32_t kept = 0;
  for (int32_t j0 = 0;; j0 += kPodLanes) {
#pragma unroll
    for (int it = 0; it < kSkip; ++it)
#pragma unroll
      for (int i = 0; i < kSkip; ++i)
        if (i < ns && j0 >= slo[i] && j0 < shi[i]) j0 = shi[i];
    const bool active = j0 < c0 && kept < k;  // (uniform within the pod's half)
    if (!__ballot(active)) break;
    const int32_t j = j0 + sub;
    const bool valid = active && j < c0;
    const int32_t n = valid ? row[j] : 0;
    bool ok = valid;
    if (a.cand) ok = ok && ((a.cand[(int64_t)p * a.W64 + (n >> 6)] >> (n & 63)) & 1ull);
    // dontschedule.Violated (strategy.go:25-44) at this node: any rule whose metric the node
    // has and whose EvaluateRule holds; rules on metrics outside the cache or with an
    // unknown operator are skipped.  kRuleBatch rules' loads in flight at once.
    const int64_t* vrow = a.vals_t + (int64_t)n * a.M;
    const uint64_t* prow = a.pres_t + (int64_t)n * a.WM;
    bool viol = false;
    if (staged) {
      for (int32_t rb = 0; __ballot(ok && rb < nr); rb += kRuleBatch) {
        int32_t m[kRuleBatch];
        int64_t v[kRuleBatch];
        uint64_t pw[kRuleBatch];
#pragma unroll
        for (int u = 0; u < kRuleBatch; ++u) m[u] = smetric[pslot][min(rb + u, kStageRules - 1)];
        // (one presence word per node when the snapshot has at most 64 metrics)
        const uint64_t pw0 = a.WM == 1 ? prow[0] : 0;
#pragma unroll
        for (int u = 0; u < kRuleBatch; ++u) {
          const int32_t mm = m[u] >= 0 ? m[u] : 0;
          v[u] = vrow[mm];
          pw[u] = a.WM == 1 ? pw0 : prow[mm >> 6];
        }
#pragma unroll
        for (int u = 0; u < kRuleBatch; ++u) {
          const LazyRule cr = srule[pslot][min(rb + u, kStageRules - 1)];
          const bool hit = rb + u < nr && m[u] >= 0 &&
                           (uint64_t)v[u] - (uint64_t)cr.lo <= cr.span &&
                           ((pw[u] >> (m[u] & 63)) & 1ull);
          viol = viol || hit;
        }
      }
    }
    for (int32_t rb = r0; !staged && __ballot(ok && rb < r1); rb += kRuleBatch) {
      pas_rule ru[kRuleBatch];
      int64_t v[kRuleBatch];
      uint64_t pw[kRuleBatch];
#pragma unroll
      for (int u = 0; u < kRuleBatch; ++u) ru[u] = a.rules[max(min(rb + u, r1 - 1), 0)];
#pragma unroll
      for (int u = 0; u < kRuleBatch; ++u) {
        const int32_t m = (ru[u].metric >= 0 && ru[u].metric < a.M) ? ru[u].metric : 0;
        v[u] = vrow[m];
        pw[u] = prow[m >> 6];
      }
#pragma unroll
      for (int u = 0; u < kRuleBatch; ++u) {
        const pas_rule rule = ru[u];
        if (rb + u >= r1 || rule.metric < 0 || rule.metric >= a.M || rule.op < 0 || rule.op > 2)
          continue;
        int64_t tm = 0;
        const int sat = target_scaled(rule.target, a.scale_tab, rule.metric, &tm);
        bool hit;
        if (rule.op == PAS_OP_LESS_THAN) hit = sat > 0 || (sat == 0 && v[u] < tm);
        else if (rule.op == PAS_OP_GREATER_THAN) hit = sat < 0 || (sat == 0 && v[u] > tm);
        else hit = sat == 0 && v[u] == tm;
        viol = viol || (hit && ((pw[u] >> (rule.metric & 63)) & 1ull));
      }
    }
    ok = ok && !viol;
    if (ok) ok = lane_fit<KMAX, QW>(a, p, n);
    const uint64_t keep = __ballot(ok) & half_mask;
    if (ok) {
      const int32_t rank = kept + __popcll(keep & below);
      if (rank < k) {
        nodes[rank] = n + a.node_base;
        keys[rank] = order_key(pr.op, mcol[n]);
      }
    }
    kept += active ? __popcll(keep) : 0;
  }
  if (!have) return;
  const int32_t len = min(kept, k);
  for (int32_t i = len + sub; i < k; i += kPodLanes) {
    keys[i] = INT64_MAX;
    nodes[i] = INT32_MAX;
  }
  if (sub == 0) a.len_out[p] = len;
}

// vals [M][N] -> vals_t [N][M] through 64 x 64 LDS tiles (coalesced both ways)
__global__ __launch_bounds__(kTpb) void transpose_vals_kernel(int32_t N, int32_t M,
                                                               const int64_t* __restrict__ vals,
                                                               int64_t* __restrict__ vals_t) {
  __shared__ int64_t tile[64][65];
  const int32_t n0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += kWaves) {
    const int32_t m = m0 + r, n = n0 + tx;
    tile[r][tx] = (m < M && n < N) ? vals[(int64_t)m * N + n] : 0;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += kWaves) {
    const int32_t n = n0 + r, m = m0 + tx;
    if (n < N && m < M) vals_t[(int64_t)n * M + m] = tile[tx][r];
  }
}

// present [M][W64] -> pres_t [N][WM]: bit m of node n's word m / 64
__global__ __launch_bounds__(kTpb) void transpose_present_kernel(
    int32_t N, int32_t M, int32_t W64, int32_t WM, const uint64_t* __restrict__ present,
    uint64_t* __restrict__ pres_t) {
  const int32_t n = blockIdx.x * kTpb + threadIdx.x;
  if (n >= N) return;
  for (int32_t w = 0; w < WM; ++w) {
    uint64_t word = 0;
    for (int32_t j = 0; j < 64 && w * 64 + j < M; ++j) {
      const uint64_t bit = (present[(int64_t)(w * 64 + j) * W64 + (n >> 6)] >> (n & 63)) & 1ull;
      word |= bit << j;
    }
    pres_t[(int64_t)n * WM + w] = word;
  }
}

}  // namespace

int tas_gas_topk_launch(pas_ctx* ctx, int32_t n_pods, int32_t n_rules, const pas_rule* d_rules,
                        const int32_t* d_rule_off, const pas_rule* d_prio,
                        const uint64_t* d_cand, int32_t max_containers, int32_t i915_index,
                        const int64_t* d_req, const uint32_t* d_req_mask,
                        const int32_t* d_n_containers, int32_t k, int32_t node_base,
                        int64_t* d_key, int32_t* d_node, int32_t* d_len, hipStream_t s) {
  if (n_pods == 0) return PAS_OK;
  TasSnapshot& t = ctx->tas;
  const GasSnapshot& g = ctx->gas;
  const int32_t N = t.n_nodes, M = t.n_metrics;
  const int32_t WM = (M + 63) / 64;
  // node-major copies, once per snapshot change
  if (t.t_epoch != t.epoch && N > 0 && M > 0) {
    const size_t bv = sizeof(int64_t) * (size_t)N * M, bp = sizeof(uint64_t) * (size_t)N * WM;
    if (t.t_bytes != bv + bp) {
      if (t.vals_t) {
        PAS_HIP(ctx, hipStreamSynchronize(s));
        PAS_HIP(ctx, hipFree(t.vals_t));
        PAS_HIP(ctx, hipFree(t.pres_t));
        t.vals_t = nullptr;
        t.pres_t = nullptr;
      }
      t.t_bytes = 0;
      PAS_HIP(ctx, hipMalloc(&t.vals_t, bv));
      PAS_HIP(ctx, hipMalloc(&t.pres_t, bp));
      t.t_bytes = bv + bp;
    }
    transpose_vals_kernel<<<dim3((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64)), kTpb, 0,
                            s>>>(N, M, t.vals, t.vals_t);
    transpose_present_kernel<<<(unsigned)((N + kTpb - 1) / kTpb), kTpb, 0, s>>>(
        N, M, (int32_t)w64(N), WM, t.present, t.pres_t);
    PAS_HIP(ctx, hipGetLastError());
    t.t_epoch = t.epoch;
    if (int e = derived_built(ctx, t.t_sync, s)) return e;
  } else if (int e = derived_wait(ctx, t.t_sync, s)) {
    return e;  // built by a call on another stream, maybe still running
  }
  TimedLaunch tl;
  timing_begin(ctx, s, PAS_K_TAS_GAS_TOPK, &tl);
  LazyTopkParams a;
  a.n_pods = n_pods;
  a.N = N;
  a.M = M;
  a.R = t.row;
  a.W64 = (int32_t)w64(N);
  a.k = k;
  a.node_base = node_base;
  a.rules = d_rules;
  a.rule_off = d_rule_off;
  a.n_rules = std::max(n_rules, 0);
  a.prio = d_prio;
  a.cand = d_cand;
  a.perm = t.perm;
  a.cnt = t.cnt;
  a.vals = t.vals;
  a.vals_t = t.vals_t;
  a.pres_t = t.pres_t;
  a.WM = WM;
  a.sorted = t.sorted;
  a.f1k = t.f1k;
  a.f32 = t.f32;
  a.scale_tab = t.scale_tab;
  a.K = g.max_cards;
  a.Q = g.n_res;
  a.C = max_containers;
  a.i915 = i915_index;
  a.n_cards = g.n_cards;
  a.cap = g.cap;
  a.used = g.used;
  a.req = d_req;
  a.mask = d_req_mask;
  a.ncont = d_n_containers;
  a.key_out = d_key;
  a.node_out = d_node;
  a.len_out = d_len;
  const unsigned grid = (unsigned)((n_pods + kPodsPerBlock - 1) / kPodsPerBlock);
  if (a.K <= 8) {
    switch (a.Q) {
      case 1: tas_gas_topk_kernel<8, 1><<<grid, kTpb, 0, s>>>(a); break;
      case 2: tas_gas_topk_kernel<8, 2><<<grid, kTpb, 0, s>>>(a); break;
      case 3: tas_gas_topk_kernel<8, 3><<<grid, kTpb, 0, s>>>(a); break;
      default: tas_gas_topk_kernel<8, kMaxRes><<<grid, kTpb, 0, s>>>(a); break;
    }
  } else if (a.K <= 16) {
    tas_gas_topk_kernel<16, kMaxRes><<<grid, kTpb, 0, s>>>(a);
  } else {
    tas_gas_topk_kernel<PAS_GAS_MAX_CARDS, kMaxRes><<<grid, kTpb, 0, s>>>(a);
  }
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

}  // namespace pas
