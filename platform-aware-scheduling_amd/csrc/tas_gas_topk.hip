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
// although only the first k passing nodes of the order are kept.  Here a wave owns a pod and
// walks its order row (the snapshot's per-metric order, tas_snapshot.hip) 64 positions at a
// time: each lane evaluates its position's node directly — candidate bit, every dontschedule
// rule of the pod (EvaluateRule on the node's value: one gather per rule), then the GAS first
// fit on the node's card usage (only for lanes still passing) — and the wave stops once k
// nodes are kept.  The result is the same list: the k first positions of the order whose
// node passes both filters.  With filter and fit rates near 1 (C5: ~0.93 and ~0.97) a pod
// needs one round, ~64 node evaluations instead of the shard's N.
//
// Records: key = order key of the node's value under the pod's operator (tas_topk.hip),
// node = global id (local + node_base); past len: key INT64_MAX, node INT32_MAX.
#include <hip/hip_runtime.h>

#include <cstdint>

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
  const pas_rule* prio;
  const uint64_t* cand;  // [P][W64] or null (every node a candidate)
  const int32_t* perm;   // [3][M][R] snapshot orders
  const int32_t* cnt;    // [M]
  const int64_t* vals;   // [M][N]
  const uint64_t* present;
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

__device__ __forceinline__ int target_milli(int64_t t, int64_t* tm) {
  constexpr int64_t kMax = INT64_MAX / 1000;
  constexpr int64_t kMin = INT64_MIN / 1000;
  if (t > kMax) return 1;
  if (t < kMin) return -1;
  *tm = t * 1000;
  return 0;
}

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
// (fully unrolled) for KMAX <= 16; the wide case keeps the copy in scratch.
template <int KMAX>
__device__ bool lane_fit(const LazyTopkParams& a, int32_t p, int32_t n) {
  const int32_t nc = a.n_cards[n];
  if (nc <= 0) return false;  // FetchNode error / no cards label (:282-298)
  constexpr int kUnroll = KMAX <= 16 ? KMAX : 1;
  const int32_t Q = a.Q;
  const int32_t ncard = min(nc, min(a.K, KMAX));
  int64_t cap[kMaxRes];
  int64_t w[KMAX][kMaxRes];
#pragma unroll
  for (int q = 0; q < kMaxRes; ++q) cap[q] = q < Q ? a.cap[(int64_t)n * Q + q] : 0;
#pragma unroll kUnroll
  for (int k = 0; k < KMAX; ++k)
#pragma unroll
    for (int q = 0; q < kMaxRes; ++q)
      w[k][q] = (k < ncard && q < Q) ? a.used[((int64_t)n * a.K + k) * Q + q] : 0;
  const int32_t nct = a.ncont[p];
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
    for (int64_t g = 0; g < num; ++g) {
      int chosen = -1;
#pragma unroll kUnroll
      for (int k = KMAX - 1; k >= 0; --k) {  // first fit = lowest k
        bool ok = k < ncard && !(m & PAS_REQ_UNKNOWN_KIND);  // (a key no capacity has)
#pragma unroll
        for (int q = 0; q < kMaxRes; ++q)
          if (q < Q && ((m >> q) & 1u)) ok = ok && kind_fits(r[q], cap[q], w[k][q]);
        chosen = ok ? k : chosen;
      }
      if (chosen < 0) return false;  // errWontFit (:249-253)
#pragma unroll kUnroll
      for (int k = 0; k < KMAX; ++k)
#pragma unroll
        for (int q = 0; q < kMaxRes; ++q)
          if (k == chosen && q < Q && ((m >> q) & 1u)) w[k][q] += r[q];
    }
  }
  return true;
}

template <int KMAX>
__global__ __launch_bounds__(kTpb) void tas_gas_topk_kernel(LazyTopkParams a) {
  const int lane = threadIdx.x & 63;
  const int32_t p = (int32_t)blockIdx.x * kWaves + (int32_t)(threadIdx.x >> 6);
  if (p >= a.n_pods) return;  // wave-uniform
  const int32_t k = a.k;
  int64_t* keys = a.key_out + (int64_t)p * k;
  int32_t* nodes = a.node_out + (int64_t)p * k;
  const pas_rule pr = a.prio[p];
  // no scheduling rule / metric not cached: empty list (telemetryscheduler.go:92-96)
  const bool listed = pr.metric >= 0 && pr.metric < a.M;
  int32_t c0 = listed ? a.cnt[pr.metric] : 0;
  // a pod past PAS_GAS_MAX_SELECTIONS is not evaluated (its fit bits are 0, as
  // pas_gas_fit_bitmap_device leaves them)
  {
    int64_t steps = 0;
    for (int32_t c = 0; c < a.ncont[p]; ++c) {
      const int64_t b = (int64_t)p * a.C + c;
      const uint32_t m = a.mask[b];
      if (a.i915 >= 0 && m != 0u && ((m >> a.i915) & 1u)) {
        const int64_t v = a.req[b * a.Q + a.i915];
        if (v > 0) steps += min(v, (int64_t)PAS_GAS_MAX_SELECTIONS + 1);
      }
    }
    if (steps > PAS_GAS_MAX_SELECTIONS) c0 = 0;
  }
  const int32_t r0 = a.rule_off[p], r1 = a.rule_off[p + 1];
  const int32_t* row =
      a.perm + ((int64_t)(pr.op == PAS_OP_GREATER_THAN ? kOrderDesc
                          : pr.op == PAS_OP_LESS_THAN  ? kOrderAsc
                                                       : kOrderIndex) *
                    a.M +
                (listed ? pr.metric : 0)) *
                   a.R;
  const int64_t* mcol = a.vals + (int64_t)(listed ? pr.metric : 0) * a.N;
  int32_t kept = 0;
  for (int32_t j0 = 0; j0 < c0 && kept < k; j0 += 64) {
    const int32_t j = j0 + lane;
    const bool valid = j < c0;
    const int32_t n = valid ? row[j] : 0;
    bool ok = valid;
    if (a.cand) ok = ok && ((a.cand[(int64_t)p * a.W64 + (n >> 6)] >> (n & 63)) & 1ull);
    // dontschedule.Violated (strategy.go:25-44) at this node: any rule whose metric the node
    // has and whose EvaluateRule holds; rules on metrics outside the cache or with an
    // unknown operator are skipped.  kRuleBatch rules' gathers in flight at once.
    bool viol = false;
    for (int32_t rb = r0; rb < r1; rb += kRuleBatch) {
      pas_rule ru[kRuleBatch];
      int64_t v[kRuleBatch];
      uint64_t pw[kRuleBatch];
#pragma unroll
      for (int u = 0; u < kRuleBatch; ++u) ru[u] = a.rules[min(rb + u, r1 - 1)];
#pragma unroll
      for (int u = 0; u < kRuleBatch; ++u) {
        const int32_t m = (ru[u].metric >= 0 && ru[u].metric < a.M) ? ru[u].metric : 0;
        v[u] = a.vals[(int64_t)m * a.N + n];
        pw[u] = a.present[(int64_t)m * a.W64 + (n >> 6)];
      }
#pragma unroll
      for (int u = 0; u < kRuleBatch; ++u) {
        const pas_rule rule = ru[u];
        if (rule.metric < 0 || rule.metric >= a.M || rule.op < 0 || rule.op > 2) continue;
        int64_t tm = 0;
        const int sat = target_milli(rule.target, &tm);
        bool hit;
        if (rule.op == PAS_OP_LESS_THAN) hit = sat > 0 || (sat == 0 && v[u] < tm);
        else if (rule.op == PAS_OP_GREATER_THAN) hit = sat < 0 || (sat == 0 && v[u] > tm);
        else hit = sat == 0 && v[u] == tm;
        viol = viol || (hit && ((pw[u] >> (n & 63)) & 1ull));
      }
    }
    ok = ok && !viol;
    if (ok) ok = lane_fit<KMAX>(a, p, n);
    const uint64_t keep = __ballot(ok);
    if (ok) {
      const int32_t rank = kept + (int32_t)__builtin_amdgcn_mbcnt_hi(
                                      (uint32_t)(keep >> 32),
                                      __builtin_amdgcn_mbcnt_lo((uint32_t)keep, 0u));
      if (rank < k) {
        nodes[rank] = n + a.node_base;
        keys[rank] = order_key(pr.op, mcol[n]);
      }
    }
    kept += (int32_t)__popcll(keep);
  }
  const int32_t len = min(kept, k);
  for (int32_t i = len + lane; i < k; i += 64) {
    keys[i] = INT64_MAX;
    nodes[i] = INT32_MAX;
  }
  if (lane == 0) a.len_out[p] = len;
}

}  // namespace

int tas_gas_topk_launch(pas_ctx* ctx, int32_t n_pods, const pas_rule* d_rules,
                        const int32_t* d_rule_off, const pas_rule* d_prio,
                        const uint64_t* d_cand, int32_t max_containers, int32_t i915_index,
                        const int64_t* d_req, const uint32_t* d_req_mask,
                        const int32_t* d_n_containers, int32_t k, int32_t node_base,
                        int64_t* d_key, int32_t* d_node, int32_t* d_len, hipStream_t s) {
  if (n_pods == 0) return PAS_OK;
  const TasSnapshot& t = ctx->tas;
  const GasSnapshot& g = ctx->gas;
  LazyTopkParams a;
  a.n_pods = n_pods;
  a.N = t.n_nodes;
  a.M = t.n_metrics;
  a.R = t.row;
  a.W64 = (int32_t)w64(t.n_nodes);
  a.k = k;
  a.node_base = node_base;
  a.rules = d_rules;
  a.rule_off = d_rule_off;
  a.prio = d_prio;
  a.cand = d_cand;
  a.perm = t.perm;
  a.cnt = t.cnt;
  a.vals = t.vals;
  a.present = t.present;
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
  TimedLaunch tl;
  timing_begin(ctx, s, PAS_K_TAS_GAS_TOPK, &tl);
  const unsigned grid = (unsigned)((n_pods + kWaves - 1) / kWaves);
  if (a.K <= 8)
    tas_gas_topk_kernel<8><<<grid, kTpb, 0, s>>>(a);
  else if (a.K <= 16)
    tas_gas_topk_kernel<16><<<grid, kTpb, 0, s>>>(a);
  else
    tas_gas_topk_kernel<PAS_GAS_MAX_CARDS><<<grid, kTpb, 0, s>>>(a);
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

}  // namespace pas
