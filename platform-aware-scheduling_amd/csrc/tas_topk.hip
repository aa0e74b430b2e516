// tas_topk.hip — per-pod top-k prioritize lists over node shards, and their exact merge.
//
// Node-sharded evaluation (BASELINE configs[4]): each GPU holds a contiguous
// node range of the snapshot and evaluates every pending pod against it.  The filter verdict
// (dontschedule.Violated, telemetryscheduler.go:184-225) is per node; the prioritize order
// (prioritizeNodesForRule / core.OrderedList, telemetryscheduler.go:128-149,
// operator.go:30-42) is global, but its first k entries are among the union of each
// shard's first k, compared by the order's key:
//   GreaterThan  value descending, ties by ascending node index
//   LessThan     value ascending,  ties by ascending node index
//   other        ascending node index (the documented order of the unsorted branch)
// So a shard emits merge records (key, global node) for its first k entries, the records of
// all shards are all-gathered, and a merge keeps the k smallest (key, node) pairs — the
// same list the whole snapshot gives (HostPriority.Score = 10 - position).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;
constexpr int64_t kKeyNone = INT64_MAX;  // past a list's end (sorts after every record)
constexpr int32_t kNodeNone = INT32_MAX;

// Merge key of a node's value under the pod's prioritize operator: ascending key order is
// the HostPriorityList order (~v reverses int64 order without overflow).
__device__ __forceinline__ int64_t order_key(int32_t op, int64_t v) {
  return op == PAS_OP_GREATER_THAN ? ~v : op == PAS_OP_LESS_THAN ? v : 0;
}

// Shard-local top-k lists (node ids local to the shard, from the eval kernel) -> merge
// records: key from the snapshot value of the pod's prioritize metric, node id + node_base.
__global__ void topk_records_kernel(int32_t n_pods, int32_t k, int32_t N, int32_t M,
                                    int32_t node_base, const pas_rule* __restrict__ prio,
                                    const int64_t* __restrict__ vals,
                                    int32_t* __restrict__ nodes, const int32_t* __restrict__ len,
                                    int64_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * kTpb + threadIdx.x;
  if (i >= (int64_t)n_pods * k) return;
  const int32_t p = (int32_t)(i / k), j = (int32_t)(i % k);
  if (j >= len[p]) {
    keys[i] = kKeyNone;
    nodes[i] = kNodeNone;
    return;
  }
  const pas_rule r = prio[p];  // a listed pod has 0 <= metric < M (tas_prep grouping)
  const int32_t n = nodes[i];
  keys[i] = order_key(r.op, vals[(int64_t)r.metric * N + n]);
  nodes[i] = n + node_base;
}

__device__ __forceinline__ bool before(int64_t ka, int32_t na, int64_t kb, int32_t nb) {
  return ka < kb || (ka == kb && na < nb);
}

// One wave per pod: the n_shards * k records of the pod are staged in LDS; each lane ranks
// its records against all of them (nodes are distinct, so ranks are distinct) and the
// records of rank < k are the merged list.
__global__ __launch_bounds__(64) void topk_merge_kernel(int32_t n_pods, int32_t k,
                                                        int32_t n_shards,
                                                        const int64_t* __restrict__ keys,
                                                        const int32_t* __restrict__ nodes,
                                                        int32_t* __restrict__ out_node,
                                                        int32_t* __restrict__ out_len) {
  extern __shared__ __attribute__((aligned(16))) int64_t rec_key[];
  const int32_t total = n_shards * k;
  int32_t* rec_node = reinterpret_cast<int32_t*>(rec_key + total);
  const int32_t p = blockIdx.x;
  const int lane = threadIdx.x;
  int32_t real = 0;
  for (int32_t i = lane; i < total; i += 64) {
    const int64_t src = ((int64_t)(i / k) * n_pods + p) * k + (i % k);  // [shard][pod][k]
    rec_key[i] = keys[src];
    rec_node[i] = nodes[src];
    real += nodes[src] != kNodeNone;
  }
  __syncthreads();
  for (int off = 32; off > 0; off >>= 1) real += __shfl_xor(real, off, 64);
  const int32_t len = min(real, k);
  int32_t* row = out_node + (int64_t)p * k;
  for (int32_t i = lane; i < total; i += 64) {
    const int64_t ki = rec_key[i];
    const int32_t ni = rec_node[i];
    if (ni == kNodeNone) continue;
    int32_t rank = 0;
    for (int32_t j = 0; j < total; ++j) rank += before(rec_key[j], rec_node[j], ki, ni);
    if (rank < k) row[rank] = ni;
  }
  for (int32_t i = len + lane; i < k; i += 64) row[i] = -1;
  if (lane == 0) out_len[p] = len;
}

}  // namespace

int tas_topk_launch(pas_ctx* ctx, int32_t n_pods, int32_t n_rules, const pas_rule* d_rules,
                    const int32_t* d_rule_off, const pas_rule* d_prio, const uint64_t* d_cand,
                    int32_t k, int32_t node_base, int64_t* d_key, int32_t* d_node,
                    int32_t* d_len, hipStream_t s) {
  if (n_pods == 0) return PAS_OK;
  const TasSnapshot& t = ctx->tas;
  // the eval kernel writes the shard-local lists into d_node (stride k), then records
  if (int rc = tas_eval_launch(ctx, n_pods, n_rules, d_rules, d_rule_off, d_prio, d_cand,
                               PAS_TAS_FILTER | PAS_TAS_PRIORITIZE, nullptr, d_node, d_len, k,
                               s))
    return rc;
  const int64_t n = (int64_t)n_pods * k;
  topk_records_kernel<<<(unsigned)((n + kTpb - 1) / kTpb), kTpb, 0, s>>>(
      n_pods, k, t.n_nodes, t.n_metrics, node_base, d_prio, t.vals, d_node, d_len, d_key);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

int topk_merge_launch(pas_ctx* ctx, int32_t n_pods, int32_t k, int32_t n_shards,
                      const int64_t* d_keys, const int32_t* d_nodes, int32_t* d_out_node,
                      int32_t* d_out_len, hipStream_t s) {
  if (n_pods == 0) return PAS_OK;
  const size_t lds = (size_t)n_shards * k * (sizeof(int64_t) + sizeof(int32_t));
  if (lds > 64 * 1024)
    return set_error(ctx, PAS_ECAPACITY, "pas_topk_merge: n_shards * k too large (LDS)");
  topk_merge_kernel<<<(unsigned)n_pods, 64, lds, s>>>(n_pods, k, n_shards, d_keys, d_nodes,
                                                      d_out_node, d_out_len);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

}  // namespace pas
