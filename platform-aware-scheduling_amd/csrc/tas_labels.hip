// tas_labels.hip — deschedule label plan: which strategy labels each node's patch adds and
// removes, from the violation bitmaps of a sweep and the labels the nodes carry.
//
// Deschedule.updateNodeLabels (deschedule/enforce.go:99-151) walks every node: for each
// strategy whose violation list holds the node it adds the strategy's label with value
// "violating" (:108-117); for every registered policy NAME none of whose strategies is
// violated it counts a "violation" (totalViolations++, :118-134 — the reference counts the
// non-violated names) and, when the node carries that label, removes it and re-adds it as
// "null" (:119-132).  The non-violated set is keyed by name (allPolicies, :89-95), and two
// strategies can share one (NamePlan, pas_internal.h).  Per node that is two 64-bit masks
// over <= 64 strategies: add by strategy, remove by the name's first strategy.  The sweep's
// output is [S][W64] bitmaps (a word = 64 nodes of one strategy), so the plan is a 64 x S
// bit transpose per word: one wave per word, lane s loads word w of strategy row s
// (violations and labels), the S words are broadcast with readlane and each lane (node)
// collects bit s of each.  HBM-bound byte work: 2 * S * 8 bytes read per 64 nodes, 16 bytes
// written per node.
//
// totalViolations is a count over the whole node list, so the kernel writes one partial
// count of violated (node, name) pairs per workgroup and a one-workgroup kernel finishes the
// sum (device-scope atomics on one address serialise across the 8 XCDs).
//
// The JSON body of one node's patch (enforce.go:21-25, 74-86) is host work on the two masks:
// pas_label_patch_json below.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

#include "json_out.h"
#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;
constexpr int kWaves = kTpb / 64;
constexpr int kMaxBlocks = 2048;  // grid-stride beyond; also the partial-count buffer size

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int s) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, s);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), s);
  return (uint64_t)hi << 32 | lo;
}

__global__ __launch_bounds__(kTpb) void label_plan_kernel(int32_t n_nodes, int32_t n_strat,
                                                          int64_t W, NamePlan names,
                                                          const uint64_t* __restrict__ viol,
                                                          const uint64_t* __restrict__ labels,
                                                          uint64_t* __restrict__ add,
                                                          uint64_t* __restrict__ rem,
                                                          int64_t* __restrict__ part) {
  __shared__ int64_t red[kWaves];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * kWaves;
  int64_t violated = 0;  // violated (node, name) pairs of this lane's nodes
  for (int64_t w = (int64_t)blockIdx.x * kWaves + wave; w < W; w += stride) {
    uint64_t vw = 0, lw = 0;
    if (lane < n_strat) {
      vw = viol[lane * W + w];
      if (labels) lw = labels[lane * W + w];
    }
    const int64_t valid = min((int64_t)64, (int64_t)n_nodes - w * 64);
    uint64_t a = 0, r = 0;
    for (int s = 0; s < n_strat; ++s) a |= ((readlane64(vw, s) >> lane) & 1ull) << s;
    if (labels)
      for (int s = 0; s < n_strat; ++s) r |= ((readlane64(lw, s) >> lane) & 1ull) << s;
    if (lane < valid) {
      const uint64_t vn = violated_names(names, a);
      violated += __popcll(vn);
      add[w * 64 + lane] = a;
      rem[w * 64 + lane] = r & names.canon & ~vn;
    }
  }
  for (int off = 32; off > 0; off >>= 1) violated += __shfl_xor(violated, off, 64);
  if (lane == 0) red[wave] = violated;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int i = 0; i < kWaves; ++i) t += red[i];
    part[blockIdx.x] = t;
  }
}

// totalViolations = the non-violated pairs = n_nodes * names - violated pairs.
__global__ __launch_bounds__(kTpb) void label_total_kernel(int32_t n_parts, int64_t pairs,
                                                           const int64_t* __restrict__ part,
                                                           int64_t* __restrict__ total) {
  __shared__ int64_t red[kWaves];
  int64_t t = 0;
  for (int i = threadIdx.x; i < n_parts; i += kTpb) t += part[i];
  for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t v = 0;
    for (int i = 0; i < kWaves; ++i) v += red[i];
    *total = pairs - v;
  }
}

// One patchValue (enforce.go:21-25): {"op":<op>,"path":"/metadata/labels/<name>","value":<v>}
void put_patch(JsonOut& o, const char* op, const char* name, const char* value) {
  o.lit("{\"op\":");
  o.str(op);
  o.lit(",\"path\":\"");
  o.str_body("/metadata/labels/");
  o.str_body(name);
  o.lit("\",\"value\":");
  o.str(value);
  o.put('}');
}

}  // namespace

int label_total_launch(pas_ctx* ctx, int32_t n_parts, int64_t pairs, const int64_t* d_part,
                       int64_t* d_total, hipStream_t s) {
  label_total_kernel<<<1, kTpb, 0, s>>>(n_parts, pairs, d_part, d_total);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

NamePlan make_name_plan(int32_t n_strat, const int32_t* name_id) {
  NamePlan np;
  uint64_t member[64] = {};
  for (int32_t s = 0; s < n_strat; ++s) {
    int32_t k = s;  // the name's first strategy
    if (name_id)
      for (int32_t t = 0; t < s; ++t)
        if (name_id[t] == name_id[s]) {
          k = t;
          break;
        }
    member[k] |= 1ull << s;
  }
  for (int32_t k = 0; k < n_strat; ++k) {
    if (!member[k]) continue;
    np.canon |= 1ull << k;
    if (member[k] == 1ull << k) {
      np.single |= 1ull << k;
    } else {
      np.key[np.n_groups] = (uint8_t)k;
      np.group[np.n_groups++] = member[k];
    }
  }
  return np;
}

int label_plan_launch(pas_ctx* ctx, int32_t n_nodes, int32_t n_strat, const NamePlan& names,
                      const uint64_t* d_viol, const uint64_t* d_labels, uint64_t* d_add,
                      uint64_t* d_rem, int64_t* d_total, hipStream_t s) {
  // the partial counts are the stream's slot buffer: plans on other streams may run beside
  int rc = PAS_OK;
  SlotScope sc(ctx, s, 0, &rc);
  if (!sc.slot) return rc;
  int64_t* part = static_cast<int64_t*>(
      slot_buf(ctx, sc.slot, kBufLabel, sizeof(int64_t) * kMaxBlocks, s, &rc));
  if (!part) return rc;
  const int64_t W = ((int64_t)n_nodes + 63) / 64;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((W + kWaves - 1) / kWaves,
                                                                   kMaxBlocks));
  TimedLaunch tl;
  timing_begin(ctx, s, PAS_K_TAS_LABELS, &tl);
  label_plan_kernel<<<blocks, kTpb, 0, s>>>(n_nodes, n_strat, W, names, d_viol, d_labels, d_add,
                                            d_rem, part);
  const int64_t pairs = (int64_t)n_nodes * __builtin_popcountll(names.canon);
  label_total_kernel<<<1, kTpb, 0, s>>>(blocks, pairs, part, d_total);
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

}  // namespace pas

// json.Marshal([]patchValue) of one node's label patch: the adds in strategy order, then a
// remove + add-"null" pair per removed label in the order of the names' first strategies
// (the reference iterates a Go map there, whose order is unspecified; the set of operations
// is the same).
extern "C" int pas_label_patch_json(int32_t n_strat, const char* const* names, uint64_t add_mask,
                                    uint64_t remove_mask, char* buf, int64_t cap, int64_t* len) {
  if (n_strat < 0 || n_strat > 64 || !names || !len || cap < 0 || (cap > 0 && !buf))
    return PAS_EINVAL;
  const uint64_t live = n_strat == 64 ? ~0ull : ((1ull << n_strat) - 1);
  if ((add_mask | remove_mask) & ~live) return PAS_EINVAL;
  for (int32_t s = 0; s < n_strat; ++s)
    if (((add_mask | remove_mask) >> s & 1) && !names[s]) return PAS_EINVAL;
  pas::JsonOut o{buf, cap};
  o.put('[');
  bool first = true;
  for (int32_t s = 0; s < n_strat; ++s)
    if (add_mask >> s & 1) {
      if (!first) o.put(',');
      pas::put_patch(o, "add", names[s], "violating");
      first = false;
    }
  for (int32_t s = 0; s < n_strat; ++s)
    if (remove_mask >> s & 1) {
      if (!first) o.put(',');
      pas::put_patch(o, "remove", names[s], "");
      o.put(',');
      pas::put_patch(o, "add", names[s], "null");
      first = false;
    }
  o.put(']');
  *len = o.pos;
  return o.pos <= cap ? PAS_OK : PAS_ECAPACITY;
}
