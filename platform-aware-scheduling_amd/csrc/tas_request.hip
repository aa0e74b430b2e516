// tas_request.hip — prioritize of one extender request in the request's own order.
//
// prioritizeNodesForRule (telemetryscheduler.go:128-149) copies the metric of every
// args.Nodes.Items entry that has one into a map (filteredNodeData, :135-139; a repeated
// name keeps one entry), and core.OrderedList (operator.go:30-42) sorts the map's entries:
// GreaterThan by value descending, LessThan ascending, any other operator not at all.  The
// reference's order among ties (and for other operators) is Go-map order, i.e. unspecified;
// SURVEY.md A.3 fixes it as the ascending position of the node in the request's candidate
// list.  This path produces exactly that order as request positions:
//
//   1. first[node] = min request position naming node        (scatter, atomicMin)
//   2. key[j] = rank(value) << pb | j for first occurrences that have the metric, where
//      rank = #values strictly before it in the operator's direction (LessThan: lower bound
//      in the snapshot's ascending sorted row; GreaterThan: cnt - upper bound; others: 0),
//      and an all-ones sentinel for every other position; count the kept positions
//   3. radix sort of the keys over bits [0, rb + pb)       (rocprim, stable, one launch set)
//   4. pos[i] = key[i] & (2^pb - 1) for i < len, -1 after
//
// The snapshot's sorted rows (tas_snapshot.hip) give every rank in one binary search, so
// no value leaves HBM except the row the search touches (L2-resident after the first
// request); the work is O(n_req) plus a sort of n_req 8-byte keys.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <rocprim/device/device_radix_sort.hpp>

#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;

inline int bit_length(int64_t x) {
  int b = 0;
  while (x > 0) {
    ++b;
    x >>= 1;
  }
  return b;
}

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + kTpb - 1) / kTpb); }

__global__ void first_pos_kernel(int32_t n_req, int32_t N, const int32_t* __restrict__ req,
                                 int32_t* __restrict__ first) {
  const int32_t j = blockIdx.x * kTpb + threadIdx.x;
  if (j >= n_req) return;
  const int32_t n = req[j];
  if (n >= 0 && n < N) atomicMin(first + n, j);
}

// Number of entries of the ascending row[0, cnt) that are < v (lower) or <= v (upper).
__device__ __forceinline__ int32_t bound(const int64_t* __restrict__ row, int32_t cnt, int64_t v,
                                         bool upper) {
  int32_t lo = 0, hi = cnt;
  while (lo < hi) {
    const int32_t mid = (int32_t)(((uint32_t)lo + (uint32_t)hi) >> 1);
    const int64_t x = row[mid];
    if (x < v || (upper && x == v)) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ void request_keys_kernel(int32_t n_req, int32_t N, int32_t R, pas_rule rule,
                                    int pb, uint64_t sentinel, const int32_t* __restrict__ req,
                                    const int32_t* __restrict__ first,
                                    const int64_t* __restrict__ vals,
                                    const uint64_t* __restrict__ present,
                                    const int32_t* __restrict__ cnt,
                                    const int64_t* __restrict__ sorted,
                                    uint64_t* __restrict__ keys, int32_t* __restrict__ len) {
  const int32_t j = blockIdx.x * kTpb + threadIdx.x;
  bool keep = false;
  uint64_t key = sentinel;
  if (j < n_req) {
    const int32_t n = req[j];
    if (n >= 0 && n < N && first[n] == j) {
      const int64_t W = ((int64_t)N + 63) >> 6;
      const uint64_t word = present[(int64_t)rule.metric * W + (n >> 6)];
      if ((word >> (n & 63)) & 1ull) {
        keep = true;
        uint64_t rank = 0;
        if (rule.op == PAS_OP_LESS_THAN || rule.op == PAS_OP_GREATER_THAN) {
          const int64_t v = vals[(int64_t)rule.metric * N + n];
          const int32_t c = cnt[rule.metric];
          const int64_t* row = sorted + (int64_t)rule.metric * R;
          rank = rule.op == PAS_OP_LESS_THAN ? (uint64_t)bound(row, c, v, false)
                                             : (uint64_t)(c - bound(row, c, v, true));
        }
        key = rank << pb | (uint64_t)j;
      }
    }
    keys[j] = key;
  }
  // one atomic per wave: the kept count of the wave's 64 positions
  const uint64_t ballot = __ballot(keep);
  if ((threadIdx.x & 63) == 0 && ballot) atomicAdd(len, (int32_t)__popcll(ballot));
}

__global__ void request_positions_kernel(int32_t n_req, uint64_t mask,
                                         const uint64_t* __restrict__ keys,
                                         const int32_t* __restrict__ len,
                                         int32_t* __restrict__ pos) {
  const int32_t i = blockIdx.x * kTpb + threadIdx.x;
  if (i >= n_req) return;
  pos[i] = i < *len ? (int32_t)(keys[i] & mask) : -1;
}

struct Bits {
  int rb, pb;
};

Bits key_bits(int32_t n_nodes, int32_t n_req) {
  // ranks are < n_nodes <= 2^rb - 1, so the all-ones rank field of the sentinel sorts last
  return Bits{bit_length(n_nodes), std::max(1, bit_length((int64_t)n_req - 1))};
}

}  // namespace

int prio_request_workspace(pas_ctx* ctx, int32_t n_req, size_t* bytes) {
  *bytes = 0;
  if (n_req == 0) return PAS_OK;  // the launch returns an empty list before any sort
  const Bits b = key_bits(ctx->tas.n_nodes, n_req);
  size_t tmp = 0;
  uint64_t* none = nullptr;
  if (rocprim::radix_sort_keys(nullptr, tmp, none, none, (size_t)n_req, 0, b.rb + b.pb) !=
      hipSuccess)
    return set_error(ctx, PAS_EDEVICE, "pas_tas_prioritize_request: sort sizing failed");
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  *bytes = up(sizeof(int32_t) * (size_t)ctx->tas.n_nodes) + 2 * up(sizeof(uint64_t) * n_req) +
           up(tmp);
  return PAS_OK;
}

int prio_request_launch(pas_ctx* ctx, const pas_rule& rule, int32_t n_req,
                        const int32_t* d_req, int32_t* d_pos, int32_t* d_len, void* ws,
                        size_t ws_bytes, hipStream_t s) {
  const TasSnapshot& t = ctx->tas;
  const int32_t N = t.n_nodes;
  PAS_HIP(ctx, hipMemsetAsync(d_len, 0, sizeof(int32_t), s));
  if (n_req == 0) return PAS_OK;
  if (rule.metric < 0 || rule.metric >= t.n_metrics) {
    // no scheduling rule / metric not cached: prioritizeNodes answers with an empty list
    PAS_HIP(ctx, hipMemsetAsync(d_pos, 0xff, sizeof(int32_t) * (size_t)n_req, s));
    return PAS_OK;
  }
  const Bits b = key_bits(N, n_req);
  const uint64_t mask = (1ull << b.pb) - 1;
  const uint64_t sentinel = (1ull << (b.rb + b.pb)) - 1;
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  char* p = static_cast<char*>(ws);
  int32_t* first = reinterpret_cast<int32_t*>(p);
  p += up(sizeof(int32_t) * (size_t)N);
  uint64_t* keys_a = reinterpret_cast<uint64_t*>(p);
  p += up(sizeof(uint64_t) * n_req);
  uint64_t* keys_b = reinterpret_cast<uint64_t*>(p);
  p += up(sizeof(uint64_t) * n_req);
  size_t tmp = ws_bytes - (size_t)(p - static_cast<char*>(ws));
  if (N > 0) PAS_HIP(ctx, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(first), INT32_MAX,
                                          (size_t)N, s));
  TimedLaunch tl;
  timing_begin(ctx, s, PAS_K_PRIO_REQUEST, &tl);
  first_pos_kernel<<<blocks_for(n_req), kTpb, 0, s>>>(n_req, N, d_req, first);
  request_keys_kernel<<<blocks_for(n_req), kTpb, 0, s>>>(
      n_req, N, t.row, rule, b.pb, sentinel, d_req, first, t.vals, t.present, t.cnt, t.sorted,
      keys_a, d_len);
  PAS_HIP(ctx, rocprim::radix_sort_keys(p, tmp, keys_a, keys_b, (size_t)n_req, 0, b.rb + b.pb,
                                        s));
  request_positions_kernel<<<blocks_for(n_req), kTpb, 0, s>>>(n_req, mask, keys_b, d_len, d_pos);
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

}  // namespace pas
