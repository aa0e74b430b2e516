// tas_list_merge.hip — exact merge of node-shard HostPriorityLists into the cluster's full list.
//
// Full-list prioritize over node shards: prioritizeNodesForRule
// (telemetryscheduler.go:128-149) lists every candidate node with the metric in
// core.OrderedList order (operator.go:30-42), i.e. ascending (key, node) with key = ~v for
// GreaterThan, v for LessThan, 0 otherwise (tas_topk.hip).  Each shard's list, as
// pas_tas_topk_device writes it with k = the shard width, is already that order over the
// shard's nodes, so the cluster list is the S-way merge of the shards' runs.  No (key, node)
// pair repeats (node ids are global and distinct), so the merge is unique.
//
// The runs are merged pairwise, log2(S) rounds (S padded to a power of two with empty runs).
// A round is a merge-path pass: a workgroup owns kTile consecutive outputs of one pair, finds
// where its first and last output cut the two runs (binary search along the diagonal),
// stages the two cut pieces (kTile records in all) in LDS, and each lane finds its own cut
// inside them and merges kItems records.  Every record is read and written once per round:
// 12 B (key + node) each way, HBM-bound like the eval kernel's list stores.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;
constexpr int kItems = 4;
constexpr int kTile = kTpb * kItems;
constexpr int64_t kKeyNone = INT64_MAX;
constexpr int32_t kNodeNone = INT32_MAX;

__device__ __forceinline__ bool before(int64_t ka, int32_t na, int64_t kb, int32_t nb) {
  return ka < kb || (ka == kb && na < nb);
}

// A round's input: record i of run s of pod p at base + s * s_stride + p * p_stride + i; runs
// s >= n_real are empty (every record a sentinel).
struct Runs {
  const int64_t* key;
  const int32_t* node;
  int64_t s_stride, p_stride;
  int32_t n_real;
};

struct RunRef {
  const int64_t* key;
  const int32_t* node;
  bool real;
};

__device__ __forceinline__ RunRef run_ref(const Runs& in, int32_t p, int32_t s) {
  const int64_t off = (int64_t)s * in.s_stride + (int64_t)p * in.p_stride;
  return {in.key + off, in.node + off, s < in.n_real};
}

__device__ __forceinline__ void load(const RunRef& r, int64_t i, int64_t* k, int32_t* n) {
  if (r.real) {
    *k = r.key[i];
    *n = r.node[i];
  } else {
    *k = kKeyNone;
    *n = kNodeNone;
  }
}

// Records of run A among the first d outputs of the stable merge of A and B (width w each;
// A first on equal records): the merge path's cut on diagonal d.
__device__ int64_t cut(const RunRef& a, const RunRef& b, int64_t w, int64_t d) {
  int64_t lo = d > w ? d - w : 0, hi = d < w ? d : w;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    int64_t ka, kb;
    int32_t na, nb;
    load(a, mid, &ka, &na);
    load(b, d - mid - 1, &kb, &nb);
    if (!before(kb, nb, ka, na)) lo = mid + 1;  // A[mid] precedes B[d - mid - 1]
    else hi = mid;
  }
  return lo;
}

// The cuts of every tile boundary of a round, [P][n_pairs][tiles + 1], one thread each (the
// dependent binary-search loads of all boundaries in flight at once, ahead of the merge).
__global__ void cuts_kernel(Runs in, int64_t w, int32_t n_pairs, int32_t tiles, int64_t n_cuts,
                            int64_t* __restrict__ cuts) {
  const int64_t t = (int64_t)blockIdx.x * kTpb + threadIdx.x;
  if (t >= n_cuts) return;
  const int32_t e = (int32_t)(t % (tiles + 1));
  const int32_t m = (int32_t)((t / (tiles + 1)) % n_pairs);
  const int32_t p = (int32_t)(t / ((int64_t)(tiles + 1) * n_pairs));
  const RunRef A = run_ref(in, p, 2 * m), B = run_ref(in, p, 2 * m + 1);
  cuts[t] = cut(A, B, w, min((int64_t)e * kTile, 2 * w));
}

// One round: pairs (2m, 2m + 1) of runs of width w -> run m of width 2w.  Blocks: (pod, pair,
// tile) in x.  Output: out_key/out_node [P][...] with row pitch out_pitch, or (final round,
// out_key null) the node ids only, sentinels as -1, positions < out_cols.
__global__ __launch_bounds__(kTpb) void merge_round_kernel(Runs in, int64_t w, int32_t n_pairs,
                                                           int32_t tiles,
                                                           const int64_t* __restrict__ cuts,
                                                           int64_t* out_key, int32_t* out_node,
                                                           int64_t out_pitch, int64_t out_cols) {
  __shared__ int64_t sk[kTile];
  __shared__ int32_t sn[kTile];
  const int64_t b = blockIdx.x;
  const int32_t tile = (int32_t)(b % tiles);
  const int32_t m = (int32_t)((b / tiles) % n_pairs);
  const int32_t p = (int32_t)(b / ((int64_t)tiles * n_pairs));
  const RunRef A = run_ref(in, p, 2 * m), B = run_ref(in, p, 2 * m + 1);
  const int64_t d0 = (int64_t)tile * kTile, d1 = min(d0 + kTile, 2 * w);
  const int64_t* bc = cuts + (b / tiles) * (tiles + 1) + tile;
  const int64_t a0 = bc[0], a1 = bc[1];
  const int64_t b0 = d0 - a0, b1 = d1 - a1;
  const int32_t na = (int32_t)(a1 - a0), nb = (int32_t)(b1 - b0);
  for (int32_t i = threadIdx.x; i < na + nb; i += kTpb) {
    int64_t k;
    int32_t n;
    if (i < na) load(A, a0 + i, &k, &n);
    else load(B, b0 + i - na, &k, &n);
    sk[i] = k;
    sn[i] = n;
  }
  __syncthreads();
  // this lane's outputs [t0, t0 + kItems) of the tile: its cut inside the staged pieces
  const int32_t t0 = threadIdx.x * kItems;
  const int32_t total = na + nb;
  if (t0 >= total) return;
  int32_t lo = max(0, t0 - nb), hi = min(t0, na);
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    const int32_t j = na + t0 - mid - 1;
    if (!before(sk[j], sn[j], sk[mid], sn[mid])) lo = mid + 1;
    else hi = mid;
  }
  int32_t i = lo, j = t0 - lo;
  const int64_t o0 = (int64_t)m * 2 * w + d0 + t0;  // output position in the pod's row
  int64_t* rk = out_key ? out_key + (int64_t)p * out_pitch : nullptr;
  int32_t* rn = out_node + (int64_t)p * out_pitch;
#pragma unroll
  for (int u = 0; u < kItems; ++u) {
    if (t0 + u >= total) break;
    const bool take_a = i < na && (j >= nb || !before(sk[na + j], sn[na + j], sk[i], sn[i]));
    const int32_t s = take_a ? i++ : na + j++;
    const int64_t o = o0 + u;
    if (rk) {
      rk[o] = sk[s];
      rn[o] = sn[s];
    } else if (o < out_cols) {  // final round: node ids, -1 past the list
      rn[o] = sn[s] != kNodeNone ? sn[s] : -1;
    }
  }
}

// The list lengths: the number of real records, i.e. the sum of the shards' lengths.
__global__ void list_len_kernel(int32_t n_pods, Runs in, int32_t n_runs, int64_t w,
                                int32_t* __restrict__ out_len) {
  const int32_t p = blockIdx.x * kTpb + threadIdx.x;
  if (p >= n_pods) return;
  int64_t total = 0;
  for (int32_t s = 0; s < n_runs; ++s) {
    const RunRef r = run_ref(in, p, s);
    if (!r.real) continue;
    int64_t lo = 0, hi = w;  // first sentinel of the run (records are sorted, sentinels last)
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (r.node[mid] != kNodeNone) lo = mid + 1;
      else hi = mid;
    }
    total += lo;
  }
  out_len[p] = (int32_t)total;
}

// One shard: its run already is the cluster's list; copy the node ids, sentinels as -1.
__global__ void single_run_kernel(int32_t n_pods, const int32_t* __restrict__ node, int64_t w,
                                  int32_t* __restrict__ out_node, int64_t out_pitch) {
  const int64_t t = (int64_t)blockIdx.x * kTpb + threadIdx.x;
  if (t >= (int64_t)n_pods * w) return;
  const int64_t p = t / w, i = t - p * w;
  const int32_t n = node[t];
  out_node[p * out_pitch + i] = n != kNodeNone ? n : -1;
}

}  // namespace

int list_merge_launch(pas_ctx* ctx, int32_t n_pods, int32_t n_shards, int32_t width,
                      const int64_t* d_keys, const int32_t* d_nodes, int32_t* d_out_node,
                      int64_t out_ld, int32_t* d_out_len, hipStream_t s) {
  if (n_pods == 0) return PAS_OK;
  int32_t rounds = 0;
  while ((1 << rounds) < n_shards) ++rounds;
  const int64_t sp = (int64_t)1 << rounds;  // runs after padding
  const int64_t row = sp * width;           // records per pod in the intermediate rows
  const int64_t cols = (int64_t)n_shards * width;
  Runs in{d_keys, d_nodes, (int64_t)n_pods * width, width, n_shards};
  list_len_kernel<<<(n_pods + kTpb - 1) / kTpb, kTpb, 0, s>>>(n_pods, in, n_shards, width,
                                                             d_out_len);
  PAS_HIP(ctx, hipGetLastError());
  if (rounds == 0) {  // one shard: no merge, no scratch
    const int64_t n = (int64_t)n_pods * width;
    single_run_kernel<<<(unsigned)((n + kTpb - 1) / kTpb), kTpb, 0, s>>>(n_pods, d_nodes, width,
                                                                        d_out_node, out_ld);
    PAS_HIP(ctx, hipGetLastError());
    return PAS_OK;
  }
  // the tile cuts of a round, then ping-pong rows [P][sp * width] for the rounds before the
  // last.  A round has n_pairs * (tiles + 1) <= sp * width / kTile + 2 * n_pairs cuts per pod.
  int acq = PAS_OK;
  SlotScope sc(ctx, s, 0, &acq);
  if (!sc.slot) return acq;
  int64_t* key_buf[2] = {nullptr, nullptr};
  int32_t* node_buf[2] = {nullptr, nullptr};
  const int64_t max_cuts = (int64_t)n_pods * ((row + kTile - 1) / kTile + 2 * sp + 2);
  int64_t* cut_buf = nullptr;
  {
    const size_t half = rounds > 1 ? (size_t)n_pods * row : 0;
    const size_t need =
        2 * half * (sizeof(int64_t) + sizeof(int32_t)) + sizeof(int64_t) * (size_t)max_cuts;
    // the stream's slot buffer: merges on other streams may run beside this one
    int rc = PAS_OK;
    char* base = static_cast<char*>(slot_buf(ctx, sc.slot, kBufMerge, need, s, &rc));
    if (!base) return rc;
    cut_buf = reinterpret_cast<int64_t*>(base);
    key_buf[0] = cut_buf + max_cuts;
    key_buf[1] = key_buf[0] + half;
    node_buf[0] = reinterpret_cast<int32_t*>(key_buf[1] + half);
    node_buf[1] = node_buf[0] + half;
  }
  auto round = [&](const Runs& rin, int64_t w, int32_t n_pairs, int64_t* ok, int32_t* on,
                   int64_t pitch) -> int {
    const int32_t tiles = (int32_t)((2 * w + kTile - 1) / kTile);
    const int64_t n_cuts = (int64_t)n_pods * n_pairs * (tiles + 1);
    cuts_kernel<<<(unsigned)((n_cuts + kTpb - 1) / kTpb), kTpb, 0, s>>>(rin, w, n_pairs, tiles,
                                                                       n_cuts, cut_buf);
    merge_round_kernel<<<(unsigned)((int64_t)n_pods * n_pairs * tiles), kTpb, 0, s>>>(
        rin, w, n_pairs, tiles, cut_buf, ok, on, pitch, cols);
    PAS_HIP(ctx, hipGetLastError());
    return PAS_OK;
  };
  for (int32_t r = 0; r < rounds; ++r) {
    const int64_t w = (int64_t)width << r;
    const int32_t n_pairs = (int32_t)(sp >> (r + 1));
    const bool last = r == rounds - 1;
    if (int rc = round(in, w, n_pairs, last ? nullptr : key_buf[r & 1],
                       last ? d_out_node : node_buf[r & 1], last ? out_ld : row))
      return rc;
    // the next round reads this round's rows: run i of width 2w at row offset i * 2w
    in = Runs{key_buf[r & 1], node_buf[r & 1], 2 * w, row, (int32_t)(sp >> (r + 1))};
  }
  return PAS_OK;
}

}  // namespace pas
