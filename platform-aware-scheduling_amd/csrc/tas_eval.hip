// tas_eval.hip — batched TAS filter + prioritize, and the deschedule sweep.
//
// Reference path, per pending pod (telemetry-aware-scheduling/pkg/telemetryscheduler/
// telemetryscheduler.go):
//   filterNodes (:184-225)            -> dontschedule.Violated (strategies/dontschedule/
//                                        strategy.go:25-44): union over rules of
//                                        {node : EvaluateRule(value, rule)}
//   prioritizeNodesForRule (:128-149) -> core.OrderedList (strategies/core/operator.go:30-42)
//                                        over the candidates that have the metric
//
// Device formulation (snapshot orders built once per snapshot by tas_snapshot.hip):
//   K ranges  rule -> range.  With the present values of metric m sorted ascending, the
//             nodes satisfying EvaluateRule (operator.go:13-26) form one contiguous range:
//               LessThan t: [0, lower_bound(t*1000))   GreaterThan t: [upper_bound(t*1000), cnt)
//               Equals   t: [lower_bound, upper_bound)
//             (t*1000 saturates: above int64 every present value is LessThan, none is
//             greater or equal; symmetric below).
//   K group   pods are bucketed by their prioritize order (metric, asc/desc/index), so
//             pods sharing a permutation / rank array run back to back (L2 locality).
//   K filter  one workgroup per pod, XCD-aware over the bucketed pod list: a node-space
//             pass bitmap in LDS (candidates, then every node of every rule range cleared;
//             this is the FilterResult), then every non-passing node mapped through the
//             order's rank array into a "drop" bitmap over order positions, written to HBM
//             with the output base of each 1024-position segment.
//   K emit    one wave per (bucket, 1024-position segment): the permutation segment is
//             read ONCE into registers and written, compacted by each pod's drop bits
//             (mbcnt), for every pod of the bucket, with 16-byte non-temporal stores.  The
//             path is therefore bound by the HBM writes of the ordered lists (§8(d)).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;
constexpr int kWaves = kTpb / 64;
constexpr int kRuleChunk = 64;
constexpr int kSegWords = 16;               // 64-bit drop words per emit segment
constexpr int kSegPos = kSegWords * 64;     // 1024 order positions per emit segment
constexpr int kGroupTpb = 1024;
constexpr int kMaxGroupMetrics = 4096;      // 3 * M + 1 buckets in LDS for K group
// LDS words reserved in front of the two bitmaps (rule chunk tables, scan partials), a
// multiple of 4 so the bitmaps stay 16-byte aligned (cdna_hip_programming G17).
constexpr int kMiscWords = 4 * kRuleChunk + 16;
static_assert(kMiscWords >= kTpb, "scan partials live in the misc words");

__device__ __forceinline__ uint64_t tail_mask64(int32_t c, int32_t n) {
  const int32_t lo = c * 64;
  if (lo >= n) return 0ull;
  if (lo + 64 <= n) return ~0ull;
  return (1ull << (n - lo)) - 1ull;
}

__device__ __forceinline__ int32_t lower_bound_i64(const int64_t* __restrict__ a, int32_t n,
                                                   int64_t x) {
  int32_t lo = 0, hi = n;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int32_t upper_bound_i64(const int64_t* __restrict__ a, int32_t n,
                                                   int64_t x) {
  int32_t lo = 0, hi = n;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// target * 1000 with saturation: +1 (above every int64 milli value), -1 (below every
// value) or 0 with *tm exact.
__device__ __forceinline__ int target_milli(int64_t t, int64_t* tm) {
  constexpr int64_t kMax = INT64_MAX / 1000;
  constexpr int64_t kMin = INT64_MIN / 1000;
  if (t > kMax) return 1;
  if (t < kMin) return -1;
  *tm = t * 1000;
  return 0;
}

__device__ __forceinline__ int order_of(int32_t op) {
  return op == PAS_OP_GREATER_THAN ? kOrderDesc : op == PAS_OP_LESS_THAN ? kOrderAsc : kOrderIndex;
}

// Exclusive scan of a[0..n) in LDS by the whole block; returns the total.
// `partial` holds blockDim.x ints of LDS.
__device__ int32_t block_exclusive_scan(int32_t* a, int32_t n, int32_t* partial) {
  const int T = blockDim.x, tid = threadIdx.x;
  const int32_t per = (n + T - 1) / T;
  const int32_t lo = min(n, tid * per), hi = min(n, lo + per);
  int32_t s = 0;
  for (int32_t i = lo; i < hi; ++i) s += a[i];
  partial[tid] = s;
  __syncthreads();
  for (int off = 1; off < T; off <<= 1) {
    const int32_t v = tid >= off ? partial[tid - off] : 0;
    __syncthreads();
    partial[tid] += v;
    __syncthreads();
  }
  int32_t run = partial[tid] - s;
  const int32_t total = partial[T - 1];
  for (int32_t i = lo; i < hi; ++i) {
    const int32_t t = a[i];
    a[i] = run;
    run += t;
  }
  __syncthreads();
  return total;
}

// ---------------------------------------------------------------------------- prep
//
// One launch, two roles: block 0 groups the pods (below); blocks 1.. map every rule to its
// range (a3).  The two are independent, so the binary searches run beside the grouping.

struct RangesParams {
  int32_t n_rules, N, M;
  const pas_rule* rules;
  const int32_t* cnt;
  const int64_t* sorted;
  int2* ranges;
};

// EvaluateRule (operator.go:13-26) over the ascending column: the nodes a rule selects form
// one range, [lower_bound, upper_bound) of t*1000 for Equals, the prefix below it for
// LessThan, the suffix above it for GreaterThan (t*1000 saturates).
__device__ void ranges_body(const RangesParams& R, int32_t r) {
  const pas_rule rule = R.rules[r];
  int2 out = make_int2(0, 0);
  if (rule.metric >= 0 && rule.metric < R.M && rule.op >= 0 && rule.op <= 2) {
    const int32_t c = R.cnt[rule.metric];
    const int64_t* sv = R.sorted + (int64_t)rule.metric * R.N;
    int64_t tm = 0;
    const int sat = target_milli(rule.target, &tm);
    int32_t lb, ub;
    if (sat > 0) { lb = ub = c; }
    else if (sat < 0) { lb = ub = 0; }
    else { lb = lower_bound_i64(sv, c, tm); ub = upper_bound_i64(sv, c, tm); }
    if (rule.op == PAS_OP_LESS_THAN) out = make_int2(0, lb);
    else if (rule.op == PAS_OP_GREATER_THAN) out = make_int2(ub, c);
    else out = make_int2(lb, ub);
  }
  R.ranges[r] = out;
}

struct GroupParams {
  int32_t P, M, N;
  uint32_t flags;
  const pas_rule* prio;
  const int32_t* rule_off;
  const int32_t* cnt;
  int2* keys;            // [P]   scratch: {bucket, cnt0} of each pod
  int32_t* pod_list;     // [P]   pods bucketed by key, bucket G (no list) last
  int32_t* group_start;  // [G+2]
  int32_t* seg_start;    // [G+1] first emit segment of each bucket
  int32_t* seg_group;    // [max_segs] bucket of each emit segment, -1 past the last
  int4* desc;            // [2P] per bucketed position: {pod, ocol, cnt0, n_seg}, {r0, r1, 0, 0}
  int32_t max_segs;
};

constexpr int kGU = 4;  // pods per thread per round of loads (all issued before use)

// Counting sort of the pods by bucket = order column (order * M + metric) of the pod's
// prioritize list, or G when it has none (no PRIORITIZE flag, metric out of range, or a
// metric no node reports: the ReadMetric error of prioritizeNodesForRule,
// telemetryscheduler.go:92-96).  Also writes the per-position pod descriptors the filter
// reads with one load, and the emit-segment table per bucket.  Loads are unconditional
// (clamped indices) so that each round's are in flight together.
__device__ void group_body(const GroupParams& g, int32_t* sh) {
  const int32_t G = 3 * g.M;
  int32_t* partial = sh;                  // [kGroupTpb]
  int32_t* hist = sh + kGroupTpb;         // [G + 1]
  const int tid = threadIdx.x;
  const bool prio = (g.flags & PAS_TAS_PRIORITIZE) != 0 && g.M > 0;
  for (int32_t i = tid; i <= G; i += kGroupTpb) hist[i] = 0;
  __syncthreads();
  for (int32_t p0 = tid; p0 < g.P; p0 += kGroupTpb * kGU) {
    pas_rule r[kGU];
    int32_t c[kGU];
    if (prio) {  // uniform: prio may be null without the PRIORITIZE flag
#pragma unroll
      for (int u = 0; u < kGU; ++u) r[u] = g.prio[min(p0 + u * kGroupTpb, g.P - 1)];
#pragma unroll
      for (int u = 0; u < kGU; ++u) c[u] = g.cnt[min(max(r[u].metric, 0), g.M - 1)];
    } else {
#pragma unroll
      for (int u = 0; u < kGU; ++u) {
        r[u] = pas_rule{-1, 0, 0};
        c[u] = 0;
      }
    }
#pragma unroll
    for (int u = 0; u < kGU; ++u) {
      const int32_t p = p0 + u * kGroupTpb;
      if (p >= g.P) continue;
      const bool listed = prio && r[u].metric >= 0 && r[u].metric < g.M && c[u] > 0;
      const int32_t key = listed ? order_of(r[u].op) * g.M + r[u].metric : G;
      g.keys[p] = make_int2(key, listed ? c[u] : 0);
      atomicAdd(&hist[key], 1);
    }
  }
  __syncthreads();
  block_exclusive_scan(hist, G + 1, partial);
  for (int32_t i = tid; i <= G; i += kGroupTpb) g.group_start[i] = hist[i];
  if (tid == 0) g.group_start[G + 1] = g.P;
  __syncthreads();
  const bool filt = (g.flags & PAS_TAS_FILTER) != 0;
  for (int32_t p0 = tid; p0 < g.P; p0 += kGroupTpb * kGU) {
    int2 kc[kGU];
    int32_t r0[kGU], r1[kGU];
#pragma unroll
    for (int u = 0; u < kGU; ++u) {
      const int32_t p = min(p0 + u * kGroupTpb, g.P - 1);
      kc[u] = g.keys[p];
      r0[u] = filt ? g.rule_off[p] : 0;
      r1[u] = filt ? g.rule_off[p + 1] : 0;
    }
#pragma unroll
    for (int u = 0; u < kGU; ++u) {
      const int32_t p = p0 + u * kGroupTpb;
      if (p >= g.P) continue;
      const int32_t key = kc[u].x, c0 = kc[u].y;
      const int32_t pos = atomicAdd(&hist[key], 1);  // order inside a bucket is free
      g.pod_list[pos] = p;
      g.desc[2 * pos] = make_int4(p, key < G ? key : -1, c0, (c0 + kSegPos - 1) / kSegPos);
      g.desc[2 * pos + 1] = make_int4(r0[u], r1[u], 0, 0);
    }
  }
  __syncthreads();
  // hist[i] now holds the end of bucket i: emit segments per non-empty bucket
  for (int32_t i = tid; i < G; i += kGroupTpb) {
    const int32_t begin = g.group_start[i];
    const int32_t c = g.cnt[i % g.M];
    hist[i] = hist[i] > begin ? (c + kSegPos - 1) / kSegPos : 0;
  }
  __syncthreads();
  const int32_t total = block_exclusive_scan(hist, G, partial);
  for (int32_t i = tid; i < G; i += kGroupTpb) g.seg_start[i] = hist[i];
  if (tid == 0) g.seg_start[G] = total;
  for (int32_t i = tid; i < G; i += kGroupTpb) {
    const int32_t end = i + 1 < G ? hist[i + 1] : total;
    for (int32_t k = hist[i]; k < end; ++k) g.seg_group[k] = i;
  }
  for (int32_t k = total + tid; k < g.max_segs; k += kGroupTpb) g.seg_group[k] = -1;
}

__global__ __launch_bounds__(kGroupTpb) void tas_prep_kernel(GroupParams g, RangesParams R) {
  extern __shared__ __attribute__((aligned(16))) int32_t sh[];
  if (blockIdx.x == 0) {
    group_body(g, sh);
    return;
  }
  const int32_t r = (int32_t)(blockIdx.x - 1) * kGroupTpb + threadIdx.x;
  if (r < R.n_rules) ranges_body(R, r);
}

// ---------------------------------------------------------------------------- filter

struct FilterParams {
  int32_t N, M, P;
  int32_t W32;   // ceil(N / 32)
  int32_t W32p;  // 2 * W64: words per LDS bitmap
  int32_t W64;
  int32_t D64;   // drop row stride in 64-bit words (multiple of kSegWords)
  int32_t S;     // seg_base row stride (= D64 / kSegWords)
  int32_t Nr;    // rank row stride
  uint32_t flags;
  const int2* ranges;
  const pas_rule* rules;
  const uint64_t* cand;
  const int32_t* perm;   // [3][M][N]
  const uint32_t* rank;  // [3][M][Nr]
  const int32_t* phi;    // [3M][M][N] composed orders, or null
  const int4* desc;      // [2P] from K group
  uint64_t* pass_out;    // [P][W64]
  uint64_t* drop;        // [P][D64]
  int32_t* seg_base;     // [P][S]
  int32_t* order_len;    // [P]
};

typedef int32_t v4i32 __attribute__((ext_vector_type(4)));
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int32_t wave_inclusive_sum(int32_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  return x;
}

// Clear bits of the LDS node bitmap `pass` -> bits at their positions in order column
// `ocol` of the LDS drop bitmap, through the rank row.  The walk is in node order, 8 lanes
// per 32-node word: lane q of a word loads the 16-byte quad of ranks of nodes 4q..4q+3 only
// when one of them is clear, so a wave instruction touches at most 8 lines and a pod moves
// one line per word with a clear bit.  (A random 4-byte gather per node moves a line per
// node: 2.6x the line traffic at the C2 shape.)  The loads are unconditional buffer loads
// (a load under a divergent branch makes the compiler wait for the previous one first); a
// lane with nothing to map passes an out-of-range offset: the range check drops the fetch.
template <int kAblate>
__device__ __forceinline__ void map_clear_bits(const FilterParams& P, const uint32_t* pass,
                                               uint32_t* drop, int32_t ocol, int tid) {
  const int32_t N = P.N;
  // buffer resource over the rank row (128-B aligned rows); built from wave-uniform
  // values only (cdna_hip_programming.md T8)
  const uint32_t* row = P.rank + (int64_t)ocol * P.Nr;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(row), 0, P.Nr * 4, 0x00020000);
  const int q = tid & 7;                       // quad of the word: nodes 4q..4q+3
  const int32_t wl = tid >> 3;                 // word slot: 32 per block step
  constexpr int UQ = 8;                        // words per lane in flight
  for (int32_t w0 = 0; w0 < P.W32; w0 += (kTpb / 8) * UQ) {
    uint32_t zq[UQ];
    v4i32 r[UQ];
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int32_t w = min(w0 + u * (kTpb / 8) + wl, P.W32 - 1);
      const int32_t lo = w * 32;
      const uint32_t tail = lo + 32 <= N ? 0xFFFFFFFFu : (1u << (N - lo)) - 1u;
      zq[u] = w0 + u * (kTpb / 8) + wl < P.W32 ? ((~pass[w] & tail) >> (4 * q)) & 0xFu : 0u;
      const uint32_t voff =
          (zq[u] && !(kAblate & 1)) ? (uint32_t)(w * 8 + q) * 16u : 0x80000000u;
      r[u] = __builtin_bit_cast(v4i32, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, 0, 0));
    }
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      if (!zq[u]) continue;
      const uint32_t rr[4] = {(uint32_t)r[u].x, (uint32_t)r[u].y, (uint32_t)r[u].z,
                              (uint32_t)r[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (((zq[u] >> j) & 1u) && rr[j] != kNoRank)
          atomicOr(&drop[rr[j] >> 5], 1u << (rr[j] & 31));
    }
  }
}

// One workgroup per pod.  Phases, each issuing its global loads before their first use:
//   1. candidates -> LDS pass bitmap over node ids;
//   2. rule ranges: 16 coalesced perm reads per thread, LDS atomicAnd into the bitmap.
//      With the composed-order index (phi, pas_tas_set_index_budget) the same range of
//      phi gives the nodes' positions in the pod's prioritize order: a second coalesced
//      read and an LDS atomicOr into the drop bitmap over positions;
//   3. without phi: every clear bit of the final bitmap (failing node or non-candidate)
//      goes to the drop bitmap through the rank row (map_clear_bits); with phi only the
//      non-candidates do, before phase 2;
//   4. drop row + kept count per 1024-position segment -> segment output bases.
// (Measured at C2: random rank gathers per failing node 0.115 ms/step; whole-row scans per
// pod are LDS-bank / VALU bound and slower; line-quad rank loads ~0.08 ms/step.)
// kAblate (diagnostic timing builds only, PAS_FILTER_ABLATE; outputs wrong): bit 1 = no
// rank loads, 2 = no LDS atomics in the rule loop, 4 = no rule loop, 8 = no row writes.
template <int kAblate>
__global__ __launch_bounds__(kTpb) void tas_filter_kernel(FilterParams P) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  int32_t* s_pref = reinterpret_cast<int32_t*>(lds);  // [kRuleChunk] prefix of range lengths
  int32_t* s_base = s_pref + kRuleChunk;              // [kRuleChunk] perm index of range start
  int32_t* s_total = s_base + kRuleChunk;             // [1]
  uint32_t* pass = lds + kMiscWords;                  // [W32p]
  uint32_t* drop = pass + P.W32p;                     // [S * 32], then segk [S]
  uint64_t* pass64 = reinterpret_cast<uint64_t*>(pass);
  uint64_t* drop64 = reinterpret_cast<uint64_t*>(drop);

  // XCD-aware placement: blocks b and b+8 share an XCD (MI355X_MICROARCH.md, Workgroup
  // dispatch), so give each XCD a contiguous run of the bucketed pod list; pods of a
  // bucket then read the same rank row from that XCD's L2.  Speed only, never correctness.
  const int32_t nb = gridDim.x, b = blockIdx.x;
  const int32_t xcd = b & 7, per_xcd = nb >> 3, rem = nb & 7;
  const int32_t pos = xcd * per_xcd + min(xcd, rem) + (b >> 3);
  const int4 d0 = P.desc[2 * pos], d1 = P.desc[2 * pos + 1];
  const int32_t pod = d0.x, ocol = d0.y, cnt0 = d0.z, n_seg = d0.w;
  const int32_t r0 = d1.x, r1 = d1.y;
  const int tid = threadIdx.x;
  const int32_t N = P.N, W64 = P.W64;
  const bool has_list = ocol >= 0;
  const bool use_phi = P.phi != nullptr && (P.flags & PAS_TAS_FILTER);
  const int32_t* __restrict__ phi_o =
      (use_phi && has_list) ? P.phi + (int64_t)ocol * P.M * N : nullptr;

  // ---- 1. candidates -> pass bitmap (args.Nodes.Items, telemetryscheduler.go:204) ----
  constexpr int kCU = 8;
  const uint64_t* __restrict__ cand = P.cand ? P.cand + (int64_t)pod * W64 : nullptr;
  for (int32_t w0 = tid; w0 < W64; w0 += kTpb * kCU) {
    uint64_t x[kCU];
#pragma unroll
    for (int u = 0; u < kCU; ++u) {
      const int32_t w = w0 + u * kTpb;
      x[u] = (cand && w < W64) ? cand[w] : ~0ull;
    }
#pragma unroll
    for (int u = 0; u < kCU; ++u) {
      const int32_t w = w0 + u * kTpb;
      if (w < W64) pass64[w] = x[u] & tail_mask64(w, N);
    }
  }
  if (has_list)
    for (int32_t w = tid; w < n_seg * kSegWords; w += kTpb) drop64[w] = 0ull;
  else if (tid == 0 && (P.flags & PAS_TAS_PRIORITIZE))
    P.order_len[pod] = 0;  // no rule / ReadMetric error -> empty HostPriorityList (:92-96)
  __syncthreads();

  // with phi, the non-candidates are the only clear bits that phase 2 does not map
  if (use_phi && has_list && cand) map_clear_bits<kAblate>(P, pass, drop, ocol, tid);

  // ---- 2. dontschedule.Violated: every node of every rule range fails the filter ----
  if ((P.flags & PAS_TAS_FILTER) && !(kAblate & 4)) {
    const int32_t* perm_asc = P.perm + (int64_t)kOrderAsc * P.M * N;
    for (int32_t c0 = r0; c0 < r1; c0 += kRuleChunk) {
      const int32_t nr = min(kRuleChunk, r1 - c0);
      if (tid < 64) {  // wave 0: rule table = prefix of range lengths (largest-index search)
        int32_t len = 0, bse = 0;
        if (tid < nr) {
          const int2 rg = P.ranges[c0 + tid];
          const int32_t m = P.rules[c0 + tid].metric;
          len = rg.y - rg.x;
          bse = (m >= 0 && m < P.M) ? m * N + rg.x : 0;
        }
        const int32_t incl = wave_inclusive_sum(len);
        const int32_t total = __shfl(incl, nr - 1, 64);  // all lanes active here
        s_base[tid] = bse;
        s_pref[tid] = tid < nr ? incl - len : INT32_MAX;
        if (tid == 0) *s_total = total;
      }
      __syncthreads();
      const int32_t total = *s_total;
      // 16 range reads in flight per thread.  Loads are unconditional (entries past the
      // end re-read the last one; clearing a bit twice is harmless): a load under a
      // divergent branch makes the compiler wait for the previous one first.
      constexpr int U = 16;
      for (int32_t base = tid; base < total; base += kTpb * U) {
        int32_t v[U], q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int32_t f = min(base + u * kTpb, total - 1);
          int32_t r = 0;  // largest r with s_pref[r] <= f (zero-length ranges are skipped)
#pragma unroll
          for (int st = kRuleChunk / 2; st > 0; st >>= 1)
            r = s_pref[r + st] <= f ? r + st : r;
          const int32_t idx = s_base[r] + (f - s_pref[r]);
          v[u] = perm_asc[idx];
          q[u] = phi_o ? phi_o[idx] : -1;  // uniform branch
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (kAblate & 2) {
            asm volatile("" ::"v"(v[u]), "v"(q[u]));
            continue;
          }
          atomicAnd(&pass[v[u] >> 5], ~(1u << (v[u] & 31)));
          if (q[u] >= 0) atomicOr(&drop[q[u] >> 5], 1u << (q[u] & 31));
        }
      }
      __syncthreads();
    }
  }
  // FilterResult row -> HBM.  Written after phase 3 when there is one: a store ahead of
  // phase 3's loads would make their first wait also wait for the store.
  const bool write_pass = (P.flags & PAS_TAS_FILTER) && !(kAblate & 8);
  uint64_t* pass_row = P.pass_out + (int64_t)pod * W64;
  if (!has_list) {
    if (write_pass)
      for (int32_t w = tid; w < W64; w += kTpb) pass_row[w] = pass64[w];
    return;
  }

  // ---- 3. without phi: every clear bit (failing node or non-candidate) -> drop ----
  if (!use_phi) map_clear_bits<kAblate>(P, pass, drop, ocol, tid);
  __syncthreads();

  // ---- 4. pass and drop rows -> HBM; kept count per segment -> segment output bases ----
  if (write_pass)
    for (int32_t w = tid; w < W64; w += kTpb) pass_row[w] = pass64[w];
  uint64_t* drow = P.drop + (int64_t)pod * P.D64;
  if (!(kAblate & 8))
    for (int32_t w = tid; w < n_seg * kSegWords; w += kTpb) drow[w] = drop64[w];
  int32_t* segk = reinterpret_cast<int32_t*>(drop + (size_t)P.S * kSegWords * 2);  // [S]
  for (int32_t sgi = tid; sgi < n_seg; sgi += kTpb) {
    int32_t kept = 0;
#pragma unroll
    for (int j = 0; j < kSegWords; ++j) {
      const int32_t c = sgi * kSegWords + j;
      kept += __popcll(~drop64[c] & tail_mask64(c, cnt0));
    }
    segk[sgi] = kept;
  }
  __syncthreads();
  if (tid < 64) {  // wave 0: exclusive scan of the segment counts
    const int32_t per = (n_seg + 63) / 64;
    const int32_t lo = min(n_seg, tid * per), hi = min(n_seg, lo + per);
    int32_t sum = 0;
    for (int32_t i = lo; i < hi; ++i) sum += segk[i];
    const int32_t incl = wave_inclusive_sum(sum);
    int32_t run = incl - sum;
    int32_t* sb = P.seg_base + (int64_t)pod * P.S;
    for (int32_t i = lo; i < hi; ++i) {
      sb[i] = run;
      run += segk[i];
    }
    if (tid == 63) P.order_len[pod] = incl;
  }
}

// ---------------------------------------------------------------------------- emit

constexpr int kEmitBatch = 16;                                   // pods per LDS fetch round
constexpr int kStageWords = ((kSegPos + 31 + 255) / 256) * 256;  // 5 x 256 (unrolled reads)
constexpr int kDumpSlot = kStageWords - 1;  // compaction target of dropped lanes (> 1055)
constexpr uint32_t kOob = 0x80000000u;      // buffer offset past every range: no access
constexpr int kNtAux = 2;                   // buffer store cache policy: nt

// One wave per (bucket, 1024-position segment): the permutation segment is read once into
// registers and written, compacted by each pod's drop bits, for every pod of the bucket.
// Per pod (ids, bases and drop words of 16 pods are fetched into LDS in one round):
//   compaction  16 x (mbcnt, one unconditional LDS write: dropped lanes write a dump slot)
//               into a stage aligned to the destination's 128-byte lines;
//   stores      range-checked buffer stores against a descriptor of the pod's run: every
//               chunk of whole lines takes an nt 16-byte store, the other full chunks a
//               plain one, the <= 2 partial chunks dword stores; a lane with nothing to
//               store passes an out-of-range offset, so there are no per-lane branches.
// Measured (scripts/diag/fill_shapes.py): the HBM write rate follows the number of
// stores in flight, so the per-pod instruction count between store bursts is what this
// layout minimises.  Waves of a block take different buckets and never synchronise.
// kAblate (diagnostic timing builds only, PAS_EMIT_ABLATE; outputs wrong): 1 = no stores.
template <int kAblate>
__global__ __launch_bounds__(kTpb) void tas_emit_kernel(
    int32_t N, int32_t M, int32_t D64, int32_t S, const int32_t* __restrict__ perm,
    const int32_t* __restrict__ cnt, const int32_t* __restrict__ pod_list,
    const int32_t* __restrict__ group_start, const int32_t* __restrict__ seg_start,
    const int32_t* __restrict__ seg_group, const uint64_t* __restrict__ drop,
    const int32_t* __restrict__ seg_base, int32_t total_segs_bound,
    int32_t* __restrict__ order_out) {
  __shared__ __attribute__((aligned(16))) int32_t stage_all[kWaves][kStageWords];
  __shared__ __attribute__((aligned(16))) uint64_t dbuf_all[kWaves][kEmitBatch][kSegWords];
  __shared__ int32_t pods_all[kWaves][kEmitBatch];
  __shared__ int32_t bases_all[kWaves][kEmitBatch];
  const int wave = threadIdx.x >> 6;
  int32_t* stage = stage_all[wave];
  uint64_t(*dbuf)[kSegWords] = dbuf_all[wave];
  int32_t* pods = pods_all[wave];
  int32_t* bases = bases_all[wave];
  const int32_t gw = __builtin_amdgcn_readfirstlane((int32_t)(blockIdx.x * kWaves + wave));
  const int lane = threadIdx.x & 63;
  if (gw >= total_segs_bound) return;
  const int32_t g = seg_group[gw];  // -1 past the last segment
  if (g < 0) return;
  const int32_t m0 = g % M;
  const int32_t order = g / M;
  const int32_t cnt0 = cnt[m0];
  const int32_t s = gw - seg_start[g];
  const int32_t* __restrict__ pm = perm + ((int64_t)order * M + m0) * N;
  const int32_t k0 = s * kSegPos + lane;
  int32_t node[kSegWords];
#pragma unroll
  for (int j = 0; j < kSegWords; ++j) {
    const int32_t kk = k0 + j * 64;
    node[j] = kk < cnt0 ? pm[kk] : 0;
  }
  const bool full = (s + 1) * kSegPos <= cnt0;  // only a bucket's last segment has a tail

  const int32_t i0 = group_start[g], i1 = group_start[g + 1];
  // Pods in batches of 16: one round of vector loads puts their ids, segment bases and
  // drop words into the wave's LDS (its wait is the only vmcnt wait of a batch); the pod
  // loop then reads LDS only, so up to 16 pods' stores stay in flight per wave.
  for (int32_t ic = i0; ic < i1; ic += kEmitBatch) {
    const int32_t nc = min(kEmitBatch, i1 - ic);
    const int32_t my_pod = pod_list[ic + min(lane & (kEmitBatch - 1), nc - 1)];
    const int pidx = lane >> 2;  // 4 lanes x 32 bytes of drop words per pod
    const int32_t dpod = __shfl(my_pod, pidx, 64);
    const int4* src = reinterpret_cast<const int4*>(drop + (int64_t)dpod * D64 +
                                                    s * kSegWords + (lane & 3) * 4);
    const int4 d0 = src[0], d1 = src[1];
    const int32_t my_base = seg_base[(int64_t)my_pod * S + s];
    int4* dst = reinterpret_cast<int4*>(&dbuf[pidx][(lane & 3) * 4]);
    dst[0] = d0;
    dst[1] = d1;
    if (lane < kEmitBatch) {
      pods[lane] = my_pod;
      bases[lane] = my_base;
    }
    __builtin_amdgcn_wave_barrier();
    for (int32_t q = 0; q < nc; ++q) {
      const int32_t pod = __builtin_amdgcn_readfirstlane(pods[q]);
      const int32_t base = __builtin_amdgcn_readfirstlane(bases[q]);
      uint64_t dw[kSegWords];
#pragma unroll
      for (int j = 0; j < kSegWords; ++j) {
        const uint64_t x = dbuf[q][j];  // broadcast read
        dw[j] = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(x >> 32)) << 32) |
                (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)x);
      }

      const int64_t gdst = (int64_t)pod * N + base;  // element index of the first entry
      const int32_t a = (int32_t)(gdst & 31);         // stage offset: 128-B line alignment
      int32_t k = a;
#pragma unroll
      for (int j = 0; j < kSegWords; ++j) {
        const uint64_t keep = ~dw[j] & (full ? ~0ull : tail_mask64(s * kSegWords + j, cnt0));
        const uint32_t below = __builtin_amdgcn_mbcnt_hi(
            (uint32_t)(keep >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)keep, 0u));
        int32_t addr;  // per-lane select on the SGPR keep mask: k + below, or the dump slot
        asm("v_cndmask_b32_e64 %0, %1, %2, %3"
            : "=v"(addr)
            : "v"(kDumpSlot), "v"(k + (int32_t)below), "s"(keep));
        stage[addr] = node[j];
        k += __popcll(keep);
      }
      __builtin_amdgcn_wave_barrier();
      // the run [a, k) of the stage goes to order_out[gdst - a + a .. gdst - a + k)
      const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
          order_out + (gdst - a), 0, k * 4, 0x00020000);
      constexpr int kChunkIters = kStageWords / 256;
      v4i32 v[kChunkIters];
#pragma unroll
      for (int it = 0; it < kChunkIters; ++it)
        v[it] = *reinterpret_cast<const v4i32*>(stage + (lane + it * 64) * 4);
      const int32_t full_lo = (a + 31) & ~31;  // first entry of the first whole line
      const int32_t full_hi = k & ~31;         // end of the last whole line
      // the <= 2 partial chunks: lanes 0..3 the chunk holding a, lanes 4..7 the one holding
      // k - 1 (the same chunk twice when both ends share it: same values, same addresses)
      const int32_t pidx = lane < 4 ? (a & ~3) + lane : (k & ~3) + (lane - 4);
      const bool pchunk_full = (pidx & ~3) >= a && (pidx & ~3) + 4 <= k;
      const bool pvalid = lane < 8 && pidx >= a && pidx < k && !pchunk_full;
      const int32_t pval = stage[pvalid ? pidx : 0];
      if (kAblate == 1) {
#pragma unroll
        for (int it = 0; it < kChunkIters; ++it)
          asm volatile("" ::"v"(v[it].x), "v"(v[it].y), "v"(v[it].z), "v"(v[it].w));
        asm volatile("" ::"v"(pval));
      } else {
#pragma unroll
        for (int it = 0; it < kChunkIters; ++it) {
          const int32_t e0 = (lane + it * 64) * 4;
          const bool nt = e0 >= full_lo && e0 + 4 <= full_hi;
          const bool plain = !nt && e0 >= a && e0 + 4 <= k;
          const uint32_t off = (uint32_t)e0 * 4u;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v[it]), rsrc,
                                                 nt ? off : kOob, 0, kNtAux);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v[it]), rsrc,
                                                 plain ? off : kOob, 0, 0);
        }
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)pval, rsrc,
                                              pvalid ? (uint32_t)pidx * 4u : kOob, 0, 0);
      }
      __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_wave_barrier();  // the next batch rewrites pods/bases/drop words
  }
}

// ---------------------------------------------------------------------------- deschedule

// One wave per 64-node word, strategies x rules in the wave loop: deschedule.Strategy.
// Violated (deschedule/strategy.go:31-50) per registered strategy, as
// nodeStatusForStrategy does (deschedule/enforce.go:154-164).
__global__ __launch_bounds__(kTpb) void tas_violations_kernel(
    int32_t N, int32_t M, int32_t W64, int32_t n_strat, const int32_t* __restrict__ rule_off,
    const pas_rule* __restrict__ rules, const int64_t* __restrict__ vals,
    const uint64_t* __restrict__ present, uint64_t* __restrict__ viol_out) {
  const int32_t gw = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (gw >= W64) return;
  const int lane = threadIdx.x & 63;
  const int32_t n = gw * 64 + lane;
  const bool valid = n < N;
  for (int32_t s = 0; s < n_strat; ++s) {
    uint64_t acc = 0;
    const int32_t r1 = rule_off[s + 1];
    for (int32_t r = rule_off[s]; r < r1; ++r) {
      const pas_rule rule = rules[r];
      if (rule.metric < 0 || rule.metric >= M || rule.op < 0 || rule.op > 2) continue;
      const uint64_t pres = present[(int64_t)rule.metric * W64 + gw];
      const int64_t v = valid ? vals[(int64_t)rule.metric * N + n] : 0;
      int64_t tm = 0;
      const int sat = target_milli(rule.target, &tm);
      bool hit;
      if (rule.op == PAS_OP_LESS_THAN) hit = sat > 0 || (sat == 0 && v < tm);
      else if (rule.op == PAS_OP_GREATER_THAN) hit = sat < 0 || (sat == 0 && v > tm);
      else hit = sat == 0 && v == tm;
      acc |= __ballot(hit && valid) & pres;
    }
    if (lane == 0) viol_out[(int64_t)s * W64 + gw] = acc;
  }
}

size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

}  // namespace

int tas_eval_launch(pas_ctx* ctx, int32_t n_pods, int32_t n_rules, const pas_rule* d_rules,
                    const int32_t* d_rule_off, const pas_rule* d_prio, const uint64_t* d_cand,
                    uint32_t flags, uint64_t* d_pass, int32_t* d_order, int32_t* d_len,
                    hipStream_t s) {
  const TasSnapshot& t = ctx->tas;
  const int32_t N = t.n_nodes, M = t.n_metrics;
  const int32_t W64 = (int32_t)w64(N);
  const int32_t S = (int32_t)((N + kSegPos - 1) / kSegPos);
  const int32_t D64 = S * kSegWords;
  const int32_t G = 3 * M;
  // LDS: misc | pass bitmap (2*W64 words) | drop bitmap (S segments x 32 words) | segk (S)
  const size_t filter_lds = sizeof(uint32_t) * ((size_t)kMiscWords + 2 * (size_t)W64 +
                                                (size_t)S * kSegWords * 2 + (size_t)S);
  if (filter_lds > 160 * 1024)
    return set_error(ctx, PAS_ECAPACITY,
                     "pas_tas_eval: n_nodes too large for the LDS bitmaps (max ~620k nodes)");
  if (M > kMaxGroupMetrics)
    return set_error(ctx, PAS_ECAPACITY, "pas_tas_eval: more than 4096 metric columns");
  const bool prio = (flags & PAS_TAS_PRIORITIZE) != 0;

  // upper bound on emit segments: at most min(P, G) non-empty buckets of S segments
  const int64_t max_segs = prio ? (int64_t)std::min(n_pods, G) * S : 0;
  if (max_segs > INT32_MAX) return set_error(ctx, PAS_ECAPACITY, "pas_tas_eval: batch too large");

  // scratch: ranges | pod_list | group_start | seg_start | seg_group | seg_base | drop | desc
  //          | keys
  const size_t sizes[9] = {
      align256(sizeof(int2) * (size_t)std::max(n_rules, 1)),
      align256(sizeof(int32_t) * (size_t)n_pods),
      align256(sizeof(int32_t) * (size_t)(G + 2)),
      align256(sizeof(int32_t) * (size_t)(G + 1)),
      align256(sizeof(int32_t) * (size_t)std::max<int64_t>(max_segs, 1)),
      prio ? align256(sizeof(int32_t) * (size_t)n_pods * S) : 0,
      prio ? align256(sizeof(uint64_t) * (size_t)n_pods * D64) : 0,
      align256(sizeof(int4) * 2 * (size_t)std::max(n_pods, 1)),
      align256(sizeof(int2) * (size_t)std::max(n_pods, 1))};
  size_t need = 0;
  for (size_t b : sizes) need += b;
  if (need > ctx->aux_bytes) {
    if (ctx->aux) {
      PAS_HIP(ctx, hipStreamSynchronize(s));
      PAS_HIP(ctx, hipFree(ctx->aux));
      ctx->aux = nullptr;
      ctx->aux_bytes = 0;
    }
    PAS_HIP(ctx, hipMalloc(&ctx->aux, need));
    ctx->aux_bytes = need;
  }
  char* cur = static_cast<char*>(ctx->aux);
  char* parts[9];
  for (int i = 0; i < 9; ++i) {
    parts[i] = cur;
    cur += sizes[i];
  }
  int2* d_ranges = reinterpret_cast<int2*>(parts[0]);
  int32_t* d_list = reinterpret_cast<int32_t*>(parts[1]);
  int32_t* d_gs = reinterpret_cast<int32_t*>(parts[2]);
  int32_t* d_ss = reinterpret_cast<int32_t*>(parts[3]);
  int32_t* d_sg = reinterpret_cast<int32_t*>(parts[4]);
  int32_t* d_sb = reinterpret_cast<int32_t*>(parts[5]);
  uint64_t* d_drop = reinterpret_cast<uint64_t*>(parts[6]);
  int4* d_desc = reinterpret_cast<int4*>(parts[7]);
  int2* d_keys = reinterpret_cast<int2*>(parts[8]);

  TimedLaunch span, tl;
  timing_begin(ctx, s, PAS_K_TAS_SPAN, &span);
  // ranges (blocks 1..) beside the grouping (block 0), one launch
  const int32_t range_rules = (flags & PAS_TAS_FILTER) ? n_rules : 0;
  RangesParams rp{range_rules, N, M, d_rules, t.cnt, t.sorted, d_ranges};
  GroupParams gp{n_pods, M,    N,    flags, d_prio, d_rule_off, t.cnt,
                 d_keys, d_list, d_gs, d_ss,  d_sg,   d_desc,     (int32_t)max_segs};
  const size_t group_lds = sizeof(int32_t) * ((size_t)kGroupTpb + G + 1);
  if (group_lds > 64 * 1024)
    PAS_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void*>(&tas_prep_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)group_lds));
  const unsigned prep_blocks = 1u + (unsigned)((range_rules + kGroupTpb - 1) / kGroupTpb);
  timing_begin(ctx, s, PAS_K_TAS_GROUP, &tl);
  tas_prep_kernel<<<prep_blocks, kGroupTpb, group_lds, s>>>(gp, rp);
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());

  FilterParams fp;
  fp.N = N;
  fp.M = M;
  fp.P = n_pods;
  fp.W32 = (int32_t)w32(N);
  fp.W32p = 2 * W64;
  fp.W64 = W64;
  fp.D64 = D64;
  fp.S = S;
  fp.Nr = t.rank_stride;
  fp.rank = t.rank;
  fp.phi = t.phi;
  fp.flags = flags;
  fp.ranges = d_ranges;
  fp.rules = d_rules;
  fp.cand = d_cand;
  fp.perm = t.perm;
  fp.pass_out = d_pass;
  fp.drop = d_drop;
  fp.seg_base = d_sb;
  fp.order_len = d_len;
  fp.desc = d_desc;
  if (filter_lds > 64 * 1024)
    for (const void* f : {reinterpret_cast<const void*>(&tas_filter_kernel<0>),
                          reinterpret_cast<const void*>(&tas_filter_kernel<1>),
                          reinterpret_cast<const void*>(&tas_filter_kernel<2>),
                          reinterpret_cast<const void*>(&tas_filter_kernel<4>),
                          reinterpret_cast<const void*>(&tas_filter_kernel<8>)})
      PAS_HIP(ctx, hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)filter_lds));
  timing_begin(ctx, s, PAS_K_TAS_FILTER, &tl);
  static const int filter_ablate = [] {
    const char* e = std::getenv("PAS_FILTER_ABLATE");
    return e ? std::atoi(e) : 0;
  }();
  const unsigned fblocks = (unsigned)n_pods;
  switch (filter_ablate) {
    case 1: tas_filter_kernel<1><<<fblocks, kTpb, filter_lds, s>>>(fp); break;
    case 2: tas_filter_kernel<2><<<fblocks, kTpb, filter_lds, s>>>(fp); break;
    case 4: tas_filter_kernel<4><<<fblocks, kTpb, filter_lds, s>>>(fp); break;
    case 8: tas_filter_kernel<8><<<fblocks, kTpb, filter_lds, s>>>(fp); break;
    default: tas_filter_kernel<0><<<fblocks, kTpb, filter_lds, s>>>(fp); break;
  }
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());

  if (prio) {
    const int64_t blocks = (max_segs + kWaves - 1) / kWaves;
    if (blocks > 0) {
      timing_begin(ctx, s, PAS_K_TAS_EMIT, &tl);
      static const int ablate = [] {
        const char* e = std::getenv("PAS_EMIT_ABLATE");
        return e ? std::atoi(e) : 0;
      }();
      if (ablate == 1)
        tas_emit_kernel<1><<<(unsigned)blocks, kTpb, 0, s>>>(N, M, D64, S, t.perm, t.cnt, d_list,
                                                             d_gs, d_ss, d_sg, d_drop, d_sb,
                                                             (int32_t)max_segs, d_order);
      else
        tas_emit_kernel<0><<<(unsigned)blocks, kTpb, 0, s>>>(N, M, D64, S, t.perm, t.cnt, d_list,
                                                             d_gs, d_ss, d_sg, d_drop, d_sb,
                                                             (int32_t)max_segs, d_order);
      timing_end(ctx, s, &tl);
      PAS_HIP(ctx, hipGetLastError());
    }
  }
  timing_end(ctx, s, &span);
  return PAS_OK;
}

int tas_violations_launch(pas_ctx* ctx, int32_t n_strat, const pas_rule* d_rules,
                          const int32_t* d_rule_off, uint64_t* d_viol, hipStream_t s) {
  const TasSnapshot& t = ctx->tas;
  const int32_t W64 = (int32_t)w64(t.n_nodes);
  if (W64 == 0) return PAS_OK;
  TimedLaunch tl;
  timing_begin(ctx, s, PAS_K_TAS_VIOLATIONS, &tl);
  tas_violations_kernel<<<(W64 + kWaves - 1) / kWaves, kTpb, 0, s>>>(
      t.n_nodes, t.n_metrics, W64, n_strat, d_rule_off, d_rules, t.vals, t.present, d_viol);
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

}  // namespace pas
