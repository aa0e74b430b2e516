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
//   K prep    (a) rule -> range.  With the present values of metric m sorted ascending,
//             the nodes satisfying EvaluateRule (operator.go:13-26) form one contiguous
//             range:  LessThan t: [0, lower_bound(t*1000))   GreaterThan t:
//             [upper_bound(t*1000), cnt)   Equals t: [lower_bound, upper_bound)
//             (t*1000 saturates: above int64 every present value is LessThan, none is
//             greater or equal; symmetric below).
//             (b) pods bucketed by their prioritize order (metric, asc/desc/index), so
//             pods streaming the same order row run back to back on one XCD.
//   K eval    one workgroup per pod: a node-space pass bitmap in LDS (candidates, then
//             every node of every rule range cleared; this is the FilterResult), then the
//             pod's order row walked in 1024-position segments and compacted by the pass
//             bits into the ordered host list.  The path is bound by the HBM writes of
//             the ordered lists.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kRuleChunk = 64;
constexpr int kSegWords = 16;             // 64-position words per order segment
constexpr int kSegPos = kSegWords * 64;   // 1024 order positions per segment
constexpr int kGroupTpb = 1024;
constexpr int kMaxGroupMetrics = 4096;    // 3 * M + 1 buckets in LDS for the grouping
// LDS words in front of the pass bitmap (rule chunk table, round counts), a multiple of 4
// so the bitmap stays 16-byte aligned (cdna_hip_programming G17).
constexpr int kMiscWords = 4 * kRuleChunk + 16;
constexpr int kStageWords = ((kSegPos + 31 + 255) / 256) * 256;  // 5 x 256 (b128 reads)
constexpr int kDumpSlot = kStageWords - 1;  // compaction target of dropped lanes (> 1055)
constexpr int kNtAux = 18;  // whole-line store cache policy: sc1 nt (streamed out, not kept in L2)
static_assert(kSegPos == kOrderPad, "order rows are padded by one segment");

typedef int32_t v4i32 __attribute__((ext_vector_type(4)));
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;

__device__ __forceinline__ uint64_t tail_mask64(int32_t c, int32_t n) {
  const int32_t lo = c * 64;
  if (lo >= n) return 0ull;
  if (lo + 64 <= n) return ~0ull;
  return (1ull << (n - lo)) - 1ull;
}

__device__ __forceinline__ int order_of(int32_t op) {
  return op == PAS_OP_GREATER_THAN ? kOrderDesc : op == PAS_OP_LESS_THAN ? kOrderAsc : kOrderIndex;
}

__device__ __forceinline__ int32_t wave_inclusive_sum(int32_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  return x;
}

// Exclusive scan of a[0..n) in LDS by wave 0 of the block (each lane a contiguous run of
// ceil(n / 64) entries), then a block barrier.
__device__ void block_exclusive_scan(int32_t* a, int32_t n) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int32_t per = (n + 63) / 64;
    const int32_t lo = min(n, lane * per), hi = min(n, lo + per);
    int32_t sum = 0;
    for (int32_t i = lo; i < hi; ++i) sum += a[i];
    int32_t run = wave_inclusive_sum(sum) - sum;
    for (int32_t i = lo; i < hi; ++i) {
      const int32_t v = a[i];
      a[i] = run;
      run += v;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------- prep
#ifndef PAS_PREP_STAMPS
#define PAS_PREP_STAMPS 0  // diagnostic builds: phase times of the prep (printf, 100 MHz ticks)
#endif
//
// One launch, two roles: block 0 groups the pods (below); blocks 1.. map every rule to its
// range (a3).  The two are independent, so the binary searches run beside the grouping.

struct RangesParams {
  int32_t n_rules, M;
  int32_t R;  // order row stride
  const pas_rule* rules;
  const int32_t* cnt;
  const int64_t* sorted;  // [M][R]
  const int64_t* f1k;     // [M][R / 1024] sorted[m][1024 a]
  const int64_t* f32;     // [M][R / 32]   sorted[m][32 b]
  int2* ranges;
  const int64_t* scale_tab;  // [M][2] the columns' fixed point (target_scaled)
};

constexpr int kRuleLanes = 8;  // lanes per rule in the range search

// Numbers of entries of a[0..n) below t (cl: v < t) and not above t (cu: v <= t), for an
// ascending a, counted by the rule's lane group (gl = lane within the group, gmask = the
// group's lanes) with every load of the window in flight at once.
template <int kMaxPerLane>
__device__ __forceinline__ void count_below(const int64_t* __restrict__ al, int32_t nl,
                                            const int64_t* __restrict__ au, int32_t nu,
                                            int64_t t, int gl, uint64_t gmask, int32_t* cl,
                                            int32_t* cu) {
  int32_t sl = 0, su = 0;
#pragma unroll
  for (int q = 0; q < kMaxPerLane; ++q) {
    const int32_t i = gl + q * kRuleLanes;
    const int64_t vl = al[min(i, max(nl - 1, 0))];
    const int64_t vu = au[min(i, max(nu - 1, 0))];
    sl += __popcll(__ballot(i < nl && vl < t) & gmask);
    su += __popcll(__ballot(i < nu && vu <= t) & gmask);
  }
  *cl = sl;
  *cu = su;
}

// EvaluateRule (operator.go:13-26) over the ascending column: the nodes a rule selects form
// one range, [lower_bound, upper_bound) of t*1000 for Equals, the prefix below it for
// LessThan, the suffix above it for GreaterThan (t*1000 saturates).  A group
// of 8 lanes per rule finds both bounds in three dependent rounds of loads: the 1024-stride
// fences (f1k), the 32-stride fences of one 1024-block (f32), the 32 values of one
// 32-block; each round counts the window's entries below the target.
__device__ void ranges_group(const RangesParams& R, int32_t r) {
  const int lane = threadIdx.x & 63, gl = lane & (kRuleLanes - 1);
  const uint64_t gmask = 0xFFull << (lane & ~(kRuleLanes - 1));
  const pas_rule rule = R.rules[r];
  int2 out = make_int2(0, 0);
  if (rule.metric >= 0 && rule.metric < R.M && rule.op >= 0 && rule.op <= 2) {
    const int32_t m = rule.metric;
    const int32_t c = R.cnt[m];
    int64_t t = 0;
    const int sat = target_scaled(rule.target, R.scale_tab, m, &t);
    int32_t lb, ub;
    if (sat != 0) {
      lb = ub = sat > 0 ? c : 0;
    } else {
      const int64_t* sv = R.sorted + (int64_t)m * R.R;
      const int64_t* f1 = R.f1k + (int64_t)m * (R.R >> 10);
      const int64_t* f2 = R.f32 + (int64_t)m * (R.R >> 5);
      const int32_t na = (c + 1023) >> 10, nb = (c + 31) >> 5;
      int32_t n1l = 0, n1u = 0;  // fences (1024 apart) below the target
      if (na <= 16 * kRuleLanes) {  // up to 131 072 nodes: every fence load in flight at once
        count_below<16>(f1, na, f1, na, t, gl, gmask, &n1l, &n1u);
      } else {
        for (int32_t i0 = 0; i0 < na; i0 += 4 * kRuleLanes) {
          int32_t a, b;
          count_below<4>(f1 + i0, na - i0, f1 + i0, na - i0, t, gl, gmask, &a, &b);
          n1l += a;
          n1u += b;
        }
      }
      // 1024-blocks holding each bound (sorted[1024 b1] is below; block 0 if none is)
      const int32_t b1l = max(n1l - 1, 0), b1u = max(n1u - 1, 0);
      int32_t n2l, n2u;
      count_below<4>(f2 + b1l * 32, n1l ? min(32, nb - b1l * 32) : 0, f2 + b1u * 32,
                     n1u ? min(32, nb - b1u * 32) : 0, t, gl, gmask, &n2l, &n2u);
      const int32_t b2l = b1l * 32 + max(n2l - 1, 0), b2u = b1u * 32 + max(n2u - 1, 0);
      int32_t n3l, n3u;
      count_below<4>(sv + b2l * 32, n1l ? min(32, c - b2l * 32) : 0, sv + b2u * 32,
                     n1u ? min(32, c - b2u * 32) : 0, t, gl, gmask, &n3l, &n3u);
      lb = n1l ? b2l * 32 + n3l : 0;
      ub = n1u ? b2u * 32 + n3u : 0;
    }
    if (rule.op == PAS_OP_LESS_THAN) out = make_int2(0, lb);
    else if (rule.op == PAS_OP_GREATER_THAN) out = make_int2(ub, c);
    else out = make_int2(lb, ub);
  }
  if (gl == 0) R.ranges[r] = out;
}

struct GroupParams {
  int32_t P, M;
  uint32_t flags;
  const pas_rule* prio;
  const int32_t* rule_off;
  const int32_t* cnt;
  int2* keys;   // [P] scratch: {bucket, cnt0} of each pod
  int4* desc;   // [2P] per bucketed position: {pod, ocol, cnt0, 0}, {r0, r1, 0, 0}
  int32_t no_group;
  int32_t n_rules;
};

// Pod / strategy i's rule span from a device rule_off (the _device entry points cannot check
// it on the host): clamped into [0, n_rules] and non-decreasing, so that an offset array that
// is not a CSR never indexes past the rules (what is computed for it is unspecified).
__device__ __forceinline__ int2 rule_span(const int32_t* off, int32_t i, int32_t n_rules) {
  const int32_t a = min(max(off[i], 0), n_rules);
  return make_int2(a, min(max(off[i + 1], a), n_rules));
}

constexpr int kGU = 4;  // pods per thread per round of loads (all issued before use)

// Counting sort of the pods by bucket = order column (order * M + metric) of the pod's
// prioritize list, or G when it has none (no PRIORITIZE flag, metric out of range, or a
// metric no node reports: the ReadMetric error of prioritizeNodesForRule,
// telemetryscheduler.go:92-96).  Writes the per-position pod descriptors the eval kernel
// reads with one load.  Loads are unconditional (clamped indices) so that each round's
// are in flight together.
__device__ void group_body(const GroupParams& g, int32_t* sh) {
  const int32_t G = 3 * g.M;
  int32_t* hist = sh;  // [G + 1]
  const int tid = threadIdx.x;
  const bool prio = (g.flags & PAS_TAS_PRIORITIZE) != 0 && g.M > 0;
  for (int32_t i = tid; i <= G; i += kGroupTpb) hist[i] = 0;
  const bool filt = (g.flags & PAS_TAS_FILTER) != 0;
#if PAS_PREP_STAMPS
  uint64_t st[6];
  st[0] = __builtin_amdgcn_s_memrealtime();
#define PAS_STAMP(i) st[i] = __builtin_amdgcn_s_memrealtime()
#else
#define PAS_STAMP(i)
#endif
  if (g.P > 0 && g.P <= kGroupTpb * kGU && g.M <= kGroupTpb) {
    // one round: every load of the pods (prioritize rule, rule offsets) in flight together,
    // the keys kept in registers between the histogram and the scatter
    // the per-metric node counts staged in LDS (after the histogram) with the same round
    int32_t* cnt = sh + G + 1;
    pas_rule r[kGU];
    int32_t c[kGU], r0[kGU], r1[kGU], key[kGU];
#pragma unroll
    for (int u = 0; u < kGU; ++u) {
      const int32_t pc = min(tid + u * kGroupTpb, g.P - 1);
      r[u] = prio ? g.prio[pc] : pas_rule{-1, 0, 0};
      const int2 sp = filt ? rule_span(g.rule_off, pc, g.n_rules) : make_int2(0, 0);
      r0[u] = sp.x;
      r1[u] = sp.y;
    }
    if (tid < g.M) cnt[tid] = g.cnt[tid];
    __syncthreads();
    PAS_STAMP(1);
#pragma unroll
    for (int u = 0; u < kGU; ++u) c[u] = prio ? cnt[min(max(r[u].metric, 0), g.M - 1)] : 0;
#pragma unroll
    for (int u = 0; u < kGU; ++u) {
      const bool listed = prio && r[u].metric >= 0 && r[u].metric < g.M && c[u] > 0;
      key[u] = listed ? order_of(r[u].op) * g.M + r[u].metric : G;
      c[u] = listed ? c[u] : 0;
      if (tid + u * kGroupTpb < g.P) atomicAdd(&hist[key[u]], 1);
    }
    __syncthreads();
    PAS_STAMP(2);
    block_exclusive_scan(hist, G + 1);
    PAS_STAMP(3);
#pragma unroll
    for (int u = 0; u < kGU; ++u) {
      const int32_t p = tid + u * kGroupTpb;
      if (p >= g.P) continue;
      int32_t pos = atomicAdd(&hist[key[u]], 1);  // order inside a bucket is free
      if (g.no_group) pos = p;
      g.desc[2 * pos] = make_int4(p, key[u] < G ? key[u] : -1, c[u], 0);
      g.desc[2 * pos + 1] = make_int4(r0[u], r1[u], 0, 0);
    }
#if PAS_PREP_STAMPS
    PAS_STAMP(4);
    __syncthreads();
    __builtin_amdgcn_s_waitcnt(0);
    PAS_STAMP(5);
    if (tid == 0)
      printf("STAMP group load %d hist %d scan %d scatter %d drain %d\n", (int)(st[1] - st[0]),
             (int)(st[2] - st[1]), (int)(st[3] - st[2]), (int)(st[4] - st[3]),
             (int)(st[5] - st[4]));
#endif
    return;
  }
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
  block_exclusive_scan(hist, G + 1);
  for (int32_t p0 = tid; p0 < g.P; p0 += kGroupTpb * kGU) {
    int2 kc[kGU];
    int32_t r0[kGU], r1[kGU];
#pragma unroll
    for (int u = 0; u < kGU; ++u) {
      const int32_t p = min(p0 + u * kGroupTpb, g.P - 1);
      kc[u] = g.keys[p];
      const int2 sp = filt ? rule_span(g.rule_off, p, g.n_rules) : make_int2(0, 0);
      r0[u] = sp.x;
      r1[u] = sp.y;
    }
#pragma unroll
    for (int u = 0; u < kGU; ++u) {
      const int32_t p = p0 + u * kGroupTpb;
      if (p >= g.P) continue;
      const int32_t key = kc[u].x, c0 = kc[u].y;
      int32_t pos = atomicAdd(&hist[key], 1);  // order inside a bucket is free
      if (g.no_group) pos = p;
      g.desc[2 * pos] = make_int4(p, key < G ? key : -1, c0, 0);
      g.desc[2 * pos + 1] = make_int4(r0[u], r1[u], 0, 0);
    }
  }
}

// PAS_PREP_ABLATE (compile time, diagnostic timing builds only; outputs wrong): 1 = no
// ranges, 2 = no grouping.  The product library is built with 0.
#ifndef PAS_PREP_ABLATE
#define PAS_PREP_ABLATE 0
#endif
__global__ __launch_bounds__(kGroupTpb) void tas_prep_kernel(GroupParams g, RangesParams R) {
  extern __shared__ __attribute__((aligned(16))) int32_t sh[];
#if PAS_PREP_STAMPS
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == 1 || blockIdx.x == gridDim.x - 1))
    printf("STAMP start block %d t %llu\n", (int)blockIdx.x, (unsigned long long)t_start);
#endif
  if (blockIdx.x == 0) {
    if (!(PAS_PREP_ABLATE & 2)) group_body(g, sh);
    return;
  }
  if (PAS_PREP_ABLATE & 1) return;
  const int32_t r =
      (int32_t)(blockIdx.x - 1) * (kGroupTpb / kRuleLanes) + (int32_t)(threadIdx.x / kRuleLanes);
  if (r < R.n_rules) ranges_group(R, r);
#if PAS_PREP_STAMPS
  __syncthreads();
  if (threadIdx.x == 0 && (blockIdx.x == 1 || blockIdx.x == gridDim.x - 1))
    printf("STAMP ranges block %d took %d end %llu\n", (int)blockIdx.x,
           (int)(__builtin_amdgcn_s_memrealtime() - t_start),
           (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
}

// ---------------------------------------------------------------------------- eval


// Barrier over the block's waves that orders LDS only: outstanding global loads and stores
// stay in flight across it (a __syncthreads would wait for them; vmcnt counts stores).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// One wave writes the kept entries of a 1024-position order segment, in position order, to
// order_out[gdst ..): node[j] holds positions j*64 + lane, keep[j] (wave-uniform) their keep
// bits.  Compaction into a wave-private LDS stage aligned to the destination's 128-byte
// lines: per j one mbcnt pair (k + kept lanes below), a select of the dump slot for dropped
// lanes, one unconditional LDS write.  Stores: the whole lines of the run with nt 16-byte
// stores, the partial head and tail lines with one dword store each.  Every store is
// unconditional and range-checked against a buffer descriptor of exactly its part of the
// run (out-of-range lanes store nothing), so there are no per-lane predicates; a call with
// no kept entries issues the same 7 stores and writes nothing.  kmax caps the entries
// stored (top-k lists).
template <int kAux>
__device__ __forceinline__ void compact_store(int32_t* stage, uint32_t stage_off,
                                              const int32_t (&node)[kSegWords],
                                              const uint64_t (&keep)[kSegWords],
                                              int32_t* order_out, int64_t gdst, int lane,
                                              int32_t kmax = kSegPos) {
  const int32_t a = (int32_t)(gdst & 31);  // stage offset: 128-B line alignment
  int32_t k = a;
#pragma unroll
  for (int j = 0; j < kSegWords; ++j) {
    const uint32_t pos = __builtin_amdgcn_mbcnt_hi(
        (uint32_t)(keep[j] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)keep[j], (uint32_t)k));
    uint32_t slot;  // per-lane select on the SGPR keep mask: k + below, or the dump slot
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(slot) : "v"(kDumpSlot), "v"(pos), "s"(keep[j]));
    *(lds_u32*)(size_t)(stage_off + slot * 4u) = (uint32_t)node[j];
    k += __popcll(keep[j]);
  }
  __builtin_amdgcn_wave_barrier();
  k = min(k, a + kmax);  // top-k: only the first kmax kept entries are stored
  int32_t* const line0 = order_out + (gdst - a);  // 128-B aligned
  const int32_t full_lo = (a + 31) & ~31;         // first entry of the first whole line
  const int32_t full_hi = max(k & ~31, full_lo);  // end of the last whole line
  const int32_t head_end = min(full_lo, k);
  const int32_t tail_lo = max(full_hi, head_end);
  constexpr int kChunkIters = kStageWords / 256;
  v4i32 v[kChunkIters];
#pragma unroll
  for (int it = 0; it < kChunkIters; ++it)
    v[it] = *reinterpret_cast<const v4i32*>(stage + (lane + it * 64) * 4);
  const int32_t hv = stage[a + lane];
  const int32_t tv = stage[tail_lo + lane];
  const __amdgpu_buffer_rsrc_t mid =
      __builtin_amdgcn_make_buffer_rsrc(line0 + full_lo, 0, (full_hi - full_lo) * 4, 0x00020000);
  const uint32_t moff = (uint32_t)(lane * 16 - full_lo * 4);  // < 0 wraps: out of range
#pragma unroll
  for (int it = 0; it < kChunkIters; ++it)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v[it]), mid,
                                           moff + it * 1024, 0, kAux);
  const __amdgpu_buffer_rsrc_t head =
      __builtin_amdgcn_make_buffer_rsrc(line0 + a, 0, (head_end - a) * 4, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32((uint32_t)hv, head, lane * 4, 0, 0);
  const __amdgpu_buffer_rsrc_t tail =
      __builtin_amdgcn_make_buffer_rsrc(line0 + tail_lo, 0, max(k - tail_lo, 0) * 4, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32((uint32_t)tv, tail, lane * 4, 0, 0);
  __builtin_amdgcn_wave_barrier();  // the next segment rewrites the stage
}

struct EvalParams {
  int32_t N, M;
  int32_t R;         // order row stride (snapshot)
  int32_t W64;
  int32_t W32p;      // words of the LDS pass bitmap: 2 * W64 + a zero word for the sentinel
  uint32_t flags;
  const int2* ranges;
  const pas_rule* rules;
  const uint64_t* cand;
  const int32_t* perm;   // [3][M][R]
  const int4* desc;      // [2P] from the prep kernel
  uint64_t* pass_out;    // [P][W64]
  int32_t* order_out;    // [P][out_stride]
  int32_t* order_len;    // [P]
  int32_t topk;          // 0: whole HostPriorityList; else its first topk entries
  int32_t out_stride;    // N, or topk
  int32_t pos_base;      // first bucketed position of this launch
  uint32_t* gpass;       // kGP: [grid][W32p] pass bitmaps in global scratch
};

// One workgroup of kW waves per pod, XCD-aware over the bucketed pod list (blocks b and b+8
// share an XCD, MI355X_MICROARCH.md; each XCD takes a contiguous run of the list, so pods
// streaming the same order row read it from one L2):
//   A. dontschedule.Violated + filterNodes (telemetryscheduler.go:184-225): candidates into
//      an LDS pass bitmap over node ids, then every node of every rule range cleared (range
//      reads of perm_asc, 16 in flight per thread, LDS atomicAnd);
//   B. prioritizeNodesForRule / OrderedList (telemetryscheduler.go:128-149,
//      operator.go:30-42): the pod's order row (metric m in ascending / descending / node
//      order) is walked in 1024-position segments, one per wave per round; a position's
//      node is kept iff its pass bit is set (failing nodes and non-candidates drop out;
//      padding positions hold a sentinel node whose bit is always clear), the round's kept
//      counts are exchanged through LDS for the output bases, and each wave writes its
//      segment's kept nodes with compact_store.  The next round's segment is loaded before
//      the exchange, and the exchange orders LDS only, so loads and stores stay in flight
//      across rounds;
//   C. FilterResult row -> HBM, HostPriorityList length.
// kS: adjacent segments per wave per round.  kAblate (diagnostic timing builds only: the
// compile-time PAS_EVAL_ABLATE, 0 in the product library; outputs wrong): 1 = no stores,
// 2 = no count exchange, 4 = no pass-bit lookups, 8 = no rule loop.
// kGP (clusters past the LDS pass bitmap, ~1.1M nodes): the pod's pass bitmap lives in a
// global scratch row instead (P.gpass, one row per workgroup of the launch; lookups are
// workgroup-coherent loads, clears are L2 atomics) — the same algorithm, slower lookups.
template <int kW, int kS, int kAblate, int kAux = kNtAux, bool kGP = false>
__global__ __launch_bounds__(kW * 64) void tas_eval_kernel(EvalParams P) {
  constexpr int T = kW * 64;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  int32_t* s_pref = reinterpret_cast<int32_t*>(lds);  // [kRuleChunk] prefix of range lengths
  int32_t* s_base = s_pref + kRuleChunk;              // [kRuleChunk] perm index of range start
  int32_t* s_total = s_base + kRuleChunk;             // [1]
  int32_t* s_cnt = s_total + 16;                      // [2][kW] kept counts per round
  const int32_t nb = gridDim.x, b = blockIdx.x;
  const int32_t xcd = b & 7, per_xcd = nb >> 3, rem = nb & 7;
  const int32_t slot = xcd * per_xcd + min(xcd, rem) + (b >> 3);
  const int32_t pos = P.pos_base + slot;
  uint32_t* pass = kGP ? P.gpass + (int64_t)slot * P.W32p : lds + kMiscWords;  // [W32p]
  uint64_t* pass64 = reinterpret_cast<uint64_t*>(pass);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform, in an SGPR
  const int lane = threadIdx.x & 63, tid = threadIdx.x;
  int32_t* stage =
      reinterpret_cast<int32_t*>(kGP ? lds + kMiscWords : pass + P.W32p) + wave * kStageWords;
  const uint32_t pass_off = kGP ? 0u : (uint32_t)(size_t)(lds_u32*)pass;  // LDS byte offsets
  const uint32_t stage_off = (uint32_t)(size_t)(lds_u32*)stage;

  const int4 d0 = P.desc[2 * pos], d1 = P.desc[2 * pos + 1];
  // block-uniform, kept in SGPRs (the output descriptors built from them must be scalar)
  const int32_t pod = __builtin_amdgcn_readfirstlane(d0.x);
  const int32_t ocol = __builtin_amdgcn_readfirstlane(d0.y);
  const int32_t cnt0 = __builtin_amdgcn_readfirstlane(d0.z);
  const int32_t r0 = __builtin_amdgcn_readfirstlane(d1.x);
  const int32_t r1 = __builtin_amdgcn_readfirstlane(d1.y);
  const int32_t N = P.N, W64 = P.W64;
  const bool has_list = ocol >= 0 && (P.flags & PAS_TAS_PRIORITIZE);

  // ---- A1. candidates -> pass bitmap (args.Nodes.Items, telemetryscheduler.go:204) ----
  constexpr int kCU = 8;
  const uint64_t* __restrict__ cand = P.cand ? P.cand + (int64_t)pod * W64 : nullptr;
  for (int32_t w0 = tid; w0 < W64; w0 += T * kCU) {
    uint64_t x[kCU];
#pragma unroll
    for (int u = 0; u < kCU; ++u) x[u] = cand ? cand[min(w0 + u * T, W64 - 1)] : ~0ull;
#pragma unroll
    for (int u = 0; u < kCU; ++u) {
      const int32_t w = w0 + u * T;
      if (w < W64) pass64[w] = x[u] & tail_mask64(w, N);
    }
  }
  for (int32_t w = 2 * W64 + tid; w < P.W32p; w += T) pass[w] = 0u;  // sentinel word
  __syncthreads();

  // ---- A2. dontschedule.Violated: every node of every rule range fails the filter ----
  if ((P.flags & PAS_TAS_FILTER) && !(kAblate & 8)) {
    const int32_t* perm_asc = P.perm + (int64_t)kOrderAsc * P.M * P.R;
    for (int32_t c0 = r0; c0 < r1; c0 += kRuleChunk) {
      const int32_t nr = min(kRuleChunk, r1 - c0);
      if (tid < 64) {  // wave 0: rule table = prefix of range lengths (largest-index search)
        int32_t len = 0, bse = 0;
        if (tid < nr) {
          const int2 rg = P.ranges[c0 + tid];
          const int32_t m = P.rules[c0 + tid].metric;
          len = rg.y - rg.x;
          bse = (m >= 0 && m < P.M) ? m * P.R + rg.x : 0;
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
      for (int32_t base = tid; base < total; base += T * U) {
        int32_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int32_t f = min(base + u * T, total - 1);
          int32_t r = 0;  // largest r with s_pref[r] <= f (zero-length ranges are skipped)
#pragma unroll
          for (int st = kRuleChunk / 2; st > 0; st >>= 1)
            r = s_pref[r + st] <= f ? r + st : r;
          v[u] = perm_asc[s_base[r] + (f - s_pref[r])];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) atomicAnd(&pass[v[u] >> 5], ~(1u << (v[u] & 31)));
      }
      __syncthreads();
    }
  }

  // ---- B. ordered list: compaction of the pod's order row by its pass bits ----
  int32_t running = 0;
  if (has_list) {
    const int32_t* __restrict__ pm = P.perm + (int64_t)ocol * P.R;
    const int32_t n_seg = (cnt0 + kSegPos - 1) / kSegPos;  // segment n_seg: all sentinel
    constexpr int kPerRound = kW * kS;  // a wave takes kS adjacent segments per round
    const int32_t rounds = (n_seg + kPerRound - 1) / kPerRound;
    const int32_t* __restrict__ lane_pm = pm + lane;
    int32_t node[kS][kSegWords];
    auto load_round = [&](int32_t (&dst)[kS][kSegWords], int32_t r) {
#pragma unroll
      for (int i = 0; i < kS; ++i) {
        const int32_t* src = lane_pm + min(r * kPerRound + wave * kS + i, n_seg) * kSegPos;
#pragma unroll
        for (int j = 0; j < kSegWords; ++j) dst[i][j] = src[j * 64];
      }
    };
    load_round(node, 0);
    {
      // The same stores as a round with nothing kept: the loop is then entered with the
      // memory-counter shape (segment loads, then the stores) of every later round, so the
      // compiler's waits for a segment never include a round's stores.
      uint64_t none[kSegWords];
#pragma unroll
      for (int j = 0; j < kSegWords; ++j) none[j] = 0;
#pragma unroll
      for (int i = 0; i < kS; ++i)
        compact_store<kAux>(stage, stage_off, node[i], none, P.order_out,
                            (int64_t)pod * P.out_stride, lane);
    }
    for (int32_t r = 0; r < rounds; ++r) {
      uint64_t keep[kS][kSegWords];
      int32_t cnt[kS];
#pragma unroll
      for (int i = 0; i < kS; ++i) {
        uint32_t w[kSegWords];
#pragma unroll
        for (int j = 0; j < kSegWords; ++j) {  // all 16 reads in flight
          uint32_t word;  // node >> 5 (bfe: the compiler's shift/mask/add form is longer)
          asm("v_bfe_u32 %0, %1, 5, 27" : "=v"(word) : "v"(node[i][j]));
          if constexpr (kGP)
            w[j] = __hip_atomic_load(pass + word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          else
            w[j] = (kAblate & 4) ? ~0u : *(lds_u32*)(size_t)(pass_off + word * 4u);
        }
        cnt[i] = 0;
#pragma unroll
        for (int j = 0; j < kSegWords; ++j) {
          keep[i][j] = __ballot(__builtin_amdgcn_ubfe(w[j], (uint32_t)node[i][j], 1u));
          cnt[i] += __popcll(keep[i][j]);
        }
      }
      int32_t nxt[kS][kSegWords];  // next round's segments, in flight across the exchange
      load_round(nxt, r + 1);
      int32_t mine = 0;
#pragma unroll
      for (int i = 0; i < kS; ++i) mine += cnt[i];
      int32_t base = running, tot = mine;  // wave-uniform: the stores' descriptors are scalar
      if (!(kAblate & 2)) {
        int32_t* cbuf = s_cnt + (r & 1) * kW;
        if (lane == 0) cbuf[wave] = mine;
        lds_barrier();
        tot = 0;
#pragma unroll
        for (int v = 0; v < kW; ++v) {
          const int32_t c = __builtin_amdgcn_readfirstlane(cbuf[v]);
          base += v < wave ? c : 0;
          tot += c;
        }
      }
      running += tot;
      // unconditional (an empty run stores nothing): a store under a branch would make the
      // next round's first use of a segment wait for every store of this round
#pragma unroll
      for (int i = 0; i < kS; ++i) {
        const int32_t kmax = P.topk ? max(P.topk - base, 0) : kSegPos;
        if (!(kAblate & 1))
          compact_store<kAux>(stage, stage_off, node[i], keep[i], P.order_out,
                              (int64_t)pod * P.out_stride + base, lane, kmax);
        base += cnt[i];
      }
      if (P.topk && running >= P.topk) break;  // uniform: every wave has the same running
#pragma unroll
      for (int i = 0; i < kS; ++i)
#pragma unroll
        for (int j = 0; j < kSegWords; ++j) node[i][j] = nxt[i][j];
    }
  }

  // ---- C. FilterResult row, HostPriorityList length ----
  if ((P.flags & PAS_TAS_FILTER) && P.pass_out) {
    uint64_t* pass_row = P.pass_out + (int64_t)pod * W64;
    for (int32_t w = tid; w < W64; w += T) pass_row[w] = pass64[w];
  }
  // no list: no rule / ReadMetric error -> empty HostPriorityList (telemetryscheduler.go:92-96)
  if (tid == 0 && (P.flags & PAS_TAS_PRIORITIZE))
    P.order_len[pod] = P.topk ? min(running, P.topk) : running;
}

// ---------------------------------------------------------------------------- deschedule

constexpr int kTpb = 256;
constexpr int kWaves = kTpb / 64;


// The sweep by column runs: a wave owns kRun consecutive 64-node words and walks the flat
// rule list one rule at a time, reading that rule's column over its words as one
// contiguous kRun * 512-byte run (every DRAM page it opens is read whole) while the next
// rule's run is already in flight.  Lane k keeps word k's violation mask of the open
// strategy (its presence word is lane k's own load); at a strategy's end lanes 0..kRun-1
// store its words with one coalesced store.
#ifndef PAS_VIOL_NT
#define PAS_VIOL_NT 1  // non-temporal column loads: each column byte is read once per sweep
#endif
// The label plan fused into the sweep (pas_tas_deschedule_device, deschedule/enforce.go:99-151,
// as label_plan_kernel in tas_labels.hip): the wave's carried-label words [S][kRun] are read
// into its LDS slice before the walk, a strategy's completed words go next to them, and after
// the walk lane l turns both into the masks of nodes (gw0 + k) * 64 + l, one word k at a time
// (bit s = bit l of word (s, k), from broadcast LDS reads; removes and the count are by policy
// name, NamePlan; the block stores its count of violated (node, name) pairs).  The run length
// is fixed at 8 words per wave here (PAS_VIOL_RUN tunes only the unfused sweep).
static_assert(kWaves == 4, "the plan's per-block count sums four waves");
struct PlanOut {
  NamePlan names;
  const uint64_t* labels;  // [S][W64] or null
  uint64_t* add;           // [N]
  uint64_t* rem;           // [N]
  int64_t* part;           // [gridDim.x] violated pairs per block
};

template <int kRun, bool kPlan = false>
__global__ __launch_bounds__(kTpb) void tas_violations_run_kernel(
    int32_t N, int32_t M, int32_t W64, int32_t n_strat, int32_t n_rules,
    const int32_t* __restrict__ rule_off,
    const pas_rule* __restrict__ rules, const int64_t* __restrict__ vals,
    const uint64_t* __restrict__ present, const int64_t* __restrict__ scale_tab,
    uint64_t* __restrict__ viol_out, PlanOut plan) {
  static_assert(kRun <= 64, "one word per lane");
  __shared__ int64_t red[kPlan ? kWaves : 1];
  __shared__ uint64_t vws[kPlan ? kWaves : 1][kPlan ? 64 : 1][kPlan ? kRun : 1];
  __shared__ uint64_t lws[kPlan ? kWaves : 1][kPlan ? 64 : 1][kPlan ? kRun : 1];
  const int32_t gw0 = (blockIdx.x * kWaves + (threadIdx.x >> 6)) * kRun;
  const int lane = threadIdx.x & 63;
  if (gw0 >= W64) {
    if constexpr (kPlan) {  // (a block's waves past the end still take part in its count)
      if (lane == 0) red[threadIdx.x >> 6] = 0;
      __syncthreads();
      if (threadIdx.x == 0) plan.part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
    }
    return;
  }
  const int32_t pw_lane = min(gw0 + lane, W64 - 1);
  // the offsets clamped into [0, n_rules] and non-decreasing (rule_span): strategy s ends at
  // or before r_end, so the walk below never passes strategy n_strat - 1
  const int32_t r_begin = min(max(rule_off[0], 0), n_rules);
  const int32_t r_end = min(max(rule_off[n_strat], r_begin), n_rules);
  int32_t s = 0;
  int32_t s_end = n_strat > 0 ? min(max(rule_off[1], r_begin), r_end) : 0;
  uint64_t acc = 0;  // lane k: word gw0 + k
  int64_t violated = 0;
  if constexpr (kPlan) {  // lane t: strategy t's carried-label words of this wave's run
    if (lane < n_strat) {
#pragma unroll
      for (int k = 0; k < kRun; ++k)
        lws[threadIdx.x >> 6][lane][k] =
            plan.labels ? plan.labels[(int64_t)lane * W64 + min(gw0 + k, W64 - 1)] : 0ull;
    }
  }
  auto flush = [&]() {
    if (lane < kRun && gw0 + lane < W64) viol_out[(int64_t)s * W64 + gw0 + lane] = acc;
    if constexpr (kPlan) {
      if (lane < kRun) vws[threadIdx.x >> 6][s][lane] = acc;
    }
    acc = 0;
  };
  // rule records arrive two rules ahead (scalar loads), so the column loads of the next rule
  // never wait for its record
  auto load = [&](const pas_rule& ru, int64_t (&v)[kRun], uint64_t* pr) {
    const int32_t m = (ru.metric >= 0 && ru.metric < M) ? ru.metric : 0;
    const int64_t* col = vals + (int64_t)m * N;
#pragma unroll
    for (int k = 0; k < kRun; ++k) {
      const int64_t* a = col + min((gw0 + k) * 64 + lane, N - 1);
      v[k] = PAS_VIOL_NT ? __builtin_nontemporal_load(a) : *a;
    }
    *pr = present[(int64_t)m * W64 + pw_lane];
  };
  pas_rule ru{}, ru1{};
  int64_t v[kRun];
  uint64_t pr = 0;
  if (r_begin < r_end) {  // (no rule records to read otherwise)
    ru = rules[r_begin];
    ru1 = rules[min(r_begin + 1, r_end - 1)];
    load(ru, v, &pr);
  }
  for (int32_t r = r_begin; r < r_end; ++r) {
    while (r >= s_end) {  // the list has passed strategy s: its words are complete
      flush();
      ++s;
      s_end = min(max(rule_off[s + 1], s_end), r_end);
    }
    const pas_rule ru2 = rules[min(r + 2, r_end - 1)];
    int64_t nv[kRun];
    uint64_t npr;
    load(ru1, nv, &npr);  // the next run in flight during this rule's compares
    if (ru.metric >= 0 && ru.metric < M && ru.op >= 0 && ru.op <= 2) {
      // the rule as the value range it hits, [lo, hi] (empty: lo > hi), once per rule: the
      // word loop is two compares per word, no branch on the operator
      int64_t tm = 0;
      const int sat = target_scaled(ru.target, scale_tab, ru.metric, &tm);
      int64_t lo = 1, hi = 0;
      if (ru.op == PAS_OP_LESS_THAN) {  // v < t
        if (sat > 0) lo = INT64_MIN, hi = INT64_MAX;
        else if (sat == 0 && tm != INT64_MIN) lo = INT64_MIN, hi = tm - 1;
      } else if (ru.op == PAS_OP_GREATER_THAN) {  // v > t
        if (sat < 0) lo = INT64_MIN, hi = INT64_MAX;
        else if (sat == 0 && tm != INT64_MAX) lo = tm + 1, hi = INT64_MAX;
      } else if (sat == 0) {  // v == t
        lo = hi = tm;
      }
#pragma unroll
      for (int k = 0; k < kRun; ++k) {
        const bool valid = (gw0 + k) * 64 + lane < N;
        const uint64_t mask = __ballot((v[k] >= lo) & (v[k] <= hi) & valid);
        acc = lane == k ? (acc | (mask & pr)) : acc;
      }
    }
    ru = ru1;
    ru1 = ru2;
    pr = npr;
#pragma unroll
    for (int k = 0; k < kRun; ++k) v[k] = nv[k];
  }
  for (; s < n_strat; ++s) flush();  // the last strategy with rules, then those without
  if constexpr (kPlan) {
    const uint64_t(*ws)[kRun] = vws[threadIdx.x >> 6];
    const uint64_t(*ls)[kRun] = lws[threadIdx.x >> 6];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    // bit l of a word: bit (l & 31) of its half l >> 5
    const bool hi = lane >= 32;
    const uint32_t sh = (uint32_t)lane & 31u;
    auto bit = [&](uint64_t w) { return ((hi ? (uint32_t)(w >> 32) : (uint32_t)w) >> sh) & 1u; };
    for (int k = 0; k < kRun; ++k) {
      uint32_t a[2] = {0u, 0u}, r[2] = {0u, 0u};
      for (int32_t t = 0; t < n_strat; ++t) {
        const int h = t >> 5;
        const uint32_t b = (uint32_t)t & 31u;
        a[h] |= bit(ws[t][k]) << b;
        r[h] |= bit(ls[t][k]) << b;
      }
      const int64_t n = (int64_t)(gw0 + k) * 64 + lane;
      if (n < N) {
        const uint64_t av = (uint64_t)a[1] << 32 | a[0], rv = (uint64_t)r[1] << 32 | r[0];
        const uint64_t vn = violated_names(plan.names, av);
        violated += __popcll(vn);
        plan.add[n] = av;
        plan.rem[n] = rv & plan.names.canon & ~vn;
      }
    }
    for (int off = 32; off > 0; off >>= 1) violated += __shfl_xor(violated, off, 64);
    if (lane == 0) red[threadIdx.x >> 6] = violated;
    __syncthreads();
    if (threadIdx.x == 0) plan.part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  }
}

size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

#ifndef PAS_EVAL_ABLATE
#define PAS_EVAL_ABLATE 0  // diagnostic timing builds only (outputs wrong); see tas_eval_kernel
#endif

// Launch shape of the eval kernel.  The PAS_EVAL_* environment overrides exist for tuning
// sweeps (scripts/tas_sweep.sh); every one of them leaves the outputs unchanged (launch
// shape, pod order across workgroups, store cache policy) — tests/test_env_knobs.py checks
// that.  Output-changing diagnostics (PAS_EVAL_ABLATE, PAS_PREP_ABLATE) are compile-time.
struct TasTuning {
  int32_t waves = 4;         // waves per eval workgroup (2, 4 or 8)
  int32_t seg_per_wave = 1;  // adjacent order segments per wave per round (1 or 2)
  int32_t no_group = 0;      // diagnostic: pods in index order (no XCD locality)
  int32_t store_aux = kNtAux;  // cache policy of the whole-line stores
};

const TasTuning& tas_tuning() {
  static const TasTuning t = [] {
    TasTuning x;
    const int w = env_int("PAS_EVAL_WAVES", x.waves);
    x.waves = w == 8 ? 8 : w == 2 ? 2 : 4;
    x.seg_per_wave = env_int("PAS_EVAL_SEGS", x.seg_per_wave) == 2 ? 2 : 1;
    x.no_group = env_int("PAS_EVAL_NOGROUP", 0);
    x.store_aux = env_int("PAS_EVAL_AUX", x.store_aux);
    return x;
  }();
  return t;
}

}  // namespace

int tas_eval_launch(pas_ctx* ctx, int32_t n_pods, int32_t n_rules, const pas_rule* d_rules,
                    const int32_t* d_rule_off, const pas_rule* d_prio, const uint64_t* d_cand,
                    uint32_t flags, uint64_t* d_pass, int32_t* d_order, int32_t* d_len,
                    int32_t topk, hipStream_t s) {
  const TasSnapshot& t = ctx->tas;
  const int32_t N = t.n_nodes, M = t.n_metrics;
  const int32_t W64 = (int32_t)w64(N);
  const int32_t G = 3 * M;
  const TasTuning& tune = tas_tuning();
  if (M > kMaxGroupMetrics)
    return set_error(ctx, PAS_ECAPACITY, "pas_tas_eval: more than 4096 metric columns");
  EvalParams ep;
  ep.N = N;
  ep.M = M;
  ep.R = t.row;
  ep.W64 = W64;
  ep.W32p = (2 * W64 + 1 + 3) & ~3;  // + the sentinel's zero word, 16-byte multiple
  size_t eval_lds =
      sizeof(uint32_t) * ((size_t)kMiscWords + ep.W32p + (size_t)tune.waves * kStageWords);
  // (kS segments of a wave share its stage: compact_store finishes with the stage first)
  // past ~1.1M nodes the pass bitmaps move to global scratch, launched in chunks of pods
  const bool global_pass = eval_lds > 160 * 1024 || env_int("PAS_EVAL_GLOBAL_PASS", 0);
  int32_t chunk = n_pods;
  size_t gpass_bytes = 0;
  if (global_pass) {
    eval_lds = sizeof(uint32_t) * ((size_t)kMiscWords + 4 * (size_t)kStageWords);
    const size_t row = sizeof(uint32_t) * (size_t)ep.W32p;
    chunk = (int32_t)std::max<size_t>(1, std::min<size_t>(n_pods, (256u << 20) / row));
    gpass_bytes = row * (size_t)chunk;  // the stream's slot buffer (below)
  }
  if (n_pods == 0) return PAS_OK;

  // scratch: ranges | desc | keys
  const size_t sizes[3] = {align256(sizeof(int2) * (size_t)std::max(n_rules, 1)),
                           align256(sizeof(int4) * 2 * (size_t)n_pods),
                           align256(sizeof(int2) * (size_t)n_pods)};
  const size_t need = sizes[0] + sizes[1] + sizes[2];
  // the stream's scratch slot: evals on two alternating streams (a pipeline of batches) run
  // beside each other, batch i + 1's prep under batch i's eval
  int rc = PAS_OK;
  AuxSlot* slot = aux_acquire(ctx, s, need, &rc);
  if (!slot) return rc;
  struct ReleaseOnExit {
    pas_ctx* c;
    AuxSlot* a;
    hipStream_t s;
    ~ReleaseOnExit() { aux_release(c, a, s); }
  } done{ctx, slot, s};
  // the global pass bitmaps are per stream too: evals on other streams may run beside this one
  void* gpass = nullptr;
  if (global_pass && !(gpass = slot_buf(ctx, slot, kBufGpass, gpass_bytes, s, &rc))) return rc;
  char* cur = static_cast<char*>(slot->p);
  int2* d_ranges = reinterpret_cast<int2*>(cur);
  int4* d_desc = reinterpret_cast<int4*>(cur + sizes[0]);
  int2* d_keys = reinterpret_cast<int2*>(cur + sizes[0] + sizes[1]);

  TimedLaunch span, tl;
  timing_begin(ctx, s, PAS_K_TAS_SPAN, &span);
  // ranges (blocks 1..) beside the grouping (block 0), one launch
  const int32_t range_rules = (flags & PAS_TAS_FILTER) ? n_rules : 0;
  RangesParams rp{range_rules, M, t.row, d_rules, t.cnt, t.sorted, t.f1k, t.f32, d_ranges,
                  t.scale_tab};
  GroupParams gp{n_pods, M,      flags,  d_prio,        d_rule_off,
                 t.cnt,  d_keys, d_desc, tune.no_group, std::max(n_rules, 0)};
  const size_t group_lds = sizeof(int32_t) * ((size_t)G + 1 + (size_t)M);  // hist | cnt
  if (group_lds > 64 * 1024)
    PAS_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void*>(&tas_prep_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)group_lds));
  constexpr int kRulesPerBlock = kGroupTpb / kRuleLanes;
  const unsigned prep_blocks =
      1u + (unsigned)((range_rules + kRulesPerBlock - 1) / kRulesPerBlock);
  timing_begin(ctx, s, PAS_K_TAS_PREP, &tl);
  tas_prep_kernel<<<prep_blocks, kGroupTpb, group_lds, s>>>(gp, rp);
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());

  ep.flags = flags;
  ep.ranges = d_ranges;
  ep.rules = d_rules;
  ep.cand = d_cand;
  ep.perm = t.perm;
  ep.desc = d_desc;
  ep.pass_out = d_pass;
  ep.order_out = d_order;
  ep.order_len = d_len;
  ep.topk = topk;
  ep.out_stride = topk ? topk : N;
  ep.pos_base = 0;
  ep.gpass = static_cast<uint32_t*>(gpass);
  using EvalFn = void (*)(EvalParams);
  constexpr int kA = PAS_EVAL_ABLATE;
  EvalFn fn = &tas_eval_kernel<4, 1, kA>;
#define PAS_EVAL_CASE(W, S) \
  if (tune.waves == W && tune.seg_per_wave == S) fn = &tas_eval_kernel<W, S, kA>;
  PAS_EVAL_CASE(4, 2) PAS_EVAL_CASE(8, 1) PAS_EVAL_CASE(8, 2) PAS_EVAL_CASE(2, 1)
  PAS_EVAL_CASE(2, 2)
#undef PAS_EVAL_CASE
  if (tune.store_aux == 0) fn = &tas_eval_kernel<4, 1, kA, 0>;
  if (tune.store_aux == 3) fn = &tas_eval_kernel<4, 1, kA, 3>;
  if (tune.store_aux == 16) fn = &tas_eval_kernel<4, 1, kA, 16>;
  if (tune.store_aux == 2) fn = &tas_eval_kernel<4, 1, kA, 2>;
  if (tune.store_aux == 19) fn = &tas_eval_kernel<4, 1, kA, 19>;
  if (global_pass) fn = &tas_eval_kernel<4, 1, kA, kNtAux, true>;
  const int32_t waves = global_pass ? 4 : tune.waves;
  if (eval_lds > 64 * 1024)
    PAS_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)eval_lds));
  timing_begin(ctx, s, PAS_K_TAS_EVAL, &tl);
  for (int32_t p0 = 0; p0 < n_pods; p0 += chunk) {
    ep.pos_base = p0;
    fn<<<(unsigned)std::min(chunk, n_pods - p0), (unsigned)(waves * 64), eval_lds, s>>>(ep);
  }
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  timing_end(ctx, s, &span);
  return PAS_OK;
}

int tas_group_launch(pas_ctx* ctx, int32_t n_pods, const pas_rule* d_prio,
                     const int32_t* d_rule_off, int4* d_desc, int2* d_keys, int32_t n_rules,
                     const pas_rule* d_rules, int2* d_ranges, hipStream_t s) {
  const TasSnapshot& t = ctx->tas;
  const int32_t M = t.n_metrics;
  if (M > kMaxGroupMetrics)
    return set_error(ctx, PAS_ECAPACITY, "more than 4096 metric columns");
  const uint32_t flags = PAS_TAS_FILTER | PAS_TAS_PRIORITIZE;
  const int32_t range_rules = d_ranges ? n_rules : 0;
  RangesParams rp{range_rules, M, t.row, d_rules, t.cnt, t.sorted, t.f1k, t.f32, d_ranges,
                  t.scale_tab};
  GroupParams gp{n_pods, M, flags, d_prio, d_rule_off, t.cnt, d_keys, d_desc, 0,
                 std::max(n_rules, 0)};
  const size_t group_lds = sizeof(int32_t) * ((size_t)3 * M + 1 + (size_t)M);
  if (group_lds > 64 * 1024)
    PAS_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void*>(&tas_prep_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)group_lds));
  constexpr int kRulesPerBlock = kGroupTpb / kRuleLanes;
  const unsigned blocks = 1u + (unsigned)((range_rules + kRulesPerBlock - 1) / kRulesPerBlock);
  tas_prep_kernel<<<blocks, kGroupTpb, group_lds, s>>>(gp, rp);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

int tas_violations_launch(pas_ctx* ctx, int32_t n_strat, int32_t n_rules,
                          const pas_rule* d_rules, const int32_t* d_rule_off, uint64_t* d_viol,
                          hipStream_t s) {
  const TasSnapshot& t = ctx->tas;
  const int32_t W64 = (int32_t)w64(t.n_nodes);
  if (W64 == 0) return PAS_OK;
  TimedLaunch tl;
  timing_begin(ctx, s, PAS_K_TAS_VIOLATIONS, &tl);
  // words per wave (an output-invariant tuning knob: PAS_VIOL_RUN = 2, 4, 8 or 16)
  static const int run = env_int("PAS_VIOL_RUN", 8);
  auto rfn = run == 2    ? &tas_violations_run_kernel<2>
             : run == 4  ? &tas_violations_run_kernel<4>
             : run == 16 ? &tas_violations_run_kernel<16>
                         : &tas_violations_run_kernel<8>;
  const int32_t per = (run == 2 || run == 4 || run == 16) ? run : 8;
  const int32_t rwaves = (W64 + per - 1) / per;
  rfn<<<(rwaves + kWaves - 1) / kWaves, kTpb, 0, s>>>(
      t.n_nodes, t.n_metrics, W64, n_strat, std::max(n_rules, 0), d_rule_off, d_rules, t.vals,
      t.present, t.scale_tab, d_viol, PlanOut{NamePlan{}, nullptr, nullptr, nullptr, nullptr});
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

int tas_deschedule_launch(pas_ctx* ctx, int32_t n_strat, int32_t n_rules,
                          const pas_rule* d_rules, const int32_t* d_rule_off, uint64_t* d_viol,
                          const NamePlan& names,
                          const uint64_t* d_labels, uint64_t* d_add, uint64_t* d_rem,
                          int64_t* d_total, hipStream_t s) {
  const TasSnapshot& t = ctx->tas;
  const int32_t N = t.n_nodes, W64 = (int32_t)w64(N);
  if (W64 == 0 || n_strat == 0) {  // no pairs: every mask 0, total 0
    if (N > 0) {
      PAS_HIP(ctx, hipMemsetAsync(d_add, 0, sizeof(uint64_t) * (size_t)N, s));
      PAS_HIP(ctx, hipMemsetAsync(d_rem, 0, sizeof(uint64_t) * (size_t)N, s));
    }
    return label_total_launch(ctx, 0, 0, nullptr, d_total, s);
  }
  constexpr int kRun = 8;
  const int32_t rwaves = (W64 + kRun - 1) / kRun;
  const int32_t blocks = (rwaves + kWaves - 1) / kWaves;
  // the per-block counts are the stream's slot buffer: sweeps on other streams may run beside
  int rc = PAS_OK;
  SlotScope sc(ctx, s, 0, &rc);
  if (!sc.slot) return rc;
  int64_t* part = static_cast<int64_t*>(
      slot_buf(ctx, sc.slot, kBufLabel, sizeof(int64_t) * (size_t)blocks, s, &rc));
  if (!part) return rc;
  TimedLaunch tl;
  timing_begin(ctx, s, PAS_K_TAS_VIOLATIONS, &tl);
  tas_violations_run_kernel<kRun, true><<<blocks, kTpb, 0, s>>>(
      N, t.n_metrics, W64, n_strat, std::max(n_rules, 0), d_rule_off, d_rules, t.vals, t.present,
      t.scale_tab, d_viol, PlanOut{names, d_labels, d_add, d_rem, part});
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  return label_total_launch(ctx, blocks, (int64_t)N * __builtin_popcountll(names.canon), part,
                            d_total, s);
}

}  // namespace pas
