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
// Device formulation (snapshot orders built by tas_snapshot.hip):
//   * rule -> range.  With the present values of metric m sorted ascending, the nodes
//     satisfying EvaluateRule (operator.go:13-26) form one contiguous range:
//       LessThan  t: [0, lower_bound(t*1000))     GreaterThan t: [upper_bound(t*1000), cnt)
//       Equals    t: [lower_bound, upper_bound)
//     (t*1000 saturates: above int64 every present value is LessThan, none is greater
//     or equal; symmetric below).  tas_ranges_kernel computes them for the batch.
//   * filter.  One workgroup per pod keeps a node-space pass bitmap in LDS (N bits),
//     initialised from the candidates, and clears the bit of every node listed in any
//     of the pod's rule ranges (perm_asc entries, read coalesced).  The bitmap is the
//     FilterResult (pass = candidate AND NOT violated).
//   * prioritize.  The order for the pod's scheduleonmetric rule (asc / desc / index) is
//     a fixed permutation of the metric's present nodes.  Every non-passing node is
//     mapped through that order's rank array into a "drop" bitmap over sorted positions
//     (LDS), the per-wave drop counts give each wave its output offset, and each wave
//     streams its slice of the permutation, writing kept entries with mbcnt compaction.
//     HBM traffic per pod: N/8 B of pass bitmap + 4 B per listed node written, the
//     permutation read (L2/MALL-resident, shared by all pods with the same metric/order).
#include <hip/hip_runtime.h>

#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;
constexpr int kWaves = kTpb / 64;
constexpr int kRuleChunk = 64;
// LDS words reserved in front of the two bitmaps (rule chunk tables + wave counts),
// a multiple of 4 so the bitmaps stay 16-byte aligned (cdna_hip_programming G17).
constexpr int kMiscWords = 4 * kRuleChunk + 16;

struct EvalParams {
  int32_t N;
  int32_t M;
  int32_t W32;   // ceil(N / 32)
  int32_t W32p;  // 2 * W64: words per LDS bitmap
  int32_t W64;
  uint32_t flags;
  const int32_t* rule_off;
  const int2* ranges;
  const pas_rule* rules;
  const pas_rule* prio;
  const uint64_t* cand;
  const int32_t* perm;   // [3][M][N]
  const uint32_t* rank;  // [3][M][N]
  const int32_t* cnt;    // [M]
  uint64_t* pass_out;
  int32_t* order_out;
  int32_t* order_len;
};

__device__ __forceinline__ uint32_t tail_mask32(int32_t w, int32_t n) {
  const int32_t lo = w * 32;
  if (lo >= n) return 0u;
  if (lo + 32 <= n) return 0xFFFFFFFFu;
  return (1u << (n - lo)) - 1u;
}

__device__ __forceinline__ uint64_t tail_mask64(int32_t c, int32_t n) {
  const int32_t lo = c * 64;
  if (lo >= n) return 0ull;
  if (lo + 64 <= n) return ~0ull;
  return (1ull << (n - lo)) - 1ull;
}

// Binary search bounds over ascending sorted values.
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

// target * 1000 with saturation: sat = +1 (above every int64 milli value), -1 (below
// every value) or 0 with *tm exact.
__device__ __forceinline__ int target_milli(int64_t t, int64_t* tm) {
  constexpr int64_t kMax = INT64_MAX / 1000;
  constexpr int64_t kMin = INT64_MIN / 1000;
  if (t > kMax) return 1;
  if (t < kMin) return -1;
  *tm = t * 1000;
  return 0;
}

// One thread per rule: its violating range in the metric's ascending order.
__global__ void tas_ranges_kernel(int32_t n_rules, const pas_rule* __restrict__ rules,
                                  const int32_t* __restrict__ cnt,
                                  const int64_t* __restrict__ sorted, int32_t N, int32_t M,
                                  int2* __restrict__ ranges) {
  const int32_t r = blockIdx.x * kTpb + threadIdx.x;
  if (r >= n_rules) return;
  const pas_rule rule = rules[r];
  int2 out = make_int2(0, 0);
  if (rule.metric >= 0 && rule.metric < M && rule.op >= 0 && rule.op <= 2) {
    const int32_t c = cnt[rule.metric];
    const int64_t* sv = sorted + (int64_t)rule.metric * N;
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
  ranges[r] = out;
}

__global__ __launch_bounds__(kTpb) void tas_eval_kernel(EvalParams P) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  int32_t* s_pref = reinterpret_cast<int32_t*>(lds);          // [kRuleChunk + 1]
  int32_t* s_lo = s_pref + (kRuleChunk + 4);                  // [kRuleChunk]
  int32_t* s_m = s_lo + kRuleChunk;                           // [kRuleChunk]
  int32_t* s_wdrop = s_m + kRuleChunk;                        // [kWaves]
  uint32_t* pass = lds + kMiscWords;                          // [W32p]
  uint32_t* drop = pass + P.W32p;                             // [W32p]

  const int32_t pod = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int32_t N = P.N;

  // ---- candidates -> pass bitmap (args.Nodes.Items, telemetryscheduler.go:204) ----
  const uint32_t* cand32 =
      P.cand ? reinterpret_cast<const uint32_t*>(P.cand + (int64_t)pod * P.W64) : nullptr;
  for (int32_t w = tid; w < P.W32p; w += kTpb) {
    const uint32_t x = cand32 ? cand32[w] : 0xFFFFFFFFu;
    pass[w] = x & tail_mask32(w, N);
  }
  __syncthreads();

  // ---- dontschedule.Violated: clear every node in any rule range ----
  if (P.flags & PAS_TAS_FILTER) {
    const int32_t r0 = P.rule_off[pod], r1 = P.rule_off[pod + 1];
    const int32_t* perm_asc = P.perm + (int64_t)kOrderAsc * P.M * N;
    for (int32_t c0 = r0; c0 < r1; c0 += kRuleChunk) {
      const int32_t nr = min(kRuleChunk, r1 - c0);
      if (tid < nr) {
        const int2 rg = P.ranges[c0 + tid];
        s_lo[tid] = rg.x;
        s_pref[tid + 1] = rg.y - rg.x;
        const int32_t m = P.rules[c0 + tid].metric;
        s_m[tid] = (m >= 0 && m < P.M) ? m : 0;
      }
      __syncthreads();
      if (tid == 0) {
        s_pref[0] = 0;
        for (int32_t i = 0; i < nr; ++i) s_pref[i + 1] += s_pref[i];
      }
      __syncthreads();
      const int32_t total = s_pref[nr];
      int32_t r = 0;
      constexpr int U = 8;
      for (int32_t base = tid; base < total; base += kTpb * U) {
        int32_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int32_t f = base + u * kTpb;
          v[u] = -1;
          if (f < total) {
            while (s_pref[r + 1] <= f) ++r;
            v[u] = perm_asc[(int64_t)s_m[r] * N + s_lo[r] + (f - s_pref[r])];
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (v[u] >= 0) atomicAnd(&pass[v[u] >> 5], ~(1u << (v[u] & 31)));
      }
      __syncthreads();
    }
    uint64_t* out = P.pass_out + (int64_t)pod * P.W64;
    for (int32_t w = tid; w < P.W64; w += kTpb)
      out[w] = (uint64_t)pass[2 * w] | ((uint64_t)pass[2 * w + 1] << 32);
  }

  if (!(P.flags & PAS_TAS_PRIORITIZE)) return;

  // ---- prioritizeNodesForRule over the candidates that passed ----
  const pas_rule pr = P.prio[pod];
  const int32_t m0 = pr.metric;
  const int32_t cnt0 = (m0 >= 0 && m0 < P.M) ? P.cnt[m0] : 0;
  if (cnt0 == 0) {  // no rule / ReadMetric error -> empty HostPriorityList (:92-96)
    if (tid == 0) P.order_len[pod] = 0;
    return;
  }
  const int order = pr.op == PAS_OP_GREATER_THAN ? kOrderDesc
                    : pr.op == PAS_OP_LESS_THAN  ? kOrderAsc
                                                 : kOrderIndex;
  const int64_t col = ((int64_t)order * P.M + m0) * N;
  const int32_t* __restrict__ pm = P.perm + col;
  const uint32_t* __restrict__ rk = P.rank + col;
  const int32_t C64 = (cnt0 + 63) / 64;
  for (int32_t w = tid; w < 2 * C64; w += kTpb) drop[w] = 0u;
  __syncthreads();

  // Map every non-passing node to its position in the order (4 gathers in flight).
  for (int32_t w = tid; w < P.W32; w += kTpb) {
    uint32_t z = ~pass[w] & tail_mask32(w, N);
    while (z) {
      int32_t n0 = -1, n1 = -1, n2 = -1, n3 = -1;
      n0 = w * 32 + __ffs(z) - 1; z &= z - 1;
      if (z) { n1 = w * 32 + __ffs(z) - 1; z &= z - 1; }
      if (z) { n2 = w * 32 + __ffs(z) - 1; z &= z - 1; }
      if (z) { n3 = w * 32 + __ffs(z) - 1; z &= z - 1; }
      const uint32_t q0 = rk[n0];
      const uint32_t q1 = n1 >= 0 ? rk[n1] : kNoRank;
      const uint32_t q2 = n2 >= 0 ? rk[n2] : kNoRank;
      const uint32_t q3 = n3 >= 0 ? rk[n3] : kNoRank;
      if (q0 != kNoRank) atomicOr(&drop[q0 >> 5], 1u << (q0 & 31));
      if (q1 != kNoRank) atomicOr(&drop[q1 >> 5], 1u << (q1 & 31));
      if (q2 != kNoRank) atomicOr(&drop[q2 >> 5], 1u << (q2 & 31));
      if (q3 != kNoRank) atomicOr(&drop[q3 >> 5], 1u << (q3 & 31));
    }
  }
  __syncthreads();

  // Each wave owns a contiguous run of 64-position chunks of the order.
  const int32_t per = (C64 + kWaves - 1) / kWaves;
  const int32_t c_begin = min(C64, wave * per);
  const int32_t c_end = min(C64, c_begin + per);
  const uint64_t* drop64 = reinterpret_cast<const uint64_t*>(drop);
  int32_t dropped = 0;
  for (int32_t c = c_begin + lane; c < c_end; c += 64)
    dropped += __popcll(drop64[c] & tail_mask64(c, cnt0));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) dropped += __shfl_xor(dropped, off, 64);
  if (lane == 0) s_wdrop[wave] = dropped;
  __syncthreads();
  int32_t drops_before = 0, drops_total = 0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) {
    drops_total += s_wdrop[i];
    if (i < wave) drops_before += s_wdrop[i];
  }
  int32_t* __restrict__ out = P.order_out + (int64_t)pod * N;
  int32_t base = c_begin * 64 - drops_before;
#pragma unroll 4
  for (int32_t c = c_begin; c < c_end; ++c) {
    const int32_t k = c * 64 + lane;
    const uint64_t keep = ~drop64[c] & tail_mask64(c, cnt0);
    const int32_t node = k < cnt0 ? pm[k] : 0;
    const uint32_t below = __builtin_amdgcn_mbcnt_hi(
        (uint32_t)(keep >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)keep, 0u));
    if ((keep >> lane) & 1ull) out[base + (int32_t)below] = node;
    base += __popcll(keep);
  }
  if (tid == 0) P.order_len[pod] = cnt0 - drops_total;
}

// Deschedule sweep: one wave per 64-node word, strategies x rules in the wave loop.
// deschedule.Strategy.Violated (deschedule/strategy.go:31-50) per registered strategy,
// as nodeStatusForStrategy does (deschedule/enforce.go:154-164).
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

}  // namespace

int tas_eval_launch(pas_ctx* ctx, int32_t n_pods, int32_t n_rules, const pas_rule* d_rules,
                    const int32_t* d_rule_off, const pas_rule* d_prio, const uint64_t* d_cand,
                    uint32_t flags, uint64_t* d_pass, int32_t* d_order, int32_t* d_len,
                    hipStream_t s) {
  const TasSnapshot& t = ctx->tas;
  const int32_t N = t.n_nodes, M = t.n_metrics;
  const int32_t W64 = (int32_t)w64(N);
  const size_t lds_bytes = sizeof(uint32_t) * ((size_t)kMiscWords + 4 * (size_t)W64);
  if (lds_bytes > 160 * 1024)
    return set_error(ctx, PAS_ECAPACITY,
                     "pas_tas_eval: n_nodes too large for the LDS bitmaps (max ~620k nodes)");
  // rule ranges live in a context-owned buffer that grows with the rule count
  const size_t need = sizeof(int2) * (size_t)std::max(n_rules, 1);
  if (need > ctx->aux_bytes) {
    if (ctx->aux) {
      PAS_HIP(ctx, hipStreamSynchronize(s));
      PAS_HIP(ctx, hipFree(ctx->aux));
      ctx->aux = nullptr;
      ctx->aux_bytes = 0;
    }
    PAS_HIP(ctx, hipMalloc(&ctx->aux, need * 2));
    ctx->aux_bytes = need * 2;
  }
  int2* d_ranges = static_cast<int2*>(ctx->aux);
  TimedLaunch tl;
  if ((flags & PAS_TAS_FILTER) && n_rules > 0) {
    timing_begin(ctx, s, PAS_K_TAS_RANGES, &tl);
    tas_ranges_kernel<<<(n_rules + kTpb - 1) / kTpb, kTpb, 0, s>>>(n_rules, d_rules, t.cnt,
                                                                   t.sorted, N, M, d_ranges);
    timing_end(ctx, s, &tl);
    PAS_HIP(ctx, hipGetLastError());
  }
  EvalParams p;
  p.N = N;
  p.M = M;
  p.W32 = (int32_t)w32(N);
  p.W32p = 2 * W64;
  p.W64 = W64;
  p.flags = flags;
  p.rule_off = d_rule_off;
  p.ranges = d_ranges;
  p.rules = d_rules;
  p.prio = d_prio;
  p.cand = d_cand;
  p.perm = t.perm;
  p.rank = t.rank;
  p.cnt = t.cnt;
  p.pass_out = d_pass;
  p.order_out = d_order;
  p.order_len = d_len;
  if (lds_bytes > 64 * 1024)
    PAS_HIP(ctx, hipFuncSetAttribute(reinterpret_cast<const void*>(&tas_eval_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds_bytes));
  timing_begin(ctx, s, PAS_K_TAS_EVAL, &tl);
  tas_eval_kernel<<<n_pods, kTpb, lds_bytes, s>>>(p);
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
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
