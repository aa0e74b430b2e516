// gas_fit.hip — batched GAS filter: one runSchedulingLogic per (pod, node).
//
// Reference (gpu-aware-scheduling/pkg/gpuscheduler/scheduler.go):
//   runSchedulingLogic (:280-338): per container, getCardsForContainerGPURequest
//   (:200-257) loops gpuNum < numI915 over the node's cards in sort.Strings order and
//   takes the first card for which checkResourceCapacity (:341-383) holds, adding the
//   per-GPU request to that card's usage (addRM, resource_map.go:38-53), so later
//   selections of the same pod see it; no fit -> errWontFit.
//
// Device formulation: one lane per node holds the node's free capacity per card and kind,
//   free[k][q] = cap[q] - used[k][q]   if cap[q] > 0 and used[k][q] >= 0, else -1
// (cards in lexicographic order; missing cards -1), built once from the frozen snapshot
// (Cache.getNodeResourceStatus, node_resource_cache.go:474-491).  For a requested kind
// with need >= 0, checkResourceCapacity (:341-383) holds exactly when need <= free: a
// non-positive capacity or negative usage gives -1, and used + need overflowing int64
// means need > INT64_MAX - used >= free.  Taking a card (addRM) is free -= need.  A
// negative need on a requested kind fails every card (:343-347).
//
// The pod loop is wave-uniform (a lane per node, the pod's values broadcast).  The prep
// kernel files each pod under a list by selection count: one selection (the common case), two,
// three, four to eight (more: the generic kernel), and by the kind it may skip (below).
// Launches per fit: gas_prep_kernel (lists), gas_rank_prep_kernel (rank groups, below),
// gas_rfit_single_kernel (one-selection pods), gas_rfit_closed_kernel (two and three
// selections in closed form), gas_rfit_seq_kernel (four to eight in order),
// gas_fit_generic_kernel (shapes past 8 cards or 8 selections).  The three fit kernels run
// side by side: the closed-form one on the caller's stream, the single-selection (store-bound)
// and sequential ones on two side streams of the call's scratch slot, forked after the prep
// launches and joined before the generic kernel.
//
// Rank compression (the ranked fit section): every "need <= free" compare of a group of at
// most 127 thresholds becomes a compare of 7-bit ranks, four cards of one kind per 32-bit
// subtraction, exactly.
//
// Kind skipping (exact, decided per pod before the fit kernels): gmin[q] = the minimum of
// free[k][q] over every card of every labelled node of the snapshot (gas_minfree_kernel).
// When a pod's total take of kind q is <= gmin[q], no check of kind q can fail anywhere, so
// its compares are dropped: the prep kernel files the pod under list 1 + q (the lowest such
// kind) or list 0, and the fit kernels instantiate one body per list.  The last kind a
// selection requests stays compared, so cards a node does not have (free -1) still fail.  In
// the C3 mix the i915 kind (1 per selection against >= 30 free) goes.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "gas_runs.h"
#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;
#ifndef PAS_GAS_SEQ_TPB
#define PAS_GAS_SEQ_TPB 128  // threads per block of the sequential kernel (two waves: its 10 KB
                             // per wave of LDS then fits the CUs the other two fit kernels leave;
                             // C3 0.687-0.691 -> 0.665-0.672 ms against 256, 0.692-0.696 at 64)
#endif
constexpr int kSeqTpb = PAS_GAS_SEQ_TPB;
#ifndef PAS_GAS_CLOSED_TPB
#define PAS_GAS_CLOSED_TPB 256  // threads per block of the closed-form kernel (128: C3 0.670 ->
                                // 0.698-0.700 ms, 64: 0.700-0.702)
#endif
constexpr int kClosedTpb = PAS_GAS_CLOSED_TPB;
#ifndef PAS_GAS_SINGLE_TPB
#define PAS_GAS_SINGLE_TPB 256  // threads per block of the single-selection kernel (128: C3
                                // 0.665-0.671 -> 0.759-0.763 ms)
#endif
constexpr int kSingleTpb = PAS_GAS_SINGLE_TPB;
#ifndef PAS_GAS_SPIN_SYNC
#define PAS_GAS_SPIN_SYNC 1  // 1: fork / join the fit's side streams with device flags (0: events)
#endif
#ifndef PAS_GAS_FAULT_INJECTION
// 1: the fault-injection build (lib/libpas_fault.so): PAS_GAS_FORCE_TIMEOUT=n makes the next
// n fits' side-stream waits give up at once, to test that the call then fails loudly
#define PAS_GAS_FAULT_INJECTION 0
#endif
#ifndef PAS_GAS_SEQ_FIRST
#define PAS_GAS_SEQ_FIRST 0  // 1: the sequential kernel before the closed-form one (diagnostic)
#endif
#ifndef PAS_GAS_BLOCKS_SINGLE
#define PAS_GAS_BLOCKS_SINGLE 8192  // target blocks of a fit grid: (node block, pod chunk) pairs
#endif
#ifndef PAS_GAS_BLOCKS_MULTI
#define PAS_GAS_BLOCKS_MULTI 8192
#endif
#ifndef PAS_GAS_BLOCKS_SEQ
#define PAS_GAS_BLOCKS_SEQ PAS_GAS_BLOCKS_MULTI  // target blocks of the sequential kernel's grid
                                                // (2 048 / 4 096 / 16 384: within +-1 %)
#endif
constexpr int kPrepTpb = 64;  // pods per prep block: small blocks spread the pods over the CUs
constexpr int kMaxCards = PAS_GAS_PACKED;  // cards of a fast-path node, in registers
constexpr int kPacked = PAS_GAS_PACKED;    // selections of a fast-path pod
// Multi-selection pods are listed by class (each class has its own loop in a fit kernel, so
// no per-pod dispatch on S): S = 2, S = 3 (closed form, gas_rfit_closed_kernel), S >= 4 in
// order, and S = 4 in closed form (lists with a skipped kind; gas_rfit_seq_kernel, rfour).
constexpr int kClasses = 4;
constexpr int kClsSeq = 2, kClsFour = 3;

// A (pod, container) step, in compare form: cmp[q] = per-GPU need of a requested kind
// (getPerGPUResourceRequest :180-190), INT64_MIN for the others, so every card passes them
// and the check needs no mask; take[q] = the need, 0 for the others (addRM).
struct alignas(16) GasStep {
  int64_t cmp[PAS_GAS_MAX_RES];
  int64_t take[PAS_GAS_MAX_RES];
  int32_t num_i915;  // getNumI915 (:192-198); 0 = no selection (skipped, :206-208, :215)
  int32_t bad;       // a requested kind has a negative per-GPU need (:343-347)
  int32_t kinds;     // bit q: kind q requested
  int32_t pad;
};

// One card selection of a pod with several, per kind q: {cmp, -take} (kinds as GasStep: the
// need of a requested kind, INT64_MIN / 0 for the others), one 16-byte load per kind.
struct alignas(16) GasSel {
  int64_t ct[PAS_GAS_MAX_RES][2];
};
// A pod with 2 or 3 selections is resolved in closed form from threshold compares on the
// snapshot free values (see rclosed): threshold j per kind, in compare form (INT64_MIN
// for kinds the selection does not request).  The 7 thresholds of a 3-selection pod:
//   0: n0   1: n1   2: n1 + t0   3: n2   4: n2 + t0   5: n2 + t1   6: n2 + t0 + t1
// (n = the selection's need, t = an earlier selection's take); a 2-selection pod uses 0-2.
// over bit j: threshold j overflows int64, so no card can pass it (:367-371).
struct alignas(16) GasThresholds {
  int64_t th[7][PAS_GAS_MAX_RES];
  int32_t over;
  int32_t pad[7];
};
// A multi-selection pod's row: its selections as GasSel (rows 0 .. S-1); a pod with 2 or 3
// selections also has its thresholds from row kThRow on.
constexpr int kThRow = 4;
static_assert(sizeof(GasThresholds) <= sizeof(GasSel) * (kPacked - kThRow), "row");
// A pod with 4 selections in a list with a skipped kind (class kClsFour) has a row of its 15
// thresholds instead (no GasSel rows): row (t, m) = 2^t - 1 + m for selection t and the set m
// of earlier selections (bit s: selection s) whose takes sit on the card,
//   0: n0  1: n1  2: n1+t0  3: n2  4: n2+t0  5: n2+t1  6: n2+t0+t1  7: n3  8: n3+t0  9: n3+t1
//   10: n3+t0+t1  11: n3+t2  12: n3+t0+t2  13: n3+t1+t2  14: n3+t0+t1+t2.
// flags: bit r row r overflows int64 (bit 0 also: a bad pod); bit 16 + t (t = 1..3) selection
// t's need equals selection t - 1's (the kernel reuses the mask).
struct alignas(16) GasFour {
  int64_t th[15][PAS_GAS_MAX_RES];
  int32_t flags;
  int32_t pad[3];
};
static_assert(sizeof(GasFour) <= sizeof(GasSel) * kPacked, "row");
constexpr int kFourSame = 16;  // GasFour::flags: first "same" bit (selection t at bit 16 + t)
constexpr int32_t kBadPod = 1 << 30;  // multi-list word flag: a selection has a negative need

// Pod with at most one card selection: its selecting step (compare form), and
// word = pod | steps << 24 | bad << 30 (steps 0: no selection, fits every labelled node).
struct alignas(16) GasSingle {
  int64_t cmp[PAS_GAS_MAX_RES];
  int32_t word;
  int32_t pad[3];
};

// getPerGPUResourceRequest: copy the container's map and, when numI915 > 1, divide
// every entry (the i915 entry included) by numI915, truncating (resource_map.go:129-145).
// A container's request row: mask and values, every load unconditional (clamped to the row),
// so they arrive together.
struct ContainerReq {
  uint32_t m;
  int64_t rv[PAS_GAS_MAX_RES];
};
__device__ __forceinline__ ContainerReq load_container(int64_t i, int32_t n_res,
                                                       const int64_t* __restrict__ req,
                                                       const uint32_t* __restrict__ mask) {
  ContainerReq c;
  c.m = mask[i];
#pragma unroll
  for (int q = 0; q < PAS_GAS_MAX_RES; ++q) c.rv[q] = req[i * n_res + min(q, n_res - 1)];
  return c;
}

// v / ni truncated toward zero (Go's int64 division), ni > 1: 32-bit unsigned division when
// both fit (the common case), else the 64-bit one.
__device__ __forceinline__ int64_t per_gpu(int64_t v, int64_t ni) {
  if (v >= 0 && v <= (int64_t)UINT32_MAX && ni <= (int64_t)UINT32_MAX)
    return (int64_t)((uint32_t)v / (uint32_t)ni);
  return v / ni;
}

__device__ GasStep container_step(const ContainerReq& cr, int32_t n_res, int32_t i915) {
  const uint32_t m = cr.m;
  const int64_t(&rv)[PAS_GAS_MAX_RES] = cr.rv;
  int64_t ni = 0;
#pragma unroll
  for (int q = 0; q < PAS_GAS_MAX_RES; ++q)
    if (q == i915 && ((m >> q) & 1u) && rv[q] > 0) ni = rv[q];
  GasStep g = {};
  g.num_i915 = m != 0u ? (int32_t)min(ni, (int64_t)PAS_GAS_MAX_SELECTIONS + 1) : 0;
  g.kinds = (int32_t)(m & ((1u << n_res) - 1u));
  g.bad = (m & PAS_REQ_UNKNOWN_KIND) ? 1 : 0;  // a key no capacity map has (:349-354)
#pragma unroll
  for (int q = 0; q < PAS_GAS_MAX_RES; ++q) {
    const bool has = q < n_res && ((m >> q) & 1u);
    int64_t v = has ? rv[q] : 0;
    if (ni > 1) v = per_gpu(v, ni);
    if (has && v < 0) g.bad = 1;
    g.take[q] = v;
    g.cmp[q] = has ? v : INT64_MIN;
  }
  return g;
}

// The list a single-selection pod is filed under: 1 + q for the lowest kind q whose need is
// within gmin[q] (every real card of every node has that much free, so the compare always
// holds), else 0.  The last kind the selection requests is kept: cards a node does not have
// read free = -1 and must keep failing.  A bad selection fails in any list.
__device__ __forceinline__ int32_t skip_list(int32_t n_res, const int64_t (&cmp)[PAS_GAS_MAX_RES],
                                             uint32_t kinds, const int64_t (&gmin)[PAS_GAS_MAX_RES]) {
  int32_t l = 0;
#pragma unroll
  for (int q = PAS_GAS_MAX_RES - 1; q >= 0; --q) {  // the lowest such kind wins
    if (q >= n_res || !((kinds >> q) & 1u) || kinds == (1u << q)) continue;
    if (cmp[q] <= gmin[q]) l = 1 + q;
  }
  return l;
}

// A slot in list `list` for each active lane: one atomic per distinct list in the wave (lanes
// of different lists hit different counters, which the compiler would leave one per lane).
// The lists are counted first (ballots only); then each list's leader lane issues its atomic,
// all of them in one instruction: one round trip to L2 instead of one per distinct list.
__device__ __forceinline__ int32_t wave_slot(int32_t* __restrict__ counts, int32_t list) {
  unsigned long long todo = __ballot(1);
  const int lane = (int)__lane_id();
  int32_t local = 0, my_leader = 0, lead_cnt = 0;
  while (todo) {
    const int leader = __builtin_ctzll(todo);
    const int32_t l = __shfl(list, leader, 64);
    const unsigned long long m = __ballot(list == l);
    if (list == l) {
      local = (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      my_leader = leader;
    }
    if (lane == leader) lead_cnt = __popcll(m);
    todo &= ~m;
  }
  int32_t base = 0;
  if (lead_cnt > 0) base = atomicAdd(&counts[list], lead_cnt);  // leaders: own list
  return __shfl(base, my_leader, 64) + local;
}

// The list a multi-selection pod is filed under: 1 + q for the lowest kind q that some
// selection requests and whose compares can be dropped: the pod's total take of q is at most
// gmin[q], so any selection's need plus any earlier takes on a card stays within every real
// card's snapshot free; and every selection requesting q requests another kind too (cards a
// node does not have must keep failing).  Else 0.
__device__ __forceinline__ int32_t multi_skip_list(int32_t n_res, uint32_t ok_mask,
                                                   uint32_t req_mask) {
  const uint32_t m = ok_mask & req_mask & ((1u << n_res) - 1u);
  return m ? 1 + __builtin_ctz(m) : 0;
}

// A fit kernel whose fork wait gave up returns at entry: its prep lists may be unwritten (the
// call reports PAS_EDEVICE, gas_fault_check).
__device__ __forceinline__ bool fit_aborted(const uint32_t* abort, uint32_t epoch) {
  return abort && __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
}

// One thread per pod files it under `single` (<= 1 selection: its selecting step, in the
// list of its skippable kind; lists [n_res + 1][n_pods]) or `multi` (several: lists
// [n_res + 1][kClasses][n_pods] of words pod | S << 24, by skippable kind as multi_skip_list
// and by class: S = 2, S = 3, S >= 4 in order, S = 4 in closed form); a multi pod's selections (containers in order, then gpuNum)
// go to the row sels[list][slot][8] of its list position.  pod_steps saturates at
// PAS_GAS_MAX_SELECTIONS + 1 (such pods only go to the generic path).  counts: [n_res + 1] single lists, then [n_res + 1][kClasses] multi lists.
struct PrepArgs {
  int32_t n_pods, max_containers, n_res, i915;
  const int64_t* req;
  const uint32_t* mask;
  const int32_t* n_containers;
  const unsigned long long* gflip;
  GasSingle* single;
  int32_t* multi;
  GasSel* sels;
  int32_t* counts;
  int32_t* big_pods;
  int32_t* n_big_pods;
  int32_t* pod_steps;
  int32_t* counts_next;
  int32_t n_counts;
  int64_t* limit_count;
  int64_t* side_count;
  uint32_t* start;  // device flags: set to the fit's epoch when the prep starts (null: events)
  uint32_t epoch;
};

// Block 0 of the prep zeroes the next fit's counts and this fit's generic-kernel counters
// (read after the prep in stream order), in place of fill launches.
template <int TPB>
__device__ __forceinline__ void prep_zero(const PrepArgs& a) {
  for (int32_t i = threadIdx.x; i < a.n_counts; i += TPB) a.counts_next[i] = 0;
  if (threadIdx.x == 0) {
    *a.limit_count = 0;
    if (a.side_count) *a.side_count = 0;
  }
}

__device__ __forceinline__ void prep_pod(const PrepArgs& a, const int32_t p) {
  const int32_t n_pods = a.n_pods, max_containers = a.max_containers, n_res = a.n_res,
                i915 = a.i915;
  const int64_t* __restrict__ req = a.req;
  const uint32_t* __restrict__ mask = a.mask;
  const int32_t* __restrict__ n_containers = a.n_containers;
  const unsigned long long* __restrict__ gflip = a.gflip;
  GasSingle* __restrict__ single = a.single;
  int32_t* __restrict__ multi = a.multi;
  GasSel* __restrict__ sels = a.sels;
  int32_t* __restrict__ counts = a.counts;
  int32_t* __restrict__ big_pods = a.big_pods;
  int32_t* __restrict__ n_big_pods = a.n_big_pods;
  int32_t* __restrict__ pod_steps = a.pod_steps;
  if (p >= n_pods) return;
  const int32_t nc = min(max(n_containers[p], 0), max_containers);
  const int64_t row = (int64_t)p * max_containers;
  // the first kPre containers' requests loaded at once (one memory latency, not one per
  // container and pass); containers past them are loaded when reached
  constexpr int kPre = 4;
  ContainerReq pre[kPre] = {};
  // (indexed by max_containers, not nc, so that they do not wait for n_containers[p]; entries
  // past nc are never used)
  if (max_containers > 0) {
#pragma unroll
    for (int c = 0; c < kPre; ++c)
      pre[c] = load_container(row + min(c, max_containers - 1), n_res, req, mask);
  }
  // their steps, once; both passes below run unrolled over them (a runtime container index
  // into these arrays would put them in scratch memory), then over containers past them
  GasStep pst[kPre];
#pragma unroll
  for (int c = 0; c < kPre; ++c) pst[c] = container_step(pre[c], n_res, i915);
  auto each_container = [&](auto&& fn) {
#pragma unroll
    for (int c = 0; c < kPre; ++c)
      if (c < nc) fn(pst[c]);
    for (int32_t c = kPre; c < nc; ++c)
      fn(container_step(load_container(row + c, n_res, req, mask), n_res, i915));
  };
  // the kind minima (kept flipped in gflip, gas_minfree_kernel)
  int64_t gmin[PAS_GAS_MAX_RES];
#pragma unroll
  for (int q = 0; q < PAS_GAS_MAX_RES; ++q)
    gmin[q] = q < n_res ? (int64_t)((unsigned long long)INT64_MAX - gflip[q]) : INT64_MAX;
  int32_t steps = 0;
  uint32_t kinds = 0;
  uint32_t skip_ok = (1u << n_res) - 1u, skip_req = 0;  // multi_skip_list
  int64_t cum[PAS_GAS_MAX_RES] = {};                     // the pod's total take per kind
  GasSingle one = {};
  int32_t one_bad = 0;
  each_container([&](const GasStep& g) {
    if (g.num_i915 > 0) {
      if (steps == 0) {
#pragma unroll
        for (int q = 0; q < PAS_GAS_MAX_RES; ++q) one.cmp[q] = g.cmp[q];
        one_bad = g.bad;
        kinds = g.kinds;
      }
      steps = min(steps + g.num_i915, PAS_GAS_MAX_SELECTIONS + 1);
      const uint32_t gk = (uint32_t)g.kinds;
      skip_req |= gk;
#pragma unroll
      for (int q = 0; q < PAS_GAS_MAX_RES; ++q) {
        if (q >= n_res || !((gk >> q) & 1u)) continue;
        // num_i915 takes, saturating: a total past INT64_MAX only has to exceed every gmin
        const int64_t add = g.take[q] > 0 ? g.take[q] : 0;
        int64_t prod;
        const bool ovf = __builtin_mul_overflow(add, (int64_t)g.num_i915, &prod);
        cum[q] = (ovf || prod > INT64_MAX - cum[q]) ? INT64_MAX : cum[q] + prod;
        if (gk == (1u << q)) skip_ok &= ~(1u << q);
      }
    }
  });
#pragma unroll
  for (int q = 0; q < PAS_GAS_MAX_RES; ++q)
    if (q < n_res && cum[q] > gmin[q]) skip_ok &= ~(1u << q);
  pod_steps[p] = steps;
  const bool one_sel = steps <= 1;
  const int32_t l = one_sel ? (steps == 1 ? skip_list(n_res, one.cmp, kinds, gmin) : 0)
                            : multi_skip_list(n_res, skip_ok, skip_req);
  const int32_t nl = n_res + 1;
  // four selections in closed form on the ranked lists (a skipped kind), else in order
  const bool four = steps == 4 && l > 0;
  const int32_t ml =
      l * kClasses + (steps == 2 ? 0 : steps == 3 ? 1 : four ? kClsFour : kClsSeq);  // multi list
  const int32_t slot = wave_slot(counts, one_sel ? l : nl + ml);
  if (one_sel) {
    one.word = p | (steps << 24) | (one_bad ? kBadPod : 0);
    // no selection: threshold INT64_MIN in every kind, so its group rank is 1 everywhere and
    // the ranked kernel's mask is non-empty exactly on the nodes that fit (a node without
    // cards has rank 0 in every card); its word is then node_ok as the reference's (:206-215)
    if (steps == 0)
#pragma unroll
      for (int q = 0; q < PAS_GAS_MAX_RES; ++q) one.cmp[q] = INT64_MIN;
    single[(int64_t)l * n_pods + slot] = one;
    return;
  }
  if (steps > kPacked) {  // gas_fit_generic_kernel; the fast kernel writes 0 first
    multi[(int64_t)ml * n_pods + slot] = p | ((kPacked + 1) << 24);
    big_pods[atomicAdd(n_big_pods, 1)] = p;
    return;
  }
  // the pod's row sits at its list position, so a batch of a list is one contiguous copy
  GasSel* out = sels + ((int64_t)ml * n_pods + slot) * kPacked;
  int32_t k = 0, bad = 0;
  // the first four selections in named registers (a runtime-indexed array would live in
  // scratch memory)
  int64_t cmp0[PAS_GAS_MAX_RES], cmp1[PAS_GAS_MAX_RES], cmp2[PAS_GAS_MAX_RES];
  int64_t cmp3[PAS_GAS_MAX_RES];
  int64_t take0[PAS_GAS_MAX_RES], take1[PAS_GAS_MAX_RES], take2[PAS_GAS_MAX_RES];
#pragma unroll
  for (int q = 0; q < PAS_GAS_MAX_RES; ++q)
    cmp0[q] = cmp1[q] = cmp2[q] = cmp3[q] = take0[q] = take1[q] = take2[q] = 0;
  each_container([&](const GasStep& g) {
    bad |= g.num_i915 > 0 ? g.bad : 0;
    // selections k .. k + num_i915 - 1 all carry this container's step
    const bool s0 = k <= 0 && 0 < k + g.num_i915, s1 = k <= 1 && 1 < k + g.num_i915;
    const bool s2 = k <= 2 && 2 < k + g.num_i915, s3 = k <= 3 && 3 < k + g.num_i915;
#pragma unroll
    for (int q = 0; q < PAS_GAS_MAX_RES; ++q) {
      cmp0[q] = s0 ? g.cmp[q] : cmp0[q];
      take0[q] = s0 ? g.take[q] : take0[q];
      cmp1[q] = s1 ? g.cmp[q] : cmp1[q];
      take1[q] = s1 ? g.take[q] : take1[q];
      cmp2[q] = s2 ? g.cmp[q] : cmp2[q];
      take2[q] = s2 ? g.take[q] : take2[q];
      cmp3[q] = s3 ? g.cmp[q] : cmp3[q];
    }
    for (int32_t r = 0; r < g.num_i915; ++r, ++k) {
      if (four) continue;  // a threshold row instead (below)
      GasSel e = {};
#pragma unroll
      for (int q = 0; q < PAS_GAS_MAX_RES; ++q) {
        e.ct[q][0] = g.cmp[q];
        e.ct[q][1] = (int64_t)(0ull - (unsigned long long)g.take[q]);
      }
      out[k] = e;
    }
  });
  if (four) {
    // row (t, m): need t plus the takes of the set m of earlier selections, overflow flagged
    // (as the two / three-selection rows below); unrequested kinds stay INT64_MIN
    GasFour* f = reinterpret_cast<GasFour*>(out);
    const int64_t* cmps[4] = {cmp0, cmp1, cmp2, cmp3};
    const int64_t* takes[3] = {take0, take1, take2};
    int32_t flags = bad ? 1 : 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int m = 0; m < (1 << t); ++m) {
        bool o = false;
#pragma unroll
        for (int q = 0; q < PAS_GAS_MAX_RES; ++q) {
          int64_t v = cmps[t][q];
          if (v != INT64_MIN) {
#pragma unroll
            for (int s = 0; s < t; ++s) {
              int64_t r;
              if (((m >> s) & 1) && !o) {
                o = __builtin_add_overflow(v, takes[s][q], &r);
                v = r;
              }
            }
          }
          f->th[(1 << t) - 1 + m][q] = v;
        }
        flags |= o ? 1 << ((1 << t) - 1 + m) : 0;
      }
      if (t > 0) {
        bool eq = true;
#pragma unroll
        for (int q = 0; q < PAS_GAS_MAX_RES; ++q) eq = eq && cmps[t][q] == cmps[t - 1][q];
        flags |= eq ? 1 << (kFourSame + t) : 0;
      }
    }
    f->flags = flags;
  }
  if (steps <= 3) {
    // thresholds: need plus the takes of a subset of the earlier selections (cards taken
    // from by exactly those selections); unrequested kinds stay INT64_MIN
    //   row 0: c0   1: c1   2: c1 + t0   3: c2   4: c2 + t0   5: c2 + t1   6: c2 + t0 + t1
    // written straight to the row (a local GasThresholds would live in scratch memory)
    GasThresholds* t = reinterpret_cast<GasThresholds*>(out + kThRow);
    auto add = [](int64_t v, int64_t d, bool& o) {
      int64_t r;
      const bool f = __builtin_add_overflow(v, d, &r);
      o = o || f;
      return r;
    };
    int32_t over = 0;
    int64_t th[7][PAS_GAS_MAX_RES];
#pragma unroll
    for (int q = 0; q < PAS_GAS_MAX_RES; ++q) {
      bool o2 = false, o4 = false, o5 = false, o6 = false;
      th[0][q] = cmp0[q];
      th[1][q] = cmp1[q];
      th[2][q] = cmp1[q] == INT64_MIN ? cmp1[q] : add(cmp1[q], take0[q], o2);
      th[3][q] = cmp2[q];
      th[4][q] = cmp2[q] == INT64_MIN ? cmp2[q] : add(cmp2[q], take0[q], o4);
      th[5][q] = cmp2[q] == INT64_MIN ? cmp2[q] : add(cmp2[q], take1[q], o5);
      if (cmp2[q] == INT64_MIN) {
        th[6][q] = cmp2[q];
      } else {
        const int64_t v = add(cmp2[q], take0[q], o6);
        th[6][q] = o6 ? v : add(v, take1[q], o6);
      }
      over |= (o2 ? 4 : 0) | (o4 ? 16 : 0) | (o5 ? 32 : 0) | (o6 ? 64 : 0);
    }
    if (steps == 2) {  // rows 3..6 unused
#pragma unroll
      for (int jj = 3; jj < 7; ++jj)
#pragma unroll
        for (int q = 0; q < PAS_GAS_MAX_RES; ++q) th[jj][q] = 0;
      over &= 7;
    }
    // full-mask rows (0, 1, 3: a selection's own need) that repeat an earlier one (the
    // selections of one container are identical): bit 8 row 1 == row 0, bit 9 row 3 == row 0,
    // bit 10 row 3 == row 1 (the ranked kernel reuses the mask)
    auto same = [&](int a, int b) {
      bool eq = true;
#pragma unroll
      for (int q = 0; q < PAS_GAS_MAX_RES; ++q) eq = eq && th[a][q] == th[b][q];
      return eq;
    };
    if (same(1, 0)) over |= 1 << 8;
    if (steps == 3 && same(3, 0)) over |= 1 << 9;
    if (steps == 3 && same(3, 1)) over |= 1 << 10;
#pragma unroll
    for (int jj = 0; jj < 7; ++jj)
#pragma unroll
      for (int q = 0; q < PAS_GAS_MAX_RES; ++q) t->th[jj][q] = th[jj][q];
    // a bad pod's row 0 never passes (rank 0x80), so its closed-form word is 0 with no branch
    t->over = over | (bad ? 1 : 0);
  }
  multi[(int64_t)ml * n_pods + slot] = p | (steps << 24) | (bad ? kBadPod : 0);
}

// One thread per pod.
__global__ __launch_bounds__(kPrepTpb) void gas_prep_kernel(PrepArgs a) {
  if (blockIdx.x == 0) prep_zero<kPrepTpb>(a);
  if (a.start && blockIdx.x == 0 && threadIdx.x == 0)  // the side streams' waits start timing
    __hip_atomic_store(a.start, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  prep_pod(a, blockIdx.x * kPrepTpb + threadIdx.x);
}

// gflip[q] = INT64_MAX - gmin[q] (kept flipped so that a zeroed buffer is the identity of the
// unsigned atomicMax): per node the minimum free over its cards, per workgroup the minimum
// over its nodes, one atomic per workgroup and kind.  Nodes without the cards label or not in
// the lister never fit, so they do not count.
__global__ __launch_bounds__(kTpb) void gas_minfree_kernel(int32_t N, int32_t K, int32_t n_res,
                                                           const int32_t* __restrict__ n_cards,
                                                           const int64_t* __restrict__ cap,
                                                           const int64_t* __restrict__ used,
                                                           unsigned long long* __restrict__ gflip,
                                                           int32_t* __restrict__ big_nodes,
                                                           int32_t* __restrict__ n_big_nodes,
                                                           int64_t* __restrict__ free_t) {
  __shared__ int64_t red[kTpb / 64][PAS_GAS_MAX_RES];
  const int32_t n = blockIdx.x * kTpb + threadIdx.x;
  const int32_t nc = n < N ? min(n_cards[n], K) : 0;
  if (nc > kMaxCards) big_nodes[atomicAdd(n_big_nodes, 1)] = n;  // gas_fit_generic_kernel
  for (int q = 0; q < n_res; ++q) {
    int64_t m = INT64_MAX;
    const int64_t c = nc > 0 ? cap[(int64_t)n * n_res + q] : 0;
    for (int k = 0; k < nc; ++k) {
      const int64_t u = used[((int64_t)n * K + k) * n_res + q];
      const int64_t f = (c > 0 && u >= 0) ? c - u : -1;
      m = f < m ? f : m;
    }
    // the card-major copy (free_t, load_free_t: -1 for cards the node does not have)
    if (n < N)
      for (int k = 0; k < kMaxCards; ++k) {
        const int64_t u = k < nc ? used[((int64_t)n * K + k) * n_res + q] : -1;
        free_t[((int64_t)k * n_res + q) * N + n] = (c > 0 && u >= 0) ? c - u : -1;
      }
    for (int off = 32; off > 0; off >>= 1) {
      const int64_t o = __shfl_xor(m, off, 64);
      m = o < m ? o : m;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][q] = m;
  }
  __syncthreads();
  if (threadIdx.x < n_res) {
    int64_t m = INT64_MAX;
    for (int w = 0; w < kTpb / 64; ++w) m = red[w][threadIdx.x] < m ? red[w][threadIdx.x] : m;
    atomicMax(&gflip[threadIdx.x], (unsigned long long)INT64_MAX - (unsigned long long)m);
  }
}

// free[k][q] = cap[q] - used[k][q] if cap[q] > 0 and used[k][q] >= 0, else -1 (and -1 for
// cards the node does not have), from the card-major copy (GasSnapshot::free_t, built by
// gas_minfree_kernel; one coalesced load per card and kind).
//
// free_t[(k Q + q) N + n] through a buffer resource per card (base free_t + k Q N, Q N values):
// the lane's byte offset n * 8 is the only per-lane operand, so no 64-bit address per card and
// kind is computed or held live (as plain pointers they spilled to scratch in the closed-form
// kernel).  gas_fit_launch bounds N so that the offsets fit 32 bits.
template <int Q>
__device__ __forceinline__ int64_t free_at(const int64_t* __restrict__ free_t, int32_t N, int k,
                                           int q, uint32_t off) {
  typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int64_t*>(free_t) + (size_t)k * Q * (uint32_t)N, 0, Q * N * 8, 0x00020000);
  const v2u32 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, q * N * 8, 0);
  return (int64_t)(((uint64_t)v.y << 32) | v.x);
}

// A lane that stores nothing (past N, or a node past 8 cards with word results) reads node 0:
// its values are never used (no store; bitmaps ballot `valid`; masks are ANDed with `live`).
template <int Q>
__device__ __forceinline__ void load_free_t(int32_t n, bool valid, int32_t N,
                                            const int64_t* __restrict__ free_t,
                                            int64_t (&free)[kMaxCards][Q]) {
  const uint32_t off = valid ? (uint32_t)n * 8u : 0u;
#pragma unroll
  for (int k = 0; k < kMaxCards; ++k)
#pragma unroll
    for (int q = 0; q < Q; ++q) free[k][q] = free_at<Q>(free_t, N, k, q, off);
}

typedef unsigned long long lane_mask;  // one bit per lane of the wave (ballot)

// One (pod, node) result: the packed word, or (kBits) the fit bit in the pod's row of a
// node bitmap, written per 64-node word by lane 0 of the wave (waves cover aligned
// 64-node ranges).
#ifndef PAS_GAS_ABLATE
#define PAS_GAS_ABLATE 0  // diagnostic timing builds only: 1 = no result stores (outputs wrong)
#endif
#ifndef PAS_GAS_RUN_FAST
#define PAS_GAS_RUN_FAST 1  // full runs of pods as straight-line code (0: every pod tested)
#endif
#ifndef PAS_GAS_STORE_AUX
#define PAS_GAS_STORE_AUX 2  // result word store cache policy: nt (0: plain global store)
#endif
// The result words: word (p, n) at w[p * ld + n] (ld >= N; pas_gas_fit_ld_device).
struct ResOut {
  uint32_t* w;
  int64_t ld;
  const uint32_t* abort;  // device flags: a wait of this fit timed out if *abort == epoch
  uint32_t epoch;
};

template <bool kBits>
__device__ __forceinline__ void put_result(ResOut res, uint64_t* __restrict__ fit, int64_t p,
                                           int32_t N, int32_t n, bool valid, uint32_t out) {
  if (PAS_GAS_ABLATE & 1) {
    if (out == (uint32_t)p * 2654435761u + 0x7fu) res.w[n] = out;  // keeps the work alive
    return;
  }
  if (kBits) {
    const uint64_t b = __ballot(valid && (out >> 31));
    if ((threadIdx.x & 63) == 0 && n < N) fit[p * ((N + 63) / 64) + (n >> 6)] = b;
  } else if (PAS_GAS_STORE_AUX) {
    // the pod's row as a buffer (lanes past N store nothing), with the store cache policy
    const __amdgpu_buffer_rsrc_t row =
        __builtin_amdgcn_make_buffer_rsrc(res.w + p * res.ld, 0, N * 4, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(out, row, valid ? n * 4 : N * 4, 0, PAS_GAS_STORE_AUX);
  } else if (valid) {
    res.w[p * res.ld + n] = out;
  }
}

// Word results of a batch of fewer than 2^31 result bytes (every C3-sized batch): one buffer
// over all rows, a row's byte offset p * ld * 4 as the store's scalar offset.  The per-row
// form (put_result above) builds a 64-bit row base and a buffer descriptor per pod, ~8 scalar
// instructions against 2 here.
struct ResSoff {
  uint32_t* w;
  uint32_t ld4;    // ld * 4
  uint32_t bytes;  // the whole result buffer, P * ld * 4 < 2^31
  __device__ ResSoff(const ResOut& r, int32_t P)
      : w(r.w), ld4((uint32_t)r.ld * 4u), bytes((uint32_t)P * ((uint32_t)r.ld * 4u)) {}
};

template <bool kBits>
__device__ __forceinline__ void put_result(ResSoff res, uint64_t* __restrict__ fit, int64_t p,
                                           int32_t N, int32_t n, bool valid, uint32_t out) {
  static_assert(!kBits, "bitmap results take put_result(ResOut)");
  // one descriptor over the whole buffer; a lane past N stores at the buffer's end (vector
  // offset = its size: out of range, dropped whether or not the check adds the scalar offset)
  const __amdgpu_buffer_rsrc_t all = __builtin_amdgcn_make_buffer_rsrc(res.w, 0, res.bytes, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(out, all, valid ? n * 4 : res.bytes,
                                        (int32_t)((uint32_t)p * res.ld4), PAS_GAS_STORE_AUX);
}

// Blocks of the fit kernels cover (node block, pod chunk) pairs.  A 1-D grid is mapped so
// that every chunk of a node block runs on the same XCD (block b runs on XCD b % 8,
// MI355X_MICROARCH.md): pairs are ordered node-major and each XCD takes a contiguous run of
// them, so a node block's snapshot rows are fetched into one L2 only.
struct BlockTile {
  int32_t node_block, chunk, chunks;
};
#ifndef PAS_GAS_POD_MAJOR
#define PAS_GAS_POD_MAJOR 0  // 1: a chunk's node blocks consecutive on an XCD (diagnostic)
#endif
__device__ __forceinline__ BlockTile block_tile(int32_t chunks) {
  const int32_t nb = gridDim.x, b = blockIdx.x;
  const int32_t xcd = b & 7, per = nb >> 3, rem = nb & 7;
  const int32_t pos = xcd * per + min(xcd, rem) + (b >> 3);
  if (PAS_GAS_POD_MAJOR) {
    const int32_t node_blocks = nb / chunks;
    return BlockTile{pos % node_blocks, pos / node_blocks, chunks};
  }
  return BlockTile{pos / chunks, pos % chunks, chunks};
}

// This block's share [*b, *e) of a device-counted list, split evenly over the chunks.
__device__ __forceinline__ void list_share(const int32_t* count, const BlockTile& bt, int32_t* b,
                                           int32_t* e) {
  const int32_t cnt = __builtin_amdgcn_readfirstlane(*count);
  const int32_t per = (cnt + bt.chunks - 1) / bt.chunks;
  *b = min(cnt, bt.chunk * per);
  *e = min(cnt, *b + per);
}

constexpr int kPodBatch = 64;  // one-selection pod records staged in LDS per round and wave

// A group of cards of the untouched-card scan: bm * 2 + (1 if need[q] <= free[q] for the C
// compared kinds), card by card from the highest, so bit k of the final mask is card k.
// The blocks declare the SCC clobber of their s_and's.  One assembly block per group issues
// every compare of the group first (they write lane
// masks), then the s_and's combining each card's kinds (with `live` when there is only one
// kind, so the carry-in always comes from a scalar write: a VALU-written SGPR read as a lane
// mask by the next VALU needs wait states inline assembly does not get), then one v_addc per
// card with its mask as carry-in.  The compares' latency is covered by the group's other
// compares; a block per group also keeps the scheduler from hoisting every card's compares
// and running out of SGPRs for their masks.
#define PAS_CMP(m, n, f) "v_cmp_le_i64_e64 %[" #m "], %[" #n "], %[" #f "]\n\t"
#define PAS_AND(d, a, b) "s_and_b64 %[" #d "], %[" #a "], %[" #b "]\n\t"
#define PAS_ADDC(r, x, m) "v_addc_co_u32_e64 %[" #r "], %[co], %[" #x "], %[" #x "], %[" #m "]\n\t"
// C = 1: 4 cards per block
__device__ __forceinline__ uint32_t push4_c1(uint32_t bm, int64_t n0, int64_t f0, int64_t f1,
                                             int64_t f2, int64_t f3, uint64_t live) {
  uint32_t r;
  uint64_t m0, m1, m2, m3, co;
  asm(PAS_CMP(m0, n0, f0) PAS_CMP(m1, n0, f1) PAS_CMP(m2, n0, f2) PAS_CMP(m3, n0, f3)
      PAS_AND(m0, m0, lv) PAS_AND(m1, m1, lv) PAS_AND(m2, m2, lv) PAS_AND(m3, m3, lv)
      PAS_ADDC(r, bm, m0) PAS_ADDC(r, r, m1) PAS_ADDC(r, r, m2) PAS_ADDC(r, r, m3)
      : [r] "=&v"(r), [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3),
        [co] "=&s"(co)
      : [n0] "v"(n0), [f0] "v"(f0), [f1] "v"(f1), [f2] "v"(f2), [f3] "v"(f3), [lv] "s"(live),
        [bm] "v"(bm)
      : "scc");
  return r;
}
// C = 2: 4 cards per block
__device__ __forceinline__ uint32_t push4_c2(uint32_t bm, int64_t n0, int64_t n1, int64_t a0,
                                             int64_t a1, int64_t b0, int64_t b1, int64_t c0,
                                             int64_t c1, int64_t d0, int64_t d1) {
  uint32_t r;
  uint64_t m0, m1, m2, m3, m4, m5, m6, m7, co;
  asm(PAS_CMP(m0, n0, a0) PAS_CMP(m1, n1, a1) PAS_CMP(m2, n0, b0) PAS_CMP(m3, n1, b1)
      PAS_CMP(m4, n0, c0) PAS_CMP(m5, n1, c1) PAS_CMP(m6, n0, d0) PAS_CMP(m7, n1, d1)
      PAS_AND(m0, m0, m1) PAS_AND(m2, m2, m3) PAS_AND(m4, m4, m5) PAS_AND(m6, m6, m7)
      PAS_ADDC(r, bm, m0) PAS_ADDC(r, r, m2) PAS_ADDC(r, r, m4) PAS_ADDC(r, r, m6)
      : [r] "=&v"(r), [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3),
        [m4] "=&s"(m4), [m5] "=&s"(m5), [m6] "=&s"(m6), [m7] "=&s"(m7), [co] "=&s"(co)
      : [n0] "v"(n0), [n1] "v"(n1), [a0] "v"(a0), [a1] "v"(a1), [b0] "v"(b0), [b1] "v"(b1),
        [c0] "v"(c0), [c1] "v"(c1), [d0] "v"(d0), [d1] "v"(d1), [bm] "v"(bm)
      : "scc");
  return r;
}
// C = 3: 2 cards per block
__device__ __forceinline__ uint32_t push2_c3(uint32_t bm, int64_t n0, int64_t n1, int64_t n2,
                                             int64_t a0, int64_t a1, int64_t a2, int64_t b0,
                                             int64_t b1, int64_t b2) {
  uint32_t r;
  uint64_t m0, m1, m2, m3, m4, m5, co;
  asm(PAS_CMP(m0, n0, a0) PAS_CMP(m1, n1, a1) PAS_CMP(m2, n2, a2) PAS_CMP(m3, n0, b0)
      PAS_CMP(m4, n1, b1) PAS_CMP(m5, n2, b2)
      PAS_AND(m0, m0, m1) PAS_AND(m3, m3, m4) PAS_AND(m0, m0, m2) PAS_AND(m3, m3, m5)
      PAS_ADDC(r, bm, m0) PAS_ADDC(r, r, m3)
      : [r] "=&v"(r), [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3),
        [m4] "=&s"(m4), [m5] "=&s"(m5), [co] "=&s"(co)
      : [n0] "v"(n0), [n1] "v"(n1), [n2] "v"(n2), [a0] "v"(a0), [a1] "v"(a1), [a2] "v"(a2),
        [b0] "v"(b0), [b1] "v"(b1), [b2] "v"(b2), [bm] "v"(bm)
      : "scc");
  return r;
}
// C = 4: 2 cards per block
__device__ __forceinline__ uint32_t push2_c4(uint32_t bm, const int64_t (&n)[4],
                                             const int64_t (&a)[4], const int64_t (&b)[4]) {
  uint32_t r;
  uint64_t m0, m1, m2, m3, m4, m5, m6, m7, co;
  asm(PAS_CMP(m0, n0, a0) PAS_CMP(m1, n1, a1) PAS_CMP(m2, n2, a2) PAS_CMP(m3, n3, a3)
      PAS_CMP(m4, n0, b0) PAS_CMP(m5, n1, b1) PAS_CMP(m6, n2, b2) PAS_CMP(m7, n3, b3)
      PAS_AND(m0, m0, m1) PAS_AND(m4, m4, m5) PAS_AND(m2, m2, m3) PAS_AND(m6, m6, m7)
      PAS_AND(m0, m0, m2) PAS_AND(m4, m4, m6)
      PAS_ADDC(r, bm, m0) PAS_ADDC(r, r, m4)
      : [r] "=&v"(r), [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3),
        [m4] "=&s"(m4), [m5] "=&s"(m5), [m6] "=&s"(m6), [m7] "=&s"(m7), [co] "=&s"(co)
      : [n0] "v"(n[0]), [n1] "v"(n[1]), [n2] "v"(n[2]), [n3] "v"(n[3]), [a0] "v"(a[0]),
        [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]), [b0] "v"(b[0]), [b1] "v"(b[1]),
        [b2] "v"(b[2]), [b3] "v"(b[3]), [bm] "v"(bm)
      : "scc");
  return r;
}
#undef PAS_CMP
#undef PAS_AND
#undef PAS_ADDC

// Bit mask of the cards k (bit k) with need[j] <= fr[k][j] for all C compared kinds.
template <int C>
__device__ __forceinline__ uint32_t fit_mask(const int64_t (&need)[C],
                                             const int64_t (&fr)[kMaxCards][C], uint64_t live) {
  uint32_t bm = 0u;
  if constexpr (C == 1) {
#ifdef PAS_C1_PERCARD
#pragma unroll
    for (int k = kMaxCards - 1; k >= 0; --k) {
      uint32_t r;
      uint64_t m0, co;
      asm("v_cmp_le_i64_e64 %1, %3, %4\n\t"
          "s_and_b64 %1, %1, %5\n\t"
          "v_addc_co_u32_e64 %0, %2, %6, %6, %1"
          : "=&v"(r), "=&s"(m0), "=&s"(co)
          : "v"(need[0]), "v"(fr[k][0]), "s"(live), "v"(bm)
          : "scc");
      bm = r;
    }
#else
    bm = push4_c1(bm, need[0], fr[7][0], fr[6][0], fr[5][0], fr[4][0], live);
    bm = push4_c1(bm, need[0], fr[3][0], fr[2][0], fr[1][0], fr[0][0], live);
#endif
  } else if constexpr (C == 2) {
    bm = push4_c2(bm, need[0], need[1], fr[7][0], fr[7][1], fr[6][0], fr[6][1], fr[5][0],
                  fr[5][1], fr[4][0], fr[4][1]);
    bm = push4_c2(bm, need[0], need[1], fr[3][0], fr[3][1], fr[2][0], fr[2][1], fr[1][0],
                  fr[1][1], fr[0][0], fr[0][1]);
  } else if constexpr (C == 3) {
#pragma unroll
    for (int k = kMaxCards - 1; k > 0; k -= 2)
      bm = push2_c3(bm, need[0], need[1], need[2], fr[k][0], fr[k][1], fr[k][2], fr[k - 1][0],
                    fr[k - 1][1], fr[k - 1][2]);
  } else {
#pragma unroll
    for (int k = kMaxCards - 1; k > 0; k -= 2) bm = push2_c4(bm, need, fr[k], fr[k - 1]);
  }
  return bm;
}

constexpr int kMB = 2;  // multi-selection pods staged in LDS per round and wave (LDS: 4 workgroups per CU)
constexpr int kRowChunks = kPacked * (int)sizeof(GasSel) / 16;  // 16-B chunks per row
template <int Q, int SKIP>
__device__ __forceinline__ uint32_t th_mask(const int64_t (&free)[kMaxCards][Q], const int64_t* th,
                                            uint64_t live) {
  constexpr int kSkip = Q == 1 ? -1 : SKIP;  // a selection's only kind is never skipped
  constexpr int kC = Q - (kSkip >= 0 ? 1 : 0);
  int64_t need[kC];
  int64_t fr[kMaxCards][kC];
#pragma unroll
  for (int q = 0, j = 0; q < Q; ++q)
    if (q != kSkip) need[j++] = th[q];
#pragma unroll
  for (int k = 0; k < kMaxCards; ++k)
#pragma unroll
    for (int q = 0, j = 0; q < Q; ++q)
      if (q != kSkip) fr[k][j++] = free[k][q];
  return fit_mask<kC>(need, fr, live);
}

// v_ffbl_b32: the lowest set bit of a lane mask, 0xFFFFFFFF for none, in one instruction (the
// C form adds a compare and a select for the zero case)
__device__ __forceinline__ uint32_t ffbl(uint32_t m) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(m));
  return r;
}
__device__ __forceinline__ uint32_t lowest(uint32_t m) { return min(ffbl(m), 8u); }  // 8: none

// ---------------------------------------------------------------------------- ranked fit
//
// Rank compression (exact).  Every compare of the one-selection and closed-form paths is
// "threshold t <= snapshot free f".  For a multiset T of at most 127 thresholds holding t,
//   t <= f  <=>  #{t' in T : t' < t} + 1  <=  #{t' in T : t' <= f}
// (t <= f: the right side counts t and everything below it; t > f: it counts only values
// below t).  Both ranks fit 7 bits, so the ranks of four cards of one kind pack into a dword
// as bytes rank + 0x80, and one 32-bit subtraction of the threshold's rank (replicated in
// every byte) tests the four cards at once: byte k of the difference keeps bit 7 exactly
// when card k passes, and no byte borrows from the next (each byte of it is >= 1).  A kind a
// row does not request has rank 0 (always passes); a row whose threshold overflows int64
// has rank 0x80 (never passes).
//
// The pods of each list are cut into groups of at most 127 thresholds per kind (127
// one-selection pods; 42 two-selection pods of 3 threshold rows; 18 three-selection pods of
// 7 rows), inside each block's chunk of the list.  gas_rank_prep_kernel sorts a group's
// thresholds per kind (counting ranks, one wave per group) and writes each threshold's rank;
// a fit kernel ranks its nodes' free values against the group once (a 7-step binary search
// per card and kind) and then tests a row against the 8 cards with 2 subtractions per kind
// and a few bit operations, instead of 8 64-bit compares and 8 mask updates per kind.
constexpr int kRankMax = 127;       // thresholds per group and kind (7-bit ranks)
constexpr int kRankItems = 128;     // sorted row length in LDS (padded with INT64_MAX)
constexpr int kRankMB = 16;         // two/three-selection pods staged per batch (64-B rows)

// A one-selection pod's ranks: g[j] = the rank of its need of compared kind j in every byte.
struct alignas(16) GasRSingle {
  uint32_t g[PAS_GAS_MAX_RES];
  int32_t word;  // as GasSingle::word
  int32_t pad[3];
};
// A two/three-selection pod's ranks: rows 0, 1, 3 (the full-mask rows: a selection's own need)
// replicated per kind; rows 2, 4, 5, 6 (checked at one chosen card) packed, byte j = kind j.
struct alignas(16) GasRMulti {
  uint32_t rep[3][PAS_GAS_MAX_RES];
  uint32_t pk[4];
};
// A four-to-eight-selection pod's ranks: selection t's need per compared kind, replicated.
struct alignas(16) GasRSeq {
  uint32_t rep[kPacked][PAS_GAS_MAX_RES];
};
// A closed-form four-selection pod's ranks: its full-mask rows (GasFour rows 0, 1, 3, 7: the
// selections' own needs) per compared kind, replicated.  Its other rows are checked at one
// card on 64-bit values (rfour).
struct alignas(16) GasRFour {
  uint32_t rep[4][PAS_GAS_MAX_RES];
};
// rword flags (free bits of a multi-list word): the full-mask rows that repeat an earlier one
constexpr uint32_t kSame01 = 1u << 28, kSame03 = 1u << 29, kSame13 = 1u << 31;

// rows per pod of a slot class: 0 one selection, 1 two, 2 three, 3 four to eight (a row per
// selection, rows past S hold INT64_MIN), 4 four in closed form (its full-mask rows)
__device__ __forceinline__ int32_t rank_rows(int32_t cls) {
  return cls == 0 ? 1 : cls == 1 ? 3 : cls == 2 ? 7 : cls == 3 ? kPacked : 4;
}
__device__ __forceinline__ int32_t rank_gs(int32_t cls) { return kRankMax / rank_rows(cls); }

__device__ __forceinline__ void rank_group(
    int32_t P, int32_t Q, const int32_t* counts, int32_t slot, int32_t gi,
    const GasSingle* __restrict__ single, const int32_t* __restrict__ multi,
    const GasSel* __restrict__ sels, int64_t* __restrict__ srt_s, int64_t* __restrict__ srt_m,
    GasRSingle* __restrict__ rsingle, GasRMulti* __restrict__ rmulti, int32_t* __restrict__ rword,
    GasRSeq* __restrict__ rseq, GasRFour* __restrict__ rfour, int64_t (*v)[kRankItems],
    uint32_t* pks) {
  const int32_t NL = Q + 1;
  const bool one = slot < NL, seq = slot >= 3 * NL && slot < 4 * NL, four = slot >= 4 * NL;
  const int32_t l = one ? slot : seq ? slot - 3 * NL : four ? slot - 4 * NL : (slot - NL) >> 1;
  const int32_t cls = one ? 0 : seq ? 3 : four ? 4 : 1 + ((slot - NL) & 1);
  const int32_t R = rank_rows(cls);
  const int32_t ml =
      l * kClasses + (seq ? kClsSeq : four ? kClsFour : cls - 1);  // multi list (cls > 0)
  const int32_t cnt = counts[one ? l : NL + ml];
  const int32_t gb = gi * rank_gs(cls), ge = min(cnt, gb + rank_gs(cls));
  const int32_t n = (ge - gb) * R;
  int64_t base = 0;
  if (one) {
    for (int32_t s = 0; s < l; ++s) base += counts[s];
  } else {
    // two- and three-selection slots in slot order, then the sequential ones, then the
    // closed-form four-selection ones
    const int32_t pairs = seq || four ? 2 * NL : slot - NL;
    for (int32_t s = 0; s < pairs; ++s)
      base += (int64_t)counts[NL + (s >> 1) * kClasses + (s & 1)] * rank_rows(1 + (s & 1));
    // list 0's sequential pods are not ranked (no groups, no rows), nor filed as four
    for (int32_t s = 1; s < (seq ? l : four ? NL : 0); ++s)
      base += (int64_t)counts[NL + s * kClasses + kClsSeq] * kPacked;
    if (four)
      for (int32_t s = 1; s < l; ++s) base += (int64_t)counts[NL + s * kClasses + kClsFour] * 4;
  }
  base += (int64_t)gb * R;
  int64_t* srt = one ? srt_s : srt_m;
  const int32_t skip = l - 1;
  const int32_t i = threadIdx.x % kRankItems, q = threadIdx.x / kRankItems;
  const bool kind = q < Q && q != skip;
  const int32_t j = q - (skip >= 0 && q > skip ? 1 : 0);  // compared-kind index
  const bool live = kind && i < n;
  const int32_t pos = gb + (i < n ? i / R : 0), row = i < n ? i % R : 0;
  const GasThresholds* th = one || seq || four
                                ? nullptr
                                : reinterpret_cast<const GasThresholds*>(
                                      sels + ((int64_t)ml * P + pos) * kPacked + kThRow);
  const GasFour* th4 =
      four ? reinterpret_cast<const GasFour*>(sels + ((int64_t)ml * P + pos) * kPacked) : nullptr;
  // a four-selection pod's full-mask rows: GasFour rows 0, 1, 3, 7
  const int32_t frow = (1 << row) - 1;
  // every global load of the group up front (one round trip): the value (padded with
  // INT64_MAX: never below an item, equal only to items past the padding), the pod word, the
  // threshold flags, the one-selection word
  const bool item = i < n;
  const int32_t mword = !one && item ? multi[(int64_t)ml * P + pos] : 0;
  const uint32_t over = !item || one || seq ? 0u
                        : four         ? (uint32_t)th4->flags >> frow
                                       : (uint32_t)th->over >> row;
  const int32_t sword = one && item ? single[(int64_t)l * P + pos].word : 0;
  int64_t y = INT64_MAX;
  if (live) {
    if (one) {
      y = single[(int64_t)l * P + pos].cmp[q];
    } else if (seq) {  // selection `row` of the pod, loaded unconditionally (INT64_MIN past S)
      const int64_t x = sels[((int64_t)ml * P + pos) * kPacked + row].ct[q][0];
      y = row < ((mword >> 24) & 0xF) ? x : INT64_MIN;
    } else if (four) {
      y = th4->th[frow][q];
    } else {
      y = th->th[row][q];
    }
  }
  v[q][i] = y;
  if (q == 0) pks[i] = 0u;
  __syncthreads();
  uint32_t g = 0u;
  if (live) {
    const int32_t n16 = (n + 15) & ~15;
    int32_t less = 0, eqb = 0;
    for (int32_t k0 = 0; k0 < n16; k0 += 16) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int64_t x = v[q][k0 + k];
        less += x < y ? 1 : 0;
        eqb += (x == y && k0 + k < i) ? 1 : 0;
      }
    }
    srt[(base + less + eqb) * PAS_GAS_MAX_RES + j] = y;
    // 0x80 never passes: an overflowing threshold, or (one selection) a bad pod, whose word
    // is then 0 on every node without a branch in the fit kernel
    g = ((over & 1u) || (sword & kBadPod)) ? 0x80u : (uint32_t)(less + 1);
    if (one) {
      rsingle[(int64_t)l * P + pos].g[j] = g * 0x01010101u;
    } else if (seq) {
      rseq[(int64_t)l * P + pos].rep[row][j] = g * 0x01010101u;
    } else if (four) {
      rfour[(int64_t)l * P + pos].rep[row][j] = g * 0x01010101u;
    } else if (row == 0 || row == 1 || row == 3) {
      rmulti[(int64_t)(l * 2 + cls - 1) * P + pos].rep[row == 3 ? 2 : row][j] = g * 0x01010101u;
    } else {
      atomicOr(&pks[i], g << (8 * j));
    }
  }
  __syncthreads();
  // one thread per item: the packed rows and the pod word
  if (threadIdx.x >= kRankItems || i >= n || seq || four) return;
  if (one) {
    rsingle[(int64_t)l * P + pos].word = sword;
    return;
  }
  const int64_t mp = (int64_t)(l * 2 + cls - 1) * P + pos;
  if (row == 2 || row >= 4) rmulti[mp].pk[row == 2 ? 0 : row - 3] = pks[i];
  if (row == 0)
    rword[mp] = (int32_t)((uint32_t)mword | (((over >> 8) & 1u) ? kSame01 : 0u) |
                          (((over >> 9) & 1u) ? kSame03 : 0u) |
                          (((over >> 10) & 1u) ? kSame13 : 0u));
}


// Each ranked list is cut into fixed groups of gs = 127 / rows pods: group g holds list
// positions [g gs, min(cnt, (g + 1) gs)).  A one-selection chunk of the fit kernel is one group
// (the grid covers ceil(P / 127) chunks); a multi-selection chunk takes ceil(G / chunks) whole
// groups of each list (G groups), so every block ranks its nodes once per full group.
__device__ __forceinline__ void chunk_groups(int32_t cnt, int32_t chunks, int32_t chunk,
                                             int32_t gs, int32_t* g0, int32_t* g1) {
  const int32_t G = (cnt + gs - 1) / gs;
  const int32_t gpc = (G + chunks - 1) / chunks;
  *g0 = min(G, chunk * gpc);
  *g1 = min(G, *g0 + gpc);
}

// One block per non-empty group (a persistent loop over the groups of every list slot), a
// thread per (item, kind).  Slots: [0, NL) the one-selection lists; NL + 2 l + c list l's
// two- (c = 0) and three-selection (c = 1) pods; then per list the sequential pods, then the
// closed-form four-selection pods (their full-mask rows).  A group's items are its pods' rows
// (pod-major).  Per compared kind: an item's rank = #{items below it} (+ #{equal items before
// it} for its sorted position), written as the sorted row (srt_*[item][kind j]) and as the
// item's rank in its pod's record.  Items of a slot sit after those of the slots before it,
// so a group's sorted rows are contiguous.
constexpr int kRankPrepTpb = kRankItems * PAS_GAS_MAX_RES;
constexpr int kRankPrepBlocks = 256;  // one per CU: a group per block at a time
struct RankArgs {
  int32_t P, Q;
  const int32_t* counts;
  const GasSingle* single;
  const int32_t* multi;
  const GasSel* sels;
  int64_t* srt_s;
  int64_t* srt_m;
  GasRSingle* rsingle;
  GasRMulti* rmulti;
  int32_t* rword;
  GasRSeq* rseq;
  GasRFour* rfour;
};
struct RankLds {
  int64_t v[PAS_GAS_MAX_RES][kRankItems];
  uint32_t pks[kRankItems];
  int32_t cnt_s[(1 + kClasses) * (PAS_GAS_MAX_RES + 1)];
};
// The groups w = first, first + stride, ... of every list slot, one at a time per block.
__device__ __forceinline__ void rank_prep_body(const RankArgs& a, int32_t first, int32_t stride,
                                               RankLds& L) {
  const int32_t P = a.P, Q = a.Q;
  const int32_t* counts = a.counts;
  int32_t (&cnt_s)[(1 + kClasses) * (PAS_GAS_MAX_RES + 1)] = L.cnt_s;
  const int32_t NL = Q + 1, slots = NL * 5;
  // the list counts, loaded once (a slot scan of dependent global loads costs a round trip each)
  if (threadIdx.x < (1 + kClasses) * NL) cnt_s[threadIdx.x] = counts[threadIdx.x];
  __syncthreads();
  counts = cnt_s;
  // slots: one-selection lists, two/three-selection pairs, sequential lists (list 0's
  // sequential pods, with no kind skipped, are evaluated on 64-bit values: no groups),
  // closed-form four-selection lists (none in list 0)
  auto slot_groups = [&](int32_t slot) {
    int32_t cnt, cls;
    if (slot < NL) {
      cnt = counts[slot], cls = 0;
    } else if (slot < 3 * NL) {
      cnt = counts[NL + ((slot - NL) >> 1) * kClasses + ((slot - NL) & 1)];
      cls = 1 + ((slot - NL) & 1);
    } else if (slot < 4 * NL) {
      cnt = slot == 3 * NL ? 0 : counts[NL + (slot - 3 * NL) * kClasses + kClsSeq], cls = 3;
    } else {
      cnt = counts[NL + (slot - 4 * NL) * kClasses + kClsFour], cls = 4;  // (list 0: none)
    }
    return (cnt + rank_gs(cls) - 1) / rank_gs(cls);
  };
  for (int32_t w = first;; w += stride) {
    // the group: w-th over the slots' groups in slot order
    int32_t slot = 0, gi = w;
    for (; slot < slots; ++slot) {
      const int32_t G = slot_groups(slot);
      if (gi < G) break;
      gi -= G;
    }
    if (slot >= slots) return;
    __syncthreads();  // the previous group's reads of v / pks are done
    rank_group(P, Q, counts, slot, gi, a.single, a.multi, a.sels, a.srt_s, a.srt_m, a.rsingle,
               a.rmulti, a.rword, a.rseq, a.rfour, L.v, L.pks);
  }
}

__global__ __launch_bounds__(kRankPrepTpb) void gas_rank_prep_kernel(RankArgs a) {
  __shared__ RankLds L;
  rank_prep_body(a, blockIdx.x, gridDim.x, L);
}


// The group's sorted rows of the C compared kinds into the wave's LDS slice [C][128]
// (positions past the group's items: INT64_MAX), each in Eytzinger (breadth-first) order: the
// i-th smallest (1-based r = i + 1 <= 127) at e(r) = 2^(6 - tz) + (r >> (tz + 1)), tz = ctz(r),
// so that level L of the search reads entries [2^L, 2^(L+1)) — consecutive, one per bank —
// instead of entries 2^(7-L) apart, which share banks (LDS bank conflicts of the sorted order:
// SQ_LDS_BANK_CONFLICT, profiles/r05_gas_sq.csv).  Entry 0 is not read; the 128th is not kept.
template <int C>
__device__ __forceinline__ void load_sorted(const int64_t* __restrict__ srt, int64_t item0,
                                            int32_t n, int64_t* lds, int lane) {
  int64_t x[2][C];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int32_t i = lane + 64 * it;
    const int64_t* p = srt + (item0 + min(i, max(n - 1, 0))) * PAS_GAS_MAX_RES;
#pragma unroll
    for (int j = 0; j < C; ++j) x[it][j] = i < n ? p[j] : INT64_MAX;
  }
  __builtin_amdgcn_wave_barrier();  // the previous group's reads of the slice are done
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const uint32_t r = (uint32_t)(lane + 64 * it) + 1u;  // 1 .. 128
    const uint32_t tz = (uint32_t)__builtin_ctz(r);
    const uint32_t e = r < 128u ? (1u << (6u - tz)) + (r >> (tz + 1u)) : 0u;  // 128: entry 0
#pragma unroll
    for (int j = 0; j < C; ++j) lds[j * kRankItems + e] = x[it][j];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// Four upper-bound levels at once: pos[k] = 2 pos[k] + (x[k] <= f[k]).  The compares go first
// (each writes a lane mask), then the adds with the masks as carry-in, each mask read three
// instructions after its compare (the VALU SGPR-write -> mask-read hazard needs two).
__device__ __forceinline__ void rank_level4(uint32_t& p0, uint32_t& p1, uint32_t& p2, uint32_t& p3,
                                            int64_t x0, int64_t x1, int64_t x2, int64_t x3,
                                            int64_t f0, int64_t f1, int64_t f2, int64_t f3) {
  uint64_t m0, m1, m2, m3, co;
  asm("v_cmp_le_i64_e64 %[m0], %[x0], %[f0]\n\t"
      "v_cmp_le_i64_e64 %[m1], %[x1], %[f1]\n\t"
      "v_cmp_le_i64_e64 %[m2], %[x2], %[f2]\n\t"
      "v_cmp_le_i64_e64 %[m3], %[x3], %[f3]\n\t"
      "v_addc_co_u32_e64 %[p0], %[co], %[p0], %[p0], %[m0]\n\t"
      "v_addc_co_u32_e64 %[p1], %[co], %[p1], %[p1], %[m1]\n\t"
      "v_addc_co_u32_e64 %[p2], %[co], %[p2], %[p2], %[m2]\n\t"
      "v_addc_co_u32_e64 %[p3], %[co], %[p3], %[p3], %[m3]"
      : [p0] "+v"(p0), [p1] "+v"(p1), [p2] "+v"(p2), [p3] "+v"(p3), [m0] "=&s"(m0),
        [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3), [co] "=&s"(co)
      : [x0] "v"(x0), [x1] "v"(x1), [x2] "v"(x2), [x3] "v"(x3), [f0] "v"(f0), [f1] "v"(f1),
        [f2] "v"(f2), [f3] "v"(f3));
}

// The node's cards ranked against the group: fa[j] = bytes rank + 0x80 of cards 0, 2, 4, 6
// (kind j), fb[j] of cards 1, 3, 5, 7.  rank = #{group thresholds <= free}, the upper bound
// found down the Eytzinger tree of the sorted row (load_sorted): from e = 1, e = 2e + (row[e]
// <= free) for 7 levels, then rank = e - 128 (an address, a compare and an add-with-carry per
// level; at most n, the padding is INT64_MAX).  The 8 cards of a kind go level by level
// together (8 LDS reads in flight).
// (the free values read from the card-major copy one kind at a time: 8 values live, not 8 Q)
template <int Q, int SKIP, int C>
__device__ __forceinline__ void rank_cards_t(const int64_t* __restrict__ free_t, int32_t n_node,
                                             bool valid, int32_t N, const int64_t* lds,
                                             int32_t n, uint32_t (&fa)[C], uint32_t (&fb)[C]) {
  const uint32_t off = valid ? (uint32_t)n_node * 8u : 0u;
#pragma unroll
  for (int q = 0, j = 0; q < Q; ++q) {
    if (q == SKIP) continue;
    int64_t f[kMaxCards];
#pragma unroll
    for (int k = 0; k < kMaxCards; ++k) f[k] = free_at<Q>(free_t, N, k, q, off);  // (load_free_t)
    uint32_t pos[kMaxCards];
#pragma unroll
    for (int k = 0; k < kMaxCards; ++k) pos[k] = 1u;
    const int64_t* row = lds + j * kRankItems;
#pragma unroll
    for (int sh = 6; sh >= 0; --sh) {
      int64_t x[kMaxCards];
#pragma unroll
      for (int k = 0; k < kMaxCards; ++k) x[k] = row[pos[k]];
      rank_level4(pos[0], pos[1], pos[2], pos[3], x[0], x[1], x[2], x[3], f[0], f[1], f[2], f[3]);
      rank_level4(pos[4], pos[5], pos[6], pos[7], x[4], x[5], x[6], x[7], f[4], f[5], f[6], f[7]);
    }
    // bytes rank + 0x80 (ranks are at most 127: the 0x80 is one OR per word)
    uint32_t a = 0u, b = 0u;
#pragma unroll
    for (int k = 0; k < kMaxCards; ++k) {
      const uint32_t r = min(pos[k] - 128u, (uint32_t)n);
      if (k & 1) b |= r << (8 * (k >> 1));
      else a |= r << (8 * (k >> 1));
    }
    fa[j] = a | 0x80808080u;
    fb[j] = b | 0x80808080u;
    ++j;
  }
}

// Card mask of a row of replicated ranks g[j]: card k passes <=> bit 4k + 3.
template <int C>
__device__ __forceinline__ uint32_t rmask(const uint32_t (&fa)[C], const uint32_t (&fb)[C],
                                          const uint32_t* g) {
  uint32_t a = 0x80808080u, b = 0x80808080u;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    a &= fa[j] - g[j];
    b &= fb[j] - g[j];
  }
  return (a >> 4) | b;
}

// lowest set bit, 0xFFFFFFFF for none (v_ffbl_b32)
__device__ __forceinline__ uint32_t lowbit(uint32_t m) { return ffbl(m); }

// p as a per-lane (VGPR) address: the pod loops read each pod's record from the wave's stage at
// fixed offsets; with a uniform (SGPR) base the compiler copies the base into a VGPR before
// every LDS read (a v_mov per read), with a VGPR base it adds the record offsets as immediates.
template <typename T>
__device__ __forceinline__ T* lane_ptr(T* p) {
  uint32_t zero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
  return reinterpret_cast<T*>(reinterpret_cast<char*>(p) + zero);
}

// Lane-private copy of the node's free values of the compared kinds (all but SKIP) in LDS,
// [card][lane][kind], so that a lane can read its chosen card's values back with one LDS read
// (registers cannot be indexed per lane).
template <int kC>
struct FreeTab {
  int64_t* base;  // this wave's table: kMaxCards * 64 * kC
  __device__ __forceinline__ int64_t* at(uint32_t card, int lane) const {
    return base + ((int64_t)card * 64 + lane) * kC;
  }
};

template <int Q, int SKIP, int kC>
__device__ __forceinline__ void fill_tab(const int64_t (&free)[kMaxCards][Q], const FreeTab<kC>& tab,
                                         int lane) {
#pragma unroll
  for (int k = 0; k < kMaxCards; ++k)
#pragma unroll
    for (int q = 0, j = 0; q < Q; ++q)
      if (q != SKIP) tab.at(k, lane)[j++] = free[k][q];
}

// fill_tab with the values read from the card-major copy (no register copy of the node's
// free values stays live in the sequential kernel).
template <int Q, int SKIP, int kC>
__device__ __forceinline__ void fill_tab_t(const int64_t* __restrict__ free_t, int32_t n,
                                           bool valid, int32_t N, const FreeTab<kC>& tab,
                                           int lane) {
  int64_t free[kMaxCards][Q];
  load_free_t<Q>(n, valid, N, free_t, free);
  fill_tab<Q, SKIP, kC>(free, tab, lane);
}

// A pod with 4 to 8 selections: the selections in order on a working copy of the free values
// (registers, loaded from the card-major copy per pod: the rare list without a skipped kind
// keeps no second copy live), each a fit mask on the copy; the chosen card's copy drops by
// the take, updated under the lanes that chose it (one branch per card some lane chose).
template <int Q, int SKIP>
__device__ __forceinline__ uint32_t multi_state(const int64_t* __restrict__ free_t, int32_t n,
                                                bool valid, int32_t N, const GasSel* rec,
                                                int32_t S, uint64_t live, uint32_t node_ok) {
  typedef int64_t v2i64 __attribute__((ext_vector_type(2)));
  int64_t w[kMaxCards][Q];
  load_free_t<Q>(n, valid, N, free_t, w);
  bool fits = true;
  uint32_t word = 0u;
  for (int32_t t = 0; t < S; ++t) {
    int64_t cmp[Q], neg[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const v2i64 ct = *reinterpret_cast<const v2i64*>(rec[t].ct[q]);
      cmp[q] = ct.x;
      neg[q] = ct.y;
    }
    const uint32_t c = lowest(th_mask<Q, SKIP>(w, cmp, live));
    fits = fits && c < 8u;
    if (!__ballot(fits)) break;
#pragma unroll
    for (int kk = 0; kk < kMaxCards; ++kk)
      if (__ballot(c == (uint32_t)kk) && c == (uint32_t)kk)
#pragma unroll
        for (int q = 0; q < Q; ++q) w[kk][q] += neg[q];
    word |= (c & 7u) << (3 * t);
  }
  return fits ? (node_ok | ((uint32_t)S << 24) | word) : 0u;
}

// A pod with several selections, in order: selection t takes the first card (lexicographic)
// whose current free covers its need (getCardsForContainerGPURequest, scheduler.go:200-257;
// addRM after each take).  A card no earlier selection of the pod took from still has its
// snapshot free, so the candidates are the fit mask of the need on the snapshot (free only
// falls: a card outside the mask cannot pass); among them a card an earlier selection s took
// from passes only if its current free cur[s] covers the need.  So
//   c_t = lowest(mask(need_t) without {c_s : s < t, need_t > cur[s]})
// and the take lowers cur of every s with c_s = c_t (a card first taken reads its snapshot
// free from the lane's LDS copy).  Registers only, unrolled over t; a selection whose need
// equals the previous one's reuses its mask (the selections of one container are identical).

// kRanked: the fit masks from the group ranks (rk: selection t's ranks per compared kind,
// replicated; fa / fb the node's card ranks) instead of 64-bit compares; card k is then bit
// 4k + 3 of a mask (rmask), else bit k.
template <int Q, int SKIP, int kC, bool kRanked = false>
__device__ __forceinline__ uint32_t multi_seq(const int64_t (*free)[Q],  // [kMaxCards][Q]; unused ranked
                                              const GasSel* rec, int32_t S, uint64_t live,
                                              uint32_t node_ok, const FreeTab<kC>& tab,
                                              int lane, uint32_t same_row,
                                              const uint32_t* rk = nullptr,
                                              const uint32_t* fa = nullptr,
                                              const uint32_t* fb = nullptr) {
  typedef int64_t v2i64 __attribute__((ext_vector_type(2)));
  int64_t fr[kMaxCards][kC];
  if constexpr (!kRanked) {
#pragma unroll
    for (int k = 0; k < kMaxCards; ++k)
#pragma unroll
      for (int q = 0, j = 0; q < Q; ++q)
        if (q != SKIP) fr[k][j++] = free[k][q];
  }
  int64_t cur[kPacked][kC];
  uint32_t cb[kPacked];  // the card of each earlier selection's entry, one-hot
  uint32_t word = 0u, m = 0u, bad_prev = 0u;
  uint64_t fit_m = __ballot(true);  // lanes whose every step so far found a card
#pragma unroll
  for (int t = 0; t < kPacked; ++t) {
    if (t >= S) break;
    int64_t need[kC], neg[kC];
#pragma unroll
    for (int q = 0, j = 0; q < Q; ++q)
      if (q != SKIP) {
        const v2i64 ct = *reinterpret_cast<const v2i64*>(rec[t].ct[q]);
        need[j] = ct.x;
        neg[j++] = ct.y;
      }
    // same_row: nibble t all ones = selection t's record equals selection t - 1's
    const bool same = t > 0 && ((same_row >> (4 * t)) & 0xFu) == 0xFu;
    if (!same) {
      if constexpr (kRanked) {
        uint32_t ga[kC], gfa[kC], gfb[kC];
#pragma unroll
        for (int j = 0; j < kC; ++j) {
          ga[j] = rk[t * PAS_GAS_MAX_RES + j];
          gfa[j] = fa[j];
          gfb[j] = fb[j];
        }
        m = rmask<kC>(gfa, gfb, ga);
      } else {
        m = fit_mask<kC>(need, fr, live);
      }
    }
    uint32_t bad = 0u;
    if (same) {
      // the need of step t - 1: the entries before t - 1 are unchanged since then (a take
      // only adds an entry, and the card taken was not in the old set), so only entry t - 1
      // is new
      bool ok = true;
#pragma unroll
      for (int j = 0; j < kC; ++j) ok = ok && need[j] <= cur[t > 0 ? t - 1 : 0][j];
      bad = bad_prev | (ok ? 0u : cb[t > 0 ? t - 1 : 0]);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < t; ++s2) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < kC; ++j) ok = ok && need[j] <= cur[s2][j];
        bad |= ok ? 0u : cb[s2];
      }
    }
    bad_prev = bad;
    // the chosen card, and its bit in the mask layout (a failed lane's later choices are
    // garbage: its word is 0 whatever they are)
    uint32_t c, bc;
    if constexpr (kRanked) {
      const uint32_t pb = lowbit(m & ~bad);
      c = pb >> 2;
      bc = 1u << (pb & 31u);
    } else {
      c = lowest(m & ~bad);
      bc = 1u << c;  // c = 8 (no card): bit 8, outside every 8-card mask
    }
    fit_m &= __ballot(c < 8u);  // (a lane mask in SGPRs: one compare per step)
    if (!fit_m) break;
    int64_t g[kC];
    {
      const int64_t* p = tab.at(min(c, 7u), lane);
#pragma unroll
      for (int j = 0; j < kC; ++j) g[j] = p[j];
    }
    // the card's newest entry (later entries override earlier ones).  Older entries of a card
    // stay: free only falls, so an older entry fails a need only when the newest one does,
    // and the checks above read them harmlessly
#pragma unroll
    for (int s2 = 0; s2 < t; ++s2) {
      const bool e = cb[s2] == bc;
#pragma unroll
      for (int j = 0; j < kC; ++j) g[j] = e ? cur[s2][j] : g[j];
    }
#pragma unroll
    for (int j = 0; j < kC; ++j) {
      g[j] += neg[j];
      cur[t][j] = g[j];
    }
    cb[t] = bc;
    word |= (c & 7u) << (3 * t);
  }
  return ((fit_m >> lane) & 1u) ? (node_ok | ((uint32_t)S << 24) | word) : 0u;
}

// Pods of 4 to 8 selections (list `list`, kind SKIP = list - 1 dropped).  Each wave stages
// the rows of kMB pods in its own LDS slice (one contiguous copy: rows sit in list order) and
// reads them back with broadcast LDS reads (values in VGPRs).  No block barrier: a wave
// waiting for its copy does not hold up the other waves of the block.
template <int Q, int SKIP, bool kBits, class RO>
__device__ __forceinline__ void multi_list(const int64_t* __restrict__ free_t, GasSel* stage,
                                           int64_t* tab_base, uint32_t node_ok,
                                           int32_t N, int32_t n, bool valid,
                                           const int32_t* __restrict__ list,
                                           const GasSel* __restrict__ sels,
                                           const int32_t* __restrict__ count, const BlockTile& bt,
                                           RO res,
                                           uint64_t* __restrict__ fit) {
  const int32_t lane = threadIdx.x & 63;
  const uint64_t live = __ballot(valid && node_ok != 0u);
  int32_t i0, i1;
  list_share(count, bt, &i0, &i1);
  // lists with a skipped kind read chosen cards back from the lane's LDS copy (kC = Q - 1)
  constexpr bool kGather = Q > 1 && SKIP >= 0;
  constexpr int kC = Q > 1 ? Q - 1 : 1;
  const FreeTab<kC> tab{tab_base};
  if (kGather && i0 < i1) fill_tab_t<Q, SKIP, kC>(free_t, n, valid, N, tab, lane);
  // a batch's rows are loaded one batch ahead: every load of the next batch is in flight
  // while this batch's pods are evaluated (rows past the batch: zeros, not read)
  constexpr int kIters = kMB * kRowChunks / 64;
  int4 v[kIters];
  int32_t wd = 0;
  auto load_batch = [&](int32_t b0) {
    const int32_t nb = max(0, min(kMB, i1 - b0));
    const int4* src = reinterpret_cast<const int4*>(sels + (int64_t)b0 * kPacked);
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int32_t c = lane + it * 64;
      v[it] = c < nb * kRowChunks ? src[c] : int4{0, 0, 0, 0};
    }
    wd = lane < nb ? list[b0 + lane] : 0;
  };
  if (i0 < i1) load_batch(i0);
  for (int32_t b0 = i0; b0 < i1; b0 += kMB) {
    const int32_t nb = min(kMB, i1 - b0);
    __builtin_amdgcn_wave_barrier();  // the previous batch's stage reads are done
#pragma unroll
    for (int it = 0; it < kIters; ++it) reinterpret_cast<int4*>(stage)[lane + it * 64] = v[it];
    // for the sequential class: which selections repeat the previous one, for the whole batch
    // in one ballot (lane l holds 16-B piece l % 4 of selection (l % 32) / 4 of row l / 32)
    static_assert(kIters == 1 && kMB * kRowChunks == 64 && sizeof(GasSel) == 64, "pieces");
    uint64_t same_m;
    {
      const int4 u = v[0];
      const int ux = __shfl_up(u.x, 4, 64), uy = __shfl_up(u.y, 4, 64);
      const int uz = __shfl_up(u.z, 4, 64), uw = __shfl_up(u.w, 4, 64);
      same_m = __ballot((lane & 31) >= 4 && u.x == ux && u.y == uy && u.z == uz && u.w == uw);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    // the batch's pod words straight from the staging register (lane j: pod j's word)
    const int32_t wcur = wd;
    load_batch(b0 + kMB);
    for (int32_t j = 0; j < nb; ++j) {
      const int32_t pw = __builtin_amdgcn_readlane(wcur, j);
      const int32_t pod = pw & 0xFFFFFF;
      const int32_t S = (pw >> 24) & 0xF;
      const GasSel* rec = stage + j * kPacked;
      if (!kBits && S > kPacked) continue;  // the generic kernel's row (it runs beside this one)
      uint32_t out = 0u;
      if (!(pw & kBadPod)) {
        if (S <= kPacked) {  // 4..8 in order (more: the generic kernel's, 0 here)
          if constexpr (kGather) {
            int64_t free[kMaxCards][Q];
            load_free_t<Q>(n, valid, N, free_t, free);
            out = multi_seq<Q, SKIP, kC>(free, rec, S, live, node_ok, tab, lane,
                                         (uint32_t)(same_m >> (32 * j)));
          } else {
            out = multi_state<Q, SKIP>(free_t, n, valid, N, rec, S, live, node_ok);
          }
        }
      }
      put_result<kBits>(res, fit, pod, N, n, valid, out);
    }
  }
}

// Pods of 4 to 8 selections of a list with a skipped kind, with fit masks from group ranks
// (multi_seq<..., true>): the list is cut into groups of 15 pods (8 rows each), a chunk takes
// whole groups; per group the node's cards are ranked once, then batches of kMB pods (their
// 64-bit rows for the current-free checks and their rank rows) are staged as in multi_list.
// LDS: the FreeTab copy, then the sorted rows of the ranking, overlaid by the batch stage.
template <int Q, int SKIP, bool kBits, class RO>
__device__ __forceinline__ void rseq_list(const int64_t* __restrict__ free_t, char* wlds,
                                          uint32_t node_ok, int32_t N, int32_t n, bool valid,
                                          const int32_t* __restrict__ list,
                                          const GasSel* __restrict__ sels,
                                          const GasRSeq* __restrict__ rq,
                                          const int64_t* __restrict__ srt, int64_t item0,
                                          int32_t cnt, const BlockTile& bt, RO res,
                                          uint64_t* __restrict__ fit) {
  constexpr int kC = Q - 1;
  const int32_t lane = threadIdx.x & 63;
  const FreeTab<kC> tab{reinterpret_cast<int64_t*>(wlds)};
  char* over = wlds + sizeof(int64_t) * kMaxCards * 64 * kC;
  int64_t* lds = reinterpret_cast<int64_t*>(over);
  GasSel* stage = reinterpret_cast<GasSel*>(over);
  GasRSeq* rstage = reinterpret_cast<GasRSeq*>(stage + kMB * kPacked);
  constexpr int32_t gs = kRankMax / kPacked;
  int32_t g0, g1;
  chunk_groups(cnt, bt.chunks, bt.chunk, gs, &g0, &g1);
  if (g0 < g1) fill_tab_t<Q, SKIP, kC>(free_t, n, valid, N, tab, lane);
  static_assert(kMB * kRowChunks == 64 && sizeof(GasSel) == 64, "one 16-B piece per lane");
  static_assert(kMB * sizeof(GasRSeq) / 16 <= 64, "rank rows");
  constexpr int kRWords = (int)(sizeof(GasRSeq) / 16);
  for (int32_t gi = g0; gi < g1; ++gi) {
    const int32_t gb = gi * gs, ge = min(cnt, gb + gs);
    load_sorted<kC>(srt, item0 + (int64_t)gb * kPacked, (ge - gb) * kPacked, lds, lane);
    uint32_t fa[kC], fb[kC];
    rank_cards_t<Q, SKIP, kC>(free_t, n, valid, N, lds, (ge - gb) * kPacked, fa, fb);
    for (int32_t b0 = gb; b0 < ge; b0 += kMB) {
      const int32_t nb = __builtin_amdgcn_readfirstlane(min(kMB, ge - b0));
      const int4* src = reinterpret_cast<const int4*>(sels + (int64_t)b0 * kPacked);
      const int4 v = lane < nb * kRowChunks ? src[lane] : int4{0, 0, 0, 0};
      const int4* rsrc = reinterpret_cast<const int4*>(rq + b0);
      const int4 rv = lane < nb * kRWords ? rsrc[lane] : int4{0, 0, 0, 0};
      const int32_t wd = lane < nb ? list[b0 + lane] : 0;
      __builtin_amdgcn_wave_barrier();  // the previous batch's (or the ranking's) reads are done
      reinterpret_cast<int4*>(stage)[lane] = v;
      if (lane < kMB * kRWords) reinterpret_cast<int4*>(rstage)[lane] = rv;
      uint64_t same_m;  // selections repeating the previous one (as multi_list)
      {
        const int ux = __shfl_up(v.x, 4, 64), uy = __shfl_up(v.y, 4, 64);
        const int uz = __shfl_up(v.z, 4, 64), uw = __shfl_up(v.w, 4, 64);
        same_m = __ballot((lane & 31) >= 4 && v.x == ux && v.y == uy && v.z == uz && v.w == uw);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
      const GasSel* st = lane_ptr(stage);  // (lane_ptr: record reads at immediate offsets)
      const GasRSeq* rst = lane_ptr(rstage);
      for (int32_t j = 0; j < nb; ++j) {
        const int32_t pw = __builtin_amdgcn_readlane(wd, j);
        const int32_t pod = pw & 0xFFFFFF;
        const int32_t S = (pw >> 24) & 0xF;
        if (!kBits && S > kPacked) continue;  // the generic kernel's row (it runs beside this one)
        uint32_t out = 0u;
        if (!(pw & kBadPod) && S <= kPacked)  // more: the generic kernel's (bitmaps: 0 here)
          out = multi_seq<Q, SKIP, kC, true>(nullptr, st + j * kPacked, S, 0, node_ok, tab, lane,
                                             (uint32_t)(same_m >> (32 * j)),
                                             &rst[j].rep[0][0], fa, fb);
        put_result<kBits>(res, fit, pod, N, n, valid, out);
      }
    }
  }
}

// Four-selection pods in closed form (class kClsFour: lists with a skipped kind).  Selection t
// takes the first card whose free covers its need plus the takes already on that card
// (getCardsForContainerGPURequest, scheduler.go:200-257; addRM, resource_map.go:38-53).  A
// card no earlier selection took from passes iff it is in the mask of the selection's own need
// (ranks, as rclosed); a card that earlier selections took from passes iff its snapshot free
// covers the threshold row of exactly those selections (GasFour), checked at that one card on
// its 64-bit free values from the lane's LDS copy (FreeTab).  With e_ab = (c_a == c_b):
//   c0 = lowest(m0)
//   c1 = min(lowest(m1 \ {c0}), c0 if row 2 fits at c0)
//   c2 = min(lowest(m2 \ {c0, c1}), c0 if row (e01 ? 6 : 4) fits at c0,
//            c1 if !e01 and row 5 fits at c1)
//   c3 = min(lowest(m3 \ {c0, c1, c2}), c0 if row 8 + 2 e01 + 4 e02 fits at c0,
//            c1 if !e01 and row 9 + 4 e12 fits at c1, c2 if !e02, !e12 and row 11 fits at c2)
// Card positions are mask bit positions 4c + 3 (0xFFFFFFFF: none, as rclosed).
// The pod's GasFour from row 2 on, as staged in LDS (rows 0, 1, 3, 7 are ranked instead).
struct alignas(16) FourStage {
  int64_t th[13][PAS_GAS_MAX_RES];  // GasFour rows 2 .. 14
  int32_t flags;
  int32_t pad[3];
};
static_assert(sizeof(FourStage) + 2 * sizeof(int64_t) * PAS_GAS_MAX_RES == sizeof(GasFour) &&
                  offsetof(GasFour, flags) == 15 * sizeof(int64_t) * PAS_GAS_MAX_RES,
              "FourStage is GasFour from row 2 on");
constexpr int kFourMB = 4;  // four-selection pods staged per batch and wave

template <int Q, int SKIP, int kC>
__device__ __forceinline__ uint32_t rfour(const uint32_t (&fa)[kC], const uint32_t (&fb)[kC],
                                          const GasRFour& rk, const FourStage& st, uint32_t flags,
                                          const FreeTab<kC>& tab, int lane) {
  constexpr uint32_t kNone = ~0u;
  auto mask = [&](int t) {
    uint32_t g[kC];
#pragma unroll
    for (int j = 0; j < kC; ++j) g[j] = rk.rep[t][j];
    return rmask<kC>(fa, fb, g);
  };
  auto load = [&](uint32_t p, int64_t (&f)[kC]) {
    const int64_t* x = tab.at(min(p >> 2, 7u), lane);
#pragma unroll
    for (int j = 0; j < kC; ++j) f[j] = x[j];
  };
  // row r >= 2 fits at a card of snapshot free f (and does not overflow).  Every check is
  // evaluated and combined with bitwise operations: straight-line compares and lane-mask
  // logic, no divergent branches around the threshold loads
  auto fits = [&](int r, const int64_t (&f)[kC]) {
    bool ok = ((flags >> r) & 1u) == 0u;
#pragma unroll
    for (int q = 0, j = 0; q < Q; ++q)
      if (q != SKIP) ok = ok & (st.th[r - 2][q] <= f[j++]);
    return ok;
  };
  const uint32_t m0 = mask(0);
  const uint32_t m1 = ((flags >> (kFourSame + 1)) & 1u) ? m0 : mask(1);
  const uint32_t m2 = ((flags >> (kFourSame + 2)) & 1u) ? m1 : mask(2);
  const uint32_t m3 = ((flags >> (kFourSame + 3)) & 1u) ? m2 : mask(3);
  int64_t f0[kC], f1[kC], f2[kC];
  const uint32_t p0 = lowbit(m0);
  load(p0, f0);
  const uint32_t b0 = 1u << (p0 & 31u);
  const uint32_t p1 = min(lowbit(m1 & ~b0), fits(2, f0) ? p0 : kNone);
  load(p1, f1);
  const uint32_t b1 = 1u << (p1 & 31u);
  const bool e01 = p0 == p1;
  const bool r4 = fits(4, f0), r6 = fits(6, f0), r5 = fits(5, f1);
  const bool a0 = (e01 & r6) | (!e01 & r4);
  const bool a1 = !e01 & r5;
  const uint32_t p2 = min(lowbit(m2 & ~(b0 | b1)), min(a0 ? p0 : kNone, a1 ? p1 : kNone));
  load(p2, f2);
  const uint32_t b2 = 1u << (p2 & 31u);
  const bool e02 = p0 == p2, e12 = p1 == p2;
  const bool r8 = fits(8, f0), r10 = fits(10, f0), r12 = fits(12, f0), r14 = fits(14, f0);
  const bool r9 = fits(9, f1), r13 = fits(13, f1), r11 = fits(11, f2);
  const bool c0 = (e01 & ((e02 & r14) | (!e02 & r10))) | (!e01 & ((e02 & r12) | (!e02 & r8)));
  const bool c1 = !e01 & ((e12 & r13) | (!e12 & r9));
  const bool c2 = !e02 & !e12 & r11;
  const uint32_t p3 = min(min(lowbit(m3 & ~(b0 | b1 | b2)), c0 ? p0 : kNone),
                          min(c1 ? p1 : kNone, c2 ? p2 : kNone));
  // card fields as arithmetic shifts: a selection without a card makes the word negative
  const int32_t word = ((int32_t)p0 >> 2) | (((int32_t)p1 >> 2) << 3) |
                       (((int32_t)p2 >> 2) << 6) | (((int32_t)p3 >> 2) << 9);
  return (uint32_t)min(word ^ (int32_t)(0x80000000u | (4u << 24)), 0);
}

// The closed-form four-selection pods of a list with a skipped kind: groups of 31 pods (their
// 4 full-mask rows ranked), a chunk takes whole groups; per group the node's cards are ranked
// once, then batches of kFourMB pods (FourStage + GasRFour) are staged as in rseq_list.
template <int Q, int SKIP, bool kBits, class RO>
__device__ __forceinline__ void rfour_list(const int64_t* __restrict__ free_t, char* wlds,
                                           uint32_t node_ok, int32_t N, int32_t n, bool valid,
                                           const int32_t* __restrict__ list,
                                           const GasSel* __restrict__ sels,
                                           const GasRFour* __restrict__ rf,
                                           const int64_t* __restrict__ srt, int64_t item0,
                                           int32_t cnt, const BlockTile& bt, RO res,
                                           uint64_t* __restrict__ fit) {
  constexpr int kC = Q - 1;
  const int32_t lane = threadIdx.x & 63;
  const FreeTab<kC> tab{reinterpret_cast<int64_t*>(wlds)};
  char* over = wlds + sizeof(int64_t) * kMaxCards * 64 * kC;
  int64_t* lds = reinterpret_cast<int64_t*>(over);
  FourStage* stage = reinterpret_cast<FourStage*>(over);
  GasRFour* rstage = reinterpret_cast<GasRFour*>(stage + kFourMB);
  constexpr int32_t gs = kRankMax / 4;
  int32_t g0, g1;
  chunk_groups(cnt, bt.chunks, bt.chunk, gs, &g0, &g1);
  if (g0 < g1) fill_tab_t<Q, SKIP, kC>(free_t, n, valid, N, tab, lane);
  constexpr int kPieces = (int)(sizeof(FourStage) / 16), kRPieces = (int)(sizeof(GasRFour) / 16);
  constexpr int kIters = (kFourMB * kPieces + 63) / 64;
  static_assert(kFourMB * kRPieces <= 64, "rank rows");
  constexpr size_t kSkipRows = 2 * sizeof(int64_t) * PAS_GAS_MAX_RES;  // GasFour rows 0, 1
  for (int32_t gi = g0; gi < g1; ++gi) {
    const int32_t gb = gi * gs, ge = min(cnt, gb + gs);
    load_sorted<kC>(srt, item0 + (int64_t)gb * 4, (ge - gb) * 4, lds, lane);
    uint32_t fa[kC], fb[kC];
    rank_cards_t<Q, SKIP, kC>(free_t, n, valid, N, lds, (ge - gb) * 4, fa, fb);
    for (int32_t b0 = gb; b0 < ge; b0 += kFourMB) {
      const int32_t nb = __builtin_amdgcn_readfirstlane(min(kFourMB, ge - b0));
      int4 v[kIters];
#pragma unroll
      for (int it = 0; it < kIters; ++it) {
        const int32_t c = lane + 64 * it, pod = c / kPieces, pc = c % kPieces;
        const int4* src = reinterpret_cast<const int4*>(
            reinterpret_cast<const char*>(sels + (int64_t)(b0 + min(pod, nb - 1)) * kPacked) +
            kSkipRows);
        v[it] = pod < nb ? src[pc] : int4{0, 0, 0, 0};
      }
      const int4 rv = lane < nb * kRPieces ? reinterpret_cast<const int4*>(rf + b0)[lane]
                                           : int4{0, 0, 0, 0};
      const int32_t wd = lane < nb ? list[b0 + lane] : 0;
      __builtin_amdgcn_wave_barrier();  // the previous batch's (or the ranking's) reads are done
#pragma unroll
      for (int it = 0; it < kIters; ++it)
        if (lane + 64 * it < kFourMB * kPieces) reinterpret_cast<int4*>(stage)[lane + 64 * it] = v[it];
      if (lane < kFourMB * kRPieces) reinterpret_cast<int4*>(rstage)[lane] = rv;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
      const FourStage* st = lane_ptr(stage);  // (lane_ptr: record reads at immediate offsets)
      const GasRFour* rst = lane_ptr(rstage);
#pragma unroll
      for (int j = 0; j < kFourMB; ++j) {
        if (j >= nb) break;
        const int32_t pod = __builtin_amdgcn_readlane(wd, j) & 0xFFFFFF;
        const uint32_t flags = (uint32_t)__builtin_amdgcn_readfirstlane(st[j].flags);
        uint32_t out = rfour<Q, SKIP, kC>(fa, fb, rst[j], st[j], flags, tab, lane);
        if constexpr (kBits) out = out ? node_ok : 0u;
        put_result<kBits>(res, fit, pod, N, n, valid, out);
      }
    }
  }
}

// The closed-form four-selection lists l = 1 .. Q (list 0 files its four-selection pods as
// sequential ones).  item0: the first sorted row of list 1's groups (after the sequential ones).
template <int Q, bool kBits, int l = 1, class RO>
__device__ __forceinline__ void four_lists(const int64_t* __restrict__ free_t, char* wlds,
                                           uint32_t node_ok, int32_t N, int32_t n, bool valid,
                                           int32_t P, const int32_t* __restrict__ multi,
                                           const GasSel* __restrict__ sels,
                                           const GasRFour* __restrict__ rf,
                                           const int64_t* __restrict__ srt, int64_t item0,
                                           const int32_t* __restrict__ counts, const BlockTile& bt,
                                           RO res, uint64_t* __restrict__ fit) {
  constexpr int L = l * kClasses + kClsFour;
  const int32_t cnt = __builtin_amdgcn_readfirstlane(counts[L]);
  rfour_list<Q, l - 1, kBits>(free_t, wlds, node_ok, N, n, valid, multi + (int64_t)L * P,
                              sels + (int64_t)L * P * kPacked, rf + (int64_t)l * P, srt, item0,
                              cnt, bt, res, fit);
  __builtin_amdgcn_wave_barrier();
  if constexpr (l < Q)
    four_lists<Q, kBits, l + 1>(free_t, wlds, node_ok, N, n, valid, P, multi, sels, rf, srt,
                                item0 + (int64_t)cnt * 4, counts, bt, res, fit);
}

// The lists of pods with 4 to 8 selections (class 2 of each kind-skip list): ranked where a
// kind is skipped (rseq_list), else on 64-bit values (multi_list).  item0: the first sorted
// row of list 1's groups (after the two- and three-selection lists' rows).
template <int Q, bool kBits, int l = 0, class RO>
__device__ __forceinline__ void seq_lists(const int64_t* __restrict__ free_t, char* wlds,
                                          uint32_t node_ok, int32_t N, int32_t n, bool valid,
                                          int32_t P, const int32_t* __restrict__ multi,
                                          const GasSel* __restrict__ sels,
                                          const GasRSeq* __restrict__ rq,
                                          const int64_t* __restrict__ srt, int64_t item0,
                                          const int32_t* __restrict__ counts, const BlockTile& bt,
                                          RO res, uint64_t* __restrict__ fit) {
  constexpr int L = l * kClasses + 2;
  int32_t cnt = 0;
  if constexpr (l == 0 || Q == 1) {
    GasSel* stage = reinterpret_cast<GasSel*>(wlds);
    int64_t* tab = reinterpret_cast<int64_t*>(stage + kPacked * kMB);
    multi_list<Q, l - 1, kBits>(free_t, stage, tab, node_ok, N, n, valid, multi + (int64_t)L * P,
                                sels + (int64_t)L * P * kPacked, counts + L, bt, res, fit);
  } else {
    cnt = __builtin_amdgcn_readfirstlane(counts[L]);
    rseq_list<Q, l - 1, kBits>(free_t, wlds, node_ok, N, n, valid, multi + (int64_t)L * P,
                               sels + (int64_t)L * P * kPacked, rq + (int64_t)l * P, srt, item0,
                               cnt, bt, res, fit);
  }
  __builtin_amdgcn_wave_barrier();
  if constexpr (l < Q)
    seq_lists<Q, kBits, l + 1>(free_t, wlds, node_ok, N, n, valid, P, multi, sels, rq, srt,
                               item0 + (int64_t)cnt * kPacked, counts, bt, res, fit);
}


template <int Q, int SKIP, bool kBits, class RO>
__device__ __forceinline__ void rsingle_list(const int64_t* __restrict__ free_t,
                                             uint32_t node_ok, int32_t N, int32_t n, bool valid,
                                             const GasRSingle* __restrict__ rs,
                                             const int64_t* __restrict__ srt, int64_t item0,
                                             int32_t cnt, const BlockTile& bt, int64_t* lds,
                                             GasRSingle* stage, RO res,
                                             uint64_t* __restrict__ fit) {
  constexpr int kSkip = Q == 1 ? -1 : SKIP;
  constexpr int C = Q - (kSkip >= 0 ? 1 : 0);
  const int lane = threadIdx.x & 63;
  // this chunk's group (one-selection lists: chunk = group)
  const int32_t gb = min(cnt, bt.chunk * kRankMax), ge = min(cnt, gb + kRankMax);
  if (gb >= ge) return;
  uint32_t fa[C], fb[C];
  // the node's free values only while ranking, one kind at a time (registers for the pod loop)
  load_sorted<C>(srt, item0 + gb, ge - gb, lds, lane);
  rank_cards_t<Q, kSkip, C>(free_t, n, valid, N, lds, ge - gb, fa, fb);
  // a node that fits nothing (no cards label, not in the lister, past the fast kernels' card
  // count) as eight cards of rank 0: every one-selection row compares at least one kind of
  // rank >= 1 (the last kind a selection requests is never skipped), so its mask is empty
  // and the pod loop needs no node_ok (pods without a selection still take node_ok)
#pragma unroll
  for (int j = 0; j < C; ++j) {
    fa[j] = node_ok ? fa[j] : 0x80808080u;
    fb[j] = node_ok ? fb[j] : 0x80808080u;
  }
  // Every pod takes one path: a pod without a selection ranks 1 in every kind and a bad pod
  // 0x80 (gas_prep_kernel, rank_group), so m is empty exactly where its word is 0, and
  //   word = m ? base | lowest card : 0,  base = 0x81000000 (one selection) / 0x80000000 (none)
  // is min_i32((ffbl(m) >> 2) ^ base, 0): ffbl(0) = -1 turns base into a positive value.
  auto one_pod = [&](const GasRSingle& r, int32_t w) {
    const int64_t pod = w & 0xFFFFFF;
    uint32_t g[C];
#pragma unroll
    for (int jj = 0; jj < C; ++jj) g[jj] = r.g[jj];
    const uint32_t m = rmask<C>(fa, fb, g);
    uint32_t out;
    if constexpr (kBits) {
      out = m ? 0x80000000u : 0u;
    } else {
      // base = 0x80000000 | steps << 24 (steps <= 1): one scalar AND, a three-input XOR
      const int32_t sbits = (int32_t)((uint32_t)w & 0x0F000000u);
      out = (uint32_t)min((((int32_t)ffbl(m) >> 2) ^ sbits) ^ (int32_t)0x80000000u, 0);
    }
    put_result<kBits>(res, fit, pod, N, n, valid, out);
  };
  for (int32_t b0 = gb; b0 < ge; b0 += kPodBatch) {
    const int32_t nb = __builtin_amdgcn_readfirstlane(min(kPodBatch, ge - b0));
    constexpr int kWords = (int)(sizeof(GasRSingle) / 16);
    constexpr int kIters = kPodBatch * kWords / 64;
    const int4* src = reinterpret_cast<const int4*>(rs + b0);
    int4 v[kIters];
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int32_t c = lane + it * 64;
      v[it] = c < nb * kWords ? src[c] : int4{0, 0, 0, 0};
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < kIters; ++it) reinterpret_cast<int4*>(stage)[lane + it * 64] = v[it];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    // pods in pairs: both records read (broadcast LDS reads) before the first one's tests;
    // eight pods per iteration, so the records' LDS offsets are constants off one address
    for (int32_t j0 = 0; j0 < nb; j0 += 8) {
      const GasRSingle* st = lane_ptr(stage) + j0;
      if (PAS_GAS_RUN_FAST && j0 + 8 <= nb) {
        // a full run of 8: straight-line code (no exit test between pods), so the pods'
        // record reads and tests interleave
        GasRSingle r[8];
        int32_t w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = st[u];
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = __builtin_amdgcn_readfirstlane(r[u].word);
#pragma unroll
        for (int u = 0; u < 8; ++u) one_pod(r[u], w[u]);
        continue;
      }
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        if (j0 + u >= nb) break;
        const GasRSingle r0 = st[u], r1 = st[u + 1];
        const int32_t w0 = __builtin_amdgcn_readfirstlane(r0.word);
        const int32_t w1 = __builtin_amdgcn_readfirstlane(r1.word);
        one_pod(r0, w0);
        if (j0 + u + 1 < nb) one_pod(r1, w1);
      }
    }
  }
}

template <int Q, bool kBits, int L = 0, class RO>
__device__ __forceinline__ void rsingle_lists(const int64_t* __restrict__ free_t,
                                              uint32_t node_ok, int32_t N, int32_t n, bool valid,
                                              int32_t P, const GasRSingle* __restrict__ rs,
                                              const int64_t* __restrict__ srt, int64_t item0,
                                              const int32_t* __restrict__ counts,
                                              const BlockTile& bt, int64_t* lds,
                                              GasRSingle* stage, RO res,
                                              uint64_t* __restrict__ fit) {
  const int32_t cnt = __builtin_amdgcn_readfirstlane(counts[L]);
  rsingle_list<Q, L - 1, kBits>(free_t, node_ok, N, n, valid, rs + (int64_t)L * P, srt, item0,
                                cnt, bt, lds, stage, res, fit);
  if constexpr (L < Q)
    rsingle_lists<Q, kBits, L + 1>(free_t, node_ok, N, n, valid, P, rs, srt, item0 + cnt, counts,
                                   bt, lds, stage, res, fit);
}

// LDS of one wave of the one-selection path: the group's sorted rows, then the pod stage.
template <int Q>
struct SingleLds {
  static constexpr size_t kBytes = sizeof(int64_t) * Q * kRankItems + sizeof(GasRSingle) * kPodBatch;
};

template <int Q, bool kBits, class RO>
__device__ __forceinline__ void rfit_single_body(
    const BlockTile& bt, char* wlds, int32_t N, int32_t P, const int32_t* __restrict__ n_cards,
    const int64_t* __restrict__ free_t, const GasRSingle* __restrict__ rs,
    const int64_t* __restrict__ srt, const int32_t* __restrict__ counts, RO res,
    uint64_t* __restrict__ fit) {
  // chunks past every list's end: nothing to load
  int32_t most = 0;
#pragma unroll
  for (int l = 0; l <= Q; ++l) most = max(most, counts[l]);
  if (bt.chunk * kRankMax >= __builtin_amdgcn_readfirstlane(most)) return;
  const int32_t n = bt.node_block * kSingleTpb + threadIdx.x;
  const bool in = n < N;
  const int32_t nc = in ? n_cards[n] : 0;
  // word results: a node past the fast kernels' card count is the generic kernel's alone (it
  // runs beside them), so its lane stores nothing here
  const bool valid = in && (kBits || nc <= kMaxCards);
  const uint32_t node_ok = (nc > 0 && nc <= kMaxCards) ? 0x80000000u : 0u;
  int64_t* lds = reinterpret_cast<int64_t*>(wlds);
  GasRSingle* stage = reinterpret_cast<GasRSingle*>(wlds + sizeof(int64_t) * Q * kRankItems);
  rsingle_lists<Q, kBits>(free_t, node_ok, N, n, valid, P, rs, srt, 0, counts, bt, lds, stage,
                          res, fit);
}

// kSoff: word results through put_result(ResSoff) (a batch of < 2^31 result bytes)
template <int Q, bool kBits, bool kSoff>
__global__ __launch_bounds__(kSingleTpb) void gas_rfit_single_kernel(
    int32_t N, int32_t K, int32_t P, const int32_t* __restrict__ n_cards,
    const int64_t* __restrict__ free_t, const GasRSingle* __restrict__ rs, const int64_t* __restrict__ srt,
    const int32_t* __restrict__ counts, int32_t chunks, ResOut res,
    uint64_t* __restrict__ fit) {
  __shared__ int4 smem[kSingleTpb / 64][SingleLds<Q>::kBytes / 16];  // a slice per wave
  if (fit_aborted(res.abort, res.epoch)) return;
  const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr (kSoff)
    rfit_single_body<Q, kBits>(block_tile(chunks), reinterpret_cast<char*>(smem[wave]), N, P,
                               n_cards, free_t, rs, srt, counts, ResSoff(res, P), fit);
  else
    rfit_single_body<Q, kBits>(block_tile(chunks), reinterpret_cast<char*>(smem[wave]), N, P,
                               n_cards, free_t, rs, srt, counts, res, fit);
}

// A row of packed ranks (byte j = kind j) checked at one card: x = the card's packed ranks
// + 0x80 (the lane's table), every compared byte keeps bit 7.
template <int C>
__device__ __forceinline__ bool rpoint(uint32_t x, uint32_t gp) {
  constexpr uint32_t kMc = C == 1 ? 0x80u : C == 2 ? 0x8080u : C == 3 ? 0x808080u : 0x80808080u;
  return ((x - gp) & kMc) == kMc;
}

// Two- and three-selection pods in closed form on ranks.  Selection t takes the first card
// whose free covers its need plus the takes already on that card (getCardsForContainerGPU-
// Request, scheduler.go:200-257; addRM, resource_map.go:38-53); which earlier takes those are
// depends only on the earlier choices, so every combination is one threshold row
// (GasThresholds):
//   c0 = lowest(m0)
//   c1 = min(lowest(m1 without c0), c0 if row 2 fits at c0)
//   c2 = min(lowest(m3 without c0, c1),
//            c0 == c1 ? (c0 if row 6 fits at c0) : min(c0 if row 4 fits at c0, c1 if row 5 at c1))
// Masks of rows 0, 1, 3 from the group ranks; rows 2, 4, 5, 6 checked at the chosen card on
// its packed ranks from the lane's table.  Card positions are bit positions 4c + 3
// (0xFFFFFFFF: none), so min() picks the lower card and none loses.
template <int C, int S>
__device__ __forceinline__ uint32_t rclosed(const uint32_t (&fa)[C], const uint32_t (&fb)[C],
                                           const GasRMulti& r, uint32_t w, const uint32_t* tab,
                                           int lane, uint32_t node_ok) {
  uint32_t g0[C], g1[C];
#pragma unroll
  for (int j = 0; j < C; ++j) {
    g0[j] = r.rep[0][j];
    g1[j] = r.rep[1][j];
  }
  const uint32_t m0 = rmask<C>(fa, fb, g0);
  const uint32_t m1 = (w & kSame01) ? m0 : rmask<C>(fa, fb, g1);
  const uint32_t p0 = lowbit(m0);
  const uint32_t x0 = tab[min(p0 >> 2, 7u) * 64 + lane];
  const uint32_t u1 = lowbit(m1 & ~(1u << (p0 & 31u)));
  const uint32_t p1 = rpoint<C>(x0, r.pk[0]) ? min(u1, p0) : u1;
  // card fields as arithmetic shifts: a selection without a card (position -1) makes the
  // word negative, whatever the other fields hold
  int32_t word = ((int32_t)p0 >> 2) | (((int32_t)p1 >> 2) << 3);
  if constexpr (S == 3) {
    uint32_t g3[C];
#pragma unroll
    for (int j = 0; j < C; ++j) g3[j] = r.rep[2][j];
    const uint32_t m3 = (w & kSame03) ? m0 : (w & kSame13) ? m1 : rmask<C>(fa, fb, g3);
    const uint32_t x1 = tab[min(p1 >> 2, 7u) * 64 + lane];
    // c0 == c1: row 6 at c0; else row 4 at c0, row 5 at c1 (every check evaluated, combined
    // bitwise: no divergent branch)
    const bool e01 = p0 == p1;
    const bool r6 = rpoint<C>(x0, r.pk[3]), r4 = rpoint<C>(x0, r.pk[1]);
    const bool r5 = rpoint<C>(x1, r.pk[2]);
    const uint32_t touched = min(((e01 & r6) | (!e01 & r4)) ? p0 : ~0u, (!e01 & r5) ? p1 : ~0u);
    const uint32_t un = lowbit(m3 & ~(1u << (p0 & 31u)) & ~(1u << (p1 & 31u)));
    const uint32_t p2 = min(un, touched);
    word |= ((int32_t)p2 >> 2) << 6;
  }
  // base = pass | S: a complete word xors to a negative value (kept by the min), a negative
  // word to a positive one (0).  A node without cards (every free -1) has empty masks, so
  // node_ok is not needed here; bitmap results take it at the caller.
  (void)node_ok;
  return (uint32_t)min(word ^ (int32_t)(0x80000000u | ((uint32_t)S << 24)), 0);
}

template <int Q, int SKIP, int S, bool kBits, class RO>
__device__ __forceinline__ void rmulti_list(const int64_t* __restrict__ free_t, uint32_t node_ok,
                                            int32_t N, int32_t n, bool valid,
                                            const GasRMulti* __restrict__ rm,
                                            const int32_t* __restrict__ rw,
                                            const int64_t* __restrict__ srt, int64_t item0,
                                            int32_t cnt, const BlockTile& bt, int64_t* lds,
                                            GasRMulti* stage, uint32_t* tab,
                                            RO res,
                                            uint64_t* __restrict__ fit) {
  constexpr int kSkip = Q == 1 ? -1 : SKIP;
  constexpr int C = Q - (kSkip >= 0 ? 1 : 0);
  constexpr int R = S == 2 ? 3 : 7;
  const int lane = threadIdx.x & 63;
  constexpr int32_t gs = kRankMax / R;
  int32_t g0, g1;
  chunk_groups(cnt, bt.chunks, bt.chunk, gs, &g0, &g1);
  for (int32_t gi = g0; gi < g1; ++gi) {
    const int32_t gb = gi * gs, ge = min(cnt, gb + gs);
    load_sorted<C>(srt, item0 + (int64_t)gb * R, (ge - gb) * R, lds, lane);
    uint32_t fa[C], fb[C];
    rank_cards_t<Q, kSkip, C>(free_t, n, valid, N, lds, (ge - gb) * R, fa, fb);
    // the lane's table: card k's packed ranks (byte j = kind j)
#pragma unroll
    for (int k = 0; k < kMaxCards; ++k) {
      uint32_t x = 0u;
#pragma unroll
      for (int j = 0; j < C; ++j)
        x |= (((k & 1 ? fb[j] : fa[j]) >> (8 * (k >> 1))) & 0xFFu) << (8 * j);
      tab[k * 64 + lane] = x;
    }
    for (int32_t b0 = gb; b0 < ge; b0 += kRankMB) {
      const int32_t nb = __builtin_amdgcn_readfirstlane(min(kRankMB, ge - b0));
      constexpr int kWords = (int)(sizeof(GasRMulti) / 16);
      static_assert(kRankMB * kWords == 64, "one 16-B piece per lane");
      const int4* src = reinterpret_cast<const int4*>(rm + b0);
      const int4 v = lane < nb * kWords ? src[lane] : int4{0, 0, 0, 0};
      const int32_t wd = lane < nb ? rw[b0 + lane] : 0;
      __builtin_amdgcn_wave_barrier();
      reinterpret_cast<int4*>(stage)[lane] = v;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
      // four pods per iteration: their records' LDS offsets are constants off one address
      for (int32_t j0 = 0; j0 < nb; j0 += 4) {
        const GasRMulti* st = lane_ptr(stage) + j0;
        if (PAS_GAS_RUN_FAST && j0 + 4 <= nb) {  // a full run: straight-line, as rsingle_list
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t w = (uint32_t)__builtin_amdgcn_readlane(wd, j0 + u);
            uint32_t out = rclosed<C, S>(fa, fb, st[u], w, tab, lane, node_ok);
            if constexpr (kBits) out = out ? node_ok : 0u;
            put_result<kBits>(res, fit, w & 0xFFFFFF, N, n, valid, out);
          }
          continue;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (j0 + u >= nb) break;
          const uint32_t w = (uint32_t)__builtin_amdgcn_readlane(wd, j0 + u);
          const int64_t pod = w & 0xFFFFFF;
          // (a bad pod's row 0 ranks 0x80: its word comes out 0)
          uint32_t out = rclosed<C, S>(fa, fb, st[u], w, tab, lane, node_ok);
          if constexpr (kBits) out = out ? node_ok : 0u;
          put_result<kBits>(res, fit, pod, N, n, valid, out);
        }
      }
    }
  }
}

template <int Q, bool kBits, int L = 0, class RO>
__device__ __forceinline__ void rmulti_lists(const int64_t* __restrict__ free_t, uint32_t node_ok,
                                             int32_t N, int32_t n, bool valid, int32_t P,
                                             const GasRMulti* __restrict__ rm,
                                             const int32_t* __restrict__ rw,
                                             const int64_t* __restrict__ srt, int64_t item0,
                                             const int32_t* __restrict__ counts,
                                             const BlockTile& bt, int64_t* lds, GasRMulti* stage,
                                             uint32_t* tab, RO res,
                                             uint64_t* __restrict__ fit) {
  // slot L: list L / 2, class L % 2 (S = 2 + L % 2); counts of the multi lists [l][kClasses]
  constexpr int l = L / 2, S = 2 + L % 2;
  const int32_t cnt = __builtin_amdgcn_readfirstlane(counts[l * kClasses + L % 2]);
  rmulti_list<Q, l - 1, S, kBits>(free_t, node_ok, N, n, valid, rm + (int64_t)L * P,
                                  rw + (int64_t)L * P, srt, item0, cnt, bt, lds, stage, tab, res,
                                  fit);
  if constexpr (L + 1 < (Q + 1) * 2)
    rmulti_lists<Q, kBits, L + 1>(free_t, node_ok, N, n, valid, P, rm, rw, srt,
                                  item0 + (int64_t)cnt * (S == 2 ? 3 : 7), counts, bt, lds,
                                  stage, tab, res, fit);
}

// Pods with several selections, two kernels so that each gets the registers of its own phase:
// the two- and three-selection lists on ranks (ranked straight from free_t, no register copy of
// the node's free values: 7 waves per SIMD instead of the other kernel's 4), then the lists
// that read the node's 64-bit free values (FreeTab): four to eight selections in order, and
// the closed-form four-selection lists.  (Three-selection pods in that closed form, 3 ranked
// rows instead of 7: the closed kernel's VALU 134 -> 65 M, the other's 74 -> 138 M, C3 0.57-0.59
// -> 0.62 ms: the 4-wave kernel became the fit's critical path.)
template <int Q>
struct MultiLds {
  static constexpr int kC = Q > 1 ? Q - 1 : 1;
  // the closed-form kernel: a group's sorted rows (ranking only), overlaid by the pod batch
  // stage (pod loop only), then the lane's packed-rank table
  static constexpr size_t kRows = sizeof(int64_t) * Q * kRankItems;
  static constexpr size_t kRowsOrStage =
      kRows > sizeof(GasRMulti) * kRankMB ? kRows : sizeof(GasRMulti) * kRankMB;
  static constexpr size_t kRanked = kRowsOrStage + sizeof(uint32_t) * kMaxCards * 64;
  // the sequential kernel: the FreeTab copy, then the sorted rows overlaid by a batch stage
  // (sequential pods or closed-form four-selection pods)
  static constexpr size_t cmax(size_t a, size_t b) { return a > b ? a : b; }
  static constexpr size_t kSeqOver =
      cmax(sizeof(int64_t) * kC * kRankItems,
           cmax(sizeof(GasSel) * kPacked * kMB + sizeof(GasRSeq) * kMB,
                (sizeof(FourStage) + sizeof(GasRFour)) * kFourMB));
  static constexpr size_t kSeq = sizeof(int64_t) * kMaxCards * 64 * kC + kSeqOver;
};

template <int Q, bool kBits, class RO>
__device__ __forceinline__ void rfit_closed_body(
    const BlockTile& bt, char* w, int32_t N, int32_t P, const int32_t* __restrict__ n_cards,
    const int64_t* __restrict__ free_t, const GasRMulti* __restrict__ rm,
    const int32_t* __restrict__ rw, const int64_t* __restrict__ srt,
    const int32_t* __restrict__ counts, RO res, uint64_t* __restrict__ fit) {
  const int32_t n = bt.node_block * kClosedTpb + threadIdx.x;
  const bool in = n < N;
  const int32_t nc = in ? n_cards[n] : 0;
  // word results: a node past the fast kernels' card count is the generic kernel's alone (it
  // runs beside them), so its lane stores nothing here
  const bool valid = in && (kBits || nc <= kMaxCards);
  const uint32_t node_ok = (nc > 0 && nc <= kMaxCards) ? 0x80000000u : 0u;
  int64_t* lds = reinterpret_cast<int64_t*>(w);
  GasRMulti* stage = reinterpret_cast<GasRMulti*>(w);  // overlays the rows (MultiLds)
  uint32_t* tab = reinterpret_cast<uint32_t*>(w + MultiLds<Q>::kRowsOrStage);
  rmulti_lists<Q, kBits>(free_t, node_ok, N, n, valid, P, rm, rw, srt, 0, counts, bt, lds, stage,
                         tab, res, fit);
}

// Waves per SIMD the closed-form kernel is compiled for.  Its LDS (the sorted rows overlaid
// by the pod stage, MultiLds) allows 8 below four kinds.  With all three fit kernels side by
// side, same box, C3 ms: 5 waves (96 VGPRs, 16 B of scratch per lane, the rows and the stage
// apart) 0.710-0.723 -> 6 waves 0.684-0.692 -> overlay 0.660-0.668 -> 7 waves (72 VGPRs,
// 112 B) 0.648-0.649; 8 waves (64 VGPRs, 144 B) 0.669-0.672; 4 waves 0.743-0.748.
#ifndef PAS_GAS_CLOSED_WAVES
#define PAS_GAS_CLOSED_WAVES 7
#endif
template <int Q>
constexpr int closed_waves() { return Q < 4 ? PAS_GAS_CLOSED_WAVES : 5; }
template <int Q, bool kBits, bool kSoff>
__global__ __launch_bounds__(kClosedTpb) __attribute__((amdgpu_waves_per_eu(closed_waves<Q>()))) void gas_rfit_closed_kernel(
    int32_t N, int32_t K, int32_t P, const int32_t* __restrict__ n_cards,
    const int64_t* __restrict__ free_t, const GasRMulti* __restrict__ rm,
    const int32_t* __restrict__ rw, const int64_t* __restrict__ srt,
    const int32_t* __restrict__ counts, int32_t chunks, ResOut res, uint64_t* __restrict__ fit) {
  __shared__ int4 smem[kClosedTpb / 64][MultiLds<Q>::kRanked / 16];
  if (fit_aborted(res.abort, res.epoch)) return;
  const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr (kSoff)
    rfit_closed_body<Q, kBits>(block_tile(chunks), reinterpret_cast<char*>(smem[wave]), N, P,
                               n_cards, free_t, rm, rw, srt, counts, ResSoff(res, P), fit);
  else
    rfit_closed_body<Q, kBits>(block_tile(chunks), reinterpret_cast<char*>(smem[wave]), N, P,
                               n_cards, free_t, rm, rw, srt, counts, res, fit);
}

template <int Q, bool kBits, class RO>
__device__ __forceinline__ void rfit_seq_body(
    const BlockTile& bt, char* w, int32_t N, int32_t P, const int32_t* __restrict__ n_cards,
    const int64_t* __restrict__ free_t, const GasRSeq* __restrict__ rq,
    const GasRFour* __restrict__ rf, const int64_t* __restrict__ srt,
    const int32_t* __restrict__ multi, const GasSel* __restrict__ sels,
    const int32_t* __restrict__ counts, RO res, uint64_t* __restrict__ fit) {
  const int32_t n = bt.node_block * kSeqTpb + threadIdx.x;
  const bool in = n < N;
  const int32_t nc = in ? n_cards[n] : 0;
  // word results: a node past the fast kernels' card count is the generic kernel's alone (it
  // runs beside them), so its lane stores nothing here
  const bool valid = in && (kBits || nc <= kMaxCards);
  const uint32_t node_ok = (nc > 0 && nc <= kMaxCards) ? 0x80000000u : 0u;
  // the sequential lists' sorted rows follow every two- and three-selection list's rows
  int64_t item_seq = 0;
#pragma unroll
  for (int l = 0; l <= Q; ++l)
    item_seq += (int64_t)counts[l * kClasses] * 3 + (int64_t)counts[l * kClasses + 1] * 7;
  seq_lists<Q, kBits>(free_t, w, node_ok, N, n, valid, P, multi, sels, rq, srt,
                      __builtin_amdgcn_readfirstlane(item_seq), counts, bt, res, fit);
  if constexpr (Q > 1) {
    // the closed-form four-selection lists' rows follow the ranked sequential lists' rows
    int64_t item_four = item_seq;
#pragma unroll
    for (int l = 1; l <= Q; ++l) item_four += (int64_t)counts[l * kClasses + kClsSeq] * kPacked;
    four_lists<Q, kBits>(free_t, w, node_ok, N, n, valid, P, multi, sels, rf, srt,
                         __builtin_amdgcn_readfirstlane(item_four), counts, bt, res, fit);
  }
}

template <int Q, bool kBits, bool kSoff>
__global__ __launch_bounds__(kSeqTpb) void gas_rfit_seq_kernel(
    int32_t N, int32_t K, int32_t P, const int32_t* __restrict__ n_cards,
    const int64_t* __restrict__ free_t, const GasRSeq* __restrict__ rq,
    const GasRFour* __restrict__ rf, const int64_t* __restrict__ srt,
    const int32_t* __restrict__ multi, const GasSel* __restrict__ sels,
    const int32_t* __restrict__ counts, int32_t chunks, ResOut res, uint64_t* __restrict__ fit) {
  __shared__ int4 smem[kSeqTpb / 64][MultiLds<Q>::kSeq / 16];
  if (fit_aborted(res.abort, res.epoch)) return;
  const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr (kSoff)
    rfit_seq_body<Q, kBits>(block_tile(chunks), reinterpret_cast<char*>(smem[wave]), N, P,
                            n_cards, free_t, rq, rf, srt, multi, sels, counts, ResSoff(res, P), fit);
  else
    rfit_seq_body<Q, kBits>(block_tile(chunks), reinterpret_cast<char*>(smem[wave]), N, P,
                            n_cards, free_t, rq, rf, srt, multi, sels, counts, res, fit);
}

// ---------------------------------------------------------------------------- generic path
//
// (pod, node) pairs outside the fast kernels' shapes: pods with more than 8 selections
// (every node) and nodes with more than 8 cards (every other pod).  One thread per pair runs
// runSchedulingLogic (scheduler.go:280-338) as the reference writes it: per container
// getPerGPUResourceRequest, then per gpuNum the first card in lexicographic order passing
// checkResourceCapacity (:341-383) on the usage with the pod's earlier takes (addRM); a
// container of more than PAS_GAS_MAX_SELECTIONS selections as card runs (gas_runs.h), its
// pod's word then PAS_GAS_SEL_LIMIT.  The state is private (KMAX cards;
// 64-card snapshots put it in scratch): this is the rare path, not a hot kernel.  Words
// overwrite the fast kernels' zeros; bitmap bits are or-ed in; selections that do not pack
// go to the side buffer.
struct GenericArgs {
  int32_t N, K, Q, C, i915;
  const int32_t* n_cards;
  const int64_t* cap;
  const int64_t* used;
  const int64_t* req;
  const uint32_t* mask;
  const int32_t* ncont;
  const int32_t* big_pods;
  const int32_t* n_big_pods;
  const int32_t* big_nodes;
  const int32_t* n_big_nodes;
  const int32_t* pod_steps;
  int32_t n_pods;
  uint32_t* res;
  int64_t ld;  // result row pitch
  uint64_t* fit;
  pas_gas_selection* side;
  int64_t side_cap;
  unsigned long long* side_count;
  unsigned long long* limit_count;
  const uint32_t* abort;  // as ResOut
  uint32_t epoch;
};

__device__ __forceinline__ bool kind_fits(int64_t need, int64_t cap, int64_t used) {
  if (need < 0 || cap <= 0 || used < 0) return false;
  const int64_t sum = (int64_t)((uint64_t)used + (uint64_t)need);
  return sum >= 0 && cap >= sum;
}

template <int KMAX>
__device__ void fit_pair(const GenericArgs& a, int32_t p, int32_t n) {
  const int32_t Q = a.Q;
  uint32_t word = 0u;
  uint8_t sel[PAS_GAS_MAX_SELECTIONS];
  int64_t nsel = 0;  // the first PAS_GAS_MAX_SELECTIONS are recorded
  bool fits = false;
  const int32_t nc = a.n_cards[n];
  if (nc > 0) {  // FetchNode error / no cards label (:282-298)
    fits = true;
    const int32_t ncard = min(nc, min(a.K, KMAX));
    int64_t w[KMAX][PAS_GAS_MAX_RES];  // readNodeResources copy (node_resource_cache.go:474-491)
    int64_t cap[PAS_GAS_MAX_RES];
    for (int q = 0; q < Q; ++q) cap[q] = a.cap[(int64_t)n * Q + q];
    for (int k = 0; k < ncard; ++k)
      for (int q = 0; q < Q; ++q) w[k][q] = a.used[((int64_t)n * a.K + k) * Q + q];
    // (clamped as gas_prep_kernel does: a device n_containers past max_containers never
    // indexes past the pod's request rows)
    const int32_t nct = min(max(a.ncont[p], 0), a.C);
    for (int32_t c = 0; fits && c < nct; ++c) {
      const int64_t b = (int64_t)p * a.C + c;
      const uint32_t m = a.mask[b];
      if (m == 0u) continue;  // no GPU resources: no cards (:206-208)
      int64_t r[PAS_GAS_MAX_RES];
      for (int q = 0; q < Q; ++q) r[q] = a.req[b * Q + q];
      int64_t num = 0;  // getNumI915 (:192-198)
      if (a.i915 >= 0 && ((m >> a.i915) & 1u) && r[a.i915] > 0) num = r[a.i915];
      if (num > 1)
        for (int q = 0; q < Q; ++q) r[q] /= num;  // getPerGPUResourceRequest (:180-190)
      if (num > kRunsFrom) {  // the pod has more than PAS_GAS_MAX_SELECTIONS: count only
        fits = container_runs<KMAX>(Q, m, r, num, cap, w, ncard,
                                    [&](int, int64_t t) { nsel += t; });
        continue;
      }
      for (int64_t g = 0; g < num; ++g) {
        int chosen = -1;
        for (int k = 0; k < ncard && chosen < 0; ++k) {
          bool ok = !(m & PAS_REQ_UNKNOWN_KIND);  // a key no capacity map has (:349-354)
          for (int q = 0; q < Q; ++q)
            if ((m >> q) & 1u) ok = ok && kind_fits(r[q], cap[q], w[k][q]);
          if (ok) chosen = k;
        }
        if (chosen < 0) {  // errWontFit (:249-253)
          fits = false;
          break;
        }
        for (int q = 0; q < Q; ++q)
          if ((m >> q) & 1u) w[chosen][q] += r[q];  // addRM after a passing check
        if (nsel < PAS_GAS_MAX_SELECTIONS) sel[nsel] = (uint8_t)chosen;
        ++nsel;
      }
    }
  }
  if (fits && nsel > PAS_GAS_MAX_SELECTIONS) {
    word = 0x80000000u | ((uint32_t)PAS_GAS_SEL_LIMIT << 24);  // selection reported at bind
  } else if (fits) {
    bool packable = nsel <= kPacked;
    for (int32_t j = 0; j < nsel; ++j) packable = packable && sel[j] < kMaxCards;
    if (packable) {
      word = 0x80000000u | ((uint32_t)nsel << 24);
      for (int32_t j = 0; j < nsel; ++j) word |= (uint32_t)sel[j] << (3 * j);
    } else {
      word = 0x80000000u | ((uint32_t)PAS_GAS_SEL_EXTENDED << 24);
      if (a.side_count) {
        const unsigned long long slot = atomicAdd(a.side_count, 1ull);
        if ((int64_t)slot < a.side_cap) {
          pas_gas_selection& rec = a.side[slot];
          rec.pod = p;
          rec.node = n;
          rec.n_sel = (int32_t)nsel;
          rec.reserved = 0;
          for (int32_t j = 0; j < PAS_GAS_MAX_SELECTIONS; ++j) rec.card[j] = j < nsel ? sel[j] : 0;
        }
      }
    }
  }
  if (a.fit) {
    if (fits)
      atomicOr(reinterpret_cast<unsigned long long*>(a.fit) + (int64_t)p * ((a.N + 63) / 64) +
                   (n >> 6),
               1ull << (n & 63));
  } else {
    a.res[(int64_t)p * a.ld + n] = word;
  }
}

template <int KMAX>
__global__ __launch_bounds__(64) void gas_fit_generic_kernel(GenericArgs a) {
  if (fit_aborted(a.abort, a.epoch)) return;
  const int64_t nbp = *a.n_big_pods, nbn = *a.n_big_nodes;
  const int64_t seg_a = nbp * a.N, total = seg_a + (int64_t)a.n_pods * nbn;
  for (int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 64) {
    int32_t p, n;
    if (i < seg_a) {  // a pod with more than 8 selections, every node
      p = a.big_pods[i / a.N];
      n = (int32_t)(i % a.N);
      // more than PAS_GAS_MAX_SELECTIONS: evaluated, counted (pas_gas_limit_count)
      if (n == 0 && a.pod_steps[p] > PAS_GAS_MAX_SELECTIONS) atomicAdd(a.limit_count, 1ull);
    } else {  // a node with more than 8 cards, every pod the fast kernels evaluated
      const int64_t j = i - seg_a;
      p = (int32_t)(j / nbn);
      n = a.big_nodes[j % nbn];
      if (a.pod_steps[p] > kPacked) continue;  // done in the first segment
    }
    fit_pair<KMAX>(a, p, n);
  }
}

// Device-side fork / join of the fit's streams (PAS_GAS_SPIN_SYNC): a one-thread kernel
// sets a flag to the fit's epoch after the work before it on its stream; another waits on
// flags before the work after it on its stream.  Host order is the deadlock guard: every
// wait is enqueued after the signal it waits for (so is every event wait), so streams that
// share a hardware queue still reach the signal first.  A wait gives up rather than hang: a
// fork wait first waits for the fit's prep to start on the caller's stream (start; up to
// limit_start, the caller's earlier work on that stream), then for the prep's signal (up to
// limit); the join wait for the side streams' signals (limit).  A wait that gives up aborts
// the fit (its fit kernels return at entry, fit_aborted) and sets the context's fault word,
// which the call's synchronization reports as PAS_EDEVICE (gas_fault_check).  force: a
// debug-forced timeout (PAS_GAS_FORCE_TIMEOUT).
__global__ __launch_bounds__(64) void gas_signal_kernel(uint32_t* flag, uint32_t epoch) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
struct WaitArgs {
  const uint32_t* flags;  // [n]
  int32_t n;
  const uint32_t* start;  // fork waits: the prep-started flag, else null
  uint32_t epoch;
  uint64_t limit, limit_start;  // 100 MHz ticks
  uint32_t* abort;
  uint32_t* fault;  // host-pinned
  int32_t force;
};
__global__ __launch_bounds__(64) void gas_wait_kernel(WaitArgs a) {
  if (threadIdx.x != 0) return;
  auto give_up = [&]() {
    __hip_atomic_store(a.abort, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.fault, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  if (a.force) {
    give_up();
    return;
  }
  auto reached = [&](const uint32_t* f) {
    return (int32_t)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - a.epoch) >=
           0;
  };
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (a.start)
    while (!reached(a.start)) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.limit_start) {
        give_up();
        return;
      }
      __builtin_amdgcn_s_sleep(8);
    }
  t0 = __builtin_amdgcn_s_memrealtime();
  for (int32_t i = 0; i < a.n; ++i)
    while (!reached(a.flags + i)) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.limit) {
        give_up();
        return;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// The fork / join mode of a context: PAS_GAS_SYNC=events|flags, else flags unless a tool that
// runs kernels one at a time is attached (rocprofv3 counter collection or thread trace,
// AMD_SERIALIZE_KERNEL): such a tool may start a wait kernel before the signal it waits for
// and hold every other kernel back until the wait gives up, so events are used there.
int gas_sync_mode() {
  auto on = [](const char* v) { return v && *v && std::strcmp(v, "0") != 0; };
  if (const char* m = std::getenv("PAS_GAS_SYNC")) {
    if (!std::strcmp(m, "events")) return 0;
    if (!std::strcmp(m, "flags")) return 1;
  }
  if (on(std::getenv("ROCPROF_COUNTER_COLLECTION")) ||
      on(std::getenv("ROCPROF_ADVANCED_THREAD_TRACE")) || on(std::getenv("AMD_SERIALIZE_KERNEL")))
    return 0;
  return PAS_GAS_SPIN_SYNC ? 1 : 0;
}

}  // namespace

int gas_fault_check(pas_ctx* ctx) {
  if (!ctx->gas_sync_fault || !__atomic_load_n(ctx->gas_sync_fault, __ATOMIC_ACQUIRE))
    return PAS_OK;
  // the fit kernels of a fit whose join gave up may still be running on its side streams
  for (AuxSlot& a : ctx->aux_slot) {
    if (a.side) (void)hipStreamSynchronize(a.side);
    if (a.side2) (void)hipStreamSynchronize(a.side2);
  }
  __atomic_store_n(ctx->gas_sync_fault, 0u, __ATOMIC_RELEASE);
  return set_error(ctx, PAS_EDEVICE,
                   "pas_gas_fit: a side-stream wait of a fit timed out, so that fit's results "
                   "are incomplete (set PAS_GAS_SYNC=events under kernel-serializing tools)");
}

int gas_fit_launch(pas_ctx* ctx, int32_t n_pods, int32_t max_containers, int32_t i915_index,
                   const int64_t* d_req, const uint32_t* d_req_mask,
                   const int32_t* d_n_containers, uint32_t* d_res, int64_t ld_res, uint64_t* d_fit,
                   pas_gas_selection* d_side, int64_t side_cap, int64_t* d_side_count,
                   hipStream_t s) {
  const GasSnapshot& g = ctx->gas;
  const int32_t N = g.n_nodes, Q = g.n_res, K = g.max_cards;
  constexpr int32_t kCounts = (1 + kClasses) * (PAS_GAS_MAX_RES + 1) + 1;  // lists + generic pods
  if (Q < 1 || Q > PAS_GAS_MAX_RES) return set_error(ctx, PAS_EINVAL, "pas_gas_fit: n_res out of range");
  if (n_pods > (1 << 24)) return set_error(ctx, PAS_ECAPACITY, "pas_gas_fit: > 2^24 pods");
  // the fit kernels' 32-bit byte offsets into the card-major free table (free_at)
  if ((int64_t)N * PAS_GAS_MAX_RES * 8 > INT32_MAX)
    return set_error(ctx, PAS_ECAPACITY, "pas_gas_fit: more than 2^26 nodes");
  // scratch: single-selection records [Q+1][P] | multi-selection pod words [Q+1][3][P] |
  // their selection rows [Q+1][3][P][8] | the generic path's pods [P] and per-pod selection
  // counts [P] | list counts [Q+1] + [(Q+1)3] and the generic pod count (zeroed together).  The flipped
  // kind minima and the generic path's nodes depend on the snapshot alone: they sit in
  // g.derived and are recomputed only after the snapshot changed.
  const int32_t NL = Q + 1;
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t b_single = al(sizeof(GasSingle) * (size_t)NL * n_pods);
  const size_t b_multi = al(sizeof(int32_t) * (size_t)NL * kClasses * n_pods);
  const size_t b_sels = al(sizeof(GasSel) * kPacked * (size_t)NL * kClasses * n_pods);
  const size_t b_pods = al(sizeof(int32_t) * (size_t)n_pods);
  // ranked paths: pod records and sorted rows (items: <= P one-selection, <= 7P closed-form)
  const size_t b_rs = al(sizeof(GasRSingle) * (size_t)NL * n_pods);
  const size_t b_rm = al(sizeof(GasRMulti) * (size_t)NL * 2 * n_pods);
  const size_t b_rw = al(sizeof(int32_t) * (size_t)NL * 2 * n_pods);
  const size_t b_srs = al(sizeof(int64_t) * PAS_GAS_MAX_RES * (size_t)n_pods);
  const size_t b_srm = al(sizeof(int64_t) * PAS_GAS_MAX_RES * kPacked * (size_t)n_pods);
  const size_t b_rq = al(sizeof(GasRSeq) * (size_t)NL * n_pods);
  const size_t b_rf = al(sizeof(GasRFour) * (size_t)NL * n_pods);
  const bool empty = N == 0 || n_pods == 0;
  const size_t need = empty ? 0
                            : b_single + b_multi + b_sels + 2 * b_pods + b_rs + b_rm + b_rw +
                                  b_srs + b_srm + b_rq + b_rf;
  // the stream's scratch slot (ordered after its previous user on another stream)
  int rc = PAS_OK;
  AuxSlot* slot = aux_acquire(ctx, s, need, &rc);
  if (!slot) return rc;
  if (!slot->gas_limit) PAS_HIP(ctx, hipMalloc(&slot->gas_limit, sizeof(int64_t)));
  if (!slot->gas_counts) {  // both sets zero before their first use
    int32_t* c = nullptr;
    PAS_HIP(ctx, hipMalloc(&c, 2 * kCounts * sizeof(int32_t)));
    if (hipMemsetAsync(c, 0, 2 * kCounts * sizeof(int32_t), s) != hipSuccess) {
      (void)hipFree(c);
      return set_error(ctx, PAS_EDEVICE, "pas_gas_fit: counts init failed");
    }
    slot->gas_counts = c;
    slot->gas_counts_set = 0;
  }
  ctx->gas_last_slot = (int)(slot - ctx->aux_slot);
  // every exit from here records the slot's event on s (a later call on another stream
  // waits for it before it reuses the slot)
  struct ReleaseOnExit {
    pas_ctx* c;
    AuxSlot* a;
    hipStream_t s;
    ~ReleaseOnExit() { aux_release(c, a, s); }
  } done{ctx, slot, s};
  if (empty) {
    PAS_HIP(ctx, hipMemsetAsync(slot->gas_limit, 0, sizeof(int64_t), s));
    if (d_side_count) PAS_HIP(ctx, hipMemsetAsync(d_side_count, 0, sizeof(int64_t), s));
    return PAS_OK;
  }
  char* base = static_cast<char*>(slot->p);
  GasSingle* single = reinterpret_cast<GasSingle*>(base);
  base += b_single;
  int32_t* multi = reinterpret_cast<int32_t*>(base);
  base += b_multi;
  GasSel* sels = reinterpret_cast<GasSel*>(base);
  base += b_sels;
  int32_t* big_pods = reinterpret_cast<int32_t*>(base);
  base += b_pods;
  int32_t* pod_steps = reinterpret_cast<int32_t*>(base);
  base += b_pods;
  GasRSingle* rsingle = reinterpret_cast<GasRSingle*>(base);
  base += b_rs;
  GasRMulti* rmulti = reinterpret_cast<GasRMulti*>(base);
  base += b_rm;
  int32_t* rword = reinterpret_cast<int32_t*>(base);
  base += b_rw;
  int64_t* srt_s = reinterpret_cast<int64_t*>(base);
  base += b_srs;
  int64_t* srt_m = reinterpret_cast<int64_t*>(base);
  base += b_srm;
  GasRSeq* rseq = reinterpret_cast<GasRSeq*>(base);
  base += b_rq;
  GasRFour* rfour = reinterpret_cast<GasRFour*>(base);
  base += b_rf;
  // this fit's list counts (zeroed by the previous fit's prep kernel, or at allocation) and
  // the other set, which this fit's prep kernel zeroes for the next one
  int32_t* counts = slot->gas_counts + kCounts * slot->gas_counts_set;
  int32_t* counts_next = slot->gas_counts + kCounts * (1 - slot->gas_counts_set);
  int32_t* n_big_pods = counts + (1 + kClasses) * (PAS_GAS_MAX_RES + 1);
  unsigned long long* gflip = static_cast<unsigned long long*>(g.derived);
  int32_t* n_big_nodes = reinterpret_cast<int32_t*>(gflip + PAS_GAS_MAX_RES);
  int32_t* big_nodes = reinterpret_cast<int32_t*>(static_cast<char*>(g.derived) + 64);
  // The fit forks two side streams of its slot after its prep launches (the one-selection
  // and generic kernels on one, the sequential kernel on the other; the closed-form kernel
  // stays on s) and joins them at the end.  Fork / join: device flags (per slot, set to the
  // slot's fit epoch), else events (gas_sync_mode).
  if (ctx->gas_sync_mode < 0) {
    ctx->gas_sync_mode = gas_sync_mode();
    if (ctx->gas_sync_mode) {
      PAS_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->gas_sync_fault), sizeof(uint32_t),
                                 hipHostMallocCoherent));
      *ctx->gas_sync_fault = 0;
#if PAS_GAS_FAULT_INJECTION  // lib/libpas_fault.so only (tests/test_gas_sync.py)
      if (const char* f = std::getenv("PAS_GAS_FORCE_TIMEOUT"))
        ctx->gas_force_timeouts = std::atoi(f);
#endif
    }
  }
  // a wait of an earlier fit that gave up and was not reported by a synchronization yet
  if (int e = gas_fault_check(ctx)) return e;
  // side streams and events exist before the fork, and every exit after the fork joins them
  // (Joins), so a later user of the slot never waits on an event that does not cover
  // side-stream work
  if (!slot->side) {
    PAS_HIP(ctx, hipStreamCreateWithFlags(&slot->side, hipStreamNonBlocking));
    PAS_HIP(ctx, hipStreamCreateWithFlags(&slot->side2, hipStreamNonBlocking));
    PAS_HIP(ctx, hipEventCreateWithFlags(&slot->fork, hipEventDisableTiming));
    PAS_HIP(ctx, hipEventCreateWithFlags(&slot->join, hipEventDisableTiming));
    PAS_HIP(ctx, hipEventCreateWithFlags(&slot->join2, hipEventDisableTiming));
  }
  hipStream_t const ss = slot->side, qs = slot->side2;
  const bool kFlags = ctx->gas_sync_mode == 1;
  // limits (100 MHz ticks): a side-stream wait for the prep to START, up to 30 s (it may sit
  // behind the caller's earlier work on s); then for the prep's signal, and the join's wait
  // for the side streams, 1 s plus 1 ns per (pod, node) pair, far past any fit
  const uint64_t limit = 100000000ull + (uint64_t)n_pods * (uint64_t)N / 10u;
  const uint64_t limit_start = 3000000000ull;
  uint32_t* sync = nullptr;  // [prep done, side done, side2 done, abort, prep started]
  uint32_t epoch = 0;
  if (kFlags) {
    if (!slot->gas_sync) {
      uint32_t* f = nullptr;
      PAS_HIP(ctx, hipMalloc(&f, 8 * sizeof(uint32_t)));
      // zero before any side stream can read them (once per slot)
      if (hipMemsetAsync(f, 0, 8 * sizeof(uint32_t), s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess) {
        (void)hipFree(f);
        return set_error(ctx, PAS_EDEVICE, "pas_gas_fit: sync flags init failed");
      }
      slot->gas_sync = f;
      slot->gas_epoch = 0;
    }
    sync = slot->gas_sync;
    epoch = ++slot->gas_epoch;
    if (epoch == 0) epoch = ++slot->gas_epoch;  // flags start at 0: never wait for epoch 0
  }
  uint32_t* const abort_flag = kFlags ? sync + 3 : nullptr;
  TimedLaunch tl;
  timing_begin(ctx, s, PAS_K_GAS_PREP, &tl);
  if (ctx->gas.derived_epoch != ctx->gas.epoch) {
    PAS_HIP(ctx, hipMemsetAsync(gflip, 0, 64, s));
    gas_minfree_kernel<<<(N + kTpb - 1) / kTpb, kTpb, 0, s>>>(N, K, Q, g.n_cards, g.cap, g.used,
                                                             gflip, big_nodes, n_big_nodes,
                                                             static_cast<int64_t*>(g.free_t));
    PAS_HIP(ctx, hipGetLastError());
    ctx->gas.derived_epoch = ctx->gas.epoch;
    if (int e = derived_built(ctx, ctx->gas.derived_sync, s)) return e;
  } else if (int e = derived_wait(ctx, ctx->gas.derived_sync, s)) {
    return e;  // built by a fit on another stream, maybe still running
  }
  const PrepArgs pa{n_pods, max_containers, Q, i915_index, d_req, d_req_mask, d_n_containers,
                    gflip, single, multi, sels, counts, big_pods, n_big_pods, pod_steps,
                    counts_next, kCounts, slot->gas_limit, d_side_count,
                    kFlags ? sync + 4 : nullptr, epoch};
  const RankArgs ra{n_pods, Q, counts, single, multi, sels, srt_s, srt_m, rsingle, rmulti, rword,
                    rseq, rfour};
  gas_prep_kernel<<<(n_pods + kPrepTpb - 1) / kPrepTpb, kPrepTpb, 0, s>>>(pa);
  PAS_HIP(ctx, hipGetLastError());
  // the prep kernel ran: the other set is zeroed (on s) for the slot's next fit
  slot->gas_counts_set = 1 - slot->gas_counts_set;
  // grids: (node block, pod chunk) pairs, ~8192 blocks; each kernel splits each of its
  // device-counted lists evenly over the chunks
  const int32_t nb_s = (N + kSingleTpb - 1) / kSingleTpb;  // the single-selection kernel's
  const int32_t ch_s = (n_pods + kRankMax - 1) / kRankMax;  // fixed one-group chunks
  const int32_t nb_c = (N + kClosedTpb - 1) / kClosedTpb;  // the closed-form kernel's
  const int32_t ch_c = std::max(1, std::min(n_pods, (PAS_GAS_BLOCKS_MULTI + nb_c - 1) / nb_c));
  const int32_t nb_q = (N + kSeqTpb - 1) / kSeqTpb;  // the sequential kernel's node blocks
  const int32_t ch_q = std::max(1, std::min(n_pods, (PAS_GAS_BLOCKS_SEQ + nb_q - 1) / nb_q));
  gas_rank_prep_kernel<<<kRankPrepBlocks, kRankPrepTpb, 0, s>>>(ra);
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  timing_begin(ctx, s, PAS_K_GAS_FIT, &tl);
  const bool bits = d_fit != nullptr;
  // the wide shapes: the lists' lengths are on the device, so the grid is fixed and threads
  // past the work return at once
  GenericArgs ga;
  ga.N = N;
  ga.K = K;
  ga.Q = Q;
  ga.C = max_containers;
  ga.i915 = i915_index;
  ga.n_cards = g.n_cards;
  ga.cap = g.cap;
  ga.used = g.used;
  ga.req = d_req;
  ga.mask = d_req_mask;
  ga.ncont = d_n_containers;
  ga.big_pods = big_pods;
  ga.n_big_pods = n_big_pods;
  ga.big_nodes = big_nodes;
  ga.n_big_nodes = n_big_nodes;
  ga.pod_steps = pod_steps;
  ga.n_pods = n_pods;
  ga.res = d_res;
  ga.ld = ld_res;
  ga.fit = d_fit;
  ga.side = d_side;
  ga.side_cap = d_side ? side_cap : 0;
  ga.side_count = reinterpret_cast<unsigned long long*>(d_side_count);
  ga.limit_count = reinterpret_cast<unsigned long long*>(slot->gas_limit);
  ga.abort = abort_flag;
  ga.epoch = epoch;
  const ResOut ro{d_res, ld_res, abort_flag, epoch};
  auto generic = [&](hipStream_t st) {
    constexpr int kGenericBlocks = 512;
    if (K <= 8)
      gas_fit_generic_kernel<8><<<kGenericBlocks, 64, 0, st>>>(ga);
    else if (K <= 16)
      gas_fit_generic_kernel<16><<<kGenericBlocks, 64, 0, st>>>(ga);
    else
      gas_fit_generic_kernel<PAS_GAS_MAX_CARDS><<<kGenericBlocks, 64, 0, st>>>(ga);
  };
  struct Joins {
    AuxSlot* a;
    hipStream_t s;
    bool forked = false;  // side streams forked and not yet joined
    hipError_t join() {
      hipError_t e = hipEventRecord(a->join, a->side);
      if (e == hipSuccess) e = hipStreamWaitEvent(s, a->join, 0);
      if (e == hipSuccess) e = hipEventRecord(a->join2, a->side2);
      if (e == hipSuccess) e = hipStreamWaitEvent(s, a->join2, 0);
      forked = false;
      return e;
    }
    ~Joins() {
      if (forked) (void)join();  // an error exit: runs before ReleaseOnExit records the slot
    }
  } joins{slot, s};
  // the fork, after the rank prep: flags — a signal kernel on s, a wait kernel at the head of
  // each side stream (enqueued after the signal); else events
  if (kFlags) {
    int32_t force = 0;  // PAS_GAS_FORCE_TIMEOUT: the side streams' waits give up at once
    if (ctx->gas_force_timeouts > 0) {
      force = 1;
      --ctx->gas_force_timeouts;
    }
    gas_signal_kernel<<<1, 64, 0, s>>>(sync, epoch);
    const WaitArgs fw{sync, 1, sync + 4, epoch, limit, limit_start, abort_flag,
                      ctx->gas_sync_fault, force};
    gas_wait_kernel<<<1, 64, 0, ss>>>(fw);
    gas_wait_kernel<<<1, 64, 0, qs>>>(fw);
  } else {
    PAS_HIP(ctx, hipEventRecord(slot->fork, s));
    PAS_HIP(ctx, hipStreamWaitEvent(ss, slot->fork, 0));
    PAS_HIP(ctx, hipStreamWaitEvent(qs, slot->fork, 0));
  }
  joins.forked = true;
  PAS_HIP(ctx, hipGetLastError());
  // streams of the single-selection (ss), closed-form (s) and sequential (qs) kernels:
  // disjoint pods, disjoint result rows.  Word results: the generic kernel writes its (pod,
  // node) words alone (the fast kernels skip pods past 8 selections and nodes past 8 cards),
  // so it runs beside them, after the single-selection kernel on ss; bitmap rows are or-ed
  // into the fast kernels' words, so it runs after the join
  // word results of < 2^31 bytes: row offsets as the stores' 32-bit scalar offsets (ResSoff)
  const bool soff = !bits && (int64_t)n_pods * ld_res * 4 < ((int64_t)1 << 31);
  switch (Q * 4 + (bits ? 1 : 0) * 2 + (soff ? 1 : 0)) {
#define PAS_GAS_CASE(QQ, B, SO)                                                                \
  case QQ * 4 + B * 2 + SO:                                                                    \
    if (PAS_GAS_SEQ_FIRST)                                                                     \
      gas_rfit_seq_kernel<QQ, B, SO><<<nb_q * ch_q, kSeqTpb, 0, qs>>>(                         \
          N, K, n_pods, g.n_cards, static_cast<int64_t*>(g.free_t), rseq, rfour, srt_m, multi, \
          sels, counts + NL, ch_q, ro, d_fit);                                                  \
    gas_rfit_closed_kernel<QQ, B, SO><<<nb_c * ch_c, kClosedTpb, 0, s>>>(                      \
        N, K, n_pods, g.n_cards, static_cast<int64_t*>(g.free_t), rmulti, rword, srt_m,         \
        counts + NL, ch_c, ro, d_fit);                                                          \
    if (!PAS_GAS_SEQ_FIRST)                                                                    \
      gas_rfit_seq_kernel<QQ, B, SO><<<nb_q * ch_q, kSeqTpb, 0, qs>>>(                         \
          N, K, n_pods, g.n_cards, static_cast<int64_t*>(g.free_t), rseq, rfour, srt_m, multi, \
          sels, counts + NL, ch_q, ro, d_fit);                                                  \
    gas_rfit_single_kernel<QQ, B, SO><<<nb_s * ch_s, kSingleTpb, 0, ss>>>(                     \
        N, K, n_pods, g.n_cards, static_cast<int64_t*>(g.free_t), rsingle, srt_s, counts,       \
        ch_s, ro, d_fit);                                                                       \
    break;
    PAS_GAS_CASE(1, 0, 0) PAS_GAS_CASE(2, 0, 0) PAS_GAS_CASE(3, 0, 0) PAS_GAS_CASE(4, 0, 0)
    PAS_GAS_CASE(1, 0, 1) PAS_GAS_CASE(2, 0, 1) PAS_GAS_CASE(3, 0, 1) PAS_GAS_CASE(4, 0, 1)
    PAS_GAS_CASE(1, 1, 0) PAS_GAS_CASE(2, 1, 0) PAS_GAS_CASE(3, 1, 0) PAS_GAS_CASE(4, 1, 0)
#undef PAS_GAS_CASE
    default: return set_error(ctx, PAS_EINVAL, "pas_gas_fit: n_res out of range");
  }
  if (!bits) generic(ss);
  if (kFlags) {
    // the join: each side stream sets its flag after its work; s waits for both (enqueued
    // after the signals)
    gas_signal_kernel<<<1, 64, 0, ss>>>(sync + 1, epoch);
    gas_signal_kernel<<<1, 64, 0, qs>>>(sync + 2, epoch);
    gas_wait_kernel<<<1, 64, 0, s>>>(
        WaitArgs{sync + 1, 2, nullptr, epoch, limit, 0, abort_flag, ctx->gas_sync_fault, 0});
    PAS_HIP(ctx, hipGetLastError());
    joins.forked = false;
  } else {
    PAS_HIP(ctx, joins.join());
  }
  if (bits) generic(s);
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

}  // namespace pas
