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
// The pod loop is wave-uniform: pod records sit in SGPRs, so each card check is one 64-bit
// compare against an SGPR.  The prep kernel splits the batch: pods with at most one card
// selection (the common case: one container, one i915) go to a kernel that only reads free;
// pods with several selections go to a kernel that takes cards in a working copy
// (per-card lane-masked updates), so the first kernel keeps a small register footprint.
//
// Kind skipping (exact, decided per pod before the fit kernels): gmin[q] = the minimum of
// free[k][q] over every card of every labelled node of the snapshot (gas_minfree_kernel).
// When a single-selection pod's need of kind q is <= gmin[q], no check of kind q can fail
// anywhere, so its compares are dropped: the prep kernel files the pod under list 1 + q (the
// lowest such kind) or list 0, and the single kernel instantiates one body per list, so the
// skip costs nothing per (pod, node).  The last kind the selection requests stays compared,
// so cards a node does not have (free -1 everywhere) still fail.  In the C3 mix the i915
// kind (1 per selection against >= 30 free) goes: single kernel 502 -> 381 us.  The same
// for multi-selection pods (bound = need plus the takes before it) measured 1587 -> 1609 us,
// so that kernel keeps every kind: it is not bound by its compares.
#include <hip/hip_runtime.h>

#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;
constexpr int kMaxCards = PAS_GAS_MAX_CARDS;
constexpr int kPodBatch = 64;  // pod records staged in LDS per round

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

// One card selection of a pod with several: compare and take vectors (kinds as GasStep).
struct alignas(16) GasSel {
  int64_t cmp[PAS_GAS_MAX_RES];
  int64_t take[PAS_GAS_MAX_RES];
  int32_t bad;
  int32_t pad[3];
};

// Pod with at most one card selection: its selecting step, or steps == 0.
struct alignas(16) GasSingle {
  int64_t cmp[PAS_GAS_MAX_RES];
  int32_t pod;
  int32_t steps;
  int32_t bad;
  int32_t pad;
};

// getPerGPUResourceRequest: copy the container's map and, when numI915 > 1, divide
// every entry (the i915 entry included) by numI915, truncating (resource_map.go:129-145).
__device__ GasStep container_step(int64_t i, int32_t n_res, int32_t i915,
                                  const int64_t* __restrict__ req,
                                  const uint32_t* __restrict__ mask) {
  const uint32_t m = mask[i];
  int64_t ni = 0;
  if (i915 >= 0 && ((m >> i915) & 1u)) {
    const int64_t v = req[i * n_res + i915];
    if (v > 0) ni = v;
  }
  GasStep g = {};
  g.num_i915 = m != 0u ? (int32_t)min(ni, (int64_t)PAS_GAS_MAX_SELECTIONS + 1) : 0;
  g.kinds = (int32_t)(m & ((1u << n_res) - 1u));
#pragma unroll
  for (int q = 0; q < PAS_GAS_MAX_RES; ++q) {
    const bool has = q < n_res && ((m >> q) & 1u);
    int64_t v = has ? req[i * n_res + q] : 0;
    if (ni > 1) v /= ni;
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
                                             uint32_t kinds,
                                             const unsigned long long* __restrict__ gflip) {
  for (int q = 0; q < n_res; ++q) {
    if (!((kinds >> q) & 1u) || kinds == (1u << q)) continue;
    const int64_t gmin = (int64_t)((unsigned long long)INT64_MAX - gflip[q]);
    if (cmp[q] <= gmin) return 1 + q;
  }
  return 0;
}

// A slot in list `list` for each active lane: one atomic per distinct list in the wave (lanes
// of different lists hit different counters, which the compiler would leave one per lane).
__device__ __forceinline__ int32_t wave_slot(int32_t* __restrict__ counts, int32_t list) {
  unsigned long long todo = __ballot(1);
  int32_t slot = 0;
  while (todo) {
    const int leader = __builtin_ctzll(todo);
    const int32_t l = __shfl(list, leader, 64);
    const unsigned long long m = __ballot(list == l);
    int32_t base = 0;
    if ((int)__lane_id() == leader) base = atomicAdd(&counts[l], __popcll(m));
    base = __shfl(base, leader, 64);
    if (list == l)
      slot = base + (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
    todo &= ~m;
  }
  return slot;
}

// One thread per pod files it under `single` (<= 1 selection: its selecting step, in the
// list of its skippable kind; lists [n_res + 1][n_pods]) or `multi` (several: its steps,
// containers in order then gpuNum, into its row of `sels`; more than PAS_GAS_MAX_SELECTIONS
// are beyond the packed result and keep only the count).  counts: [n_res + 1] single lists,
// then the multi list.
__global__ void gas_prep_kernel(int32_t n_pods, int32_t max_containers, int32_t n_res,
                                int32_t i915, const int64_t* __restrict__ req,
                                const uint32_t* __restrict__ mask,
                                const int32_t* __restrict__ n_containers,
                                const unsigned long long* __restrict__ gflip,
                                GasSingle* __restrict__ single, int32_t* __restrict__ multi,
                                GasSel* __restrict__ sels, int32_t* __restrict__ counts) {
  const int32_t p = blockIdx.x * kTpb + threadIdx.x;
  if (p >= n_pods) return;
  const int32_t nc = min(max(n_containers[p], 0), max_containers);
  const int64_t row = (int64_t)p * max_containers;
  int32_t steps = 0;
  uint32_t kinds = 0;
  GasSingle one = {};
  one.pod = p;
  for (int32_t c = 0; c < nc; ++c) {
    const GasStep g = container_step(row + c, n_res, i915, req, mask);
    if (g.num_i915 > 0) {
      if (steps == 0) {
#pragma unroll
        for (int q = 0; q < PAS_GAS_MAX_RES; ++q) one.cmp[q] = g.cmp[q];
        one.bad = g.bad;
        kinds = g.kinds;
      }
      steps = min(steps + g.num_i915, PAS_GAS_MAX_SELECTIONS + 1);
    }
  }
  const bool one_sel = steps <= 1;
  const int32_t l = steps == 1 ? skip_list(n_res, one.cmp, kinds, gflip) : 0;
  const int32_t slot = wave_slot(counts, one_sel ? l : n_res + 1);
  if (one_sel) {
    one.steps = steps;
    single[(int64_t)l * n_pods + slot] = one;
    return;
  }
  multi[slot] = p | (steps << 24);
  if (steps > PAS_GAS_MAX_SELECTIONS) return;
  GasSel* out = sels + (int64_t)slot * PAS_GAS_MAX_SELECTIONS;
  int32_t k = 0;
  for (int32_t c = 0; c < nc; ++c) {
    const GasStep g = container_step(row + c, n_res, i915, req, mask);
    for (int32_t r = 0; r < g.num_i915; ++r, ++k) {
      GasSel e = {};
#pragma unroll
      for (int q = 0; q < PAS_GAS_MAX_RES; ++q) {
        e.cmp[q] = g.cmp[q];
        e.take[q] = g.take[q];
      }
      e.bad = g.bad;
      out[k] = e;
    }
  }
}

// gflip[q] = INT64_MAX - gmin[q] (kept flipped so that a zeroed buffer is the identity of the
// unsigned atomicMax): per node the minimum free over its cards, per workgroup the minimum
// over its nodes, one atomic per workgroup and kind.  Nodes without the cards label or not in
// the lister never fit, so they do not count.
__global__ __launch_bounds__(kTpb) void gas_minfree_kernel(int32_t N, int32_t K, int32_t n_res,
                                                           const int32_t* __restrict__ n_cards,
                                                           const int64_t* __restrict__ cap,
                                                           const int64_t* __restrict__ used,
                                                           unsigned long long* __restrict__ gflip) {
  __shared__ int64_t red[kTpb / 64][PAS_GAS_MAX_RES];
  const int32_t n = blockIdx.x * kTpb + threadIdx.x;
  const int32_t nc = n < N ? min(n_cards[n], K) : 0;
  for (int q = 0; q < n_res; ++q) {
    int64_t m = INT64_MAX;
    const int64_t c = nc > 0 ? cap[(int64_t)n * n_res + q] : 0;
    for (int k = 0; k < nc; ++k) {
      const int64_t u = used[((int64_t)n * K + k) * n_res + q];
      const int64_t f = (c > 0 && u >= 0) ? c - u : -1;
      m = f < m ? f : m;
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
// cards the node does not have).
template <int Q>
__device__ __forceinline__ void load_free(int32_t n, bool valid, int32_t ncard, int32_t K,
                                          const int64_t* __restrict__ cap,
                                          const int64_t* __restrict__ used,
                                          int64_t (&free)[kMaxCards][Q]) {
  int64_t cap_r[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) cap_r[q] = valid ? cap[(int64_t)n * Q + q] : 0;
#pragma unroll
  for (int k = 0; k < kMaxCards; ++k)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int64_t u = k < ncard ? used[((int64_t)n * K + k) * Q + q] : -1;
      free[k][q] = (cap_r[q] > 0 && u >= 0) ? cap_r[q] - u : -1;
    }
}

typedef unsigned long long lane_mask;  // one bit per lane of the wave (ballot)

// First card (lexicographic rank) passing checkResourceCapacity, or -1: cmp[q] <= free[k][q]
// for every kind (cmp is INT64_MIN for kinds the container does not request).
template <int Q, int SKIP>
__device__ __forceinline__ int first_fit(const int64_t (&free)[kMaxCards][Q],
                                         const int64_t (&cmp)[Q]) {
  int chosen = -1;
#pragma unroll
  for (int k = kMaxCards - 1; k >= 0; --k) {  // first fit = lowest k
    bool ok = true;
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (q != SKIP) ok &= cmp[q] <= free[k][q];  // lane masks and-ed in SALU
    chosen = ok ? k : chosen;                    // one select per card
  }
  return chosen;
}

// A wave-uniform value copied into a VGPR pair, so that selects against the condition mask
// (VCC, one scalar operand) do not re-materialise it per use.
__device__ __forceinline__ int64_t to_vgpr64(int64_t x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)((uint64_t)x >> 32);
  asm volatile("v_mov_b32 %0, %0" : "+v"(lo));
  asm volatile("v_mov_b32 %0, %0" : "+v"(hi));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int64_t uniform64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// One (pod, node) result: the packed word, or (kBits) the fit bit in the pod's row of a
// node bitmap, written per 64-node word by lane 0 of the wave (waves cover aligned
// 64-node ranges).
template <bool kBits>
__device__ __forceinline__ void put_result(uint32_t* __restrict__ res, uint64_t* __restrict__ fit,
                                           int64_t p, int32_t N, int32_t n, bool valid,
                                           uint32_t out) {
  if (kBits) {
    const uint64_t b = __ballot(valid && (out >> 31));
    if ((threadIdx.x & 63) == 0 && n < N) fit[p * ((N + 63) / 64) + (n >> 6)] = b;
  } else if (valid) {
    res[p * N + n] = out;
  }
}

// This block's share [*b, *e) of a device-counted list, split evenly over gridDim.y.
__device__ __forceinline__ void list_share(const int32_t* count, int32_t* b, int32_t* e) {
  const int32_t cnt = __builtin_amdgcn_readfirstlane(*count);
  const int32_t per = (cnt + (int32_t)gridDim.y - 1) / (int32_t)gridDim.y;
  *b = min(cnt, (int32_t)blockIdx.y * per);
  *e = min(cnt, *b + per);
}

// Pods with at most one selection, list `l` (kind SKIP = l - 1 dropped): a read-only first
// fit per (pod, node lane), pod records staged in LDS per batch and read into SGPRs.
template <int Q, int SKIP, bool kBits>
__device__ __forceinline__ void single_list(const int64_t (&free)[kMaxCards][Q],
                                            uint32_t node_ok, int32_t N, int32_t n, bool valid,
                                            const GasSingle* __restrict__ single,
                                            const int32_t* __restrict__ count, GasSingle* stage,
                                            uint32_t* __restrict__ res,
                                            uint64_t* __restrict__ fit) {
  int32_t i0, i1;
  list_share(count, &i0, &i1);
  for (int32_t b0 = i0; b0 < i1; b0 += kPodBatch) {
    const int32_t nb = min(kPodBatch, i1 - b0);
    constexpr int kWords = (int)(sizeof(GasSingle) / 16);
    const int4* src = reinterpret_cast<const int4*>(single + b0);
    int4* dst = reinterpret_cast<int4*>(stage);
    for (int32_t i = threadIdx.x; i < nb * kWords; i += kTpb) dst[i] = src[i];
    __syncthreads();
    for (int32_t j = 0; j < nb; ++j) {
      const GasSingle& r = stage[j];  // broadcast LDS reads, then SGPRs
      const int64_t pod = __builtin_amdgcn_readfirstlane(r.pod);
      uint32_t out = node_ok;
      if (__builtin_amdgcn_readfirstlane(r.steps) == 1) {
        int64_t cmp[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) cmp[q] = q == SKIP ? 0 : uniform64(r.cmp[q]);
        const int k =
            __builtin_amdgcn_readfirstlane(r.bad) ? -1 : first_fit<Q, SKIP>(free, cmp);
        out = k >= 0 ? (node_ok | (1u << 24) | (uint32_t)k) : 0u;
      }
      put_result<kBits>(res, fit, pod, N, n, valid, out);
    }
    __syncthreads();  // the next batch rewrites the stage
  }
}

template <int Q, bool kBits, int L = 0>
__device__ __forceinline__ void single_lists(const int64_t (&free)[kMaxCards][Q],
                                             uint32_t node_ok, int32_t N, int32_t n, bool valid,
                                             int32_t P, const GasSingle* __restrict__ single,
                                             const int32_t* __restrict__ counts,
                                             GasSingle* stage, uint32_t* __restrict__ res,
                                             uint64_t* __restrict__ fit) {
  single_list<Q, L - 1, kBits>(free, node_ok, N, n, valid, single + (int64_t)L * P, counts + L,
                               stage, res, fit);
  if constexpr (L < Q)
    single_lists<Q, kBits, L + 1>(free, node_ok, N, n, valid, P, single, counts, stage, res,
                                  fit);
}

template <int Q, bool kBits>
__global__ __launch_bounds__(kTpb) void gas_fit_single_kernel(
    int32_t N, int32_t K, int32_t P, const int32_t* __restrict__ n_cards,
    const int64_t* __restrict__ cap, const int64_t* __restrict__ used,
    const GasSingle* __restrict__ single, const int32_t* __restrict__ counts,
    uint32_t* __restrict__ res, uint64_t* __restrict__ fit) {
  __shared__ GasSingle stage[kPodBatch];
  const int32_t n = blockIdx.x * kTpb + threadIdx.x;
  const bool valid = n < N;
  const int32_t nc = valid ? n_cards[n] : 0;
  int64_t free[kMaxCards][Q];
  load_free<Q>(n, valid, min(nc, K), K, cap, used, free);
  // FetchNode error / missing cards label -> errWontFit before any container (:282-298)
  const uint32_t node_ok = nc > 0 ? 0x80000000u : 0u;
  single_lists<Q, kBits>(free, node_ok, N, n, valid, P, single, counts, stage, res, fit);
}

// The compare / take fields of one selection record, kinds [0, Q) (scalar loads).
struct SelHead {
  int64_t cmp[PAS_GAS_MAX_RES];
  int64_t take[PAS_GAS_MAX_RES];
  int32_t bad;
};
template <int Q>
__device__ __forceinline__ SelHead sel_head(const GasSel* e) {
  SelHead h = {};
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    h.cmp[q] = e->cmp[q];
    h.take[q] = e->take[q];
  }
  h.bad = e->bad;
  return h;
}

// Pods with several selections: the steps in order (containers, then gpuNum), each taking
// the first fitting card (free drops by the need for the following steps).  Two
// selections need no state (the second sees the first take added to card c0's need);
// more work on a copy of free.  One list: dropping a kind from the compares does not pay
// here (measured: 1711 us with or without it for C3; the multi-selection pods are not bound
// by their compares).
template <int Q, bool kBits>
__global__ __launch_bounds__(kTpb) void gas_fit_multi_kernel(
    int32_t N, int32_t K, const int32_t* __restrict__ n_cards, const int64_t* __restrict__ cap,
    const int64_t* __restrict__ used, const int32_t* __restrict__ multi,
    const GasSel* __restrict__ sels, const int32_t* __restrict__ counts,
    uint32_t* __restrict__ res, uint64_t* __restrict__ fit) {
  const int32_t n = blockIdx.x * kTpb + threadIdx.x;
  const bool valid = n < N;
  const int32_t nc = valid ? n_cards[n] : 0;
  int64_t free[kMaxCards][Q];
  load_free<Q>(n, valid, min(nc, K), K, cap, used, free);
  const uint32_t node_ok = nc > 0 ? 0x80000000u : 0u;
  int32_t i0, i1;
  list_share(counts, &i0, &i1);
  // pod words and selection records are wave-uniform: scalar loads straight into SGPRs (a
  // selection used to cost a dozen readfirstlanes from an LDS stage)
  // The next pod's word and first two selections are loaded one iteration ahead: otherwise
  // every pod waits on two scalar-load round trips before its first compare.
  {
    SelHead nh = {}, nh1 = {};
    int32_t npw = 0;
    if (i0 < i1) {
      npw = multi[i0];
      nh = sel_head<Q>(sels + (int64_t)i0 * PAS_GAS_MAX_SELECTIONS);
      nh1 = sel_head<Q>(sels + (int64_t)i0 * PAS_GAS_MAX_SELECTIONS + 1);
    }
    for (int32_t i = i0; i < i1; ++i) {
      const GasSel* stage_j = sels + (int64_t)i * PAS_GAS_MAX_SELECTIONS;
      const int32_t pw = npw;
      const SelHead e0 = nh, e1 = nh1;
      if (i + 1 < i1) {
        npw = multi[i + 1];
        nh = sel_head<Q>(stage_j + PAS_GAS_MAX_SELECTIONS);
        nh1 = sel_head<Q>(stage_j + PAS_GAS_MAX_SELECTIONS + 1);
      }
      const int64_t p = pw & 0xFFFFFF;
      const int32_t steps = pw >> 24;
      uint32_t out = 0u;
      if (steps == 2) {
        // two selections without touching free: the second one sees card c0 with the
        // first take added to its need, every other card as it was
        int64_t cmp0[Q], cmp1[Q], cmp1t[Q];
        bool ovf = false;  // need1 + take0 beyond int64: card c0 cannot take the second
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          cmp0[q] = uniform64(e0.cmp[q]);
          cmp1[q] = uniform64(e1.cmp[q]);
          // INT64_MIN + 0 stays unrequested
          ovf |= __builtin_add_overflow(cmp1[q], uniform64(e0.take[q]), &cmp1t[q]);
        }
        const int c0 = __builtin_amdgcn_readfirstlane(e0.bad) ? -1 : first_fit<Q, -1>(free, cmp0);
        int c1 = -1;
        if (!__builtin_amdgcn_readfirstlane(e1.bad)) {
          // card k fits the second selection: cmp1 <= free (k != c0) or cmp1t <= free
          // (k == c0; never when need1 + take0 overflows, a uniform and rare case)
          if (!ovf) {
#pragma unroll
            for (int k = kMaxCards - 1; k >= 0; --k) {
              bool ok = true;
#pragma unroll
              for (int q = 0; q < Q; ++q)
                ok &= (c0 == k ? cmp1t[q] : cmp1[q]) <= free[k][q];
              c1 = ok ? k : c1;
            }
          } else {
#pragma unroll
            for (int k = kMaxCards - 1; k >= 0; --k) {
              bool ok = c0 != k;
#pragma unroll
              for (int q = 0; q < Q; ++q) ok &= cmp1[q] <= free[k][q];
              c1 = ok ? k : c1;
            }
          }
        }
        out = (c0 >= 0 && c1 >= 0) ? (node_ok | (2u << 24) | (uint32_t)c0 | ((uint32_t)c1 << 3))
                                   : 0u;
      } else if (steps <= PAS_GAS_MAX_SELECTIONS) {
        // three or more selections: take cards in a working copy of free
        int64_t w[kMaxCards][Q];
#pragma unroll
        for (int k = 0; k < kMaxCards; ++k)
#pragma unroll
          for (int q = 0; q < Q; ++q) w[k][q] = free[k][q];
        bool fits = true;
        uint32_t word = 0;
        // the next step's record is loaded before the current step's compares (slot
        // min(t + 1, 7) of the row is always in bounds)
        SelHead e = e0;
        for (int32_t t = 0; t < steps; ++t) {
          const SelHead en = sel_head<Q>(stage_j + min(t + 1, PAS_GAS_MAX_SELECTIONS - 1));
          int64_t cmp[Q], take[Q];
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            cmp[q] = uniform64(e.cmp[q]);
            take[q] = uniform64(e.take[q]);
          }
          const int k = __builtin_amdgcn_readfirstlane(e.bad) ? -1 : first_fit<Q, -1>(w, cmp);
          fits = fits && k >= 0;
          // per card taken by some lane of the wave (uniform branch), a per-lane select: a
          // divergent branch around the update would make the compiler copy the array
          int64_t tv[Q];  // the takes in VGPRs once per step (a select may read one SGPR)
#pragma unroll
          for (int q = 0; q < Q; ++q) tv[q] = to_vgpr64(take[q]);
#pragma unroll
          for (int kk = 0; kk < kMaxCards; ++kk)
            if (__ballot(k == kk))
#pragma unroll
              for (int q = 0; q < Q; ++q) w[kk][q] -= k == kk ? tv[q] : 0;
          word |= (uint32_t)(k & 7) << (3 * t);
          e = en;
        }
        out = fits ? (node_ok | ((uint32_t)steps << 24) | word) : 0u;
      }
      put_result<kBits>(res, fit, p, N, n, valid, out);
    }
  }
}

}  // namespace

int gas_fit_launch(pas_ctx* ctx, int32_t n_pods, int32_t max_containers, int32_t i915_index,
                   const int64_t* d_req, const uint32_t* d_req_mask,
                   const int32_t* d_n_containers, uint32_t* d_res, uint64_t* d_fit,
                   hipStream_t s) {
  const GasSnapshot& g = ctx->gas;
  const int32_t N = g.n_nodes, Q = g.n_res, K = g.max_cards;
  if (N == 0 || n_pods == 0) return PAS_OK;
  // scratch: single-selection records [Q+1][P] | multi-selection pod words [P] | their
  // selection rows [P][8] | the flipped kind minima [4] and counts [Q+2] (zeroed together)
  if (n_pods > (1 << 24)) return set_error(ctx, PAS_ECAPACITY, "pas_gas_fit: > 2^24 pods");
  const int32_t NL = Q + 1;
  const size_t b_single = (sizeof(GasSingle) * (size_t)NL * n_pods + 255) & ~size_t(255);
  const size_t b_multi = (sizeof(int32_t) * (size_t)n_pods + 255) & ~size_t(255);
  const size_t b_sels =
      (sizeof(GasSel) * PAS_GAS_MAX_SELECTIONS * (size_t)n_pods + 255) & ~size_t(255);
  constexpr size_t b_tail = (PAS_GAS_MAX_RES + 2) * sizeof(int32_t) +
                            PAS_GAS_MAX_RES * sizeof(unsigned long long);
  const size_t need = b_single + b_multi + b_sels + b_tail;
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
  char* base = static_cast<char*>(ctx->aux);
  GasSingle* single = reinterpret_cast<GasSingle*>(base);
  int32_t* multi = reinterpret_cast<int32_t*>(base + b_single);
  GasSel* sels = reinterpret_cast<GasSel*>(base + b_single + b_multi);
  unsigned long long* gflip =
      reinterpret_cast<unsigned long long*>(base + b_single + b_multi + b_sels);
  int32_t* counts = reinterpret_cast<int32_t*>(gflip + PAS_GAS_MAX_RES);
  TimedLaunch tl;
  timing_begin(ctx, s, PAS_K_GAS_PREP, &tl);
  PAS_HIP(ctx, hipMemsetAsync(gflip, 0, b_tail, s));
  gas_minfree_kernel<<<(N + kTpb - 1) / kTpb, kTpb, 0, s>>>(N, K, Q, g.n_cards, g.cap, g.used,
                                                           gflip);
  gas_prep_kernel<<<(n_pods + kTpb - 1) / kTpb, kTpb, 0, s>>>(
      n_pods, max_containers, Q, i915_index, d_req, d_req_mask, d_n_containers, gflip, single,
      multi, sels, counts);
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  // grids: node blocks x pod chunks, ~4096 blocks for the whole batch; each kernel splits
  // each of its device-counted lists evenly over its chunks
  const int32_t node_blocks = (N + kTpb - 1) / kTpb;
  const int32_t chunks = std::max(1, std::min(n_pods, (4096 + node_blocks - 1) / node_blocks));
  const dim3 grid((unsigned)node_blocks, (unsigned)chunks);
  timing_begin(ctx, s, PAS_K_GAS_FIT, &tl);
  const bool bits = d_fit != nullptr;
  switch (Q * 2 + (bits ? 1 : 0)) {
#define PAS_GAS_CASE(QQ, B)                                                                    \
  case QQ * 2 + B:                                                                             \
    gas_fit_single_kernel<QQ, B><<<grid, kTpb, 0, s>>>(N, K, n_pods, g.n_cards, g.cap, g.used, \
                                                       single, counts, d_res, d_fit);          \
    gas_fit_multi_kernel<QQ, B><<<grid, kTpb, 0, s>>>(N, K, g.n_cards, g.cap, g.used, multi,   \
                                                      sels, counts + NL, d_res, d_fit);        \
    break;
    PAS_GAS_CASE(1, 0) PAS_GAS_CASE(2, 0) PAS_GAS_CASE(3, 0) PAS_GAS_CASE(4, 0)
    PAS_GAS_CASE(1, 1) PAS_GAS_CASE(2, 1) PAS_GAS_CASE(3, 1) PAS_GAS_CASE(4, 1)
#undef PAS_GAS_CASE
    default: return set_error(ctx, PAS_EINVAL, "pas_gas_fit: n_res out of range");
  }
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

}  // namespace pas
