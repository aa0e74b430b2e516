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

// The list a multi-selection pod is filed under: 1 + q for the lowest kind q that some
// selection requests and whose compare can be dropped from every selection's scan of the
// cards the pod has not taken from yet (untouched cards hold their snapshot free, >= gmin[q]):
// each selection either does not request q or needs at most gmin[q] of it and requests
// another kind too (cards a node does not have must keep failing).  Cards the pod has taken
// from are always compared on every kind.  Else 0.
__device__ __forceinline__ int32_t multi_skip_list(int32_t n_res, uint32_t ok_mask,
                                                   uint32_t req_mask) {
  const uint32_t m = ok_mask & req_mask & ((1u << n_res) - 1u);
  return m ? 1 + __builtin_ctz(m) : 0;
}

// One thread per pod files it under `single` (<= 1 selection: its selecting step, in the
// list of its skippable kind; lists [n_res + 1][n_pods]) or `multi` (several: lists
// [n_res + 1][n_pods] of words pod | S << 24, by skippable kind as multi_skip_list); a multi
// pod's selections (containers in order, then gpuNum) go to its own row sels[pod][8].  More
// than PAS_GAS_MAX_SELECTIONS selections are beyond the packed result and keep only the
// count.  counts: [n_res + 1] single lists, then [n_res + 1] multi lists.
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
  uint32_t skip_ok = (1u << n_res) - 1u, skip_req = 0;  // multi_skip_list
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
      const uint32_t gk = (uint32_t)g.kinds;
      skip_req |= gk;
      for (int q = 0; q < n_res; ++q) {
        if (!((gk >> q) & 1u)) continue;
        const int64_t gmin = (int64_t)((unsigned long long)INT64_MAX - gflip[q]);
        if (g.cmp[q] > gmin || gk == (1u << q)) skip_ok &= ~(1u << q);
      }
    }
  }
  const bool one_sel = steps <= 1;
  const int32_t l = one_sel ? (steps == 1 ? skip_list(n_res, one.cmp, kinds, gflip) : 0)
                            : multi_skip_list(n_res, skip_ok, skip_req);
  const int32_t nl = n_res + 1;
  const int32_t slot = wave_slot(counts, one_sel ? l : nl + l);
  if (one_sel) {
    one.steps = steps;
    single[(int64_t)l * n_pods + slot] = one;
    return;
  }
  multi[(int64_t)l * n_pods + slot] = p | (steps << 24);
  if (steps > PAS_GAS_MAX_SELECTIONS) return;
  GasSel* out = sels + (int64_t)p * PAS_GAS_MAX_SELECTIONS;
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

// Blocks of the fit kernels cover (node block, pod chunk) pairs.  A 1-D grid is mapped so
// that every chunk of a node block runs on the same XCD (block b runs on XCD b % 8,
// MI355X_MICROARCH.md): pairs are ordered node-major and each XCD takes a contiguous run of
// them, so a node block's snapshot rows are fetched into one L2 only.
struct BlockTile {
  int32_t node_block, chunk, chunks;
};
__device__ __forceinline__ BlockTile block_tile(int32_t chunks) {
  const int32_t nb = gridDim.x, b = blockIdx.x;
  const int32_t xcd = b & 7, per = nb >> 3, rem = nb & 7;
  const int32_t pos = xcd * per + min(xcd, rem) + (b >> 3);
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

// Pods with at most one selection, list `l` (kind SKIP = l - 1 dropped): a read-only first
// fit per (pod, node lane), pod records staged in LDS per batch and read into SGPRs.
template <int Q, int SKIP, bool kBits>
__device__ __forceinline__ void single_list(const int64_t (&free)[kMaxCards][Q],
                                            uint32_t node_ok, int32_t N, int32_t n, bool valid,
                                            const GasSingle* __restrict__ single,
                                            const int32_t* __restrict__ count, GasSingle* stage,
                                            const BlockTile& bt, uint32_t* __restrict__ res,
                                            uint64_t* __restrict__ fit) {
  int32_t i0, i1;
  list_share(count, bt, &i0, &i1);
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
                                             GasSingle* stage, const BlockTile& bt,
                                             uint32_t* __restrict__ res,
                                             uint64_t* __restrict__ fit) {
  single_list<Q, L - 1, kBits>(free, node_ok, N, n, valid, single + (int64_t)L * P, counts + L,
                               stage, bt, res, fit);
  if constexpr (L < Q)
    single_lists<Q, kBits, L + 1>(free, node_ok, N, n, valid, P, single, counts, stage, bt, res,
                                  fit);
}

template <int Q, bool kBits>
__global__ __launch_bounds__(kTpb) void gas_fit_single_kernel(
    int32_t N, int32_t K, int32_t P, const int32_t* __restrict__ n_cards,
    const int64_t* __restrict__ cap, const int64_t* __restrict__ used,
    const GasSingle* __restrict__ single, const int32_t* __restrict__ counts, int32_t chunks,
    uint32_t* __restrict__ res, uint64_t* __restrict__ fit) {
  __shared__ GasSingle stage[kPodBatch];
  const BlockTile bt = block_tile(chunks);
  const int32_t n = bt.node_block * kTpb + threadIdx.x;
  const bool valid = n < N;
  const int32_t nc = valid ? n_cards[n] : 0;
  int64_t free[kMaxCards][Q];
  load_free<Q>(n, valid, min(nc, K), K, cap, used, free);
  // FetchNode error / missing cards label -> errWontFit before any container (:282-298)
  const uint32_t node_ok = nc > 0 ? 0x80000000u : 0u;
  single_lists<Q, kBits>(free, node_ok, N, n, valid, P, single, counts, stage, bt, res, fit);
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

// Lane mask of a <= v (a wave-uniform, in SGPRs): the compare writes the mask directly.
__device__ __forceinline__ uint64_t le_mask(int64_t a, int64_t v) {
  uint64_t m;
  asm("v_cmp_le_i64_e64 %0, %1, %2" : "=s"(m) : "s"(a), "v"(v));
  return m;
}

// bm * 2 + (this lane's bit of `mask`): one v_addc with the lane mask as carry-in.  Cards are
// pushed from the last to the first, so bit k of the result is card k.  `mask` must come from
// a scalar instruction (an s_and of compare masks): a VALU-written SGPR read as a lane mask by
// the next VALU instruction needs wait states that inline assembly does not get.
__device__ __forceinline__ uint32_t push_bit(uint32_t bm, uint64_t mask) {
  uint32_t r;
  uint64_t carry_out;
  asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(carry_out) : "v"(bm), "s"(mask));
  return r;
}

constexpr int kMT = 128;  // threads per multi-selection block
// LDS working copy of the lanes' free capacity: cur[k][q][tid] for cards k < 8, plus row 8
// where lanes without a fitting card put their takes (never read as a real card).
template <int Q>
constexpr size_t multi_lds_bytes() { return sizeof(int64_t) * 9 * Q * kMT; }

// Pods with several selections (list `list`, kind SKIP = list - 1 dropped from the scans of
// untouched cards): the selections in order (containers, then gpuNum), each taking the first
// card that passes checkResourceCapacity (:341-383) with the pod's earlier takes (addRM,
// resource_map.go:38-53) included.
//   * Cards the pod has not taken from yet still hold the snapshot's free values, which stay
//     in registers: one compare per (card, kind), the per-card verdicts packed into a lane
//     bit mask bm (bit k = card k), masked by the cards not taken from (tm_not).
//   * Cards it has taken from are the cards of the earlier selections (slots s < t); their
//     current free lives in the lane's LDS column and is compared on every kind.
//   * The selection is the lowest card of either set; taking it subtracts the need from the
//     LDS column (ds_add_u64 of -need, no return).  After the pod the touched cards' columns
//     are rewritten from the registers.
// The per-lane state of one pod's selections: slot s = the card taken at selection s and the
// LDS index of its column.
struct MultiState {
  uint32_t tm_not;  // bit k set: card k not taken from yet
  uint32_t word;    // packed card ranks
  bool fits;
  int32_t slot_c[PAS_GAS_MAX_SELECTIONS];
  int32_t slot_a[PAS_GAS_MAX_SELECTIONS];
};

// Selection T of the pod (recursion = full unroll, so slots are registers); returns when the
// pod has no more selections or no node of the wave can still fit it.
template <int Q, int SKIP, int T>
__device__ __forceinline__ void multi_step(const int64_t (&free)[kMaxCards][Q], int64_t* cur,
                                           int32_t tid, uint64_t live_mask, int32_t S,
                                           const GasSel* rec, SelHead e, MultiState& st) {
  if constexpr (T < PAS_GAS_MAX_SELECTIONS) {
    if (T >= S) return;
    if (e.bad) {  // a negative need fails every card (:343-347)
      st.fits = false;
      return;
    }
    // next record's scalar loads in flight during this selection
    const SelHead en = sel_head<Q>(rec + min(T + 1, PAS_GAS_MAX_SELECTIONS - 1));
    // untouched cards: snapshot free in registers; per card the kinds' compare masks and-ed
    // in SALU (with the live lanes, so the mask is always a scalar result)
    constexpr int kCompared = Q - (SKIP >= 0 ? 1 : 0);
    uint32_t bm = 0u;
#pragma unroll
    for (int k = kMaxCards - 1; k >= 0; --k) {
      uint64_t m = ~0ull;
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (q != SKIP) m &= le_mask(e.cmp[q], free[k][q]);
      if (kCompared == 1) m &= live_mask;  // one compare: an s_and makes the mask scalar
      bm = push_bit(bm, m);
    }
    const uint32_t u = bm & st.tm_not;
    uint32_t c = u ? (uint32_t)__builtin_ctz(u) : 8u;
    // touched cards: current free in LDS, every kind
#pragma unroll
    for (int sl = 0; sl < T; ++sl) {
      bool ok = true;
#pragma unroll
      for (int q = 0; q < Q; ++q) ok &= e.cmp[q] <= cur[st.slot_a[sl] + q * kMT];
      c = ok ? min(c, (uint32_t)st.slot_c[sl]) : c;
    }
    st.fits = st.fits && c < 8u;
    if (!__ballot(st.fits)) return;  // no node of the wave fits the pod any more
    st.slot_c[T] = (int32_t)c;
    st.slot_a[T] = (int32_t)c * (Q * kMT) + tid;
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (e.take[q] != 0)
        atomicAdd(reinterpret_cast<unsigned long long*>(&cur[st.slot_a[T] + q * kMT]),
                  (unsigned long long)(-e.take[q]));
    st.tm_not &= ~(1u << c);
    st.word |= (c & 7u) << (3 * T);
    multi_step<Q, SKIP, T + 1>(free, cur, tid, live_mask, S, rec, en, st);
  }
}

// Pods with several selections (list `list`, kind SKIP = list - 1 dropped from the scans of
// untouched cards): the selections in order (containers, then gpuNum), each taking the first
// card that passes checkResourceCapacity (:341-383) with the pod's earlier takes (addRM,
// resource_map.go:38-53) included.
//   * Cards the pod has not taken from yet still hold the snapshot's free values, which stay
//     in registers: one compare per (card, kind), the per-card verdicts packed into a lane
//     bit mask bm (bit k = card k), masked by the cards not taken from (tm_not).
//   * Cards it has taken from are the cards of the earlier selections (slots s < t); their
//     current free lives in the lane's LDS column and is compared on every kind.
//   * The selection is the lowest card of either set; taking it subtracts the need from the
//     LDS column (ds_add_u64 of -need, no return).  After the pod the touched cards' columns
//     are rewritten from the registers.
template <int Q, int SKIP, bool kBits>
__device__ __forceinline__ void multi_list(const int64_t (&free)[kMaxCards][Q], int64_t* cur,
                                           uint32_t node_ok, int32_t N, int32_t n, bool valid,
                                           const int32_t* __restrict__ list,
                                           const GasSel* __restrict__ sels,
                                           const int32_t* __restrict__ count, const BlockTile& bt,
                                           uint32_t* __restrict__ res,
                                           uint64_t* __restrict__ fit) {
  const int32_t tid = threadIdx.x;
  const bool live = valid && node_ok != 0u;
  const uint64_t live_mask = __ballot(live);
  int32_t i0, i1;
  list_share(count, bt, &i0, &i1);
  for (int32_t i = i0; i < i1; ++i) {
    const int32_t pw = list[i];
    const int64_t pod = pw & 0xFFFFFF;
    const int32_t S = pw >> 24;
    uint32_t out = 0u;
    if (S <= PAS_GAS_MAX_SELECTIONS) {
      const GasSel* rec = sels + pod * PAS_GAS_MAX_SELECTIONS;
      MultiState st;
      st.tm_not = 0xFFu;
      st.word = 0u;
      st.fits = live;
      multi_step<Q, SKIP, 0>(free, cur, tid, live_mask, S, rec, sel_head<Q>(rec), st);
      out = st.fits ? (node_ok | ((uint32_t)S << 24) | st.word) : 0u;
      // restore the touched cards' columns
#pragma unroll
      for (int k = 0; k < kMaxCards; ++k) {
        const bool touched = !((st.tm_not >> k) & 1u);
        if (__ballot(touched) && touched)
#pragma unroll
          for (int q = 0; q < Q; ++q) cur[(k * Q + q) * kMT + tid] = free[k][q];
      }
    }
    put_result<kBits>(res, fit, pod, N, n, valid, out);
  }
}

template <int Q, bool kBits, int L = 0>
__device__ __forceinline__ void multi_lists(const int64_t (&free)[kMaxCards][Q], int64_t* cur,
                                            uint32_t node_ok, int32_t N, int32_t n, bool valid,
                                            int32_t P, const int32_t* __restrict__ multi,
                                            const GasSel* __restrict__ sels,
                                            const int32_t* __restrict__ counts,
                                            const BlockTile& bt, uint32_t* __restrict__ res,
                                            uint64_t* __restrict__ fit) {
  multi_list<Q, L - 1, kBits>(free, cur, node_ok, N, n, valid, multi + (int64_t)L * P, sels,
                              counts + L, bt, res, fit);
  if constexpr (L < Q)
    multi_lists<Q, kBits, L + 1>(free, cur, node_ok, N, n, valid, P, multi, sels, counts, bt,
                                 res, fit);
}

template <int Q, bool kBits>
__global__ __launch_bounds__(kMT) void gas_fit_multi_kernel(
    int32_t N, int32_t K, int32_t P, const int32_t* __restrict__ n_cards,
    const int64_t* __restrict__ cap, const int64_t* __restrict__ used,
    const int32_t* __restrict__ multi, const GasSel* __restrict__ sels,
    const int32_t* __restrict__ counts, int32_t chunks, uint32_t* __restrict__ res,
    uint64_t* __restrict__ fit) {
  extern __shared__ __attribute__((aligned(16))) int64_t cur[];
  const BlockTile bt = block_tile(chunks);
  const int32_t n = bt.node_block * kMT + threadIdx.x;
  const bool valid = n < N;
  const int32_t nc = valid ? n_cards[n] : 0;
  int64_t free[kMaxCards][Q];
  load_free<Q>(n, valid, min(nc, K), K, cap, used, free);
#pragma unroll
  for (int k = 0; k < kMaxCards; ++k)
#pragma unroll
    for (int q = 0; q < Q; ++q) cur[(k * Q + q) * kMT + threadIdx.x] = free[k][q];
  const uint32_t node_ok = nc > 0 ? 0x80000000u : 0u;
  multi_lists<Q, kBits>(free, cur, node_ok, N, n, valid, P, multi, sels, counts, bt, res, fit);
}

}  // namespace

int gas_fit_launch(pas_ctx* ctx, int32_t n_pods, int32_t max_containers, int32_t i915_index,
                   const int64_t* d_req, const uint32_t* d_req_mask,
                   const int32_t* d_n_containers, uint32_t* d_res, uint64_t* d_fit,
                   hipStream_t s) {
  const GasSnapshot& g = ctx->gas;
  const int32_t N = g.n_nodes, Q = g.n_res, K = g.max_cards;
  if (N == 0 || n_pods == 0) return PAS_OK;
  // scratch: single-selection records [Q+1][P] | multi-selection pod words [Q+1][P] | their
  // selection rows [P][8] | the flipped kind minima [4] and counts [2(Q+1)] (zeroed together)
  if (n_pods > (1 << 24)) return set_error(ctx, PAS_ECAPACITY, "pas_gas_fit: > 2^24 pods");
  const int32_t NL = Q + 1;
  const size_t b_single = (sizeof(GasSingle) * (size_t)NL * n_pods + 255) & ~size_t(255);
  const size_t b_multi = (sizeof(int32_t) * (size_t)NL * n_pods + 255) & ~size_t(255);
  const size_t b_sels =
      (sizeof(GasSel) * PAS_GAS_MAX_SELECTIONS * (size_t)n_pods + 255) & ~size_t(255);
  constexpr size_t b_tail = 2 * (PAS_GAS_MAX_RES + 1) * sizeof(int32_t) +
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
  // grids: (node block, pod chunk) pairs, ~4096 blocks for the single kernel and ~8192 for
  // the multi kernel (half the nodes per block); each kernel splits each of its
  // device-counted lists evenly over the chunks
  const int32_t nb_s = (N + kTpb - 1) / kTpb, nb_m = (N + kMT - 1) / kMT;
  const int32_t ch_s = std::max(1, std::min(n_pods, (4096 + nb_s - 1) / nb_s));
  const int32_t ch_m = std::max(1, std::min(n_pods, (8192 + nb_m - 1) / nb_m));
  timing_begin(ctx, s, PAS_K_GAS_FIT, &tl);
  const bool bits = d_fit != nullptr;
  switch (Q * 2 + (bits ? 1 : 0)) {
#define PAS_GAS_CASE(QQ, B)                                                                    \
  case QQ * 2 + B:                                                                             \
    gas_fit_single_kernel<QQ, B><<<nb_s * ch_s, kTpb, 0, s>>>(                                 \
        N, K, n_pods, g.n_cards, g.cap, g.used, single, counts, ch_s, d_res, d_fit);           \
    gas_fit_multi_kernel<QQ, B><<<nb_m * ch_m, kMT, multi_lds_bytes<QQ>(), s>>>(               \
        N, K, n_pods, g.n_cards, g.cap, g.used, multi, sels, counts + NL, ch_m, d_res, d_fit); \
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
