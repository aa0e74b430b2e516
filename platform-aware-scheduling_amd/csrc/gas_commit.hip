// gas_commit.hip — bind-time commit of GAS card selections into the resident snapshot.
//
// GASExtender.bindNode (gpu-aware-scheduling/pkg/gpuscheduler/scheduler.go:385-445) runs
// runSchedulingLogic for the pod on the chosen node once more (:417-421), then
// Cache.adjustPodResources(add) (node_resource_cache.go:240-287) adds, per container, the
// request divided by the container's card count to each card of its annotation segment, all
// or nothing (checkPodResourceAdjustment on a copy first, :187-238).  A pod leaving the node
// runs adjustPodResources(remove): subtractRM per card (resource_map.go:55-73, 103-127: a
// negative amount or a key the card lacks is an input error; results clamp at zero).
//
// Here both patch the device-resident used[N][K][Q] in place, so the frozen snapshot stays
// consistent across binds without a re-upload.  The host sorts the operations by node
// (stable); one thread owns each node and applies that node's operations in call order, so
// operations on one node see each other exactly as the reference's serialised binds do.
// This is latency work (a few thousand operations per call at most), not a hot kernel.
#include <hip/hip_runtime.h>

#include "gas_runs.h"
#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 64;
constexpr int kMaxRes = PAS_GAS_MAX_RES;

// checkResourceCapacity (scheduler.go:341-383) for one requested kind.
__device__ __forceinline__ bool kind_fits(int64_t need, int64_t cap, int64_t used) {
  if (need < 0 || cap <= 0 || used < 0) return false;
  const int64_t sum = (int64_t)((uint64_t)used + (uint64_t)need);
  return sum >= 0 && cap >= sum;
}

struct BindArgs {
  int32_t K, Q, C, i915;
  const int32_t* order;    // operation indices sorted by node (stable)
  const int32_t* seg_off;  // [n_seg + 1] into order
  const int32_t* op_pod;
  const int32_t* op_node;
  const int32_t* n_cards;
  const int64_t* cap;
  int64_t* used;
  const int64_t* req;      // [n_pods][C][Q]
  const uint32_t* mask;    // [n_pods][C]
  const int32_t* ncont;    // [n_pods]
  const int32_t* cpc;      // release: [n_ops][C] cards per container
  const int32_t* cards;    // release: [n_ops][cards_stride]
  int32_t cards_stride;    // 8 (pas_gas_release) or PAS_GAS_MAX_SELECTIONS (_ex)
  uint32_t* res_out;       // bind: [n_ops]
  int32_t* status;         // [n_ops]
  uint8_t* cards_out;      // bind_ex: [n_ops][PAS_GAS_MAX_SELECTIONS] or null
  int32_t* nsel_out;       // bind_ex: [n_ops] or null
  int64_t* counts_out;     // bind_counts: [n_ops][C][K] or null
  const int64_t* counts;   // release_counts: [n_ops][C][K] (else cpc / cards)
};

// KMAX: the snapshot's max_cards rounded up to 8 / 16 / 64 (the per-thread copies live in
// registers for the common shapes, in scratch for 64-card snapshots).
template <int KMAX>
__global__ __launch_bounds__(kTpb) void gas_bind_kernel(int32_t n_seg, BindArgs a) {
  const int32_t sgi = blockIdx.x * kTpb + threadIdx.x;
  if (sgi >= n_seg) return;
  const int32_t K = a.K, Q = a.Q, C = a.C;
  const int32_t n = a.op_node[a.order[a.seg_off[sgi]]];
  const int32_t ncard = min(a.n_cards[n], K);
  int64_t* un = a.used + (int64_t)n * K * Q;
  int64_t u[KMAX][kMaxRes], cap[kMaxRes];
  for (int k = 0; k < K; ++k)
    for (int q = 0; q < Q; ++q) u[k][q] = un[k * Q + q];
  for (int q = 0; q < Q; ++q) cap[q] = a.cap[(int64_t)n * Q + q];
  for (int32_t i = a.seg_off[sgi]; i < a.seg_off[sgi + 1]; ++i) {
    const int32_t op = a.order[i];
    const int32_t p = a.op_pod[op];
    // runSchedulingLogic on the node's current usage: a working copy (readNodeResources,
    // node_resource_cache.go:474-491), first fit per selection, takes accumulate (addRM)
    int64_t w[KMAX][kMaxRes];
    for (int k = 0; k < K; ++k)
      for (int q = 0; q < Q; ++q) w[k][q] = u[k][q];
    bool fits = ncard > 0;  // FetchNode error / no cards label (:282-298)
    uint32_t word = 0;
    int64_t nsel = 0;
    bool packable = true;
    uint8_t* sel_out = a.cards_out ? a.cards_out + (int64_t)op * PAS_GAS_MAX_SELECTIONS : nullptr;
    if (sel_out)
      for (int j = 0; j < PAS_GAS_MAX_SELECTIONS; ++j) sel_out[j] = 0;
    int64_t* cnt = a.counts_out ? a.counts_out + (int64_t)op * C * K : nullptr;
    if (cnt)
      for (int64_t j = 0; j < (int64_t)C * K; ++j) cnt[j] = 0;
    for (int32_t c = 0; fits && c < a.ncont[p]; ++c) {
      const int64_t b = (int64_t)p * C + c;
      const uint32_t m = a.mask[b];
      if (m == 0u) continue;  // no GPU resources: no cards (:206-208)
      int64_t r[kMaxRes];
      for (int q = 0; q < Q; ++q) r[q] = a.req[b * Q + q];
      int64_t num = 0;  // getNumI915 (:192-198)
      if (a.i915 >= 0 && ((m >> a.i915) & 1u) && r[a.i915] > 0) num = r[a.i915];
      if (num > 1)
        for (int q = 0; q < Q; ++q) r[q] /= num;  // getPerGPUResourceRequest (:180-190)
      if (num > kRunsFrom) {  // more than PAS_GAS_MAX_SELECTIONS: card runs (gas_runs.h)
        fits = container_runs<KMAX>(Q, m, r, num, cap, w, ncard, [&](int k, int64_t t) {
          if (cnt) cnt[(int64_t)c * K + k] += t;
        });
        nsel += num;
        packable = false;
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
        if (nsel < PAS_GAS_PACKED) word |= (uint32_t)chosen << (3 * nsel);
        packable = packable && chosen < PAS_GAS_PACKED;
        if (sel_out && nsel < PAS_GAS_MAX_SELECTIONS) sel_out[nsel] = (uint8_t)chosen;
        if (cnt) cnt[(int64_t)c * K + chosen] += 1;
        ++nsel;
      }
    }
    if (!fits) {
      a.res_out[op] = 0u;
      a.status[op] = PAS_GAS_WONT_FIT;
      if (a.nsel_out) a.nsel_out[op] = 0;
      if (sel_out)  // the selections of a bind that did not fit are not reported
        for (int j = 0; j < PAS_GAS_MAX_SELECTIONS; ++j) sel_out[j] = 0;
      if (cnt)
        for (int64_t j = 0; j < (int64_t)C * K; ++j) cnt[j] = 0;
      continue;
    }
    // the pas_gas_fit word: selections that do not pack are PAS_GAS_SEL_EXTENDED, more than
    // PAS_GAS_MAX_SELECTIONS PAS_GAS_SEL_LIMIT (cards_out zero, n_sel -1: counts_out has them)
    const bool wide = nsel > PAS_GAS_MAX_SELECTIONS;
    a.res_out[op] = nsel <= PAS_GAS_PACKED && packable
                        ? 0x80000000u | ((uint32_t)nsel << 24) | word
                        : 0x80000000u | ((uint32_t)(wide ? PAS_GAS_SEL_LIMIT
                                                         : PAS_GAS_SEL_EXTENDED) << 24);
    if (a.nsel_out) a.nsel_out[op] = wide ? -1 : (int32_t)nsel;
    if (sel_out && wide)
      for (int j = 0; j < PAS_GAS_MAX_SELECTIONS; ++j) sel_out[j] = 0;
    // adjustPodResources(add) with that annotation adds request / numCards (= numI915) to
    // each selected card: exactly the working copy's takes, which cannot overflow after the
    // capacity checks
    for (int k = 0; k < K; ++k)
      for (int q = 0; q < Q; ++q) u[k][q] = w[k][q];
    a.status[op] = PAS_GAS_OK;
  }
  for (int k = 0; k < K; ++k)
    for (int q = 0; q < Q; ++q) un[k * Q + q] = u[k][q];
}

template <int KMAX>
__global__ __launch_bounds__(kTpb) void gas_release_kernel(int32_t n_seg, BindArgs a) {
  const int32_t sgi = blockIdx.x * kTpb + threadIdx.x;
  if (sgi >= n_seg) return;
  const int32_t K = a.K, Q = a.Q, C = a.C;
  const int32_t n = a.op_node[a.order[a.seg_off[sgi]]];
  const int32_t ncard = max(0, min(a.n_cards[n], K));
  int64_t* un = a.used + (int64_t)n * K * Q;
  int64_t u[KMAX][kMaxRes];
  for (int k = 0; k < K; ++k)
    for (int q = 0; q < Q; ++q) u[k][q] = un[k * Q + q];
  for (int32_t i = a.seg_off[sgi]; i < a.seg_off[sgi + 1]; ++i) {
    const int32_t op = a.order[i];
    const int32_t p = a.op_pod[op];
    int64_t w[KMAX][kMaxRes];  // checkPodResourceAdjustment's copy
    for (int k = 0; k < K; ++k)
      for (int q = 0; q < Q; ++q) w[k][q] = u[k][q];
    bool ok = true;
    int32_t off = 0;
    if (a.counts) {  // the annotation as counts per container and card (any length)
      const int64_t* cnt = a.counts + (int64_t)op * C * K;
      for (int32_t c = 0; ok && c < a.ncont[p]; ++c) {
        int64_t kc = 0;  // numCards (the host checked that the sum does not overflow)
        for (int k = 0; k < K; ++k) kc += cnt[(int64_t)c * K + k];
        if (kc <= 0) continue;  // empty annotation segment
        const int64_t b = (int64_t)p * C + c;
        const uint32_t m = a.mask[b];
        if (m & PAS_REQ_UNKNOWN_KIND) ok = false;
        int64_t r[kMaxRes];
        for (int q = 0; q < Q; ++q) r[q] = a.req[b * Q + q] / kc;  // divide(numCards)
        for (int k = 0; ok && k < K; ++k) {
          const int64_t t = cnt[(int64_t)c * K + k];
          if (t <= 0) continue;
          for (int q = 0; q < Q; ++q) {
            if (!((m >> q) & 1u)) continue;
            if (r[q] < 0 || k >= ncard) {  // negative amount / a card the label lacks
              ok = false;
              break;
            }
            w[k][q] = subtract_times(w[k][q], r[q], t);
          }
        }
      }
    }
    for (int32_t c = 0; !a.counts && ok && c < a.ncont[p]; ++c) {
      const int32_t kc = a.cpc[(int64_t)op * C + c];
      if (kc <= 0) continue;  // empty annotation segment
      const int64_t b = (int64_t)p * C + c;
      const uint32_t m = a.mask[b];
      int64_t r[kMaxRes];
      for (int q = 0; q < Q; ++q) r[q] = a.req[b * Q + q] / kc;  // divide(numCards)
      // subtractRM of a key no card map has (a kind outside the snapshot) -> errInput
      if (m & PAS_REQ_UNKNOWN_KIND) ok = false;
      for (int32_t j = 0; ok && j < kc; ++j) {
        const int32_t k = a.cards[(int64_t)op * a.cards_stride + off + j];
        const bool known = k >= 0 && k < ncard;
        for (int q = 0; q < Q; ++q) {
          if (!((m >> q) & 1u)) continue;
          // subtract: negative amount or a key the card lacks -> errInput
          if (r[q] < 0 || !known) {
            ok = false;
            break;
          }
          const int64_t v = (int64_t)((uint64_t)w[k][q] - (uint64_t)r[q]);  // Go wraps
          w[k][q] = v < 0 ? 0 : v;  // capped to zero
        }
      }
      off += kc;
    }
    if (!ok) {
      a.status[op] = PAS_GAS_ERR_INPUT;
      continue;
    }
    for (int k = 0; k < K; ++k)
      for (int q = 0; q < Q; ++q) u[k][q] = w[k][q];
    a.status[op] = PAS_GAS_OK;
  }
  for (int k = 0; k < K; ++k)
    for (int q = 0; q < Q; ++q) un[k * Q + q] = u[k][q];
}

}  // namespace

int gas_commit_launch(pas_ctx* ctx, bool release, int32_t n_seg, int32_t max_containers,
                      int32_t i915_index, const int32_t* d_order, const int32_t* d_seg_off,
                      const int32_t* d_pod, const int32_t* d_node, const int64_t* d_req,
                      const uint32_t* d_mask, const int32_t* d_ncont, const int32_t* d_cpc,
                      const int32_t* d_cards, int32_t cards_stride, uint32_t* d_res,
                      int32_t* d_status, uint8_t* d_cards_out, int32_t* d_nsel_out,
                      int64_t* d_counts_out, const int64_t* d_counts, hipStream_t s) {
  if (n_seg == 0) return PAS_OK;
  GasSnapshot& g = ctx->gas;
  BindArgs a{g.max_cards, g.n_res,  max_containers, i915_index, d_order, d_seg_off,
             d_pod,       d_node,   g.n_cards,      g.cap,      g.used,  d_req,
             d_mask,      d_ncont,  d_cpc,          d_cards,    cards_stride,
             d_res,       d_status, d_cards_out,    d_nsel_out, d_counts_out, d_counts};
  const unsigned blocks = (unsigned)((n_seg + kTpb - 1) / kTpb);
#define PAS_COMMIT(KM)                                       \
  if (release)                                               \
    gas_release_kernel<KM><<<blocks, kTpb, 0, s>>>(n_seg, a); \
  else                                                       \
    gas_bind_kernel<KM><<<blocks, kTpb, 0, s>>>(n_seg, a);
  if (g.max_cards <= 8) {
    PAS_COMMIT(8)
  } else if (g.max_cards <= 16) {
    PAS_COMMIT(16)
  } else {
    PAS_COMMIT(PAS_GAS_MAX_CARDS)
  }
#undef PAS_COMMIT
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

}  // namespace pas
