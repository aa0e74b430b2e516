// gas_fit.hip — batched GAS filter: one runSchedulingLogic per (pod, node).
//
// Reference (gpu-aware-scheduling/pkg/gpuscheduler/scheduler.go):
//   runSchedulingLogic (:280-338): per container, getCardsForContainerGPURequest
//   (:200-257) loops gpuNum < numI915 over the node's cards in sort.Strings order and
//   takes the first card for which checkResourceCapacity (:341-383) holds, adding the
//   per-GPU request to that card's usage (addRM, resource_map.go:38-53), so later
//   selections of the same pod see it; no fit -> errWontFit.
//
// Device formulation: one lane per node, holding the node's frozen per-card usage
// (Cache.getNodeResourceStatus, node_resource_cache.go:474-491) in registers, walks a
// chunk of pods (the pod loop is wave-uniform, so container/step tables are scalar
// loads).  checkResourceCapacity for a requested kind q with need >= 0 and cap > 0 is
// exactly   0 <= used <= cap - need   (then used + need cannot overflow), i.e. one
// unsigned 64-bit compare against slack = cap - need; kinds not requested get
// slack = UINT64_MAX.  A negative need or non-positive cap on a requested kind makes
// the container unplaceable on this node (:343-354).
#include <hip/hip_runtime.h>

#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;
constexpr int kMaxCards = PAS_GAS_MAX_CARDS;

// Per (pod, container) step table built by gas_prep_kernel.
struct alignas(16) GasContainer {
  int64_t req[PAS_GAS_MAX_RES];  // per-GPU request (getPerGPUResourceRequest :180-190); 0 if
                                 // the kind is not requested
  uint32_t mask;                 // requested kinds
  int32_t num_i915;              // getNumI915 (:192-198)
  int32_t pad[2];
};

// getPerGPUResourceRequest: copy the container's map and, when numI915 > 1, divide
// every entry (the i915 entry included) by numI915, truncating (resource_map.go:129-145).
__global__ void gas_prep_kernel(int32_t n, int32_t n_res, int32_t i915,
                                const int64_t* __restrict__ req,
                                const uint32_t* __restrict__ mask,
                                GasContainer* __restrict__ out) {
  const int32_t i = blockIdx.x * kTpb + threadIdx.x;
  if (i >= n) return;
  GasContainer g;
  g.mask = mask[i];
  int64_t ni = 0;
  if (i915 >= 0 && ((g.mask >> i915) & 1u)) {
    const int64_t v = req[(int64_t)i * n_res + i915];
    if (v > 0) ni = v;
  }
  g.num_i915 = (int32_t)ni;
#pragma unroll
  for (int q = 0; q < PAS_GAS_MAX_RES; ++q) {
    int64_t v = 0;
    if (q < n_res && ((g.mask >> q) & 1u)) {
      v = req[(int64_t)i * n_res + q];
      if (ni > 1) v /= ni;
    }
    g.req[q] = v;
  }
  g.pad[0] = g.pad[1] = 0;
  out[i] = g;
}

template <int Q>
__global__ __launch_bounds__(kTpb) void gas_fit_kernel(
    int32_t N, int32_t K, const int32_t* __restrict__ n_cards, const int64_t* __restrict__ cap,
    const int64_t* __restrict__ used, int32_t n_pods, int32_t pods_per_block, int32_t C, int32_t max_containers,
    const GasContainer* __restrict__ table, const int32_t* __restrict__ n_containers,
    uint32_t* __restrict__ res) {
  const int32_t n = blockIdx.x * kTpb + threadIdx.x;
  const bool valid = n < N;
  const int32_t nc = valid ? n_cards[n] : 0;
  int64_t cap_r[Q];
  int64_t snap[kMaxCards][Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) cap_r[q] = valid ? cap[(int64_t)n * Q + q] : 0;
#pragma unroll
  for (int k = 0; k < kMaxCards; ++k)
#pragma unroll
    for (int q = 0; q < Q; ++q)
      snap[k][q] = (valid && k < K) ? used[((int64_t)n * K + k) * Q + q] : 0;

  const int32_t p0 = blockIdx.y * pods_per_block;
  const int32_t p1 = min(n_pods, p0 + pods_per_block);
  for (int32_t p = p0; p < p1; ++p) {
    // FetchNode error / missing cards label -> errWontFit before any container
    // (scheduler.go:282-298).
    bool fits = nc > 0;
    uint32_t word = 0;
    int32_t nsel = 0;
    int64_t u[kMaxCards][Q];
#pragma unroll
    for (int k = 0; k < kMaxCards; ++k)
#pragma unroll
      for (int q = 0; q < Q; ++q) u[k][q] = snap[k][q];
    const int32_t ncont = min(n_containers[p], max_containers);
    for (int32_t c = 0; c < ncont; ++c) {
      const GasContainer& g = table[(int64_t)p * C + c];
      const uint32_t mask = g.mask;
      const int32_t ni = g.num_i915;
      if (mask == 0u || ni == 0) continue;  // no GPU request / zero gpuNum iterations
      uint64_t slack[Q];
      bool placeable = true;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if ((mask >> q) & 1u) {
          const int64_t need = g.req[q];
          if (need < 0 || cap_r[q] <= 0) placeable = false;
          const int64_t s = (int64_t)((uint64_t)cap_r[q] - (uint64_t)need);
          if (s < 0) placeable = false;
          slack[q] = (uint64_t)s;
        } else {
          slack[q] = ~0ull;
        }
      }
      if (!placeable) fits = false;
      for (int32_t step = 0; step < ni; ++step) {
        int chosen = -1;
#pragma unroll
        for (int k = kMaxCards - 1; k >= 0; --k) {  // first fit = lowest k
          bool ok = k < nc;
#pragma unroll
          for (int q = 0; q < Q; ++q) ok = ok && ((uint64_t)u[k][q] <= slack[q]);
          if (ok) chosen = k;
        }
        if (chosen < 0) fits = false;
#pragma unroll
        for (int k = 0; k < kMaxCards; ++k)
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (chosen == k) u[k][q] += g.req[q];
        word |= (uint32_t)(chosen & 7) << (3 * nsel);
        ++nsel;
      }
    }
    if (valid)
      res[(int64_t)p * N + n] = fits ? (0x80000000u | ((uint32_t)nsel << 24) | word) : 0u;
  }
}

}  // namespace

int gas_fit_launch(pas_ctx* ctx, int32_t n_pods, int32_t max_containers, int32_t i915_index,
                   const int64_t* d_req, const uint32_t* d_req_mask,
                   const int32_t* d_n_containers, uint32_t* d_res, hipStream_t s) {
  const GasSnapshot& g = ctx->gas;
  const int32_t N = g.n_nodes, Q = g.n_res, K = g.max_cards;
  if (N == 0 || n_pods == 0) return PAS_OK;
  const int32_t C = std::max(max_containers, 1);
  const size_t table_bytes = sizeof(GasContainer) * (size_t)n_pods * C;
  if (table_bytes > ctx->aux_bytes) {
    if (ctx->aux) {
      PAS_HIP(ctx, hipStreamSynchronize(s));
      PAS_HIP(ctx, hipFree(ctx->aux));
      ctx->aux = nullptr;
      ctx->aux_bytes = 0;
    }
    PAS_HIP(ctx, hipMalloc(&ctx->aux, table_bytes));
    ctx->aux_bytes = table_bytes;
  }
  GasContainer* table = static_cast<GasContainer*>(ctx->aux);
  TimedLaunch tl;
  const int32_t n_entries = n_pods * max_containers;
  if (n_entries > 0) {
    timing_begin(ctx, s, PAS_K_GAS_PREP, &tl);
    gas_prep_kernel<<<(n_entries + kTpb - 1) / kTpb, kTpb, 0, s>>>(n_entries, Q, i915_index,
                                                                  d_req, d_req_mask, table);
    timing_end(ctx, s, &tl);
    PAS_HIP(ctx, hipGetLastError());
  }
  const int32_t node_blocks = (N + kTpb - 1) / kTpb;
  const int32_t target_blocks = 4096;
  int32_t chunks = std::max(1, std::min(n_pods, (target_blocks + node_blocks - 1) / node_blocks));
  const int32_t ppb = (n_pods + chunks - 1) / chunks;
  chunks = (n_pods + ppb - 1) / ppb;
  const dim3 grid((unsigned)node_blocks, (unsigned)chunks);
  timing_begin(ctx, s, PAS_K_GAS_FIT, &tl);
  switch (Q) {
    case 1: gas_fit_kernel<1><<<grid, kTpb, 0, s>>>(N, K, g.n_cards, g.cap, g.used, n_pods, ppb, C, max_containers, table, d_n_containers, d_res); break;
    case 2: gas_fit_kernel<2><<<grid, kTpb, 0, s>>>(N, K, g.n_cards, g.cap, g.used, n_pods, ppb, C, max_containers, table, d_n_containers, d_res); break;
    case 3: gas_fit_kernel<3><<<grid, kTpb, 0, s>>>(N, K, g.n_cards, g.cap, g.used, n_pods, ppb, C, max_containers, table, d_n_containers, d_res); break;
    default: gas_fit_kernel<4><<<grid, kTpb, 0, s>>>(N, K, g.n_cards, g.cap, g.used, n_pods, ppb, C, max_containers, table, d_n_containers, d_res); break;
  }
  timing_end(ctx, s, &tl);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

}  // namespace pas
