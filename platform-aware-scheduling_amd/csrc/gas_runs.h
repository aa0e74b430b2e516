// gas_runs.h — one container's card selections as runs on ascending cards (device helpers).
//
// getCardsForContainerGPURequest (gpu-aware-scheduling/pkg/gpuscheduler/scheduler.go:200-257)
// picks numI915 times the first card, in sort.Strings order, that passes
// checkResourceCapacity (:341-383) on the usage with the container's earlier takes, and adds
// the per-GPU request there (addRM).  Every selection of a container carries the same request
// and a card only loses free capacity by being taken, so a card the scan has passed never
// fits again within the container: the selections are runs on ascending cards, card k taking
// min(remaining, T_k), T_k = the takes its free capacity allows.  That is O(cards) per
// container for any numI915 — the reference puts no bound on it (the GPU plugin's
// -shared-dev-num lets one card take hundreds of selections) — where the literal loop is
// O(numI915 · cards).  The kernels keep the literal loop up to PAS_GAS_MAX_SELECTIONS
// selections per container and use the runs past it; the oracle keeps the literal loop
// everywhere, so the parity tests check the two against each other.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pas.h"

namespace pas {

// Containers with more selections than this go through container_runs.
constexpr int64_t kRunsFrom = PAS_GAS_MAX_SELECTIONS;

// Takes of per-GPU request r (kinds: mask bits) that a card with usage w admits under the
// per-GPU capacity cap: take t + 1 passes checkResourceCapacity iff every requested kind has
// r >= 0, cap > 0, w + t·r >= 0 without overflow and w + t·r <= cap (free-capacity form).  A
// request of a kind outside the snapshot has no capacity key (:349-354): no take.
template <int QW = PAS_GAS_MAX_RES>
__device__ __forceinline__ int64_t card_takes(int32_t Q, uint32_t m, const int64_t* r,
                                              const int64_t* cap, const int64_t* w) {
  if (m & PAS_REQ_UNKNOWN_KIND) return 0;
  int64_t t = INT64_MAX;
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    if (q >= Q || !((m >> q) & 1u)) continue;
    if (r[q] < 0 || cap[q] <= 0 || w[q] < 0 || w[q] > cap[q]) return 0;
    if (r[q] > 0) t = min(t, (cap[q] - w[q]) / r[q]);
  }
  return t;
}

// The container's num selections as runs over cards 0 .. ncard-1 (w: the working copy
// [card][kind], updated); emit(card, takes) per run.  False = a selection fits no card
// (errWontFit, :249-253).  num >= 1.
template <int KMAX, int QW = PAS_GAS_MAX_RES, class Emit>
__device__ bool container_runs(int32_t Q, uint32_t m, const int64_t* r, int64_t num,
                               const int64_t* cap, int64_t (&w)[KMAX][QW],
                               int32_t ncard, Emit emit) {
  // unrolled for register-resident copies (KMAX <= 16), so w is never indexed dynamically
  constexpr int kUnroll = KMAX <= 16 ? KMAX : 1;
  int64_t rem = num;
#pragma unroll kUnroll
  for (int k = 0; k < KMAX; ++k) {
    if (k < ncard && rem > 0) {
      const int64_t t = min(rem, card_takes<QW>(Q, m, r, cap, w[k]));
      if (t > 0) {
        // t·r[q] <= cap[q] - w[q]: no overflow
#pragma unroll
        for (int q = 0; q < QW; ++q)
          if (q < Q && ((m >> q) & 1u)) w[k][q] += t * r[q];
        rem -= t;
        emit(k, t);
      }
    }
  }
  return rem == 0;
}

// subtractRM of amount r, t times, from a usage value (resource_map.go:103-127): Go's int64
// subtraction wraps, a negative result is set to zero.  After the first subtraction the value
// is >= 0 and r >= 0, so the rest cannot wrap: max(0, v - (t-1)·r).
__device__ __forceinline__ int64_t subtract_times(int64_t w, int64_t r, int64_t t) {
  if (t <= 0) return w;
  int64_t v = (int64_t)((uint64_t)w - (uint64_t)r);
  v = v < 0 ? 0 : v;
  const int64_t rest = t - 1;
  if (rest == 0 || r == 0) return v;
  return rest > v / r ? 0 : v - rest * r;
}

}  // namespace pas
