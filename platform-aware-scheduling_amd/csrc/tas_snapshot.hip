// tas_snapshot.hip — device-side build of the resident TAS snapshot.
//
// The reference re-derives node order per request: core.OrderedList ranges over the
// metric's map and sort.Slice-s it with Quantity.Cmp on every prioritize call
// (telemetry-aware-scheduling/pkg/strategies/core/operator.go:30-42), and every
// dontschedule rule scans the whole metric map (dontschedule/strategy.go:33-41).
// Here the snapshot (one AutoUpdatingCache refresh, cache/autoupdating.go:37-59) is
// sorted once per metric into three orders — ascending, descending, node index — each
// with its inverse (rank).  A rule's violating set is then a contiguous range of the
// ascending order, and a pod's prioritize list is a compaction of one order.
//
// Ties: rocPRIM's segmented radix sorts are stable in both directions, and the input
// is in node-index order, so equal values stay in ascending node index (the
// documented tie-break; the reference's is unspecified Go-map order).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;

// popc[i] = number of present nodes in bitmap word i (words beyond M*W are 0).
__global__ void popc_words(const uint64_t* __restrict__ present, int64_t total_words,
                           int32_t N, int64_t W, uint32_t* __restrict__ popc) {
  const int64_t i = (int64_t)blockIdx.x * kTpb + threadIdx.x;
  if (i > total_words) return;
  uint32_t c = 0;
  if (i < total_words) {
    uint64_t bits = present[i];
    const int64_t w = i % W;
    const int64_t lo = w * 64;
    if (lo + 64 > N) bits &= (N - lo) >= 64 ? ~0ull : ((1ull << (N - lo)) - 1);
    c = (uint32_t)__popcll(bits);
  }
  popc[i] = c;
}

// Compact the present nodes of each metric in node-index order (order kOrderIndex):
// perm[2][m][pos] = n, rank[2][m][n] = pos, vals_c[m][pos] = vals[m][n].
__global__ void compact_present(const uint64_t* __restrict__ present,
                                const int64_t* __restrict__ vals,
                                const uint32_t* __restrict__ scan, int32_t N, int32_t Nr,
                                int32_t M, int64_t W, int32_t* __restrict__ perm_index,
                                uint32_t* __restrict__ rank_index,
                                int64_t* __restrict__ vals_c) {
  const int64_t i = (int64_t)blockIdx.x * kTpb + threadIdx.x;
  if (i >= (int64_t)M * W) return;
  const int64_t m = i / W, w = i % W;
  uint64_t bits = present[i];
  const int64_t lo = w * 64;
  if (lo + 64 > N) bits &= (N - lo) >= 64 ? ~0ull : ((1ull << (N - lo)) - 1);
  uint32_t pos = scan[i] - scan[m * W];
  const int64_t col = m * (int64_t)N;
  while (bits) {
    const int b = __ffsll((unsigned long long)bits) - 1;
    bits &= bits - 1;
    const int32_t n = (int32_t)(lo + b);
    perm_index[col + pos] = n;
    rank_index[m * (int64_t)Nr + n] = pos;
    vals_c[col + pos] = vals[col + n];
    ++pos;
  }
}

__global__ void segment_bounds(const uint32_t* __restrict__ scan, int32_t N, int32_t M,
                               int64_t W, int32_t* __restrict__ cnt,
                               int32_t* __restrict__ seg_begin, int32_t* __restrict__ seg_end) {
  const int m = blockIdx.x * kTpb + threadIdx.x;
  if (m >= M) return;
  const int32_t c = (int32_t)(scan[(m + 1) * W] - scan[m * W]);
  cnt[m] = c;
  seg_begin[m] = m * N;
  seg_end[m] = m * N + c;
}

// rank[o][m][perm[o][m][k]] = k for k < cnt[m]
__global__ void invert_order(const int32_t* __restrict__ perm, const int32_t* __restrict__ cnt,
                             int32_t N, int32_t Nr, uint32_t* __restrict__ rank) {
  const int m = blockIdx.y;
  const int32_t k = blockIdx.x * kTpb + threadIdx.x;
  if (k >= cnt[m]) return;
  rank[(int64_t)m * Nr + perm[(int64_t)m * N + k]] = (uint32_t)k;
}

// phi[ocol][m][k] = rank[ocol][perm_asc[m][k]] for k < cnt[m].  Blocks run ocol-major
// (grid z), so one rank row serves all M metrics from L2 while it is hot.
__global__ void compose_orders(const int32_t* __restrict__ perm_asc,
                               const uint32_t* __restrict__ rank,
                               const int32_t* __restrict__ cnt, int32_t N, int32_t Nr,
                               int32_t M, int32_t* __restrict__ phi) {
  const int32_t m = blockIdx.y;
  const int32_t ocol = blockIdx.z;
  const int32_t k = blockIdx.x * kTpb + threadIdx.x;
  if (k >= cnt[m]) return;
  const int32_t n = perm_asc[(int64_t)m * N + k];
  phi[((int64_t)ocol * M + m) * N + k] = (int32_t)rank[(int64_t)ocol * Nr + n];
}

}  // namespace

// The composed-order index, when it fits the context's budget (pas.h,
// pas_tas_set_index_budget); otherwise none (the evaluation then uses the rank arrays).
static int build_phi(pas_ctx* ctx, int32_t N, int32_t M, hipStream_t s) {
  TasSnapshot& t = ctx->tas;
  const size_t need = sizeof(int32_t) * 3 * (size_t)M * (size_t)M * (size_t)N;
  size_t cap = 0;
  if (ctx->tas_index_budget >= 0) {
    cap = (size_t)ctx->tas_index_budget;
  } else {
    size_t free_b = 0, total_b = 0;
    PAS_HIP(ctx, hipMemGetInfo(&free_b, &total_b));
    cap = (free_b + (t.phi ? t.phi_bytes : 0)) / 4;
  }
  if (need == 0 || need > cap) {
    if (t.phi) {
      PAS_HIP(ctx, hipStreamSynchronize(s));
      PAS_HIP(ctx, hipFree(t.phi));
    }
    t.phi = nullptr;
    t.phi_bytes = 0;
    return PAS_OK;
  }
  if (!t.phi || t.phi_bytes != need) {
    if (t.phi) {
      PAS_HIP(ctx, hipStreamSynchronize(s));
      PAS_HIP(ctx, hipFree(t.phi));
      t.phi = nullptr;
    }
    PAS_HIP(ctx, hipMalloc(&t.phi, need));
    t.phi_bytes = need;
  }
  const dim3 grid((unsigned)((N + kTpb - 1) / kTpb), (unsigned)M, (unsigned)(3 * M));
  compose_orders<<<grid, kTpb, 0, s>>>(t.perm + (size_t)kOrderAsc * M * N, t.rank, t.cnt, N,
                                       t.rank_stride, M, t.phi);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

int tas_snapshot_build(pas_ctx* ctx, uint64_t gen, int32_t N, int32_t M,
                       const int64_t* d_vals, const uint64_t* d_present, hipStream_t s) {
  TasSnapshot& t = ctx->tas;
  t.valid = false;
  const int64_t W = w64(N);
  const int64_t MN = (int64_t)M * N;
  const int32_t Nr = (int32_t)rank_row(N);
  const int64_t MNr = (int64_t)M * Nr;
  if (MNr > 0x7fffffffLL)
    return set_error(ctx, PAS_ECAPACITY, "TAS snapshot: n_metrics * n_nodes must be < 2^31");
  if (t.n_nodes != N || t.n_metrics != M || !t.cnt) {
    PAS_HIP(ctx, hipStreamSynchronize(s));
    free_tas(ctx);
    const size_t mn = (size_t)std::max<int64_t>(MN, 1);
    const size_t mw = (size_t)std::max<int64_t>((int64_t)M * W, 1);
    const size_t mm = (size_t)std::max(M, 1);
    PAS_HIP(ctx, hipMalloc(&t.vals, sizeof(int64_t) * mn));
    PAS_HIP(ctx, hipMalloc(&t.present, sizeof(uint64_t) * mw));
    PAS_HIP(ctx, hipMalloc(&t.cnt, sizeof(int32_t) * mm));
    PAS_HIP(ctx, hipMalloc(&t.sorted, sizeof(int64_t) * mn));
    // +1024 entries: the emit loader reads whole 1024-position segments unconditionally
    PAS_HIP(ctx, hipMalloc(&t.perm, sizeof(int32_t) * (mn * kNumOrders + 1024)));
    PAS_HIP(ctx, hipMalloc(&t.rank,
                           sizeof(uint32_t) * (size_t)std::max<int64_t>(MNr, 1) * kNumOrders));
    PAS_HIP(ctx, hipMalloc(&t.vals_c, sizeof(int64_t) * mn));
    PAS_HIP(ctx, hipMalloc(&t.word_scan, sizeof(uint32_t) * (mw + 1)));
    PAS_HIP(ctx, hipMalloc(&t.seg_begin, sizeof(int32_t) * mm));
    PAS_HIP(ctx, hipMalloc(&t.seg_end, sizeof(int32_t) * mm));
    // temp storage for the sorts (the descending form needs the same or less)
    size_t sort_bytes = 0, sort_bytes_desc = 0, scan_bytes = 0;
    PAS_HIP(ctx, rocprim::segmented_radix_sort_pairs(
                     nullptr, sort_bytes, t.vals_c, t.sorted, t.perm, t.perm, (unsigned)MN,
                     (unsigned)M, t.seg_begin, t.seg_end, 0, 64, s));
    PAS_HIP(ctx, rocprim::segmented_radix_sort_pairs_desc(
                     nullptr, sort_bytes_desc, t.vals_c, t.sorted, t.perm, t.perm, (unsigned)MN,
                     (unsigned)M, t.seg_begin, t.seg_end, 0, 64, s));
    PAS_HIP(ctx, rocprim::exclusive_scan(nullptr, scan_bytes, t.word_scan, t.word_scan,
                                         0u, (size_t)(mw + 1), rocprim::plus<uint32_t>(), s));
    t.sort_tmp_bytes = std::max<size_t>(std::max(sort_bytes, sort_bytes_desc), 16);
    t.scan_tmp_bytes = std::max<size_t>(scan_bytes, 16);
    PAS_HIP(ctx, hipMalloc(&t.sort_tmp, t.sort_tmp_bytes));
    PAS_HIP(ctx, hipMalloc(&t.scan_tmp, t.scan_tmp_bytes));
    t.n_nodes = N;
    t.n_metrics = M;
    t.rank_stride = Nr;
  }
  if (MN > 0) {
    if (d_vals != t.vals)
      PAS_HIP(ctx, hipMemcpyAsync(t.vals, d_vals, sizeof(int64_t) * MN,
                                  hipMemcpyDeviceToDevice, s));
    if (d_present != t.present)
      PAS_HIP(ctx, hipMemcpyAsync(t.present, d_present, sizeof(uint64_t) * M * W,
                                  hipMemcpyDeviceToDevice, s));
    const int64_t mw = (int64_t)M * W;
    // popcounts into rank (scratch at this point; MNr >= M*W + 1), then scan into word_scan
    uint32_t* popc = t.rank;
    popc_words<<<(unsigned)((mw + 1 + kTpb - 1) / kTpb), kTpb, 0, s>>>(t.present, mw, N, W,
                                                                         popc);
    PAS_HIP(ctx, hipGetLastError());
    size_t scan_bytes = t.scan_tmp_bytes;
    PAS_HIP(ctx, rocprim::exclusive_scan(t.scan_tmp, scan_bytes, popc, t.word_scan, 0u,
                                         (size_t)(mw + 1), rocprim::plus<uint32_t>(), s));
    PAS_HIP(ctx, hipMemsetAsync(t.rank, 0xFF, sizeof(uint32_t) * MNr * kNumOrders, s));
    int32_t* perm_asc = t.perm + (size_t)kOrderAsc * MN;
    int32_t* perm_desc = t.perm + (size_t)kOrderDesc * MN;
    int32_t* perm_index = t.perm + (size_t)kOrderIndex * MN;
    compact_present<<<(unsigned)((mw + kTpb - 1) / kTpb), kTpb, 0, s>>>(
        t.present, t.vals, t.word_scan, N, Nr, M, W, perm_index,
        t.rank + (size_t)kOrderIndex * MNr, t.vals_c);
    PAS_HIP(ctx, hipGetLastError());
    segment_bounds<<<(M + kTpb - 1) / kTpb, kTpb, 0, s>>>(t.word_scan, N, M, W, t.cnt,
                                                        t.seg_begin, t.seg_end);
    PAS_HIP(ctx, hipGetLastError());
    size_t sort_bytes = t.sort_tmp_bytes;
    // descending first (its key output lands in `sorted` and is then overwritten)
    PAS_HIP(ctx, rocprim::segmented_radix_sort_pairs_desc(
                     t.sort_tmp, sort_bytes, t.vals_c, t.sorted, perm_index, perm_desc,
                     (unsigned)MN, (unsigned)M, t.seg_begin, t.seg_end, 0, 64, s));
    sort_bytes = t.sort_tmp_bytes;
    PAS_HIP(ctx, rocprim::segmented_radix_sort_pairs(
                     t.sort_tmp, sort_bytes, t.vals_c, t.sorted, perm_index, perm_asc,
                     (unsigned)MN, (unsigned)M, t.seg_begin, t.seg_end, 0, 64, s));
    const dim3 grid((unsigned)((N + kTpb - 1) / kTpb), (unsigned)M);
    invert_order<<<grid, kTpb, 0, s>>>(perm_asc, t.cnt, N, Nr, t.rank + (size_t)kOrderAsc * MNr);
    PAS_HIP(ctx, hipGetLastError());
    invert_order<<<grid, kTpb, 0, s>>>(perm_desc, t.cnt, N, Nr,
                                        t.rank + (size_t)kOrderDesc * MNr);
    PAS_HIP(ctx, hipGetLastError());
    if (int rc = build_phi(ctx, N, M, s)) return rc;
  }
  t.gen = gen;
  t.valid = true;
  return PAS_OK;
}

}  // namespace pas
