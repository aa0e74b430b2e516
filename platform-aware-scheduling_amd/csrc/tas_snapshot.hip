// tas_snapshot.hip — device-side build of the resident TAS snapshot.
//
// The reference re-derives node order per request: core.OrderedList ranges over the
// metric's map and sort.Slice-s it with Quantity.Cmp on every prioritize call
// (telemetry-aware-scheduling/pkg/strategies/core/operator.go:30-42), and every
// dontschedule rule scans the whole metric map (dontschedule/strategy.go:33-41).
// Here the snapshot (one AutoUpdatingCache refresh, cache/autoupdating.go:37-59) is
// sorted once per metric into three orders — ascending, descending, node index.  A
// rule's violating set is then a contiguous range of the ascending order, and a pod's
// prioritize list is a compaction of one order by the pod's pass bits.
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
// perm[2][m][pos] = n, vals_c[m][pos] = vals[m][n].
__global__ void compact_present(const uint64_t* __restrict__ present,
                                const int64_t* __restrict__ vals,
                                const uint32_t* __restrict__ scan, int32_t N, int32_t R,
                                int32_t M, int64_t W, int32_t* __restrict__ perm_index,
                                int64_t* __restrict__ vals_c) {
  const int64_t i = (int64_t)blockIdx.x * kTpb + threadIdx.x;
  if (i >= (int64_t)M * W) return;
  const int64_t m = i / W, w = i % W;
  uint64_t bits = present[i];
  const int64_t lo = w * 64;
  if (lo + 64 > N) bits &= (N - lo) >= 64 ? ~0ull : ((1ull << (N - lo)) - 1);
  uint32_t pos = scan[i] - scan[m * W];
  const int64_t row = m * (int64_t)R;
  const int64_t col = m * (int64_t)N;
  while (bits) {
    const int b = __ffsll((unsigned long long)bits) - 1;
    bits &= bits - 1;
    const int32_t n = (int32_t)(lo + b);
    perm_index[row + pos] = n;
    vals_c[row + pos] = vals[col + n];
    ++pos;
  }
}

__global__ void segment_bounds(const uint32_t* __restrict__ scan, int32_t R, int32_t M,
                               int64_t W, int32_t* __restrict__ cnt,
                               int32_t* __restrict__ seg_begin, int32_t* __restrict__ seg_end) {
  const int m = blockIdx.x * kTpb + threadIdx.x;
  if (m >= M) return;
  const int32_t c = (int32_t)(scan[(m + 1) * W] - scan[m * W]);
  cnt[m] = c;
  seg_begin[m] = m * R;
  seg_end[m] = m * R + c;
}

// f32[m][b] = sorted[m][32 b], and f1k[m][a] = sorted[m][1024 a], for positions < cnt[m]
__global__ void build_fences(const int64_t* __restrict__ sorted, const int32_t* __restrict__ cnt,
                             int32_t R, int32_t M, int64_t* __restrict__ f1k,
                             int64_t* __restrict__ f32) {
  const int32_t nb = R >> 5;
  const int64_t i = (int64_t)blockIdx.x * kTpb + threadIdx.x;
  if (i >= (int64_t)M * nb) return;
  const int32_t m = (int32_t)(i / nb), b = (int32_t)(i % nb);
  const int64_t v = b * 32 < cnt[m] ? sorted[(int64_t)m * R + b * 32] : 0;
  f32[i] = v;
  if ((b & 31) == 0) f1k[(int64_t)m * (R >> 10) + (b >> 5)] = v;
}

}  // namespace

int tas_snapshot_build(pas_ctx* ctx, uint64_t gen, int32_t N, int32_t M,
                       const int64_t* d_vals, const uint64_t* d_present, hipStream_t s) {
  TasSnapshot& t = ctx->tas;
  t.valid = false;
  const int64_t W = w64(N);
  const int64_t MN = (int64_t)M * N;
  const int32_t R = (int32_t)order_row(N);
  const int64_t MR = (int64_t)M * R;
  if (MR * kNumOrders > 0x7fffffffLL)
    return set_error(ctx, PAS_ECAPACITY,
                     "TAS snapshot: 3 * n_metrics * padded n_nodes must be < 2^31");
  if (t.n_nodes != N || t.n_metrics != M || !t.cnt) {
    PAS_HIP(ctx, hipStreamSynchronize(s));
    free_tas(ctx);
    const size_t mn = (size_t)std::max<int64_t>(MN, 1);
    const size_t mr = (size_t)std::max<int64_t>(MR, 1);
    const size_t mw = (size_t)std::max<int64_t>((int64_t)M * W, 1);
    const size_t mm = (size_t)std::max(M, 1);
    PAS_HIP(ctx, hipMalloc(&t.vals, sizeof(int64_t) * mn));
    PAS_HIP(ctx, hipMalloc(&t.present, sizeof(uint64_t) * mw));
    PAS_HIP(ctx, hipMalloc(&t.cnt, sizeof(int32_t) * mm));
    // sorted doubles as the popcount scratch of the build (mr >= mw + 1)
    PAS_HIP(ctx, hipMalloc(&t.sorted, sizeof(int64_t) * mr));
    PAS_HIP(ctx, hipMalloc(&t.perm, sizeof(int32_t) * mr * kNumOrders));
    PAS_HIP(ctx, hipMalloc(&t.vals_c, sizeof(int64_t) * mr));
    PAS_HIP(ctx, hipMalloc(&t.f1k, sizeof(int64_t) * (mr / 1024 + 1)));
    PAS_HIP(ctx, hipMalloc(&t.f32, sizeof(int64_t) * (mr / 32 + 1)));
    PAS_HIP(ctx, hipMalloc(&t.word_scan, sizeof(uint32_t) * (mw + 1)));
    PAS_HIP(ctx, hipMalloc(&t.seg_begin, sizeof(int32_t) * mm));
    PAS_HIP(ctx, hipMalloc(&t.seg_end, sizeof(int32_t) * mm));
    // temp storage for the sorts (the descending form needs the same or less)
    size_t sort_bytes = 0, sort_bytes_desc = 0, scan_bytes = 0;
    PAS_HIP(ctx, rocprim::segmented_radix_sort_pairs(
                     nullptr, sort_bytes, t.vals_c, t.sorted, t.perm, t.perm, (unsigned)MR,
                     (unsigned)M, t.seg_begin, t.seg_end, 0, 64, s));
    PAS_HIP(ctx, rocprim::segmented_radix_sort_pairs_desc(
                     nullptr, sort_bytes_desc, t.vals_c, t.sorted, t.perm, t.perm, (unsigned)MR,
                     (unsigned)M, t.seg_begin, t.seg_end, 0, 64, s));
    PAS_HIP(ctx, rocprim::exclusive_scan(nullptr, scan_bytes, t.word_scan, t.word_scan,
                                         0u, (size_t)(mw + 1), rocprim::plus<uint32_t>(), s));
    t.sort_tmp_bytes = std::max<size_t>(std::max(sort_bytes, sort_bytes_desc), 16);
    t.scan_tmp_bytes = std::max<size_t>(scan_bytes, 16);
    PAS_HIP(ctx, hipMalloc(&t.sort_tmp, t.sort_tmp_bytes));
    PAS_HIP(ctx, hipMalloc(&t.scan_tmp, t.scan_tmp_bytes));
    t.n_nodes = N;
    t.n_metrics = M;
    t.row = R;
  }
  if (MN > 0) {
    if (d_vals != t.vals)
      PAS_HIP(ctx, hipMemcpyAsync(t.vals, d_vals, sizeof(int64_t) * MN,
                                  hipMemcpyDeviceToDevice, s));
    if (d_present != t.present)
      PAS_HIP(ctx, hipMemcpyAsync(t.present, d_present, sizeof(uint64_t) * M * W,
                                  hipMemcpyDeviceToDevice, s));
    const int64_t mw = (int64_t)M * W;
    uint32_t* popc = reinterpret_cast<uint32_t*>(t.sorted);
    popc_words<<<(unsigned)((mw + 1 + kTpb - 1) / kTpb), kTpb, 0, s>>>(t.present, mw, N, W,
                                                                         popc);
    PAS_HIP(ctx, hipGetLastError());
    size_t scan_bytes = t.scan_tmp_bytes;
    PAS_HIP(ctx, rocprim::exclusive_scan(t.scan_tmp, scan_bytes, popc, t.word_scan, 0u,
                                         (size_t)(mw + 1), rocprim::plus<uint32_t>(), s));
    // every order position past cnt[m] holds the sentinel (the sorts write [0, cnt) only)
    PAS_HIP(ctx, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(t.perm), (int)(W * 64),
                                   (size_t)MR * kNumOrders, s));
    int32_t* perm_asc = t.perm + (size_t)kOrderAsc * MR;
    int32_t* perm_desc = t.perm + (size_t)kOrderDesc * MR;
    int32_t* perm_index = t.perm + (size_t)kOrderIndex * MR;
    compact_present<<<(unsigned)((mw + kTpb - 1) / kTpb), kTpb, 0, s>>>(
        t.present, t.vals, t.word_scan, N, R, M, W, perm_index, t.vals_c);
    PAS_HIP(ctx, hipGetLastError());
    segment_bounds<<<(M + kTpb - 1) / kTpb, kTpb, 0, s>>>(t.word_scan, R, M, W, t.cnt,
                                                        t.seg_begin, t.seg_end);
    PAS_HIP(ctx, hipGetLastError());
    size_t sort_bytes = t.sort_tmp_bytes;
    // descending first (its key output lands in `sorted` and is then overwritten)
    PAS_HIP(ctx, rocprim::segmented_radix_sort_pairs_desc(
                     t.sort_tmp, sort_bytes, t.vals_c, t.sorted, perm_index, perm_desc,
                     (unsigned)MR, (unsigned)M, t.seg_begin, t.seg_end, 0, 64, s));
    sort_bytes = t.sort_tmp_bytes;
    PAS_HIP(ctx, rocprim::segmented_radix_sort_pairs(
                     t.sort_tmp, sort_bytes, t.vals_c, t.sorted, perm_index, perm_asc,
                     (unsigned)MR, (unsigned)M, t.seg_begin, t.seg_end, 0, 64, s));
    build_fences<<<(unsigned)((MR / 32 + kTpb - 1) / kTpb), kTpb, 0, s>>>(t.sorted, t.cnt, R, M,
                                                                          t.f1k, t.f32);
    PAS_HIP(ctx, hipGetLastError());
  }
  t.gen = gen;
  t.valid = true;
  return PAS_OK;
}

}  // namespace pas
