// tas_snapshot.hip — device-side build of the resident TAS snapshot, whole or per column.
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
// The cache refreshes one metric at a time (updateAllMetrics -> updateMetric ->
// WriteMetric replaces the metric's whole node map, autoupdating.go:45-73), so a column is
// the unit of update: tas_snapshot_update rebuilds the orders of the given columns only.
//
// Build of C columns (all M for a full upload):
//   1. per-word popcounts of the columns' presence bitmaps and their exclusive scan;
//   2. compaction, one thread per order position j of a column: a present node j goes to
//      its rank among the column's present nodes (coalesced: consecutive present nodes,
//      consecutive positions), positions past cnt get a pad;
//   3. one device-wide stable radix sort of keys {value, column} with node ids as values
//      (C*R pairs: every column occupies exactly R sorted positions, pads last), then the
//      same with {~value, column} for the descending order.  The keyed device-wide sort
//      fills the GPU, where a segmented sort runs one workgroup per column;
//   4. placement into the snapshot rows, with the range-search fences.
// Ties: the sorts are stable and the compacted input is in node-index order, so equal
// values stay in ascending node index in both orders (the documented tie-break; the
// reference's is unspecified Go-map order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "pas_internal.h"

namespace pas {
namespace {

constexpr int kTpb = 256;

// Sort key: the column's value (or ~value for the descending order) below the column
// index; pads carry INT64_MAX and follow every value of their column (stable sort, pads
// after the column's present nodes in the input).
struct SortKey {
  int64_t v;
  uint32_t c;
  uint32_t pad;
};
struct SortKeyBits {
  __host__ __device__ rocprim::tuple<uint32_t&, int64_t&> operator()(SortKey& k) const {
    return rocprim::tuple<uint32_t&, int64_t&>(k.c, k.v);
  }
};

__device__ __forceinline__ int32_t row_of(const int32_t* rows, int32_t c) {
  return rows ? rows[c] : c;
}

__device__ __forceinline__ uint64_t word_mask(uint64_t bits, int64_t w, int32_t N) {
  const int64_t lo = w * 64;
  return lo + 64 > N ? bits & ((N - lo) >= 64 ? ~0ull : ((1ull << (N - lo)) - 1)) : bits;
}

// popc[c*W + w] = present nodes in word w of column c; the last entry (c*W == C*W) is 0 so
// the exclusive scan yields every column's end.
__global__ void popc_words(const uint64_t* __restrict__ present, int64_t total_words,
                           int32_t N, int64_t W, uint32_t* __restrict__ popc) {
  const int64_t i = (int64_t)blockIdx.x * kTpb + threadIdx.x;
  if (i > total_words) return;
  popc[i] = i < total_words ? (uint32_t)__popcll(word_mask(present[i], i % W, N)) : 0u;
}

// One thread per (column c, order position j < R).
__global__ void compact_keys(const uint64_t* __restrict__ present,
                             const int64_t* __restrict__ vals, const uint32_t* __restrict__ scan,
                             const int32_t* __restrict__ rows, int32_t C, int32_t N, int32_t R,
                             int64_t W, int32_t MR, SortKey* __restrict__ keys,
                             int32_t* __restrict__ ids, int32_t* __restrict__ perm_index) {
  const int64_t i = (int64_t)blockIdx.x * kTpb + threadIdx.x;
  if (i >= (int64_t)C * R) return;
  const int32_t c = (int32_t)(i / R), j = (int32_t)(i % R);
  const int64_t m = row_of(rows, c);
  const uint32_t base = scan[(int64_t)c * W];
  const int32_t cnt = (int32_t)(scan[(int64_t)(c + 1) * W] - base);
  const int32_t sentinel = (int32_t)(W * 64);
  const int64_t out = (int64_t)c * R;
  if (j < N) {
    const int64_t w = j >> 6;
    const uint64_t bits = word_mask(present[(int64_t)c * W + w], w, N);
    if ((bits >> (j & 63)) & 1ull) {
      const int32_t pos = (int32_t)(scan[(int64_t)c * W + w] - base) +
                          __popcll(bits & ((1ull << (j & 63)) - 1ull));
      keys[out + pos] = SortKey{vals[(int64_t)c * N + j], (uint32_t)c, 0u};
      ids[out + pos] = j;
      perm_index[(int64_t)kOrderIndex * MR + m * R + pos] = j;
    }
  }
  if (j >= cnt) {
    keys[out + j] = SortKey{INT64_MAX, (uint32_t)c, 0u};
    ids[out + j] = sentinel;
    perm_index[(int64_t)kOrderIndex * MR + m * R + j] = sentinel;
  }
}

// Ascending result -> sorted / perm_asc rows and the fences (f32[m][b] = sorted[32 b],
// f1k[m][a] = sorted[1024 a], 0 past cnt); the input keys become the descending keys.
__global__ void place_asc(const SortKey* __restrict__ skeys, const int32_t* __restrict__ sids,
                          SortKey* __restrict__ keys, const uint32_t* __restrict__ scan,
                          const int32_t* __restrict__ rows, int32_t C, int32_t R, int64_t W,
                          int32_t MR, int64_t* __restrict__ sorted, int32_t* __restrict__ perm,
                          int32_t* __restrict__ cnt_out, int64_t* __restrict__ f1k,
                          int64_t* __restrict__ f32) {
  const int64_t i = (int64_t)blockIdx.x * kTpb + threadIdx.x;
  if (i >= (int64_t)C * R) return;
  const int32_t c = (int32_t)(i / R), j = (int32_t)(i % R);
  const int64_t m = row_of(rows, c);
  const int32_t cnt = (int32_t)(scan[(int64_t)(c + 1) * W] - scan[(int64_t)c * W]);
  const int64_t v = skeys[i].v;
  sorted[m * R + j] = v;
  perm[(int64_t)kOrderAsc * MR + m * R + j] = sids[i];
  if ((j & 31) == 0) {
    const int64_t f = j < cnt ? v : 0;
    f32[m * (R >> 5) + (j >> 5)] = f;
    if ((j & 1023) == 0) f1k[m * (R >> 10) + (j >> 10)] = f;
  }
  if (j == 0) cnt_out[m] = cnt;
  if (j < cnt) keys[i].v = ~keys[i].v;  // v1 < v2 <=> ~v1 > ~v2 (no overflow)
}

__global__ void place_desc(const int32_t* __restrict__ sids, const int32_t* __restrict__ rows,
                           int32_t C, int32_t R, int32_t MR, int32_t* __restrict__ perm) {
  const int64_t i = (int64_t)blockIdx.x * kTpb + threadIdx.x;
  if (i >= (int64_t)C * R) return;
  const int32_t c = (int32_t)(i / R), j = (int32_t)(i % R);
  perm[(int64_t)kOrderDesc * MR + (int64_t)row_of(rows, c) * R + j] = sids[i];
}

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + kTpb - 1) / kTpb); }

inline unsigned bits_for(int32_t c) {  // bits of the column index in the sort key
  unsigned b = 1;
  while (b < 31 && (int64_t(1) << b) < c) ++b;
  return b;
}

// Orders of C columns whose values / presence sit at vals [C][N] / present [C][W]
// (rows: snapshot row of each column, nullptr = identity).
int build_columns(pas_ctx* ctx, int32_t C, const int32_t* d_rows, const int64_t* vals,
                  const uint64_t* present, hipStream_t s) {
  TasSnapshot& t = ctx->tas;
  const int32_t N = t.n_nodes, R = t.row;
  const int64_t W = w64(N);
  const int32_t MR = t.n_metrics * R;
  const int64_t cw = (int64_t)C * W;
  const int64_t cr = (int64_t)C * R;
  popc_words<<<blocks_for(cw + 1), kTpb, 0, s>>>(present, cw, N, W, t.popc);
  PAS_HIP(ctx, hipGetLastError());
  size_t scan_bytes = t.scan_tmp_bytes;
  PAS_HIP(ctx, rocprim::exclusive_scan(t.scan_tmp, scan_bytes, t.popc, t.word_scan, 0u,
                                       (size_t)(cw + 1), rocprim::plus<uint32_t>(), s));
  SortKey* ka = static_cast<SortKey*>(t.keys_a);
  SortKey* kb = static_cast<SortKey*>(t.keys_b);
  compact_keys<<<blocks_for(cr), kTpb, 0, s>>>(present, vals, t.word_scan, d_rows, C, N, R, W, MR,
                                              ka, t.ids_a, t.perm);
  PAS_HIP(ctx, hipGetLastError());
  const unsigned end_bit = 64 + bits_for(C);
  size_t sort_bytes = t.sort_tmp_bytes;
  PAS_HIP(ctx, rocprim::radix_sort_pairs(t.sort_tmp, sort_bytes, ka, kb, t.ids_a, t.ids_b,
                                         (size_t)cr, SortKeyBits{}, 0u, end_bit, s));
  place_asc<<<blocks_for(cr), kTpb, 0, s>>>(kb, t.ids_b, ka, t.word_scan, d_rows, C, R, W, MR,
                                           t.sorted, t.perm, t.cnt, t.f1k, t.f32);
  PAS_HIP(ctx, hipGetLastError());
  sort_bytes = t.sort_tmp_bytes;
  PAS_HIP(ctx, rocprim::radix_sort_pairs(t.sort_tmp, sort_bytes, ka, kb, t.ids_a, t.ids_b,
                                         (size_t)cr, SortKeyBits{}, 0u, end_bit, s));
  place_desc<<<blocks_for(cr), kTpb, 0, s>>>(t.ids_b, d_rows, C, R, MR, t.perm);
  PAS_HIP(ctx, hipGetLastError());
  return PAS_OK;
}

}  // namespace

__global__ void scale_fill_kernel(int64_t* tab, int32_t M) {
  const int32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m < M) {
    tab[2 * m] = 1000;
    tab[2 * m + 1] = INT64_MAX / 1000;
  }
}

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
    PAS_HIP(ctx, hipMalloc(&t.sorted, sizeof(int64_t) * mr));
    PAS_HIP(ctx, hipMalloc(&t.perm, sizeof(int32_t) * mr * kNumOrders));
    PAS_HIP(ctx, hipMalloc(&t.f1k, sizeof(int64_t) * (mr / 1024 + 1)));
    PAS_HIP(ctx, hipMalloc(&t.f32, sizeof(int64_t) * (mr / 32 + 1)));
    PAS_HIP(ctx, hipMalloc(&t.keys_a, sizeof(SortKey) * mr));
    PAS_HIP(ctx, hipMalloc(&t.keys_b, sizeof(SortKey) * mr));
    PAS_HIP(ctx, hipMalloc(&t.ids_a, sizeof(int32_t) * mr));
    PAS_HIP(ctx, hipMalloc(&t.ids_b, sizeof(int32_t) * mr));
    PAS_HIP(ctx, hipMalloc(&t.popc, sizeof(uint32_t) * (mw + 1)));
    PAS_HIP(ctx, hipMalloc(&t.word_scan, sizeof(uint32_t) * (mw + 1)));
    PAS_HIP(ctx, hipMalloc(&t.rows, sizeof(int32_t) * mm));
    PAS_HIP(ctx, hipMalloc(&t.scale_tab, sizeof(int64_t) * 2 * mm));
    // temp storage for the largest (whole-snapshot) sort and scan
    size_t sort_bytes = 0, scan_bytes = 0;
    SortKey* ka = static_cast<SortKey*>(t.keys_a);
    SortKey* kb = static_cast<SortKey*>(t.keys_b);
    PAS_HIP(ctx, rocprim::radix_sort_pairs(nullptr, sort_bytes, ka, kb, t.ids_a, t.ids_b,
                                           (size_t)mr, SortKeyBits{}, 0u,
                                           64 + bits_for(std::max(M, 1)), s));
    PAS_HIP(ctx, rocprim::exclusive_scan(nullptr, scan_bytes, t.popc, t.word_scan, 0u,
                                         (size_t)(mw + 1), rocprim::plus<uint32_t>(), s));
    t.sort_tmp_bytes = std::max<size_t>(sort_bytes, 16);
    t.scan_tmp_bytes = std::max<size_t>(scan_bytes, 16);
    PAS_HIP(ctx, hipMalloc(&t.sort_tmp, t.sort_tmp_bytes));
    PAS_HIP(ctx, hipMalloc(&t.scan_tmp, t.scan_tmp_bytes));
    t.n_nodes = N;
    t.n_metrics = M;
    t.row = R;
  }
  if (M > 0) {
    // every column milli until pas_tas_snapshot_set_scale says otherwise
    scale_fill_kernel<<<(M + 255) / 256, 256, 0, s>>>(t.scale_tab, M);
    PAS_HIP(ctx, hipGetLastError());
    if (MN > 0 && d_vals != t.vals)
      PAS_HIP(ctx, hipMemcpyAsync(t.vals, d_vals, sizeof(int64_t) * MN,
                                  hipMemcpyDeviceToDevice, s));
    if (MN > 0 && d_present != t.present)
      PAS_HIP(ctx, hipMemcpyAsync(t.present, d_present, sizeof(uint64_t) * M * W,
                                  hipMemcpyDeviceToDevice, s));
    if (int rc = build_columns(ctx, M, nullptr, t.vals, t.present, s)) return rc;
  }
  t.gen = gen;
  t.valid = true;
  ++t.epoch;
  return PAS_OK;
}

int tas_snapshot_update(pas_ctx* ctx, uint64_t gen, int32_t n_cols, const int32_t* cols,
                        const int64_t* d_vals, const uint64_t* d_present, hipStream_t s) {
  TasSnapshot& t = ctx->tas;
  const int32_t N = t.n_nodes;
  const int64_t W = w64(N);
  if (n_cols > 0) {
    // the new columns into their snapshot rows, then their orders
    for (int32_t c = 0; c < n_cols && N > 0; ++c) {
      const int64_t m = cols[c];
      PAS_HIP(ctx, hipMemcpyAsync(t.vals + m * N, d_vals + (int64_t)c * N, sizeof(int64_t) * N,
                                  hipMemcpyDeviceToDevice, s));
      PAS_HIP(ctx, hipMemcpyAsync(t.present + m * W, d_present + (int64_t)c * W,
                                  sizeof(uint64_t) * W, hipMemcpyDeviceToDevice, s));
    }
    // cols is a caller-owned host array: wait for its copy before returning
    PAS_HIP(ctx, hipMemcpyAsync(t.rows, cols, sizeof(int32_t) * n_cols, hipMemcpyHostToDevice,
                                s));
    PAS_HIP(ctx, hipStreamSynchronize(s));
    t.valid = false;
    if (int rc = build_columns(ctx, n_cols, t.rows, d_vals, d_present, s)) return rc;
  }
  t.gen = gen;
  t.valid = true;
  ++t.epoch;
  return PAS_OK;
}

}  // namespace pas
