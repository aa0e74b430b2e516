// Diagnostic microbenchmark (not product code): HBM write rate for the emit kernel's
// output pieces (3.7 KB runs of int32 in 4096 rows of 100k entries), no loads.
#include <hip/hip_runtime.h>
#include <cstdint>

// one wave per piece; mode 0 row-major, 1 segment-major
extern "C" __global__ void write_pieces(int32_t* out, int rows, int segs, int mode, int piece) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= rows * segs) return;
  const int r = mode == 0 ? w / segs : w % rows;
  const int s = mode == 0 ? w % segs : w / rows;
  int32_t* dst = out + (int64_t)r * 100000 + (int64_t)s * piece;
  for (int e = lane * 4; e + 4 <= piece; e += 256)
    *reinterpret_cast<int4*>(dst + e) = make_int4(r, s, e, lane);
}

// persistent waves: wave g of G handles pieces g, g+G, ... (mode 2: row-major interleave,
// mode 3: each wave a contiguous run of pieces)
extern "C" __global__ void write_pieces_persistent(int32_t* out, int rows, int segs, int mode,
                                                   int piece) {
  const int G = gridDim.x * 4;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int total = rows * segs;
  const int per = (total + G - 1) / G;
  for (int i = 0; i < per; ++i) {
    const int w = mode == 2 ? g + i * G : g * per + i;
    if (w >= total) break;
    const int r = w / segs, s = w % segs;
    int32_t* dst = out + (int64_t)r * 100000 + (int64_t)s * piece;
    for (int e = lane * 4; e + 4 <= piece; e += 256)
      *reinterpret_cast<int4*>(dst + e) = make_int4(r, s, e, lane);
  }
}

extern "C" int run(int32_t* out, int rows, int segs, int mode, int piece, int iters, int wg,
                   float* ms) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&] {
    if (mode < 2)
      write_pieces<<<(rows * segs + 3) / 4, 256>>>(out, rows, segs, mode, piece);
    else
      write_pieces_persistent<<<wg, 256>>>(out, rows, segs, mode, piece);
  };
  launch();
  (void)hipEventRecord(a);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(ms, a, b);
  *ms /= iters;
  return 0;
}

typedef int v4i __attribute__((ext_vector_type(4)));
// linear grid-stride fill of n int32 (int4 per lane); nt = non-temporal stores
template <bool NT>
__global__ void fill_linear(int32_t* out, int64_t n4) {
  v4i* o = reinterpret_cast<v4i*>(out);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const v4i v = {(int)i, 1, 2, 3};
    if (NT) __builtin_nontemporal_store(v, o + i); else o[i] = v;
  }
}
// pieces (row-major interleaved persistent) with non-temporal stores
__global__ void write_pieces_nt(int32_t* out, int rows, int segs, int piece) {
  const int G = gridDim.x * 4;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int total = rows * segs;
  for (int w = g; w < total; w += G) {
    const int r = w / segs, s = w % segs;
    int32_t* dst = out + (int64_t)r * 100000 + (int64_t)s * piece;
    for (int e = lane * 4; e + 4 <= piece; e += 256)
      __builtin_nontemporal_store((v4i){r, s, e, lane}, reinterpret_cast<v4i*>(dst + e));
  }
}

extern "C" int run2(int32_t* out, int64_t n, int kind, int wg, int iters, float* ms) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&] {
    if (kind == 0) fill_linear<false><<<wg, 256>>>(out, n / 4);
    else if (kind == 1) fill_linear<true><<<wg, 256>>>(out, n / 4);
    else write_pieces_nt<<<wg, 256>>>(out, 4096, 98, 928);
  };
  launch();
  (void)hipEventRecord(a);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(ms, a, b);
  *ms /= iters;
  return 0;
}

// pieces, dword NT stores (one 256-B store instruction per 64 entries)
__global__ void write_pieces_nt_dword(int32_t* out, int rows, int segs, int piece) {
  const int G = gridDim.x * 4;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int total = rows * segs;
  for (int w = g; w < total; w += G) {
    const int r = w / segs, s = w % segs;
    int32_t* dst = out + (int64_t)r * 100000 + (int64_t)s * piece + 3;  // unaligned start
    for (int e = lane; e < piece - 3; e += 64) __builtin_nontemporal_store(r + e, dst + e);
  }
}
extern "C" int run3(int32_t* out, int wg, int iters, float* ms) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  write_pieces_nt_dword<<<wg, 256>>>(out, 4096, 98, 928);
  (void)hipEventRecord(a);
  for (int i = 0; i < iters; ++i) write_pieces_nt_dword<<<wg, 256>>>(out, 4096, 98, 928);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(ms, a, b);
  *ms /= iters;
  return 0;
}

// runs of R consecutive pieces of one row per wave task (R * piece contiguous entries)
__global__ void write_runs_nt(int32_t* out, int rows, int segs, int piece, int R) {
  const int G = gridDim.x * 4;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int per_row = (segs + R - 1) / R;
  const int total = rows * per_row;
  for (int w = g; w < total; w += G) {
    const int r = w / per_row, c = w % per_row;
    const int s0 = c * R, s1 = min(segs, s0 + R);
    int32_t* dst = out + (int64_t)r * 100000 + (int64_t)s0 * piece;
    const int len = (s1 - s0) * piece;
    for (int e = lane * 4; e + 4 <= len; e += 256)
      __builtin_nontemporal_store((v4i){r, c, e, lane}, reinterpret_cast<v4i*>(dst + e));
  }
}
extern "C" int run4(int32_t* out, int wg, int R, int iters, float* ms) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  write_runs_nt<<<wg, 256>>>(out, 4096, 98, 928, R);
  (void)hipEventRecord(a);
  for (int i = 0; i < iters; ++i) write_runs_nt<<<wg, 256>>>(out, 4096, 98, 928, R);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(ms, a, b);
  *ms /= iters;
  return 0;
}

// linear fill, U 16-byte stores per lane per iteration (consecutive 1 KB wave chunks)
template <int U, bool NT>
__global__ void fill_unrolled(int32_t* out, int64_t n4) {
  v4i* o = reinterpret_cast<v4i*>(out);
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t base = wave * 64 * U; base < n4; base += waves * 64 * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 64 + lane;
      const v4i v = {(int)i, 1, 2, 3};
      if (i < n4) {
        if (NT) __builtin_nontemporal_store(v, o + i); else o[i] = v;
      }
    }
  }
}
extern "C" int run5(int32_t* out, int64_t n, int U, int nt, int wg, int tpb, int iters, float* ms) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&] {
#define L(UU) if (U == UU) { if (nt) fill_unrolled<UU, true><<<wg, tpb>>>(out, n / 4); \
                             else fill_unrolled<UU, false><<<wg, tpb>>>(out, n / 4); }
    L(1) L(2) L(4) L(8)
#undef L
  };
  launch();
  (void)hipEventRecord(a);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(ms, a, b);
  *ms /= iters;
  return 0;
}
