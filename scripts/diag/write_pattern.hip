// Diagnostic microbenchmark (not product code): HBM write rate for the emit kernel's
// output pieces (3.7 KB runs of int32 in 4096 rows of 100k entries) issued in different
// orders, with no loads in the kernel.
#include <hip/hip_runtime.h>
#include <cstdint>

// piece (row r, segment s) = rows * 98 pieces; each wave writes one piece of 928 ints
// mode 0: row-major  (consecutive waves -> consecutive pieces of one row)
// mode 1: segment-major (consecutive waves -> same segment of consecutive rows)
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

extern "C" int run(int32_t* out, int rows, int segs, int mode, int piece, int iters, float* ms) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int blocks = (rows * segs + 3) / 4;
  write_pieces<<<blocks, 256>>>(out, rows, segs, mode, piece);
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i) write_pieces<<<blocks, 256>>>(out, rows, segs, mode, piece);
  hipEventRecord(b);
  hipEventSynchronize(b);
  hipEventElapsedTime(ms, a, b);
  *ms /= iters;
  return 0;
}
