// Diagnostic microbenchmark (not product code): HBM write rate of the GAS result matrix
// (P rows of N int32, row pitch ld) in the store patterns of the fit kernels, no compute.
//   mode 0 (node per lane): a wave writes 256 B of one row per instruction, pods in turn
//   mode 1 (pod per lane): a wave owns R rows x a node range, tile by tile of T nodes; per
//          tile R rows x 4T bytes, T/4 lanes of 16 B per row
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void store_node_lane(uint32_t* out, int P, int N, int64_t ld, int chunks, int nt) {
  // blocks: (node block of 256, chunk of pods); each wave takes pods w, w+4, ... of its chunk
  const int nbk = (N + 255) / 256;
  const int b = blockIdx.x;
  const int nb = b / chunks, ch = b % chunks;
  const int per = (P + chunks - 1) / chunks;
  const int p0 = ch * per, p1 = min(P, p0 + per);
  const int n = nb * 256 + (int)threadIdx.x;
  if (nb >= nbk) return;
  const int wave = threadIdx.x >> 6;
  for (int p = p0 + wave; p < p1; p += 4)
    if (n < N) {
      uint32_t* d = out + p * ld + n;
      if (nt) __builtin_nontemporal_store((uint32_t)p, d);
      else *d = (uint32_t)p;
    }
}

__global__ void store_pod_lane(uint32_t* out, int P, int N, int64_t ld, int R, int range, int T,
                               int nt) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int groups = (P + R - 1) / R, ranges = (N + range - 1) / range;
  if (w >= groups * ranges) return;
  const int r = w / groups, g = w % groups;
  const int nb = r * range, ne = min(N, nb + range);
  const int lpr = T / 4, rpi = 64 / lpr;
  for (int t0 = nb; t0 < ne; t0 += T) {
    for (int it = 0; it < R / rpi; ++it) {
      const int p = g * R + it * rpi + lane / lpr, c = (lane % lpr) * 4;
      if (p < P && t0 + c + 4 <= ne) {
        u32x4 v = {(uint32_t)p, (uint32_t)t0, (uint32_t)c, 1u};
        u32x4* d = reinterpret_cast<u32x4*>(out + p * ld + t0 + c);
        if (nt) __builtin_nontemporal_store(v, d);
        else *d = v;
      }
    }
  }
}

int main(int argc, char** argv) {
  const int P = 4000, N = 50000;
  uint32_t* out;
  (void)hipMalloc(&out, (size_t)P * 50048 * 4 + 4096);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto time = [&](auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    (void)hipEventRecord(a);
    for (int i = 0; i < 10; ++i) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 10;
  };
  const double bytes = (double)P * N * 4;
  for (int64_t ld : {(int64_t)N, (int64_t)50048}) {
    for (int nt = 0; nt < 2; ++nt) {
      const int nbk = (N + 255) / 256, chunks = 21;
      float ms = time([&] { store_node_lane<<<nbk * chunks, 256>>>(out, P, N, ld, chunks, nt); });
      printf("ld=%ld nt=%d node-lane                   %7.1f us  %6.0f GB/s\n", (long)ld, nt,
             ms * 1e3, bytes / ms / 1e6);
      for (int R : {64, 128})
        for (int T : {16, 32, 64})
          for (int range : {256, 1024}) {
            const int groups = (P + R - 1) / R, ranges = (N + range - 1) / range;
            const int blocks = (groups * ranges + 3) / 4;
            float m = time([&] { store_pod_lane<<<blocks, 256>>>(out, P, N, ld, R, range, T, nt); });
            printf("ld=%ld nt=%d pod-lane R=%3d T=%2d rg=%4d %7.1f us  %6.0f GB/s\n", (long)ld, nt,
                   R, T, range, m * 1e3, bytes / m / 1e6);
          }
    }
  }
  return 0;
}
