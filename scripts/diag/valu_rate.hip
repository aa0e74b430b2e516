// valu_rate.hip — issue cost of a few integer VALU forms at full occupancy (diagnostic).
// Each lane runs 8 independent chains of one instruction form for ITERS rounds; the kernel's
// duration over 256 CUs x 32 waves gives cycles per wave instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;

template <int FORM>
__global__ __launch_bounds__(256) void body(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint64_t b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = seed * (threadIdx.x + k);
    b[k] = (uint64_t)a[k] << 32 | (a[k] ^ 0x5555u);
  }
  const uint32_t c = seed | 1u;
  const uint64_t c64 = (uint64_t)c << 32 | c;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (FORM == 0) {
        asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[k]) : "v"(c));
      } else if constexpr (FORM == 1) {
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(b[k]) : "v"(c64));
      } else if constexpr (FORM == 2) {
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x80" : "+v"(a[k]) : "v"(c), "v"(c));
      } else {
        asm volatile("v_cmp_le_i64_e32 vcc, %0, %1" : : "v"(b[k]), "v"(c64) : "vcc");
      }
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) r ^= a[k] ^ (uint32_t)b[k] ^ (uint32_t)(b[k] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int FORM>
float run(uint32_t* out, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  body<FORM><<<blocks, 256>>>(out, 3u);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) body<FORM><<<blocks, 256>>>(out, 3u + r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int blocks = cus * 8;  // 8 blocks x 4 waves = 32 waves per CU, 8 per SIMD
  uint32_t* out;
  hipMalloc(&out, sizeof(uint32_t) * blocks * 256);
  const double insts = (double)blocks * 4 * kIters * 8;  // wave instructions
  const double ghz = p.clockRate / 1e6;
  const char* names[] = {"v_sub_u32", "v_lshl_add_u64", "v_bitop3_b32", "v_cmp_le_i64"};
  float t[4] = {run<0>(out, blocks), run<1>(out, blocks), run<2>(out, blocks), run<3>(out, blocks)};
  for (int f = 0; f < 4; ++f) {
    const double per_simd = insts / (cus * 4);
    printf("%-16s %.3f ms  %.2f cycles per wave instruction per SIMD (clock %.2f GHz)\n", names[f],
           t[f], t[f] * 1e-3 * ghz * 1e9 / per_simd, ghz);
  }
  hipFree(out);
  return 0;
}
