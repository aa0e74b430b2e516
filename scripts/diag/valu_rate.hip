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
  const uint64_t msk = __ballot(a[0] & 1u), ones = __ballot(1);
  if constexpr (FORM == 11) asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1" : : "v"(c), "v"(a[1]) : "vcc");
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (FORM == 0) {
        asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[k]) : "v"(c));
      } else if constexpr (FORM == 1) {
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(b[k]) : "v"(c64));
      } else if constexpr (FORM == 2) {
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x80" : "+v"(a[k]) : "v"(c), "v"(c));
      } else if constexpr (FORM == 3) {
        asm volatile("v_cmp_le_i64_e32 vcc, %0, %1" : : "v"(b[k]), "v"(c64) : "vcc");
      } else if constexpr (FORM == 4) {  // carry-in from an SGPR pair (the search's form)
        asm volatile("v_addc_co_u32_e64 %0, s[20:21], %0, %0, s[22:23]" : "+v"(a[k]) : : "s20", "s21");
      } else if constexpr (FORM == 5) {  // carry in and out through vcc
        asm volatile("v_addc_co_u32_e32 %0, vcc, %0, %0, vcc" : "+v"(a[k]) : : "vcc");
      } else if constexpr (FORM == 6) {
        asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(a[k]) : "v"(c));
      } else if constexpr (FORM == 7) {
        asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(c));
      } else if constexpr (FORM == 8) {
        asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c), "v"(a[(k + 1) & 7]));
      } else if constexpr (FORM == 9) {
        asm volatile("v_lshrrev_b32_e32 %0, 4, %0" : "+v"(a[k]));
      } else if constexpr (FORM == 10) {  // select on a mask from a compare (SGPR pair)
        asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c), "s"(msk));
      } else if constexpr (FORM == 11) {  // vcc written by a compare before the loop
        asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(c));
      } else if constexpr (FORM == 12) {  // all-ones mask
        asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c), "s"(ones));
      } else if constexpr (FORM == 13) {  // mixed: one vcc select per three subtractions
        if (k & 3)
          asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[k]) : "v"(c));
        else
          asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(c));
      } else {  // mixed, the select on an SGPR pair
        if (k & 3)
          asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[k]) : "v"(c));
        else
          asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c), "s"(msk));
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
  const char* names[] = {"v_sub_u32",         "v_lshl_add_u64",    "v_bitop3_b32",
                         "v_cmp_le_i64",      "v_addc_co_u32_e64", "v_addc_co_u32_e32",
                         "v_lshl_add_u32",    "v_cndmask_b32_e32", "v_and_or_b32",
                         "v_lshrrev_b32",     "v_cndmask_e64 cmp", "v_cndmask_e32 vcc=",
                         "v_cndmask_e64 ~0",  "mix 1 vcc sel:3 sub", "mix 1 e64 sel:3 sub"};
  float t[15] = {run<0>(out, blocks), run<1>(out, blocks), run<2>(out, blocks),
                 run<3>(out, blocks), run<4>(out, blocks), run<5>(out, blocks),
                 run<6>(out, blocks), run<7>(out, blocks), run<8>(out, blocks),
                 run<9>(out, blocks), run<10>(out, blocks), run<11>(out, blocks),
                 run<12>(out, blocks), run<13>(out, blocks), run<14>(out, blocks)};
  for (int f = 0; f < 15; ++f) {
    const double per_simd = insts / (cus * 4);
    printf("%-20s %.3f ms  %.2f cycles per wave instruction per SIMD (clock %.2f GHz)\n", names[f],
           t[f], t[f] * 1e-3 * ghz * 1e9 / per_simd, ghz);
  }
  hipFree(out);
  return 0;
}
