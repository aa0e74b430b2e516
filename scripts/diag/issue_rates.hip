// Issue-rate microbenchmark for the GAS fit kernels' instruction mix on gfx950:
// 64-bit vs 32-bit integer compares into SGPR lane masks, SALU mask logic, v_cndmask,
// 64-bit adds, and the same mixed in the proportions the first-fit loop uses.
// (Kernels with inline-asm s_and_b64 on "+s" 64-bit operands hung on gfx950 and were
// removed.)  Every kernel runs ITERS iterations of 16 independent instructions per wave; the
// printout is the chip-wide cost per wave-instruction in SIMD cycles (at the measured
// clock) and per CU.  Build: hipcc -O3 --offload-arch=gfx950 issue_rates.hip -o issue_rates
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define ITERS 2048

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

__global__ __launch_bounds__(256) void k_cmp64(const int64_t* in, uint64_t* out, int64_t s) {
  int64_t v = in[threadIdx.x];
  uint64_t acc = 0;
  for (int it = 0; it < ITERS; ++it) {
#define C(i)                                                                         \
    {                                                                                \
      uint64_t m;                                                                    \
      asm volatile("v_cmp_le_i64_e64 %0, %1, %2" : "=s"(m) : "s"(s + i), "v"(v)); \
      acc ^= m;                                                                      \
    }
    REP16(C)
#undef C
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_cmp32(const int64_t* in, uint64_t* out, int64_t s) {
  int32_t v = (int32_t)in[threadIdx.x];
  int32_t s32 = (int32_t)s;
  uint64_t acc = 0;
  for (int it = 0; it < ITERS; ++it) {
#define C(i)                                                                          \
    {                                                                                 \
      uint64_t m;                                                                     \
      asm volatile("v_cmp_le_i32_e64 %0, %1, %2" : "=s"(m) : "s"(s32 + i), "v"(v)); \
      acc ^= m;                                                                       \
    }
    REP16(C)
#undef C
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// 16 v_cmp_i64 with no SALU consumer between them (results or-ed at the end of the batch)
__global__ __launch_bounds__(256) void k_cmp64_nosalu(const int64_t* in, uint64_t* out,
                                                      int64_t s) {
  int64_t v = in[threadIdx.x];
  uint64_t acc = 0;
  for (int it = 0; it < ITERS; ++it) {
    uint64_t m[16];
#define C(i) asm volatile("v_cmp_le_i64_e64 %0, %1, %2" : "=s"(m[i]) : "s"(s + i), "v"(v));
    REP16(C)
#undef C
    asm volatile("" ::"s"(m[0]), "s"(m[1]), "s"(m[2]), "s"(m[3]), "s"(m[4]), "s"(m[5]),
                 "s"(m[6]), "s"(m[7]));
    asm volatile("" ::"s"(m[8]), "s"(m[9]), "s"(m[10]), "s"(m[11]), "s"(m[12]), "s"(m[13]),
                 "s"(m[14]), "s"(m[15]));
    acc += it;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_cndmask(const int64_t* in, uint64_t* out, int64_t s) {
  uint32_t v = (uint32_t)in[threadIdx.x];
  uint64_t m = (uint64_t)s;
  for (int it = 0; it < ITERS; ++it) {
#define C(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(v) : "v"(i + 3), "s"(m));
    REP16(C)
#undef C
  }
  out[blockIdx.x * 256 + threadIdx.x] = v;
}

__global__ __launch_bounds__(256) void k_add64(const int64_t* in, uint64_t* out, int64_t s) {
  uint64_t v[4] = {(uint64_t)in[threadIdx.x], 1, 2, 3};
  for (int it = 0; it < ITERS; ++it) {
#define C(i) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(v[i & 3]) : "s"(s + i));
    REP16(C)
#undef C
  }
  out[blockIdx.x * 256 + threadIdx.x] = v[0] ^ v[1] ^ v[2] ^ v[3];
}

// 32-bit ALU ops of the ranked kernels (v_sub_u32, v_bitop3_b32, v_and_or_b32): 16
// independent instructions per group over 8 accumulators
__global__ __launch_bounds__(256) void k_sub32(const int64_t* in, uint64_t* out, int64_t s) {
  uint32_t v[8];
  for (int i = 0; i < 8; ++i) v[i] = (uint32_t)in[threadIdx.x] + i;
  const uint32_t s32 = (uint32_t)s;
  for (int it = 0; it < ITERS; ++it) {
#define C(i) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(v[i & 7]) : "s"(s32 + i));
    REP16(C)
#undef C
  }
  out[blockIdx.x * 256 + threadIdx.x] = v[0] ^ v[1] ^ v[2] ^ v[3] ^ v[4] ^ v[5] ^ v[6] ^ v[7];
}
__global__ __launch_bounds__(256) void k_bitop3(const int64_t* in, uint64_t* out, int64_t s) {
  uint32_t v[8];
  for (int i = 0; i < 8; ++i) v[i] = (uint32_t)in[threadIdx.x] + i;
  const uint32_t s32 = (uint32_t)s;
  for (int it = 0; it < ITERS; ++it) {
#define C(i) \
  asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x80" : "+v"(v[i & 7]) : "s"(s32 + i), "v"(v[(i + 3) & 7]));
    REP16(C)
#undef C
  }
  out[blockIdx.x * 256 + threadIdx.x] = v[0] ^ v[1] ^ v[2] ^ v[3] ^ v[4] ^ v[5] ^ v[6] ^ v[7];
}
// a dependent chain per wave (one accumulator): the single-wave latency bound
__global__ __launch_bounds__(256) void k_sub32_chain(const int64_t* in, uint64_t* out, int64_t s) {
  uint32_t v = (uint32_t)in[threadIdx.x];
  const uint32_t s32 = (uint32_t)s;
  for (int it = 0; it < ITERS; ++it) {
#define C(i) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(v) : "s"(s32 + i));
    REP16(C)
#undef C
  }
  out[blockIdx.x * 256 + threadIdx.x] = v;
}

typedef void (*Kern)(const int64_t*, uint64_t*, int64_t);

int main(int argc, char** argv) {
  const int only = argc > 1 ? atoi(argv[1]) : -1;
  setvbuf(stdout, nullptr, _IONBF, 0);
  int64_t* in;
  uint64_t* out;
  const int per_cu = argc > 2 ? atoi(argv[2]) : 8;
  const int blocks = 256 * per_cu;  // per_cu blocks (4 * per_cu waves) per CU
  hipMalloc(&in, 4096 * sizeof(int64_t));
  hipMemset(in, 0, 4096 * sizeof(int64_t));
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(uint64_t));
  struct {
    const char* name;
    Kern k;
    int valu, salu;  // per 16-instruction group
  } ks[] = {{"v_cmp_le_i64 + s_xor", k_cmp64, 16, 16},
            {"v_cmp_le_i32 + s_xor", k_cmp32, 16, 16},
            {"v_cmp_le_i64 only", k_cmp64_nosalu, 16, 0},
            {"v_cndmask_b32", k_cndmask, 16, 0},
            {"v_lshl_add_u64", k_add64, 16, 0},
            {"v_sub_u32 (8 chains)", k_sub32, 16, 0},
            {"v_bitop3_b32 (8 chains)", k_bitop3, 16, 0},
            {"v_sub_u32 (1 chain)", k_sub32_chain, 16, 0}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  const double ghz = clk_khz / 1e6;
  printf("clock %.2f GHz (attribute)\n", ghz);
  int idx = -1;
  for (auto& k : ks) {
    if (only >= 0 && ++idx != only) continue;
    fprintf(stderr, "start %s\n", k.name);
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      k.k<<<blocks, 256>>>(in, out, 5);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep < 2) continue;
      const double waves = blocks * 4.0;
      const double groups = waves * ITERS;  // 16-instruction groups
      const double simd_cycles = ms * 1e-3 * ghz * 1e9 * 256 * 4;
      printf("%d blk/CU %-34s %8.3f ms  %.2f SIMD-cycles per 16-group per wave  (%.2f per instr)\n", per_cu, k.name,
             ms, simd_cycles / groups, simd_cycles / groups / 16);
    }
  }
  return 0;
}
