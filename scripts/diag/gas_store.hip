// Diagnostic microbenchmark (not product code): HBM write rate of the GAS fit result words,
// res[P][pitch] int32, in the fit kernels' grid shape: (node block, pod chunk) blocks, a
// node block's chunks on one XCD, each block looping over its chunk's pods and storing NPL
// consecutive nodes' words per lane (one 4 * NPL-byte buffer store), no compute.
#include <hip/hip_runtime.h>
#include <cstdint>

template <int NPL>
__global__ void gas_store(uint32_t* res, int P, int N, int pitch, int chunks, int aux) {
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, per_x = nb >> 3, rem = nb & 7;
  const int pos = xcd * per_x + min(xcd, rem) + (b >> 3);
  const int node_block = pos / chunks, chunk = pos % chunks;
  const int n = (node_block * blockDim.x + threadIdx.x) * NPL;
  const int per = (P + chunks - 1) / chunks;
  const int p0 = min(P, chunk * per), p1 = min(P, p0 + per);
  for (int p = p0; p < p1; ++p) {
    const __amdgpu_buffer_rsrc_t row =
        __builtin_amdgcn_make_buffer_rsrc(res + (int64_t)p * pitch, 0, N * 4, 0x00020000);
    const uint32_t v = (uint32_t)(p ^ n);
    if (NPL == 1) {
      if (aux) __builtin_amdgcn_raw_buffer_store_b32(v, row, n * 4, 0, 2);
      else __builtin_amdgcn_raw_buffer_store_b32(v, row, n * 4, 0, 0);
    } else if (NPL == 2) {
      typedef uint32_t v2u __attribute__((ext_vector_type(2)));
      const v2u w = {v, v + 1};
      if (aux) __builtin_amdgcn_raw_buffer_store_b64(w, row, n * 4, 0, 2);
      else __builtin_amdgcn_raw_buffer_store_b64(w, row, n * 4, 0, 0);
    } else {
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      const v4u w = {v, v + 1, v + 2, v + 3};
      if (aux) __builtin_amdgcn_raw_buffer_store_b128(w, row, n * 4, 0, 2);
      else __builtin_amdgcn_raw_buffer_store_b128(w, row, n * 4, 0, 0);
    }
  }
}

extern "C" int run(uint32_t* res, int P, int N, int pitch, int npl, int tpb, int blocks_target,
                   int aux, int iters, float* ms) {
  const int node_blocks = (N + tpb * npl - 1) / (tpb * npl);
  const int chunks = (blocks_target + node_blocks - 1) / node_blocks;
  auto launch = [&] {
    const dim3 g(node_blocks * chunks);
    if (npl == 1) gas_store<1><<<g, tpb>>>(res, P, N, pitch, chunks, aux);
    else if (npl == 2) gas_store<2><<<g, tpb>>>(res, P, N, pitch, chunks, aux);
    else gas_store<4><<<g, tpb>>>(res, P, N, pitch, chunks, aux);
  };
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch();
  (void)hipEventRecord(a);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(ms, a, b);
  *ms /= iters;
  return 0;
}
