// Diagnostic microbenchmark (not product code): HBM write rate of the GAS fit result words,
// res[P][pitch] int32, in the fit kernels' grid shape: (node block, pod chunk) blocks, a
// node block's chunks on one XCD, each block looping over its chunk's pods and storing NPL
// consecutive nodes' words per lane (one 4 * NPL-byte buffer store), no compute.
// map 0: a node block's chunks consecutive (the fit kernels'); 1: a chunk's node blocks
// consecutive (blocks resident together write whole rows); 2: a plain linear fill of the same
// bytes (grid-stride, 16-B stores), the ceiling without the row structure.
#include <hip/hip_runtime.h>
#include <cstdint>

template <int NPL>
__global__ void gas_store(uint32_t* res, int P, int N, int pitch, int chunks, int aux, int map) {
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, per_x = nb >> 3, rem = nb & 7;
  const int pos = xcd * per_x + min(xcd, rem) + (b >> 3);
  const int node_blocks = nb / chunks;
  const int node_block = map == 1 || map == 6 ? pos % node_blocks : pos / chunks;
  const int chunk = map == 1 || map == 6 ? pos / node_blocks : pos % chunks;
  const int n = (node_block * blockDim.x + threadIdx.x) * NPL;
  const int per = (P + chunks - 1) / chunks;
  const int p0 = min(P, chunk * per), p1 = min(P, p0 + per);
  // map 6: chunk c takes pods c, c + chunks, c + 2 chunks, ... (blocks resident together, in
  // lockstep, write consecutive rows)
  const int pstep = map == 6 ? chunks : 1;
  const int pa = map == 6 ? chunk : p0, pb = map == 6 ? P : p1;
  for (int p = pa; p < pb; p += pstep) {
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

__global__ void linear_fill(uint32_t* res, int64_t words, int aux) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i * 4 < words; i += stride) {
    const v4u w = {(uint32_t)i, 1u, 2u, 3u};
    if (aux) __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(res) + i);
    else reinterpret_cast<v4u*>(res)[i] = w;
  }
}

// map 3: one-shot linear fill, a block per 4096 * U contiguous bytes (no grid-stride loop)
template <int U>
__global__ void oneshot_fill(uint32_t* res, int64_t words, int aux) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const int64_t base = (int64_t)blockIdx.x * blockDim.x * U;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * blockDim.x + threadIdx.x;
    if (i * 4 < words) {
      const v4u w = {(uint32_t)i, 1u, 2u, 3u};
      if (aux) __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(res) + i);
      else reinterpret_cast<v4u*>(res)[i] = w;
    }
  }
}

// maps 4 / 5: one-shot row pieces, a block per (pod, node block) storing NPL words per lane
// once: 4 in row-major block order (a row's pieces consecutive), 5 column-major (a node
// block's rows consecutive)
template <int NPL>
__global__ void oneshot_rows(uint32_t* res, int P, int N, int pitch, int node_blocks, int aux,
                             int colmajor) {
  const int b = blockIdx.x;
  const int pod = colmajor ? b % P : b / node_blocks;
  const int nb = colmajor ? b / P : b % node_blocks;
  const int n = (nb * blockDim.x + threadIdx.x) * NPL;
  const __amdgpu_buffer_rsrc_t row =
      __builtin_amdgcn_make_buffer_rsrc(res + (int64_t)pod * pitch, 0, N * 4, 0x00020000);
  const uint32_t v = (uint32_t)(pod ^ n);
  if (NPL == 1) {
    if (aux) __builtin_amdgcn_raw_buffer_store_b32(v, row, n * 4, 0, 2);
    else __builtin_amdgcn_raw_buffer_store_b32(v, row, n * 4, 0, 0);
  } else {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u w = {v, v + 1, v + 2, v + 3};
    if (aux) __builtin_amdgcn_raw_buffer_store_b128(w, row, n * 4, 0, 2);
    else __builtin_amdgcn_raw_buffer_store_b128(w, row, n * 4, 0, 0);
  }
}

// map 7: row streams (the TAS ordered lists' pattern): a block writes whole rows front to back
// (4 KB per iteration: 16 B per lane), blocks b, b + G, ... of a G-block grid
__global__ void row_streams(uint32_t* res, int P, int N, int pitch, int aux) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  for (int p = blockIdx.x; p < P; p += gridDim.x) {
    const __amdgpu_buffer_rsrc_t row =
        __builtin_amdgcn_make_buffer_rsrc(res + (int64_t)p * pitch, 0, N * 4, 0x00020000);
    for (int n = threadIdx.x * 4; n < N; n += blockDim.x * 4) {
      const v4u w = {(uint32_t)p, (uint32_t)n, 2u, 3u};
      if (aux) __builtin_amdgcn_raw_buffer_store_b128(w, row, n * 4, 0, 2);
      else __builtin_amdgcn_raw_buffer_store_b128(w, row, n * 4, 0, 0);
    }
  }
}

extern "C" int run(uint32_t* res, int P, int N, int pitch, int npl, int tpb, int blocks_target,
                   int aux, int map, int iters, float* ms) {
  const int node_blocks = (N + tpb * npl - 1) / (tpb * npl);
  const int chunks = (blocks_target + node_blocks - 1) / node_blocks;
  auto launch = [&] {
    const dim3 g(node_blocks * chunks);
    const int64_t vecs = ((int64_t)P * N + 3) / 4;
    if (map == 7) {
      row_streams<<<blocks_target, tpb>>>(res, P, N, pitch, aux);
    } else if (map == 4 || map == 5) {
      const int nbk = (N + tpb * npl - 1) / (tpb * npl);
      if (npl == 1) oneshot_rows<1><<<P * nbk, tpb>>>(res, P, N, pitch, nbk, aux, map == 5);
      else oneshot_rows<4><<<P * nbk, tpb>>>(res, P, N, pitch, nbk, aux, map == 5);
    } else if (map == 2) linear_fill<<<blocks_target, tpb>>>(res, (int64_t)P * N, aux);
    else if (map == 3 && npl == 1) oneshot_fill<1><<<(vecs + tpb - 1) / tpb, tpb>>>(res, (int64_t)P * N, aux);
    else if (map == 3 && npl == 4) oneshot_fill<4><<<(vecs + 4 * tpb - 1) / (4 * tpb), tpb>>>(res, (int64_t)P * N, aux);
    else if (map == 3) oneshot_fill<16><<<(vecs + 16 * tpb - 1) / (16 * tpb), tpb>>>(res, (int64_t)P * N, aux);
    else if (npl == 1) gas_store<1><<<g, tpb>>>(res, P, N, pitch, chunks, aux, map);
    else if (npl == 2) gas_store<2><<<g, tpb>>>(res, P, N, pitch, chunks, aux, map);
    else gas_store<4><<<g, tpb>>>(res, P, N, pitch, chunks, aux, map);
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
