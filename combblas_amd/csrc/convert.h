// gfx950 kernels of the device format conversions:
//
//   tuples -> DCSC   SpTuples(edges) / SortColBased / RemoveDuplicates + SpDCCols(const SpTuples&)
//                    [SpTuples.cpp:52-118, 271-300; SpDCCols.cpp:109-183]: a radix sort of
//                    key = col*m + row (stable: duplicates keep their input order), duplicate runs
//                    summed left to right (one thread per run, deterministic), self loops dropped on
//                    request, then column heads -> jc/cp. Replaces the serial 0.87 s DCSC build at C1.
//   DCSC -> tuples   SpTuples(const SpDCCols&) [SpTuples.cpp:181-200]: column ids expanded from cp.
//
// Included once by spgemm.hip (one translation unit).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace cbh {

__global__ void tuple_keys_kernel(const int32_t* __restrict__ rows, const int64_t* __restrict__ cols, int64_t nnz,
                                  int64_t m, int64_t n, uint64_t* __restrict__ key, int64_t* __restrict__ idx,
                                  int* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const int64_t r = rows[i], c = cols[i];
  if (r < 0 || r >= m || c < 0 || c >= n) {
    atomicOr(&err[2], 1);
    key[i] = 0;
  } else {
    key[i] = (uint64_t)c * (uint64_t)m + (uint64_t)r;
  }
  idx[i] = i;
}

// head[i] = 1 where a new (row, col) starts (and it is kept), over the sorted keys
__global__ void tuple_heads_kernel(const uint64_t* __restrict__ key, int64_t nnz, int64_t m, bool drop_loops,
                                   int64_t* __restrict__ head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const uint64_t k = key[i];
  bool h = i == 0 || key[i - 1] != k;
  if (drop_loops && (int64_t)(k / (uint64_t)m) == (int64_t)(k % (uint64_t)m)) h = false;
  head[i] = h ? 1 : 0;
}

// one thread per distinct kept key: its run of duplicates summed in input order (stable sort)
template <class V>
__global__ void tuple_reduce_kernel(const uint64_t* __restrict__ key, const int64_t* __restrict__ perm,
                                    const int64_t* __restrict__ head, const int64_t* __restrict__ pos, int64_t nnz,
                                    int64_t m, const V* __restrict__ vin, int32_t* __restrict__ ir,
                                    uint64_t* __restrict__ ukey, V* __restrict__ vout) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz || !head[i]) return;
  const uint64_t k = key[i];
  V acc = vin[perm[i]];
  for (int64_t j = i + 1; j < nnz && key[j] == k; ++j) {
    if constexpr (sizeof(V) == 1) acc = (V)(acc | vin[perm[j]]);  // bool: duplicates are ignored (OR)
    else acc += vin[perm[j]];
  }
  const int64_t o = pos[i];
  ir[o] = (int32_t)(k % (uint64_t)m);
  ukey[o] = k;
  vout[o] = acc;
}

// column heads over the unique keys -> flag, then jc/cp from their exclusive scan
__global__ void col_heads_kernel(const uint64_t* __restrict__ ukey, int64_t nnz, int64_t m, int64_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  flag[i] = (i == 0 || ukey[i - 1] / (uint64_t)m != ukey[i] / (uint64_t)m) ? 1 : 0;
}
__global__ void col_fill_kernel(const uint64_t* __restrict__ ukey, const int64_t* __restrict__ flag,
                                const int64_t* __restrict__ cpos, int64_t nnz, int64_t m, int64_t* __restrict__ jc,
                                int64_t* __restrict__ cp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  if (flag[i]) {
    jc[cpos[i]] = (int64_t)(ukey[i] / (uint64_t)m);
    cp[cpos[i]] = i;
  }
}

// DCSC -> tuples: one wave per nonzero column writes its column id over its entries
__global__ __launch_bounds__(256) void expand_cols_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp,
                                                          int64_t nzc, int64_t* __restrict__ cols) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nzc) return;
  const int64_t j = jc[c];
  for (int64_t p = cp[c] + lane; p < cp[c + 1]; p += 64) cols[p] = j;
}

}  // namespace cbh
