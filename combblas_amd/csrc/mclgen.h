// mclgen.h -- config C5's protein-similarity-like input on the device (cbh_gen_planted_partition).
//
// The reference ships no generator for HipMCL's inputs; this follows the stated
// recipe of combblas_amd/mclgen.py: a planted-partition graph with power-law cluster sizes
// (2 + floor(6 * Lomax(alpha))), avg_deg / 2 draws per vertex of which a fraction p_in land inside
// the vertex's cluster (uniform member) and the rest anywhere, cluster members scattered over the
// vertex ids by a random permutation, symmetric, uniform (0, 1] weights, unit self loops, every
// column divided by its sum (MakeColStochastic, Applications/MCL.cpp:390-396). Every random draw is
// a counter-based hash of (seed, stream, index), so the matrix depends on (n, avg_deg, seed, p_in,
// alpha) only -- the same on every run, device and driver (the C++ C5 harness and bench_mcl.py
// build the identical input). Included by spgemm.hip.
#pragma once

namespace cbh {

__host__ __device__ __forceinline__ uint64_t gen_mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// uniform double in [0, 1) of draw i of stream s
__host__ __device__ __forceinline__ double gen_u01(uint64_t seed, uint64_t s, uint64_t i) {
  return (double)(gen_mix(seed ^ gen_mix(s * 0x632BE59BD9B4E019ull + i)) >> 11) * (1.0 / 9007199254740992.0);
}

__global__ void gen_cluster_of_kernel(const int64_t* __restrict__ start, int64_t ncl, int64_t n,
                                      int32_t* __restrict__ cl) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  int64_t lo = 0, hi = ncl;  // last cluster with start <= v
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (start[mid] <= v) lo = mid;
    else hi = mid;
  }
  cl[v] = (int32_t)lo;
}

__global__ void gen_perm_keys_kernel(uint64_t seed, int64_t n, uint64_t* __restrict__ key, int32_t* __restrict__ val) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  key[v] = gen_mix(seed ^ gen_mix(0xA5A5ull * 0x632BE59BD9B4E019ull + (uint64_t)v));
  val[v] = (int32_t)v;
}

// draw d: vertex v = d / half, its neighbour u; key = min(perm) * n + max(perm), or ~0 for a loop
__global__ void gen_edge_keys_kernel(uint64_t seed, int64_t d0, int64_t cnt, int64_t half, int64_t n, double p_in,
                                     const int32_t* __restrict__ cl, const int64_t* __restrict__ start,
                                     const int32_t* __restrict__ perm, uint64_t* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cnt) return;
  const int64_t d = d0 + i;
  const int64_t v = d / half;
  const int32_t c = cl[v];
  const int64_t s0 = start[c], sz = start[c + 1] - s0;
  int64_t u;
  if (gen_u01(seed, 1, (uint64_t)d) < p_in) {
    u = s0 + (int64_t)(gen_u01(seed, 2, (uint64_t)d) * (double)sz);
    if (u >= s0 + sz) u = s0 + sz - 1;
  } else {
    u = (int64_t)(gen_u01(seed, 3, (uint64_t)d) * (double)n);
    if (u >= n) u = n - 1;
  }
  const int64_t a = perm[v], b = perm[u];
  key[i] = a == b ? ~0ull : (uint64_t)(a < b ? a : b) * (uint64_t)n + (uint64_t)(a < b ? b : a);
}

__global__ void gen_head_kernel(const uint64_t* __restrict__ k, int64_t cnt, int64_t* __restrict__ head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cnt) head[i] = (k[i] != ~0ull && (i == 0 || k[i] != k[i - 1])) ? 1 : 0;
}

// unique pair q (key K) -> entries (lo, hi) and (hi, lo) with weight 1 - u in (0, 1]; then the loops
__global__ void gen_tuples_kernel(uint64_t seed, const uint64_t* __restrict__ k, const int64_t* __restrict__ head,
                                  const int64_t* __restrict__ pos, int64_t cnt, int64_t npairs, int64_t n,
                                  int32_t* __restrict__ rows, int64_t* __restrict__ cols, double* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cnt && head[i]) {
    const int64_t q = pos[i];
    const uint64_t K = k[i];
    const int64_t lo = (int64_t)(K / (uint64_t)n), hi = (int64_t)(K % (uint64_t)n);
    const double w = 1.0 - gen_u01(seed, 4, K);
    rows[2 * q] = (int32_t)lo;
    cols[2 * q] = hi;
    vals[2 * q] = w;
    rows[2 * q + 1] = (int32_t)hi;
    cols[2 * q + 1] = lo;
    vals[2 * q + 1] = w;
  }
  if (i < n) {
    rows[2 * npairs + i] = (int32_t)i;
    cols[2 * npairs + i] = i;
    vals[2 * npairs + i] = 1.0;
  }
}

// MakeColStochastic: every column divided by its sum (wave per column, a fixed summation order)
__global__ __launch_bounds__(256) void gen_col_stochastic_kernel(const int64_t* __restrict__ cp, int64_t nzc,
                                                                 double* __restrict__ num) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nzc) return;
  double s = 0;
  for (int64_t p = cp[c] + lane; p < cp[c + 1]; p += 64) s += num[p];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  for (int64_t p = cp[c] + lane; p < cp[c + 1]; p += 64) num[p] /= s;
}

}  // namespace cbh
