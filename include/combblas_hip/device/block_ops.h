// block_ops.h -- workgroup-level building blocks of the gfx950 SpGEMM kernels (task_kernel.h,
// combblas_amd/csrc/apps.h): device-side bounds-guard reporting, block scans (sum, exclusive,
// prefix-max for the owner map), row-sorted lower bounds, and the table constants.
//
// Numeric tables use an ORDER-PRESERVING slot map (slot = (row-lo)*T/(hi-lo)) with forward linear
// probing that never wraps (kGuard slots past T): keys end up globally sorted once each run of
// occupied slots is sorted (proof in DESIGN.md §3.3), replacing the per-column std::sort
// (mtSpGEMM.h:434). A sub-tile whose probes exceed kPmax (clustered rows) or run off the table
// is retried with half the row range.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "semiring.h"

namespace cbh {

constexpr int32_t kEmpty = -1;
constexpr int kGuard = 64;  // numeric tables: extra slots past T (probing never wraps)
constexpr int kPmax = 64;   // probe limit before the tile is split in half

constexpr int kMaxLists = 16;

// Records a violated bounds guard instead of faulting: err[2] = count, err[3] |= 1<<site, and the
// first failure's context in err[4..15].
__device__ __forceinline__ void guard_fail(int* err, int site, int64_t v0 = 0, int64_t v1 = 0, int64_t v2 = 0,
                                           int64_t v3 = 0, int64_t v4 = 0, int64_t v5 = 0) {
  atomicAdd(&err[2], 1);
  atomicOr(&err[3], 1 << site);
  if (atomicCAS(&err[4], 0, site) == 0) {
    err[5] = (int)v0;
    err[6] = (int)v1;
    err[7] = (int)v2;
    err[8] = (int)v3;
    err[9] = (int)v4;
    err[10] = (int)v5;
    err[11] = (int)blockIdx.x;
    err[12] = (int)threadIdx.x;
  }
}

// The wave scans below use GFX9-only DPP controls (row_bcast:15/31, wave_shr:1); the library is
// built for gfx950 only (build.py), and any other device target stops here rather than miscompiling.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "block_ops.h: the DPP wave scans are GFX9 (gfx950) code"
#endif

// Inclusive scans across a wavefront: DPP row shifts 1/2/4/8 and the GFX9 row broadcasts 15/31
// (the sequence LLVM's atomic optimizer emits for gfx9) -- VALU moves instead of six ds_bpermute
// round trips through LDS (round 4: A^2 144.3 -> 150.1 GFLOP/s, every task kernel faster).
// Lanes without a source read `ident`.
__device__ __forceinline__ int wave_incl_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}
__device__ __forceinline__ int wave_incl_max(int v, int ident) {
  int y;
  y = __builtin_amdgcn_update_dpp(ident, v, 0x111, 0xf, 0xf, false);
  v = y > v ? y : v;
  y = __builtin_amdgcn_update_dpp(ident, v, 0x112, 0xf, 0xf, false);
  v = y > v ? y : v;
  y = __builtin_amdgcn_update_dpp(ident, v, 0x114, 0xf, 0xf, false);
  v = y > v ? y : v;
  y = __builtin_amdgcn_update_dpp(ident, v, 0x118, 0xf, 0xf, false);
  v = y > v ? y : v;
  y = __builtin_amdgcn_update_dpp(ident, v, 0x142, 0xa, 0xf, false);
  v = y > v ? y : v;
  y = __builtin_amdgcn_update_dpp(ident, v, 0x143, 0xc, 0xf, false);
  v = y > v ? y : v;
  return v;
}
// the previous lane's value (lane 0: ident)
__device__ __forceinline__ int wave_prev(int v, int ident) {
  return __builtin_amdgcn_update_dpp(ident, v, 0x138, 0xf, 0xf, false);  // wave_shr:1
}

template <int NW>
__device__ __forceinline__ int block_sum_int(int v, int* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  int t = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) t += red[w];
  return t;
}

// In-place exclusive scan of x[0..n) (LDS), x[n] = total. All threads must call.
template <int BS>
__device__ __forceinline__ void block_scan_excl(int32_t* x, int n, int* red) {
  constexpr int NW = BS / 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int carry = 0;
  for (int base = 0; base < n; base += BS) {
    const int i = base + tid;
    const int v = i < n ? x[i] : 0;
    const int s = wave_incl_sum(v);
    if (lane == 63) red[wid] = s;
    __syncthreads();
    int wpre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int r = red[w];
      wpre += (w < wid) ? r : 0;
      tot += r;
    }
    if (i < n) x[i] = carry + wpre + s - v;
    carry += tot;
    __syncthreads();
  }
  if (tid == 0) x[n] = carry;
  __syncthreads();
}

// In-place inclusive prefix-max of own[0..WIN) (LDS); each thread owns E = WIN/BS contiguous slots.
template <int BS, int WIN, class OT = int32_t>
__device__ __forceinline__ void block_max_scan(OT* own, int* red) {
  constexpr int E = WIN / BS, NW = BS / 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int v[E];
  int m = -1;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int x = own[tid * E + e];
    m = x > m ? x : m;
    v[e] = m;
  }
  const int s = wave_incl_max(m, -1);
  if (lane == 63) red[wid] = s;
  const int ex = wave_prev(s, -1);
  __syncthreads();
  int wpre = -1;
#pragma unroll
  for (int w = 0; w < NW; ++w)
    if (w < wid) wpre = red[w] > wpre ? red[w] : wpre;
  const int carry = ex > wpre ? ex : wpre;
#pragma unroll
  for (int e = 0; e < E; ++e) own[tid * E + e] = (OT)(v[e] > carry ? v[e] : carry);
  __syncthreads();
}

// first q in [lo, hi) with p[q] >= key (p sorted ascending); global memory.
__device__ __forceinline__ int lower_bound_rows(const int32_t* __restrict__ p, int lo, int hi, int64_t key) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)p[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// Galloping lower bound from `lo`: the next tile's segment usually ends a few entries later,
// so probe lo, lo+1, lo+3, lo+7, ... (same cache line) before bisecting.
__device__ __forceinline__ int gallop_rows(const int32_t* __restrict__ p, int lo, int hi, int64_t key) {
  if (lo >= hi || (int64_t)p[lo] >= key) return lo;
  int step = 1, prev = lo;
  while (true) {
    const int nx = lo + step;
    if (nx >= hi) return lower_bound_rows(p, prev + 1, hi, key);
    if ((int64_t)p[nx] >= key) return lower_bound_rows(p, prev + 1, nx, key);
    prev = nx;
    step <<= 1;
  }
}
// first i in [0, n] with x[i] >= key (x sorted); LDS.
__device__ __forceinline__ int lower_bound_lds(const int32_t* x, int n, int key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (x[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

}  // namespace cbh
