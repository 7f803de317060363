// C-ABI implementation of the gfx950 semiring SpGEMM hot path (include/combblas_hip.h).
//
// Pipeline of one cbh_spgemm call (reference stages in brackets):
//   densify_cp     A's DCSC -> dense column pointers        [Dcsc::ConstructAux/FillColInds, dcsc.cpp:983-1010,1282-1344]
//   flop_kernel    flop_j, rmin_j, rmax_j per column of B    [estimateFLOP, mtSpGEMM.h:1057-1134]
//   bin_*          columns binned by flop (symbolic) / nnz (numeric), large bins ordered by size
//   task_kernel<TSYM>  exact nnz per task (row range of a column)  [estimateNNZ_Hash, mtSpGEMM.h:806-933]
//   hipcub scan    task / column offsets of C                  [prefixsum, mtSpGEMM.h:23-70]
//   task_kernel<TNUM|TDENSE>  values, rows ascending           [LocalHybridSpGEMM loop, mtSpGEMM.h:289-441]
//   cbh_merge      task_kernel in merge mode                   [MultiwayMerge, MultiwayMerge.h:411-526]
//   compact_cols   drop empty columns -> DCSC of C            [SpDCCols(SpTuples), SpDCCols.cpp:109-183]
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/combblas_hip.h"
#include "../../include/combblas_hip/device/numeric.h"
#include "../../include/combblas_hip/device/merge2.h"
#include "apps.h"
#include "convert.h"
#include "blocks.h"
#include "mclgen.h"

using namespace cbh;

// ============================================================================ context / matrices
struct cbh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  int64_t phase_budget = 0;
  double bmp_frac = -1.0;  // < 0: bmp_frac() (cbh_ctx_set_bitmap_fraction)
  bool timing = false;
  cbh_kernel_times times{-1, -1, -1, 0};
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  int* d_err = nullptr;  // 32 ints: [0..15] device-side error flags (check_err), [16] sub-tile retries
  void* ws = nullptr;  // persistent phase workspace (hipMalloc'd once, grow-only): a ~150 GB
  int64_t ws_bytes = 0;  // buffer must not be re-mapped on every product
  cbh_alloc_fn alloc = nullptr;
  cbh_free_fn release = nullptr;
  void* alloc_user = nullptr;
  // per-launch instrumentation (cbh_ctx_enable_timing): events around every tile-kernel launch
  struct Rec {
    int kind;
    size_t e0, e1;
    double bytes;
  };
  // stream-ordered block cache of the default allocator (see dalloc): free blocks by size and
  // the size of every live block
  std::multimap<size_t, void*> cache;
  std::unordered_map<void*, size_t> live;
  size_t cached_bytes = 0;
  // CBH_CACHE_CAP_GB; above it cached blocks go back to HIP (shrink_cache). Default, set at
  // cbh_ctx_create: 0.9 of the device -- a product near HBM capacity (scale-22 A^2: 108 GB of
  // stored bitmaps; C5's 190 GB output arena) otherwise re-maps its scratch every call; OOM,
  // the RCCL setup (cbh_ctx_release) and cbh_ctx_trim give memory to other allocators
  size_t cache_cap = size_t(128) << 30;
  bool poison = false;  // CBH_ALLOC_POISON=1: freed blocks are filled with 0xFF and never reused
  std::vector<void*> quarantine;
  std::vector<hipEvent_t> evpool;
  size_t evused = 0;
  std::vector<Rec> recs;
  double k_ms[CBH_K_NKINDS] = {0};
  int64_t k_launch[CBH_K_NKINDS] = {0};
  double k_bytes[CBH_K_NKINDS] = {0};
  cbh_phase_fn phase_fn = nullptr;  // per-phase consumer of cbh_spgemm_phased
  void* phase_user = nullptr;
  // pinned staging of the chunked host transfers (cbh_mat_upload_chunks / _download_chunks):
  // two halves of pin_bytes / 2, grow-only, with one event per half
  void* pin = nullptr;
  size_t pin_bytes = 0;
  hipEvent_t pin_ev[2] = {nullptr, nullptr};
};

struct cbh_mat {
  int64_t m = 0, n = 0, nnz = 0, nzc = 0;
  int dtype = CBH_F64;
  int64_t vbytes = 8;  // bytes per value (dtype's size; CBH_OPAQUE: the caller's)
  int64_t* cp = nullptr;
  int64_t* jc = nullptr;
  int32_t* ir = nullptr;
  void* num = nullptr;
  bool owned = true;
  bool borrowed_rows = false;  // ir / num live in a cbh_arena (not freed with the block)
};

// Output arena of the phased MCL drivers: the pruned pieces of every phase are written back to
// back into one pair of row / value arrays, which then become the concatenated result's arrays
// without a copy (cbh_arena_concat) -- a near-capacity product never holds the pieces and their
// concatenation at once.
struct cbh_arena {
  int32_t* ir = nullptr;
  char* num = nullptr;
  int64_t cap = 0, used = 0, vbytes = 8;
  bool overflow = false;  // a piece did not fit: it was allocated on its own (cbh_arena_concat copies)
};

static size_t dtype_size(int dt) {
  switch (dt) {
    case CBH_F64: case CBH_I64: return 8;
    case CBH_F32: case CBH_I32: return 4;
    case CBH_BOOL: return 1;
  }
  return 0;
}

// a HIP call's status as a library code (the context's error text set), for paths that must free
// what they hold before returning instead of CBH_HIP's early return
static int hip_rc(cbh_ctx* ctx, hipError_t e, const char* what);
#define CBH_HIP(ctx, call)                                                                       \
  do {                                                                                           \
    hipError_t e_ = (call);                                                                      \
    if (e_ != hipSuccess) {                                                                      \
      (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                            \
      return (e_ == hipErrorOutOfMemory || e_ == hipErrorMemoryAllocation) ? CBH_E_OOM : CBH_E_HIP; \
    }                                                                                            \
  } while (0)

#define CBH_TRY(x)            \
  do {                        \
    int rc_ = (x);            \
    if (rc_ != CBH_OK) return rc_; \
  } while (0)

static int fail(cbh_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}
static int hip_rc(cbh_ctx* ctx, hipError_t e, const char* what) {
  if (e == hipSuccess) return CBH_OK;
  return fail(ctx, (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? CBH_E_OOM : CBH_E_HIP,
              std::string(what) + ": " + hipGetErrorString(e));
}

// Default device allocator: a per-context cache of hipMalloc'd blocks, reused in stream order.
// Every kernel and copy of a context runs on its one stream, so a block freed by an earlier call
// can be handed to a later allocation without a sync: the stream finishes the old users first.
// (hipMallocAsync's default pool, used before, handed overlapping blocks to live allocations on
// repeated phased products in processes where torch had not initialised HIP first.)
// Sizes are rounded to 512 B (< 1 MiB) or 2 MiB; a cached block is reused for a request of at
// least half its size. On OOM cached blocks go back to HIP (after a stream sync, as many as the
// request needs, then all of them) and the request is retried; the cache also sheds blocks when
// it grows past cache_cap, on cbh_ctx_release and (all) on cbh_ctx_trim.
// Debug mode CBH_ALLOC_POISON=1 (read at cbh_ctx_create): a freed block is overwritten with 0xFF
// on the stream and quarantined until the context is destroyed, so a use after free reads NaN /
// -1 row ids instead of a later allocation's data (tests/test_allocator_gpu.py).
static size_t alloc_class(size_t bytes) {
  return bytes < (size_t(1) << 20) ? (bytes + 511) & ~size_t(511) : (bytes + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
}
static void release_cache(cbh_ctx* ctx) {
  (void)hipStreamSynchronize(ctx->stream);
  static const bool diag = std::getenv("CBH_MEMDIAG") != nullptr;
  int nerr = 0;
  hipError_t last = hipSuccess;
  for (auto& kv : ctx->cache) {
    const hipError_t e = hipFree(kv.second);
    if (e != hipSuccess) {
      ++nerr;
      last = e;
    }
  }
  if (diag && !ctx->cache.empty())
    std::fprintf(stderr, "[cbh memdiag] release_cache: %zu blocks, %.2f GB, %d hipFree errors (%s)\n", ctx->cache.size(),
                 ctx->cached_bytes / 1e9, nerr, hipGetErrorString(last));
  (void)hipGetLastError();
  ctx->cache.clear();
  ctx->cached_bytes = 0;
  for (void* q : ctx->quarantine) (void)hipFree(q);
  ctx->quarantine.clear();
}
// frees cached blocks until the cache holds at most `keep` bytes: each time the smallest block
// that alone covers what is still to go, else the largest (a near-capacity product re-maps only
// what it must, and a cache just over its cap keeps its big blocks: C5's C++ driver then reuses
// its 190 GB output arena from the second call on instead of re-mapping it)
static void shrink_cache(cbh_ctx* ctx, size_t keep) {
  if (ctx->cached_bytes <= keep || ctx->cache.empty()) return;
  (void)hipStreamSynchronize(ctx->stream);
  while (ctx->cached_bytes > keep && !ctx->cache.empty()) {
    auto it = ctx->cache.lower_bound(ctx->cached_bytes - keep);
    if (it == ctx->cache.end()) it = std::prev(ctx->cache.end());
    (void)hipFree(it->second);
    ctx->cached_bytes -= it->first;
    ctx->cache.erase(it);
  }
  (void)hipGetLastError();
}
template <class T>
static int dalloc(cbh_ctx* ctx, T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  const size_t bytes = ((count * sizeof(T)) + 255) & ~size_t(255);
  if (ctx->alloc) {
    *p = reinterpret_cast<T*>(ctx->alloc(ctx->alloc_user, (int64_t)bytes, ctx->stream));
    if (!*p) return fail(ctx, CBH_E_OOM, "allocator callback failed for " + std::to_string(bytes) + " bytes");
    return CBH_OK;
  }
  const size_t cls = alloc_class(bytes);
  auto it = ctx->cache.lower_bound(cls);
  // a cached block serves a request up to twice its size; above 1 GB only up to 1/8 larger (a 26 GB
  // request served by a 39 GB block left C5's third MCL call 13 GB short)
  const size_t slack = cls >= (size_t(1) << 30) ? cls / 8 : cls;
  if (it != ctx->cache.end() && it->first - cls <= slack) {
    void* q = it->second;
    ctx->live[q] = it->first;
    ctx->cached_bytes -= it->first;
    ctx->cache.erase(it);
    *p = reinterpret_cast<T*>(q);
    return CBH_OK;
  }
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, cls);
  if (e != hipSuccess && !ctx->cache.empty()) {  // give back cached blocks, largest first, until it fits
    (void)hipGetLastError();
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    const size_t margin = size_t(1) << 30;
    const size_t need = cls + margin > fr ? cls + margin - fr : 0;
    shrink_cache(ctx, ctx->cached_bytes > need ? ctx->cached_bytes - need : 0);
    e = hipMalloc(&q, cls);
    if (e != hipSuccess && !ctx->cache.empty()) {
      (void)hipGetLastError();
      release_cache(ctx);
      e = hipMalloc(&q, cls);
    }
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    size_t live = 0;
    for (auto& kv : ctx->live) live += kv.second;
    return fail(ctx, CBH_E_OOM, "hipMalloc(" + std::to_string(cls) + "): " + hipGetErrorString(e) + " (device free " +
                                    std::to_string(fr) + " of " + std::to_string(tot) + ", context live " +
                                    std::to_string(live) + ", workspace " + std::to_string(ctx->ws_bytes) + ")");
  }
  ctx->live[q] = cls;
  *p = reinterpret_cast<T*>(q);
  return CBH_OK;
}
static void dfree(cbh_ctx* ctx, void* p) {
  if (!p) return;
  if (ctx->release) {
    ctx->release(ctx->alloc_user, p, ctx->stream);
    return;
  }
  auto it = ctx->live.find(p);
  if (it == ctx->live.end()) return;  // not ours (wrapped device arrays are never freed here)
  if (ctx->poison) {
    (void)hipMemsetAsync(p, 0xFF, it->second, ctx->stream);
    ctx->quarantine.push_back(p);
    ctx->live.erase(it);
    return;
  }
  ctx->cache.emplace(it->second, p);
  ctx->cached_bytes += it->second;
  ctx->live.erase(it);
  if (ctx->cached_bytes > ctx->cache_cap) shrink_cache(ctx, ctx->cache_cap);
}

// RAII holder for scratch allocations of one call.
struct Scratch {
  cbh_ctx* ctx;
  std::vector<void*> ptrs;
  explicit Scratch(cbh_ctx* c) : ctx(c) {}
  template <class T>
  int get(T** p, size_t count) {
    int rc = dalloc(ctx, p, count);
    if (rc == CBH_OK) ptrs.push_back(*p);
    return rc;
  }
  // frees one allocation of this holder before the call ends (no-op for foreign pointers)
  void drop(void* p) {
    for (auto it = ptrs.begin(); it != ptrs.end(); ++it)
      if (*it == p) {
        dfree(ctx, p);
        ptrs.erase(it);
        return;
      }
  }
  ~Scratch() {
    for (void* p : ptrs) dfree(ctx, p);
  }
};

// ============================================================================ auxiliary kernels
__global__ void densify_cp_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp, int64_t nzc,
                                  int64_t n, int64_t nnz, int64_t* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > n) return;
  int64_t lo = 0, hi = nzc;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (jc[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  out[k] = lo < nzc ? cp[lo] : nnz;
}

// One wave per nonzero column of B: flops, and the row range any product can reach
// (A's columns are row-sorted, so first/last entries bound them).
__global__ __launch_bounds__(256) void flop_kernel(const int64_t* __restrict__ Acp, const int32_t* __restrict__ Air,
                                                   const int64_t* __restrict__ Bcp, const int32_t* __restrict__ Bir,
                                                   int64_t nzc, int64_t ncolA, int64_t* __restrict__ flop,
                                                   int32_t* __restrict__ rmin, int32_t* __restrict__ rmax, int* err) {
  const int lane = threadIdx.x & 63;
  const int64_t col = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (col >= nzc) return;
  int64_t f = 0;
  int32_t mn = INT32_MAX, mx = -1;
  for (int64_t p = Bcp[col] + lane; p < Bcp[col + 1]; p += 64) {
    const int32_t k = Bir[p];
    if (k < 0 || k >= ncolA) {  // B row id outside A's columns: report, do not index
      guard_fail(err, 11, col, k, ncolA);
      continue;
    }
    const int64_t s = Acp[k], e = Acp[k + 1];
    if (e > s) {
      f += e - s;
      mn = min(mn, Air[s]);
      mx = max(mx, Air[e - 1]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    f += __shfl_xor(f, o);
    mn = min(mn, __shfl_xor(mn, o));
    mx = max(mx, __shfl_xor(mx, o));
  }
  if (lane == 0) {
    flop[col] = f;
    rmin[col] = f ? mn : 0;
    rmax[col] = f ? mx : 0;
  }
}

// Bins: 0 = no work, 1 = small (work <= cap1), 2 = mid (work <= cap2), 3 + (kSub-1-lg) = large,
// lg = floor(log2 work): laid out in bin order so the large list runs from the heaviest columns down.
constexpr int kSub = 48;
constexpr int kNB = 3 + kSub;
constexpr int kGroups = 3;  // small, mid, large

struct BinCaps {
  int64_t cap1, cap2;
};

__device__ __forceinline__ int bin_of(int64_t w, BinCaps k) {
  if (w <= 0) return 0;
  if (w <= k.cap1) return 1;
  if (w <= k.cap2) return 2;
  int lg = 63 - __clzll((unsigned long long)w);
  if (lg > kSub - 1) lg = kSub - 1;
  return 3 + (kSub - 1 - lg);
}
__device__ __forceinline__ int group_of(int b) { return b <= 1 ? 0 : (b == 2 ? 1 : 2); }

// Optional per-group unit sums for the roofline (groups small/mid/large): sums[g] = sum of
// units[item] (algorithmic entries an item moves).
__global__ __launch_bounds__(256) void bin_count_kernel(const int64_t* __restrict__ work, int64_t n, BinCaps caps,
                                                        unsigned long long* __restrict__ counts,
                                                        const int64_t* __restrict__ units,
                                                        unsigned long long* __restrict__ sums) {
  __shared__ unsigned int h[kNB];
  __shared__ unsigned long long ssum[kGroups];
  for (int i = threadIdx.x; i < kNB; i += blockDim.x) h[i] = 0;
  if (threadIdx.x < kGroups) ssum[threadIdx.x] = 0;
  __syncthreads();
  unsigned long long loc[kGroups] = {0, 0, 0};
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x) {
    const int b = bin_of(work[c], caps);
    atomicAdd(&h[b], 1u);
    if (sums && units && b > 0) loc[group_of(b)] += (unsigned long long)units[c];
  }
  if (sums)
    for (int i = 0; i < kGroups; ++i)
      if (loc[i]) atomicAdd(&ssum[i], loc[i]);
  __syncthreads();
  for (int i = threadIdx.x; i < kNB; i += blockDim.x)
    if (h[i]) atomicAdd(&counts[i], (unsigned long long)h[i]);
  if (sums && threadIdx.x < kGroups && ssum[threadIdx.x]) atomicAdd(&sums[threadIdx.x], ssum[threadIdx.x]);
}

__global__ __launch_bounds__(256) void bin_scatter_kernel(const int64_t* __restrict__ work, int64_t n, int64_t col0,
                                                          BinCaps caps, unsigned long long* __restrict__ cursor,
                                                          int32_t* __restrict__ cols) {
  __shared__ unsigned int h[kNB];
  __shared__ unsigned long long base[kNB];
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int i = threadIdx.x; i < kNB; i += blockDim.x) h[i] = 0;
  __syncthreads();
  int b = -1;
  unsigned int r = 0;
  if (c < n) {
    b = bin_of(work[c], caps);
    r = atomicAdd(&h[b], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kNB; i += blockDim.x)
    base[i] = h[i] ? atomicAdd(&cursor[i], (unsigned long long)h[i]) : 0ull;
  __syncthreads();
  if (b > 0) cols[base[b] + r] = (int32_t)(c + col0);
}

// launch order inside a bin by row block (rowkey): keys = bin * 256 + rowkey, bin 0 last
__global__ void bin_key_kernel(const int64_t* __restrict__ work, int64_t n, int64_t col0, BinCaps caps,
                               const int32_t* __restrict__ rowkey, uint32_t* __restrict__ keys,
                               int32_t* __restrict__ vals) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const int b = bin_of(work[c], caps);
  keys[c] = b == 0 ? 0xFFFFFFFFu : (uint32_t)b * 256u + (uint32_t)(rowkey[c] & 255);
  vals[c] = (int32_t)(c + col0);
}

// per task: the row block of its middle row (tasks of one row block read the same lines of the
// hub columns of A)
__global__ void task_rowkey_kernel(const int32_t* __restrict__ tlo, const int32_t* __restrict__ thi, int64_t n,
                                   int32_t RB, int32_t* __restrict__ key) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) key[t] = (int32_t)(((int64_t)tlo[t] + thi[t]) / 2 / RB);
}

__global__ void fill_i64_kernel(int64_t* p, int64_t n, int64_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void nz_flag_kernel(const int64_t* __restrict__ nnz, int64_t n, int64_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flag[i] = nnz[i] > 0 ? 1 : 0;
}

__global__ void compact_cols_kernel(const int64_t* __restrict__ nnz, const int64_t* __restrict__ pos,
                                    const int64_t* __restrict__ Bjc, const int64_t* __restrict__ Ccp, int64_t n,
                                    int64_t* __restrict__ jc, int64_t* __restrict__ cp, int64_t base = 0) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && nnz[i] > 0) {
    jc[pos[i]] = Bjc[i];
    cp[pos[i]] = Ccp[i] - base;
  }
  if (i == n - 1) cp[pos[n]] = Ccp[n] - base;
}

// CBH_KEEP_EMPTY_COLS form of a slot range: every slot kept, offsets rebased
__global__ void keep_cols_kernel(const int64_t* __restrict__ Bjc, const int64_t* __restrict__ Ccp, int64_t n,
                                 int64_t base, int64_t* __restrict__ jc, int64_t* __restrict__ cp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) jc[i] = Bjc[i];
  if (i <= n) cp[i] = Ccp[i] - base;
}

__global__ void widen_i32_kernel(const int32_t* __restrict__ f, int64_t* __restrict__ o, int64_t k) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < k) o[i] = f[i];
}

// merge: mark union of column ids
__global__ void mark_cols_kernel(const int64_t* __restrict__ jc, int64_t nzc, int64_t n, int32_t* __restrict__ flag,
                                 int* err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nzc) return;
  const int64_t c = jc[i];
  if (c < 0 || c >= n) guard_fail(err, 10, i, c, n);
  else flag[c] = 1;
}
__global__ void union_cols_kernel(const int32_t* __restrict__ flag, const int64_t* __restrict__ idx, int64_t n,
                                  int64_t* __restrict__ jcC) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n && flag[k]) jcC[idx[k]] = k;
}
__global__ void merge_seg_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp, int64_t nzc,
                                 const int64_t* __restrict__ idx, int l, int nl, int64_t* __restrict__ seg_start,
                                 int64_t* __restrict__ seg_len) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nzc) return;
  const int64_t c = idx[jc[i]];
  seg_start[c * nl + l] = cp[i];
  seg_len[c * nl + l] = cp[i + 1] - cp[i];
}
struct ListRows {
  const int32_t* ir[kMaxLists];
};
__global__ void merge_work_kernel(const int64_t* __restrict__ seg_start, const int64_t* __restrict__ seg_len, int nl,
                                  ListRows lr, int64_t ncols, int64_t* __restrict__ work, int32_t* __restrict__ rmin,
                                  int32_t* __restrict__ rmax) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncols) return;
  int64_t w = 0;
  int32_t mn = INT32_MAX, mx = -1;
  for (int l = 0; l < nl; ++l) {
    const int64_t len = seg_len[c * nl + l];
    if (len > 0) {
      const int64_t s = seg_start[c * nl + l];
      w += len;
      mn = min(mn, lr.ir[l][s]);
      mx = max(mx, lr.ir[l][s + len - 1]);
    }
  }
  work[c] = w;
  rmin[c] = w ? mn : 0;
  rmax[c] = w ? mx : 0;
}

// checksum of one C block: wave per column; global entry index = gbase + local index
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
template <class VT>
__global__ __launch_bounds__(256) void checksum_kernel(const int64_t* __restrict__ colid, const int64_t* __restrict__ cp,
                                                       int64_t cbase, int64_t ncols, const int32_t* __restrict__ ir,
                                                       const VT* __restrict__ num, int64_t gbase,
                                                       double* __restrict__ vsum, unsigned long long* __restrict__ dig,
                                                       const int64_t* __restrict__ colpos = nullptr,
                                                       int64_t row_off = 0, int64_t col_off = 0) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  double s = 0;
  uint64_t d = 0;
  if (c < ncols) {
    const uint64_t col = (uint64_t)(colid[c] + col_off);
    // colpos (a block of a distributed C): the global position of the column's first entry, so that
    // the blocks' digests add up to the whole product's
    if (colpos) gbase = colpos[c] - (cp[c] - cbase);
    for (int64_t p = cp[c] - cbase + lane; p < cp[c + 1] - cbase; p += 64) {
      const VT v = num[p];
      uint64_t bits;
      if constexpr (sizeof(VT) == 8) bits = __builtin_bit_cast(uint64_t, v);
      else if constexpr (sizeof(VT) == 4) bits = (uint64_t)__builtin_bit_cast(uint32_t, v);
      else bits = (uint64_t)v;
      s += (double)v;
      d += mix64((uint64_t)(gbase + p) ^ mix64(col ^ mix64((uint64_t)(uint32_t)(ir[p] + row_off) ^ mix64(bits))));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    d += __shfl_xor(d, o);
  }
  if (lane == 0 && c < ncols) {
    atomicAdd(vsum, s);
    atomicAdd(dig, (unsigned long long)d);
  }
}

static size_t next_event(cbh_ctx* ctx) {
  if (ctx->evused == ctx->evpool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return (size_t)-1;
    ctx->evpool.push_back(e);
  }
  return ctx->evused++;
}

// Folds the recorded launch events into the per-kind totals (call after a stream sync).
static void flush_records(cbh_ctx* ctx) {
  for (const auto& r : ctx->recs) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, ctx->evpool[r.e0], ctx->evpool[r.e1]) == hipSuccess) {
      ctx->k_ms[r.kind] += ms;
      ctx->k_launch[r.kind] += 1;
      ctx->k_bytes[r.kind] += r.bytes;
    }
  }
  ctx->recs.clear();
  ctx->evused = 0;
}

// Bins the items [0, n) (column slots or tasks) by work; writes item ids + col0 into `ids`.
struct BinLists {
  int64_t small_first = 0, small_count = 0, mid_first = 0, mid_count = 0, large_first = 0, large_count = 0;
  int64_t sub_count[kSub] = {0};  // large sub-bins, index = floor(log2 work)
  double units[kGroups] = {0};    // [small|mid|large] sum of units (timing only)
};
// Unit sums are gathered only when the context records timings (bench/roofline); `units` is
// indexed like `work`.
// Inside each bin, tasks launch in row-block order (rowkey), so the tasks in flight at a time
// read one slice of A (98.3 -> 99.0 GFLOP/s at scale 22: the dense kernel's over-fetch hits L2
// more often).
static int make_bins(cbh_ctx* ctx, Scratch& S, const int64_t* work, int64_t n, int64_t col0, int32_t* ids,
                     BinLists* out, BinCaps caps, const int64_t* units = nullptr, const int32_t* rowkey = nullptr) {
  constexpr int NS = kGroups;
  unsigned long long* counts;
  CBH_TRY(S.get(&counts, 2 * kNB + NS));
  unsigned long long* sums = ctx->timing ? counts + 2 * kNB : nullptr;
  CBH_HIP(ctx, hipMemsetAsync(counts, 0, sizeof(unsigned long long) * (2 * kNB + NS), ctx->stream));
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(bin_count_kernel, dim3(std::max(grid, 1)), dim3(256), 0, ctx->stream, work, n, caps, counts,
                     units, sums);
  CBH_HIP(ctx, hipGetLastError());
  unsigned long long h[2 * kNB + NS];
  CBH_HIP(ctx, hipMemcpyAsync(h, counts, sizeof(unsigned long long) * (2 * kNB + NS), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  unsigned long long off[kNB];
  unsigned long long run = 0;
  off[0] = 0;  // bin 0 not stored
  for (int b = 1; b < kNB; ++b) {
    off[b] = run;
    run += h[b];
  }
  if (rowkey && n > 0) {
    uint32_t *kin, *kout;
    int32_t* vin;
    CBH_TRY(S.get(&kin, n));
    CBH_TRY(S.get(&kout, n));
    CBH_TRY(S.get(&vin, n));
    hipLaunchKernelGGL(bin_key_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, work, n, col0, caps,
                       rowkey, kin, vin);
    CBH_HIP(ctx, hipGetLastError());
    int32_t* vout = ids;  // the first `run` sorted items are the binned ones, in bin order
    int32_t* vtmp = nullptr;
    if ((int64_t)run < n) {  // ids holds only `run` slots: sort into scratch, copy the prefix
      CBH_TRY(S.get(&vtmp, n));
      vout = vtmp;
    }
    size_t tmp = 0;
    CBH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, kin, kout, vin, vout, (int)n, 0, 16, ctx->stream));
    void* tbuf;
    CBH_TRY(S.get(reinterpret_cast<char**>(&tbuf), tmp));
    CBH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(tbuf, tmp, kin, kout, vin, vout, (int)n, 0, 16, ctx->stream));
    if (vtmp && run > 0)
      CBH_HIP(ctx, hipMemcpyAsync(ids, vtmp, sizeof(int32_t) * run, hipMemcpyDeviceToDevice, ctx->stream));
  } else {
    unsigned long long* cursor = counts + kNB;
    CBH_HIP(ctx, hipMemcpyAsync(cursor, off, sizeof(off), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(bin_scatter_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, work, n, col0,
                       caps, cursor, ids);
    CBH_HIP(ctx, hipGetLastError());
  }
  // the host copy of `off` must outlive the async H2D copy
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (sums)
    for (int i = 0; i < NS; ++i) out->units[i] = (double)h[2 * kNB + i];
  out->small_first = 0;
  out->small_count = (int64_t)h[1];
  out->mid_first = (int64_t)h[1];
  out->mid_count = (int64_t)h[2];
  out->large_first = (int64_t)(h[1] + h[2]);
  out->large_count = (int64_t)(run - h[1] - h[2]);
  for (int lg = 0; lg < kSub; ++lg) out->sub_count[lg] = (int64_t)h[3 + (kSub - 1 - lg)];
  return CBH_OK;
}

// CBH_DIAG=1: launch every large sub-bin separately and print its time (profiling aid only).
static bool diag_enabled() {
  static int v = [] {
    const char* e = std::getenv("CBH_DIAG");
    return e ? std::atoi(e) : 0;
  }();
  return v != 0;
}
static int exclusive_scan_i64(cbh_ctx* ctx, Scratch& S, const int64_t* in, int64_t* out, int64_t n) {
  size_t tmp = 0;
  CBH_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, (int)n, ctx->stream));
  void* t;
  CBH_TRY(S.get(reinterpret_cast<char**>(&t), tmp));
  CBH_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(t, tmp, in, out, (int)n, ctx->stream));
  return CBH_OK;
}

static int sum_i64(cbh_ctx* ctx, Scratch& S, const int64_t* in, int64_t n, int64_t* d_out) {
  size_t tmp = 0;
  CBH_HIP(ctx, hipcub::DeviceReduce::Sum(nullptr, tmp, in, d_out, (int)n, ctx->stream));
  void* t;
  CBH_TRY(S.get(reinterpret_cast<char**>(&t), tmp));
  CBH_HIP(ctx, hipcub::DeviceReduce::Sum(t, tmp, in, d_out, (int)n, ctx->stream));
  return CBH_OK;
}

static inline unsigned blocks_for(int64_t n, int bs) { return (unsigned)std::max<int64_t>(1, (n + bs - 1) / bs); }
// grid cap of the wave-strided kernels (an AQL dispatch counts work-items in 32 bits: a direct
// grid of blocks_for(n, 4) x 256 threads overflows from n = 2^26 items)
constexpr unsigned kWaveGridCap = 1u << 16;
// CBH_TEST_GRID_CAP=<blocks> lowers the cap so that a small product exercises the wave-strided
// loops' wrap-around (tests/test_regress_gpu.py); read on every launch so a test can set it
static unsigned wave_grid_cap() {
  const char* e = std::getenv("CBH_TEST_GRID_CAP");
  const long v = e ? std::atol(e) : 0;
  return v > 0 && v < (long)kWaveGridCap ? (unsigned)v : kWaveGridCap;
}

static int check_err(cbh_ctx* ctx) {
  int h[16];
  CBH_HIP(ctx, hipMemcpyAsync(h, ctx->d_err, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (ctx->timing) flush_records(ctx);
  if (h[0] || h[1] || h[2]) {
    CBH_HIP(ctx, hipMemsetAsync(ctx->d_err, 0, sizeof(h), ctx->stream));
    return fail(ctx, CBH_E_INTERNAL,
                "device consistency check failed (count mismatch " + std::to_string(h[0]) + ", split failure " +
                    std::to_string(h[1]) + ", bounds guards " + std::to_string(h[2]) + " sites mask " +
                    std::to_string(h[3]) + "; first: site " + std::to_string(h[4]) + " ctx " + std::to_string(h[5]) +
                    " " + std::to_string(h[6]) + " " + std::to_string(h[7]) + " " + std::to_string(h[8]) + " " +
                    std::to_string(h[9]) + " " + std::to_string(h[10]) + " block " + std::to_string(h[11]) +
                    " thread " + std::to_string(h[12]) + ")");
  }
  return CBH_OK;
}

// ============================================================================ task plan (spgemm)
// Every nonzero column j of B becomes S_j tasks: equal-width row ranges of [rmin_j, rmax_j]
// with about kTaskFlops products each (S_j = 1 for light columns). Tasks of a column are
// consecutive and in row order, so the exclusive scan of the per-task counts gives every task
// its output offset and C's column pointers are the offsets of each column's first task.
// (round 3: 65536 / 262144 vs 131072 -> 121.8 / 124.9 vs 124.8 GFLOP/s at scale 22; round 4 with the
// 2048-slot hash table: 133.7 / 140.3 vs 139.5, symbolic 221 / 184 vs 194 ms)
#ifndef CBH_TASK_FLOPS  // (A/B hook: build variants only)
#define CBH_TASK_FLOPS 262144
#endif
constexpr int64_t kTaskFlops = CBH_TASK_FLOPS;
constexpr int64_t kMergeTaskFlops = 131072;  // merge tasks (list entries per task; not re-measured)

// Row blocks: C's rows are cut into blocks of RB rows (kRowBlocks blocks); interior task
// boundaries of a split column sit on block boundaries, where the row-block table of A gives
// every hub entry's position directly (hub_fill_kernel); short columns bisect.
constexpr int64_t kRowBlocks = 256;  // (128 / 192 / 384: 130.9 / 131.3 / 131.4 vs 132.2 GFLOP/s, aligned sub-tiles)
// rows per block: a multiple of 32 from 32 rows up, so that block boundaries are stored-bitmap word boundaries
static int32_t row_block(int64_t m) {
  const int64_t rb = std::max<int64_t>(1, (m + kRowBlocks - 1) / kRowBlocks);
  return (int32_t)(rb >= 32 ? (rb + 31) & ~int64_t(31) : rb);  // small matrices keep fine blocks
}

__global__ void task_count_kernel(const int64_t* __restrict__ flop, const int32_t* __restrict__ rmin,
                                  const int32_t* __restrict__ rmax, int64_t n, int64_t ft, int32_t RB,
                                  int64_t* __restrict__ S) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t f = flop[i];
  int64_t s = 0;
  if (f > 0) {
    const int64_t nb = (int64_t)(rmax[i] / RB) - rmin[i] / RB + 1;  // row blocks the column touches
    s = (f + ft - 1) / ft;
    if (s > nb) s = nb;
    if (s < 1) s = 1;
  }
  S[i] = s;
}

// one wave per column: task s takes row blocks [b0 + nb*s/S, b0 + nb*(s+1)/S) (clipped to
// [rmin, rmax] at the column's ends); per-task work and roofline units are split in proportion
// to the blocks so that they sum exactly to the column's totals
__global__ __launch_bounds__(256) void task_fill_kernel(const int64_t* __restrict__ tstart, const int64_t* __restrict__ flop,
                                                        const int32_t* __restrict__ rmin, const int32_t* __restrict__ rmax,
                                                        const int64_t* __restrict__ Bcp, int64_t n, int32_t RB,
                                                        int32_t* __restrict__ tcol, int32_t* __restrict__ tlo,
                                                        int32_t* __restrict__ thi, uint8_t* __restrict__ tfull,
                                                        int64_t* __restrict__ twork, int64_t* __restrict__ tunits) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= n) return;
  const int64_t t0 = tstart[c], S = tstart[c + 1] - t0;
  if (S <= 0) return;
  const int64_t f = flop[c], b = Bcp[c + 1] - Bcp[c];
  const int64_t b0 = rmin[c] / RB, nb = (int64_t)(rmax[c] / RB) - b0 + 1;
  for (int64_t s = lane; s < S; s += 64) {
    const int64_t t = t0 + s;
    const int64_t c0 = nb * s / S, c1 = nb * (s + 1) / S;
    tcol[t] = (int32_t)c;
    tlo[t] = s == 0 ? (rmin[c] & ~31) : (int32_t)((b0 + c0) * RB);  // word-aligned start (stored bitmaps)
    thi[t] = s == S - 1 ? rmax[c] + 1 : (int32_t)((b0 + c1) * RB);
    tfull[t] = (uint8_t)((s == 0 ? 1 : 0) | (s == S - 1 ? 2 : 0));
    twork[t] = f * c1 / nb - f * c0 / nb;
    tunits[t] = (b + f) * c1 / nb - (b + f) * c0 / nb;
  }
}

// Row-block table of the hub columns of A (>= kHubMin entries; wave per hub column):
// hub h owns pairs [h*(nblk+2), +nblk+2): pair 0 = the column's start (int64), pair 1 + x =
// (first position of A(:,k), relative to its start, whose row is >= x*RB, the row there or
// kNoRow), for x = 0..nblk. Task and sub-tile boundaries (multiples of
// RB) and the stop search of long segments (task_kernel.h stop_search) read it -- one 8-B load
// gives a cursor and its row; short columns bisect instead. At scale 22: 288 K hub columns (82 %
// of A's entries), 593 MB, instead of a table over all 4.2 M columns.
constexpr int64_t kHubMin = 32;  // (8 / 16 / 64: 132.5 / 131.5 / 130.6 vs 132.2 GFLOP/s at scale 22)
__global__ void hub_flag_kernel(const int64_t* __restrict__ Acp, int64_t ncol, int64_t minlen, int64_t* __restrict__ flag) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < ncol) flag[k] = (Acp[k + 1] - Acp[k]) >= minlen ? 1 : 0;
}
__global__ void hub_index_kernel(const int64_t* __restrict__ flag, const int64_t* __restrict__ pos, int64_t ncol,
                                 int32_t* __restrict__ hidx) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < ncol) hidx[k] = flag[k] ? (int32_t)pos[k] : -1;
}
__global__ __launch_bounds__(256) void hub_fill_kernel(const int64_t* __restrict__ Acp, const int32_t* __restrict__ Air,
                                                       const int32_t* __restrict__ hidx, int64_t ncol, int32_t RB,
                                                       int64_t nblk, int32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= ncol) return;
  const int32_t h = hidx[k];
  if (h < 0) return;
  const int64_t base = Acp[k], len = Acp[k + 1] - base;
  if (lane == 0) reinterpret_cast<int64_t*>(out)[(int64_t)h * (nblk + 2)] = base;  // pair 0: the column start
  int2* o = reinterpret_cast<int2*>(out) + (int64_t)h * (nblk + 2) + 1;
  for (int64_t p = lane; p < len; p += 64) {
    const int32_t r = Air[base + p];
    const int64_t bc = r / RB;
    const int64_t bp = p > 0 ? Air[base + p - 1] / RB : -1;
    for (int64_t x = bp + 1; x <= bc; ++x) o[x] = make_int2((int32_t)p, r);
  }
  const int64_t blast = len > 0 ? Air[base + len - 1] / RB : -1;
  for (int64_t x = blast + 1 + lane; x <= nblk; x += 64) o[x] = make_int2((int32_t)len, kNoRow);
}

// entries of every task that may run chunked (more than the smallest EMAX), else 0
__global__ void chunk_count_kernel(const int32_t* __restrict__ tcol, const int64_t* __restrict__ Bcp, int64_t ntasks,
                                   int64_t emin, int64_t* __restrict__ cnt) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntasks) return;
  const int32_t c = tcol[t];
  const int64_t ne = Bcp[c + 1] - Bcp[c];
  cnt[t] = ne > emin ? ne : 0;
}

__global__ void iota_scaled_kernel(int64_t* __restrict__ x, int64_t n, int64_t k) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = i * k;
}
__global__ void gather_i64_kernel(const int64_t* __restrict__ src, const int64_t* __restrict__ idx, int64_t n,
                                  int64_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}
__global__ void diff_i64_kernel(const int64_t* __restrict__ x, int64_t n, int64_t* __restrict__ d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = x[i + 1] - x[i];
}
__global__ void add_i64_kernel(const int64_t* __restrict__ x, const int64_t* __restrict__ y, int64_t n,
                               int64_t* __restrict__ o) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = x[i] + y[i];
}

// Stored row bitmaps (TaskArgs::bmp): words of every dense CANDIDATE, a large-symbolic task that
// the dense split could choose by its flop estimate (the outputs the split decides on are at most
// the flops, and dense_subtiles only grows with the work), else 0. The symbolic pass writes the
// candidates' bitmaps while it counts; the dense kernel reads them instead of marking rows again.
// When they do not all fit the budget, the candidates with the highest flop density are kept
// (quarter-octave density classes: words per class, then a class threshold).
constexpr int kBmpClasses = 96;
__device__ __forceinline__ int bmp_class(int64_t w, int64_t span) {
  const float x = (float)w * 65536.0f / (float)span;  // flops per 2^16 rows
  const int b = (int)(4.0f * log2f(x > 1.0f ? x : 1.0f));
  return b < kBmpClasses ? b : kBmpClasses - 1;
}
__global__ __launch_bounds__(256) void bmp_count_kernel(const int64_t* __restrict__ twork, const int32_t* __restrict__ tlo,
                                                        const int32_t* __restrict__ thi, int64_t n, int64_t T,
                                                        int64_t capd, int64_t nwb, int64_t minwork, int64_t dr4,
                                                        int64_t cr4, int min_class, int64_t* __restrict__ words,
                                                        unsigned long long* __restrict__ class_words) {
  __shared__ unsigned long long h[kBmpClasses];
  for (int i = threadIdx.x; i < kBmpClasses; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) {
    const int64_t w = twork[t], span = (int64_t)thi[t] - tlo[t];
    const int64_t we = w * 4 / cr4;  // outputs expected of the flops at compression ratio cr4 / 4
    int64_t nw = (w > minwork && span > 0 && dense_subtiles(we, span, T, capd, nwb, dr4) > 0) ? (span + 31) / 32 : 0;
    if (nw > 0) {
      const int b = bmp_class(w, span);
      if (b < min_class) nw = 0;
      else if (class_words) atomicAdd(&h[b], (unsigned long long)nw);
    }
    words[t] = nw;
  }
  __syncthreads();
  if (class_words)
    for (int i = threadIdx.x; i < kBmpClasses; i += blockDim.x)
      if (h[i]) atomicAdd(&class_words[i], h[i]);
}

// numeric tasks split between the dense (bitmap-rank) and the hash kernels: wd / wh = the task's
// output count in the kernel it goes to, 0 in the other. Dense needs a stored bitmap (boff). The
// compression ratio routes the short tasks: a task with few outputs but more than wavemax products
// (cr above wavemax / outputs) goes to the mid workgroup kernel, whose 256 threads share its
// products, instead of one wave (a 64-lane wave would walk them alone: a launch's tail task).
__global__ void dense_split_kernel(const int64_t* __restrict__ tcnt, const int32_t* __restrict__ tlo,
                                   const int32_t* __restrict__ thi, const int64_t* __restrict__ boff,
                                   const int64_t* __restrict__ flops, int64_t n, int64_t T, int64_t capd, int64_t nwb,
                                   int64_t dr4, int64_t smallcap, int64_t wavemax, int enable,
                                   int64_t* __restrict__ wd, int64_t* __restrict__ wh) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int64_t w = tcnt[t];
  const bool d = enable && boff != nullptr && boff[t + 1] > boff[t] && w > smallcap &&
                 dense_subtiles(w, (int64_t)thi[t] - tlo[t], T, capd, nwb, dr4) > 0;
  wd[t] = d ? w : 0;
  wh[t] = d ? 0 : (w > 0 && w <= smallcap && flops && flops[t] > wavemax ? smallcap + 1 : w);
}
#ifndef CBH_SYM_SPLIT4  // (A/B hook) bitmap sub-tiles allowed per hash sub-tile, in quarters
#define CBH_SYM_SPLIT4 4
#endif
// symbolic tasks split between the one-workgroup-per-CU bitmap kernel (dense_kernel.h, SYM) and
// the task kernels: wb / wh = the task's flops in the kernel it goes to, 0 in the other. A large
// task (flops > midcap) runs the bitmap kernel when it stores its bitmap (a dense candidate) or when
// its row bitmap needs no more sub-tiles (of nws_rows rows) than the task kernel's key hash (of
// hashcap keys) would; the small and mid tasks keep their kernels.
__global__ void sym_split_kernel(const int64_t* __restrict__ twork, const int32_t* __restrict__ tlo,
                                 const int32_t* __restrict__ thi, const int64_t* __restrict__ boff, int64_t n,
                                 int64_t midcap, int64_t hashcap, int64_t nws_rows, int64_t* __restrict__ wb,
                                 int64_t* __restrict__ wh) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int64_t w = twork[t], span = (int64_t)thi[t] - tlo[t];
  bool b = false;
  if (w > midcap && span > 0) {
    const bool store = boff != nullptr && boff[t + 1] > boff[t];
    b = store || 4 * ((span + nws_rows - 1) / nws_rows) <= CBH_SYM_SPLIT4 * ((w + hashcap - 1) / hashcap);
  }
  wb[t] = b ? w : 0;
  wh[t] = b ? 0 : w;
}

// share of the free HBM the phase workspace of cbh_spgemm_phased takes (CBH_PHASE_FRAC)
static double phase_frac() {
  static double v = [] {
    const char* e = std::getenv("CBH_PHASE_FRAC");
    return e ? std::atof(e) : 0.5;
  }();
  return v;
}
// compression ratio (quarters) a dense candidate's flops are divided by before the dense test
// (5/4, 6/4, 8/4 and 12/4 measured flat or slower than 4/4)
static int64_t bmp_cr4() {  // CBH_BMP_CR4 overrides (A/B)
  static int64_t v = [] {
    const char* e = std::getenv("CBH_BMP_CR4");
    return e ? std::max<int64_t>(1, std::atoll(e)) : int64_t(4);
  }();
  return v;
}
static double bmp_frac() {
  static double v = [] {
    const char* e = std::getenv("CBH_BMP_FRAC");
    return e ? std::atof(e) : 0.4;
  }();
  return v;
}

// task_kernel launch with optional HIP-event timing (kernel configurations: device/numeric.h;
// measured at scale 22: a 1024-thread workgroup with an 8192-slot table, half the sub-tiles, ran
// 28 % slower than two 512-thread workgroups per CU with 4096 slots)
// `launch` (a hipError_t-returning callable) between two timing events of kernel class `kind`
template <class F>
static int timed_launch(cbh_ctx* ctx, int kind, double bytes, F&& launch) {
  size_t e0 = (size_t)-1;
  if (ctx->timing && kind >= 0) {
    e0 = next_event(ctx);
    if (e0 != (size_t)-1) (void)hipEventRecord(ctx->evpool[e0], ctx->stream);
  }
  CBH_HIP(ctx, launch());
  if (e0 != (size_t)-1) {
    const size_t e1 = next_event(ctx);
    if (e1 != (size_t)-1) {
      (void)hipEventRecord(ctx->evpool[e1], ctx->stream);
      ctx->recs.push_back({kind, e0, e1, bytes});
    }
  }
  return CBH_OK;
}
template <class SR, class CFG, int MODE, bool MERGE = false>
static int launch_task(cbh_ctx* ctx, const TaskArgs& args, int64_t first, int64_t count, int kind = -1,
                       double bytes = 0) {
  if (count <= 0) return CBH_OK;
  return timed_launch(ctx, kind, bytes, [&] { return launch_tasks<SR, CFG, MODE, MERGE>(args, first, count, ctx->stream); });
}

// CBH_DIAG=1: every large sub-bin launched separately with its time printed (profiling aid only)
template <class SR, class CFG, int MODE>
static int launch_task_diag(cbh_ctx* ctx, const TaskArgs& a, const BinLists& bl, const char* what) {
  int64_t first = bl.large_first;
  for (int lg = kSub - 1; lg >= 0; --lg) {
    const int64_t n = bl.sub_count[lg];
    if (!n) continue;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, ctx->stream);
    CBH_TRY((launch_task<SR, CFG, MODE>(ctx, a, first, n)));
    (void)hipEventRecord(e1, ctx->stream);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::fprintf(stderr, "[cbh diag] %s work 2^%d: %lld tasks, %.3f ms\n", what, lg, (long long)n, ms);
#ifdef CBH_STAMPS
    {
      unsigned long long hs[24];
      (void)hipMemcpyFromSymbol(hs, HIP_SYMBOL(g_stamps), sizeof(hs));
      const unsigned long long z[24] = {0};
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z));
      double tot = 0;
      for (int k = 0; k < 12; ++k) tot += (double)hs[k];
      std::fprintf(stderr, "[cbh stamps]   chunk-subtiles=%llu overflows=%llu products=%llu\n", hs[13], hs[14], hs[15]);
      std::fprintf(stderr, "[cbh stamps]   wg=%llu cyc/wg=%.0f  setup %.1f%% clear %.1f%% entries %.1f%% scan %.1f%% own %.1f%% products %.1f%% | ovf-check %.1f%% cursor+count %.1f%% place %.1f%% end-sync %.1f%% | tail %.1f%%\n",
                   hs[12], tot / std::max(1ull, hs[12]), 100 * hs[0] / tot, 100 * hs[1] / tot, 100 * hs[2] / tot,
                   100 * hs[3] / tot, 100 * hs[4] / tot, 100 * hs[5] / tot, 100 * hs[8] / tot, 100 * hs[9] / tot,
                   100 * hs[10] / tot, 100 * hs[6] / tot, 100 * hs[7] / tot);
      char pshare[48] = "n/a: dense windows count no products";  // (products are counted by the hash kernels)
      if (hs[15]) std::snprintf(pshare, sizeof(pshare), "%.1f%%", 100.0 * hs[19] / hs[15]);
      std::fprintf(stderr, "[cbh stamps]   entry-visits=%llu active=%llu (%.1f%%) short=%llu (%.1f%% of active) short-products=%llu (%s) committed=%llu\n",
                   hs[16], hs[17], 100.0 * hs[17] / std::max(1ull, hs[16]), hs[18], 100.0 * hs[18] / std::max(1ull, hs[17]),
                   hs[19], pshare, hs[20]);
    }
#endif
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    first += n;
  }
  return CBH_OK;
}

struct Plan {  // device arrays describing C = A*B (B's nonzero column slots, tasks)
  int64_t nzcB = 0, ntasks = 0;
  int64_t* Adense = nullptr;  // A.n + 1
  int64_t* flop = nullptr;    // nzcB + 1
  int32_t* rmin = nullptr;
  int32_t* rmax = nullptr;
  int64_t* tstart = nullptr;  // nzcB + 1: first task of each column
  int32_t* tcol = nullptr;    // per task
  int32_t* tlo = nullptr;
  int32_t* thi = nullptr;
  uint8_t* tfull = nullptr;
  int64_t* twork = nullptr;   // flops estimate
  int64_t* tunits = nullptr;  // roofline units (B entries + products), later + outputs
  int64_t* tcnt = nullptr;    // ntasks + 1: outputs per task
  int64_t* toff = nullptr;    // ntasks + 1: output offset per task
  int32_t* order = nullptr;   // ntasks: launch order
  int64_t* nnz = nullptr;     // nzcB + 1
  int64_t* Ccp = nullptr;     // nzcB + 1
  int32_t* hidx = nullptr;    // hub row-block table of A (see hub_fill_kernel)
  int32_t* htab = nullptr;
  int64_t nblk = 0;
  int32_t RB = 1;
  int64_t* goff = nullptr;    // ntasks + 1: HBM cursor-state offsets of chunked tasks (null: none)
  int64_t* gcur0 = nullptr;
  int64_t* gcur1 = nullptr;
  int64_t* gend = nullptr;
  int32_t* trk = nullptr;     // per task: row block of its middle row (launch order key)
  int32_t* gnx0 = nullptr;    // row at each committed cursor (double-buffered like gcur)
  int32_t* gnx1 = nullptr;
  int32_t* ghub = nullptr;    // hub id of each chunked entry's A column
  int64_t* gbase = nullptr;   // its start (the stop search's column base)
  int64_t* boff = nullptr;    // ntasks + 1: stored-bitmap word offsets (see bmp_count_kernel)
  uint32_t* bmp = nullptr;    // null: no stored bitmaps (dense kernel off)
  int64_t total_flops = 0, total_nnz = 0;
};

static TaskArgs task_args(const cbh_mat* A, const cbh_mat* B, const Plan& P, cbh_ctx* ctx) {
  TaskArgs a;
  std::memset(&a, 0, sizeof(a));
  a.Acp = P.Adense;
  a.Air = A->ir;
  a.Anum = A->num;
  a.Bcp = B->cp;
  a.Bir = B->ir;
  a.Bnum = B->num;
  a.order = P.order;
  a.hidx = P.hidx;
  a.htab = P.htab;
  a.nblk = P.nblk;
  a.RB = P.htab ? P.RB : 0;
  a.tcol = P.tcol;
  a.tlo = P.tlo;
  a.thi = P.thi;
  a.tfull = P.tfull;
  a.err = ctx->d_err;
  a.nnzA = A->nnz;
  a.ncolA = A->n;
  a.ntasks = P.ntasks;
  a.ccap = INT64_MAX;
  a.goff = P.goff;
  a.gcur0 = P.gcur0;
  a.gcur1 = P.gcur1;
  a.gend = P.gend;
  a.gnx0 = P.gnx0;
  a.gnx1 = P.gnx1;
  a.ghub = P.ghub;
  a.gbase = P.gbase;
  a.boff = P.bmp ? P.boff : nullptr;
  a.bmp = P.bmp;
  return a;
}

// count_only: the caller needs the counts alone (cbh_spgemm_symbolic, EstPerProcessNnzSUMMA), so no
// dense-candidate bitmaps are sized, stored or kept
static int run_symbolic(cbh_ctx* ctx, Scratch& S, const cbh_mat* A, const cbh_mat* B, Plan& P, bool count_only = false) {
  P.nzcB = B->nzc;
  const int64_t n = P.nzcB;
  CBH_TRY(S.get(&P.Adense, A->n + 1));
  CBH_TRY(S.get(&P.flop, n + 1));
  CBH_TRY(S.get(&P.rmin, n));
  CBH_TRY(S.get(&P.rmax, n));
  CBH_TRY(S.get(&P.tstart, n + 1));
  CBH_TRY(S.get(&P.nnz, n + 1));
  CBH_TRY(S.get(&P.Ccp, n + 1));
  int64_t* scnt;
  CBH_TRY(S.get(&scnt, n + 1));
  int64_t* d_tot;
  CBH_TRY(S.get(&d_tot, 3));
  hipLaunchKernelGGL(densify_cp_kernel, dim3(blocks_for(A->n + 1, 256)), dim3(256), 0, ctx->stream, A->jc, A->cp,
                     A->nzc, A->n, A->nnz, P.Adense);
  hipLaunchKernelGGL(flop_kernel, dim3(blocks_for(n, 4)), dim3(256), 0, ctx->stream, P.Adense, A->ir, B->cp, B->ir, n,
                     A->n, P.flop, P.rmin, P.rmax, ctx->d_err);
  CBH_HIP(ctx, hipGetLastError());
  CBH_TRY(sum_i64(ctx, S, P.flop, n, d_tot));
  P.RB = row_block(A->m);
  hipLaunchKernelGGL(task_count_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, P.flop, P.rmin, P.rmax, n,
                     kTaskFlops, P.RB, scnt);
  CBH_HIP(ctx, hipMemsetAsync(scnt + n, 0, sizeof(int64_t), ctx->stream));
  CBH_TRY(exclusive_scan_i64(ctx, S, scnt, P.tstart, n + 1));
  int64_t h[2];
  CBH_HIP(ctx, hipMemcpyAsync(&h[1], P.tstart + n, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipMemcpyAsync(&h[0], d_tot, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  P.total_flops = h[0];
  P.ntasks = h[1];
  if (P.ntasks > INT32_MAX) return fail(ctx, CBH_E_INTERNAL, "more than 2^31 tasks");
  const int64_t nt = std::max<int64_t>(P.ntasks, 1);
  CBH_TRY(S.get(&P.tcol, nt));
  CBH_TRY(S.get(&P.tlo, nt));
  CBH_TRY(S.get(&P.thi, nt));
  CBH_TRY(S.get(&P.tfull, nt));
  CBH_TRY(S.get(&P.twork, nt));
  CBH_TRY(S.get(&P.tunits, nt));
  CBH_TRY(S.get(&P.tcnt, nt + 1));
  CBH_TRY(S.get(&P.toff, nt + 1));
  CBH_TRY(S.get(&P.order, nt));
  CBH_TRY(S.get(&P.trk, nt));
  hipLaunchKernelGGL(task_fill_kernel, dim3(blocks_for(n, 4)), dim3(256), 0, ctx->stream, P.tstart, P.flop, P.rmin,
                     P.rmax, B->cp, n, P.RB, P.tcol, P.tlo, P.thi, P.tfull, P.twork, P.tunits);
  CBH_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(task_rowkey_kernel, dim3(blocks_for(P.ntasks, 256)), dim3(256), 0, ctx->stream, P.tlo, P.thi,
                     P.ntasks, P.RB, P.trk);
  {  // row-block table of A's hub columns: task boundaries and long-segment stops
    int64_t *hflag, *hpos;
    CBH_TRY(S.get(&hflag, A->n + 1));
    CBH_TRY(S.get(&hpos, A->n + 1));
    CBH_TRY(S.get(&P.hidx, std::max<int64_t>(A->n, 1)));
    hipLaunchKernelGGL(hub_flag_kernel, dim3(blocks_for(A->n, 256)), dim3(256), 0, ctx->stream, P.Adense, A->n, kHubMin,
                       hflag);
    CBH_HIP(ctx, hipMemsetAsync(hflag + A->n, 0, sizeof(int64_t), ctx->stream));
    CBH_TRY(exclusive_scan_i64(ctx, S, hflag, hpos, A->n + 1));
    int64_t nhub = 0;
    CBH_HIP(ctx, hipMemcpyAsync(&nhub, hpos + A->n, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (nhub > 0) {
      P.nblk = (A->m + P.RB - 1) / P.RB;
      hipLaunchKernelGGL(hub_index_kernel, dim3(blocks_for(A->n, 256)), dim3(256), 0, ctx->stream, hflag, hpos, A->n,
                         P.hidx);
      CBH_TRY(S.get(&P.htab, 2 * (size_t)nhub * (size_t)(P.nblk + 2)));  // start + (position, row) pairs
      hipLaunchKernelGGL(hub_fill_kernel, dim3(blocks_for(A->n, 4)), dim3(256), 0, ctx->stream, P.Adense, A->ir, P.hidx,
                         A->n, P.RB, P.nblk, P.htab);
      CBH_HIP(ctx, hipGetLastError());
    }
  }
  {  // HBM cursor state for tasks with more B entries than the smallest chunk (EMAX)
    int64_t* gcnt;
    CBH_TRY(S.get(&gcnt, nt + 1));
    CBH_TRY(S.get(&P.goff, nt + 1));
    hipLaunchKernelGGL(chunk_count_kernel, dim3(blocks_for(nt, 256)), dim3(256), 0, ctx->stream, P.tcol, B->cp,
                       P.ntasks, (int64_t)kChunkMin, gcnt);
    CBH_HIP(ctx, hipGetLastError());
    CBH_HIP(ctx, hipMemsetAsync(gcnt + P.ntasks, 0, sizeof(int64_t), ctx->stream));
    CBH_TRY(exclusive_scan_i64(ctx, S, gcnt, P.goff, P.ntasks + 1));
    int64_t gtot = 0;
    CBH_HIP(ctx, hipMemcpyAsync(&gtot, P.goff + P.ntasks, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (gtot > 0) {
      CBH_TRY(S.get(&P.gcur0, (size_t)gtot));
      CBH_TRY(S.get(&P.gcur1, (size_t)gtot));
      CBH_TRY(S.get(&P.gend, (size_t)gtot));
      CBH_TRY(S.get(&P.gnx0, (size_t)gtot));
      CBH_TRY(S.get(&P.gnx1, (size_t)gtot));
      CBH_TRY(S.get(&P.ghub, (size_t)gtot));
      CBH_TRY(S.get(&P.gbase, (size_t)gtot));
    } else {
      P.goff = nullptr;
    }
  }
  if (!count_only) {  // stored row bitmaps of the dense candidates, within CBH_BMP_FRAC (default 0.4) of the HBM
    using CD = TaskCfg<PlusTimesD<double>, kSplitHashT, TNumLarge::BS, TNumLarge::EMAX, TNumLarge::U, MODE_TDENSE>;  // split pricing
    int64_t* bw;
    unsigned long long* cw;
    CBH_TRY(S.get(&bw, nt + 1));
    CBH_TRY(S.get(&cw, kBmpClasses));
    CBH_TRY(S.get(&P.boff, nt + 1));
    CBH_HIP(ctx, hipMemsetAsync(cw, 0, sizeof(unsigned long long) * kBmpClasses, ctx->stream));
    hipLaunchKernelGGL(bmp_count_kernel, dim3(blocks_for(nt, 256)), dim3(256), 0, ctx->stream, P.twork, P.tlo, P.thi,
                       P.ntasks, kSplitHashT, (int64_t)CD::CAPD, (int64_t)CD::NWB, kSymMidCap, (int64_t)kDRatio4,
                       bmp_cr4(), 0, bw, cw);
    CBH_HIP(ctx, hipGetLastError());
    unsigned long long hc[kBmpClasses];
    CBH_HIP(ctx, hipMemcpyAsync(hc, cw, sizeof(hc), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    size_t freeb = 0, totb = 0;
    CBH_HIP(ctx, hipMemGetInfo(&freeb, &totb));
    // within a fraction of the device (not of what is free: later calls find the earlier call's
    // bitmaps in the block cache and the phase workspace resident), densest classes first
    const double frac = ctx->bmp_frac >= 0 ? ctx->bmp_frac : bmp_frac();
    const double cap_words = std::min(frac * (double)totb, 0.9 * (double)(freeb + ctx->cached_bytes)) / 4.0;
    double words = 0;
    int min_class = kBmpClasses;
    while (min_class > 0 && words + (double)hc[min_class - 1] <= cap_words) words += (double)hc[--min_class];
    if (min_class > 0 && words > 0)  // drop the classes that did not fit
      hipLaunchKernelGGL(bmp_count_kernel, dim3(blocks_for(nt, 256)), dim3(256), 0, ctx->stream, P.twork, P.tlo, P.thi,
                         P.ntasks, kSplitHashT, (int64_t)CD::CAPD, (int64_t)CD::NWB, kSymMidCap, (int64_t)kDRatio4,
                         bmp_cr4(), min_class, bw, nullptr);
    CBH_HIP(ctx, hipMemsetAsync(bw + P.ntasks, 0, sizeof(int64_t), ctx->stream));
    CBH_TRY(exclusive_scan_i64(ctx, S, bw, P.boff, P.ntasks + 1));
    if (words > 0) CBH_TRY(S.get(&P.bmp, (size_t)words));
    if (diag_enabled()) {
      double all = 0;
      for (int i = 0; i < kBmpClasses; ++i) all += (double)hc[i];
      std::fprintf(stderr, "[cbh diag] stored bitmaps: %.3f of %.3f GB (density classes >= %d)\n", words * 4e-9,
                   all * 4e-9, min_class);
    }
  }
  CBH_HIP(ctx, hipMemsetAsync(P.tcnt, 0, sizeof(int64_t) * (nt + 1), ctx->stream));
  BinLists bl, bb;
#if CBH_SYM_V2
  {  // the large bitmap tasks to the one-workgroup-per-CU kernel, the rest to the task kernels
    using CS = DenseCfg<PlusTimesD<int64_t>, TSym2::BS, TSym2::EL, TSym2::U, TSym2::LDSB, KSYMB>;
    constexpr int64_t kHashKeys = (int64_t)kSymWords * kSymFill8 / 8;  // TSymLarge's key-hash capacity
    int64_t *wb, *wh;
    CBH_TRY(S.get(&wb, nt));
    CBH_TRY(S.get(&wh, nt));
    hipLaunchKernelGGL(sym_split_kernel, dim3(blocks_for(P.ntasks, 256)), dim3(256), 0, ctx->stream, P.twork, P.tlo,
                       P.thi, P.bmp ? P.boff : nullptr, P.ntasks, (int64_t)kSymMidCap, kHashKeys, 32ll * CS::NWS, wb,
                       wh);
    CBH_HIP(ctx, hipGetLastError());
    CBH_TRY(make_bins(ctx, S, wh, P.ntasks, 0, P.order, &bl, BinCaps{kSymWaveCap, kSymMidCap}, P.tunits, P.trk));
    const int64_t nh = bl.small_count + bl.mid_count + bl.large_count;
    CBH_TRY(make_bins(ctx, S, wb, P.ntasks, 0, P.order + nh, &bb, BinCaps{kSymWaveCap, kSymMidCap}, P.tunits, P.trk));
    bb.large_first += nh;  // (wb holds large tasks only)
  }
#else
  CBH_TRY(make_bins(ctx, S, P.twork, P.ntasks, 0, P.order, &bl, BinCaps{kSymWaveCap, kSymMidCap}, P.tunits, P.trk));
#endif
  TaskArgs a = task_args(A, B, P, ctx);
  a.twork = P.twork;
  a.cnt = P.tcnt;
  using Dummy = PlusTimesD<int64_t>;
  // algorithmic bytes of the symbolic pass: row ids of B and of every gathered A entry + pointers
  const double sb_l = 4.0 * bl.units[2] + 16.0 * bl.large_count;
  const double sb_s = 4.0 * bl.units[0] + 16.0 * bl.small_count;
  const double sb_m = 4.0 * bl.units[1] + 16.0 * bl.mid_count;
  const double sb_b = 4.0 * bb.units[2] + 16.0 * bb.large_count;
  if (bb.large_count > 0)
    CBH_TRY(timed_launch(ctx, CBH_K_SYM_BMP, sb_b, [&] {
      return launch_dense<Dummy, TSym2::BS, TSym2::EL, TSym2::U, TSym2::LDSB, KSYMB>(a, bb.large_first, bb.large_count,
                                                                                     ctx->stream);
    }));
  if (diag_enabled()) CBH_TRY((launch_task_diag<Dummy, TSymLarge, MODE_TSYM>(ctx, a, bl, "symbolic")));
  else CBH_TRY((launch_task<Dummy, TSymLarge, MODE_TSYM>(ctx, a, bl.large_first, bl.large_count, CBH_K_SYM_LARGE, sb_l)));
  CBH_TRY((launch_task<Dummy, TSymMid, MODE_TSYM>(ctx, a, bl.mid_first, bl.mid_count, CBH_K_SYM_MID, sb_m)));
  if (bl.small_count > 0)  // one task per wave (wave_kernel.h)
    CBH_TRY(timed_launch(ctx, CBH_K_SYM_SMALL, sb_s, [&] {
      return launch_waves<Dummy, WSymSmall::TW, WSymSmall::WPB, WSymSmall::U, MODE_TSYM>(a, bl.small_first, bl.small_count,
                                                                                        ctx->stream);
    }));
  // task offsets -> column pointers of C
  CBH_TRY(exclusive_scan_i64(ctx, S, P.tcnt, P.toff, P.ntasks + 1));
  hipLaunchKernelGGL(gather_i64_kernel, dim3(blocks_for(n + 1, 256)), dim3(256), 0, ctx->stream, P.toff, P.tstart,
                     n + 1, P.Ccp);
  hipLaunchKernelGGL(diff_i64_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, P.Ccp, n, P.nnz);
  CBH_HIP(ctx, hipMemsetAsync(P.nnz + n, 0, sizeof(int64_t), ctx->stream));
  // roofline units of the numeric pass: + outputs
  hipLaunchKernelGGL(add_i64_kernel, dim3(blocks_for(P.ntasks, 256)), dim3(256), 0, ctx->stream, P.tunits, P.tcnt,
                     P.ntasks, P.tunits);
  CBH_HIP(ctx, hipGetLastError());
  CBH_HIP(ctx, hipMemcpyAsync(&h[1], P.Ccp + n, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  P.total_nnz = h[1];
  return check_err(ctx);
}

// numeric over the tasks of column slots [c0, c1) (task ids [t0, t1)) writing C entries at toff-cbase
template <class SR>
static int run_numeric(cbh_ctx* ctx, Scratch& S, const cbh_mat* A, const cbh_mat* B, Plan& P, int64_t t0, int64_t t1,
                       int64_t cbase, int32_t* Cir, void* Cnum, int64_t* launches, int64_t ccap) {
  if (t1 <= t0) return CBH_OK;
  // tasks whose sub-tiles fit a bitmap run the dense (bitmap-rank) kernel, the rest the hash
  // kernels (task_kernel.h dense_subtiles: the same plan the kernel re-derives)
  using CD = TaskCfg<SR, kSplitHashT, TNumLarge::BS, TNumLarge::EMAX, TNumLarge::U, MODE_TDENSE>;  // split pricing
  const int64_t nt = t1 - t0;
  int64_t *wd, *wh;
  CBH_TRY(S.get(&wd, nt));
  CBH_TRY(S.get(&wh, nt));
  hipLaunchKernelGGL(dense_split_kernel, dim3(blocks_for(nt, 256)), dim3(256), 0, ctx->stream, P.tcnt + t0, P.tlo + t0,
                     P.thi + t0, P.bmp ? P.boff + t0 : nullptr, P.twork + t0, nt, kSplitHashT, (int64_t)CD::CAPD,
                     (int64_t)CD::NWB, (int64_t)kDRatio4, kSmallCap, kWaveProducts,
                     1, wd, wh);
  CBH_HIP(ctx, hipGetLastError());
  BinLists bd, bl;
  CBH_TRY(make_bins(ctx, S, wd, nt, t0, P.order, &bd, BinCaps{kSmallCap, kSmallCap}, P.tunits + t0, P.trk + t0));
  const int64_t nd = bd.small_count + bd.mid_count + bd.large_count;
  CBH_TRY(make_bins(ctx, S, wh, nt, t0, P.order + nd, &bl, BinCaps{kSmallCap, kMidCap}, P.tunits + t0, P.trk + t0));
  bl.small_first += nd;
  bl.mid_first += nd;
  bl.large_first += nd;
  TaskArgs a = task_args(A, B, P, ctx);
  a.twork = P.tcnt;
  a.toff = P.toff;
  a.cbase = cbase;
  a.Cir = Cir;
  a.Cnum = Cnum;
  a.ccap = ccap;
  // algorithmic bytes: (s_i+s_v) * (nnz(B) + flops + nnz(C)) + pointers
  constexpr double eb = 4.0 + sizeof(typename SR::val_t);
  const double nb_d = eb * bd.units[2] + 16.0 * bd.large_count;
  const double nb_l = eb * bl.units[2] + 16.0 * bl.large_count;
  const double nb_s = eb * bl.units[0] + 16.0 * bl.small_count;
  const double nb_m = eb * bl.units[1] + 16.0 * bl.mid_count;
  if (diag_enabled()) {
    {  // per numeric bin: tasks, outputs, products (flop estimate), compression ratio, rows spanned
      std::vector<int64_t> hd(nt), hh(nt), hc(nt), hw(nt);
      std::vector<int32_t> hlo(nt), hhi(nt);
      CBH_HIP(ctx, hipMemcpyAsync(hd.data(), wd, nt * 8, hipMemcpyDeviceToHost, ctx->stream));
      CBH_HIP(ctx, hipMemcpyAsync(hh.data(), wh, nt * 8, hipMemcpyDeviceToHost, ctx->stream));
      CBH_HIP(ctx, hipMemcpyAsync(hc.data(), P.tcnt + t0, nt * 8, hipMemcpyDeviceToHost, ctx->stream));
      CBH_HIP(ctx, hipMemcpyAsync(hw.data(), P.twork + t0, nt * 8, hipMemcpyDeviceToHost, ctx->stream));
      CBH_HIP(ctx, hipMemcpyAsync(hlo.data(), P.tlo + t0, nt * 4, hipMemcpyDeviceToHost, ctx->stream));
      CBH_HIP(ctx, hipMemcpyAsync(hhi.data(), P.thi + t0, nt * 4, hipMemcpyDeviceToHost, ctx->stream));
      std::vector<int64_t> hb(P.bmp ? nt + 1 : 0);
      if (P.bmp) CBH_HIP(ctx, hipMemcpyAsync(hb.data(), P.boff + t0, (nt + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
      CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
      if (P.bmp) {  // stored bitmap words the numeric split uses, and those of tasks it sends to hash
        double used = 0, unused = 0, unused_tasks = 0;
        for (int64_t t = 0; t < nt; ++t) {
          const double w = (double)(hb[t + 1] - hb[t]);
          if (w <= 0) continue;
          if (hd[t] > 0) used += w;
          else unused += w, unused_tasks += 1;
        }
        std::fprintf(stderr, "[cbh diag] stored bitmap words: dense %.4g GB, to hash %.4g GB (%.0f tasks)\n",
                     used * 4e-9, unused * 4e-9, unused_tasks);
      }
      const char* names[4] = {"wave (<=256 out)", "mid (<=1024 out)", "hash large", "dense"};
      double st[4][4] = {{0}};  // tasks, outputs, flops, span
      for (int64_t t = 0; t < nt; ++t) {
        int k;
        if (hd[t] > 0) k = 3;
        else if (hh[t] <= 0) continue;
        else k = hh[t] <= kSmallCap ? 0 : (hh[t] <= kMidCap ? 1 : 2);
        st[k][0] += 1;
        st[k][1] += (double)hc[t];
        st[k][2] += (double)hw[t];
        st[k][3] += (double)(hhi[t] - hlo[t]);
      }
      for (int k = 0; k < 4; ++k)
        if (st[k][0] > 0)
          std::fprintf(stderr, "[cbh diag] bin %-17s tasks %.0f outputs %.4g flops %.4g cr %.2f out/task %.0f density %.3g%%\n",
                       names[k], st[k][0], st[k][1], st[k][2], st[k][2] / std::max(1.0, st[k][1]),
                       st[k][1] / st[k][0], 100.0 * st[k][1] / std::max(1.0, st[k][3]));
    }
#if CBH_DENSE_V2
    CBH_TRY(timed_launch(ctx, CBH_K_NUM_DENSE, nb_d, [&] {
      return launch_dense_numeric<SR>(a, bd.large_first, bd.large_count, ctx->stream);
    }));
#else
    CBH_TRY((launch_task_diag<SR, TNumLarge, MODE_TDENSE>(ctx, a, bd, "numeric dense")));
#endif
    CBH_TRY((launch_task_diag<SR, TNumHash, MODE_TNUM>(ctx, a, bl, "numeric hash")));
  }
  if (!diag_enabled()) {
    if (bd.large_count > 0)
      CBH_TRY(timed_launch(ctx, CBH_K_NUM_DENSE, nb_d, [&] {
        return launch_dense_numeric<SR>(a, bd.large_first, bd.large_count, ctx->stream);
      }));
#if CBH_HASH_V2
    if (bl.large_count > 0)
      CBH_TRY(timed_launch(ctx, CBH_K_NUM_LARGE, nb_l, [&] {
        return launch_dense<SR, THash2::BS, THash2::EL, THash2::U, THash2::LDSB, KHASH>(a, bl.large_first,
                                                                                        bl.large_count, ctx->stream);
      }));
#else
    CBH_TRY((launch_task<SR, TNumHash, MODE_TNUM>(ctx, a, bl.large_first, bl.large_count, CBH_K_NUM_LARGE, nb_l)));
#endif
  }
  CBH_TRY((launch_task<SR, TNumMid, MODE_TNUM>(ctx, a, bl.mid_first, bl.mid_count, CBH_K_NUM_MID, nb_m)));
  if (bl.small_count > 0)  // one task per wave (wave_kernel.h)
    CBH_TRY(timed_launch(ctx, CBH_K_NUM_SMALL, nb_s, [&] {
      return launch_small_numeric<SR, TNumSmall>(a, bl.small_first, bl.small_count, ctx->stream);
    }));
  if (launches) *launches += (bd.large_count > 0);
  if (launches) *launches += (bl.large_count > 0) + (bl.mid_count > 0) + (bl.small_count > 0);
  return CBH_OK;
}

// The reference-order pass (device/order_kernel.h) over C's tasks after the throughput pass
template <class SR>
static int run_reference_order(cbh_ctx* ctx, Scratch& S, const cbh_mat* A, const cbh_mat* B, Plan& P, cbh_mat* out,
                               uint32_t flags) {
  const int branch = (flags & CBH_ORDER_HEAP) ? 1 : ((flags & CBH_ORDER_HASH) ? 2 : 0);
  TaskArgs a = task_args(A, B, P, ctx);
  a.twork = P.tcnt;
  a.toff = P.toff;
  a.cbase = 0;
  a.Cir = out->ir;
  a.Cnum = out->num;
  a.ccap = P.total_nnz;
  unsigned char* scratch;
  CBH_TRY(S.get(&scratch, (int64_t)ord_scratch_bytes<SR>(B->nnz, P.ntasks, P.total_nnz)));
  CBH_HIP(ctx, (launch_reference_order<Ordered<SR>>(a, scratch, B->nnz, P.total_nnz, branch, ctx->stream)));
  return check_err(ctx);
}

// ============================================================================ semiring dispatch
template <class F>
static int dispatch_sr(cbh_ctx* ctx, cbh_semiring sr, int dtype, F&& f) {
  switch (sr) {
    case CBH_SR_PLUS_TIMES:
      if (dtype == CBH_F64) return f(PlusTimesD<double>{});
      if (dtype == CBH_I64) return f(PlusTimesD<int64_t>{});
      if (dtype == CBH_F32) return f(PlusTimesD<float>{});
      if (dtype == CBH_I32) return f(PlusTimesD<int32_t>{});
      if (dtype == CBH_BOOL) return f(OrAndD{});
      break;
    case CBH_SR_SELECT_MAX:
      if (dtype == CBH_F64) return f(SelectMaxD<double>{});
      if (dtype == CBH_I64) return f(SelectMaxD<int64_t>{});
      break;
    case CBH_SR_MIN_PLUS:
      if (dtype == CBH_F64) return f(MinPlusD<double>{});
      if (dtype == CBH_I64) return f(MinPlusD<int64_t>{});
      break;
    case CBH_SR_OR_AND:
      if (dtype == CBH_BOOL) return f(OrAndD{});
      break;
    default:
      break;
  }
  return fail(ctx, CBH_E_ARG, "unsupported semiring/dtype combination (sr=" + std::to_string((int)sr) +
                                  ", dtype=" + std::to_string(dtype) + ")");
}

static int new_mat(cbh_ctx* ctx, int64_t m, int64_t n, int64_t nnz, int64_t nzc, int dtype, cbh_mat** out,
                   int64_t vbytes = 0) {
  cbh_mat* M = new cbh_mat;
  M->m = m;
  M->n = n;
  M->nnz = nnz;
  M->nzc = nzc;
  M->dtype = dtype;
  M->vbytes = vbytes > 0 ? vbytes : (int64_t)dtype_size(dtype);
  int rc = dalloc(ctx, &M->cp, nzc + 1);
  if (rc == CBH_OK) rc = dalloc(ctx, &M->jc, nzc);
  if (rc == CBH_OK) rc = dalloc(ctx, &M->ir, nnz);
  if (rc == CBH_OK) rc = dalloc(ctx, reinterpret_cast<char**>(&M->num), nnz * M->vbytes);
  if (rc != CBH_OK) {
    cbh_mat_free(ctx, M);
    return rc;
  }
  *out = M;
  return CBH_OK;
}

// C's allocation once the symbolic pass knows nnz(C). The dense candidates' stored bitmaps were
// sized before nnz(C) was known (up to CBH_BMP_FRAC of the device): when C does not fit beside
// them, they are dropped -- every task then runs on the hash kernels -- and C is allocated again.
static int new_result(cbh_ctx* ctx, Scratch& S, Plan& P, int64_t m, int64_t n, int64_t nnz, int64_t nzc, int dtype,
                      cbh_mat** out, int64_t vbytes = 0) {
  int rc = new_mat(ctx, m, n, nnz, nzc, dtype, out, vbytes);
  if (rc == CBH_OK && P.bmp != nullptr && std::getenv("CBH_TEST_RESULT_OOM")) {  // test hook: the fallback below
    cbh_mat_free(ctx, *out);
    *out = nullptr;
    rc = fail(ctx, CBH_E_OOM, "CBH_TEST_RESULT_OOM");
  }
  if (rc != CBH_E_OOM || P.bmp == nullptr) return rc;
  S.drop(P.bmp);
  P.bmp = nullptr;
  release_cache(ctx);
  if (diag_enabled()) std::fprintf(stderr, "[cbh diag] C does not fit beside the stored bitmaps: dense windows off\n");
  return new_mat(ctx, m, n, nnz, nzc, dtype, out, vbytes);
}

static int empty_result(cbh_ctx* ctx, int64_t m, int64_t n, int dtype, cbh_mat** C) {
  CBH_TRY(new_mat(ctx, m, n, 0, 0, dtype, C));
  CBH_HIP(ctx, hipMemsetAsync((*C)->cp, 0, sizeof(int64_t), ctx->stream));
  return CBH_OK;
}

static int validate_pair(cbh_ctx* ctx, const cbh_mat* A, const cbh_mat* B) {
  if (!ctx || !A || !B) return fail(ctx, CBH_E_ARG, "null argument");
  if (A == B) return fail(ctx, CBH_E_MATRIXALIAS, "A and B alias (ParFriends.h:172-179)");
  if (A->n != B->m) return fail(ctx, CBH_E_DIMMISMATCH, "A.getncol() != B.getnrow()");
  if (A->dtype != B->dtype) return fail(ctx, CBH_E_ARG, "A and B dtypes differ");
  if (A->m > INT32_MAX) return fail(ctx, CBH_E_DIMMISMATCH, "local row count exceeds 32-bit row ids");
  return CBH_OK;
}

static void ev_record(cbh_ctx* ctx, int i) {
  if (ctx->timing) (void)hipEventRecord(ctx->ev[i], ctx->stream);
}
static float ev_ms(cbh_ctx* ctx, int a, int b) {
  float ms = -1;
  if (ctx->timing) (void)hipEventElapsedTime(&ms, ctx->ev[a], ctx->ev[b]);
  return ms;
}

// ============================================================================ C-ABI
extern "C" {

const char* cbh_version(void) { return "combblas_hip 0.1 (gfx950)"; }

int cbh_device_count(int* n) {
  if (!n) return CBH_E_ARG;
  *n = 0;
  if (hipGetDeviceCount(n) != hipSuccess || *n <= 0) {
    *n = 0;
    return CBH_E_NODEVICE;
  }
  return CBH_OK;
}

int cbh_device_pci_id(int device, char* buf, int len) {
  if (!buf || len < 13) return CBH_E_ARG;
  return hipDeviceGetPCIBusId(buf, len, device) == hipSuccess ? CBH_OK : CBH_E_HIP;
}

int cbh_ctx_device(cbh_ctx* ctx, int* device) {
  if (!ctx || !device) return CBH_E_ARG;
  *device = ctx->device;
  return CBH_OK;
}

int cbh_ctx_create(int device, cbh_ctx** out) {
  if (!out) return CBH_E_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return CBH_E_NODEVICE;
  if (device < 0 || device >= ndev) return CBH_E_ARG;
  cbh_ctx* c = new cbh_ctx;
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return CBH_E_HIP;
  }
  c->own_stream = true;
  if (const char* v = std::getenv("CBH_ALLOC_POISON")) c->poison = std::atoi(v) != 0;
  {
    size_t freeb = 0, totb = 0;
    // 0.9 of the device: a phased near-capacity driver (C5's C++ MemEfficientSpGEMM) reuses its
    // 190 GB output arena and phase blocks from step to step (0.5 re-mapped ~130 GB per step, 3 s;
    // 0.85 still re-mapped ~60 GB: 8.3 s per step against 2.8 s at 0.9); other
    // allocators get memory back through the OOM path (largest cached blocks first) and the RCCL
    // setup (releases what it needs when less than 8 GB is free)
    if (hipMemGetInfo(&freeb, &totb) == hipSuccess && totb > 0) c->cache_cap = totb / 10 * 9;
  }
  if (const char* v = std::getenv("CBH_CACHE_CAP_GB")) c->cache_cap = size_t(std::atof(v) * double(size_t(1) << 30));
  for (auto& e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) {
      delete c;
      return CBH_E_HIP;
    }
  if (hipMalloc(&c->d_err, 32 * sizeof(int)) != hipSuccess || hipMemset(c->d_err, 0, 32 * sizeof(int)) != hipSuccess) {
    delete c;
    return CBH_E_HIP;
  }
  *out = c;
  return CBH_OK;
}

int cbh_ctx_destroy(cbh_ctx* ctx) {
  if (!ctx) return CBH_OK;
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->d_err) (void)hipFree(ctx->d_err);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : ctx->evpool) (void)hipEventDestroy(e);
  if (ctx->ws) (void)hipFree(ctx->ws);
  if (ctx->pin) (void)hipHostFree(ctx->pin);
  for (auto& e : ctx->pin_ev)
    if (e) (void)hipEventDestroy(e);
  release_cache(ctx);
  for (auto& kv : ctx->live) (void)hipFree(kv.first);  // matrices not freed by the caller
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return CBH_OK;
}

int cbh_ctx_set_stream(cbh_ctx* ctx, void* s) {
  if (!ctx) return CBH_E_ARG;
  if (ctx->own_stream) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamDestroy(ctx->stream);
    ctx->own_stream = false;
  }
  if (s) {
    ctx->stream = reinterpret_cast<hipStream_t>(s);
  } else {
    CBH_HIP(ctx, hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    ctx->own_stream = true;
  }
  return CBH_OK;
}

void* cbh_ctx_stream(cbh_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

int cbh_ctx_synchronize(cbh_ctx* ctx) {
  if (!ctx) return CBH_E_ARG;
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return CBH_OK;
}

int cbh_ctx_trim(cbh_ctx* ctx) {
  if (!ctx) return CBH_E_ARG;
  release_cache(ctx);
  if (ctx->ws) {
    (void)hipFree(ctx->ws);
    ctx->ws = nullptr;
    ctx->ws_bytes = 0;
  }
  CBH_HIP(ctx, hipGetLastError());
  return CBH_OK;
}

int cbh_ctx_release(cbh_ctx* ctx, int64_t bytes) {
  if (!ctx || bytes < 0) return CBH_E_ARG;
  shrink_cache(ctx, ctx->cached_bytes > (size_t)bytes ? ctx->cached_bytes - (size_t)bytes : 0);
  CBH_HIP(ctx, hipGetLastError());
  return CBH_OK;
}

const char* cbh_last_error(cbh_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int cbh_ctx_alloc(cbh_ctx* ctx, int64_t bytes, void** p) {
  if (!ctx || !p || bytes < 0) return CBH_E_ARG;
  *p = nullptr;
  unsigned char* q = nullptr;
  CBH_TRY(dalloc(ctx, &q, (size_t)(bytes > 0 ? bytes : 1)));
  *p = q;
  return CBH_OK;
}

int cbh_ctx_free(cbh_ctx* ctx, void* p) {
  if (!ctx) return CBH_E_ARG;
  if (p) dfree(ctx, p);
  return CBH_OK;
}

int cbh_hash_config(int64_t* table_slots, int64_t* threads, int64_t* per_thread) {
#if CBH_HASH_V2
  using CH = DenseCfg<PlusTimesD<double>, THash2::BS, THash2::EL, THash2::U, THash2::LDSB, KHASH>;
  if (table_slots) *table_slots = CH::TH;
  if (threads) *threads = THash2::BS;
  if (per_thread) *per_thread = THash2::U;
#else
  if (table_slots) *table_slots = TNumHash::T;
  if (threads) *threads = TNumHash::BS;
  if (per_thread) *per_thread = TNumHash::U;
#endif
  return CBH_OK;
}

int cbh_ctx_memory(cbh_ctx* ctx, int64_t* live_bytes, int64_t* cached_bytes, int64_t* device_free,
                   int64_t* device_total) {
  if (!ctx) return CBH_E_ARG;
  size_t live = 0;
  for (auto& kv : ctx->live) live += kv.second;
  size_t fr = 0, tot = 0;
  CBH_HIP(ctx, hipMemGetInfo(&fr, &tot));
  if (live_bytes) *live_bytes = (int64_t)live;
  if (cached_bytes) *cached_bytes = (int64_t)ctx->cached_bytes;
  if (device_free) *device_free = (int64_t)fr;
  if (device_total) *device_total = (int64_t)tot;
  return CBH_OK;
}

int cbh_ctx_take_retries(cbh_ctx* ctx, int64_t* subtile_retries) {
  if (!ctx || !subtile_retries) return CBH_E_ARG;
  int h = 0;
  CBH_HIP(ctx, hipMemcpyAsync(&h, ctx->d_err + 16, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipMemsetAsync(ctx->d_err + 16, 0, sizeof(int), ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  *subtile_retries = h;
  return CBH_OK;
}

int cbh_ctx_set_allocator(cbh_ctx* ctx, cbh_alloc_fn alloc, cbh_free_fn release, void* user) {
  if (!ctx || (alloc == nullptr) != (release == nullptr)) return CBH_E_ARG;
  ctx->alloc = alloc;
  ctx->release = release;
  ctx->alloc_user = user;
  return CBH_OK;
}

int cbh_ctx_set_phase_consumer(cbh_ctx* ctx, cbh_phase_fn fn, void* user) {
  if (!ctx) return CBH_E_ARG;
  ctx->phase_fn = fn;
  ctx->phase_user = user;
  return CBH_OK;
}

int cbh_ctx_set_phase_budget(cbh_ctx* ctx, int64_t bytes) {
  if (!ctx || bytes < 0) return CBH_E_ARG;
  ctx->phase_budget = bytes;
  return CBH_OK;
}

int cbh_ctx_set_bitmap_fraction(cbh_ctx* ctx, double frac) {
  if (!ctx || frac > 1.0) return CBH_E_ARG;
  ctx->bmp_frac = frac;
  return CBH_OK;
}

int cbh_kernel_stats(cbh_ctx* ctx, int kind, cbh_kernel_stat* out) {
  if (!ctx || !out || kind < 0 || kind >= CBH_K_NKINDS) return CBH_E_ARG;
  out->ms = ctx->k_ms[kind];
  out->launches = ctx->k_launch[kind];
  out->alg_bytes = ctx->k_bytes[kind];
  return CBH_OK;
}

int cbh_kernel_stats_reset(cbh_ctx* ctx) {
  if (!ctx) return CBH_E_ARG;
  for (int k = 0; k < CBH_K_NKINDS; ++k) {
    ctx->k_ms[k] = 0;
    ctx->k_launch[k] = 0;
    ctx->k_bytes[k] = 0;
  }
  return CBH_OK;
}

int cbh_ctx_enable_timing(cbh_ctx* ctx, int enable) {
  if (!ctx) return CBH_E_ARG;
  ctx->timing = enable != 0;
  return CBH_OK;
}

int cbh_last_kernel_times(cbh_ctx* ctx, cbh_kernel_times* t) {
  if (!ctx || !t) return CBH_E_ARG;
  *t = ctx->times;
  return CBH_OK;
}

int cbh_mat_upload(cbh_ctx* ctx, const cbh_dcsc* h, cbh_dtype dtype, cbh_mat** out) {
  if (!ctx || !h || !out || dtype_size(dtype) == 0) return fail(ctx, CBH_E_ARG, "bad upload arguments");
  if (h->nnz < 0 || h->nzc < 0 || h->m < 0 || h->n < 0) return fail(ctx, CBH_E_DIMMISMATCH, "negative sizes");
  cbh_mat* M;
  CBH_TRY(new_mat(ctx, h->m, h->n, h->nnz, h->nzc, dtype, &M));
  const size_t vs = dtype_size(dtype);
  if (h->nzc > 0) {
    CBH_HIP(ctx, hipMemcpyAsync(M->cp, h->cp, sizeof(int64_t) * (h->nzc + 1), hipMemcpyHostToDevice, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(M->jc, h->jc, sizeof(int64_t) * h->nzc, hipMemcpyHostToDevice, ctx->stream));
  } else {
    CBH_HIP(ctx, hipMemsetAsync(M->cp, 0, sizeof(int64_t), ctx->stream));
  }
  if (h->nnz > 0) {
    CBH_HIP(ctx, hipMemcpyAsync(M->ir, h->ir, sizeof(int32_t) * h->nnz, hipMemcpyHostToDevice, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(M->num, h->num, vs * h->nnz, hipMemcpyHostToDevice, ctx->stream));
  }
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // host buffers may be released on return
  *out = M;
  return CBH_OK;
}

int cbh_mat_wrap_device(cbh_ctx* ctx, const cbh_dcsc* d, cbh_dtype dtype, cbh_mat** out) {
  if (!ctx || !d || !out || dtype_size(dtype) == 0) return fail(ctx, CBH_E_ARG, "bad wrap arguments");
  cbh_mat* M = new cbh_mat;
  M->m = d->m;
  M->n = d->n;
  M->nnz = d->nnz;
  M->nzc = d->nzc;
  M->dtype = dtype;
  M->vbytes = (int64_t)dtype_size(dtype);
  M->cp = const_cast<int64_t*>(d->cp);
  M->jc = const_cast<int64_t*>(d->jc);
  M->ir = const_cast<int32_t*>(d->ir);
  M->num = const_cast<void*>(d->num);
  M->owned = false;
  *out = M;
  return CBH_OK;
}

int cbh_mat_info(const cbh_mat* M, int64_t* m, int64_t* n, int64_t* nnz, int64_t* nzc, int* dtype) {
  if (!M) return CBH_E_ARG;
  if (m) *m = M->m;
  if (n) *n = M->n;
  if (nnz) *nnz = M->nnz;
  if (nzc) *nzc = M->nzc;
  if (dtype) *dtype = M->dtype;
  return CBH_OK;
}

int cbh_mat_device_arrays(const cbh_mat* M, const int64_t** cp, const int64_t** jc, const int32_t** ir,
                          const void** num) {
  if (!M) return CBH_E_ARG;
  if (cp) *cp = M->cp;
  if (jc) *jc = M->jc;
  if (ir) *ir = M->ir;
  if (num) *num = M->num;
  return CBH_OK;
}

}  // extern "C"

// the two pinned staging halves for chunks of `chunk` entries of (int32 row, vb-byte value)
static int pinned_halves(cbh_ctx* ctx, int64_t chunk, int64_t vb, char* half[2]) {
  const size_t hb = (size_t)chunk * (size_t)(4 + vb) + 256;
  if (ctx->pin_bytes < 2 * hb) {
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->pin) (void)hipHostFree(ctx->pin);
    ctx->pin = nullptr;
    ctx->pin_bytes = 0;
    CBH_HIP(ctx, hipHostMalloc(&ctx->pin, 2 * hb, hipHostMallocDefault));
    ctx->pin_bytes = 2 * hb;
  }
  for (auto& e : ctx->pin_ev)
    if (!e) CBH_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  half[0] = reinterpret_cast<char*>(ctx->pin);
  half[1] = half[0] + ctx->pin_bytes / 2;
  return CBH_OK;
}
static int64_t chunk_entries(int64_t chunk) { return chunk > 0 ? chunk : (int64_t)4 << 20; }

extern "C" {

int cbh_mat_upload_chunks(cbh_ctx* ctx, int64_t m, int64_t n, int64_t nnz, int64_t nzc, const int64_t* cp,
                          const int64_t* jc, cbh_dtype dtype, int64_t value_bytes, int64_t chunk, cbh_fill_fn fill,
                          void* user, cbh_mat** out) {
  if (!ctx || !out || !fill || nnz < 0 || nzc < 0 || m < 0 || n < 0 || (nzc > 0 && (!cp || !jc)))
    return fail(ctx, CBH_E_ARG, "bad chunked upload arguments");
  const int64_t vb = dtype == CBH_OPAQUE ? value_bytes : (int64_t)dtype_size(dtype);
  if (vb <= 0) return fail(ctx, CBH_E_ARG, "bad value size");
  if (m > INT32_MAX) return fail(ctx, CBH_E_DIMMISMATCH, "local rows exceed int32");
  *out = nullptr;
  cbh_mat* M;
  CBH_TRY(new_mat(ctx, m, n, nnz, nzc, dtype, &M, vb));
  int rc = CBH_OK;
  auto body = [&]() -> int {
    if (nzc > 0) {
      CBH_HIP(ctx, hipMemcpyAsync(M->cp, cp, sizeof(int64_t) * (nzc + 1), hipMemcpyHostToDevice, ctx->stream));
      CBH_HIP(ctx, hipMemcpyAsync(M->jc, jc, sizeof(int64_t) * nzc, hipMemcpyHostToDevice, ctx->stream));
    } else {
      CBH_HIP(ctx, hipMemsetAsync(M->cp, 0, sizeof(int64_t), ctx->stream));
    }
    const int64_t ch = chunk_entries(chunk);
    char* half[2];
    CBH_TRY(pinned_halves(ctx, ch, vb, half));
    bool used[2] = {false, false};
    for (int64_t f = 0, k = 0; f < nnz; f += ch, ++k) {
      const int h = (int)(k & 1);
      const int64_t cnt = std::min(ch, nnz - f);
      if (used[h]) CBH_HIP(ctx, hipEventSynchronize(ctx->pin_ev[h]));  // the copy out of this half is done
      int32_t* sir = reinterpret_cast<int32_t*>(half[h]);
      char* snum = half[h] + (((size_t)ch * 4 + 255) & ~size_t(255));
      const int r = fill(user, f, cnt, sir, snum);
      if (r != 0) return fail(ctx, r, "upload fill callback returned " + std::to_string(r));
      CBH_HIP(ctx, hipMemcpyAsync(M->ir + f, sir, sizeof(int32_t) * cnt, hipMemcpyHostToDevice, ctx->stream));
      CBH_HIP(ctx, hipMemcpyAsync(reinterpret_cast<char*>(M->num) + f * vb, snum, (size_t)(vb * cnt),
                                  hipMemcpyHostToDevice, ctx->stream));
      CBH_HIP(ctx, hipEventRecord(ctx->pin_ev[h], ctx->stream));
      used[h] = true;
    }
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // cp / jc may be released on return
    return CBH_OK;
  };
  rc = body();
  if (rc != CBH_OK) {
    (void)hipStreamSynchronize(ctx->stream);
    cbh_mat_free(ctx, M);
    return rc;
  }
  *out = M;
  return CBH_OK;
}

int cbh_mat_download_chunks(cbh_ctx* ctx, const cbh_mat* M, int64_t* cp, int64_t* jc, int64_t chunk, cbh_take_fn take,
                            void* user) {
  if (!ctx || !M || !take) return fail(ctx, CBH_E_ARG, "bad chunked download arguments");
  if (cp) CBH_HIP(ctx, hipMemcpyAsync(cp, M->cp, sizeof(int64_t) * (M->nzc + 1), hipMemcpyDeviceToHost, ctx->stream));
  if (jc && M->nzc) CBH_HIP(ctx, hipMemcpyAsync(jc, M->jc, sizeof(int64_t) * M->nzc, hipMemcpyDeviceToHost, ctx->stream));
  const int64_t nnz = M->nnz, vb = M->vbytes;
  const int64_t ch = chunk_entries(chunk);
  char* half[2];
  CBH_TRY(pinned_halves(ctx, ch, vb, half));
  auto issue = [&](int64_t f, int h) -> int {
    const int64_t cnt = std::min(ch, nnz - f);
    char* snum = half[h] + (((size_t)ch * 4 + 255) & ~size_t(255));
    CBH_HIP(ctx, hipMemcpyAsync(half[h], M->ir + f, sizeof(int32_t) * cnt, hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(snum, reinterpret_cast<const char*>(M->num) + f * vb, (size_t)(vb * cnt),
                                hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipEventRecord(ctx->pin_ev[h], ctx->stream));
    return CBH_OK;
  };
  // CBH_XFER_DIAG=1: where a download's time goes -- waiting for the copy engine vs the caller's
  // host-side conversion (take), per call on stderr
  static const bool diag = std::getenv("CBH_XFER_DIAG") != nullptr;
  const auto t_start = std::chrono::steady_clock::now();
  double wait_s = 0, take_s = 0;
  if (nnz > 0) CBH_TRY(issue(0, 0));
  for (int64_t f = 0, k = 0; f < nnz; f += ch, ++k) {
    const int h = (int)(k & 1);
    if (f + ch < nnz) CBH_TRY(issue(f + ch, h ^ 1));  // the next chunk moves while this one is taken
    const auto t0 = std::chrono::steady_clock::now();
    CBH_HIP(ctx, hipEventSynchronize(ctx->pin_ev[h]));
    const auto t1 = std::chrono::steady_clock::now();
    const int64_t cnt = std::min(ch, nnz - f);
    const int r = take(user, f, cnt, reinterpret_cast<const int32_t*>(half[h]),
                       half[h] + (((size_t)ch * 4 + 255) & ~size_t(255)));
    wait_s += std::chrono::duration<double>(t1 - t0).count();
    take_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    if (r != 0) {
      (void)hipStreamSynchronize(ctx->stream);
      return fail(ctx, r, "download take callback returned " + std::to_string(r));
    }
  }
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (diag && nnz > 0) {
    const double tot = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    std::fprintf(stderr, "[cbh xfer] download %lld entries (%.1f MB device format) in %lld chunks: %.2f ms total, "
                         "copy-engine wait %.2f ms, take %.2f ms (%.1f GB/s device format)\n",
                 (long long)nnz, nnz * (4.0 + vb) / 1e6, (long long)((nnz + ch - 1) / ch), tot * 1e3, wait_s * 1e3,
                 take_s * 1e3, nnz * (4.0 + vb) / tot / 1e9);
  }
  return CBH_OK;
}

int cbh_mat_copy_out(cbh_ctx* ctx, const cbh_mat* M, int64_t* cp, int64_t* jc, int32_t* ir, void* num,
                     int dst_on_device) {
  if (!ctx || !M) return CBH_E_ARG;
  const hipMemcpyKind k = dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  if (cp) CBH_HIP(ctx, hipMemcpyAsync(cp, M->cp, sizeof(int64_t) * (M->nzc + 1), k, ctx->stream));
  if (jc && M->nzc) CBH_HIP(ctx, hipMemcpyAsync(jc, M->jc, sizeof(int64_t) * M->nzc, k, ctx->stream));
  if (ir && M->nnz) CBH_HIP(ctx, hipMemcpyAsync(ir, M->ir, sizeof(int32_t) * M->nnz, k, ctx->stream));
  if (num && M->nnz) CBH_HIP(ctx, hipMemcpyAsync(num, M->num, M->vbytes * M->nnz, k, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return CBH_OK;
}

int cbh_mat_free(cbh_ctx* ctx, cbh_mat* M) {
  if (!M) return CBH_OK;
  if (M->owned && ctx) {
    dfree(ctx, M->cp);
    dfree(ctx, M->jc);
    if (!M->borrowed_rows) {
      dfree(ctx, M->ir);
      dfree(ctx, M->num);
    }
  }
  delete M;
  return CBH_OK;
}

int cbh_mat_upload_bytes(cbh_ctx* ctx, const cbh_dcsc* h, int64_t value_bytes, cbh_mat** out) {
  if (!ctx || !h || !out || value_bytes <= 0) return fail(ctx, CBH_E_ARG, "bad upload arguments");
  if (h->nnz < 0 || h->nzc < 0 || h->m < 0 || h->n < 0) return fail(ctx, CBH_E_DIMMISMATCH, "negative sizes");
  cbh_mat* M;
  CBH_TRY(new_mat(ctx, h->m, h->n, h->nnz, h->nzc, CBH_OPAQUE, &M, value_bytes));
  if (h->nzc > 0) {
    CBH_HIP(ctx, hipMemcpyAsync(M->cp, h->cp, sizeof(int64_t) * (h->nzc + 1), hipMemcpyHostToDevice, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(M->jc, h->jc, sizeof(int64_t) * h->nzc, hipMemcpyHostToDevice, ctx->stream));
  } else {
    CBH_HIP(ctx, hipMemsetAsync(M->cp, 0, sizeof(int64_t), ctx->stream));
  }
  if (h->nnz > 0) {
    CBH_HIP(ctx, hipMemcpyAsync(M->ir, h->ir, sizeof(int32_t) * h->nnz, hipMemcpyHostToDevice, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(M->num, h->num, value_bytes * h->nnz, hipMemcpyHostToDevice, ctx->stream));
  }
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  *out = M;
  return CBH_OK;
}

int64_t cbh_mat_value_bytes(const cbh_mat* M) { return M ? M->vbytes : 0; }

int cbh_mat_create(cbh_ctx* ctx, int64_t m, int64_t n, int64_t nnz, int64_t nzc, cbh_dtype dtype, int64_t value_bytes,
                   cbh_mat** out) {
  if (!ctx || !out || m < 0 || n < 0 || nnz < 0 || nzc < 0) return fail(ctx, CBH_E_ARG, "bad create arguments");
  const int64_t vb = dtype == CBH_OPAQUE ? value_bytes : (int64_t)dtype_size(dtype);
  if (vb <= 0) return fail(ctx, CBH_E_ARG, "unknown value size");
  CBH_TRY(new_mat(ctx, m, n, nnz, nzc, dtype, out, vb));
  if (nzc == 0) CBH_HIP(ctx, hipMemsetAsync((*out)->cp, 0, sizeof(int64_t), ctx->stream));
  return CBH_OK;
}

int cbh_mat_clone(cbh_ctx* ctx, const cbh_mat* S, cbh_mat** out) {
  if (!ctx || !S || !out) return fail(ctx, CBH_E_ARG, "bad clone arguments");
  cbh_mat* M;
  CBH_TRY(new_mat(ctx, S->m, S->n, S->nnz, S->nzc, S->dtype, &M, S->vbytes));
  CBH_HIP(ctx, hipMemcpyAsync(M->cp, S->cp, sizeof(int64_t) * (S->nzc + 1), hipMemcpyDeviceToDevice, ctx->stream));
  if (S->nzc) CBH_HIP(ctx, hipMemcpyAsync(M->jc, S->jc, sizeof(int64_t) * S->nzc, hipMemcpyDeviceToDevice, ctx->stream));
  if (S->nnz) {
    CBH_HIP(ctx, hipMemcpyAsync(M->ir, S->ir, sizeof(int32_t) * S->nnz, hipMemcpyDeviceToDevice, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(M->num, S->num, S->vbytes * S->nnz, hipMemcpyDeviceToDevice, ctx->stream));
  }
  *out = M;
  return CBH_OK;
}

int cbh_spgemm_symbolic(cbh_ctx* ctx, const cbh_mat* A, const cbh_mat* B, int64_t* flops, int64_t* nnzC,
                        int64_t* col_flops_dev, int64_t* col_nnz_dev) {
  CBH_TRY(validate_pair(ctx, A, B));
  if (A->nnz == 0 || B->nnz == 0) {
    if (flops) *flops = 0;
    if (nnzC) *nnzC = 0;
    if (col_flops_dev && B->nzc) CBH_HIP(ctx, hipMemsetAsync(col_flops_dev, 0, sizeof(int64_t) * B->nzc, ctx->stream));
    if (col_nnz_dev && B->nzc) CBH_HIP(ctx, hipMemsetAsync(col_nnz_dev, 0, sizeof(int64_t) * B->nzc, ctx->stream));
    return CBH_OK;
  }
  Scratch S(ctx);
  Plan P;
  CBH_TRY(run_symbolic(ctx, S, A, B, P, true));
  if (flops) *flops = P.total_flops;
  if (nnzC) *nnzC = P.total_nnz;
  if (col_flops_dev)
    CBH_HIP(ctx, hipMemcpyAsync(col_flops_dev, P.flop, sizeof(int64_t) * P.nzcB, hipMemcpyDeviceToDevice, ctx->stream));
  if (col_nnz_dev)
    CBH_HIP(ctx, hipMemcpyAsync(col_nnz_dev, P.nnz, sizeof(int64_t) * P.nzcB, hipMemcpyDeviceToDevice, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return CBH_OK;
}

int cbh_spgemm(cbh_ctx* ctx, cbh_semiring sr, const cbh_mat* A, const cbh_mat* B, uint32_t flags, cbh_mat** C) {
  CBH_TRY(validate_pair(ctx, A, B));
  if (!C) return fail(ctx, CBH_E_ARG, "null output");
  *C = nullptr;
  ctx->times = cbh_kernel_times{-1, -1, -1, 0};
  if (A->nnz == 0 || B->nnz == 0) return empty_result(ctx, A->m, B->n, A->dtype, C);
  return dispatch_sr(ctx, sr, A->dtype, [&](auto srv) -> int {
    using SR = decltype(srv);
    Scratch S(ctx);
    Plan P;
    ev_record(ctx, 0);
    CBH_TRY(run_symbolic(ctx, S, A, B, P));
    ev_record(ctx, 1);
    cbh_mat* out;
    const bool keep = (flags & CBH_KEEP_EMPTY_COLS) != 0;
    int64_t nzcC = P.nzcB;
    int64_t* pos = nullptr;
    if (!keep) {
      int64_t* flag;
      CBH_TRY(S.get(&flag, P.nzcB + 1));
      CBH_TRY(S.get(&pos, P.nzcB + 1));
      hipLaunchKernelGGL(nz_flag_kernel, dim3(blocks_for(P.nzcB + 1, 256)), dim3(256), 0, ctx->stream, P.nnz,
                         P.nzcB + 1, flag);
      CBH_TRY(exclusive_scan_i64(ctx, S, flag, pos, P.nzcB + 1));
      CBH_HIP(ctx, hipMemcpyAsync(&nzcC, pos + P.nzcB, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
      CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    CBH_TRY(new_result(ctx, S, P, A->m, B->n, P.total_nnz, nzcC, A->dtype, &out));
    int64_t launches = 0;
    int rc = run_numeric<SR>(ctx, S, A, B, P, 0, P.ntasks, 0, out->ir, out->num, &launches, P.total_nnz);
    if (rc == CBH_OK && (flags & (CBH_ORDER_HYBRID | CBH_ORDER_HEAP | CBH_ORDER_HASH)))
      rc = run_reference_order<SR>(ctx, S, A, B, P, out, flags);
    if (rc == CBH_OK) {
      if (keep) {
        rc = hip_rc(ctx, hipMemcpyAsync(out->jc, B->jc, sizeof(int64_t) * P.nzcB, hipMemcpyDeviceToDevice, ctx->stream),
                    "hipMemcpyAsync(C.jc)");
        if (rc == CBH_OK)
          rc = hip_rc(ctx, hipMemcpyAsync(out->cp, P.Ccp, sizeof(int64_t) * (P.nzcB + 1), hipMemcpyDeviceToDevice, ctx->stream),
                      "hipMemcpyAsync(C.cp)");
      } else {
        hipLaunchKernelGGL(compact_cols_kernel, dim3(blocks_for(P.nzcB, 256)), dim3(256), 0, ctx->stream, P.nnz, pos,
                           B->jc, P.Ccp, P.nzcB, out->jc, out->cp);
      }
      ev_record(ctx, 2);
      if (rc == CBH_OK) rc = check_err(ctx);
    }
    if (rc != CBH_OK) {
      cbh_mat_free(ctx, out);
      return rc;
    }
    if (ctx->timing) {
      ctx->times.symbolic_ms = ev_ms(ctx, 0, 1);
      ctx->times.numeric_ms = ev_ms(ctx, 1, 2);
      ctx->times.total_ms = ev_ms(ctx, 0, 2);
      ctx->times.numeric_launches = launches;
    }
    *C = out;
    return CBH_OK;
  });
}

int cbh_spgemm_phased(cbh_ctx* ctx, cbh_semiring sr, const cbh_mat* A, const cbh_mat* B, uint32_t flags,
                      cbh_phase_stats* st) {
  CBH_TRY(validate_pair(ctx, A, B));
  if (!st) return fail(ctx, CBH_E_ARG, "null stats");
  std::memset(st, 0, sizeof(*st));
  ctx->times = cbh_kernel_times{-1, -1, -1, 0};
  if (A->nnz == 0 || B->nnz == 0) return CBH_OK;
  return dispatch_sr(ctx, sr, A->dtype, [&](auto srv) -> int {
    using SR = decltype(srv);
    using VT = typename SR::val_t;
    Scratch S(ctx);
    Plan P;
    ev_record(ctx, 0);
    CBH_TRY(run_symbolic(ctx, S, A, B, P));
    ev_record(ctx, 1);
    const size_t esz = sizeof(int32_t) + sizeof(VT);
    int64_t budget_bytes = ctx->phase_budget;
    if (budget_bytes <= 0) {
      if (ctx->ws_bytes > 0) {
        budget_bytes = ctx->ws_bytes - 512;
      } else {
        size_t freeb = 0, totb = 0;
        CBH_HIP(ctx, hipMemGetInfo(&freeb, &totb));
        budget_bytes = (int64_t)(freeb * phase_frac());
      }
    }
    int64_t budget = std::max<int64_t>(1, std::min<int64_t>(budget_bytes / (int64_t)esz, P.total_nnz));
    // phase boundaries over B's column slots from the exact column offsets
    std::vector<int64_t> hcp(P.nzcB + 1), hts(P.nzcB + 1);
    CBH_HIP(ctx, hipMemcpyAsync(hcp.data(), P.Ccp, sizeof(int64_t) * (P.nzcB + 1), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(hts.data(), P.tstart, sizeof(int64_t) * (P.nzcB + 1), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    int64_t maxcol = 0;
    for (int64_t c = 0; c < P.nzcB; ++c) maxcol = std::max(maxcol, hcp[c + 1] - hcp[c]);
    budget = std::max(budget, maxcol);
    auto cut_with = [&](int64_t bud) {
      std::vector<int64_t> cs{0};
      while (cs.back() < P.nzcB) {
        const int64_t c0 = cs.back();
        const int64_t lim = hcp[c0] + bud;
        int64_t c1 = (int64_t)(std::upper_bound(hcp.begin() + c0 + 1, hcp.end(), lim) - hcp.begin()) - 1;
        if (c1 <= c0) c1 = c0 + 1;
        cs.push_back(c1);
      }
      return cs;
    };
    std::vector<int64_t> cuts = cut_with(budget);
    // balance: the greedy cuts leave a short last phase that pays its own launch tails; the same
    // number of phases at an even share of the entries (plus the widest column of slack) is kept
    // when it needs no more phases
    if (cuts.size() > 2) {
      const int64_t np = (int64_t)cuts.size() - 1;
      const int64_t even = std::min(budget, (P.total_nnz + np - 1) / np + maxcol);
      std::vector<int64_t> bal = cut_with(even);
      if (bal.size() == cuts.size()) cuts.swap(bal);
    }
    const int64_t maxphase = [&] {
      int64_t mx = 0;
      for (size_t i = 1; i < cuts.size(); ++i) mx = std::max(mx, hcp[cuts[i]] - hcp[cuts[i - 1]]);
      return mx;
    }();
    int32_t* ir;
    VT* num;
    auto hnow = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double ta = hnow();
    const int64_t ir_bytes = ((maxphase * (int64_t)sizeof(int32_t)) + 255) & ~int64_t(255);
    const int64_t need = ir_bytes + maxphase * (int64_t)sizeof(VT) + 256;
    if (ctx->ws_bytes < need) {
      CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
      if (ctx->ws) (void)hipFree(ctx->ws);
      ctx->ws = nullptr;
      ctx->ws_bytes = 0;
      if (hipMalloc(&ctx->ws, (size_t)need) != hipSuccess) {
        (void)hipGetLastError();
        if (P.bmp) {  // the workspace does not fit beside the stored bitmaps: dense windows off
          S.drop(P.bmp);
          P.bmp = nullptr;
        }
        release_cache(ctx);
        CBH_HIP(ctx, hipMalloc(&ctx->ws, (size_t)need));
      }
      ctx->ws_bytes = need;
    }
    ir = reinterpret_cast<int32_t*>(ctx->ws);
    num = reinterpret_cast<VT*>(reinterpret_cast<char*>(ctx->ws) + ir_bytes);
    if (diag_enabled()) {
      CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
      std::fprintf(stderr, "[cbh diag] phased: %zu phases, budget %lld entries, alloc %.1f ms\n", cuts.size() - 1,
                   (long long)budget, hnow() - ta);
    }
    double* d_sum;
    unsigned long long* d_dig;
    CBH_TRY(S.get(&d_sum, 1));
    CBH_TRY(S.get(&d_dig, 1));
    CBH_HIP(ctx, hipMemsetAsync(d_sum, 0, sizeof(double), ctx->stream));
    CBH_HIP(ctx, hipMemsetAsync(d_dig, 0, sizeof(unsigned long long), ctx->stream));
    int64_t launches = 0;
    int64_t *vcp = nullptr, *vjc = nullptr;  // per-phase consumer: the view's rebased pointers / ids
    if (ctx->phase_fn) {
      int64_t maxn = 0;
      for (size_t i = 1; i < cuts.size(); ++i) maxn = std::max(maxn, cuts[i] - cuts[i - 1]);
      CBH_TRY(S.get(&vcp, maxn + 1));
      CBH_TRY(S.get(&vjc, std::max<int64_t>(maxn, 1)));
    }
    for (size_t i = 1; i < cuts.size(); ++i) {
      const int64_t c0 = cuts[i - 1], c1 = cuts[i];
      const double tp = hnow();
      CBH_TRY(run_numeric<SR>(ctx, S, A, B, P, hts[c0], hts[c1], hcp[c0], ir, num, &launches, maxphase));
      if (ctx->phase_fn) {
        CBH_TRY(check_err(ctx));  // the consumer sees only a phase whose guards all passed
        hipLaunchKernelGGL(keep_cols_kernel, dim3(blocks_for(c1 - c0 + 1, 256)), dim3(256), 0, ctx->stream, B->jc + c0,
                           P.Ccp + c0, c1 - c0, hcp[c0], vjc, vcp);
        CBH_HIP(ctx, hipGetLastError());
        cbh_mat view;
        view.m = A->m;
        view.n = B->n;
        view.nnz = hcp[c1] - hcp[c0];
        view.nzc = c1 - c0;
        view.dtype = A->dtype;
        view.vbytes = (int64_t)sizeof(VT);
        view.cp = vcp;
        view.jc = vjc;
        view.ir = ir;
        view.num = num;
        view.owned = false;
        const int rc = ctx->phase_fn(ctx->phase_user, (int64_t)i - 1, c0, c1, &view);
        if (rc != CBH_OK) return fail(ctx, rc, "phase consumer returned " + std::to_string(rc));
      }
      if (diag_enabled()) {
        CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
        std::fprintf(stderr, "[cbh diag] phase %zu: cols [%lld,%lld) %.1f ms host wall\n", i, (long long)c0,
                     (long long)c1, hnow() - tp);
      }
      if (flags & CBH_PHASE_CHECKSUM) {
        hipLaunchKernelGGL(checksum_kernel<VT>, dim3(blocks_for(c1 - c0, 4)), dim3(256), 0, ctx->stream, B->jc + c0,
                           P.Ccp + c0, hcp[c0], c1 - c0, ir, num, hcp[c0], d_sum, d_dig);
        CBH_HIP(ctx, hipGetLastError());
      }
    }
    ev_record(ctx, 2);
    CBH_TRY(check_err(ctx));
    double hs = 0;
    unsigned long long hd = 0;
    CBH_HIP(ctx, hipMemcpyAsync(&hs, d_sum, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(&hd, d_dig, sizeof(hd), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    st->flops = P.total_flops;
    st->nnz = P.total_nnz;
    st->phases = (int64_t)cuts.size() - 1;
    st->value_sum = hs;
    st->digest = hd;
    if (ctx->timing) {
      ctx->times.symbolic_ms = ev_ms(ctx, 0, 1);
      ctx->times.numeric_ms = ev_ms(ctx, 1, 2);
      ctx->times.total_ms = ev_ms(ctx, 0, 2);
      ctx->times.numeric_launches = launches;
    }
    return CBH_OK;
  });
}

// ---------------------------------------------------------------------------- user-semiring plans
// The semiring-independent half of cbh_spgemm (symbolic pass, task plan, binning, compaction);
// the caller launches the numeric kernels of its own semiring in between (device/numeric.h).
}  // extern "C"
struct cbh_plan {
  cbh_ctx* ctx = nullptr;
  const cbh_mat* A = nullptr;
  const cbh_mat* B = nullptr;
  Scratch S;
  Plan P;
  int64_t* pos = nullptr;  // nonempty-column positions of C (compaction)
  int64_t nzcC = 0;
  explicit cbh_plan(cbh_ctx* c) : ctx(c), S(c) {}
};
extern "C" {

int cbh_plan_create(cbh_ctx* ctx, const cbh_mat* A, const cbh_mat* B, cbh_plan** out) {
  if (!ctx || !A || !B || !out) return fail(ctx, CBH_E_ARG, "null argument");
  if (A == B) return fail(ctx, CBH_E_MATRIXALIAS, "A and B alias (ParFriends.h:172-179)");
  if (A->n != B->m) return fail(ctx, CBH_E_DIMMISMATCH, "A.getncol() != B.getnrow()");
  if (A->m > INT32_MAX) return fail(ctx, CBH_E_DIMMISMATCH, "local row count exceeds 32-bit row ids");
  *out = nullptr;
  cbh_plan* p = new cbh_plan(ctx);
  p->A = A;
  p->B = B;
  if (A->nnz > 0 && B->nnz > 0) {
    const int rc = run_symbolic(ctx, p->S, A, B, p->P);
    if (rc != CBH_OK) {
      delete p;
      return rc;
    }
  }
  *out = p;
  return CBH_OK;
}

int cbh_plan_info(const cbh_plan* p, int64_t* flops, int64_t* nnzC) {
  if (!p) return CBH_E_ARG;
  if (flops) *flops = p->P.total_flops;
  if (nnzC) *nnzC = p->P.total_nnz;
  return CBH_OK;
}

int cbh_plan_numeric(cbh_plan* p, cbh_dtype dtype, int64_t value_bytes, uint32_t flags, cbh_mat** C,
                     cbh_numeric_plan* out) {
  if (!p || !C || !out || value_bytes <= 0) return fail(p ? p->ctx : nullptr, CBH_E_ARG, "bad plan arguments");
  cbh_ctx* ctx = p->ctx;
  Plan& P = p->P;
  *C = nullptr;
  std::memset(out, 0, sizeof(*out));
  out->stream = ctx->stream;
  if (P.ntasks == 0) {  // empty operand or product: an empty C (mtSpGEMM.h:224-227)
    CBH_TRY(new_mat(ctx, p->A->m, p->B->n, 0, 0, dtype, C, value_bytes));
    CBH_HIP(ctx, hipMemsetAsync((*C)->cp, 0, sizeof(int64_t), ctx->stream));
    return CBH_OK;
  }
  int64_t* flag;
  CBH_TRY(p->S.get(&flag, P.nzcB + 1));
  CBH_TRY(p->S.get(&p->pos, P.nzcB + 1));
  hipLaunchKernelGGL(nz_flag_kernel, dim3(blocks_for(P.nzcB + 1, 256)), dim3(256), 0, ctx->stream, P.nnz, P.nzcB + 1,
                     flag);
  CBH_TRY(exclusive_scan_i64(ctx, p->S, flag, p->pos, P.nzcB + 1));
  CBH_HIP(ctx, hipMemcpyAsync(&p->nzcC, p->pos + P.nzcB, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  CBH_TRY(new_result(ctx, p->S, P, p->A->m, p->B->n, P.total_nnz, P.nzcB, dtype, C, value_bytes));
  // bins: dense (built-in, lock-free semirings only), then hash large / small
  using CD = TaskCfg<PlusTimesD<double>, kSplitHashT, TNumLarge::BS, TNumLarge::EMAX, TNumLarge::U, MODE_TDENSE>;  // split pricing
  const int64_t nt = P.ntasks;
  int64_t *wd, *wh;
  CBH_TRY(p->S.get(&wd, nt));
  CBH_TRY(p->S.get(&wh, nt));
  hipLaunchKernelGGL(dense_split_kernel, dim3(blocks_for(nt, 256)), dim3(256), 0, ctx->stream, P.tcnt, P.tlo, P.thi,
                     P.bmp ? P.boff : nullptr, P.twork, nt,
                     kSplitHashT, (int64_t)CD::CAPD, (int64_t)CD::NWB, (int64_t)kDRatio4, kSmallCap, kWaveProducts,
                     !(flags & CBH_PLAN_NO_DENSE) ? 1 : 0, wd, wh);
  CBH_HIP(ctx, hipGetLastError());
  BinLists bd, bl;
  CBH_TRY(make_bins(ctx, p->S, wd, nt, 0, P.order, &bd, BinCaps{kSmallCap, kSmallCap}, nullptr, P.trk));
  const int64_t nd = bd.small_count + bd.mid_count + bd.large_count;
  CBH_TRY(make_bins(ctx, p->S, wh, nt, 0, P.order + nd, &bl, BinCaps{kSmallCap, kMidCap}, nullptr, P.trk));
  const cbh_mat* A = p->A;
  const cbh_mat* B = p->B;
  out->Acp = P.Adense;
  out->Air = A->ir;
  out->Anum = A->num;
  out->Bcp = B->cp;
  out->Bir = B->ir;
  out->Bnum = B->num;
  out->hidx = P.hidx;
  out->htab = P.htab;
  out->nblk = P.nblk;
  out->RB = P.htab ? P.RB : 0;
  out->tcol = P.tcol;
  out->tlo = P.tlo;
  out->thi = P.thi;
  out->tfull = P.tfull;
  out->tcnt = P.tcnt;
  out->toff = P.toff;
  out->goff = P.goff;
  out->gcur0 = P.gcur0;
  out->gcur1 = P.gcur1;
  out->gend = P.gend;
  out->gnx0 = P.gnx0;
  out->gnx1 = P.gnx1;
  out->ghub = P.ghub;
  out->gbase = P.gbase;
  out->boff = P.bmp ? P.boff : nullptr;
  out->bmp = P.bmp;
  out->err = ctx->d_err;
  out->nnzA = A->nnz;
  out->ncolA = A->n;
  out->ntasks = P.ntasks;
  out->order = P.order;
  out->dense_first = bd.large_first;
  out->dense_count = bd.large_count;
  out->large_first = nd + bl.large_first;
  out->large_count = bl.large_count;
  out->small_first = nd + bl.small_first;
  out->small_count = bl.small_count;
  out->mid_first = nd + bl.mid_first;
  out->mid_count = bl.mid_count;
  return CBH_OK;
}

int cbh_plan_finish(cbh_plan* p, cbh_mat* C, uint32_t flags) {
  if (!p || !C) return fail(p ? p->ctx : nullptr, CBH_E_ARG, "bad plan arguments");
  cbh_ctx* ctx = p->ctx;
  Plan& P = p->P;
  if (P.ntasks == 0) return CBH_OK;
  if (flags & CBH_KEEP_EMPTY_COLS) {
    CBH_HIP(ctx, hipMemcpyAsync(C->jc, p->B->jc, sizeof(int64_t) * P.nzcB, hipMemcpyDeviceToDevice, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(C->cp, P.Ccp, sizeof(int64_t) * (P.nzcB + 1), hipMemcpyDeviceToDevice, ctx->stream));
  } else {
    hipLaunchKernelGGL(compact_cols_kernel, dim3(blocks_for(P.nzcB, 256)), dim3(256), 0, ctx->stream, P.nnz, p->pos,
                       p->B->jc, P.Ccp, P.nzcB, C->jc, C->cp);
    C->nzc = p->nzcC;
  }
  CBH_HIP(ctx, hipGetLastError());
  return check_err(ctx);
}

int cbh_plan_destroy(cbh_plan* p) {
  delete p;
  return CBH_OK;
}

int cbh_plan_col_nnz(const cbh_plan* p, int64_t* col_nnz_dev) {
  if (!p || !col_nnz_dev) return fail(p ? p->ctx : nullptr, CBH_E_ARG, "bad plan arguments");
  cbh_ctx* ctx = p->ctx;
  const int64_t n = p->B->nzc;
  if (n == 0) return CBH_OK;
  if (p->P.ntasks == 0) CBH_HIP(ctx, hipMemsetAsync(col_nnz_dev, 0, sizeof(int64_t) * n, ctx->stream));
  else CBH_HIP(ctx, hipMemcpyAsync(col_nnz_dev, p->P.nnz, sizeof(int64_t) * n, hipMemcpyDeviceToDevice, ctx->stream));
  return CBH_OK;
}

int cbh_plan_spgemm_slots(cbh_plan* p, cbh_semiring sr, int64_t s0, int64_t s1, uint32_t flags, cbh_mat** C) {
  if (!p || !C) return fail(p ? p->ctx : nullptr, CBH_E_ARG, "bad plan arguments");
  cbh_ctx* ctx = p->ctx;
  const cbh_mat* A = p->A;
  const cbh_mat* B = p->B;
  *C = nullptr;
  if (s0 < 0 || s1 < s0 || s1 > B->nzc) return fail(ctx, CBH_E_ARG, "slot range outside B's nonzero columns");
  if (A->dtype != B->dtype) return fail(ctx, CBH_E_ARG, "A and B dtypes differ");
  Plan& P = p->P;
  if (P.ntasks == 0 || s1 == s0) return empty_result(ctx, A->m, B->n, A->dtype, C);
  return dispatch_sr(ctx, sr, A->dtype, [&](auto srv) -> int {
    using SR = decltype(srv);
    Scratch S(ctx);
    const int64_t n = s1 - s0;
    int64_t h[4];
    CBH_HIP(ctx, hipMemcpyAsync(&h[0], P.tstart + s0, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(&h[1], P.tstart + s1, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(&h[2], P.Ccp + s0, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(&h[3], P.Ccp + s1, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    const bool keep = (flags & CBH_KEEP_EMPTY_COLS) != 0;
    int64_t nzcC = n;
    int64_t* pos = nullptr;
    if (!keep) {
      int64_t* flag;
      CBH_TRY(S.get(&flag, n + 1));
      CBH_TRY(S.get(&pos, n + 1));
      hipLaunchKernelGGL(nz_flag_kernel, dim3(blocks_for(n + 1, 256)), dim3(256), 0, ctx->stream, P.nnz + s0, n + 1,
                         flag);
      CBH_TRY(exclusive_scan_i64(ctx, S, flag, pos, n + 1));
      CBH_HIP(ctx, hipMemcpyAsync(&nzcC, pos + n, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    }
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const int64_t nnz = h[3] - h[2];
    cbh_mat* out;
    CBH_TRY(new_result(ctx, p->S, P, A->m, B->n, nnz, nzcC, A->dtype, &out));
    int rc = run_numeric<SR>(ctx, S, A, B, P, h[0], h[1], h[2], out->ir, out->num, nullptr, nnz);
    if (rc == CBH_OK) {
      if (keep)
        hipLaunchKernelGGL(keep_cols_kernel, dim3(blocks_for(n + 1, 256)), dim3(256), 0, ctx->stream, B->jc + s0,
                           P.Ccp + s0, n, h[2], out->jc, out->cp);
      else
        hipLaunchKernelGGL(compact_cols_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, P.nnz + s0, pos,
                           B->jc + s0, P.Ccp + s0, n, out->jc, out->cp, h[2]);
      rc = check_err(ctx);
    }
    if (rc != CBH_OK) {
      cbh_mat_free(ctx, out);
      return rc;
    }
    *C = out;
    return CBH_OK;
  });
}

extern "C++" {
// Two lists: the streaming merge path (device/merge2.h) -- head counts per chunk, a scan over the
// chunks (C's offsets and column pointers), the write pass. CBH_MERGE2=0 keeps the task kernels'
// hash merge for every list count (A/B hook).
static bool merge2_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("CBH_MERGE2");
    return !(e && std::atoi(e) == 0);
  }();
  return v;
}
template <class SR>
static int merge_two(cbh_ctx* ctx, Scratch& S, SR, const cbh_mat* const* parts, int64_t ncols, const int64_t* jcC,
                     const int64_t* seg_start, const int64_t* seg_len, cbh_mat** C) {
  const cbh_mat* P0 = parts[0];
  int64_t *nch, *cstart;
  CBH_TRY(S.get(&nch, ncols + 1));
  CBH_TRY(S.get(&cstart, ncols + 1));
  hipLaunchKernelGGL(merge2_nchunks_kernel, dim3(blocks_for(ncols, 256)), dim3(256), 0, ctx->stream, seg_len, ncols, nch);
  CBH_HIP(ctx, hipMemsetAsync(nch + ncols, 0, sizeof(int64_t), ctx->stream));
  CBH_TRY(exclusive_scan_i64(ctx, S, nch, cstart, ncols + 1));
  int64_t nchunks = 0;
  CBH_HIP(ctx, hipMemcpyAsync(&nchunks, cstart + ncols, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (nchunks > INT32_MAX) return fail(ctx, CBH_E_INTERNAL, "more than 2^31 merge chunks");
  int32_t* chunk_col;
  int64_t *ccnt, *coff, *Ccp;
  CBH_TRY(S.get(&chunk_col, nchunks));
  CBH_TRY(S.get(&ccnt, nchunks + 1));
  CBH_TRY(S.get(&coff, nchunks + 1));
  CBH_TRY(S.get(&Ccp, ncols + 1));
  hipLaunchKernelGGL(merge2_fill_kernel, dim3(blocks_for(ncols, 256)), dim3(256), 0, ctx->stream, cstart, ncols,
                     chunk_col);
  constexpr int WPB = 4;
  const unsigned grid = (unsigned)((nchunks + WPB - 1) / WPB);
  const int64_t in = P0->nnz + parts[1]->nnz;
  CBH_TRY(timed_launch(ctx, CBH_K_MERGE_SYM, 4.0 * (double)in, [&] {
    hipLaunchKernelGGL((merge2_kernel<SR, false, WPB>), dim3(grid), dim3(64 * WPB), 0, ctx->stream, chunk_col, nchunks,
                       cstart, seg_start, seg_len, P0->ir, P0->num, parts[1]->ir, parts[1]->num, ccnt,
                       (const int64_t*)nullptr, (int32_t*)nullptr, (void*)nullptr);
    return hipGetLastError();
  }));
  CBH_HIP(ctx, hipMemsetAsync(ccnt + nchunks, 0, sizeof(int64_t), ctx->stream));
  CBH_TRY(exclusive_scan_i64(ctx, S, ccnt, coff, nchunks + 1));
  hipLaunchKernelGGL(gather_i64_kernel, dim3(blocks_for(ncols + 1, 256)), dim3(256), 0, ctx->stream, coff, cstart,
                     ncols + 1, Ccp);
  int64_t total = 0;
  CBH_HIP(ctx, hipMemcpyAsync(&total, coff + nchunks, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  CBH_TRY(check_err(ctx));
  cbh_mat* out;
  CBH_TRY(new_mat(ctx, P0->m, P0->n, total, ncols, P0->dtype, &out, P0->vbytes));
  constexpr double eb = 4.0 + sizeof(typename SR::val_t);  // entries read + outputs written
  int rc = timed_launch(ctx, CBH_K_MERGE_NUM, eb * (double)(in + total), [&] {
    hipLaunchKernelGGL((merge2_kernel<SR, true, WPB>), dim3(grid), dim3(64 * WPB), 0, ctx->stream, chunk_col, nchunks,
                       cstart, seg_start, seg_len, P0->ir, P0->num, parts[1]->ir, parts[1]->num, (int64_t*)nullptr,
                       coff, out->ir, out->num);
    return hipGetLastError();
  });
  if (rc == CBH_OK)
    rc = hip_rc(ctx, hipMemcpyAsync(out->jc, jcC, sizeof(int64_t) * ncols, hipMemcpyDeviceToDevice, ctx->stream),
                "hipMemcpyAsync(C.jc)");
  if (rc == CBH_OK)
    rc = hip_rc(ctx, hipMemcpyAsync(out->cp, Ccp, sizeof(int64_t) * (ncols + 1), hipMemcpyDeviceToDevice, ctx->stream),
                "hipMemcpyAsync(C.cp)");
  if (rc == CBH_OK) rc = check_err(ctx);
  if (rc != CBH_OK) {
    cbh_mat_free(ctx, out);
    return rc;
  }
  *C = out;
  return CBH_OK;
}
}  // extern "C++"

int cbh_merge(cbh_ctx* ctx, cbh_semiring sr, int nlists, const cbh_mat* const* parts, cbh_mat** C) {
  if (!ctx || !C || nlists < 0 || (nlists > 0 && !parts)) return fail(ctx, CBH_E_ARG, "bad merge arguments");
  if (nlists > kMaxLists) return fail(ctx, CBH_E_ARG, "at most 16 lists per merge; merge hierarchically");
  *C = nullptr;
  if (nlists == 0) return fail(ctx, CBH_E_ARG, "merge of zero lists has no dimensions");
  const cbh_mat* P0 = parts[0];
  for (int l = 0; l < nlists; ++l) {
    if (!parts[l]) return fail(ctx, CBH_E_ARG, "null list");
    if (parts[l]->m != P0->m || parts[l]->n != P0->n)
      return fail(ctx, CBH_E_DIMMISMATCH, "Dimensions of SpTuples do not match on multiwayMerge()");
    if (parts[l]->dtype != P0->dtype) return fail(ctx, CBH_E_ARG, "list dtypes differ");
  }
  const int dtype = P0->dtype;
  const size_t vs = dtype_size(dtype);
  if (nlists == 1) {  // MultiwayMerge.h:420-439: one list is copied
    cbh_mat* out;
    CBH_TRY(new_mat(ctx, P0->m, P0->n, P0->nnz, P0->nzc, dtype, &out));
    CBH_HIP(ctx, hipMemcpyAsync(out->cp, P0->cp, sizeof(int64_t) * (P0->nzc + 1), hipMemcpyDeviceToDevice, ctx->stream));
    if (P0->nzc) CBH_HIP(ctx, hipMemcpyAsync(out->jc, P0->jc, sizeof(int64_t) * P0->nzc, hipMemcpyDeviceToDevice, ctx->stream));
    if (P0->nnz) {
      CBH_HIP(ctx, hipMemcpyAsync(out->ir, P0->ir, sizeof(int32_t) * P0->nnz, hipMemcpyDeviceToDevice, ctx->stream));
      CBH_HIP(ctx, hipMemcpyAsync(out->num, P0->num, vs * P0->nnz, hipMemcpyDeviceToDevice, ctx->stream));
    }
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *C = out;
    return CBH_OK;
  }
  return dispatch_sr(ctx, sr, dtype, [&](auto srv) -> int {
    using SR = decltype(srv);
    Scratch S(ctx);
    const int64_t n = P0->n;
    int32_t* flag;
    int64_t *idx, *flag64;
    CBH_TRY(S.get(&flag, n + 1));
    CBH_TRY(S.get(&flag64, n + 1));
    CBH_TRY(S.get(&idx, n + 1));
    CBH_HIP(ctx, hipMemsetAsync(flag, 0, sizeof(int32_t) * (n + 1), ctx->stream));
    for (int l = 0; l < nlists; ++l)
      if (parts[l]->nzc)
        hipLaunchKernelGGL(mark_cols_kernel, dim3(blocks_for(parts[l]->nzc, 256)), dim3(256), 0, ctx->stream,
                           parts[l]->jc, parts[l]->nzc, n, flag, ctx->d_err);
    // widen flags for the int64 scan
    hipLaunchKernelGGL(widen_i32_kernel, dim3(blocks_for(n + 1, 256)), dim3(256), 0, ctx->stream, flag, flag64, n + 1);
    CBH_TRY(exclusive_scan_i64(ctx, S, flag64, idx, n + 1));
    int64_t ncols = 0;
    CBH_HIP(ctx, hipMemcpyAsync(&ncols, idx + n, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    CBH_TRY(check_err(ctx));  // column ids outside [0, n): stop before they index anything
    if (ncols == 0) return empty_result(ctx, P0->m, n, dtype, C);
    int64_t *jcC, *seg_start, *seg_len, *work, *Ccp;
    int32_t *rmin, *rmax;
    CBH_TRY(S.get(&jcC, ncols));
    CBH_TRY(S.get(&seg_start, ncols * nlists));
    CBH_TRY(S.get(&seg_len, ncols * nlists));
    CBH_TRY(S.get(&work, ncols + 1));
    CBH_TRY(S.get(&Ccp, ncols + 1));
    CBH_TRY(S.get(&rmin, ncols));
    CBH_TRY(S.get(&rmax, ncols));
    hipLaunchKernelGGL(union_cols_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, flag, idx, n, jcC);
    CBH_HIP(ctx, hipMemsetAsync(seg_len, 0, sizeof(int64_t) * ncols * nlists, ctx->stream));
    CBH_HIP(ctx, hipMemsetAsync(seg_start, 0, sizeof(int64_t) * ncols * nlists, ctx->stream));
    ListRows lr;
    std::memset(&lr, 0, sizeof(lr));
    for (int l = 0; l < nlists; ++l) {
      lr.ir[l] = parts[l]->ir;
      if (parts[l]->nzc)
        hipLaunchKernelGGL(merge_seg_kernel, dim3(blocks_for(parts[l]->nzc, 256)), dim3(256), 0, ctx->stream,
                           parts[l]->jc, parts[l]->cp, parts[l]->nzc, idx, l, nlists, seg_start, seg_len);
    }
    if (nlists == 2 && merge2_enabled()) return merge_two(ctx, S, SR{}, parts, ncols, jcC, seg_start, seg_len, C);
    hipLaunchKernelGGL(merge_work_kernel, dim3(blocks_for(ncols, 256)), dim3(256), 0, ctx->stream, seg_start, seg_len,
                       nlists, lr, ncols, work, rmin, rmax);
    CBH_HIP(ctx, hipGetLastError());
    // task-parallel merge: every union column becomes row-range tasks of ~kMergeTaskFlops list
    // entries (as the SpGEMM's columns), symbolic -> scan -> numeric on the task kernels in
    // merge mode (entries = the lists' segments of the column; task_kernel.h MERGE)
    const int32_t RB = (int32_t)std::max<int64_t>(1, (P0->m + kRowBlocks - 1) / kRowBlocks);
    int64_t *bcp, *scnt, *tstart;
    CBH_TRY(S.get(&bcp, ncols + 1));
    CBH_TRY(S.get(&scnt, ncols + 1));
    CBH_TRY(S.get(&tstart, ncols + 1));
    hipLaunchKernelGGL(iota_scaled_kernel, dim3(blocks_for(ncols + 1, 256)), dim3(256), 0, ctx->stream, bcp, ncols + 1,
                       (int64_t)nlists);
    hipLaunchKernelGGL(task_count_kernel, dim3(blocks_for(ncols, 256)), dim3(256), 0, ctx->stream, work, rmin, rmax,
                       ncols, kMergeTaskFlops, RB, scnt);
    CBH_HIP(ctx, hipMemsetAsync(scnt + ncols, 0, sizeof(int64_t), ctx->stream));
    CBH_TRY(exclusive_scan_i64(ctx, S, scnt, tstart, ncols + 1));
    int64_t ntasks = 0;
    CBH_HIP(ctx, hipMemcpyAsync(&ntasks, tstart + ncols, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (ntasks > INT32_MAX) return fail(ctx, CBH_E_INTERNAL, "more than 2^31 merge tasks");
    const int64_t nt = std::max<int64_t>(ntasks, 1);
    int32_t *tcol, *tlo, *thi, *order;
    uint8_t* tfull;
    int64_t *twork, *tunits, *tcnt, *toff;
    CBH_TRY(S.get(&tcol, nt));
    CBH_TRY(S.get(&tlo, nt));
    CBH_TRY(S.get(&thi, nt));
    CBH_TRY(S.get(&tfull, nt));
    CBH_TRY(S.get(&twork, nt));
    CBH_TRY(S.get(&tunits, nt));
    CBH_TRY(S.get(&tcnt, nt + 1));
    CBH_TRY(S.get(&toff, nt + 1));
    CBH_TRY(S.get(&order, nt));
    hipLaunchKernelGGL(task_fill_kernel, dim3(blocks_for(ncols, 4)), dim3(256), 0, ctx->stream, tstart, work, rmin, rmax,
                       bcp, ncols, RB, tcol, tlo, thi, tfull, twork, tunits);
    CBH_HIP(ctx, hipGetLastError());
    CBH_HIP(ctx, hipMemsetAsync(tcnt, 0, sizeof(int64_t) * (nt + 1), ctx->stream));
    TaskArgs ta;
    std::memset(&ta, 0, sizeof(ta));
    ta.Bcp = bcp;
    ta.tcol = tcol;
    ta.tlo = tlo;
    ta.thi = thi;
    ta.tfull = tfull;
    ta.err = ctx->d_err;
    ta.nnzA = INT64_MAX;
    ta.ncolA = INT64_MAX;
    ta.ntasks = ntasks;
    ta.ccap = INT64_MAX;
    ta.mstart = seg_start;
    ta.mlen = seg_len;
    ta.nl = nlists;
    for (int l = 0; l < nlists; ++l) {
      ta.lir[l] = parts[l]->ir;
      ta.lnum[l] = parts[l]->num;
    }
    // symbolic: distinct rows per task
    BinLists bs;
    CBH_TRY(make_bins(ctx, S, twork, ntasks, 0, order, &bs, BinCaps{kSmallCap, kSmallCap}, tunits));
    ta.order = order;
    ta.twork = twork;
    ta.cnt = tcnt;
    using Dummy = PlusTimesD<int64_t>;
    CBH_TRY((launch_task<Dummy, TSymLarge, MODE_TSYM, true>(ctx, ta, bs.large_first, bs.large_count, CBH_K_MERGE_SYM,
                                                             4.0 * bs.units[2])));
    CBH_TRY((launch_task<Dummy, TSymSmall, MODE_TSYM, true>(ctx, ta, bs.small_first, bs.small_count + bs.mid_count,
                                                             CBH_K_MERGE_SYM, 4.0 * (bs.units[0] + bs.units[1]))));
    CBH_TRY(exclusive_scan_i64(ctx, S, tcnt, toff, ntasks + 1));
    hipLaunchKernelGGL(gather_i64_kernel, dim3(blocks_for(ncols + 1, 256)), dim3(256), 0, ctx->stream, toff, tstart,
                       ncols + 1, Ccp);
    hipLaunchKernelGGL(add_i64_kernel, dim3(blocks_for(ntasks, 256)), dim3(256), 0, ctx->stream, tunits, tcnt, ntasks,
                       tunits);
    int64_t total = 0;
    CBH_HIP(ctx, hipMemcpyAsync(&total, Ccp + ncols, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    CBH_TRY(check_err(ctx));
    cbh_mat* out;
    CBH_TRY(new_mat(ctx, P0->m, n, total, ncols, dtype, &out, P0->vbytes));
    BinLists bl;
    int rc = make_bins(ctx, S, tcnt, ntasks, 0, order, &bl, BinCaps{kSmallCap, kSmallCap}, tunits);
    if (rc == CBH_OK) {
      ta.twork = tcnt;
      ta.cnt = nullptr;
      ta.toff = toff;
      ta.cbase = 0;
      ta.Cir = out->ir;
      ta.Cnum = out->num;
      constexpr double eb = 4.0 + sizeof(typename SR::val_t);  // entries read + outputs written
      rc = launch_task<SR, TNumLargeFor<SR>, MODE_TNUM, true>(ctx, ta, bl.large_first, bl.large_count, CBH_K_MERGE_NUM,
                                                               eb * bl.units[2]);
      if (rc == CBH_OK)
        rc = launch_task<SR, TNumSmallFor<SR>, MODE_TNUM, true>(ctx, ta, bl.small_first, bl.small_count + bl.mid_count,
                                                                 CBH_K_MERGE_NUM, eb * (bl.units[0] + bl.units[1]));
    }
    if (rc == CBH_OK) {
      rc = hip_rc(ctx, hipMemcpyAsync(out->jc, jcC, sizeof(int64_t) * ncols, hipMemcpyDeviceToDevice, ctx->stream),
                  "hipMemcpyAsync(C.jc)");
      if (rc == CBH_OK)
        rc = hip_rc(ctx, hipMemcpyAsync(out->cp, Ccp, sizeof(int64_t) * (ncols + 1), hipMemcpyDeviceToDevice, ctx->stream),
                    "hipMemcpyAsync(C.cp)");
      if (rc == CBH_OK) rc = check_err(ctx);
    }
    if (rc != CBH_OK) {
      cbh_mat_free(ctx, out);
      return rc;
    }
    *C = out;
    return CBH_OK;
  });
}

// ============================================================================ callers around the hot path
// (TC's masked product, EWiseMult, HipMCL's column prune/select/recover)

}  // extern "C"

static int mat_checksum(cbh_ctx* ctx, const cbh_mat* M, int64_t row_off, int64_t col_off, const int64_t* col_pos,
                        double* value_sum, uint64_t* digest) {
  if (!ctx || !M || !value_sum || !digest) return fail(ctx, CBH_E_ARG, "null argument");
  Scratch S(ctx);
  double* d_sum;
  unsigned long long* d_dig;
  int64_t* d_pos = nullptr;
  CBH_TRY(S.get(&d_sum, 1));
  CBH_TRY(S.get(&d_dig, 1));
  if (col_pos && M->nzc > 0) {
    CBH_TRY(S.get(&d_pos, M->nzc));
    CBH_HIP(ctx, hipMemcpyAsync(d_pos, col_pos, sizeof(int64_t) * M->nzc, hipMemcpyHostToDevice, ctx->stream));
  }
  CBH_HIP(ctx, hipMemsetAsync(d_sum, 0, sizeof(double), ctx->stream));
  CBH_HIP(ctx, hipMemsetAsync(d_dig, 0, sizeof(unsigned long long), ctx->stream));
  auto run = [&](auto tag) {
    using VT = decltype(tag);
    hipLaunchKernelGGL(checksum_kernel<VT>, dim3(blocks_for(M->nzc, 4)), dim3(256), 0, ctx->stream, M->jc, M->cp,
                       (int64_t)0, M->nzc, M->ir, reinterpret_cast<const VT*>(M->num), (int64_t)0, d_sum, d_dig, d_pos,
                       row_off, col_off);
  };
  if (M->nzc > 0) {
    switch (M->dtype) {
      case CBH_F64: run(double{}); break;
      case CBH_I64: run(int64_t{}); break;
      case CBH_F32: run(float{}); break;
      case CBH_I32: run(int32_t{}); break;
      case CBH_BOOL: run(uint8_t{}); break;
      default: return fail(ctx, CBH_E_ARG, "checksum: opaque value type");
    }
    CBH_HIP(ctx, hipGetLastError());
  }
  double hs = 0;
  unsigned long long hd = 0;
  CBH_HIP(ctx, hipMemcpyAsync(&hs, d_sum, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipMemcpyAsync(&hd, d_dig, sizeof(hd), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  *value_sum = hs;
  *digest = hd;
  return CBH_OK;
}

extern "C" int cbh_mat_checksum(cbh_ctx* ctx, const cbh_mat* M, double* value_sum, uint64_t* digest) {
  return mat_checksum(ctx, M, 0, 0, nullptr, value_sum, digest);
}

extern "C" int cbh_mat_checksum_global(cbh_ctx* ctx, const cbh_mat* M, int64_t row_off, int64_t col_off,
                                       const int64_t* col_pos, double* value_sum, uint64_t* digest) {
  if (!col_pos && M && M->nzc > 0) return fail(ctx, CBH_E_ARG, "checksum_global: col_pos is required");
  return mat_checksum(ctx, M, row_off, col_off, col_pos, value_sum, digest);
}

extern "C" int cbh_transpose(cbh_ctx* ctx, const cbh_mat* A, cbh_mat** AT) {
  if (!ctx || !A || !AT) return fail(ctx, CBH_E_ARG, "null argument");
  *AT = nullptr;
  if (A->n > INT32_MAX) return fail(ctx, CBH_E_DIMMISMATCH, "transpose: column count exceeds 32-bit row ids");
  if (A->nnz == 0) return empty_result(ctx, A->n, A->m, A->dtype, AT);
  Scratch S(ctx);
  int32_t* trow;
  int64_t* tcol;
  CBH_TRY(S.get(&trow, A->nnz));
  CBH_TRY(S.get(&tcol, A->nnz));
  hipLaunchKernelGGL(transpose_tuples_kernel, dim3(blocks_for(A->nzc, 4)), dim3(256), 0, ctx->stream, A->jc, A->cp,
                     A->nzc, A->ir, trow, tcol);
  CBH_HIP(ctx, hipGetLastError());
  return cbh_tuples_to_dcsc(ctx, A->n, A->m, A->nnz, trow, tcol, A->num, (cbh_dtype)A->dtype, 0, AT);
}

// entries sharing one longer list that make it a hub group (apps.h); CBH_DOT_HUB_MIN overrides
// (read per call), 0 keeps every long entry on the wave kernel's merge / binary search. C4 at
// R-MAT scale 24 (profiles/r06/tc_hub), final kernels: 2048 / 512 / 256 / 128 -> 4.80 / 4.52 /
// 4.50 / 4.45 s per step (8.11 s without groups); the thread mode alone measured best at 2048
// before the reciprocal buckets (a group needs entries enough to fill its workgroups' threads
// over every window of its longer list)
static int dot_hub_min() {
  const char* e = std::getenv("CBH_DOT_HUB_MIN");
  return e ? std::max(0, std::atoi(e)) : 128;
}

// longer / shorter list length above which a long entry is a hub candidate (CBH_DOT_HUB_RATIO,
// read per call; default kDotMergeRatio: exactly the wave kernel's binary-search entries)
static int dot_hub_ratio() {
  const char* e = std::getenv("CBH_DOT_HUB_RATIO");
  return e ? std::max(1, std::atoi(e)) : kDotMergeRatio;
}

// longer / shorter list length at or below which a long entry is a wave-mode hub candidate
// (CBH_DOT_HUB_WAVE, read per call; 0 = no wave mode). C4 at scale 24 (profiles/r06/tc_hub):
// 0 / 2 / 8 / 12 / 16 / 24 / 32 / 64 -> 7.56 / 7.58 / 7.24 / 6.66 / 6.66 / 6.53 / 6.77 / 6.77 s
static int dot_hub_wave() {
  const char* e = std::getenv("CBH_DOT_HUB_WAVE");
  return e ? std::max(0, std::atoi(e)) : 24;
}

// entries per wave-mode hub group (CBH_DOT_HUB_WMIN, read per call; default: the thread mode's)
static int dot_hub_wmin(int hub_min) {
  const char* e = std::getenv("CBH_DOT_HUB_WMIN");
  return e ? std::max(1, std::atoi(e)) : hub_min;
}

// C = (A*B) .* M, dot form (apps.h, "masked SpGEMM, dot form")
template <class SR>
static int masked_dot(cbh_ctx* ctx, const cbh_mat* A, const cbh_mat* B, const cbh_mat* M, bool pattern, cbh_mat** C) {
  using VT = typename SR::val_t;
  if (M->nnz > INT32_MAX) return fail(ctx, CBH_E_ARG, "dot-form mask: at most 2^31-1 entries");
  cbh_mat* AT = nullptr;
  CBH_TRY(cbh_transpose(ctx, A, &AT));
  struct ATGuard {
    cbh_ctx* c;
    cbh_mat* m;
    ~ATGuard() { cbh_mat_free(c, m); }
  } atg{ctx, AT};
  Scratch S(ctx);
  const int64_t nm = M->nnz, nzc = M->nzc;
  int64_t *ATd, *Bd, *Mcol, *npiece, *poff, *hits, *off, *flag, *pos;
  int32_t *lthr, *llong, *item;
  unsigned long long* counts;
  VT* Tnum;
  uint8_t* Tflag;
  CBH_TRY(S.get(&ATd, A->m + 1));
  CBH_TRY(S.get(&Bd, B->n + 1));
  CBH_TRY(S.get(&Mcol, nm));
  CBH_TRY(S.get(&lthr, nm));
  CBH_TRY(S.get(&llong, nm));
  CBH_TRY(S.get(&npiece, nm + 1));
  CBH_TRY(S.get(&counts, 3));
  CBH_TRY(S.get(&Tnum, nm));
  CBH_TRY(S.get(&Tflag, nm));
  hipLaunchKernelGGL(densify_cp_kernel, dim3(blocks_for(A->m + 1, 256)), dim3(256), 0, ctx->stream, AT->jc, AT->cp,
                     AT->nzc, A->m, AT->nnz, ATd);
  hipLaunchKernelGGL(densify_cp_kernel, dim3(blocks_for(B->n + 1, 256)), dim3(256), 0, ctx->stream, B->jc, B->cp,
                     B->nzc, B->n, B->nnz, Bd);
  hipLaunchKernelGGL(expand_cols_kernel, dim3(blocks_for(nzc, 4)), dim3(256), 0, ctx->stream, M->jc, M->cp, nzc, Mcol);
  CBH_HIP(ctx, hipMemsetAsync(counts, 0, 3 * sizeof(unsigned long long), ctx->stream));
  DotArgs a{ATd, AT->ir, AT->num, Bd, B->ir, B->num, Mcol, M->ir, nm, A->m, B->n, Tnum, Tflag, ctx->d_err};
  // hub groups (apps.h): entries of the binary-search branch grouped by their longer list
  const int64_t K = B->n + A->m;  // group keys: j < nB (B(:, j) longer), nB + i (A(i, :) longer)
  // (the group tables take ~40 B per key and mode: skipped for masks far sparser than their shape)
  const int hub_min = K <= 8 * nm + (int64_t(1) << 20) ? dot_hub_min() : 0;
  const int hub_wave = dot_hub_wave();
  const int hub_wmin = dot_hub_wmin(hub_min);
  int32_t *gcount = nullptr, *lcand = nullptr;  // K thread-mode keys, then K wave-mode keys
  if (hub_min > 0) {
    CBH_TRY(S.get(&gcount, 2 * K));
    CBH_TRY(S.get(&lcand, nm));
    CBH_HIP(ctx, hipMemsetAsync(gcount, 0, sizeof(int32_t) * 2 * K, ctx->stream));
  }
  hipLaunchKernelGGL(dot_classify_kernel, dim3(blocks_for(nm, 256)), dim3(256), 0, ctx->stream, a, lthr, llong, npiece,
                     counts, hub_min, dot_hub_ratio(), hub_wave, gcount, lcand);
  CBH_HIP(ctx, hipGetLastError());
  unsigned long long cnt[3];
  CBH_HIP(ctx, hipMemcpyAsync(cnt, counts, sizeof(cnt), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  CBH_TRY(check_err(ctx));
  const int64_t nthr = (int64_t)cnt[0], ncand = (int64_t)cnt[2];
  int64_t nlong = (int64_t)cnt[1], nh = 0, nhitems = 0, nhthr = 0;
  int64_t *goff = nullptr, *ioff = nullptr;
  int32_t* hs = nullptr;
  if (ncand > 0) {
    int64_t *glen, *gitems;
    int32_t* gcur;
    const int64_t K2 = 2 * K;
    CBH_TRY(S.get(&glen, K2 + 1));
    CBH_TRY(S.get(&gitems, K2 + 1));
    CBH_TRY(S.get(&goff, K2 + 1));
    CBH_TRY(S.get(&ioff, K2 + 1));
    CBH_TRY(S.get(&gcur, K2));
    CBH_TRY(S.get(&hs, ncand));
    hipLaunchKernelGGL(dot_hub_sizes_kernel, dim3(blocks_for(K2, 256)), dim3(256), 0, ctx->stream, gcount, K, hub_min,
                       hub_wmin, glen, gitems);
    CBH_HIP(ctx, hipMemsetAsync(glen + K2, 0, sizeof(int64_t), ctx->stream));
    CBH_HIP(ctx, hipMemsetAsync(gitems + K2, 0, sizeof(int64_t), ctx->stream));
    CBH_TRY(exclusive_scan_i64(ctx, S, glen, goff, K2 + 1));
    CBH_TRY(exclusive_scan_i64(ctx, S, gitems, ioff, K2 + 1));
    CBH_HIP(ctx, hipMemsetAsync(gcur, 0, sizeof(int32_t) * K2, ctx->stream));
    hipLaunchKernelGGL(dot_hub_route_kernel, dim3(blocks_for(ncand, 256)), dim3(256), 0, ctx->stream, a, lcand, ncand,
                       gcount, hub_min, hub_wmin, hub_wave, goff, gcur, hs, llong, npiece, counts);
    CBH_HIP(ctx, hipGetLastError());
    int64_t h3[3];
    CBH_HIP(ctx, hipMemcpyAsync(&h3[0], goff + K2, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(&h3[1], ioff + K, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(&h3[2], ioff + K2, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(cnt, counts, sizeof(cnt), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    nh = h3[0];
    nhthr = h3[1];
    nhitems = h3[2];
    if (nh + ((int64_t)cnt[1] - nlong) != ncand) return fail(ctx, CBH_E_INTERNAL, "dot-form hub routing lost entries");
    nlong = (int64_t)cnt[1];
    if (diag_enabled())
      std::fprintf(stderr, "[cbh diag] dot hub: %lld candidates, %lld grouped (%lld thread-mode + %lld wave-mode work items), %lld long\n",
                   (long long)ncand, (long long)nh, (long long)nhthr, (long long)(nhitems - nhthr), (long long)nlong);
  }
  if (nthr > 0)
    hipLaunchKernelGGL(dot_thread_kernel<SR>, dim3(blocks_for(nthr, 256)), dim3(256), 0, ctx->stream, a, lthr, nthr);
  if (nlong > 0) {
    CBH_TRY(S.get(&poff, nlong + 1));
    CBH_HIP(ctx, hipMemsetAsync(npiece + nlong, 0, sizeof(int64_t), ctx->stream));
    CBH_TRY(exclusive_scan_i64(ctx, S, npiece, poff, nlong + 1));
    int64_t nitems = 0;
    CBH_HIP(ctx, hipMemcpyAsync(&nitems, poff + nlong, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (nitems > INT32_MAX) return fail(ctx, CBH_E_ARG, "dot-form mask: too many pieces");
    VT* pval;
    uint8_t* phit;
    CBH_TRY(S.get(&item, nitems));
    CBH_TRY(S.get(&pval, nitems));
    CBH_TRY(S.get(&phit, nitems));
    // wave-strided kernels: capped grids (a dispatch's work-item count is 32-bit)
    hipLaunchKernelGGL(dot_items_kernel, dim3(std::min(blocks_for(nlong, 4), wave_grid_cap())), dim3(256), 0, ctx->stream,
                       poff, nlong, item);
    hipLaunchKernelGGL(dot_wave_kernel<SR>, dim3(std::min(blocks_for(nitems, 4), wave_grid_cap())), dim3(256), 0,
                       ctx->stream, a, llong, poff, item, nitems, pval, phit);
    hipLaunchKernelGGL(dot_fold_kernel<SR>, dim3(blocks_for(nlong, 256)), dim3(256), 0, ctx->stream, a, llong, poff,
                       nlong, pval, phit);
  }
  if (nhthr > 0)
    hipLaunchKernelGGL(dot_hub_kernel<SR>, dim3((unsigned)std::min<int64_t>(nhthr, wave_grid_cap())), dim3(kHubBS), 0,
                       ctx->stream, a, ioff, K, nhthr, goff, hs);
  if (nhitems > nhthr)
    hipLaunchKernelGGL(dot_hub_wave_kernel<SR>, dim3((unsigned)std::min<int64_t>(nhitems - nhthr, wave_grid_cap())),
                       dim3(kHubBS), 0, ctx->stream, a, ioff, K, nhthr, nhitems, goff, hs);
  CBH_HIP(ctx, hipGetLastError());
  CBH_TRY(S.get(&hits, nzc + 1));
  CBH_TRY(S.get(&off, nzc + 1));
  CBH_TRY(S.get(&flag, nzc + 1));
  CBH_TRY(S.get(&pos, nzc + 1));
  const VT* Mnum = reinterpret_cast<const VT*>(M->num);
  hipLaunchKernelGGL((dot_collect_kernel<VT, false, false>), dim3(blocks_for(nzc, 4)), dim3(256), 0, ctx->stream, M->cp,
                     M->ir, Mnum, nzc, Tflag, Tnum, hits, nullptr, nullptr, nullptr);
  CBH_HIP(ctx, hipMemsetAsync(hits + nzc, 0, sizeof(int64_t), ctx->stream));
  CBH_TRY(exclusive_scan_i64(ctx, S, hits, off, nzc + 1));
  hipLaunchKernelGGL(nz_flag_kernel, dim3(blocks_for(nzc + 1, 256)), dim3(256), 0, ctx->stream, hits, nzc + 1, flag);
  CBH_TRY(exclusive_scan_i64(ctx, S, flag, pos, nzc + 1));
  int64_t h[2];
  CBH_HIP(ctx, hipMemcpyAsync(&h[0], off + nzc, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipMemcpyAsync(&h[1], pos + nzc, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  CBH_TRY(check_err(ctx));
  cbh_mat* out;
  CBH_TRY(new_mat(ctx, A->m, B->n, h[0], h[1], A->dtype, &out));
  if (pattern)
    hipLaunchKernelGGL((dot_collect_kernel<VT, true, true>), dim3(blocks_for(nzc, 4)), dim3(256), 0, ctx->stream, M->cp,
                       M->ir, Mnum, nzc, Tflag, Tnum, hits, off, out->ir, reinterpret_cast<VT*>(out->num));
  else
    hipLaunchKernelGGL((dot_collect_kernel<VT, true, false>), dim3(blocks_for(nzc, 4)), dim3(256), 0, ctx->stream, M->cp,
                       M->ir, Mnum, nzc, Tflag, Tnum, hits, off, out->ir, reinterpret_cast<VT*>(out->num));
  hipLaunchKernelGGL(compact_cols_kernel, dim3(blocks_for(nzc, 256)), dim3(256), 0, ctx->stream, hits, pos, M->jc, off,
                     nzc, out->jc, out->cp);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cbh_mat_free(ctx, out);
    return fail(ctx, CBH_E_HIP, std::string("masked dot: ") + hipGetErrorString(e));
  }
  *C = out;
  return CBH_OK;
}

extern "C" {

int cbh_spgemm_masked(cbh_ctx* ctx, cbh_semiring sr, const cbh_mat* A, const cbh_mat* B, const cbh_mat* M,
                      uint32_t flags, cbh_mat** C) {
  CBH_TRY(validate_pair(ctx, A, B));
  if (!M || !C) return fail(ctx, CBH_E_ARG, "null mask or output");
  if (M->m != A->m || M->n != B->n) return fail(ctx, CBH_E_DIMMISMATCH, "mask dimensions differ from A*B's");
  if (M->dtype != A->dtype) return fail(ctx, CBH_E_ARG, "mask dtype differs from A's");
  if ((flags & CBH_MASK_DOT) && (flags & CBH_MASK_EXPAND)) return fail(ctx, CBH_E_ARG, "DOT and EXPAND both set");
  *C = nullptr;
  if (A->nnz == 0 || B->nnz == 0 || M->nnz == 0) return empty_result(ctx, A->m, B->n, A->dtype, C);
  const bool pattern = (flags & CBH_MASK_PATTERN) != 0;
  const bool dot = (flags & CBH_MASK_DOT) || (!(flags & CBH_MASK_EXPAND) && A->nnz >= 65536);
  if (dot)
    return dispatch_sr(ctx, sr, A->dtype,
                       [&](auto srv) -> int { return masked_dot<decltype(srv)>(ctx, A, B, M, pattern, C); });
  if (B->nzc > INT32_MAX) return fail(ctx, CBH_E_ARG, "too many columns for one launch");
  return dispatch_sr(ctx, sr, A->dtype, [&](auto srv) -> int {
    using SR = decltype(srv);
    using VT = typename SR::val_t;
    Scratch S(ctx);
    const int64_t nb = B->nzc;
    int64_t *Adense, *mslot, *hits, *off, *flag, *pos;
    int32_t* Tir;
    VT* Tnum;
    CBH_TRY(S.get(&Adense, A->n + 1));
    CBH_TRY(S.get(&mslot, nb));
    CBH_TRY(S.get(&hits, nb + 1));
    CBH_TRY(S.get(&off, nb + 1));
    CBH_TRY(S.get(&flag, nb + 1));
    CBH_TRY(S.get(&pos, nb + 1));
    CBH_TRY(S.get(&Tir, M->nnz));
    CBH_TRY(S.get(&Tnum, M->nnz));
    hipLaunchKernelGGL(densify_cp_kernel, dim3(blocks_for(A->n + 1, 256)), dim3(256), 0, ctx->stream, A->jc, A->cp,
                       A->nzc, A->n, A->nnz, Adense);
    hipLaunchKernelGGL(match_slots_kernel, dim3(blocks_for(nb, 256)), dim3(256), 0, ctx->stream, B->jc, nb, M->jc,
                       M->nzc, mslot);
    CBH_HIP(ctx, hipMemsetAsync(hits + nb, 0, sizeof(int64_t), ctx->stream));
    MaskArgs a{Adense, A->ir, A->num, B->cp, B->ir, B->num, nb, mslot, M->cp, M->ir, M->num, Tir, Tnum, hits,
               ctx->d_err, A->nnz, A->n};
    if (pattern)
      hipLaunchKernelGGL((masked_kernel<SR, 2048, 256, 256, true>), dim3((unsigned)nb), dim3(256), 0, ctx->stream, a);
    else
      hipLaunchKernelGGL((masked_kernel<SR, 2048, 256, 256, false>), dim3((unsigned)nb), dim3(256), 0, ctx->stream, a);
    CBH_HIP(ctx, hipGetLastError());
    CBH_TRY(exclusive_scan_i64(ctx, S, hits, off, nb + 1));
    hipLaunchKernelGGL(nz_flag_kernel, dim3(blocks_for(nb + 1, 256)), dim3(256), 0, ctx->stream, hits, nb + 1, flag);
    CBH_TRY(exclusive_scan_i64(ctx, S, flag, pos, nb + 1));
    int64_t h[2];
    CBH_HIP(ctx, hipMemcpyAsync(&h[0], off + nb, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(&h[1], pos + nb, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    CBH_TRY(check_err(ctx));
    cbh_mat* out;
    CBH_TRY(new_mat(ctx, A->m, B->n, h[0], h[1], A->dtype, &out));
    hipLaunchKernelGGL(gather_cols_kernel<VT>, dim3(blocks_for(nb, 4)), dim3(256), 0, ctx->stream, mslot, M->cp, hits,
                       off, nb, Tir, Tnum, out->ir, reinterpret_cast<VT*>(out->num));
    hipLaunchKernelGGL(compact_cols_kernel, dim3(blocks_for(nb, 256)), dim3(256), 0, ctx->stream, hits, pos, B->jc, off,
                       nb, out->jc, out->cp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      cbh_mat_free(ctx, out);
      return fail(ctx, CBH_E_HIP, std::string("masked compaction: ") + hipGetErrorString(e));
    }
    *C = out;
    return CBH_OK;
  });
}

int cbh_ewise_mult(cbh_ctx* ctx, const cbh_mat* A, const cbh_mat* B, cbh_mat** C) {
  if (!ctx || !A || !B || !C) return fail(ctx, CBH_E_ARG, "null argument");
  if (A->m != B->m || A->n != B->n) return fail(ctx, CBH_E_DIMMISMATCH, "EWiseMult operands differ in shape");
  if (A->dtype != B->dtype) return fail(ctx, CBH_E_ARG, "EWiseMult operands differ in dtype");
  *C = nullptr;
  if (A->nnz == 0 || B->nnz == 0) return empty_result(ctx, A->m, A->n, A->dtype, C);
  auto run = [&](auto tag) -> int {
    using VT = decltype(tag);
    Scratch S(ctx);
    const int64_t na = A->nzc;
    int64_t *bslot, *hits, *off, *flag, *pos;
    CBH_TRY(S.get(&bslot, na));
    CBH_TRY(S.get(&hits, na + 1));
    CBH_TRY(S.get(&off, na + 1));
    CBH_TRY(S.get(&flag, na + 1));
    CBH_TRY(S.get(&pos, na + 1));
    hipLaunchKernelGGL(match_slots_kernel, dim3(blocks_for(na, 256)), dim3(256), 0, ctx->stream, A->jc, na, B->jc,
                       B->nzc, bslot);
    CBH_HIP(ctx, hipMemsetAsync(hits + na, 0, sizeof(int64_t), ctx->stream));
    const VT* an = reinterpret_cast<const VT*>(A->num);
    const VT* bn = reinterpret_cast<const VT*>(B->num);
    hipLaunchKernelGGL((ewise_kernel<VT, false>), dim3(blocks_for(na, 4)), dim3(256), 0, ctx->stream, A->cp, A->ir, an,
                       na, bslot, B->cp, B->ir, bn, hits, nullptr, nullptr, nullptr);
    CBH_HIP(ctx, hipGetLastError());
    CBH_TRY(exclusive_scan_i64(ctx, S, hits, off, na + 1));
    hipLaunchKernelGGL(nz_flag_kernel, dim3(blocks_for(na + 1, 256)), dim3(256), 0, ctx->stream, hits, na + 1, flag);
    CBH_TRY(exclusive_scan_i64(ctx, S, flag, pos, na + 1));
    int64_t h[2];
    CBH_HIP(ctx, hipMemcpyAsync(&h[0], off + na, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(&h[1], pos + na, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    cbh_mat* out;
    CBH_TRY(new_mat(ctx, A->m, A->n, h[0], h[1], A->dtype, &out));
    hipLaunchKernelGGL((ewise_kernel<VT, true>), dim3(blocks_for(na, 4)), dim3(256), 0, ctx->stream, A->cp, A->ir, an,
                       na, bslot, B->cp, B->ir, bn, hits, off, out->ir, reinterpret_cast<VT*>(out->num));
    hipLaunchKernelGGL(compact_cols_kernel, dim3(blocks_for(na, 256)), dim3(256), 0, ctx->stream, hits, pos, A->jc, off,
                       na, out->jc, out->cp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      cbh_mat_free(ctx, out);
      return fail(ctx, CBH_E_HIP, std::string("ewise: ") + hipGetErrorString(e));
    }
    *C = out;
    return CBH_OK;
  };
  switch (A->dtype) {
    case CBH_F64: return run(double{});
    case CBH_I64: return run(int64_t{});
    case CBH_F32: return run(float{});
    case CBH_I32: return run(int32_t{});
    case CBH_BOOL: return run(uint8_t{});
  }
  return fail(ctx, CBH_E_ARG, "unknown dtype");
}

static int need_f64(cbh_ctx* ctx, const cbh_mat* A) {
  if (!ctx || !A) return fail(ctx, CBH_E_ARG, "null argument");
  if (A->dtype != CBH_F64) return fail(ctx, CBH_E_ARG, "the MCL column operations take f64 matrices");
  return CBH_OK;
}

int cbh_col_stats(cbh_ctx* ctx, const cbh_mat* A, double hard, double* cnt, double* cntp, double* sump) {
  CBH_TRY(need_f64(ctx, A));
  if (!cnt || !cntp || !sump) return fail(ctx, CBH_E_ARG, "null output vector");
  const size_t nb = sizeof(double) * (size_t)A->n;
  CBH_HIP(ctx, hipMemsetAsync(cnt, 0, nb, ctx->stream));
  CBH_HIP(ctx, hipMemsetAsync(cntp, 0, nb, ctx->stream));
  CBH_HIP(ctx, hipMemsetAsync(sump, 0, nb, ctx->stream));
  if (A->nzc > 0) {
    hipLaunchKernelGGL(colstat_kernel, dim3(blocks_for(A->nzc, 4)), dim3(256), 0, ctx->stream, A->jc, A->cp,
                       reinterpret_cast<const double*>(A->num), A->nzc, hard, cnt, cntp, sump);
    CBH_HIP(ctx, hipGetLastError());
  }
  return CBH_OK;
}

int cbh_kselect_hist(cbh_ctx* ctx, const cbh_mat* A, const int32_t* active_index, int64_t nactive,
                     const uint64_t* prefix, int shift, uint32_t* hist) {
  CBH_TRY(need_f64(ctx, A));
  if (shift < 0 || shift > 56 || shift % 8) return fail(ctx, CBH_E_ARG, "radix shift must be 0, 8, ..., 56");
  if (nactive <= 0) return CBH_OK;
  if (!active_index || !prefix || !hist) return fail(ctx, CBH_E_ARG, "null argument");
  CBH_HIP(ctx, hipMemsetAsync(hist, 0, sizeof(uint32_t) * 256 * (size_t)nactive, ctx->stream));
  if (A->nzc > 0) {
    if (A->nzc > INT32_MAX) return fail(ctx, CBH_E_ARG, "too many columns for one launch");
    hipLaunchKernelGGL(kselect_hist_kernel, dim3((unsigned)A->nzc), dim3(256), 0, ctx->stream, A->jc, A->cp,
                       reinterpret_cast<const double*>(A->num), A->nzc, active_index, prefix, shift, hist);
    CBH_HIP(ctx, hipGetLastError());
  }
  return CBH_OK;
}

int cbh_kselect_pick(cbh_ctx* ctx, int64_t nactive, const uint32_t* hist, uint64_t* prefix, int64_t* rank,
                     int shift) {
  if (!ctx) return CBH_E_ARG;
  if (nactive <= 0) return CBH_OK;
  if (!hist || !prefix || !rank) return fail(ctx, CBH_E_ARG, "null argument");
  hipLaunchKernelGGL(kselect_pick_kernel, dim3(blocks_for(nactive, 256)), dim3(256), 0, ctx->stream, nactive, hist,
                     prefix, rank, shift);
  CBH_HIP(ctx, hipGetLastError());
  return CBH_OK;
}

int cbh_kselect_value(cbh_ctx* ctx, int64_t nactive, const uint64_t* prefix, double* out) {
  if (!ctx) return CBH_E_ARG;
  if (nactive <= 0) return CBH_OK;
  if (!prefix || !out) return fail(ctx, CBH_E_ARG, "null argument");
  hipLaunchKernelGGL(kselect_value_kernel, dim3(blocks_for(nactive, 256)), dim3(256), 0, ctx->stream, nactive, prefix,
                     out);
  CBH_HIP(ctx, hipGetLastError());
  return CBH_OK;
}

int cbh_col_stats_kept(cbh_ctx* ctx, const cbh_mat* A, const double* thresh, double* cntk, double* sumk) {
  CBH_TRY(need_f64(ctx, A));
  if (!thresh || !cntk || !sumk) return fail(ctx, CBH_E_ARG, "null argument");
  const size_t nb = sizeof(double) * (size_t)A->n;
  CBH_HIP(ctx, hipMemsetAsync(cntk, 0, nb, ctx->stream));
  CBH_HIP(ctx, hipMemsetAsync(sumk, 0, nb, ctx->stream));
  if (A->nzc > 0) {
    hipLaunchKernelGGL(colstat_kept_kernel, dim3(blocks_for(A->nzc, 4)), dim3(256), 0, ctx->stream, A->jc, A->cp,
                       reinterpret_cast<const double*>(A->num), A->nzc, thresh, cntk, sumk);
    CBH_HIP(ctx, hipGetLastError());
  }
  return CBH_OK;
}

int cbh_kselect_cols(cbh_ctx* ctx, const cbh_mat* A, const int32_t* active_index, int64_t nactive, int64_t k,
                     double* out) {
  CBH_TRY(need_f64(ctx, A));
  if (k < 1) return fail(ctx, CBH_E_ARG, "k must be >= 1");
  if (nactive <= 0) return CBH_OK;
  if (!active_index || !out) return fail(ctx, CBH_E_ARG, "null argument");
  const int64_t nzc = A->nzc;
  if (nzc <= 0) return CBH_OK;
  const double* num = reinterpret_cast<const double*>(A->num);
  // columns of <= 64*R entries: a wave each (keys in registers); <= 256*RB: a workgroup each (keys
  // in registers); <= kSelLong: a workgroup each streaming the keys every round
  constexpr int R = 48, RB = 32;
  constexpr int64_t kSelLong = 1 << 17;
  const int64_t wgrid = std::min<int64_t>((nzc + 3) / 4, 16384);
  hipLaunchKernelGGL(kselect_wave_kernel<R>, dim3((unsigned)wgrid), dim3(256), 0, ctx->stream, A->jc, A->cp, num, nzc,
                     active_index, k, out);
  const int64_t grid = std::min<int64_t>(nzc, 8192);  // workgroups stride over the slots
  hipLaunchKernelGGL((kselect_block_kernel<RB, true>), dim3((unsigned)grid), dim3(256), 0, ctx->stream, A->jc, A->cp,
                     num, nzc, active_index, k, out, (int64_t)64 * R, (int64_t)256 * RB);
  hipLaunchKernelGGL((kselect_block_kernel<1, false>), dim3((unsigned)grid), dim3(256), 0, ctx->stream, A->jc, A->cp,
                     num, nzc, active_index, k, out, (int64_t)256 * RB, kSelLong);
  CBH_HIP(ctx, hipGetLastError());
  // longer columns: chunked over workgroups, 8 radix passes with per-column global histograms
  Scratch S(ctx);
  int64_t *flag, *pos;
  CBH_TRY(S.get(&flag, nzc + 1));
  CBH_TRY(S.get(&pos, nzc + 1));
  hipLaunchKernelGGL(kselect_long_flag_kernel, dim3(blocks_for(nzc + 1, 256)), dim3(256), 0, ctx->stream, A->jc, A->cp,
                     nzc, active_index, kSelLong, flag);
  CBH_TRY(exclusive_scan_i64(ctx, S, flag, pos, nzc + 1));
  int64_t nl = 0;
  CBH_HIP(ctx, hipMemcpyAsync(&nl, pos + nzc, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (nl == 0) return CBH_OK;
  int64_t *list, *nch, *cpos, *rank;
  uint64_t* prefix;
  uint32_t* hist;
  CBH_TRY(S.get(&list, nl));
  CBH_TRY(S.get(&nch, nl + 1));
  CBH_TRY(S.get(&cpos, nl + 1));
  CBH_TRY(S.get(&rank, nl));
  CBH_TRY(S.get(&prefix, nl));
  CBH_TRY(S.get(&hist, 256 * nl));
  CBH_HIP(ctx, hipMemsetAsync(nch + nl, 0, sizeof(int64_t), ctx->stream));
  hipLaunchKernelGGL(kselect_long_list_kernel, dim3(blocks_for(nzc, 256)), dim3(256), 0, ctx->stream, A->cp, nzc, flag,
                     pos, k, list, nch, rank, prefix);
  CBH_TRY(exclusive_scan_i64(ctx, S, nch, cpos, nl + 1));
  int64_t nchunks = 0;
  CBH_HIP(ctx, hipMemcpyAsync(&nchunks, cpos + nl, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  int32_t* map;
  CBH_TRY(S.get(&map, nchunks));
  hipLaunchKernelGGL(kselect_long_map_kernel, dim3(blocks_for(nl, 256)), dim3(256), 0, ctx->stream, nl, nch, cpos, map);
  const unsigned hgrid = (unsigned)std::min<int64_t>(nchunks, 16384);
  for (int shift = 56; shift >= 0; shift -= 8) {
    CBH_HIP(ctx, hipMemsetAsync(hist, 0, sizeof(uint32_t) * 256 * (size_t)nl, ctx->stream));
    hipLaunchKernelGGL(kselect_long_hist_kernel, dim3(hgrid), dim3(256), 0, ctx->stream, A->cp, num, list, cpos, map,
                       nchunks, prefix, shift, hist);
    hipLaunchKernelGGL(kselect_pick_kernel, dim3(blocks_for(nl, 256)), dim3(256), 0, ctx->stream, nl, hist, prefix, rank,
                       shift);
  }
  hipLaunchKernelGGL(kselect_long_out_kernel, dim3(blocks_for(nl, 256)), dim3(256), 0, ctx->stream, nl, list, A->jc,
                     active_index, prefix, out);
  CBH_HIP(ctx, hipGetLastError());
  return CBH_OK;  // (the scratch returns to the stream-ordered cache)
}

static int prune_columns_impl(cbh_ctx* ctx, const cbh_mat* A, const double* thresh, cbh_arena* ar, cbh_mat** C);
int cbh_prune_columns(cbh_ctx* ctx, const cbh_mat* A, const double* thresh, cbh_mat** C) {
  return prune_columns_impl(ctx, A, thresh, nullptr, C);
}
static int prune_columns_impl(cbh_ctx* ctx, const cbh_mat* A, const double* thresh, cbh_arena* ar, cbh_mat** C) {
  CBH_TRY(need_f64(ctx, A));
  if (!thresh || !C) return fail(ctx, CBH_E_ARG, "null argument");
  *C = nullptr;
  if (A->nnz == 0) return empty_result(ctx, A->m, A->n, A->dtype, C);
  Scratch S(ctx);
  const int64_t nz = A->nzc;
  int64_t *kept, *off, *flag, *pos;
  CBH_TRY(S.get(&kept, nz + 1));
  CBH_TRY(S.get(&off, nz + 1));
  CBH_TRY(S.get(&flag, nz + 1));
  CBH_TRY(S.get(&pos, nz + 1));
  const double* num = reinterpret_cast<const double*>(A->num);
  CBH_HIP(ctx, hipMemsetAsync(kept + nz, 0, sizeof(int64_t), ctx->stream));
  hipLaunchKernelGGL(prune_col_kernel<false>, dim3(blocks_for(nz, 4)), dim3(256), 0, ctx->stream, A->jc, A->cp, A->ir,
                     num, nz, thresh, kept, nullptr, nullptr, nullptr);
  CBH_HIP(ctx, hipGetLastError());
  CBH_TRY(exclusive_scan_i64(ctx, S, kept, off, nz + 1));
  hipLaunchKernelGGL(nz_flag_kernel, dim3(blocks_for(nz + 1, 256)), dim3(256), 0, ctx->stream, kept, nz + 1, flag);
  CBH_TRY(exclusive_scan_i64(ctx, S, flag, pos, nz + 1));
  int64_t h[2];
  CBH_HIP(ctx, hipMemcpyAsync(&h[0], off + nz, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipMemcpyAsync(&h[1], pos + nz, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  cbh_mat* out;
  if (ar && !ar->overflow && ar->vbytes == 8 && ar->used + h[0] <= ar->cap) {  // rows and values into the arena
    CBH_TRY(new_mat(ctx, A->m, A->n, 0, h[1], A->dtype, &out));
    dfree(ctx, out->ir);
    dfree(ctx, out->num);
    out->nnz = h[0];
    out->ir = ar->ir + ar->used;
    out->num = ar->num + ar->used * ar->vbytes;
    out->borrowed_rows = true;
    ar->used += h[0];
  } else {
    if (ar) ar->overflow = true;
    CBH_TRY(new_mat(ctx, A->m, A->n, h[0], h[1], A->dtype, &out));
  }
  hipLaunchKernelGGL(prune_col_kernel<true>, dim3(blocks_for(nz, 4)), dim3(256), 0, ctx->stream, A->jc, A->cp, A->ir,
                     num, nz, thresh, kept, off, out->ir, reinterpret_cast<double*>(out->num));
  hipLaunchKernelGGL(compact_cols_kernel, dim3(blocks_for(nz, 256)), dim3(256), 0, ctx->stream, kept, pos, A->jc, off,
                     nz, out->jc, out->cp);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cbh_mat_free(ctx, out);
    return fail(ctx, CBH_E_HIP, std::string("prune: ") + hipGetErrorString(e));
  }
  *C = out;
  return CBH_OK;
}

// ---------------------------------------------------------------------------- block column ops
int cbh_mat_col_slice(cbh_ctx* ctx, const cbh_mat* M, int64_t c0, int64_t c1, cbh_mat** out) {
  if (!ctx || !M || !out) return fail(ctx, CBH_E_ARG, "null argument");
  if (c0 < 0 || c1 < c0 || c1 > M->n) return fail(ctx, CBH_E_ARG, "column range outside the block");
  *out = nullptr;
  if (M->nzc == 0) {
    CBH_TRY(new_mat(ctx, M->m, c1 - c0, 0, 0, M->dtype, out, M->vbytes));
    CBH_HIP(ctx, hipMemsetAsync((*out)->cp, 0, sizeof(int64_t), ctx->stream));
    return CBH_OK;
  }
  Scratch S(ctx);
  int64_t* d;
  CBH_TRY(S.get(&d, 4));
  hipLaunchKernelGGL(col_range_kernel, dim3(1), dim3(64), 0, ctx->stream, M->jc, M->cp, M->nzc, c0, c1, d);
  CBH_HIP(ctx, hipGetLastError());
  int64_t h[4];
  CBH_HIP(ctx, hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  const int64_t nzc = h[1] - h[0], nnz = h[3] - h[2];
  cbh_mat* C;
  CBH_TRY(new_mat(ctx, M->m, c1 - c0, nnz, nzc, M->dtype, &C, M->vbytes));
  hipLaunchKernelGGL(add_const_i64_kernel, dim3(blocks_for(nzc + 1, 256)), dim3(256), 0, ctx->stream, M->cp + h[0],
                     nzc + 1, -h[2], C->cp);
  if (nzc > 0)
    hipLaunchKernelGGL(add_const_i64_kernel, dim3(blocks_for(nzc, 256)), dim3(256), 0, ctx->stream, M->jc + h[0], nzc,
                       -c0, C->jc);
  if (nnz > 0) {
    CBH_HIP(ctx, hipMemcpyAsync(C->ir, M->ir + h[2], sizeof(int32_t) * nnz, hipMemcpyDeviceToDevice, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(C->num, static_cast<const char*>(M->num) + h[2] * M->vbytes, (size_t)(nnz * M->vbytes),
                                hipMemcpyDeviceToDevice, ctx->stream));
  }
  CBH_HIP(ctx, hipGetLastError());
  *out = C;
  return CBH_OK;
}

int cbh_mat_col_view(cbh_ctx* ctx, const cbh_mat* M, int64_t c0, int64_t c1, cbh_mat** out) {
  if (!ctx || !M || !out) return fail(ctx, CBH_E_ARG, "null argument");
  if (c0 < 0 || c1 < c0 || c1 > M->n) return fail(ctx, CBH_E_ARG, "column range outside the block");
  *out = nullptr;
  if (M->nzc == 0) {
    CBH_TRY(new_mat(ctx, M->m, c1 - c0, 0, 0, M->dtype, out, M->vbytes));
    CBH_HIP(ctx, hipMemsetAsync((*out)->cp, 0, sizeof(int64_t), ctx->stream));
    return CBH_OK;
  }
  Scratch S(ctx);
  int64_t* d;
  CBH_TRY(S.get(&d, 4));
  hipLaunchKernelGGL(col_range_kernel, dim3(1), dim3(64), 0, ctx->stream, M->jc, M->cp, M->nzc, c0, c1, d);
  CBH_HIP(ctx, hipGetLastError());
  int64_t h[4];
  CBH_HIP(ctx, hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  const int64_t nzc = h[1] - h[0], nnz = h[3] - h[2];
  cbh_mat* C;
  CBH_TRY(new_mat(ctx, M->m, c1 - c0, 0, nzc, M->dtype, &C, M->vbytes));
  dfree(ctx, C->ir);
  dfree(ctx, C->num);
  C->nnz = nnz;
  C->ir = M->ir + h[2];
  C->num = static_cast<char*>(M->num) + h[2] * M->vbytes;
  C->borrowed_rows = true;
  hipLaunchKernelGGL(add_const_i64_kernel, dim3(blocks_for(nzc + 1, 256)), dim3(256), 0, ctx->stream, M->cp + h[0],
                     nzc + 1, -h[2], C->cp);
  if (nzc > 0)
    hipLaunchKernelGGL(add_const_i64_kernel, dim3(blocks_for(nzc, 256)), dim3(256), 0, ctx->stream, M->jc + h[0], nzc,
                       -c0, C->jc);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cbh_mat_free(ctx, C);
    return fail(ctx, CBH_E_HIP, std::string("col_view: ") + hipGetErrorString(e));
  }
  *out = C;
  return CBH_OK;
}

int cbh_mat_row_slice(cbh_ctx* ctx, const cbh_mat* M, int64_t r0, int64_t r1, cbh_mat** out) {
  if (!ctx || !M || !out) return fail(ctx, CBH_E_ARG, "null argument");
  if (r0 < 0 || r1 < r0 || r1 > M->m) return fail(ctx, CBH_E_ARG, "row range outside the block");
  *out = nullptr;
  if (M->nzc == 0) {
    CBH_TRY(new_mat(ctx, r1 - r0, M->n, 0, 0, M->dtype, out, M->vbytes));
    CBH_HIP(ctx, hipMemsetAsync((*out)->cp, 0, sizeof(int64_t), ctx->stream));
    return CBH_OK;
  }
  Scratch S(ctx);
  const int64_t nz = M->nzc;
  int64_t *first, *cnt, *off, *flag, *pos;
  CBH_TRY(S.get(&first, nz + 1));
  CBH_TRY(S.get(&cnt, nz + 1));
  CBH_TRY(S.get(&off, nz + 1));
  CBH_TRY(S.get(&flag, nz + 1));
  CBH_TRY(S.get(&pos, nz + 1));
  hipLaunchKernelGGL(row_range_kernel, dim3(blocks_for(nz, 256)), dim3(256), 0, ctx->stream, M->cp, M->ir, nz,
                     (int32_t)r0, (int32_t)r1, first, cnt);
  CBH_HIP(ctx, hipMemsetAsync(cnt + nz, 0, sizeof(int64_t), ctx->stream));
  CBH_TRY(exclusive_scan_i64(ctx, S, cnt, off, nz + 1));
  hipLaunchKernelGGL(nz_flag_kernel, dim3(blocks_for(nz + 1, 256)), dim3(256), 0, ctx->stream, cnt, nz + 1, flag);
  CBH_TRY(exclusive_scan_i64(ctx, S, flag, pos, nz + 1));
  int64_t h[2];
  CBH_HIP(ctx, hipMemcpyAsync(&h[0], off + nz, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipMemcpyAsync(&h[1], pos + nz, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  cbh_mat* C;
  CBH_TRY(new_mat(ctx, r1 - r0, M->n, h[0], h[1], M->dtype, &C, M->vbytes));
  hipLaunchKernelGGL(row_slice_copy_kernel, dim3(blocks_for(nz, 4)), dim3(256), 0, ctx->stream, first, cnt, off, M->ir,
                     static_cast<const char*>(M->num), nz, (int32_t)r0, M->vbytes, C->ir, static_cast<char*>(C->num));
  hipLaunchKernelGGL(compact_cols_kernel, dim3(blocks_for(nz, 256)), dim3(256), 0, ctx->stream, cnt, pos, M->jc, off, nz,
                     C->jc, C->cp);
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess && h[1] == 0) (void)hipMemsetAsync(C->cp, 0, sizeof(int64_t), ctx->stream);
  if (e != hipSuccess) {
    cbh_mat_free(ctx, C);
    return fail(ctx, CBH_E_HIP, std::string("row slice: ") + hipGetErrorString(e));
  }
  *out = C;
  return CBH_OK;
}

int cbh_mat_rebase_cols(cbh_ctx* ctx, cbh_mat* M, int64_t c0, int64_t n) {
  if (!ctx || !M || c0 < 0 || n < 0) return fail(ctx, CBH_E_ARG, "bad rebase arguments");
  if (M->nzc > 0) {
    int64_t h[2];
    CBH_HIP(ctx, hipMemcpyAsync(&h[0], M->jc, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipMemcpyAsync(&h[1], M->jc + M->nzc - 1, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (h[0] < c0 || h[1] >= c0 + n) return fail(ctx, CBH_E_ARG, "columns outside [c0, c0 + n)");
    hipLaunchKernelGGL(add_const_i64_kernel, dim3(blocks_for(M->nzc, 256)), dim3(256), 0, ctx->stream, M->jc, M->nzc, -c0,
                       M->jc);
    CBH_HIP(ctx, hipGetLastError());
  }
  M->n = n;
  return CBH_OK;
}

int cbh_mat_col_concat(cbh_ctx* ctx, int k, const cbh_mat* const* parts, cbh_mat** out) {
  if (!ctx || !out || k < 1 || !parts) return fail(ctx, CBH_E_ARG, "bad concat arguments");
  *out = nullptr;
  int64_t m = 0, n = 0, nnz = 0, nzc = 0;
  for (int i = 0; i < k; ++i) {
    if (!parts[i]) return fail(ctx, CBH_E_ARG, "null block");
    if (parts[i]->dtype != parts[0]->dtype || parts[i]->vbytes != parts[0]->vbytes)
      return fail(ctx, CBH_E_ARG, "blocks of different value types");
    m = std::max(m, parts[i]->m);
    n += parts[i]->n;
    nnz += parts[i]->nnz;
    nzc += parts[i]->nzc;
  }
  cbh_mat* C;
  CBH_TRY(new_mat(ctx, m, n, nnz, nzc, parts[0]->dtype, &C, parts[0]->vbytes));
  const int64_t vb = parts[0]->vbytes;
  int64_t coff = 0, eoff = 0, zoff = 0;
  for (int i = 0; i < k; ++i) {
    const cbh_mat* P = parts[i];
    if (P->nzc > 0) {
      hipLaunchKernelGGL(add_const_i64_kernel, dim3(blocks_for(P->nzc, 256)), dim3(256), 0, ctx->stream, P->cp, P->nzc,
                         eoff, C->cp + zoff);
      hipLaunchKernelGGL(add_const_i64_kernel, dim3(blocks_for(P->nzc, 256)), dim3(256), 0, ctx->stream, P->jc, P->nzc,
                         coff, C->jc + zoff);
    }
    if (P->nnz > 0) {
      CBH_HIP(ctx, hipMemcpyAsync(C->ir + eoff, P->ir, sizeof(int32_t) * P->nnz, hipMemcpyDeviceToDevice, ctx->stream));
      CBH_HIP(ctx, hipMemcpyAsync(static_cast<char*>(C->num) + eoff * vb, P->num, (size_t)(P->nnz * vb),
                                  hipMemcpyDeviceToDevice, ctx->stream));
    }
    coff += P->n;
    eoff += P->nnz;
    zoff += P->nzc;
  }
  CBH_HIP(ctx, hipMemcpyAsync(C->cp + nzc, &nnz, sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // nnz is a host local
  CBH_HIP(ctx, hipGetLastError());
  *out = C;
  return CBH_OK;
}

// cbh_mat_col_concat that releases the parts as it goes, one array kind at a time (pointers, then
// rows, then values): the peak is the parts plus the largest output array, not twice the matrix
// (a C5 step's pruned pieces are 148 GB; a copying concatenation would need 296 GB beside A and B)
// The consuming concatenation. arena: the pruned pieces' arena when they borrow its rows and values
// but could not take them over (cbh_arena_concat's fallback): its rows / values are released as soon
// as they are copied, like an owned part's. On a failure after C's allocation both C and every part
// are released (the parts are half consumed by then), and the error is returned.
static int concat_consume(cbh_ctx* ctx, int k, cbh_mat** parts, cbh_mat** out, cbh_arena* arena) {
  if (!ctx || !out || k < 1 || !parts) return fail(ctx, CBH_E_ARG, "bad concat arguments");
  *out = nullptr;
  int64_t m = 0, n = 0, nnz = 0, nzc = 0;
  for (int i = 0; i < k; ++i) {
    if (!parts[i]) return fail(ctx, CBH_E_ARG, "null block");
    if (parts[i]->dtype != parts[0]->dtype || parts[i]->vbytes != parts[0]->vbytes)
      return fail(ctx, CBH_E_ARG, "blocks of different value types");
    m = std::max(m, parts[i]->m);
    n += parts[i]->n;
    nnz += parts[i]->nnz;
    nzc += parts[i]->nzc;
  }
  cbh_mat* C = new cbh_mat;
  C->m = m;
  C->n = n;
  C->nnz = nnz;
  C->nzc = nzc;
  C->dtype = parts[0]->dtype;
  C->vbytes = parts[0]->vbytes;
  const int64_t vb = C->vbytes;
  auto release = [&](auto member, bool rows) {  // rows: ir / num, which arena pieces only borrow
    for (int i = 0; i < k; ++i)
      if (parts[i]->owned && !(rows && parts[i]->borrowed_rows)) {
        dfree(ctx, parts[i]->*member);
        parts[i]->*member = nullptr;
      }
  };
  const int rc = [&]() -> int {  // (CBH_HIP / CBH_TRY return from here)
  CBH_TRY(dalloc(ctx, &C->cp, nzc + 1));
  CBH_TRY(dalloc(ctx, &C->jc, nzc));
  int64_t coff = 0, eoff = 0, zoff = 0;
  for (int i = 0; i < k; ++i) {
    const cbh_mat* P = parts[i];
    if (P->nzc > 0) {
      hipLaunchKernelGGL(add_const_i64_kernel, dim3(blocks_for(P->nzc, 256)), dim3(256), 0, ctx->stream, P->cp, P->nzc,
                         eoff, C->cp + zoff);
      hipLaunchKernelGGL(add_const_i64_kernel, dim3(blocks_for(P->nzc, 256)), dim3(256), 0, ctx->stream, P->jc, P->nzc,
                         coff, C->jc + zoff);
    }
    coff += P->n;
    eoff += P->nnz;
    zoff += P->nzc;
  }
  CBH_HIP(ctx, hipGetLastError());
  release(&cbh_mat::cp, false);
  release(&cbh_mat::jc, false);
  if (std::getenv("CBH_MEMDIAG")) {
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    std::fprintf(stderr, "[cbh memdiag] concat: %d parts, device free %.2f GB, rows need %.2f GB\n", k, fr / 1e9,
                 nnz * 4 / 1e9);
  }
  CBH_TRY(dalloc(ctx, &C->ir, nnz));
  eoff = 0;
  for (int i = 0; i < k; ++i) {
    if (parts[i]->nnz > 0)
      CBH_HIP(ctx, hipMemcpyAsync(C->ir + eoff, parts[i]->ir, sizeof(int32_t) * parts[i]->nnz, hipMemcpyDeviceToDevice,
                                  ctx->stream));
    eoff += parts[i]->nnz;
  }
  release(&cbh_mat::ir, true);
  if (arena) {  // (stream-ordered: the copies above run first)
    dfree(ctx, arena->ir);
    arena->ir = nullptr;
  }
  if (std::getenv("CBH_MEMDIAG")) {
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    std::fprintf(stderr, "[cbh memdiag] concat: rows copied and released, device free %.2f GB, values need %.2f GB\n",
                 fr / 1e9, nnz * vb / 1e9);
  }
  CBH_TRY(dalloc(ctx, reinterpret_cast<char**>(&C->num), nnz * vb));
  eoff = 0;
  for (int i = 0; i < k; ++i) {
    if (parts[i]->nnz > 0)
      CBH_HIP(ctx, hipMemcpyAsync(static_cast<char*>(C->num) + eoff * vb, parts[i]->num, (size_t)(parts[i]->nnz * vb),
                                  hipMemcpyDeviceToDevice, ctx->stream));
    eoff += parts[i]->nnz;
  }
  release(&cbh_mat::num, true);
  if (arena) {
    dfree(ctx, arena->num);
    arena->num = nullptr;
    arena->cap = arena->used = 0;
  }
  CBH_HIP(ctx, hipMemcpyAsync(C->cp + nzc, &nnz, sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // nnz is a host local
  CBH_HIP(ctx, hipGetLastError());
  return CBH_OK;
  }();
  for (int i = 0; i < k; ++i) {
    cbh_mat_free(ctx, parts[i]);
    parts[i] = nullptr;
  }
  if (rc != CBH_OK) {
    cbh_mat_free(ctx, C);
    return rc;
  }
  *out = C;
  return CBH_OK;
}

int cbh_mat_col_concat_consume(cbh_ctx* ctx, int k, cbh_mat** parts, cbh_mat** out) {
  return concat_consume(ctx, k, parts, out, nullptr);
}

int cbh_arena_create(cbh_ctx* ctx, int64_t capacity, int64_t value_bytes, cbh_arena** out) {
  if (!ctx || !out || capacity < 0 || value_bytes <= 0) return fail(ctx, CBH_E_ARG, "bad arena arguments");
  *out = nullptr;
  cbh_arena* a = new cbh_arena;
  a->cap = capacity;
  a->vbytes = value_bytes;
  int rc = dalloc(ctx, &a->ir, (size_t)capacity);
  if (rc == CBH_OK) rc = dalloc(ctx, &a->num, (size_t)(capacity * value_bytes));
  if (rc != CBH_OK) {
    dfree(ctx, a->ir);
    delete a;
    return rc;
  }
  *out = a;
  return CBH_OK;
}
int cbh_arena_destroy(cbh_ctx* ctx, cbh_arena* a) {
  if (!a) return CBH_OK;
  if (ctx) {
    dfree(ctx, a->ir);
    dfree(ctx, a->num);
  }
  delete a;
  return CBH_OK;
}
// The pieces side by side (as cbh_mat_col_concat_consume). When they were all pruned into the arena,
// back to back in order, their rows and values already form the result's arrays: the result takes
// the arena's arrays over (the arena is left empty) and only the column pointers and ids are built.
int cbh_arena_concat(cbh_ctx* ctx, int k, cbh_mat** parts, cbh_arena* a, cbh_mat** out) {
  if (!ctx || !out || k < 1 || !parts || !a) return fail(ctx, CBH_E_ARG, "bad arena concat arguments");
  bool contiguous = !a->overflow;
  int64_t off = 0, m = 0, n = 0, nzc = 0;
  for (int i = 0; i < k && contiguous; ++i) {
    const cbh_mat* P = parts[i];
    if (!P) return fail(ctx, CBH_E_ARG, "null block");
    if (P->nnz > 0 && (!P->borrowed_rows || P->ir != a->ir + off || static_cast<char*>(P->num) != a->num + off * a->vbytes))
      contiguous = false;
    off += P->nnz;
  }
  if (!contiguous || off != a->used) return concat_consume(ctx, k, parts, out, a);
  for (int i = 0; i < k; ++i) {
    m = std::max(m, parts[i]->m);
    n += parts[i]->n;
    nzc += parts[i]->nzc;
  }
  cbh_mat* C = new cbh_mat;
  C->m = m;
  C->n = n;
  C->nnz = off;
  C->nzc = nzc;
  C->dtype = parts[0]->dtype;
  C->vbytes = parts[0]->vbytes;
  int rc = dalloc(ctx, &C->cp, nzc + 1);
  if (rc == CBH_OK) rc = dalloc(ctx, &C->jc, nzc);
  if (rc != CBH_OK) {
    cbh_mat_free(ctx, C);
    return rc;
  }
  int64_t coff = 0, eoff = 0, zoff = 0;
  for (int i = 0; i < k; ++i) {
    const cbh_mat* P = parts[i];
    if (P->nzc > 0) {
      hipLaunchKernelGGL(add_const_i64_kernel, dim3(blocks_for(P->nzc, 256)), dim3(256), 0, ctx->stream, P->cp, P->nzc,
                         eoff, C->cp + zoff);
      hipLaunchKernelGGL(add_const_i64_kernel, dim3(blocks_for(P->nzc, 256)), dim3(256), 0, ctx->stream, P->jc, P->nzc,
                         coff, C->jc + zoff);
    }
    coff += P->n;
    eoff += P->nnz;
    zoff += P->nzc;
  }
  C->ir = a->ir;  // the arena's arrays become the result's (capacity >= nnz)
  C->num = a->num;
  a->ir = nullptr;
  a->num = nullptr;
  a->cap = a->used = 0;
  CBH_HIP(ctx, hipMemcpyAsync(C->cp + nzc, &off, sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // off is a host local
  CBH_HIP(ctx, hipGetLastError());
  for (int i = 0; i < k; ++i) {
    cbh_mat_free(ctx, parts[i]);
    parts[i] = nullptr;
  }
  *out = C;
  return CBH_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------- MCLPruneRecoverySelect
// Kselect1 of the flagged columns into thresh (see cbh_mcl_prune_recovery_select)
static int mcl_kselect(cbh_ctx* ctx, Scratch& S, const cbh_mat* A, const int64_t* flag, const double* tot, int64_t k,
                       cbh_allreduce_fn colsum, void* user, double* thresh) {
  const int64_t n = A->n;
  int64_t* pos;
  int32_t* aidx;
  CBH_TRY(S.get(&pos, n + 1));
  CBH_TRY(S.get(&aidx, n));
  CBH_TRY(exclusive_scan_i64(ctx, S, flag, pos, n + 1));
  int64_t nact = 0;
  CBH_HIP(ctx, hipMemcpyAsync(&nact, pos + n, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (nact == 0) return CBH_OK;
  hipLaunchKernelGGL(active_index_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, n, flag, pos, aidx);
  double *kth, *totact;
  CBH_TRY(S.get(&kth, nact));
  CBH_TRY(S.get(&totact, nact));
  if (!colsum) {  // columns held whole: one launch, columns staged in LDS
    const double dmin = 2.2250738585072014e-308;
    hipLaunchKernelGGL(fill_f64_kernel, dim3(blocks_for(nact, 256)), dim3(256), 0, ctx->stream, kth, nact, dmin);
    CBH_TRY(cbh_kselect_cols(ctx, A, aidx, nact, k, kth));
    hipLaunchKernelGGL(kselect_scatter_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, n, aidx, kth,
                       (const double*)nullptr, thresh);
  } else {  // 8 radix passes, digit histograms summed over the processor column
    int64_t* rank;
    uint64_t* prefix;
    uint32_t* hist;
    CBH_TRY(S.get(&rank, nact));
    CBH_TRY(S.get(&prefix, nact));
    CBH_TRY(S.get(&hist, 256 * nact));
    hipLaunchKernelGGL(kselect_rank_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, n, aidx, tot, k, rank,
                       prefix, totact);
    for (int shift = 56; shift >= 0; shift -= 8) {
      CBH_TRY(cbh_kselect_hist(ctx, A, aidx, nact, prefix, shift, hist));
      const int rc = colsum(user, hist, 256 * nact, CBH_REDUCE_U32);
      if (rc != 0) return fail(ctx, rc, "processor-column reduction of the Kselect histograms failed");
      CBH_TRY(cbh_kselect_pick(ctx, nact, hist, prefix, rank, shift));
    }
    CBH_TRY(cbh_kselect_value(ctx, nact, prefix, kth));
    hipLaunchKernelGGL(kselect_scatter_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, n, aidx, kth, totact,
                       thresh);
  }
  CBH_HIP(ctx, hipGetLastError());
  return CBH_OK;
}

static int mcl_prune_impl(cbh_ctx* ctx, const cbh_mat* A, double hardThreshold, int64_t selectNum, int64_t recoverNum,
                          double recoverPct, cbh_allreduce_fn colsum, void* user, cbh_arena* ar, cbh_mat** C);
extern "C" int cbh_mcl_prune_recovery_select(cbh_ctx* ctx, const cbh_mat* A, double hardThreshold, int64_t selectNum,
                                             int64_t recoverNum, double recoverPct, cbh_allreduce_fn colsum,
                                             void* user, cbh_mat** C) {
  return mcl_prune_impl(ctx, A, hardThreshold, selectNum, recoverNum, recoverPct, colsum, user, nullptr, C);
}
extern "C" int cbh_mcl_prune_recovery_select_arena(cbh_ctx* ctx, const cbh_mat* A, double hardThreshold,
                                                   int64_t selectNum, int64_t recoverNum, double recoverPct,
                                                   cbh_allreduce_fn colsum, void* user, cbh_arena* ar, cbh_mat** C) {
  return mcl_prune_impl(ctx, A, hardThreshold, selectNum, recoverNum, recoverPct, colsum, user, ar, C);
}
static int mcl_prune_impl(cbh_ctx* ctx, const cbh_mat* A, double hardThreshold, int64_t selectNum, int64_t recoverNum,
                          double recoverPct, cbh_allreduce_fn colsum, void* user, cbh_arena* ar, cbh_mat** C) {
  CBH_TRY(need_f64(ctx, A));
  if (!C) return fail(ctx, CBH_E_ARG, "null output");
  *C = nullptr;
  const int64_t n = A->n;
  if (n == 0) return empty_result(ctx, A->m, A->n, A->dtype, C);
  Scratch S(ctx);
  double *st, *thresh, *kept;
  int64_t *rec, *sel, *s2;
  CBH_TRY(S.get(&st, 3 * n));  // cnt | cntp | sump, reduced in one call
  CBH_TRY(S.get(&thresh, n));
  CBH_TRY(S.get(&kept, 2 * n));
  CBH_TRY(S.get(&rec, n + 1));
  CBH_TRY(S.get(&sel, n + 1));
  CBH_TRY(S.get(&s2, n + 1));
  double *cnt = st, *cntp = st + n, *sump = st + 2 * n;
  CBH_TRY(cbh_col_stats(ctx, A, hardThreshold, cnt, cntp, sump));
  if (colsum) {
    const int rc = colsum(user, st, 3 * n, CBH_REDUCE_F64);
    if (rc != 0) return fail(ctx, rc, "processor-column reduction of the column statistics failed");
  }
  hipLaunchKernelGGL(mcl_flags_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, n, cnt, cntp, sump,
                     hardThreshold, selectNum, recoverNum, recoverPct, thresh, rec, sel);
  CBH_HIP(ctx, hipGetLastError());
  // recovery: the recoverNum-th largest of the UNPRUNED column (A.Kselect, ParFriends.h:221-236)
  if (recoverNum > 0) CBH_TRY(mcl_kselect(ctx, S, A, rec, cnt, recoverNum, colsum, user, thresh));
  if (selectNum > 0) {  // selection (:239-270), then recovery of what selection left too thin (:272-330)
    CBH_TRY(mcl_kselect(ctx, S, A, sel, cnt, selectNum, colsum, user, thresh));
    if (recoverNum > 0) {
      CBH_TRY(cbh_col_stats_kept(ctx, A, thresh, kept, kept + n));
      if (colsum) {
        const int rc = colsum(user, kept, 2 * n, CBH_REDUCE_F64);
        if (rc != 0) return fail(ctx, rc, "processor-column reduction of the kept statistics failed");
      }
      hipLaunchKernelGGL(mcl_recheck_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, n, sel, kept,
                         kept + n, recoverNum, recoverPct, s2);
      CBH_TRY(mcl_kselect(ctx, S, A, s2, cnt, recoverNum, colsum, user, thresh));
    }
  }
  return prune_columns_impl(ctx, A, thresh, ar, C);  // PruneColumn(pruneCols, less, true) (:343)
}

// ============================================================================ format conversions
// SURVEY.md §8(f)3 (kernels in convert.h): the SpTuples -> SpDCCols build and back, on the device.
template <class V>
static void launch_tuple_reduce(cbh_ctx* ctx, const uint64_t* key, const int64_t* perm, const int64_t* head,
                                const int64_t* pos, int64_t nnz, int64_t m, const void* vin, int32_t* ir, uint64_t* ukey,
                                void* vout) {
  hipLaunchKernelGGL(tuple_reduce_kernel<V>, dim3(blocks_for(nnz, 256)), dim3(256), 0, ctx->stream, key, perm, head, pos,
                     nnz, m, reinterpret_cast<const V*>(vin), ir, ukey, reinterpret_cast<V*>(vout));
}

extern "C" int cbh_tuples_to_dcsc(cbh_ctx* ctx, int64_t m, int64_t n, int64_t nnz, const int32_t* rows,
                                  const int64_t* cols, const void* vals, cbh_dtype dtype, uint32_t flags,
                                  cbh_mat** out) {
  if (!ctx || !out || nnz < 0 || m < 0 || n < 0 || dtype_size(dtype) == 0 || (nnz > 0 && (!rows || !cols || !vals)))
    return fail(ctx, CBH_E_ARG, "bad tuples_to_dcsc arguments");
  *out = nullptr;
  if (m > INT32_MAX) return fail(ctx, CBH_E_DIMMISMATCH, "local row count exceeds 32-bit row ids");
  if (nnz > INT32_MAX) return fail(ctx, CBH_E_ARG, "at most 2^31-1 tuples per conversion");
  if (m > 0 && n > (int64_t)(UINT64_MAX / 2 / (uint64_t)m)) return fail(ctx, CBH_E_ARG, "m*n exceeds 63-bit keys");
  if (nnz == 0 || m == 0 || n == 0) return empty_result(ctx, m, n, dtype, out);
  Scratch S(ctx);
  uint64_t *k0, *k1, *ukey;
  int64_t *i0, *i1, *head, *pos, *flag, *cpos;
  int32_t* ir;
  char* vout;
  const size_t vs = dtype_size(dtype);
  CBH_TRY(S.get(&k0, nnz));
  CBH_TRY(S.get(&k1, nnz));
  CBH_TRY(S.get(&i0, nnz));
  CBH_TRY(S.get(&i1, nnz));
  CBH_TRY(S.get(&head, nnz + 1));
  CBH_TRY(S.get(&pos, nnz + 1));
  hipLaunchKernelGGL(tuple_keys_kernel, dim3(blocks_for(nnz, 256)), dim3(256), 0, ctx->stream, rows, cols, nnz, m, n,
                     k0, i0, ctx->d_err);
  CBH_HIP(ctx, hipGetLastError());
  int end_bit = 1;
  while (end_bit < 64 && (((uint64_t)m * (uint64_t)n - 1) >> end_bit) != 0) ++end_bit;
  size_t tmp = 0;
  CBH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, k0, k1, i0, i1, (int)nnz, 0, end_bit, ctx->stream));
  char* t;
  CBH_TRY(S.get(&t, tmp));
  CBH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(t, tmp, k0, k1, i0, i1, (int)nnz, 0, end_bit, ctx->stream));
  hipLaunchKernelGGL(tuple_heads_kernel, dim3(blocks_for(nnz, 256)), dim3(256), 0, ctx->stream, k1, nnz, m,
                     (flags & CBH_TUPLES_DROP_LOOPS) != 0, head);
  CBH_HIP(ctx, hipMemsetAsync(head + nnz, 0, sizeof(int64_t), ctx->stream));
  CBH_TRY(exclusive_scan_i64(ctx, S, head, pos, nnz + 1));
  int64_t u = 0;
  CBH_HIP(ctx, hipMemcpyAsync(&u, pos + nnz, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (u == 0) {
    CBH_TRY(check_err(ctx));
    return empty_result(ctx, m, n, dtype, out);
  }
  CBH_TRY(S.get(&ir, u));
  CBH_TRY(S.get(&ukey, u));
  CBH_TRY(S.get(&vout, u * vs));
  CBH_TRY(S.get(&flag, u + 1));
  CBH_TRY(S.get(&cpos, u + 1));
  switch (dtype) {
    case CBH_F64: launch_tuple_reduce<double>(ctx, k1, i1, head, pos, nnz, m, vals, ir, ukey, vout); break;
    case CBH_I64: launch_tuple_reduce<int64_t>(ctx, k1, i1, head, pos, nnz, m, vals, ir, ukey, vout); break;
    case CBH_F32: launch_tuple_reduce<float>(ctx, k1, i1, head, pos, nnz, m, vals, ir, ukey, vout); break;
    case CBH_I32: launch_tuple_reduce<int32_t>(ctx, k1, i1, head, pos, nnz, m, vals, ir, ukey, vout); break;
    default: launch_tuple_reduce<uint8_t>(ctx, k1, i1, head, pos, nnz, m, vals, ir, ukey, vout); break;
  }
  CBH_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(col_heads_kernel, dim3(blocks_for(u, 256)), dim3(256), 0, ctx->stream, ukey, u, m, flag);
  CBH_HIP(ctx, hipMemsetAsync(flag + u, 0, sizeof(int64_t), ctx->stream));
  CBH_TRY(exclusive_scan_i64(ctx, S, flag, cpos, u + 1));
  int64_t nzc = 0;
  CBH_HIP(ctx, hipMemcpyAsync(&nzc, cpos + u, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  cbh_mat* M;
  CBH_TRY(new_mat(ctx, m, n, u, nzc, dtype, &M));
  hipLaunchKernelGGL(col_fill_kernel, dim3(blocks_for(u, 256)), dim3(256), 0, ctx->stream, ukey, flag, cpos, u, m, M->jc,
                     M->cp);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(M->cp + nzc, &u, sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(M->ir, ir, sizeof(int32_t) * u, hipMemcpyDeviceToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(M->num, vout, vs * u, hipMemcpyDeviceToDevice, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  int rc = e == hipSuccess ? check_err(ctx) : fail(ctx, CBH_E_HIP, std::string("tuples_to_dcsc: ") + hipGetErrorString(e));
  if (rc != CBH_OK) {
    cbh_mat_free(ctx, M);
    return rc;
  }
  *out = M;
  return CBH_OK;
}

// config C5's input (mclgen.h): planted partition, symmetric, unit loops, column-stochastic, f64
extern "C" int cbh_gen_planted_partition(cbh_ctx* ctx, int64_t n, int64_t avg_deg, uint64_t seed, double p_in,
                                         double alpha, cbh_mat** out) {
  if (!ctx || !out || n < 2 || n > INT32_MAX || avg_deg < 2 || !(alpha > 0) || !(p_in >= 0 && p_in <= 1))
    return fail(ctx, CBH_E_ARG, "bad planted-partition arguments");
  *out = nullptr;
  const int64_t half = avg_deg / 2, draws = n * half;
  if (draws > INT32_MAX) return fail(ctx, CBH_E_ARG, "n * avg_deg / 2 must stay below 2^31 draws");
  std::vector<int64_t> start{0};  // power-law cluster sizes 2 + floor(6 * Lomax(alpha)), summing to n
  for (uint64_t i = 0; start.back() < n; ++i) {
    const double lomax = std::pow(1.0 - gen_u01(seed, 0, i), -1.0 / alpha) - 1.0;
    const double sz = std::min((double)n, 2.0 + std::floor(6.0 * lomax));
    start.push_back(std::min<int64_t>(n, start.back() + (int64_t)sz));
  }
  const int64_t ncl = (int64_t)start.size() - 1;
  Scratch S(ctx);
  int64_t *dstart, *head, *pos;
  int32_t *cl, *perm, *pval;
  uint64_t *pkey, *pkey2, *key, *key2;
  CBH_TRY(S.get(&dstart, ncl + 1));
  CBH_TRY(S.get(&cl, n));
  CBH_TRY(S.get(&perm, n));
  CBH_TRY(S.get(&pval, n));
  CBH_TRY(S.get(&pkey, n));
  CBH_TRY(S.get(&pkey2, n));
  CBH_HIP(ctx, hipMemcpyAsync(dstart, start.data(), sizeof(int64_t) * (ncl + 1), hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(gen_cluster_of_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, dstart, ncl, n, cl);
  hipLaunchKernelGGL(gen_perm_keys_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, seed, n, pkey, pval);
  CBH_HIP(ctx, hipGetLastError());
  size_t tmp = 0;
  CBH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, pkey, pkey2, pval, perm, (int)n, 0, 64, ctx->stream));
  char* t;
  CBH_TRY(S.get(&t, tmp));
  CBH_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(t, tmp, pkey, pkey2, pval, perm, (int)n, 0, 64, ctx->stream));
  CBH_TRY(S.get(&key, draws));
  CBH_TRY(S.get(&key2, draws));
  hipLaunchKernelGGL(gen_edge_keys_kernel, dim3(blocks_for(draws, 256)), dim3(256), 0, ctx->stream, seed, (int64_t)0,
                     draws, half, n, p_in, cl, dstart, perm, key);
  CBH_HIP(ctx, hipGetLastError());
  tmp = 0;
  CBH_HIP(ctx, hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, key, key2, (int)draws, 0, 64, ctx->stream));
  char* t2;
  CBH_TRY(S.get(&t2, tmp));
  CBH_HIP(ctx, hipcub::DeviceRadixSort::SortKeys(t2, tmp, key, key2, (int)draws, 0, 64, ctx->stream));
  S.drop(t2);
  S.drop(key);
  CBH_TRY(S.get(&head, draws + 1));
  CBH_TRY(S.get(&pos, draws + 1));
  hipLaunchKernelGGL(gen_head_kernel, dim3(blocks_for(draws, 256)), dim3(256), 0, ctx->stream, key2, draws, head);
  CBH_HIP(ctx, hipMemsetAsync(head + draws, 0, sizeof(int64_t), ctx->stream));
  CBH_TRY(exclusive_scan_i64(ctx, S, head, pos, draws + 1));
  int64_t npairs = 0;
  CBH_HIP(ctx, hipMemcpyAsync(&npairs, pos + draws, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  const int64_t total = 2 * npairs + n;
  if (total > INT32_MAX) return fail(ctx, CBH_E_ARG, "planted partition above 2^31 entries");
  int32_t* rows;
  int64_t* cols;
  double* vals;
  CBH_TRY(S.get(&rows, total));
  CBH_TRY(S.get(&cols, total));
  CBH_TRY(S.get(&vals, total));
  hipLaunchKernelGGL(gen_tuples_kernel, dim3(blocks_for(std::max(draws, n), 256)), dim3(256), 0, ctx->stream, seed, key2,
                     head, pos, draws, npairs, n, rows, cols, vals);
  CBH_HIP(ctx, hipGetLastError());
  S.drop(key2);
  S.drop(head);
  S.drop(pos);
  cbh_mat* M = nullptr;
  CBH_TRY(cbh_tuples_to_dcsc(ctx, n, n, total, rows, cols, vals, CBH_F64, 0, &M));
  hipLaunchKernelGGL(gen_col_stochastic_kernel, dim3(blocks_for(M->nzc, 4)), dim3(256), 0, ctx->stream, M->cp, M->nzc,
                     reinterpret_cast<double*>(M->num));
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cbh_mat_free(ctx, M);
    return fail(ctx, CBH_E_HIP, std::string("gen_col_stochastic: ") + hipGetErrorString(e));
  }
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  *out = M;
  return CBH_OK;
}

extern "C" int cbh_dcsc_to_tuples(cbh_ctx* ctx, const cbh_mat* M, int32_t* rows, int64_t* cols, void* vals) {
  if (!ctx || !M || (M->nnz > 0 && (!rows || !cols || !vals))) return fail(ctx, CBH_E_ARG, "bad dcsc_to_tuples arguments");
  if (M->nnz == 0) return CBH_OK;
  CBH_HIP(ctx, hipMemcpyAsync(rows, M->ir, sizeof(int32_t) * M->nnz, hipMemcpyDeviceToDevice, ctx->stream));
  CBH_HIP(ctx, hipMemcpyAsync(vals, M->num, M->vbytes * M->nnz, hipMemcpyDeviceToDevice, ctx->stream));
  hipLaunchKernelGGL(expand_cols_kernel, dim3(blocks_for(M->nzc, 4)), dim3(256), 0, ctx->stream, M->jc, M->cp, M->nzc,
                     cols);
  CBH_HIP(ctx, hipGetLastError());
  CBH_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return CBH_OK;
}
