// gfx950 kernels of the SpGEMM hot path.
//
// One workgroup owns one output column j (one nonzero column of B, or one column of the
// merged result). The column's products are accumulated in LDS; columns whose output does not
// fit are cut into ROW TILES [lo,hi) processed one after another by the same workgroup (each B
// entry keeps a cursor into its row-sorted A column), so every product is visited once per pass
// and no global-memory atomics are ever needed (DESIGN.md §3.2 explains why global hashing is
// avoided on MI355X).
//
//   MODE_SYM      distinct rows per column in an LDS hash of keys  -> estimateNNZ_Hash (mtSpGEMM.h:806-933)
//   MODE_SYM_BMP  the same count from an LDS BITMAP over the tile's rows (heavy columns: no
//                 hashing, no overflow, 32*T rows per tile)
//   MODE_NUM      SR::add(SR::multiply(a,b)) per row in an order-preserving LDS hash, column
//                 written with rows ascending                       -> LocalHybridSpGEMM (mtSpGEMM.h:289-441)
//   *_MRG         entries are the k partial lists of the column    -> MultiwayMerge (MultiwayMerge.h:411-526)
//
// Load balance inside the workgroup: per tile, each entry i (one B nonzero -> one A column
// segment) contributes seg_i products; an LDS exclusive scan gives offsets, and products are
// processed in windows of WIN: an owner map (segment starts scattered, then a block max-scan)
// tells each product its entry with ONE LDS read; consecutive lanes take consecutive products
// (coalesced within a segment).
//
// Numeric tables use an ORDER-PRESERVING slot map (slot = (row-lo)*T/(hi-lo)) with forward linear
// probing that never wraps: keys end up globally sorted once each run of occupied slots is sorted
// (proof in DESIGN.md §3.3), replacing the per-column std::sort (mtSpGEMM.h:434). A tile whose
// probes exceed kPmax (clustered rows) or run off the table is retried with half the row range.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "semiring.h"

namespace cbh {

constexpr int32_t kEmpty = -1;
constexpr int kGuard = 64;  // numeric tables: extra slots past T (probing never wraps)
constexpr int kPmax = 64;   // probe limit before the tile is split in half

enum : int { MODE_SYM = 0, MODE_NUM = 1, MODE_SYM_MRG = 2, MODE_NUM_MRG = 3, MODE_SYM_BMP = 4, MODE_SYM_BMP_MRG = 6 };
constexpr int kMaxLists = 16;

struct TileArgs {
  // gather side (A), dense column pointers (A.n + 1 entries)
  const int64_t* Acp;
  const int32_t* Air;
  const void* Anum;
  // SpGEMM entries: B in DCSC (cp over B's nonzero columns)
  const int64_t* Bcp;
  const int32_t* Bir;
  const void* Bnum;
  // merge entries: per output column c and list l, segment [seg_start, seg_start+seg_len)
  const int64_t* seg_start;
  const int64_t* seg_len;
  const int32_t* lir[kMaxLists];
  const void* lnum[kMaxLists];
  int nlists;
  // schedule: column slots handled by this launch
  const int32_t* cols;
  int64_t ncols;
  const int64_t* work;  // per column slot: flops (symbolic) or nnz (numeric)
  const int32_t* rmin;  // per column slot: smallest / largest row any product can hit
  const int32_t* rmax;
  // outputs
  int32_t* gcur[2];  // chunked columns: per-B-entry cursors, double-buffered by tile parity
  int64_t* nnz_out;  // symbolic: per column slot
  const int64_t* Ccp;  // numeric: per column slot output offsets (exclusive scan of nnz)
  int64_t cbase;       // subtracted from Ccp (phase base)
  int32_t* Cir;
  void* Cnum;
  int* err;  // [0] numeric count mismatch, [1] split failure, [2] bounds guard, [3] guard site
  // sizes for the device-side bounds guards (a violated guard sets err[2] and skips the access)
  int64_t nnzA, ncolA, nnzB, ccap, nslots;
};

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

template <class SR, int T, int BS, int EMAX, int MODE>
struct TileCfg {
  static constexpr bool NUM = (MODE & 1) != 0;
  static constexpr bool MRG = (MODE & 2) != 0;
  static constexpr bool BMP = (MODE & 4) != 0;
  using val_t = typename SR::val_t;
  using acc_t = typename SR::acc_t;
  static constexpr int TA = NUM ? T + kGuard : T;  // table slots (bitmap: 32-bit words)
  static constexpr int NW = BS / 64;
  static constexpr int WIN = 4 * BS;  // products per owner-map window
  static constexpr size_t al(size_t x) { return (x + 15) & ~size_t(15); }
  static constexpr size_t o_keys = 0;
  static constexpr size_t o_vals = al(o_keys + sizeof(int32_t) * TA);
  static constexpr size_t o_base = al(o_vals + (NUM ? sizeof(acc_t) * TA : 0));
  static constexpr size_t o_scale = al(o_base + sizeof(int64_t) * EMAX);
  static constexpr size_t o_len = al(o_scale + ((NUM && !MRG) ? sizeof(val_t) * EMAX : 0));
  static constexpr size_t o_cur = al(o_len + sizeof(int32_t) * EMAX);
  static constexpr size_t o_stop = al(o_cur + sizeof(int32_t) * EMAX);
  static constexpr size_t o_off = al(o_stop + sizeof(int32_t) * EMAX);
  static constexpr size_t o_own = al(o_off + sizeof(int32_t) * (EMAX + 1));
  static constexpr size_t o_list = al(o_own + sizeof(int32_t) * WIN);
  static constexpr size_t o_red = al(o_list + (MRG ? EMAX : 0));
  static constexpr size_t bytes = al(o_red + sizeof(int32_t) * (NW + 4));
};

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
    int s = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      int y = __shfl_up(s, d);
      if (lane >= d) s += y;
    }
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
  int s = m;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(s, d);
    if (lane >= d) s = y > s ? y : s;
  }
  if (lane == 63) red[wid] = s;
  int ex = __shfl_up(s, 1);
  if (lane == 0) ex = -1;
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

template <class SR, int T, int BS, int EMAX, int MODE>
__global__ __launch_bounds__(BS) void tile_kernel(TileArgs a) {
  using C = TileCfg<SR, T, BS, EMAX, MODE>;
  using val_t = typename C::val_t;
  using acc_t = typename C::acc_t;
  constexpr bool NUM = C::NUM, MRG = C::MRG, BMP = C::BMP;
  constexpr int TA = C::TA, NW = C::NW, WIN = C::WIN;
  static_assert(BMP || (T & (T - 1)) == 0, "hash tables must be a power of two");
  static_assert(!(BMP && NUM), "bitmap mode is symbolic only");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int32_t* keys = reinterpret_cast<int32_t*>(smem + C::o_keys);
  uint32_t* words = reinterpret_cast<uint32_t*>(smem + C::o_keys);
  acc_t* vals = reinterpret_cast<acc_t*>(smem + C::o_vals);
  int64_t* ebase = reinterpret_cast<int64_t*>(smem + C::o_base);
  val_t* escale = reinterpret_cast<val_t*>(smem + C::o_scale);
  int32_t* elen = reinterpret_cast<int32_t*>(smem + C::o_len);
  int32_t* ecur = reinterpret_cast<int32_t*>(smem + C::o_cur);
  int32_t* estop = reinterpret_cast<int32_t*>(smem + C::o_stop);
  int32_t* eoff = reinterpret_cast<int32_t*>(smem + C::o_off);
  int32_t* own = reinterpret_cast<int32_t*>(smem + C::o_own);
  uint8_t* elist = reinterpret_cast<uint8_t*>(smem + C::o_list);
  int32_t* red = reinterpret_cast<int32_t*>(smem + C::o_red);  // NW wave slots + flags
  volatile int32_t* flag_ovf = red + NW;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t ci = blockIdx.x;
  if (ci >= a.ncols) return;
  const int c = a.cols[ci];
  if (c < 0 || c >= a.nslots) {
    if (threadIdx.x == 0) guard_fail(a.err, 6);
    return;
  }

  int64_t e0, ne;
  if constexpr (!MRG) {
    e0 = a.Bcp[c];
    ne = a.Bcp[c + 1] - e0;
  } else {
    e0 = (int64_t)c * a.nlists;
    ne = a.nlists;
  }
  const int64_t work = a.work[c];
  if (work <= 0) {
    if (!NUM && tid == 0) a.nnz_out[c] = 0;
    return;
  }
  const int64_t rlo = a.rmin[c], rhi = (int64_t)a.rmax[c] + 1;
  const int64_t span = rhi - rlo;
  int64_t R;
  if constexpr (BMP) {
    R = (span + 32ll * T - 1) / (32ll * T);
  } else {
    constexpr int64_t cap = T / 2;
    R = (work + cap - 1) / cap;
    if (R > span) R = span;
  }
  const int64_t wnom = (span + R - 1) / R;
  const bool chunked = ne > EMAX;
  const int nchunks = chunked ? (int)((ne + EMAX - 1) / EMAX) : 1;

  // Loads entries [first, first+cnt) of the column into LDS. Cursors persist across tiles: in LDS
  // when the column fits (ne <= EMAX), otherwise in HBM (gcur, double-buffered by the parity of
  // committed tiles so a retried tile re-reads the same starts).
  int tpar = 0;
  auto load_entries = [&](int64_t first, int cnt, int64_t lo) {
    for (int i = tid; i < cnt; i += BS) {
      int64_t base, len;
      int l = 0;
      if constexpr (!MRG) {
        const int64_t p = e0 + first + i;
        const int32_t k = a.Bir[p];
        if (k < 0 || k >= a.ncolA) {
          guard_fail(a.err, 1);
          base = 0;
          len = 0;
        } else {
          base = a.Acp[k];
          len = a.Acp[k + 1] - base;
          if (base < 0 || len < 0 || base + len > a.nnzA) {
            guard_fail(a.err, 2);
            base = 0;
            len = 0;
          }
        }
        if constexpr (NUM) escale[i] = reinterpret_cast<const val_t*>(a.Bnum)[p];
      } else {
        l = (int)(first + i);
        base = a.seg_start[e0 + l];
        len = a.seg_len[e0 + l];
        elist[i] = (uint8_t)l;
      }
      ebase[i] = base;
      elen[i] = (int32_t)len;
      int cur = 0;
      if (chunked && lo > rlo && len > 0) {
        if (!MRG && a.gcur[0]) {
          // L1-bypassing (sc1) load: another workgroup on this CU may have pulled this line into
          // the vector L1 before this column's previous tile stored it (MI355X_MICROARCH.md,
          // inter-workgroup visibility); L2 holds the value written by this workgroup.
          cur = __hip_atomic_load(&a.gcur[tpar][e0 + first + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          const int32_t* rows = MRG ? a.lir[l] + base : a.Air + base;
          cur = lower_bound_rows(rows, 0, (int)len, lo);
        }
      }
      if (cur < 0 || cur > len) {
        guard_fail(a.err, 3, MODE, c, first + i, cur, len, lo);
        cur = (int)len;
      }
      ecur[i] = cur;
    }
  };

  if (!chunked) {
    load_entries(0, (int)ne, rlo);
    __syncthreads();
  }

  int64_t out_pos = 0, out_end = 0;
  if constexpr (NUM) {
    out_pos = a.Ccp[c] - a.cbase;
    out_end = a.Ccp[c + 1] - a.cbase;
  }
  int64_t count_total = 0;

  int64_t lo = rlo;
  int64_t w = wnom;
  while (lo < rhi) {
    const int64_t hi = (lo + w < rhi) ? lo + w : rhi;
    const int64_t tw = hi - lo;
    const int nwords = BMP ? (int)((tw + 31) >> 5) : 0;
    // order-preserving slot map for numeric tables: slot = ((row-lo) * scale) >> 32 < T
    const uint64_t scale = ((uint64_t)T << 32) / (uint64_t)tw;
    if constexpr (BMP) {
      for (int s = tid; s < nwords; s += BS) words[s] = 0u;
    } else {
      for (int s = tid; s < TA; s += BS) {
        keys[s] = kEmpty;
        if constexpr (NUM) vals[s] = SR::identity();
      }
    }
    if (tid == 0) *flag_ovf = 0;
    __syncthreads();

    for (int ch = 0; ch < nchunks; ++ch) {
      int nec = (int)ne;
      if (chunked) {
        const int64_t first = (int64_t)ch * EMAX;
        nec = (int)((ne - first) < EMAX ? (ne - first) : EMAX);
        load_entries(first, nec, lo);
        __syncthreads();
      }
      // segment of each entry inside [lo, hi)
      const int64_t first = (int64_t)ch * EMAX;
      for (int i = tid; i < nec; i += BS) {
        const int cur = ecur[i], len = elen[i];
        int stop = len;
        if (hi < rhi && cur < len) {
          const int32_t* rows = MRG ? a.lir[elist[i]] + ebase[i] : a.Air + ebase[i];
          stop = gallop_rows(rows, cur, len, hi);
        }
        estop[i] = stop;
        eoff[i] = stop - cur;
        // plain store: the line stays in this XCD's L2 (an sc1 store would write through and drop
        // it, and a later sc1 load could then read memory before the write lands)
        if (!MRG && chunked && a.gcur[0]) a.gcur[tpar ^ 1][e0 + first + i] = stop;
      }
      // __syncthreads() waits only for LDS (lgkmcnt): make the cursor stores reach L2 before the
      // next tile's L1-bypassing loads of them.
      if (!MRG && chunked && a.gcur[0]) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      block_scan_excl<BS>(eoff, nec, red);
      const int P = eoff[nec];
      for (int w0 = 0; w0 < P; w0 += WIN) {
        const int wn = (P - w0) < WIN ? (P - w0) : WIN;
        // owner map of products [w0, w0+wn): starts of non-empty segments, then prefix-max
        const int ia = lower_bound_lds(eoff, nec, w0);
        const int ib = lower_bound_lds(eoff, nec, w0 + wn);
        for (int x = tid; x < WIN; x += BS) own[x] = (x == 0) ? ia - 1 : -1;
        __syncthreads();
        for (int i = ia + tid; i < ib; i += BS) {
          const int s0 = eoff[i];
          if (eoff[i + 1] > s0) own[s0 - w0] = i;
        }
        __syncthreads();
        block_max_scan<BS, WIN>(own, red);
        for (int x = tid; x < wn; x += BS) {
          if (!BMP && *flag_ovf) break;
          const int i = own[x];
          const int p = w0 + x;
          const int64_t q = ebase[i] + ecur[i] + (p - eoff[i]);
          if (i < 0 || i >= nec || q < 0 || (!MRG && q >= a.nnzA)) {
            guard_fail(a.err, 4, MODE * 1000 + (chunked ? 100 : 0) + ch, c, i, nec, p, (i >= 0 && i < nec) ? ecur[i] * 100000 + eoff[i] : -7);
            continue;
          }
          int32_t r;
          val_t v{};
          if constexpr (!MRG) {
            r = a.Air[q];
            if constexpr (NUM) v = SR::multiply(reinterpret_cast<const val_t*>(a.Anum)[q], escale[i]);
          } else {
            const int l = elist[i];
            r = a.lir[l][q];
            if constexpr (NUM) v = reinterpret_cast<const val_t*>(a.lnum[l])[q];
          }
          if constexpr (BMP) {
            const uint32_t d = (uint32_t)(r - lo);
            if ((int64_t)r < lo || (int64_t)r >= hi) {
              guard_fail(a.err, 7, c, i + 1000 * ch + (chunked ? 1000000 : 0), r, lo, hi, ecur[i] * 100000 + estop[i]);
              continue;
            }
            atomicOr(&words[d >> 5], 1u << (d & 31));
          } else if constexpr (NUM) {
            if ((int64_t)r < lo || (int64_t)r >= hi) {
              guard_fail(a.err, 8, c, i, r, lo, hi, ecur[i] * 100000 + estop[i]);
              continue;
            }
            bool ok = false;
            uint32_t s = (uint32_t)(((uint64_t)(r - lo) * scale) >> 32);
            for (int probe = 0; probe < kPmax && s < (uint32_t)TA; ++probe, ++s) {
              int32_t k = reinterpret_cast<volatile int32_t*>(keys)[s];
              if (k == kEmpty) k = atomicCAS(&keys[s], kEmpty, r);
              if (k == kEmpty || k == r) {
                SR::lds_acc(&vals[s], v);
                ok = true;
                break;
              }
            }
            if (!ok) *flag_ovf = 1;
          } else {
            constexpr int LG = __builtin_ctz(T);
            bool ok = false;
            uint32_t s = ((uint32_t)r * 0x9E3779B1u) >> (32 - LG);
            for (int probe = 0; probe < 2 * kPmax; ++probe, s = (s + 1) & (T - 1)) {
              int32_t k = reinterpret_cast<volatile int32_t*>(keys)[s];
              if (k == kEmpty) k = atomicCAS(&keys[s], kEmpty, r);
              if (k == kEmpty || k == r) {
                ok = true;
                break;
              }
            }
            if (!ok) *flag_ovf = 1;
          }
        }
        __syncthreads();
        if (!BMP && *flag_ovf) break;
      }
      if (!BMP && *flag_ovf) break;
    }
    if (!BMP && *flag_ovf) {  // table could not hold the tile: halve the row range and redo it
      __syncthreads();
      if (tw == 1) {  // cannot happen (one row always fits); fail loudly rather than loop
        if (tid == 0) atomicOr(&a.err[1], 1);
        return;
      }
      w = (tw + 1) / 2;
      continue;
    }
    // commit the tile
    if (!chunked)
      for (int i = tid; i < (int)ne; i += BS) ecur[i] = estop[i];
    else
      tpar ^= 1;
    if constexpr (BMP) {
      int cnt = 0;
      for (int s = tid; s < nwords; s += BS) cnt += __popc(words[s]);
      count_total += block_sum_int<NW>(cnt, red);
    } else if constexpr (!NUM) {
      int cnt = 0;
      for (int s = tid; s < TA; s += BS) cnt += (keys[s] != kEmpty);
      count_total += block_sum_int<NW>(cnt, red);
    } else {
      // sort each run of occupied slots (keys are globally ordered across runs)
      for (int s = tid; s < TA; s += BS) {
        if (keys[s] != kEmpty && (s == 0 || keys[s - 1] == kEmpty)) {
          int e = s + 1;
          while (e < TA && keys[e] != kEmpty) ++e;
          for (int x = s + 1; x < e; ++x) {
            const int32_t kx = keys[x];
            const acc_t vx = vals[x];
            int y = x - 1;
            while (y >= s && keys[y] > kx) {
              keys[y + 1] = keys[y];
              vals[y + 1] = vals[y];
              --y;
            }
            keys[y + 1] = kx;
            vals[y + 1] = vx;
          }
        }
      }
      __syncthreads();
      // compaction in slot order -> coalesced column write
      for (int base = 0; base < TA; base += BS) {
        const int s = base + tid;
        const bool occ = (s < TA) && keys[s] != kEmpty;
        const uint64_t mask = __ballot(occ);
        const int pre = __popcll(mask & ((1ull << lane) - 1ull));
        if (lane == 0) red[wid] = __popcll(mask);
        __syncthreads();
        int wpre = 0, tot = 0;
#pragma unroll
        for (int x = 0; x < NW; ++x) {
          const int rr = red[x];
          wpre += (x < wid) ? rr : 0;
          tot += rr;
        }
        if (occ) {
          const int64_t o = out_pos + wpre + pre;
          if (o >= a.ccap) guard_fail(a.err, 5);
          else if (o < out_end) {
            a.Cir[o] = keys[s];
            reinterpret_cast<val_t*>(a.Cnum)[o] = SR::finalize(vals[s]);
          }
        }
        out_pos += tot;
        __syncthreads();
      }
    }
    lo = hi;
    w = wnom;
    __syncthreads();
  }
  if constexpr (!NUM) {
    if (tid == 0) a.nnz_out[c] = count_total;
  } else {
    if (tid == 0 && out_pos != out_end) atomicAdd(&a.err[0], 1);
  }
}

}  // namespace cbh
