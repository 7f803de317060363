// gfx950 kernels of the SpGEMM hot path.
//
// One workgroup owns one output column j (one nonzero column of B, or one column of the
// merged result). The column's products are accumulated in an LDS hash table; columns whose
// output does not fit the table are cut into ROW TILES [lo,hi) processed one after another by
// the same workgroup, so every product is hashed exactly once and no global-memory atomics
// are ever needed (see DESIGN.md §3 for why global hashing is avoided on MI355X).
//
//   symbolic (MODE_SYM*) : counts distinct rows per column   -> estimateNNZ_Hash (mtSpGEMM.h:806-933)
//   numeric  (MODE_NUM*) : accumulates SR::add(SR::multiply(a,b)) and writes the column with
//                          rows ascending                      -> LocalHybridSpGEMM hash branch
//                                                                (mtSpGEMM.h:362-440) / heap branch
//   merge    (MODE_*MRG) : same kernel, entries are the k partial lists of a column
//                                                              -> MultiwayMerge (MultiwayMerge.h:411-526)
//
// Work per workgroup is load-balanced across threads by flattening the column's products:
// entry i (one B nonzero -> one A column segment) contributes seg_i products, an LDS exclusive
// scan of seg_i gives offsets, and thread t handles products t, t+BS, ... (consecutive lanes
// read consecutive A entries: coalesced within a segment).
//
// Numeric tables use an ORDER-PRESERVING hash (slot = (row-lo)*T/(hi-lo)) with forward linear
// probing and no wrap-around: keys then end up globally sorted once each run of occupied slots
// is sorted (proof in DESIGN.md §3.3), which replaces the reference's per-column std::sort
// (mtSpGEMM.h:434) by short in-place insertion sorts. A tile whose probes exceed kPmax (a
// clustered row distribution) is retried with half the row range.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "semiring.h"

namespace cbh {

constexpr int32_t kEmpty = -1;
constexpr int kGuard = 64;  // numeric tables: extra slots past T (probing never wraps)
constexpr int kPmax = 64;   // probe limit before the tile is split in half

enum : int { MODE_SYM = 0, MODE_NUM = 1, MODE_SYM_MRG = 2, MODE_NUM_MRG = 3 };
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
  int64_t* nnz_out;  // symbolic: per column slot
  const int64_t* Ccp;  // numeric: per column slot output offsets (exclusive scan of nnz)
  int64_t cbase;       // subtracted from Ccp (phase base)
  int32_t* Cir;
  void* Cnum;
  int* err;  // [0] numeric count mismatch, [1] column too large
};

template <class SR, int T, int BS, int EMAX, int MODE>
struct TileCfg {
  static constexpr bool NUM = (MODE & 1) != 0;
  static constexpr bool MRG = (MODE & 2) != 0;
  using val_t = typename SR::val_t;
  using acc_t = typename SR::acc_t;
  static constexpr int TA = NUM ? T + kGuard : T;
  static constexpr int NW = BS / 64;
  static constexpr size_t al(size_t x) { return (x + 15) & ~size_t(15); }
  static constexpr size_t o_keys = 0;
  static constexpr size_t o_vals = al(o_keys + sizeof(int32_t) * TA);
  static constexpr size_t o_base = al(o_vals + (NUM ? sizeof(acc_t) * TA : 0));
  static constexpr size_t o_scale = al(o_base + sizeof(int64_t) * EMAX);
  static constexpr size_t o_len = al(o_scale + ((NUM && !MRG) ? sizeof(val_t) * EMAX : 0));
  static constexpr size_t o_cur = al(o_len + sizeof(int32_t) * EMAX);
  static constexpr size_t o_stop = al(o_cur + sizeof(int32_t) * EMAX);
  static constexpr size_t o_off = al(o_stop + sizeof(int32_t) * EMAX);
  static constexpr size_t o_list = al(o_off + sizeof(int32_t) * (EMAX + 1));
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

// first q in [lo, hi) with p[q] >= key (p sorted ascending); global memory.
__device__ __forceinline__ int lower_bound_rows(const int32_t* __restrict__ p, int lo, int hi, int64_t key) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)p[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

template <class SR, int T, int BS, int EMAX, int MODE>
__global__ __launch_bounds__(BS) void tile_kernel(TileArgs a) {
  using C = TileCfg<SR, T, BS, EMAX, MODE>;
  using val_t = typename C::val_t;
  using acc_t = typename C::acc_t;
  constexpr bool NUM = C::NUM, MRG = C::MRG;
  constexpr int TA = C::TA, NW = C::NW;
  static_assert((T & (T - 1)) == 0, "T must be a power of two");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int32_t* keys = reinterpret_cast<int32_t*>(smem + C::o_keys);
  acc_t* vals = reinterpret_cast<acc_t*>(smem + C::o_vals);
  int64_t* ebase = reinterpret_cast<int64_t*>(smem + C::o_base);
  val_t* escale = reinterpret_cast<val_t*>(smem + C::o_scale);
  int32_t* elen = reinterpret_cast<int32_t*>(smem + C::o_len);
  int32_t* ecur = reinterpret_cast<int32_t*>(smem + C::o_cur);
  int32_t* estop = reinterpret_cast<int32_t*>(smem + C::o_stop);
  int32_t* eoff = reinterpret_cast<int32_t*>(smem + C::o_off);
  uint8_t* elist = reinterpret_cast<uint8_t*>(smem + C::o_list);
  int32_t* red = reinterpret_cast<int32_t*>(smem + C::o_red);  // NW wave slots + flags
  volatile int32_t* flag_ovf = red + NW;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t ci = blockIdx.x;
  if (ci >= a.ncols) return;
  const int c = a.cols[ci];

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
  constexpr int64_t cap = T / 2;
  int64_t R = (work + cap - 1) / cap;
  if (R > span) R = span;
  const int64_t wnom = (span + R - 1) / R;
  const bool chunked = ne > EMAX;
  const int nchunks = chunked ? (int)((ne + EMAX - 1) / EMAX) : 1;

  // Loads entries [first, first+cnt) of the column into LDS. In chunked mode the cursor is
  // re-derived for every tile by binary search; otherwise cursors persist across tiles.
  auto load_entries = [&](int64_t first, int cnt, int64_t lo) {
    for (int i = tid; i < cnt; i += BS) {
      int64_t base, len;
      int l = 0;
      if constexpr (!MRG) {
        const int64_t p = e0 + first + i;
        const int32_t k = a.Bir[p];
        base = a.Acp[k];
        len = a.Acp[k + 1] - base;
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
        const int32_t* rows = MRG ? a.lir[l] + base : a.Air + base;
        cur = lower_bound_rows(rows, 0, (int)len, lo);
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
    // order-preserving slot map for numeric tables: slot = ((row-lo) * scale) >> 32 < T
    const uint64_t scale = ((uint64_t)T << 32) / (uint64_t)tw;
    for (int s = tid; s < TA; s += BS) {
      keys[s] = kEmpty;
      if constexpr (NUM) vals[s] = SR::identity();
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
      for (int i = tid; i < nec; i += BS) {
        const int cur = ecur[i], len = elen[i];
        int stop = len;
        if (hi < rhi && cur < len) {
          const int32_t* rows = MRG ? a.lir[elist[i]] + ebase[i] : a.Air + ebase[i];
          stop = lower_bound_rows(rows, cur, len, hi);
        }
        estop[i] = stop;
        eoff[i] = stop - cur;
      }
      __syncthreads();
      block_scan_excl<BS>(eoff, nec, red);
      const int P = eoff[nec];
      for (int p = tid; p < P; p += BS) {
        if (*flag_ovf) break;
        // entry owning product p: last i with eoff[i] <= p
        int lo_i = 0, hi_i = nec;
        while (hi_i - lo_i > 1) {
          const int mid = (lo_i + hi_i) >> 1;
          if (eoff[mid] <= p) lo_i = mid;
          else hi_i = mid;
        }
        const int i = lo_i;
        const int64_t q = ebase[i] + ecur[i] + (p - eoff[i]);
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
        bool ok = false;
        if constexpr (NUM) {
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
        } else {
          constexpr int LG = __builtin_ctz(T);
          uint32_t s = ((uint32_t)r * 0x9E3779B1u) >> (32 - LG);
          for (int probe = 0; probe < 2 * kPmax; ++probe, s = (s + 1) & (T - 1)) {
            int32_t k = reinterpret_cast<volatile int32_t*>(keys)[s];
            if (k == kEmpty) k = atomicCAS(&keys[s], kEmpty, r);
            if (k == kEmpty || k == r) {
              ok = true;
              break;
            }
          }
        }
        if (!ok) *flag_ovf = 1;
      }
      __syncthreads();
      if (*flag_ovf) break;
    }
    if (*flag_ovf) {  // table could not hold the tile: halve the row range and redo it
      __syncthreads();
      w = (tw > 1) ? (tw + 1) / 2 : 1;
      if (tw == 1) {  // cannot happen (one row always fits); fail loudly rather than loop
        if (tid == 0) atomicOr(&a.err[1], 1);
        return;
      }
      continue;
    }
    // commit the tile
    if (!chunked)
      for (int i = tid; i < (int)ne; i += BS) ecur[i] = estop[i];
    if constexpr (!NUM) {
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
          if (o < out_end) {
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
