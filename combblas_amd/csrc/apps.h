// gfx950 kernels for the callers either side of the SpGEMM hot path:
//
//   masked_kernel        C = (A*B) .* M in one pass         [TC.cpp:108-110: Mult_AnXBn_Synch(L, L) then
//                                                             C.EWiseMult(L, false) = Friends.h:834-887]
//   ewise_kernel         C = A .* B (pattern intersection, values multiplied)   [Friends.h:834-887]
//   colstat_kernel       per-column count, count and sum of the entries above a threshold
//                                                           [SpParMat::Reduce(Column, ...), ParFriends.h:196-200]
//   kselect_hist/pick    k-th largest value per active column, radix select over order-preserving
//                        keys; histograms can be summed over a processor column between passes
//                                                           [SpParMat::Kselect1, SpParMat.cpp:1413-1700]
//   prune_col_kernel     keep entries !(v < thresh[col])    [Dcsc::PruneColumn, dcsc.cpp:699-760]
//   colstat_kept_kernel  count / sum of what PruneColumn(thresh) keeps, per column
//   kselect_wave/block   Kselect1 of whole local columns: a wave / a workgroup per column (keys in
//                        registers or streamed); kselect_long_* for the longest, chunked
//
// Included once by spgemm.hip (one translation unit).
#pragma once
#include "../../include/combblas_hip/device/task_kernel.h"

namespace cbh {

// ---------------------------------------------------------------------------- masked SpGEMM
// One workgroup per nonzero column slot c of B whose column also exists in M. The mask column's
// rows are staged in LDS in chunks of MCAP (sorted); the products whose rows fall in the chunk's
// row range are flattened over the workgroup (segment scan + binary search for the owner), each
// product's row is looked up in the staged rows by binary search and accumulated with SR::add
// (a zero-valued product still creates the entry, as explicit zeros do in the reference). Hits
// are written in mask order (rows ascending) at Mcp[ms] + rank into a temporary indexed like M;
// the per-column hit counts drive the final compaction. PATTERN: values are the semiring sums
// (the mask only selects); otherwise they are multiplied by M's values (EWiseMult).
struct MaskArgs {
  const int64_t* Acp;  // A dense column pointers (A.n + 1)
  const int32_t* Air;
  const void* Anum;
  const int64_t* Bcp;  // B DCSC (per slot)
  const int32_t* Bir;
  const void* Bnum;
  int64_t nzcB;
  const int64_t* mslot;  // per B slot: M's slot with the same column id, -1 if none
  const int64_t* Mcp;
  const int32_t* Mir;
  const void* Mnum;
  int32_t* Tir;  // temporary output, nnz(M) slots, indexed like M
  void* Tnum;
  int64_t* hits;  // per B slot
  int* err;
  int64_t nnzA, ncolA;
};

template <class SR, int MCAP, int BS, int EMAX, bool PATTERN>
__global__ __launch_bounds__(BS) void masked_kernel(MaskArgs a) {
  using val_t = typename SR::val_t;
  using acc_t = typename SR::acc_t;
  constexpr int NW = BS / 64;
  static_assert(EMAX >= BS, "the hit scan reuses eoff[0..BS]");
  __shared__ int32_t mrow[MCAP];
  __shared__ acc_t acc[MCAP];
  __shared__ int32_t hit[MCAP];
  __shared__ int64_t ebeg[EMAX];
  __shared__ int32_t eoff[EMAX + 1];
  __shared__ val_t escale[EMAX];
  __shared__ int red[2 * NW + 4];
  const int tid = threadIdx.x;
  const int64_t c = blockIdx.x;
  if (c >= a.nzcB) return;
  const int64_t ms = a.mslot[c];
  if (ms < 0) {
    if (tid == 0) a.hits[c] = 0;
    return;
  }
  const int64_t m0 = a.Mcp[ms], m1 = a.Mcp[ms + 1];
  const int64_t e0 = a.Bcp[c], ne = a.Bcp[c + 1] - e0;
  int64_t nhits = 0;
  for (int64_t x0 = m0; x0 < m1; x0 += MCAP) {
    const int cnt = (int)((m1 - x0) < MCAP ? (m1 - x0) : MCAP);
    for (int i = tid; i < cnt; i += BS) {
      mrow[i] = a.Mir[x0 + i];
      acc[i] = SR::identity();
      hit[i] = 0;
    }
    __syncthreads();
    const int32_t rlo = mrow[0], rhi = mrow[cnt - 1];
    for (int64_t f0 = 0; f0 < ne; f0 += EMAX) {
      const int nec = (int)((ne - f0) < EMAX ? (ne - f0) : EMAX);
      // segment of every entry inside [rlo, rhi]
      for (int i = tid; i < nec; i += BS) {
        const int64_t p = e0 + f0 + i;
        const int32_t k = a.Bir[p];
        int64_t s = 0, e = 0;
        if (k >= 0 && k < a.ncolA) {
          const int64_t base = a.Acp[k], end = a.Acp[k + 1];
          s = lb_rows64(a.Air, base, end, rlo);
          e = lb_rows64(a.Air, s, end, rhi + 1);  // row ids are < m < 2^31 - 1
        } else {
          guard_fail(a.err, 20, c, k);
        }
        ebeg[i] = s;
        eoff[i] = (int32_t)(e - s);
        escale[i] = reinterpret_cast<const val_t*>(a.Bnum)[p];
      }
      __syncthreads();
      block_scan_excl<BS>(eoff, nec, red);
      const int P = eoff[nec];
      for (int x = tid; x < P; x += BS) {
        // owner: the last entry whose segment starts at or before x (LDS binary search)
        int lo = 0, hi = nec - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (eoff[mid] <= x) lo = mid;
          else hi = mid - 1;
        }
        const int64_t q = ebeg[lo] + (x - eoff[lo]);
        const int32_t r = a.Air[q];
        const val_t av = reinterpret_cast<const val_t*>(a.Anum)[q];
        int l2 = 0, h2 = cnt;  // mask lookup
        while (l2 < h2) {
          const int mid = (l2 + h2) >> 1;
          if (mrow[mid] < r) l2 = mid + 1;
          else h2 = mid;
        }
        if (l2 < cnt && mrow[l2] == r) {
          SR::lds_acc(&acc[l2], SR::multiply(av, escale[lo]));
          hit[l2] = 1;
        }
      }
      __syncthreads();
    }
    // hits of this chunk in mask order
    int carry = 0;
    for (int base = 0; base < cnt; base += BS) {
      const int i = base + tid;
      const int h = (i < cnt) ? hit[i] : 0;
      eoff[tid] = h;
      __syncthreads();
      block_scan_excl<BS>(eoff, BS, red);
      if (h) {
        const int64_t pos = m0 + nhits + carry + eoff[tid];
        a.Tir[pos] = mrow[i];
        val_t v = SR::finalize(acc[i]);
        if constexpr (!PATTERN) v = (val_t)(v * reinterpret_cast<const val_t*>(a.Mnum)[x0 + i]);  // Friends.h:871
        reinterpret_cast<val_t*>(a.Tnum)[pos] = v;
      }
      carry += eoff[BS];
      __syncthreads();
    }
    nhits += carry;
    __syncthreads();
  }
  if (tid == 0) a.hits[c] = nhits;
}

// ---------------------------------------------------------------------------- masked SpGEMM, dot form
// C = (A*B) .* M evaluated per MASK ENTRY (i, j): the sorted k-lists of row i of A (column i of
// AT = A') and of column j of B are intersected, SR::add of SR::multiply(A(i,k), B(k,j)) over the
// common k in ascending order; the entry exists iff the intersection is not empty (explicit zeros
// count, as in the expanding form). Work is sum over mask entries of the shorter list (x a search
// in the longer one), instead of the full flops of A*B: TC's (L*L) .* L at R-MAT scale 24
// enumerates ~10^12 products of the symmetric pattern, the dot form a few 10^10 probes.
// Mask entries are classified by the shorter list: short (thread per entry, galloping merge),
// long (pieces of kDotPiece elements, one wave per piece, partials reduced in piece order).
constexpr int kDotThread = 64;   // shorter list <= this: one thread per entry
constexpr int kDotPiece = 2048;  // long entries: elements of the shorter list per wave piece
constexpr int kDotMergeRatio = 8;  // long entries: merge when longer <= 8 x shorter, else binary search

struct DotArgs {
  const int64_t* ATd;  // AT dense column pointers (A.m + 1): row i of A = AT(:, i), rows = k
  const int32_t* ATir;
  const void* ATnum;
  const int64_t* Bd;  // B dense column pointers (B.n + 1)
  const int32_t* Bir;
  const void* Bnum;
  const int64_t* Mcol;  // per mask entry: its column id
  const int32_t* Mir;
  int64_t nnzM, mA, nB;
  void* Tnum;      // per mask entry: the sum (where Tflag)
  uint8_t* Tflag;  // per mask entry: intersection not empty
  int* err;
};

// first q in [lo, hi) with rows[q] >= key by galloping from lo
__device__ __forceinline__ int64_t dot_gallop(const int32_t* __restrict__ rows, int64_t lo, int64_t hi, int32_t key) {
  if (lo >= hi || rows[lo] >= key) return lo;
  return gallop64(rows, lo + 1, hi, key);
}

template <class V>
__device__ __forceinline__ V shfl_down_val(V v, int d) {
  if constexpr (sizeof(V) == 8) {
    return __builtin_bit_cast(V, (unsigned long long)__shfl_down(__builtin_bit_cast(unsigned long long, v), d));
  } else if constexpr (sizeof(V) == 4) {
    return __builtin_bit_cast(V, (unsigned)__shfl_down(__builtin_bit_cast(unsigned, v), d));
  } else {
    static_assert(sizeof(V) == 1, "value width");
    return (V)__shfl_down((int)v, d);
  }
}

// the two lists of mask entry p; returns false (and counts a guard) on out-of-range ids
__device__ __forceinline__ bool dot_lists(const DotArgs& a, int64_t p, int64_t& a0, int64_t& a1, int64_t& b0,
                                          int64_t& b1) {
  const int64_t i = a.Mir[p], j = a.Mcol[p];
  if (i < 0 || i >= a.mA || j < 0 || j >= a.nB) return false;
  a0 = a.ATd[i];
  a1 = a.ATd[i + 1];
  b0 = a.Bd[j];
  b1 = a.Bd[j + 1];
  return true;
}

// class of every mask entry: 0 = empty intersection for sure (a list is empty: flag 0 written
// here), 1 = thread, 2 = long (pieces), 3 = hub candidate (hub_min > 0 and the longer list at most
// hub_wave x the shorter -- a wave-mode group, key + nB + mA -- or more than hub_ratio x the
// shorter -- a thread-mode group, key: counted into its group, gcount[key]). Waves append their
// entries to the class lists with one atomic per class; npiece[x] = pieces of long entry x.
__global__ __launch_bounds__(256) void dot_classify_kernel(DotArgs a, int32_t* __restrict__ lthr,
                                                           int32_t* __restrict__ llong, int64_t* __restrict__ npiece,
                                                           unsigned long long* __restrict__ counts, int hub_min,
                                                           int hub_ratio, int hub_wave, int32_t* __restrict__ gcount,
                                                           int32_t* __restrict__ lcand) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int cls = -1;
  int64_t ls = 0;
  if (p < a.nnzM) {
    int64_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
    if (!dot_lists(a, p, a0, a1, b0, b1)) atomicOr(&a.err[2], 1);
    const bool a_short = (a1 - a0) <= (b1 - b0);
    ls = a_short ? (a1 - a0) : (b1 - b0);
    const int64_t ll = a_short ? (b1 - b0) : (a1 - a0);
    cls = ls <= 0 ? 0 : (ls <= kDotThread ? 1 : 2);
    if (cls == 0) a.Tflag[p] = 0;
    if (cls == 2 && hub_min > 0) {
      const bool wave = hub_wave > 0 && ll <= (int64_t)hub_wave * ls;
      if (wave || ll > hub_ratio * ls) {
        cls = 3;
        const int64_t key = a_short ? (int64_t)a.Mcol[p] : a.nB + (int64_t)a.Mir[p];
        atomicAdd(&gcount[key + (wave ? a.nB + a.mA : 0)], 1);
      }
    }
  }
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint64_t m1 = __ballot(cls == 1), m2 = __ballot(cls == 2), m3 = __ballot(cls == 3);
  unsigned long long base1 = 0, base2 = 0, base3 = 0;
  if (lane == 0) {
    if (m1) base1 = atomicAdd(&counts[0], (unsigned long long)__popcll(m1));
    if (m2) base2 = atomicAdd(&counts[1], (unsigned long long)__popcll(m2));
    if (m3) base3 = atomicAdd(&counts[2], (unsigned long long)__popcll(m3));
  }
  base1 = __shfl(base1, 0);
  base2 = __shfl(base2, 0);
  base3 = __shfl(base3, 0);
  if (cls == 1) lthr[base1 + __popcll(m1 & lt)] = (int32_t)p;
  if (cls == 2) {
    const int64_t x = (int64_t)base2 + __popcll(m2 & lt);
    llong[x] = (int32_t)p;
    npiece[x] = (ls + kDotPiece - 1) / kDotPiece;
  }
  if (cls == 3) lcand[base3 + __popcll(m3 & lt)] = (int32_t)p;
}

// thread per short entry: the shorter list drives, the longer one is galloped through
template <class SR>
__global__ __launch_bounds__(256) void dot_thread_kernel(DotArgs a, const int32_t* __restrict__ list, int64_t n) {
  using val_t = typename SR::val_t;
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n) return;
  const int64_t p = list[x];
  int64_t a0, a1, b0, b1;
  if (!dot_lists(a, p, a0, a1, b0, b1)) return;
  const val_t* __restrict__ av = reinterpret_cast<const val_t*>(a.ATnum);
  const val_t* __restrict__ bv = reinterpret_cast<const val_t*>(a.Bnum);
  val_t acc{};
  bool hit = false;
  if (a1 - a0 <= b1 - b0) {
    int64_t q = b0;
    for (int64_t s = a0; s < a1 && q < b1; ++s) {
      const int32_t k = a.ATir[s];
      q = dot_gallop(a.Bir, q, b1, k);
      if (q < b1 && a.Bir[q] == k) {
        const val_t pr = SR::multiply(av[s], bv[q]);
        acc = hit ? SR::add(acc, pr) : pr;
        hit = true;
      }
    }
  } else {
    int64_t q = a0;
    for (int64_t s = b0; s < b1 && q < a1; ++s) {
      const int32_t k = a.Bir[s];
      q = dot_gallop(a.ATir, q, a1, k);
      if (q < a1 && a.ATir[q] == k) {
        const val_t pr = SR::multiply(av[q], bv[s]);
        acc = hit ? SR::add(acc, pr) : pr;
        hit = true;
      }
    }
  }
  a.Tflag[p] = hit ? 1 : 0;
  if (hit) reinterpret_cast<val_t*>(a.Tnum)[p] = acc;
}

// piece -> (long entry, piece number): item y of long entry x for y in [poff[x], poff[x+1])
__global__ __launch_bounds__(256) void dot_items_kernel(const int64_t* __restrict__ poff, int64_t nlong,
                                                        int32_t* __restrict__ item_entry) {
  const int lane = threadIdx.x & 63;
  // wave-strided: a grid's work-item count is 32-bit (AQL dispatch), so the grid is capped
  for (int64_t x = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); x < nlong; x += (int64_t)gridDim.x * 4)
    for (int64_t y = poff[x] + lane; y < poff[x + 1]; y += 64) item_entry[y] = (int32_t)x;
}

// piece y of a long entry (one wave): a merge of the two lists when their lengths are within
// kDotMergeRatio, else lanes take 64 consecutive elements of the shorter list at a time and
// binary-search them in the longer one (bounded below by the previous batch's last position); the
// lane partials are folded in lane order into the piece's partial
template <class SR>
__device__ __forceinline__ void dot_piece(const DotArgs& a, const int32_t* __restrict__ llong,
                                          const int64_t* __restrict__ poff, const int32_t* __restrict__ item_entry,
                                          int64_t y, void* __restrict__ pval, uint8_t* __restrict__ phit, int lane) {
  using val_t = typename SR::val_t;
  const int32_t x = item_entry[y];
  const int64_t p = llong[x];
  int64_t a0, a1, b0, b1;
  if (!dot_lists(a, p, a0, a1, b0, b1)) {
    if (lane == 0) phit[y] = 0;
    return;
  }
  const val_t* __restrict__ av = reinterpret_cast<const val_t*>(a.ATnum);
  const val_t* __restrict__ bv = reinterpret_cast<const val_t*>(a.Bnum);
  const bool a_short = a1 - a0 <= b1 - b0;
  const int32_t* __restrict__ srow = a_short ? a.ATir : a.Bir;
  const int32_t* __restrict__ lrow = a_short ? a.Bir : a.ATir;
  const int64_t s0 = (a_short ? a0 : b0) + (y - poff[x]) * (int64_t)kDotPiece;
  const int64_t s1e = a_short ? a1 : b1;
  const int64_t s1 = s0 + kDotPiece < s1e ? s0 + kDotPiece : s1e;
  int64_t lo = a_short ? b0 : a0;
  const int64_t hi = a_short ? b1 : a1;
  val_t acc{};
  bool hit = false;
  if ((hi - lo) <= kDotMergeRatio * (s1e - (a_short ? a0 : b0))) {
    // comparable lengths: merge. The wave walks this piece of the shorter list and the longer
    // list in chunks of 64 (coalesced loads); every undecided element not above the longer
    // chunk's last value is looked up among its 64 values by a shuffle binary search; the
    // shorter chunk advances once all its elements are decided, else the longer one does.
    // (Measured at scale 24: 8.1 s; loading 3 chunks ahead 8.8 s; staging 1024-element blocks
    // in LDS with lockstep LDS searches 11.3 s.)
    int64_t lp = lb_rows64(lrow, lo, hi, srow[s0]);
    int64_t sp = s0;
    int32_t sv = sp + lane < s1 ? srow[sp + lane] : kNoRow;
    bool und = sp + lane < s1;
    while (sp < s1 && lp < hi) {
      const int32_t lv = lp + lane < hi ? lrow[lp + lane] : kNoRow;
      const int32_t lmax = __shfl(lv, 63);
      int pos = 0;
#pragma unroll
      for (int st = 32; st >= 1; st >>= 1)
        if (__shfl(lv, pos + st - 1) < sv) pos += st;
      const int32_t at = __shfl(lv, pos & 63);
      if (und && sv <= lmax) {
        und = false;
        if (pos < 64 && at == sv) {
          const int64_t s = sp + lane, q = lp + pos;
          const val_t pr = a_short ? SR::multiply(av[s], bv[q]) : SR::multiply(av[q], bv[s]);
          acc = hit ? SR::add(acc, pr) : pr;
          hit = true;
        }
      }
      if (__ballot(und) == 0ull) {
        sp += 64;
        und = sp + lane < s1;
        sv = und ? srow[sp + lane] : kNoRow;
      } else {
        lp += 64;
      }
    }
  } else {
    // much longer other list: every element binary-searches it (an interpolation start measured
    // slower: 9.7 vs 8.1 s at scale 24 -- the bisection's first levels are shared L2 hits). Round 5
    // measured this branch at 3.5 of the 8.1 s (a build without the search: 4.6 s) and two ways to
    // shorten it, both slower: an 8-ary search with 7 splitter loads per level (15.3 s: its deep
    // levels fetch 7 distinct lines each) and the top levels from an LDS sample of the longer
    // list, 1024 rows per wave (8.24 vs 8.14 s: the shared top levels were never the cost)
    for (int64_t base = s0; base < s1 && lo < hi; base += 64) {
      const int64_t s = base + lane;
      int64_t q = hi;
      if (s < s1) {
        const int32_t k = srow[s];
        q = lb_rows64(lrow, lo, hi, k);
        if (q < hi && lrow[q] == k) {
          const val_t pr = a_short ? SR::multiply(av[s], bv[q]) : SR::multiply(av[q], bv[s]);
          acc = hit ? SR::add(acc, pr) : pr;
          hit = true;
        }
      }
      // the next batch's keys are larger than every key of this one
      const int last = (s1 - base) < 64 ? (int)(s1 - base) - 1 : 63;
      lo = __shfl(q, last);
    }
  }
  // fold lanes in order: lane l absorbs lane l + d (higher lanes hold larger k)
  for (int d = 1; d < 64; d <<= 1) {
    const val_t o = shfl_down_val(acc, d);
    const int oh = __shfl_down((int)hit, d);
    if ((lane & (2 * d - 1)) == 0 && lane + d < 64 && oh) {
      acc = hit ? SR::add(acc, o) : o;
      hit = true;
    }
  }
  if (lane == 0) {
    phit[y] = hit ? 1 : 0;
    if (hit) reinterpret_cast<val_t*>(pval)[y] = acc;
  }
}

template <class SR>
__global__ __launch_bounds__(256) void dot_wave_kernel(DotArgs a, const int32_t* __restrict__ llong,
                                                       const int64_t* __restrict__ poff,
                                                       const int32_t* __restrict__ item_entry, int64_t nitems,
                                                       void* __restrict__ pval, uint8_t* __restrict__ phit) {
  const int lane = threadIdx.x & 63;
  // wave-strided over the pieces (the grid is capped: a dispatch counts work-items in 32 bits)
  for (int64_t y = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); y < nitems; y += (int64_t)gridDim.x * 4)
    dot_piece<SR>(a, llong, poff, item_entry, y, pval, phit, lane);
}

// long entry x: its pieces folded in order
template <class SR>
__global__ __launch_bounds__(256) void dot_fold_kernel(DotArgs a, const int32_t* __restrict__ llong,
                                                       const int64_t* __restrict__ poff, int64_t nlong,
                                                       const void* __restrict__ pval, const uint8_t* __restrict__ phit) {
  using val_t = typename SR::val_t;
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= nlong) return;
  val_t acc{};
  bool hit = false;
  for (int64_t y = poff[x]; y < poff[x + 1]; ++y)
    if (phit[y]) {
      const val_t v = reinterpret_cast<const val_t*>(pval)[y];
      acc = hit ? SR::add(acc, v) : v;
      hit = true;
    }
  const int64_t p = llong[x];
  a.Tflag[p] = hit ? 1 : 0;
  if (hit) reinterpret_cast<val_t*>(a.Tnum)[p] = acc;
}

// ---- hub groups (round 6): the entries whose longer list is more than kDotMergeRatio x the
// shorter (dot_piece's binary-search branch) share their longer list with many other entries when
// it is a hub's: the mask column j of a long B(:, j) holds |M(:, j)| entries that all intersect it,
// and the mask row i of a long A(i, :) as many. Such entries are grouped by their longer list (key
// j, or nB + i) when at least hub_min of them share it. A workgroup takes a chunk of up to kHubECh
// entries of one group (kHubEPT per thread, their cursors, partials and hit flags in registers)
// and walks the group's longer list in windows of kHubWin rows: each window is staged in LDS with a
// bucket directory over its row range, and every thread advances each of its entries' shorter-list
// cursor through the window's row range, looking every element up in LDS (one directory read and
// ~1-2 row reads) instead of binary-searching the longer list in HBM. Products fold in ascending k
// (windows in order, elements in order inside a window).
constexpr int kHubWin = 8192;   // longer-list rows per window (LDS: 32 KB rows + 16 KB directory)
constexpr int kHubBS = 512;     // threads per hub workgroup
constexpr int kHubEPT = 8;      // entries per thread
constexpr int kHubECh = kHubBS * kHubEPT;  // entries per work item
constexpr int kHubBatch = 8;    // shorter-list elements a thread loads at once
constexpr int kHubEPW = 8;      // wave mode: entries per wave
constexpr int kHubWCh = (kHubBS / 64) * kHubEPW;  // wave mode: entries per work item

// group key of a hub candidate: j (B(:, j) longer) or nB + i (A(i, :) longer), + nB + mA in wave mode
__device__ __forceinline__ int64_t dot_hub_key(const DotArgs& a, int64_t p, int hub_wave, bool& ok) {
  int64_t a0, a1, b0, b1;
  ok = dot_lists(a, p, a0, a1, b0, b1);
  if (!ok) return 0;
  const bool a_short = (a1 - a0) <= (b1 - b0);
  const int64_t ls = a_short ? (a1 - a0) : (b1 - b0), ll = a_short ? (b1 - b0) : (a1 - a0);
  const bool wave = hub_wave > 0 && ll <= (int64_t)hub_wave * ls;
  return (a_short ? (int64_t)a.Mcol[p] : a.nB + (int64_t)a.Mir[p]) + (wave ? a.nB + a.mA : 0);
}
// the longer list of group key (either mode): B(:, j) for j < nB, else A(i, :) = AT(:, i)
__device__ __forceinline__ void dot_hub_list(const DotArgs& a, int64_t key, int64_t& l0, int64_t& l1,
                                             const int32_t*& lrow) {
  if (key >= a.nB + a.mA) key -= a.nB + a.mA;
  if (key < a.nB) {
    l0 = a.Bd[key];
    l1 = a.Bd[key + 1];
    lrow = a.Bir;
  } else {
    l0 = a.ATd[key - a.nB];
    l1 = a.ATd[key - a.nB + 1];
    lrow = a.ATir;
  }
}

// per group key (K thread-mode keys, then K wave-mode keys): entries (glen: count when >= hub_min,
// else 0) and work items (entry chunks of the mode)
__global__ __launch_bounds__(256) void dot_hub_sizes_kernel(const int32_t* __restrict__ gcount, int64_t K, int hub_min,
                                                            int hub_wmin, int64_t* __restrict__ glen,
                                                            int64_t* __restrict__ gitems) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= 2 * K) return;
  const int64_t c = gcount[k] >= (k < K ? hub_min : hub_wmin) ? gcount[k] : 0;
  const int64_t ch = k < K ? kHubECh : kHubWCh;
  glen[k] = c;
  gitems[k] = (c + ch - 1) / ch;
}

// hub candidates: into their group (goff + a per-group cursor) when the group has >= hub_min
// entries, else back to the long list (pieces of the wave kernel)
__global__ __launch_bounds__(256) void dot_hub_route_kernel(DotArgs a, const int32_t* __restrict__ lcand, int64_t n,
                                                            const int32_t* __restrict__ gcount, int hub_min, int hub_wmin,
                                                            int hub_wave,
                                                            const int64_t* __restrict__ goff, int32_t* __restrict__ gcur,
                                                            int32_t* __restrict__ hs, int32_t* __restrict__ llong,
                                                            int64_t* __restrict__ npiece,
                                                            unsigned long long* __restrict__ counts) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  bool back = false;
  int64_t p = 0, ls = 0;
  if (x < n) {
    p = lcand[x];
    bool ok;
    const int64_t key = dot_hub_key(a, p, hub_wave, ok);
    if (ok && gcount[key] >= (key < a.nB + a.mA ? hub_min : hub_wmin)) {
      hs[goff[key] + atomicAdd(&gcur[key], 1)] = (int32_t)p;
    } else {
      int64_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
      dot_lists(a, p, a0, a1, b0, b1);
      ls = (a1 - a0) < (b1 - b0) ? (a1 - a0) : (b1 - b0);
      back = true;
    }
  }
  const uint64_t m = __ballot(back);
  unsigned long long base = 0;
  if (lane == 0 && m) base = atomicAdd(&counts[1], (unsigned long long)__popcll(m));
  base = __shfl(base, 0);
  if (back) {
    const int64_t y = (int64_t)base + __popcll(m & ((1ull << lane) - 1ull));
    llong[y] = (int32_t)p;
    npiece[y] = (ls + kDotPiece - 1) / kDotPiece;
  }
}

// one workgroup per (group, entry chunk), grid-strided over the work items
#ifndef CBH_HUB_MINB  // (A/B hook) workgroups per CU the hub kernels' register budget is sized for
#define CBH_HUB_MINB 1
#endif
template <class SR>
__global__ __launch_bounds__(kHubBS, CBH_HUB_MINB) void dot_hub_kernel(DotArgs a, const int64_t* __restrict__ ioff, int64_t K,
                                                         int64_t nitems, const int64_t* __restrict__ goff,
                                                         const int32_t* __restrict__ hs) {
  using val_t = typename SR::val_t;
  __shared__ int32_t s_rows[kHubWin + 1];  // + a sentinel above every row
  __shared__ uint16_t s_dir[kHubWin + 1];
  const val_t* __restrict__ av = reinterpret_cast<const val_t*>(a.ATnum);
  const val_t* __restrict__ bv = reinterpret_cast<const val_t*>(a.Bnum);
  for (int64_t it = blockIdx.x; it < nitems; it += gridDim.x) {
    // the group: last key with ioff[key] <= it (keys without items have ioff[key] == ioff[key + 1])
    int64_t lo = 0, hi = K;
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (ioff[mid] <= it) lo = mid;
      else hi = mid;
    }
    const int64_t key = lo;
    int64_t l0, l1;
    const int32_t* lrow;
    dot_hub_list(a, key, l0, l1, lrow);
    const bool b_long = key < a.nB;  // the shorter lists are A(i, :) = AT(:, i), else B(:, j)
    const int32_t* __restrict__ srow = b_long ? a.ATir : a.Bir;
    const int64_t* __restrict__ sd = b_long ? a.ATd : a.Bd;
    const int64_t g0 = goff[key], ge = goff[key + 1] - g0;
    const int64_t ebase = (it - ioff[key]) * kHubECh;
    int64_t cur[kHubEPT], send[kHubEPT];
    val_t acc[kHubEPT];
    bool hit[kHubEPT];
    const int32_t first = lrow[l0];
    // each level of loads issued for all entries before the next (see the wave mode)
    int64_t pe[kHubEPT], sid[kHubEPT];
#pragma unroll
    for (int j = 0; j < kHubEPT; ++j) {
      const int64_t e = ebase + j * kHubBS + threadIdx.x;
      pe[j] = e < ge ? (int64_t)hs[g0 + e] : -1;
      acc[j] = val_t{};
      hit[j] = false;
    }
#pragma unroll
    for (int j = 0; j < kHubEPT; ++j) sid[j] = pe[j] < 0 ? 0 : (b_long ? (int64_t)a.Mir[pe[j]] : (int64_t)a.Mcol[pe[j]]);
#pragma unroll
    for (int j = 0; j < kHubEPT; ++j) {
      cur[j] = pe[j] < 0 ? 0 : sd[sid[j]];
      send[j] = pe[j] < 0 ? 0 : sd[sid[j] + 1];
    }
    // (thread mode: the shorter list is much shorter than the longer one; a bisection to the first
    // window's first row saves the walk over the elements below it)
#pragma unroll
    for (int j = 0; j < kHubEPT; ++j)
      if (pe[j] >= 0) cur[j] = lb_rows64(srow, cur[j], send[j], first);
    for (int64_t w0 = l0; w0 < l1; w0 += kHubWin) {
      const int n = (int)((l1 - w0) < kHubWin ? (l1 - w0) : kHubWin);
      __syncthreads();  // the previous window's readers are done with the LDS
      for (int t = threadIdx.x; t < n; t += kHubBS) s_rows[t] = lrow[w0 + t];
      if (threadIdx.x == 0) s_rows[n] = INT32_MAX;
      __syncthreads();
      const int32_t r_lo = s_rows[0], r_hi = s_rows[n - 1];
      const int64_t span = (int64_t)r_hi - r_lo + 1;
      // buckets over [r_lo, r_hi]: bucket(k) ~ (k - r_lo) * n / span (monotone in k); s_dir[b] =
      // first row index whose bucket >= b (b in [0, n]): element t fills (bucket(t - 1), bucket(t)]
      // ~(k - r_lo) * n / span by a 0.32 reciprocal and one __umulhi (span >= n as the rows are
      // distinct, so the scale is at most 2^32, clamped to 2^32 - 1: monotone, below n)
      const uint64_t bs64 = ((uint64_t)n << 32) / (uint64_t)span;
      const uint32_t bscale = bs64 > 0xffffffffull ? 0xffffffffu : (uint32_t)bs64;
      auto bucket = [&](int32_t k) -> int { return (int)__umulhi((uint32_t)(k - r_lo), bscale); };
      for (int t = threadIdx.x; t <= n; t += kHubBS) {
        const int bt = t < n ? bucket(s_rows[t]) : n;
        const int bp = t > 0 ? bucket(s_rows[t - 1]) : -1;
        for (int b = bp + 1; b <= bt; ++b) s_dir[b] = (uint16_t)t;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kHubEPT; ++j) {
        int64_t s = cur[j];
        bool more = s < send[j];
        while (more) {
          // kHubBatch elements per step, loaded together (independent loads, mostly one line)
          int32_t kk[kHubBatch];
#pragma unroll
          for (int u = 0; u < kHubBatch; ++u) kk[u] = s + u < send[j] ? srow[s + u] : INT32_MAX;
          int used = kHubBatch;
#pragma unroll
          for (int u = 0; u < kHubBatch; ++u) {
            const int32_t k = kk[u];
            if (used < kHubBatch) continue;
            if (k > r_hi) {  // past the window (or the list: INT32_MAX)
              used = u;
              continue;
            }
            if (k < r_lo) continue;  // (between the previous window's last row and this one's first)
            // the first row >= k from the bucket's first row on (the sentinel ends the walk)
            int q = s_dir[bucket(k)];
            int32_t r = s_rows[q];
            while (r < k) r = s_rows[++q];
            if (r == k) {
              const int64_t qg = w0 + q, sq = s + u;
              const val_t pr = b_long ? SR::multiply(av[sq], bv[qg]) : SR::multiply(av[qg], bv[sq]);
              acc[j] = hit[j] ? SR::add(acc[j], pr) : pr;
              hit[j] = true;
            }
          }
          s += used;
          more = used == kHubBatch && s < send[j];
        }
        cur[j] = s < send[j] ? s : send[j];
      }
    }
#pragma unroll
    for (int j = 0; j < kHubEPT; ++j) {
      const int64_t e = ebase + j * kHubBS + threadIdx.x;
      if (e < ge) {
        const int64_t p = hs[g0 + e];
        a.Tflag[p] = hit[j] ? 1 : 0;
        if (hit[j]) reinterpret_cast<val_t*>(a.Tnum)[p] = acc[j];
      }
    }
  }
}

// wave mode (the entries whose longer list is at most hub_wave x the shorter): one wave per entry,
// kHubEPW entries per wave, the lanes taking 64 consecutive shorter-list elements per step
// (coalesced) and looking them up in the staged window; the elements inside a window are a prefix
// of the rest of the (sorted) list, so a step advances the cursor by the ballot's count. Lane
// partials are folded in lane order at the end (as dot_piece's).
template <class SR>
__global__ __launch_bounds__(kHubBS, CBH_HUB_MINB) void dot_hub_wave_kernel(DotArgs a, const int64_t* __restrict__ ioff, int64_t K,
                                                              int64_t it0, int64_t it1, const int64_t* __restrict__ goff,
                                                              const int32_t* __restrict__ hs) {
  using val_t = typename SR::val_t;
  __shared__ int32_t s_rows[kHubWin + 1];  // + a sentinel above every row
  __shared__ uint16_t s_dir[kHubWin + 1];
  const val_t* __restrict__ av = reinterpret_cast<const val_t*>(a.ATnum);
  const val_t* __restrict__ bv = reinterpret_cast<const val_t*>(a.Bnum);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t it = it0 + blockIdx.x; it < it1; it += gridDim.x) {
    int64_t lo = K, hi = 2 * K;  // the group: last wave-mode key with ioff[key] <= it
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (ioff[mid] <= it) lo = mid;
      else hi = mid;
    }
    const int64_t gkey = lo;
    int64_t l0, l1;
    const int32_t* lrow;
    dot_hub_list(a, gkey, l0, l1, lrow);
    const bool b_long = gkey - K < a.nB;  // the shorter lists are A(i, :) = AT(:, i), else B(:, j)
    const int32_t* __restrict__ srow = b_long ? a.ATir : a.Bir;
    const int64_t* __restrict__ sd = b_long ? a.ATd : a.Bd;
    const int64_t g0 = goff[gkey], ge = goff[gkey + 1] - g0;
    const int64_t ebase = (it - ioff[gkey]) * kHubWCh;
    int64_t cur[kHubEPW], send[kHubEPW];
    val_t acc[kHubEPW];
    bool hit[kHubEPW];
    // the entries' shorter lists, each level of loads issued for all entries before the next; the
    // cursors start at the lists' heads (elements below the first window are skipped by the walk)
    int64_t pe[kHubEPW], sid[kHubEPW];
#pragma unroll
    for (int j = 0; j < kHubEPW; ++j) {
      const int64_t e = ebase + j * (kHubBS / 64) + wid;
      pe[j] = e < ge ? (int64_t)hs[g0 + e] : -1;  // (wave-uniform)
      acc[j] = val_t{};
      hit[j] = false;
    }
#pragma unroll
    for (int j = 0; j < kHubEPW; ++j) sid[j] = pe[j] < 0 ? 0 : (b_long ? (int64_t)a.Mir[pe[j]] : (int64_t)a.Mcol[pe[j]]);
#pragma unroll
    for (int j = 0; j < kHubEPW; ++j) {
      cur[j] = pe[j] < 0 ? 0 : sd[sid[j]];
      send[j] = pe[j] < 0 ? 0 : sd[sid[j] + 1];
    }
    for (int64_t w0 = l0; w0 < l1; w0 += kHubWin) {
      const int n = (int)((l1 - w0) < kHubWin ? (l1 - w0) : kHubWin);
      __syncthreads();
      for (int t = threadIdx.x; t < n; t += kHubBS) s_rows[t] = lrow[w0 + t];
      if (threadIdx.x == 0) s_rows[n] = INT32_MAX;
      __syncthreads();
      const int32_t r_lo = s_rows[0], r_hi = s_rows[n - 1];
      const int64_t span = (int64_t)r_hi - r_lo + 1;
      // ~(k - r_lo) * n / span by a 0.32 reciprocal and one __umulhi (span >= n as the rows are
      // distinct, so the scale is at most 2^32, clamped to 2^32 - 1: monotone, below n)
      const uint64_t bs64 = ((uint64_t)n << 32) / (uint64_t)span;
      const uint32_t bscale = bs64 > 0xffffffffull ? 0xffffffffu : (uint32_t)bs64;
      auto bucket = [&](int32_t k) -> int { return (int)__umulhi((uint32_t)(k - r_lo), bscale); };
      for (int t = threadIdx.x; t <= n; t += kHubBS) {
        const int bt = t < n ? bucket(s_rows[t]) : n;
        const int bp = t > 0 ? bucket(s_rows[t - 1]) : -1;
        for (int b = bp + 1; b <= bt; ++b) s_dir[b] = (uint16_t)t;
      }
      __syncthreads();
      // the first step of entry 0, then of every next entry, loads while the previous one is walked
      int32_t knext = cur[0] + lane < send[0] ? srow[cur[0] + lane] : INT32_MAX;
#pragma unroll
      for (int j = 0; j < kHubEPW; ++j) {
        int64_t s = cur[j];
        // one step ahead: the next 64 elements load while this step looks its elements up
        int32_t kn = knext;
        if (j + 1 < kHubEPW) knext = cur[j + 1] + lane < send[j + 1] ? srow[cur[j + 1] + lane] : INT32_MAX;
        while (s < send[j]) {
          const int64_t q = s + lane;
          const int32_t k = kn;
          const bool in = k <= r_hi;
          const int nin = __popcll(__ballot(in));
          kn = nin == 64 && q + 64 < send[j] ? srow[q + 64] : INT32_MAX;
          if (in && k >= r_lo) {
            // the first row >= k from the bucket's first row on (the sentinel ends the walk)
            int x = s_dir[bucket(k)];
            int32_t r = s_rows[x];
            while (r < k) r = s_rows[++x];
            if (r == k) {
              const int64_t qg = w0 + x;
              const val_t pr = b_long ? SR::multiply(av[q], bv[qg]) : SR::multiply(av[qg], bv[q]);
              acc[j] = hit[j] ? SR::add(acc[j], pr) : pr;
              hit[j] = true;
            }
          }
          s += nin;
          if (nin < 64) break;
        }
        cur[j] = s;
      }
    }
#pragma unroll
    for (int j = 0; j < kHubEPW; ++j) {
      val_t v = acc[j];
      bool h = hit[j];
      for (int d = 1; d < 64; d <<= 1) {  // lane l absorbs lane l + d: lanes in order
        const val_t o = shfl_down_val(v, d);
        const int oh = __shfl_down((int)h, d);
        if ((lane & (2 * d - 1)) == 0 && lane + d < 64 && oh) {
          v = h ? SR::add(v, o) : o;
          h = true;
        }
      }
      const int64_t e = ebase + j * (kHubBS / 64) + wid;
      if (lane == 0 && e < ge) {
        const int64_t p = hs[g0 + e];
        a.Tflag[p] = h ? 1 : 0;
        if (h) reinterpret_cast<val_t*>(a.Tnum)[p] = v;
      }
    }
  }
}

// hits per mask column (wave per slot) and, with WRITE, the compaction of the hit entries in
// mask order: C(ir, num) at off[slot] + rank, num = sum * M's value (EWiseMult, Friends.h:871)
// unless PATTERN
template <class V, bool WRITE, bool PATTERN>
__global__ __launch_bounds__(256) void dot_collect_kernel(const int64_t* __restrict__ Mcp, const int32_t* __restrict__ Mir,
                                                          const V* __restrict__ Mnum, int64_t nzcM,
                                                          const uint8_t* __restrict__ Tflag, const V* __restrict__ Tnum,
                                                          int64_t* __restrict__ hits, const int64_t* __restrict__ off,
                                                          int32_t* __restrict__ Cir, V* __restrict__ Cnum) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nzcM) return;
  const uint64_t lt = (1ull << lane) - 1ull;
  int64_t o = WRITE ? off[s] : 0;
  for (int64_t base = Mcp[s]; base < Mcp[s + 1]; base += 64) {
    const int64_t p = base + lane;
    const bool h = p < Mcp[s + 1] && Tflag[p];
    const uint64_t m = __ballot(h);
    if (WRITE && h) {
      const int64_t d = o + __popcll(m & lt);
      Cir[d] = Mir[p];
      V v = Tnum[p];
      if constexpr (!PATTERN) v = (V)(v * Mnum[p]);
      Cnum[d] = v;
    }
    o += __popcll(m);
  }
  if (!WRITE && lane == 0) hits[s] = o;
}

// A's entries as the tuples of A' (wave per column slot): row = A's column id, col = A's row id
__global__ __launch_bounds__(256) void transpose_tuples_kernel(const int64_t* __restrict__ jc,
                                                               const int64_t* __restrict__ cp, int64_t nzc,
                                                               const int32_t* __restrict__ ir, int32_t* __restrict__ trow,
                                                               int64_t* __restrict__ tcol) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nzc) return;
  const int32_t j = (int32_t)jc[c];
  for (int64_t p = cp[c] + lane; p < cp[c + 1]; p += 64) {
    trow[p] = j;
    tcol[p] = ir[p];
  }
}

// per slot of X: Y's slot holding the same column id (both jc arrays ascending), -1 if none
__global__ void match_slots_kernel(const int64_t* __restrict__ Xjc, int64_t nzcX, const int64_t* __restrict__ Yjc,
                                   int64_t nzcY, int64_t* __restrict__ yslot) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nzcX) return;
  const int64_t col = Xjc[i];
  int64_t lo = 0, hi = nzcY;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (Yjc[mid] < col) lo = mid + 1;
    else hi = mid;
  }
  yslot[i] = (lo < nzcY && Yjc[lo] == col) ? lo : -1;
}

// compaction of a temporary whose column c starts at src_cp[sslot[c]]: wave per column copies
// its hits[c] entries to off[c]
template <class V>
__global__ __launch_bounds__(256) void gather_cols_kernel(const int64_t* __restrict__ sslot,
                                                          const int64_t* __restrict__ src_cp,
                                                          const int64_t* __restrict__ hits,
                                                          const int64_t* __restrict__ off, int64_t ncols,
                                                          const int32_t* __restrict__ Tir, const V* __restrict__ Tnum,
                                                          int32_t* __restrict__ Cir, V* __restrict__ Cnum) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= ncols) return;
  const int64_t h = hits[c];
  if (h <= 0) return;
  const int64_t src = src_cp[sslot[c]], dst = off[c];
  for (int64_t i = lane; i < h; i += 64) {
    Cir[dst + i] = Tir[src + i];
    Cnum[dst + i] = Tnum[src + i];
  }
}

// C = A .* B (Friends.h:834-887, exclude = false): wave per A slot; each A entry looks its row up
// in B's column (binary search), matches are compacted by ballot in A's row order. Pass 1
// counts (hits per A slot), pass 2 writes at off[slot].
template <class V, bool WRITE>
__global__ __launch_bounds__(256) void ewise_kernel(const int64_t* __restrict__ Acp, const int32_t* __restrict__ Air,
                                                    const V* __restrict__ Anum, int64_t nzcA,
                                                    const int64_t* __restrict__ bslot, const int64_t* __restrict__ Bcp,
                                                    const int32_t* __restrict__ Bir, const V* __restrict__ Bnum,
                                                    int64_t* __restrict__ hits, const int64_t* __restrict__ off,
                                                    int32_t* __restrict__ Cir, V* __restrict__ Cnum) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nzcA) return;
  const int64_t bs = bslot[s];
  int64_t o = WRITE ? off[s] : 0;
  if (bs >= 0) {
    const int64_t b0 = Bcp[bs], b1 = Bcp[bs + 1];
    const int64_t p0 = Acp[s], p1 = Acp[s + 1];
    for (int64_t base = p0; base < p1; base += 64) {
      const int64_t p = base + lane;
      bool hit = false;
      int64_t q = 0;
      if (p < p1) {
        const int32_t r = Air[p];
        q = lb_rows64(Bir, b0, b1, r);
        hit = q < b1 && Bir[q] == r;
      }
      const uint64_t m = __ballot(hit);
      if (WRITE && hit) {
        const int64_t d = o + __popcll(m & ((1ull << lane) - 1ull));
        Cir[d] = Air[p];
        Cnum[d] = (V)(Anum[p] * Bnum[q]);
      }
      o += __popcll(m);
    }
  }
  if (!WRITE && lane == 0) hits[s] = o;
}

// ---------------------------------------------------------------------------- MCL column ops
// Wave per nonzero column slot; outputs dense over the n local columns (index jc[slot]), zero
// where a column has no slot:
//   cnt[col]  = nnz of the column                 (A.Reduce(Column, plus, 0, v->1))
//   cntp[col] = entries with v > hard             (nnz of A.Prune(v <= hard))
//   sump[col] = sum of those entries              (PrunedA.Reduce(Column, plus, 0))
__global__ __launch_bounds__(256) void colstat_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp,
                                                      const double* __restrict__ num, int64_t nzc, double hard,
                                                      double* __restrict__ cnt, double* __restrict__ cntp,
                                                      double* __restrict__ sump) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nzc) return;
  const int64_t p0 = cp[s], p1 = cp[s + 1];
  double n1 = 0, s1 = 0;
  for (int64_t p = p0 + lane; p < p1; p += 64) {
    const double v = num[p];
    if (v > hard) {
      n1 += 1.0;
      s1 += v;
    }
  }
  // the reference sums a column serially; counts are exact, this reduction tree's sum can differ
  // from the serial one in the last bits
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    n1 += __shfl_xor(n1, o);
    s1 += __shfl_xor(s1, o);
  }
  if (lane == 0) {
    const int64_t col = jc[s];
    cnt[col] = (double)(p1 - p0);
    cntp[col] = n1;
    sump[col] = s1;
  }
}

// colstat_kept_kernel: per column, count and sum of the entries that PruneColumn(thresh) keeps
// (!(v < thresh[col])) -- the statistics of the pruned matrix without forming it
__global__ __launch_bounds__(256) void colstat_kept_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp,
                                                           const double* __restrict__ num, int64_t nzc,
                                                           const double* __restrict__ thresh, double* __restrict__ cntk,
                                                           double* __restrict__ sumk) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nzc) return;
  const int64_t col = jc[s];
  const double t = thresh[col];
  const int64_t p0 = cp[s], p1 = cp[s + 1];
  double n1 = 0, s1 = 0;
  for (int64_t p = p0 + lane; p < p1; p += 64) {
    const double v = num[p];
    if (!(v < t)) {
      n1 += 1.0;
      s1 += v;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    n1 += __shfl_xor(n1, o);
    s1 += __shfl_xor(s1, o);
  }
  if (lane == 0) {
    cntk[col] = n1;
    sumk[col] = s1;
  }
}

// order-preserving map of a double onto uint64 (larger value -> larger key)
__device__ __forceinline__ uint64_t fkey(double v) {
  uint64_t b;
  __builtin_memcpy(&b, &v, 8);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double fval(uint64_t k) {
  const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  double v;
  __builtin_memcpy(&v, &b, 8);
  return v;
}

// One radix-select pass (8 bits at `shift`) for the active columns: hist[a*256 + d] = number of
// the column's keys that match prefix[a] above the digit and have digit d. Workgroup per slot.
__global__ __launch_bounds__(256) void kselect_hist_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp,
                                                           const double* __restrict__ num, int64_t nzc,
                                                           const int32_t* __restrict__ aidx,
                                                           const uint64_t* __restrict__ prefix, int shift,
                                                           uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const int64_t s = blockIdx.x;
  if (s >= nzc) return;
  const int32_t ai = aidx[jc[s]];
  if (ai < 0) return;
  const int tid = threadIdx.x;
  h[tid] = 0;
  __syncthreads();
  const uint64_t pre = prefix[ai];
  const uint64_t himask = shift >= 56 ? 0ull : (~0ull << (shift + 8));
  for (int64_t p = cp[s] + tid; p < cp[s + 1]; p += 256) {
    const uint64_t key = fkey(num[p]);
    if ((key & himask) == pre) atomicAdd(&h[(key >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(int64_t)ai * 256 + tid] = h[tid];
}

// Thread per active column: the digit holding descending rank[a] (largest digits first); rank
// becomes the rank inside that digit. rank < 0 marks an empty column (left alone).
__global__ void kselect_pick_kernel(int64_t nact, const uint32_t* __restrict__ hist, uint64_t* __restrict__ prefix,
                                    int64_t* __restrict__ rank, int shift) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= nact) return;
  int64_t r = rank[a];
  if (r < 0) return;
  const uint32_t* H = hist + a * 256;
  int b = 255;
  for (; b > 0; --b) {
    if (r < (int64_t)H[b]) break;
    r -= H[b];
  }
  prefix[a] |= (uint64_t)b << shift;
  rank[a] = r;
}

__global__ void kselect_value_kernel(int64_t nact, const uint64_t* __restrict__ prefix, double* __restrict__ out) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a < nact) out[a] = fval(prefix[a]);
}

// Kselect1 of whole local columns (the k-th largest value of every active column, the smallest
// when the column has fewer than k entries): a radix select over order-preserving keys, one
// launch per column-length class -- a wave per column up to 64*R entries and a workgroup per
// column up to 256*RB entries, the keys in registers; a workgroup per longer column that streams
// the keys and moves the candidates left after the first digit into LDS; kselect_long_* for the
// longest. The 8-bit digits start at the highest bit in which the column's keys differ (a
// min/max reduction first: the sign and most exponent bits of MCL's probabilities are common to
// a column, and a digit over them put every key on one bin); bins are per wave; the digit holding
// descending rank r is found by one wave (lane l owns bins 255-4l .. 252-4l, a shuffle prefix
// and a ballot); a bin holding a single key ends the select.

__device__ __forceinline__ void sel_minmax_shfl(uint64_t& lo, uint64_t& hi) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
}
// the digit pick, in every lane of one wave: c[j] = count of bin 255-4*lane-j
struct SelPick {
  int d;
  int64_t r;
  int one;
};
__device__ __forceinline__ SelPick sel_pick(const uint32_t (&c)[4], int64_t r) {
  const int lane = threadIdx.x & 63;
  uint32_t sum = c[0] + c[1] + c[2] + c[3];
  uint32_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  const uint64_t m = __ballot((int64_t)incl > r);
  const int L = __ffsll((long long)m) - 1;
  int64_t rr = r - (int64_t)(incl - sum);
  int d = 255 - 4 * lane, one = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (rr < (int64_t)c[j]) {
      d = 255 - 4 * lane - j;
      one = c[j] == 1u;
      break;
    }
    rr -= c[j];
  }
  return {__shfl(d, L), __shfl(rr, L), __shfl(one, L)};
}
// the first digit's position from the keys' min and max: top = highest differing bit, pre = the
// common bits above it (lo == hi: every key equal, pre = that key and top = -1)
__device__ __forceinline__ void sel_start(uint64_t lo, uint64_t hi, int& top, uint64_t& pre) {
  if (lo == hi) {
    top = -1;
    pre = lo;
    return;
  }
  top = 63 - __clzll((long long)(lo ^ hi));
  pre = top >= 63 ? 0ull : (lo & (~0ull << (top + 1)));
}

// One WAVE per column of at most 64*R entries, the keys held in registers (R per lane, all loads
// of a column in flight at once), the 256 bins in a per-wave LDS slice.
template <int R>
__global__ __launch_bounds__(256) void kselect_wave_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp,
                                                           const double* __restrict__ num, int64_t nzc,
                                                           const int32_t* __restrict__ aidx, int64_t k,
                                                           double* __restrict__ out) {
  __shared__ uint32_t hist[4][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t* h = hist[w];
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t s = (int64_t)blockIdx.x * 4 + w; s < nzc; s += nwaves) {
    const int32_t ai = aidx[jc[s]];
    const int64_t p0 = cp[s], n = cp[s + 1] - p0;
    if (ai < 0 || n <= 0 || n > 64 * R) continue;  // uniform over the wave
    uint64_t key[R];
    uint64_t lo = ~0ull, hi = 0ull;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int64_t i = (int64_t)j * 64 + lane;
      key[j] = i < n ? fkey(num[p0 + i]) : 0ull;
    }
#pragma unroll
    for (int j = 0; j < R; ++j)
      if ((int64_t)j * 64 + lane < n) {
        lo = key[j] < lo ? key[j] : lo;
        hi = key[j] > hi ? key[j] : hi;
      }
    sel_minmax_shfl(lo, hi);
    int64_t r = (n >= k ? k : n) - 1;
    int top;
    uint64_t pre;
    sel_start(lo, hi, top, pre);
    while (top >= 0) {
      const int shift = top >= 7 ? top - 7 : 0;
      const uint64_t himask = top >= 63 ? 0ull : (~0ull << (top + 1));
      const uint32_t dmask = (uint32_t)((2u << (top - shift)) - 1u);
#pragma unroll
      for (int j = 0; j < 4; ++j) h[lane * 4 + j] = 0u;
      wave_lds_sync();
#pragma unroll
      for (int j = 0; j < R; ++j)
        if ((int64_t)j * 64 + lane < n && (key[j] & himask) == pre) atomicAdd(&h[(uint32_t)(key[j] >> shift) & dmask], 1u);
      wave_lds_sync();
      uint32_t c[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) c[j] = h[255 - 4 * lane - j];
      const SelPick pk = sel_pick(c, r);
      wave_lds_sync();  // every lane has read its bins before the next digit clears them
      pre |= (uint64_t)pk.d << shift;
      r = pk.r;
      top = shift - 1;
      if (pk.one && top >= 0) {  // one key left under the prefix: it is the answer
        const uint64_t m2 = ~0ull << shift;
        uint64_t found = 0;
        bool has = false;
#pragma unroll
        for (int j = 0; j < R; ++j)
          if ((int64_t)j * 64 + lane < n && (key[j] & m2) == pre) {
            found = key[j];
            has = true;
          }
        pre = __shfl(found, __ffsll((long long)__ballot(has)) - 1);
        break;
      }
    }
    if (lane == 0) out[ai] = fval(pre);
  }
}

// One WORKGROUP of 256 threads per column of min_n < n <= max_n entries.
// REG (max_n <= 256*R): the keys in registers. Otherwise the keys are streamed (HBM / L2): the
// min/max and the first digit's histogram take one read each, then the candidates under the first
// digit move into LDS (one more read) when at most kSelCand of them are left -- the usual case --
// and the remaining digits run on them; a larger remainder keeps streaming.
constexpr int kSelCand = 4096;
template <int R, bool REG>
__global__ __launch_bounds__(256) void kselect_block_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp,
                                                            const double* __restrict__ num, int64_t nzc,
                                                            const int32_t* __restrict__ aidx, int64_t k,
                                                            double* __restrict__ out, int64_t min_n, int64_t max_n) {
  constexpr int RK = REG ? R : 1;
  __shared__ uint64_t cand[REG ? 1 : kSelCand];
  __shared__ uint32_t h[4][256];
  __shared__ uint64_t s_mm[2][4];
  __shared__ uint64_t s_key;
  __shared__ int s_d, s_one;
  __shared__ uint32_t s_nc;
  __shared__ int64_t s_r;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int64_t s = blockIdx.x; s < nzc; s += gridDim.x) {
    const int32_t ai = aidx[jc[s]];
    const int64_t p0 = cp[s], n = cp[s + 1] - p0;
    if (ai < 0 || n <= min_n || n > max_n) continue;  // uniform over the workgroup
    uint64_t key[RK];
    int64_t nk = n;       // keys in the current source
    int src = REG ? 0 : 1;  // 0 registers, 1 HBM stream, 2 LDS candidates
    if (REG) {
#pragma unroll
      for (int j = 0; j < RK; ++j) {
        const int64_t i = (int64_t)j * 256 + tid;
        key[j] = i < n ? fkey(num[p0 + i]) : 0ull;
      }
    }
    // f(key) over this thread's valid keys of the current source
    auto each = [&](auto&& f) {
      if (src == 0) {
#pragma unroll
        for (int j = 0; j < RK; ++j)
          if ((int64_t)j * 256 + tid < nk) f(key[j]);
      } else if (src == 1) {
        for (int64_t i = tid; i < nk; i += 256) f(fkey(num[p0 + i]));
      } else {
        for (int64_t i = tid; i < nk; i += 256) f(cand[i]);
      }
    };
    uint64_t lo = ~0ull, hi = 0ull;
    each([&](uint64_t x) {
      lo = x < lo ? x : lo;
      hi = x > hi ? x : hi;
    });
    sel_minmax_shfl(lo, hi);
    if (lane == 0) {
      s_mm[0][w] = lo;
      s_mm[1][w] = hi;
    }
    __syncthreads();
    lo = s_mm[0][0];
    hi = s_mm[1][0];
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      lo = s_mm[0][j] < lo ? s_mm[0][j] : lo;
      hi = s_mm[1][j] > hi ? s_mm[1][j] : hi;
    }
    int64_t r = (n >= k ? k : n) - 1;
    int top;
    uint64_t pre;
    sel_start(lo, hi, top, pre);
    while (top >= 0) {
      const int shift = top >= 7 ? top - 7 : 0;
      const uint64_t himask = top >= 63 ? 0ull : (~0ull << (top + 1));
      const uint32_t dmask = (uint32_t)((2u << (top - shift)) - 1u);
      h[0][tid] = h[1][tid] = h[2][tid] = h[3][tid] = 0u;
      __syncthreads();
      each([&](uint64_t x) {
        if ((x & himask) == pre) atomicAdd(&h[w][(uint32_t)(x >> shift) & dmask], 1u);
      });
      __syncthreads();
      if (tid < 64) {
        uint32_t c[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int b = 255 - 4 * lane - j;
          c[j] = h[0][b] + h[1][b] + h[2][b] + h[3][b];
        }
        const SelPick pk = sel_pick(c, r);
        if (lane == 0) {
          s_d = pk.d;
          s_r = pk.r;
          s_one = pk.one;
        }
        // the chosen bin's count, for the move into LDS
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (255 - 4 * lane - j == pk.d) s_nc = c[j];
      }
      __syncthreads();
      pre |= (uint64_t)s_d << shift;
      r = s_r;
      top = shift - 1;
      const uint64_t m2 = ~0ull << shift;
      if (s_one && top >= 0) {  // one key left under the prefix: it is the answer
        each([&](uint64_t x) {
          if ((x & m2) == pre) s_key = x;
        });
        __syncthreads();
        pre = s_key;
        break;
      }
      if (!REG && src == 1 && top >= 0 && s_nc <= (uint32_t)kSelCand) {  // candidates -> LDS
        const uint32_t nc = s_nc;
        __syncthreads();  // s_nc read by every thread before it is reused as the fill counter
        if (tid == 0) s_nc = 0;
        __syncthreads();
        each([&](uint64_t x) {
          if ((x & m2) == pre) cand[atomicAdd(&s_nc, 1u)] = x;
        });
        __syncthreads();
        src = 2;
        nk = nc;
      }
    }
    if (tid == 0) out[ai] = fval(pre);
    __syncthreads();
  }
}

// The longest columns (a near-dense column of an MCL iterate can hold millions of entries, which
// one workgroup would stream alone for every round): every such column is cut into chunks of
// kSelChunk entries, each radix pass runs
// over all chunks of all long columns at once (LDS histogram per chunk, added to the column's
// global 256 bins), and kselect_pick_kernel picks the digit per column between passes.
constexpr int kSelChunk = 8192;
__global__ void kselect_long_flag_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp, int64_t nzc,
                                         const int32_t* __restrict__ aidx, int64_t min_n, int64_t* __restrict__ flag) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > nzc) return;
  flag[s] = (s < nzc && aidx[jc[s]] >= 0 && cp[s + 1] - cp[s] > min_n) ? 1 : 0;
}
// list[l] = slot of long column l; nch[l] = its chunk count; rank / prefix initialised
__global__ void kselect_long_list_kernel(const int64_t* __restrict__ cp, int64_t nzc, const int64_t* __restrict__ flag,
                                         const int64_t* __restrict__ pos, int64_t k, int64_t* __restrict__ list,
                                         int64_t* __restrict__ nch, int64_t* __restrict__ rank,
                                         uint64_t* __restrict__ prefix) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nzc || !flag[s]) return;
  const int64_t l = pos[s], n = cp[s + 1] - cp[s];
  list[l] = s;
  nch[l] = (n + kSelChunk - 1) / kSelChunk;
  rank[l] = (n >= k ? k : n) - 1;
  prefix[l] = 0;
}
__global__ void kselect_long_map_kernel(int64_t nl, const int64_t* __restrict__ nch, const int64_t* __restrict__ cpos,
                                        int32_t* __restrict__ map) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nl) return;
  for (int64_t c = 0; c < nch[l]; ++c) map[cpos[l] + c] = (int32_t)l;
}
__global__ __launch_bounds__(256) void kselect_long_hist_kernel(const int64_t* __restrict__ cp,
                                                                const double* __restrict__ num,
                                                                const int64_t* __restrict__ list,
                                                                const int64_t* __restrict__ cpos,
                                                                const int32_t* __restrict__ map, int64_t nchunks,
                                                                const uint64_t* __restrict__ prefix, int shift,
                                                                uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const int tid = threadIdx.x;
  const uint64_t himask = shift >= 56 ? 0ull : (~0ull << (shift + 8));
  for (int64_t g = blockIdx.x; g < nchunks; g += gridDim.x) {
    const int32_t l = map[g];
    const int64_t s = list[l], c = g - cpos[l];
    const int64_t p1 = cp[s + 1], b0 = cp[s] + c * kSelChunk, b1 = b0 + kSelChunk < p1 ? b0 + kSelChunk : p1;
    const uint64_t pre = prefix[l];
    h[tid] = 0u;
    __syncthreads();
    for (int64_t p = b0 + tid; p < b1; p += 256) {
      const uint64_t key = fkey(num[p]);
      if ((key & himask) == pre) atomicAdd(&h[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (h[tid]) atomicAdd(&hist[(int64_t)l * 256 + tid], h[tid]);
    __syncthreads();
  }
}
__global__ void kselect_long_out_kernel(int64_t nl, const int64_t* __restrict__ list, const int64_t* __restrict__ jc,
                                        const int32_t* __restrict__ aidx, const uint64_t* __restrict__ prefix,
                                        double* __restrict__ out) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l < nl) out[aidx[jc[list[l]]]] = fval(prefix[l]);
}

// keep entry (i, col) iff !(v < thresh[col]): pass 1 counts per slot, pass 2 copies
template <bool COPY>
__global__ __launch_bounds__(256) void prune_col_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp,
                                                        const int32_t* __restrict__ ir, const double* __restrict__ num,
                                                        int64_t nzc, const double* __restrict__ thresh,
                                                        int64_t* __restrict__ kept, const int64_t* __restrict__ off,
                                                        int32_t* __restrict__ oir, double* __restrict__ onum) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nzc) return;
  const double t = thresh[jc[s]];
  const int64_t p0 = cp[s], p1 = cp[s + 1];
  int64_t o = COPY ? off[s] : 0;
  for (int64_t b = p0; b < p1; b += 64) {
    const int64_t p = b + lane;
    const double v = p < p1 ? num[p] : 0.0;
    const bool keep = p < p1 && !(v < t);
    const uint64_t m = __ballot(keep);
    if (COPY && keep) {
      const int64_t d = o + __popcll(m & ((1ull << lane) - 1ull));
      oir[d] = ir[p];
      onum[d] = v;
    }
    o += __popcll(m);
  }
  if (!COPY && lane == 0) kept[s] = o;
}

}  // namespace cbh
