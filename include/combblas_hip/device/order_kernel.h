// order_kernel.h -- REFERENCE-ORDER numeric pass: every output of C folded in exactly the order
// the reference's LocalHybridSpGEMM (mtSpGEMM.h:289-441) folds it, so that a semiring whose add is
// not commutative or associative (Select2ndSRing, Semirings.h:143-163; any user semiring not
// marked arrival_order_ok, HipSpGEMMDevice.h) -- and floating-point PlusTimes sums -- match the
// stock path bit for bit. Per column the reference picks a branch by cr = flops / nnz (:310):
//   * cr < 2, the HEAP branch (:311-360): std::make_heap / pop_heap / push_heap over HeapEntry
//     (HeapEntry.h: min-heap on the row only), restated below as libstdc++'s __adjust_heap /
//     __push_heap so that equal rows pop in the same order; repeated rows fold add(old, new) (:341).
//     Inherently serial: ONE THREAD per heap-branch column (order_heap_kernel).
//   * otherwise the HASH branch (:362-437): products in B-entry order, within an entry in A-column
//     order, each folded add(new, old) into its row's slot (:408) -- so a row's value is the fold
//     of its products in increasing B-entry order, whatever the table. ONE WAVE PER TASK
//     (order_fold_kernel): the throughput pass has already written C's rows (sorted), the wave
//     walks the task's products in B-entry order 64 at a time, finds each product's output by a
//     binary search of its row in the task's rows, and folds the products of one output in lane
//     order (= B-entry order): conflicting lanes of a batch go in rounds, the lowest lane of each
//     output first (an LDS owner table, ds_min).
// The throughput kernels (task_kernel.h) accumulate in arrival order, exact for a commutative,
// associative add (integers, bool, min / max); this pass runs after them on the same C.
#pragma once
#include "wave_kernel.h"  // task_kernel.h, wave_lds_sync

namespace cbh {

template <class SR, class = void>
struct sr_ordered : std::false_type {};
template <class SR>
struct sr_ordered<SR, std::void_t<decltype(SR::kOrdered)>> : std::integral_constant<bool, SR::kOrdered> {};

// a built-in functor in reference order (the library's CBH_ORDER_* flags, HipSpGEMMKernels.h)
template <class SR>
struct Ordered : SR {
  static constexpr bool kOrdered = true;
};

template <class SR>
struct OrdHeapEntry {  // HeapEntry<IT, NT1> (HeapEntry.h): operator< is "key greater"
  int64_t key;
  int64_t runr;
  typename sr_a_type<SR>::type num;
};

template <class E>
__device__ __forceinline__ bool heap_less(const E& a, const E& b) {
  return a.key > b.key;  // HeapEntry::operator<
}
// libstdc++ std::__push_heap (bits/stl_heap.h)
template <class E>
__device__ void ord_push_heap(E* first, int64_t hole, int64_t top, E value) {
  int64_t parent = (hole - 1) / 2;
  while (hole > top && heap_less(first[parent], value)) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}
// libstdc++ std::__adjust_heap
template <class E>
__device__ void ord_adjust_heap(E* first, int64_t hole, int64_t len, E value) {
  const int64_t top = hole;
  int64_t child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (heap_less(first[child], first[child - 1])) child--;
    first[hole] = first[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    first[hole] = first[child - 1];
    hole = child - 1;
  }
  ord_push_heap(first, hole, top, value);
}
template <class E>
__device__ void ord_make_heap(E* first, int64_t len) {
  if (len < 2) return;
  int64_t parent = (len - 2) / 2;
  while (true) {
    ord_adjust_heap(first, parent, len, first[parent]);
    if (parent == 0) return;
    parent--;
  }
}
template <class E>
__device__ void ord_pop_heap(E* first, int64_t len) {  // std::pop_heap(first, first + len)
  if (len > 1) {
    const E value = first[len - 1];
    first[len - 1] = first[0];
    ord_adjust_heap(first, 0, len - 1, value);
  }
}
template <class E>
__device__ void ord_push_heap_back(E* first, int64_t len) {  // std::push_heap(first, first + len)
  ord_push_heap(first, len - 1, 0, first[len - 1]);
}

template <class SR>
struct OrdScratch {
  OrdHeapEntry<SR>* heap;  // nnz(B) entries: a heap column's heap at its B entries' offsets
  int64_t* cfirst;         // nnz(B): colinds[j].first / .second of the reference
  int64_t* csecond;
  uint8_t* tbranch;        // per task: 1 its column takes the heap branch, 2 the hash branch
  uint8_t* seen;           // per output of C: the hash-branch fold has stored its first product
};
enum : uint8_t { kOrdHeap = 1, kOrdHash = 2 };

// branch of every column (its first task decides for all its tasks): cr = flops / nnz(C(:, j))
// (mtSpGEMM.h:310); branch 1 / 2 forces LocalSpGEMM's heap / LocalSpGEMMHash's hash
__global__ __launch_bounds__(256) void order_classify_kernel(TaskArgs a, uint8_t* tbranch, int branch) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.ntasks) return;
  const int32_t c = a.tcol[t];
  if (t > 0 && a.tcol[t - 1] == c) return;  // the column's first task classifies it
  int64_t t2 = t + 1;
  while (t2 < a.ntasks && a.tcol[t2] == c) ++t2;
  const int64_t nnzc = a.toff[t2] - a.toff[t];
  int64_t flops = 0;
  for (int64_t p = a.Bcp[c]; p < a.Bcp[c + 1]; ++p) {
    const int32_t k = a.Bir[p];
    if (k >= 0 && k < a.ncolA) flops += a.Acp[k + 1] - a.Acp[k];
  }
  const bool heap = branch == 1 || (branch == 0 && nnzc > 0 && (double)flops / (double)nnzc < 2.0);
  for (int64_t u = t; u < t2; ++u) tbranch[u] = heap ? kOrdHeap : kOrdHash;
}

// The heap branch, one thread per heap-branch column (its first task's thread): rewrites the
// column's rows and values from the restated heap sequence.
template <class SR>
__global__ __launch_bounds__(64) void order_heap_kernel(TaskArgs a, OrdScratch<SR> s) {
  using val_t = typename SR::val_t;
  using a_t = typename sr_a_type<SR>::type;
  using b_t = typename sr_b_type<SR>::type;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.ntasks) return;
  const int32_t c = a.tcol[t];
  if (t > 0 && a.tcol[t - 1] == c) return;  // the column's first task walks it
  if (s.tbranch[t] != kOrdHeap) return;
  int64_t t2 = t + 1;
  while (t2 < a.ntasks && a.tcol[t2] == c) ++t2;
  const int64_t cstart = a.toff[t] - a.cbase, cend = a.toff[t2] - a.cbase;
  const int64_t e0 = a.Bcp[c];
  const int64_t nnzcolB = a.Bcp[c + 1] - e0;
  const a_t* Anum = reinterpret_cast<const a_t*>(a.Anum);
  const b_t* Bnum = reinterpret_cast<const b_t*>(a.Bnum);
  val_t* Cnum = reinterpret_cast<val_t*>(a.Cnum);
  int64_t* cf = s.cfirst + e0;
  int64_t* cs = s.csecond + e0;
  for (int64_t j = 0; j < nnzcolB; ++j) {  // FillColInds: A(:, B(j, c)) for every B entry
    const int32_t k = a.Bir[e0 + j];
    int64_t f = 0, l = 0;
    if (k >= 0 && k < a.ncolA) {
      f = a.Acp[k];
      l = a.Acp[k + 1];
    } else {
      guard_fail(a.err, 1, c, k);
    }
    cf[j] = f;
    cs[j] = l;
  }
  if (cend > a.ccap) {
    guard_fail(a.err, 5, c, cend);
    return;
  }
  int64_t cur = cstart;
  OrdHeapEntry<SR>* w = s.heap + e0;
  int64_t hsize = 0;
  for (int64_t j = 0; j < nnzcolB; ++j)
    if (cf[j] != cs[j]) w[hsize++] = OrdHeapEntry<SR>{(int64_t)a.Air[cf[j]], j, Anum[cf[j]]};
  ord_make_heap(w, hsize);
  while (hsize > 0) {
    ord_pop_heap(w, hsize);
    OrdHeapEntry<SR>& top = w[hsize - 1];
    const int64_t locb = top.runr;
    const val_t mrhs = SR::multiply(top.num, Bnum[e0 + locb]);
    if (cur > cstart && (int64_t)a.Cir[cur - 1] == top.key) {
      Cnum[cur - 1] = SR::add(Cnum[cur - 1], mrhs);
    } else if (cur < cend) {
      if (a.Cir[cur] != (int32_t)top.key) guard_fail(a.err, 12, c, cur);  // the throughput pass's row
      Cnum[cur] = mrhs;
      ++cur;
    } else {
      guard_fail(a.err, 5, c, cur);
      return;
    }
    if (++cf[locb] != cs[locb]) {
      top.key = a.Air[cf[locb]];
      top.num = Anum[cf[locb]];
      ord_push_heap_back(w, hsize);
    } else {
      --hsize;
    }
  }
  if (cur != cend) atomicAdd(&a.err[0], 1);
}

// a lane's value of any trivially copyable type (in 4-byte words)
template <class T>
__device__ __forceinline__ T shfl_any(const T& v, int src) {
  constexpr int W = (int)((sizeof(T) + 3) / 4);
  int w[W] = {};
  __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
  for (int i = 0; i < W; ++i) w[i] = __shfl(w[i], src);
  T out;
  __builtin_memcpy(&out, w, sizeof(T));
  return out;
}

// first q in [lo, hi) with rows[q] >= key (rows sorted, int64 positions)
__device__ __forceinline__ int64_t lb_out(const int32_t* __restrict__ rows, int64_t lo, int64_t hi, int32_t key) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (rows[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// The hash branch, one wave per task of a hash-branch column: the task's products in B-entry
// order, each folded into its output (found in the task's sorted rows) -- the first product of
// an output stored as is, every later one folded add(new, old) (mtSpGEMM.h:401-416). A batch of 64
// products spans one or more B entries; products of one entry have distinct rows, and lanes are in
// entry order, so folding each output's products lowest lane first is the reference's order.
template <class SR>
__global__ __launch_bounds__(64) void order_fold_kernel(TaskArgs a, OrdScratch<SR> s) {
  using val_t = typename SR::val_t;
  using a_t = typename sr_a_type<SR>::type;
  using b_t = typename sr_b_type<SR>::type;
  constexpr int kOwn = 256;  // LDS owner table (outputs hashed by position; a shared slot only adds a round)
  __shared__ uint32_t own[kOwn];
  const int lane = threadIdx.x;
  const int64_t t = blockIdx.x;
  if (t >= a.ntasks || s.tbranch[t] != kOrdHash) return;
  const int32_t c = a.tcol[t];
  const int64_t e0 = a.Bcp[c], ne = a.Bcp[c + 1] - e0;
  const int32_t lo = a.tlo[t], hi = a.thi[t];
  const int64_t out0 = a.toff[t] - a.cbase, out1 = a.toff[t + 1] - a.cbase;
  if (out1 <= out0 || hi <= lo) return;
  if (out1 > a.ccap) {
    if (lane == 0) guard_fail(a.err, 5, c, out1);
    return;
  }
  const int32_t* __restrict__ Air = a.Air;
  const a_t* __restrict__ Anum = reinterpret_cast<const a_t*>(a.Anum);
  const b_t* __restrict__ Bnum = reinterpret_cast<const b_t*>(a.Bnum);
  val_t* Cnum = reinterpret_cast<val_t*>(a.Cnum);
  const int32_t* Cir = a.Cir;
  for (int x = lane; x < kOwn; x += 64) own[x] = 64u;
  wave_lds_sync();
  int bad = 0;
  for (int64_t jb = 0; jb < ne; jb += 64) {
    // lane i: entry jb + i's segment inside the task's rows, and B's value
    const int64_t j = jb + lane;
    int64_t s0 = 0;
    int len = 0;
    b_t bv{};
    if (j < ne) {
      const int32_t k = a.Bir[e0 + j];
      if (k >= 0 && k < a.ncolA) {
        const int64_t base = a.Acp[k], end = a.Acp[k + 1];
        s0 = lb_rows64(Air, base, end, lo);
        len = (int)(lb_rows64(Air, s0, end, hi) - s0);
        bv = Bnum[e0 + j];
      } else {
        bad |= 1 << 1;
      }
    }
    const int incl = wave_incl_sum(len);
    const int off = incl - len;  // exclusive offset of this lane's products
    const int total = __builtin_amdgcn_readlane(incl, 63);
    for (int x0 = 0; x0 < total; x0 += 64) {
      const int x = x0 + lane;
      const bool valid = x < total;
      // owning lane: the last lane whose offset is <= x (offsets ascend; that lane has products,
      // since the next lane's offset -- or the total -- lies past x)
      int ow = 0;
#pragma unroll
      for (int step = 32; step > 0; step >>= 1) {
        const int cand = ow + step;  // <= 63
        if (__shfl(off, cand) <= x) ow = cand;
      }
      const int64_t ps0 = shfl_any(s0, ow);
      const int poff = __shfl(off, ow);
      const b_t pbv = shfl_any(bv, ow);
      int64_t pos = -1;
      val_t prod{};
      if (valid) {
        const int64_t q = ps0 + (x - poff);
        const int32_t row = Air[q];
        prod = SR::multiply(Anum[q], pbv);
        pos = lb_out(Cir, out0, out1, row);
        if (pos >= out1 || Cir[pos] != row) {
          bad |= 1 << 12;  // a product row the throughput pass did not write
          pos = -1;
        }
      }
      bool pending = pos >= 0;
      const uint32_t h = (uint32_t)(pos & (kOwn - 1));
      while (__ballot(pending)) {
        if (pending) atomicMin(&own[h], (uint32_t)lane);
        wave_lds_sync();
        const bool win = pending && own[h] == (uint32_t)lane;
        if (win) {
          if (s.seen[pos]) {
            Cnum[pos] = SR::add(prod, Cnum[pos]);
          } else {
            Cnum[pos] = prod;
            s.seen[pos] = 1;
          }
        }
        __threadfence_block();  // this round's folds before the next round's loads of the same output
        wave_lds_sync();
        if (win) {
          own[h] = 64u;
          pending = false;
        }
        wave_lds_sync();
      }
    }
  }
  if (bad) guard_fail(a.err, 31 - __clz(bad), c, bad, lo);
}

// The reference-order pass over a plan's C, after the throughput numeric pass has written C's rows
// (and arrival-order values): classification, the heap columns (a thread each), the hash tasks (a
// wave each), all on `stream`. Scratch (from the caller's allocator): see ord_scratch_bytes.
// branch: 0 the hybrid (LocalHybridSpGEMM), 1 heap only (LocalSpGEMM), 2 hash only (LocalSpGEMMHash).
template <class SR>
size_t ord_scratch_bytes(int64_t nnzB, int64_t ntasks, int64_t nnzC) {
  const size_t nb = (size_t)(nnzB > 0 ? nnzB : 1);
  return nb * (sizeof(OrdHeapEntry<SR>) + 2 * sizeof(int64_t)) + (size_t)ntasks + (size_t)nnzC + 64;
}
template <class SR>
hipError_t launch_reference_order(const TaskArgs& a, void* scratch, int64_t nnzB, int64_t nnzC, int branch,
                                  hipStream_t st) {
  if (a.ntasks <= 0) return hipSuccess;
  const size_t nb = (size_t)(nnzB > 0 ? nnzB : 1);
  char* p = static_cast<char*>(scratch);
  OrdScratch<SR> s{};
  s.heap = reinterpret_cast<OrdHeapEntry<SR>*>(p);
  p += nb * sizeof(OrdHeapEntry<SR>);
  s.cfirst = reinterpret_cast<int64_t*>(p);
  p += nb * sizeof(int64_t);
  s.csecond = reinterpret_cast<int64_t*>(p);
  p += nb * sizeof(int64_t);
  s.tbranch = reinterpret_cast<uint8_t*>(p);
  p += a.ntasks;
  s.seen = reinterpret_cast<uint8_t*>(p);
  hipError_t e = hipMemsetAsync(s.seen, 0, (size_t)(nnzC > 0 ? nnzC : 1), st);
  if (e != hipSuccess) return e;
  const unsigned g = (unsigned)((a.ntasks + 255) / 256);
  hipLaunchKernelGGL(order_classify_kernel, dim3(g), dim3(256), 0, st, a, s.tbranch, branch);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(order_heap_kernel<SR>, dim3((unsigned)((a.ntasks + 63) / 64)), dim3(64), 0, st, a, s);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int64_t kMaxGrid = (1ll << 32) / 64 - 1;
  for (int64_t off = 0; off < a.ntasks; off += kMaxGrid) {
    TaskArgs b = a;
    const int64_t n = a.ntasks - off < kMaxGrid ? a.ntasks - off : kMaxGrid;
    // (the fold kernel indexes tasks by block id: slices shift the task arrays)
    b.tcol = a.tcol + off;
    b.tlo = a.tlo + off;
    b.thi = a.thi + off;
    b.toff = a.toff + off;
    b.ntasks = n;
    OrdScratch<SR> so = s;
    so.tbranch = s.tbranch + off;
    hipLaunchKernelGGL(order_fold_kernel<SR>, dim3((unsigned)n), dim3(64), 0, st, b, so);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace cbh
