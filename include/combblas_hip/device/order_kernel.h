// order_kernel.h -- REFERENCE-ORDER numeric pass for semirings whose add is not commutative
// (Select2ndSRing, Semirings.h:143-163; any user semiring marked SR::kOrdered): the device
// re-executes LocalHybridSpGEMM's per-column algorithm (mtSpGEMM.h:289-441) exactly, one thread
// per output column, so every output is folded in the reference's own order:
//   * cr = flops / nnz of the column < 2: the HEAP branch (mtSpGEMM.h:311-360) -- std::make_heap /
//     pop_heap / push_heap over HeapEntry (HeapEntry.h: min-heap on the row only), restated below as
//     libstdc++'s __adjust_heap / __push_heap so that equal rows pop in the same order; repeated
//     rows fold add(old, new) (:341);
//   * otherwise the HASH branch (:362-437): the reference's table (ht_size = 2^k >= nnz, >= 16,
//     slot (row*107) & (ht_size-1), linear probing), products in B-entry order folded
//     add(new, old) (:408), then the occupied slots sorted by row (:434).
// The throughput kernels (task_kernel.h) accumulate in arrival order, which is exact for a
// commutative, associative add only; this pass is the correctness path for the others (and gives
// bit-exact f64 PlusTimes sums as well when a caller marks the semiring ordered). It is not a hot
// path: one thread walks a whole column.
#pragma once
#include "task_kernel.h"

namespace cbh {

template <class SR, class = void>
struct sr_ordered : std::false_type {};
template <class SR>
struct sr_ordered<SR, std::void_t<decltype(SR::kOrdered)>> : std::integral_constant<bool, SR::kOrdered> {};

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
  OrdHeapEntry<SR>* heap;  // nnz(B) entries: a column's heap at its B entries' offsets
  int64_t* cfirst;         // nnz(B): colinds[j].first / .second of the reference
  int64_t* csecond;
  int64_t* hkey;           // hash tables: 2 * nnz(C) + 16 * ntasks slots
  typename SR::val_t* hval;
};

template <class SR>
__global__ __launch_bounds__(64) void order_kernel(TaskArgs a, OrdScratch<SR> s, int branch) {
  using val_t = typename SR::val_t;
  using a_t = typename sr_a_type<SR>::type;
  using b_t = typename sr_b_type<SR>::type;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.ntasks) return;
  const int32_t c = a.tcol[t];
  if (t > 0 && a.tcol[t - 1] == c) return;  // the column's first task walks it
  int64_t t2 = t + 1;
  while (t2 < a.ntasks && a.tcol[t2] == c) ++t2;
  const int64_t cstart = a.toff[t] - a.cbase, cend = a.toff[t2] - a.cbase;
  const int64_t nnzcolC = cend - cstart;
  const int64_t e0 = a.Bcp[c];
  const int64_t nnzcolB = a.Bcp[c + 1] - e0;
  const a_t* Anum = reinterpret_cast<const a_t*>(a.Anum);
  const b_t* Bnum = reinterpret_cast<const b_t*>(a.Bnum);
  val_t* Cnum = reinterpret_cast<val_t*>(a.Cnum);
  int64_t* cf = s.cfirst + e0;
  int64_t* cs = s.csecond + e0;
  int64_t flops = 0;
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
    flops += l - f;
  }
  if (nnzcolC <= 0) {
    if (flops > 0) atomicAdd(&a.err[0], 1);
    return;
  }
  if (cend > a.ccap) {
    guard_fail(a.err, 5, c, cend);
    return;
  }
  const double cr = (double)flops / (double)nnzcolC;  // mtSpGEMM.h:310
  int64_t cur = cstart;
  if (branch == 1 || (branch == 0 && cr < 2.0)) {  // heap branch
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
        a.Cir[cur] = (int32_t)top.key;
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
  } else {  // hash branch
    int64_t ht = 16;
    while (ht < nnzcolC) ht <<= 1;
    int64_t* hk = s.hkey + 2 * cstart + 16 * t;
    val_t* hv = s.hval + 2 * cstart + 16 * t;
    for (int64_t x = 0; x < ht; ++x) hk[x] = -1;
    for (int64_t j = 0; j < nnzcolB; ++j) {
      const b_t bv = Bnum[e0 + j];
      for (int64_t k = cf[j]; k < cs[j]; ++k) {
        const val_t mrhs = SR::multiply(Anum[k], bv);
        const int64_t key = a.Air[k];
        int64_t h = (key * 107) & (ht - 1);
        while (true) {
          if (hk[h] == key) {
            hv[h] = SR::add(mrhs, hv[h]);
            break;
          } else if (hk[h] == -1) {
            hk[h] = key;
            hv[h] = mrhs;
            break;
          }
          h = (h + 1) & (ht - 1);
        }
      }
    }
    int64_t n = 0;
    for (int64_t x = 0; x < ht; ++x)
      if (hk[x] != -1) {
        hk[n] = hk[x];
        hv[n] = hv[x];
        ++n;
      }
    if (n != nnzcolC) {
      atomicAdd(&a.err[0], 1);
      return;
    }
    // sort by row (keys are distinct, so any correct sort is the reference's std::sort result):
    // heapsort in place
    auto sift = [&](int64_t root, int64_t len) {
      while (true) {
        int64_t ch = 2 * root + 1;
        if (ch >= len) return;
        if (ch + 1 < len && hk[ch + 1] > hk[ch]) ++ch;
        if (hk[ch] <= hk[root]) return;
        const int64_t tk = hk[root];
        hk[root] = hk[ch];
        hk[ch] = tk;
        const val_t tv = hv[root];
        hv[root] = hv[ch];
        hv[ch] = tv;
        root = ch;
      }
    };
    for (int64_t r = n / 2 - 1; r >= 0; --r) sift(r, n);
    for (int64_t e = n - 1; e > 0; --e) {
      const int64_t tk = hk[0];
      hk[0] = hk[e];
      hk[e] = tk;
      const val_t tv = hv[0];
      hv[0] = hv[e];
      hv[e] = tv;
      sift(0, e);
    }
    for (int64_t x = 0; x < n; ++x) {
      a.Cir[cstart + x] = (int32_t)hk[x];
      Cnum[cstart + x] = hv[x];
    }
    cur = cstart + n;
  }
  if (cur != cend) atomicAdd(&a.err[0], 1);
}

// The numeric pass of a plan in reference order (every task id; the first task of each column
// walks the column). nnzB: B's entries (heap and column-range scratch). branch: 0 the hybrid
// (LocalHybridSpGEMM), 1 heap only (LocalSpGEMM), 2 hash only (LocalSpGEMMHash). The scratch is
// allocated here and freed after the launch has completed.
template <class SR>
hipError_t run_numeric_plan_ordered(const cbh_numeric_plan& p, int32_t* Cir, void* Cnum, int64_t ccap,
                                    int64_t nnzB, int branch = 0) {
  using val_t = typename SR::val_t;
  hipStream_t st = reinterpret_cast<hipStream_t>(p.stream);
  TaskArgs a{};
  a.Acp = p.Acp;
  a.Air = p.Air;
  a.Anum = p.Anum;
  a.Bcp = p.Bcp;
  a.Bir = p.Bir;
  a.Bnum = p.Bnum;
  a.tcol = p.tcol;
  a.toff = p.toff;
  a.cbase = 0;
  a.Cir = Cir;
  a.Cnum = Cnum;
  a.ccap = ccap;
  a.err = p.err;
  a.nnzA = p.nnzA;
  a.ncolA = p.ncolA;
  a.ntasks = p.ntasks;
  if (p.ntasks <= 0) return hipSuccess;
  OrdScratch<SR> s{};
  const size_t nb = (size_t)std::max<int64_t>(nnzB, 1);
  const size_t nh = (size_t)(2 * ccap + 16 * p.ntasks);
  hipError_t e = hipSuccess;
  void* blk[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  const size_t sz[5] = {nb * sizeof(OrdHeapEntry<SR>), nb * sizeof(int64_t), nb * sizeof(int64_t),
                        nh * sizeof(int64_t), nh * sizeof(val_t)};
  for (int i = 0; i < 5 && e == hipSuccess; ++i) e = hipMalloc(&blk[i], sz[i]);
  if (e == hipSuccess) {
    s.heap = static_cast<OrdHeapEntry<SR>*>(blk[0]);
    s.cfirst = static_cast<int64_t*>(blk[1]);
    s.csecond = static_cast<int64_t*>(blk[2]);
    s.hkey = static_cast<int64_t*>(blk[3]);
    s.hval = static_cast<val_t*>(blk[4]);
    hipLaunchKernelGGL(order_kernel<SR>, dim3((unsigned)((p.ntasks + 63) / 64)), dim3(64), 0, st, a, s, branch);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  for (int i = 0; i < 5; ++i)  // (after the synchronize: nothing in flight reads them)
    if (blk[i]) {
      const hipError_t f = hipFree(blk[i]);
      if (e == hipSuccess) e = f;
    }
  return e;
}

}  // namespace cbh
