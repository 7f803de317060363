// ============================================================================================
// TEST INFRASTRUCTURE ONLY — the CPU oracle. It is the checker for the HIP path and the
// "port" CPU baseline leg of bench.py; no product code links, imports or calls it.
//
// A plain C++ restatement (written from the reference's behaviour, not copied) of CombBLAS's
// local SpGEMM hot path, exposed through a small C ABI for the Python tests:
//   oracle_spgemm kernel=0  LocalHybridSpGEMM  include/CombBLAS/mtSpGEMM.h:213-460
//                          (cr = flop/nnz per column, mtSpGEMM.h:310; cr<2 -> heap merge :311-360
//                           with HeapEntry's key-only ordering HeapEntry.h:50-55; else linear-probe
//                           hash (key*107)&(size-1), size = pow2 >= max(16,nnz) :366-420, add(new,old)
//                           :408, then compaction + sort by row :425-439)
//                  kernel=1  LocalSpGEMMHash(sort=true)  mtSpGEMM.h:463-656
//                  kernel=2  LocalSpGEMMHash(sort=false) (rows in hash-slot order, mtSpGEMM.h:624-634)
//                  kernel=3  LocalSpGEMM (heap only)     mtSpGEMM.h:74-202
//   oracle_symbolic          estimateFLOP mtSpGEMM.h:1057-1134, estimateNNZ_Hash :806-933
//   oracle_merge             MultiwayMerge MultiwayMerge.h:411-526 (k-way heap merge on (col,row),
//                            SR::add(acc, next) on duplicates :210-214)
//   oracle_digest            value sum + order-sensitive digest, same definition as the device
//                            checksum_kernel (combblas_amd/csrc/spgemm.hip)
// Parity pinning: tests/test_oracle.py checks this restatement against fixtures produced by the
// reference itself (oracle/_ref/ref_harness, tests/golden/make_golden.py).
// ============================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <functional>
#include <limits>
#include <thread>
#include <vector>

extern "C" {
typedef struct or_mat {
  int64_t m, n, nnz, nzc;
  int64_t* cp;  // nzc+1
  int64_t* jc;  // nzc
  int32_t* ir;  // nnz
  void* num;    // nnz
  int dtype;    // 0 f64, 1 i64, 2 bool(u8), 3 f32, 4 i32
  int owned;
} or_mat;
}

namespace {

// ---------------------------------------------------------------- semirings (Semirings.h)
template <class T>
struct PlusTimes {
  static T add(T a, T b) { return a + b; }
  static T multiply(T a, T b) { return a * b; }
};
template <class T>
struct SelectMax {
  static T add(T a, T b) { return std::max(a, b); }
  static T multiply(T a, T b) { return a * b; }
};
template <class T>
struct MinPlus {
  static T add(T a, T b) { return std::min(a, b); }
  static T multiply(T a, T b) {
    const T inf = std::numeric_limits<T>::max();
    return (a == inf || b == inf) ? inf : a + b;
  }
};
struct OrAnd {
  static uint8_t add(uint8_t a, uint8_t b) { return (uint8_t)((a != 0) || (b != 0)); }
  static uint8_t multiply(uint8_t a, uint8_t b) { return (uint8_t)((a != 0) && (b != 0)); }
};

template <class T>
struct View {
  int64_t m, n, nnz, nzc;
  const int64_t *cp, *jc;
  const int32_t* ir;
  const T* num;
};
template <class T>
View<T> view(const or_mat* a) {
  return View<T>{a->m, a->n, a->nnz, a->nzc, a->cp, a->jc, a->ir, reinterpret_cast<const T*>(a->num)};
}

or_mat* alloc_mat(int64_t m, int64_t n, int64_t nnz, int64_t nzc, int dtype, size_t vs) {
  or_mat* r = (or_mat*)std::calloc(1, sizeof(or_mat));
  r->m = m;
  r->n = n;
  r->nnz = nnz;
  r->nzc = nzc;
  r->dtype = dtype;
  r->owned = 1;
  r->cp = (int64_t*)std::malloc(sizeof(int64_t) * (nzc + 1));
  r->jc = (int64_t*)std::malloc(sizeof(int64_t) * (nzc ? nzc : 1));
  r->ir = (int32_t*)std::malloc(sizeof(int32_t) * (nnz ? nnz : 1));
  r->num = std::malloc(vs * (nnz ? nnz : 1));
  r->cp[0] = 0;
  return r;
}

template <class F>
void parallel_for(int64_t n, int nthreads, F&& f) {
  if (nthreads <= 1 || n < 64) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> th;
  // interleaved chunks of 64 columns for balance (OpenMP dynamic-ish)
  std::atomic<int64_t> next(0);
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&] {
      for (;;) {
        int64_t b = next.fetch_add(64);
        if (b >= n) break;
        int64_t e = std::min(n, b + 64);
        for (int64_t i = b; i < e; ++i) f(i);
      }
    });
  for (auto& x : th) x.join();
}

struct ColRange {
  int64_t first, second;
};

// FillColInds equivalent: A column ranges for the row ids of B(:, i).
template <class T>
void fill_colinds(const View<T>& A, const std::vector<int64_t>& apos, const View<T>& B, int64_t i,
                  std::vector<ColRange>& ci) {
  const int64_t b0 = B.cp[i], nb = B.cp[i + 1] - b0;
  ci.resize(nb);
  for (int64_t j = 0; j < nb; ++j) {
    const int64_t k = B.ir[b0 + j];
    const int64_t p = (k >= 0 && k < (int64_t)apos.size()) ? apos[k] : -1;
    if (p < 0) ci[j] = {0, 0};
    else ci[j] = {A.cp[p], A.cp[p + 1]};
  }
}

template <class T>
std::vector<int64_t> dense_pos(const View<T>& A) {
  std::vector<int64_t> pos(A.n, -1);
  for (int64_t i = 0; i < A.nzc; ++i) pos[A.jc[i]] = i;
  return pos;
}

int64_t ht_size_for(int64_t need) {
  int64_t s = 16;
  while (s < need) s <<= 1;
  return s;
}

// distinct rows of column i (estimateNNZ_Hash), table sized by flops
template <class T>
int64_t nnz_hash(const View<T>& A, const std::vector<ColRange>& ci, int64_t flop, std::vector<int64_t>& ht) {
  const int64_t sz = ht_size_for(flop);
  ht.assign(sz, -1);
  int64_t cnt = 0;
  for (const ColRange& r : ci)
    for (int64_t k = r.first; k < r.second; ++k) {
      const int64_t key = A.ir[k];
      int64_t h = (key * 107) & (sz - 1);
      for (;;) {
        if (ht[h] == key) break;
        if (ht[h] == -1) {
          ht[h] = key;
          ++cnt;
          break;
        }
        h = (h + 1) & (sz - 1);
      }
    }
  return cnt;
}

template <class T>
struct HeapE {  // same ordering semantics as HeapEntry (key only, inverted => min-heap)
  int64_t key, runr;
  T num;
  bool operator<(const HeapE& o) const { return key > o.key; }
};

template <class SR, class T>
void column_heap(const View<T>& A, const View<T>& B, int64_t i, std::vector<ColRange> ci, int64_t* orow, T* oval,
                 int64_t& cnt) {
  std::vector<HeapE<T>> w;
  w.reserve(ci.size());
  for (size_t j = 0; j < ci.size(); ++j)
    if (ci[j].first != ci[j].second) w.push_back(HeapE<T>{A.ir[ci[j].first], (int64_t)j, A.num[ci[j].first]});
  std::make_heap(w.begin(), w.end());
  int64_t hs = (int64_t)w.size();
  cnt = 0;
  while (hs > 0) {
    std::pop_heap(w.begin(), w.begin() + hs);
    HeapE<T>& top = w[hs - 1];
    const int64_t lb = top.runr;
    const T prod = SR::multiply(top.num, B.num[B.cp[i] + lb]);
    if (cnt > 0 && orow[cnt - 1] == top.key) oval[cnt - 1] = SR::add(oval[cnt - 1], prod);
    else {
      orow[cnt] = top.key;
      oval[cnt] = prod;
      ++cnt;
    }
    if (++ci[lb].first != ci[lb].second) {
      top.key = A.ir[ci[lb].first];
      top.num = A.num[ci[lb].first];
      std::push_heap(w.begin(), w.begin() + hs);
    } else {
      --hs;
    }
  }
}

template <class SR, class T>
void column_hash(const View<T>& A, const View<T>& B, int64_t i, const std::vector<ColRange>& ci, int64_t nnzcol,
                 bool sorted, int64_t* orow, T* oval) {
  const int64_t sz = ht_size_for(nnzcol);
  std::vector<std::pair<int64_t, T>> ht(sz, std::make_pair((int64_t)-1, T()));
  for (size_t j = 0; j < ci.size(); ++j) {
    const T bv = B.num[B.cp[i] + j];
    for (int64_t k = ci[j].first; k < ci[j].second; ++k) {
      const T prod = SR::multiply(A.num[k], bv);
      const int64_t key = A.ir[k];
      int64_t h = (key * 107) & (sz - 1);
      for (;;) {
        if (ht[h].first == key) {
          ht[h].second = SR::add(prod, ht[h].second);
          break;
        }
        if (ht[h].first == -1) {
          ht[h].first = key;
          ht[h].second = prod;
          break;
        }
        h = (h + 1) & (sz - 1);
      }
    }
  }
  int64_t idx = 0;
  for (int64_t s = 0; s < sz; ++s)
    if (ht[s].first != -1) ht[idx++] = ht[s];
  if (sorted)
    std::sort(ht.begin(), ht.begin() + idx,
              [](const std::pair<int64_t, T>& a, const std::pair<int64_t, T>& b) { return a.first < b.first; });
  for (int64_t s = 0; s < idx; ++s) {
    orow[s] = ht[s].first;
    oval[s] = ht[s].second;
  }
}

template <class SR, class T>
or_mat* spgemm(const or_mat* Am, const or_mat* Bm, int kernel, int nthreads, size_t vs) {
  View<T> A = view<T>(Am), B = view<T>(Bm);
  const int64_t nzc = B.nzc;
  std::vector<int64_t> apos = dense_pos(A);
  std::vector<int64_t> flop(nzc, 0), nnz(nzc, 0);
  // symbolic: estimateFLOP + nnz (hash for hybrid/hash kernels, exact distinct count either way)
  parallel_for(nzc, nthreads, [&](int64_t i) {
    thread_local std::vector<ColRange> ci;
    thread_local std::vector<int64_t> ht;
    fill_colinds(A, apos, B, i, ci);
    int64_t f = 0;
    for (auto& r : ci) f += r.second - r.first;
    flop[i] = f;
    nnz[i] = nnz_hash(A, ci, f, ht);
  });
  std::vector<int64_t> ptr(nzc + 1, 0);
  for (int64_t i = 0; i < nzc; ++i) ptr[i + 1] = ptr[i] + nnz[i];
  std::vector<int64_t> rows(ptr[nzc]);
  std::vector<T> vals(ptr[nzc]);
  parallel_for(nzc, nthreads, [&](int64_t i) {
    thread_local std::vector<ColRange> ci;
    fill_colinds(A, apos, B, i, ci);
    int64_t* orow = rows.data() + ptr[i];
    T* oval = vals.data() + ptr[i];
    bool heap = false;
    if (kernel == 3) heap = true;
    else if (kernel == 0) heap = ((double)flop[i] / (double)nnz[i]) < 2.0;  // NaN (0/0) -> hash
    if (heap) {
      int64_t cnt;
      column_heap<SR, T>(A, B, i, ci, orow, oval, cnt);
    } else {
      column_hash<SR, T>(A, B, i, ci, nnz[i], kernel != 2, orow, oval);
    }
  });
  // tuples -> DCSC (drop empty columns, SpDCCols(SpTuples))
  int64_t nzcC = 0;
  for (int64_t i = 0; i < nzc; ++i) nzcC += nnz[i] > 0;
  or_mat* C = alloc_mat(A.m, B.n, ptr[nzc], nzcC, Am->dtype, vs);
  int64_t c = 0;
  for (int64_t i = 0; i < nzc; ++i)
    if (nnz[i] > 0) {
      C->jc[c] = B.jc[i];
      C->cp[c + 1] = ptr[i + 1];
      ++c;
    }
  for (int64_t p = 0; p < ptr[nzc]; ++p) {
    C->ir[p] = (int32_t)rows[p];
    reinterpret_cast<T*>(C->num)[p] = vals[p];
  }
  return C;
}

template <class SR, class T>
or_mat* merge(int nl, const or_mat* const* L, size_t vs) {
  // union of columns, then per column a k-way merge with ties combined in list order
  std::vector<int64_t> cols;
  for (int l = 0; l < nl; ++l) cols.insert(cols.end(), L[l]->jc, L[l]->jc + L[l]->nzc);
  std::sort(cols.begin(), cols.end());
  cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
  std::vector<std::vector<int64_t>> pos(nl);
  for (int l = 0; l < nl; ++l) {
    pos[l].assign(cols.size(), -1);
    size_t q = 0;
    for (int64_t i = 0; i < L[l]->nzc; ++i) {
      while (cols[q] != L[l]->jc[i]) ++q;
      pos[l][q] = i;
    }
  }
  std::vector<int64_t> cp(cols.size() + 1, 0);
  std::vector<int32_t> rows;
  std::vector<T> vals;
  for (size_t c = 0; c < cols.size(); ++c) {
    std::vector<std::pair<int64_t, int64_t>> cur(nl, {0, 0});  // [pos, end) into list l
    for (int l = 0; l < nl; ++l)
      if (pos[l][c] >= 0) cur[l] = {L[l]->cp[pos[l][c]], L[l]->cp[pos[l][c] + 1]};
    for (;;) {
      int64_t best = std::numeric_limits<int64_t>::max();
      for (int l = 0; l < nl; ++l)
        if (cur[l].first < cur[l].second) best = std::min<int64_t>(best, L[l]->ir[cur[l].first]);
      if (best == std::numeric_limits<int64_t>::max()) break;
      bool first = true;
      T acc{};
      for (int l = 0; l < nl; ++l)
        if (cur[l].first < cur[l].second && L[l]->ir[cur[l].first] == best) {
          const T v = reinterpret_cast<const T*>(L[l]->num)[cur[l].first++];
          acc = first ? v : SR::add(acc, v);
          first = false;
        }
      rows.push_back((int32_t)best);
      vals.push_back(acc);
    }
    cp[c + 1] = (int64_t)rows.size();
  }
  or_mat* C = alloc_mat(L[0]->m, L[0]->n, (int64_t)rows.size(), (int64_t)cols.size(), L[0]->dtype, vs);
  std::copy(cols.begin(), cols.end(), C->jc);
  std::copy(cp.begin(), cp.end(), C->cp);
  std::copy(rows.begin(), rows.end(), C->ir);
  std::copy(vals.begin(), vals.end(), reinterpret_cast<T*>(C->num));
  return C;
}

template <template <class> class S, class F>
or_mat* by_type(int dtype, F&& f) {
  switch (dtype) {
    case 0: return f(S<double>{}, double{}, 8);
    case 1: return f(S<int64_t>{}, int64_t{}, 8);
    case 3: return f(S<float>{}, float{}, 4);
    case 4: return f(S<int32_t>{}, int32_t{}, 4);
  }
  return nullptr;
}

template <class F>
or_mat* dispatch(int sr, int dtype, F&& f) {
  if (dtype == 2) return f(OrAnd{}, uint8_t{}, 1);  // bool: OR-AND regardless of sr id (PlusTimes<bool>)
  if (sr == 0) return by_type<PlusTimes>(dtype, f);
  if (sr == 1) return by_type<SelectMax>(dtype, f);
  if (sr == 2) return by_type<MinPlus>(dtype, f);
  return nullptr;
}

uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

}  // namespace

extern "C" {

or_mat* oracle_spgemm(int sr, int dtype, int kernel, const or_mat* A, const or_mat* B, int nthreads) {
  if (!A || !B || A->n != B->m) return nullptr;
  return dispatch(sr, dtype, [&](auto srv, auto tv, size_t vs) -> or_mat* {
    using SR = decltype(srv);
    using T = decltype(tv);
    return spgemm<SR, T>(A, B, kernel, nthreads, vs);
  });
}

or_mat* oracle_merge(int sr, int dtype, int nlists, const or_mat* const* L) {
  if (nlists <= 0) return nullptr;
  return dispatch(sr, dtype, [&](auto srv, auto tv, size_t vs) -> or_mat* {
    using SR = decltype(srv);
    using T = decltype(tv);
    return merge<SR, T>(nlists, L, vs);
  });
}

int oracle_symbolic(const or_mat* Am, const or_mat* Bm, int64_t* flops, int64_t* nnzC, int64_t* colflop,
                    int64_t* colnnz, int nthreads) {
  if (!Am || !Bm || Am->n != Bm->m) return 3002;
  View<uint8_t> A{Am->m, Am->n, Am->nnz, Am->nzc, Am->cp, Am->jc, Am->ir, nullptr};
  View<uint8_t> B{Bm->m, Bm->n, Bm->nnz, Bm->nzc, Bm->cp, Bm->jc, Bm->ir, nullptr};
  std::vector<int64_t> apos = dense_pos(A);
  std::vector<int64_t> f(B.nzc), z(B.nzc);
  parallel_for(B.nzc, nthreads, [&](int64_t i) {
    thread_local std::vector<ColRange> ci;
    thread_local std::vector<int64_t> ht;
    fill_colinds(A, apos, B, i, ci);
    int64_t s = 0;
    for (auto& r : ci) s += r.second - r.first;
    f[i] = s;
    z[i] = nnz_hash(A, ci, s, ht);
  });
  int64_t tf = 0, tz = 0;
  for (int64_t i = 0; i < B.nzc; ++i) {
    tf += f[i];
    tz += z[i];
    if (colflop) colflop[i] = f[i];
    if (colnnz) colnnz[i] = z[i];
  }
  if (flops) *flops = tf;
  if (nnzC) *nnzC = tz;
  return 0;
}

// value sum and digest = sum_p mix64(p ^ mix64(col ^ mix64(row ^ mix64(bits)))) (mod 2^64)
int oracle_digest(const or_mat* C, double* vsum, uint64_t* digest) {
  double s = 0;
  uint64_t d = 0;
  for (int64_t c = 0; c < C->nzc; ++c)
    for (int64_t p = C->cp[c]; p < C->cp[c + 1]; ++p) {
      uint64_t bits = 0;
      double v = 0;
      switch (C->dtype) {
        case 0: { double x = ((const double*)C->num)[p]; std::memcpy(&bits, &x, 8); v = x; break; }
        case 1: { int64_t x = ((const int64_t*)C->num)[p]; bits = (uint64_t)x; v = (double)x; break; }
        case 2: { uint8_t x = ((const uint8_t*)C->num)[p]; bits = x; v = x; break; }
        case 3: { float x = ((const float*)C->num)[p]; uint32_t b; std::memcpy(&b, &x, 4); bits = b; v = x; break; }
        case 4: { int32_t x = ((const int32_t*)C->num)[p]; bits = (uint64_t)(uint32_t)x; v = x; break; }
      }
      s += v;
      d += mix64((uint64_t)p ^ mix64((uint64_t)C->jc[c] ^ mix64((uint64_t)(uint32_t)C->ir[p] ^ mix64(bits))));
    }
  *vsum = s;
  *digest = d;
  return 0;
}

void oracle_free(or_mat* C) {
  if (!C || !C->owned) return;
  std::free(C->cp);
  std::free(C->jc);
  std::free(C->ir);
  std::free(C->num);
  std::free(C);
}

}  // extern "C"
