// HipSpGEMM.h -- C++ drop-in adaptor: CombBLAS's local SpGEMM entry points on the gfx950 path.
//
// Include AFTER "CombBLAS/CombBLAS.h". It provides
//   combblas_hip::LocalHybridSpGEMM<SR,NTO>(A, B, clearA, clearB, aux)   (mtSpGEMM.h:213-217)
//   combblas_hip::LocalSpGEMMHash<SR,NTO>(A, B, clearA, clearB, sort)    (mtSpGEMM.h:463-467)
//   combblas_hip::LocalSpGEMM<SR,NTO>(A, B, clearA, clearB)              (mtSpGEMM.h:74-78)
//   combblas_hip::MultiwayMerge<SR>(ArrSpTups, mdim, ndim, delarrs)      (MultiwayMerge.h:411-412)
//   combblas_hip::mult_synch_host<SR>(A, B, clearA, clearB)              (Mult_AnXBn_Synch, ParFriends.h:1004-1108)
// with the reference signatures and ownership rules (heap SpTuples* the caller deletes, tuples
// allocated with ::operator new and flagged isOperatorNew, clearA/clearB delete the inputs,
// delarrs deletes the merged lists), and the macro
//   COMBBLAS_HIP_INSTANTIATE(SR, IT, NT)
// that declares explicit specializations of combblas::LocalHybridSpGEMM / LocalSpGEMMHash /
// LocalSpGEMM / MultiwayMerge / MultiwayMergeHash and, for SpParMats over SpDCCols<IT,NT>,
// Mult_AnXBn_Synch (PSpGEMM's driver) for that semiring and types, so that the UNCHANGED reference
// drivers (PSpGEMM -> Mult_AnXBn_Synch, ParFriends.h:1004-1108; MemEfficientSpGEMM; the 3D
// drivers) instantiate the HIP versions. Use it at namespace scope, after this header and before
// the first call that instantiates a driver. Built-in semirings map to device functors through
// combblas_hip::semiring_traits (specialize it for a user semiring whose device functor exists).
//
// All device work goes through the C-ABI in combblas_hip.h; link with libcombblas_hip.so.
// Errors raise MPI_Abort with the library's code (3001/3002/3005 mirror SpDefs.h), as the
// reference drivers do (ParFriends.h:160-181).
#pragma once

#include <mpi.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <limits>
#include <memory>
#include <tuple>
#include <type_traits>
#include <vector>

#include "../combblas_hip.h"

namespace combblas_hip {

// ------------------------------------------------------------------ type/semiring mapping
inline cbh_ctx* context();

// value type -> dtype code (CBH_OPAQUE for any other trivially copyable type: user semirings)
template <class NT>
struct dtype_of { static constexpr cbh_dtype value = CBH_OPAQUE; };
template <> struct dtype_of<double> { static constexpr cbh_dtype value = CBH_F64; };
template <> struct dtype_of<int64_t> { static constexpr cbh_dtype value = CBH_I64; };
template <> struct dtype_of<float> { static constexpr cbh_dtype value = CBH_F32; };
template <> struct dtype_of<int32_t> { static constexpr cbh_dtype value = CBH_I32; };
template <> struct dtype_of<bool> { static constexpr cbh_dtype value = CBH_BOOL; };

inline int upload_dcsc(const cbh_dcsc& h, cbh_dtype dt, int64_t vbytes, cbh_mat** out) {
  return dt == CBH_OPAQUE ? cbh_mat_upload_bytes(context(), &h, vbytes, out) : cbh_mat_upload(context(), &h, dt, out);
}

template <class SR>
struct semiring_traits;  // specialize: static constexpr cbh_semiring code
template <class T1, class T2>
struct semiring_traits<combblas::PlusTimesSRing<T1, T2>> { static constexpr cbh_semiring code = CBH_SR_PLUS_TIMES; };
template <class T1, class T2>
struct semiring_traits<combblas::SelectMaxSRing<T1, T2>> { static constexpr cbh_semiring code = CBH_SR_SELECT_MAX; };
template <class T1, class T2>
struct semiring_traits<combblas::MinPlusSRing<T1, T2>> { static constexpr cbh_semiring code = CBH_SR_MIN_PLUS; };

inline void die(cbh_ctx* ctx, int rc, const char* what) {
  std::fprintf(stderr, "combblas_hip: %s failed (%d): %s\n", what, rc, ctx ? cbh_last_error(ctx) : "");
  MPI_Abort(MPI_COMM_WORLD, rc);
}

// One context per process (one rank drives one GPU, CommGrid semantics). The device is
// COMBBLAS_HIP_DEVICE when set, else the node-local rank (LOCAL_RANK, MPI_LOCALRANKID,
// OMPI_COMM_WORLD_LOCAL_RANK). A device that cannot be opened is fatal: no silent fallback to
// GPU 0, where a mis-set rank would share a device with another rank (RCCL refuses that). More
// local ranks than devices is allowed only as an explicit rehearsal -- COMBBLAS_HIP_SHARE_DEVICE=1
// or the host-staged transport COMBBLAS_HIP_COMM=mpi -- and then maps local rank modulo devices.
// The RCCL transport also checks that the members of each communicator on one node hold distinct
// devices (SpParMatDev.h, rccl_comm_for).
inline bool device_sharing_allowed() {
  const char* s = std::getenv("COMBBLAS_HIP_SHARE_DEVICE");
  const char* c = std::getenv("COMBBLAS_HIP_COMM");
  return (s && std::atoi(s) != 0) || (c && std::strcmp(c, "mpi") == 0);
}
inline int local_rank_env() {
  for (const char* k : {"LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK"})
    if (const char* v = std::getenv(k)) return std::atoi(v);
  return 0;
}
inline cbh_ctx* context() {
  static cbh_ctx* ctx = nullptr;
  if (!ctx) {
    int ndev = 0;
    if (cbh_device_count(&ndev) != CBH_OK) die(nullptr, CBH_E_NODEVICE, "cbh_device_count (no GPU)");
    int dev;
    if (const char* e = std::getenv("COMBBLAS_HIP_DEVICE")) {
      dev = std::atoi(e);
    } else {
      dev = local_rank_env();
      if (dev >= ndev) {
        if (!device_sharing_allowed()) {
          std::fprintf(stderr,
                       "combblas_hip: node-local rank %d but only %d visible GPU(s); set COMBBLAS_HIP_DEVICE, or "
                       "COMBBLAS_HIP_SHARE_DEVICE=1 to share devices (host-staged rehearsals only)\n",
                       dev, ndev);
          MPI_Abort(MPI_COMM_WORLD, CBH_E_NODEVICE);
        }
        dev %= ndev;
      }
    }
    int rc = cbh_ctx_create(dev, &ctx);
    if (rc != CBH_OK) {
      std::fprintf(stderr, "combblas_hip: cannot open GPU %d of %d\n", dev, ndev);
      die(nullptr, rc, "cbh_ctx_create");
    }
  }
  return ctx;
}

struct MatGuard {
  cbh_mat* m = nullptr;
  ~MatGuard() {
    if (m) cbh_mat_free(context(), m);
  }
};

// Host <-> device transfers of the adaptors go through the context's pinned staging in chunks
// (cbh_mat_upload_chunks / cbh_mat_download_chunks): the copy engine moves one chunk while the
// OpenMP threads below convert the next (int64 row ids <-> int32, SpTuples' AoS layout).
// Per-process totals of the adaptor's stages (seconds), printed per driver call with
// COMBBLAS_HIP_TIMING=1 and read by the drop-in bench harness.
struct AdaptorTimes {
  double upload = 0, kernel = 0, merge = 0, download = 0, build = 0;
  int64_t calls = 0;
};
inline AdaptorTimes& adaptor_times() {
  static AdaptorTimes t;
  return t;
}
inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
inline bool timing_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("COMBBLAS_HIP_TIMING");
    return e && std::atoi(e) != 0;
  }();
  return v;
}

// SpDCCols<IT,NT> (Dcsc arrays) -> device matrix. Row ids narrowed to the local int32 layout.
template <class IT, class NT>
cbh_mat* upload(const combblas::SpDCCols<IT, NT>& A) {
  static_assert(std::is_trivially_copyable<NT>::value, "device values must be trivially copyable");
  const int64_t m = A.getnrow(), n = A.getncol();
  if (m > std::numeric_limits<int32_t>::max()) die(context(), CBH_E_DIMMISMATCH, "local rows exceed int32");
  combblas::Dcsc<IT, NT>* d = A.getnnz() > 0 ? A.GetDCSC() : nullptr;
  const int64_t nnz = d ? (int64_t)d->nz : 0, nzc = d ? (int64_t)d->nzc : 0;
  std::vector<int64_t> cpv, jcv;
  const int64_t *cp = nullptr, *jc = nullptr;
  if (d) {
    if (std::is_same<IT, int64_t>::value) {
      cp = reinterpret_cast<const int64_t*>(d->cp);
      jc = reinterpret_cast<const int64_t*>(d->jc);
    } else {
      cpv.assign(d->cp, d->cp + nzc + 1);
      jcv.assign(d->jc, d->jc + nzc);
      cp = cpv.data();
      jc = jcv.data();
    }
  }
  struct Src {
    const IT* ir;
    const NT* num;
  } src{d ? d->ir : nullptr, d ? d->numx : nullptr};
  cbh_fill_fn fill = [](void* u, int64_t f, int64_t cnt, int32_t* ir, void* num) -> int {
    const Src* s = static_cast<const Src*>(u);
    NT* out = static_cast<NT*>(num);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < cnt; ++i) {
      ir[i] = static_cast<int32_t>(s->ir[f + i]);
      out[i] = s->num[f + i];
    }
    return 0;
  };
  cbh_mat* out = nullptr;
  int rc = cbh_mat_upload_chunks(context(), m, n, nnz, nzc, cp, jc, dtype_of<NT>::value, (int64_t)sizeof(NT), 0, fill,
                                 &src, &out);
  if (rc != CBH_OK) die(context(), rc, "cbh_mat_upload_chunks");
  return out;
}

// column-sorted SpTuples -> device DCSC. sort_rows: rows inside a column may be in any order (the
// unsorted outputs of the stock LocalSpGEMMHash / MultiwayMergeHash(sorted=false), mtSpGEMM.h:624-634);
// they are sorted per column on the way up, as the device merge reads row-sorted segments.
template <class IT, class NT>
cbh_mat* upload(const combblas::SpTuples<IT, NT>& T, bool sort_rows = false) {
  cbh_dcsc h{};
  h.m = T.getnrow();
  h.n = T.getncol();
  h.nnz = T.getnnz();
  if (h.m > std::numeric_limits<int32_t>::max()) die(context(), CBH_E_DIMMISMATCH, "local rows exceed int32");
  std::vector<int64_t> cp, jc;
  std::vector<int32_t> ir(h.nnz);
  std::unique_ptr<NT[]> num(new NT[h.nnz > 0 ? h.nnz : 1]);  // not std::vector: vector<bool> has no data()
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < h.nnz; ++i) {
    ir[i] = static_cast<int32_t>(T.rowindex(i));
    num[i] = T.numvalue(i);
  }
  // column heads (the tuples are column-sorted): counted per block, offsets by a scan over the
  // blocks, written per block -- both passes parallel
  constexpr int64_t kBlocks = 256;
  const int64_t bl = (h.nnz + kBlocks - 1) / kBlocks;
  std::vector<int64_t> heads(kBlocks + 1, 0);
  auto head = [&T](int64_t i) { return i == 0 || T.colindex(i) != T.colindex(i - 1); };
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < kBlocks; ++b) {
    int64_t c = 0;
    for (int64_t i = b * bl, e = std::min(h.nnz, (b + 1) * bl); i < e; ++i) c += head(i) ? 1 : 0;
    heads[b + 1] = c;
  }
  for (int64_t b = 0; b < kBlocks; ++b) heads[b + 1] += heads[b];
  h.nzc = heads[kBlocks];
  cp.resize(h.nzc + 1);
  jc.resize(h.nzc);
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < kBlocks; ++b) {
    int64_t k = heads[b];
    for (int64_t i = b * bl, e = std::min(h.nnz, (b + 1) * bl); i < e; ++i)
      if (head(i)) {
        cp[k] = i;
        jc[k++] = T.colindex(i);
      }
  }
  cp[h.nzc] = h.nnz;
  const int64_t ncols_up = (int64_t)cp.size() - 1;
  if (sort_rows)
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t c = 0; c < ncols_up; ++c) {
      const int64_t b = cp[c], e = cp[c + 1];
      bool sorted = true;
      for (int64_t i = b + 1; i < e && sorted; ++i) sorted = ir[i - 1] < ir[i];
      if (sorted) continue;
      std::vector<std::pair<int32_t, NT>> col;
      for (int64_t i = b; i < e; ++i) col.emplace_back(ir[i], num[i]);
      std::sort(col.begin(), col.end(), [](const std::pair<int32_t, NT>& x, const std::pair<int32_t, NT>& y) {
        return x.first < y.first;
      });
      for (int64_t i = b; i < e; ++i) {
        ir[i] = col[i - b].first;
        num[i] = col[i - b].second;
      }
    }
  h.cp = cp.data();
  h.jc = jc.data();
  h.ir = ir.data();
  h.num = reinterpret_cast<const void*>(num.get());
  cbh_mat* out = nullptr;
  int rc = upload_dcsc(h, dtype_of<NT>::value, (int64_t)sizeof(NT), &out);
  if (rc != CBH_OK) die(context(), rc, "cbh_mat_upload");
  return out;
}

// The arrays a download fills are fresh allocations (SpDCCols / ::operator new): every 4 KB page
// faults at its first write inside the take callback. Transparent huge pages for them (where the
// host's THP mode is "madvise") fault 2 MB at a time; COMBBLAS_HIP_NO_THP=1 skips the advice.
inline void advise_huge(void* p, size_t bytes) {
  static const bool off = std::getenv("COMBBLAS_HIP_NO_THP") != nullptr;
  constexpr uintptr_t kHuge = uintptr_t(2) << 20;
  if (off || bytes < 2 * kHuge) return;
  const uintptr_t b = (reinterpret_cast<uintptr_t>(p) + kHuge - 1) & ~(kHuge - 1);
  const uintptr_t e = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(kHuge - 1);
  if (e > b) (void)madvise(reinterpret_cast<void*>(b), e - b, MADV_HUGEPAGE);
}

// device DCSC -> SpTuples<IT,NT>* (column-sorted; ::operator new tuples, mtSpGEMM.h:272,453). The
// tuples are packed from the pinned chunks by the OpenMP threads, blocks of 4096 entries each
// finding their first column by one bisection of cp.
template <class IT, class NT>
combblas::SpTuples<IT, NT>* download_tuples(cbh_mat* C) {
  int64_t m, n, nnz, nzc;
  cbh_mat_info(C, &m, &n, &nnz, &nzc, nullptr);
  if (nnz == 0) return new combblas::SpTuples<IT, NT>(0, (IT)m, (IT)n);
  std::vector<int64_t> cp(nzc + 1), jc(nzc);
  auto* tuples = static_cast<std::tuple<IT, IT, NT>*>(::operator new(sizeof(std::tuple<IT, IT, NT>) * nnz));
  advise_huge(tuples, sizeof(std::tuple<IT, IT, NT>) * (size_t)nnz);
  struct Dst {
    std::tuple<IT, IT, NT>* t;
    const int64_t* cp;
    const int64_t* jc;
    int64_t nzc;
  } dst{tuples, cp.data(), jc.data(), nzc};
  cbh_take_fn take = [](void* u, int64_t f, int64_t cnt, const int32_t* ir, const void* num) -> int {
    const Dst* d = static_cast<const Dst*>(u);
    const NT* v = static_cast<const NT*>(num);
    const int64_t nb = (cnt + 4095) / 4096;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nb; ++b) {
      const int64_t p0 = f + b * 4096, p1 = std::min(f + cnt, p0 + 4096);
      int64_t c = (int64_t)(std::upper_bound(d->cp, d->cp + d->nzc + 1, p0) - d->cp) - 1;
      for (int64_t p = p0; p < p1; ++p) {
        while (d->cp[c + 1] <= p) ++c;
        d->t[p] = std::make_tuple((IT)ir[p - f], (IT)d->jc[c], v[p - f]);
      }
    }
    return 0;
  };
  int rc = cbh_mat_download_chunks(context(), C, cp.data(), jc.data(), 0, take, &dst);
  if (rc != CBH_OK) die(context(), rc, "cbh_mat_download_chunks");
  return new combblas::SpTuples<IT, NT>(nnz, (IT)m, (IT)n, tuples, true, true);
}

// device DCSC -> a host SpDCCols<IT,NT> built directly (no SpTuples round trip): the Dcsc arrays
// are allocated by SpDCCols(nnz, m, n, nzc) (SpDCCols.cpp:55-62) and filled from the chunks.
template <class IT, class NT>
combblas::SpDCCols<IT, NT>* download_dcsc(const cbh_mat* C) {
  int64_t m, n, nnz, nzc;
  cbh_mat_info(C, &m, &n, &nnz, &nzc, nullptr);
  if (nnz == 0) return new combblas::SpDCCols<IT, NT>((IT)0, (IT)m, (IT)n, (IT)0);
  auto* S = new combblas::SpDCCols<IT, NT>((IT)nnz, (IT)m, (IT)n, (IT)nzc);
  combblas::Dcsc<IT, NT>* d = S->GetDCSC();
  std::vector<int64_t> cpv, jcv;
  int64_t *cp, *jc;
  if (std::is_same<IT, int64_t>::value) {
    cp = reinterpret_cast<int64_t*>(d->cp);
    jc = reinterpret_cast<int64_t*>(d->jc);
  } else {
    cpv.resize(nzc + 1);
    jcv.resize(nzc);
    cp = cpv.data();
    jc = jcv.data();
  }
  struct Dst {
    IT* ir;
    NT* num;
  } dst{d->ir, d->numx};
  cbh_take_fn take = [](void* u, int64_t f, int64_t cnt, const int32_t* ir, const void* num) -> int {
    const Dst* t = static_cast<const Dst*>(u);
    const NT* v = static_cast<const NT*>(num);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < cnt; ++i) {
      t->ir[f + i] = (IT)ir[i];
      t->num[f + i] = v[i];
    }
    return 0;
  };
  advise_huge(d->ir, sizeof(IT) * (size_t)nnz);  // first-touch faults of the fresh arrays (take callback)
  advise_huge(d->numx, sizeof(NT) * (size_t)nnz);
  int rc = cbh_mat_download_chunks(context(), C, cp, jc, 0, take, &dst);
  if (rc != CBH_OK) die(context(), rc, "cbh_mat_download_chunks");
  if (!std::is_same<IT, int64_t>::value) {
    std::copy(cpv.begin(), cpv.end(), d->cp);
    std::copy(jcv.begin(), jcv.end(), d->jc);
  }
  return S;
}

// MultiwayMerge of any number of device partials (MultiwayMerge.h:411-526 takes any count): one
// cbh_merge per group of at most kMaxLists (16) lists, the group results merged again until one
// is left; every input and intermediate is freed. Takes ownership of `parts` (non-empty).
inline cbh_mat* merge_all(cbh_semiring sr, std::vector<cbh_mat*> parts) {
  constexpr size_t kGroup = 16;  // cbh_merge's list limit (kMaxLists)
  while (parts.size() > 1) {
    std::vector<cbh_mat*> next;
    for (size_t g = 0; g < parts.size(); g += kGroup) {
      const size_t k = std::min(kGroup, parts.size() - g);
      if (k == 1) {
        next.push_back(parts[g]);
        continue;
      }
      cbh_mat* C = nullptr;
      int rc = cbh_merge(context(), sr, (int)k, parts.data() + g, &C);
      if (rc != CBH_OK) die(context(), rc, "cbh_merge");
      for (size_t i = g; i < g + k; ++i) cbh_mat_free(context(), parts[i]);
      next.push_back(C);
    }
    parts.swap(next);
  }
  return parts[0];
}

// COMBBLAS_HIP_ORDER=reference (read per call): the built-in semirings also fold every output in
// the reference's own order (cbh_spgemm's CBH_ORDER_* flags, device/order_kernel.h), so that
// floating-point sums are bit-identical to the stock kernel named by `branch` -- 0
// LocalHybridSpGEMM, 1 LocalSpGEMM (heap), 2 LocalSpGEMMHash (hash). Default: arrival order
// (exact for integer, bool, min and max; f64 sums within the Higham bound).
inline uint32_t order_flags(int branch) {
  const char* e = std::getenv("COMBBLAS_HIP_ORDER");
  if (!e || std::strcmp(e, "reference") != 0) return 0u;
  return branch == 1 ? CBH_ORDER_HEAP : (branch == 2 ? CBH_ORDER_HASH : CBH_ORDER_HYBRID);
}

template <class SR, class NTO, class IT, class NT1, class NT2>
combblas::SpTuples<IT, NTO>* LocalHybridSpGEMM(const combblas::SpDCCols<IT, NT1>& A,
                                               const combblas::SpDCCols<IT, NT2>& B, bool clearA, bool clearB,
                                               IT* aux = nullptr, int branch = 0) {
  static_assert(std::is_same<NT1, NTO>::value && std::is_same<NT2, NTO>::value,
                "device path: input and output value types must match (T1 == T2 == T_promote)");
  (void)aux;
  const IT mdim = A.getnrow(), ndim = B.getncol();
  combblas::SpTuples<IT, NTO>* out;
  if (A.isZero() || B.isZero()) {
    out = new combblas::SpTuples<IT, NTO>(0, mdim, ndim);  // mtSpGEMM.h:224-227
  } else {
    MatGuard a, b, c;
    a.m = upload(A);
    b.m = upload(B);
    int rc = cbh_spgemm(context(), semiring_traits<SR>::code, a.m, b.m, CBH_SORTED_ROWS | order_flags(branch), &c.m);
    if (rc != CBH_OK) die(context(), rc, "cbh_spgemm");
    out = download_tuples<IT, NTO>(c.m);
  }
  if (clearA) delete const_cast<combblas::SpDCCols<IT, NT1>*>(&A);
  if (clearB) delete const_cast<combblas::SpDCCols<IT, NT2>*>(&B);
  return out;
}

template <class SR, class NTO, class IT, class NT1, class NT2>
combblas::SpTuples<IT, NTO>* LocalSpGEMMHash(const combblas::SpDCCols<IT, NT1>& A,
                                             const combblas::SpDCCols<IT, NT2>& B, bool clearA, bool clearB,
                                             bool sort = true) {
  (void)sort;  // ascending rows are a valid order for the unsorted contract
  return combblas_hip::LocalHybridSpGEMM<SR, NTO>(A, B, clearA, clearB, (IT*)nullptr, 2);
}

template <class SR, class NTO, class IT, class NT1, class NT2>
combblas::SpTuples<IT, NTO>* LocalSpGEMM(const combblas::SpDCCols<IT, NT1>& A, const combblas::SpDCCols<IT, NT2>& B,
                                         bool clearA, bool clearB) {
  return combblas_hip::LocalHybridSpGEMM<SR, NTO>(A, B, clearA, clearB, (IT*)nullptr, 1);
}

template <class SR, class IT, class NT>
combblas::SpTuples<IT, NT>* MultiwayMerge(std::vector<combblas::SpTuples<IT, NT>*>& lists, IT mdim = 0, IT ndim = 0,
                                          bool delarrs = false, bool unsorted_rows = false) {
  const int nlists = (int)lists.size();
  if (nlists == 0) return new combblas::SpTuples<IT, NT>(0, mdim, ndim);
  if (nlists == 1) {
    if (delarrs) return lists[0];  // MultiwayMerge.h:422-425 steals the input
    // MultiwayMerge.h:426-438: a copy of the one list, no dimension check (pure data movement;
    // ::operator new storage, filled in parallel, no value-initialisation pass)
    const int64_t nnz = lists[0]->getnnz();
    auto* t = static_cast<std::tuple<IT, IT, NT>*>(::operator new(sizeof(std::tuple<IT, IT, NT>) * (nnz > 0 ? nnz : 1)));
    const std::tuple<IT, IT, NT>* src = lists[0]->tuples;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nnz; ++i) t[i] = src[i];
    return new combblas::SpTuples<IT, NT>(nnz, mdim, ndim, t, false, true);
  }
  for (int i = 0; i < nlists; ++i)
    if (mdim != lists[i]->getnrow() || ndim != lists[i]->getncol()) {
      std::fprintf(stderr, "Dimensions of SpTuples do not match on multiwayMerge()\n");
      return new combblas::SpTuples<IT, NT>(0, 0, 0);
    }
  std::vector<MatGuard> g(nlists);
  std::vector<const cbh_mat*> parts(nlists);
  for (int i = 0; i < nlists; ++i) parts[i] = g[i].m = upload(*lists[i], unsorted_rows);
  // cbh_merge takes at most 16 lists: merge in groups of 16, then the group results, and so on
  std::vector<cbh_mat*> cur;
  if (nlists > 16)
    for (int i = 0; i < nlists; ++i) {  // the hierarchy owns (and frees) the uploaded lists
      cur.push_back(g[i].m);
      g[i].m = nullptr;
    }
  MatGuard c;
  if (cur.empty()) {
    int rc = cbh_merge(context(), semiring_traits<SR>::code, nlists, parts.data(), &c.m);
    if (rc != CBH_OK) die(context(), rc, "cbh_merge");
  } else {
    while (cur.size() > 1) {
      std::vector<cbh_mat*> next;
      for (size_t g0 = 0; g0 < cur.size(); g0 += 16) {
        const size_t k = std::min<size_t>(16, cur.size() - g0);
        if (k == 1) {
          next.push_back(cur[g0]);
          continue;
        }
        cbh_mat* r = nullptr;
        int rc = cbh_merge(context(), semiring_traits<SR>::code, (int)k, cur.data() + g0, &r);
        if (rc != CBH_OK) die(context(), rc, "cbh_merge");
        for (size_t i = g0; i < g0 + k; ++i) cbh_mat_free(context(), cur[i]);
        next.push_back(r);
      }
      cur.swap(next);
    }
    c.m = cur[0];
  }
  combblas::SpTuples<IT, NT>* out = download_tuples<IT, NT>(c.m);
  if (delarrs)
    for (auto* l : lists) delete l;
  return out;
}

// MultiwayMergeHash (MultiwayMerge.h:536-684): same contract; inputs may have unsorted rows inside
// a column, the output has rows ascending (a valid order for sorted=false as well)
template <class SR, class IT, class NT>
combblas::SpTuples<IT, NT>* MultiwayMergeHash(std::vector<combblas::SpTuples<IT, NT>*>& lists, IT mdim = 0,
                                              IT ndim = 0, bool delarrs = false, bool sorted = true) {
  (void)sorted;
  return combblas_hip::MultiwayMerge<SR, IT, NT>(lists, mdim, ndim, delarrs, true);
}

// Mult_AnXBn_Synch (ParFriends.h:1004-1108) for SpParMats over the stock SpDCCols with a built-in
// semiring: the reference's SUMMA stage loop and host MPI broadcasts of the stage blocks
// (SpParHelper::GetSetSizes / BCastMatrix, unchanged), every stage block uploaded through the
// pinned chunks and multiplied on the device, the stage partials merged on the device
// (MultiwayMerge), and C downloaded straight into the result's Dcsc arrays -- no SpTuples, no
// host merge copy and no serial SpDCCols(SpTuples) conversion (SpDCCols.cpp:109-183).
// clearA / clearB leave A / B with an empty block (the reference deletes it and sets NULL).
template <class SR, class IU, class NU>
combblas::SpParMat<IU, NU, combblas::SpDCCols<IU, NU>> mult_synch_host(
    combblas::SpParMat<IU, NU, combblas::SpDCCols<IU, NU>>& A, combblas::SpParMat<IU, NU, combblas::SpDCCols<IU, NU>>& B,
    bool clearA, bool clearB) {
  typedef combblas::SpDCCols<IU, NU> DER;
  if (!combblas::CheckSpGEMMCompliance(A, B)) return combblas::SpParMat<IU, NU, DER>();
  AdaptorTimes& T = adaptor_times();
  const AdaptorTimes before = T;
  int stages, dummy;
  std::shared_ptr<combblas::CommGrid> GridC =
      ProductGrid(A.getcommgrid().get(), B.getcommgrid().get(), stages, dummy, dummy);
  const IU C_m = A.seq().getnrow(), C_n = B.seq().getncol();
  IU** ARecvSizes = combblas::SpHelper::allocate2D<IU>(DER::esscount, stages);
  IU** BRecvSizes = combblas::SpHelper::allocate2D<IU>(DER::esscount, stages);
  combblas::SpParHelper::GetSetSizes(A.seq(), ARecvSizes, A.getcommgrid()->GetRowWorld());
  combblas::SpParHelper::GetSetSizes(B.seq(), BRecvSizes, B.getcommgrid()->GetColWorld());
  const int Aself = A.getcommgrid()->GetRankInProcRow();
  const int Bself = B.getcommgrid()->GetRankInProcCol();
  std::vector<cbh_mat*> parts;
  for (int i = 0; i < stages; ++i) {
    std::vector<IU> ess;
    DER* ARecv = &A.seq();
    if (i != Aself) {
      for (int j = 0; j < DER::esscount; ++j) ess.push_back(ARecvSizes[j][i]);
      ARecv = new DER();
    }
    combblas::SpParHelper::BCastMatrix(GridC->GetRowWorld(), *ARecv, ess, i);
    ess.clear();
    DER* BRecv = &B.seq();
    if (i != Bself) {
      for (int j = 0; j < DER::esscount; ++j) ess.push_back(BRecvSizes[j][i]);
      BRecv = new DER();
    }
    combblas::SpParHelper::BCastMatrix(GridC->GetColWorld(), *BRecv, ess, i);
    if (!ARecv->isZero() && !BRecv->isZero()) {
      const double t0 = now_s();
      MatGuard a, b;
      a.m = upload(*ARecv);
      b.m = upload(*BRecv);
      const double t1 = now_s();
      cbh_mat* Ci = nullptr;
      int rc = cbh_spgemm(context(), semiring_traits<SR>::code, a.m, b.m, CBH_SORTED_ROWS | order_flags(0), &Ci);
      if (rc != CBH_OK) die(context(), rc, "cbh_spgemm");
      T.upload += t1 - t0;
      T.kernel += now_s() - t1;
      int64_t nnz = 0;
      cbh_mat_info(Ci, nullptr, nullptr, &nnz, nullptr, nullptr);
      if (nnz > 0) parts.push_back(Ci);  // `if(!C_cont->isZero()) tomerge.push_back`
      else cbh_mat_free(context(), Ci);
    }
    if (i != Aself) delete ARecv;  // the reference's clearA / clearB = i != self
    if (i != Bself) delete BRecv;
  }
  combblas::SpHelper::deallocate2D(ARecvSizes, DER::esscount);
  combblas::SpHelper::deallocate2D(BRecvSizes, DER::esscount);
  if (clearA) A.seq() = DER();
  if (clearB) B.seq() = DER();
  const double t2 = now_s();
  DER* C;
  if (parts.empty()) {
    C = new DER((IU)0, C_m, C_n, (IU)0);
  } else {
    cbh_mat* Cd = parts.size() == 1 ? parts[0] : merge_all(semiring_traits<SR>::code, parts);
    const double t3 = now_s();
    T.merge += t3 - t2;
    C = download_dcsc<IU, NU>(Cd);
    cbh_mat_free(context(), Cd);
    T.download += now_s() - t3;
  }
  T.calls += 1;
  if (timing_enabled())
    std::fprintf(stderr, "[combblas_hip] Mult_AnXBn_Synch: upload %.1f ms, kernel %.1f ms, merge %.1f ms, download %.1f ms\n",
                 1e3 * (T.upload - before.upload), 1e3 * (T.kernel - before.kernel), 1e3 * (T.merge - before.merge),
                 1e3 * (T.download - before.download));
  return combblas::SpParMat<IU, NU, DER>(C, GridC);
}

}  // namespace combblas_hip

// Route the reference's own drivers to the device path for (SR, IT, NT): explicit
// specializations of the combblas:: function templates, forwarding to combblas_hip::.
#define COMBBLAS_HIP_INSTANTIATE(SR, IT, NT)                                                                  \
  namespace combblas {                                                                                        \
  template <>                                                                                                 \
  inline SpTuples<IT, NT>* LocalHybridSpGEMM<SR, NT, IT, NT, NT>(const SpDCCols<IT, NT>& A,                  \
                                                                 const SpDCCols<IT, NT>& B, bool clearA,      \
                                                                 bool clearB, IT* aux) {                      \
    return combblas_hip::LocalHybridSpGEMM<SR, NT>(A, B, clearA, clearB, aux);                               \
  }                                                                                                           \
  template <>                                                                                                 \
  inline SpTuples<IT, NT>* LocalSpGEMMHash<SR, NT, IT, NT, NT>(const SpDCCols<IT, NT>& A,                    \
                                                               const SpDCCols<IT, NT>& B, bool clearA,        \
                                                               bool clearB, bool sort) {                      \
    return combblas_hip::LocalSpGEMMHash<SR, NT>(A, B, clearA, clearB, sort);                                \
  }                                                                                                           \
  template <>                                                                                                 \
  inline SpTuples<IT, NT>* LocalSpGEMM<SR, NT, IT, NT, NT>(const SpDCCols<IT, NT>& A, const SpDCCols<IT, NT>& B, \
                                                           bool clearA, bool clearB) {                        \
    return combblas_hip::LocalSpGEMM<SR, NT>(A, B, clearA, clearB);                                          \
  }                                                                                                           \
  template <>                                                                                                 \
  inline SpTuples<IT, NT>* MultiwayMerge<SR, IT, NT>(std::vector<SpTuples<IT, NT>*> & L, IT mdim, IT ndim,    \
                                                     bool delarrs) {                                          \
    return combblas_hip::MultiwayMerge<SR, IT, NT>(L, mdim, ndim, delarrs);                                  \
  }                                                                                                           \
  template <>                                                                                                 \
  inline SpTuples<IT, NT>* MultiwayMergeHash<SR, IT, NT>(std::vector<SpTuples<IT, NT>*> & L, IT mdim, IT ndim, \
                                                         bool delarrs, bool sorted) {                         \
    return combblas_hip::MultiwayMergeHash<SR, IT, NT>(L, mdim, ndim, delarrs, sorted);                      \
  }                                                                                                           \
  template <>                                                                                                 \
  inline SpParMat<IT, NT, SpDCCols<IT, NT>>                                                                   \
  Mult_AnXBn_Synch<SR, NT, SpDCCols<IT, NT>, IT, NT, NT, SpDCCols<IT, NT>, SpDCCols<IT, NT>>(                 \
      SpParMat<IT, NT, SpDCCols<IT, NT>> & A, SpParMat<IT, NT, SpDCCols<IT, NT>> & B, bool clearA, bool clearB) { \
    return combblas_hip::mult_synch_host<SR, IT, NT>(A, B, clearA, clearB);                                  \
  }                                                                                                           \
  }
