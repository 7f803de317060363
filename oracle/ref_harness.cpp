// TEST INFRASTRUCTURE ONLY. Built by oracle/Makefile against the reference sources
// under $(COMBBLAS_REF) (default /root/reference) into oracle/_ref/ref_harness.
// Nothing in the product library links or calls this.
//
// It drives the reference's own code so that the CPU restatement (oracle/spgemm_oracle.cpp)
// and the HIP path can be pinned against it:
//   gen   <scale> <ef> <out.cbm>                      DistEdgeList::GenGraph500Data(packed) +
//                                                     SpParMat(DEL, removeloops=false)  (TC.cpp:139-148)
//   mult  <sr> <kernel> <A.cbm> <B.cbm> <out.cbm>     LocalHybridSpGEMM / LocalSpGEMMHash / LocalSpGEMM
//                                                     (mtSpGEMM.h:74,213,463)
//   merge <sr> <out.cbm> <in1.cbm> ...                MultiwayMerge (MultiwayMerge.h:411)
//   synch <sr> <A.cbm> <B.cbm> <out.cbm|-> [reps]     Mult_AnXBn_Synch on a 1x1 grid (ParFriends.h:1004),
//                                                     prints wall time per call (MPI_Wtime)
//   slice <scale> <ef> <col0> <col1> <reps> <sr> [stride]
//                                                     CPU baseline: A (scale, ef) times the columns
//                                                     c0 <= c < c1, (c-c0) % stride == 0 of A, with
//                                                     Mult_AnXBn_Synch on any square rank count; JSON
//   digest <scale> <ef> <block> <sr>                 digest + value sum of the whole C = A*A by column
//                                                     blocks of B (LocalHybridSpGEMM), one JSON line per block
//   tc    <scale> <L.cbm> <C.cbm> [reps]              Applications/TC.cpp:62-121 on one rank (C = (L*L).*L);
//                                                     reps: warm-up + median of reps timed passes
//   mcl   <A.cbm> <out.cbm> <hard> <select> <recover> <pct>
//                                                     MCLPruneRecoverySelect (ParFriends.h:185-353)
//   galerkin <A.cbm> <R.cbm> <stride> <reps>          CPU baseline of C3: GalerkinNew.cpp:99-106's
//                                                     S = R', AT = PSpGEMM(A, R_s), SAT = PSpGEMM(S, AT)
//                                                     with R_s = R's columns c % stride == 0; JSON
//   mclexp <A.cbm> <stride> <reps> <hard> <select> <recover> <pct>
//                                                     CPU baseline of C5: MCL.cpp:574-577's expansion
//                                                     MemEfficientSpGEMM(A, A_s) with the prune, A_s =
//                                                     A's columns c % stride == 0; JSON
// sr: pt_f64 | pt_i64 | max_i64 | min_i64 | bool ; kernel: hybrid | hash | hashu | heap
#include <mpi.h>
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "CombBLAS/CombBLAS.h"
#include "cbm_io.h"

using namespace combblas;

// Globals some reference translation units expect to be defined by the application.
double cblas_alltoalltime, cblas_allgathertime, cblas_mergeconttime, cblas_transvectime, cblas_localspmvtime;
MTRand GlobalMT(123);

// Boolean OR-AND semiring with the same contract as the test-defined KTipsSR
// (ReleaseTests/KTipsTest.cpp:12-20).
template <class T>
struct OrAndSRing {
  static T id() { return static_cast<T>(0); }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_LOR; }
  static T add(const T& a, const T& b) { return (a || b); }
  static T multiply(const T& a, const T& b) { return (a && b); }
  static void axpy(T a, const T& x, T& y) { y = add(y, multiply(a, x)); }
};

template <class NT>
static NT value_of(const cbm::Dcsc& d, int64_t i) {
  return d.vtype == cbm::F64 ? static_cast<NT>(d.vf[i]) : static_cast<NT>(d.vi[i]);
}

template <class NT>
static uint32_t vtype_of() {
  if (std::is_same<NT, double>::value) return cbm::F64;
  if (std::is_same<NT, bool>::value) return cbm::U8;
  return cbm::I64;
}

template <class NT>
static SpDCCols<int64_t, NT>* to_spdccols(const cbm::Dcsc& d) {
  if (d.nnz() == 0) return new SpDCCols<int64_t, NT>(0, d.m, d.n, 0);
  auto* s = new SpDCCols<int64_t, NT>(d.nnz(), d.m, d.n, d.nzc());
  Dcsc<int64_t, NT>* dc = s->GetDCSC();
  for (int64_t i = 0; i < d.nzc(); ++i) dc->jc[i] = d.jc[i];
  for (int64_t i = 0; i <= d.nzc(); ++i) dc->cp[i] = d.cp[i];
  for (int64_t i = 0; i < d.nnz(); ++i) {
    dc->ir[i] = d.ir[i];
    dc->numx[i] = value_of<NT>(d, i);
  }
  return s;
}

template <class NT>
static cbm::Dcsc from_spdccols(const SpDCCols<int64_t, NT>& s) {
  cbm::Dcsc d;
  d.vtype = vtype_of<NT>();
  d.m = s.getnrow();
  d.n = s.getncol();
  if (s.getnnz() == 0) {
    d.cp.push_back(0);
    return d;
  }
  Dcsc<int64_t, NT>* dc = s.GetDCSC();
  d.jc.assign(dc->jc, dc->jc + dc->nzc);
  d.cp.assign(dc->cp, dc->cp + dc->nzc + 1);
  d.ir.resize(dc->nz);
  for (int64_t i = 0; i < dc->nz; ++i) d.ir[i] = (int32_t)dc->ir[i];
  if (d.vtype == cbm::F64) {
    d.vf.resize(dc->nz);
    for (int64_t i = 0; i < dc->nz; ++i) d.vf[i] = (double)dc->numx[i];
  } else {
    d.vi.resize(dc->nz);
    for (int64_t i = 0; i < dc->nz; ++i) d.vi[i] = (int64_t)dc->numx[i];
  }
  return d;
}

template <class NT>
static cbm::Dcsc from_sptuples(SpTuples<int64_t, NT>* t) {
  // Column-sorted tuples -> DCSC in the tuples' own order (SpDCCols.cpp:109-183).
  SpDCCols<int64_t, NT> s(*t, false);
  return from_spdccols<NT>(s);
}

static double now() { return MPI_Wtime(); }

template <class SR, class NT>
static int do_mult(const std::string& kernel, const std::string& fa, const std::string& fb, const std::string& fo) {
  cbm::Dcsc a = cbm::read(fa), b = cbm::read(fb);
  SpDCCols<int64_t, NT>* A = to_spdccols<NT>(a);
  SpDCCols<int64_t, NT>* B = to_spdccols<NT>(b);
  SpTuples<int64_t, NT>* C = nullptr;
  double t0 = now();
  if (kernel == "hybrid")
    C = LocalHybridSpGEMM<SR, NT>(*A, *B, false, false);
  else if (kernel == "hash")
    C = LocalSpGEMMHash<SR, NT>(*A, *B, false, false, true);
  else if (kernel == "hashu")
    C = LocalSpGEMMHash<SR, NT>(*A, *B, false, false, false);
  else if (kernel == "heap")
    C = LocalSpGEMM<SR, NT>(*A, *B, false, false);
  else {
    std::fprintf(stderr, "unknown kernel %s\n", kernel.c_str());
    return 2;
  }
  double t1 = now();
  std::fprintf(stderr, "kernel=%s nnzC=%lld time=%.6f\n", kernel.c_str(), (long long)C->getnnz(), t1 - t0);
  cbm::write(fo, from_sptuples<NT>(C));
  delete C;
  delete A;
  delete B;
  return 0;
}

template <class SR, class NT>
static int do_merge(const std::string& fo, const std::vector<std::string>& ins) {
  std::vector<SpTuples<int64_t, NT>*> lists;
  int64_t m = 0, n = 0;
  for (auto& f : ins) {
    cbm::Dcsc d = cbm::read(f);
    m = d.m;
    n = d.n;
    SpDCCols<int64_t, NT>* s = to_spdccols<NT>(d);
    lists.push_back(new SpTuples<int64_t, NT>(*s));
    delete s;
  }
  SpTuples<int64_t, NT>* C = MultiwayMerge<SR>(lists, m, n, true);
  cbm::write(fo, from_sptuples<NT>(C));
  if (lists.size() != 1) delete C;
  return 0;
}

template <class SR, class NT>
static int do_synch(const std::string& fa, const std::string& fb, const std::string& fo, int reps) {
  typedef SpDCCols<int64_t, NT> DER;
  std::shared_ptr<CommGrid> grid(new CommGrid(MPI_COMM_WORLD, 0, 0));
  cbm::Dcsc a = cbm::read(fa), b = cbm::read(fb);
  SpParMat<int64_t, NT, DER> A(to_spdccols<NT>(a), grid);
  SpParMat<int64_t, NT, DER> B(to_spdccols<NT>(b), grid);
  SpParMat<int64_t, NT, DER> C = Mult_AnXBn_Synch<SR, NT, DER>(A, B);  // warm-up
  for (int r = 0; r < reps; ++r) {
    double t0 = now();
    C = Mult_AnXBn_Synch<SR, NT, DER>(A, B);
    double t1 = now();
    std::printf("synch_time %.6f\n", t1 - t0);
  }
  if (fo != "-") cbm::write(fo, from_spdccols<NT>(C.seq()));
  return 0;
}

static SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>>* gen_rmat(int scale, int ef) {
  double init[4] = {.57, .19, .19, .05};
  DistEdgeList<int64_t>* DEL = new DistEdgeList<int64_t>();
  DEL->GenGraph500Data(init, scale, ef, true, true);
  auto* A = new SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>>(*DEL, false);
  delete DEL;
  return A;
}

static int do_gen(int scale, int ef, const std::string& fo) {
  auto* A = gen_rmat(scale, ef);
  cbm::write(fo, from_spdccols<int64_t>(A->seq()));
  delete A;
  return 0;
}

// CPU baseline on a bounded column block of the north-star workload: C = A * A(:, c0:c1).
template <class SR, class NT>
static int do_slice(int scale, int ef, int64_t c0, int64_t c1, int reps, int64_t stride) {
  // Any square number of MPI ranks p (mpirun -np p): the generator distributes A over the
  // sqrt(p) x sqrt(p) grid exactly as TC.cpp does, B = A(:, c0:c1) via SpParMat::PruneI on global
  // column ids (all n columns kept, as a ColSplit piece), one untimed warm-up call, then `reps`
  // timed Mult_AnXBn_Synch calls (barrier + MPI_Wtime, max over ranks); prints the median.
  typedef SpDCCols<int64_t, NT> DER;
  int rank = 0, nprocs = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
  double tg0 = now();
  auto* G = gen_rmat(scale, ef);
  double tg1 = now();
  typedef SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>> GMat;
  GMat GB(*G);
  GB.PruneI([c0, c1, stride](const std::tuple<int64_t, int64_t, int64_t>& t) {
    const int64_t c = std::get<1>(t);
    return c < c0 || c >= c1 || (c - c0) % stride != 0;
  });
  // flops = sum_k nnz(A(:,k)) * nnz(B(k,:)) (EstimateFLOP's count; the reference's EstimateFLOP
  // faults on ranks whose B block is empty, so the same sum is formed from two Reduce()s)
  int64_t flops = 0;
  {
    auto one = [](int64_t) { return (int64_t)1; };
    FullyDistVec<int64_t, int64_t> ca = G->Reduce(Column, std::plus<int64_t>(), (int64_t)0, one);
    FullyDistVec<int64_t, int64_t> rb = GB.Reduce(Row, std::plus<int64_t>(), (int64_t)0, one);
    int64_t loc = 0;
    for (int64_t i = 0; i < ca.LocArrSize(); ++i) loc += ca.GetLocArr()[i] * rb.GetLocArr()[i];
    MPI_Allreduce(&loc, &flops, 1, MPI_INT64_T, MPI_SUM, MPI_COMM_WORLD);
  }
  SpParMat<int64_t, NT, DER> A(*G);
  SpParMat<int64_t, NT, DER> B(GB);
  delete G;
  std::vector<double> ts;
  int64_t nnzc = 0;
  for (int r = -1; r < reps; ++r) {  // r = -1: warm-up
    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = now();
    SpParMat<int64_t, NT, DER> C = Mult_AnXBn_Synch<SR, NT, DER>(A, B);
    double t1 = now(), dt = t1 - t0, mx = 0;
    MPI_Allreduce(&dt, &mx, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    if (r >= 0) ts.push_back(mx);
    nnzc = C.getnnz();
  }
  std::sort(ts.begin(), ts.end());
  double med = ts[ts.size() / 2];
  int nthreads = 1;
#ifdef THREADED
#pragma omp parallel
  {
#pragma omp master
    nthreads = omp_get_num_threads();
  }
#endif
  if (rank == 0)
    std::printf("{\"flops\": %lld, \"nnzC\": %lld, \"median_s\": %.6f, \"min_s\": %.6f, \"max_s\": %.6f, "
                "\"reps\": %d, \"warmup\": 1, \"gflops\": %.6f, \"ranks\": %d, \"threads\": %d, \"gen_s\": %.3f, "
                "\"col0\": %lld, \"col1\": %lld, \"stride\": %lld}\n",
                (long long)flops, (long long)nnzc, med, ts.front(), ts.back(), reps, 2.0 * flops / med / 1e9, nprocs,
                nthreads, tg1 - tg0, (long long)c0, (long long)c1, (long long)stride);
  return 0;
}

// Digest of the WHOLE product C = A*A (R-MAT scale, ef) computed by the reference's own
// LocalHybridSpGEMM (mtSpGEMM.h:212-460) one column block of B at a time (B = A(:, c0:c1), all n
// columns kept, as a ColSplit piece), so that the output never has to be held at once (scale 22:
// 24.8 G entries). Entries are visited in C order (columns ascending, rows as the kernel emits
// them) with a running global index, so the sum over blocks is the same order-sensitive digest
// as tests/helpers.py digest() / the device checksum_kernel over the whole C. Prints one JSON line
// per block and a final total.
static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
template <class NT>
static uint64_t bits_of(NT v) {
  if (std::is_same<NT, double>::value) {
    uint64_t b;
    std::memcpy(&b, &v, 8);
    return b;
  }
  return (uint64_t)(int64_t)v;
}
template <class SR, class NT>
static int do_digest(int scale, int ef, int64_t block) {
  auto* G = gen_rmat(scale, ef);
  cbm::Dcsc a = from_spdccols<int64_t>(G->seq());
  delete G;
  SpDCCols<int64_t, NT>* A = to_spdccols<NT>(a);
  // column sums and row sums of A for the closed form sum(C) = sum_k colsum_k(A) * rowsum_k(A)
  uint64_t gidx = 0, dig = 0;
  long double vsum_exact = 0;
  for (int64_t c0 = 0; c0 < a.n; c0 += block) {
    const int64_t c1 = std::min<int64_t>(a.n, c0 + block);
    cbm::Dcsc b;
    b.vtype = a.vtype;
    b.m = a.m;
    b.n = a.n;
    b.cp.push_back(0);
    for (int64_t i = 0; i < a.nzc(); ++i) {
      if (a.jc[i] < c0 || a.jc[i] >= c1) continue;
      b.jc.push_back(a.jc[i]);
      for (int64_t p = a.cp[i]; p < a.cp[i + 1]; ++p) {
        b.ir.push_back(a.ir[p]);
        b.vi.push_back(a.vi[p]);
      }
      b.cp.push_back((int64_t)b.ir.size());
    }
    SpDCCols<int64_t, NT>* B = to_spdccols<NT>(b);
    double t0 = now();
    SpTuples<int64_t, NT>* C = LocalHybridSpGEMM<SR, NT>(*A, *B, false, false);
    double t1 = now();
    const int64_t nnz = C->getnnz();
    uint64_t bd = 0;
    double bs = 0;
    for (int64_t i = 0; i < nnz; ++i) {
      const NT v = C->numvalue(i);
      const uint64_t p = gidx + (uint64_t)i;
      bd += mix64(p ^ mix64((uint64_t)C->colindex(i) ^ mix64((uint64_t)(uint32_t)C->rowindex(i) ^ mix64(bits_of<NT>(v)))));
      bs += (double)v;
    }
    std::printf("{\"block\": [%lld, %lld], \"gbase\": %llu, \"nnz\": %lld, \"sum\": %.1f, \"digest\": \"%llu\", "
                "\"kernel_s\": %.3f}\n",
                (long long)c0, (long long)c1, (unsigned long long)gidx, (long long)nnz, bs, (unsigned long long)bd,
                t1 - t0);
    std::fflush(stdout);
    gidx += (uint64_t)nnz;
    dig += bd;
    vsum_exact += bs;
    delete C;
    delete B;
  }
  std::printf("{\"total\": true, \"nnz\": %llu, \"sum\": %.1f, \"digest\": \"%llu\"}\n", (unsigned long long)gidx,
              (double)vsum_exact, (unsigned long long)dig);
  delete A;
  return 0;
}

// Applications/TC.cpp:62-121 on one rank (global = local indices): symmetrise, set values to 1,
// L = tril with the upper entries kept as explicit zeros, C = (L*L) .* L, triangles = sum(C).
// Writes L and C, prints the triangle count.
static int do_tc(int scale, const std::string& fl, const std::string& fc, int reps) {
  typedef SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>> Mat;
  Mat* A = gen_rmat(scale, 16);
  A->RemoveLoops();
  Mat AT = *A;
  AT.Transpose();
  *A += AT;
  A->Apply([](int64_t) { return (int64_t)1; });
  Mat L = *A;
  for (auto colit = L.seq().begcol(); colit != L.seq().endcol(); ++colit)
    for (auto nzit = L.seq().begnz(colit); nzit != L.seq().endnz(colit); ++nzit)
      if (nzit.rowid() < colit.colid()) nzit.value() = 0;
  Mat Lt = L;
  // TC.cpp:108-115 timed: the product, the mask and the reduction (the CPU baseline of bench_tc.py);
  // reps > 0: one untimed warm-up pass, then the median of `reps` timed passes
  auto pass = [&](Mat& C, int64_t& result) {
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    C = Mult_AnXBn_Synch<PlusTimesSRing<int64_t, int64_t>, int64_t, SpDCCols<int64_t, int64_t>>(L, Lt);
    C.EWiseMult(L, false);
    FullyDistVec<int64_t, int64_t> tri = C.Reduce(Column, std::plus<int64_t>(), static_cast<int64_t>(0));
    result = tri.Reduce(std::plus<int64_t>(), static_cast<int64_t>(0));
    MPI_Barrier(MPI_COMM_WORLD);
    return MPI_Wtime() - t0;
  };
  Mat C;
  int64_t result = 0;
  std::vector<double> ts;
  if (reps > 0) pass(C, result);
  for (int r = 0; r < (reps > 0 ? reps : 1); ++r) {
    Mat Cr;
    ts.push_back(pass(Cr, result));
    if (r == 0) C = Cr;
  }
  std::sort(ts.begin(), ts.end());
  const double tc_s = ts[ts.size() / 2];
  if (!fl.empty() && fl != "-") cbm::write(fl, from_spdccols<int64_t>(L.seq()));
  if (!fc.empty() && fc != "-") cbm::write(fc, from_spdccols<int64_t>(C.seq()));
  std::printf("{\"triangles\": %lld, \"nnzL\": %lld, \"nnzC\": %lld, \"tc_s\": %.6f, \"reps\": %d, \"threads\": %d}\n",
              (long long)result, (long long)L.getnnz(), (long long)C.getnnz(), tc_s, (int)ts.size(),
              omp_get_max_threads());
  delete A;
  return 0;
}

// HipMCL post-expansion step (ParFriends.h:185-353, kselectVersion 1) on one rank: reads the
// expanded matrix (f64), writes it after MCLPruneRecoverySelect.
static int do_mcl(const std::string& fa, const std::string& fo, double hard, int64_t sel, int64_t rec, double pct) {
  typedef SpDCCols<int64_t, double> DER;
  std::shared_ptr<CommGrid> grid(new CommGrid(MPI_COMM_WORLD, 0, 0));
  cbm::Dcsc a = cbm::read(fa);
  SpParMat<int64_t, double, DER> A(to_spdccols<double>(a), grid);
  MCLPruneRecoverySelect(A, hard, sel, rec, pct, 1);
  cbm::write(fo, from_spdccols<double>(A.seq()));
  std::printf("{\"nnz\": %lld}\n", (long long)A.getnnz());
  return 0;
}

// keeps the columns c % stride == 0 of d (all n columns kept, as a ColSplit piece)
static cbm::Dcsc column_sample(const cbm::Dcsc& d, int64_t stride) {
  cbm::Dcsc o;
  o.vtype = d.vtype;
  o.m = d.m;
  o.n = d.n;
  o.cp.push_back(0);
  for (int64_t i = 0; i < d.nzc(); ++i) {
    if (d.jc[i] % stride != 0) continue;
    o.jc.push_back(d.jc[i]);
    for (int64_t p = d.cp[i]; p < d.cp[i + 1]; ++p) {
      o.ir.push_back(d.ir[p]);
      if (d.vtype == cbm::F64) o.vf.push_back(d.vf[p]);
      else o.vi.push_back(d.vi[p]);
    }
    o.cp.push_back((int64_t)o.ir.size());
  }
  return o;
}

// semiring multiplies of X*Y on one rank: sum over Y's entries (k, j) of nnz(X(:, k))
template <class NT>
static int64_t local_flops(const SpDCCols<int64_t, NT>& X, const SpDCCols<int64_t, NT>& Y) {
  if (X.getnnz() == 0 || Y.getnnz() == 0) return 0;
  std::vector<int64_t> cn(X.getncol(), 0);
  const Dcsc<int64_t, NT>* dx = X.GetDCSC();
  for (int64_t i = 0; i < dx->nzc; ++i) cn[dx->jc[i]] = dx->cp[i + 1] - dx->cp[i];
  const Dcsc<int64_t, NT>* dy = Y.GetDCSC();
  int64_t f = 0;
  for (int64_t p = 0; p < dy->nz; ++p) f += cn[dy->ir[p]];
  return f;
}

static int nthreads_of() {
  int nthreads = 1;
#ifdef THREADED
#pragma omp parallel
  {
#pragma omp master
    nthreads = omp_get_num_threads();
  }
#endif
  return nthreads;
}

// GalerkinNew.cpp:99-106 on one rank: S = T' (Transpose), AT = PSpGEMM<PTDD>(A, T), SAT =
// PSpGEMM<PTDD>(S, AT), on the column sample T_s of T (SAT(:, J) = S * (A * T(:, J)) exactly).
// One untimed warm-up, then `reps` timed pairs of products; prints the median.
static int do_galerkin(const std::string& fa, const std::string& fr, int64_t stride, int reps) {
  typedef PlusTimesSRing<double, double> PTDD;
  typedef SpDCCols<int64_t, double> DER;
  typedef SpParMat<int64_t, double, DER> Mat;
  std::shared_ptr<CommGrid> grid(new CommGrid(MPI_COMM_WORLD, 0, 0));
  cbm::Dcsc a = cbm::read(fa), r = cbm::read(fr);
  Mat A(to_spdccols<double>(a), grid);
  Mat T(to_spdccols<double>(r), grid);
  Mat Ts(to_spdccols<double>(column_sample(r, stride)), grid);
  Mat S = T;
  S.Transpose();
  std::vector<double> ts;
  int64_t f1 = 0, f2 = 0, nnz_at = 0, nnz_sat = 0;
  double vsum = 0;
  for (int it = -1; it < reps; ++it) {
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = now();
    Mat AT = PSpGEMM<PTDD>(A, Ts);
    Mat SAT = PSpGEMM<PTDD>(S, AT);
    MPI_Barrier(MPI_COMM_WORLD);
    const double dt = now() - t0;
    if (it >= 0) ts.push_back(dt);
    f1 = local_flops<double>(A.seq(), Ts.seq());
    f2 = local_flops<double>(S.seq(), AT.seq());
    nnz_at = AT.getnnz();
    nnz_sat = SAT.getnnz();
    vsum = 0;
    if (SAT.seq().getnnz()) {
      const Dcsc<int64_t, double>* d = SAT.seq().GetDCSC();
      for (int64_t p = 0; p < d->nz; ++p) vsum += d->numx[p];
    }
  }
  std::sort(ts.begin(), ts.end());
  const double med = ts[ts.size() / 2];
  std::printf("{\"flops\": %lld, \"flops_AR\": %lld, \"flops_RtAR\": %lld, \"nnzAT\": %lld, \"nnzSAT\": %lld, "
              "\"value_sum\": %.17g, \"median_s\": %.6f, \"min_s\": %.6f, \"reps\": %d, \"gflops\": %.6f, "
              "\"threads\": %d, \"stride\": %lld, \"cols\": %lld}\n",
              (long long)(f1 + f2), (long long)f1, (long long)f2, (long long)nnz_at, (long long)nnz_sat, vsum, med,
              ts.front(), reps, 2.0 * (f1 + f2) / med / 1e9, nthreads_of(), (long long)stride,
              (long long)Ts.seq().getnzc());
  return 0;
}

// MCL.cpp:574-577 (layers == 1) on one rank: the expansion MemEfficientSpGEMM<PTFF>(A, A_s, phases
// = 1, prunelimit, select, recover_num, recover_pct, kselectVersion 1, hash kernel) with its
// MCLPruneRecoverySelect, on the column sample A_s of the right operand.
static int do_mclexp(const std::string& fa, int64_t stride, int reps, double hard, int64_t sel, int64_t rec,
                     double pct) {
  typedef PlusTimesSRing<double, double> PTFF;
  typedef SpDCCols<int64_t, double> DER;
  typedef SpParMat<int64_t, double, DER> Mat;
  std::shared_ptr<CommGrid> grid(new CommGrid(MPI_COMM_WORLD, 0, 0));
  cbm::Dcsc a = cbm::read(fa);
  Mat A(to_spdccols<double>(a), grid);
  Mat B(to_spdccols<double>(column_sample(a, stride)), grid);
  const int64_t flops = local_flops<double>(A.seq(), B.seq());
  std::vector<double> ts;
  int64_t nnzc = 0;
  for (int it = -1; it < reps; ++it) {
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = now();
    Mat C = MemEfficientSpGEMM<PTFF, double, DER>(A, B, 1, hard, (int64_t)sel, (int64_t)rec, pct, 1, 1, (int64_t)0);
    MPI_Barrier(MPI_COMM_WORLD);
    const double dt = now() - t0;
    if (it >= 0) ts.push_back(dt);
    nnzc = C.getnnz();
  }
  std::sort(ts.begin(), ts.end());
  const double med = ts[ts.size() / 2];
  std::printf("{\"flops\": %lld, \"nnz_after_prune\": %lld, \"median_s\": %.6f, \"min_s\": %.6f, \"reps\": %d, "
              "\"gflops\": %.6f, \"threads\": %d, \"stride\": %lld, \"cols\": %lld}\n",
              (long long)flops, (long long)nnzc, med, ts.front(), reps, 2.0 * flops / med / 1e9, nthreads_of(),
              (long long)stride, (long long)B.seq().getnzc());
  return 0;
}

#define DISPATCH_SR(sr, CALL)                                                   \
  if (sr == "pt_f64") {                                                         \
    typedef PlusTimesSRing<double, double> SR;                                  \
    typedef double NT;                                                          \
    return CALL;                                                                \
  } else if (sr == "pt_i64") {                                                  \
    typedef PlusTimesSRing<int64_t, int64_t> SR;                                \
    typedef int64_t NT;                                                         \
    return CALL;                                                                \
  } else if (sr == "max_i64") {                                                 \
    typedef SelectMaxSRing<int64_t, int64_t> SR;                                \
    typedef int64_t NT;                                                         \
    return CALL;                                                                \
  } else if (sr == "min_i64") {                                                 \
    typedef MinPlusSRing<int64_t, int64_t> SR;                                  \
    typedef int64_t NT;                                                         \
    return CALL;                                                                \
  } else if (sr == "bool") {                                                    \
    typedef OrAndSRing<bool> SR;                                                \
    typedef bool NT;                                                            \
    return CALL;                                                                \
  }

static int run(int argc, char** argv) {
  if (argc < 2) return 2;
  std::string mode = argv[1];
  if (mode == "gen" && argc == 5) return do_gen(std::atoi(argv[2]), std::atoi(argv[3]), argv[4]);
  if (mode == "mult" && argc == 7) {
    std::string sr = argv[2];
    DISPATCH_SR(sr, (do_mult<SR, NT>(argv[3], argv[4], argv[5], argv[6])));
  }
  if (mode == "merge" && argc >= 5) {
    std::string sr = argv[2];
    std::vector<std::string> ins(argv + 4, argv + argc);
    DISPATCH_SR(sr, (do_merge<SR, NT>(argv[3], ins)));
  }
  if (mode == "synch" && argc >= 6) {
    std::string sr = argv[2];
    int reps = argc > 6 ? std::atoi(argv[6]) : 1;
    DISPATCH_SR(sr, (do_synch<SR, NT>(argv[3], argv[4], argv[5], reps)));
  }
  if (mode == "slice" && (argc == 8 || argc == 9)) {
    std::string sr = argv[7];
    const int64_t stride = argc == 9 ? std::max<int64_t>(1, std::atoll(argv[8])) : 1;
    DISPATCH_SR(sr, (do_slice<SR, NT>(std::atoi(argv[2]), std::atoi(argv[3]), std::atoll(argv[4]),
                                      std::atoll(argv[5]), std::atoi(argv[6]), stride)));
  }
  if (mode == "digest" && argc == 6) {
    std::string sr = argv[5];
    DISPATCH_SR(sr, (do_digest<SR, NT>(std::atoi(argv[2]), std::atoi(argv[3]), std::atoll(argv[4]))));
  }
  if (mode == "tc" && (argc == 5 || argc == 6))
    return do_tc(std::atoi(argv[2]), argv[3], argv[4], argc == 6 ? std::atoi(argv[5]) : 0);
  if (mode == "mcl" && argc == 8)
    return do_mcl(argv[2], argv[3], std::atof(argv[4]), std::atoll(argv[5]), std::atoll(argv[6]), std::atof(argv[7]));
  if (mode == "galerkin" && argc == 6) return do_galerkin(argv[2], argv[3], std::atoll(argv[4]), std::atoi(argv[5]));
  if (mode == "mclexp" && argc == 9)
    return do_mclexp(argv[2], std::atoll(argv[3]), std::atoi(argv[4]), std::atof(argv[5]), std::atoll(argv[6]),
                     std::atoll(argv[7]), std::atof(argv[8]));
  std::fprintf(stderr, "bad arguments\n");
  return 2;
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rc = run(argc, argv);
  MPI_Finalize();
  return rc;
}
