// Drop-in integration test (built by `make -C oracle ref` into oracle/_ref/dropin_harness; it
// compiles the reference's headers, so its binary lives with the other reference builds). This
// translation unit is built with g++, as the reference is; the device kernels of the
// test-defined semirings are instantiated in dropin_kernels.hip (hipcc).
//
// The reference's UNCHANGED Mult_AnXBn_Synch (ParFriends.h:1004-1108) runs twice per case on the
// same R-MAT input: once for a semiring routed to the gfx950 kernels, once for a value-identical
// semiring that is not specialized (the stock OpenMP LocalHybridSpGEMM). The two DCSC results
// must match exactly (structure, row order and values).
//   built-in semirings (COMBBLAS_HIP_INSTANTIATE, library kernels through the C-ABI):
//     PlusTimesSRing<double,double>, SelectMaxSRing<int64_t,int64_t>
//   header-instantiated (COMBBLAS_HIP_INSTANTIATE_DEVICE, HipSpGEMMDevice.h):
//     KTipsDev    -- test-defined bool OR-AND with the KTipsSR contract (KTipsTest.cpp:12-20)
//     MinMaxSR    -- test-defined semiring over a two-field struct, int64 inputs (NT != NTO, as
//                    SegTest.cpp:165-171's KmerIntersect<int64_t, CommonKmers>)
//     PlusTimesSRing<double,int64_t> -- promotion NT1 != NT2 -> T_promote = double
//     Select2ndSRing<int64,int64,int64> -- non-commutative add (reference order, order_kernel.h)
//     PTOrdDev    -- f64 PlusTimes marked reference_order: non-dyadic sums bit-exact
//     AffineDev   -- an UNMARKED non-commutative f64 semiring: reference order by default
//   PlusTimesSRing<double,double> again with COMBBLAS_HIP_ORDER=reference on non-dyadic values
//     (library kernels + the reference-order pass, cbh_spgemm CBH_ORDER_HYBRID)
//   dropin_harness <scale>      -> prints "DROPIN <case> OK nnz=..." lines, exit 0 on success
#include <mpi.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "CombBLAS/CombBLAS.h"
#include "combblas_hip/HipSpGEMMDevice.h"

using namespace combblas;

double cblas_alltoalltime, cblas_allgathertime, cblas_mergeconttime, cblas_transvectime, cblas_localspmvtime;
MTRand GlobalMT(123);

#include "dropin_semirings.h"

// the value-identical stock semirings of the built-in cases
template <class T>
struct CpuPlusTimes {
  static T id() { return 0; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_SUM; }
  static T add(const T& a, const T& b) { return a + b; }
  static T multiply(const T& a, const T& b) { return a * b; }
  static void axpy(T a, const T& x, T& y) { y += a * x; }
};
template <class T>
struct CpuSelectMax {
  static T id() { return -1; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_MAX; }
  static T add(const T& a, const T& b) { return std::max(a, b); }
  static T multiply(const T& a, const T& b) { return a * b; }
  static void axpy(T a, const T& x, T& y) { y = std::max(y, a * x); }
};
struct CpuPlusTimesDI {  // PlusTimesSRing<double,int64_t> on the stock path
  static double id() { return 0; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_SUM; }
  static double add(const double& a, const double& b) { return a + b; }
  static double multiply(const double& a, const int64_t& b) { return a * static_cast<double>(b); }
  static void axpy(double a, const int64_t& x, double& y) { y += a * x; }
};

typedef PlusTimesSRing<double, double> PTDD;
typedef SelectMaxSRing<int64_t, int64_t> SMLL;
typedef PlusTimesSRing<double, int64_t> PTDI;
COMBBLAS_HIP_INSTANTIATE(PTDD, int64_t, double)
COMBBLAS_HIP_INSTANTIATE(SMLL, int64_t, int64_t)
COMBBLAS_HIP_INSTANTIATE_DEVICE(KTipsDev, int64_t, bool, bool, bool)
COMBBLAS_HIP_INSTANTIATE_DEVICE(MinMaxDev, int64_t, int64_t, int64_t, MinMax)
COMBBLAS_HIP_INSTANTIATE_DEVICE(PTDI, int64_t, double, int64_t, double)
typedef Select2ndSRing<int64_t, int64_t, int64_t> S2LL;
COMBBLAS_HIP_INSTANTIATE_DEVICE(S2LL, int64_t, int64_t, int64_t, int64_t)
COMBBLAS_HIP_INSTANTIATE_DEVICE(PTOrdDev, int64_t, double, double, double)
COMBBLAS_HIP_INSTANTIATE_DEVICE(AffineDev, int64_t, double, double, double)

template <class NT>
static bool same(const SpDCCols<int64_t, NT>& x, const SpDCCols<int64_t, NT>& y) {
  if (x.getnnz() != y.getnnz() || x.getnrow() != y.getnrow() || x.getncol() != y.getncol()) return false;
  if (x.getnnz() == 0) return true;
  Dcsc<int64_t, NT>* a = x.GetDCSC();
  Dcsc<int64_t, NT>* b = y.GetDCSC();
  if (a->nzc != b->nzc) return false;
  for (int64_t i = 0; i < a->nzc; ++i)
    if (a->jc[i] != b->jc[i] || a->cp[i + 1] != b->cp[i + 1]) return false;
  for (int64_t i = 0; i < a->nz; ++i)
    if (a->ir[i] != b->ir[i] || !(a->numx[i] == b->numx[i])) return false;
  return true;
}

// value = f(row, col, value) on the local block (1 rank: local ids are global), as TC.cpp:72-87 edits L
template <class NT, class F>
static void set_values(SpParMat<int64_t, NT, SpDCCols<int64_t, NT>>& M, F f) {
  for (auto colit = M.seq().begcol(); colit != M.seq().endcol(); ++colit)
    for (auto nzit = M.seq().begnz(colit); nzit != M.seq().endnz(colit); ++nzit)
      nzit.value() = f(nzit.rowid(), colit.colid(), nzit.value());
}

template <class NTO, class SRH, class SRC, class NA, class NB>
static int run_case(const char* name, SpParMat<int64_t, NA, SpDCCols<int64_t, NA>>& A,
                    SpParMat<int64_t, NB, SpDCCols<int64_t, NB>>& B) {
  typedef SpDCCols<int64_t, NTO> DER;
  std::fprintf(stderr, "case %s: device\n", name);
  double t0 = MPI_Wtime();
  SpParMat<int64_t, NTO, DER> Ch = Mult_AnXBn_Synch<SRH, NTO, DER>(A, B);  // device path
  double t1 = MPI_Wtime();
  std::fprintf(stderr, "case %s: stock\n", name);
  SpParMat<int64_t, NTO, DER> Cc = Mult_AnXBn_Synch<SRC, NTO, DER>(A, B);  // stock reference path
  double t2 = MPI_Wtime();
  bool ok = same(Ch.seq(), Cc.seq());
  std::printf("DROPIN %s %s nnz=%lld hip_s=%.3f cpu_s=%.3f\n", name, ok ? "OK" : "MISMATCH", (long long)Ch.getnnz(),
              t1 - t0, t2 - t1);
  std::fflush(stdout);
  return ok ? 0 : 1;
}

// C1 line (bench_c1.py): PSpGEMM<PlusTimesSRing<double,double>> -- the reference's MultTest.cpp:161-181
// plumbing, Mult_AnXBn_Synch on SpParMat<int64_t, double, SpDCCols> -- on the device path
// (COMBBLAS_HIP_INSTANTIATE) and on the stock OpenMP path, first call and the median of `reps`
// warm calls each, the device calls split into the adaptor's stages. Prints one BENCHC1 JSON line.
static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : (v.size() % 2 ? v[v.size() / 2] : 0.5 * (v[v.size() / 2 - 1] + v[v.size() / 2]));
}
static int bench_c1(int scale, int reps) {
  double init[4] = {.57, .19, .19, .05};
  DistEdgeList<int64_t>* DEL = new DistEdgeList<int64_t>();
  DEL->GenGraph500Data(init, scale, 16, true, true);
  SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>> G(*DEL, false);
  delete DEL;
  typedef SpDCCols<int64_t, double> DER;
  SpParMat<int64_t, double, DER> A(G), B(G);
  combblas_hip::AdaptorTimes& T = combblas_hip::adaptor_times();
  double t0 = MPI_Wtime();
  SpParMat<int64_t, double, DER> C = Mult_AnXBn_Synch<PTDD, double, DER>(A, B);
  const double first = MPI_Wtime() - t0;
  std::vector<double> dev, up, ker, mer, down, cpu;
  // every timed call initialises a fresh SpParMat (SpParMat's operator= deep-copies the block,
  // SpParMat.cpp:725-738); its destruction stays outside the timed region
  for (int r = 0; r < reps; ++r) {
    const combblas_hip::AdaptorTimes b = T;
    t0 = MPI_Wtime();
    {
      SpParMat<int64_t, double, DER> Cr = Mult_AnXBn_Synch<PTDD, double, DER>(A, B);
      dev.push_back(MPI_Wtime() - t0);
    }
    up.push_back(T.upload - b.upload);
    ker.push_back(T.kernel - b.kernel);
    mer.push_back(T.merge - b.merge);
    down.push_back(T.download - b.download);
  }
  t0 = MPI_Wtime();
  SpParMat<int64_t, double, DER> Cc = Mult_AnXBn_Synch<CpuPlusTimes<double>, double, DER>(A, B);
  const double cpu_first = MPI_Wtime() - t0;
  for (int r = 0; r < reps; ++r) {
    t0 = MPI_Wtime();
    SpParMat<int64_t, double, DER> Cr = Mult_AnXBn_Synch<CpuPlusTimes<double>, double, DER>(A, B);
    cpu.push_back(MPI_Wtime() - t0);
  }
  const bool ok = same(C.seq(), Cc.seq());
  // flops = sum_k nnz(A(:,k)) * nnz(B(k,:)) on the one rank (EstimateFLOP)
  std::vector<int64_t> rowcnt(A.seq().getnrow(), 0);
  Dcsc<int64_t, double>* da = A.seq().GetDCSC();
  for (int64_t i = 0; i < da->nz; ++i) rowcnt[da->ir[i]]++;
  int64_t flops = 0;
  for (int64_t c = 0; c < da->nzc; ++c) flops += (da->cp[c + 1] - da->cp[c]) * rowcnt[da->jc[c]];
  const char* omp = std::getenv("OMP_NUM_THREADS");
  std::printf("BENCHC1 {\"scale\": %d, \"nnzA\": %lld, \"nnzC\": %lld, \"flops\": %lld, \"match\": %s, \"reps\": %d, "
              "\"first_s\": %.6f, \"warm_s\": %.6f, \"upload_s\": %.6f, \"kernel_s\": %.6f, \"merge_s\": %.6f, "
              "\"download_s\": %.6f, \"cpu_first_s\": %.6f, \"cpu_s\": %.6f, \"cpu_threads\": %s}\n",
              scale, (long long)A.getnnz(), (long long)C.getnnz(), (long long)flops, ok ? "true" : "false", reps, first,
              median(dev), median(up), median(ker), median(mer), median(down), cpu_first, median(cpu), omp ? omp : "0");
  std::fflush(stdout);
  return ok ? 0 : 1;
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  if (argc > 1 && std::string(argv[1]) == "bench") {
    int rc = 0;
    {
      rc = bench_c1(argc > 2 ? std::atoi(argv[2]) : 16, argc > 3 ? std::atoi(argv[3]) : 5);
    }
    MPI_Finalize();
    return rc;
  }
  int scale = argc > 1 ? std::atoi(argv[1]) : 12;
  int bad = 0;
  {  // every CombBLAS object must be destroyed before MPI_Finalize
    double init[4] = {.57, .19, .19, .05};
    DistEdgeList<int64_t>* DEL = new DistEdgeList<int64_t>();
    DEL->GenGraph500Data(init, scale, 16, true, true);
    typedef SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>> PMatI;
    PMatI G(*DEL, false);
    delete DEL;
    SpParMat<int64_t, double, SpDCCols<int64_t, double>> Ad(G), Bd(G);
    bad += run_case<double, PTDD, CpuPlusTimes<double>>("PSpGEMM<PlusTimes<double>>", Ad, Bd);
    PMatI Ai(G), Bi(G);
    bad += run_case<int64_t, SMLL, CpuSelectMax<int64_t>>("PSpGEMM<SelectMax<int64>>", Ai, Bi);
    SpParMat<int64_t, bool, SpDCCols<int64_t, bool>> Ab(G), Bb(G);
    bad += run_case<bool, KTipsDev, KTipsCpu>("PSpGEMM<user KTipsSR bool>", Ab, Bb);
    // values that differ per entry (multiplicities alone make most products equal)
    PMatI Av(G), Bv(G);
    set_values(Av, [](int64_t r, int64_t c, int64_t x) { return x * ((r * 7919 + c * 31) % 23 - 11); });
    set_values(Bv, [](int64_t r, int64_t c, int64_t x) { return x * ((r * 104729 + c * 17) % 19 - 9); });
    bad += run_case<MinMax, MinMaxDev, MinMaxCpu>("PSpGEMM<user struct MinMax, int64 -> struct>", Av, Bv);
    bad += run_case<double, PTDI, CpuPlusTimesDI>("PSpGEMM<PlusTimes<double,int64> promotion>", Ad, Bi);
    // non-commutative add: Select2nd keeps the first product of the hash branch, the last popped of
    // the heap branch (mtSpGEMM.h:341, :408)
    bad += run_case<int64_t, S2LL, Select2ndCpu>("PSpGEMM<Select2nd<int64> reference order>", Av, Bv);
    // non-dyadic f64 sums in the reference's order
    SpParMat<int64_t, double, SpDCCols<int64_t, double>> Af(G), Bf(G);
    set_values(Af, [](int64_t r, int64_t c, double x) { return x * (0.1 + 1e-3 * ((r * 7919 + c * 31) % 97)); });
    set_values(Bf, [](int64_t r, int64_t c, double x) { return x * (0.3 - 1e-3 * ((r * 104729 + c * 17) % 89)); });
    bad += run_case<double, PTOrdDev, PTOrdCpu>("PSpGEMM<PlusTimes<double> reference order, non-dyadic>", Af, Bf);
    // an unmarked non-commutative, non-associative user semiring: reference order by default
    bad += run_case<double, AffineDev, AffineCpu>("PSpGEMM<unmarked user affine f64, default reference order>", Af, Bf);
    // the built-in f64 PlusTimes through the library kernels with COMBBLAS_HIP_ORDER=reference
    setenv("COMBBLAS_HIP_ORDER", "reference", 1);
    bad += run_case<double, PTDD, CpuPlusTimes<double>>("PSpGEMM<PlusTimes<double>> COMBBLAS_HIP_ORDER=reference, non-dyadic",
                                                          Af, Bf);
    unsetenv("COMBBLAS_HIP_ORDER");
  }
  MPI_Finalize();
  return bad ? 1 : 0;
}
