// Drop-in integration test (built by `make -C oracle ref` into oracle/_ref/dropin_harness; it
// compiles the reference's headers, so its binary lives with the other reference builds).
//
// The reference's UNCHANGED Mult_AnXBn_Synch (ParFriends.h:1004-1108) is instantiated twice on the
// same R-MAT input: once for PlusTimesSRing<double,double> / SelectMaxSRing<int64_t,int64_t>,
// which COMBBLAS_HIP_INSTANTIATE routes to the gfx950 kernels through the C-ABI, and once for
// value-identical local semirings that are not specialized (stock OpenMP LocalHybridSpGEMM).
// The two DCSC results must match exactly (structure, row order and values).
//   dropin_harness <scale>      -> prints "DROPIN <case> OK nnz=..." lines, exit 0 on success
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <memory>

#include "CombBLAS/CombBLAS.h"
#include "combblas_hip/HipSpGEMM.h"

using namespace combblas;

double cblas_alltoalltime, cblas_allgathertime, cblas_mergeconttime, cblas_transvectime, cblas_localspmvtime;
MTRand GlobalMT(123);

typedef PlusTimesSRing<double, double> PTDD;
typedef SelectMaxSRing<int64_t, int64_t> SMLL;
COMBBLAS_HIP_INSTANTIATE(PTDD, int64_t, double)
COMBBLAS_HIP_INSTANTIATE(SMLL, int64_t, int64_t)

// value-identical semirings that stay on the stock CPU path
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

template <class NT, class SRH, class SRC>
static int run_case(const char* name, SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>>& G) {
  typedef SpDCCols<int64_t, NT> DER;
  SpParMat<int64_t, NT, DER> A(G);
  SpParMat<int64_t, NT, DER> B(G);
  double t0 = MPI_Wtime();
  SpParMat<int64_t, NT, DER> Ch = Mult_AnXBn_Synch<SRH, NT, DER>(A, B);  // device path
  double t1 = MPI_Wtime();
  SpParMat<int64_t, NT, DER> Cc = Mult_AnXBn_Synch<SRC, NT, DER>(A, B);  // stock reference path
  double t2 = MPI_Wtime();
  bool ok = same(Ch.seq(), Cc.seq());
  std::printf("DROPIN %s %s nnz=%lld hip_s=%.3f cpu_s=%.3f\n", name, ok ? "OK" : "MISMATCH", (long long)Ch.getnnz(),
              t1 - t0, t2 - t1);
  return ok ? 0 : 1;
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int scale = argc > 1 ? std::atoi(argv[1]) : 12;
  int bad = 0;
  {  // every CombBLAS object must be destroyed before MPI_Finalize
    double init[4] = {.57, .19, .19, .05};
    DistEdgeList<int64_t>* DEL = new DistEdgeList<int64_t>();
    DEL->GenGraph500Data(init, scale, 16, true, true);
    SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>> G(*DEL, false);
    delete DEL;
    bad += run_case<double, PlusTimesSRing<double, double>, CpuPlusTimes<double>>("PSpGEMM<PlusTimes<double>>", G);
    bad += run_case<int64_t, SelectMaxSRing<int64_t, int64_t>, CpuSelectMax<int64_t>>("PSpGEMM<SelectMax<int64>>", G);
  }
  MPI_Finalize();
  return bad ? 1 : 0;
}
