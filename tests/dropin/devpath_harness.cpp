// Device-resident SUMMA through the reference's API (include/combblas_hip/SpParMatDev.h): the
// operands are SpParMat<IT, NT, SpDCColsDev<IT, NT>>, the reference's own PSpGEMM<SR>
// (SpParMat.h:454-467) dispatches to the device-resident Mult_AnXBn_Synch overload, and every
// block, stage partial and the product stay in HBM (RCCL broadcasts; COMBBLAS_HIP_COMM=mpi: host
// staged). Each rank's block of C is compared with the stock Mult_AnXBn_Synch on host blocks.
// Built by `make -C oracle ref` into oracle/_ref/devpath_harness (g++, as the reference).
//   [mpirun -np P] devpath_harness <scale> [reps]   -> "DEVPATH <case> OK ..." lines (rank 0)
#include <mpi.h>

#include <cstdio>
#include <cstdlib>

#include "CombBLAS/CombBLAS.h"
#include "combblas_hip/SpParMatDev.h"

using namespace combblas;

double cblas_alltoalltime, cblas_allgathertime, cblas_mergeconttime, cblas_transvectime, cblas_localspmvtime;
MTRand GlobalMT(123);

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

template <class NT, class SRD, class SRC>
static int run_case(const char* name, SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>>& G, int reps) {
  typedef SpDCCols<int64_t, NT> HD;
  typedef combblas_hip::SpDCColsDev<int64_t, NT> DD;
  SpParMat<int64_t, NT, HD> A(G), B(G);
  SpParMat<int64_t, NT, DD> Ad = combblas_hip::to_device(A), Bd = combblas_hip::to_device(B);
  SpParMat<int64_t, NT, DD> Cd = PSpGEMM<SRD>(Ad, Bd);  // warm-up (RCCL communicators, kernels)
  cbh_ctx_synchronize(combblas_hip::context());
  double best = 1e30;
  for (int r = 0; r < reps; ++r) {
    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = MPI_Wtime();
    Cd = PSpGEMM<SRD>(Ad, Bd);  // the reference's PSpGEMM -> device-resident Mult_AnXBn_Synch
    cbh_ctx_synchronize(combblas_hip::context());
    double dt = MPI_Wtime() - t0, mx = 0;
    MPI_Allreduce(&dt, &mx, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    best = std::min(best, mx);
  }
  SpParMat<int64_t, NT, HD> Ch = combblas_hip::to_host(Cd);
  double t1 = MPI_Wtime();
  SpParMat<int64_t, NT, HD> Cc = Mult_AnXBn_Synch<SRC, NT, HD>(A, B);  // stock reference path
  double cpu = MPI_Wtime() - t1;
  int ok = same(Ch.seq(), Cc.seq()) ? 1 : 0, all = 0;
  // the overlapped drivers on the device (ParFriends.h:1110-1235, :798-997): the same C
  SpParMat<int64_t, NT, DD> Co = Mult_AnXBn_Overlap<SRD, NT, DD>(Ad, Bd);
  SpParMat<int64_t, NT, HD> Coh = combblas_hip::to_host(Co);
  SpParMat<int64_t, NT, DD> Cb = Mult_AnXBn_DoubleBuff<SRD, NT, DD>(Ad, Bd);
  SpParMat<int64_t, NT, HD> Cbh = combblas_hip::to_host(Cb);
  const int ok_over = same(Coh.seq(), Cc.seq()) ? 1 : 0, ok_dbuf = same(Cbh.seq(), Cc.seq()) ? 1 : 0;
  int all_over = 0, all_dbuf = 0;
  MPI_Allreduce(&ok_over, &all_over, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
  MPI_Allreduce(&ok_dbuf, &all_dbuf, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
  MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
  int rank = 0, np = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &np);
  const int64_t nnz = Cc.getnnz();
  if (rank == 0) {
    std::printf("DEVPATH %s %s ranks=%d nnz=%lld hip_s=%.4f cpu_s=%.4f transport=%s\n", name, all ? "OK" : "MISMATCH",
                np, (long long)nnz, best, cpu, combblas_hip::use_mpi_transport() ? "mpi" : "rccl");
    std::printf("DEVPATH %s/Mult_AnXBn_Overlap %s ranks=%d\n", name, all_over ? "OK" : "MISMATCH", np);
    std::printf("DEVPATH %s/Mult_AnXBn_DoubleBuff %s ranks=%d\n", name, all_dbuf ? "OK" : "MISMATCH", np);
  }
  std::fflush(stdout);
  return (all && all_over && all_dbuf) ? 0 : 1;
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  const int scale = argc > 1 ? std::atoi(argv[1]) : 12;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
  int bad = 0;
  {
    double init[4] = {.57, .19, .19, .05};
    DistEdgeList<int64_t>* DEL = new DistEdgeList<int64_t>();
    DEL->GenGraph500Data(init, scale, 16, true, true);
    SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>> G(*DEL, false);
    delete DEL;
    bad += run_case<double, PlusTimesSRing<double, double>, CpuPlusTimes<double>>("PSpGEMM<PlusTimes<double>>", G, reps);
    bad += run_case<int64_t, SelectMaxSRing<int64_t, int64_t>, CpuSelectMax<int64_t>>("PSpGEMM<SelectMax<int64>>", G,
                                                                                       reps);
  }
  MPI_Finalize();
  return bad ? 1 : 0;
}
