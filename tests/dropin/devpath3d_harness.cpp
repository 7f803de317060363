// Device-resident PHASED and 3D drivers behind the reference's own API
// (include/combblas_hip/ParFriendsDev.h): operands are SpParMat / SpParMat3D over SpDCColsDev, the
// reference's driver names -- MemEfficientSpGEMM (ParFriends.h:449-730, with
// MCLPruneRecoverySelect :185-353 per phase), Mult_AnXBn_SUMMA3D (:2918-3208) and
// MemEfficientSpGEMM3D (:3214-3705) -- resolve to the device overloads (stage broadcasts, fiber
// reduce-scatter and processor-column reductions over RCCL; COMBBLAS_HIP_COMM=mpi: host staged),
// and every rank's block is compared, column by column as sorted sets, with the STOCK drivers on
// host blocks (the OpenMP kernels; a value-identical, unspecialized semiring). R-MAT edge
// multiplicities make every double sum exact. Built by `make -C oracle ref` (g++, as the reference).
//   [mpirun -np P] devpath3d_harness <scale> <layers>  -> "DEVPATH3D <case> OK ..." lines (rank 0)
#include <mpi.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <tuple>
#include <utility>
#include <vector>

#include "CombBLAS/CombBLAS.h"
#include "combblas_hip/ParFriendsDev.h"

using namespace combblas;

double cblas_alltoalltime, cblas_allgathertime, cblas_mergeconttime, cblas_transvectime, cblas_localspmvtime;
double mcl_Abcasttime, mcl_Bbcasttime, mcl_localspgemmtime, mcl_multiwaymergetime, mcl_kselecttime,
    mcl_prunecolumntime, mcl_symbolictime, mcl3d_conversiontime, mcl3d_symbolictime, mcl3d_Abcasttime,
    mcl3d_Bbcasttime, mcl3d_SUMMAtime, mcl3d_localspgemmtime, mcl3d_SUMMAmergetime, mcl3d_reductiontime,
    mcl3d_3dmergetime, mcl3d_kselecttime, mcl3d_totaltime, mcl3d_floptime, mcl3d_proc_flop_mean, mcl3d_proc_flop_std,
    mcl3d_proc_nnzc_pre_red, mcl3d_proc_nnzc_post_red;
int64_t mcl_memory, mcl3d_layer_flop, mcl3d_layer_nnzc, mcl3d_nnzc, mcl3d_flop, mcl3d_max_proc_flop,
    mcl3d_max_proc_nnzc_pre_red, mcl3d_max_proc_nnzc_post_red;
MTRand GlobalMT(123);

struct CpuPlusTimes {  // PlusTimesSRing<double,double> on the stock path
  static double id() { return 0; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_SUM; }
  static double add(const double& a, const double& b) { return a + b; }
  static double multiply(const double& a, const double& b) { return a * b; }
  static void axpy(double a, const double& x, double& y) { y += a * x; }
};
typedef PlusTimesSRing<double, double> PTDD;

typedef SpDCCols<int64_t, double> DCols;
typedef SpParMat<int64_t, double, DCols> PMat;
typedef SpParMat3D<int64_t, double, DCols> PMat3D;

// the local block's columns as sorted (row, value) sets
static std::vector<std::pair<int64_t, std::vector<std::pair<int64_t, double>>>> columns(DCols& M) {
  std::vector<std::pair<int64_t, std::vector<std::pair<int64_t, double>>>> out;
  for (auto colit = M.begcol(); colit != M.endcol(); ++colit) {
    std::vector<std::pair<int64_t, double>> col;
    for (auto nzit = M.begnz(colit); nzit != M.endnz(colit); ++nzit) col.emplace_back(nzit.rowid(), nzit.value());
    std::sort(col.begin(), col.end());
    if (!col.empty()) out.emplace_back(colit.colid(), std::move(col));
  }
  return out;
}

static int report(const char* name, PMat& Ch, PMat& Cc, double hip_s, double cpu_s) {
  int myrank, nprocs;
  MPI_Comm_rank(MPI_COMM_WORLD, &myrank);
  MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
  int bad = (columns(Ch.seq()) == columns(Cc.seq())) ? 0 : 1;
  if (Ch.getnrow() != Cc.getnrow() || Ch.getncol() != Cc.getncol()) bad = 1;
  int anybad = 0;
  MPI_Allreduce(&bad, &anybad, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
  const int64_t nnz = Ch.getnnz(), nnzc = Cc.getnnz();  // collective
  if (nnz != nnzc) anybad = 1;
  if (myrank == 0) {
    std::printf("DEVPATH3D %s %s nnz=%lld ranks=%d hip_s=%.3f cpu_s=%.3f transport=%s\n", name, anybad ? "MISMATCH" : "OK",
                (long long)nnz, nprocs, hip_s, cpu_s,
                combblas_hip::use_mpi_transport() ? "mpi" : "rccl");
    std::fflush(stdout);
  }
  return anybad;
}

// 3D results compared block by block (both runs distribute C the same way): Convert2D builds a
// square 2D grid of the world, which 2 and 8 ranks do not have
static int report3d(const char* name, PMat3D& Ch, PMat3D& Cc, double hip_s, double cpu_s) {
  int myrank, nprocs;
  MPI_Comm_rank(MPI_COMM_WORLD, &myrank);
  MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
  int bad = (columns(*Ch.seqptr()) == columns(*Cc.seqptr())) ? 0 : 1;
  if (Ch.seqptr()->getnrow() != Cc.seqptr()->getnrow() || Ch.seqptr()->getncol() != Cc.seqptr()->getncol()) bad = 1;
  int64_t loc[2] = {Ch.seqptr()->getnnz(), Cc.seqptr()->getnnz()}, tot[2] = {0, 0};
  MPI_Allreduce(loc, tot, 2, MPI_INT64_T, MPI_SUM, MPI_COMM_WORLD);
  int anybad = 0;
  MPI_Allreduce(&bad, &anybad, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
  if (tot[0] != tot[1]) anybad = 1;
  if (myrank == 0) {
    std::printf("DEVPATH3D %s %s nnz=%lld ranks=%d hip_s=%.3f cpu_s=%.3f transport=%s\n", name, anybad ? "MISMATCH" : "OK",
                (long long)tot[0], nprocs, hip_s, cpu_s,
                combblas_hip::use_mpi_transport() ? "mpi" : "rccl");
    std::fflush(stdout);
  }
  return anybad;
}

static bool is_square(int p) {
  const int r = (int)std::lround(std::sqrt((double)p));
  return r * r == p;
}

// The R-MAT input on a gr x gc grid of MPI_COMM_WORLD. DistEdgeList and SpParMat(DEL) need a square
// world (CommGrid.cpp:45-52 aborts otherwise), so for 2 or 8 ranks every rank generates the whole
// matrix on MPI_COMM_SELF and keeps its block (SpParMat::Owner's split: m/gr rows per block, the
// last one taking the remainder; local ids) -- the 3D drivers then redistribute it by tuples
// (SpParMat3D's non-special constructor takes any 2D grid shape).
static PMat make_input(int scale, int gr, int gc) {
  double init[4] = {.57, .19, .19, .05};
  if (gr == gc) {
    DistEdgeList<int64_t>* DEL = new DistEdgeList<int64_t>();
    DEL->GenGraph500Data(init, scale, 16, true, true);
    SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>> G(*DEL, false);
    delete DEL;
    return PMat(G);
  }
  MPI_Comm self = MPI_COMM_SELF;
  DistEdgeList<int64_t>* DEL = new DistEdgeList<int64_t>(self);
  DEL->GenGraph500Data(init, scale, 16, true, true);
  SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>> G(*DEL, false);
  delete DEL;
  int myrank;
  MPI_Comm_rank(MPI_COMM_WORLD, &myrank);
  const int64_t m = G.getnrow(), n = G.getncol();
  const int pr = myrank / gc, pc = myrank % gc;
  const int64_t rper = m / gr, cper = n / gc;
  const int64_t r0 = pr * rper, r1 = pr == gr - 1 ? m : r0 + rper;
  const int64_t c0 = pc * cper, c1 = pc == gc - 1 ? n : c0 + cper;
  std::vector<std::tuple<int64_t, int64_t, double>> t;
  auto& S = G.seq();
  for (auto colit = S.begcol(); colit != S.endcol(); ++colit) {
    const int64_t c = colit.colid();
    if (c < c0 || c >= c1) continue;
    for (auto nzit = S.begnz(colit); nzit != S.endnz(colit); ++nzit)
      if (nzit.rowid() >= r0 && nzit.rowid() < r1)
        t.emplace_back(nzit.rowid() - r0, c - c0, (double)nzit.value());
  }
  auto* owned = new std::tuple<int64_t, int64_t, double>[t.size()];  // SpTuples delete[]s its array
  std::copy(t.begin(), t.end(), owned);
  SpTuples<int64_t, double> tup((int64_t)t.size(), r1 - r0, c1 - c0, owned, true);
  std::shared_ptr<CommGrid> grid(new CommGrid(MPI_COMM_WORLD, gr, gc));
  return PMat(new DCols(tup, false), grid);
}

typedef combblas_hip::SpDCColsDev<int64_t, double> DDev;
typedef SpParMat<int64_t, double, DDev> DMat;
typedef SpParMat3D<int64_t, double, DDev> DMat3D;

int main(int argc, char** argv) {
  int provided;
  MPI_Init_thread(&argc, &argv, MPI_THREAD_SERIALIZED, &provided);
  const int scale = argc > 1 ? std::atoi(argv[1]) : 10;
  const int layers = argc > 2 ? std::atoi(argv[2]) : 0;
  int nprocs;
  MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
  int bad = 0;
  {  // every CombBLAS object must be destroyed before MPI_Finalize
    int gr = (int)std::lround(std::sqrt((double)nprocs)), gc = gr;
    if (gr * gc != nprocs) {  // 2 -> 1 x 2, 8 -> 2 x 4
      gr = (int)std::lround(std::sqrt((double)(nprocs / 2)));
      gc = nprocs / gr;
    }
    PMat A = make_input(scale, gr, gc), B = make_input(scale, gr, gc);
    const double hard = 1.5, pct = 0.9;
    const int64_t sel = 40, rec = 60;
    if (is_square(nprocs)) {
      DMat Ad = combblas_hip::to_device(A), Bd = combblas_hip::to_device(B);
      PMat Cc = MemEfficientSpGEMM<CpuPlusTimes, double, DCols>(A, B, 1, hard, sel, rec, pct, 1, 1, 0);
      // 1 and 3 phases; the memory model (EstPerProcessNnzSUMMA on the device) with a budget
      // small enough to force several phases: the pruned product is the same in every case
      const int64_t mem_cases[3][2] = {{1, 0}, {3, 0}, {1, 1}};
      for (const auto& mc : mem_cases) {
        char name[96];
        std::snprintf(name, sizeof(name), "MemEfficientSpGEMM<phases=%lld,perProcessMemory=%lld,prune>",
                      (long long)mc[0], (long long)mc[1]);
        // perProcessMemory in GB: 1 GB leaves phases to the model at these sizes
        double t0 = MPI_Wtime();
        DMat Cd = MemEfficientSpGEMM<PTDD, double, DDev>(Ad, Bd, (int)mc[0], hard, sel, rec, pct, 1, 1, mc[1]);
        cbh_ctx_synchronize(combblas_hip::context());
        double t1 = MPI_Wtime();
        PMat Ch = combblas_hip::to_host(Cd);
        bad += report(name, Ch, Cc, t1 - t0, 0.0);
      }
    }
    if (layers > 0 && nprocs % layers == 0 && is_square(nprocs / layers)) {
      PMat3D A3(A, layers, true, false), B3(B, layers, false, false);
      DMat3D A3d = combblas_hip::to_device(A3), B3d = combblas_hip::to_device(B3);
      {
        double t0 = MPI_Wtime();
        DMat3D C3d = Mult_AnXBn_SUMMA3D<PTDD, double, DDev, int64_t, double, double>(A3d, B3d);
        cbh_ctx_synchronize(combblas_hip::context());
        double t1 = MPI_Wtime();
        PMat3D C3c = Mult_AnXBn_SUMMA3D<CpuPlusTimes, double, DCols, int64_t, double, double, DCols, DCols>(A3, B3);
        double t2 = MPI_Wtime();
        PMat3D C3h = combblas_hip::to_host(C3d);
        bad += report3d("Mult_AnXBn_SUMMA3D", C3h, C3c, t1 - t0, t2 - t1);
      }
      for (int phases : {1, 2}) {
        char name[96];
        std::snprintf(name, sizeof(name), "MemEfficientSpGEMM3D<phases=%d,prune>", phases);
        double t0 = MPI_Wtime();
        DMat3D C3d = MemEfficientSpGEMM3D<PTDD, double, DDev, int64_t, double, double>(A3d, B3d, phases, hard, sel,
                                                                                       rec, pct, 1, 1, 0);
        cbh_ctx_synchronize(combblas_hip::context());
        double t1 = MPI_Wtime();
        PMat3D C3c = MemEfficientSpGEMM3D<CpuPlusTimes, double, DCols, int64_t, double, double, DCols, DCols>(
            A3, B3, phases, hard, sel, rec, pct, 1, 1, 0);
        double t2 = MPI_Wtime();
        PMat3D C3h = combblas_hip::to_host(C3d);
        bad += report3d(name, C3h, C3c, t1 - t0, t2 - t1);
      }
    }
  }
  MPI_Finalize();
  return bad ? 1 : 0;
}
