// Drop-in test of the reference's STANDALONE 3D SpGEMM layer (3DSpGEMM/: CCGrid.h, SplitMatDist.h,
// SUMMALayer.h, Reductions.h, Multiplier.h -- the `mpipspgemm` driver's path), built by
// `make -C oracle ref` twice from this one source with g++, as the reference is:
//   oracle/_ref/dropin3ds_harness  -- COMBBLAS_HIP_INSTANTIATE(PlusTimesSRing<double,double>, int64_t,
//                                     double): the layer's LocalSpGEMM (SUMMALayer.h:78) and both
//                                     MultiwayMerge calls (Reductions.h:119,143) run on the gfx950
//                                     kernels through the C-ABI;
//   oracle/_ref/stock3ds_harness   -- -DCBH_STOCK: the same code on the reference's own OpenMP kernels.
// Flow (mpipspgemm.cpp's column-threaded case): CCGrid(layers, gridcols); on layer 0 a packed R-MAT
// (deterministic, unlike GenMat's time-seeded permutation) on the layer's 2D grid; SplitMat of A by
// columns and of B by rows down the fibers (SplitMatDist.h:143-213); multiply(splitA, splitB, CMG,
// false, true) (Multiplier.h:10-61: SUMMALayer's stage broadcasts and local products, then
// ReduceAll_threaded's merge and the fiber reduce-scatter ParallelReduce_Alltoall_threaded).
// Every rank prints an order-sensitive digest of its block of C; tests/test_dropin3d_gpu.py
// compares the binaries rank by rank (a third, oracle/_ref/devpath3ds_harness, -DCBH_DEVPATH, runs
// the device-resident overloads of the same layer, see below). Values are edge multiplicities: every double sum is exact.
//   mpirun -np P dropin3ds_harness <scale> <layers> [bt]   (P / layers a square: 1x1xc or 2x2xc)
// bt: mpipspgemm.cpp's outer-product case (:176-179): splitB transposed locally, multiply(splitA,
// splitB, CMG, true, false) -- the reference's MultiplyReturnTuples(..., isBT) stock, the device
// overload's transpose-back on the device with -DCBH_DEVPATH.
#include <mpi.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "CombBLAS/CombBLAS.h"
#if !defined(CBH_STOCK) && !defined(CBH_DEVPATH)
#include "combblas_hip/HipSpGEMM.h"
typedef combblas::PlusTimesSRing<double, double> PTDD;
COMBBLAS_HIP_INSTANTIATE(PTDD, int64_t, double)
#endif
#include "Glue.h"
#include "CCGrid.h"
#include "Reductions.h"
#include "SUMMALayer.h"
#include "Multiplier.h"
#include "SplitMatDist.h"
#ifdef CBH_DEVPATH
// oracle/_ref/devpath3ds_harness: the split blocks uploaded once (SpDCColsDev) and the layer run by the
// device overloads of include/combblas_hip/Dev3DSpGEMM.h (RCCL stage broadcasts and fiber exchange;
// COMBBLAS_HIP_COMM=mpi host-stages them when ranks share one GPU); C downloaded for the digest
#include "combblas_hip/Dev3DSpGEMM.h"
#endif

using namespace combblas;

// the layer's timers (Glue.h declares them extern; mpipspgemm.cpp defines them)
double comm_bcast, comm_reduce, comm_split, comp_summa, comp_reduce, comp_reduce_layer, comp_result, comp_trans,
    comp_split;
double cblas_alltoalltime, cblas_allgathertime, cblas_mergeconttime, cblas_transvectime, cblas_localspmvtime;
MTRand GlobalMT(123);

typedef SpDCCols<int64_t, double> DCols;

// layer 0: the packed Graph500 R-MAT on the layer's 2D grid (its local block); other layers: empty
static DCols* make_input(CCGrid& CMG, int scale) {
  if (CMG.layer_grid != 0) return new DCols();
  double init[4] = {.57, .19, .19, .05};
  DistEdgeList<int64_t>* DEL = new DistEdgeList<int64_t>(CMG.layerWorld);
  DEL->GenGraph500Data(init, scale, 16, true, true);
  SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>> G(*DEL, false);
  delete DEL;
  SpParMat<int64_t, double, DCols> A(G);
  return new DCols(A.seq());
}

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// order-sensitive digest of a DCSC block: columns in order, rows in stored order, value bits
static uint64_t block_digest(DCols& M) {
  uint64_t d = 0, k = 0;
  for (auto colit = M.begcol(); colit != M.endcol(); ++colit)
    for (auto nzit = M.begnz(colit); nzit != M.endnz(colit); ++nzit) {
      uint64_t bits;
      const double v = nzit.value();
      std::memcpy(&bits, &v, sizeof(bits));
      d += mix64(k++ ^ mix64((uint64_t)colit.colid() ^ mix64((uint64_t)nzit.rowid() ^ mix64(bits))));
    }
  return d;
}

int main(int argc, char** argv) {
  int provided;
  MPI_Init_thread(&argc, &argv, MPI_THREAD_SERIALIZED, &provided);
  const int scale = argc > 1 ? std::atoi(argv[1]) : 10;
  const int layers = argc > 2 ? std::atoi(argv[2]) : 2;
  const bool bt = argc > 3 && std::strcmp(argv[3], "bt") == 0;
  int nprocs, myrank;
  MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
  MPI_Comm_rank(MPI_COMM_WORLD, &myrank);
  const int per_layer = nprocs / layers;
  const int gc = (int)std::lround(std::sqrt((double)per_layer));
  if (layers < 1 || per_layer * layers != nprocs || gc * gc != per_layer) {
    if (myrank == 0) std::fprintf(stderr, "ranks / layers must be a square\n");
    MPI_Abort(MPI_COMM_WORLD, 2);
  }
  {  // every CombBLAS object must be destroyed before MPI_Finalize
    CCGrid CMG(layers, gc);
    DCols splitA, splitB;
    DCols* A = make_input(CMG, scale);
    DCols* B = make_input(CMG, scale);
    SplitMat(CMG, A, splitA, false);
    SplitMat(CMG, B, splitB, true);  // row split
    delete A;
    delete B;
    if (bt) splitB.Transpose();  // locally transposed for the outer product
#ifdef CBH_DEVPATH
    combblas_hip::SpDCColsDev<int64_t, double> dA(splitA), dB(splitB);
    delete multiply(dA, dB, CMG, bt, !bt);  // first call: HIP context, code objects, communicators
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    combblas_hip::SpDCColsDev<int64_t, double>* Cd = multiply(dA, dB, CMG, bt, !bt);
    const double t1 = MPI_Wtime();
    DCols* C = Cd->to_host();
    delete Cd;
#else
    DCols* C = multiply(splitA, splitB, CMG, bt, !bt);  // first call: HIP context, code objects
    delete C;
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    C = multiply(splitA, splitB, CMG, bt, !bt);
    const double t1 = MPI_Wtime();
#endif
    const uint64_t dg = block_digest(*C);
    int64_t nnz = C->getnnz(), tot = 0;
    MPI_Allreduce(&nnz, &tot, 1, MPI_INT64_T, MPI_SUM, MPI_COMM_WORLD);
    for (int r = 0; r < nprocs; ++r) {
      if (r == myrank) {
        std::printf("BLOCK3DS rank=%d layer=%d m=%lld n=%lld nnz=%lld digest=%016llx\n", myrank, CMG.layer_grid,
                    (long long)C->getnrow(), (long long)C->getncol(), (long long)nnz, (unsigned long long)dg);
        std::fflush(stdout);
      }
      MPI_Barrier(MPI_COMM_WORLD);
    }
    if (myrank == 0) {
      std::printf("TOTAL3DS grid=%dx%dx%d nnz=%lld multiply_s=%.4f\n", gc, gc, layers, (long long)tot, t1 - t0);
      std::fflush(stdout);
    }
    delete C;
  }
  MPI_Finalize();
  return 0;
}
