// Dev3DSpGEMM.h -- the reference's STANDALONE 3D SpGEMM layer (3DSpGEMM/: the `mpipspgemm` driver's
// CCGrid / SplitMat / SUMMALayer / ReduceAll_threaded / ParallelReduce_Alltoall_threaded /
// multiply) for device-resident blocks.
//
// Include after the reference's 3DSpGEMM headers (CCGrid.h, SUMMALayer.h, Reductions.h,
// Multiplier.h). The overloads below take SpDCColsDev blocks where the reference takes SpDCCols,
// so a driver that keeps its split blocks on the device (splitA = SpDCColsDev(splitA_host) after
// SplitMat) runs the same layer with every stage block, partial and reduce-scatter piece in HBM:
//   SUMMALayer                 SUMMALayer.h:24-97    stage blocks broadcast on CMG.rowWorld /
//                                                    colWorld with RCCL (BCastMatrix), local products
//                                                    on the device (LocalSpGEMM's contract)
//   ReduceAll_threaded         Reductions.h:136-155  the stage partials merged on the device
//                                                    (MultiwayMerge), then the fiber reduce-scatter
//   ParallelReduce_Alltoall_threaded  Reductions.h:36-132  column pieces at findColSplitters' cuts
//                                                    (i * (n / c); the last takes the remainder),
//                                                    exchanged over CMG.fiberWorld with grouped
//                                                    ncclSend / ncclRecv, merged on the device
//   multiply                   Multiplier.h:10-61    SUMMALayer + ReduceAll_threaded, the layer's
//                                                    timers kept (comm_bcast, comp_summa, ...)
// One deliberate difference (as in combblas_amd/spgemm3d.py): every fiber rank rebases its
// piece's column ids by its chunk START; the reference shifts the last rank by its remainder-sized
// width (Reductions.h:99-102), which agrees only when the layer count divides the column count.
// PlusTimesSRing<NT,NT> is the semiring, as the reference's layer hard-codes (SUMMALayer.h:27,
// Reductions.h:136). Link as for ParFriendsDev.h (libcombblas_hip.so, librccl.so, MPI).
#pragma once

#include "ParFriendsDev.h"

namespace combblas {

template <typename IT, typename NT>
void SUMMALayer(combblas_hip::SpDCColsDev<IT, NT>& SplitA, combblas_hip::SpDCColsDev<IT, NT>& SplitB,
                std::vector<combblas_hip::SpDCColsDev<IT, NT>*>& C, CCGrid& CMG, bool isBT, bool threaded) {
  typedef PlusTimesSRing<NT, NT> PTNN;
  // the outer-product mode (mpipspgemm.cpp:176-179: SplitB locally transposed, threaded = false ->
  // MultiplyReturnTuples(A, B, false, isBT), SUMMALayer.h:80-86): every received B block is
  // transposed back on the device (cbh_transpose) and the product runs as in the threaded mode;
  // with threaded = true the reference's LocalSpGEMM ignores isBT, and so does this overload
  const bool transposeB = isBT && !threaded;
  const int stages = CMG.GridCols;
  auto Asizes = combblas_hip::GetSetSizes(SplitA, CMG.rowWorld);
  auto Bsizes = combblas_hip::GetSetSizes(SplitB, CMG.colWorld);
  const int Aself = CMG.RankInRow, Bself = CMG.RankInCol;
  for (int i = 0; i < stages; ++i) {
    const double bcast_beg = MPI_Wtime();
    combblas_hip::SpDCColsDev<IT, NT> Arecv, Brecv;
    combblas_hip::SpDCColsDev<IT, NT>& Ai = (i == Aself) ? SplitA : Arecv;
    combblas_hip::SpDCColsDev<IT, NT>& Bi = (i == Bself) ? SplitB : Brecv;
    combblas_hip::BCastMatrix(CMG.rowWorld, Ai, Asizes[i], i);
    combblas_hip::BCastMatrix(CMG.colWorld, Bi, Bsizes[i], i);
    combblas_hip::hip_check(hipStreamSynchronize(reinterpret_cast<hipStream_t>(cbh_ctx_stream(combblas_hip::context()))), "hipStreamSynchronize");
    comm_bcast += MPI_Wtime() - bcast_beg;
    const double summa_beg = MPI_Wtime();
    cbh_mat* Ci;
    if (transposeB) {
      cbh_mat* Bt = nullptr;
      const int rc = cbh_transpose(combblas_hip::context(), Bi.mat(), &Bt);
      if (rc != CBH_OK) combblas_hip::die(combblas_hip::context(), rc, "cbh_transpose");
      Ci = combblas_hip::local_multiply<PTNN, NT, NT, NT>(Ai.mat(), Bt);
      cbh_mat_free(combblas_hip::context(), Bt);
    } else {
      Ci = combblas_hip::local_multiply<PTNN, NT, NT, NT>(Ai.mat(), Bi.mat());
    }
    comp_summa += MPI_Wtime() - summa_beg;
    C.push_back(new combblas_hip::SpDCColsDev<IT, NT>(Ci));  // received blocks are freed with Arecv / Brecv
  }
}

template <typename SR, typename IT, typename NT>
combblas_hip::SpDCColsDev<IT, NT>* ParallelReduce_Alltoall_threaded(MPI_Comm& fibWorld,
                                                                     combblas_hip::SpDCColsDev<IT, NT>*& localmerged) {
  int fprocs = 1;
  MPI_Comm_size(fibWorld, &fprocs);
  if (fprocs == 1) return localmerged;
  const double beg = MPI_Wtime();
  const int64_t ndim = localmerged->getncol();
  const auto cuts = combblas_hip::colsplit_cuts(ndim, fprocs);  // findColSplitters: i * (ndim / fprocs)
  std::vector<int64_t> div(fprocs);
  for (int j = 0; j < fprocs; ++j) div[j] = cuts[j + 1] - cuts[j];
  cbh_mat* C = combblas_hip::fiber_reduce_scatter(combblas_hip::semiring_traits<SR>::code, localmerged->release(), div,
                                                  fibWorld, combblas_hip::dtype_of<NT>::value, (int64_t)sizeof(NT));
  delete localmerged;
  localmerged = nullptr;
  comm_reduce += MPI_Wtime() - beg;
  return new combblas_hip::SpDCColsDev<IT, NT>(C);
}

template <typename NT, typename IT>
combblas_hip::SpDCColsDev<IT, NT>* ReduceAll_threaded(std::vector<combblas_hip::SpDCColsDev<IT, NT>*>& unreducedC,
                                                       CCGrid& CMG) {
  typedef PlusTimesSRing<NT, NT> PTNN;
  const double beg = MPI_Wtime();
  const int64_t m = unreducedC[0]->getnrow(), n = unreducedC[0]->getncol();
  std::vector<cbh_mat*> parts;
  for (auto* p : unreducedC) {
    if (p->getnnz() > 0) parts.push_back(p->release());
    delete p;
  }
  unreducedC.clear();
  cbh_mat* merged = nullptr;
  if (parts.empty()) {
    int rc = cbh_mat_create(combblas_hip::context(), m, n, 0, 0, combblas_hip::dtype_of<NT>::value, (int64_t)sizeof(NT),
                            &merged);
    if (rc != CBH_OK) combblas_hip::die(combblas_hip::context(), rc, "cbh_mat_create");
  } else {
    merged = parts.size() == 1 ? parts[0] : combblas_hip::merge_all(combblas_hip::semiring_traits<PTNN>::code, parts);
  }
  comp_reduce += MPI_Wtime() - beg;
  auto* local = new combblas_hip::SpDCColsDev<IT, NT>(merged);
  return ParallelReduce_Alltoall_threaded<PTNN>(CMG.fiberWorld, local);
}

template <typename IT, typename NT>
combblas_hip::SpDCColsDev<IT, NT>* multiply(combblas_hip::SpDCColsDev<IT, NT>& splitA,
                                            combblas_hip::SpDCColsDev<IT, NT>& splitB, CCGrid& CMG, bool isBT,
                                            bool threaded) {
  comm_bcast = 0, comm_reduce = 0, comp_summa = 0, comp_reduce = 0, comp_result = 0, comp_reduce_layer = 0;
  std::vector<combblas_hip::SpDCColsDev<IT, NT>*> unreducedC;
  SUMMALayer(splitA, splitB, unreducedC, CMG, isBT, threaded);
  combblas_hip::SpDCColsDev<IT, NT>* C = ReduceAll_threaded<NT>(unreducedC, CMG);
  combblas_hip::hip_check(hipStreamSynchronize(reinterpret_cast<hipStream_t>(cbh_ctx_stream(combblas_hip::context()))), "hipStreamSynchronize");
  return C;
}

}  // namespace combblas
