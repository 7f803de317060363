// HipSpGEMMDevice.h -- the drop-in for semirings the library was NOT built with. Host code:
// include AFTER "CombBLAS/CombBLAS.h" in the translation units that run the reference drivers
// (compiled with the application's own compiler, as the reference is -- g++), and use
//
//   COMBBLAS_HIP_INSTANTIATE_DEVICE(SR, IT, NT1, NT2, NTO)
//
// to declare explicit specializations of combblas::LocalHybridSpGEMM / LocalSpGEMMHash /
// LocalSpGEMM <SR, NTO, IT, NT1, NT2> (mtSpGEMM.h:74,213,463), so that the UNCHANGED reference
// drivers (PSpGEMM -> Mult_AnXBn_Synch, ParFriends.h:1004-1108; SpParMat.h:454-467 with its
// promote_trait NT1 != NT2 -> T_promote) run the product on the device. The device kernels for
// the semiring are instantiated in ONE hipcc-compiled translation unit with
// COMBBLAS_HIP_DEVICE_KERNELS(SR, IT, NT1, NT2, NTO) from HipSpGEMMKernels.h. Supported:
//   * a user semiring with the reference's static-functor contract (Semirings.h:143-255) whose
//     add and multiply are __host__ __device__ -- e.g. the bool OR-AND KTipsSR
//     (ReleaseTests/KTipsTest.cpp:12-20) or a semiring over a struct value (SegTest.cpp:35-61):
//     the kernels accumulate under a per-slot lock with SR::add (any trivially copyable NTO);
//   * the reference's PlusTimesSRing / SelectMaxSRing / MinPlusSRing with NT1 != NT2 (promotion).
// The semiring-independent half (symbolic pass, task plan, binning, C's allocation, column
// compaction) runs in libcombblas_hip.so through the cbh_plan_* C-ABI (include/combblas_hip.h).
//
// Exact-parity note: the device accumulates the products of one output in no fixed order, so a
// semiring whose add is commutative and associative (integers, bool, min/max, structs of such)
// matches the reference bit for bit; a non-commutative add (Select2ndSRing, KmerIntersect's
// "first/second" fields) is computed with the reference's hash-branch argument order
// add(new, old) but in arrival order, which the reference itself does not fix either (its
// heap branch folds add(old, new), mtSpGEMM.h:341 vs :408).
#pragma once

#include "HipSpGEMM.h"

namespace combblas_hip {
// defined in HipSpGEMMKernels.h, explicitly instantiated by COMBBLAS_HIP_DEVICE_KERNELS (hipcc)
template <class SR, class NTO, class IT, class NT1, class NT2>
combblas::SpTuples<IT, NTO>* DeviceLocalSpGEMM(const combblas::SpDCCols<IT, NT1>& A,
                                               const combblas::SpDCCols<IT, NT2>& B, bool clearA, bool clearB);
}  // namespace combblas_hip

#define COMBBLAS_HIP_INSTANTIATE_DEVICE(SR, IT, NT1, NT2, NTO)                                                  \
  namespace combblas {                                                                                          \
  template <>                                                                                                   \
  inline SpTuples<IT, NTO>* LocalHybridSpGEMM<SR, NTO, IT, NT1, NT2>(const SpDCCols<IT, NT1>& A,              \
                                                                    const SpDCCols<IT, NT2>& B, bool clearA,   \
                                                                    bool clearB, IT* aux) {                    \
    (void)aux;                                                                                                  \
    return combblas_hip::DeviceLocalSpGEMM<SR, NTO, IT, NT1, NT2>(A, B, clearA, clearB);                                     \
  }                                                                                                             \
  template <>                                                                                                   \
  inline SpTuples<IT, NTO>* LocalSpGEMMHash<SR, NTO, IT, NT1, NT2>(const SpDCCols<IT, NT1>& A,                \
                                                                  const SpDCCols<IT, NT2>& B, bool clearA,     \
                                                                  bool clearB, bool sort) {                    \
    (void)sort; /* ascending rows are a valid order for the unsorted contract */                               \
    return combblas_hip::DeviceLocalSpGEMM<SR, NTO, IT, NT1, NT2>(A, B, clearA, clearB);                                     \
  }                                                                                                             \
  template <>                                                                                                   \
  inline SpTuples<IT, NTO>* LocalSpGEMM<SR, NTO, IT, NT1, NT2>(const SpDCCols<IT, NT1>& A,                    \
                                                              const SpDCCols<IT, NT2>& B, bool clearA,         \
                                                              bool clearB) {                                   \
    return combblas_hip::DeviceLocalSpGEMM<SR, NTO, IT, NT1, NT2>(A, B, clearA, clearB);                                     \
  }                                                                                                             \
  }
