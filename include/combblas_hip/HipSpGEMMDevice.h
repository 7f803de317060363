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
// Exact-parity note: the throughput kernels accumulate the products of one output in arrival
// order, so a semiring whose add is commutative and associative (integers, bool, min/max, structs
// of such) matches the reference bit for bit. A semiring marked reference_order (below: the
// reference's Select2ndSRing; any application semiring it specializes) instead runs the
// reference's own per-column algorithm on the device -- heap branch for cr < 2 with libstdc++'s
// heap order and add(old, new), hash branch otherwise with add(new, old) in B-entry order
// (mtSpGEMM.h:311-437, device/order_kernel.h) -- so even a non-commutative add, or floating-point
// sums, match the stock path bit for bit. That pass walks a column per thread: a correctness
// path, not the throughput one.
#pragma once

#include "HipSpGEMM.h"

namespace combblas_hip {
// semirings computed in the reference's own accumulation order (device/order_kernel.h). An
// application marks its own semiring with
//   template <> struct combblas_hip::reference_order<MySR> : std::true_type {};
// visible in both translation units (before COMBBLAS_HIP_DEVICE_KERNELS).
template <class SR>
struct reference_order : std::false_type {};
template <class T1, class T2, class OUT>
struct reference_order<combblas::Select2ndSRing<T1, T2, OUT>> : std::true_type {};  // add(x, y) = y

// defined in HipSpGEMMKernels.h, explicitly instantiated by COMBBLAS_HIP_DEVICE_KERNELS (hipcc).
// branch: which reference kernel a reference_order semiring follows -- 0 LocalHybridSpGEMM (heap for
// cr < 2, hash otherwise), 1 LocalSpGEMM (heap), 2 LocalSpGEMMHash (hash); the others ignore it.
template <class SR, class NTO, class IT, class NT1, class NT2>
combblas::SpTuples<IT, NTO>* DeviceLocalSpGEMM(const combblas::SpDCCols<IT, NT1>& A,
                                               const combblas::SpDCCols<IT, NT2>& B, bool clearA, bool clearB,
                                               int branch = 0);
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
    return combblas_hip::DeviceLocalSpGEMM<SR, NTO, IT, NT1, NT2>(A, B, clearA, clearB, 2);                                  \
  }                                                                                                             \
  template <>                                                                                                   \
  inline SpTuples<IT, NTO>* LocalSpGEMM<SR, NTO, IT, NT1, NT2>(const SpDCCols<IT, NT1>& A,                    \
                                                              const SpDCCols<IT, NT2>& B, bool clearA,         \
                                                              bool clearB) {                                   \
    return combblas_hip::DeviceLocalSpGEMM<SR, NTO, IT, NT1, NT2>(A, B, clearA, clearB, 1);                                  \
  }                                                                                                             \
  }
