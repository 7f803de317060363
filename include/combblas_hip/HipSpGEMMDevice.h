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
// Exact-parity contract: the throughput kernels accumulate the products of one output in arrival
// order, which is exact only when add is commutative and associative on the values (integers,
// bool, min / max). Arrival order is therefore OPT-IN: a semiring runs in it only when
// arrival_order_ok<SR> says so -- true for the built-in PlusTimes / SelectMax / MinPlus over
// integer and bool values and for SelectMax / MinPlus over floating values; an application marks
// its own commutative semiring with
//   template <> struct combblas_hip::arrival_order_ok<MySR> : std::true_type {};
// Every other semiring -- any unmarked user semiring, PlusTimes over float / double, the
// reference's Select2ndSRing -- gets the reference's own accumulation order on the device: after
// the throughput pass, every output is re-folded as LocalHybridSpGEMM folds it (heap branch for
// cr < 2 with libstdc++'s heap order and add(old, new), a thread per column; hash branch
// otherwise, add(new, old) in B-entry order, a wave per task; mtSpGEMM.h:311-437,
// device/order_kernel.h), so even a non-commutative add, or floating-point sums, match the stock
// path bit for bit. reference_order<SR> forces that order for a semiring marked arrival_order_ok.
// (Built-in semirings through COMBBLAS_HIP_INSTANTIATE run the library's kernels: arrival order
// unless the caller passes cbh_spgemm's CBH_ORDER_* flags.)
#pragma once

#include "HipSpGEMM.h"

namespace combblas_hip {
template <class SR>
struct arrival_order_ok : std::false_type {};
template <class T1, class T2>
struct arrival_order_ok<combblas::PlusTimesSRing<T1, T2>>
    : std::integral_constant<bool, !std::is_floating_point<T1>::value && !std::is_floating_point<T2>::value> {};
template <class T1, class T2>
struct arrival_order_ok<combblas::SelectMaxSRing<T1, T2>> : std::true_type {};  // max: exact in any order
template <class T1, class T2>
struct arrival_order_ok<combblas::MinPlusSRing<T1, T2>> : std::true_type {};    // min: exact in any order
// forces the reference's order for a semiring marked arrival_order_ok (visible in both
// translation units, before COMBBLAS_HIP_DEVICE_KERNELS)
template <class SR>
struct reference_order : std::false_type {};
template <class T1, class T2, class OUT>
struct reference_order<combblas::Select2ndSRing<T1, T2, OUT>> : std::true_type {};  // add(x, y) = y
// the order the device pass uses for SR over these value types (a PlusTimes sum in a floating
// output type is not order-free, whatever SR's own template arguments say)
template <class SR>
struct is_plus_times : std::false_type {};
template <class T1, class T2>
struct is_plus_times<combblas::PlusTimesSRing<T1, T2>> : std::true_type {};
template <class SR, class NT1, class NT2, class NTO>
struct ordered_semiring
    : std::integral_constant<bool, reference_order<SR>::value || !arrival_order_ok<SR>::value ||
                                       (is_plus_times<SR>::value && std::is_floating_point<NTO>::value)> {};

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
