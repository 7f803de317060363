// HipSpGEMMKernels.h -- device half of HipSpGEMMDevice.h: compile ONE translation unit with
// hipcc that includes "CombBLAS/CombBLAS.h", this header and the semiring definitions, and
// instantiates the gfx950 kernels of each semiring the application routes to the device:
//
//   COMBBLAS_HIP_DEVICE_KERNELS(SR, IT, NT1, NT2, NTO)
//
// (the same arguments as COMBBLAS_HIP_INSTANTIATE_DEVICE in the host translation units). Only
// this definition of combblas_hip::DeviceLocalSpGEMM runs here: the reference drivers stay in
// the host translation units, built by the application's own compiler.
//
// Floating-point contract: compile this translation unit with -ffp-contract=off. hipcc fuses a*b+c
// into one fma by default, the reference's host build (g++ on x86-64) rounds the product and the
// sum separately, and the reference-order pass reproduces the stock kernel's values bit for bit only
// with the same roundings. The pragma below turns fusion off for everything parsed after this header
// (a semiring defined in a header included later); a semiring defined before it needs the flag.
#pragma once

#include "HipSpGEMMDevice.h"
#include "device/numeric.h"

#pragma clang fp contract(off)

namespace combblas_hip {

// reference semiring type -> device functor; every semiring not known to be order-free runs in the
// reference's accumulation order (ordered_semiring, HipSpGEMMDevice.h)
template <class SR, class NT1, class NT2, class NTO>
struct device_semiring {
  using type = cbh::UserSRD<SR, NT1, NT2, NTO, ordered_semiring<SR, NT1, NT2, NTO>::value>;
};
template <class T1, class T2, class NT1, class NT2, class NTO>
struct device_semiring<combblas::PlusTimesSRing<T1, T2>, NT1, NT2, NTO> {
  using base = typename std::conditional<std::is_same<NT1, NTO>::value && std::is_same<NT2, NTO>::value,
                                         cbh::PlusTimesD<NTO>, cbh::PlusTimesPromoteD<NT1, NT2, NTO>>::type;
  using type = typename std::conditional<ordered_semiring<combblas::PlusTimesSRing<T1, T2>, NT1, NT2, NTO>::value,
                                         cbh::Ordered<base>, base>::type;
};

// SelectMaxSRing / MinPlusSRing with NT1 != NT2: the reference's functions are host-only, so the
// device functor restates them (Semirings.h:165-187, 235-255) in T_promote = NTO.
template <class NT1, class NT2, class NTO>
struct SelectMaxPromoteD {
  using a_t = NT1;
  using b_t = NT2;
  using val_t = NTO;
  using acc_t = NTO;
  static constexpr bool kLocked = true;
  static __device__ __forceinline__ NTO multiply(NT1 a, NT2 b) { return static_cast<NTO>(a) * static_cast<NTO>(b); }
  static __device__ __forceinline__ NTO add(NTO a, NTO b) { return a < b ? b : a; }
  static __device__ __forceinline__ NTO identity() { return NTO(); }
  static __device__ __forceinline__ NTO finalize(NTO a) { return a; }
};
template <class NT1, class NT2, class NTO>
struct MinPlusPromoteD {
  using a_t = NT1;
  using b_t = NT2;
  using val_t = NTO;
  using acc_t = NTO;
  static constexpr bool kLocked = true;
  static __device__ __forceinline__ NTO multiply(NT1 a, NT2 b) {
    const NTO x = static_cast<NTO>(a), y = static_cast<NTO>(b), inf = std::numeric_limits<NTO>::max();
    return (x == inf || y == inf) ? inf : x + y;
  }
  static __device__ __forceinline__ NTO add(NTO a, NTO b) { return b < a ? b : a; }
  static __device__ __forceinline__ NTO identity() { return NTO(); }
  static __device__ __forceinline__ NTO finalize(NTO a) { return a; }
};
// Select2ndSRing (Semirings.h:143-163): host-only functions restated; reference-order accumulation
template <class OUT, class NT1, class NT2, class NTO>
struct Select2ndD {
  using a_t = NT1;
  using b_t = NT2;
  using val_t = NTO;
  using acc_t = NTO;
  static constexpr bool kLocked = true;
  static constexpr bool kOrdered = true;
  static __device__ __forceinline__ NTO multiply(const NT1&, const NT2& b) {
    return static_cast<NTO>(static_cast<OUT>(b));
  }
  static __device__ __forceinline__ NTO add(const NTO&, const NTO& y) { return y; }
  static __device__ __forceinline__ NTO identity() { return NTO(); }
  static __device__ __forceinline__ NTO finalize(const NTO& a) { return a; }
};
template <class T1, class T2, class OUT, class NT1, class NT2, class NTO>
struct device_semiring<combblas::Select2ndSRing<T1, T2, OUT>, NT1, NT2, NTO> {
  using type = Select2ndD<OUT, NT1, NT2, NTO>;
};
template <class T1, class T2, class NT1, class NT2, class NTO>
struct device_semiring<combblas::SelectMaxSRing<T1, T2>, NT1, NT2, NTO> {
  using base = SelectMaxPromoteD<NT1, NT2, NTO>;
  using type = typename std::conditional<ordered_semiring<combblas::SelectMaxSRing<T1, T2>, NT1, NT2, NTO>::value,
                                         cbh::Ordered<base>, base>::type;
};
template <class T1, class T2, class NT1, class NT2, class NTO>
struct device_semiring<combblas::MinPlusSRing<T1, T2>, NT1, NT2, NTO> {
  using base = MinPlusPromoteD<NT1, NT2, NTO>;
  using type = typename std::conditional<ordered_semiring<combblas::MinPlusSRing<T1, T2>, NT1, NT2, NTO>::value,
                                         cbh::Ordered<base>, base>::type;
};

// returnedSAID (mtSpGEMM.h:337): the reference's heap branch drops a product for which the
// semiring's multiply raised its "said" flag. A device multiply cannot raise a host flag, so a
// semiring with a settable flag (returnedSAID(bool), Applications/TwitterEdge.h:261) is rejected at
// compile time; one whose returnedSAID() is a plain query is checked once per call on the host.
template <class SR, class = void>
struct said_settable : std::false_type {};
template <class SR>
struct said_settable<SR, std::void_t<decltype(SR::returnedSAID(true))>> : std::true_type {};
template <class SR, class = void>
struct said_query : std::false_type {};
template <class SR>
struct said_query<SR, std::void_t<decltype(SR::returnedSAID())>> : std::true_type {};

// C = A*B on the device for any (SR, NT1, NT2, NTO): library plan + caller-instantiated kernels.
template <class SR, class NTO, class IT, class NT1, class NT2>
combblas::SpTuples<IT, NTO>* DeviceLocalSpGEMM(const combblas::SpDCCols<IT, NT1>& A,
                                               const combblas::SpDCCols<IT, NT2>& B, bool clearA, bool clearB,
                                               int branch) {
  using DSR = typename device_semiring<SR, NT1, NT2, NTO>::type;
  static_assert(std::is_trivially_copyable<NTO>::value, "device values must be trivially copyable");
  static_assert(!said_settable<SR>::value,
                "combblas_hip: a semiring whose multiply sets a returnedSAID flag (mtSpGEMM.h:337) cannot run on "
                "the device (its multiply would have to raise a host flag per product)");
  if constexpr (said_query<SR>::value)
    if (SR::returnedSAID()) die(nullptr, CBH_E_ARG, "returnedSAID() is true before the product (mtSpGEMM.h:337)");
  const IT mdim = A.getnrow(), ndim = B.getncol();
  combblas::SpTuples<IT, NTO>* out;
  if (A.isZero() || B.isZero()) {
    out = new combblas::SpTuples<IT, NTO>(0, mdim, ndim);  // mtSpGEMM.h:224-227
  } else {
    cbh_ctx* ctx = context();
    MatGuard a, b, c;
    a.m = upload(A);
    b.m = upload(B);
    cbh_plan* plan = nullptr;
    int rc = cbh_plan_create(ctx, a.m, b.m, &plan);
    if (rc != CBH_OK) die(ctx, rc, "cbh_plan_create");
    cbh_numeric_plan np;
    rc = cbh_plan_numeric(plan, dtype_of<NTO>::value, (int64_t)sizeof(NTO), cbh::plan_flags<DSR>(), &c.m, &np);
    if (rc != CBH_OK) die(ctx, rc, "cbh_plan_numeric");
    const int64_t *cp, *jc;
    const int32_t* ir;
    const void* num;
    cbh_mat_device_arrays(c.m, &cp, &jc, &ir, &num);
    int64_t nnzC = 0;
    cbh_mat_info(c.m, nullptr, nullptr, &nnzC, nullptr, nullptr);
    hipError_t e = cbh::run_numeric_plan<DSR>(np, const_cast<int32_t*>(ir), const_cast<void*>(num), nnzC);
    if constexpr (cbh::sr_ordered<DSR>::value) {  // then every output re-folded in the reference's own order
      if (e == hipSuccess) {
        void* scratch = nullptr;
        const int64_t nnzB = (int64_t)B.getnnz();
        rc = cbh_ctx_alloc(ctx, (int64_t)cbh::ord_scratch_bytes<DSR>(nnzB, np.ntasks, nnzC), &scratch);
        if (rc != CBH_OK) die(ctx, rc, "cbh_ctx_alloc (reference-order scratch)");
        cbh::TaskArgs ta = cbh::numeric_args(np, 0, const_cast<int32_t*>(ir), const_cast<void*>(num), nnzC);
        e = cbh::launch_reference_order<DSR>(ta, scratch, nnzB, nnzC, branch, reinterpret_cast<hipStream_t>(np.stream));
        cbh_ctx_free(ctx, scratch);  // stream-ordered: the launches above run first
      }
    }
    if (e != hipSuccess) {
      std::fprintf(stderr, "combblas_hip: numeric launch failed: %s\n", hipGetErrorString(e));
      MPI_Abort(MPI_COMM_WORLD, CBH_E_HIP);
    }
    rc = cbh_plan_finish(plan, c.m, 0);
    if (rc != CBH_OK) die(ctx, rc, "cbh_plan_finish");
    cbh_plan_destroy(plan);
    out = download_tuples<IT, NTO>(c.m);
  }
  if (clearA) delete const_cast<combblas::SpDCCols<IT, NT1>*>(&A);
  if (clearB) delete const_cast<combblas::SpDCCols<IT, NT2>*>(&B);
  return out;
}

}  // namespace combblas_hip


#define COMBBLAS_HIP_DEVICE_KERNELS(SR, IT, NT1, NT2, NTO)                                                   \
  template combblas::SpTuples<IT, NTO>* combblas_hip::DeviceLocalSpGEMM<SR, NTO, IT, NT1, NT2>(            \
      const combblas::SpDCCols<IT, NT1>&, const combblas::SpDCCols<IT, NT2>&, bool, bool, int);
