// Device-side semiring functors, inlined into the SpGEMM/merge kernels as template
// parameters. Each mirrors a reference semiring's static contract (Semirings.h) --
// multiply(a,b) with A's value first (mtSpGEMM.h:401), add(x,y) -- plus what the
// device path needs on top of it:
//   identity()   a TRUE two-sided identity of add, used to pre-fill LDS accumulators
//                (the reference's SR::id() is not always one: SelectMaxSRing::id() is -1).
//   lds_acc()    atomic "acc = add(acc, v)" on an LDS slot (ds_add_f64 / ds_max_i64 / ...).
// val_t is the element type in HBM; acc_t the LDS accumulator type (bool widens to u32
// so it can use ds_or_b32). Optional members: a_t / b_t (A's and B's value types when they
// differ from val_t -- the reference's NT1 / NT2 -> T_promote), kLocked (the kernels accumulate
// under a per-slot lock with SR::add instead of SR::lds_acc: any trivially copyable value type,
// e.g. a user semiring's struct; the first product of a slot is stored as is, every later one is
// folded in with add(new, old) -- the reference's hash-branch order, mtSpGEMM.h:401-416).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <limits>
#include <type_traits>

namespace cbh {

template <class SR, class = void>
struct sr_a_type { using type = typename SR::val_t; };
template <class SR>
struct sr_a_type<SR, std::void_t<typename SR::a_t>> { using type = typename SR::a_t; };
template <class SR, class = void>
struct sr_b_type { using type = typename SR::val_t; };
template <class SR>
struct sr_b_type<SR, std::void_t<typename SR::b_t>> { using type = typename SR::b_t; };
template <class SR, class = void>
struct sr_locked : std::false_type {};
template <class SR>
struct sr_locked<SR, std::void_t<decltype(SR::kLocked)>> : std::integral_constant<bool, SR::kLocked> {};

template <class T>
struct PlusTimesD {  // PlusTimesSRing<T,T>, Semirings.h:212-232
  using val_t = T;
  using acc_t = T;
  static __device__ __forceinline__ acc_t identity() {
    // -0.0 (not +0.0) so that add(identity, -0.0) keeps the sign, as x alone would.
    if constexpr (std::is_floating_point<T>::value) return (T)-0.0;
    else return (T)0;
  }
  static __device__ __forceinline__ T multiply(T a, T b) { return a * b; }
  static __device__ __forceinline__ T add(T a, T b) { return a + b; }
  static __device__ __forceinline__ void lds_acc(acc_t* p, T v) {
    if constexpr (sizeof(T) == 8 && !std::is_floating_point<T>::value)
      atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v);
    else if constexpr (sizeof(T) == 4 && !std::is_floating_point<T>::value)
      atomicAdd(reinterpret_cast<unsigned int*>(p), (unsigned int)v);
    else
      atomicAdd(p, v);
  }
  static __device__ __forceinline__ val_t finalize(acc_t a) { return a; }
};

template <class T>
struct SelectMaxD {  // SelectMaxSRing<T,T>, Semirings.h:165-187
  using val_t = T;
  using acc_t = T;
  static __device__ __forceinline__ acc_t identity() { return std::numeric_limits<T>::lowest(); }
  static __device__ __forceinline__ T multiply(T a, T b) { return a * b; }
  static __device__ __forceinline__ T add(T a, T b) { return a < b ? b : a; }  // std::max(a,b)
  static __device__ __forceinline__ void lds_acc(acc_t* p, T v) {
    if constexpr (std::is_same<T, int64_t>::value) atomicMax(reinterpret_cast<long long*>(p), (long long)v);
    else if constexpr (std::is_same<T, int32_t>::value) atomicMax(p, v);
    else atomic_generic(p, v);
  }
  static __device__ __forceinline__ void atomic_generic(acc_t* p, T v) {
    static_assert(sizeof(T) == 8 || sizeof(T) == 4, "width");
    if constexpr (sizeof(T) == 8) {
      unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
      unsigned long long old = *q, assumed;
      do {
        assumed = old;
        T cur = __builtin_bit_cast(T, assumed);
        T nv = add(cur, v);
        if (__builtin_bit_cast(unsigned long long, nv) == assumed) return;
        old = atomicCAS(q, assumed, __builtin_bit_cast(unsigned long long, nv));
      } while (old != assumed);
    } else {
      unsigned int* q = reinterpret_cast<unsigned int*>(p);
      unsigned int old = *q, assumed;
      do {
        assumed = old;
        T cur = __builtin_bit_cast(T, assumed);
        T nv = add(cur, v);
        if (__builtin_bit_cast(unsigned int, nv) == assumed) return;
        old = atomicCAS(q, assumed, __builtin_bit_cast(unsigned int, nv));
      } while (old != assumed);
    }
  }
  static __device__ __forceinline__ val_t finalize(acc_t a) { return a; }
};

template <class T>
struct MinPlusD {  // MinPlusSRing<T,T>, Semirings.h:235-255 (multiply = inf_plus, Semirings.h:40-47)
  using val_t = T;
  using acc_t = T;
  static __device__ __forceinline__ acc_t identity() { return std::numeric_limits<T>::max(); }
  static __device__ __forceinline__ T multiply(T a, T b) {
    const T inf = std::numeric_limits<T>::max();
    return (a == inf || b == inf) ? inf : a + b;
  }
  static __device__ __forceinline__ T add(T a, T b) { return b < a ? b : a; }  // std::min(a,b)
  static __device__ __forceinline__ void lds_acc(acc_t* p, T v) {
    if constexpr (std::is_same<T, int64_t>::value) atomicMin(reinterpret_cast<long long*>(p), (long long)v);
    else if constexpr (std::is_same<T, int32_t>::value) atomicMin(p, v);
    else {
      unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
      unsigned long long old = *q, assumed;
      do {
        assumed = old;
        T nv = add(__builtin_bit_cast(T, assumed), v);
        if (__builtin_bit_cast(unsigned long long, nv) == assumed) return;
        old = atomicCAS(q, assumed, __builtin_bit_cast(unsigned long long, nv));
      } while (old != assumed);
    }
  }
  static __device__ __forceinline__ val_t finalize(acc_t a) { return a; }
};

struct OrAndD {  // boolean OR-AND: PlusTimesSRing<bool,bool> / KTipsSR (ReleaseTests/KTipsTest.cpp:12-20)
  using val_t = uint8_t;
  using acc_t = uint32_t;
  static __device__ __forceinline__ acc_t identity() { return 0u; }
  static __device__ __forceinline__ uint8_t multiply(uint8_t a, uint8_t b) { return (uint8_t)((a != 0) & (b != 0)); }
  static __device__ __forceinline__ uint8_t add(uint8_t a, uint8_t b) { return (uint8_t)((a != 0) | (b != 0)); }
  static __device__ __forceinline__ void lds_acc(acc_t* p, uint8_t v) {
    if (v) atomicOr(p, 1u);
  }
  static __device__ __forceinline__ val_t finalize(acc_t a) { return (uint8_t)(a != 0); }
};

// PlusTimesSRing<T1,T2> with T1 != T2 (Semirings.h:212-232): multiply in T_promote = TO.
template <class T1, class T2, class TO>
struct PlusTimesPromoteD {
  using a_t = T1;
  using b_t = T2;
  using val_t = TO;
  using acc_t = TO;
  static __device__ __forceinline__ acc_t identity() { return PlusTimesD<TO>::identity(); }
  static __device__ __forceinline__ TO multiply(T1 a, T2 b) { return static_cast<TO>(a) * static_cast<TO>(b); }
  static __device__ __forceinline__ TO add(TO a, TO b) { return a + b; }
  static __device__ __forceinline__ void lds_acc(acc_t* p, TO v) { PlusTimesD<TO>::lds_acc(p, v); }
  static __device__ __forceinline__ val_t finalize(acc_t a) { return a; }
};

// A user semiring with the reference's static-functor contract (Semirings.h:143-255; e.g.
// ReleaseTests/KTipsTest.cpp:12-20, Applications/SegTestApp/SegTest.cpp:35-61) whose add and
// multiply are callable on the device (__host__ __device__). Accumulated under the slot lock.
template <class USR, class NT1, class NT2, class NTO, bool ORD = false>
struct UserSRD {
  using a_t = NT1;
  using b_t = NT2;
  using val_t = NTO;
  using acc_t = NTO;
  static constexpr bool kLocked = true;
  static constexpr bool kOrdered = ORD;  // reference-order accumulation (order_kernel.h)
  static_assert(std::is_trivially_copyable<NTO>::value, "device values must be trivially copyable");
  static __device__ __forceinline__ NTO multiply(const NT1& a, const NT2& b) { return USR::multiply(a, b); }
  static __device__ __forceinline__ NTO add(const NTO& x, const NTO& y) { return USR::add(x, y); }
  static __device__ __forceinline__ acc_t identity() { return acc_t(); }  // never read: first product is stored
  static __device__ __forceinline__ val_t finalize(const acc_t& a) { return a; }
};

}  // namespace cbh
