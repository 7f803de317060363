// Device-side semiring functors, inlined into the SpGEMM/merge kernels as template
// parameters. Each mirrors a reference semiring's static contract (Semirings.h) --
// multiply(a,b) with A's value first (mtSpGEMM.h:401), add(x,y) -- plus what the
// device path needs on top of it:
//   identity()   a TRUE two-sided identity of add, used to pre-fill LDS accumulators
//                (the reference's SR::id() is not always one: SelectMaxSRing::id() is -1).
//   lds_acc()    atomic "acc = add(acc, v)" on an LDS slot (ds_add_f64 / ds_max_i64 / ...).
// val_t is the element type in HBM; acc_t the LDS accumulator type (bool widens to u32
// so it can use ds_or_b32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <limits>

namespace cbh {

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

}  // namespace cbh
