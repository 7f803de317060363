// Test-defined semirings of the drop-in harness, shared by the g++ translation unit that runs the
// reference drivers (dropin_harness.cpp) and the hipcc one that instantiates their device
// kernels (dropin_kernels.hip). add/multiply are callable on the device (CBH_HD).
#pragma once
#include <mpi.h>

#include <cstdint>
#include <ostream>

#ifdef __HIP__
#define CBH_HD __host__ __device__
#else
#define CBH_HD
#endif

// KTipsSR with device-callable add/multiply (ReleaseTests/KTipsTest.cpp:12-20)
struct KTipsDev {
  static bool id() { return false; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_LOR; }
  CBH_HD static bool add(const bool& a, const bool& b) { return a || b; }
  CBH_HD static bool multiply(const bool& a, const bool& b) { return a && b; }
  static void axpy(bool a, const bool& x, bool& y) { y = add(y, multiply(a, x)); }
};
struct KTipsCpu {  // the same semiring on the stock path
  static bool id() { return false; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_LOR; }
  static bool add(const bool& a, const bool& b) { return a || b; }
  static bool multiply(const bool& a, const bool& b) { return a && b; }
  static void axpy(bool a, const bool& x, bool& y) { y = add(y, multiply(a, x)); }
};

// a two-field struct value: (smallest, largest) product reaching each output
struct MinMax {
  int64_t lo = 0, hi = 0;
  bool operator==(const MinMax& o) const { return lo == o.lo && hi == o.hi; }
  friend std::ostream& operator<<(std::ostream& os, const MinMax& m) { return os << "(" << m.lo << "," << m.hi << ")"; }
};
struct MinMaxDev {
  static MinMax id() { return MinMax(); }
  static bool returnedSAID() { return false; }
  CBH_HD static MinMax add(const MinMax& a, const MinMax& b) {
    MinMax r;
    r.lo = a.lo < b.lo ? a.lo : b.lo;
    r.hi = a.hi > b.hi ? a.hi : b.hi;
    return r;
  }
  CBH_HD static MinMax multiply(const int64_t& a, const int64_t& b) {
    MinMax r;
    r.lo = r.hi = a * b - 3 * a + b;  // not symmetric in (a, b): catches swapped operands
    return r;
  }
};
// f64 PlusTimes computed in the REFERENCE'S accumulation order on the device (reference_order,
// HipSpGEMMDevice.h -> device/order_kernel.h): with non-dyadic values the sums must still equal the
// stock path's bit for bit
struct PTOrdDev {
  static double id() { return 0.0; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_SUM; }
  CBH_HD static double add(const double& a, const double& b) { return a + b; }
  CBH_HD static double multiply(const double& a, const double& b) { return a * b; }
  static void axpy(double a, const double& x, double& y) { y += a * x; }
};
struct PTOrdCpu {
  static double id() { return 0.0; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_SUM; }
  static double add(const double& a, const double& b) { return a + b; }
  static double multiply(const double& a, const double& b) { return a * b; }
  static void axpy(double a, const double& x, double& y) { y += a * x; }
};
// Select2ndSRing<int64,int64,int64> (Semirings.h:143-163) on the stock path: add(x, y) = y
struct Select2ndCpu {
  static int64_t id() { return 0; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_MAX; }
  static int64_t add(const int64_t&, const int64_t& b) { return b; }
  static int64_t multiply(const int64_t&, const int64_t& b) { return b; }
  static void axpy(int64_t a, const int64_t& x, int64_t& y) { y = multiply(a, x); }
};
// an UNMARKED user semiring whose add is neither commutative nor associative, over non-dyadic
// doubles: the device path must fold it in the reference's order by default (HipSpGEMMDevice.h)
struct AffineDev {
  static double id() { return 0.0; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_SUM; }
  CBH_HD static double add(const double& a, const double& b) { return 0.75 * a + b; }
  CBH_HD static double multiply(const double& a, const double& b) { return a * b - 0.125 * b; }
};
struct AffineCpu {
  static double id() { return 0.0; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_SUM; }
  static double add(const double& a, const double& b) { return 0.75 * a + b; }
  static double multiply(const double& a, const double& b) { return a * b - 0.125 * b; }
};
namespace combblas_hip {
template <>
struct reference_order<PTOrdDev> : std::true_type {};
template <>
struct arrival_order_ok<MinMaxDev> : std::true_type {};  // min / max per field: order-free (opt-in)
}  // namespace combblas_hip

struct MinMaxCpu {
  static MinMax id() { return MinMax(); }
  static bool returnedSAID() { return false; }
  static MinMax add(const MinMax& a, const MinMax& b) { return MinMaxDev::add(a, b); }
  static MinMax multiply(const int64_t& a, const int64_t& b) { return MinMaxDev::multiply(a, b); }
};

