// Small host-side helpers shared by the C-ABI translation units.
// Thread pool-free parallel_for over std::thread: the library must not depend on
// an OpenMP runtime (the reference's -DTHREADED OpenMP loops are replaced by
// device kernels; host loops here only assemble synthetic inputs).
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <vector>

namespace cbh {

inline int host_threads() {
  static int n = [] {
    const char* e = std::getenv("CBH_HOST_THREADS");
    int v = e ? std::atoi(e) : 0;
    if (v <= 0) {
      // The GPU box exports OMP_NUM_THREADS (its CPU share); honour it.
      const char* o = std::getenv("OMP_NUM_THREADS");
      v = o ? std::atoi(o) : 0;
    }
    if (v <= 0) v = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(v, 64));
  }();
  return n;
}

// Calls f(begin, end, tid) over [0, n) split into contiguous chunks, one per thread.
template <class F>
void parallel_chunks(int64_t n, F&& f) {
  int nt = host_threads();
  if (n < 4096 || nt == 1) {
    f((int64_t)0, n, 0);
    return;
  }
  nt = (int)std::min<int64_t>(nt, n / 1024);
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int t = 0; t < nt; ++t) {
    int64_t b = n * t / nt, e = n * (t + 1) / nt;
    th.emplace_back([&f, b, e, t] { f(b, e, t); });
  }
  for (auto& x : th) x.join();
}

}  // namespace cbh
