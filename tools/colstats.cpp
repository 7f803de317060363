// Dev tool: per-column work statistics of R-MAT A^2 (flop_j, nnzC_j, nnzB_j) used to size
// the symbolic/numeric bins. Not part of the product or the tests.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cmath>
#include <thread>
#include <atomic>
extern "C" int cbh_rmat_edges(int, uint64_t, int64_t, int64_t, int64_t*, int64_t*);
extern "C" int cbh_edges_to_csc(int64_t, int64_t, int64_t, const int64_t*, const int64_t*, int, int64_t*, int32_t*, int64_t*, int64_t*);
int main(int argc, char** argv) {
  int scale = atoi(argv[1]); int64_t n = 1LL << scale, M = n * 16;
  std::vector<int64_t> s(M), d(M), cp(n + 1), cnt(M); std::vector<int32_t> ir(M); int64_t nnz;
  cbh_rmat_edges(scale, 0xDECAFBAD, 0, M, s.data(), d.data());
  cbh_edges_to_csc(n, n, M, s.data(), d.data(), 0, cp.data(), ir.data(), cnt.data(), &nnz);
  std::vector<int64_t>().swap(s); std::vector<int64_t>().swap(d);
  std::vector<int64_t> flop(n), nnzc(n), bj(n);
  int nt = std::thread::hardware_concurrency();
  std::atomic<int64_t> next(0);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back([&] {
    std::vector<int64_t> mark(n, -1);
    for (;;) { int64_t j = next.fetch_add(64); if (j >= n) break;
      for (int64_t jj = j; jj < std::min(n, j + 64); ++jj) {
        int64_t f = 0, c = 0;
        for (int64_t p = cp[jj]; p < cp[jj + 1]; ++p) { int64_t k = ir[p];
          for (int64_t q = cp[k]; q < cp[k + 1]; ++q) { ++f; if (mark[ir[q]] != jj) { mark[ir[q]] = jj; ++c; } } }
        flop[jj] = f; nnzc[jj] = c; bj[jj] = cp[jj + 1] - cp[jj]; } } });
  for (auto& x : th) x.join();
  int64_t F = 0, C = 0, nzc = 0; for (int64_t j = 0; j < n; ++j) { F += flop[j]; C += nnzc[j]; nzc += bj[j] > 0; }
  printf("scale %d n %lld nnzA %lld nzcB %lld flops %lld nnzC %lld\n", scale, (long long)n, (long long)nnz, (long long)nzc, (long long)F, (long long)C);
  // histogram by nnzC buckets (powers of 2): columns, flop share, nnzC share, sum bj, sum bj*ceil(nnzc/1024)
  const char* hdr = "bucket(nnzC<=)   cols     flop%%   nnzC%%   maxflop   max_bj   sum_bj*tiles(cap1024)/flop\n";
  printf("%s", hdr);
  for (int b = 0; b <= 24; ++b) {
    int64_t lo = b == 0 ? 0 : (1LL << (b - 1)) + 1, hi = 1LL << b; if (b == 0) hi = 1;
    int64_t cols = 0, f = 0, c = 0, mf = 0, mb = 0; double ov = 0;
    for (int64_t j = 0; j < n; ++j) if (bj[j] > 0 && nnzc[j] >= lo && nnzc[j] <= hi) { ++cols; f += flop[j]; c += nnzc[j]; mf = std::max(mf, flop[j]); mb = std::max(mb, bj[j]); ov += (double)bj[j] * ((nnzc[j] + 1023) / 1024); }
    if (cols) printf("%10lld %8lld %8.3f %8.3f %10lld %8lld %8.4f\n", (long long)hi, (long long)cols, 100.0 * f / F, 100.0 * c / C, (long long)mf, (long long)mb, f ? ov / f : 0);
  }
  printf("by nnzB (b_j) bucket: cols flop%% nnzC%% maxnnzC\n");
  for (int b = 0; b <= 20; ++b) {
    int64_t lo = b == 0 ? 1 : (1LL << (b - 1)) + 1, hi = 1LL << b;
    int64_t cols = 0, f = 0, c = 0, mc = 0;
    for (int64_t j = 0; j < n; ++j) if (bj[j] >= lo && bj[j] <= hi) { ++cols; f += flop[j]; c += nnzc[j]; mc = std::max(mc, nnzc[j]); }
    if (cols) printf("%8lld %8lld %8.3f %8.3f %10lld\n", (long long)hi, (long long)cols, 100.0 * f / F, 100.0 * c / C, (long long)mc);
  }
}
