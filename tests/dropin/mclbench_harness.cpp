// Config C5 through the C++ driver HipMCL calls (Applications/MCL.cpp:574-577:
// MemEfficientSpGEMM<PTFF, ...>(A, A, phases, prunelimit, select, recover_num, recover_pct,
// kselectVersion, computationKernel, perProcessMem)), on the device-resident overload of
// include/combblas_hip/ParFriendsDev.h: SpParMat over SpDCColsDev, one rank (a 1x1 grid), the stage
// pair planned once (StagePlans), every phase's block pruned on the device by
// MCLPruneRecoverySelect (ParFriends.h:185-353) and the pieces concatenated.
// Built by `make -C oracle ref` (g++, the reference's headers) into oracle/_ref/mclbench_harness.
//
// Input: the library's planted-partition generator (cbh_gen_planted_partition, the same matrix as
// bench_mcl.py --driver lib). Check: `check_cols` sampled columns of the device result against the
// reference's own STOCK MemEfficientSpGEMM + MCLPruneRecoverySelect on those columns of the right
// operand (host SpDCCols, OpenMP kernels; rows exact, values within 1e-12 relative -- the f64 sums
// run in another order). CPU baseline: the same stock call on every `stride`-th column, one warm-up
// and the median of 3, 1 rank x OMP_NUM_THREADS.
//   mclbench_harness <log2n> <deg> <steps> <phases> <check_cols> <cpu_stride>
//     -> one "BENCHC5CPP {json}" line
#include <mpi.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "CombBLAS/CombBLAS.h"
#include "combblas_hip/ParFriendsDev.h"

using namespace combblas;

double cblas_alltoalltime, cblas_allgathertime, cblas_mergeconttime, cblas_transvectime, cblas_localspmvtime;
double mcl_Abcasttime, mcl_Bbcasttime, mcl_localspgemmtime, mcl_multiwaymergetime, mcl_kselecttime,
    mcl_prunecolumntime, mcl_symbolictime, mcl3d_conversiontime, mcl3d_symbolictime, mcl3d_Abcasttime,
    mcl3d_Bbcasttime, mcl3d_SUMMAtime, mcl3d_localspgemmtime, mcl3d_SUMMAmergetime, mcl3d_reductiontime,
    mcl3d_3dmergetime, mcl3d_kselecttime, mcl3d_totaltime, mcl3d_floptime, mcl3d_proc_flop_mean, mcl3d_proc_flop_std,
    mcl3d_proc_nnzc_pre_red, mcl3d_proc_nnzc_post_red;
int64_t mcl_memory, mcl3d_layer_flop, mcl3d_layer_nnzc, mcl3d_nnzc, mcl3d_flop, mcl3d_max_proc_flop,
    mcl3d_max_proc_nnzc_pre_red, mcl3d_max_proc_nnzc_post_red;
MTRand GlobalMT(123);

struct CpuPlusTimes {  // PlusTimesSRing<double,double> on the stock path
  static double id() { return 0; }
  static bool returnedSAID() { return false; }
  static MPI_Op mpi_op() { return MPI_SUM; }
  static double add(const double& a, const double& b) { return a + b; }
  static double multiply(const double& a, const double& b) { return a * b; }
  static void axpy(double a, const double& x, double& y) { y += a * x; }
};
typedef PlusTimesSRing<double, double> PTDD;
typedef SpDCCols<int64_t, double> DCols;
typedef SpParMat<int64_t, double, DCols> PMat;
typedef combblas_hip::SpDCColsDev<int64_t, double> DDev;
typedef SpParMat<int64_t, double, DDev> DMat;

// MCL.cpp's defaults (prunelimit, select, recover_num, recover_pct)
static const double kHard = 1e-4, kPct = 0.9;
static const int64_t kSelect = 1100, kRecover = 1400;

// the columns `cols` of a host block, as an m x cols.size() block (column i = column cols[i])
static DCols* columns_of(DCols& A, const std::vector<int64_t>& cols) {
  Dcsc<int64_t, double>* d = A.GetDCSC();
  std::vector<std::tuple<int64_t, int64_t, double>> t;
  for (size_t i = 0; i < cols.size(); ++i) {
    const int64_t* it = std::lower_bound(d->jc, d->jc + d->nzc, cols[i]);
    if (it == d->jc + d->nzc || *it != cols[i]) continue;
    const int64_t s = it - d->jc;
    for (int64_t p = d->cp[s]; p < d->cp[s + 1]; ++p) t.emplace_back(d->ir[p], (int64_t)i, d->numx[p]);
  }
  auto* owned = new std::tuple<int64_t, int64_t, double>[t.size()];
  std::copy(t.begin(), t.end(), owned);
  SpTuples<int64_t, double> tup((int64_t)t.size(), A.getnrow(), (int64_t)cols.size(), owned, true);
  return new DCols(tup, false);
}

static uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static double median3(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  int provided;
  MPI_Init_thread(&argc, &argv, MPI_THREAD_SERIALIZED, &provided);
  const int log2n = argc > 1 ? std::atoi(argv[1]) : 16;
  const int64_t deg = argc > 2 ? std::atoll(argv[2]) : 100;
  const int steps = argc > 3 ? std::atoi(argv[3]) : 2;
  int phases = argc > 4 ? std::atoi(argv[4]) : 0;  // MCL.cpp's -phases; 0: C's phase blocks within 0.25 of free HBM
  const int ncheck = argc > 5 ? std::atoi(argv[5]) : 100;
  const int64_t stride = argc > 6 ? std::atoll(argv[6]) : 0;
  const int64_t n = int64_t(1) << log2n;
  int rc = 0;
  {
    cbh_ctx* ctx = combblas_hip::context();
    double t0 = MPI_Wtime();
    cbh_mat *Am = nullptr, *Bm = nullptr;
    if (cbh_gen_planted_partition(ctx, n, deg, 7, 0.9, 1.6, &Am) != CBH_OK ||
        cbh_mat_clone(ctx, Am, &Bm) != CBH_OK)
      combblas_hip::die(ctx, CBH_E_INTERNAL, "generator");
    const double tgen = MPI_Wtime() - t0;
    int64_t flops = 0, nnzC = 0, nnzA = 0;
    if (cbh_spgemm_symbolic(ctx, Am, Bm, &flops, &nnzC, nullptr, nullptr) != CBH_OK)
      combblas_hip::die(ctx, CBH_E_INTERNAL, "symbolic");
    cbh_mat_info(Am, nullptr, nullptr, &nnzA, nullptr, nullptr);
    if (phases <= 0) {  // as the Python mirror plans them (parfriends._budget_entries): 12-byte entries
      size_t fr = 0, tot = 0;
      (void)hipMemGetInfo(&fr, &tot);
      const double budget = 0.25 * (double)fr / 12.0;  // (room beside each phase for the output arena)
      phases = std::max(1, (int)std::ceil((double)nnzC / budget));
    }
    std::shared_ptr<CommGrid> grid(new CommGrid(MPI_COMM_WORLD, 1, 1));
    DMat A(new DDev(Am), grid), B(new DDev(Bm), grid);
    auto run = [&]() {
      return MemEfficientSpGEMM<PTDD, double, DDev>(A, B, phases, kHard, kSelect, kRecover, kPct, 1, 1, 0);
    };
    // every step's C is a fresh object initialised from the call (SpParMat's operator= deep-copies
    // the block, SpParMat.cpp:725-738) and freed before the next step (~100 GB at 2^24)
    { DMat Cw = run(); }  // warm-up
    cbh_ctx_synchronize(ctx);
    MPI_Barrier(MPI_COMM_WORLD);
    cbh_kernel_stats_reset(ctx);
    cbh_ctx_enable_timing(ctx, 1);  // per-kernel-class HIP events (the roofline of the line)
    double total = 0;
    for (int s = 0; s < steps; ++s) {
      cbh_ctx_synchronize(ctx);
      t0 = MPI_Wtime();
      {
        DMat Cs = run();
        cbh_ctx_synchronize(ctx);
        total += MPI_Wtime() - t0;
        combblas_hip::memdiag("step returned");
      }
      combblas_hip::memdiag("step result freed");
    }
    const double step_s = total / steps;
    cbh_ctx_enable_timing(ctx, 0);
    std::string ks = "[";
    for (int k = 0; k < CBH_K_NKINDS; ++k) {
      cbh_kernel_stat st{};
      cbh_kernel_stats(ctx, k, &st);
      char buf[160];
      std::snprintf(buf, sizeof(buf), "%s[%.6f, %lld, %.1f]", k ? ", " : "", st.ms, (long long)st.launches, st.alg_bytes);
      ks += buf;
    }
    ks += "]";
    DMat C = run();  // the result the check samples (untimed)
    const int64_t kept = C.getnnz();

    // the check: sampled columns against the stock driver on those columns of B
    std::unique_ptr<DCols> Ah(combblas_hip::download_dcsc<int64_t, double>(A.seq().mat()));
    std::vector<int64_t> sample;
    for (uint64_t i = 0; (int)sample.size() < ncheck; ++i) {
      const int64_t c = (int64_t)(mix64(11 ^ mix64(i)) % (uint64_t)n);
      if (std::find(sample.begin(), sample.end(), c) == sample.end()) sample.push_back(c);
    }
    std::sort(sample.begin(), sample.end());
    PMat Ahp(new DCols(*Ah), grid), Bsp(columns_of(*Ah, sample), grid);
    PMat Cs = MemEfficientSpGEMM<CpuPlusTimes, double, DCols>(Ahp, Bsp, 1, kHard, kSelect, kRecover, kPct, 1, 1, 0);
    Dcsc<int64_t, double>* ds = Cs.seq().getnnz() > 0 ? Cs.seq().GetDCSC() : nullptr;
    int64_t row_bad = 0, val_bad = 0, checked = 0;
    double maxrel = 0;
    for (size_t i = 0; i < sample.size(); ++i) {
      cbh_mat* piece = nullptr;
      if (cbh_mat_col_slice(ctx, C.seq().mat(), sample[i], sample[i] + 1, &piece) != CBH_OK)
        combblas_hip::die(ctx, CBH_E_INTERNAL, "col_slice");
      int64_t pn = 0, pz = 0;
      cbh_mat_info(piece, nullptr, nullptr, &pn, &pz, nullptr);
      std::vector<int32_t> ir(pn);
      std::vector<double> num(pn);
      std::vector<int64_t> cp(pz + 1), jc(pz);
      cbh_mat_copy_out(ctx, piece, cp.data(), jc.data(), ir.data(), num.data(), 0);
      cbh_mat_free(ctx, piece);
      std::vector<std::pair<int64_t, double>> exp;
      if (ds) {
        const int64_t* it = std::lower_bound(ds->jc, ds->jc + ds->nzc, (int64_t)i);
        if (it != ds->jc + ds->nzc && *it == (int64_t)i)
          for (int64_t p = ds->cp[it - ds->jc]; p < ds->cp[it - ds->jc + 1]; ++p) exp.emplace_back(ds->ir[p], ds->numx[p]);
      }
      std::sort(exp.begin(), exp.end());
      ++checked;
      if ((int64_t)exp.size() != pn) {
        ++row_bad;
        continue;
      }
      bool rows_ok = true, vals_ok = true;
      for (int64_t q = 0; q < pn; ++q) {
        if (exp[q].first != ir[q]) rows_ok = false;
        const double rel = std::fabs(exp[q].second - num[q]) / std::max(std::fabs(exp[q].second), 1e-300);
        maxrel = std::max(maxrel, rel);
        if (rel > 1e-12) vals_ok = false;
      }
      row_bad += rows_ok ? 0 : 1;
      val_bad += (rows_ok && !vals_ok) ? 1 : 0;
    }

    // CPU baseline: the stock call on every stride-th column (about 3e8 multiplies by default)
    const int64_t st = stride > 0 ? stride : std::max<int64_t>(1, flops / 300000000);
    std::vector<int64_t> bcols;
    for (int64_t c = 0; c < n; c += st) bcols.push_back(c);
    PMat Bcp(columns_of(*Ah, bcols), grid);
    int64_t cpu_flops = 0;
    {
      Dcsc<int64_t, double>* da = Ah->GetDCSC();
      std::vector<int64_t> colnnz(n, 0);
      for (int64_t c = 0; c < da->nzc; ++c) colnnz[da->jc[c]] = da->cp[c + 1] - da->cp[c];
      Dcsc<int64_t, double>* db = Bcp.seq().GetDCSC();
      for (int64_t p = 0; p < db->nz; ++p) cpu_flops += colnnz[db->ir[p]];
    }
    std::vector<double> cpu;
    int64_t cpu_kept = 0;
    for (int r = 0; r < 4; ++r) {  // one warm-up, then the median of 3
      const double c0 = MPI_Wtime();
      PMat Cc = MemEfficientSpGEMM<CpuPlusTimes, double, DCols>(Ahp, Bcp, 1, kHard, kSelect, kRecover, kPct, 1, 1, 0);
      if (r > 0) cpu.push_back(MPI_Wtime() - c0);
      cpu_kept = Cc.getnnz();
    }
    const char* omp = std::getenv("OMP_NUM_THREADS");
    const bool ok = row_bad == 0 && val_bad == 0 && checked == ncheck;
    std::printf("BENCHC5CPP {\"n\": %lld, \"deg\": %lld, \"nnzA\": %lld, \"flops\": %lld, \"nnzC_unpruned\": %lld, "
                "\"nnz_after_prune\": %lld, \"steps\": %d, \"step_s\": %.6f, \"gen_s\": %.3f, \"phases\": %d, "
                "\"check_cols\": %lld, \"row_mismatches\": %lld, \"value_mismatches\": %lld, \"max_rel\": %.3e, "
                "\"ok\": %s, \"cpu_stride\": %lld, \"cpu_cols\": %lld, \"cpu_flops\": %lld, \"cpu_kept\": %lld, "
                "\"cpu_s\": %.6f, \"cpu_threads\": %s, \"kernel_stats\": %s}\n",
                (long long)n, (long long)deg, (long long)nnzA, (long long)flops, (long long)nnzC, (long long)kept, steps,
                step_s, tgen, phases, (long long)checked, (long long)row_bad, (long long)val_bad, maxrel,
                ok ? "true" : "false", (long long)st, (long long)bcols.size(), (long long)cpu_flops,
                (long long)cpu_kept, median3(cpu), omp ? omp : "0", ks.c_str());
    std::fflush(stdout);
    rc = ok ? 0 : 1;
  }
  MPI_Finalize();
  return rc;
}
