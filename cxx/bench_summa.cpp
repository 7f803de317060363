// bench_summa -- the N-GPU line of bench.py through the C++ host path north_star names: the
// reference's own distributed types (SpParMat / SpParMat3D) over device-resident blocks
// (combblas_hip::SpDCColsDev), whose driver calls resolve to the device overloads of
// include/combblas_hip/SpParMatDev.h and ParFriendsDev.h (RCCL broadcasts, fiber exchange).
//
//   mpirun -np P bench_summa <scale> <steps> <warmup> [phases]
//
// P square (1, 4, 9): 2D SUMMA on a sqrt(P) x sqrt(P) grid. With one phase the step is the
//   reference's PSpGEMM<PlusTimesSRing<double,double>> -> Mult_AnXBn_Synch (ParFriends.h:1004-1108);
//   when C does not fit it is MemEfficientSpGEMM's phase loop (StagePlans) without the prune.
// P = L * q^2 otherwise (2 = 1x1x2, 8 = 2x2x2): 3D SUMMA, the layer SUMMA + fiber reduce-scatter of
//   Mult_AnXBn_SUMMA3D (ParFriends.h:2918-3208) in MemEfficientSpGEMM3D's phase layout (a scale-22
//   layer product is ~178 GB per rank at P = 2).
// phases 0 (default): planned once, before the timed region, from the exact nnz of the stage plans.
// Input: the packed Graph500 R-MAT of the reference (DistEdgeList::GenGraph500Data, scramble,
// edge factor 16; values = edge multiplicities as double), A and B separate copies.
// Timing: `warmup` untimed steps, then exactly `steps` steps bracketed by device synchronize +
// MPI_Barrier, max over ranks. Then an untimed verification (verify_product): nnz, value sum and
// the reference's order-sensitive digest of the whole product assembled from the ranks' pieces.
// Rank 0 prints one JSON line.
#include <mpi.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
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

typedef PlusTimesSRing<double, double> PTDD;
typedef SpDCCols<int64_t, double> DCols;
typedef SpParMat<int64_t, double, DCols> PMat;
typedef SpParMat3D<int64_t, double, DCols> PMat3D;
typedef combblas_hip::SpDCColsDev<int64_t, double> DDev;
typedef SpParMat<int64_t, double, DDev> DMat;
typedef SpParMat3D<int64_t, double, DDev> DMat3D;

static bool is_square(int p) {
  const int r = (int)std::lround(std::sqrt((double)p));
  return r * r == p;
}

// The R-MAT input on a gr x gc grid of MPI_COMM_WORLD. DistEdgeList and SpParMat(DEL) need a square
// world (CommGrid.cpp:45-52), so for other worlds every rank generates the whole matrix on
// MPI_COMM_SELF and keeps its block (SpParMat::Owner's split; local ids).
static PMat make_input(int scale, int gr, int gc) {
  double init[4] = {.57, .19, .19, .05};
  if (gr == gc) {
    DistEdgeList<int64_t>* DEL = new DistEdgeList<int64_t>();
    DEL->GenGraph500Data(init, scale, 16, true, true);
    SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>> G(*DEL, false);
    delete DEL;
    return PMat(G);
  }
  MPI_Comm self = MPI_COMM_SELF;
  DistEdgeList<int64_t>* DEL = new DistEdgeList<int64_t>(self);
  DEL->GenGraph500Data(init, scale, 16, true, true);
  SpParMat<int64_t, int64_t, SpDCCols<int64_t, int64_t>> G(*DEL, false);
  delete DEL;
  int myrank;
  MPI_Comm_rank(MPI_COMM_WORLD, &myrank);
  const int64_t m = G.getnrow(), n = G.getncol();
  const int pr = myrank / gc, pc = myrank % gc;
  const int64_t rper = m / gr, cper = n / gc;
  const int64_t r0 = pr * rper, r1 = pr == gr - 1 ? m : r0 + rper;
  const int64_t c0 = pc * cper, c1 = pc == gc - 1 ? n : c0 + cper;
  std::vector<std::tuple<int64_t, int64_t, double>> t;
  auto& S = G.seq();
  for (auto colit = S.begcol(); colit != S.endcol(); ++colit) {
    const int64_t c = colit.colid();
    if (c < c0 || c >= c1) continue;
    for (auto nzit = S.begnz(colit); nzit != S.endnz(colit); ++nzit)
      if (nzit.rowid() >= r0 && nzit.rowid() < r1) t.emplace_back(nzit.rowid() - r0, c - c0, (double)nzit.value());
  }
  auto* owned = new std::tuple<int64_t, int64_t, double>[t.size()];  // SpTuples delete[]s its array
  std::copy(t.begin(), t.end(), owned);
  SpTuples<int64_t, double> tup((int64_t)t.size(), r1 - r0, c1 - c0, owned, true);
  std::shared_ptr<CommGrid> grid(new CommGrid(MPI_COMM_WORLD, gr, gc));
  return PMat(new DCols(tup, false), grid);
}

// A final piece of this rank's share of C: the block and the offset of its first column inside the
// rank's column range (2D: the rank's block of C; 3D: its fiber chunk of the layer block)
typedef std::function<void(cbh_mat*, int64_t)> Consumer;

// phases such that every phase's partials and its merge / exchange output (3 x 12 bytes per
// entry of the largest local product) fit in half the free HBM of the tightest rank
static int plan_phases(int64_t local_nnz) {
  int64_t gnnz = 0;
  MPI_Allreduce(&local_nnz, &gnnz, 1, MPI_INT64_T, MPI_MAX, MPI_COMM_WORLD);
  int64_t live = 0, cached = 0, fr = 0, tot = 0;
  cbh_ctx_memory(combblas_hip::context(), &live, &cached, &fr, &tot);
  double budget = 0.5 * (double)(fr + cached), gb = 0;
  MPI_Allreduce(&budget, &gb, 1, MPI_DOUBLE, MPI_MIN, MPI_COMM_WORLD);
  return std::max(1, (int)std::ceil(3.0 * 12.0 * (double)gnnz / gb));
}

// one step of the phased driver: the SUMMA stage blocks broadcast and every stage pair planned once
// (StagePlans; the symbolic pass is inside the step), then per phase the numeric pass of its
// columns with the stage partials merged (2D: MemEfficientSpGEMM's loop, ParFriends.h:449-730,
// without the prune) or the layer partial fiber-reduce-scattered (3D: MemEfficientSpGEMM3D's loop,
// :3214-3705 -- phase p = piece p of each of the L column chunks of B's layer block).
static void phased_step(DDev& Aloc, CommGrid* GA, DDev& Bloc, CommGrid* GB, CommGrid3D* g3, const std::vector<int64_t>& div3,
                        int& phases, const Consumer& consume) {
  const cbh_semiring sr = combblas_hip::semiring_traits<PTDD>::code;
  const int dt = combblas_hip::dtype_of<double>::value;
  combblas_hip::StagePlans<int64_t, double, double> SP(Aloc, GA, Bloc, GB);
  if (phases <= 0) phases = plan_phases(SP.nnz);
  if (!g3) {
    const int64_t n = Bloc.getncol();
    const auto cuts = phases == 1 ? std::vector<int64_t>{0, n}
                                  : combblas_hip::balanced_cuts(SP.col_nnz(n, SP.GridC->GetColWorld()), phases);
    for (size_t p = 0; p + 1 < cuts.size(); ++p) consume(SP.piece(sr, dt, 8, cuts[p], cuts[p + 1]), cuts[p]);
    return;
  }
  const int L = (int)div3.size(), me = g3->GetRankInFiber();
  std::vector<std::vector<int64_t>> piece(L);
  int64_t c0 = 0;
  for (int c = 0; c < L; ++c) {
    piece[c] = combblas_hip::colsplit_cuts(div3[c], phases);
    for (auto& x : piece[c]) x += c0;
    c0 += div3[c];
  }
  // phase p's fiber exchange (communication stream) overlaps phase p+1's products (context
  // stream): MemEfficientSpGEMM3D's schedule in ParFriendsDev.h
  std::unique_ptr<combblas_hip::FiberExchange> inflight;
  int inflight_p = -1;
  for (int p = 0; p < phases; ++p) {
    std::vector<cbh_mat*> parts;
    std::vector<int64_t> lb(L);
    for (int c = 0; c < L; ++c) {
      parts.push_back(SP.piece(sr, dt, 8, piece[c][p], piece[c][p + 1]));
      lb[c] = piece[c][p + 1] - piece[c][p];
    }
    combblas_hip::trace("products issued", p);
    cbh_mat* P = combblas_hip::col_concat(parts);
    if (inflight) {
      consume(combblas_hip::fiber_exchange_finish(*inflight), piece[me][inflight_p] - piece[me][0]);
      combblas_hip::trace("exchange merged", inflight_p);
    }
    inflight.reset(new combblas_hip::FiberExchange(
        combblas_hip::fiber_exchange_start(sr, P, lb, g3->GetFiberWorld(), dt, 8)));
    inflight_p = p;
    combblas_hip::trace("exchange posted", p);
  }
  if (inflight) {
    consume(combblas_hip::fiber_exchange_finish(*inflight), piece[me][inflight_p] - piece[me][0]);
    combblas_hip::trace("exchange merged", inflight_p);
  }
}

static int64_t exscan_i64(int64_t v, MPI_Comm comm) {
  int64_t out = 0;
  MPI_Exscan(&v, &out, 1, MPI_INT64_T, MPI_SUM, comm);
  int r = 0;
  MPI_Comm_rank(comm, &r);
  return r == 0 ? 0 : out;
}

// Where this rank's share of C sits in the whole product: the first global row and column of its
// column range, its column count, and the communicator of the ranks holding the same columns
// (ordered by their rows: the processor column of the 2D grid, or of the layer grid for one fiber
// chunk in 3D)
struct Share {
  int64_t row_off = 0, col_off = 0, ncols = 0;
  MPI_Comm colcomm = MPI_COMM_NULL;
};
static Share share_of(DDev& Aloc, CommGrid* GA, DDev& Bloc, CommGrid* GB, CommGrid3D* g3, const std::vector<int64_t>& div3) {
  Share s;
  s.row_off = exscan_i64(Aloc.getnrow(), GA->GetColWorld());  // C's rows are A's block rows
  s.col_off = exscan_i64(Bloc.getncol(), GB->GetRowWorld());
  s.ncols = Bloc.getncol();
  int color = GB->GetRankInProcRow();
  if (g3) {
    const int me = g3->GetRankInFiber(), L = (int)div3.size();
    for (int c = 0; c < me; ++c) s.col_off += div3[c];
    s.ncols = div3[me];
    color = color * L + me;
  }
  // ranks with the same column range: same processor column (and fiber chunk); key = row offset
  MPI_Comm_split(MPI_COMM_WORLD, color, (int)std::min<int64_t>(s.row_off, INT32_MAX), &s.colcomm);
  return s;
}

// The reference's order-sensitive digest of the WHOLE product from the distributed pieces
// (tests/golden/make_golden_s22.py's definition; cbh_mat_checksum_global): every entry's position
// in C's global DCSC order is (entries of the global columns before its column) + (entries of its
// column in the row ranges above this rank's) + (its index in the piece's column). Pass 1 counts
// the entries per column of this rank's range, the collective sums place every column's first
// entry, pass 2 digests the pieces of a second run of the product.
struct Verify {
  int64_t nnz = 0;
  double vsum = 0;
  uint64_t digest = 0;
};
static Verify verify_product(const std::function<void(const Consumer&)>& product, const Share& sh) {
  cbh_ctx* ctx = combblas_hip::context();
  Verify v;
  std::vector<int64_t> cnt((size_t)sh.ncols, 0);
  product([&](cbh_mat* M, int64_t rel) {
    DDev blk(M);  // frees the piece
    const int64_t nzc = blk.getnzc();
    v.nnz += blk.getnnz();
    if (blk.getnnz() == 0) return;
    double vs = 0;
    uint64_t dg = 0;
    int rc = cbh_mat_checksum(ctx, M, &vs, &dg);
    if (rc != CBH_OK) combblas_hip::die(ctx, rc, "cbh_mat_checksum");
    v.vsum += vs;
    std::vector<int64_t> cp((size_t)nzc + 1), jc((size_t)nzc);
    rc = cbh_mat_copy_out(ctx, M, cp.data(), jc.data(), nullptr, nullptr, 0);
    if (rc != CBH_OK) combblas_hip::die(ctx, rc, "cbh_mat_copy_out");
    for (int64_t k = 0; k < nzc; ++k) cnt[(size_t)(rel + jc[k])] += cp[k + 1] - cp[k];
  });
  // column starts: rows above (exclusive scan over the column communicator), column totals, and the
  // entries of every column range left of this one (one leader per range)
  std::vector<int64_t> above((size_t)sh.ncols, 0), tot((size_t)sh.ncols, 0);
  int crank = 0;
  MPI_Comm_rank(sh.colcomm, &crank);
  MPI_Exscan(cnt.data(), above.data(), (int)sh.ncols, MPI_INT64_T, MPI_SUM, sh.colcomm);
  if (crank == 0) std::fill(above.begin(), above.end(), 0);
  MPI_Allreduce(cnt.data(), tot.data(), (int)sh.ncols, MPI_INT64_T, MPI_SUM, sh.colcomm);
  int64_t range_total = 0;
  for (int64_t t : tot) range_total += t;
  int np = 1;
  MPI_Comm_size(MPI_COMM_WORLD, &np);
  int64_t mine[3] = {sh.col_off, range_total, crank == 0 ? 1 : 0};
  std::vector<int64_t> all(3 * (size_t)np);
  MPI_Allgather(mine, 3, MPI_INT64_T, all.data(), 3, MPI_INT64_T, MPI_COMM_WORLD);
  int64_t base = 0;
  for (int r = 0; r < np; ++r)
    if (all[3 * r + 2] && all[3 * r] < sh.col_off) base += all[3 * r + 1];
  std::vector<int64_t> start((size_t)sh.ncols);
  for (int64_t j = 0; j < sh.ncols; ++j) {
    start[(size_t)j] = base + above[(size_t)j];
    base += tot[(size_t)j];
  }
  product([&](cbh_mat* M, int64_t rel) {
    DDev blk(M);
    const int64_t nzc = blk.getnzc();
    if (blk.getnnz() == 0) return;
    std::vector<int64_t> jc((size_t)nzc), pos((size_t)nzc);
    int rc = cbh_mat_copy_out(ctx, M, nullptr, jc.data(), nullptr, nullptr, 0);
    if (rc != CBH_OK) combblas_hip::die(ctx, rc, "cbh_mat_copy_out");
    for (int64_t k = 0; k < nzc; ++k) pos[(size_t)k] = start[(size_t)(rel + jc[k])];
    double vs = 0;
    uint64_t dg = 0;
    rc = cbh_mat_checksum_global(ctx, M, sh.row_off, sh.col_off + rel, pos.data(), &vs, &dg);
    if (rc != CBH_OK) combblas_hip::die(ctx, rc, "cbh_mat_checksum_global");
    v.digest += dg;
  });
  return v;
}

int main(int argc, char** argv) {
  int provided;
  MPI_Init_thread(&argc, &argv, MPI_THREAD_SERIALIZED, &provided);
  const int scale = argc > 1 ? std::atoi(argv[1]) : 18;
  const int steps = argc > 2 ? std::atoi(argv[2]) : 3;
  const int warmup = argc > 3 ? std::atoi(argv[3]) : 1;
  int phases = argc > 4 ? std::atoi(argv[4]) : 0;  // 0: planned from the exact nnz
  int myrank, nprocs;
  MPI_Comm_rank(MPI_COMM_WORLD, &myrank);
  MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
  {  // every CombBLAS object must be destroyed before MPI_Finalize
    int layers = 1;
    while (nprocs % layers || !is_square(nprocs / layers)) ++layers;  // 2 -> 2 layers of 1x1, 8 -> 2 of 2x2
    const bool twod = layers == 1;
    int gr = (int)std::lround(std::sqrt((double)nprocs)), gc = gr;
    if (!twod) {  // the 2D input grid the 3D constructor redistributes from: 2 -> 1 x 2, 8 -> 2 x 4
      gr = (int)std::lround(std::sqrt((double)(nprocs / 2)));
      gc = nprocs / gr;
    }
    const double tg = MPI_Wtime();
    PMat A = make_input(scale, gr, gc), B = make_input(scale, gr, gc);
    std::unique_ptr<DMat> Ad, Bd;
    std::unique_ptr<DMat3D> A3d, B3d;
    std::vector<int64_t> div3;
    char grid[96];
    if (twod) {
      Ad.reset(new DMat(combblas_hip::to_device(A)));
      Bd.reset(new DMat(combblas_hip::to_device(B)));
      std::snprintf(grid, sizeof(grid), "2D SUMMA %dx%d", gr, gc);
    } else {
      PMat3D A3(A, layers, true, false), B3(B, layers, false, false);
      A3d.reset(new DMat3D(combblas_hip::to_device(A3)));
      B3d.reset(new DMat3D(combblas_hip::to_device(B3)));
      std::vector<int64_t> d;
      B3d->CalculateColSplitDistributionOfLayer(d);
      div3.assign(d.begin(), d.end());
      const int q = (int)std::lround(std::sqrt((double)(nprocs / layers)));
      std::snprintf(grid, sizeof(grid), "3D SUMMA %dx%dx%d", q, q, layers);
    }
    A.FreeMemory();
    B.FreeMemory();
    cbh_ctx_synchronize(combblas_hip::context());
    const double setup_s = MPI_Wtime() - tg;
    // one product. 2D with one phase: the reference's PSpGEMM itself (-> the device
    // Mult_AnXBn_Synch of SpParMatDev.h); otherwise the phased loop above
    auto product = [&](const Consumer& consume) {
      if (twod && phases == 1) {
        DMat C = PSpGEMM<PTDD>(*Ad, *Bd);
        consume(C.seq().release(), 0);
        return;
      }
      if (twod)
        return phased_step(Ad->seq(), Ad->getcommgrid().get(), Bd->seq(), Bd->getcommgrid().get(), nullptr, div3,
                           phases, consume);
      return phased_step(*A3d->GetLayerMat()->seqptr(), A3d->GetLayerMat()->getcommgrid().get(),
                         *B3d->GetLayerMat()->seqptr(), B3d->GetLayerMat()->getcommgrid().get(),
                         A3d->getcommgrid3D().get(), div3, phases, consume);
    };
    const Consumer discard = [](cbh_mat* M, int64_t) { cbh_mat_free(combblas_hip::context(), M); };
    if (phases <= 0) {  // plan the phase count once (a symbolic pass), outside the timed region
      std::unique_ptr<combblas_hip::StagePlans<int64_t, double, double>> SP;
      if (twod)
        SP.reset(new combblas_hip::StagePlans<int64_t, double, double>(Ad->seq(), Ad->getcommgrid().get(), Bd->seq(),
                                                                       Bd->getcommgrid().get()));
      else
        SP.reset(new combblas_hip::StagePlans<int64_t, double, double>(
            *A3d->GetLayerMat()->seqptr(), A3d->GetLayerMat()->getcommgrid().get(), *B3d->GetLayerMat()->seqptr(),
            B3d->GetLayerMat()->getcommgrid().get()));
      phases = plan_phases(SP->nnz);  // with the plans (and their stored bitmaps) still resident
      // 3D over RCCL: at least 4 phases, so that all but a quarter of the fiber exchange runs under
      // the next phase's products (one phase would leave the whole exchange exposed)
      if (!twod && !combblas_hip::use_mpi_transport()) phases = std::max(phases, 4);
    }
    if (myrank == 0) std::fprintf(stderr, "[bench_summa] setup %.1f s, %d phase(s); warm-up\n", setup_s, phases);
    for (int w = 0; w < warmup; ++w) product(discard);
    cbh_ctx_synchronize(combblas_hip::context());
    cbh_ctx_enable_timing(combblas_hip::context(), 1);  // per-kind HIP-event totals of the timed steps
    cbh_kernel_stats_reset(combblas_hip::context());
    if (myrank == 0) std::fprintf(stderr, "[bench_summa] %d timed step(s)\n", steps);
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    for (int k = 0; k < steps; ++k) product(discard);
    cbh_ctx_synchronize(combblas_hip::context());
    MPI_Barrier(MPI_COMM_WORLD);
    double dt = (MPI_Wtime() - t0) / std::max(steps, 1), mx = 0;
    MPI_Allreduce(&dt, &mx, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    cbh_ctx_enable_timing(combblas_hip::context(), 0);
    std::string kstats;  // rank 0's kernel classes: {"kind": [ms, launches, alg_bytes], ...}
    {
      static const char* names[CBH_K_NKINDS] = {"sym_large", "sym_small", "num_large", "num_small", "merge_sym",
                                                 "merge_num", "num_dense", "sym_mid", "num_mid", "sym_bmp"};
      char buf[160];
      for (int k = 0; k < CBH_K_NKINDS; ++k) {
        cbh_kernel_stat st{};
        if (cbh_kernel_stats(combblas_hip::context(), k, &st) != CBH_OK || st.launches == 0) continue;
        std::snprintf(buf, sizeof(buf), "%s\"%s\": [%.4f, %lld, %.0f]", kstats.empty() ? "" : ", ", names[k], st.ms,
                      (long long)st.launches, st.alg_bytes);
        kstats += buf;
      }
    }
    if (myrank == 0) std::fprintf(stderr, "[bench_summa] %.1f ms/step; verification step\n", mx * 1e3);
    // verification (untimed, two runs of the product): nnz, value sum and the whole product's digest
    const Share sh = twod ? share_of(Ad->seq(), Ad->getcommgrid().get(), Bd->seq(), Bd->getcommgrid().get(), nullptr, div3)
                          : share_of(*A3d->GetLayerMat()->seqptr(), A3d->GetLayerMat()->getcommgrid().get(),
                                     *B3d->GetLayerMat()->seqptr(), B3d->GetLayerMat()->getcommgrid().get(),
                                     A3d->getcommgrid3D().get(), div3);
    const Verify v = verify_product(product, sh);
    cbh_ctx_synchronize(combblas_hip::context());
    int64_t nnz = 0;
    double vsum = 0;
    MPI_Allreduce(&v.nnz, &nnz, 1, MPI_INT64_T, MPI_SUM, MPI_COMM_WORLD);
    MPI_Allreduce(&v.vsum, &vsum, 1, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD);
    std::vector<uint64_t> digs((size_t)nprocs);  // summed mod 2^64 on rank 0 (MPI_SUM on unsigned may not wrap)
    MPI_Gather(&v.digest, 1, MPI_UINT64_T, digs.data(), 1, MPI_UINT64_T, 0, MPI_COMM_WORLD);
    uint64_t digest = 0;
    for (uint64_t d : digs) digest += d;
    MPI_Comm colcomm = sh.colcomm;
    MPI_Comm_free(&colcomm);
    if (myrank == 0) {
      const char* drv = twod ? (phases == 1 ? "PSpGEMM -> Mult_AnXBn_Synch (SpParMatDev.h)"
                                            : "MemEfficientSpGEMM phase loop without prune (ParFriendsDev.h StagePlans)")
                             : "MemEfficientSpGEMM3D phase loop without prune (layer SUMMA + fiber reduce-scatter)";
      std::printf("{\"ms_per_step\": %.3f, \"steps\": %d, \"warmup\": %d, \"ranks\": %d, \"grid\": \"%s\", "
                  "\"driver\": \"%s\", \"phases\": %d, \"nnzC\": %lld, \"value_sum\": %.1f, \"digest\": \"%llu\", \"setup_s\": %.3f, "
                  "\"transport\": \"%s\", \"kernel_stats_rank0\": {%s}}\n",
                  mx * 1e3, steps, warmup, nprocs, grid, drv, phases, (long long)nnz, vsum, (unsigned long long)digest, setup_s,
                  combblas_hip::use_mpi_transport() ? "mpi (host staged)" : "rccl", kstats.c_str());
      std::fflush(stdout);
    }
  }
  MPI_Finalize();
  return 0;
}
