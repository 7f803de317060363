// ParFriendsDev.h -- the reference's PHASED and 3D SpGEMM drivers for device-resident blocks.
//
// Overloads, for SpParMat / SpParMat3D over SpDCColsDev (more specialized than the reference's
// templates, so HipMCL's own calls -- Applications/MCL.cpp:574-577 -- resolve to them):
//   MCLPruneRecoverySelect   ParFriends.h:185-353   whole local block on the device
//                                                   (cbh_mcl_prune_recovery_select), column
//                                                   statistics and Kselect histograms summed over
//                                                   the processor column with ncclAllReduce
//   EstPerProcessNnzSUMMA    ParFriends.h:1243-1340 stage broadcasts + device symbolic pass
//   MemEfficientSpGEMM       ParFriends.h:449-730   the stage blocks broadcast once and every stage
//                                                   pair planned once (StagePlans: one symbolic
//                                                   pass, which also feeds the memory model); per
//                                                   phase the numeric pass of B's ColSplit columns,
//                                                   the stage partials merged, MCLPruneRecoverySelect,
//                                                   the pruned pieces concatenated (ColConcatenate)
//   Mult_AnXBn_SUMMA3D       ParFriends.h:2918-3208 layer SUMMA, then the fiber reduce-scatter
//                                                   (:3097-3183) as device column pieces exchanged
//                                                   with grouped ncclSend / ncclRecv and merged
//   MemEfficientSpGEMM3D     ParFriends.h:3214-3705 B's layer block cut in `layers` chunks, each in
//                                                   `phases` pieces; the layer's stage pairs planned
//                                                   once; phase p = piece p of every chunk: layer
//                                                   numeric pass, fiber reduce-scatter, prune on the
//                                                   layer grid, concatenation
// Every block, stage partial and piece stays in HBM; only sizes (essentials) cross the host.
// COMBBLAS_HIP_COMM=mpi stages the exchanges through host MPI instead of RCCL (test rehearsal of
// several ranks sharing one GPU).
#pragma once

#include <cmath>

#include "CombBLAS/CommGrid3D.h"
#include "CombBLAS/SpParMat3D.h"
#include "SpParMatDev.h"

namespace combblas_hip {

inline cbh_mat* col_slice(const cbh_mat* M, int64_t c0, int64_t c1) {
  cbh_mat* out = nullptr;
  int rc = cbh_mat_col_slice(context(), M, c0, c1, &out);
  if (rc != CBH_OK) die(context(), rc, "cbh_mat_col_slice");
  return out;
}
// ColConcatenate of the blocks, released as they are consumed (peak: the blocks + one output array)
inline cbh_mat* col_concat(std::vector<cbh_mat*>& parts) {
  cbh_mat* out = nullptr;
  int rc = cbh_mat_col_concat_consume(context(), (int)parts.size(), parts.data(), &out);
  if (rc != CBH_OK) die(context(), rc, "cbh_mat_col_concat_consume");
  parts.clear();
  return out;
}
// COMBBLAS_HIP_MEMDIAG=1: the device memory state at the phased drivers' milestones (stderr)
inline bool memdiag_on() {
  static const bool on = std::getenv("COMBBLAS_HIP_MEMDIAG") != nullptr;
  return on;
}
inline void memdiag(const char* where) {
  if (!memdiag_on()) return;
  static double last = 0;
  cbh_ctx_synchronize(context());
  const double now = MPI_Wtime();
  int64_t live = 0, cached = 0, fr = 0, tot = 0;
  cbh_ctx_memory(context(), &live, &cached, &fr, &tot);
  std::printf("[memdiag] %-28s +%8.1f ms  live %.2f GB, cached %.2f GB, device free %.2f of %.2f GB\n", where,
              last > 0 ? (now - last) * 1e3 : 0.0, live / 1e9, cached / 1e9, fr / 1e9, tot / 1e9);
  std::fflush(stdout);
  last = now;
}
// Device bytes one phase of MemEfficientSpGEMM allocates beside its product piece (an upper bound
// read off the library's allocations): the numeric pass's task binning (< 64 B per output entry
// of the piece is generous: a task covers thousands), MCLPruneRecoverySelect's column arrays
// (cbh_mcl_prune_recovery_select: 9 eight-byte words per column) and its three Kselect calls
// (per active column: 4 words, and 256 four-byte digit counts when the columns are reduced over
// a processor column), the merge of per-stage partials (a second piece), plus 2 GB for the
// allocator's size classes and the runtime. Round 5 used a constant 12 GB here.
inline int64_t phase_scratch_bytes(int64_t phase_nnz, int64_t phase_cols, bool merges) {
  const int64_t numeric = phase_nnz / 8;
  const int64_t prune = phase_cols * (9 * 8 + 3 * (4 * 8 + 256 * 4));
  const int64_t merge = merges ? phase_nnz * 12 : 0;
  return numeric + prune + merge + (int64_t(2) << 30);
}
// The output arena's capacity (entries) for a phased call of this context: the room `fit` left
// beside the phase, at most `limit`, but the capacity of the context's previous arena when that
// still fits -- identical requests are served from the allocator's cache by the block the previous
// result freed (C5's C++ line: a smaller second arena could not use the first one's block, and
// re-mapping ~200 GB inside the first timed call cost 5.9 s). Fresh sizes are
// rounded down to 1 GiB of entries so that small changes in free memory repeat the same request.
// Per-context state (round 5 kept a function-static `last_pruned` shared by every call site).
inline int64_t arena_capacity(cbh_ctx* ctx, int64_t fit, int64_t limit) {
  static std::map<const cbh_ctx*, int64_t> prev;
  int64_t cap = std::min(fit, limit);
  if (cap <= 0) return 0;
  auto it = prev.find(ctx);
  if (it != prev.end() && it->second <= cap) return it->second;
  const int64_t g = int64_t(1) << 30;
  if (cap > 2 * g) cap = cap / g * g;
  prev[ctx] = cap;
  return cap;
}
inline std::vector<int64_t> essentials(const cbh_mat* M) {  // {nnz, m, n, nzc}
  int64_t m = 0, n = 0, nnz = 0, nzc = 0;
  cbh_mat_info(M, &m, &n, &nnz, &nzc, nullptr);
  return {nnz, m, n, nzc};
}
// SpDCCols::ColSplit(parts) cuts: (i+1) * (n/parts), the last piece takes the remainder
// phase cuts with an even share of the product's entries (cnt: exact nnz per column): the pieces
// of a phase loop then have nearly one size, so the context allocator serves every phase from the
// block the first one left in its cache (ColSplit's even column counts gave C5 pieces of 44 to
// 58 GB, and each larger one re-mapped its block: 0.5-0.9 s per such phase). C does not depend on
// the cuts.
inline std::vector<int64_t> balanced_cuts(const std::vector<int64_t>& cnt, int parts) {
  const int64_t n = (int64_t)cnt.size();
  int64_t total = 0;
  for (int64_t v : cnt) total += v;
  std::vector<int64_t> c{0};
  int64_t cum = 0, col = 0;
  for (int p = 1; p < parts && col < n; ++p) {
    const int64_t target = (int64_t)((double)total * p / parts);
    while (col < n && cum < target) cum += cnt[(size_t)col++];  // the first column past the share
    if (col <= c.back() && col < n) cum += cnt[(size_t)col++];  // every phase keeps >= 1 column
    if (col >= n) break;
    c.push_back(col);
  }
  c.push_back(n);
  return c;
}
inline bool even_column_cuts() {  // COMBBLAS_HIP_EVEN_CUTS=1: the reference's ColSplit cuts
  const char* e = std::getenv("COMBBLAS_HIP_EVEN_CUTS");
  return e && std::atoi(e) != 0;
}

inline std::vector<int64_t> colsplit_cuts(int64_t n, int parts) {
  std::vector<int64_t> c{0};
  for (int i = 1; i < parts; ++i) c.push_back(i * (n / parts));
  c.push_back(n);
  return c;
}

// in-place sum of a device buffer over an MPI communicator (the cbh_allreduce_fn of
// cbh_mcl_prune_recovery_select): ncclAllReduce on the mirrored RCCL communicator, or host staged
inline int comm_allreduce_sum(void* user, void* buf, int64_t count, int type) {
  MPI_Comm comm = *static_cast<MPI_Comm*>(user);
  hipStream_t s = reinterpret_cast<hipStream_t>(cbh_ctx_stream(context()));
  const size_t esz = type == CBH_REDUCE_F64 ? sizeof(double) : sizeof(uint32_t);
  if (use_mpi_transport()) {
    std::vector<char> h(esz * (size_t)count);
    if (hipMemcpyAsync(h.data(), buf, h.size(), hipMemcpyDeviceToHost, s) != hipSuccess) return CBH_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return CBH_E_HIP;
    MPI_Allreduce(MPI_IN_PLACE, h.data(), (int)count, type == CBH_REDUCE_F64 ? MPI_DOUBLE : MPI_UINT32_T, MPI_SUM, comm);
    if (hipMemcpyAsync(buf, h.data(), h.size(), hipMemcpyHostToDevice, s) != hipSuccess) return CBH_E_HIP;
    return hipStreamSynchronize(s) == hipSuccess ? 0 : CBH_E_HIP;
  }
  ncclComm_t nc = rccl_comm_for(comm);
  return ncclAllReduce(buf, buf, (size_t)count, type == CBH_REDUCE_F64 ? ncclFloat64 : ncclUint32, ncclSum, nc, s) ==
                 ncclSuccess
             ? 0
             : CBH_E_HIP;
}

// MCLPruneRecoverySelect of a device block whose columns are split over `colworld`
inline cbh_mat* mcl_prune_block(const cbh_mat* A, MPI_Comm colworld, double hard, int64_t selectNum,
                                int64_t recoverNum, double recoverPct, cbh_arena* arena = nullptr) {
  int size = 1;
  MPI_Comm_size(colworld, &size);
  MPI_Comm comm = colworld;
  cbh_mat* C = nullptr;
  int rc = cbh_mcl_prune_recovery_select_arena(context(), A, hard, selectNum, recoverNum, recoverPct,
                                               size > 1 ? comm_allreduce_sum : nullptr, &comm, arena, &C);
  if (rc != CBH_OK) die(context(), rc, "cbh_mcl_prune_recovery_select");
  return C;
}

// The fiber reduce-scatter of Mult_AnXBn_SUMMA3D (ParFriends.h:3097-3183) on device blocks: the
// layer partial P is cut into column pieces of widths div[0..L) (ids rebased), piece j goes to
// fiber rank j -- essentials by MPI_Alltoall, the arrays by grouped ncclSend / ncclRecv (host
// staged with COMBBLAS_HIP_COMM=mpi) -- and the L pieces of this rank's chunk are merged
// (MultiwayMergeHash there; the device merge keeps rows sorted). P is freed.
//
// In two halves so that a phase loop can overlap the exchange of phase p with the products of
// phase p+1 (the reference's Mult_AnXBn_Overlap idea, ParFriends.h:1110-1235, applied to the 3D
// drivers' fiber step, :3143-3183): fiber_exchange_start posts the transfers on the communication
// stream (RCCL) behind an event that orders the freshly allocated receive blocks after the context
// stream's work, and returns; fiber_exchange_finish makes the context stream wait for them, frees
// the sent pieces (stream-ordered, after the wait) and merges. The host-staged transport completes
// the exchange inside start (MPI is synchronous here). COMBBLAS_HIP_TRACE=1 prints when each half
// is issued (the rehearsal's evidence of the schedule).
struct FiberExchange {
  cbh_mat* P = nullptr;  // the layer partial: the pieces are views of it (cbh_mat_col_view), freed last
  std::vector<cbh_mat*> send, recv;
  std::vector<int64_t> ress;
  int me = 0, L = 1;
  int64_t width = 0;
  hipEvent_t done = nullptr;
  cbh_semiring sr = CBH_SR_PLUS_TIMES;
  int dtype = CBH_F64;
  int64_t vbytes = 8;
};
inline bool trace_on() {
  static const bool v = [] {
    const char* e = std::getenv("COMBBLAS_HIP_TRACE");
    return e && std::atoi(e) != 0;
  }();
  return v;
}
inline void trace(const char* what, int phase) {
  if (!trace_on()) return;
  int r = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &r);
  std::fprintf(stderr, "[trace] rank %d %.6f %s phase %d\n", r, MPI_Wtime(), what, phase);
}
inline FiberExchange fiber_exchange_start(cbh_semiring sr, cbh_mat* P, const std::vector<int64_t>& div, MPI_Comm fiber,
                                          int dtype, int64_t vbytes) {
  FiberExchange X;
  X.sr = sr;
  X.dtype = dtype;
  X.vbytes = vbytes;
  MPI_Comm_size(fiber, &X.L);
  MPI_Comm_rank(fiber, &X.me);
  const int L = X.L, me = X.me;
  X.width = div[me];
  X.send.assign(L, nullptr);
  X.recv.assign(L, nullptr);
  // the pieces are views of P (rows and values not copied: a scale-22 layer partial at 1x1x2 is
  // ~180 GB); P lives until the exchange is finished and merged
  X.P = P;
  int64_t c0 = 0;
  for (int j = 0; j < L; ++j) {
    int rc = cbh_mat_col_view(context(), P, c0, c0 + div[j], &X.send[j]);
    if (rc != CBH_OK) die(context(), rc, "cbh_mat_col_view");
    c0 += div[j];
  }
  std::vector<int64_t> sess(4 * (size_t)L);
  X.ress.assign(4 * (size_t)L, 0);
  for (int j = 0; j < L; ++j) {
    const auto e = essentials(X.send[j]);
    std::copy(e.begin(), e.end(), sess.begin() + 4 * j);
  }
  MPI_Alltoall(sess.data(), 4, MPI_INT64_T, X.ress.data(), 4, MPI_INT64_T, fiber);
  X.recv[me] = X.send[me];
  X.send[me] = nullptr;
  for (int j = 0; j < L; ++j) {
    if (j == me) continue;
    int rc = cbh_mat_create(context(), X.ress[4 * j + 1], X.ress[4 * j + 2], X.ress[4 * j], X.ress[4 * j + 3],
                            (cbh_dtype)dtype, vbytes, &X.recv[j]);
    if (rc != CBH_OK) die(context(), rc, "cbh_mat_create");
  }
  struct Arrs {
    void* p[4];
    size_t b[4];
  };
  auto arrays = [&](cbh_mat* M) {
    const int64_t *cp, *jc;
    const int32_t* ir;
    const void* num;
    cbh_mat_device_arrays(M, &cp, &jc, &ir, &num);
    const auto e = essentials(M);
    return Arrs{{const_cast<int64_t*>(cp), const_cast<int64_t*>(jc), const_cast<int32_t*>(ir), const_cast<void*>(num)},
                {sizeof(int64_t) * (size_t)(e[3] + 1), sizeof(int64_t) * (size_t)e[3], sizeof(int32_t) * (size_t)e[0],
                 (size_t)vbytes * (size_t)e[0]}};
  };
  hipStream_t s = reinterpret_cast<hipStream_t>(cbh_ctx_stream(context()));
  if (use_mpi_transport()) {  // host-staged pairwise exchange (synchronous)
    for (int d = 1; d < L; ++d) {
      const int to = (me + d) % L, from = (me - d + L) % L;
      const Arrs a = arrays(X.send[to]), b = arrays(X.recv[from]);
      for (int k = 0; k < 4; ++k) {
        std::vector<char> hs(a.b[k]), hr(b.b[k]);
        if (a.b[k]) {
          hip_check(hipMemcpyAsync(hs.data(), a.p[k], a.b[k], hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
          hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
        }
        mpi_sendrecv_bytes(hs.data(), a.b[k], to, hr.data(), b.b[k], from, k, fiber);
        if (b.b[k]) {
          hip_check(hipMemcpyAsync(b.p[k], hr.data(), b.b[k], hipMemcpyHostToDevice, s), "hipMemcpyAsync");
          hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
        }
      }
    }
  } else if (L > 1) {
    ncclComm_t nc = rccl_comm_for(fiber);
    hipStream_t cs = comm_stream();
    hipEvent_t ready;
    hip_check(hipEventCreateWithFlags(&ready, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventRecord(ready, s), "hipEventRecord");  // the slices and receive blocks exist
    hip_check(hipStreamWaitEvent(cs, ready, 0), "hipStreamWaitEvent");
    hip_check(hipEventDestroy(ready), "hipEventDestroy");
    rccl_check(ncclGroupStart(), "ncclGroupStart");
    for (int j = 0; j < L; ++j) {
      if (j == me) continue;
      const Arrs a = arrays(X.send[j]), b = arrays(X.recv[j]);
      for (int k = 0; k < 4; ++k) {
        if (a.b[k]) rccl_check(ncclSend(a.p[k], a.b[k], ncclUint8, j, nc, cs), "ncclSend");
        if (b.b[k]) rccl_check(ncclRecv(b.p[k], b.b[k], ncclUint8, j, nc, cs), "ncclRecv");
      }
    }
    rccl_check(ncclGroupEnd(), "ncclGroupEnd");
    hip_check(hipEventCreateWithFlags(&X.done, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventRecord(X.done, cs), "hipEventRecord");
  }
  return X;
}
inline cbh_mat* fiber_exchange_finish(FiberExchange& X) {
  if (X.done) {  // the context stream waits for the transfers; the sent slices are freed after them
    hip_check(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(cbh_ctx_stream(context())), X.done, 0),
              "hipStreamWaitEvent");
    hip_check(hipEventDestroy(X.done), "hipEventDestroy");
    X.done = nullptr;
  }
  for (cbh_mat* m : X.send)
    if (m) cbh_mat_free(context(), m);
  X.send.clear();
  cbh_mat* own = X.recv[X.me];  // a view of P
  std::vector<cbh_mat*> nonempty;
  for (int j = 0; j < X.L; ++j)
    if (essentials(X.recv[j])[0] > 0) nonempty.push_back(X.recv[j]);
  cbh_mat* C = nullptr;
  if (nonempty.empty()) {
    int rc = cbh_mat_create(context(), X.ress[4 * X.me + 1], X.width, 0, 0, (cbh_dtype)X.dtype, X.vbytes, &C);
    if (rc != CBH_OK) die(context(), rc, "cbh_mat_create");
  } else if (nonempty.size() == 1 && nonempty[0] != own) {
    C = nonempty[0];  // a received block: owned
  } else if (nonempty.size() == 1) {
    int rc = cbh_mat_clone(context(), own, &C);  // the view must not outlive P
    if (rc != CBH_OK) die(context(), rc, "cbh_mat_clone");
  } else {
    // (cbh_merge of the pieces, 16 at a time as merge_all, without freeing the inputs here)
    std::vector<cbh_mat*> cur(nonempty.begin(), nonempty.end());
    std::vector<cbh_mat*> made;
    while (cur.size() > 1) {
      std::vector<cbh_mat*> next;
      for (size_t g = 0; g < cur.size(); g += 16) {
        const size_t k = std::min<size_t>(16, cur.size() - g);
        if (k == 1) {
          next.push_back(cur[g]);
          continue;
        }
        cbh_mat* r = nullptr;
        int rc = cbh_merge(context(), X.sr, (int)k, cur.data() + g, &r);
        if (rc != CBH_OK) die(context(), rc, "cbh_merge");
        made.push_back(r);
        next.push_back(r);
      }
      cur.swap(next);
    }
    C = cur[0];
    for (cbh_mat* m : made)
      if (m != C) cbh_mat_free(context(), m);
  }
  for (int j = 0; j < X.L; ++j)
    if (X.recv[j] != C) cbh_mat_free(context(), X.recv[j]);
  X.recv.clear();
  cbh_mat_free(context(), X.P);  // (stream-ordered after the merge that read its views)
  X.P = nullptr;
  return C;
}
inline cbh_mat* fiber_reduce_scatter(cbh_semiring sr, cbh_mat* P, const std::vector<int64_t>& div, MPI_Comm fiber,
                                     int dtype, int64_t vbytes) {
  FiberExchange X = fiber_exchange_start(sr, P, div, fiber, dtype, vbytes);
  return fiber_exchange_finish(X);
}

// The SUMMA stage pairs of C = A * B for a phase loop. The reference re-broadcasts the stage blocks
// and re-multiplies them in every phase (ParFriends.h:560-669 inside its phase loop); here every
// stage block is broadcast ONCE and kept in HBM. Default (round 5): the stages' blocks are then
// concatenated into this rank's strips A(r, :) = [A_0 ... A_{s-1}] and B(:, c) = [B_0; ...; B_{s-1}]
// and planned as ONE product -- sum_i A_i B_i in one pass, no stage partial written and no
// MultiwayMerge (the Python drivers' form; C is the same matrix, f64 sums in
// another order). COMBBLAS_HIP_STAGE_PLANS=per-stage keeps one plan per stage pair and merges the
// stage partials per phase, as the reference does. Either way a phase runs only the numeric pass of
// its columns (cbh_plan_spgemm_slots) and the memory model reads the exact nnz off the plans
// instead of a separate EstPerProcessNnzSUMMA pass.
inline bool per_stage_plans() {
  static const bool v = [] {
    const char* e = std::getenv("COMBBLAS_HIP_STAGE_PLANS");
    return e && std::strcmp(e, "per-stage") == 0;
  }();
  return v;
}
template <class IU, class NU1, class NU2>
class StagePlans {
 public:
  StagePlans(SpDCColsDev<IU, NU1>& Aloc, combblas::CommGrid* GA, SpDCColsDev<IU, NU2>& Bloc, combblas::CommGrid* GB) {
    int dummy;
    GridC = ProductGrid(GA, GB, stages, dummy, dummy);  // found by ADL (a friend of CommGrid)
    m = Aloc.getnrow();
    auto Asizes = GetSetSizes(Aloc, GA->GetRowWorld());
    auto Bsizes = GetSetSizes(Bloc, GB->GetColWorld());
    const int Aself = GA->GetRankInProcRow(), Bself = GB->GetRankInProcCol();
    const bool concat = stages > 1 && !per_stage_plans();
    // per-stage plans stay resident through the phase loop: their stored dense-task bitmaps share
    // ONE budget (0.4 of the device) instead of taking up to 0.4 each
    if (stages > 1 && !concat) cbh_ctx_set_bitmap_fraction(context(), 0.4 / stages);
    std::vector<SpDCColsDev<IU, NU1>*> As;
    std::vector<SpDCColsDev<IU, NU2>*> Bs;
    for (int i = 0; i < stages; ++i) {
      SpDCColsDev<IU, NU1>* Ai = &Aloc;
      SpDCColsDev<IU, NU2>* Bi = &Bloc;
      if (i != Aself) {
        Ahold.emplace_back(new SpDCColsDev<IU, NU1>());
        Ai = Ahold.back().get();
      }
      if (i != Bself) {
        Bhold.emplace_back(new SpDCColsDev<IU, NU2>());
        Bi = Bhold.back().get();
      }
      BCastMatrix(GridC->GetRowWorld(), *Ai, Asizes[i], i);
      BCastMatrix(GridC->GetColWorld(), *Bi, Bsizes[i], i);
      if (concat) {
        As.push_back(Ai);
        Bs.push_back(Bi);
      } else {
        add_plan(*Ai, *Bi);
      }
    }
    if (concat) {
      // A strip: the stage blocks side by side; B strip: stacked, as the transpose of the side-by-side
      // transposes (rows stay ascending in every column)
      std::vector<const cbh_mat*> ap;
      for (auto* a : As) ap.push_back(a->mat());
      cbh_mat* ac = nullptr;
      int rc = cbh_mat_col_concat(context(), (int)ap.size(), ap.data(), &ac);
      if (rc != CBH_OK) die(context(), rc, "cbh_mat_col_concat");
      Acat.reset(new SpDCColsDev<IU, NU1>(ac));
      std::vector<cbh_mat*> bt;
      for (auto* b : Bs) {
        cbh_mat* t = nullptr;
        rc = cbh_transpose(context(), b->mat(), &t);
        if (rc != CBH_OK) die(context(), rc, "cbh_transpose");
        bt.push_back(t);
      }
      cbh_mat *btc = nullptr, *bc = nullptr;
      rc = cbh_mat_col_concat(context(), (int)bt.size(), const_cast<const cbh_mat* const*>(bt.data()), &btc);
      if (rc != CBH_OK) die(context(), rc, "cbh_mat_col_concat");
      for (cbh_mat* t : bt) cbh_mat_free(context(), t);
      rc = cbh_transpose(context(), btc, &bc);
      if (rc != CBH_OK) die(context(), rc, "cbh_transpose");
      cbh_mat_free(context(), btc);
      Bcat.reset(new SpDCColsDev<IU, NU2>(bc));
      Ahold.clear();  // the received stage blocks are copied into the strips
      Bhold.clear();
      add_plan(*Acat, *Bcat);
    }
    if (stages > 1 && !concat) cbh_ctx_set_bitmap_fraction(context(), -1.0);
  }
  ~StagePlans() {
    for (cbh_plan* p : plans)
      if (p) cbh_plan_destroy(p);
  }
  StagePlans(const StagePlans&) = delete;
  StagePlans& operator=(const StagePlans&) = delete;
  // C(:, c0:c1) as an m x (c1 - c0) block with rebased column ids (a ColSplit piece of B times A,
  // ParFriends.h:591-669), the stages' partials merged on the device
  cbh_mat* piece(cbh_semiring sr, int dtype, int64_t vbytes, int64_t c0, int64_t c1) {
    std::vector<cbh_mat*> parts;
    for (size_t i = 0; i < plans.size(); ++i) {
      if (!plans[i]) continue;
      const std::vector<int64_t>& jc = bjc[i];
      const int64_t s0 = std::lower_bound(jc.begin(), jc.end(), c0) - jc.begin();
      const int64_t s1 = std::lower_bound(jc.begin(), jc.end(), c1) - jc.begin();
      if (s1 <= s0) continue;
      cbh_mat* C = nullptr;
      int rc = cbh_plan_spgemm_slots(plans[i], sr, s0, s1, 0, &C);
      if (rc != CBH_OK) die(context(), rc, "cbh_plan_spgemm_slots");
      if (essentials(C)[0] > 0) parts.push_back(C);
      else cbh_mat_free(context(), C);
    }
    cbh_mat* out = nullptr;
    if (parts.empty()) {
      int rc = cbh_mat_create(context(), m, c1 - c0, 0, 0, (cbh_dtype)dtype, vbytes, &out);
      if (rc != CBH_OK) die(context(), rc, "cbh_mat_create");
      return out;
    }
    out = parts.size() == 1 ? parts[0] : merge_all(sr, parts);
    int rc = cbh_mat_rebase_cols(context(), out, c0, c1 - c0);
    if (rc != CBH_OK) die(context(), rc, "cbh_mat_rebase_cols");
    return out;
  }
  // exact nnz of every local column of C (n columns), summed over the stages' plans and then over
  // `comm` (the processor column: MCLPruneRecoverySelect's column sums pair its ranks up, so they
  // must cut their phases identically)
  std::vector<int64_t> col_nnz(int64_t n, MPI_Comm comm) const {
    std::vector<int64_t> cnt((size_t)n, 0);
    for (size_t i = 0; i < plans.size(); ++i) {
      if (!plans[i] || bjc[i].empty()) continue;
      const size_t nzc = bjc[i].size();
      // (scratch from the context allocator: the block cache deliberately holds the previous call's
      // phase blocks, and its OOM path gives them back where a raw hipMalloc would abort)
      void* dv = nullptr;
      int rc = cbh_ctx_alloc(context(), (int64_t)(nzc * sizeof(int64_t)), &dv);
      if (rc != CBH_OK) die(context(), rc, "cbh_ctx_alloc");
      int64_t* d = static_cast<int64_t*>(dv);
      rc = cbh_plan_col_nnz(plans[i], d);
      if (rc != CBH_OK) die(context(), rc, "cbh_plan_col_nnz");
      std::vector<int64_t> h(nzc);
      hipStream_t cs = reinterpret_cast<hipStream_t>(cbh_ctx_stream(context()));
      hip_check(hipMemcpyAsync(h.data(), d, nzc * sizeof(int64_t), hipMemcpyDeviceToHost, cs), "hipMemcpyAsync");
      hip_check(hipStreamSynchronize(cs), "hipStreamSynchronize");
      cbh_ctx_free(context(), d);
      for (size_t sl = 0; sl < nzc; ++sl) cnt[(size_t)bjc[i][sl]] += h[sl];
    }
    int csize = 1;
    MPI_Comm_size(comm, &csize);
    if (csize > 1) MPI_Allreduce(MPI_IN_PLACE, cnt.data(), (int)n, MPI_INT64_T, MPI_SUM, comm);
    return cnt;
  }
  bool merges() const { return plans.size() > 1; }  // a phase merges per-stage partials
  std::shared_ptr<combblas::CommGrid> GridC;
  int stages = 0;
  int64_t m = 0;
  int64_t nnz = 0;  // exact nnz of the whole local product, summed over the stages

 private:
  std::vector<std::unique_ptr<SpDCColsDev<IU, NU1>>> Ahold;  // received stage blocks
  std::vector<std::unique_ptr<SpDCColsDev<IU, NU2>>> Bhold;
  std::unique_ptr<SpDCColsDev<IU, NU1>> Acat;  // the concatenated strips (default form)
  std::unique_ptr<SpDCColsDev<IU, NU2>> Bcat;
  std::vector<cbh_plan*> plans;
  std::vector<std::vector<int64_t>> bjc;  // host column ids of every plan's B operand
  // one symbolic pass over A_i * B_i: its exact nnz and B's column ids (the phase cuts' slots)
  void add_plan(SpDCColsDev<IU, NU1>& Ai, SpDCColsDev<IU, NU2>& Bi) {
    cbh_plan* p = nullptr;
    std::vector<int64_t> jc;
    if (Ai.getnnz() > 0 && Bi.getnnz() > 0) {
      int rc = cbh_plan_create(context(), Ai.mat(), Bi.mat(), &p);
      if (rc != CBH_OK) die(context(), rc, "cbh_plan_create");
      int64_t f = 0, z = 0;
      cbh_plan_info(p, &f, &z);
      nnz += z;
      jc.resize((size_t)Bi.getnzc());
      rc = cbh_mat_copy_out(context(), Bi.mat(), nullptr, jc.data(), nullptr, nullptr, 0);
      if (rc != CBH_OK) die(context(), rc, "cbh_mat_copy_out");
    }
    plans.push_back(p);
    bjc.push_back(std::move(jc));
  }
};

// the product 3D grid of C (ParFriends.h:3200-3203 / 3700: a fresh CommGrid3D of A's shape)
template <class IU, class NU1, class DER>
std::shared_ptr<combblas::CommGrid3D> product_grid3d(combblas::SpParMat3D<IU, NU1, DER>& A) {
  auto g = A.getcommgrid3D();
  return std::shared_ptr<combblas::CommGrid3D>(new combblas::CommGrid3D(g->GetWorld(), g->GetGridLayers(),
                                                                          g->GetGridRows(), g->GetGridCols(),
                                                                          A.isSpecial()));
}

// SpParMat3D<.., SpDCCols> -> SpParMat3D<.., SpDCColsDev> on the same 3D grid, and back
template <class IT, class NT>
combblas::SpParMat3D<IT, NT, SpDCColsDev<IT, NT>> to_device(combblas::SpParMat3D<IT, NT, combblas::SpDCCols<IT, NT>>& A) {
  return combblas::SpParMat3D<IT, NT, SpDCColsDev<IT, NT>>(new SpDCColsDev<IT, NT>(*A.seqptr()), A.getcommgrid3D(),
                                                           A.isColSplit(), A.isSpecial());
}
template <class IT, class NT>
combblas::SpParMat3D<IT, NT, combblas::SpDCCols<IT, NT>> to_host(combblas::SpParMat3D<IT, NT, SpDCColsDev<IT, NT>>& A) {
  return combblas::SpParMat3D<IT, NT, combblas::SpDCCols<IT, NT>>(A.seqptr()->to_host(), A.getcommgrid3D(),
                                                                  A.isColSplit(), A.isSpecial());
}

}  // namespace combblas_hip

namespace combblas {

template <typename IT, typename NT>
void MCLPruneRecoverySelect(SpParMat<IT, NT, combblas_hip::SpDCColsDev<IT, NT>>& A, NT hardThreshold, IT selectNum,
                            IT recoverNum, NT recoverPct, int kselectVersion) {
  static_assert(std::is_same<NT, double>::value, "device MCLPruneRecoverySelect: double values");
  (void)kselectVersion;  // Kselect1 semantics either way (radix select of the exact k-th value)
  cbh_mat* C = combblas_hip::mcl_prune_block(A.seq().mat(), A.getcommgrid()->GetColWorld(), hardThreshold,
                                             (int64_t)selectNum, (int64_t)recoverNum, recoverPct);
  A.seq().reset(C);
}

// EstPerProcessNnzSUMMA (ParFriends.h:1243-1340): per stage the broadcast blocks' exact product
// nnz (device symbolic pass), summed over the stages, max over the world
template <typename IU, typename NU1, typename NU2>
int64_t EstPerProcessNnzSUMMA(SpParMat<IU, NU1, combblas_hip::SpDCColsDev<IU, NU1>>& A,
                              SpParMat<IU, NU2, combblas_hip::SpDCColsDev<IU, NU2>>& B, bool hashEstimate) {
  (void)hashEstimate;
  if (A.getncol() != B.getnrow()) MPI_Abort(MPI_COMM_WORLD, DIMMISMATCH);
  int stages, dummy;
  std::shared_ptr<CommGrid> GridC = ProductGrid(A.getcommgrid().get(), B.getcommgrid().get(), stages, dummy, dummy);
  auto Asizes = combblas_hip::GetSetSizes(A.seq(), A.getcommgrid()->GetRowWorld());
  auto Bsizes = combblas_hip::GetSetSizes(B.seq(), B.getcommgrid()->GetColWorld());
  const int Aself = A.getcommgrid()->GetRankInProcRow(), Bself = B.getcommgrid()->GetRankInProcCol();
  int64_t nnz = 0;
  for (int i = 0; i < stages; ++i) {
    combblas_hip::SpDCColsDev<IU, NU1> Arecv;
    combblas_hip::SpDCColsDev<IU, NU2> Brecv;
    auto& Ai = (i == Aself) ? A.seq() : Arecv;
    auto& Bi = (i == Bself) ? B.seq() : Brecv;
    combblas_hip::BCastMatrix(GridC->GetRowWorld(), Ai, Asizes[i], i);
    combblas_hip::BCastMatrix(GridC->GetColWorld(), Bi, Bsizes[i], i);
    int64_t flops = 0, z = 0;
    if (Ai.getnnz() > 0 && Bi.getnnz() > 0) {
      int rc = cbh_spgemm_symbolic(combblas_hip::context(), Ai.mat(), Bi.mat(), &flops, &z, nullptr, nullptr);
      if (rc != CBH_OK) combblas_hip::die(combblas_hip::context(), rc, "cbh_spgemm_symbolic");
    }
    nnz += z;
  }
  int64_t mx = 0;
  MPI_Allreduce(&nnz, &mx, 1, MPI_INT64_T, MPI_MAX, GridC->GetWorld());
  return mx;
}

template <typename SR, typename NUO, typename UDERO, typename IU, typename NU1, typename NU2>
SpParMat<IU, NUO, UDERO> MemEfficientSpGEMM(SpParMat<IU, NU1, combblas_hip::SpDCColsDev<IU, NU1>>& A,
                                            SpParMat<IU, NU2, combblas_hip::SpDCColsDev<IU, NU2>>& B, int phases,
                                            NUO hardThreshold, IU selectNum, IU recoverNum, NUO recoverPct,
                                            int kselectVersion, int computationKernel, int64_t perProcessMemory) {
  static_assert(std::is_same<UDERO, combblas_hip::SpDCColsDev<IU, NUO>>::value,
                "device-resident operands give a device-resident product");
  (void)computationKernel;  // hash and heap contracts are both met by the device kernel
  if (A.getncol() != B.getnrow()) {
    SpParHelper::Print("Can not multiply, dimensions does not match\n");
    MPI_Abort(MPI_COMM_WORLD, DIMMISMATCH);
  }
  if (phases < 1 || phases >= A.getncol()) phases = 1;
  // the plans (and their scratch) live for the phase loop only: the concatenation of the pruned
  // pieces below needs a second copy of them in HBM (no cache release here: the block cache
  // holds the previous call's phase blocks, which this call's phases reuse -- releasing them first
  // made C5's third MCL call run out of memory)
  combblas_hip::memdiag("MemEfficientSpGEMM start");
  std::unique_ptr<combblas_hip::StagePlans<IU, NU1, NU2>> SPp(
      new combblas_hip::StagePlans<IU, NU1, NU2>(A.seq(), A.getcommgrid().get(), B.seq(), B.getcommgrid().get()));
  combblas_hip::StagePlans<IU, NU1, NU2>& SP = *SPp;
  combblas_hip::memdiag("stage plans");
  std::shared_ptr<CommGrid> GridC = SP.GridC;
  if (perProcessMemory > 0) {  // the reference's memory model (ParFriends.h:480-520), exact nnz per stage
    int p;
    MPI_Comm_size(GridC->GetWorld(), &p);
    const int64_t perNNZMem_in = sizeof(IU) * 2 + sizeof(NU1), perNNZMem_out = sizeof(IU) * 2 + sizeof(NUO);
    int64_t lannz = A.getlocalnnz(), gannz = 0;
    MPI_Allreduce(&lannz, &gannz, 1, MPI_INT64_T, MPI_MAX, GridC->GetWorld());
    const int64_t inputMem = gannz * perNNZMem_in * 4;
    int64_t asquareNNZ = 0;  // EstPerProcessNnzSUMMA: the plans' exact nnz, max over the world
    MPI_Allreduce(&SP.nnz, &asquareNNZ, 1, MPI_INT64_T, MPI_MAX, GridC->GetWorld());
    const int64_t asquareMem = asquareNNZ * perNNZMem_out * 2;
    const int64_t lcols = std::max<int64_t>(1, B.getlocalcols());
    const int64_t d = (int64_t)std::ceil((asquareNNZ * std::sqrt((double)p)) / lcols);
    const int64_t k = std::min(int64_t(std::max(selectNum, recoverNum)), d);
    const int64_t kselectmem = lcols * k * 8 * 3;
    const int64_t outputMem = (int64_t)((lcols * k) / std::sqrt((double)p)) * perNNZMem_in * 2;
    const int64_t remainingMem = perProcessMemory * 1000000000 - inputMem - outputMem;
    if (remainingMem > 0) phases = 1 + (int)((asquareMem + kselectmem) / remainingMem);
  }
  const IU C_n = B.seq().getncol();
  // phase cuts: an even share of the exact entries per phase (balanced_cuts); the reference's even
  // column counts with COMBBLAS_HIP_EVEN_CUTS=1. Either way C is the same matrix.
  const std::vector<int64_t> ccnt = SP.col_nnz(C_n, GridC->GetColWorld());
  const auto cuts = combblas_hip::even_column_cuts() ? combblas_hip::colsplit_cuts(C_n, phases)
                                                     : combblas_hip::balanced_cuts(ccnt, phases);
  phases = (int)cuts.size() - 1;
  int64_t max_phase_nnz = 0;
  for (int p = 0; p < phases; ++p) {
    int64_t z = 0;
    for (int64_t c = cuts[p]; c < cuts[p + 1]; ++c) z += ccnt[(size_t)c];
    max_phase_nnz = std::max(max_phase_nnz, z);
  }
  std::vector<cbh_mat*> toconcatenate;
  // the pruned pieces go back to back into one arena whose arrays become C's: the memory beside
  // A, B, the plans, the largest phase product (its exact nnz; twice that when per-stage partials
  // are merged) and the scratch of one phase (combblas_hip::phase_scratch_bytes), at most the
  // unpruned nnz; the same capacity as the previous call of this context when it still fits
  // (arena_capacity), so that the block the previous result freed serves it again
  cbh_arena* arena = nullptr;
  {
    cbh_ctx* ctx = combblas_hip::context();
    int64_t live = 0, cached = 0, fr = 0, tot = 0;
    cbh_ctx_memory(ctx, &live, &cached, &fr, &tot);
    const int64_t eb = (int64_t)(sizeof(int32_t) + sizeof(NUO));
    int64_t max_phase_cols = 0;
    for (int p = 0; p < phases; ++p) max_phase_cols = std::max<int64_t>(max_phase_cols, cuts[p + 1] - cuts[p]);
    const int64_t phase_bytes = max_phase_nnz * (SP.merges() ? 2 : 1) * eb;
    const int64_t reserve = combblas_hip::phase_scratch_bytes(max_phase_nnz, max_phase_cols, SP.merges());
    const int64_t cap = combblas_hip::arena_capacity(ctx, (fr + cached - phase_bytes - reserve) / eb, SP.nnz);
    if (combblas_hip::memdiag_on())
      std::printf("[memdiag] arena %.2f GB (phase piece %.2f GB, phase scratch bound %.2f GB)\n", cap * eb / 1e9,
                  phase_bytes / 1e9, reserve / 1e9);
    if (cap > 0 && sizeof(NUO) == 8 && cbh_arena_create(ctx, cap, (int64_t)sizeof(NUO), &arena) != CBH_OK)
      arena = nullptr;  // (no room: the pieces are allocated one by one and concatenated)
  }
  combblas_hip::memdiag("phase loop start");
  for (int p = 0; p < phases; ++p) {
    cbh_mat* Cp = SP.piece(combblas_hip::semiring_traits<SR>::code, combblas_hip::dtype_of<NUO>::value,
                           (int64_t)sizeof(NUO), cuts[p], cuts[p + 1]);
    combblas_hip::memdiag("phase product");
    SpParMat<IU, NUO, UDERO> OnePieceOfC(new UDERO(Cp), GridC);
    // MCLPruneRecoverySelect (ParFriends.h:185-353) with its rows and values written into the arena
    cbh_mat* Cpr = combblas_hip::mcl_prune_block(OnePieceOfC.seq().mat(), GridC->GetColWorld(), hardThreshold,
                                                 (int64_t)selectNum, (int64_t)recoverNum, recoverPct, arena);
    OnePieceOfC.seq().reset(Cpr);
    toconcatenate.push_back(OnePieceOfC.seq().release());
    combblas_hip::memdiag("phase pruned");
  }
  SPp.reset();
  combblas_hip::memdiag("before concatenation");
  cbh_mat* Cm = nullptr;
  if (arena) {
    const int rc = cbh_arena_concat(combblas_hip::context(), (int)toconcatenate.size(), toconcatenate.data(), arena, &Cm);
    cbh_arena_destroy(combblas_hip::context(), arena);
    if (rc != CBH_OK) combblas_hip::die(combblas_hip::context(), rc, "cbh_arena_concat");
    toconcatenate.clear();
  } else {
    Cm = combblas_hip::col_concat(toconcatenate);
  }
  combblas_hip::memdiag("concatenated");
  (void)kselectVersion;
  return SpParMat<IU, NUO, UDERO>(new UDERO(Cm), GridC);
}

template <typename SR, typename NUO, typename UDERO, typename IU, typename NU1, typename NU2>
SpParMat3D<IU, NUO, UDERO> Mult_AnXBn_SUMMA3D(SpParMat3D<IU, NU1, combblas_hip::SpDCColsDev<IU, NU1>>& A,
                                              SpParMat3D<IU, NU2, combblas_hip::SpDCColsDev<IU, NU2>>& B) {
  static_assert(std::is_same<UDERO, combblas_hip::SpDCColsDev<IU, NUO>>::value,
                "device-resident operands give a device-resident product");
  if (A.getncol() != B.getnrow()) {
    SpParHelper::Print("Can not multiply, dimensions does not match\n");
    MPI_Abort(MPI_COMM_WORLD, DIMMISMATCH);
  }
  std::vector<IU> div3;
  B.CalculateColSplitDistributionOfLayer(div3);
  std::shared_ptr<CommGrid> G;
  cbh_mat* P = combblas_hip::summa_blocks<SR, NUO>(*A.GetLayerMat()->seqptr(), A.GetLayerMat()->getcommgrid().get(),
                                                   *B.GetLayerMat()->seqptr(), B.GetLayerMat()->getcommgrid().get(), G);
  std::vector<int64_t> div(div3.begin(), div3.end());
  cbh_mat* C = combblas_hip::fiber_reduce_scatter(combblas_hip::semiring_traits<SR>::code, P, div,
                                                  A.getcommgrid3D()->GetFiberWorld(), combblas_hip::dtype_of<NUO>::value,
                                                  (int64_t)sizeof(NUO));
  return SpParMat3D<IU, NUO, UDERO>(new UDERO(C), combblas_hip::product_grid3d(A), A.isColSplit(), A.isSpecial());
}

template <typename SR, typename NUO, typename UDERO, typename IU, typename NU1, typename NU2>
SpParMat3D<IU, NUO, UDERO> MemEfficientSpGEMM3D(SpParMat3D<IU, NU1, combblas_hip::SpDCColsDev<IU, NU1>>& A,
                                                SpParMat3D<IU, NU2, combblas_hip::SpDCColsDev<IU, NU2>>& B, int phases,
                                                NUO hardThreshold, IU selectNum, IU recoverNum, NUO recoverPct,
                                                int kselectVersion, int computationKernel, int64_t perProcessMemory) {
  static_assert(std::is_same<UDERO, combblas_hip::SpDCColsDev<IU, NUO>>::value,
                "device-resident operands give a device-resident product");
  (void)computationKernel;
  if (A.getncol() != B.getnrow()) {
    SpParHelper::Print("Can not multiply, dimensions does not match\n");
    MPI_Abort(MPI_COMM_WORLD, DIMMISMATCH);
  }
  if (phases < 1 || phases >= B.getncol()) phases = 1;
  // (no cache release at the start, as in the 2D driver: the previous call's phase blocks are what
  // this call's phases reuse; a new RCCL communicator frees what it needs itself, rccl_comm_for)
  auto g3 = A.getcommgrid3D();
  // the layer SUMMA's stage pairs, planned once for every phase (freed before the concatenation)
  std::unique_ptr<combblas_hip::StagePlans<IU, NU1, NU2>> SPp(new combblas_hip::StagePlans<IU, NU1, NU2>(
      *A.GetLayerMat()->seqptr(), A.GetLayerMat()->getcommgrid().get(), *B.GetLayerMat()->seqptr(),
      B.GetLayerMat()->getcommgrid().get()));
  combblas_hip::StagePlans<IU, NU1, NU2>& SP = *SPp;
  if (perProcessMemory > 0) {  // the reference's 3D memory model (ParFriends.h:3247-3290)
    int p;
    MPI_Comm_size(g3->GetLayerWorld(), &p);
    const int64_t perNNZMem_in = sizeof(IU) * 2 + sizeof(NU1), perNNZMem_out = sizeof(IU) * 2 + sizeof(NUO);
    int64_t lannz = A.GetLayerMat()->getlocalnnz(), gannz = 0;
    MPI_Allreduce(&lannz, &gannz, 1, MPI_INT64_T, MPI_MAX, g3->GetWorld());
    const int64_t ginputMem = gannz * perNNZMem_in * 5;
    int64_t asquareNNZ = 0;  // EstPerProcessNnzSUMMA on the layer: the plans' exact nnz, max over the layer
    MPI_Allreduce(&SP.nnz, &asquareNNZ, 1, MPI_INT64_T, MPI_MAX, SP.GridC->GetWorld());
    int64_t gasquareNNZ = 0;
    MPI_Allreduce(&asquareNNZ, &gasquareNNZ, 1, MPI_INT64_T, MPI_MAX, g3->GetFiberWorld());
    const int64_t gasquareMem = gasquareNNZ * perNNZMem_out * 2;
    const int64_t lcols = std::max<int64_t>(1, B.GetLayerMat()->getlocalcols());
    const int64_t d = (int64_t)std::ceil(((gasquareNNZ / g3->GetGridLayers()) * std::sqrt((double)p)) / lcols);
    const int64_t k = std::min(int64_t(std::max(selectNum, recoverNum)), d);
    const int64_t postMem = (int64_t)std::ceil(((lcols / g3->GetGridLayers()) * k) / std::sqrt((double)p)) *
                            perNNZMem_out * 2;
    const double remainingMem = perProcessMemory * 1000000000.0 - ginputMem - postMem;
    const int64_t kselectMem = lcols * k * (int64_t)sizeof(NUO) * 3;
    int calc = remainingMem > 0 ? (int)std::ceil((gasquareMem + kselectMem) / remainingMem) : -1, gcalc = 0;
    MPI_Allreduce(&calc, &gcalc, 1, MPI_INT, MPI_MAX, g3->GetFiberWorld());
    if (gcalc > phases) phases = gcalc;
  }
  std::vector<IU> div3;
  B.CalculateColSplitDistributionOfLayer(div3);
  const int L = g3->GetGridLayers(), me = g3->GetRankInFiber();
  // B's layer block: `L` chunks of div3 columns, each cut in `phases` pieces (ColSplit)
  std::vector<std::vector<int64_t>> piece(L);  // column offsets of chunk c's pieces in the layer block
  int64_t c0 = 0;
  for (int c = 0; c < L; ++c) {
    auto cuts = combblas_hip::colsplit_cuts((int64_t)div3[c], phases);
    for (auto& x : cuts) x += c0;
    piece[c] = cuts;
    c0 += div3[c];
  }
  std::vector<cbh_mat*> toconcatenate;
  // phase p's fiber exchange runs on the communication stream while phase p+1's products run on
  // the context stream; its merge and prune follow them (fiber_exchange_start / _finish)
  auto finish = [&](combblas_hip::FiberExchange& X, int p) {
    cbh_mat* Cp = combblas_hip::fiber_exchange_finish(X);
    combblas_hip::trace("exchange merged", p);
    SpParMat<IU, NUO, UDERO> phaseResultantLayer(new UDERO(Cp), g3->GetLayerWorld());
    MCLPruneRecoverySelect(phaseResultantLayer, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion);
    toconcatenate.push_back(phaseResultantLayer.seq().release());
  };
  std::unique_ptr<combblas_hip::FiberExchange> inflight;
  for (int p = 0; p < phases; ++p) {
    // OnePieceOfB = piece p of every chunk (ParFriends.h:3414-3440): the layer product of those
    // columns is the concatenation of the chunk pieces' products
    std::vector<cbh_mat*> parts;
    std::vector<int64_t> lb(L);
    for (int c = 0; c < L; ++c) {
      parts.push_back(SP.piece(combblas_hip::semiring_traits<SR>::code, combblas_hip::dtype_of<NUO>::value,
                               (int64_t)sizeof(NUO), piece[c][p], piece[c][p + 1]));
      lb[c] = piece[c][p + 1] - piece[c][p];
    }
    combblas_hip::trace("products issued", p);
    cbh_mat* P = combblas_hip::col_concat(parts);
    if (inflight) finish(*inflight, p - 1);  // (after phase p's products were issued)
    inflight.reset(new combblas_hip::FiberExchange(combblas_hip::fiber_exchange_start(
        combblas_hip::semiring_traits<SR>::code, P, lb, g3->GetFiberWorld(), combblas_hip::dtype_of<NUO>::value,
        (int64_t)sizeof(NUO))));
    combblas_hip::trace("exchange posted", p);
  }
  if (inflight) finish(*inflight, phases - 1);
  (void)me;
  SPp.reset();
  return SpParMat3D<IU, NUO, UDERO>(new UDERO(combblas_hip::col_concat(toconcatenate)),
                                    combblas_hip::product_grid3d(A), A.isColSplit(), A.isSpecial());
}

}  // namespace combblas
