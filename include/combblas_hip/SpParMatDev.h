// SpParMatDev.h -- device-resident distributed SpGEMM behind the reference's own API.
//
//   typedef combblas::SpParMat<int64_t, double, combblas_hip::SpDCColsDev<int64_t, double>> DMat;
//   DMat A = combblas_hip::to_device(Ahost), B = combblas_hip::to_device(Bhost);
//   DMat C = combblas::PSpGEMM<combblas::PlusTimesSRing<double, double>>(A, B);   // SpParMat.h:454-467
//   auto Ch = combblas_hip::to_host(C);
//
// SpDCColsDev<IT,NT> is a DER (the local-block type parameter of SpParMat, like SpDCCols) whose
// Dcsc arrays live in HBM (a cbh_mat). For SpParMats over it, the overload of
// combblas::Mult_AnXBn_Synch below is more specialized than the reference's generic one
// (ParFriends.h:1004-1108), so the reference's PSpGEMM (and any code that calls
// Mult_AnXBn_Synch<SR, NUO, UDERO>) runs the same 2D SUMMA with every block kept in HBM:
//   GetSetSizes      host MPI_Allgather of the 4 essentials per rank (scalars; SpParHelper.cpp:797-808)
//   BCastMatrix      cp / jc / ir / num broadcast DEVICE TO DEVICE on the row (A) and column (B)
//                    communicators with RCCL (ncclBroadcast over xGMI; SpParHelper.cpp:581-599)
//   local multiply   cbh_spgemm (LocalHybridSpGEMM, mtSpGEMM.h:212-460)
//   MultiwayMerge    cbh_merge of the stage partials on the device (MultiwayMerge.h:411-526)
// -- no host copy of any block, partial or result. The RCCL communicators mirror the
// reference's MPI ones (CommGrid.cpp:37-75: world, row and column splits): one ncclComm per MPI
// communicator, bootstrapped by an MPI_Bcast of the ncclUniqueId from the communicator's rank 0.
// COMBBLAS_HIP_COMM=mpi selects a host-staged MPI_Bcast transport instead (test rehearsal of
// several ranks sharing one GPU, which RCCL does not allow).
//
// Link: libcombblas_hip.so, librccl.so (/opt/rocm/lib), libamdhip64.so, MPI.
#pragma once

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <vector>

#include "HipSpGEMM.h"

namespace combblas_hip {

// ------------------------------------------------------------------ the device-resident block
template <class IT, class NT>
class SpDCColsDev {
 public:
  typedef IT LocalIT;
  typedef NT LocalNT;
  static const int esscount = 4;  // nnz, m, n, nzc (SpDCCols.h esscount, SpDCCols.cpp:787-795)

  SpDCColsDev() { mat_ = make_empty(0, 0); }
  SpDCColsDev(IT m, IT n) { mat_ = make_empty(m, n); }
  explicit SpDCColsDev(cbh_mat* m) : mat_(m) {}  // takes ownership
  explicit SpDCColsDev(const combblas::SpDCCols<IT, NT>& host) { mat_ = upload(host); }
  SpDCColsDev(const SpDCColsDev& o) {  // deep copy, as SpDCCols's (SpDCCols.cpp:214-226)
    int rc = cbh_mat_clone(context(), o.mat_, &mat_);
    if (rc != CBH_OK) die(context(), rc, "cbh_mat_clone");
  }
  SpDCColsDev& operator=(const SpDCColsDev& o) {
    if (this != &o) {
      cbh_mat* m = nullptr;
      int rc = cbh_mat_clone(context(), o.mat_, &m);
      if (rc != CBH_OK) die(context(), rc, "cbh_mat_clone");
      reset(m);
    }
    return *this;
  }
  ~SpDCColsDev() { reset(nullptr); }

  IT getnrow() const { return (IT)info(0); }
  IT getncol() const { return (IT)info(1); }
  IT getnnz() const { return (IT)info(2); }
  IT getnzc() const { return (IT)info(3); }
  bool isZero() const { return getnnz() == 0; }
  // SpDCCols::GetEssentials (SpDCCols.cpp:46): {nnz, m, n, nzc}
  std::vector<IT> GetEssentials() const { return {getnnz(), getnrow(), getncol(), getnzc()}; }

  cbh_mat* mat() const { return mat_; }
  void reset(cbh_mat* m) {
    if (mat_) cbh_mat_free(context(), mat_);
    mat_ = m;
  }
  cbh_mat* release() {
    cbh_mat* m = mat_;
    mat_ = nullptr;
    return m;
  }
  // one download of the whole block (the only device -> host copy of the path)
  combblas::SpDCCols<IT, NT>* to_host() const {
    combblas::SpTuples<IT, NT>* t = download_tuples<IT, NT>(mat_);
    auto* d = new combblas::SpDCCols<IT, NT>(*t, false);
    delete t;
    return d;
  }

 private:
  static cbh_mat* make_empty(IT m, IT n) {
    cbh_mat* out = nullptr;
    int rc = cbh_mat_create(context(), m, n, 0, 0, dtype_of<NT>::value, (int64_t)sizeof(NT), &out);
    if (rc != CBH_OK) die(context(), rc, "cbh_mat_create");
    return out;
  }
  int64_t info(int k) const {
    int64_t v[4] = {0, 0, 0, 0};
    cbh_mat_info(mat_, &v[0], &v[1], &v[2], &v[3], nullptr);
    return v[k];
  }
  cbh_mat* mat_ = nullptr;
};

// ------------------------------------------------------------------ RCCL communicators of a grid
inline bool use_mpi_transport() {
  static const bool v = [] {
    const char* e = std::getenv("COMBBLAS_HIP_COMM");
    return e && std::strcmp(e, "mpi") == 0;
  }();
  return v;
}

// HIP runtime calls of the device drivers: a failed copy, event or synchronize (where an
// asynchronous kernel fault surfaces) aborts the job with the HIP code, as rccl_check does for RCCL,
// so a host-staged exchange can never ship stale host data over MPI
inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "combblas_hip: %s failed: %s (%d)\n", what, hipGetErrorString(e), (int)e);
    MPI_Abort(MPI_COMM_WORLD, CBH_E_HIP);
  }
}

// host-staged transport (COMBBLAS_HIP_COMM=mpi): MPI counts are int, so messages go in pieces of
// at most 1 GiB
constexpr size_t kMpiPiece = size_t(1) << 30;
inline void mpi_bcast_bytes(void* buf, size_t bytes, int root, MPI_Comm comm) {
  for (size_t o = 0; o < bytes; o += kMpiPiece)
    MPI_Bcast(static_cast<char*>(buf) + o, (int)std::min(kMpiPiece, bytes - o), MPI_BYTE, root, comm);
}
inline void mpi_sendrecv_bytes(const void* sbuf, size_t sbytes, int to, void* rbuf, size_t rbytes, int from, int tag,
                               MPI_Comm comm) {
  // pieces in order, each side counting its own (MPI keeps the order of one pair's messages)
  std::vector<MPI_Request> req;
  for (size_t o = 0; o < rbytes; o += kMpiPiece) {
    req.emplace_back();
    MPI_Irecv(static_cast<char*>(rbuf) + o, (int)std::min(kMpiPiece, rbytes - o), MPI_BYTE, from, tag, comm, &req.back());
  }
  for (size_t o = 0; o < sbytes; o += kMpiPiece) {
    req.emplace_back();
    MPI_Isend(static_cast<const char*>(sbuf) + o, (int)std::min(kMpiPiece, sbytes - o), MPI_BYTE, to, tag, comm,
              &req.back());
  }
  if (!req.empty()) MPI_Waitall((int)req.size(), req.data(), MPI_STATUSES_IGNORE);
}

// when less than `want` bytes of device memory are free, cached blocks of the context allocator go
// back to HIP (largest first, as many as make `want` free): before RCCL allocates a communicator's
// buffers, and at the start of a phased product, whose arena and phase pieces are sized from the
// free memory (the block cache may hold a large share of the HBM)
inline void ensure_device_free(int64_t want = int64_t(8) << 30) {
  int64_t fr = 0, tot = 0;
  cbh_ctx_memory(context(), nullptr, nullptr, &fr, &tot);
  if (fr < want) cbh_ctx_release(context(), want - fr);
}

inline void rccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    std::fprintf(stderr, "combblas_hip: %s failed: %s\n", what, ncclGetErrorString(r));
    MPI_Abort(MPI_COMM_WORLD, CBH_E_HIP);
  }
}

// ncclComm_t for an MPI communicator, one per MEMBERSHIP (the communicator's ranks in
// MPI_COMM_WORLD, in communicator rank order): created collectively (ncclUniqueId from the
// communicator's rank 0 over MPI_Bcast) the first time a communicator with those members is used,
// then kept for the process. The reference's ProductGrid builds a fresh CommGrid -- fresh row and
// column MPI communicators -- for every product (CommGrid.cpp:164-180), so a communicator-keyed
// ncclComm paid ncclCommInitRank's bootstrap on every call (round 4 keyed it by the MPI handle and
// destroyed it with the communicator). Every member of a membership ran the same creation (SPMD),
// so all of them find it in their caches. An attribute on the MPI communicator remembers the
// lookup (no delete callback: the ncclComm outlives the communicator).
inline std::map<std::vector<int>, ncclComm_t>& rccl_cache() {
  static std::map<std::vector<int>, ncclComm_t> m;
  return m;
}
inline int rccl_keyval() {
  static int kv = [] {
    int k = MPI_KEYVAL_INVALID;
    MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, MPI_COMM_NULL_DELETE_FN, &k, nullptr);
    return k;
  }();
  return kv;
}
inline std::vector<int> world_ranks(MPI_Comm comm) {
  MPI_Group g, wg;
  MPI_Comm_group(comm, &g);
  MPI_Comm_group(MPI_COMM_WORLD, &wg);
  int n = 0;
  MPI_Group_size(g, &n);
  std::vector<int> in(n), out(n);
  for (int i = 0; i < n; ++i) in[i] = i;
  MPI_Group_translate_ranks(g, n, in.data(), wg, out.data());
  MPI_Group_free(&g);
  MPI_Group_free(&wg);
  return out;
}
// The members of an RCCL communicator that share a node must drive distinct GPUs (RCCL refuses two
// ranks on one device, and a rank whose device resolution went wrong would otherwise surface as an
// RCCL error deep inside a product): the node's members gather their devices' PCI bus ids.
inline void check_distinct_devices(MPI_Comm comm) {
  MPI_Comm node;
  MPI_Comm_split_type(comm, MPI_COMM_TYPE_SHARED, 0, MPI_INFO_NULL, &node);
  int n = 1;
  MPI_Comm_size(node, &n);
  if (n > 1) {
    int dev = -1;
    cbh_ctx_device(context(), &dev);
    char mine[32] = {0};
    if (cbh_device_pci_id(dev, mine, (int)sizeof(mine)) != CBH_OK) std::snprintf(mine, sizeof(mine), "dev%d", dev);
    std::vector<char> all(32 * (size_t)n);
    MPI_Allgather(mine, 32, MPI_CHAR, all.data(), 32, MPI_CHAR, node);
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j)
        if (std::strncmp(&all[32 * (size_t)i], &all[32 * (size_t)j], 32) == 0) {
          std::fprintf(stderr,
                       "combblas_hip: node-local ranks %d and %d of an RCCL communicator share GPU %s (set one "
                       "device per rank, or COMBBLAS_HIP_COMM=mpi for a shared-GPU rehearsal)\n",
                       i, j, &all[32 * (size_t)i]);
          MPI_Abort(MPI_COMM_WORLD, CBH_E_NODEVICE);
        }
  }
  MPI_Comm_free(&node);
}

// The cached communicators are released when MPI finalizes (the delete callback of an attribute
// on MPI_COMM_SELF runs first thing in MPI_Finalize): after the context stream has drained, each
// is aborted -- a local teardown that waits on no peer, so ranks that finish at different times
// cannot hang each other at exit (ncclCommDestroy's implicit finalize may synchronize with peers).
inline int rccl_release_all(MPI_Comm, int, void*, void*) {
  auto& cache = rccl_cache();
  if (!cache.empty()) {
    (void)cbh_ctx_synchronize(context());
    for (auto& kv : cache) (void)ncclCommAbort(kv.second);
    cache.clear();
  }
  return MPI_SUCCESS;
}
inline void rccl_register_teardown() {
  static bool done = [] {
    int kv = MPI_KEYVAL_INVALID;
    MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, rccl_release_all, &kv, nullptr);
    MPI_Comm_set_attr(MPI_COMM_SELF, kv, nullptr);
    return true;
  }();
  (void)done;
}

inline ncclComm_t rccl_comm_for(MPI_Comm comm) {
  void* attr = nullptr;
  int found = 0;
  MPI_Comm_get_attr(comm, rccl_keyval(), &attr, &found);
  if (found && attr) return *static_cast<ncclComm_t*>(attr);
  auto& cache = rccl_cache();
  const std::vector<int> key = world_ranks(comm);
  auto it = cache.find(key);
  if (it == cache.end()) {
    int rank = 0, size = 1;
    MPI_Comm_rank(comm, &rank);
    MPI_Comm_size(comm, &size);
    check_distinct_devices(comm);
    rccl_register_teardown();
    // RCCL's buffers are not the context allocator's: only a NEW communicator needs device memory
    // freed (releasing on every uncached MPI communicator emptied the block cache the
    // phased drivers reuse, as 783b081 found for the 2D driver's start)
    ensure_device_free();
    ncclUniqueId id;
    if (rank == 0) rccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    MPI_Bcast(&id, (int)sizeof(id), MPI_BYTE, 0, comm);
    ncclComm_t c;
    rccl_check(ncclCommInitRank(&c, size, id, rank), "ncclCommInitRank");
    it = cache.emplace(key, c).first;
  }
  MPI_Comm_set_attr(comm, rccl_keyval(), &it->second);  // std::map nodes are stable
  return it->second;
}

// SpParHelper::BCastMatrix (SpParHelper.cpp:581-599) on device blocks, in two halves: non-root
// ranks allocate from the essentials {nnz, m, n, nzc} (SpDCCols::Create), then cp, jc, ir and the
// values are broadcast device to device on `s` (the context stream, or the overlapped drivers'
// communication stream).
template <class IT, class NT>
void bcast_alloc(MPI_Comm comm, SpDCColsDev<IT, NT>& M, const std::vector<IT>& ess, int root) {
  int rank = 0;
  MPI_Comm_rank(comm, &rank);
  if (rank == root) return;
  cbh_mat* m = nullptr;
  int rc = cbh_mat_create(context(), ess[1], ess[2], ess[0], ess[3], dtype_of<NT>::value, (int64_t)sizeof(NT), &m);
  if (rc != CBH_OK) die(context(), rc, "cbh_mat_create");
  M.reset(m);
}
template <class IT, class NT>
void bcast_arrays(MPI_Comm comm, SpDCColsDev<IT, NT>& M, const std::vector<IT>& ess, int root, hipStream_t s,
                  bool grouped = false);
template <class IT, class NT>
void BCastMatrix(MPI_Comm comm, SpDCColsDev<IT, NT>& M, const std::vector<IT>& ess, int root) {
  bcast_alloc(comm, M, ess, root);
  bcast_arrays(comm, M, ess, root, reinterpret_cast<hipStream_t>(cbh_ctx_stream(context())));
}
// grouped: the caller brackets several broadcasts in one ncclGroupStart / ncclGroupEnd
template <class IT, class NT>
void bcast_arrays(MPI_Comm comm, SpDCColsDev<IT, NT>& M, const std::vector<IT>& ess, int root, hipStream_t s,
                  bool grouped) {
  int rank = 0, csize = 1;
  MPI_Comm_rank(comm, &rank);
  MPI_Comm_size(comm, &csize);
  if (csize == 1) return;  // the root's own block: nothing moves (and no communicator is created)
  const int64_t *cp, *jc;
  const int32_t* ir;
  const void* num;
  cbh_mat_device_arrays(M.mat(), &cp, &jc, &ir, &num);
  const int64_t nnz = ess[0], nzc = ess[3];
  struct Piece {
    void* p;
    size_t bytes;
  } pieces[4] = {{const_cast<int64_t*>(cp), sizeof(int64_t) * (size_t)(nzc + 1)},
                 {const_cast<int64_t*>(jc), sizeof(int64_t) * (size_t)nzc},
                 {const_cast<int32_t*>(ir), sizeof(int32_t) * (size_t)nnz},
                 {const_cast<void*>(num), sizeof(NT) * (size_t)nnz}};
  if (use_mpi_transport()) {  // host-staged rehearsal transport
    for (const Piece& x : pieces) {
      if (!x.bytes) continue;
      std::vector<char> h(x.bytes);
      if (rank == root) {
        hip_check(hipMemcpyAsync(h.data(), x.p, x.bytes, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
        hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
      }
      mpi_bcast_bytes(h.data(), x.bytes, root, comm);
      if (rank != root) {
        hip_check(hipMemcpyAsync(x.p, h.data(), x.bytes, hipMemcpyHostToDevice, s), "hipMemcpyAsync");
        hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
      }
    }
    return;
  }
  ncclComm_t nc = rccl_comm_for(comm);
  if (!grouped) rccl_check(ncclGroupStart(), "ncclGroupStart");
  for (const Piece& x : pieces)
    if (x.bytes) rccl_check(ncclBroadcast(x.p, x.p, x.bytes, ncclUint8, root, nc, s), "ncclBroadcast");
  if (!grouped) rccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

// SpParHelper::GetSetSizes (SpParHelper.cpp:797-808): essentials of every rank of comm1d
template <class IT, class NT>
std::vector<std::vector<IT>> GetSetSizes(const SpDCColsDev<IT, NT>& M, MPI_Comm comm1d) {
  int size = 1;
  MPI_Comm_size(comm1d, &size);
  std::vector<IT> mine = M.GetEssentials(), all(4 * (size_t)size);
  MPI_Allgather(mine.data(), 4 * (int)sizeof(IT), MPI_BYTE, all.data(), 4 * (int)sizeof(IT), MPI_BYTE, comm1d);
  std::vector<std::vector<IT>> out(size);
  for (int r = 0; r < size; ++r) out[r].assign(all.begin() + 4 * r, all.begin() + 4 * r + 4);
  return out;
}

// the built-in semiring code of SR (semiring_traits in HipSpGEMM.h)
template <class SR, class NUO, class NU1, class NU2>
cbh_mat* local_multiply(const cbh_mat* A, const cbh_mat* B) {
  static_assert(std::is_same<NU1, NUO>::value && std::is_same<NU2, NUO>::value,
                "device-resident SUMMA: built-in semirings over one value type");
  cbh_mat* C = nullptr;
  int rc = cbh_spgemm(context(), semiring_traits<SR>::code, A, B, CBH_SORTED_ROWS, &C);
  if (rc != CBH_OK) die(context(), rc, "cbh_spgemm");
  return C;
}

// The SUMMA stage loop of Mult_AnXBn_Synch (ParFriends.h:1004-1108) over two device blocks on their
// grids (the local blocks of A and B, or B's phase piece): sizes exchanged on the host
// (GetSetSizes), stage blocks broadcast device to device on the product grid's row (A) and column
// (B) communicators, multiplied on the device, the non-empty stage partials merged on the device.
// Returns the product block (an m x n matrix even when empty); GridC = ProductGrid(GA, GB).
template <class SR, class NUO, class IU, class NU1, class NU2>
cbh_mat* summa_blocks(SpDCColsDev<IU, NU1>& Aloc, combblas::CommGrid* GA, SpDCColsDev<IU, NU2>& Bloc,
                      combblas::CommGrid* GB, std::shared_ptr<combblas::CommGrid>& GridC) {
  int stages, dummy;
  GridC = ProductGrid(GA, GB, stages, dummy, dummy);  // found by ADL (a friend of CommGrid)
  const IU C_m = Aloc.getnrow(), C_n = Bloc.getncol();
  auto Asizes = GetSetSizes(Aloc, GA->GetRowWorld());
  auto Bsizes = GetSetSizes(Bloc, GB->GetColWorld());
  const int Aself = GA->GetRankInProcRow();
  const int Bself = GB->GetRankInProcCol();
  std::vector<cbh_mat*> tomerge;
  for (int i = 0; i < stages; ++i) {
    SpDCColsDev<IU, NU1> Arecv;
    SpDCColsDev<IU, NU2> Brecv;
    SpDCColsDev<IU, NU1>& Ai = (i == Aself) ? Aloc : Arecv;
    SpDCColsDev<IU, NU2>& Bi = (i == Bself) ? Bloc : Brecv;
    BCastMatrix(GridC->GetRowWorld(), Ai, Asizes[i], i);
    BCastMatrix(GridC->GetColWorld(), Bi, Bsizes[i], i);
    cbh_mat* Ci = local_multiply<SR, NUO, NU1, NU2>(Ai.mat(), Bi.mat());
    int64_t nnz = 0;
    cbh_mat_info(Ci, nullptr, nullptr, &nnz, nullptr, nullptr);
    if (nnz > 0) tomerge.push_back(Ci);  // `if(!C_cont->isZero()) tomerge.push_back`
    else cbh_mat_free(context(), Ci);
  }  // received blocks are freed at the end of their stage (the reference's clearA/clearB = i != self)
  if (tomerge.empty()) {
    cbh_mat* C = nullptr;
    int rc = cbh_mat_create(context(), C_m, C_n, 0, 0, dtype_of<NUO>::value, (int64_t)sizeof(NUO), &C);
    if (rc != CBH_OK) die(context(), rc, "cbh_mat_create");
    return C;
  }
  if (tomerge.size() == 1) return tomerge[0];  // one partial: it is the product (no copy round trip)
  return merge_all(semiring_traits<SR>::code, tomerge);
}

// The stage broadcasts of the overlapped drivers run on a stream of their own: the multiply of
// stage i (context stream) waits only for stage i's broadcasts (an event), so later stages' RCCL
// transfers overlap it (Mult_AnXBn_Overlap, ParFriends.h:1110-1235: MPI_Ibcast of every stage
// up front, each multiply after MPI_Waitall of its stage).
inline hipStream_t comm_stream() {
  static hipStream_t s = [] {
    hipStream_t x = nullptr;
    if (hipStreamCreateWithFlags(&x, hipStreamNonBlocking) != hipSuccess) die(context(), CBH_E_HIP, "hipStreamCreate");
    return x;
  }();
  return s;
}

// SUMMA over two device blocks with every stage's broadcasts posted up front on comm_stream():
// receive blocks are allocated first (their memory ordered before the transfers by an event on
// the context stream), stage i's multiply waits on stage i's event; the non-empty stage products
// are appended to `partials` (merged by the caller). The host-staged transport
// (COMBBLAS_HIP_COMM=mpi) runs the stages one after another.
template <class SR, class NUO, class IU, class NU1, class NU2>
void summa_overlap(SpDCColsDev<IU, NU1>& Aloc, combblas::CommGrid* GA, SpDCColsDev<IU, NU2>& Bloc,
                   combblas::CommGrid* GB, std::shared_ptr<combblas::CommGrid>& GridC, std::vector<cbh_mat*>& partials) {
  int stages, dummy;
  GridC = ProductGrid(GA, GB, stages, dummy, dummy);  // found by ADL (a friend of CommGrid)
  auto Asizes = GetSetSizes(Aloc, GA->GetRowWorld());
  auto Bsizes = GetSetSizes(Bloc, GB->GetColWorld());
  const int Aself = GA->GetRankInProcRow(), Bself = GB->GetRankInProcCol();
  std::vector<std::unique_ptr<SpDCColsDev<IU, NU1>>> Ar(stages);
  std::vector<std::unique_ptr<SpDCColsDev<IU, NU2>>> Br(stages);
  auto Ai = [&](int i) -> SpDCColsDev<IU, NU1>& { return i == Aself ? Aloc : *Ar[i]; };
  auto Bi = [&](int i) -> SpDCColsDev<IU, NU2>& { return i == Bself ? Bloc : *Br[i]; };
  for (int i = 0; i < stages; ++i) {
    if (i != Aself) Ar[i].reset(new SpDCColsDev<IU, NU1>());
    if (i != Bself) Br[i].reset(new SpDCColsDev<IU, NU2>());
    bcast_alloc(GridC->GetRowWorld(), Ai(i), Asizes[i], i);
    bcast_alloc(GridC->GetColWorld(), Bi(i), Bsizes[i], i);
  }
  hipStream_t cs = comm_stream(), ks = reinterpret_cast<hipStream_t>(cbh_ctx_stream(context()));
  const bool overlap = !use_mpi_transport();
  std::vector<hipEvent_t> done(stages, nullptr);
  if (overlap) {
    MPI_Comm rw = GridC->GetRowWorld(), cw = GridC->GetColWorld();
    int rws = 1, cws = 1;
    MPI_Comm_size(rw, &rws);
    MPI_Comm_size(cw, &cws);
    if (rws > 1) (void)rccl_comm_for(rw);  // communicators exist before the grouped calls
    if (cws > 1) (void)rccl_comm_for(cw);
    hipEvent_t ready;
    if (hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess) die(context(), CBH_E_HIP, "hipEventCreate");
    hip_check(hipEventRecord(ready, ks), "hipEventRecord");  // the receive blocks' memory: ordered after the context stream's work
    hip_check(hipStreamWaitEvent(cs, ready, 0), "hipStreamWaitEvent");
    hip_check(hipEventDestroy(ready), "hipEventDestroy");
    for (int i = 0; i < stages; ++i) {
      rccl_check(ncclGroupStart(), "ncclGroupStart");
      bcast_arrays(rw, Ai(i), Asizes[i], i, cs, true);
      bcast_arrays(cw, Bi(i), Bsizes[i], i, cs, true);
      rccl_check(ncclGroupEnd(), "ncclGroupEnd");
      if (hipEventCreateWithFlags(&done[i], hipEventDisableTiming) != hipSuccess) die(context(), CBH_E_HIP, "hipEventCreate");
      hip_check(hipEventRecord(done[i], cs), "hipEventRecord");
    }
  }
  for (int i = 0; i < stages; ++i) {
    if (overlap) {
      hip_check(hipStreamWaitEvent(ks, done[i], 0), "hipStreamWaitEvent");
    } else {
      bcast_arrays(GridC->GetRowWorld(), Ai(i), Asizes[i], i, ks);
      bcast_arrays(GridC->GetColWorld(), Bi(i), Bsizes[i], i, ks);
    }
    cbh_mat* Ci = local_multiply<SR, NUO, NU1, NU2>(Ai(i).mat(), Bi(i).mat());
    int64_t nnz = 0;
    cbh_mat_info(Ci, nullptr, nullptr, &nnz, nullptr, nullptr);
    if (nnz > 0) partials.push_back(Ci);
    else cbh_mat_free(context(), Ci);
    if (i != Aself) Ar[i].reset();  // the reference's clearA / clearB = i != self
    if (i != Bself) Br[i].reset();
  }
  for (hipEvent_t e : done)
    if (e) hip_check(hipEventDestroy(e), "hipEventDestroy");
}

inline cbh_mat* merge_partials(cbh_semiring sr, std::vector<cbh_mat*>& parts, int64_t m, int64_t n, int dtype,
                               int64_t vbytes) {
  if (parts.empty()) {
    cbh_mat* C = nullptr;
    int rc = cbh_mat_create(context(), m, n, 0, 0, (cbh_dtype)dtype, vbytes, &C);
    if (rc != CBH_OK) die(context(), rc, "cbh_mat_create");
    return C;
  }
  cbh_mat* C = parts.size() == 1 ? parts[0] : merge_all(sr, parts);
  parts.clear();
  return C;
}

// SpParMat<.., SpDCCols> <-> SpParMat<.., SpDCColsDev>: one upload / download of the local block
template <class IT, class NT>
combblas::SpParMat<IT, NT, SpDCColsDev<IT, NT>> to_device(combblas::SpParMat<IT, NT, combblas::SpDCCols<IT, NT>>& A) {
  return combblas::SpParMat<IT, NT, SpDCColsDev<IT, NT>>(new SpDCColsDev<IT, NT>(A.seq()), A.getcommgrid());
}
template <class IT, class NT>
combblas::SpParMat<IT, NT, combblas::SpDCCols<IT, NT>> to_host(combblas::SpParMat<IT, NT, SpDCColsDev<IT, NT>>& A) {
  return combblas::SpParMat<IT, NT, combblas::SpDCCols<IT, NT>>(A.seq().to_host(), A.getcommgrid());
}

}  // namespace combblas_hip

namespace combblas {

// (equal value types: promote.h's promote_trait<T, T> already gives T)
template <class IT, class NT1, class NT2>
struct promote_trait<combblas_hip::SpDCColsDev<IT, NT1>, combblas_hip::SpDCColsDev<IT, NT2>,
                     typename std::enable_if<!std::is_same<NT1, NT2>::value>::type> {
  typedef combblas_hip::SpDCColsDev<IT, typename promote_trait<NT1, NT2>::T_promote> T_promote;
};

// Mult_AnXBn_Synch (ParFriends.h:1004-1108) for device-resident operands: the same SUMMA stage
// loop, sizes exchanged on the host, blocks broadcast and multiplied in HBM, partials merged on
// the device, C returned device-resident.
template <typename SR, typename NUO, typename UDERO, typename IU, typename NU1, typename NU2>
SpParMat<IU, NUO, UDERO> Mult_AnXBn_Synch(SpParMat<IU, NU1, combblas_hip::SpDCColsDev<IU, NU1>>& A,
                                          SpParMat<IU, NU2, combblas_hip::SpDCColsDev<IU, NU2>>& B,
                                          bool clearA = false, bool clearB = false) {
  static_assert(std::is_same<UDERO, combblas_hip::SpDCColsDev<IU, NUO>>::value,
                "device-resident operands give a device-resident product");
  if (!CheckSpGEMMCompliance(A, B)) return SpParMat<IU, NUO, UDERO>();
  std::shared_ptr<CommGrid> GridC;
  cbh_mat* C = combblas_hip::summa_blocks<SR, NUO>(A.seq(), A.getcommgrid().get(), B.seq(), B.getcommgrid().get(), GridC);
  if (clearA) A.seq() = combblas_hip::SpDCColsDev<IU, NU1>();
  if (clearB) B.seq() = combblas_hip::SpDCColsDev<IU, NU2>();
  return SpParMat<IU, NUO, UDERO>(new UDERO(C), GridC);
}

// Mult_AnXBn_Overlap (ParFriends.h:1110-1235) for device-resident operands: every stage's
// broadcasts posted up front on the communication stream, each stage's multiply as soon as its
// blocks have arrived, the partials merged on the device.
template <typename SR, typename NUO, typename UDERO, typename IU, typename NU1, typename NU2>
SpParMat<IU, NUO, UDERO> Mult_AnXBn_Overlap(SpParMat<IU, NU1, combblas_hip::SpDCColsDev<IU, NU1>>& A,
                                            SpParMat<IU, NU2, combblas_hip::SpDCColsDev<IU, NU2>>& B,
                                            bool clearA = false, bool clearB = false) {
  static_assert(std::is_same<UDERO, combblas_hip::SpDCColsDev<IU, NUO>>::value,
                "device-resident operands give a device-resident product");
  if (!CheckSpGEMMCompliance(A, B)) return SpParMat<IU, NUO, UDERO>();
  const IU C_m = A.seq().getnrow(), C_n = B.seq().getncol();
  std::shared_ptr<CommGrid> GridC;
  std::vector<cbh_mat*> parts;
  combblas_hip::summa_overlap<SR, NUO>(A.seq(), A.getcommgrid().get(), B.seq(), B.getcommgrid().get(), GridC, parts);
  if (clearA) A.seq() = combblas_hip::SpDCColsDev<IU, NU1>();
  if (clearB) B.seq() = combblas_hip::SpDCColsDev<IU, NU2>();
  cbh_mat* C = combblas_hip::merge_partials(combblas_hip::semiring_traits<SR>::code, parts, C_m, C_n,
                                            combblas_hip::dtype_of<NUO>::value, (int64_t)sizeof(NUO));
  return SpParMat<IU, NUO, UDERO>(new UDERO(C), GridC);
}

// Mult_AnXBn_DoubleBuff (ParFriends.h:798-997) for device-resident operands: the inner dimension
// in two halves (SpDCCols::Split of A's columns and of the transposed B), each half a SUMMA round with overlapped broadcasts of half-blocks -- 2 * stages
// partials, merged on the device.
template <typename SR, typename NUO, typename UDERO, typename IU, typename NU1, typename NU2>
SpParMat<IU, NUO, UDERO> Mult_AnXBn_DoubleBuff(SpParMat<IU, NU1, combblas_hip::SpDCColsDev<IU, NU1>>& A,
                                               SpParMat<IU, NU2, combblas_hip::SpDCColsDev<IU, NU2>>& B,
                                               bool clearA = false, bool clearB = false) {
  static_assert(std::is_same<UDERO, combblas_hip::SpDCColsDev<IU, NUO>>::value,
                "device-resident operands give a device-resident product");
  if (!CheckSpGEMMCompliance(A, B)) return SpParMat<IU, NUO, UDERO>();
  const IU C_m = A.seq().getnrow(), C_n = B.seq().getncol();
  // SpDCCols::Split: columns [0, n/2) and [n/2, n) of A's block; of B's transposed block, so B's
  // rows [0, m/2) and [m/2, m) -- each rank cuts its own block (stage i's A and B halves meet on
  // the same k range: A_i's columns are B_i's rows)
  const int64_t ka = A.seq().getncol(), kb = B.seq().getnrow();
  cbh_ctx* ctx = combblas_hip::context();
  cbh_mat *a1 = nullptr, *a2 = nullptr, *b1 = nullptr, *b2 = nullptr;
  if (cbh_mat_col_slice(ctx, A.seq().mat(), 0, ka / 2, &a1) != CBH_OK ||
      cbh_mat_col_slice(ctx, A.seq().mat(), ka / 2, ka, &a2) != CBH_OK ||
      cbh_mat_row_slice(ctx, B.seq().mat(), 0, kb / 2, &b1) != CBH_OK ||
      cbh_mat_row_slice(ctx, B.seq().mat(), kb / 2, kb, &b2) != CBH_OK)
    combblas_hip::die(ctx, CBH_E_INTERNAL, "DoubleBuff split");
  if (clearA) A.seq() = combblas_hip::SpDCColsDev<IU, NU1>();
  if (clearB) B.seq() = combblas_hip::SpDCColsDev<IU, NU2>();
  std::shared_ptr<CommGrid> GridC;
  std::vector<cbh_mat*> parts;
  {
    combblas_hip::SpDCColsDev<IU, NU1> A1(a1);
    combblas_hip::SpDCColsDev<IU, NU2> B1(b1);
    combblas_hip::summa_overlap<SR, NUO>(A1, A.getcommgrid().get(), B1, B.getcommgrid().get(), GridC, parts);
  }
  {
    combblas_hip::SpDCColsDev<IU, NU1> A2(a2);
    combblas_hip::SpDCColsDev<IU, NU2> B2(b2);
    combblas_hip::summa_overlap<SR, NUO>(A2, A.getcommgrid().get(), B2, B.getcommgrid().get(), GridC, parts);
  }
  cbh_mat* C = combblas_hip::merge_partials(combblas_hip::semiring_traits<SR>::code, parts, C_m, C_n,
                                            combblas_hip::dtype_of<NUO>::value, (int64_t)sizeof(NUO));
  return SpParMat<IU, NUO, UDERO>(new UDERO(C), GridC);
}

}  // namespace combblas
