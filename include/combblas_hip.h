/*
 * combblas_hip.h — C-ABI of the MI355X (gfx950) semiring SpGEMM hot path.
 *
 * Plain pointers and sizes only (no torch / no C++ types). The C++ drop-in adaptor
 * (include/combblas_hip/HipSpGEMM.h) and the Python host mirror (combblas_amd/) both
 * sit on top of this interface. Every entry point names the reference interface it
 * replaces:
 *
 *   cbh_spgemm            LocalHybridSpGEMM<SR,NTO>        include/CombBLAS/mtSpGEMM.h:213-460
 *                         LocalSpGEMMHash<SR,NTO>(sort)     include/CombBLAS/mtSpGEMM.h:463-656
 *                         LocalSpGEMM<SR,NTO> (heap)        include/CombBLAS/mtSpGEMM.h:74-202
 *   cbh_spgemm_symbolic   estimateFLOP + estimateNNZ_Hash   include/CombBLAS/mtSpGEMM.h:1057-1134, 806-933
 *                         (+ prefixsum, mtSpGEMM.h:23-70)
 *   cbh_merge             MultiwayMerge<SR>                 include/CombBLAS/MultiwayMerge.h:411-526
 *                         MultiwayMergeHash<SR>             include/CombBLAS/MultiwayMerge.h:536-684
 *   cbh_mat_*             SpDCCols / Dcsc storage           include/CombBLAS/dcsc.h:124-130,
 *                         (GetEssentials / Create)           SpDCCols.cpp:46,787-845
 *   cbh_spgemm_phased     MemEfficientSpGEMM phase loop     include/CombBLAS/ParFriends.h:449-730
 *                         (B split into column phases, SpDCCols::ColSplit SpDCCols.cpp:936-1090)
 *   cbh_rmat_edges        RefGen21::make_graph (packed)     include/CombBLAS/RefGen21.h:246-301
 *   cbh_edges_to_csc      SpParMat(DistEdgeList, removeloops) SpParMat.cpp:3140-3253, SpTuples.cpp:70-118
 *
 * Status codes mirror the reference's MPI_Abort codes (include/CombBLAS/SpDefs.h:72-78):
 * 0 ok, 3001 GRIDMISMATCH, 3002 DIMMISMATCH, 3005 MATRIXALIAS, plus CBH_E_* below.
 * Threading: one host thread per context (the reference calls the kernel from one thread
 * per MPI rank). The library never calls MPI.
 */
#ifndef COMBBLAS_HIP_H
#define COMBBLAS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- status codes */
#define CBH_OK 0
#define CBH_E_GRIDMISMATCH 3001 /* SpDefs.h GRIDMISMATCH */
#define CBH_E_DIMMISMATCH 3002  /* SpDefs.h DIMMISMATCH: A.getncol() != B.getnrow(), bad sizes */
#define CBH_E_MATRIXALIAS 3005  /* SpDefs.h MATRIXALIAS */
#define CBH_E_HIP 4001          /* a HIP runtime call failed (see cbh_last_error) */
#define CBH_E_OOM 4002          /* device allocation failed */
#define CBH_E_ARG 4003          /* invalid argument (null pointer, unknown semiring/dtype) */
#define CBH_E_INTERNAL 4004     /* a device-side consistency check failed */
#define CBH_E_NODEVICE 4005     /* no HIP device visible */

/* ---------------------------------------------------------------- semirings / value types
 * Built-in semirings (Semirings.h). The value type is both input and output type
 * (T1 == T2 == T_promote), as in every hot-path call site listed in SURVEY.md §8(a).   */
typedef enum cbh_semiring {
  CBH_SR_PLUS_TIMES = 0, /* PlusTimesSRing<T,T>   Semirings.h:212-232 */
  CBH_SR_SELECT_MAX = 1, /* SelectMaxSRing<T,T>   Semirings.h:165-187: add=max, multiply=a*b */
  CBH_SR_MIN_PLUS = 2,   /* MinPlusSRing<T,T>     Semirings.h:235-255: add=min, multiply=inf_plus */
  CBH_SR_OR_AND = 3,     /* boolean OR-AND (PlusTimesSRing<bool,bool>, KTipsSR) */
  CBH_SR_SELECT_2ND = 4  /* Select2ndSRing<T,T,T> Semirings.h:143-163 (non-commutative add) */
} cbh_semiring;

typedef enum cbh_dtype {
  CBH_F64 = 0,   /* double  */
  CBH_I64 = 1,   /* int64_t */
  CBH_BOOL = 2,  /* bool, one byte per value */
  CBH_F32 = 3,   /* float   */
  CBH_I32 = 4,   /* int32_t */
  CBH_OPAQUE = 5 /* a user value type of a fixed byte size (cbh_mat_upload_bytes; user semirings) */
} cbh_dtype;

/* cbh_spgemm flags */
#define CBH_SORTED_ROWS 0x1u   /* rows sorted within each column (LocalHybridSpGEMM, LocalSpGEMMHash sort=true) */
#define CBH_KEEP_EMPTY_COLS 0x2u /* keep C columns of B's nzc even when empty (SpTuples view); default drops them (DCSC) */
/* Reference-order accumulation (device/order_kernel.h): after the throughput pass, every output is
 * re-folded in exactly the order the reference folds it, so floating-point sums (and any
 * non-commutative add) are bit-identical to the stock kernel's: CBH_ORDER_HYBRID follows
 * LocalHybridSpGEMM (heap branch for columns with cr = flops / nnz < 2, hash branch otherwise,
 * mtSpGEMM.h:310), CBH_ORDER_HEAP LocalSpGEMM, CBH_ORDER_HASH LocalSpGEMMHash. Without them the
 * products of one output are summed in arrival order (exact for integer, bool, min and max). */
#define CBH_ORDER_HYBRID 0x200u
#define CBH_ORDER_HEAP 0x400u
#define CBH_ORDER_HASH 0x800u

/* ---------------------------------------------------------------- matrices
 * A local sparse block in DCSC form (combblas::Dcsc: cp[nzc+1], jc[nzc], ir[nnz], numx[nnz]).
 * Row ids are local 32-bit (a local block has < 2^31 rows); column pointers and nnz are 64-bit. */
typedef struct cbh_dcsc {
  int64_t m, n;      /* SpDCCols::getnrow()/getncol() */
  int64_t nnz, nzc;  /* SpDCCols::getnnz()/getnzc() */
  const int64_t* cp; /* nzc+1 */
  const int64_t* jc; /* nzc   */
  const int32_t* ir; /* nnz   */
  const void* num;   /* nnz values of dtype */
} cbh_dcsc;

typedef struct cbh_ctx cbh_ctx; /* one device + one stream + a stream-ordered memory pool */
typedef struct cbh_mat cbh_mat; /* a device-resident DCSC block */

int cbh_ctx_create(int device, cbh_ctx** ctx);
int cbh_ctx_destroy(cbh_ctx* ctx);
/* Visible HIP devices (CBH_E_NODEVICE when none) and the PCI bus id of one ("0000:xx:00.0"): the
 * C++ adaptors resolve a rank's device with them and check that node-local RCCL peers hold
 * distinct devices (HipSpGEMM.h context(), SpParMatDev.h rccl_comm_for). */
int cbh_device_count(int* n);
int cbh_device_pci_id(int device, char* buf, int len);
/* The device a context drives. */
int cbh_ctx_device(cbh_ctx* ctx, int* device);
/* Use an existing hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL = own stream. */
int cbh_ctx_set_stream(cbh_ctx* ctx, void* hip_stream);
void* cbh_ctx_stream(cbh_ctx* ctx);
int cbh_ctx_synchronize(cbh_ctx* ctx);
/* Synchronize and return the context's cached device blocks and phase workspace to HIP (the
 * default allocator keeps freed blocks for reuse in stream order).                            */
int cbh_ctx_trim(cbh_ctx* ctx);
/* Synchronize and return at least `bytes` of the context's cached device blocks to HIP, largest
 * first (all of them if fewer are cached); live blocks and the phase workspace stay. */
int cbh_ctx_release(cbh_ctx* ctx, int64_t bytes);
const char* cbh_last_error(cbh_ctx* ctx);
/* Device scratch from the context's allocator (its block cache, and on OOM its fallback of
 * returning cached blocks to HIP), stream-ordered on the context's stream: the caller's kernels
 * that use it must run on that stream (cbh_ctx_stream), and cbh_ctx_free may be called as soon as
 * they are enqueued. */
int cbh_ctx_alloc(cbh_ctx* ctx, int64_t bytes, void** ptr);
int cbh_ctx_free(cbh_ctx* ctx, void* ptr);
/* Sub-tiles the task kernels retried with half the row range (table overflow, commit queue) since
 * the last call; resets the counter (diagnostics and tests). */
int cbh_ctx_take_retries(cbh_ctx* ctx, int64_t* subtile_retries);
/* Memory held by the context's default allocator (live blocks, cached free blocks) and the
 * device's free / total memory (hipMemGetInfo); any pointer may be NULL. */
int cbh_ctx_memory(cbh_ctx* ctx, int64_t* live_bytes, int64_t* cached_bytes, int64_t* device_free,
                   int64_t* device_total);
/* The large numeric hash kernel's configuration: home slots T of its order-preserving table (plus
 * 64 guard slots; a sub-tile plans T/2 outputs), threads per workgroup, products per thread per
 * gather step. */
int cbh_hash_config(int64_t* table_slots, int64_t* threads, int64_t* per_thread);
/* Route every device allocation of this context through caller callbacks (e.g. the torch
 * caching allocator), stream-ordered on `stream`. NULL alloc restores the built-in block cache.        */
typedef void* (*cbh_alloc_fn)(void* user, int64_t bytes, void* stream);
typedef void (*cbh_free_fn)(void* user, void* ptr, void* stream);
int cbh_ctx_set_allocator(cbh_ctx* ctx, cbh_alloc_fn alloc, cbh_free_fn release, void* user);
/* Workspace budget for cbh_spgemm_phased (bytes of output buffer per phase); 0 = auto. */
int cbh_ctx_set_phase_budget(cbh_ctx* ctx, int64_t bytes);
/* Share of the device's HBM one plan's stored dense-task bitmaps may take (default CBH_BMP_FRAC,
 * 0.4); 0 = store none (the dense tasks run the hash kernels). Callers holding several plans at
 * once (the C++ phase loop's stage plans) split one budget between them. A negative value
 * restores the default.                                                                          */
int cbh_ctx_set_bitmap_fraction(cbh_ctx* ctx, double frac);

/* Copy a host DCSC into a new device matrix (SpParHelper::BCastMatrix receive side / upload). */
int cbh_mat_upload(cbh_ctx* ctx, const cbh_dcsc* host, cbh_dtype dtype, cbh_mat** out);
/* Copy a host DCSC whose values are an opaque type of value_bytes bytes (a user semiring's NT). */
int cbh_mat_upload_bytes(cbh_ctx* ctx, const cbh_dcsc* host, int64_t value_bytes, cbh_mat** out);
/* An uninitialised device matrix of the given sizes (the receive side of a broadcast,
 * SpDCCols::Create(essentials), SpDCCols.cpp:787-795); value_bytes is used for CBH_OPAQUE. */
int cbh_mat_create(cbh_ctx* ctx, int64_t m, int64_t n, int64_t nnz, int64_t nzc, cbh_dtype dtype,
                   int64_t value_bytes, cbh_mat** out);
/* A device copy of a matrix (SpDCCols copy constructor, SpDCCols.cpp:214-226). */
int cbh_mat_clone(cbh_ctx* ctx, const cbh_mat* src, cbh_mat** out);
/* Bytes per value of a matrix (any dtype). */
int64_t cbh_mat_value_bytes(const cbh_mat* mat);
/* Wrap device arrays without copying. The caller keeps them alive until cbh_mat_free. */
int cbh_mat_wrap_device(cbh_ctx* ctx, const cbh_dcsc* dev, cbh_dtype dtype, cbh_mat** out);
/* Sizes (host pointers, any may be NULL). */
int cbh_mat_info(const cbh_mat* mat, int64_t* m, int64_t* n, int64_t* nnz, int64_t* nzc, int* dtype);
/* Device pointers of the matrix arrays (valid until cbh_mat_free). */
int cbh_mat_device_arrays(const cbh_mat* mat, const int64_t** cp, const int64_t** jc,
                          const int32_t** ir, const void** num);
/* Chunked host transfers through the context's pinned staging buffers (the drop-in adaptors'
 * SpDCCols <-> device path, HipSpGEMM.h). Entries move in chunks of `chunk` (<= 0: 4 M); while
 * the copy engine moves chunk k+1, the callback converts chunk k on the host (the adaptor's
 * OpenMP threads: int64 row ids <-> the device's int32, AoS tuples, ...).
 *   upload: cbh_fill_fn writes entries [first, first+count) into the staging arrays ir / num
 *           (num: value_bytes per entry); cp / jc are copied as given (nzc + 1 and nzc int64s).
 *   download: cbh_take_fn reads entries [first, first+count) of the matrix from staging.
 * A callback returning nonzero aborts the transfer with that code.                           */
typedef int (*cbh_fill_fn)(void* user, int64_t first, int64_t count, int32_t* ir, void* num);
typedef int (*cbh_take_fn)(void* user, int64_t first, int64_t count, const int32_t* ir, const void* num);
int cbh_mat_upload_chunks(cbh_ctx* ctx, int64_t m, int64_t n, int64_t nnz, int64_t nzc, const int64_t* cp,
                          const int64_t* jc, cbh_dtype dtype, int64_t value_bytes, int64_t chunk,
                          cbh_fill_fn fill, void* user, cbh_mat** out);
int cbh_mat_download_chunks(cbh_ctx* ctx, const cbh_mat* mat, int64_t* cp, int64_t* jc, int64_t chunk,
                            cbh_take_fn take, void* user);
/* Copy the matrix arrays to caller buffers; dst_on_device selects hipMemcpy direction. */
int cbh_mat_copy_out(cbh_ctx* ctx, const cbh_mat* mat, int64_t* cp, int64_t* jc, int32_t* ir,
                     void* num, int dst_on_device);
int cbh_mat_free(cbh_ctx* ctx, cbh_mat* mat);

/* ---------------------------------------------------------------- the hot path
 * C = A * B over semiring sr. A, B, C share dtype. C is a new device matrix (caller frees).
 * Output contract = LocalHybridSpGEMM's SpTuples converted to SpDCCols: columns in B's
 * order, rows ascending within each column, explicit zeros kept, empty columns dropped
 * unless CBH_KEEP_EMPTY_COLS.                                                            */
int cbh_spgemm(cbh_ctx* ctx, cbh_semiring sr, const cbh_mat* A, const cbh_mat* B, uint32_t flags,
               cbh_mat** C);
/* Symbolic only: total flops (estimateFLOP) and exact nnz(C) (estimateNNZ_Hash).
 * Optional per-column outputs (device pointers, length B.nzc) may be NULL.               */
int cbh_spgemm_symbolic(cbh_ctx* ctx, const cbh_mat* A, const cbh_mat* B, int64_t* flops,
                        int64_t* nnzC, int64_t* col_flops_dev, int64_t* col_nnz_dev);
/* k-way merge of column-sorted partial products with SR::add on duplicates. */
int cbh_merge(cbh_ctx* ctx, cbh_semiring sr, int nlists, const cbh_mat* const* parts, cbh_mat** C);

/* Phased C = A * B for products larger than HBM: B's columns are processed in phases whose
 * output fits the phase budget; each phase's C block is materialised in device memory and
 * folded into the statistics below, then its buffer is reused. */
typedef struct cbh_phase_stats {
  int64_t flops;        /* number of SR::multiply calls (EstimateFLOP) */
  int64_t nnz;          /* nnz(C) */
  int64_t phases;       /* number of column phases used */
  double value_sum;     /* sum of C's values as double (checksum) */
  uint64_t digest;      /* order-sensitive digest of (col,row,value bits) in C order */
} cbh_phase_stats;
#define CBH_PHASE_CHECKSUM 0x100u /* also compute value_sum/digest (extra read of each phase) */
int cbh_spgemm_phased(cbh_ctx* ctx, cbh_semiring sr, const cbh_mat* A, const cbh_mat* B,
                      uint32_t flags, cbh_phase_stats* stats);
/* Per-phase consumer of cbh_spgemm_phased (the role of MemEfficientSpGEMM's per-phase
 * MCLPruneRecoverySelect + ColConcatenate, ParFriends.h:694-721): called once per phase, in
 * column order, after the phase's numeric launches were queued on the context stream, with a
 * NON-OWNING view of C(:, B's column slots [slot0, slot1)) -- an m x B.n DCSC that keeps the
 * phase's empty columns (CBH_KEEP_EMPTY_COLS form). The view's arrays live in the phase
 * workspace and are overwritten by the next phase: copy (cbh_mat_clone), reduce or prune it on
 * the context stream before returning. A nonzero return aborts the product with that code.
 * fn = NULL removes the consumer.                                                              */
typedef int (*cbh_phase_fn)(void* user, int64_t phase, int64_t slot0, int64_t slot1, const cbh_mat* Cphase);
int cbh_ctx_set_phase_consumer(cbh_ctx* ctx, cbh_phase_fn fn, void* user);

/* Timing of the last cbh_spgemm/cbh_spgemm_phased call, per kernel class, measured with
 * hipEvents on the context stream (milliseconds; -1 when not recorded).                  */
typedef struct cbh_kernel_times {
  double symbolic_ms, numeric_ms, total_ms;
  int64_t numeric_launches;
} cbh_kernel_times;
int cbh_last_kernel_times(cbh_ctx* ctx, cbh_kernel_times* t);
int cbh_ctx_enable_timing(cbh_ctx* ctx, int enable);

/* Per-kernel-class totals accumulated while timing is enabled: HIP-event time of every launch,
 * launch count, and the ALGORITHMIC bytes those launches processed (SURVEY.md §8(d):
 * (s_i+s_v)*(nnz(B)+flops+nnz(C)) + column pointers; the symbolic pass counts row ids only).  */
#define CBH_K_SYM_LARGE 0 /* task_kernel<...,8192,512,512,16,MODE_TSYM>    symbolic hash, work > 2048   */
#define CBH_K_SYM_SMALL 1 /* wave_kernel<...,2048,4,4,0>                  symbolic, one task per wave  */
#define CBH_K_NUM_LARGE 2 /* task_kernel<SR,2048,512,512,4,MODE_TNUM>     numeric hash sub-tiles       */
#define CBH_K_NUM_SMALL 3 /* wave_kernel<SR,512,4,4,1>                    numeric, one task per wave   */
#define CBH_K_MERGE_SYM 4
#define CBH_K_MERGE_NUM 5
#define CBH_K_NUM_DENSE 6 /* dense_kernel<SR,1024,1024,8,163776,KDENSE>   numeric bitmap-rank windows  */
#define CBH_K_SYM_MID 7   /* task_kernel<...,4096,256,256,4,MODE_TSYM>    symbolic, mid-size tasks     */
#define CBH_K_NUM_MID 8   /* task_kernel<SR,2048,256,256,4,MODE_TNUM>     numeric, mid-size tasks      */
#define CBH_K_SYM_BMP 9   /* dense_kernel<...,1024,1024,8,163776,KSYMB>   symbolic bitmap tasks        */
#define CBH_K_NKINDS 10
typedef struct cbh_kernel_stat {
  double ms;
  int64_t launches;
  double alg_bytes;
} cbh_kernel_stat;
int cbh_kernel_stats(cbh_ctx* ctx, int kind, cbh_kernel_stat* out);
int cbh_kernel_stats_reset(cbh_ctx* ctx);

/* ---------------------------------------------------------------- user semirings
 * LocalHybridSpGEMM<SR,NTO>(SpDCCols<IT,NT1>, SpDCCols<IT,NT2>) for a semiring the library was
 * not built with (Semirings.h:143-255 contract; NT1 != NT2 promotion). The library runs what
 * does not depend on the semiring -- the symbolic pass (estimateFLOP + estimateNNZ_Hash), the
 * task plan, the binning, C's allocation and column compaction -- and the caller launches the
 * numeric kernels instantiated for its semiring from the header-only device code
 * (include/combblas_hip/HipSpGEMMDevice.h -> device/numeric.h: cbh::run_numeric_plan<SR>) on
 * the plan's stream, between cbh_plan_numeric and cbh_plan_finish.                          */
typedef struct cbh_plan cbh_plan;
typedef struct cbh_numeric_plan {
  const int64_t* Acp; const int32_t* Air; const void* Anum;  /* A: dense column pointers, rows, values */
  const int64_t* Bcp; const int32_t* Bir; const void* Bnum;  /* B: DCSC pointers, rows, values         */
  const int32_t* hidx; const int32_t* htab; int64_t nblk; int32_t RB; /* hub row-block table: start + (position, row) pairs */
  const int32_t* tcol; const int32_t* tlo; const int32_t* thi; const uint8_t* tfull; /* tasks    */
  const int64_t* tcnt; const int64_t* toff;                  /* outputs per task, output offsets  */
  const int64_t* goff; int64_t* gcur0; int64_t* gcur1; int64_t* gend; /* chunked-task cursors    */
  int32_t* gnx0; int32_t* gnx1;                              /* rows at those cursors             */
  int* err;                                                  /* device consistency flags          */
  int64_t nnzA, ncolA, ntasks;
  const int32_t* order;                                      /* task ids in launch order          */
  int64_t dense_first, dense_count, large_first, large_count, small_first, small_count;
  void* stream;                                              /* hipStream_t of the context        */
  int64_t mid_first, mid_count;                              /* mid-size hash tasks (<= 1024 out) */
  const int64_t* boff; uint32_t* bmp;                        /* stored row bitmaps of dense tasks */
  int32_t* ghub;                                             /* hub id of each chunked-task entry */
  int64_t* gbase;                                            /* its A column's start              */
} cbh_numeric_plan;
/* bin every task for the hash kernels: the dense (bitmap-rank) kernel needs a lock-free SR::add
 * and 8-byte accumulators, the layout the plan's dense split is computed for (numeric.h
 * dense_capable<SR>) */
#define CBH_PLAN_NO_DENSE 0x1u
/* Symbolic pass of C = A*B (A and B values may differ in type); the plan owns its scratch. */
int cbh_plan_create(cbh_ctx* ctx, const cbh_mat* A, const cbh_mat* B, cbh_plan** plan);
int cbh_plan_info(const cbh_plan* plan, int64_t* flops, int64_t* nnzC);
/* Allocate C (value_bytes per value, CBH_OPAQUE unless it matches a built-in dtype the caller
 * names in dtype) and bin the tasks; fills the launch description. */
int cbh_plan_numeric(cbh_plan* plan, cbh_dtype dtype, int64_t value_bytes, uint32_t flags, cbh_mat** C,
                     cbh_numeric_plan* out);
/* After the caller's numeric launches: C's column pointers / ids (CBH_KEEP_EMPTY_COLS honoured)
 * and the device-side consistency checks. */
int cbh_plan_finish(cbh_plan* plan, cbh_mat* C, uint32_t flags);
int cbh_plan_destroy(cbh_plan* plan);
/* Phase loops over one planned product (MemEfficientSpGEMM, ParFriends.h:449-730: per phase a
 * LocalSpGEMM of A with a column slice of B) without a second symbolic pass: the exact nnz of
 * every nonzero column slot of B (device int64[B.nzc]), and C = A * B(:, slots [s0, s1)) for a
 * built-in semiring -- the same m x B.n matrix cbh_spgemm returns for that column slice.      */
int cbh_plan_col_nnz(const cbh_plan* plan, int64_t* col_nnz_dev);
int cbh_plan_spgemm_slots(cbh_plan* plan, cbh_semiring sr, int64_t s0, int64_t s1, uint32_t flags, cbh_mat** C);

/* ---------------------------------------------------------------- callers around the hot path
 * (device kernels in combblas_amd/csrc/apps.h)                           */
/* C = (A*B) .* M in one pass: Applications/TC.cpp:108-110 (Mult_AnXBn_Synch(L, L) then
 * C.EWiseMult(L, false), Friends.h:834-887). Pattern = pattern(A*B) ∩ pattern(M) (explicit zeros
 * count), rows ascending; values SR-sum * M(i,j), or the SR-sum alone with CBH_MASK_PATTERN.
 * Two evaluation orders, same result: EXPAND enumerates the products of A*B whose rows fall in
 * the mask column (work = flops of A*B); DOT intersects row i of A (A transposed on the device)
 * with column j of B for every mask entry (work = sum of the shorter lists) -- TC at scale 24.
 * Default: DOT when nnz(A) >= 65536, else EXPAND; the flags force one.                         */
#define CBH_MASK_PATTERN 0x4u
#define CBH_MASK_EXPAND 0x8u
#define CBH_MASK_DOT 0x10u
int cbh_spgemm_masked(cbh_ctx* ctx, cbh_semiring sr, const cbh_mat* A, const cbh_mat* B, const cbh_mat* M,
                      uint32_t flags, cbh_mat** C);
/* AT = A' on the device (SpDCCols::Transpose, SpDCCols.cpp): rows ascending in every column.
 * A.n < 2^31, nnz(A) < 2^31.                                                                   */
int cbh_transpose(cbh_ctx* ctx, const cbh_mat* A, cbh_mat** AT);
/* Value sum and order-sensitive digest of a block, the definition cbh_spgemm_phased's
 * CBH_PHASE_CHECKSUM and the oracle use: sum over entries p (in DCSC order) of
 * mix64(p ^ mix64(col ^ mix64(row ^ mix64(value bits)))) mod 2^64. Built-in dtypes only.        */
int cbh_mat_checksum(cbh_ctx* ctx, const cbh_mat* M, double* value_sum, uint64_t* digest);
/* The same for one block of a distributed C: its rows and column ids are offset by row_off /
 * col_off, and col_pos (host, M's nzc entries) holds the position of each nonzero column's first
 * entry in the WHOLE product's DCSC order, so that the blocks' digests sum (mod 2^64) to the
 * whole product's (bench_summa checks the N-rank product against the reference's digest). */
int cbh_mat_checksum_global(cbh_ctx* ctx, const cbh_mat* M, int64_t row_off, int64_t col_off, const int64_t* col_pos,
                            double* value_sum, uint64_t* digest);
/* C = A .* B (SpParMat::EWiseMult(B, false) -> Friends.h:834-887): intersection, values A*B. */
int cbh_ewise_mult(cbh_ctx* ctx, const cbh_mat* A, const cbh_mat* B, cbh_mat** C);
/* HipMCL column operations on f64 blocks (ParFriends.h:185-353). Vectors are device arrays over
 * the block's n columns.
 *   cbh_col_stats      cnt = nnz per column, cntp / sump = count / sum of the entries > hard
 *                      (A.Reduce(Column,...) and Prune(v <= hard).Reduce(Column,...), :196-200)
 *   cbh_kselect_*      SpParMat::Kselect1 (SpParMat.cpp:1413-1700) as an 8-pass radix select:
 *                      per pass, hist (nactive x 256) of the keys matching prefix above the digit
 *                      at `shift` (56, 48, ..., 0), then pick the digit holding rank (descending).
 *                      Histograms may be summed over a processor column between the two calls.
 *                      active_index[col] = slot in the active list or -1.
 *   cbh_kselect_cols   the same Kselect1 for columns held whole by this block, in one launch:
 *                      out[active_index[col]] = k-th largest (the smallest when fewer than k);
 *                      active columns without entries keep what out held (the caller's fill)
 *   cbh_prune_columns  keep entries with !(v < thresh[col]) (Dcsc::PruneColumn, dcsc.cpp:699-760)
 *   cbh_col_stats_kept count / sum of the entries cbh_prune_columns(thresh) would keep, per column
 *                      (ParFriends.h:318-329: the recovery check on the selected matrix) */
int cbh_col_stats(cbh_ctx* ctx, const cbh_mat* A, double hard, double* cnt, double* cntp, double* sump);
int cbh_kselect_hist(cbh_ctx* ctx, const cbh_mat* A, const int32_t* active_index, int64_t nactive,
                     const uint64_t* prefix, int shift, uint32_t* hist);
int cbh_kselect_pick(cbh_ctx* ctx, int64_t nactive, const uint32_t* hist, uint64_t* prefix, int64_t* rank,
                     int shift);
int cbh_kselect_value(cbh_ctx* ctx, int64_t nactive, const uint64_t* prefix, double* out);
int cbh_kselect_cols(cbh_ctx* ctx, const cbh_mat* A, const int32_t* active_index, int64_t nactive, int64_t k,
                     double* out);
int cbh_prune_columns(cbh_ctx* ctx, const cbh_mat* A, const double* thresh, cbh_mat** C);
int cbh_col_stats_kept(cbh_ctx* ctx, const cbh_mat* A, const double* thresh, double* cntk, double* sumk);

/* Whole-block MCLPruneRecoverySelect (ParFriends.h:185-353) on the device: column statistics,
 * recovery / selection Kselect1 (recoverNum-th / selectNum-th largest), the recovery check after
 * selection, then PruneColumn -- C is the pruned block (a new matrix; A is kept). Where the block's
 * columns are split over a processor column, `colsum` (non-NULL) sums a device buffer over it in
 * place (MPI_Allreduce / ncclAllReduce, the reference's Reduce(Column, ...) and Kselect1 gathers):
 * count values of type CBH_REDUCE_F64 (double) or CBH_REDUCE_U32 (uint32 histograms), queued on
 * the context stream; a nonzero return aborts with that code. NULL: columns held whole.          */
#define CBH_REDUCE_F64 0
#define CBH_REDUCE_U32 1
typedef int (*cbh_allreduce_fn)(void* user, void* dev_buf, int64_t count, int type);
int cbh_mcl_prune_recovery_select(cbh_ctx* ctx, const cbh_mat* A, double hardThreshold, int64_t selectNum,
                                  int64_t recoverNum, double recoverPct, cbh_allreduce_fn colsum, void* user,
                                  cbh_mat** C);
/* Output arena of the phased MCL drivers (MemEfficientSpGEMM, ParFriends.h:449-730): the pruned
 * pieces of every phase are written back to back into one pair of row / value arrays of
 * `capacity` entries, which cbh_arena_concat hands to the concatenated result without a copy -- a
 * near-capacity product never holds its pieces and their concatenation at once (C5: 148 GB).
 *   cbh_mcl_prune_recovery_select_arena  as cbh_mcl_prune_recovery_select; C's rows and values are
 *       written into the arena when they fit (C then borrows them), else allocated as usual
 *   cbh_arena_concat  the k pieces side by side (cbh_mat_col_concat_consume semantics: the parts are
 *       freed and cleared); without a copy of rows and values when the parts tile the arena in order
 *   cbh_arena_destroy frees whatever the arena still owns                                       */
typedef struct cbh_arena cbh_arena;
int cbh_arena_create(cbh_ctx* ctx, int64_t capacity, int64_t value_bytes, cbh_arena** out);
int cbh_arena_destroy(cbh_ctx* ctx, cbh_arena* arena);
int cbh_mcl_prune_recovery_select_arena(cbh_ctx* ctx, const cbh_mat* A, double hardThreshold, int64_t selectNum,
                                        int64_t recoverNum, double recoverPct, cbh_allreduce_fn colsum, void* user,
                                        cbh_arena* arena, cbh_mat** C);
int cbh_arena_concat(cbh_ctx* ctx, int k, cbh_mat** parts, cbh_arena* arena, cbh_mat** out);

/* ---------------------------------------------------------------- block column operations
 *   cbh_mat_col_slice   columns [c0, c1) of M as a new m x (c1-c0) block, ids rebased
 *                       (one piece of SpDCCols::ColSplit, SpDCCols.cpp:936-1012)
 *   cbh_mat_col_concat  the k blocks side by side (SpDCCols::ColConcatenate, SpDCCols.cpp:1014-1090):
 *                       rows = the largest m, columns offset by the earlier blocks' n            */
int cbh_mat_col_slice(cbh_ctx* ctx, const cbh_mat* M, int64_t c0, int64_t c1, cbh_mat** out);
/* The same column range as a VIEW: its column pointers and ids are its own (rebased), its rows and
 * values are M's own arrays (not copied, not freed with the view): free the view before M. The 3D
 * drivers' fiber exchange sends a layer partial's column pieces from it without copying them. */
int cbh_mat_col_view(cbh_ctx* ctx, const cbh_mat* M, int64_t c0, int64_t c1, cbh_mat** view);
int cbh_mat_col_concat(cbh_ctx* ctx, int k, const cbh_mat* const* parts, cbh_mat** out);
/* The same, releasing the parts as they are consumed (one array kind at a time: pointers, rows,
 * values), so the peak is the parts plus the largest output array instead of twice the matrix;
 * every parts[i] is freed and set to NULL -- on success, and also on a failure past the argument
 * checks (the parts are half consumed by then; no result is produced). ColConcatenate also
 * empties its inputs. cbh_arena_concat's copying fallback (pieces not tiling the arena) releases
 * the arena's rows and values as soon as they are copied.                                      */
int cbh_mat_col_concat_consume(cbh_ctx* ctx, int k, cbh_mat** parts, cbh_mat** out);
/* Rows [r0, r1) of the block as an (r1 - r0) x n block, row ids rebased, empty columns dropped
 * (Mult_AnXBn_DoubleBuff's row halves of B). */
int cbh_mat_row_slice(cbh_ctx* ctx, const cbh_mat* M, int64_t r0, int64_t r1, cbh_mat** out);
/* In place: the block's columns [c0, c0 + n) become columns [0, n) of an m x n block (a phase
 * piece of a plan's slot product, which keeps B's column ids, rebased like a ColSplit piece). */
int cbh_mat_rebase_cols(cbh_ctx* ctx, cbh_mat* M, int64_t c0, int64_t n);

/* ---------------------------------------------------------------- format conversions (device)
 *   cbh_tuples_to_dcsc  device COO (rows, cols, vals; any order, duplicates allowed) -> a DCSC block:
 *                       SpTuples::SortColBased + duplicate combination (sum; OR for bool, as
 *                       SpTuples(edges) SpTuples.cpp:70-118 and RemoveDuplicates :271-300 with the
 *                       default SumOp) + SpDCCols(const SpTuples&) SpDCCols.cpp:109-183.
 *                       CBH_TUPLES_DROP_LOOPS removes row == col entries (removeloops). nnz < 2^31.
 *   cbh_dcsc_to_tuples  a DCSC block -> device COO, column-sorted (SpTuples(const SpDCCols&),
 *                       SpTuples.cpp:181-200); buffers of M's nnz entries. */
#define CBH_TUPLES_DROP_LOOPS 0x1u
int cbh_tuples_to_dcsc(cbh_ctx* ctx, int64_t m, int64_t n, int64_t nnz, const int32_t* rows, const int64_t* cols,
                       const void* vals, cbh_dtype dtype, uint32_t flags, cbh_mat** out);
int cbh_dcsc_to_tuples(cbh_ctx* ctx, const cbh_mat* M, int32_t* rows, int64_t* cols, void* vals);

/* Config C5's input on the device (combblas_amd/csrc/mclgen.h): a planted-partition graph of n
 * vertices, power-law cluster sizes (2 + floor(6 * Lomax(alpha))), avg_deg / 2 draws per vertex
 * (a fraction p_in inside the vertex's cluster), symmetric, uniform (0, 1] weights, unit loops,
 * column-stochastic (MakeColStochastic, MCL.cpp:390-396); f64. Counter-based draws: the matrix
 * depends on the arguments only. n * avg_deg / 2 < 2^31.                                       */
int cbh_gen_planted_partition(cbh_ctx* ctx, int64_t n, int64_t avg_deg, uint64_t seed, double p_in, double alpha,
                              cbh_mat** out);

/* ---------------------------------------------------------------- inputs (host side) */
int cbh_rmat_edges(int scale, uint64_t userseed, int64_t start_edge, int64_t end_edge, int64_t* src,
                   int64_t* dst);
int cbh_edges_to_csc(int64_t m, int64_t n, int64_t nedges, const int64_t* rows, const int64_t* cols,
                     int removeloops, int64_t* colptr, int32_t* rowidx, int64_t* count,
                     int64_t* nnz_out);

/* Library version / build tag (for logs). */
const char* cbh_version(void);

#ifdef __cplusplus
}
#endif
#endif /* COMBBLAS_HIP_H */
