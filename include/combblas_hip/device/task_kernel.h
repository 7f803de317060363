// gfx950 SpGEMM kernels, TASK-PARALLEL form (the SpGEMM hot path; merges still use block_ops.h).
//
// A task is one row range [lo, hi) of one output column j (one nonzero column of B). Heavy
// columns are cut into tasks of about kTaskFlops products, so the heaviest column of R-MAT
// scale 22 (15.7 M products, 752 K outputs) spreads over hundreds of workgroups instead of one
// (the per-column row-tile loop of block_ops.h was tail-bound). R-MAT rows are scrambled
// (uniform), so equal-width row ranges carry equal work.
//
// Inside a task the range is processed in SUB-TILES that fit one LDS table, one after another.
// Every B entry k of the column keeps, in LDS, a cursor into its row-sorted A column and the row
// at that cursor: an entry with no product in the current sub-tile costs one LDS read (no global
// traffic); an active one finds the end of its segment (stop_search: 8 independent row loads,
// then, for long A columns, the row-block table of the hub columns bounds the search to one
// block). Products of a sub-tile are flattened (LDS scan of segment lengths), each thread
// gathers U of them before any table update (memory-level parallelism), and an owner map
// (segment starts + block max-scan) names the entry.
//
//   symbolic (MODE_TSYM): distinct rows of the task -> cnt[task]        [estimateNNZ_Hash, mtSpGEMM.h:806-933]
//            sub-tile = an LDS bitmap over 32*TA rows (exact, no hashing) or, for sparse ranges,
//            an LDS key hash of <= TA/2 products -- whichever needs fewer sub-tiles.
//   offsets : exclusive scan of cnt over tasks (a column's tasks are consecutive, in row order),
//             so every task knows where its outputs go and C's column pointers fall out.
//   numeric (MODE_TNUM): SR::add(SR::multiply(a,b)) into an order-preserving LDS hash (slot =
//            (row-lo)*T/(hi-lo), forward probing), sub-tiles of <= T/2 outputs, written at
//            toff[task] with rows ascending                              [LocalHybridSpGEMM, mtSpGEMM.h:289-441]
//            Commit without sorting: keys in different runs of occupied slots are already in
//            order, so slot s goes to (occupied slots before its run) + (rank of
//            its key inside the run) -- replaces the per-column std::sort (mtSpGEMM.h:434).
// Columns with more than EMAX entries are processed in entry chunks whose cursors live in HBM
// between sub-tiles (double-buffered, so that a retried sub-tile restarts from committed ones).
#pragma once

// CBH_GATHER_PIN (default 1): pin the window gathers before the updates (sweep() below)
// CBH_HASH_BATCH (A/B hook, default 0): the numeric hash issues the first probe of all U products
// of a batch before using any result, instead of probing each product to completion before the
// next one starts. Measured slower (round 6, profiles/r06/hash_batch: hash 236.7 -> 251.2 ms per
// scale-22 product): the kernel is issue-bound, not latency-bound, and the per-product pending
// flags cost more SALU mask arithmetic than the overlapped probes save
#ifndef CBH_HASH_BATCH
#define CBH_HASH_BATCH 0
#endif
#ifndef CBH_PROBE_BOUND
#define CBH_PROBE_BOUND 0
#endif
#ifndef CBH_GUARD_BRANCHLESS  // the numeric hash's per-product range guard as flag + clamp, not a
#define CBH_GUARD_BRANCHLESS 1  // branch (round 6: hash 229.4 -> 227.1 ms; on the dense kernel flat)
#endif
#ifndef CBH_GATHER_PIN
#define CBH_GATHER_PIN 1
#endif
#include "block_ops.h"

namespace cbh {

enum : int { MODE_TSYM = 0, MODE_TNUM = 1, MODE_TDENSE = 2 };
constexpr int32_t kNoRow = 0x7fffffff;
// cursor row not loaded yet (< every row range: the entry counts as active, and its first
// segment search starts AT the cursor, whose row the search loads with the following ones)
constexpr int32_t kUnknownRow = -2;
constexpr bool kAlignSubtiles = true;  // sub-tiles and dense windows end on row-block boundaries
constexpr int kSymWords = 12160;  // bitmap words of the large symbolic configuration (see TaskCfg::TA)
// numeric sub-tile: planned outputs, in eighths of the T home slots (3/8 and 5/8 measured slower:
// 97.6 and 93.5 vs 98.6 GFLOP/s at scale 22 with T 4096; 5/8 again with T 2048: hash 434 vs 360 ms)
constexpr int kFill8 = 4;
#ifndef CBH_FILL16  // (A/B hook) numeric sub-tile plan in sixteenths of T (8 = kFill8 / 8 = 1/2)
#define CBH_FILL16 8
#endif
// symbolic key-hash sub-tiles: keys, in eighths of TA (6/8 measured flat: symbolic 197 vs 193 ms)
constexpr int kSymFill8 = 4;
// dense numeric sub-tile capacity in quarters of T: 3 = 3072 values for T = 4096 (2 and 4
// measured slower: 98.7 / 104.5 vs 105.3 GFLOP/s at scale 22)
constexpr int kCapD4 = 3;
// a task runs dense when its dense sub-tiles are at most kDRatio4/4 of its hash sub-tiles. Round 4
// (2048-slot hash table, 262144-flop tasks): 5/6/7/8/10 -> 140.3/142.3/142.7/142.1/141.4 GFLOP/s at
// scale 22; rounds 2-3 had found 4..12 flat around 5 with the 4096-slot hash table.
// Round 5 (dense tasks on dense_kernel.h): 7/9/12 -> 164.4/165.6/165.1 and 164.0/165.2 (7 vs 9).
#ifndef CBH_DRATIO4  // (A/B hook: build variants only)
#define CBH_DRATIO4 9
#endif
constexpr int kDRatio4 = CBH_DRATIO4;

// Diagnostic build only (-DCBH_STAMPS, libcombblas_hip_stamps.so): thread 0 of every workgroup
// adds the s_memtime cycles of each kernel phase (delimited by block barriers) into g_stamps.
#ifdef CBH_STAMPS
// [0..11] phase cycles, [12] workgroups, [13] chunk-subtiles, [14] overflows, [15] products,
// [16] entry visits, [17] active entry visits, [18] active entries whose segment ends inside the
// 8-row window (short), [19] products of those, [20] hash sub-tile occupied slots (commit)
__device__ unsigned long long g_stamps[24];
#define CBH_STAMP(k)                                    \
  do {                                                  \
    if (threadIdx.x == 0) {                             \
      const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
      st_[k] += t_ - t_prev_;                           \
      t_prev_ = t_;                                     \
    }                                                   \
  } while (0)
#else
#define CBH_STAMP(k) \
  do {               \
  } while (0)
#endif

struct TaskArgs {
  const int64_t* Acp;  // A dense column pointers (A.n + 1)
  const int32_t* Air;
  const void* Anum;
  const int64_t* Bcp;  // B DCSC column pointers (per nonzero column slot)
  const int32_t* Bir;
  const void* Bnum;
  const int32_t* order;  // task ids in launch order
  int64_t norder;
  // row-block table of the HUB columns of A (>= kHubMin entries): hidx[k] = hub id or -1. Hub h
  // owns nblk + 2 int32 pairs from pair h*(nblk+2): pair 0 is the column's start (int64), pair
  // 1 + b = (first position of A(:,k), relative to its start, whose row is >= b*RB, the row there
  // or kNoRow), b = 0..nblk: one 8-B load gives a cursor and its row, and the start loads beside
  // it. Task and sub-tile boundaries sit on multiples of RB; RB = 0: no table.
  const int32_t* hidx;
  const int32_t* htab;
  int64_t nblk;
  int32_t RB;
  const int32_t* tcol;   // per task: column slot j
  const int32_t* tlo;    // per task: row range [lo, hi)
  const int32_t* thi;
  const uint8_t* tfull;  // per task: bit0 = lo is the column's first row, bit1 = hi past its last row
  const int64_t* twork;  // symbolic: flops of the task (estimate); numeric: exact output count
  int64_t* cnt;          // symbolic output
  const int64_t* toff;   // numeric: output offset of every task
  int64_t cbase;
  int32_t* Cir;
  void* Cnum;
  int64_t ccap;
  int* err;
  int64_t nnzA, ncolA, ntasks;
  // chunked tasks (more than EMAX entries): entry cursors kept in HBM between sub-tiles, double
  // buffered so that a retried sub-tile restarts from the last committed cursors; goff = per-task
  // offset into them
  const int64_t* goff;
  int64_t* gcur0;
  int64_t* gcur1;
  int64_t* gend;
  // the row at each committed cursor (kNoRow: done), same double buffering: a later sub-tile
  // knows which entries are idle without gathering A, and loads the rest of an entry's state
  // only when it is active
  int32_t* gnx0;
  int32_t* gnx1;
  int32_t* ghub;  // hub id of each chunked entry's A column (-1: none), written at its first visit
  int64_t* gbase;  // start of each chunked hub entry's A column, written at its first visit: the
                   // stop search reads it from here (coalesced) instead of the hub table's row
  // stored row bitmaps of the dense candidates (bmp_count_kernel): task t owns words
  // [boff[t], boff[t+1]) of bmp, bit x of word w = row tlo[t] + 32 w + x. The large symbolic kernel
  // writes them while it counts; the dense numeric kernel reads them instead of a marking pass.
  const int64_t* boff;
  uint32_t* bmp;
  // merge mode (MultiwayMerge of k partial lists): entry l of output column slot c is list l's
  // segment [mstart[c*nl+l], +mlen[c*nl+l]) of lir[l] / lnum[l]; no multiply
  const int64_t* mstart;
  const int64_t* mlen;
  int nl;
  const int32_t* lir[kMaxLists];
  const void* lnum[kMaxLists];
};

// first q in [lo, hi) with rows[q] >= key (rows sorted); global memory, 64-bit positions.
__device__ __forceinline__ int64_t lb_rows64(const int32_t* __restrict__ rows, int64_t lo, int64_t hi, int32_t key) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (rows[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// galloping lower bound from lo (rows[lo-1] < key is known): lo, lo+1, lo+3, lo+7, ...
__device__ __forceinline__ int64_t gallop64(const int32_t* __restrict__ rows, int64_t lo, int64_t hi, int32_t key) {
  int64_t step = 1, prev = lo;
  int64_t nx = lo;
  while (nx < hi) {
    if (rows[nx] >= key) return lb_rows64(rows, prev, nx, key);
    prev = nx + 1;
    nx = lo + step;
    step <<= 1;
  }
  return lb_rows64(rows, prev, hi, key);
}

// End of an active entry's segment inside the sub-tile: first q in [lo, hi) with rows[q] >= key.
// The W rows after lo are loaded at once (independent loads, mostly one cache line): at scale 22
// most segments of short A columns end there in one round trip. Past them, a hub column's
// row-block table (blk: first position of each RB-row block, relative to the column start
// `base`) bounds the stop to one block -- a few dozen rows of one or two cache lines -- instead
// of a galloping search of ~2 log2(segment) dependent loads; short columns gallop. Also returns
// the row at the stop (kNoRow past hi), the next sub-tile's cursor row. Sub-tiles and dense
// windows end on row-block boundaries where they can (kAlignSubtiles), and there a hub's stop is
// the table entry itself: one load instead of the preload, the table and a bisection. The column
// start (`base`) comes from the entry state, not from the hub table's row (round 5: one random
// 128-B line less per active hub visit, A^2 153.3 -> 155.5 GFLOP/s). Round 5 also tried the
// preload FIRST at aligned stops (CBH_STOP_TABLE_FIRST=0: its rows are the line the gather reads
// anyway, and half the dense kernel's active segments end inside it): 147.3 GFLOP/s, dense 275 ->
// 299 ms -- the extra dependent round trip of the long segments costs more than the table lines.
#ifndef CBH_STOP_TABLE_FIRST
#define CBH_STOP_TABLE_FIRST 1
#endif
#ifndef CBH_LAZY_CLEAR  // (A/B hook) see the sub-tile loop of task_kernel
#define CBH_LAZY_CLEAR 0
#endif
#ifndef CBH_STOP_PREFETCH  // (A/B hook) the next sub-tile's hub table pairs loaded during the current one
#define CBH_STOP_PREFETCH 0
#endif
// pf_key / pf: the table pair of block boundary pf_key when the caller prefetched it (the task
// kernel loads the NEXT sub-tile's pair of every hub entry during the current sub-tile, so the
// one-load stop costs no round trip when its sub-tile comes; CBH_STOP_PREFETCH)
template <int W>
__device__ __forceinline__ int64_t stop_search(const int32_t* __restrict__ rows, int64_t lo, int64_t hi, int32_t key,
                                               const int2* __restrict__ blk, int64_t base, int32_t RB,
                                               int32_t& row_at, int32_t pf_key = -1, int2 pf = int2{0, 0}) {
#if CBH_STOP_TABLE_FIRST
  if (blk != nullptr && key % RB == 0) {  // a row-block boundary (aligned sub-tiles): one table load
    const int2 e = key == pf_key ? pf : blk[key / RB];
    const int64_t s0 = base + e.x;
    const int64_t stop = s0 < lo ? lo : (s0 > hi ? hi : s0);
    row_at = stop >= hi ? kNoRow : (stop == s0 ? e.y : rows[stop]);
    return stop;
  }
#endif
  int32_t v[W];
#pragma unroll
  for (int w = 0; w < W; ++w) v[w] = (lo + w < hi) ? rows[lo + w] : kNoRow;
  int c = 0;
  int32_t at = kNoRow;
#pragma unroll
  for (int w = W - 1; w >= 0; --w) {
    c += v[w] < key ? 1 : 0;
    at = v[w] >= key ? v[w] : at;
  }
  if (c < W) {
    row_at = at;
    return lo + c;
  }
  lo += W;
  int64_t stop;
  if (blk != nullptr && key % RB == 0) {  // a row-block boundary (aligned sub-tiles): one table load
    const int2 e = key == pf_key ? pf : blk[key / RB];
    const int64_t s0 = base + e.x;
    stop = s0 < lo ? lo : (s0 > hi ? hi : s0);
    row_at = stop >= hi ? kNoRow : (stop == s0 ? e.y : rows[stop]);
    return stop;
  }
  if (blk != nullptr) {
    const int32_t b = key / RB;
    const int64_t s0 = base + blk[b].x, s1 = base + blk[b + 1].x;
    stop = lb_rows64(rows, s0 > lo ? s0 : lo, s1 < hi ? s1 : hi, key);
  } else {
    stop = gallop64(rows, lo, hi, key);
  }
  row_at = stop < hi ? rows[stop] : kNoRow;
  return stop;
}

// Slot update of a locked semiring (sr_locked): the key word doubles as the slot's lock (bit 31;
// rows are < 2^31 - 1). Claims an empty slot with the lock held and stores the first product,
// or, if the slot holds row r, takes the lock and folds v in with SR::add(v, old) (new value
// first, as the reference's hash branch, mtSpGEMM.h:408). Returns false if the slot belongs to
// another row. SIMT-safe: every loop iteration makes ONE acquire attempt per lane and a lane that
// acquires releases in the same iteration, so no lane ever waits on a lock held by a lane of its
// own wave that the divergent branch order has not run yet.
constexpr uint32_t kLockBit = 0x80000000u;
template <class SR>
__device__ __forceinline__ bool locked_insert(int32_t* key, typename SR::acc_t* val, int32_t r,
                                              const typename SR::val_t& v) {
  const int32_t locked = (int32_t)((uint32_t)r | kLockBit);
  bool done = false, mine = true;
  while (!done) {
    int32_t k = kEmpty;
    if (__hip_atomic_compare_exchange_strong(key, &k, locked, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP)) {
      *val = v;  // first product of the slot
      __hip_atomic_store(key, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      done = true;
    } else if ((int32_t)((uint32_t)k & ~kLockBit) != r) {
      mine = false;  // another row's slot: probe on
      done = true;
    } else {
      int32_t e = r;
      if (__hip_atomic_compare_exchange_strong(key, &e, locked, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP)) {
        *val = SR::add(v, *val);
        __hip_atomic_store(key, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        done = true;
      }
    }
  }
  return mine;
}

// Exclusive prefix sum of one int per thread over the block (thread order); total = block sum.
// Uses red[0..NW); all threads must call.
template <int BS>
__device__ __forceinline__ int block_excl_sum(int v, int* red, int& total) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int s = wave_incl_sum(v);
  __syncthreads();  // red may still be read by a previous user
  if (lane == 63) red[wid] = s;
  __syncthreads();
  int wpre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int r = red[w];
    wpre += (w < wid) ? r : 0;
    tot += r;
  }
  total = tot;
  return wpre + s - v;
}

// Numeric task plan shared by the binning (host launch) and the kernel: a task runs DENSE when a
// bitmap over each sub-tile's rows fits the NWB LDS words and the sub-tiles it then needs (at
// most 15/16 of CAPD outputs each) are not more than 5/4 of the hash sub-tiles (T/2 outputs;
// 4/4, 8/4 and 12/4 measured slower). Returns the dense sub-tile count, or 0 when the task stays
// on the hash.
__host__ __device__ inline int64_t dense_subtiles(int64_t work, int64_t span, int64_t T, int64_t capd, int64_t nwb,
                                                  int64_t dratio4 = kDRatio4) {
  if (work <= 0 || span <= 0) return 0;
  const int64_t cap = T / 2;
  const int64_t R = (work + cap - 1) / cap;
  const int64_t cd = capd * 15 / 16;
  int64_t Rd = (work + cd - 1) / cd;
  const int64_t Rw = (span + 32 * nwb - 1) / (32 * nwb);
  Rd = Rd > Rw ? Rd : Rw;
  return 4 * Rd <= dratio4 * R ? Rd : 0;
}

// Rank commit of one batch of the queue Q[0, qtot) of occupied slots of an order-preserving table
// (slot order), by one wave: a run of occupied slots is a run of queue entries with
// consecutive slots, so slot Q[q] goes to output out_pos + (start of its run in the queue) + (keys of
// its run smaller than its key). Run boundaries come from comparing each slot with its queue
// neighbours (shuffles), run extents from two ballots, ranks from shuffling the run's keys.
// A wave commits a contiguous queue range [b0, qend) whose ends are run starts (queue_run_start),
// in batches of up to 64 entries that also end where a run starts (`used` returns the entries a
// batch committed), so no run crosses a batch edge: the dependent LDS walks across the edges of
// fixed 64-entry batches -- the longest chains of the commit -- remain only for runs longer than a
// batch and for a wave edge with no run start within 64 entries (round 4: hash 292 -> 284 ms at
// scale 22; tests/test_commit_logic.py replays the algorithm against a sort on random queues).
// Returns guard bits (1 << 5: an output position outside the task).
template <class SR>
__device__ __forceinline__ int rank_commit_batch(const int32_t* keys, const typename SR::acc_t* vals,
                                                 const int16_t* Q, int qtot, int qend, int b0, int& used,
                                                 int64_t out_pos, int64_t out_end, int64_t ccap,
                                                 int32_t* __restrict__ Cir, typename SR::val_t* __restrict__ Cnum) {
  const int lane = threadIdx.x & 63;
  int bad = 0;
  const int q = b0 + lane;
  // entries are loaded up to the queue's end, so that runs (and their ends) are seen across the
  // wave's range end; this batch commits the ones before qend and before `limit`
  const bool loaded = q < qtot;
  const bool inq = q < qend;
  const int sq = loaded ? (int)Q[q] : -4;
  const int32_t key = loaded ? keys[sq] : kNoRow;
  const int sup = __shfl_up(sq, 1);
  const int sdn = __shfl_down(sq, 1);
  const int sprev = lane == 0 ? (b0 > 0 ? (int)Q[b0 - 1] : -10) : sup;
  const int snext = (q + 1 < qtot) ? (lane == 63 ? (int)Q[q + 1] : sdn) : -10;
  const uint64_t mstart = __ballot(loaded && sq != sprev + 1);
  const uint64_t mend = __ballot(loaded && snext != sq + 1);
  // a full batch inside the range whose last run goes on past it stops where that run starts
  int limit = 64;
  if (b0 + 64 <= qend && ((mend >> 63) & 1ull) == 0ull && mstart != 0ull) {
    const int last = 63 - __clzll(mstart);
    if (last > 0) limit = last;
  }
  used = qend - b0 < limit ? qend - b0 : limit;
  const bool valid = inq && lane < limit;
  const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  const uint64_t below = mstart & upto;
  const uint64_t above = mend & ~((1ull << lane) - 1ull);
  const int rs = below ? 63 - __clzll(below) : -1;  // run start lane (-1: before the batch)
  const int re = above ? __ffsll((long long)above) - 1 : 64;  // run end lane (64: after it)
  const int lo_l = rs < 0 ? 0 : rs, hi_l = re > 63 ? 63 : re;
  int rank = 0;
  for (int j = 0;; j += 4) {
    if (__ballot(valid && lo_l + j <= hi_l) == 0ull) break;
    const int32_t k0 = __shfl(key, (lo_l + j) & 63);
    const int32_t k1 = __shfl(key, (lo_l + j + 1) & 63);
    const int32_t k2 = __shfl(key, (lo_l + j + 2) & 63);
    const int32_t k3 = __shfl(key, (lo_l + j + 3) & 63);
    if (valid) {
      rank += (lo_l + j <= hi_l && k0 < key) ? 1 : 0;
      rank += (lo_l + j + 1 <= hi_l && k1 < key) ? 1 : 0;
      rank += (lo_l + j + 2 <= hi_l && k2 < key) ? 1 : 0;
      rank += (lo_l + j + 3 <= hi_l && k3 < key) ? 1 : 0;
    }
  }
  int rstart = b0 + lo_l;
  if (valid && rs < 0) {  // (only when no run start lay near a wave's nominal cut)
    int qq = b0 - 1;
    while (qq >= 0 && (int)Q[qq] == (int)Q[qq + 1] - 1) {
      rank += keys[Q[qq]] < key ? 1 : 0;
      --qq;
    }
    rstart = qq + 1;
  }
  if (valid && re > 63) {  // the run goes on past the batch (longer than 64 entries)
    int qq = b0 + 64;
    while (qq < qtot && (int)Q[qq] == (int)Q[qq - 1] + 1) {
      rank += keys[Q[qq]] < key ? 1 : 0;
      ++qq;
    }
  }
  if (valid) {
    const int64_t pos = out_pos + rstart + rank;
    if (pos >= out_end || pos >= ccap || pos < out_pos) {
      bad |= 1 << 5;
    } else {
      Cir[pos] = key;
      Cnum[pos] = SR::finalize(vals[sq]);
    }
  }
  return bad;
}
// the first run start at or after queue index nom (wave-uniform); nom itself when none lies within
// 64 entries (the batches then walk across that edge)
__device__ __forceinline__ int queue_run_start(const int16_t* Q, int qtot, int nom) {
  if (nom <= 0) return 0;
  if (nom >= qtot) return qtot;
  const int lane = threadIdx.x & 63;
  const int x = nom + lane;
  const bool st = x >= qtot || (int)Q[x] != (int)Q[x - 1] + 1;
  const uint64_t m = __ballot(st);
  return m ? nom + __ffsll((long long)m) - 1 : nom;
}

template <class SR, int T, int BS, int EMAX, int U, int MODE>
struct TaskCfg {
  static constexpr bool NUM = MODE != MODE_TSYM;
  static constexpr bool DENSE = MODE == MODE_TDENSE;
  using val_t = typename SR::val_t;
  using acc_t = typename SR::acc_t;
  using a_t = typename sr_a_type<SR>::type;  // A's values (NT1)
  using b_t = typename sr_b_type<SR>::type;  // B's values (NT2)
  // slots (symbolic: 32-bit words, a key hash over the first T or a bitmap over all TA). The large
  // symbolic configuration fills two workgroups' share of LDS with bitmap words: 12160 words =
  // 389 K rows per sub-tile instead of 262 K, so fewer sub-tiles re-scan a column's entries
  static constexpr int TA = NUM ? T + kGuard : (T >= 8192 && BS >= 512 ? kSymWords : T);
  static constexpr int NW = BS / 64;
  static constexpr int WIN = U * BS;
  // owner map entries are entry indices (< EMAX): 16 bits leave LDS room for larger windows
  using own_t = int16_t;
  static_assert(EMAX < 32768, "owner map entries are 16-bit");
  static constexpr size_t al(size_t x) { return (x + 15) & ~size_t(15); }
  static constexpr size_t o_keys = 0;
  static constexpr size_t o_vals = al(o_keys + sizeof(int32_t) * TA);
  static constexpr size_t o_pos = al(o_vals + (NUM ? sizeof(acc_t) * TA : 0));
  // dense numeric windows (MODE_TDENSE) share the two tables' LDS [0, o_pos) between values (from
  // the bottom; the output rows are not stored: the commit reads them off the bitmap) and the
  // window's bitmap words with their int16 prefix popcounts (6 B per word, from the top). The
  // plan (dense_subtiles, the stored-bitmap candidates) prices a task with the split at the
  // widest window: CAPD values and NWB words (3072 and 4224 = 135 K rows for T = 4096 with f64).
  static constexpr int CAPD = T / 4 * kCapD4;
  static constexpr size_t o_dvals = o_keys;
  static constexpr size_t o_dbits = al(o_dvals + sizeof(acc_t) * CAPD);
  static constexpr int NWB = NUM ? (int)((o_pos - o_dbits) / 6) / 8 * 8 : 0;
  static_assert(!DENSE || o_dbits + 6 * NWB <= o_pos, "dense bitmap and prefix fit the tables");
  // o_end: two int32 arrays, the entry's remaining length in the task (end - cursor) and the cursor's
  // offset in its A column (cursor - column start, so the stop search needs no hub-table load for
  // the start); columns have < 2^31 rows
  static constexpr size_t o_end = al(o_pos + sizeof(int64_t) * EMAX);
  static constexpr size_t o_scale = al(o_end + sizeof(int64_t) * EMAX);
  static constexpr size_t o_next = al(o_scale + (NUM ? sizeof(b_t) * EMAX : 0));
  static constexpr size_t o_next2 = al(o_next + sizeof(int32_t) * EMAX);
  static constexpr size_t o_col = al(o_next2 + sizeof(int32_t) * EMAX);
  static constexpr size_t o_off = al(o_col + sizeof(int32_t) * EMAX);
  static constexpr size_t o_own = al(o_off + sizeof(int32_t) * (EMAX + 1));
  static constexpr size_t o_red = al(o_own + sizeof(own_t) * WIN);
  static constexpr size_t bytes = al(o_red + sizeof(int32_t) * (2 * NW + 4));
};

// MERGE: the entries of a task are the k lists' segments of its output column (MultiwayMerge,
// MultiwayMerge.h:411-526); rows and values are addressed through list 0's arrays plus a
// per-list element offset (all device allocations share one address space, 256-byte aligned),
// so the sub-tile machinery above runs unchanged and the "product" is the list value itself.
// Waves per SIMD the launch bounds ask for: groups of >= 512 threads get as many waves as the LDS
// lets share a CU (160 KB: two 80 KB groups of 512 threads -> 4 waves per SIMD -> <= 128 VGPRs);
// smaller groups keep 4.
template <int BS, size_t BYTES>
constexpr int task_waves_per_eu() {
  if (BS < 512) return 4;
  const int groups = (int)(163840 / (BYTES > 0 ? BYTES : 1));
  const int w = (groups < 1 ? 1 : groups) * (BS / 64) / 4;
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}
template <class SR, int T, int BS, int EMAX, int U, int MODE, bool MERGE = false>
__global__ __launch_bounds__(BS, (task_waves_per_eu<BS, TaskCfg<SR, T, BS, EMAX, U, MODE>::bytes>())) void task_kernel(TaskArgs a) {
  using C = TaskCfg<SR, T, BS, EMAX, U, MODE>;
  using val_t = typename C::val_t;
  using acc_t = typename C::acc_t;
  using a_t = typename C::a_t;
  using b_t = typename C::b_t;
  constexpr bool NUM = C::NUM;
  constexpr bool LOCKED = sr_locked<SR>::value;
  static_assert(!(LOCKED && C::DENSE), "locked (user-semiring) accumulation runs on the hash kernels");
  constexpr int TA = C::TA, NW = C::NW, WIN = C::WIN;
  static_assert((T & (T - 1)) == 0, "table size must be a power of two");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int32_t* keys = reinterpret_cast<int32_t*>(smem + C::o_keys);
  uint32_t* words = reinterpret_cast<uint32_t*>(smem + C::o_keys);
  acc_t* vals = reinterpret_cast<acc_t*>(smem + (C::DENSE ? C::o_dvals : C::o_vals));
  // epos: cursor (absolute index into A); between the segment scan and the end of the sub-tile
  // it holds cursor - exclusive offset (the gather base of the entry's products)
  int64_t* epos = reinterpret_cast<int64_t*>(smem + C::o_pos);
  int32_t* erem = reinterpret_cast<int32_t*>(smem + C::o_end);    // end of the A column in the task - cursor
  int32_t* ecoff = erem + EMAX;                                    // cursor - start of the A column
  b_t* escale = reinterpret_cast<b_t*>(smem + C::o_scale);        // B value
  int32_t* enext = reinterpret_cast<int32_t*>(smem + C::o_next);  // row at the cursor (kNoRow: done)
  int32_t* enext2 = reinterpret_cast<int32_t*>(smem + C::o_next2);  // row at the sub-tile's stop
  int32_t* ecol = reinterpret_cast<int32_t*>(smem + C::o_col);    // hub id of the A column (-1: none)
  int32_t* eoff = reinterpret_cast<int32_t*>(smem + C::o_off);
  typename C::own_t* own = reinterpret_cast<typename C::own_t*>(smem + C::o_own);
  int32_t* red = reinterpret_cast<int32_t*>(smem + C::o_red);
  __shared__ int32_t s_ovf;  // overflow flag of the current sub-tile (LDS; read after barriers)
  __shared__ int64_t s_vdelta[kMaxLists];  // merge: list l's value index - row index (elements)
  static_assert(!MERGE || EMAX >= kMaxLists, "merge entries fit one chunk");

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int32_t* __restrict__ rowsA = MERGE ? a.lir[0] : a.Air;
  const val_t* __restrict__ valsA = reinterpret_cast<const val_t*>(MERGE ? a.lnum[0] : a.Anum);
#ifdef CBH_STAMPS
  uint64_t st_[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t t_prev_ = __builtin_amdgcn_s_memtime();
  unsigned long long dg_active = 0, dg_short = 0, dg_shortp = 0;
#endif
  if ((int64_t)blockIdx.x >= a.norder) return;
  const int32_t task = a.order[blockIdx.x];
  if (task < 0 || task >= a.ntasks) {
    if (tid == 0) guard_fail(a.err, 9, task);
    return;
  }
  const int32_t c = a.tcol[task];
  const int64_t e0 = MERGE ? 0 : a.Bcp[c];
  const int64_t ne = MERGE ? a.nl : a.Bcp[c + 1] - e0;
  const int64_t work = a.twork[task];
  const int32_t tlo = a.tlo[task], thi = a.thi[task];
  const uint8_t full = a.tfull[task];
  if (work <= 0 || thi <= tlo) {
    if (!NUM && tid == 0) a.cnt[task] = 0;
    return;
  }
  const int64_t span = (int64_t)thi - tlo;
  const bool chunked = ne > EMAX;
  const int nchunks = chunked ? (int)((ne + EMAX - 1) / EMAX) : 1;
  // sub-tile plan of the hash and symbolic kernels (uniform in rows). Tasks whose output rows are
  // dense enough run the DENSE kernel instead (windows of the stored row bitmap, below): their
  // bitmap's prefix popcounts give every row its output rank directly, so values accumulate in
  // row order and the commit is a straight copy (no hashing, no probing, no rank search).
  bool bitmap = false;
  constexpr bool dense = C::DENSE;
  // symbolic: a dense candidate's bitmap is stored for the dense numeric kernel (word-aligned
  // sub-tiles, always the bitmap form)
  const bool store = !NUM && a.bmp != nullptr && a.boff[task + 1] > a.boff[task];
  int64_t R = 1;
  if constexpr (!dense) {
    constexpr int64_t cap = NUM ? (int64_t)T * CBH_FILL16 / 16 : (int64_t)TA * kSymFill8 / 8;  // outputs (keys) per sub-tile
    R = (work + cap - 1) / cap;
    if constexpr (!NUM) {
      const int64_t Rb = (span + 32ll * TA - 1) / (32ll * TA);
      if (Rb <= R || store) {
        bitmap = true;
        R = Rb;
      }
    }
    if (R > span) R = span;
    if (R < 1) R = 1;
  }
  int64_t wnom = (span + R - 1) / R;
  if (store) wnom = (wnom + 31) & ~int64_t(31);  // <= 32*TA: R >= span / (32*TA)
  // sub-tiles of a task cut in several end on row-block boundaries (hub stops are one table load)
  // once they span a few blocks: the task's blocks are dealt into R runs of wblk whole blocks (R
  // unchanged, except a bitmap sub-tile's row limit), so a sub-tile holds up to one block more than
  // the nominal width. Stored bitmaps keep their word alignment (tlo and RB are multiples of 32).
  const bool align = kAlignSubtiles && !dense && R >= 2 && a.RB > 0 && wnom >= 4ll * a.RB &&
                     (!store || ((a.RB & 31) == 0 && (tlo & 31) == 0));
  int64_t wblk = 0;  // blocks per aligned sub-tile
  if (align) {
    const int64_t nbt = ((int64_t)thi + a.RB - 1) / a.RB - tlo / a.RB;
    int64_t Ra = R;
    if (bitmap) {
      const int64_t bmax = 32ll * TA / a.RB;  // >= 4: wnom <= 32*TA
      Ra = (nbt + bmax - 1) / bmax;
    }
    wblk = (nbt + Ra - 1) / Ra;
    wnom = wblk * a.RB;
  }

  // violated bounds guards are recorded in a register and reported once at the end: a guard_fail
  // (global atomics with return values) inside a hot loop makes the compiler drain vmcnt there
  int bad = 0;  // bit k: guard site k violated
  // hub h's block pairs (TaskArgs::htab); entries keep h in ecol and their column start as the
  // cursor's column offset (ecoff), so a sub-tile's stop search loads only the pair it needs
  auto hub_tab = [&](int32_t h) -> const int2* {
    return reinterpret_cast<const int2*>(a.htab) + (int64_t)h * (a.nblk + 2) + 1;
  };
  // entry state of entries [first, first+cnt): cursor at the first row >= lo
  const int64_t go = chunked ? a.goff[task] : 0;
  int par = 0;  // which HBM cursor buffer holds the committed cursors
  auto load_entries = [&](int64_t first, int cnt, int32_t lo, int32_t hi, bool lo_is_start, bool from_state) {
    if constexpr (MERGE) {  // entry i = list i; positions are list 0-relative row indices
      for (int i = tid; i < cnt; i += BS) {
        const int64_t rdelta = (int64_t)(a.lir[i] - a.lir[0]);
        s_vdelta[i] = (int64_t)(reinterpret_cast<const val_t*>(a.lnum[i]) - valsA) - rdelta;
        ecol[i] = -1;
        const int64_t base = a.mstart[(int64_t)c * a.nl + i] + rdelta;
        const int64_t end = base + a.mlen[(int64_t)c * a.nl + i];
        int64_t cend = end;
        if (!(full & 2) && base < end) cend = lb_rows64(rowsA, base, end, thi);
        int64_t pos = base;
        if (!lo_is_start && base < cend) pos = lb_rows64(rowsA, base, cend, lo);
        epos[i] = pos;
        erem[i] = (int32_t)(cend - pos);
        ecoff[i] = 0;
        enext[i] = pos < cend ? rowsA[pos] : kNoRow;
      }
      return;
    }
    for (int i = tid; i < cnt; i += BS) {
      const int64_t p = e0 + first + i;
      if (from_state) {  // later sub-tile of a chunked task: committed cursor and its row from HBM
        // (the column was validated at the entry's first visit: an invalid one is idle for good)
        const int64_t g = go + first + i;
        const int32_t nx = (par ? a.gnx1 : a.gnx0)[g];
        const int32_t h = a.ghub[g];
        const int64_t cur = (par ? a.gcur1 : a.gcur0)[g];
        epos[i] = cur;
        enext[i] = nx;
        ecol[i] = h;
        if (nx >= hi) continue;  // idle in this sub-tile: segments() reads only the cursor and its row
        erem[i] = (int32_t)(a.gend[g] - cur);
        ecoff[i] = h >= 0 ? (int32_t)(cur - a.gbase[g]) : 0;
        if constexpr (NUM) escale[i] = reinterpret_cast<const b_t*>(a.Bnum)[p];
        continue;
      }
      const int32_t k = a.Bir[p];
      if constexpr (NUM) escale[i] = reinterpret_cast<const b_t*>(a.Bnum)[p];
      if (k < 0 || k >= a.ncolA) {
        bad |= 1 << 1;
        ecol[i] = -1;
        epos[i] = 0;
        erem[i] = ecoff[i] = 0;
        enext[i] = kNoRow;
        if (chunked) {
          a.gend[go + first + i] = 0;
          (par ? a.gcur1 : a.gcur0)[go + first + i] = 0;
          (par ? a.gnx1 : a.gnx0)[go + first + i] = kNoRow;
          a.ghub[go + first + i] = -1;
        }
        continue;
      }
      int64_t base = a.Acp[k], end = a.Acp[k + 1];
      if (base < 0 || end < base || end > a.nnzA) {
        bad |= 1 << 2;
        base = end = 0;
      }
      // the entry is clamped to the task's rows: its end is the first row >= thi. Interior task
      // boundaries sit on row-block boundaries, so a hub column finds both ends in its block
      // table (one load each); short columns bisect.
      const int32_t h = (base < end && a.RB > 0) ? a.hidx[k] : -1;
      ecol[i] = h;
      const int2* blk = h >= 0 ? hub_tab(h) : nullptr;
      int64_t cend = end;
      if (!(full & 2) && base < end) {
        if (blk && thi % a.RB == 0) cend = base + blk[thi / a.RB].x;
        else cend = lb_rows64(rowsA, base, end, thi);
      }
      int64_t pos = base;
      int32_t known = kUnknownRow;  // the row at the cursor, when the block table gave it
      if (!lo_is_start && base < cend) {
        if (blk && lo % a.RB == 0) {
          const int2 e = blk[lo / a.RB];
          pos = base + e.x;
          known = e.y;
        } else {
          pos = lb_rows64(rowsA, base, cend, lo);
        }
        if (pos > cend) pos = cend;
      }
      epos[i] = pos;
      erem[i] = (int32_t)(cend - pos);
      ecoff[i] = (int32_t)(pos - base);
      const int32_t nx = pos < cend ? known : kNoRow;
      enext[i] = nx;
      if (chunked) {  // the first sub-tile's cursors are committed state too
        a.gend[go + first + i] = cend;
        a.gbase[go + first + i] = base;
        (par ? a.gcur1 : a.gcur0)[go + first + i] = pos;
        (par ? a.gnx1 : a.gnx0)[go + first + i] = nx;
        a.ghub[go + first + i] = h;
      }
    }
  };
  // segment of every entry inside [lo, hi) (idle entries -- next row >= hi -- cost one LDS read),
  // then the exclusive scan of the segment lengths; epos becomes the gather base (cursor - offset).
  // Returns the sub-tile's product count P.
  // hi_next: the next sub-tile's end when it is a row-block boundary inside the task (-1: none).
  // Entries kept in LDS (one per thread: unchunked tasks) then load the hub table pair of that
  // boundary now, into registers, so the next sub-tile's stop search finds it there.
  int32_t pf_key = -1;
  int2 pf_e = int2{0, 0};
  auto segments = [&](int nec, int32_t hi, bool hi_is_end, int32_t hi_next) -> int {
#ifdef CBH_STAMPS
    if (tid == 0) atomicAdd(&g_stamps[16], (unsigned long long)nec);
#endif
    for (int i = tid; i < nec; i += BS) {
      const int32_t nx = enext[i];
      const int64_t p = epos[i];
      int64_t stop = p;
      int32_t nx2 = nx;
      const int32_t h = MERGE ? -1 : ecol[i];
      if (nx < hi) {
#ifdef CBH_STAMPS
        dg_active++;
#endif
        const int64_t end = p + erem[i];
        if (hi_is_end) {
          stop = end;
          nx2 = kNoRow;
        } else {
          const int2* blk = h >= 0 ? hub_tab(h) : nullptr;
          stop = stop_search<8>(rowsA, nx == kUnknownRow ? p : p + 1, end, hi, blk, p - ecoff[i], a.RB, nx2, pf_key,
                                pf_e);
        }
      }
#if CBH_STOP_PREFETCH
      if (!MERGE && !chunked && hi_next > 0 && h >= 0 && nx2 < hi_next) {  // still has rows before hi_next
        pf_e = hub_tab(h)[hi_next / a.RB];
        pf_key = hi_next;
      }
#endif
      eoff[i] = (int32_t)(stop - p);
      enext2[i] = nx2;
#ifdef CBH_STAMPS
      if (nx < hi && stop - p < 8) {
        dg_short++;
        dg_shortp += (unsigned long long)(stop - p);
      }
#endif
    }
    __syncthreads();
    CBH_STAMP(2);
    block_scan_excl<BS>(eoff, nec, red);
    for (int i = tid; i < nec; i += BS) epos[i] -= eoff[i];
    return eoff[nec];
  };
  // the U products of the current window this thread holds
  int32_t r[U];
  val_t av[U];  // numeric: A value * B value (the product), once values are gathered
  // One sweep over the windows of the current entry set: owner map, gather U products per
  // thread (all loads in flight), then `upd(u)` for every product this thread holds.
  // upd(u) updates the table with product u of the current batch; a non-null `batch(wn)` replaces
  // the per-product calls (the numeric hash's batched first probes, CBH_HASH_BATCH)
  auto sweep = [&](int nec, int P, bool with_vals, auto&& upd, auto&& batch) {
    int carry = -1;  // owner of the product just before the window
    for (int w0 = 0; w0 < P; w0 += WIN) {
      const int wn = (P - w0) < WIN ? (P - w0) : WIN;
      for (int x = tid; x < WIN; x += BS) own[x] = (typename C::own_t)((x == 0) ? carry : -1);
      __syncthreads();
      for (int i = tid; i < nec; i += BS) {
        const int s0 = eoff[i];
        if (s0 >= w0 && s0 < w0 + wn && eoff[i + 1] > s0) own[s0 - w0] = (typename C::own_t)i;
      }
      __syncthreads();
      block_max_scan<BS, WIN>(own, red);
      carry = own[wn - 1];
      CBH_STAMP(4);
      if (__hip_atomic_load(&s_ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
      // branch-free gather: lanes past the window re-read product 0 and are masked afterwards
#if CBH_GATHER_PIN
      a_t ar[U];  // numeric: A's value of each product; the multiply waits until all U are loaded
      int oi[U];
#endif
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int x0 = tid + u * BS;
        const int x = x0 < wn ? x0 : 0;
        const int i = own[x];
        const int64_t q = epos[i] + w0 + x;
        r[u] = rowsA[q];
        if constexpr (NUM && MERGE) {
          if (with_vals) av[u] = valsA[q + s_vdelta[i]];
        } else if constexpr (NUM) {
#if CBH_GATHER_PIN
          if (with_vals) {
            ar[u] = reinterpret_cast<const a_t*>(a.Anum)[q];
            oi[u] = i;
          }
#else
          if (with_vals) av[u] = SR::multiply(reinterpret_cast<const a_t*>(a.Anum)[q], escale[i]);
#endif
        }
      }
#if CBH_GATHER_PIN
      // every gathered row and value is materialised here, after all U gathers were issued, and
      // the multiplies follow: otherwise the compiler sinks product 0's value load into upd's
      // bounds-checked branch behind a vmcnt(0) for its row (two dependent HBM round trips per
      // window), or, with a multiply right after each load, waits out each load in turn
#pragma unroll
      for (int u = 0; u < U; ++u) {
        asm volatile("" ::"v"(r[u]));
        if constexpr (NUM && MERGE && std::is_arithmetic<val_t>::value && (sizeof(val_t) == 4 || sizeof(val_t) == 8))
          if (with_vals) asm volatile("" ::"v"(av[u]));
        if constexpr (NUM && !MERGE && std::is_arithmetic<a_t>::value && (sizeof(a_t) == 4 || sizeof(a_t) == 8))
          if (with_vals) asm volatile("" ::"v"(ar[u]));
      }
      if constexpr (NUM && !MERGE) {
        if (with_vals) {
#pragma unroll
          for (int u = 0; u < U; ++u) av[u] = SR::multiply(ar[u], escale[oi[u]]);
        }
      }
#endif
      if constexpr (std::is_same<std::decay_t<decltype(batch)>, std::nullptr_t>::value) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (tid + u * BS < wn) upd(u);
      } else {
        batch(wn);
      }
      __syncthreads();
      CBH_STAMP(5);
    }
  };
  auto set_ovf = [&]() { __hip_atomic_store(&s_ovf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };

  if (!chunked) {
    load_entries(0, (int)ne, tlo, thi, (full & 1) != 0, false);
  }
  __syncthreads();
  CBH_STAMP(0);

  int64_t out_pos = 0, out_end = 0;
  if constexpr (NUM) {
    out_pos = a.toff[task] - a.cbase;
    out_end = a.toff[task + 1] - a.cbase;
  }
  int my_count = 0;  // symbolic hash: keys this thread inserted first

  int32_t lo = tlo;
  if constexpr (dense) {
    // DENSE numeric sub-tiles are windows of the task's row bitmap, stored by the symbolic pass
    // (TaskArgs::bmp): the word prefix popcounts give every row its output rank before any product
    // is gathered, so one value pass accumulates the products at their ranks, nothing overflows,
    // windows without outputs are skipped, and the commit walks the bitmap (no row ids stored).
    // The two hash tables' LDS (TB bytes) holds the values from the bottom and the window's words
    // and prefixes (6 B per word) from the top: a window loads as many words as the task's output
    // density says fill the values, and is cut where its outputs would overrun them -- dense
    // columns get wide windows (5760 values at 18 % density), sparse ones long bitmaps.
    const int64_t bw0 = a.boff[task];
    const int64_t nwt = a.boff[task + 1] - bw0;
    if (a.bmp == nullptr || nwt != (span + 31) / 32) {
      if (tid == 0) guard_fail(a.err, 10, c, task, nwt, span);
      return;
    }
    const uint32_t* __restrict__ tb = a.bmp + bw0;
    __shared__ int32_t s_cut;
    constexpr int64_t TB = (int64_t)C::o_pos;
    int64_t wdes = TB * nwt / ((int64_t)sizeof(acc_t) * work + 6 * nwt);  // words whose outputs fill the rest
    wdes = wdes < 64 ? 64 : (wdes > C::NWB ? C::NWB : wdes);
    // window ends snap to row-block boundaries when that keeps >= 3/4 of the window
    const bool dalign = kAlignSubtiles && a.RB > 0 && (a.RB & 31) == 0 && (tlo & 31) == 0;
    const int64_t dbw = dalign ? a.RB / 32 : 1;  // words per row block
    bool inited = !chunked;  // chunked: HBM entry state is written by the first processed window
    constexpr int KW = (C::NWB + BS - 1) / BS;  // window words per thread
    uint32_t pre[KW];
    int64_t pre_w0 = -1;
    int64_t w0 = 0;
    while (w0 < nwt) {
      const int wl = (int)((nwt - w0) < wdes ? (nwt - w0) : wdes);
      const int dbase = (int)((TB - 6 * wl) & ~int64_t(15));
      uint32_t* dw = reinterpret_cast<uint32_t*>(smem + dbase);
      int16_t* dp = reinterpret_cast<int16_t*>(smem + dbase + 4 * wl);
      const int capv = dbase / (int)sizeof(acc_t);
      const int kw = (wl + BS - 1) / BS;
      if (pre_w0 == w0) {  // words gathered while the previous window was cut (same thread mapping)
#pragma unroll
        for (int j = 0; j < KW; ++j)
          if (tid + j * BS < wl) dw[tid + j * BS] = pre[j];
      } else {
        for (int x = tid; x < wl; x += BS) dw[x] = tb[w0 + x];
      }
      if (tid == 0) {
        s_cut = wl;
        __hip_atomic_store(&s_ovf, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // sweep() reads it
      }
      __syncthreads();
      // exclusive popcount prefix per word (thread-consecutive words), clamped to int16 past the
      // cut, and the word where the prefix passes the value capacity
      int tsum = 0;
      for (int k = 0; k < kw; ++k) {
        const int x = tid * kw + k;
        tsum += x < wl ? __popc(dw[x]) : 0;
      }
      int wtotal = 0;
      int ex = block_excl_sum<BS>(tsum, red, wtotal);
      for (int k = 0; k < kw; ++k) {
        const int x = tid * kw + k;
        if (x < wl) {
          const int pc = __popc(dw[x]);
          dp[x] = (int16_t)(ex < 32767 ? ex : 32767);
          if (ex <= capv && ex + pc > capv) s_cut = x;
          ex += pc;
        }
      }
      __syncthreads();
      CBH_STAMP(1);
      int cut = s_cut;
      if (dalign && tlo + 32 * (w0 + cut) < thi) {  // snap the window end down to a row-block boundary
        // (an absolute one: a column's first task starts at its first row's word, not on a block;
        // relative snapping missed stop_search's one-load hub path: dense 300 -> 280 ms)
        const int64_t tw0 = tlo / 32;
        const int64_t cb = (tw0 + w0 + cut) / dbw * dbw - tw0 - w0;
        if (cb > 0 && cb * 4 >= 3ll * cut) cut = (int)cb;
      }
      const int dtotal = cut < wl ? (int)dp[cut] : wtotal;
      {  // the next window's words: their loads overlap this window's entry loads
        const int64_t w0n = w0 + cut;
        if (w0n < nwt) {
          const int wln = (int)((nwt - w0n) < wdes ? (nwt - w0n) : wdes);
#pragma unroll
          for (int j = 0; j < KW; ++j) pre[j] = (tid + j * BS < wln) ? tb[w0n + tid + j * BS] : 0u;
          pre_w0 = w0n;
        }
      }
      lo = (int32_t)(tlo + 32 * w0);
      const int64_t hcut = tlo + 32 * (w0 + cut);
      const int32_t hi = (int32_t)(hcut < thi ? hcut : thi);
      const uint32_t tw = (uint32_t)(hi - lo);
      if (dtotal > 0) {
        // the window's accumulators (LDS below dbase; an earlier window's words may have been there)
        for (int x = tid; x < dtotal; x += BS) vals[x] = SR::identity();
        auto place = [&](int u) {
          const uint32_t d = (uint32_t)(r[u] - lo);
          if (d >= tw) {
            bad |= 1 << 8;
            return;
          }
          const uint32_t wv = dw[d >> 5];
          if (!((wv >> (d & 31)) & 1u)) bad |= 1 << 11;  // a product row the symbolic pass did not mark
          const int slot = dp[d >> 5] + __popc(wv & ((1u << (d & 31)) - 1u));
          SR::lds_acc(&vals[slot], av[u]);
        };
        for (int ch = 0; ch < nchunks; ++ch) {
          int nec = (int)ne;
          if (chunked) {
            const int64_t first = (int64_t)ch * EMAX;
            nec = (int)((ne - first) < EMAX ? (ne - first) : EMAX);
            load_entries(first, nec, lo, hi, lo == tlo && (full & 1), inited);
            __syncthreads();
          }
          const int P = segments(nec, hi, hi == thi, -1);
          CBH_STAMP(3);
          if (chunked) {  // this chunk's cursors after the window, into the other buffer
            int64_t* gn = par ? a.gcur0 : a.gcur1;
            int32_t* gx = par ? a.gnx0 : a.gnx1;
            for (int i = tid; i < nec; i += BS) {
              gn[go + (int64_t)ch * EMAX + i] = epos[i] + eoff[i + 1];
              gx[go + (int64_t)ch * EMAX + i] = enext2[i];
            }
            // no store wait: the thread that wrote an entry's cursor is the one that reloads it
          }
          sweep(nec, P, true, place, nullptr);  // ends with a barrier: the entry state may be reloaded
        }
        // commit: values are in row order (rank q = output out_pos + q: coalesced); the rows are
        // read off the bitmap, word x's set bits being ranks dp[x]..
        if (out_pos + dtotal > out_end || out_pos + dtotal > a.ccap) {
          bad |= 1 << 5;
        } else {
          for (int q = tid; q < dtotal; q += BS)
            reinterpret_cast<val_t*>(a.Cnum)[out_pos + q] = SR::finalize(vals[q]);
          for (int x = tid; x < cut; x += BS) {
            uint32_t wv = dw[x];
            int32_t* cr = a.Cir + out_pos + dp[x];
            while (wv) {
              *cr++ = lo + 32 * x + __builtin_ctz(wv);
              wv &= wv - 1u;
            }
          }
        }
        out_pos += dtotal;
        if (chunked) {
          par ^= 1;
          inited = true;
        } else {
          for (int i = tid; i < (int)ne; i += BS) {
            const int sg = eoff[i + 1] - eoff[i];
            epos[i] += eoff[i + 1];
            erem[i] -= sg;
            ecoff[i] += sg;
            enext[i] = enext2[i];
          }
        }
      }
      w0 += cut;
      __syncthreads();
      CBH_STAMP(6);
    }
  }
  int64_t w = wnom;
  // CBH_LAZY_CLEAR (A/B hook): a committed hash sub-tile resets only its occupied slots (listed in
  // the commit queue) instead of the next sub-tile clearing all T + 64 slots
  constexpr bool LAZY = CBH_LAZY_CLEAR && NUM && !LOCKED && !MERGE;
  bool table_clean = false;
  int lazy_q = 0;
  while (!dense && lo < thi) {
    int64_t he = (int64_t)lo + w;
    if (align) {
      if (w == wnom) {
        he = ((int64_t)lo / a.RB + wblk) * a.RB;
      } else {  // a retried (halved) sub-tile: its end snaps down to a block boundary
        const int64_t hb = he / a.RB * a.RB;
        if (hb > lo) he = hb;
      }
    }
    const int32_t hi = (int32_t)(he < thi ? he : thi);
    const bool hi_is_end = hi == thi;  // entry ends are clamped to the task (load_entries)
    // the next nominal sub-tile's end, when it is an interior row-block boundary (stop prefetch)
    int32_t hi_next = -1;
    if (align && !hi_is_end) {
      const int64_t hn = ((int64_t)hi / a.RB + wblk) * a.RB;
      if (hn < thi) hi_next = (int32_t)hn;
    }
    const uint32_t tw = (uint32_t)(hi - lo);
    const uint64_t scale = ((uint64_t)T << 32) / (uint64_t)tw;  // numeric order-preserving slot map
    const int nwd = (int)((tw + 31) >> 5);
    if (!NUM && bitmap) {
      for (int s = tid; s < nwd; s += BS) words[s] = 0u;
    } else if (!(LAZY && table_clean)) {
      for (int s = tid; s < TA; s += BS) {
        keys[s] = kEmpty;
        if constexpr (NUM && !LOCKED) vals[s] = SR::identity();
      }
    }
    if constexpr (LAZY) table_clean = false;  // (a retried sub-tile leaves the table dirty)
    if (tid == 0) __hip_atomic_store(&s_ovf, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const int count_before = my_count;
    __syncthreads();
    CBH_STAMP(1);

    for (int ch = 0; ch < nchunks; ++ch) {
      int nec = (int)ne;
      if (chunked) {
        const int64_t first = (int64_t)ch * EMAX;
        nec = (int)((ne - first) < EMAX ? (ne - first) : EMAX);
        load_entries(first, nec, lo, hi, lo == tlo && (full & 1), lo != tlo);
        __syncthreads();
      }
      const int P = segments(nec, hi, hi_is_end, hi_next);
#ifdef CBH_STAMPS
      if (tid == 0) {
        atomicAdd(&g_stamps[13], 1ull);
        atomicAdd(&g_stamps[15], (unsigned long long)P);
      }
#endif
      CBH_STAMP(3);
      if (!NUM && bitmap) {
        sweep(
            nec, P, false,
            [&](int u) {
              const uint32_t d = (uint32_t)(r[u] - lo);
              if (d >= tw) bad |= 1 << 8;
              else atomicOr(&words[d >> 5], 1u << (d & 31));
            },
            nullptr);
      } else if constexpr (NUM && !LOCKED && CBH_HASH_BATCH) {
        // every product's first probe issued before any result is used (U CAS in flight per
        // thread instead of U dependent probe chains); the products whose home slot holds another
        // row probe on afterwards, one by one
        sweep(nec, P, true, [&](int) {}, [&](int wn) {
          uint32_t hs[U];
          int32_t hk[U];
          bool need[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            need[u] = false;
            hs[u] = 0;
            if (tid + u * BS < wn) {
              const uint32_t d = (uint32_t)(r[u] - lo);
              if (d >= tw) bad |= 1 << 8;
              else {
                hs[u] = (uint32_t)(((uint64_t)d * scale) >> 32);
                need[u] = true;
              }
            }
          }
#pragma unroll
          for (int u = 0; u < U; ++u) hk[u] = need[u] ? atomicCAS(&keys[hs[u]], kEmpty, r[u]) : kEmpty;
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (need[u] && (hk[u] == kEmpty || hk[u] == r[u])) {
              SR::lds_acc(&vals[hs[u]], av[u]);
              need[u] = false;
            }
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (need[u]) {
              bool ok = false;
              uint32_t sl = hs[u] + 1;
              for (int probe = 1; probe < kPmax && sl < (uint32_t)TA; ++probe, ++sl) {
                const int32_t k = atomicCAS(&keys[sl], kEmpty, r[u]);
                if (k == kEmpty || k == r[u]) {
                  SR::lds_acc(&vals[sl], av[u]);
                  ok = true;
                  break;
                }
              }
              if (!ok) set_ovf();
            }
        });
      } else if constexpr (NUM) {
        sweep(nec, P, true, [&](int u) {
          const val_t vv = av[u];
          uint32_t d = (uint32_t)(r[u] - lo);
#if CBH_GUARD_BRANCHLESS
          // a row outside the sub-tile (never, unless the plan is inconsistent) is flagged and
          // clamped into it instead of branching around the insert: the flag fails the call
          bad |= d >= tw ? 1 << 8 : 0;
          d = d < tw ? d : 0u;
#else
          if (d >= tw) {
            bad |= 1 << 8;
            return;
          }
#endif
          uint32_t s = (uint32_t)(((uint64_t)d * scale) >> 32);
          bool ok = false;
          if constexpr (LOCKED) {
            for (int probe = 0; probe < kPmax && s < (uint32_t)TA; ++probe, ++s)
              if (locked_insert<SR>(&keys[s], &vals[s], r[u], vv)) {
                ok = true;
                break;
              }
          } else {
            // (s < T + kPmax - 1 <= TA for every probe: no end-of-table test -- round 6, hash 237.4
            // -> 229.2 ms per scale-22 product, the kernel being issue-bound; CBH_PROBE_BOUND=1
            // restores it for A/B)
            static_assert(kGuard >= kPmax, "forward probes stay inside the guard slots");
            for (int probe = 0; probe < kPmax && (!CBH_PROBE_BOUND || s < (uint32_t)TA); ++probe, ++s) {
              const int32_t k = atomicCAS(&keys[s], kEmpty, r[u]);
              if (k == kEmpty || k == r[u]) {
                SR::lds_acc(&vals[s], vv);
                ok = true;
                break;
              }
            }
          }
          if (!ok) set_ovf();
        }, nullptr);
      } else {
        sweep(nec, P, false, [&](int u) {
          const uint32_t d = (uint32_t)(r[u] - lo);
          if (d >= tw) {
            bad |= 1 << 8;
            return;
          }
          // key hash over all TA words (12160 for the large configuration: the bitmap's LDS), slot
          // = multiplicative hash scaled to TA
          uint32_t s = (uint32_t)(((uint64_t)((uint32_t)r[u] * 0x9E3779B1u) * (uint64_t)TA) >> 32);
          bool ok = false;
          for (int probe = 0; probe < 2 * kPmax; ++probe, s = (s + 1 == (uint32_t)TA) ? 0u : s + 1) {
            const int32_t k = atomicCAS(&keys[s], kEmpty, r[u]);
            if (k == kEmpty) ++my_count;
            if (k == kEmpty || k == r[u]) {
              ok = true;
              break;
            }
          }
          if (!ok) set_ovf();
        }, nullptr);
      }
      if (__hip_atomic_load(&s_ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
        for (int i = tid; i < nec; i += BS) epos[i] += eoff[i];  // back to the cursors
        break;
      }
      if (chunked) {  // this chunk's cursors (and their rows) after the sub-tile, into the other buffer
        int64_t* gn = par ? a.gcur0 : a.gcur1;
        int32_t* gx = par ? a.gnx0 : a.gnx1;
        for (int i = tid; i < nec; i += BS) {
          gn[go + (int64_t)ch * EMAX + i] = epos[i] + eoff[i + 1];
          gx[go + (int64_t)ch * EMAX + i] = enext2[i];
        }
        // (no store wait: the thread that wrote an entry's cursor is the one that reloads it)
        __syncthreads();  // entry state is reloaded by the next chunk
      }
    }
    // hash numeric: occupied slots per wave (slot ranges of SPW) -> every wave's queue offset and
    // the total; a sub-tile whose occupied slots exceed the commit queue is retried like an overflow
    constexpr int SPW = ((TA + NW - 1) / NW + 63) / 64 * 64;
    constexpr int NBW = SPW / 64;  // occupancy ballots per wave
    int qbase = 0, qtot = 0;
    // occupancy masks of this wave's slot range, kept for the queue compaction of the commit
    uint64_t occm[NUM ? NBW : 1];
    if constexpr (NUM) {
      const int sb = wid * SPW < TA ? wid * SPW : TA;
      const int se = sb + SPW < TA ? sb + SPW : TA;
      int wc = 0;
#pragma unroll
      for (int b = 0; b < NBW; ++b) {
        const int sl = sb + 64 * b + lane;
        occm[b] = __ballot(sl < se && keys[sl] != kEmpty);
        wc += __popcll(occm[b]);
      }
      if (lane == 0) red[NW + wid] = wc;
      __syncthreads();
#pragma unroll
      for (int x = 0; x < NW; ++x) {
        const int rr = red[NW + x];
        qbase += (x < wid) ? rr : 0;
        qtot += rr;
      }
    }
    const bool ovf_now = __hip_atomic_load(&s_ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (qtot > WIN || ovf_now) {  // table could not hold the sub-tile: halve the row range, redo
      // restore the cursors segments() moved, unless the insertion overflow already did. A hash
      // sub-tile that inserted fine but occupies more slots than the commit queue holds lands
      // here unrestored.
      if (!chunked && !ovf_now)
        for (int i = tid; i < (int)ne; i += BS) epos[i] += eoff[i];
      __syncthreads();
      my_count = count_before;
      if (tid == 0) atomicAdd(&a.err[16], 1);  // retry counter (cbh_ctx_take_retries)
      if (tw == 1) {
        if (tid == 0) atomicOr(&a.err[1], 1);
        return;
      }
      w = (tw + 1) / 2;
#ifdef CBH_STAMPS
      if (tid == 0) atomicAdd(&g_stamps[14], 1ull);
#endif
      continue;
    }
    CBH_STAMP(8);
    par ^= chunked ? 1 : 0;  // the cursors written during this sub-tile are now the committed ones
    if (!chunked)  // advance the cursors past the committed sub-tile
      for (int i = tid; i < (int)ne; i += BS) {
        const int sg = eoff[i + 1] - eoff[i];
        epos[i] += eoff[i + 1];
        erem[i] -= sg;
        ecoff[i] += sg;
        enext[i] = enext2[i];
      }
    CBH_STAMP(9);
    if (!NUM && bitmap) {
      uint32_t* sb = store ? a.bmp + a.boff[task] + ((lo - tlo) >> 5) : nullptr;
      for (int s = tid; s < nwd; s += BS) {
        const uint32_t wv = words[s];
        my_count += __popc(wv);
        if (store) sb[s] = wv;
      }
    } else if constexpr (NUM) {
      // rank commit. The occupied slots are compacted in slot order into a queue Q (the owner
      // map's LDS, dead here): queue index q = occupied slots before Q[q]. A run of occupied
      // slots is a run of consecutive queue entries with consecutive slots, so slot Q[q] goes
      // to (start of its run in the queue) + (keys of its run smaller than its key). Each wave
      // takes a queue range cut at run starts, in batches of <= 64 entries that end at run starts
      // (rank_commit_batch: boundaries by shuffles, extents by ballots, ranks by shuffling the
      // run's keys; runs are short at fill 1/2).
      int16_t* Q = reinterpret_cast<int16_t*>(own);
      {
        const int sb = wid * SPW < TA ? wid * SPW : TA;
        const uint64_t lt = (1ull << lane) - 1ull;
        int qo = qbase;
#pragma unroll
        for (int b = 0; b < NBW; ++b) {
          const uint64_t mask = occm[b];
          if ((mask >> lane) & 1ull) Q[qo + __popcll(mask & lt)] = (int16_t)(sb + 64 * b + lane);
          qo += __popcll(mask);
        }
      }
      __syncthreads();
      {  // wave w commits the queue range between the run starts nearest w and w + 1 NW-ths of it
        const int per = (qtot + NW - 1) / NW;
        const int qs = queue_run_start(Q, qtot, wid * per);
        const int qe = wid == NW - 1 ? qtot : queue_run_start(Q, qtot, (wid + 1) * per);
        for (int b0 = qs; b0 < qe;) {
          int used = 0;
          bad |= rank_commit_batch<SR>(keys, vals, Q, qtot, qe, b0, used, out_pos, out_end, a.ccap, a.Cir,
                                       reinterpret_cast<val_t*>(a.Cnum));
          b0 += used;
        }
      }
      out_pos += qtot;
      if constexpr (LAZY) lazy_q = qtot;
#ifdef CBH_STAMPS
      if (tid == 0) atomicAdd(&g_stamps[20], (unsigned long long)qtot);
#endif
    }
    lo = hi;
    w = wnom;
    __syncthreads();
    if constexpr (LAZY) {  // (after the commit's barrier: every read of the table is done)
      const int16_t* Q = reinterpret_cast<const int16_t*>(own);
      for (int q = tid; q < lazy_q; q += BS) {
        const int sl = Q[q];
        keys[sl] = kEmpty;
        vals[sl] = SR::identity();
      }
      table_clean = true;  // (the next sub-tile's first barrier orders these before its inserts)
    }
    CBH_STAMP(6);
  }
  if constexpr (!NUM) {
    const int total = block_sum_int<NW>(my_count, red);
    if (tid == 0) a.cnt[task] = total;
  } else {
    if (tid == 0 && out_pos != out_end) atomicAdd(&a.err[0], 1);
  }
  if (bad) guard_fail(a.err, 31 - __clz(bad), c, bad, lo);
#ifdef CBH_STAMPS
  CBH_STAMP(7);
  if (tid == 0) {
    for (int k = 0; k < 12; ++k) atomicAdd(&g_stamps[k], (unsigned long long)st_[k]);
    atomicAdd(&g_stamps[12], 1ull);
  }
  if (dg_active) atomicAdd(&g_stamps[17], dg_active);
  if (dg_short) atomicAdd(&g_stamps[18], dg_short);
  if (dg_shortp) atomicAdd(&g_stamps[19], dg_shortp);
#endif
}

}  // namespace cbh
