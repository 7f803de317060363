// dense_kernel.h -- the DENSE numeric kernel (bitmap-rank windows) of the hash-SpGEMM's dense
// tasks [LocalHybridSpGEMM, mtSpGEMM.h:289-441, for output columns whose rows are dense enough],
// round 5 layout: ONE workgroup of BS threads per CU with the whole LDS, and wave-independent
// product processing inside a window.
//
// What a dense task computes is unchanged from task_kernel<MODE_TDENSE> (task_kernel.h): the task's
// output rows are the set bits of its row bitmap, stored by the symbolic pass; a WINDOW is a run of
// bitmap words whose popcount prefix gives every row its output rank, so products accumulate at
// their ranks (SR::lds_acc) and the commit writes values coalesced and rows off the bitmap.
//
// Why a new kernel: the round-4 dense kernel was bound by fetched bytes (383 GB per scale-22 phase
// for 158 GB algorithmic, 87 % of the achievable fabric rate), and half of those bytes were paid per
// ACTIVE ENTRY VISIT -- every window revisits every B entry whose A segment has products in it,
// fetching the partial row / value lines at both ends of the segment and a hub-table line. The
// visits per product fall with the window's width, and the window is bounded by LDS. So:
//  * one 1024-thread workgroup per CU owns all 160 KB of LDS: about twice the rows per window of
//    two 80 KB workgroups (the same 16 waves per CU);
//  * that alone measured flat in round 3 because every phase of a window was block-synchronous
//    (one latency chain per workgroup): here only the window's setup, the segment scan and the
//    commit are block-wide; the products of a window are cut into one contiguous range per wave
//    and every wave walks its range on its own (owner entry by a per-wave start map and a DPP
//    max-scan, no owner-map barriers), so the waves' gathers overlap each other's latency.
//
// Per window, per chunk of <= EL entries (LDS-resident state when the task has <= EL entries,
// HBM cursor state otherwise):
//   phase 1 (thread per entry): segment [cursor, stop) inside the window (stop_search), the entry
//           advanced; block scan of (length, active flag) -> the ACTIVE entries compacted to
//           (start offset, gather base, B value) -- every compacted entry has >= 1 product, so at
//           most 64 of them start inside any 64-product batch;
//   phase 2 (wave-independent): wave w takes products [w*P/NW, (w+1)*P/NW); per step of up to
//           64*U products the 64 entries after the current one write their start slot into the
//           wave's byte map (one LDS load, one store each), a DPP max-scan per 64-product batch
//           gives every lane its entry, and all U batches gather before any update (the multiply
//           by B's value waits for the accumulate: a multiply right after its load made the
//           compiler drain vmcnt per batch).
#pragma once
#include "wave_kernel.h"  // task_kernel.h, wave_lds_sync

namespace cbh {

// bitmap words per int16 window prefix: 2 (round 6) -- a 64-bit word per rank lookup, 5 instead
// of 6 bytes of LDS per word, so a window spans ~10 % more rows at the dense tasks' density (dense
// 262.5 -> 254.5 ms per scale-22 product); 1 and 4 for A/B
#ifndef CBH_DENSE_PAIRS
#define CBH_DENSE_PAIRS 2
#endif
// registers per thread that prefetch the next window's first words (the rest load at its start)
#ifndef CBH_DENSE2_PREFETCH
#define CBH_DENSE2_PREFETCH 8
#endif

// kernel kinds of dense_kernel: numeric dense windows, symbolic bitmap sub-tiles, numeric hash
// sub-tiles (the order-preserving LDS hash of task_kernel.h with a table of ~7 K slots)
enum : int { KDENSE = 0, KSYMB = 1, KHASH = 2 };

template <class SR, int BS, int EL, int U, int LDSB, int KIND = KDENSE>
struct DenseCfg {
  using acc_t = typename SR::acc_t;
  using b_t = typename sr_b_type<SR>::type;
  static constexpr bool NUM = KIND != KSYMB;
  static constexpr bool ROLL = KIND == KHASH;  // sub-tiles may overflow and be retried: cursors commit after
  static constexpr int NW = BS / 64;
  static constexpr size_t al(size_t x) { return (x + 15) & ~size_t(15); }
  // entry state (LDS-resident tasks): cursor, row at the cursor, end - cursor, cursor - column
  // start, hub id, B value (numeric only)
  static constexpr size_t o_cur = 0;
  static constexpr size_t o_nx = al(o_cur + sizeof(int64_t) * EL);
  static constexpr size_t o_rem = al(o_nx + sizeof(int32_t) * EL);
  static constexpr size_t o_coff = al(o_rem + sizeof(int32_t) * EL);
  static constexpr size_t o_hub = al(o_coff + sizeof(int32_t) * EL);
  static constexpr size_t o_scale = al(o_hub + sizeof(int32_t) * EL);
  // hash: the cursors after the current sub-tile, committed only when it did not overflow
  static constexpr size_t o_pcur = al(o_scale + (NUM ? sizeof(b_t) * EL : 0));
  static constexpr size_t o_pnx = al(o_pcur + (ROLL ? sizeof(int64_t) * EL : 0));
  // compacted active entries of the current chunk: start offset (+ the total at [nact]), gather
  // base (cursor - start offset), B value (numeric only)
  static constexpr size_t o_cstart = al(o_pnx + (ROLL ? sizeof(int32_t) * EL : 0));
  static constexpr size_t o_cbase = al(o_cstart + sizeof(int32_t) * (EL + 1));
  static constexpr size_t o_cscale = al(o_cbase + sizeof(int64_t) * EL);
  static constexpr size_t o_own = al(o_cscale + (NUM ? sizeof(b_t) * EL : 0));  // NW x 512-byte owner maps
  static constexpr size_t o_red = al(o_own + 512 * NW);
  static constexpr size_t o_win = al(o_red + sizeof(int32_t) * (4 * NW + 8));
  // numeric: the window -- values from the bottom, the window's words and int16 prefixes (6 B per
  // word) from the top (as task_kernel's dense windows); symbolic: the sub-tile's row bitmap
  static constexpr size_t TB = (LDSB - o_win) & ~size_t(15);
  static constexpr size_t bytes = o_win + TB;
  static constexpr int NWB = (int)((TB - 64) / 6) / 8 * 8;  // widest window (all words, no values)
  static constexpr int NWS = (int)(TB / 4) / 64 * 64;      // symbolic bitmap words (32 rows each)
  // hash: TH home slots + kGuard (forward probing never wraps), keys then values; the commit queue
  // (int16 slot ids) reuses the compacted arrays
  static constexpr int TH0 = ((int)((TB - 32) / (sizeof(int32_t) + sizeof(acc_t))) - kGuard) / 64 * 64;
  static constexpr int THQ = ((int)((o_own - o_cstart) / 2) - kGuard) / 64 * 64;  // the queue's bound
  static constexpr int TH1 = TH0 < THQ ? TH0 : THQ;
#ifdef CBH_HASH2_TH_MAX  // (A/B hook: the task kernel's 2048-slot table on this kernel)
  static constexpr int TH = TH1 < CBH_HASH2_TH_MAX ? TH1 : CBH_HASH2_TH_MAX;
#else
  static constexpr int TH = TH1;
#endif
  static constexpr int TA = TH + kGuard;
  static constexpr size_t o_hvals = al(sizeof(int32_t) * TA);  // (relative to o_win)
  static_assert(KIND != KHASH || (o_hvals + sizeof(acc_t) * TA <= TB && 2 * TA <= o_own - o_cstart && TA < 32768),
                "hash table and commit queue fit");
  static_assert(NWB <= 32767, "int16 window prefixes");
  static_assert(bytes <= 163840, "one workgroup's LDS");
  static_assert(EL <= BS && EL % 64 == 0, "at most one entry per thread per chunk");
  static_assert(U >= 1 && U <= 8, "a lane's owner counts are the 8 bytes of one word");
};

// exclusive block scan of two ints per thread (thread order); totals in ta / tb. Uses red[0, 2*NW).
template <int BS>
__device__ __forceinline__ void block_excl_sum2(int& a, int& b, int* red, int& ta, int& tb) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int sa = wave_incl_sum(a), sb = wave_incl_sum(b);
  __syncthreads();  // red may still be read by a previous user
  if (lane == 63) {
    red[wid] = sa;
    red[NW + wid] = sb;
  }
  __syncthreads();
  int pa = 0, pb = 0, xa = 0, xb = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int ra = red[w], rb = red[NW + w];
    pa += (w < wid) ? ra : 0;
    pb += (w < wid) ? rb : 0;
    xa += ra;
    xb += rb;
  }
  a = pa + sa - a;
  b = pb + sb - b;
  ta = xa;
  tb = xb;
}

// KDENSE: the numeric dense tasks (windows of the stored bitmap, values by rank);
// KSYMB: the symbolic pass's bitmap tasks (sub-tiles of NWS words, rows marked with atomicOr,
// distinct rows counted and, for a dense candidate, its bitmap stored) -- estimateNNZ_Hash
// (mtSpGEMM.h:806-933) for the tasks whose row bitmap is cheaper than a key hash;
// KHASH: the numeric hash tasks (LocalHybridSpGEMM's hash branch, mtSpGEMM.h:362-437): sub-tiles of
// up to TH/2 outputs in task_kernel's order-preserving LDS hash (slot (row-lo)*TH/(hi-lo), forward
// probing, rank commit without a sort); a sub-tile that overflows its probes is
// retried with half the rows, so its entries' cursors commit only after it succeeded.
template <class SR, int BS, int EL, int U, int LDSB, int KIND = KDENSE>
__global__ __launch_bounds__(BS, BS >= 1024 ? 4 : 6) void dense_kernel(TaskArgs a) {  // 16 (24) waves per CU
  constexpr bool SYM = KIND == KSYMB;
  using C = DenseCfg<SR, BS, EL, U, LDSB, KIND>;
  using val_t = typename SR::val_t;
  using acc_t = typename SR::acc_t;
  using a_t = typename sr_a_type<SR>::type;
  using b_t = typename C::b_t;
  constexpr int NW = C::NW;
  constexpr bool NUM = C::NUM;
  constexpr bool ROLL = C::ROLL;
  static_assert(!sr_locked<SR>::value, "the dense kernel accumulates with SR::lds_acc");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int64_t* scur = reinterpret_cast<int64_t*>(smem + C::o_cur);
  int32_t* snx = reinterpret_cast<int32_t*>(smem + C::o_nx);
  int32_t* srem = reinterpret_cast<int32_t*>(smem + C::o_rem);
  int32_t* scoff = reinterpret_cast<int32_t*>(smem + C::o_coff);
  int32_t* shub = reinterpret_cast<int32_t*>(smem + C::o_hub);
  b_t* sscale = reinterpret_cast<b_t*>(smem + C::o_scale);
  int64_t* pcur = reinterpret_cast<int64_t*>(smem + C::o_pcur);
  int32_t* pnx = reinterpret_cast<int32_t*>(smem + C::o_pnx);
  int32_t* cstart = reinterpret_cast<int32_t*>(smem + C::o_cstart);
  int64_t* cbase = reinterpret_cast<int64_t*>(smem + C::o_cbase);
  b_t* cscale = reinterpret_cast<b_t*>(smem + C::o_cscale);
  int32_t* red = reinterpret_cast<int32_t*>(smem + C::o_red);
  unsigned char* win = smem + C::o_win;
  acc_t* vals = reinterpret_cast<acc_t*>(win);
  __shared__ int32_t s_cut;
  __shared__ int32_t s_ovf;  // hash: the current sub-tile overflowed (read after barriers)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint8_t* ownb = smem + C::o_own + 512 * wid;
  const int32_t* __restrict__ rowsA = a.Air;
  const a_t* __restrict__ valsA = reinterpret_cast<const a_t*>(a.Anum);
  if ((int64_t)blockIdx.x >= a.norder) return;
  const int32_t task = a.order[blockIdx.x];
  if (task < 0 || task >= a.ntasks) {
    if (tid == 0) guard_fail(a.err, 9, task);
    return;
  }
  const int32_t c = a.tcol[task];
  const int64_t e0 = a.Bcp[c];
  const int64_t ne = a.Bcp[c + 1] - e0;
  const int64_t work = a.twork[task];
  const int32_t tlo = a.tlo[task], thi = a.thi[task];
  const uint8_t full = a.tfull[task];
  if (work <= 0 || thi <= tlo) {
    if (!NUM && tid == 0) a.cnt[task] = 0;
    return;
  }
  const int64_t span = (int64_t)thi - tlo;
  const bool chunked = ne > EL;
  const int nchunks = (int)((ne + EL - 1) / EL);
  const int64_t go = chunked ? a.goff[task] : 0;
  int bad = 0;
  auto hub_tab = [&](int32_t h) -> const int2* {
    return reinterpret_cast<const int2*>(a.htab) + (int64_t)h * (a.nblk + 2) + 1;
  };

  // An entry's state at its first visit: the cursor at the first row >= lo of its A column clamped
  // to the task's rows (the block table of a hub column gives both ends at row-block boundaries)
  struct Ent {
    int64_t cur;
    int32_t nx, rem, coff, hub;
    b_t scale;
  };
  auto first_visit = [&](int64_t i, int32_t lo, bool lo_is_start) -> Ent {
    Ent e;
    const int64_t p = e0 + i;
    const int32_t k = a.Bir[p];
    if constexpr (NUM) e.scale = reinterpret_cast<const b_t*>(a.Bnum)[p];
    e.cur = 0;
    e.nx = kNoRow;
    e.rem = e.coff = 0;
    e.hub = -1;
    if (k < 0 || k >= a.ncolA) {
      bad |= 1 << 1;
      return e;
    }
    int64_t base = a.Acp[k], end = a.Acp[k + 1];
    if (base < 0 || end < base || end > a.nnzA) {
      bad |= 1 << 2;
      return e;
    }
    const int32_t h = (base < end && a.RB > 0) ? a.hidx[k] : -1;
    const int2* blk = h >= 0 ? hub_tab(h) : nullptr;
    int64_t cend = end;
    if (!(full & 2) && base < end) {
      if (blk && thi % a.RB == 0) cend = base + blk[thi / a.RB].x;
      else cend = lb_rows64(rowsA, base, end, thi);
    }
    int64_t pos = base;
    int32_t known = kUnknownRow;
    if (!lo_is_start && base < cend) {
      if (blk && lo % a.RB == 0) {
        const int2 t = blk[lo / a.RB];
        pos = base + t.x;
        known = t.y;
      } else {
        pos = lb_rows64(rowsA, base, cend, lo);
      }
      if (pos > cend) pos = cend;
    }
    e.cur = pos;
    e.nx = pos < cend ? known : kNoRow;
    e.rem = (int32_t)(cend - pos);
    e.coff = (int32_t)(pos - base);
    e.hub = h;
    if (chunked) {
      a.gend[go + i] = cend;
      a.gbase[go + i] = base;
      a.ghub[go + i] = h;
    }
    return e;
  };
  if (!chunked) {
    if (tid < ne) {
      const Ent e = first_visit(tid, tlo, (full & 1) != 0);
      scur[tid] = e.cur;
      snx[tid] = e.nx;
      srem[tid] = e.rem;
      scoff[tid] = e.coff;
      shub[tid] = e.hub;
      if constexpr (NUM) sscale[tid] = e.scale;
    }
  }
  bool inited = !chunked;  // chunked: the HBM entry state is written by the first processed range
  int par = 0;  // hash, chunked: which HBM cursor buffer holds the committed cursors (gcur0 / gcur1)

  // Every product of the row range [lo, hi) (all chunks of the task's entries): phase 1 moves each
  // entry's cursor past the range and compacts the active entries, phase 2 (wave-independent)
  // gathers the products and calls place(row, A value, compacted entry) for each.
  auto run_chunks = [&](int32_t lo, int32_t hi, auto&& place) {
    const bool hi_is_end = hi == thi;
    for (int ch = 0; ch < nchunks; ++ch) {
      // ---- phase 1: this chunk's entries (thread per entry)
      const int64_t i = (int64_t)ch * EL + tid;
      int len = 0;
      int64_t cur0 = 0;
      b_t scale{};
      if (tid < EL && i < ne) {
        Ent e;
        if (!chunked) {
          e.cur = scur[tid];
          e.nx = snx[tid];
        } else if (!inited) {
          e = first_visit(i, lo, lo == tlo && (full & 1));
        } else {
          e.cur = (par ? a.gcur1 : a.gcur0)[go + i];
          e.nx = (par ? a.gnx1 : a.gnx0)[go + i];
        }
        cur0 = e.cur;
        int64_t ncur = e.cur;  // the cursor past the range, and its row
        int32_t nnx = e.nx;
        if (e.nx < hi) {
          if (!chunked) {
            e.rem = srem[tid];
            e.coff = scoff[tid];
            e.hub = shub[tid];
            if constexpr (NUM) e.scale = sscale[tid];
          } else if (inited) {
            e.hub = a.ghub[go + i];
            e.rem = (int32_t)(a.gend[go + i] - e.cur);
            e.coff = e.hub >= 0 ? (int32_t)(e.cur - a.gbase[go + i]) : 0;
            if constexpr (NUM) e.scale = reinterpret_cast<const b_t*>(a.Bnum)[e0 + i];
          }
          int64_t stop;
          int32_t nx2;
          if (hi_is_end) {
            stop = e.cur + e.rem;
            nx2 = kNoRow;
          } else {
            const int2* blk = e.hub >= 0 ? hub_tab(e.hub) : nullptr;
            stop = stop_search<8>(rowsA, e.nx == kUnknownRow ? e.cur : e.cur + 1, e.cur + e.rem, hi, blk,
                                  e.cur - e.coff, a.RB, nx2);
          }
          len = (int)(stop - e.cur);
          if constexpr (NUM) scale = e.scale;
          ncur = stop;
          nnx = nx2;
          if (!ROLL && !chunked) {
            scur[tid] = stop;
            snx[tid] = nx2;
            srem[tid] = e.rem - len;
            scoff[tid] = e.coff + len;
          }
        }
        if constexpr (ROLL) {  // pending until the sub-tile commits (hash_commit_cursors)
          if (!chunked) {
            pcur[tid] = ncur;
            pnx[tid] = nnx;
          } else {
            (par ? a.gcur0 : a.gcur1)[go + i] = ncur;
            (par ? a.gnx0 : a.gnx1)[go + i] = nnx;
          }
        } else if (chunked && (ncur != e.cur || !inited)) {  // (an idle entry's state is unchanged)
          a.gcur0[go + i] = ncur;
          a.gnx0[go + i] = nnx;
        }
      }
      int off = len, aidx = len > 0 ? 1 : 0;
      int P = 0, nact = 0;
      block_excl_sum2<BS>(off, aidx, red, P, nact);
      P = __builtin_amdgcn_readfirstlane(P);
      nact = __builtin_amdgcn_readfirstlane(nact);
      if (len > 0) {
        cstart[aidx] = off;
        cbase[aidx] = cur0 - off;
        if constexpr (NUM) cscale[aidx] = scale;
      }
      if (tid == 0) cstart[nact] = P;
      __syncthreads();
      // ---- phase 2: wave w walks products [w*P/NW, (w+1)*P/NW) on its own
      const int pb = (int)((int64_t)P * wid / NW), pe = (int)((int64_t)P * (wid + 1) / NW);
      if (pb < pe) {
        // the compacted entry owning product pb: the last one starting at or before it
        int elo = 0;
        {
          int l0 = 0, h0 = nact;  // cstart[0] = 0 <= pb < P = cstart[nact]
          while (h0 - l0 > 1) {
            const int m = (l0 + h0) >> 1;
            if (cstart[m] <= pb) l0 = m;
            else h0 = m;
          }
          elo = __builtin_amdgcn_readfirstlane(l0);
        }
        // per step, up to 64*U products [x0, x0 + len): the 64 compacted entries after elo are
        // loaded once (lane j: entry elo+1+j, start s_j relative to x0; starts are distinct since
        // every compacted entry has a product) and scatter j+1 into the wave's byte map at their
        // start, laid out [lane][u] so that lane l reads the U positions u*64+l as ONE 8-byte
        // word; per batch u a DPP max-scan plus the carry from batch u-1 then counts the entries
        // starting at or before the lane's product. The step ends where the 64th entry starts
        // (entries past it are not loaded), at least 63 products on.
        for (int x0 = pb; x0 < pe;) {
          if (ROLL && __hip_atomic_load(&s_ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
          const int ae = elo + 1 + lane;
          const int s = ae <= nact ? cstart[ae] - x0 : (1 << 30);  // >= 1
          const int s63 = __builtin_amdgcn_readlane(s, 63);
          int len = pe - x0 < 64 * U ? pe - x0 : 64 * U;
          if (s63 < len) len = s63;
          *reinterpret_cast<uint64_t*>(ownb + 8 * lane) = 0ull;
          wave_lds_sync();
          if (s < len) ownb[8 * (s & 63) + (s >> 6)] = (uint8_t)(lane + 1);
          wave_lds_sync();
          const uint64_t ow = *reinterpret_cast<const uint64_t*>(ownb + 8 * lane);
          wave_lds_sync();  // ownb is rewritten by the next step
          int32_t r[U];
          a_t va[U];
          int ev[U];
          int carry = 0;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            r[u] = kNoRow;
            if (u * 64 >= len) continue;  // wave-uniform
            const int cnt0 = wave_incl_max((int)((ow >> (8 * u)) & 0xffu), 0);
            const int cnt = cnt0 > carry ? cnt0 : carry;
            carry = __builtin_amdgcn_readlane(cnt, 63);
            const int x = u * 64 + lane;
            if (x < len) {
              const int e = elo + cnt;
              ev[u] = e;
              const int64_t q = cbase[e] + x0 + x;
              r[u] = rowsA[q];
              if constexpr (NUM) va[u] = valsA[q];
            }
          }
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (r[u] != kNoRow) place(r[u], va[u], ev[u]);
          elo += __popcll(__ballot(s <= len));
          x0 += len;
        }
      }
      __syncthreads();  // the compacted arrays are rewritten by the next chunk
    }
  };

  if constexpr (KIND == KHASH) {
    // ---------------- numeric hash: sub-tiles of up to TH/2 planned outputs (task_kernel's plan)
    int32_t* keys = reinterpret_cast<int32_t*>(win);
    acc_t* hv = reinterpret_cast<acc_t*>(win + C::o_hvals);
    int16_t* Q = reinterpret_cast<int16_t*>(smem + C::o_cstart);  // commit queue (after the products)
    constexpr int TH = C::TH, TA = C::TA;
    int64_t out_pos = a.toff[task] - a.cbase;
    const int64_t out_end = a.toff[task + 1] - a.cbase;
    constexpr int64_t cap = (int64_t)TH * kFill8 / 8;  // outputs per sub-tile
    int64_t R = (work + cap - 1) / cap;
    if (R > span) R = span;
    if (R < 1) R = 1;
    int64_t wnom = (span + R - 1) / R;
    const bool align = kAlignSubtiles && R >= 2 && a.RB > 0 && wnom >= 4ll * a.RB;
    int64_t wblk = 0;
    if (align) {
      const int64_t nbt = ((int64_t)thi + a.RB - 1) / a.RB - tlo / a.RB;
      wblk = (nbt + R - 1) / R;
      wnom = wblk * a.RB;
    }
    constexpr int SPW = ((TA + NW - 1) / NW + 63) / 64 * 64;  // slots per wave in the commit
    constexpr int NBW = SPW / 64;
    int32_t lo = tlo;
    int64_t w = wnom;
    while (lo < thi) {
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
      const uint32_t tw = (uint32_t)(hi - lo);
      const uint64_t scl = ((uint64_t)TH << 32) / (uint64_t)tw;  // order-preserving slot map
      for (int x = tid; x < TA; x += BS) {
        keys[x] = kEmpty;
        hv[x] = SR::identity();
      }
      if (tid == 0) s_ovf = 0;
      // (phase 1's block scan orders the clearing before any insertion)
      run_chunks(lo, hi, [&](int32_t r, const a_t& av, int e) {
        const uint32_t d = (uint32_t)(r - lo);
        if (d >= tw) {
          bad |= 1 << 8;
          return;
        }
        uint32_t sl = (uint32_t)(((uint64_t)d * scl) >> 32);
        bool ok = false;
        for (int probe = 0; probe < kPmax && sl < (uint32_t)TA; ++probe, ++sl) {
          const int32_t k = atomicCAS(&keys[sl], kEmpty, r);
          if (k == kEmpty || k == r) {
            SR::lds_acc(&hv[sl], SR::multiply(av, cscale[e]));
            ok = true;
            break;
          }
        }
        if (!ok) __hip_atomic_store(&s_ovf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      });
      if (__builtin_amdgcn_readfirstlane(s_ovf)) {  // retry with half the rows (pending cursors dropped)
        if (tid == 0) atomicAdd(&a.err[16], 1);   // retry counter (cbh_ctx_take_retries)
        if (tw == 1) {
          if (tid == 0) atomicOr(&a.err[1], 1);
          return;
        }
        w = (tw + 1) / 2;
        __syncthreads();
        continue;
      }
      // the sub-tile is final: its entries' cursors commit
      if (!chunked) {
        if (tid < ne) {
          const int sg = (int)(pcur[tid] - scur[tid]);
          scur[tid] = pcur[tid];
          snx[tid] = pnx[tid];
          srem[tid] -= sg;
          scoff[tid] += sg;
        }
      } else {
        par ^= 1;
      }
      inited = true;
      // rank commit (task_kernel.h): occupied slots per wave -> the queue in slot
      // order -> every wave commits a queue range cut at run starts
      int qbase = 0, qtot = 0;
      uint64_t occm[NBW];
      {
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
      {
        const int per = (qtot + NW - 1) / NW;
        const int qs = queue_run_start(Q, qtot, wid * per);
        const int qe = wid == NW - 1 ? qtot : queue_run_start(Q, qtot, (wid + 1) * per);
        for (int b0 = qs; b0 < qe;) {
          int used = 0;
          bad |= rank_commit_batch<SR>(keys, hv, Q, qtot, qe, b0, used, out_pos, out_end, a.ccap, a.Cir,
                                       reinterpret_cast<val_t*>(a.Cnum));
          b0 += used;
        }
      }
      out_pos += qtot;
      lo = hi;
      w = wnom;
      __syncthreads();  // the table and the queue are reused by the next sub-tile
    }
    if (tid == 0 && out_pos != out_end) atomicAdd(&a.err[0], 1);
    if (bad) guard_fail(a.err, 31 - __clz(bad), c, bad, tlo);
  } else if constexpr (SYM) {
    // ---------------- symbolic: sub-tiles of up to NWS bitmap words; with a row-block table they
    // are dealt whole row blocks (hub stops are one table load), as task_kernel's sub-tiles
    const bool store = a.bmp != nullptr && a.boff[task + 1] > a.boff[task];
    uint32_t* words = reinterpret_cast<uint32_t*>(win);
    constexpr int64_t SW = 32ll * C::NWS;  // rows per sub-tile at most
    const int64_t R = (span + SW - 1) / SW;
    const bool align = a.RB > 0 && (a.RB & 31) == 0 && (tlo & 31) == 0 && R >= 2;
    int64_t wblk = 0, wrow = ((span + R - 1) / R + 31) & ~int64_t(31);
    if (align) {
      const int64_t nbt = ((int64_t)thi + a.RB - 1) / a.RB - tlo / a.RB;
      const int64_t bmax = SW / a.RB;
      const int64_t Ra = (nbt + bmax - 1) / bmax;
      wblk = (nbt + Ra - 1) / Ra;
    }
    if (store && a.boff[task + 1] - a.boff[task] != (span + 31) / 32) {
      if (tid == 0) guard_fail(a.err, 10, c, task, a.boff[task + 1] - a.boff[task], span);
      return;
    }
    int my_count = 0;
    int32_t lo = tlo;
    while (lo < thi) {
      int64_t he = align ? ((int64_t)lo / a.RB + wblk) * a.RB : (int64_t)lo + wrow;
      const int32_t hi = (int32_t)(he < thi ? he : thi);
      const uint32_t tw = (uint32_t)(hi - lo);
      const int nwd = (int)((tw + 31) >> 5);
      for (int x = tid; x < nwd; x += BS) words[x] = 0u;
      // (phase 1's block scan orders the clearing before any product is marked)
      run_chunks(lo, hi, [&](int32_t r, const a_t&, int) {
        const uint32_t d = (uint32_t)(r - lo);
        if (d >= tw) bad |= 1 << 8;
        else atomicOr(&words[d >> 5], 1u << (d & 31));
      });
      inited = true;
      uint32_t* sb = store ? a.bmp + a.boff[task] + ((lo - tlo) >> 5) : nullptr;
      for (int x = tid; x < nwd; x += BS) {
        const uint32_t wv = words[x];
        my_count += __popc(wv);
        if (store) sb[x] = wv;
      }
      __syncthreads();  // the words are cleared for the next sub-tile
      lo = hi;
    }
    const int total = block_sum_int<NW>(my_count, red);
    if (tid == 0) a.cnt[task] = total;
    if (bad) guard_fail(a.err, 31 - __clz(bad), c, bad, tlo);
    return;
  } else {
    // ---------------- numeric dense: windows of the stored row bitmap
    int64_t out_pos = a.toff[task] - a.cbase;
    const int64_t out_end = a.toff[task + 1] - a.cbase;
    const int64_t bw0 = a.boff[task];
    const int64_t nwt = a.boff[task + 1] - bw0;
    if (a.bmp == nullptr || nwt != (span + 31) / 32) {
      if (tid == 0) guard_fail(a.err, 10, c, task, nwt, span);
      return;
    }
    const uint32_t* __restrict__ tb = a.bmp + bw0;
    constexpr int64_t TB = (int64_t)C::TB;
    // G bitmap words per int16 prefix (CBH_DENSE_PAIRS: 2, a 64-bit word per rank lookup): 4 + 2 / G
    // bytes of LDS per word, so a window spans more rows for the same values
    constexpr int G = CBH_DENSE_PAIRS;
    static_assert(G == 1 || G == 2 || G == 4, "bitmap words per prefix");
    constexpr int64_t kWB2 = 4 * G + 2;  // bytes per G words (words + prefix)
    constexpr int NWBG = (int)((TB - 64) * G / kWB2) / 8 * 8;
    int64_t wdes = TB * nwt * G / ((int64_t)sizeof(acc_t) * work * G + kWB2 * nwt);  // words whose outputs fill the rest
    wdes = wdes < 64 ? 64 : (wdes > NWBG ? NWBG : wdes);
    wdes &= ~int64_t(G - 1);
    const bool dalign = kAlignSubtiles && a.RB > 0 && (a.RB & 31) == 0 && (tlo & 31) == 0;
    const int64_t dbw = dalign ? a.RB / 32 : 1;  // words per row block
    constexpr int KW0 = (C::NWB + BS - 1) / BS;
    constexpr int KW = KW0 < CBH_DENSE2_PREFETCH ? KW0 : CBH_DENSE2_PREFETCH;
    uint32_t pre[KW > 0 ? KW : 1];
    int64_t pre_w0 = -1;
    int64_t w0 = 0;
    __syncthreads();
    while (w0 < nwt) {
      const int wl = (int)((nwt - w0) < wdes ? (nwt - w0) : wdes);
      const int ng = (wl + G - 1) / G;  // prefix groups of the window (an odd last word padded)
      const int dbase = (int)((TB - 4 * G * ng - 2 * ng) & ~int64_t(15));
      uint32_t* dw = reinterpret_cast<uint32_t*>(win + dbase);
      int16_t* dp = reinterpret_cast<int16_t*>(win + dbase + 4 * G * ng);
      // group g: its G words (one LDS load of 4 G bytes); its popcount; the set bits below `bit`
      auto gpop = [&](int g) -> int {
        if constexpr (G == 4) {
          const uint4 v = reinterpret_cast<const uint4*>(dw)[g];
          return __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
        } else if constexpr (G == 2) {
          return __popcll(reinterpret_cast<const uint64_t*>(dw)[g]);
        } else {
          return __popc(dw[g]);
        }
      };
      auto grank = [&](int g, uint32_t bit, bool& set) -> int {
        if constexpr (G == 4) {
          const uint4 v = reinterpret_cast<const uint4*>(dw)[g];
          const uint32_t wi = bit >> 5, b = bit & 31u;
          const uint32_t w = wi == 0 ? v.x : (wi == 1 ? v.y : (wi == 2 ? v.z : v.w));
          set = (w >> b) & 1u;
          return (wi > 0 ? __popc(v.x) : 0) + (wi > 1 ? __popc(v.y) : 0) + (wi > 2 ? __popc(v.z) : 0) +
                 __popc(w & ((1u << b) - 1u));
        } else if constexpr (G == 2) {
          const uint64_t w = reinterpret_cast<const uint64_t*>(dw)[g];
          set = (w >> bit) & 1ull;
          return (int)__popcll(w & ((1ull << bit) - 1ull));
        } else {
          const uint32_t w = dw[g];
          set = (w >> bit) & 1u;
          return __popc(w & ((1u << bit) - 1u));
        }
      };
      const int capv = dbase / (int)sizeof(acc_t);
      const int kw = (ng + BS - 1) / BS;
      {
        int x = tid;
        if (pre_w0 == w0) {
#pragma unroll
          for (int j = 0; j < KW; ++j)
            if (tid + j * BS < wl) dw[tid + j * BS] = pre[j];
          x += KW * BS;
        }
        for (; x < wl; x += BS) dw[x] = tb[w0 + x];
        if (tid < ng * G - wl) dw[wl + tid] = 0u;  // (the last group's missing words)
      }
      if (tid == 0) s_cut = ng;
      __syncthreads();
      int tsum = 0;
      for (int k = 0; k < kw; ++k) {
        const int x = tid * kw + k;
        tsum += x < ng ? gpop(x) : 0;
      }
      int wtotal = 0;
      int ex = block_excl_sum<BS>(tsum, red, wtotal);
      for (int k = 0; k < kw; ++k) {
        const int x = tid * kw + k;
        if (x < ng) {
          const int pc = gpop(x);
          dp[x] = (int16_t)(ex < 32767 ? ex : 32767);
          if (ex <= capv && ex + pc > capv) s_cut = x;
          ex += pc;
        }
      }
      __syncthreads();
      const int cutg = __builtin_amdgcn_readfirstlane(s_cut);  // (block-uniform values kept in SGPRs)
      int cut = cutg * G < wl ? cutg * G : wl;  // in words
      if (dalign && tlo + 32 * (w0 + cut) < thi) {  // window ends snap down to absolute row blocks
        const int64_t tw0 = tlo / 32;
        int64_t cb = (tw0 + w0 + cut) / dbw * dbw - tw0 - w0;
        cb &= ~int64_t(G - 1);
        if (cb > 0 && cb * 4 >= 3ll * cut) cut = (int)cb;
      }
      const int dtotal = __builtin_amdgcn_readfirstlane(cut < wl ? (int)dp[cut / G] : wtotal);
      // the next window's words, loaded before this window's commit (not before its products: KW
      // registers live across the product phase spilled)
      auto prefetch_next = [&]() {
        const int64_t w0n = w0 + cut;
        if (KW > 0 && w0n < nwt) {
          const int wln = (int)((nwt - w0n) < wdes ? (nwt - w0n) : wdes);
#pragma unroll
          for (int j = 0; j < KW; ++j) pre[j] = (tid + j * BS < wln) ? tb[w0n + tid + j * BS] : 0u;
          pre_w0 = w0n;
        }
      };
      const int32_t lo = (int32_t)(tlo + 32 * w0);
      const int64_t hcut = tlo + 32 * (w0 + cut);
      const int32_t hi = (int32_t)(hcut < thi ? hcut : thi);
      const uint32_t tw = (uint32_t)(hi - lo);
      if (dtotal > 0) {
        for (int x = tid; x < dtotal; x += BS) vals[x] = SR::identity();
        // (phase 1's block scan orders the initialisation before any accumulation)
        run_chunks(lo, hi, [&](int32_t r, const a_t& av, int e) {
          const uint32_t d = (uint32_t)(r - lo);
          if (d >= tw) {
            bad |= 1 << 8;
            return;
          }
          constexpr int SH = G == 4 ? 7 : (G == 2 ? 6 : 5);
          bool set = false;
          const int slot = dp[d >> SH] + grank((int)(d >> SH), d & (32u * G - 1u), set);
          if (!set) bad |= 1 << 11;  // a product row the symbolic pass did not mark
          SR::lds_acc(&vals[slot], SR::multiply(av, cscale[e]));
        });
        inited = true;
        prefetch_next();
        // commit: values in row order (rank q = output out_pos + q), rows off the bitmap
        if (out_pos + dtotal > out_end || out_pos + dtotal > a.ccap) {
          bad |= 1 << 5;
        } else {
          for (int q = tid; q < dtotal; q += BS)
            reinterpret_cast<val_t*>(a.Cnum)[out_pos + q] = SR::finalize(vals[q]);
          const int cg = (cut + G - 1) / G;
          for (int x = tid; x < cg; x += BS) {
            int32_t* cr = a.Cir + out_pos + dp[x];
#pragma unroll
            for (int k = 0; k < G; ++k) {
              uint32_t wv = dw[G * x + k];
              while (wv) {
                *cr++ = lo + 32 * (G * x + k) + __builtin_ctz(wv);
                wv &= wv - 1u;
              }
            }
          }
        }
        out_pos += dtotal;
      } else {
        prefetch_next();
      }
      w0 += cut;
      __syncthreads();
    }
    if (tid == 0 && out_pos != out_end) atomicAdd(&a.err[0], 1);
    if (bad) guard_fail(a.err, 31 - __clz(bad), c, bad, tlo);
  }
}

// Launches dense_kernel over order[first, first+count) (grid slices below 2^32 work-items).
template <class SR, int BS, int EL, int U, int LDSB, int KIND = KDENSE>
hipError_t launch_dense(const TaskArgs& args, int64_t first, int64_t count, hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  using C = DenseCfg<SR, BS, EL, U, LDSB, KIND>;
  auto kern = dense_kernel<SR, BS, EL, U, LDSB, KIND>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)C::bytes);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int64_t kMaxGrid = ((1ll << 32) - 1) / BS;
  for (int64_t off = 0; off < count; off += kMaxGrid) {
    const int64_t n = count - off < kMaxGrid ? count - off : kMaxGrid;
    TaskArgs b = args;
    b.order = args.order + first + off;
    b.norder = n;
    hipLaunchKernelGGL(kern, dim3((unsigned)n), dim3(BS), C::bytes, stream, b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace cbh
