// wave_kernel.h -- short tasks, ONE TASK PER WAVEFRONT (north_star: "per-wavefront LDS hash
// tables for short rows"; the reference's short-column branch is the heap of mtSpGEMM.h:311-360).
//
// A workgroup of WPB waves runs WPB independent tasks: each wave owns a slice of the workgroup's
// LDS (its table) and never waits on another wave -- no block barriers, no block scans, no owner
// map. Per chunk of 64 B entries (one per lane) the wave loads each entry's A segment bounds,
// takes a shuffle scan of the segment lengths, and flattens the products: lane p finds its entry
// by a 6-step shuffle search over the exclusive offsets and gathers U products before any table
// update. Tasks come from the small bins, so one table holds the whole task (no sub-tiles):
//   symbolic (MODE_TSYM): multiplicative key hash of TW >= 2 x products slots (never fills), the
//            count of first insertions -> cnt[task]                       [estimateNNZ_Hash]
//   numeric  (MODE_TNUM): the same key hash (TW >= 2 x outputs) with SR::add(SR::multiply(a,b))
//            into the slot's accumulator, then a COUNTING commit: the occupied keys are compacted
//            into a list and every key's output position is the number of smaller keys in it
//            (broadcast LDS reads, no dependent chains; <= TW/2 keys). The workgroup kernels'
//            order-preserving slot map (slot = (row-lo)*T/span) is not used here: short columns of
//            structured matrices (C3's stencil x prolongation) cluster their rows in a few narrow
//            bands, which it maps to a few home slots -- probe chains of ~25 CAS per product.
#pragma once
#include "task_kernel.h"

namespace cbh {

// LDS visibility between the lanes of one wave (the wave's LDS operations complete in order;
// this keeps the compiler from moving them across the hand-off)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <class SR, int TW, int MODE>
struct WaveCfg {
  static constexpr bool NUM = MODE == MODE_TNUM;
  using acc_t = typename SR::acc_t;
  using b_t = typename sr_b_type<SR>::type;
  static constexpr int NOUT = TW / 2;  // outputs (keys) a task may have
  static constexpr size_t al(size_t x) { return (x + 15) & ~size_t(15); }
  static constexpr size_t o_keys = 0;
  static constexpr size_t o_vals = al(sizeof(int32_t) * TW);
  static constexpr size_t o_base = al(o_vals + (NUM ? sizeof(acc_t) * TW : 0));  // 64 gather bases
  static constexpr size_t o_scale = al(o_base + sizeof(int64_t) * 64);           // 64 B values
  static constexpr size_t o_klist = al(o_scale + (NUM ? sizeof(b_t) * 64 : 0));   // commit: keys (+4 pad)
  static constexpr size_t o_q = al(o_klist + (NUM ? sizeof(int32_t) * (NOUT + 4) : 0));  // their slots
  static constexpr size_t bytes = al(o_q + (NUM ? sizeof(int16_t) * NOUT : 0));  // per wave
};

template <class SR, int TW, int WPB, int U, int MODE>
__global__ __launch_bounds__(64 * WPB) void wave_kernel(TaskArgs a) {
  using C = WaveCfg<SR, TW, MODE>;
  using val_t = typename SR::val_t;
  using acc_t = typename SR::acc_t;
  using a_t = typename sr_a_type<SR>::type;
  using b_t = typename C::b_t;
  constexpr bool NUM = C::NUM;
  constexpr bool LOCKED = sr_locked<SR>::value;
  static_assert((TW & (TW - 1)) == 0 && TW >= 64, "table size must be a power of two");
  static_assert(MODE == MODE_TSYM || MODE == MODE_TNUM, "wave kernel: symbolic or numeric hash");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t slot = (int64_t)blockIdx.x * WPB + wid;
  if (slot >= a.norder) return;  // waves are independent: nothing below waits on another wave
  unsigned char* wb = smem + (size_t)wid * C::bytes;
  int32_t* keys = reinterpret_cast<int32_t*>(wb + C::o_keys);
  acc_t* vals = reinterpret_cast<acc_t*>(wb + C::o_vals);
  int64_t* ebase = reinterpret_cast<int64_t*>(wb + C::o_base);
  b_t* escale = reinterpret_cast<b_t*>(wb + C::o_scale);
  int32_t* klist = reinterpret_cast<int32_t*>(wb + C::o_klist);
  int16_t* Q = reinterpret_cast<int16_t*>(wb + C::o_q);
  const int32_t* __restrict__ rowsA = a.Air;

  const int32_t task = a.order[slot];
  if (task < 0 || task >= a.ntasks) {
    if (lane == 0) guard_fail(a.err, 9, task);
    return;
  }
  const int32_t c = a.tcol[task];
  const int64_t e0 = a.Bcp[c];
  const int64_t ne = a.Bcp[c + 1] - e0;
  const int64_t work = a.twork[task];
  const int32_t tlo = a.tlo[task], thi = a.thi[task];
  const uint8_t full = a.tfull[task];
  if (work <= 0 || thi <= tlo) {
    if (!NUM && lane == 0) a.cnt[task] = 0;
    return;
  }
  for (int s = lane; s < TW; s += 64) {
    keys[s] = kEmpty;
    if constexpr (NUM && !LOCKED) vals[s] = SR::identity();
  }
  const uint32_t tw = (uint32_t)(thi - tlo);
  int my_count = 0;  // symbolic: keys this lane inserted first
  int bad = 0;
  wave_lds_sync();

  for (int64_t eb = 0; eb < ne; eb += 64) {
    const int64_t i = eb + lane;
    int64_t pos = 0;
    int len = 0;
    if (i < ne) {
      const int32_t k = a.Bir[e0 + i];
      if (k < 0 || k >= a.ncolA) {
        bad |= 1 << 1;
      } else {
        int64_t b0 = a.Acp[k], b1 = a.Acp[k + 1];
        if (b0 < 0 || b1 < b0 || b1 > a.nnzA) {
          bad |= 1 << 2;
          b0 = b1 = 0;
        }
        // clamp to the task's rows (small tasks usually own whole columns: full == 3)
        if (!(full & 2) && b0 < b1) b1 = lb_rows64(rowsA, b0, b1, thi);
        if (!(full & 1) && b0 < b1) b0 = lb_rows64(rowsA, b0, b1, tlo);
        pos = b0;
        len = (int)(b1 - b0);
        if constexpr (NUM) escale[lane] = reinterpret_cast<const b_t*>(a.Bnum)[e0 + i];
      }
    }
    int incl = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    const int total = __shfl(incl, 63);
    const int excl = incl - len;
    ebase[lane] = pos - excl;  // product p of this entry reads A at ebase + p
    wave_lds_sync();
    for (int p0 = 0; p0 < total; p0 += 64 * U) {
      int32_t r[U];
      val_t av[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + u * 64 + lane;
        const int pp = p < total ? p : total - 1;
        // owner: the last lane whose exclusive offset is <= pp (lanes without products share
        // their successor's offset; lanes past the chunk hold offset `total`)
        int j = 0;
#pragma unroll
        for (int st = 32; st > 0; st >>= 1) {
          const int ex = __shfl(excl, j + st);
          if (ex <= pp) j += st;
        }
        const int64_t q = ebase[j] + pp;
        r[u] = rowsA[q];
        if constexpr (NUM) av[u] = SR::multiply(reinterpret_cast<const a_t*>(a.Anum)[q], escale[j]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (p0 + u * 64 + lane >= total) continue;
        const uint32_t d = (uint32_t)(r[u] - tlo);
        if (d >= tw) {
          bad |= 1 << 8;
          continue;
        }
        // key hash with wrap-around probing: at most TW/2 distinct keys, so a free slot is always
        // found (the bins guarantee the bound; a key past it is a count mismatch below)
        constexpr int LG = __builtin_ctz(TW);
        uint32_t s = ((uint32_t)r[u] * 0x9E3779B1u) >> (32 - LG);
        for (int probe = 0; probe < TW; ++probe, s = (s + 1) & (TW - 1)) {
          if constexpr (NUM && LOCKED) {
            if (locked_insert<SR>(&keys[s], &vals[s], r[u], av[u])) break;
          } else {
            const int32_t k = atomicCAS(&keys[s], kEmpty, r[u]);
            if constexpr (!NUM) {
              if (k == kEmpty) ++my_count;
            }
            if (k == kEmpty || k == r[u]) {
              if constexpr (NUM) SR::lds_acc(&vals[s], av[u]);
              break;
            }
          }
        }
      }
    }
    wave_lds_sync();  // the next chunk overwrites ebase / escale
  }

  if constexpr (!NUM) {
    int t = my_count;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if (lane == 0) a.cnt[task] = t;
  } else {
    // occupied keys (and their slots) compacted into a list; a key's output position is the
    // number of smaller keys in the list (keys are distinct rows): 4 keys per lane, the list read
    // by broadcast in 16-byte groups
    const uint64_t lt = (1ull << lane) - 1ull;
    int n = 0;
    for (int b = 0; b < TW / 64; ++b) {
      const int sl = 64 * b + lane;
      const int32_t k = keys[sl];
      const uint64_t m = __ballot(k != kEmpty);
      const int at = n + __popcll(m & lt);
      if (k != kEmpty && at < C::NOUT) {
        klist[at] = k;
        Q[at] = (int16_t)sl;
      }
      n += __popcll(m);
    }
    const int64_t out_pos = a.toff[task] - a.cbase;
    const int64_t out_end = a.toff[task + 1] - a.cbase;
    if (n > C::NOUT || out_pos + n != out_end) {
      if (lane == 0) atomicAdd(&a.err[0], 1);  // count mismatch with the symbolic pass
    } else {
      if (lane < 4) klist[n + lane] = kNoRow;  // pad of the 16-byte groups (> every row)
      wave_lds_sync();
      constexpr int NK = C::NOUT / 64;
      int32_t key[NK];
      int rank[NK];
#pragma unroll
      for (int i = 0; i < NK; ++i) {
        key[i] = 64 * i + lane < n ? klist[64 * i + lane] : kNoRow;
        rank[i] = 0;
      }
      const int nk = (n + 63) / 64;
      for (int t = 0; t < n; t += 4) {
        const int4 v = *reinterpret_cast<const int4*>(&klist[t]);
#pragma unroll
        for (int i = 0; i < NK; ++i)
          if (i < nk) rank[i] += (v.x < key[i]) + (v.y < key[i]) + (v.z < key[i]) + (v.w < key[i]);
      }
      val_t* __restrict__ Cnum = reinterpret_cast<val_t*>(a.Cnum);
#pragma unroll
      for (int i = 0; i < NK; ++i) {
        const int q = 64 * i + lane;
        if (q < n) {
          const int64_t pos = out_pos + rank[i];
          if (pos >= out_end || pos >= a.ccap) {
            bad |= 1 << 5;
          } else {
            a.Cir[pos] = key[i];
            Cnum[pos] = SR::finalize(vals[Q[q]]);
          }
        }
      }
    }
  }
  if (bad) guard_fail(a.err, 31 - __clz(bad), c, bad, task);
}

// Launches wave_kernel over order[first, first+count) in grid slices below 2^32 work-items.
template <class SR, int TW, int WPB, int U, int MODE>
hipError_t launch_waves(const TaskArgs& args, int64_t first, int64_t count, hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  using C = WaveCfg<SR, TW, MODE>;
  auto kern = wave_kernel<SR, TW, WPB, U, MODE>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)(C::bytes * WPB));
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int64_t kMaxTasks = ((1ll << 32) - 1) / 64 / WPB * WPB;
  for (int64_t off = 0; off < count; off += kMaxTasks) {
    const int64_t n = count - off < kMaxTasks ? count - off : kMaxTasks;
    TaskArgs b = args;
    b.order = args.order + first + off;
    b.norder = n;
    hipLaunchKernelGGL(kern, dim3((unsigned)((n + WPB - 1) / WPB)), dim3(64 * WPB), C::bytes * WPB, stream, b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace cbh
