// numeric.h -- host-side launch of the numeric SpGEMM kernels for one semiring, shared by the
// library (built-in semirings, combblas_amd/csrc/spgemm.hip) and by user translation units that
// instantiate the kernels for their own semiring (combblas_hip/HipSpGEMMDevice.h). Compile with
// hipcc. The symbolic pass, the task plan and its binning stay in libcombblas_hip.so; they reach
// this code as a cbh_numeric_plan (include/combblas_hip.h, cbh_plan_numeric).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../combblas_hip.h"
#include "dense_kernel.h"
#include "order_kernel.h"
#include "task_kernel.h"
#include "wave_kernel.h"

namespace cbh {

// task-kernel configurations: T slots, BS threads, EMAX entries per chunk, U products per thread
struct TSymSmall { static constexpr int T = 512, BS = 128, EMAX = 256, U = 4; };
// 16 products per thread per window: half the owner-map windows of U = 8, for 12160 instead of
// 13312 bitmap words so that two groups still share a CU (symbolic 201 -> 196 ms at scale 22)
#ifndef CBH_SYM_BS
#define CBH_SYM_BS 512
#endif
#ifndef CBH_SYM_U
#define CBH_SYM_U 16
#endif
#ifndef CBH_SYM_T
#define CBH_SYM_T 8192
#endif
struct TSymLarge { static constexpr int T = CBH_SYM_T, BS = CBH_SYM_BS, EMAX = 512, U = CBH_SYM_U; };
// mid-size symbolic tasks (kSmallCap < products <= kSymMidCap): one sub-tile in a 16 KB key
// table, five workgroups per CU, so the per-task setup latency overlaps
constexpr int kSymMid = 2048;  // (1024 / 4096 measured no better)
struct TSymMid { static constexpr int T = 2 * kSymMid, BS = 256, EMAX = 256, U = 4; };
struct TNumSmall { static constexpr int T = 512, BS = 128, EMAX = 256, U = 4; };
// (T = 8192 with 1024-thread groups, one per CU: 89.1 vs 98.2 GFLOP/s at scale 22)
#ifndef CBH_DENSE_T
#define CBH_DENSE_T 4096
#endif
#ifndef CBH_DENSE_U
#define CBH_DENSE_U 8
#endif
struct TNumLarge { static constexpr int T = CBH_DENSE_T, BS = 512, EMAX = 512, U = CBH_DENSE_U; };
// the table size the dense split rule prices a task with (dense_subtiles: the hash alternative's
// sub-tiles and the dense windows' CAPD / NWB), independent of the kernels' own table sizes
constexpr int64_t kSplitHashT = 4096;
// the library's large hash bin (MODE_TNUM; the dense windows keep TNumLarge): a 2048-slot table
// and 4 products per thread per window keep a group at 53 KB of LDS and <= 80 VGPRs, so THREE
// groups share a CU (24 waves instead of 16): hash 375 -> 360 ms per scale-22 A^2 (A/B twice,
// DESIGN.md §4). T 4096 / U 8 (two groups per CU), 1024 threads / U 4 and 768 threads / U 5
// (VGPR spills), and 5/8 fill of the 2048 table measured slower.
#ifndef CBH_HASH_T
#define CBH_HASH_T 2048
#endif
#ifndef CBH_HASH_BS
#define CBH_HASH_BS 512
#endif
#ifndef CBH_HASH_U
#define CBH_HASH_U 4
#endif
#ifndef CBH_HASH_EMAX
#define CBH_HASH_EMAX 512
#endif
struct TNumHash { static constexpr int T = CBH_HASH_T, BS = CBH_HASH_BS, EMAX = CBH_HASH_EMAX, U = CBH_HASH_U; };
// mid-size hash tasks (kSmallCap < outputs <= kMidCap) of the library's A^2 path: a quarter of the
// large kernel's LDS, so four workgroups share a CU and the per-task setup latency overlaps
constexpr int kMidOut = 1024;  // (512 / 2048 measured no better)
struct TNumMid { static constexpr int T = 2 * kMidOut, BS = 256, EMAX = 256, U = 4; };  // (U 8: flat)
// wider accumulators (user value types) keep the large table within ~50 KB of LDS
template <class SR>
struct TNumLargeFor {
  static constexpr int bytes = (int)(sizeof(int32_t) + sizeof(typename SR::acc_t));
  static constexpr int T = bytes <= 12 ? 4096 : (bytes <= 24 ? 2048 : (bytes <= 48 ? 1024 : 512));
  static constexpr int BS = 512, EMAX = 512, U = 8;
};
template <class SR>
struct TNumMidFor {
  static constexpr int bytes = (int)(sizeof(int32_t) + sizeof(typename SR::acc_t));
  static constexpr int T = bytes <= 12 ? 2 * kMidOut : (bytes <= 24 ? kMidOut : 512);
  static constexpr int BS = 256, EMAX = 256, U = 4;
};
template <class SR>
struct TNumSmallFor {
  static constexpr int bytes = (int)(sizeof(int32_t) + sizeof(typename SR::acc_t));
  static constexpr int T = bytes <= 48 ? 512 : 256;
  static constexpr int BS = 128, EMAX = 256, U = 4;
};
// one task per wavefront (wave_kernel.h) for the small bins: numeric tasks of <= kSmallCap outputs
// in a 512-slot key hash (counting commit), symbolic tasks of <= kSymWaveCap products in a key hash of
// twice that; four waves (four tasks) per workgroup
struct WNumSmall { static constexpr int TW = 512, WPB = 4, U = 4; };
constexpr int kSymWaveCap = 1024;
// numeric tasks of <= kSmallCap outputs but more products than this (compression ratio above
// kWaveProducts / outputs) go to the mid workgroup kernel instead (dense_split_kernel)
constexpr int64_t kWaveProducts = 8192;
struct WSymSmall { static constexpr int TW = 2 * kSymWaveCap, WPB = 4, U = 4; };
// user value types: the wave table while a wave's LDS stays within ~16 KB
template <class SR>
constexpr bool wave_numeric_ok() {
  return sizeof(typename SR::acc_t) <= 16 && sizeof(typename sr_b_type<SR>::type) <= 16;
}
constexpr int64_t kChunkMin = 256;  // tasks with more B entries than this keep cursors in HBM
constexpr int64_t kSmallCap = 256;  // numeric tasks with <= kSmallCap outputs run the small kernel
constexpr int64_t kMidCap = kMidOut;  // ... with <= kMidCap the mid kernel (library numeric pass)
constexpr int64_t kSymMidCap = kSymMid;  // symbolic tasks with <= kSymMidCap products: the mid kernel
static_assert(kChunkMin <= TSymSmall::EMAX && kChunkMin <= TSymMid::EMAX && kChunkMin <= TSymLarge::EMAX &&
                  kChunkMin <= TNumSmall::EMAX && kChunkMin <= TNumMid::EMAX &&
                  kChunkMin <= TNumLarge::EMAX && kChunkMin <= TNumHash::EMAX,
              "every chunked task needs HBM cursor state");

// Launches task_kernel<SR, CFG, MODE> over order[first, first+count) on `stream`, in grid slices
// of fewer than 2^32 work-items (an AQL dispatch counts work-items in 32 bits). The dynamic-LDS
// attribute is set once per instantiation.
template <class SR, class CFG, int MODE, bool MERGE = false>
hipError_t launch_tasks(const TaskArgs& args, int64_t first, int64_t count, hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  using C = TaskCfg<SR, CFG::T, CFG::BS, CFG::EMAX, CFG::U, MODE>;
  auto kern = task_kernel<SR, CFG::T, CFG::BS, CFG::EMAX, CFG::U, MODE, MERGE>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)C::bytes);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int64_t kMaxGrid = ((1ll << 32) - 1) / CFG::BS;
  for (int64_t off = 0; off < count; off += kMaxGrid) {
    const int64_t n = std::min(kMaxGrid, count - off);
    TaskArgs b = args;
    b.order = args.order + first + off;
    b.norder = n;
    hipLaunchKernelGGL(kern, dim3((unsigned)n), dim3(CFG::BS), C::bytes, stream, b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Kernel arguments of the numeric pass from the library's plan; C's entries go to Cir/Cnum at
// toff[task] - cbase.
inline TaskArgs numeric_args(const cbh_numeric_plan& p, int64_t cbase, int32_t* Cir, void* Cnum, int64_t ccap) {
  TaskArgs a{};
  a.Acp = p.Acp;
  a.Air = p.Air;
  a.Anum = p.Anum;
  a.Bcp = p.Bcp;
  a.Bir = p.Bir;
  a.Bnum = p.Bnum;
  a.order = p.order;
  a.hidx = p.hidx;
  a.htab = p.htab;
  a.nblk = p.nblk;
  a.RB = p.RB;
  a.tcol = p.tcol;
  a.tlo = p.tlo;
  a.thi = p.thi;
  a.tfull = p.tfull;
  a.twork = p.tcnt;
  a.toff = p.toff;
  a.cbase = cbase;
  a.Cir = Cir;
  a.Cnum = Cnum;
  a.ccap = ccap;
  a.err = p.err;
  a.nnzA = p.nnzA;
  a.ncolA = p.ncolA;
  a.ntasks = p.ntasks;
  a.goff = p.goff;
  a.gcur0 = p.gcur0;
  a.gcur1 = p.gcur1;
  a.gend = p.gend;
  a.gnx0 = p.gnx0;
  a.gnx1 = p.gnx1;
  a.ghub = p.ghub;
  a.gbase = p.gbase;
  a.boff = p.boff;
  a.bmp = p.bmp;
  return a;
}

// The dense (bitmap-rank) kernel accumulates with SR::lds_acc, so it needs a lock-free add, and the
// library's dense split (cbh_plan_numeric, dense_split_kernel) is computed for the CAPD / NWB
// layout of 8-byte accumulators: other semirings plan with CBH_PLAN_NO_DENSE.
template <class SR>
constexpr bool dense_capable() {
  return !sr_locked<SR>::value && sizeof(typename SR::acc_t) == 8;
}
template <class SR>
constexpr uint32_t plan_flags() {
  return dense_capable<SR>() ? 0u : CBH_PLAN_NO_DENSE;
}

// The dense (bitmap-rank) tasks: dense_kernel.h (round 5: one 1024-thread workgroup per CU with
// the whole LDS, wave-independent products); CBH_DENSE_V2=0 builds the round-4 task_kernel form.
#ifndef CBH_DENSE_V2
#define CBH_DENSE_V2 1
#endif
#ifndef CBH_DENSE2_BS
#define CBH_DENSE2_BS 1024
#endif
#ifndef CBH_DENSE2_U
#define CBH_DENSE2_U 8
#endif
#ifndef CBH_DENSE2_LDS
#define CBH_DENSE2_LDS 163776  // 160 KiB less the kernel's static LDS (s_cut)
#endif
#ifndef CBH_DENSE2_EL  // B entries per chunk (LDS-resident entry state); tasks with more keep it in HBM
#define CBH_DENSE2_EL 512  // round 6 (r6n/r6o, profiles/r06/el_ab): 1024 -> 512 frees entry-state LDS
#endif                     // for wider windows, dense 255.3 -> 250.3 ms; 256 is slower (271.7 ms)
struct TDense2 {
  static constexpr int BS = CBH_DENSE2_BS, EL = CBH_DENSE2_EL, U = CBH_DENSE2_U, LDSB = CBH_DENSE2_LDS;
};
template <class SR>
hipError_t launch_dense_numeric(const TaskArgs& a, int64_t first, int64_t count, hipStream_t s) {
#if CBH_DENSE_V2
  return launch_dense<SR, TDense2::BS, TDense2::EL, TDense2::U, TDense2::LDSB, KDENSE>(a, first, count, s);
#else
  return launch_tasks<SR, TNumLarge, MODE_TDENSE>(a, first, count, s);
#endif
}

// The symbolic pass's large bitmap tasks: the same one-workgroup-per-CU kernel (dense_kernel.h,
// SYM = true: sub-tiles of ~940 K rows instead of task_kernel's 389 K); CBH_SYM_V2=0 keeps them on
// task_kernel<MODE_TSYM>.
#ifndef CBH_SYM_V2
#define CBH_SYM_V2 1
#endif
#ifndef CBH_SYM2_U  // (A/B hook: build variants only)
#define CBH_SYM2_U 8
#endif
#ifndef CBH_SYM2_EL  // B entries per chunk of the symbolic bitmap kernel: 512 (round 6) widens
#define CBH_SYM2_EL 512  // its windows, so more tasks take it: sym_bmp + sym_large 172.1 -> 170.8 ms
#endif
struct TSym2 {
  static constexpr int BS = 1024, EL = CBH_SYM2_EL, U = CBH_SYM2_U, LDSB = 163776;
};
// The numeric hash tasks of the large bin on the same kernel (KHASH: ~7.4 K-slot order-preserving
// table, sub-tiles of ~3.7 K outputs instead of task_kernel's 1 K; U 4: U 8 spills at the 128-VGPR
// bound of 16 waves per CU) -- built with CBH_HASH_V2=1 only: correct (the GPU suite and the
// scale-22 digests pass on it) but slower at scale 22, hash 269.9 -> 343.8 ms (A/B r5f,
// profiles/r05/hash): the hash tasks are short (~9 K outputs, ~2.4 of its sub-tiles each), and one
// workgroup per CU leaves their per-task setup and block scans uncovered, which task_kernel's three
// 53 KB workgroups per CU overlap. Two 512-thread groups per CU (80 KB, ~3.5 K slots) and four
// 256-thread groups (40 KB) were slower still: hash 280.7 / 279.5 vs 234.1 ms (r5h2,
// profiles/r05/hash). TNumHash stays the shipped hash kernel.
#ifndef CBH_HASH_V2
#define CBH_HASH_V2 0
#endif
#ifndef CBH_HASH2_BS  // (A/B hooks: build variants only)
#define CBH_HASH2_BS 1024
#endif
#ifndef CBH_HASH2_EL
#define CBH_HASH2_EL CBH_HASH2_BS
#endif
#ifndef CBH_HASH2_LDS
#define CBH_HASH2_LDS 163776
#endif
struct THash2 {
  static constexpr int BS = CBH_HASH2_BS, EL = CBH_HASH2_EL, U = 4, LDSB = CBH_HASH2_LDS;
};

// Numeric tasks of the small bin: one per wave (wave_kernel.h); wide user value types keep the
// workgroup kernel CFG.
template <class SR, class CFG>
hipError_t launch_small_numeric(const TaskArgs& a, int64_t first, int64_t count, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  if constexpr (wave_numeric_ok<SR>())
    return launch_waves<SR, WNumSmall::TW, WNumSmall::WPB, WNumSmall::U, MODE_TNUM>(a, first, count, s);
  return launch_tasks<SR, CFG, MODE_TNUM>(a, first, count, s);
}

// The numeric pass of a plan for semiring SR: dense tasks (if the plan binned any), hash tasks of
// the large, mid and small kernels, all on the plan's stream. C is the matrix cbh_plan_numeric
// allocated with plan_flags<SR>().
template <class SR>
hipError_t run_numeric_plan(const cbh_numeric_plan& p, int32_t* Cir, void* Cnum, int64_t ccap) {
  const TaskArgs a = numeric_args(p, 0, Cir, Cnum, ccap);
  hipStream_t s = reinterpret_cast<hipStream_t>(p.stream);
  hipError_t e = hipSuccess;
  if constexpr (dense_capable<SR>()) {
    e = launch_dense_numeric<SR>(a, p.dense_first, p.dense_count, s);
    if (e != hipSuccess) return e;
  } else if (p.dense_count > 0) {
    return hipErrorInvalidValue;  // planned without CBH_PLAN_NO_DENSE
  }
  e = launch_tasks<SR, TNumLargeFor<SR>, MODE_TNUM>(a, p.large_first, p.large_count, s);
  if (e != hipSuccess) return e;
  e = launch_tasks<SR, TNumMidFor<SR>, MODE_TNUM>(a, p.mid_first, p.mid_count, s);
  if (e != hipSuccess) return e;
  return launch_small_numeric<SR, TNumSmallFor<SR>>(a, p.small_first, p.small_count, s);
}

}  // namespace cbh
