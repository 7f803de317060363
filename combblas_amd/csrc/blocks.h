// gfx950 kernels of the block operations around the phased / 3D drivers and HipMCL's prune:
//
//   column slice     SpDCCols::ColSplit piece [c0, c1) (SpDCCols.cpp:936-1012, Dcsc::ColSplit):
//                    the slot range by two lower bounds on jc, then cp / jc rebased, ir / num copied
//   row slice        rows [r0, r1) of every column, ids rebased (Mult_AnXBn_DoubleBuff's row halves of
//                    B: Transpose + Split + Transpose, ParFriends.h:823-828)
//   column concat    SpDCCols::ColConcatenate (SpDCCols.cpp:1014-1090): column ids and pointers
//                    offset by the earlier blocks' columns / entries
//   MCL masks        MCLPruneRecoverySelect's per-column decisions (ParFriends.h:196-330): which
//                    columns recover, which select, which recover after selection, their k-th value
//                    scattered into the per-column prune threshold
// Included once by spgemm.hip (one translation unit).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace cbh {

// out = {first slot with jc >= c0, first slot with jc >= c1, cp at both}
__global__ void col_range_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp, int64_t nzc,
                                 int64_t c0, int64_t c1, int64_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t s[2];
  const int64_t key[2] = {c0, c1};
  for (int t = 0; t < 2; ++t) {
    int64_t lo = 0, hi = nzc;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (jc[mid] < key[t]) lo = mid + 1;
      else hi = mid;
    }
    s[t] = lo;
  }
  out[0] = s[0];
  out[1] = s[1];
  out[2] = cp[s[0]];
  out[3] = cp[s[1]];
}

// row slice [r0, r1) of every column (rows sorted): first and count of its entries in the range
__global__ void row_range_kernel(const int64_t* __restrict__ cp, const int32_t* __restrict__ ir, int64_t nzc, int32_t r0,
                                 int32_t r1, int64_t* __restrict__ first, int64_t* __restrict__ cnt) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nzc) return;
  int64_t b[2];
  const int32_t key[2] = {r0, r1};
  for (int t = 0; t < 2; ++t) {
    int64_t lo = cp[c], hi = cp[c + 1];
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (ir[mid] < key[t]) lo = mid + 1;
      else hi = mid;
    }
    b[t] = lo;
  }
  first[c] = b[0];
  cnt[c] = b[1] - b[0];
}
// the kept columns' entries (wave per column): rows rebased by -r0, values copied (vb bytes each)
__global__ __launch_bounds__(256) void row_slice_copy_kernel(const int64_t* __restrict__ first,
                                                             const int64_t* __restrict__ cnt,
                                                             const int64_t* __restrict__ off, const int32_t* __restrict__ ir,
                                                             const char* __restrict__ num, int64_t nzc, int32_t r0,
                                                             int64_t vb, int32_t* __restrict__ oir, char* __restrict__ onum) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nzc) return;
  const int64_t f = first[c], k = cnt[c], o = off[c];
  for (int64_t i = lane; i < k; i += 64) oir[o + i] = ir[f + i] - r0;
  for (int64_t i = lane; i < k * vb; i += 64) onum[o * vb + i] = num[f * vb + i];
}

__global__ void fill_f64_kernel(double* __restrict__ p, int64_t n, double v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void add_const_i64_kernel(const int64_t* __restrict__ in, int64_t n, int64_t delta, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i] + delta;
}

// recovery / selection flags of every local column from the (processor-column summed) statistics
// cnt = nnz, cntp / sump = count / sum of the entries > hardThreshold (ParFriends.h:196-253):
//   recover: cntp < recoverNum, cnt > cntp, sump < recoverPct
//   select : not recover, cntp > selectNum (selectNum > 0)
// thresh starts at hardThreshold
__global__ void mcl_flags_kernel(int64_t n, const double* __restrict__ cnt, const double* __restrict__ cntp,
                                 const double* __restrict__ sump, double hard, int64_t selectNum, int64_t recoverNum,
                                 double recoverPct, double* __restrict__ thresh, int64_t* __restrict__ rec,
                                 int64_t* __restrict__ sel) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const bool r = cntp[j] < (double)recoverNum && cnt[j] > cntp[j] && sump[j] < recoverPct;
  rec[j] = r ? 1 : 0;
  sel[j] = (selectNum > 0 && !r && cntp[j] > (double)selectNum) ? 1 : 0;
  thresh[j] = hard;
}

// the selected columns that need recovery after selection (ParFriends.h:318-340): kept count and
// sum of PruneColumn(A, thresh) below recoverNum / recoverPct
__global__ void mcl_recheck_kernel(int64_t n, const int64_t* __restrict__ sel, const double* __restrict__ cntk,
                                   const double* __restrict__ sumk, int64_t recoverNum, double recoverPct,
                                   int64_t* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  out[j] = (sel[j] && cntk[j] < (double)recoverNum && sumk[j] < recoverPct) ? 1 : 0;
}

// active index of every flagged column (its slot in the active list; -1 elsewhere) from the
// exclusive scan of the flags
__global__ void active_index_kernel(int64_t n, const int64_t* __restrict__ flag, const int64_t* __restrict__ pos,
                                    int32_t* __restrict__ aidx) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) aidx[j] = flag[j] ? (int32_t)pos[j] : -1;
}

// radix-select ranks of the active columns (Kselect1: the k-th largest, the smallest when a column
// has fewer than k entries) from their processor-column totals; prefix keys start at 0
__global__ void kselect_rank_kernel(int64_t n, const int32_t* __restrict__ aidx, const double* __restrict__ tot,
                                    int64_t k, int64_t* __restrict__ rank, uint64_t* __restrict__ prefix,
                                    double* __restrict__ totact) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || aidx[j] < 0) return;
  const int64_t a = aidx[j];
  const int64_t t = (int64_t)tot[j];
  rank[a] = t >= k ? k - 1 : t - 1;
  prefix[a] = 0;
  totact[a] = tot[j];
}

// thresh[col] = k-th value of the active column (DBL_MIN where it has no entries: Kselect1's
// numeric_limits<double>::min())
__global__ void kselect_scatter_kernel(int64_t n, const int32_t* __restrict__ aidx, const double* __restrict__ kth,
                                       const double* __restrict__ totact, double* __restrict__ thresh) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || aidx[j] < 0) return;
  const int64_t a = aidx[j];
  thresh[j] = (totact == nullptr || totact[a] > 0) ? kth[a] : 2.2250738585072014e-308;
}

}  // namespace cbh
