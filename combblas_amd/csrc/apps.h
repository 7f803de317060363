// gfx950 kernels for the callers either side of the SpGEMM hot path:
//
//   masked_kernel        C = (A*B) .* M in one pass         [TC.cpp:108-110: Mult_AnXBn_Synch(L, L) then
//                                                             C.EWiseMult(L, false) = Friends.h:834-887]
//   ewise_kernel         C = A .* B (pattern intersection, values multiplied)   [Friends.h:834-887]
//   colstat_kernel       per-column count, count and sum of the entries above a threshold
//                                                           [SpParMat::Reduce(Column, ...), ParFriends.h:196-200]
//   kselect_hist/pick    k-th largest value per active column, radix select over order-preserving
//                        keys; histograms can be summed over a processor column between passes
//                                                           [SpParMat::Kselect1, SpParMat.cpp:1413-1700]
//   prune_col_kernel     keep entries !(v < thresh[col])    [Dcsc::PruneColumn, dcsc.cpp:699-760]
//
// Included once by spgemm.hip (one translation unit).
#pragma once
#include "../../include/combblas_hip/device/task_kernel.h"

namespace cbh {

// ---------------------------------------------------------------------------- masked SpGEMM
// One workgroup per nonzero column slot c of B whose column also exists in M. The mask column's
// rows are staged in LDS in chunks of MCAP (sorted); the products whose rows fall in the chunk's
// row range are flattened over the workgroup (segment scan + binary search for the owner), each
// product's row is looked up in the staged rows by binary search and accumulated with SR::add
// (a zero-valued product still creates the entry, as explicit zeros do in the reference). Hits
// are written in mask order (rows ascending) at Mcp[ms] + rank into a temporary indexed like M;
// the per-column hit counts drive the final compaction. PATTERN: values are the semiring sums
// (the mask only selects); otherwise they are multiplied by M's values (EWiseMult).
struct MaskArgs {
  const int64_t* Acp;  // A dense column pointers (A.n + 1)
  const int32_t* Air;
  const void* Anum;
  const int64_t* Bcp;  // B DCSC (per slot)
  const int32_t* Bir;
  const void* Bnum;
  int64_t nzcB;
  const int64_t* mslot;  // per B slot: M's slot with the same column id, -1 if none
  const int64_t* Mcp;
  const int32_t* Mir;
  const void* Mnum;
  int32_t* Tir;  // temporary output, nnz(M) slots, indexed like M
  void* Tnum;
  int64_t* hits;  // per B slot
  int* err;
  int64_t nnzA, ncolA;
};

template <class SR, int MCAP, int BS, int EMAX, bool PATTERN>
__global__ __launch_bounds__(BS) void masked_kernel(MaskArgs a) {
  using val_t = typename SR::val_t;
  using acc_t = typename SR::acc_t;
  constexpr int NW = BS / 64;
  static_assert(EMAX >= BS, "the hit scan reuses eoff[0..BS]");
  __shared__ int32_t mrow[MCAP];
  __shared__ acc_t acc[MCAP];
  __shared__ int32_t hit[MCAP];
  __shared__ int64_t ebeg[EMAX];
  __shared__ int32_t eoff[EMAX + 1];
  __shared__ val_t escale[EMAX];
  __shared__ int red[2 * NW + 4];
  const int tid = threadIdx.x;
  const int64_t c = blockIdx.x;
  if (c >= a.nzcB) return;
  const int64_t ms = a.mslot[c];
  if (ms < 0) {
    if (tid == 0) a.hits[c] = 0;
    return;
  }
  const int64_t m0 = a.Mcp[ms], m1 = a.Mcp[ms + 1];
  const int64_t e0 = a.Bcp[c], ne = a.Bcp[c + 1] - e0;
  int64_t nhits = 0;
  for (int64_t x0 = m0; x0 < m1; x0 += MCAP) {
    const int cnt = (int)((m1 - x0) < MCAP ? (m1 - x0) : MCAP);
    for (int i = tid; i < cnt; i += BS) {
      mrow[i] = a.Mir[x0 + i];
      acc[i] = SR::identity();
      hit[i] = 0;
    }
    __syncthreads();
    const int32_t rlo = mrow[0], rhi = mrow[cnt - 1];
    for (int64_t f0 = 0; f0 < ne; f0 += EMAX) {
      const int nec = (int)((ne - f0) < EMAX ? (ne - f0) : EMAX);
      // segment of every entry inside [rlo, rhi]
      for (int i = tid; i < nec; i += BS) {
        const int64_t p = e0 + f0 + i;
        const int32_t k = a.Bir[p];
        int64_t s = 0, e = 0;
        if (k >= 0 && k < a.ncolA) {
          const int64_t base = a.Acp[k], end = a.Acp[k + 1];
          s = lb_rows64(a.Air, base, end, rlo);
          e = lb_rows64(a.Air, s, end, rhi + 1);  // row ids are < m < 2^31 - 1
        } else {
          guard_fail(a.err, 20, c, k);
        }
        ebeg[i] = s;
        eoff[i] = (int32_t)(e - s);
        escale[i] = reinterpret_cast<const val_t*>(a.Bnum)[p];
      }
      __syncthreads();
      block_scan_excl<BS>(eoff, nec, red);
      const int P = eoff[nec];
      for (int x = tid; x < P; x += BS) {
        // owner: the last entry whose segment starts at or before x (LDS binary search)
        int lo = 0, hi = nec - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (eoff[mid] <= x) lo = mid;
          else hi = mid - 1;
        }
        const int64_t q = ebeg[lo] + (x - eoff[lo]);
        const int32_t r = a.Air[q];
        const val_t av = reinterpret_cast<const val_t*>(a.Anum)[q];
        int l2 = 0, h2 = cnt;  // mask lookup
        while (l2 < h2) {
          const int mid = (l2 + h2) >> 1;
          if (mrow[mid] < r) l2 = mid + 1;
          else h2 = mid;
        }
        if (l2 < cnt && mrow[l2] == r) {
          SR::lds_acc(&acc[l2], SR::multiply(av, escale[lo]));
          hit[l2] = 1;
        }
      }
      __syncthreads();
    }
    // hits of this chunk in mask order
    int carry = 0;
    for (int base = 0; base < cnt; base += BS) {
      const int i = base + tid;
      const int h = (i < cnt) ? hit[i] : 0;
      eoff[tid] = h;
      __syncthreads();
      block_scan_excl<BS>(eoff, BS, red);
      if (h) {
        const int64_t pos = m0 + nhits + carry + eoff[tid];
        a.Tir[pos] = mrow[i];
        val_t v = SR::finalize(acc[i]);
        if constexpr (!PATTERN) v = (val_t)(v * reinterpret_cast<const val_t*>(a.Mnum)[x0 + i]);  // Friends.h:871
        reinterpret_cast<val_t*>(a.Tnum)[pos] = v;
      }
      carry += eoff[BS];
      __syncthreads();
    }
    nhits += carry;
    __syncthreads();
  }
  if (tid == 0) a.hits[c] = nhits;
}

// per slot of X: Y's slot holding the same column id (both jc arrays ascending), -1 if none
__global__ void match_slots_kernel(const int64_t* __restrict__ Xjc, int64_t nzcX, const int64_t* __restrict__ Yjc,
                                   int64_t nzcY, int64_t* __restrict__ yslot) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nzcX) return;
  const int64_t col = Xjc[i];
  int64_t lo = 0, hi = nzcY;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (Yjc[mid] < col) lo = mid + 1;
    else hi = mid;
  }
  yslot[i] = (lo < nzcY && Yjc[lo] == col) ? lo : -1;
}

// compaction of a temporary whose column c starts at src_cp[sslot[c]]: wave per column copies
// its hits[c] entries to off[c]
template <class V>
__global__ __launch_bounds__(256) void gather_cols_kernel(const int64_t* __restrict__ sslot,
                                                          const int64_t* __restrict__ src_cp,
                                                          const int64_t* __restrict__ hits,
                                                          const int64_t* __restrict__ off, int64_t ncols,
                                                          const int32_t* __restrict__ Tir, const V* __restrict__ Tnum,
                                                          int32_t* __restrict__ Cir, V* __restrict__ Cnum) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= ncols) return;
  const int64_t h = hits[c];
  if (h <= 0) return;
  const int64_t src = src_cp[sslot[c]], dst = off[c];
  for (int64_t i = lane; i < h; i += 64) {
    Cir[dst + i] = Tir[src + i];
    Cnum[dst + i] = Tnum[src + i];
  }
}

// C = A .* B (Friends.h:834-887, exclude = false): wave per A slot; each A entry looks its row up
// in B's column (binary search), matches are compacted by ballot in A's row order. Pass 1
// counts (hits per A slot), pass 2 writes at off[slot].
template <class V, bool WRITE>
__global__ __launch_bounds__(256) void ewise_kernel(const int64_t* __restrict__ Acp, const int32_t* __restrict__ Air,
                                                    const V* __restrict__ Anum, int64_t nzcA,
                                                    const int64_t* __restrict__ bslot, const int64_t* __restrict__ Bcp,
                                                    const int32_t* __restrict__ Bir, const V* __restrict__ Bnum,
                                                    int64_t* __restrict__ hits, const int64_t* __restrict__ off,
                                                    int32_t* __restrict__ Cir, V* __restrict__ Cnum) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nzcA) return;
  const int64_t bs = bslot[s];
  int64_t o = WRITE ? off[s] : 0;
  if (bs >= 0) {
    const int64_t b0 = Bcp[bs], b1 = Bcp[bs + 1];
    const int64_t p0 = Acp[s], p1 = Acp[s + 1];
    for (int64_t base = p0; base < p1; base += 64) {
      const int64_t p = base + lane;
      bool hit = false;
      int64_t q = 0;
      if (p < p1) {
        const int32_t r = Air[p];
        q = lb_rows64(Bir, b0, b1, r);
        hit = q < b1 && Bir[q] == r;
      }
      const uint64_t m = __ballot(hit);
      if (WRITE && hit) {
        const int64_t d = o + __popcll(m & ((1ull << lane) - 1ull));
        Cir[d] = Air[p];
        Cnum[d] = (V)(Anum[p] * Bnum[q]);
      }
      o += __popcll(m);
    }
  }
  if (!WRITE && lane == 0) hits[s] = o;
}

// ---------------------------------------------------------------------------- MCL column ops
// Wave per nonzero column slot; outputs dense over the n local columns (index jc[slot]), zero
// where a column has no slot:
//   cnt[col]  = nnz of the column                 (A.Reduce(Column, plus, 0, v->1))
//   cntp[col] = entries with v > hard             (nnz of A.Prune(v <= hard))
//   sump[col] = sum of those entries              (PrunedA.Reduce(Column, plus, 0))
__global__ __launch_bounds__(256) void colstat_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp,
                                                      const double* __restrict__ num, int64_t nzc, double hard,
                                                      double* __restrict__ cnt, double* __restrict__ cntp,
                                                      double* __restrict__ sump) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nzc) return;
  const int64_t p0 = cp[s], p1 = cp[s + 1];
  double n1 = 0, s1 = 0;
  for (int64_t p = p0 + lane; p < p1; p += 64) {
    const double v = num[p];
    if (v > hard) {
      n1 += 1.0;
      s1 += v;
    }
  }
  // the reference sums a column serially; counts are exact, this reduction tree's sum can differ
  // from the serial one in the last bits
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    n1 += __shfl_xor(n1, o);
    s1 += __shfl_xor(s1, o);
  }
  if (lane == 0) {
    const int64_t col = jc[s];
    cnt[col] = (double)(p1 - p0);
    cntp[col] = n1;
    sump[col] = s1;
  }
}

// order-preserving map of a double onto uint64 (larger value -> larger key)
__device__ __forceinline__ uint64_t fkey(double v) {
  uint64_t b;
  __builtin_memcpy(&b, &v, 8);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double fval(uint64_t k) {
  const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  double v;
  __builtin_memcpy(&v, &b, 8);
  return v;
}

// One radix-select pass (8 bits at `shift`) for the active columns: hist[a*256 + d] = number of
// the column's keys that match prefix[a] above the digit and have digit d. Workgroup per slot.
__global__ __launch_bounds__(256) void kselect_hist_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp,
                                                           const double* __restrict__ num, int64_t nzc,
                                                           const int32_t* __restrict__ aidx,
                                                           const uint64_t* __restrict__ prefix, int shift,
                                                           uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const int64_t s = blockIdx.x;
  if (s >= nzc) return;
  const int32_t ai = aidx[jc[s]];
  if (ai < 0) return;
  const int tid = threadIdx.x;
  h[tid] = 0;
  __syncthreads();
  const uint64_t pre = prefix[ai];
  const uint64_t himask = shift >= 56 ? 0ull : (~0ull << (shift + 8));
  for (int64_t p = cp[s] + tid; p < cp[s + 1]; p += 256) {
    const uint64_t key = fkey(num[p]);
    if ((key & himask) == pre) atomicAdd(&h[(key >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(int64_t)ai * 256 + tid] = h[tid];
}

// Thread per active column: the digit holding descending rank[a] (largest digits first); rank
// becomes the rank inside that digit. rank < 0 marks an empty column (left alone).
__global__ void kselect_pick_kernel(int64_t nact, const uint32_t* __restrict__ hist, uint64_t* __restrict__ prefix,
                                    int64_t* __restrict__ rank, int shift) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= nact) return;
  int64_t r = rank[a];
  if (r < 0) return;
  const uint32_t* H = hist + a * 256;
  int b = 255;
  for (; b > 0; --b) {
    if (r < (int64_t)H[b]) break;
    r -= H[b];
  }
  prefix[a] |= (uint64_t)b << shift;
  rank[a] = r;
}

__global__ void kselect_value_kernel(int64_t nact, const uint64_t* __restrict__ prefix, double* __restrict__ out) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a < nact) out[a] = fval(prefix[a]);
}

// keep entry (i, col) iff !(v < thresh[col]): pass 1 counts per slot, pass 2 copies
template <bool COPY>
__global__ __launch_bounds__(256) void prune_col_kernel(const int64_t* __restrict__ jc, const int64_t* __restrict__ cp,
                                                        const int32_t* __restrict__ ir, const double* __restrict__ num,
                                                        int64_t nzc, const double* __restrict__ thresh,
                                                        int64_t* __restrict__ kept, const int64_t* __restrict__ off,
                                                        int32_t* __restrict__ oir, double* __restrict__ onum) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nzc) return;
  const double t = thresh[jc[s]];
  const int64_t p0 = cp[s], p1 = cp[s + 1];
  int64_t o = COPY ? off[s] : 0;
  for (int64_t b = p0; b < p1; b += 64) {
    const int64_t p = b + lane;
    const double v = p < p1 ? num[p] : 0.0;
    const bool keep = p < p1 && !(v < t);
    const uint64_t m = __ballot(keep);
    if (COPY && keep) {
      const int64_t d = o + __popcll(m & ((1ull << lane) - 1ull));
      oir[d] = ir[p];
      onum[d] = v;
    }
    o += __popcll(m);
  }
  if (!COPY && lane == 0) kept[s] = o;
}

}  // namespace cbh
