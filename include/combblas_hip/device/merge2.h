// merge2.h -- the two-list MultiwayMerge (MultiwayMerge.h:411-526 for k = 2: two SUMMA stage
// partials, or a 3D fiber's own and received pieces) as a streaming MERGE PATH instead of the
// task kernels' LDS hash (task_kernel.h MERGE mode).
//
// Both lists hold, per column, rows ascending and unique, so the merged column is the sorted
// union, an entry present in both lists folded with SR::add(list-0 value, list-1 value). The
// union columns' entries are cut along merge-path diagonals into chunks of kChunk inputs; one
// wavefront walks one chunk 64 outputs at a time:
//   * a step's window: lane t holds a[i0 + t] and b[j0 + t] (coalesced loads; a[i0 - 1] as a
//     wave-uniform scalar);
//   * lane l finds the co-rank of diagonal l + 1 inside the window (how many of the first l + 1
//     outputs come from a; ties emit a first) by a 7-step binary search over shuffled window
//     values, so output l is a[i0 + x_l] or b[j0 + l - x_l], x_l taken from lane l - 1;
//   * an output from b whose row equals the a-row emitted just before it is that entry's second
//     half: not a head. An a-output whose row equals the next b (b[j0 + l - x_l]) folds that b's
//     value in -- also when that b opens the next step or chunk, which then sees it as a tail;
//   * heads are numbered by a ballot prefix.
// Pass 1 counts the heads of every chunk; an exclusive scan over the chunks (they are in column
// order, and C is laid out column by column) gives every chunk its output offset and every column
// its pointer; pass 2 repeats the walk and writes rows and values at those offsets. Traffic: the
// rows twice, the values and C once -- streaming, no LDS table, no commit.
#pragma once
#include "block_ops.h"

namespace cbh {

constexpr int kMerge2Chunk = 64 * 32;  // inputs per wavefront (merge-path diagonals)

// chunks per union column c: ceil((len0 + len1) / kChunk) (seg_len holds [c * 2 + l])
__global__ __launch_bounds__(256) void merge2_nchunks_kernel(const int64_t* __restrict__ seg_len, int64_t ncols,
                                                             int64_t* __restrict__ nch) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncols) return;
  const int64_t len = seg_len[2 * c] + seg_len[2 * c + 1];
  nch[c] = (len + kMerge2Chunk - 1) / kMerge2Chunk;
}
// chunk -> its column (thread per column writes its chunks)
__global__ __launch_bounds__(256) void merge2_fill_kernel(const int64_t* __restrict__ cstart, int64_t ncols,
                                                          int32_t* __restrict__ chunk_col) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncols) return;
  for (int64_t k = cstart[c]; k < cstart[c + 1]; ++k) chunk_col[k] = (int32_t)c;
}

// co-rank: the number of a-elements among the first d outputs of merge(a[0, na), b[0, nb)), ties a first
__device__ __forceinline__ int64_t merge2_corank(const int32_t* __restrict__ a, int64_t na, const int32_t* __restrict__ b,
                                                 int64_t nb, int64_t d) {
  int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= b[d - 1 - mid]) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// One wavefront per chunk (blockDim 64 * WPB, wave w of block k takes chunk k * WPB + w).
// WRITE = false: head count per chunk into cnt[k]; WRITE = true: rows / values at off[k].
template <class SR, bool WRITE, int WPB>
__global__ __launch_bounds__(64 * WPB) void merge2_kernel(const int32_t* __restrict__ chunk_col, int64_t nchunks,
                                                          const int64_t* __restrict__ cstart,
                                                          const int64_t* __restrict__ seg_start,
                                                          const int64_t* __restrict__ seg_len,
                                                          const int32_t* __restrict__ ir0, const void* __restrict__ num0,
                                                          const int32_t* __restrict__ ir1, const void* __restrict__ num1,
                                                          int64_t* __restrict__ cnt, const int64_t* __restrict__ off,
                                                          int32_t* __restrict__ Cir, void* __restrict__ Cnum) {
  using val_t = typename SR::val_t;
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (k >= nchunks) return;
  const int32_t c = chunk_col[k];
  const int64_t sa = seg_start[2 * c], na = seg_len[2 * c];
  const int64_t sb = seg_start[2 * c + 1], nb = seg_len[2 * c + 1];
  const int32_t* __restrict__ a = ir0 + sa;
  const int32_t* __restrict__ b = ir1 + sb;
  const val_t* __restrict__ av = reinterpret_cast<const val_t*>(num0) + sa;
  const val_t* __restrict__ bv = reinterpret_cast<const val_t*>(num1) + sb;
  const int64_t total = na + nb;
  const int64_t d0 = (k - cstart[c]) * kMerge2Chunk;
  const int64_t d1 = d0 + kMerge2Chunk < total ? d0 + kMerge2Chunk : total;
  int64_t i0 = merge2_corank(a, na, b, nb, d0);  // (every lane: same loads, one transaction each)
  int64_t j0 = d0 - i0;
  int64_t out = WRITE ? off[k] : 0;
  int64_t heads = 0;
  constexpr int32_t kEnd = 0x7fffffff;  // past a list's end (rows are < 2^31 - 1)
  for (int64_t d = d0; d < d1; d += 64) {
    const int len = d1 - d < 64 ? (int)(d1 - d) : 64;
    const int32_t ra = i0 + lane < na ? a[i0 + lane] : kEnd;
    const int32_t rb = j0 + lane < nb ? b[j0 + lane] : kEnd;
    const int32_t am1 = i0 > 0 ? a[i0 - 1] : -1;
    // every index below stays inside the window: the search probes a[mid], b[l - mid] with
    // mid < min(l + 1, 64); an a-output's next b is b[j0 + l - x_l], l - x_l <= 63
    auto geta = [&](int t) -> int32_t {  // a[i0 + t], t in [-1, 63]
      const int32_t s = __shfl(ra, t & 63);
      return t < 0 ? am1 : s;
    };
    auto getb = [&](int t) -> int32_t { return __shfl(rb, t & 63); };  // b[j0 + t], t in [0, 63]
    // co-rank of local diagonal l + 1 inside the window: x in [max(0, l + 1 - 64), min(l + 1, 64)]
    const int dl = lane + 1;
    int lo = dl > 64 ? dl - 64 : 0, hi = dl < 64 ? dl : 64;
#pragma unroll
    for (int it = 0; it < 7; ++it) {
      const int mid = (lo + hi) >> 1;
      const bool go = lo < hi;
      const bool right = geta(mid) <= getb(dl - 1 - mid);  // (shuffles by every lane: uniform control)
      if (go) {
        if (right) lo = mid + 1;
        else hi = mid;
      }
    }
    const int xn = lo;              // x_{l+1}
    const int xu = __shfl_up(xn, 1);
    const int x = lane == 0 ? 0 : xu;  // x_l
    const bool froma = xn > x;
    const int ia = x, jb = lane - x;  // window indices of the candidates
    // (every shuffle by every lane: a ds_bpermute reads nothing useful from an inactive lane)
    const int32_t ga = geta(ia), gb = getb(jb), gprev = geta(ia - 1);
    const int32_t row = froma ? ga : gb;
    const bool valid = lane < len;
    // an a-output whose row equals the next b (gb) folds it in; a b-output equal to the a before
    // it is that pair's tail
    const bool pair = froma && gb == row;
    const bool tail = !froma && gprev == row;
    const bool head = valid && !tail;
    const uint64_t hm = __ballot(head);
    if constexpr (WRITE) {
      if (head) {
        const int64_t q = out + __popcll(hm & ((1ull << lane) - 1ull));
        val_t v;
        if (froma) {
          v = av[i0 + ia];
          if (pair) v = SR::add(v, bv[j0 + jb]);
        } else {
          v = bv[j0 + jb];
        }
        Cir[q] = row;
        reinterpret_cast<val_t*>(Cnum)[q] = v;
      }
    }
    out += __popcll(hm);
    heads += __popcll(hm);
    // advance by the co-rank of diagonal len
    const int xlen = __shfl(xn, len - 1);
    i0 += xlen;
    j0 += len - xlen;
  }
  if constexpr (!WRITE) {
    if (lane == 0) cnt[k] = heads;
  }
}

}  // namespace cbh
