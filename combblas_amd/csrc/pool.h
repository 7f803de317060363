// Splitting block pool of the context allocator (large requests, see spgemm.hip's dalloc).
//
// Host-only bookkeeping over segments the caller maps (hipMalloc) and unmaps (hipFree): a request
// takes the best-fitting free block of any segment and splits off the rest; a freed block
// coalesces with the free neighbours of its own segment (never across segments, which may be
// adjacent in the address space); a segment whose blocks are all free can be handed back whole.
// No device calls here, so tests/test_pool_cpu.py drives it from a plain C++ program.
#pragma once

#include <algorithm>
#include <cstddef>
#include <iterator>
#include <map>
#include <set>
#include <utility>
#include <vector>

namespace cbh {

struct BlockPool {
  struct Seg {
    size_t size = 0, free_bytes = 0;
  };
  std::map<char*, Seg> segs;                      // by base address
  std::map<char*, std::pair<size_t, bool>> blk;   // every block: size, free
  std::set<std::pair<size_t, char*>> fr;          // free blocks by (size, address)
  size_t free_bytes = 0;                          // bytes of free blocks (all segments)

  bool owns(const void* p) const { return blk.count(const_cast<char*>(static_cast<const char*>(p))) != 0; }

  std::map<char*, Seg>::iterator seg_of(char* q) {
    auto it = segs.upper_bound(q);
    return --it;  // q lies in a block: some segment starts at or below it
  }

  // a freshly mapped segment of `size` bytes whose single block is handed out at once
  void add_live_segment(char* base, size_t size) {
    segs[base] = Seg{size, 0};
    blk[base] = {size, false};
  }

  // best-fitting free block of at least `size` bytes (split when larger); nullptr when none fits
  char* take(size_t size) {
    auto it = fr.lower_bound({size, nullptr});
    if (it == fr.end()) return nullptr;
    const size_t s = it->first;
    char* q = it->second;
    fr.erase(it);
    blk[q] = {size, false};
    if (s > size) {
      blk[q + size] = {s - size, true};
      fr.insert({s - size, q + size});
    }
    seg_of(q)->second.free_bytes -= size;
    free_bytes -= size;
    return q;
  }

  // returns block q (of `size` bytes, as handed out) to the pool
  void put(char* q, size_t size) {
    auto sg = seg_of(q);
    char* const sbase = sg->first;
    char* const send = sbase + sg->second.size;
    sg->second.free_bytes += size;
    free_bytes += size;
    auto it = blk.find(q);
    auto nx = std::next(it);
    if (nx != blk.end() && nx->first == q + size && nx->first < send && nx->second.second) {
      fr.erase({nx->second.first, nx->first});
      size += nx->second.first;
      blk.erase(nx);
    }
    if (it != blk.begin()) {
      auto pv = std::prev(it);
      if (pv->first >= sbase && pv->second.second && pv->first + pv->second.first == q) {
        fr.erase({pv->second.first, pv->first});
        size += pv->second.first;
        blk.erase(it);
        it = pv;
      }
    }
    it->second = {size, true};
    fr.insert({size, it->first});
  }

  // fully free segments, largest first
  std::vector<std::pair<size_t, char*>> whole_segments() const {
    std::vector<std::pair<size_t, char*>> w;
    for (auto& kv : segs)
      if (kv.second.free_bytes == kv.second.size) w.push_back({kv.second.size, kv.first});
    std::sort(w.rbegin(), w.rend());
    return w;
  }

  // forgets a fully free segment (the caller unmaps it); returns its size
  size_t drop_segment(char* base) {
    auto sg = segs.find(base);
    const size_t size = sg->second.size;
    fr.erase({size, base});
    blk.erase(base);
    free_bytes -= size;
    segs.erase(sg);
    return size;
  }
};

}  // namespace cbh
