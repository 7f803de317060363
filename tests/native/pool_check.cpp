// Randomised check of cbh::BlockPool (combblas_amd/csrc/pool.h): segments are slices of one host
// arena placed back to back (so coalescing across a segment edge would be caught), requests of
// mixed sizes are taken / returned in random order, and after every step the bookkeeping must
// tile each segment exactly, keep no two adjacent free blocks, and agree with the live set.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <vector>

#include "../../combblas_amd/csrc/pool.h"

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAIL line %d: %s\n", __LINE__, #c);             \
      if (++fails > 5) std::exit(1);                               \
    }                                                              \
  } while (0)

static void invariants(cbh::BlockPool& P, const std::map<char*, size_t>& live) {
  size_t freeb = 0;
  for (auto& kv : P.segs) {
    char* b = kv.first;
    char* e = b + kv.second.size;
    size_t sf = 0;
    bool prev_free = false;
    char* at = b;
    for (auto it = P.blk.find(b); it != P.blk.end() && it->first < e; ++it) {
      CHECK(it->first == at);  // blocks tile the segment
      const bool f = it->second.second;
      CHECK(!(f && prev_free));  // free neighbours are always merged
      if (f) {
        sf += it->second.first;
        CHECK(P.fr.count({it->second.first, it->first}) == 1);
      } else {
        auto l = live.find(it->first);
        CHECK(l != live.end() && l->second == it->second.first);
      }
      prev_free = f;
      at += it->second.first;
    }
    CHECK(at == e);
    CHECK(sf == kv.second.free_bytes);
    freeb += sf;
  }
  CHECK(freeb == P.free_bytes);
  CHECK(P.fr.size() <= P.blk.size());
  size_t nfree = 0;
  for (auto& kv : P.blk) nfree += kv.second.second;
  CHECK(nfree == P.fr.size());
}

int main(int argc, char** argv) {
  const unsigned seed = argc > 1 ? (unsigned)std::atoi(argv[1]) : 1u;
  const int steps = argc > 2 ? std::atoi(argv[2]) : 20000;
  std::mt19937_64 rng(seed);
  const size_t Q = 64;  // quantum (the library's is 2 MiB; the logic is scale-free)
  std::vector<char> arena(Q * 1000000);
  size_t top = 0;  // next segment's offset: segments are adjacent in the address space
  cbh::BlockPool P;
  std::map<char*, size_t> live;
  size_t mapped = 0, unmapped = 0, reused = 0;
  for (int s = 0; s < steps; ++s) {
    const int op = (int)(rng() % 10);
    if (op < 6 || live.empty()) {
      const size_t size = Q * (1 + rng() % ((rng() % 4 == 0) ? 4000 : 60));
      char* q = P.take(size);
      if (q) {
        ++reused;
      } else {
        if (top + size > arena.size()) {  // out of "device" memory: give whole segments back
          for (auto& w : P.whole_segments()) P.drop_segment(w.second), ++unmapped;
          if (top + size > arena.size()) continue;
        }
        q = arena.data() + top;
        top += size;
        P.add_live_segment(q, size);
        ++mapped;
      }
      CHECK(live.count(q) == 0);
      // the block must not overlap any live block
      auto nx = live.lower_bound(q);
      if (nx != live.end()) CHECK(q + size <= nx->first);
      if (nx != live.begin()) {
        auto pv = std::prev(nx);
        CHECK(pv->first + pv->second <= q);
      }
      live[q] = size;
    } else {
      auto it = live.begin();
      std::advance(it, (long)(rng() % live.size()));
      P.put(it->first, it->second);
      live.erase(it);
    }
    if (s % 97 == 0 || s == steps - 1) invariants(P, live);
    if (fails) break;
  }
  for (auto& kv : live) P.put(kv.first, kv.second);
  live.clear();
  invariants(P, live);
  const auto whole = P.whole_segments();
  CHECK(whole.size() == P.segs.size());  // everything returned: every segment is one free block
  CHECK(P.blk.size() == P.segs.size());
  for (auto& w : whole) P.drop_segment(w.second);
  CHECK(P.segs.empty() && P.blk.empty() && P.fr.empty() && P.free_bytes == 0);
  std::printf("seed %u: %d steps, %zu segments mapped, %zu dropped, %zu requests served from the pool, %s\n", seed,
              steps, mapped, unmapped, reused, fails ? "FAIL" : "ok");
  return fails ? 1 : 0;
}
