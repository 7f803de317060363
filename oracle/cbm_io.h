// TEST INFRASTRUCTURE ONLY (oracle/). Never linked into the product library.
//
// "CBM1": a tiny binary DCSC container used to move matrices between the
// reference harness (oracle/_ref), the CPU restatement (oracle/) and the
// Python tests. Layout (little endian):
//   char magic[4] = "CBM1"; uint32 vtype (0=f64, 1=i64, 2=u8/bool);
//   int64 m, n, nnz, nzc;
//   int64 jc[nzc]; int64 cp[nzc+1]; int32 ir[nnz]; value[nnz] (8 B, or 1 B for vtype 2)
// The arrays mirror combblas::Dcsc {jc, cp, ir, numx} (include/CombBLAS/dcsc.h:124-130).
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace cbm {

enum VType : uint32_t { F64 = 0, I64 = 1, U8 = 2 };

struct Dcsc {
  uint32_t vtype = F64;
  int64_t m = 0, n = 0;
  std::vector<int64_t> jc, cp;  // cp.size() == jc.size()+1 (or 0 when empty)
  std::vector<int32_t> ir;
  std::vector<double> vf;   // vtype F64
  std::vector<int64_t> vi;  // vtype I64 / U8 (stored widened)
  int64_t nnz() const { return (int64_t)ir.size(); }
  int64_t nzc() const { return (int64_t)jc.size(); }
};

inline void write(const std::string& path, const Dcsc& d) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::fwrite("CBM1", 1, 4, f);
  std::fwrite(&d.vtype, 4, 1, f);
  int64_t hdr[4] = {d.m, d.n, d.nnz(), d.nzc()};
  std::fwrite(hdr, 8, 4, f);
  std::fwrite(d.jc.data(), 8, d.jc.size(), f);
  std::vector<int64_t> cp = d.cp;
  if (cp.empty()) cp.push_back(0);
  std::fwrite(cp.data(), 8, cp.size(), f);
  std::fwrite(d.ir.data(), 4, d.ir.size(), f);
  if (d.vtype == F64) {
    std::fwrite(d.vf.data(), 8, d.vf.size(), f);
  } else if (d.vtype == I64) {
    std::fwrite(d.vi.data(), 8, d.vi.size(), f);
  } else {
    std::vector<uint8_t> b(d.vi.size());
    for (size_t i = 0; i < b.size(); ++i) b[i] = d.vi[i] ? 1 : 0;
    std::fwrite(b.data(), 1, b.size(), f);
  }
  std::fclose(f);
}

inline Dcsc read(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  char mg[4];
  Dcsc d;
  int64_t hdr[4];
  if (std::fread(mg, 1, 4, f) != 4 || std::memcmp(mg, "CBM1", 4) != 0) throw std::runtime_error("bad magic");
  if (std::fread(&d.vtype, 4, 1, f) != 1 || std::fread(hdr, 8, 4, f) != 4) throw std::runtime_error("short header");
  d.m = hdr[0];
  d.n = hdr[1];
  int64_t nnz = hdr[2], nzc = hdr[3];
  d.jc.resize(nzc);
  d.cp.resize(nzc + 1);
  d.ir.resize(nnz);
  size_t ok = std::fread(d.jc.data(), 8, nzc, f) + std::fread(d.cp.data(), 8, nzc + 1, f) +
              std::fread(d.ir.data(), 4, nnz, f);
  if (ok != (size_t)(2 * nzc + 1 + nnz)) throw std::runtime_error("short body");
  if (d.vtype == F64) {
    d.vf.resize(nnz);
    if (std::fread(d.vf.data(), 8, nnz, f) != (size_t)nnz) throw std::runtime_error("short values");
  } else if (d.vtype == I64) {
    d.vi.resize(nnz);
    if (std::fread(d.vi.data(), 8, nnz, f) != (size_t)nnz) throw std::runtime_error("short values");
  } else {
    std::vector<uint8_t> b(nnz);
    if (std::fread(b.data(), 1, nnz, f) != (size_t)nnz) throw std::runtime_error("short values");
    d.vi.assign(b.begin(), b.end());
  }
  std::fclose(f);
  return d;
}

}  // namespace cbm
