// pmc_calib.hip -- known-byte read kernels that calibrate rocprofv3's FETCH_SIZE on gfx950 for the
// access widths the task kernels use. MI355X_MICROARCH.md §HBM pins
// FETCH_SIZE = 1/2 of the bytes only for 16-B/lane coalesced streams; the SpGEMM kernels read
// 4-B row ids and 8-B values in short column segments and single-lane gathers.
//
// Every kernel reads a 4 GiB buffer (16x the 256 MiB Infinity Cache) so nothing is re-read
// on-die; each 128-B line that is touched is touched by exactly one wave instruction. Printed per
// kernel: the bytes of the whole 128-B lines touched (`line_bytes`) and the bytes the lanes
// asked for (`useful_bytes`). tools/pmc_calib.py divides FETCH_SIZE x 1024 by them.
//   stream16 / stream8 / stream4 : coalesced streams, 16 / 8 / 4 B per lane
//   seg256  : one wave reads one 256-B segment (4 B/lane), segments in permuted order
//   seg128x8: one wave reads 128-B runs of 8-B values (16 lanes each, 4 runs), permuted
//   gather8 / gather4 : every lane reads 8 / 4 B from its own line, lines in permuted order
// Build: hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/bin/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                              \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

constexpr uint64_t kBytes = uint64_t(4) << 30;
constexpr uint64_t kLines = kBytes / 128;
constexpr uint64_t kOdd = 0x9E3779B1ull;  // odd: i -> i * kOdd mod 2^k is a bijection

__device__ inline void sink_if(uint64_t acc, uint64_t* sink) {
  if (acc == 0x5DEECE66Dull) sink[0] = acc;  // never true for the zero-filled buffer: keeps the loads
}

template <class V>
__global__ void stream_kernel(const V* __restrict__ p, uint64_t n, uint64_t* sink) {
  uint64_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const V v = p[i];
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(V) / 4); ++k) acc += w[k];
  }
  sink_if(acc, sink);
}

// one wave per 256-B segment, segment s = (wave * kOdd) mod nseg
__global__ void seg256_kernel(const uint32_t* __restrict__ p, uint64_t nseg, uint64_t* sink) {
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 64;
  const int lane = threadIdx.x & 63;
  uint64_t acc = 0;
  for (uint64_t w = wave; w < nseg; w += (uint64_t)gridDim.x * blockDim.x / 64) {
    const uint64_t s = (w * kOdd) & (nseg - 1);
    acc += p[s * 64 + lane];
  }
  sink_if(acc, sink);
}

// 16 lanes read one 128-B line of 8-B values; the 4 quarter-waves read 4 permuted lines
__global__ void seg128x8_kernel(const uint64_t* __restrict__ p, uint64_t nlines, uint64_t* sink) {
  const uint64_t q = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 16;
  const int l = threadIdx.x & 15;
  uint64_t acc = 0;
  for (uint64_t w = q; w < nlines; w += (uint64_t)gridDim.x * blockDim.x / 16) {
    const uint64_t s = (w * kOdd) & (nlines - 1);
    acc += p[s * 16 + l];
  }
  sink_if(acc, sink);
}

// every lane reads one value from its own line: line = ((i0 + lane id) * kOdd) mod kLines, for
// `count` lane ids (distinct lines spread over the whole buffer)
template <class V>
__global__ void gather_kernel(const V* __restrict__ p, uint64_t i0, uint64_t count, uint64_t* sink) {
  uint64_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s = ((i0 + i) * kOdd) & (kLines - 1);
    acc += (uint64_t)p[s * (128 / sizeof(V))];
  }
  sink_if(acc, sink);
}

int main() {
  void* buf = nullptr;
  uint64_t* sink = nullptr;
  CK(hipMalloc(&buf, kBytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 0, kBytes));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid(256 * 64), block(256);
  // launch(0): warm-up (TLB); launch(1): timed. Both dispatches touch the same byte counts.
  auto run = [&](const char* name, auto launch, double line_bytes, double useful_bytes) {
    launch(0);
    CK(hipEventRecord(e0));
    launch(1);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("CALIB %s line_bytes=%.0f useful_bytes=%.0f ms=%.4f line_GBps=%.1f\n", name, line_bytes, useful_bytes,
                ms, line_bytes / (ms * 1e6));
  };
  const double B = (double)kBytes;
  run("stream16", [&](int) { stream_kernel<uint4><<<grid, block>>>((const uint4*)buf, kBytes / 16, sink); }, B, B);
  run("stream8", [&](int) { stream_kernel<uint2><<<grid, block>>>((const uint2*)buf, kBytes / 8, sink); }, B, B);
  run("stream4", [&](int) { stream_kernel<uint32_t><<<grid, block>>>((const uint32_t*)buf, kBytes / 4, sink); }, B, B);
  run("seg256", [&](int) { seg256_kernel<<<grid, block>>>((const uint32_t*)buf, kBytes / 256, sink); }, B, B);
  run("seg128x8", [&](int) { seg128x8_kernel<<<grid, block>>>((const uint64_t*)buf, kLines, sink); }, B, B);
  // gathers: 1/16 of the lines per dispatch, the warm-up and the timed dispatch on disjoint lines
  // (so the timed one cannot hit lines the warm-up left in the Infinity Cache)
  const uint64_t g = kLines / 16;
  run("gather8", [&](int k) { gather_kernel<uint64_t><<<grid, block>>>((const uint64_t*)buf, k * g, g, sink); },
      g * 128.0, g * 8.0);
  run("gather4", [&](int k) { gather_kernel<uint32_t><<<grid, block>>>((const uint32_t*)buf, (2 + k) * g, g, sink); },
      g * 128.0, g * 4.0);
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
