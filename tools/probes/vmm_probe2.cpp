// Probe 2: (a) within one reservation, is physical memory freed by unmap+release reused when other
// offsets of the same reservation are mapped? (b) per-chunk reservations at address hints: honoured,
// and is memory returned by hipMemAddressFree of one chunk's reservation?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
static double freegb() {
  size_t f = 0, t = 0;
  hipMemGetInfo(&f, &t);
  return f / 1e9;
}
int main() {
  hipSetDevice(0);
  hipFree(nullptr);
  hipMemAllocationProp prop;
  std::memset(&prop, 0, sizeof(prop));
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemAccessDesc acc;
  std::memset(&acc, 0, sizeof(acc));
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  const size_t C = size_t(256) << 20, N = 32;
  auto map = [&](char* at, hipMemGenericAllocationHandle_t* h) {
    hipError_t e1 = hipMemCreate(h, C, &prop, 0), e2 = hipMemMap(at, C, 0, *h, 0), e3 = hipMemSetAccess(at, C, &acc, 1);
    return (int)e1 * 10000 + (int)e2 * 100 + (int)e3;
  };
  // (a)
  void* va = nullptr;
  hipMemAddressReserve(&va, C * N * 2, C, nullptr, 0);
  std::vector<hipMemGenericAllocationHandle_t> h(2 * N);
  std::printf("(a) start %.3f\n", freegb());
  for (size_t c = 0; c < N; ++c) map((char*)va + c * C, &h[c]);
  std::printf("(a) mapped [0,N) %.3f\n", freegb());
  for (size_t c = 0; c < N; ++c) {
    hipMemUnmap((char*)va + c * C, C);
    hipMemRelease(h[c]);
  }
  std::printf("(a) unmapped [0,N) %.3f\n", freegb());
  int bad = 0;
  for (size_t c = N; c < 2 * N; ++c) bad |= map((char*)va + c * C, &h[c]);
  std::printf("(a) mapped [N,2N) %.3f (err %d)\n", freegb(), bad);
  for (size_t c = N; c < 2 * N; ++c) {
    hipMemUnmap((char*)va + c * C, C);
    hipMemRelease(h[c]);
  }
  hipMemAddressFree(va, C * N * 2);
  std::printf("(a) address freed %.3f\n", freegb());
  // (b)
  void* win = nullptr;
  hipMemAddressReserve(&win, C * N, C, nullptr, 0);
  hipMemAddressFree(win, C * N);
  std::vector<void*> r(N, nullptr);
  int honoured = 0;
  for (size_t c = 0; c < N; ++c) {
    char* hint = (char*)win + c * C;
    hipError_t e = hipMemAddressReserve(&r[c], C, C, hint, 0);
    honoured += (e == hipSuccess && r[c] == hint);
    bad = map((char*)r[c], &h[c]);
    if (bad) std::printf("(b) chunk %zu map err %d\n", c, bad);
  }
  std::printf("(b) %d of %zu hints honoured, mapped %.3f\n", honoured, N, freegb());
  hipMemset(win, 3, C * N);
  hipError_t es = hipDeviceSynchronize();
  std::printf("(b) memset across chunk reservations: %d\n", (int)es);
  for (size_t c = 0; c < N / 2; ++c) {
    hipMemUnmap(r[c], C);
    hipMemRelease(h[c]);
    hipMemAddressFree(r[c], C);
  }
  std::printf("(b) half unmapped + reservations freed %.3f\n", freegb());
  for (size_t c = 0; c < N / 2; ++c) {
    char* hint = (char*)win + c * C;
    hipError_t e = hipMemAddressReserve(&r[c], C, C, hint, 0);
    if (e != hipSuccess || r[c] != hint) std::printf("(b) re-reserve chunk %zu: %d %p vs %p\n", c, (int)e, r[c], hint);
    map((char*)r[c], &h[c]);
  }
  std::printf("(b) re-mapped half %.3f\n", freegb());
  for (size_t c = 0; c < N; ++c) {
    hipMemUnmap(r[c], C);
    hipMemRelease(h[c]);
    hipMemAddressFree(r[c], C);
  }
  std::printf("(b) all freed %.3f\n", freegb());
  return 0;
}
