// Probe: does hipMemUnmap + hipMemRelease of 256 MiB chunks give the memory back to the device?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
static void info(const char* w) {
  size_t f = 0, t = 0;
  hipMemGetInfo(&f, &t);
  std::printf("%-34s free %.3f GB\n", w, f / 1e9);
}
int main() {
  hipSetDevice(0);
  hipFree(nullptr);
  hipMemAllocationProp prop;
  std::memset(&prop, 0, sizeof(prop));
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t g = 0, gr = 0;
  hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityMinimum);
  hipMemGetAllocationGranularity(&gr, &prop, hipMemAllocationGranularityRecommended);
  std::printf("granularity min %zu recommended %zu\n", g, gr);
  const size_t C = size_t(256) << 20, N = 64;
  void* va = nullptr;
  hipError_t e = hipMemAddressReserve(&va, C * N * 2, C, nullptr, 0);
  std::printf("reserve %d %p\n", (int)e, va);
  info("start");
  std::vector<hipMemGenericAllocationHandle_t> h(N);
  hipMemAccessDesc acc;
  std::memset(&acc, 0, sizeof(acc));
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  for (size_t c = 0; c < N; ++c) {
    hipError_t e1 = hipMemCreate(&h[c], C, &prop, 0);
    hipError_t e2 = hipMemMap((char*)va + c * C, C, 0, h[c], 0);
    hipError_t e3 = hipMemSetAccess((char*)va + c * C, C, &acc, 1);
    if (e1 || e2 || e3) std::printf("chunk %zu: create %d map %d access %d\n", c, (int)e1, (int)e2, (int)e3);
  }
  info("mapped 16 GiB");
  hipMemset(va, 1, C * N);
  hipDeviceSynchronize();
  info("touched");
  for (size_t c = 0; c < N / 2; ++c) {
    hipError_t e1 = hipMemUnmap((char*)va + c * C, C);
    hipError_t e2 = hipMemRelease(h[c]);
    if (e1 || e2) std::printf("chunk %zu: unmap %d release %d\n", c, (int)e1, (int)e2);
  }
  info("unmapped+released half");
  hipDeviceSynchronize();
  info("after sync");
  // re-map the same addresses with new handles
  for (size_t c = 0; c < N / 2; ++c) {
    hipError_t e1 = hipMemCreate(&h[c], C, &prop, 0);
    hipError_t e2 = hipMemMap((char*)va + c * C, C, 0, h[c], 0);
    hipError_t e3 = hipMemSetAccess((char*)va + c * C, C, &acc, 1);
    if (e1 || e2 || e3) std::printf("remap chunk %zu: create %d map %d access %d\n", c, (int)e1, (int)e2, (int)e3);
  }
  info("remapped half");
  // release the handle first, then unmap (handle freed when the mapping goes)
  for (size_t c = 0; c < N; ++c) {
    hipError_t e2 = hipMemRelease(h[c]);
    hipError_t e1 = hipMemUnmap((char*)va + c * C, C);
    if (e1 || e2) std::printf("chunk %zu: release %d unmap %d\n", c, (int)e2, (int)e1);
  }
  info("released+unmapped all");
  e = hipMemAddressFree(va, C * N * 2);
  std::printf("address free %d\n", (int)e);
  info("after address free");
  return 0;
}
