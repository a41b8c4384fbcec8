// VMM allocation timing probe: one contiguous virtual range backed by
// CHUNK_GB physical allocations (hipMemCreate + hipMemMap), first touched
// by hipMemset:  tools/probe/vmm_probe CHUNK_GB TOTAL_GB
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
int main(int argc, char** argv) {
  const double chunk = argc > 1 ? atof(argv[1]) : 16, total = argc > 2 ? atof(argv[2]) : 128;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto sec = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
  auto t0 = now();
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  printf("init %.3f s\n", sec(t0, now()));
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gran = 0;
  CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  const size_t cb = ((size_t)(chunk * (1ull << 30)) + gran - 1) / gran * gran;
  const int n = (int)((total + chunk - 1) / chunk);
  printf("granularity %zu, %d chunks of %zu\n", gran, n, cb);
  auto a = now();
  void* va = nullptr;
  CK(hipMemAddressReserve(&va, cb * n, 0, nullptr, 0));
  std::vector<hipMemGenericAllocationHandle_t> h(n);
  for (int k = 0; k < n; k++) {
    auto c0 = now();
    CK(hipMemCreate(&h[k], cb, &prop, 0));
    CK(hipMemMap((char*)va + (size_t)k * cb, cb, 0, h[k], 0));
    printf("chunk %d: create+map %.3f s\n", k, sec(c0, now()));
  }
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(va, cb * n, &acc, 1));
  auto m = now();
  CK(hipMemset(va, 0, cb * n));
  CK(hipDeviceSynchronize());
  printf("reserve+create+map+access %.3f s, memset all %.3f s\n", sec(a, m), sec(m, now()));
  for (int k = 0; k < n; k++) { CK(hipMemUnmap((char*)va + (size_t)k * cb, cb)); CK(hipMemRelease(h[k])); }
  CK(hipMemAddressFree(va, cb * n));
  return 0;
}
