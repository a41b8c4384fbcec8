// Allocation timing probe (tools/probe/alloc_chunks CHUNK_GB TOTAL_GB): hipMalloc of CHUNK_GB chunks until TOTAL_GB, each
// followed by a hipMemset, timed separately (fresh process).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
int main(int argc, char** argv) {
  const double chunk = argc > 1 ? atof(argv[1]) : 16, total = argc > 2 ? atof(argv[2]) : 128;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto t0 = now();
  if (hipSetDevice(0) != hipSuccess) return 1;
  hipFree(nullptr);
  printf("init %.3f s\n", std::chrono::duration<double>(now() - t0).count());
  std::vector<void*> ptrs;
  for (double done = 0; done < total; done += chunk) {
    const size_t b = (size_t)(chunk * (1ull << 30));
    void* p = nullptr;
    auto a = now();
    if (hipMalloc(&p, b) != hipSuccess) { printf("malloc failed at %.0f GB\n", done); break; }
    auto m = now();
    if (hipMemset(p, 0, b) != hipSuccess || hipDeviceSynchronize() != hipSuccess) { printf("memset failed\n"); break; }
    auto s = now();
    printf("chunk at %5.0f GB: malloc %.3f s memset %.3f s\n", done, std::chrono::duration<double>(m - a).count(),
           std::chrono::duration<double>(s - m).count());
    ptrs.push_back(p);
  }
  for (void* p : ptrs) hipFree(p);
  return 0;
}
