#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>
int main() {
  auto t0 = std::chrono::steady_clock::now();
  hipSetDevice(0);
  auto t1 = std::chrono::steady_clock::now();
  hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  void* p; hipMalloc(&p, 1 << 20);
  auto t2 = std::chrono::steady_clock::now();
  hipMalloc(&p, 16ull << 30);
  auto t3 = std::chrono::steady_clock::now();
  printf("{\"set_device_s\": %.4f, \"stream_small_malloc_s\": %.4f, \"malloc_16GB_s\": %.4f}\n",
         std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count(),
         std::chrono::duration<double>(t3 - t2).count());
  return 0;
}
