// Time hipMalloc + first touch for large scratch sizes (design data for the
// posterior scratch budget): ./alloc_probe GB...
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
__global__ void touch(char* p, size_t n) {
  for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4096; i < n; i += (size_t)gridDim.x * blockDim.x * 4096) p[i] = 1;
}
int main(int argc, char** argv) {
  using clk = std::chrono::steady_clock;
  hipFree(0);
  for (int a = 1; a < argc; a++) {
    const size_t gb = strtoull(argv[a], 0, 10);
    const size_t n = gb << 30;
    char* p = nullptr;
    auto t0 = clk::now();
    hipError_t e = hipMalloc(&p, n);
    auto t1 = clk::now();
    touch<<<4096, 256>>>(p, n);
    hipDeviceSynchronize();
    auto t2 = clk::now();
    printf("%zu GB: malloc %s %.3f s, touch %.3f s\n", gb, hipGetErrorString(e),
           std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count());
    fflush(stdout);
  }
  return 0;
}
