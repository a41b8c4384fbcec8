// hbm_stream -- the on-box HBM bandwidth the rooflines divide by (BASELINE.md
// section 4: re-measure the vendor 8 TB/s with a stream kernel).
//   tools/probe/hbm_stream [GiB] [reps]  -> one JSON line on stdout
// Three kernels over a buffer far larger than the 8 XCDs' L2 + the 256 MB
// MALL: read (16-byte loads, per-thread sums kept live by one conditional
// store), write (16-byte stores) and copy (read + write).  Grid-stride
// loops, 8 workgroups per CU resident; each kernel is timed with HIP events
// over `reps` launches after one warm-up, and the best rate is reported
// (bytes moved / time, 1 GB = 1e9 B).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                        \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                          \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_read(const v4f* __restrict__ a, size_t n, float* sink) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const v4f v = __builtin_nontemporal_load(a + i);
    s += v.x + v.y + v.z + v.w;
  }
  if (s == -1.2345f) sink[0] = s;  // never true for the zero-filled buffer; keeps the loads
}

__global__ __launch_bounds__(256) void k_write(v4f* __restrict__ a, size_t n) {
  const v4f z = {1.f, 2.f, 3.f, 4.f};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(z, a + i);
}

__global__ __launch_bounds__(256) void k_copy(const v4f* __restrict__ a, v4f* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 8.0;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const size_t bytes = (size_t)(gib * (1ull << 30)) & ~(size_t)4095;
  const size_t n = bytes / sizeof(v4f);
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  v4f *a = nullptr, *b = nullptr;
  float* sink = nullptr;
  CHK(hipMalloc(&a, bytes));
  CHK(hipMalloc(&b, bytes));
  CHK(hipMalloc(&sink, 4));
  CHK(hipMemset(a, 0, bytes));
  CHK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const dim3 grid(cus * 8), block(256);
  double best[3] = {0, 0, 0};
  for (int k = 0; k < 3; k++) {
    for (int r = -1; r < reps; r++) {
      CHK(hipEventRecord(e0, 0));
      if (k == 0) hipLaunchKernelGGL(k_read, grid, block, 0, 0, a, n, sink);
      if (k == 1) hipLaunchKernelGGL(k_write, grid, block, 0, 0, b, n);
      if (k == 2) hipLaunchKernelGGL(k_copy, grid, block, 0, 0, a, b, n);
      CHK(hipGetLastError());
      CHK(hipEventRecord(e1, 0));
      CHK(hipEventSynchronize(e1));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      const double moved = (double)bytes * (k == 2 ? 2 : 1);
      if (r >= 0 && ms > 0) best[k] = fmax(best[k], moved / (ms * 1e-3) / 1e9);
    }
  }
  printf("{\"buffer_gib\": %.2f, \"reps\": %d, \"cus\": %d, \"read_gbps\": %.1f, \"write_gbps\": %.1f, "
         "\"copy_gbps\": %.1f}\n",
         gib, reps, cus, best[0], best[1], best[2]);
  CHK(hipFree(a));
  CHK(hipFree(b));
  CHK(hipFree(sink));
  return 0;
}
