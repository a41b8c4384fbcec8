// pk_rate -- issue rate of packed f32 (v_pk_add_f32 / v_pk_mul_f32) against
// scalar f32 (v_add_f32 / v_mul_f32) on gfx950, at the occupancy of the
// posterior sweeps (6 waves per SIMD) and at one wave per SIMD.
//   tools/probe/pk_rate  -> one JSON line: lane-operations per second for each
// Each thread runs K independent add/mul chains (scalar) or K/2 packed chains
// of two (the same lane-operations), 4096 iterations, results kept live by one
// conditional store; K = 8 and K = 32 (enough independent work per wave for
// the issue rate, not the dependency latency, to bound it).  Built with -fno-slp-vectorize so the scalar form stays
// scalar.  DESIGN §9 (the v_pk A/B of round 4).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHK(x)                                                                        \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                          \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIter = 4096;

template <int K>
__global__ __launch_bounds__(256) void k_scalar(float a, float b, float* sink) {
  float x[K];
  for (int k = 0; k < K; ++k) x[k] = threadIdx.x * 1e-3f + k;
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = x[k] * a + b;   // -ffp-contract=off: v_mul + v_add
  }
  float s = 0;
  for (int k = 0; k < K; ++k) s += x[k];
  if (s == 12345.f) sink[threadIdx.x] = s;
}

template <int K>
__global__ __launch_bounds__(256) void k_packed(float a, float b, float* sink) {
  f2 x[K / 2];
  for (int k = 0; k < K / 2; ++k) x[k] = f2{threadIdx.x * 1e-3f + 2 * k, threadIdx.x * 1e-3f + 2 * k + 1};
  const f2 av = {a, a}, bv = {b, b};
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int k = 0; k < K / 2; ++k) x[k] = x[k] * av + bv;   // v_pk_mul_f32 + v_pk_add_f32
  }
  float s = 0;
  for (int k = 0; k < K / 2; ++k) s += x[k].x + x[k].y;
  if (s == 12345.f) sink[threadIdx.x] = s;
}

template <typename K>
static float time_ms(K kern, int blocks, float* sink) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, 0.999f, 1e-3f, sink);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, 0.999f, 1e-3f, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  float* sink;
  CHK(hipMalloc(&sink, 1024 * sizeof(float)));
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("{");
  const int waves_per_simd[2] = {6, 1};
  bool first = true;
  auto run = [&](auto ks, auto kp, int K) {
    for (int w = 0; w < 2; ++w) {
      // 256-thread blocks = 4 waves = one per SIMD
      const int blocks = cus * waves_per_simd[w];
      const double ops = (double)blocks * 256 * kIter * 2 * K;   // lane-ops: K chains x (mul + add)
      const double winst = ops / 64;                              // scalar wave-instructions
      const float ts = time_ms(ks, blocks, sink), tp = time_ms(kp, blocks, sink);
      printf("%s\"chains_%d_waves_per_simd_%d\": {\"scalar_ms\": %.4f, \"packed_ms\": %.4f, "
             "\"scalar_wave_instr_per_s\": %.4g, \"packed_wave_instr_per_s\": %.4g, \"packed_over_scalar_time\": %.3f}",
             first ? "" : ", ", K, waves_per_simd[w], ts, tp, winst / (ts * 1e-3), winst / 2 / (tp * 1e-3), tp / ts);
      first = false;
    }
  };
  run(k_scalar<8>, k_packed<8>, 8);
  run(k_scalar<32>, k_packed<32>, 32);
  printf("}\n");
  CHK(hipGetLastError());
  return 0;
}
