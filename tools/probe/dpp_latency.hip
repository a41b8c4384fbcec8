// Dependent-chain latency of one wave (one workgroup, nothing else on the
// device): cycles per step of v = max3(a, v, shift(v)) for the shift forms
// the MEA's skewed wavefront can use -- DPP wave_shr:1 (the kernel's),
// DPP row_shr:1 (within 16-lane rows), no shift -- and of the MEA step with
// a readlane insert.  tools/probe/dpp_latency -> one JSON line.
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int N = 4096;
template <int MODE>
__global__ __launch_bounds__(64) void k_chain(float* out, long long* cyc, float a) {
  float v = threadIdx.x * 1e-3f, ins = 0.5f;
  const long long t0 = clock64();
#pragma unroll 16
  for (int k = 0; k < N; ++k) {
    float s;
    if (MODE == 0) s = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(ins), __float_as_int(v), 0x138, 0xf, 0xf, false));
    else if (MODE == 1) s = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(ins), __float_as_int(v), 0x111, 0xf, 0xf, false));
    else if (MODE == 2) s = v;
    else s = __int_as_float(__builtin_amdgcn_update_dpp(__int_as_float(0) == 0 ? __float_as_int(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k & 63))) : 0,
                                                        __float_as_int(v), 0x138, 0xf, 0xf, false));
    v = fmaxf(fmaxf(a + ins, v), s);
    ins = s;
  }
  const long long t1 = clock64();
  out[threadIdx.x] = v;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  float* out;
  long long* cyc;
  if (hipMalloc(&out, 256) != hipSuccess || hipMalloc(&cyc, 8) != hipSuccess) return 1;
  const char* names[] = {"wave_shr", "row_shr", "none", "wave_shr+readlane"};
  printf("{");
  for (int m = 0; m < 4; ++m) {
    long long best = 1LL << 62;
    for (int rep = 0; rep < 5; ++rep) {
      if (m == 0) hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, out, cyc, 0.25f);
      if (m == 1) hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, out, cyc, 0.25f);
      if (m == 2) hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, out, cyc, 0.25f);
      if (m == 3) hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(64), 0, 0, out, cyc, 0.25f);
      long long c = 0;
      if (hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
      best = c < best ? c : best;
    }
    printf("%s\"%s\": %.1f", m ? ", " : "", names[m], (double)best / N);
  }
  printf(", \"unit\": \"clock64 cycles per step\"}\n");
  return 0;
}
