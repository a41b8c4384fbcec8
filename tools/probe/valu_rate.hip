// valu_rate -- chip-wide VALU issue rate on gfx950 by instruction kind and
// waves per SIMD (the VALU peak that DESIGN §4 and bench.py's valu_issue
// divide by).  Each wave runs 32 independent chains of one instruction (inline
// asm, so nothing is folded or reordered), 4096 iterations; blocks of 256
// threads (one wave per SIMD), cus * W blocks for W waves per SIMD; 3 timed
// launches after one warm-up.  Prints one JSON line: per instruction kind and
// W, wave-instructions per second and cycles per wave-instruction per SIMD at
// the measured clock (hipDeviceAttributeClockRate, the boost clock; under load
// the clock may be lower, so cycles are an upper bound on the SIMD's cost).
//   tools/probe/valu_rate   (build: hipcc --offload-arch=gfx950 -O3)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                               \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
      return 1;                                                              \
    }                                                                        \
  } while (0)

constexpr int kChains = 32;
constexpr int kIter = 4096;

#define OP2(ins) asm volatile(ins " %0, %1, %0" : "+v"(x[k]) : "v"(a))
#define OP3(ins) asm volatile(ins " %0, %1, %2, %0" : "+v"(x[k]) : "v"(a), "v"(b))

template <int KIND>
__global__ __launch_bounds__(256) void k_rate(uint32_t a, uint32_t b, uint32_t* sink) {
  uint32_t x[kChains];
  const uint64_t m = 0x5555555555555555ull ^ (uint64_t)a;
#pragma unroll
  for (int k = 0; k < kChains; ++k) x[k] = threadIdx.x + k;
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int k = 0; k < kChains; ++k) {
      if constexpr (KIND == 0) OP2("v_add_f32");
      if constexpr (KIND == 1) OP3("v_fma_f32");
      if constexpr (KIND == 2) OP2("v_mul_f32");
      if constexpr (KIND == 3) OP2("v_add_u32");
      if constexpr (KIND == 4) OP2("v_and_b32");
      if constexpr (KIND == 5) OP2("v_bcnt_u32_b32");
      if constexpr (KIND == 6) OP3("v_lshl_add_u32");
      if constexpr (KIND == 7) OP3("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x40 ;");
      if constexpr (KIND == 8) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 bound_ctrl:0" : "+v"(x[k]) : "v"(a));
      if constexpr (KIND == 9) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[k]) : "v"(a));
      if constexpr (KIND == 10) asm volatile("v_add_f32 %0, %1, %0" : "+v"(x[k]) : "s"(a));     // SGPR operand
      if constexpr (KIND == 11) asm volatile("v_add_f32 %0, 0x3f7ff000, %0" : "+v"(x[k]));      // literal operand
      if constexpr (KIND == 12) asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(x[k]));             // inline constant
      if constexpr (KIND == 13) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(x[k]) : "v"(a), "s"(m));  // SGPR-pair mask
      if constexpr (KIND == 14) asm volatile("v_max_f32 %0, %1, %0" : "+v"(x[k]) : "v"(a));
      if constexpr (KIND == 15) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(x[k]));
      if constexpr (KIND == 16) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[k]) : "v"(a), "s"(b));  // one SGPR operand
      if constexpr (KIND == 17) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(x[k]) : "s"(a));     // SGPR operand
      if constexpr (KIND == 18) OP2("v_lshlrev_b32");
      if constexpr (KIND == 19) OP2("v_sub_f32");
      if constexpr (KIND == 20) OP2("v_min_f32");
      if constexpr (KIND == 21) OP2("v_mov_b32 %0, %1 ;");
      if constexpr (KIND == 22) OP3("v_mad_u32_u24");
      if constexpr (KIND == 23) OP3("v_add3_u32");
      if constexpr (KIND == 24) asm volatile("v_cmp_le_f32 vcc, %1, %0\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[k]) : "v"(a) : "vcc");  // pair
      if constexpr (KIND == 25) asm volatile("v_cmp_le_f32 vcc, %1, %0" : : "v"(x[k]), "v"(a) : "vcc");
      if constexpr (KIND == 26) OP2("v_max_u32");
      if constexpr (KIND == 27) OP2("v_xor_b32");
      if constexpr (KIND == 28) OP3("v_lshl_or_b32");
      if constexpr (KIND == 29) asm volatile("v_max3_f32 %0, %1, %2, %0" : "+v"(x[k]) : "v"(a), "v"(b));
      if constexpr (KIND == 30) asm volatile("v_add_co_u32_e32 %0, vcc, %1, %0" : "+v"(x[k]) : "v"(a) : "vcc");  // carry out to VCC
      if constexpr (KIND == 31) asm volatile("v_sub_co_u32_e32 %0, vcc, %0, %1" : "+v"(x[k]) : "v"(a) : "vcc");
      if constexpr (KIND == 32) {  // carry out to an SGPR pair
        uint64_t c_;
        asm volatile("v_add_co_u32_e64 %0, %1, %2, %0" : "+v"(x[k]), "=s"(c_) : "v"(a));
      }
      if constexpr (KIND == 33) OP2("v_mul_u32_u24");
      if constexpr (KIND == 34) asm volatile("v_cmp_ne_u32_e32 vcc, %1, %0" : : "v"(x[k]), "v"(a) : "vcc");
      if constexpr (KIND == 35) OP2("v_lshlrev_b16");
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kChains; ++k) s ^= x[k];
  if (s == 0x12345678u) sink[threadIdx.x] = s;
}

// 64-bit chains: x[k] a register pair
template <int KIND>
__global__ __launch_bounds__(256) void k_rate64(double a, double b, double* sink) {
  double x[kChains / 2];
#pragma unroll
  for (int k = 0; k < kChains / 2; ++k) x[k] = threadIdx.x + k;
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int k = 0; k < kChains / 2; ++k) {
      if constexpr (KIND == 0) asm volatile("v_add_f64 %0, %1, %0" : "+v"(x[k]) : "v"(a));
      if constexpr (KIND == 1) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(x[k]) : "v"(a), "v"(b));
      if constexpr (KIND == 2) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(x[k]) : "v"(a));
      if constexpr (KIND == 3) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(x[k]) : "v"(a), "v"(b));
    }
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < kChains / 2; ++k) s += x[k];
  if (s == 12345.0) sink[threadIdx.x] = s;
}

template <typename F>
static float time_ms(F launch) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  launch();
  hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms / 3;
}

int main() {
  void* sink;
  CHK(hipMalloc(&sink, 1024 * sizeof(double)));
  int cus = 0, khz = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, 0));
  const double hz = khz * 1e3;
  printf("{\"cus\": %d, \"clock_hz\": %.4g", cus, hz);
  const char* names32[] = {"v_add_f32", "v_fma_f32", "v_mul_f32", "v_add_u32", "v_and_b32",
                           "v_bcnt_u32_b32", "v_lshl_add_u32", "v_bitop3_b32", "v_mov_b32_dpp", "v_cndmask_b32_vcc",
                           "v_add_f32_sgpr", "v_add_f32_literal", "v_add_f32_inline", "v_cndmask_b32_sgpr", "v_max_f32",
                           "v_cvt_i32_f32", "v_fma_f32_sgpr", "v_mul_f32_sgpr",
                           "v_lshlrev_b32", "v_sub_f32", "v_min_f32", "v_mov_b32", "v_mad_u32_u24", "v_add3_u32",
                           "v_cmp_e32+v_cndmask_vcc_pair", "v_cmp_le_f32_vcc", "v_max_u32", "v_xor_b32", "v_lshl_or_b32",
                           "v_max3_f32", "v_add_co_u32_vcc", "v_sub_co_u32_vcc", "v_add_co_u32_sgpr_pair",
                           "v_mul_u32_u24", "v_cmp_ne_u32_vcc", "v_lshlrev_b16"};
  const char* names64[] = {"v_add_f64", "v_fma_f64", "v_pk_add_f32", "v_pk_fma_f32"};
  const int waves[] = {1, 2, 4, 8};
  auto report = [&](const char* name, int W, double chains, float ms) {
    const double blocks = (double)cus * W;
    const double winst = blocks * 4 * chains * kIter;  // 4 waves per block
    const double rate = winst / (ms * 1e-3);
    const double cyc = (double)cus * 4 * hz / rate;     // SIMD-cycles per wave-instruction
    printf(", \"%s_w%d\": {\"ms\": %.4f, \"wave_instr_per_s\": %.4g, \"simd_cycles_per_instr\": %.2f}", name, W, ms,
           rate, cyc);
  };
  auto run32 = [&](auto kern, const char* name) {
    for (int W : waves) {
      const int blocks = cus * W;
      const float ms = time_ms([&] {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, 0x3f7ff000u, 0x3a800000u, (uint32_t*)sink);
      });
      report(name, W, kChains, ms);
    }
  };
  auto run64 = [&](auto kern, const char* name) {
    for (int W : waves) {
      const int blocks = cus * W;
      const float ms = time_ms([&] {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, 0.999, 1e-3, (double*)sink);
      });
      report(name, W, kChains / 2, ms);
    }
  };
  run32(k_rate<0>, names32[0]);
  run32(k_rate<1>, names32[1]);
  run32(k_rate<2>, names32[2]);
  run32(k_rate<3>, names32[3]);
  run32(k_rate<4>, names32[4]);
  run32(k_rate<5>, names32[5]);
  run32(k_rate<6>, names32[6]);
  run32(k_rate<7>, names32[7]);
  run32(k_rate<8>, names32[8]);
  run32(k_rate<9>, names32[9]);
  run32(k_rate<10>, names32[10]);
  run32(k_rate<11>, names32[11]);
  run32(k_rate<12>, names32[12]);
  run32(k_rate<13>, names32[13]);
  run32(k_rate<14>, names32[14]);
  run32(k_rate<15>, names32[15]);
  run32(k_rate<16>, names32[16]);
  run32(k_rate<17>, names32[17]);
  if (getenv("VALU_RATE_MORE")) {
    run32(k_rate<18>, names32[18]);
    run32(k_rate<19>, names32[19]);
    run32(k_rate<20>, names32[20]);
    run32(k_rate<21>, names32[21]);
    run32(k_rate<22>, names32[22]);
    run32(k_rate<23>, names32[23]);
    run32(k_rate<24>, names32[24]);
    run32(k_rate<25>, names32[25]);
    run32(k_rate<26>, names32[26]);
    run32(k_rate<27>, names32[27]);
    run32(k_rate<28>, names32[28]);
    run32(k_rate<29>, names32[29]);
  }
  if (getenv("VALU_RATE_CARRY")) {
    run32(k_rate<30>, names32[30]);
    run32(k_rate<31>, names32[31]);
    run32(k_rate<32>, names32[32]);
    run32(k_rate<33>, names32[33]);
    run32(k_rate<34>, names32[34]);
    run32(k_rate<35>, names32[35]);
    run32(k_rate<3>, names32[3]);
    run32(k_rate<5>, names32[5]);
  }
  run64(k_rate64<0>, names64[0]);
  run64(k_rate64<1>, names64[1]);
  run64(k_rate64<2>, names64[2]);
  run64(k_rate64<3>, names64[3]);
  printf("}\n");
  CHK(hipGetLastError());
  return 0;
}
