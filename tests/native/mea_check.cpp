// MEA on SIMD lanes (cpnp::mea_path_simd) against the serial recurrence
// (cpnp::mea_path_serial): random posteriors, quantised ones (ties in every
// compare of ChooseBestOfThree), every shape from 1 x 1 up, both lane counts.
// Prints "ok <cases>" or the first mismatch.
#include <stdio.h>
#include <string.h>
#include <random>
#include <vector>

#include "msa_host.h"

int main(int argc, char** argv) {
  const int lanes = argc > 1 ? atoi(argv[1]) : 8;
  std::mt19937 rng(7);
  int cases = 0;
  for (int it = 0; it < 3000; it++) {
    const int L1 = 1 + (int)(rng() % (it < 1500 ? 40 : 300)), L2 = 1 + (int)(rng() % (it < 1500 ? 40 : 300));
    const int mode = it % 3;  // 0: uniform, 1: quantised (ties), 2: sparse (mostly 0)
    std::vector<float> P((size_t)(L1 + 1) * (L2 + 1), 0.f);
    for (auto& v : P) {
      const float u = (float)(rng() % 1000000) / 1e6f;
      v = mode == 0 ? u : mode == 1 ? (float)(rng() % 4) * 0.25f : (rng() % 10 == 0 ? u : 0.f);
    }
    float s0 = 0, s1 = 0;
    const std::string a = cpnp::mea_path_serial(L1, L2, P.data(), &s0);
    const std::string b = cpnp::mea_path_simd(L1, L2, P.data(), &s1, lanes);
    if (a != b || memcmp(&s0, &s1, 4) != 0) {
      printf("mismatch L1=%d L2=%d mode=%d score %.9g vs %.9g\n%s\n%s\n", L1, L2, mode, s0, s1, a.c_str(), b.c_str());
      return 1;
    }
    cases++;
  }
  printf("ok %d\n", cases);
  return 0;
}
