// pool.h -- host threads for the CLIs' host stages (tree, progressive
// alignment, refinement, profile posteriors on the host).  A persistent pool
// whose idle workers block on a condition variable: with OpenMP's default
// spin-waiting, idle threads burned the CPU the serial stages between the
// short parallel regions needed (a 4-sequence quickprobs run took 1.1 s
// instead of 0.05 s), and libgomp reads OMP_WAIT_POLICY before main, so the
// drop-ins could not set it themselves.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <functional>

namespace mlpr {

// OMP_NUM_THREADS when set (the references' knob), else the hardware
// threads; at most 16
int host_threads();

// body(t, T) on T threads, the caller being t = 0; returns when all are
// done.  Nested calls (from inside a body) run body(0, 1) on the caller.
void parallel(int T, const std::function<void(int, int)>& body);

// iterations [0, n) in T contiguous chunks (schedule(static))
template <class F>
void parallel_for(int64_t n, int T, F f) {
  if (T <= 1 || n <= 1) {
    for (int64_t i = 0; i < n; i++) f(i);
    return;
  }
  T = (int)std::min<int64_t>(T, n);
  parallel(T, [&](int t, int TT) {
    const int64_t b = n * t / TT, e = n * (t + 1) / TT;
    for (int64_t i = b; i < e; i++) f(i);
  });
}

// iterations handed out one at a time (schedule(dynamic))
template <class F>
void parallel_for_dynamic(int64_t n, int T, F f) {
  if (T <= 1 || n <= 1) {
    for (int64_t i = 0; i < n; i++) f(i);
    return;
  }
  std::atomic<int64_t> next(0);
  parallel((int)std::min<int64_t>(T, n), [&](int, int) {
    for (int64_t i; (i = next.fetch_add(1)) < n;) f(i);
  });
}

}  // namespace mlpr
