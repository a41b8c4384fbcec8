// Background-allocation probe (tools/probe/alloc_bg BASE_GB BG_GB): does a
// hipMalloc that waits for the driver (a process that follows a large
// release) block the other thread's launches and synchronisations?  The main
// thread holds BASE_GB and runs 64 MB hipMemsetAsync + hipStreamSynchronize
// rounds while a second thread allocates BG_GB; reports the background
// allocation's time and the main thread's slowest round during it.
// tools/probe/alloc_bg BASE_GB BG_GB exit: returns from main 0.1 s after
// starting the background allocation (thread detached; the caller times the
// process: does exit wait for the allocation?); ... _exit: the same with _exit(0).
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <unistd.h>
#include <cstring>
int main(int argc, char** argv) {
  const double base = argc > 1 ? atof(argv[1]) : 16, bg = argc > 2 ? atof(argv[2]) : 48;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto sec = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
  auto t0 = now();
  if (hipSetDevice(0) != hipSuccess) return 1;
  hipFree(nullptr);
  printf("init %.3f s\n", sec(t0, now()));
  void* pb = nullptr;
  auto a = now();
  if (hipMalloc(&pb, (size_t)(base * (1ull << 30))) != hipSuccess) { printf("base malloc failed\n"); return 1; }
  printf("base %.0f GB malloc %.3f s\n", base, sec(a, now()));
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  std::atomic<int> done{0};
  double bg_s = 0;
  void* pg = nullptr;
  auto tb = now();
  std::thread th([&] {
    hipSetDevice(0);
    auto s = now();
    const hipError_t e = hipMalloc(&pg, (size_t)(bg * (1ull << 30)));
    bg_s = sec(s, now());
    if (e != hipSuccess) printf("background malloc failed\n");
    done = 1;
  });
  if (argc > 3) {
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    printf("leaving main after %.3f s (background done: %d)\n", sec(tb, now()), (int)done);
    fflush(stdout);
    th.detach();
    if (!strcmp(argv[3], "_exit")) _exit(0);
    return 0;
  }
  int rounds = 0;
  double worst = 0, total = 0;
  for (;;) {
    auto r = now();
    hipMemsetAsync(pb, rounds & 255, 64u << 20, st);
    hipStreamSynchronize(st);
    const double d = sec(r, now());
    worst = d > worst ? d : worst;
    total += d;
    ++rounds;
    if (done || sec(tb, now()) > 20) break;
  }
  th.join();
  printf("background %.0f GB malloc %.3f s; main thread meanwhile %d rounds, slowest %.4f s, mean %.5f s\n", bg, bg_s,
         rounds, worst, total / rounds);
  if (pg) hipFree(pg);
  hipFree(pb);
  return 0;
}
