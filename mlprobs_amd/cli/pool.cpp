// pool.cpp -- see pool.h
#include "pool.h"

#include <stdlib.h>

#include <condition_variable>
#include <exception>
#include <mutex>
#include <thread>
#include <vector>

namespace mlpr {

namespace {

thread_local bool t_inside = false;   // in a worker, or the caller inside a region

struct Pool {
  std::vector<std::thread> workers;
  std::mutex m, run;
  std::condition_variable go, done;
  const std::function<void(int, int)>* job = nullptr;
  int T = 0, remaining = 0;
  uint64_t gen = 0;
  std::exception_ptr error;   // the first exception a worker's body threw (rethrown on the caller)

  void loop(int id) {
    t_inside = true;
    uint64_t seen = 0;
    std::unique_lock<std::mutex> l(m);
    for (;;) {
      go.wait(l, [&] { return gen != seen; });
      seen = gen;
      if (id >= T) continue;
      const std::function<void(int, int)>* j = job;
      const int TT = T;
      l.unlock();
      std::exception_ptr e;
      try {
        (*j)(id, TT);
      } catch (...) {
        e = std::current_exception();
      }
      l.lock();
      if (e && !error) error = e;
      if (--remaining == 0) done.notify_one();
    }
  }
};

Pool& pool() {
  static Pool* p = new Pool();   // never destroyed: idle workers stay blocked until the process exits
  return *p;
}

}  // namespace

int host_threads() {
  static const int n = [] {
    const char* e = getenv("OMP_NUM_THREADS");
    int t = e && atoi(e) > 0 ? atoi(e) : (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, 16));
  }();
  return n;
}

void parallel(int T, const std::function<void(int, int)>& body) {
  if (T <= 1 || t_inside) {
    body(0, 1);
    return;
  }
  Pool& p = pool();
  std::lock_guard<std::mutex> one_region(p.run);   // regions from several host threads take turns
  {
    std::lock_guard<std::mutex> l(p.m);
    while ((int)p.workers.size() < T - 1) {
      const int id = (int)p.workers.size() + 1;
      p.workers.emplace_back([&p, id] { p.loop(id); });
    }
    p.job = &body;
    p.T = T;
    p.remaining = T - 1;
    ++p.gen;
  }
  p.go.notify_all();
  // the caller's share: whatever it throws, the workers still run `body`
  // (which lives in the caller's frame), so wait for them before unwinding;
  // a worker's exception is rethrown here
  struct Inside {
    Inside() { t_inside = true; }
    ~Inside() { t_inside = false; }
  };
  std::exception_ptr mine;
  {
    Inside in;
    try {
      body(0, T);
    } catch (...) {
      mine = std::current_exception();
    }
  }
  std::unique_lock<std::mutex> l(p.m);
  p.done.wait(l, [&] { return p.remaining == 0; });
  std::exception_ptr theirs = p.error;
  p.error = nullptr;
  p.job = nullptr;
  l.unlock();
  if (mine) std::rethrow_exception(mine);
  if (theirs) std::rethrow_exception(theirs);
}

}  // namespace mlpr
