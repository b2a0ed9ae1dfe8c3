// host_pool.h — the seam's host worker pool (commit.hip): host_threads() sizes a loop,
// parallel_ranges() forks it over persistent workers.  Header-only so tools/pool_probe.cpp can
// time the fork-join on a GPU box's host.
#pragma once
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>

// Worker count for host loops over `items` units of work (requests x signatures).
static unsigned host_threads(size_t items) {
  if (items < (1u << 16)) return 1;
  static const unsigned cap = [] {
    const char *v = getenv("TMED_HOST_THREADS");  // default 16: one GPU's share of a node's cores
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const unsigned want = v ? (unsigned)std::max(1, atoi(v)) : 16u;
    return std::min(want, hw);
  }();
  return cap;
}

// Persistent host workers: a seam call runs ~8 parallel phases per batch (a light-client call
// ~60), so the fork-join itself must cost little.  One region runs at a time (callers serialise
// on run_mu); the region's parts are claimed through ONE atomic word (generation | parts | next),
// so a worker can never take a part of a region it did not see published, and the region's job
// stays valid until its last part is done.  Workers spin on the word for a while after each
// region (the next phase of the same batch follows within microseconds) and then sleep on a
// condition variable.  The pool is started on first use and never torn down (its idle workers
// end with the process).  A call made from a worker runs serially.
namespace {
struct HostPool {
  using Job = std::function<void(unsigned)>;
  std::mutex run_mu;                 // one region at a time
  std::atomic<uint64_t> word{0};     // gen (24 bits) | parts (16) | next part (24)
  std::atomic<unsigned> done{0};     // parts finished in the current region
  const Job *job = nullptr;          // the current region's job (valid while a part is unfinished)
  std::exception_ptr err;            // the region's first exception, rethrown by run() after the join
  std::mutex err_mu;
  std::mutex m;
  std::condition_variable cv;
  static thread_local bool in_worker;
  static thread_local bool in_region;  // the caller while it runs parts of its own region
  // Polling before a worker sleeps: a short pause loop, then sched_yield (a worker that polls must not
  // take the CPU from the threads doing the work when the host has fewer cores than threads).
  static constexpr int kPause = 1000, kYield = 200;

  static uint64_t gen_of(uint64_t w) { return w >> 40; }
  static unsigned parts_of(uint64_t w) { return (unsigned)((w >> 24) & 0xffffu); }
  static unsigned next_of(uint64_t w) { return (unsigned)(w & 0xffffffu); }

  // Claim and run parts of the region published in `word` until none is left.
  void work() {
    for (;;) {
      uint64_t w = word.load(std::memory_order_acquire);
      if (next_of(w) >= parts_of(w)) return;
      if (!word.compare_exchange_weak(w, w + 1, std::memory_order_acq_rel)) continue;
      try {
        (*job)(next_of(w));  // the region cannot complete before this part: job is its own
      } catch (...) {        // a part that throws still counts as done: run() joins, then rethrows
        std::lock_guard<std::mutex> g(err_mu);
        if (!err) err = std::current_exception();
      }
      done.fetch_add(1, std::memory_order_release);
    }
  }
  explicit HostPool(unsigned n) {
    for (unsigned i = 0; i < n; i++)
      std::thread([this] {
        in_worker = true;
        uint64_t seen = 0;
        for (;;) {
          int spins = 0;
          while (gen_of(word.load(std::memory_order_acquire)) == seen) {
            if (++spins < kPause) {
              __builtin_ia32_pause();
              continue;
            }
            if (spins < kPause + kYield) {
              std::this_thread::yield();
              continue;
            }
            std::unique_lock<std::mutex> lk(m);
            cv.wait(lk, [&] { return gen_of(word.load(std::memory_order_acquire)) != seen; });
            break;
          }
          seen = gen_of(word.load(std::memory_order_acquire));
          work();
        }
      }).detach();
  }
  void run(unsigned parts, const Job &f) {
    std::lock_guard<std::mutex> lk(run_mu);
    job = &f;
    done.store(0, std::memory_order_relaxed);
    const uint64_t g = (gen_of(word.load(std::memory_order_relaxed)) + 1) & 0xffffffu;
    word.store((g << 40) | ((uint64_t)parts << 24), std::memory_order_release);
    {
      std::lock_guard<std::mutex> wk(m);  // sleeping workers re-check the word under m
    }
    cv.notify_all();
    in_region = true;
    work();  // never throws: parts' exceptions are caught and kept in err
    in_region = false;
    int spins = 0;
    while (done.load(std::memory_order_acquire) < parts)
      if (++spins < kPause) __builtin_ia32_pause();
      else std::this_thread::yield();
    std::exception_ptr e;
    {
      std::lock_guard<std::mutex> g(err_mu);
      std::swap(e, err);
    }
    if (e) std::rethrow_exception(e);  // every part has finished: no worker still reads the job
  }
  static HostPool &get() {
    static HostPool *p = new HostPool(std::max(1u, host_threads(~(size_t)0) - 1));
    return *p;
  }
};
thread_local bool HostPool::in_worker = false;
thread_local bool HostPool::in_region = false;
}  // namespace

// Tests (tmed_test_pool_jitter): each part of a region starts after a pseudo-random delay of up to
// this many microseconds, so a part that reads what another part of the same region writes sees
// it unwritten in some runs instead of almost never (0: off, the product default).
inline std::atomic<int> g_pool_jitter_us{0};
inline void pool_jitter(unsigned t) {
  const int us = g_pool_jitter_us.load(std::memory_order_relaxed);
  if (us <= 0) return;
  static std::atomic<uint64_t> ctr{0};
  uint64_t x = (ctr.fetch_add(1, std::memory_order_relaxed) + 1) * 0x9e3779b97f4a7c15ull ^ ((uint64_t)t << 32);
  x ^= x >> 31;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 29;
  std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(x % (uint64_t)us)));
}

// f(lo, hi, t) over nt contiguous parts of [0, n) (part t; each part runs exactly once, on some
// thread: per-part buffers are indexed by t).
template <class F>
static void parallel_ranges(size_t n, unsigned nt, F &&f) {
  if (nt <= 1 || n < 2 || HostPool::in_worker || HostPool::in_region) { f(0, n, 0u); return; }
  if (nt > n) nt = (unsigned)n;
  if (nt > 0xffffu) nt = 0xffffu;
  const HostPool::Job job = [&](unsigned t) {
    pool_jitter(t);
    f(n * t / nt, n * (t + 1) / nt, t);
  };
  HostPool::get().run(nt, job);
}
