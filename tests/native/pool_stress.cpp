// pool_stress.cpp — TEST-ONLY stress of the seam's host worker pool
// (tendermint-fork_amd/csrc/host_pool.h), built with ThreadSanitizer by
// tests/test_native_sanitizers.py.  Several caller threads run regions back to back (the pool
// serialises them), with random part counts, nested calls from inside a part (run serially),
// and parts that throw (the region still joins, then run() rethrows on the caller).  Every part
// of every region must run exactly once and every region's sum must come out exact.
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <random>
#include <stdexcept>
#include <thread>
#include <vector>

#include "host_pool.h"

int main(int argc, char **argv) {
  const int callers = argc > 1 ? atoi(argv[1]) : 4;
  const int regions = argc > 2 ? atoi(argv[2]) : 3000;
  setenv("TMED_HOST_THREADS", "8", 1);
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int c = 0; c < callers; c++)
    th.emplace_back([&, c] {
      std::mt19937 rng(1234u + c);
      for (int r = 0; r < regions; r++) {
        const size_t n = 1 + rng() % 5000;
        const unsigned nt = 1 + rng() % 12;
        const bool thrower = rng() % 17 == 0;
        std::vector<unsigned> hits(nt, 0);  // per-part slots (each part runs once, on some thread)
        std::vector<long long> sums(nt, 0);
        bool threw = false;
        try {
          parallel_ranges(n, nt, [&](size_t lo, size_t hi, unsigned t) {
            hits[t]++;
            long long s = 0;
            for (size_t i = lo; i < hi; i++) s += (long long)i;
            if (hi - lo > 8 && t == 1) {  // a nested call (from a worker or the caller) runs serially
              long long inner = 0;
              parallel_ranges(hi - lo, 4, [&](size_t a, size_t b, unsigned) {
                for (size_t i = a; i < b; i++) inner += 1;
              });
              if (inner != (long long)(hi - lo)) bad++;
            }
            sums[t] = s;
            if (thrower && t == 0) throw std::runtime_error("part failed");
          });
        } catch (const std::runtime_error &) {
          threw = true;
        }
        const unsigned parts = (nt > n ? (unsigned)n : nt);
        long long total = 0;
        for (unsigned t = 0; t < nt; t++) {
          if (t < parts && hits[t] != 1) bad++;
          if (t >= parts && hits[t] != 0) bad++;
          total += sums[t];
        }
        if (thrower != threw) bad++;
        if (!thrower && total != (long long)n * (long long)(n - 1) / 2) bad++;
      }
    });
  for (auto &t : th) t.join();
  printf("pool_stress callers %d regions %d: %d bad\n", callers, regions, bad.load());
  return bad.load() ? 1 : 0;
}
