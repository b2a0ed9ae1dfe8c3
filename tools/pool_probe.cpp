// pool_probe — fork-join cost of the seam's host pool (csrc/host_pool.h) on this host.
// Runs back-to-back regions of 16 parts with (a) no work, (b) ~20 us of work per part, and
// (c) the same after the caller idles 100 us / 1 ms between regions (workers spinning, yielding
// or asleep, as between a batch's phases); prints one JSON line per case with the region's
// wall time and its overhead over the slowest part.
// Build: g++ -O2 -std=c++17 -pthread tools/pool_probe.cpp -o tools/pool_probe
#include <stdio.h>

#include <chrono>
#include <vector>

#include "../tendermint-fork_amd/csrc/host_pool.h"

using Clock = std::chrono::steady_clock;
static double us_since(Clock::time_point t) { return std::chrono::duration<double, std::micro>(Clock::now() - t).count(); }

static volatile double sink;
static void busy(double us) {
  const auto t = Clock::now();
  double x = 1.0;
  while (us_since(t) < us) x = x * 1.0000001 + 1e-9;
  sink = x;
}

int main() {
  const unsigned nt = host_threads(~(size_t)0);
  struct Case { const char *name; double work_us, gap_us; };
  const Case cases[] = {{"empty", 0, 0}, {"work20", 20, 0}, {"work20_gap100", 20, 100}, {"work20_gap1000", 20, 1000},
                        {"empty_gap100", 0, 100}, {"empty_gap1000", 0, 1000}};
  for (const Case &c : cases) {
    std::vector<double> wall, over;
    for (int it = 0; it < 400; it++) {
      if (c.gap_us > 0) busy(c.gap_us);
      std::vector<double> part(nt, 0.0);
      const auto t0 = Clock::now();
      parallel_ranges(nt * 64, nt, [&](size_t, size_t, unsigned t) {
        const auto tp = Clock::now();
        if (c.work_us > 0) busy(c.work_us);
        part[t] = us_since(tp);
      });
      const double w = us_since(t0);
      double mx = 0;
      for (double p : part) mx = std::max(mx, p);
      if (it >= 20) { wall.push_back(w); over.push_back(w - mx); }
    }
    std::sort(wall.begin(), wall.end());
    std::sort(over.begin(), over.end());
    auto pct = [](const std::vector<double> &v, double q) { return v[(size_t)(q * (v.size() - 1))]; };
    printf("{\"case\": \"%s\", \"threads\": %u, \"wall_us_p50\": %.1f, \"wall_us_p90\": %.1f, \"overhead_us_p50\": %.1f, "
           "\"overhead_us_p90\": %.1f, \"overhead_us_max\": %.1f}\n",
           c.name, nt, pct(wall, 0.5), pct(wall, 0.9), pct(over, 0.5), pct(over, 0.9), over.back());
  }
  return 0;
}
