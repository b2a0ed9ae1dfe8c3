// keycache_fuzz.cpp — TEST-ONLY randomized check of the seam's key-set cache policy
// (tendermint-fork_amd/csrc/keycache.h) over a host stand-in for the device pool, built with
// AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_native_sanitizers.py.  Calls are
// emulated as the seam makes them (commit.hip keycache_resolve): pin, resolve sets (fast path or
// lookup, may_reset only before the call's first keyed set), hold the entries, check at the end of
// the call that every held index still names the set's own key in the pool, unpin.  Two calls may
// overlap.  Between calls: deferred builds drained, failing appends, budget / LRU limits changed.
// Exit status 0 = every invariant held (the sanitizers abort on a memory or UB error).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "keycache.h"

using namespace tmed;

namespace {
struct HostPool {
  std::vector<uint8_t> keys;
  size_t cap = 0;
  int fail_next = 0;
  size_t capacity_keys() const { return cap; }
  int append(const uint8_t *pubs, size_t m) {
    if (fail_next) {
      fail_next = 0;
      return -4;
    }
    keys.insert(keys.end(), pubs, pubs + 32 * m);
    return 0;
  }
  void reset() { keys.clear(); }
};

int failures = 0;
#define CHECK(c, ...)                                      \
  do {                                                     \
    if (!(c)) {                                            \
      if (failures++ < 20) {                               \
        fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
        fprintf(stderr, __VA_ARGS__);                      \
        fputc('\n', stderr);                               \
      }                                                    \
    }                                                      \
  } while (0)

struct Held {
  const KcSet *e;
  int set;
};
struct Call {
  bool open = false, keyed_any = false;
  std::vector<Held> held;
};
}  // namespace

int main(int argc, char **argv) {
  const unsigned seed = argc > 1 ? (unsigned)atoi(argv[1]) : 1u;
  const int iters = argc > 2 ? atoi(argv[2]) : 200000;
  std::mt19937_64 rng(seed);
  auto rnd = [&](uint64_t n) { return n ? rng() % n : 0; };

  // a universe of keys (a few repeated on purpose) and sets drawn from it
  const size_t U = 2500;
  std::vector<uint8_t> uni(32 * U);
  for (auto &b : uni) b = (uint8_t)rng();
  for (int r = 0; r < 10; r++) memcpy(&uni[32 * rnd(U)], &uni[32 * rnd(U)], 32);
  std::vector<std::vector<uint8_t>> sets;
  std::vector<std::vector<uint8_t>> hashes;
  for (int s = 0; s < 60; s++) {
    const size_t n = 1 + rnd(s < 50 ? 200 : 700);
    const size_t base = rnd(U);
    std::vector<uint8_t> p(32 * n);
    for (size_t i = 0; i < n; i++) {
      const size_t k = rnd(4) ? (base + i) % U : rnd(U);  // mostly a sliding window (C3-like)
      memcpy(&p[32 * i], &uni[32 * k], 32);
    }
    if (n > 3 && rnd(5) == 0) memcpy(&p[32 * 1], &p[32 * 0], 32);  // a key twice in one set
    sets.push_back(p);
    std::vector<uint8_t> h(32);
    for (auto &b : h) b = (uint8_t)rng();
    hashes.push_back(h);
  }

  KeyCache<HostPool> kc(HostPool{{}, 300 + rnd(1500), 0});
  Call calls[2];
  uint64_t last_lookups = 0;

  auto check_held = [&](const Held &h) {
    const std::vector<uint8_t> &p = sets[h.set];
    const size_t n = p.size() / 32;
    CHECK(h.e->idx.size() == n, "held entry size %zu != %zu", h.e->idx.size(), n);
    for (size_t i = 0; i < n && i < h.e->idx.size(); i++) {
      const uint32_t ix = h.e->idx[i];
      CHECK((size_t)ix * 32 + 32 <= kc.be.keys.size(), "index %u past the pool (%zu keys)", ix,
            kc.be.keys.size() / 32);
      if ((size_t)ix * 32 + 32 <= kc.be.keys.size())
        CHECK(memcmp(&kc.be.keys[32 * (size_t)ix], &p[32 * i], 32) == 0, "set %d key %zu: pool index %u holds another key",
              h.set, i, ix);
    }
  };

  for (int it = 0; it < iters && failures == 0; it++) {
    const int c = (int)rnd(2);
    Call &cl = calls[c];
    const int op = (int)rnd(100);
    if (!cl.open) {
      if (op < 70) {
        kc.pin();
        cl.open = true;
        cl.keyed_any = false;
        cl.held.clear();
      } else if (op < 85) {
        (void)kc.drain_pending();  // the worker between calls
      } else if (op < 90) {
        kc.be.fail_next = 1;
      } else if (op < 94) {
        kc.max_sets = 1 + rnd(80);
        kc.max_set_bytes = 1 + rnd(1u << 20);
      } else if (op < 97) {
        // the budget changes (tmed_keycache_config); a pool past it is dropped when no call holds it
        kc.be.cap = 100 + rnd(2500);
        if (kc.users() == 0 && kc.pool_keys() > kc.be.capacity_keys()) kc.reset();
      } else {
        const int s = (int)rnd(sets.size());
        kc.defer(sets[s].data(), sets[s].size() / 32, rnd(100000));
      }
      continue;
    }
    if (op < 80) {  // resolve one set in this call
      const int s = (int)rnd(sets.size());
      const std::vector<uint8_t> &p = sets[s];
      const size_t n = p.size() / 32;
      const int hk = (int)rnd(4);  // 0: digest key; 1: its hash; 2: another set's hash (stale); 3: digest
      const uint8_t *h = hk == 1 ? hashes[s].data() : hk == 2 ? hashes[rnd(hashes.size())].data() : nullptr;
      const KcKey key = kc_key(p.data(), n, h);
      const size_t sigs = rnd(2) ? rnd(4000) : rnd(2048 * n * 2 + 1);
      const KcSet *hold = nullptr;
      bool keyed = false;
      if (rnd(2)) {  // the fast path of keycache_resolve
        hold = kc.find(key);
        if (hold && kc.same_keys(*hold, p.data(), n)) {
          kc.hit(*hold, sigs);
          keyed = true;
        } else {
          hold = nullptr;
        }
      }
      if (!keyed) keyed = kc.lookup(p.data(), n, key, sigs, !cl.keyed_any, hold, rnd(10) == 0);
      if (keyed) {
        CHECK(hold != nullptr, "keyed without an entry");
        if (hold) {
          cl.held.push_back({hold, s});
          check_held(cl.held.back());
        }
        cl.keyed_any = true;
      }
    } else if (op < 90) {  // the call ends: every entry it holds still names its keys
      for (const Held &hd : cl.held) check_held(hd);
      cl.held.clear();
      cl.open = false;
      kc.unpin();
    } else {
      const std::vector<uint8_t> &p = sets[rnd(sets.size())];
      (void)kc.missing_keys(p.data(), p.size() / 32);
      (void)kc.all_pooled(p.data(), p.size() / 32);
    }
    CHECK(kc.pool_keys() == kc.be.keys.size() / 32, "pool_keys %zu != backend keys %zu", kc.pool_keys(),
          kc.be.keys.size() / 32);
    CHECK(kc.st.lookups >= last_lookups, "lookups went backwards");
    last_lookups = kc.st.lookups;
    CHECK(kc.st.hits <= kc.st.lookups && kc.st.keyed_sets + kc.st.generic_sets == kc.st.lookups,
          "counters inconsistent");
  }
  for (Call &cl : calls)
    if (cl.open) {
      for (const Held &hd : cl.held) check_held(hd);
      kc.unpin();
    }
  printf("keycache_fuzz seed %u iters %d: lookups %llu hits %llu keyed %llu generic %llu resets %llu evicted %llu "
         "pool %zu failures %d\n",
         seed, iters, (unsigned long long)kc.st.lookups, (unsigned long long)kc.st.hits,
         (unsigned long long)kc.st.keyed_sets, (unsigned long long)kc.st.generic_sets,
         (unsigned long long)kc.st.pool_resets, (unsigned long long)kc.st.sets_evicted, kc.pool_keys(), failures);
  return failures ? 1 : 0;
}
