// keycache_test.cpp — TEST-ONLY host build of the seam's key-set cache policy
// (tendermint-fork_amd/csrc/keycache.h) over a host stand-in for the device pool, so the
// policy (hits, deferred builds, amortised builds, budget resets, pinning, LRU bounds, byte
// compare on hits) is checked in a container without a GPU (tests/test_keycache_policy.py).
#include <stdint.h>
#include <string.h>

#include <vector>

#include "keycache.h"

using namespace tmed;

namespace {
struct HostPool {
  std::vector<uint8_t> keys;  // the pool's keys in index order
  size_t cap = 0;
  int fail_next = 0;
  size_t capacity_keys() const { return cap; }
  int append(const uint8_t *pubs, size_t m) {
    if (fail_next) { fail_next = 0; return -4; }
    keys.insert(keys.end(), pubs, pubs + 32 * m);
    return 0;
  }
  void reset() { keys.clear(); }
};
struct Kct {
  KeyCache<HostPool> kc;
  explicit Kct(size_t cap) : kc(HostPool{{}, cap, 0}) {}
};
}  // namespace

extern "C" {
void *kct_new(size_t cap_keys) { return new Kct(cap_keys); }
void kct_free(void *h) { delete (Kct *)h; }
void kct_limits(void *h, size_t max_sets, size_t max_bytes) {
  Kct *t = (Kct *)h;
  t->kc.max_sets = max_sets;
  t->kc.max_set_bytes = max_bytes;
}
void kct_pin(void *h) { ((Kct *)h)->kc.pin(); }
void kct_unpin(void *h) { ((Kct *)h)->kc.unpin(); }
void kct_fail_next_append(void *h) { ((Kct *)h)->kc.be.fail_next = 1; }
// 1 keyed (idx_out[i] = pool index of key i), 0 generic.  fast: try the find/compare/hit path first.
int kct_lookup(void *h, const uint8_t *pubs, size_t n, const uint8_t *set_hash, size_t sigs, int may_reset,
               int force, int fast, uint32_t *idx_out) {
  KeyCache<HostPool> &kc = ((Kct *)h)->kc;
  const KcKey key = kc_key(pubs, n, set_hash);
  const KcSet *hold = nullptr;
  bool keyed = false;
  if (fast) {
    hold = kc.find(key);
    if (hold && kc.same_keys(*hold, pubs, n)) {
      kc.hit(*hold, sigs);
      keyed = true;
    } else {
      hold = nullptr;
    }
  }
  if (!keyed) keyed = kc.lookup(pubs, n, key, sigs, may_reset != 0, hold, force != 0);
  if (keyed) memcpy(idx_out, hold->idx.data(), 4 * n);
  return keyed ? 1 : 0;
}
size_t kct_missing(void *h, const uint8_t *pubs, size_t n) { return ((Kct *)h)->kc.missing_keys(pubs, n); }
int kct_drain(void *h) { return ((Kct *)h)->kc.drain_pending(); }
// lookups, hits, keyed_sets, generic_sets, keyed_sigs, generic_sigs, keys_appended, keys_deferred,
// pool_resets, sets_evicted, pool_keys, sets_cached, pending_keys, backend_keys
void kct_stats(void *h, uint64_t out[14]) {
  const KeyCache<HostPool> &kc = ((Kct *)h)->kc;
  const KcCounters &s = kc.st;
  const uint64_t v[14] = {s.lookups, s.hits, s.keyed_sets, s.generic_sets, s.keyed_sigs, s.generic_sigs,
                          s.keys_appended, s.keys_deferred, s.pool_resets, s.sets_evicted, kc.pool_keys(),
                          kc.sets_cached(), kc.pending_keys(), kc.be.keys.size() / 32};
  memcpy(out, v, sizeof v);
}
int kct_pool_key(void *h, uint32_t i, uint8_t out[32]) {
  const HostPool &p = ((Kct *)h)->kc.be;
  if ((size_t)i * 32 + 32 > p.keys.size()) return -1;
  memcpy(out, &p.keys[(size_t)i * 32], 32);
  return 0;
}
size_t kct_retired(void *h) { return ((Kct *)h)->kc.retired(); }
int kct_all_pooled(void *h, const uint8_t *pubs, size_t n) { return ((Kct *)h)->kc.all_pooled(pubs, n) ? 1 : 0; }
void kct_defer(void *h, const uint8_t *pubs, size_t n, size_t sigs) { ((Kct *)h)->kc.defer(pubs, n, sigs); }
void kct_digest(const uint8_t *pubs, size_t n, uint8_t out[32]) { kc_digest(pubs, n, out); }
}
