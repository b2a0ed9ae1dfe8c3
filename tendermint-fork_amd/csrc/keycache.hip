// keycache.hip — the commit seam's validator-set key cache on the device (keycache.h policy;
// SURVEY.md §8f f2): one pooled Keyset per context, grown by keyset_append on the context stream.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <thread>

#include "ctx.h"
#include "keycache.h"

namespace tmed {

// The pool: a Keyset in ctx->keysets marked `pooled` (unreachable through the public handles, so no
// caller can free or extend it), created at the first append.  Appends are ordered on the context
// stream in front of the kernels that read them; the caller holds ctx->mu.
struct KcBackendDev {
  tmed_ctx *c = nullptr;
  uint64_t handle = 0;
  size_t capacity_keys() const { return std::max<size_t>(1, c->kc_budget / keyset_bytes_per_key(c)); }
  int append(const uint8_t *pubs, size_t m) {
    (void)hipSetDevice(c->device);
    if (!handle) {
      handle = c->next_keyset++;
      Keyset &k = c->keysets[handle];
      k.pooled = true;
    }
    int rc = keyset_append(c, c->keysets[handle], pubs, m, c->stream, capacity_keys());
    if (rc == TMED_OK) (void)ctx_bcomb24(c);  // the key-cached throughput kernel's B comb
    return rc;
  }
  void reset() {
    if (!handle) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->lane1.s) (void)hipStreamSynchronize(c->lane1.s);
    auto it = c->keysets.find(handle);
    if (it != c->keysets.end()) {
      free_keyset(it->second);
      c->keysets.erase(it);
    }
    handle = 0;
  }
};

// The keys a generic call queued are built by a worker thread of the context after the call has
// returned, so the first call against a new set costs what a generic call costs (the build's
// uploads and launches, ~30 us of host time, stay off the caller's critical path).  The worker
// takes ctx->mu like any call; tmed_keycache_wait joins it.
struct KeyCacheDev {
  KeyCache<KcBackendDev> kc;
  std::mutex wm;  // worker state (never held together with ctx->mu by the caller side)
  std::condition_variable wcv;
  bool want = false, busy = false, stop = false;
  std::thread worker;
  explicit KeyCacheDev(tmed_ctx *c) : kc(KcBackendDev{c, 0}) {
    worker = std::thread([this, c] {
      std::unique_lock<std::mutex> lk(wm);
      for (;;) {
        wcv.wait(lk, [&] { return want || stop; });
        if (stop) return;
        want = false;
        busy = true;
        lk.unlock();
        {
          std::lock_guard<std::mutex> g(c->mu);
          (void)kc.drain_pending();  // a failed build leaves those sets generic
        }
        lk.lock();
        busy = false;
        wcv.notify_all();
      }
    });
  }
  void kick() {
    std::lock_guard<std::mutex> lk(wm);
    want = true;
    wcv.notify_all();
  }
  void wait_idle() {
    std::unique_lock<std::mutex> lk(wm);
    wcv.wait(lk, [&] { return !want && !busy; });
  }
  ~KeyCacheDev() {
    {
      std::lock_guard<std::mutex> lk(wm);
      stop = true;
      wcv.notify_all();
    }
    worker.join();
  }
};

static KeyCache<KcBackendDev> &cache_of(tmed_ctx *c) {
  if (!c->kc) c->kc = new KeyCacheDev(c);
  return c->kc->kc;
}

void keycache_destroy(tmed_ctx *c) {  // ctx->mu not held: the worker may be waiting for it
  if (!c->kc) return;
  KeyCacheDev *d = c->kc;
  d->wait_idle();
  {
    std::lock_guard<std::mutex> lk(c->mu);
    c->kc = nullptr;
  }
  delete d;  // joins the worker
  // the pool's Keyset is freed with the context's key sets
}

// ---- the seam's side (commit.hip keycache_resolve); the caller holds ctx->mu -----------------
uint64_t keycache_pool_handle(const tmed_ctx *c) { return c->kc ? c->kc->kc.be.handle : 0; }
const KcSet *keycache_find(tmed_ctx *c, const KcKey &key) { return cache_of(c).find(key); }
bool keycache_same_keys(const tmed_ctx *c, const KcSet &e, const uint8_t *pubs, size_t n) {
  return c->kc && c->kc->kc.same_keys(e, pubs, n);
}
uint64_t keycache_call_tick(tmed_ctx *c) { return cache_of(c).call_tick(); }
void keycache_hits(tmed_ctx *c, size_t sets, size_t sigs) { cache_of(c).hits(sets, sigs); }
void keycache_touch(tmed_ctx *c) { (void)cache_of(c); }
void keycache_hit(tmed_ctx *c, const KcSet &e, size_t sigs) { cache_of(c).hit(e, sigs); }
void keycache_pin(tmed_ctx *c) { cache_of(c).pin(); }
void keycache_unpin(tmed_ctx *c) { cache_of(c).unpin(); }
// true: the set's signatures take the key-cached kernels in this call, *handle = the pool and
// hold->idx its index there.
bool keycache_lookup(tmed_ctx *c, const uint8_t *pubs, size_t n, const KcKey &key, size_t sigs, bool may_reset,
                     uint64_t *handle, const KcSet *&hold, bool force_build) {
  KeyCache<KcBackendDev> &kc = cache_of(c);
  if (!kc.lookup(pubs, n, key, sigs, may_reset, hold, force_build)) return false;
  *handle = kc.be.handle;
  return true;
}
size_t keycache_missing(tmed_ctx *c, const uint8_t *pubs, size_t n, std::unordered_set<Pub32, Pub32Hash> *seen) {
  return cache_of(c).missing_keys(pubs, n, seen);
}
int keycache_drain(tmed_ctx *c) { return c->kc ? c->kc->kc.drain_pending() : TMED_OK; }
void keycache_after_call(tmed_ctx *c) {
  if (c->kc && c->kc->kc.has_work()) c->kc->kick();
}
bool keycache_all_pooled(tmed_ctx *c, const uint8_t *pubs, size_t n) { return cache_of(c).all_pooled(pubs, n); }
void keycache_defer(tmed_ctx *c, const uint8_t *pubs, size_t n, size_t sigs) { cache_of(c).defer(pubs, n, sigs); }

}  // namespace tmed

using namespace tmed;

extern "C" {

int tmed_keycache_config(tmed_ctx *c, int enabled, size_t budget_bytes) {
  if (!c || enabled < -1 || enabled > 1) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (enabled >= 0) c->kc_on = enabled != 0;
  if (budget_bytes) {
    c->kc_budget = budget_bytes;
    // a pool already past the new budget is dropped at once (no call can hold it: we hold ctx->mu
    // and calls pin it only while resolving under that lock or running)
    if (c->kc && c->kc->kc.users() == 0 && c->kc->kc.pool_keys() > c->kc->kc.be.capacity_keys()) c->kc->kc.reset();
  }
  return TMED_OK;
}

int tmed_keycache_stats(tmed_ctx *c, tmed_keycache_counters *o) {
  if (!c || !o) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  memset(o, 0, sizeof *o);
  o->enabled = c->kc_on ? 1 : 0;
  o->budget_bytes = c->kc_budget;
  if (!c->kc) return TMED_OK;
  const KeyCache<KcBackendDev> &kc = c->kc->kc;
  const KcCounters &s = kc.st;
  o->lookups = s.lookups;
  o->hits = s.hits;
  o->keyed_sets = s.keyed_sets;
  o->generic_sets = s.generic_sets;
  o->keys_appended = s.keys_appended;
  o->keys_deferred = s.keys_deferred;
  o->pool_resets = s.pool_resets;
  o->sets_evicted = s.sets_evicted;
  o->keyed_sigs = s.keyed_sigs;
  o->generic_sigs = s.generic_sigs;
  o->pool_keys = kc.pool_keys();
  o->pool_capacity_keys = kc.be.capacity_keys();
  o->sets_cached = kc.sets_cached();
  o->pending_keys = kc.pending_keys();
  auto it = c->keysets.find(kc.be.handle);
  if (kc.be.handle && it != c->keysets.end()) {
    const Keyset &k = it->second;
    o->pool_bytes = k.cap * 33 + k.comb_room() * kCombBytesPerKey + k.comba_room() * kCombABytesPerKey;
    o->pool_a_window_bits = !k.comba.empty() && k.comba_n == k.n ? kCombABits : 8;
  }
  return TMED_OK;
}

int tmed_keycache_wait(tmed_ctx *c) {
  if (!c) return TMED_EINVAL;
  KeyCacheDev *d;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    d = c->kc;
  }
  if (d) d->wait_idle();
  std::lock_guard<std::mutex> lk(c->mu);
  (void)hipSetDevice(c->device);
  return map_err(hipStreamSynchronize(c->stream));
}

int tmed_keycache_flush(tmed_ctx *c) {
  if (!c) return TMED_EINVAL;
  if (c->kc) c->kc->wait_idle();
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->kc) return TMED_OK;
  if (c->kc->kc.users() > 0) return TMED_EINVAL;  // a call in flight holds indexes into the pool
  c->kc->kc.reset();
  return TMED_OK;
}

int tmed_keycache_warm(tmed_ctx *c, const tmed_valset *vals) {
  if (!c || !vals || (vals->n && !vals->pubkeys)) return TMED_EINVAL;
  if (vals->n == 0 || vals->keyset) return TMED_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  KeyCache<KcBackendDev> &kc = cache_of(c);
  (void)hipSetDevice(c->device);
  int rc = keycache_drain(c);
  if (rc != TMED_OK) return rc;
  const KcSet *hold = nullptr;
  uint64_t h = 0;
  kc.pin();
  // the missing keys are built now, whatever a call's size would say
  const bool keyed = keycache_lookup(c, vals->pubkeys, vals->n, kc_key(vals->pubkeys, vals->n, vals->set_hash), 0,
                                     true, &h, hold, /*force_build=*/true);
  kc.unpin();
  if (!keyed) return TMED_ENOMEM;  // does not fit the pool's budget
  return map_err(hipStreamSynchronize(c->stream));
}

}  // extern "C"
