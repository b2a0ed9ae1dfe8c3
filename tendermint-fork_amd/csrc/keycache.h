// keycache.h — the per-context validator-set key cache behind the commit seam.
//
// The reference decodes A inside every Verify (crypto/ed25519/ed25519.go:148-155).  Its callers
// verify commit after commit against the SAME validator set (state/validation.go:93-96 checks
// LastCommit against LastValidators every block; blockchain/v0/reactor.go:366-367 checks every
// buffered block against state.Validators; light/verifier.go:58,73-76 checks headers against sets
// that change by a few keys per height).  This cache makes those callers reach the key-cached
// kernels with no handle management on their side:
//
//   * ONE pool key set per context (a Keyset in ctx->keysets, grown by appending keys; indexes of
//     keys already in it never change).  A pubkey is stored once however many sets hold it, so a
//     light client's per-height sets share their keys.
//   * set entries keyed by ValidatorSet.Hash() (types/validator_set.go:347-353) when the caller
//     passes it (tmed_valset.set_hash), else by a digest of the ordered key bytes; an entry holds a
//     copy of the set's keys (compared byte for byte on every hit: a stale or colliding key can
//     only cost a miss, never a wrong index) and the set's index into the pool.
//   * policy on a miss: if every key is already in the pool, the set is keyed at once; if the
//     call's own signatures amortise building the new keys' combs (>= kAmortizeSigsPerKey per new
//     key, a blocksync window or a large light-client batch), the keys are appended in stream
//     order before this call's kernels and the set is keyed at once; otherwise (the first commit
//     of a new set: C1) this call takes the generic kernels and the new keys are appended right
//     after it (deferred), so the NEXT call against the set is keyed.
//   * bounds: the pool holds at most capacity_keys() keys (the HBM budget); when a set does not
//     fit, the pool is reset if no other call holds indexes into it, else the set stays generic.
//     Set entries are bounded in count and host bytes (least recently used first out).
//
// Host-only logic, templated on a backend (the device pool in keycache.hip; a host stand-in in
// tests/native/keycache_test.cpp, which checks the policy on the CPU).
//   Backend::append(const uint8_t *pubs, size_t m) -> int   append m keys (TMED_OK or an error)
//   Backend::capacity_keys() -> size_t                      pool keys the budget allows
//   Backend::reset()                                        drop every key of the pool
#pragma once
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace tmed {

struct KcKey {
  uint8_t d[32];
  uint64_t n;
  uint8_t from_hash;  // d is the caller's ValidatorSet.Hash(), not the key digest
  bool operator==(const KcKey &o) const { return n == o.n && from_hash == o.from_hash && memcmp(d, o.d, 32) == 0; }
};
struct KcKeyHash {
  size_t operator()(const KcKey &k) const {
    uint64_t x;
    memcpy(&x, k.d, 8);
    return (size_t)((x ^ (k.n * 0x9E3779B97F4A7C15ull)) + k.from_hash);
  }
};

struct Pub32 {
  uint64_t w[4];
  bool operator==(const Pub32 &o) const { return memcmp(w, o.w, 32) == 0; }
};
struct Pub32Hash {
  size_t operator()(const Pub32 &p) const {  // keys are attacker-choosable: mix every word
    uint64_t h = p.w[0] * 0x9E3779B97F4A7C15ull;
    h = (h ^ (h >> 29) ^ p.w[1]) * 0xBF58476D1CE4E5B9ull;
    h = (h ^ (h >> 31) ^ p.w[2]) * 0x94D049BB133111EBull;
    h = (h ^ (h >> 30) ^ p.w[3]) * 0x9E3779B97F4A7C15ull;
    return (size_t)(h ^ (h >> 32));
  }
};
inline Pub32 pub32(const uint8_t *p) {
  Pub32 k;
  memcpy(k.w, p, 32);
  return k;
}

// 256-bit digest of n ordered 32-byte keys: four independent multiply-xorshift lanes, one per
// 8-byte word of a key, then a cross-lane finish.  Not cryptographic: an entry found by digest is
// still compared byte for byte, so a collision only costs a miss.
inline void kc_digest(const uint8_t *pubs, size_t n, uint8_t out[32]) {
  uint64_t a[4] = {0x243F6A8885A308D3ull, 0x13198A2E03707344ull, 0xA4093822299F31D0ull, 0x082EFA98EC4E6C89ull};
  for (size_t i = 0; i < n; i++) {
    uint64_t w[4];
    memcpy(w, pubs + 32 * i, 32);
    for (int l = 0; l < 4; l++) {
      uint64_t x = (a[l] ^ w[l]) * 0x9E3779B97F4A7C15ull;
      a[l] = x ^ (x >> 31) ^ (uint64_t)i;
    }
  }
  for (int r = 0; r < 2; r++)
    for (int l = 0; l < 4; l++) {
      uint64_t x = (a[l] + a[(l + 1) & 3] + (uint64_t)n) * 0xBF58476D1CE4E5B9ull;
      a[l] = x ^ (x >> 27);
    }
  memcpy(out, a, 32);
}

inline KcKey kc_key(const uint8_t *pubs, size_t n, const uint8_t *set_hash) {
  KcKey k;
  k.n = n;
  k.from_hash = set_hash ? 1 : 0;
  if (set_hash)
    memcpy(k.d, set_hash, 32);
  else
    kc_digest(pubs, n, k.d);
  return k;
}

// address -> first validator index with that address (GetByAddress, types/validator_set.go:270-278
// returns the first match).  Flat open-addressing table: a light-client batch looks up ~59
// addresses per Trusting request, one request per trusted set (C3: 10k sets x 175 validators).
struct AddrIndex {
  const uint8_t *addrs = nullptr;  // the set's n x 20 address array
  std::vector<int32_t> vals;       // validator index, -1 = empty
  size_t mask = 0, n = 0;
  bool unique = true;              // no address occurs twice (then position i is its own first match)
  static size_t slot_of(const uint8_t *p) {  // addresses are SHA-256 truncations: 8 bytes mix well
    uint64_t a;
    memcpy(&a, p, 8);
    return (size_t)((a * 0x9E3779B97F4A7C15ull) >> 20);
  }
  void build(const uint8_t *addresses, size_t count) {
    addrs = addresses;
    n = count;
    unique = true;
    size_t cap = 16;
    while (cap < 2 * n + 1) cap <<= 1;
    mask = cap - 1;
    vals.assign(cap, -1);
    for (size_t v = 0; v < n; v++) {
      const uint8_t *a = addresses + 20 * v;
      size_t h = slot_of(a) & mask;
      while (vals[h] >= 0 && memcmp(addrs + 20 * (size_t)vals[h], a, 20) != 0) h = (h + 1) & mask;
      if (vals[h] < 0) vals[h] = (int32_t)v;  // keep the first match
      else unique = false;
    }
  }
  // validator i of the set when it has this address and addresses are unique (a commit's
  // signature i is usually validator i of a neighbouring set: one sequential compare instead of
  // two cold reads of the index), else -2 (ask find)
  int32_t at(const uint8_t *addr, size_t i) const {
    return unique && i < n && memcmp(addrs + 20 * i, addr, 20) == 0 ? (int32_t)i : -2;
  }
  // software prefetch for a lookup a few signatures ahead (the index and the set's address copy
  // are cold at a light-client batch's ~10k sets): the slot, then the address it holds
  void prefetch_slot(const uint8_t *addr) const { __builtin_prefetch(&vals[slot_of(addr) & mask]); }
  void prefetch_entry(const uint8_t *addr) const {
    const int32_t v = vals[slot_of(addr) & mask];
    if (v >= 0) __builtin_prefetch(addrs + 20 * (size_t)v);
  }
  int32_t find(const uint8_t *addr) const {
    size_t h = slot_of(addr) & mask;
    while (vals[h] >= 0) {
      if (memcmp(addrs + 20 * (size_t)vals[h], addr, 20) == 0) return vals[h];
      h = (h + 1) & mask;
    }
    return -1;
  }
};

// One cached validator set: validator i -> pool index (the byte compare of a hit reads the keys
// through it from the pool's own key table: KeyCache::same_keys); and, built at the first
// LightTrusting request against it, its address index over a private copy of the addresses that
// request passed (a later request uses it only if its addresses are the same bytes:
// tmed_valset.addresses is not part of the cache key).
struct KcSet {
  std::vector<uint32_t> idx;
  std::atomic<uint64_t> tick{0};  // LRU: the call that last used it (set from a call's threads)
  void touch(uint64_t t) { tick.store(t, std::memory_order_relaxed); }
  size_t bytes() const { return 4 * idx.size() + 64; }
  // nullptr when `addrs` (n x 20) differ from the addresses the cached index was built from
  const AddrIndex *addr_index(const uint8_t *addrs, size_t n) const {
    std::call_once(addr_once_, [&] {
      addr_copy_.assign(addrs, addrs + 20 * n);
      addr_ix_.build(addr_copy_.data(), n);
    });
    return addr_copy_.size() == 20 * n && memcmp(addr_copy_.data(), addrs, 20 * n) == 0 ? &addr_ix_ : nullptr;
  }

 private:
  mutable std::once_flag addr_once_;
  mutable std::vector<uint8_t> addr_copy_;
  mutable AddrIndex addr_ix_;
};


// Counters (tmed_keycache_stats).
struct KcCounters {
  uint64_t lookups = 0, hits = 0;         // set lookups; hits on a cached entry
  uint64_t keyed_sets = 0;                // lookups that gave the key-cached kernels
  uint64_t generic_sets = 0;              // lookups that stayed generic this call
  uint64_t keys_appended = 0;             // keys built into the pool (at once or deferred)
  uint64_t keys_deferred = 0;             // of those, queued behind a generic call
  uint64_t pool_resets = 0;               // the pool was emptied to fit a set
  uint64_t sets_evicted = 0;              // entries dropped by the count / byte bound
  uint64_t keyed_sigs = 0, generic_sigs = 0;  // signatures of requests resolved each way
};

// Signatures of a call per new key at which its keys are built BEFORE the call instead of by the
// worker after a generic call.  The keys get built either way, on the same device, so for a
// throughput caller building first only swaps generic verifies (~9.5 ns) for keyed ones (~1.8 ns);
// the threshold bounds what a single call waits for: a key's radix-256 + radix-2^12 combs cost
// ~50 us of batched device time (~5k generic verifies); the latency-size batches never reach it
// (a lone key's comb-base chain is ~0.5 ms serial, more than a generic commit).
constexpr size_t kKcAmortizeSigsPerKey = 2048;

template <class Backend>
class KeyCache {
 public:
  static constexpr size_t kAmortizeSigsPerKey = kKcAmortizeSigsPerKey;

  explicit KeyCache(Backend b) : be(std::move(b)) {}

  Backend be;
  size_t max_sets = 1u << 16;
  size_t max_set_bytes = (size_t)512 << 20;
  KcCounters st;

  size_t pool_keys() const { return slot_.size(); }

  // A cached set's keys are the caller's, byte for byte: key i against pool key idx[i] (the pool's
  // key table: a few hundred KB, cache-resident, against a private copy of every set's keys —
  // ~5.6 KB per 175-validator set, 56 MB for a light client's 10k sets, read back on every call).
  // A stale set_hash or a digest collision therefore costs a miss, never a wrong index.
  bool same_keys(const KcSet &e, const uint8_t *pubs, size_t n) const {
    if (e.idx.size() != n) return false;
    const uint8_t *pk = keys_.data();
    for (size_t i = 0; i < n; i++) {
      uint64_t a[4], b[4];
      memcpy(a, pk + 32 * (size_t)e.idx[i], 32);
      memcpy(b, pubs + 32 * i, 32);
      if (((a[0] ^ b[0]) | (a[1] ^ b[1]) | (a[2] ^ b[2]) | (a[3] ^ b[3])) != 0) return false;
    }
    return true;
  }
  size_t sets_cached() const { return sets_.size(); }
  size_t pending_keys() const { return pending_.size() / 32; }
  bool has_work() const { return !pending_.empty() || !deferred_.empty(); }
  int users() const { return users_; }
  size_t retired() const { return retired_.size(); }

  // A seam call holds the pool (no reset while its resolved indexes are in use) from before its
  // first lookup until it has collected its last batch.  Entries dropped meanwhile (LRU bound, a
  // reset, a mismatching key) are retired, not freed, until no call is pinned: the entry pointers
  // a call resolved (and their idx / address index) stay valid for the whole call without a
  // reference count per entry (a light-client batch resolves ~10k sets).
  void pin() { users_++; }
  void unpin() {
    if (users_ > 0) users_--;
    if (users_ == 0) retired_.clear();
  }

  // Fast path of a call resolving many sets: the cached entry under `key` (nullptr if none), to be
  // compared with the set's keys; a match is then recorded with touch(call_tick()) + hits().
  // Read-only (safe from several threads at once while the caller holds the lock).
  const KcSet *find(const KcKey &key) const {
    auto it = sets_.find(key);
    return it == sets_.end() ? nullptr : it->second.get();
  }
  uint64_t call_tick() { return ++tick_; }
  void hits(size_t sets, size_t sigs) {
    st.lookups += sets;
    st.hits += sets;
    st.keyed_sets += sets;
    st.keyed_sigs += sigs;
  }
  void hit(const KcSet &e, size_t sigs) {
    const_cast<KcSet &>(e).touch(call_tick());
    hits(1, sigs);
  }

  // Resolve one set for a call that pinned the pool.  Returns true (keyed: *hold->idx are the
  // pool indexes of validators 0..n-1, valid while hold lives and the call is pinned) or false
  // (generic this call).  may_reset: the call has resolved no keyed set yet.
  // force_build: build missing keys now whatever the call's size (tmed_keycache_warm).
  bool lookup(const uint8_t *pubs, size_t n, const KcKey &key, size_t sigs, bool may_reset,
              const KcSet *&hold, bool force_build = false) {
    st.lookups++;
    auto it = sets_.find(key);
    if (it != sets_.end()) {
      KcSet &s = *it->second;
      if (same_keys(s, pubs, n)) {
        s.touch(++tick_);
        st.hits++;
        return keyed(it->second.get(), sigs, hold);
      }
      drop_(it);  // same key, other keys (a stale or wrong set_hash, a digest collision)
    }
    auto e = std::make_unique<KcSet>();
    e->idx.resize(n);
    std::vector<size_t> fresh;  // first position of each key the pool lacks
    if (!resolve_(*e, pubs, fresh)) return generic(sigs);  // more distinct new keys than the pool can hold
    if (fresh.empty()) return insert_keyed(std::move(e), key, sigs, hold);
    const size_t nf = fresh.size();
    if (slot_.size() + nf > be.capacity_keys()) {
      if (!(may_reset && users_ <= 1) || nf > be.capacity_keys()) return generic(sigs);
      reset();
      st.pool_resets++;
      fresh.clear();
      if (!resolve_(*e, pubs, fresh)) return generic(sigs);
    }
    if (!force_build && sigs < kAmortizeSigsPerKey * fresh.size()) {  // generic now, keys built after the call
      for (size_t f : fresh) {
        const Pub32 k = pub32(pubs + 32 * f);
        if (pend_set_.insert(k).second) pending_.insert(pending_.end(), pubs + 32 * f, pubs + 32 * f + 32);
      }
      return generic(sigs);
    }
    std::vector<uint8_t> add(32 * fresh.size());
    for (size_t j = 0; j < fresh.size(); j++) memcpy(&add[32 * j], pubs + 32 * fresh[j], 32);
    if (!append_(add.data(), fresh.size())) return generic(sigs);
    resolve_(*e, pubs, fresh);  // every key present now
    return insert_keyed(std::move(e), key, sigs, hold);
  }

  // Every key of the set already in the pool (stops at the first missing one).
  bool all_pooled(const uint8_t *pubs, size_t n) const {
    for (size_t i = 0; i < n; i++)
      if (!slot_.count(pub32(pubs + 32 * i))) return false;
    return true;
  }

  // A set of a small call (too few signatures to pay for even one key) whose keys are not all
  // pooled: the call runs generic, and its keys are only copied here — which of them the pool lacks
  // is worked out by drain_pending, after the call (the first commit of a new set pays no
  // per-key lookups).  Counted like lookup()'s deferred path.
  void defer(const uint8_t *pubs, size_t n, size_t sigs) {
    st.lookups++;
    generic(sigs);
    deferred_.insert(deferred_.end(), pubs, pubs + 32 * n);
  }

  // Distinct keys of a set that the pool lacks (not counting those already in *seen, which
  // collects them across the sets of one call): a call builds every missing key at once when its
  // signatures amortise them all (kAmortizeSigsPerKey each), as a blocksync window or a large
  // light-client batch does.
  size_t missing_keys(const uint8_t *pubs, size_t n, std::unordered_set<Pub32, Pub32Hash> *seen = nullptr) const {
    std::unordered_set<Pub32, Pub32Hash> local;
    if (!seen) seen = &local;
    size_t m = 0;
    for (size_t i = 0; i < n; i++) {
      const Pub32 k = pub32(pubs + 32 * i);
      if (!slot_.count(k) && seen->insert(k).second) m++;
    }
    return m;
  }

  // Build the keys queued by generic calls (after such a call has collected its results).
  int drain_pending() {
    for (size_t r = 0; r < deferred_.size() / 32; r++) {  // the deferred sets' keys the pool lacks
      const Pub32 k = pub32(&deferred_[32 * r]);
      if (!slot_.count(k) && pend_set_.insert(k).second)
        pending_.insert(pending_.end(), &deferred_[32 * r], &deferred_[32 * r] + 32);
    }
    deferred_.clear();
    if (pending_.empty()) return 0;
    std::vector<uint8_t> add;
    add.swap(pending_);
    pend_set_.clear();
    // keys another call appended meanwhile are skipped
    size_t w = 0;
    for (size_t r = 0; r < add.size() / 32; r++)
      if (!slot_.count(pub32(&add[32 * r]))) {
        if (w != r) memcpy(&add[32 * w], &add[32 * r], 32);
        w++;
      }
    if (w == 0) return 0;
    if (slot_.size() + w > be.capacity_keys()) {
      if (users_ > 0 || w > be.capacity_keys()) return 0;  // dropped: the sets stay generic
      reset();
      st.pool_resets++;
    }
    st.keys_deferred += w;
    return append_(add.data(), w) ? 0 : -1;
  }

  void reset() {
    be.reset();
    slot_.clear();
    keys_.clear();
    if (users_ > 0)
      for (auto &kv : sets_) retired_.push_back(std::move(kv.second));
    sets_.clear();
    set_bytes_ = 0;
    pending_.clear();
    pend_set_.clear();
    deferred_.clear();
  }

 private:
  bool keyed(const KcSet *e, size_t sigs, const KcSet *&hold) {
    hold = e;
    st.keyed_sets++;
    st.keyed_sigs += sigs;
    return true;
  }
  bool generic(size_t sigs) {
    st.generic_sets++;
    st.generic_sigs += sigs;
    return false;
  }
  // idx of every key already in the pool; `fresh` gets the first position of each key it lacks.
  // False when there are more such keys than the pool could ever hold.
  bool resolve_(KcSet &e, const uint8_t *pubs, std::vector<size_t> &fresh) {
    const size_t n = e.idx.size();
    std::unordered_map<Pub32, uint32_t, Pub32Hash> local;  // new keys repeated inside the set
    for (size_t i = 0; i < n; i++) {
      const Pub32 k = pub32(pubs + 32 * i);
      auto s = slot_.find(k);
      if (s != slot_.end()) {
        e.idx[i] = s->second;
        continue;
      }
      auto l = local.find(k);
      if (l != local.end()) {
        e.idx[i] = l->second;
        continue;
      }
      const uint32_t provisional = (uint32_t)(slot_.size() + fresh.size());
      local.emplace(k, provisional);
      e.idx[i] = provisional;
      fresh.push_back(i);
      if (fresh.size() > be.capacity_keys()) return false;
    }
    return true;
  }
  bool append_(const uint8_t *keys, size_t m) {
    if (be.append(keys, m) != 0) return false;
    for (size_t j = 0; j < m; j++) slot_.emplace(pub32(keys + 32 * j), (uint32_t)slot_.size());
    keys_.insert(keys_.end(), keys, keys + 32 * m);
    st.keys_appended += m;
    return true;
  }
  bool insert_keyed(std::unique_ptr<KcSet> e, const KcKey &key, size_t sigs, const KcSet *&hold) {
    e->touch(++tick_);
    set_bytes_ += e->bytes();
    const KcSet *p = e.get();
    sets_[key] = std::move(e);
    if (sets_.size() > max_sets || set_bytes_ > max_set_bytes) evict_();
    return keyed(p, sigs, hold);
  }
  void drop_(typename std::unordered_map<KcKey, std::unique_ptr<KcSet>, KcKeyHash>::iterator it) {
    set_bytes_ -= it->second->bytes();
    if (users_ > 0) retired_.push_back(std::move(it->second));
    sets_.erase(it);
  }
  // Least recently used quarter out (calls in flight keep theirs: retired_).
  void evict_() {
    std::vector<uint64_t> ticks;
    ticks.reserve(sets_.size());
    for (auto &kv : sets_) ticks.push_back(kv.second->tick.load(std::memory_order_relaxed));
    const size_t k = std::max<size_t>(1, ticks.size() / 4);
    std::nth_element(ticks.begin(), ticks.begin() + (k - 1), ticks.end());
    const uint64_t cut = ticks[k - 1];
    for (auto it = sets_.begin(); it != sets_.end();) {
      auto nx = std::next(it);
      if (it->second->tick.load(std::memory_order_relaxed) <= cut) {
        drop_(it);
        st.sets_evicted++;
      }
      it = nx;
    }
  }

  std::unordered_map<Pub32, uint32_t, Pub32Hash> slot_;  // pool index of every key in the pool
  std::vector<uint8_t> keys_;  // the pool's keys in index order (32 B each): same_keys reads them
  std::unordered_map<KcKey, std::unique_ptr<KcSet>, KcKeyHash> sets_;
  std::vector<std::unique_ptr<KcSet>> retired_;  // dropped while a call was pinned
  std::vector<uint8_t> pending_;  // keys queued by generic calls
  std::vector<uint8_t> deferred_;  // keys of deferred sets, not yet checked against the pool
  std::unordered_set<Pub32, Pub32Hash> pend_set_;
  size_t set_bytes_ = 0;
  uint64_t tick_ = 0;
  int users_ = 0;
};

}  // namespace tmed
