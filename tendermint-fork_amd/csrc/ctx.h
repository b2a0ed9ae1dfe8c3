// ctx.h — tmed_ctx internals shared by the host-side translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/tmed25519.h"
#include "kernels.h"
#include "keycache.h"

struct tmed_ctx;
struct BsStream;  // commit.hip: the context's blocksync batch stream

namespace tmed {

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 4 + 256;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct HostBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 4 + 256;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

inline int map_err(hipError_t e) {
  if (e == hipSuccess) return TMED_OK;
  if (e == hipErrorOutOfMemory) return TMED_ENOMEM;
  return TMED_EHIP;
}

// A validator set's key material resident in HBM.  Keys are appended
// (tmed_keyset_extend, the key-set cache's pool): the buffers hold `cap` keys, keys [0, n) are
// built, and the index of a key never changes.
struct Keyset {
  size_t n = 0, cap = 0;
  uint8_t *d_pub = nullptr;   // cap x 32 raw encodings (hashed into k)
  uint8_t *d_ok = nullptr;    // cap: Point.SetBytes accepted the key
  // The combs in chunks of kKeyChunkKeys keys (kernels.h kKeyChunk*): chunk c holds keys
  // [c * 512, c * 512 + keys[c]); every chunk but the last allocated one is full.  comb: signed
  // radix-256 comb of -A (kCombBytesPerKey a key).  comba: radix-2^12 comb of -A for the throughput
  // kernel (kernels.h kCombA*), keys [0, comba_n) built (at the set's first throughput batch and for
  // keys appended after it: keyset.hip comba_extend; none / comba_failed: TMED_KS_ACOMB=0 or no
  // memory -> the radix-256 comb).
  std::vector<int4 *> comb, comba;
  std::vector<uint32_t> comb_keys, comba_keys;
  // device: the chunk bases, tab_chunks of the radix-256 comb then tab_chunks of the radix-2^12
  // comb (the kernels' tables); entries are set on the set's stream as chunks appear.  tab_chunks:
  // kKeyChunksMax for the cache's pool, else the chunks the set's keys need (rounded up to a power
  // of two, grown with the set: keyset_reserve)
  int4 **d_tab = nullptr;
  int4 **h_tab = nullptr;  // pinned mirror (the source of the entries' copies)
  size_t tab_chunks = 0;
  size_t comba_n = 0;
  bool comba_failed = false;
  bool pooled = false;  // the context's key-set cache pool: not reachable through the public handles
  const int4 *const *comb_tab() const { return d_tab; }
  const int4 *const *comba_tab() const { return d_tab + tab_chunks; }
  size_t comb_room() const { return comb.empty() ? 0 : (comb.size() - 1) * (size_t)kKeyChunkKeys + comb_keys.back(); }
  size_t comba_room() const { return comba.empty() ? 0 : (comba.size() - 1) * (size_t)kKeyChunkKeys + comba_keys.back(); }
  // the row of entry (window w, j) of key v: radix-256 / radix-2^12
  int4 *comb_row(size_t v, size_t row) const {
    return comb[v >> kKeyChunkBits] + ((v & (kKeyChunkKeys - 1)) * kCombWindows * kCombEntries + row) * kCombEntryInt4;
  }
  int4 *comba_row_of(size_t v, size_t row) const {
    return comba[v >> kKeyChunkBits] + ((v & (kKeyChunkKeys - 1)) * kCombARowsPerKey + row) * kCombEntryInt4;
  }
};

int build_comb(tmed_ctx *c, const uint8_t *d_pubs, size_t n, int negate, uint8_t *d_ok, int4 *d_comb);
// Append m keys (host pointer) to k on stream s: adds comb chunks when needed (the pool's hold
// kKeyChunkKeys keys, up to max_cap; an explicit set's last chunk holds exactly its keys and is
// replaced by a larger one when the set grows), uploads the keys through the context's pinned key
// staging and queues their radix-256 combs; nothing waits for the build (later work on s is ordered
// behind it).  TMED_EINVAL past max_cap keys.
int keyset_append(tmed_ctx *c, Keyset &k, const uint8_t *pubkeys, size_t m, hipStream_t s, size_t max_cap);
// Device bytes one key of a key set can take (radix-256 comb + radix-2^12 comb + encoding + flag).
size_t keyset_bytes_per_key(const tmed_ctx *c);
// The public key set of `handle` (nullptr for unknown and pooled handles).
Keyset *find_keyset(tmed_ctx *c, uint64_t handle);
// The commit seam's key-set cache (keycache.hip, keycache.h); every call below holds ctx->mu.
struct KeyCacheDev;
void keycache_destroy(tmed_ctx *c);
void bs_destroy(tmed_ctx *c);  // commit.hip: the blocksync batch stream (before keycache_destroy)
struct Lane;
void lane_release(Lane &L);    // keyset.hip: the second kernel lane's stream and scratch
bool lanes_on();               // keyset.hip: TMED_LANES != 1
void keycache_pin(tmed_ctx *c);    // a seam call resolving sets: no pool reset until it unpins
void keycache_unpin(tmed_ctx *c);
uint64_t keycache_pool_handle(const tmed_ctx *c);  // 0 before the first key is built
// KeyCache::find: read-only, callable from several threads while the caller holds ctx->mu (after
// keycache_touch has created the cache)
const KcSet *keycache_find(tmed_ctx *c, const KcKey &key);
// a cached set's keys equal pubs[0, n) byte for byte (read-only: safe from a call's threads under ctx->mu)
bool keycache_same_keys(const tmed_ctx *c, const KcSet &e, const uint8_t *pubs, size_t n);
uint64_t keycache_call_tick(tmed_ctx *c);                        // KeyCache::call_tick
void keycache_hits(tmed_ctx *c, size_t sets, size_t sigs);       // KeyCache::hits
void keycache_touch(tmed_ctx *c);
void keycache_hit(tmed_ctx *c, const KcSet &e, size_t sigs);  // KeyCache::hit
bool keycache_all_pooled(tmed_ctx *c, const uint8_t *pubs, size_t n);  // KeyCache::all_pooled
void keycache_defer(tmed_ctx *c, const uint8_t *pubs, size_t n, size_t sigs);  // KeyCache::defer
bool keycache_lookup(tmed_ctx *c, const uint8_t *pubs, size_t n, const KcKey &key, size_t sigs, bool may_reset,
                     uint64_t *handle, const KcSet *&hold, bool force_build = false);
int keycache_drain(tmed_ctx *c);  // build the keys queued behind generic calls (asynchronously)
void keycache_after_call(tmed_ctx *c);  // wake the context's key-build worker when keys are queued
size_t keycache_missing(tmed_ctx *c, const uint8_t *pubs, size_t n, std::unordered_set<Pub32, Pub32Hash> *seen);

// Commit-seam device path (f1): stage votes (key refs, signatures, per-commit templates,
// template index / flag / timestamp per vote), assemble sign-bytes on the device, verify
// (generic when keyset == 0, key-cached otherwise), return one byte per vote.
// Opt-in ZIP-215 rule (zip215.hip): batch equation by MSM, bisection, exact single-check fallback.
int zip215_verify_device(tmed_ctx *c, const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                         uint32_t n, uint8_t *out, hipStream_t s, bool msg_slots);

int verify_votes_device(tmed_ctx *c, uint64_t keyset, const uint8_t *keys, const uint8_t *sigs,
                        const uint8_t *tmpl, size_t n_tmpl, const uint32_t *tmpl_idx, const uint8_t *flags,
                        const int64_t *ts_sec, const int32_t *ts_nanos, uint32_t m, uint8_t *out);

// Zero-copy form of the same: votes_stage() returns pointers into the pinned staging area
// of one of the context's vote slots; the caller fills them; votes_enqueue() queues
// copy-in, assembly, verification and copy-out on the context stream; votes_collect()
// waits for that slot and returns the bits.  votes_launch() = enqueue + collect.  Three
// slots let a pipelined caller (tmed_blocksync_verify) stage batch b+1 on the host while
// the device copies batch b in and runs batch b-1.  The caller holds ctx->mu across stage..collect.
struct VoteStage {
  int slot = 0;
  Keyset *ks = nullptr;
  uint32_t m = 0;
  size_t n_tmpl = 0, total = 0;
  size_t o_key = 0, o_sig = 0, o_tmpl = 0, o_tidx = 0, o_flag = 0, o_sec = 0, o_nan = 0;
  uint8_t *key = nullptr, *sig = nullptr, *tmpl = nullptr, *flag = nullptr;
  uint32_t *tidx = nullptr;
  int64_t *sec = nullptr;
  int32_t *nan = nullptr;
  bool zc = false;  // the kernels read the pinned staging buffer directly (votes_enqueue)
  bool timed = true;  // kernel-time events recorded (tmed_last_kernel_ms)
  bool keys_checked = false;  // every key-set index < the key set's size (checked while staging)
  bool copy_timed = false;    // cp0 / cp1 recorded around the copy-in (TMED_TRACE)
  // Signature runs DMA'd straight from pinned caller memory (tmed_host_alloc / _register) into
  // the device copy of the sig array at dst (bytes from the sig array's start); the staging area
  // holds the rest.  sig_direct: every signature arrives that way (the staged sig region is not copied).
  struct Dma {
    size_t dst;
    const void *src;
    size_t bytes;
  };
  std::vector<Dma> dma;
  bool sig_direct = false;
  // Kernel lane: 0 = the context stream; 1 = the second kernel stream of the key-cached
  // throughput batches (its own scratch, ctx.h Lane), so consecutive batches of the pipelined seam
  // overlap on the device (one batch's small kernels beside the other's main kernel).
  int lane = 0;
};
// Batches of at least this many staged bytes are copied on the context's copy stream (and may take
// their signatures straight from pinned caller memory): votes_enqueue.
constexpr size_t kVoteCopyStreamMin = 1u << 20;
bool host_pinned(const void *p, size_t bytes);  // inside one tmed_host_alloc / _register range
// staged-vote batches up to this size skip the copies (kernels read / write pinned host memory)
constexpr size_t kVoteZeroCopyMax = 256u << 10;
// Raw host batches of at most this many signatures record no kernel-time events by default.
constexpr size_t kLatencyUntimedMax = 1024;
int votes_stage(tmed_ctx *c, uint64_t keyset, uint32_t m, size_t n_tmpl, VoteStage &st, int slot = 0);
// The shared radix-2^24 B comb (tmed_capi.hip), acquired on the first call; null: radix 2^16.
const int4 *ctx_bcomb24(tmed_ctx *c);
// Tests: microseconds of delay queued in front of the seam's producer-side copies (tmed_test_stream_delay).
uint32_t test_stream_delay_us();
int votes_enqueue(tmed_ctx *c, VoteStage &st);
int votes_collect(tmed_ctx *c, const VoteStage &st, uint8_t *out);
int votes_launch(tmed_ctx *c, VoteStage &st, uint8_t *out);
void free_keyset(Keyset &k);

}  // namespace tmed

namespace tmed {
struct VoteSlot {
  DevBuf d_votes, d_vmsg, d_off, d_out;
  HostBuf h_votes, h_out;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // around the device work of the slot's last batch
  hipEvent_t done = nullptr;                // after its copy-out
  hipEvent_t copied = nullptr;              // its staged votes are on the device (copy stream)
  hipEvent_t cp0 = nullptr, cp1 = nullptr;  // around its copy-in (TMED_TRACE only)
};
}  // namespace tmed

namespace tmed {
// The second kernel lane of the pipelined seam (VoteStage::lane 1): a stream and the scratch its
// key-cached throughput kernels write (prep hand-off, batched-finish buffers, key order), allocated
// at its first use.  Key-set pool buffers are shared read-only; pool growth (keyset_reserve)
// synchronises both lanes before it frees anything.
struct Lane {
  hipStream_t s = nullptr;
  int4 *d_prep = nullptr, *d_fin = nullptr, *d_fin_pre = nullptr;
  DevBuf d_korder;
  bool failed = false;  // no stream / memory: every batch stays on lane 0
};
}  // namespace tmed

struct tmed_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // H2D of staged votes, so batch b's copy overlaps b-1's kernels
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  float last_ms = 0.f;
  float last_copy_ms = 0.f, last_copy_gap_ms = 0.f;  // TMED_TRACE: copy-in of the last collected batch, copy end -> kernels
  hipEvent_t trace_t0 = nullptr;  // TMED_TRACE: origin of last_at (recorded by the pipelined seam)
  float last_at[4] = {0, 0, 0, 0};  // copy start, copy end, kernels start, kernels end (ms after trace_t0)
  std::mutex mu;
  int4 *d_bcomb = nullptr;  // signed radix-256 comb of +B (shared)
  int4 *d_b16 = nullptr;    // j*B, j = 0..32768 (main-kernel variant 5), built at init
  int4 *d_bcomb16 = nullptr;  // radix-2^16 comb of +B (key-cached throughput kernel), 67 MB
  int4 *d_b26 = nullptr;      // radix-2^26 B tables of the half-size main kernel (8.6 GB, shared per device)
  int4 *d_b24 = nullptr;      // radix-2^24 B comb of the key-cached main kernel (11.8 GB, shared per device)
  bool b24_tried = false;     // d_b24 acquired (or given up) at the first key-set load
  bool b24_on = true;         // TMED_B24 at tmed_init
  bool acomb_on = true;         // TMED_KS_ACOMB at tmed_init (radix-2^12 -A combs, keyset.hip comba_extend)
  // TMED_TEST_FAIL_KS_ALLOC=n at tmed_init (tests only): the context's n-th key-set device allocation
  // (keyset.hip ks_malloc: table, encodings, comb chunks, build scratch) reports out of memory
  int test_fail_ks_alloc = 0;
  int4 *d_slab = nullptr;
  int4 *d_prep = nullptr;
  int4 *d_fin = nullptr;      // batched-finish hand-off (kFinBytes)
  int4 *d_fin_pre = nullptr;  // batched-finish prefix products (kFinPreBytes)
  uint32_t slab_slots = 0;
  uint32_t chunk = 0;     // signatures per prep/main launch pair (0 = slab_slots); env TMED_CHUNK
  int main_waves = 6;     // main-kernel path (6: half-size scalars, verify_hs.h; 5: full-length Straus + finish); env TMED_MAIN_WAVES
  uint32_t lat_max = 24576;  // key-cached batches up to this size take the latency kernels (crossover ~32k,
                             // profiles/r01/session3/lat_sweep.jsonl); env TMED_LAT_MAX
  int4 *d_glat = nullptr;    // generic latency mode hand-off (kGLatHandBytes)
  uint32_t glat_max = 24576;  // generic batches up to this size take the latency kernels (crossover ~32k,
                              // profiles/r02/s6/sweep_glat*.jsonl); env TMED_GLAT_MAX
  bool timing = false;    // tmed_set_kernel_timing
  uint32_t last_hs_count = 0;  // signatures of the last half-size chunk in d_prep (tmed_window_stats)
  tmed::KernelTimer timer;
  tmed::DevBuf d_a, d_b, d_msg, d_off, d_out, d_c;
  tmed::HostBuf h_a, h_b, h_msg, h_off, h_out, h_c;
  tmed::VoteSlot vslot[3];  // the blocksync pipeline (commit.hip BsStream: two slots, three when the signatures go direct)
  BsStream *bs = nullptr;   // batches of submitted blocksync windows in flight (tmed_blocksync_submit)
  tmed::Lane lane1;         // the pipelined seam's second kernel lane (VoteStage::lane)
  tmed::DevBuf d_merkle_a, d_merkle_b, d_merkle_idx;  // Merkle level digests (ping-pong) + level indexes
  tmed::DevBuf d_korder;  // key-grouped order of a key-cached batch: counts / cursors + permutation
  tmed::DevBuf d_zip;     // ZIP-215 batch mode scratch (zip215.hip zip_bufs: points, digits, sort, buckets)
  bool zip_dense = false; // ZIP-215: the last large chunk had failures (zip215.hip: decide the next one singly first)
  tmed::HostBuf h_zip;    // pinned word: failures counted in the last singly decided chunk
  hipEvent_t zip_ev = nullptr;  // that count's copy (read at the next chunk)
  bool zip_count_pending = false;
  std::unordered_map<uint64_t, tmed::Keyset> keysets;
  uint64_t next_keyset = 1;
  tmed::KeyCacheDev *kc = nullptr;  // key-set cache of the commit seam (keycache.hip), created at first use
  bool kc_on = true;                // TMED_KEYCACHE at tmed_init / tmed_keycache_config
  size_t kc_budget = (size_t)160 << 30;  // its pool's HBM budget (~25k keys at 6.3 MB: a light client's and a replay's sets together)
  tmed::DevBuf d_kbases;            // comb-base scratch of keyset_append (ordered on the context stream)
  tmed::HostBuf h_kup;              // pinned staging of keys keyset_append uploads
  hipEvent_t kup_ev = nullptr;      // the last upload from h_kup (reused after it completes)
  // The verify scratch (slab, prep hand-off, finish buffers) is shared by every call on the
  // context, but the device-pointer entry points run on the CALLER's stream: each user of
  // the scratch first makes its stream wait for the previous user (scratch_ev, whatever its
  // stream), then records itself.  Both under mu.
  hipEvent_t scratch_ev = nullptr;
  bool scratch_foreign = false;  // the last user was a caller's stream (scratch_ev marks its end)
};

namespace tmed {
// Calls on the context's own stream are ordered by the stream itself; an event is recorded
// or waited on only when the user changes to or from a caller's stream.  (A caller's stream
// is only ever recorded on inside that caller's own call: it may be gone afterwards.)
inline hipError_t scratch_acquire(tmed_ctx *c, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (s == c->stream) {
    if (c->scratch_foreign) e = hipStreamWaitEvent(s, c->scratch_ev, 0);
  } else {
    if (!c->scratch_foreign) e = hipEventRecord(c->scratch_ev, c->stream);  // the tail covers its last use
    if (e == hipSuccess) e = hipStreamWaitEvent(s, c->scratch_ev, 0);
  }
  return e;
}
// Signatures in the last chunk launch_verify runs for an n-signature call (chunks of `chunk`
// inside blocks of kFinCap).
inline uint32_t last_chunk_count(uint32_t n, uint32_t chunk) {
  if (n == 0) return 0;
  const uint32_t m = n - (n - 1) / kFinCap * kFinCap;
  return m - (m - 1) / chunk * chunk;
}
// A generic (uncached-key) batch on stream s: the latency kernels (latency.hip) up to
// c->glat_max signatures, the throughput pipeline above.  Inside a scratch_acquire/release pair.
// va: assemble the vote sign-bytes inside the latency kernels (only when n <= glat_max, where
// generic_uses_glat says they run; the caller then skips assemble_votes).
inline bool generic_uses_glat(const tmed_ctx *c, uint32_t n) { return n <= c->glat_max; }
inline hipError_t generic_verify(tmed_ctx *c, const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs,
                                 const uint32_t *off, uint32_t n, uint8_t *out, hipStream_t s, bool msg_slots,
                                 KernelTimer *timer, const VoteAsm *va = nullptr) {
  if (generic_uses_glat(c, n)) {
    c->last_hs_count = 0;  // no half-size hand-off in d_prep (tmed_window_stats)
    return launch_verify_glat(pub, sig, msgs, off, n, out, c->d_bcomb16, c->d_glat, s, msg_slots, timer, va);
  }
  if (va) return hipErrorInvalidValue;
  hipError_t e = launch_verify(pub, sig, msgs, off, n, out, c->d_slab, c->slab_slots, BTabs{c->d_b16, c->d_bcomb16, c->d_b26},
                               c->d_prep, c->d_fin, c->d_fin_pre, s, c->chunk, c->main_waves, msg_slots, timer);
  c->last_hs_count = (e != hipSuccess || c->main_waves == 5) ? 0 : last_chunk_count(n, c->chunk);
  return e;
}
inline hipError_t scratch_release(tmed_ctx *c, hipStream_t s) {
  c->scratch_foreign = s != c->stream;
  return c->scratch_foreign ? hipEventRecord(c->scratch_ev, s) : hipSuccess;
}
}  // namespace tmed
