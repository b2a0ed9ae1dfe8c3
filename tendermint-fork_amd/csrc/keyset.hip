// keyset.hip — per-validator-set key cache (§8b "tmed_keyset_load").
//
// A validator set's keys are decoded once (Go Point.SetBytes rule) and each key
// gets a signed radix-256 comb of -A in HBM (528 KB/key; 10k validators = 5.3 GB
// of the 288 GB), so a verification needs 32 + 32 mixed additions and no
// doublings instead of ~256 doublings + 128 additions + a decompression.
// The reference has no such cache (it decodes A inside every Verify); callers
// key the cache by ValidatorSet.Hash() (types/validator_set.go:347-353).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>

#include "ctx.h"

using namespace tmed;

namespace tmed {

int build_comb(tmed_ctx *c, const uint8_t *d_pubs, size_t n, int negate, uint8_t *d_ok, int4 *d_comb) {
  int32_t *d_bases = nullptr;
  hipError_t e = hipMalloc((void **)&d_bases, n * kCombWindows * 40 * sizeof(int32_t));
  if (e == hipSuccess) e = launch_comb_bases(d_pubs, (uint32_t)n, negate, d_ok, d_bases, c->stream);
  if (e == hipSuccess) e = launch_comb_fill(d_bases, (uint32_t)n, d_comb, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (d_bases) (void)hipFree(d_bases);
  return map_err(e);
}

// Every key-set device allocation goes through here (TMED_TEST_FAIL_KS_ALLOC: the failure paths
// below are exercised by tests/test_gpu_keychunks.py).
static hipError_t ks_malloc(tmed_ctx *c, void **p, size_t bytes) {
  if (c->test_fail_ks_alloc > 0 && --c->test_fail_ks_alloc == 0) {
    *p = nullptr;
    return hipErrorOutOfMemory;
  }
  return hipMalloc(p, bytes);
}

static void free_chunks(std::vector<int4 *> &ch, std::vector<uint32_t> &keys) {
  for (int4 *p : ch) (void)hipFree(p);
  ch.clear();
  keys.clear();
}

void free_keyset(Keyset &k) {
  if (k.d_pub) (void)hipFree(k.d_pub);
  if (k.d_ok) (void)hipFree(k.d_ok);
  free_chunks(k.comb, k.comb_keys);
  free_chunks(k.comba, k.comba_keys);
  if (k.d_tab) (void)hipFree(k.d_tab);
  if (k.h_tab) (void)hipHostFree(k.h_tab);
  k = Keyset();
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Key-grouped visiting order for the throughput kernels (launch_key_order): the comb rows a
// signature reads are random 128-B lines of its key's 528-KB comb; with the signatures of a
// 10k-key set in random order the lanes in flight span the whole 5.3 GB and the main kernel
// ran 3.27 ms per 2^20 against 2.02 ms with them in key order (profiles/r03/s3).
static bool key_order_on(const Keyset &k, uint32_t n) {
  return n >= 4096 && k.n > 1 && k.n <= kKeyOrderMaxKeys;
}

// Chunks of one comb (kernels.h kKeyChunk*, bytes_per_key a key) with room for keys [0, want): a
// missing chunk c is allocated for min(kKeyChunkKeys, limit - c * 512) keys (limit >= want); a
// partial chunk too small for `want` is replaced by a larger one, its built keys (those below
// `built`) copied over on s and the old chunk left in `retired` (freed by the caller once the
// streams reading it are drained).  Each new base goes into the set's table, ordered on s.
static hipError_t chunks_grow(tmed_ctx *ctx, std::vector<int4 *> &ch, std::vector<uint32_t> &keys, int4 **h_tab, int4 **d_tab,
                              size_t want, size_t limit, size_t bytes_per_key, size_t built, hipStream_t s,
                              std::vector<void *> &retired) {
  for (size_t c = 0; c * kKeyChunkKeys < want; c++) {
    const size_t first = c * kKeyChunkKeys;
    const size_t need = std::min<size_t>(kKeyChunkKeys, want - first);
    if (c < ch.size() && keys[c] >= need) continue;
    const size_t alloc = std::min<size_t>(kKeyChunkKeys, std::max(need, limit - first));
    int4 *p = nullptr;
    hipError_t e = ks_malloc(ctx, (void **)&p, alloc * bytes_per_key);
    if (e != hipSuccess) return e;
    if (c < ch.size()) {
      const size_t nb = built > first ? std::min<size_t>(built - first, keys[c]) : 0;
      if (nb) e = hipMemcpyAsync(p, ch[c], nb * bytes_per_key, hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) {
        (void)hipFree(p);
        return e;
      }
      retired.push_back(ch[c]);
      ch[c] = p;
      keys[c] = (uint32_t)alloc;
    } else {
      ch.push_back(p);
      keys.push_back((uint32_t)alloc);
    }
    h_tab[c] = p;
    e = hipMemcpyAsync(d_tab + c, h_tab + c, sizeof(int4 *), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Free what chunks_grow / keyset_reserve replaced, after the streams that may read it (s, the
// context stream and the second kernel lane) are drained.
static hipError_t free_retired(tmed_ctx *c, std::vector<void *> &retired, hipStream_t s) {
  if (retired.empty()) return hipSuccess;
  hipError_t e = hipStreamSynchronize(s);
  if (e == hipSuccess && s != c->stream) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess && c->lane1.s && s != c->lane1.s) e = hipStreamSynchronize(c->lane1.s);
  for (void *p : retired) (void)hipFree(p);
  retired.clear();
  return e;
}

// The radix-2^12 comb gone (no memory for it): the radix-256 comb serves the set.
static void comba_drop(Keyset &k) {
  (void)hipGetLastError();
  (void)hipDeviceSynchronize();  // no kernel of either lane still reads them (a failure path only)
  free_chunks(k.comba, k.comba_keys);
  k.comba_n = 0;
}

// The key set's radix-2^12 comb (kernels.h kCombA*) for keys [comba_n, n), on stream s (queued
// in front of the batch that needs it; the bases scratch is freed after a sync of s): at the set's
// first throughput batch, then for keys appended after it.  Its chunks mirror the radix-256 comb's.
// TMED_KS_ACOMB=0 (read at tmed_init) keeps the radix-256 comb; so does a failed allocation
// (comba_failed).
static void comba_extend(tmed_ctx *c, Keyset &k, hipStream_t s) {
  if (!c->acomb_on || k.comba_failed || k.comba_n >= k.n) return;
  std::vector<void *> retired;
  hipError_t e = chunks_grow(c, k.comba, k.comba_keys, k.h_tab + k.tab_chunks, k.d_tab + k.tab_chunks, k.n,
                             k.comb_room(), kCombABytesPerKey, k.comba_n, s, retired);
  int32_t *bases = nullptr;
  const size_t m = k.n - k.comba_n;
  if (e == hipSuccess) e = ks_malloc(c, (void **)&bases, std::min<size_t>(m, kKeyChunkKeys) * kCombAWindows * 40 * sizeof(int32_t));
  for (size_t a = k.comba_n; e == hipSuccess && a < k.n;) {  // one launch pair per chunk the keys fall in
    const size_t end = std::min<size_t>(k.n, ((a >> kKeyChunkBits) + 1) * kKeyChunkKeys);
    e = launch_build_comba(k.d_pub + 32 * a, (uint32_t)(end - a), bases, k.comba_row_of(a, 0), s);
    a = end;
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (bases) (void)hipFree(bases);
  if (e == hipSuccess) e = free_retired(c, retired, s);
  if (e == hipSuccess) {
    k.comba_n = k.n;
  } else {  // an allocation failure leaves the radix-256 comb in use
    (void)hipGetLastError();
    (void)free_retired(c, retired, s);
    comba_drop(k);
    k.comba_failed = true;
  }
}

size_t keyset_bytes_per_key(const tmed_ctx *c) {
  return 33 + kCombBytesPerKey + (c->acomb_on ? kCombABytesPerKey : 0);
}

Keyset *find_keyset(tmed_ctx *c, uint64_t handle) {
  auto it = c->keysets.find(handle);
  return it == c->keysets.end() || it->second.pooled ? nullptr : &it->second;
}

// Room for keys [0, want): the encodings and flags (33 B a key) in new buffers when they are full
// (doubling up to `limit`, the built ones copied over), the radix-256 comb's chunks added
// (chunks_grow: nothing built moves, except the keys of a partial last chunk); a synchronisation of
// s and the second lane only when a replaced buffer is freed.  The radix-2^12 comb follows at the
// next throughput batch (comba_extend).
// The set's chunk tables (device + pinned mirror) with room for `chunks` chunks per comb: the
// cache's pool takes kKeyChunksMax at once (512 KB), an explicit set what its keys need (a
// 175-key set: 8 entries), doubled when tmed_keyset_extend outgrows it — the new tables take the
// old entries, the old device table is freed with the other replaced buffers (retired), the old
// pinned mirror after s has finished the copies made from it.
static hipError_t tables_reserve(tmed_ctx *c, Keyset &k, size_t chunks, hipStream_t s,
                                 std::vector<void *> &retired) {
  if (k.d_tab && chunks <= k.tab_chunks) return hipSuccess;
  size_t cap = 8;
  while (cap < chunks) cap <<= 1;
  cap = std::min<size_t>(cap, kKeyChunksMax);
  const size_t bytes = 2 * cap * sizeof(int4 *);
  int4 **d = nullptr, **h = nullptr;
  hipError_t e = ks_malloc(c, (void **)&d, bytes);
  if (e == hipSuccess) e = hipHostMalloc((void **)&h, bytes, hipHostMallocDefault);
  if (e != hipSuccess) {
    if (d) (void)hipFree(d);
    return e;
  }
  memset(h, 0, bytes);
  if (k.h_tab) {  // the old entries: radix-256 half, then the radix-2^12 half at its new offset
    memcpy(h, k.h_tab, k.tab_chunks * sizeof(int4 *));
    memcpy(h + cap, k.h_tab + k.tab_chunks, k.tab_chunks * sizeof(int4 *));
  }
  e = hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) {
    (void)hipFree(d);
    (void)hipHostFree(h);
    return e;
  }
  if (k.h_tab) {
    (void)hipStreamSynchronize(s);  // earlier entry copies read the old mirror
    (void)hipHostFree(k.h_tab);
  }
  if (k.d_tab) retired.push_back(k.d_tab);
  k.d_tab = d;
  k.h_tab = h;
  k.tab_chunks = cap;
  return hipSuccess;
}

static int keyset_reserve(tmed_ctx *c, Keyset &k, size_t want, size_t limit, hipStream_t s) {
  hipError_t e = hipSuccess;
  std::vector<void *> retired;
  e = tables_reserve(c, k, k.pooled ? (size_t)kKeyChunksMax : (limit + kKeyChunkKeys - 1) / kKeyChunkKeys, s,
                     retired);
  if (e != hipSuccess) {
    (void)free_retired(c, retired, s);
    return map_err(e);
  }
  if (want > k.cap) {
    const size_t cap = std::max(want, std::min(2 * k.cap, limit));
    uint8_t *pub = nullptr, *ok = nullptr;
    e = ks_malloc(c, (void **)&pub, cap * 32);
    if (e == hipSuccess) e = ks_malloc(c, (void **)&ok, cap);
    if (e == hipSuccess && k.n) {
      e = hipMemcpyAsync(pub, k.d_pub, k.n * 32, hipMemcpyDeviceToDevice, s);
      if (e == hipSuccess) e = hipMemcpyAsync(ok, k.d_ok, k.n, hipMemcpyDeviceToDevice, s);
    }
    if (e != hipSuccess) {
      if (pub) (void)hipFree(pub);
      if (ok) (void)hipFree(ok);
      return map_err(e);
    }
    if (k.d_pub) retired.push_back(k.d_pub);
    if (k.d_ok) retired.push_back(k.d_ok);
    k.d_pub = pub;
    k.d_ok = ok;
    k.cap = cap;
  }
  e = chunks_grow(c, k.comb, k.comb_keys, k.h_tab, k.d_tab, want, limit, kCombBytesPerKey, k.n, s, retired);
  const hipError_t ef = free_retired(c, retired, s);
  return map_err(e != hipSuccess ? e : ef);
}

int keyset_append(tmed_ctx *c, Keyset &k, const uint8_t *pubkeys, size_t m, hipStream_t s, size_t max_cap) {
  if (m == 0) return TMED_OK;
  max_cap = std::min<size_t>(max_cap, 0xffffffu);
  if (k.n + m > max_cap) return TMED_EINVAL;
  // the pool's chunks are whole up to its budget; an explicit set holds exactly its keys
  int rc = keyset_reserve(c, k, k.n + m, k.pooled ? max_cap : k.n + m, s);
  if (rc != TMED_OK) return rc;
  // the pinned key staging and the comb-base scratch are reused once the previous build is done
  hipError_t e = hipSuccess;
  if (c->kup_ev) e = hipEventSynchronize(c->kup_ev);
  else e = hipEventCreateWithFlags(&c->kup_ev, hipEventDisableTiming);
  const size_t bbytes = m * kCombWindows * 40 * sizeof(int32_t);
  if (e == hipSuccess && bbytes > c->d_kbases.cap) e = c->d_kbases.ensure(bbytes);
  if (e == hipSuccess) e = c->h_kup.ensure(m * 32);
  if (e != hipSuccess) return map_err(e);
  memcpy(c->h_kup.p, pubkeys, m * 32);
  e = launch_test_delay(s, test_stream_delay_us());  // tests only (0): the appended keys land late
  if (e == hipSuccess) e = hipMemcpyAsync(k.d_pub + 32 * k.n, c->h_kup.p, m * 32, hipMemcpyHostToDevice, s);
  int32_t *bases = (int32_t *)c->d_kbases.p;
  if (e == hipSuccess) e = launch_comb_bases(k.d_pub + 32 * k.n, (uint32_t)m, /*negate=*/1, k.d_ok + k.n, bases, s);
  for (size_t a = k.n; e == hipSuccess && a < k.n + m;) {  // one fill launch per chunk the keys fall in
    const size_t end = std::min<size_t>(k.n + m, ((a >> kKeyChunkBits) + 1) * kKeyChunkKeys);
    e = launch_comb_fill(bases + (a - k.n) * kCombWindows * 40, (uint32_t)(end - a), k.comb_row(a, 0), s);
    a = end;
  }
  if (e == hipSuccess) e = hipEventRecord(c->kup_ev, s);
  if (e != hipSuccess) return map_err(e);
  k.n += m;
  return TMED_OK;
}

// Key-cached batch on the context's stream: latency kernels for small batches (C1: one
// commit), the throughput kernels (prep / comb main / batched finish) above c->lat_max.
static hipError_t keyset_verify(tmed_ctx *c, Keyset &k, const uint32_t *d_idx, const uint8_t *d_sig,
                                const uint8_t *d_msgs, const uint32_t *d_off, uint32_t n, uint8_t *d_out,
                                hipStream_t s, bool msg_slots, const VoteAsm *va = nullptr, Lane *lane = nullptr) {
  c->last_hs_count = 0;  // d_prep now holds another path's hand-off (tmed_window_stats)
  if (n <= c->lat_max)
    return launch_verify_keyset_lat(d_idx, (uint32_t)k.n, k.d_pub, k.d_ok, k.comb_tab(), c->d_bcomb, d_sig, d_msgs, d_off, n, d_out,
                                    c->d_fin, c->d_fin_pre, s, msg_slots, va);
  if (va) return hipErrorInvalidValue;
  if (c->d_b24) comba_extend(c, k, s);
  const int4 *const *comba = c->d_b24 && !k.comba.empty() && k.comba_n == k.n ? k.comba_tab() : nullptr;
  KernelTimer *timer = (c->timing && !msg_slots) ? &c->timer : nullptr;
  uint32_t *perm = nullptr, *scratch = nullptr;
  DevBuf &korder = lane ? lane->d_korder : c->d_korder;
  if (key_order_on(k, n)) {
    const size_t sw = key_order_scratch_words(n, (uint32_t)k.n);
    hipError_t e = korder.ensure((sw + (size_t)n) * 4);
    if (e != hipSuccess) return e;
    scratch = (uint32_t *)korder.p;
    perm = scratch + sw;
  }
  // (the key order runs in front of each chunk's prep and is charged to prep by the timer)
  return launch_verify_keyset(d_idx, (uint32_t)k.n, k.d_pub, k.d_ok, k.comb_tab(), c->d_bcomb16, d_sig, d_msgs, d_off, n,
                              d_out, lane ? lane->d_prep : c->d_prep, c->slab_slots, lane ? lane->d_fin : c->d_fin,
                              lane ? lane->d_fin_pre : c->d_fin_pre, s, msg_slots, timer, perm, scratch, c->d_b24,
                              comba);
}

static std::atomic<uint32_t> g_test_stream_delay{0};
uint32_t test_stream_delay_us() { return g_test_stream_delay.load(std::memory_order_relaxed); }

int votes_stage(tmed_ctx *c, uint64_t keyset, uint32_t m, size_t n_tmpl, VoteStage &st, int slot) {
  st.slot = slot;
  st.m = m;
  st.n_tmpl = n_tmpl;
  st.ks = nullptr;
  st.keys_checked = false;
  st.dma.clear();
  st.sig_direct = false;
  if (keyset) {
    auto it = c->keysets.find(keyset);
    if (it == c->keysets.end()) return TMED_ENOKEYSET;
    st.ks = &it->second;
  }
  (void)hipSetDevice(c->device);
  VoteSlot &vs = c->vslot[slot];
  const size_t key_bytes = keyset ? (size_t)m * 4 : (size_t)m * 32;
  st.o_key = 0;
  st.o_sig = align256(st.o_key + key_bytes);
  st.o_tmpl = align256(st.o_sig + (size_t)m * 64);
  st.o_tidx = align256(st.o_tmpl + n_tmpl * kVoteTmplBytes);
  st.o_flag = align256(st.o_tidx + (size_t)m * 4);
  st.o_sec = align256(st.o_flag + m);
  st.o_nan = align256(st.o_sec + (size_t)m * 8);
  st.total = align256(st.o_nan + (size_t)m * 4);
  hipError_t e = vs.d_votes.ensure(st.total);
  if (e == hipSuccess) e = vs.h_votes.ensure(st.total);
  if (e == hipSuccess) e = vs.d_vmsg.ensure((size_t)m * kVoteSlot);
  if (e == hipSuccess) e = vs.d_off.ensure((size_t)m * 4);
  if (e == hipSuccess) e = vs.d_out.ensure(m);
  if (e == hipSuccess) e = vs.h_out.ensure(m);
  if (e == hipSuccess && !vs.ev0) e = hipEventCreate(&vs.ev0);
  if (e == hipSuccess && !vs.ev1) e = hipEventCreate(&vs.ev1);
  if (e == hipSuccess && !vs.done) e = hipEventCreateWithFlags(&vs.done, hipEventDisableTiming);
  if (e == hipSuccess && !vs.copied) e = hipEventCreateWithFlags(&vs.copied, hipEventDisableTiming);
  if (e != hipSuccess) return map_err(e);
  uint8_t *h = (uint8_t *)vs.h_votes.p;
  st.key = h + st.o_key;
  st.sig = h + st.o_sig;
  st.tmpl = h + st.o_tmpl;
  st.tidx = (uint32_t *)(h + st.o_tidx);
  st.flag = h + st.o_flag;
  st.sec = (int64_t *)(h + st.o_sec);
  st.nan = (int32_t *)(h + st.o_nan);
  return TMED_OK;
}

namespace {
// TMED_TRACE: host time of each queueing step of votes_enqueue (one line per large batch).
struct SlowStep {
  bool on;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  char buf[256];
  int len = 0;
  void lap(const char *what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    const double us = std::chrono::duration<double, std::micro>(n - t).count();
    if (len < (int)sizeof(buf) - 40) len += snprintf(buf + len, sizeof(buf) - len, " %s=%.0fus", what, us);
    t = n;
  }
  void emit(uint32_t m) {
    if (on && len) fprintf(stderr, "[tmed] votes_enqueue m=%u%.*s\n", m, len, buf);
  }
};
}  // namespace

// The second kernel lane, created at its first use (false: unavailable, the batch takes lane 0).
static bool lane1_ready(tmed_ctx *c) {
  Lane &L = c->lane1;
  if (L.s) return true;
  if (L.failed) return false;
  hipError_t e = hipStreamCreateWithFlags(&L.s, hipStreamNonBlocking);

  if (e == hipSuccess) e = hipMalloc((void **)&L.d_prep, (size_t)c->slab_slots * kPrepSlotBytes + kPrepTailBytes);
  if (e == hipSuccess) e = hipMalloc((void **)&L.d_fin, kFinBytes);
  if (e == hipSuccess) e = hipMalloc((void **)&L.d_fin_pre, kFinPreBytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    lane_release(L);
    L.failed = true;
    return false;
  }
  return true;
}

bool lanes_on() {
  static const bool on = [] {
    const char *v = getenv("TMED_LANES");
    return !(v && v[0] == '1');
  }();
  return on;
}

void lane_release(Lane &L) {
  if (L.s) {
    (void)hipStreamSynchronize(L.s);
    (void)hipStreamDestroy(L.s);
  }
  for (int4 *p : {L.d_prep, L.d_fin, L.d_fin_pre})
    if (p) (void)hipFree(p);
  L.d_korder.release();
  L.s = nullptr;
  L.d_prep = L.d_fin = L.d_fin_pre = nullptr;
}

int votes_enqueue(tmed_ctx *c, VoteStage &st) {
  static const bool trace_steps = getenv("TMED_TRACE") != nullptr;
  SlowStep slow{trace_steps && st.total >= kVoteCopyStreamMin};
  const uint32_t m = st.m;
  if (st.ks && !st.keys_checked)
    for (uint32_t j = 0; j < m; j++)
      if (((const uint32_t *)st.key)[j] >= st.ks->n) return TMED_EINVAL;
  VoteSlot &vs = c->vslot[st.slot];
  uint8_t *d = (uint8_t *)vs.d_votes.p;
  c->last_hs_count = 0;  // the commit seam reuses d_prep (tmed_window_stats)
  // lane 1: key-cached throughput batches only (the latency kernels and the generic path use the
  // context's scratch on lane 0)
  if (st.lane == 1 && (!st.ks || st.m <= c->lat_max || !lane1_ready(c))) st.lane = 0;
  Lane *lane = st.lane == 1 ? &c->lane1 : nullptr;
  hipStream_t s = lane ? lane->s : c->stream;
  // A large copy runs on the copy stream, so it overlaps the kernels of the batch queued
  // before (the other slot; this slot's previous batch was collected before it was
  // restaged).  A small one (a single commit) stays on the kernel stream: the cross-stream
  // event would cost more latency than the copy.
  // A batch of up to kVoteZeroCopyMax staged bytes (a single commit: C1) is not copied at all:
  // the kernels read the pinned staging buffer over the bus and write the decisions into the
  // pinned result buffer, which saves the copy-in and copy-out latencies (~15 us of a 100-us
  // commit).
  st.zc = st.total <= kVoteZeroCopyMax;
  uint8_t *out_dev = (uint8_t *)vs.d_out.p;
  hipError_t e = hipSuccess;
  if (st.zc) {
    void *dh = nullptr, *dout = nullptr;
    e = hipHostGetDevicePointer(&dh, vs.h_votes.p, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&dout, vs.h_out.p, 0);
    if (e == hipSuccess) { d = (uint8_t *)dh; out_dev = (uint8_t *)dout; }
  } else if (st.total >= kVoteCopyStreamMin) {
    static const bool trace = getenv("TMED_TRACE") != nullptr;
    st.copy_timed = trace;
    if (trace && !vs.cp0 && e == hipSuccess) e = hipEventCreate(&vs.cp0);
    if (trace && !vs.cp1 && e == hipSuccess) e = hipEventCreate(&vs.cp1);
    if (trace && e == hipSuccess) e = hipEventRecord(vs.cp0, c->copy_stream);
    if (e == hipSuccess) e = launch_test_delay(c->copy_stream, test_stream_delay_us());  // tests only (0)
    const uint8_t *h = (const uint8_t *)vs.h_votes.p;
    if (st.sig_direct) {  // the staged area without its (unused) signature region
      if (e == hipSuccess) e = hipMemcpyAsync(d, h, st.o_sig, hipMemcpyHostToDevice, c->copy_stream);
      if (e == hipSuccess)
        e = hipMemcpyAsync(d + st.o_tmpl, h + st.o_tmpl, st.total - st.o_tmpl, hipMemcpyHostToDevice, c->copy_stream);
    } else if (e == hipSuccess) {
      e = hipMemcpyAsync(d, h, st.total, hipMemcpyHostToDevice, c->copy_stream);
    }
    // Signature runs straight from pinned caller memory.  Each copy command costs the DMA engine
    // ~10 us (tools/copy_overlap_probe.py: 72 MB in 1.4 ms as one copy, 2.6 ms as 128), so runs
    // of equal length at a constant source stride (one per block of a blocksync batch, every
    // commit of the same size) go as one 2-D copy.
    const size_t nd = st.dma.size();
    for (size_t r = 0; r < nd && e == hipSuccess;) {
      const VoteStage::Dma &a = st.dma[r];
      const uint8_t *s0 = (const uint8_t *)a.src;
      size_t k = r + 1;
      const ptrdiff_t pitch = k < nd ? (const uint8_t *)st.dma[k].src - s0 : 0;
      if (pitch >= (ptrdiff_t)a.bytes)
        while (k < nd && st.dma[k].bytes == a.bytes && st.dma[k].dst == a.dst + (k - r) * a.bytes &&
               (const uint8_t *)st.dma[k].src == s0 + (ptrdiff_t)(k - r) * pitch)
          k++;
      // the 2-D source region spans the gaps between the runs: one copy only when it lies inside a
      // single pinned range (runs in separate tmed_host_alloc / _register ranges go one by one)
      if (k - r >= 2 && !host_pinned(s0, (size_t)pitch * (k - r - 1) + a.bytes)) k = r + 1;
      if (k - r >= 2) {
        e = hipMemcpy2DAsync(d + st.o_sig + a.dst, a.bytes, s0, (size_t)pitch, a.bytes, k - r, hipMemcpyHostToDevice,
                             c->copy_stream);
      } else {
        e = hipMemcpyAsync(d + st.o_sig + a.dst, s0, a.bytes, hipMemcpyHostToDevice, c->copy_stream);
        k = r + 1;
      }
      r = k;
    }
    if (trace && e == hipSuccess) e = hipEventRecord(vs.cp1, c->copy_stream);
    if (e == hipSuccess) e = hipEventRecord(vs.copied, c->copy_stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, vs.copied, 0);
  } else {
    e = hipMemcpyAsync(d, vs.h_votes.p, st.total, hipMemcpyHostToDevice, s);
  }
  slow.lap("copy-in");
  // lane 0 orders itself with the context's other scratch users; lane 1 has its own scratch but
  // reads the key-set pool, whose keys are appended on the context stream (keyset_append: kup_ev)
  if (e == hipSuccess && !lane) e = scratch_acquire(c, s);
  if (e == hipSuccess && lane && c->kup_ev) e = hipStreamWaitEvent(s, c->kup_ev, 0);
  slow.lap("scratch_acquire");
  // Timing events cost ~8 us of a single commit's latency (C1 generic 249 -> 239 us, keyed
  // 97 -> 88 us): a zero-copy batch records them only under tmed_set_kernel_timing.
  st.timed = !st.zc || c->timing;
  if (e == hipSuccess && st.timed) e = hipEventRecord(vs.ev0, s);
  // the latency kernels (generic and key-cached) assemble the sign-bytes in their hash lanes (no
  // launch in front)
  const VoteAsm va{d + st.o_tmpl, (const uint32_t *)(d + st.o_tidx), d + st.o_flag, (const int64_t *)(d + st.o_sec),
                   (const int32_t *)(d + st.o_nan)};
  const bool fused = st.ks ? m <= c->lat_max : generic_uses_glat(c, m);
  if (e == hipSuccess && !fused)
    e = launch_assemble_votes(va.tmpl, va.tmpl_idx, va.flags, va.ts_sec, va.ts_nanos, m, (uint8_t *)vs.d_vmsg.p,
                              (uint32_t *)vs.d_off.p, s);
  slow.lap("assemble");
  if (e == hipSuccess) {
    if (st.ks)
      e = keyset_verify(c, *st.ks, (const uint32_t *)(d + st.o_key), d + st.o_sig, (const uint8_t *)vs.d_vmsg.p,
                        (const uint32_t *)vs.d_off.p, m, out_dev, s, /*msg_slots=*/true, fused ? &va : nullptr, lane);
    else
      e = generic_verify(c, d + st.o_key, d + st.o_sig, (const uint8_t *)vs.d_vmsg.p, (const uint32_t *)vs.d_off.p, m,
                         out_dev, s, /*msg_slots=*/true, nullptr, fused ? &va : nullptr);
  }
  slow.lap("verify launches");
  if (e == hipSuccess && st.timed) e = hipEventRecord(vs.ev1, s);
  if (e == hipSuccess && !lane) e = scratch_release(c, s);
  if (e == hipSuccess && !st.zc) e = hipMemcpyAsync(vs.h_out.p, vs.d_out.p, m, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipEventRecord(vs.done, s);
  slow.lap("copy-out");
  slow.emit(m);
  return map_err(e);
}

int votes_collect(tmed_ctx *c, const VoteStage &st, uint8_t *out) {
  VoteSlot &vs = c->vslot[st.slot];
  hipError_t e = hipEventSynchronize(vs.done);  // this slot only: a later batch may be queued behind it
  if (e != hipSuccess) return map_err(e);
  c->last_ms = 0.f;
  if (st.timed) (void)hipEventElapsedTime(&c->last_ms, vs.ev0, vs.ev1);
  c->last_copy_ms = c->last_copy_gap_ms = 0.f;
  if (st.copy_timed) {
    (void)hipEventElapsedTime(&c->last_copy_ms, vs.cp0, vs.cp1);
    if (st.timed) (void)hipEventElapsedTime(&c->last_copy_gap_ms, vs.cp1, vs.ev0);
    if (c->trace_t0) {
      (void)hipEventElapsedTime(&c->last_at[0], c->trace_t0, vs.cp0);
      (void)hipEventElapsedTime(&c->last_at[1], c->trace_t0, vs.cp1);
      if (st.timed) (void)hipEventElapsedTime(&c->last_at[2], c->trace_t0, vs.ev0);
      if (st.timed) (void)hipEventElapsedTime(&c->last_at[3], c->trace_t0, vs.ev1);
    }
  }
  memcpy(out, vs.h_out.p, st.m);
  return TMED_OK;
}

int votes_launch(tmed_ctx *c, VoteStage &st, uint8_t *out) {
  int rc = votes_enqueue(c, st);
  if (rc == TMED_OK) rc = votes_collect(c, st, out);
  return rc;
}

int verify_votes_device(tmed_ctx *c, uint64_t keyset, const uint8_t *keys, const uint8_t *sigs, const uint8_t *tmpl,
                        size_t n_tmpl, const uint32_t *tmpl_idx, const uint8_t *flags, const int64_t *ts_sec,
                        const int32_t *ts_nanos, uint32_t m, uint8_t *out) {
  if (m == 0) return TMED_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  VoteStage st;
  int rc = votes_stage(c, keyset, m, n_tmpl, st);
  if (rc != TMED_OK) return rc;
  memcpy(st.key, keys, keyset ? (size_t)m * 4 : (size_t)m * 32);
  memcpy(st.sig, sigs, (size_t)m * 64);
  memcpy(st.tmpl, tmpl, n_tmpl * kVoteTmplBytes);
  memcpy(st.tidx, tmpl_idx, (size_t)m * 4);
  memcpy(st.flag, flags, m);
  memcpy(st.sec, ts_sec, (size_t)m * 8);
  memcpy(st.nan, ts_nanos, (size_t)m * 4);
  return votes_launch(c, st, out);
}

}  // namespace tmed

extern "C" {

int tmed_keyset_load(tmed_ctx *c, const uint8_t *pubkeys, size_t n, uint64_t *handle) {
  if (!c || !handle || (n && !pubkeys) || n > 0xffffffu) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  (void)hipSetDevice(c->device);
  Keyset k;
  // room for one key at least: an index past an empty set still reads key 0's rows (and rejects)
  int rc = keyset_reserve(c, k, n ? n : 1, n ? n : 1, c->stream);
  if (rc == TMED_OK) rc = keyset_append(c, k, pubkeys, n, c->stream, n);
  if (rc == TMED_OK) rc = map_err(hipStreamSynchronize(c->stream));
  if (rc == TMED_OK) (void)ctx_bcomb24(c);  // the shared radix-2^24 B comb (null: radix 2^16)
  if (rc != TMED_OK) {
    free_keyset(k);
    return rc;
  }
  const uint64_t h = c->next_keyset++;
  c->keysets[h] = k;
  *handle = h;
  return TMED_OK;
}

int tmed_keyset_extend(tmed_ctx *c, uint64_t handle, const uint8_t *pubkeys, size_t n, uint32_t *first_index) {
  if (!c || (n && !pubkeys)) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  Keyset *k = find_keyset(c, handle);
  if (!k) return TMED_ENOKEYSET;
  if (first_index) *first_index = (uint32_t)k->n;
  if (n == 0) return TMED_OK;
  (void)hipSetDevice(c->device);
  int rc = keyset_append(c, *k, pubkeys, n, c->stream, 0xffffffu);
  if (rc == TMED_OK) rc = map_err(hipStreamSynchronize(c->stream));
  return rc;
}

int tmed_keyset_free(tmed_ctx *c, uint64_t handle) {
  if (!c) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  Keyset *k = find_keyset(c, handle);
  if (!k) return TMED_ENOKEYSET;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (c->lane1.s) (void)hipStreamSynchronize(c->lane1.s);
  free_keyset(*k);
  c->keysets.erase(handle);
  return TMED_OK;
}

int tmed_verify_batch_keyset_device(tmed_ctx *c, uint64_t handle, const uint32_t *d_val_idx, const uint8_t *d_sigs,
                                    const uint8_t *d_msgs, const uint32_t *d_msg_off, size_t n, uint8_t *d_out,
                                    void *stream) {
  if (!c) return TMED_EINVAL;
  if (n == 0) return TMED_OK;
  if (!d_val_idx || !d_sigs || !d_msgs || !d_msg_off || !d_out || n > 0xffffffffu) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  Keyset *kp = find_keyset(c, handle);
  if (!kp) return TMED_ENOKEYSET;
  Keyset &k = *kp;
  (void)hipSetDevice(c->device);
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  if (c->timing) c->timer.n = 0;
  // (one lane: split over both kernel lanes in halves, a 2^20 batch ran 3 % slower — the halves'
  // key orders spread each kernel's comb reads — profiles/r04/s10/ab_keyed_lanes.jsonl)
  hipError_t e = scratch_acquire(c, s);
  if (e == hipSuccess) e = keyset_verify(c, k, d_val_idx, d_sigs, d_msgs, d_msg_off, (uint32_t)n, d_out, s, false);
  if (e == hipSuccess) e = scratch_release(c, s);
  return map_err(e);
}

int tmed_verify_batch_keyset(tmed_ctx *c, uint64_t handle, const uint32_t *val_idx, const uint8_t *sigs,
                             const uint32_t *sig_lens, const uint8_t *msgs, const uint32_t *off, size_t n,
                             uint8_t *out) {
  if (!c || !out) return TMED_EINVAL;
  if (n == 0) return TMED_OK;
  if (!val_idx || !sigs || !off || n > 0xffffffffu) return TMED_EINVAL;
  for (size_t i = 0; i < n; i++)
    if (off[i + 1] < off[i]) return TMED_EINVAL;
  const size_t mbytes = off[n];
  if (mbytes && !msgs) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  Keyset *kp = find_keyset(c, handle);
  if (!kp) return TMED_ENOKEYSET;
  Keyset &k = *kp;
  for (size_t i = 0; i < n; i++)
    if (val_idx[i] >= k.n) return TMED_EINVAL;
  (void)hipSetDevice(c->device);
  hipError_t e = hipSuccess;
  const size_t moff = (n + 1) * 4;
  for (auto &pr : {std::make_pair(&c->d_a, n * 4), std::make_pair(&c->d_b, n * 64),
                   std::make_pair(&c->d_msg, mbytes + 16), std::make_pair(&c->d_off, moff),
                   std::make_pair(&c->d_out, n)})
    if (e == hipSuccess) e = pr.first->ensure(pr.second);
  for (auto &pr : {std::make_pair(&c->h_a, n * 4), std::make_pair(&c->h_b, n * 64),
                   std::make_pair(&c->h_msg, mbytes + 16), std::make_pair(&c->h_off, moff),
                   std::make_pair(&c->h_out, n)})
    if (e == hipSuccess) e = pr.first->ensure(pr.second);
  if (e != hipSuccess) return map_err(e);
  memcpy(c->h_a.p, val_idx, n * 4);
  memcpy(c->h_b.p, sigs, n * 64);
  if (mbytes) memcpy(c->h_msg.p, msgs, mbytes);
  memcpy(c->h_off.p, off, moff);
  hipStream_t s = c->stream;
  e = hipMemcpyAsync(c->d_a.p, c->h_a.p, n * 4, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->d_b.p, c->h_b.p, n * 64, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && mbytes) e = hipMemcpyAsync(c->d_msg.p, c->h_msg.p, mbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->d_off.p, c->h_off.p, moff, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = scratch_acquire(c, s);
  if (e == hipSuccess) e = hipEventRecord(c->ev0, s);
  if (e == hipSuccess)
    e = keyset_verify(c, k, (const uint32_t *)c->d_a.p, (const uint8_t *)c->d_b.p, (const uint8_t *)c->d_msg.p,
                      (const uint32_t *)c->d_off.p, (uint32_t)n, (uint8_t *)c->d_out.p, s, false);
  if (e == hipSuccess) e = hipEventRecord(c->ev1, s);
  if (e == hipSuccess) e = scratch_release(c, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->h_out.p, c->d_out.p, n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return map_err(e);
  (void)hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1);
  memcpy(out, c->h_out.p, n);
  if (sig_lens)
    for (size_t i = 0; i < n; i++)
      if (sig_lens[i] != 64) out[i] = 0;  // crypto/ed25519/ed25519.go:150-152
  return TMED_OK;
}

}  // extern "C"

extern "C" void tmed_test_stream_delay(int us) { tmed::g_test_stream_delay.store(us < 0 ? 0u : (uint32_t)us); }
