// commit.hip — the drop-in seam: ValidatorSet.VerifyCommit* over one GPU batch (host C++).
//
// Reference loops restated (types/validator_set.go):
//   VerifyCommit               :667-714  verify EVERY non-absent signature, tally ForBlock power
//   VerifyCommitLight          :722-765  ForBlock only, return nil as soon as tally > 2/3
//   VerifyCommitLightTrusting  :775-826  ForBlock, GetByAddress (:270-278), double-vote check
//                                        before verifying, return nil once tally > trust level
// Per batch of requests:
//   1. the reference prechecks (set size, height, BlockID.Equals, zero denominator, safeMul)
//   2. candidate selection = exactly the signatures the loop can reach: for the early-exit
//      loops, the ForBlock prefix up to the crossing computed as if every signature were
//      valid (if one in that prefix is invalid the loop stops there anyway; if none is,
//      it stops at the crossing), and for Trusting also up to the first double vote
//   3. CanonicalVote sign-bytes (signbytes.hip), ONE device batch (tmed_verify_batch)
//   4. replay of the reference loop over the validity bits — first-error index, early
//      exit, Got/Needed and error kinds come out identical by construction.
#include <atomic>
#include <chrono>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/tmed25519.h"
#include "ctx.h"
#include "host_pool.h"
#include "signbytes.h"

#include "seam_host.h"

// Host fallback of the GPU verifier for templates the device assembler cannot hold.
static int ctx_verify_host_msgs(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t n, const Cands &cands,
                                uint8_t *valid) {
  CandBatch cb;
  int rc = build_cand_batch(reqs, n, cands, cb);
  if (rc != TMED_OK) return rc;
  std::unordered_map<uint64_t, std::vector<uint32_t>> groups;
  for (size_t k = 0; k < cb.m; k++) groups[cb.keyset[k]].push_back((uint32_t)k);
  for (auto &g : groups) {
    const std::vector<uint32_t> &ix = g.second;
    const size_t m = ix.size();
    std::vector<uint8_t> pubs(m * 32), sigs(m * 64), msgs, out(m);
    std::vector<uint32_t> lens(m), offs(m + 1), vidx(m);
    size_t total = 0;
    for (size_t j = 0; j < m; j++) total += cb.offs[ix[j] + 1] - cb.offs[ix[j]];
    msgs.resize(total + 16);
    total = 0;
    for (size_t j = 0; j < m; j++) {
      const uint32_t k = ix[j];
      memcpy(&pubs[j * 32], &cb.pubs[k * 32], 32);
      memcpy(&sigs[j * 64], &cb.sigs[k * 64], 64);
      lens[j] = cb.lens[k];
      vidx[j] = cb.val_idx[k];
      const uint32_t len = cb.offs[k + 1] - cb.offs[k];
      offs[j] = (uint32_t)total;
      memcpy(&msgs[total], &cb.msgs[cb.offs[k]], len);
      total += len;
    }
    offs[m] = (uint32_t)total;
    rc = g.first == 0 ? tmed_verify_batch(ctx, pubs.data(), sigs.data(), lens.data(), msgs.data(), offs.data(), m,
                                          out.data())
                      : tmed_verify_batch_keyset(ctx, g.first, vidx.data(), sigs.data(), lens.data(), msgs.data(),
                                                 offs.data(), m, out.data());
    if (rc != TMED_OK) return rc;
    for (size_t j = 0; j < m; j++) valid[ix[j]] = out[j];
  }
  return TMED_OK;
}

// Device staging of one group's candidates into vote slot `slot`: sign-bytes are assembled on
// the device from per-commit templates, so only key references, signatures,
// flags and timestamps cross PCIe; they are written straight from the request arrays into the
// pinned staging area, run by run (multi-threaded for large batches).  The caller holds ctx->mu.
constexpr size_t kDmaMinRun = 256;  // signatures (16 KB)
static int stage_group(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t n, const Cands &cands, const Group &grp,
                       uint64_t keyset, const Templates &tp, int slot, tmed::VoteStage &st) {
  const bool keyed = keyset != 0;
  const uint32_t m = (uint32_t)grp.size(cands);
  int rc = tmed::votes_stage(ctx, keyset, m, std::max<size_t>(tp.nrows, 1), st, slot);
  if (rc != TMED_OK) return rc;
  memcpy(st.tmpl, tp.rows.data(), std::max<size_t>(tp.nrows, 1) * tmed::kVoteTmplBytes);
  std::atomic<bool> key_ok{true};
  const uint32_t nkeys = keyed ? (uint32_t)st.ks->n : 0u;
  // Signature runs in pinned caller memory go to the device by their own DMA (votes_enqueue)
  // instead of through the staging area: only batches copied on the copy stream.
  bool direct = st.total >= tmed::kVoteCopyStreamMin;
  // pinned-memory lookups once per request (a registry lookup per run took a global lock per
  // vote where runs are single votes: Trusting candidates, C3)
  // (only requests with a run long enough for its own DMA: a light-client batch has none)
  std::vector<uint8_t> req_pinned;
  if (direct) {
    req_pinned.assign(n, 0);
    const size_t *pos = grp.positions(cands);
    const size_t nr = grp.nruns(cands);
    for (size_t j = 0; j < nr; j++)
      if (pos[j + 1] - pos[j] >= kDmaMinRun) req_pinned[cands.runs[grp.run(cands, j)].req] = 2;
    bool any = false;
    for (size_t q = 0; q < n; q++) {
      if (req_pinned[q] != 2) continue;
      const tmed_commit &c = *reqs[q].commit;
      req_pinned[q] = c.n_sigs && tmed::host_pinned(c.sigs, 64 * c.n_sigs) ? 1 : 0;
      any = any || req_pinned[q];
    }
    direct = any;
  }
  const unsigned nt = host_threads(m);
  std::vector<std::vector<tmed::VoteStage::Dma>> tdma(direct ? nt : 0u);
  std::atomic<bool> all_direct{direct};
  // per run segment: one memcpy per array; the key index, the template index and short
  // signatures stay per vote
  auto fill = [&](size_t lo, size_t hi, unsigned tid) {
    bool ok = true, staged_sig = false;
    std::vector<tmed::VoteStage::Dma> mine;  // (a header of its own: see seam_plan)
    for_segments(cands, grp, lo, hi, [&](size_t j, uint32_t u0, uint32_t u1, size_t p) {
      const Run &run = cands.runs[grp.run(cands, j)];
      const tmed_commit_request &r = reqs[run.req];
      const tmed_commit &c = *r.commit;
      const size_t i = (size_t)(run.sig + (int32_t)u0);
      const int32_t v0 = run.val + (int32_t)u0;
      const size_t len = u1 - u0;
      if (keyed) {
        uint32_t *kd = reinterpret_cast<uint32_t *>(st.key) + p;
        const uint32_t *kix = r.vals->keyset_index;
        for (size_t u = 0; u < len; u++) {
          const uint32_t v = kix ? kix[v0 + (int32_t)u] : (uint32_t)(v0 + (int32_t)u);
          ok = ok && v < nkeys;
          kd[u] = v;
        }
      } else {
        memcpy(st.key + p * 32, r.vals->pubkeys + 32 * (size_t)v0, 32 * len);
      }
      // runs of at least kDmaMinRun signatures: a DMA command costs ~10 us of the copy engine
      bool dma = direct && len >= kDmaMinRun && tid < tdma.size() && req_pinned[run.req];
      if (dma && c.sig_lens)  // short signatures are zero-padded in staging
        for (size_t u = 0; u < len && dma; u++) dma = c.sig_lens[i + u] >= 64;
      if (dma) {
        mine.push_back({p * 64, c.sigs + 64 * i, 64 * len});
      } else {
        staged_sig = true;
        memcpy(st.sig + p * 64, c.sigs + 64 * i, 64 * len);
        if (c.sig_lens)
          for (size_t u = 0; u < len; u++) {
            const uint32_t sl = c.sig_lens[i + u];
            if (sl < 64) memset(st.sig + (p + u) * 64 + sl, 0, 64 - sl);
          }
      }
      std::fill(st.tidx + p, st.tidx + p + len, tp.row(cands, run.req));
      memcpy(st.flag + p, c.flags + i, len);
      memcpy(st.sec + p, c.ts_seconds + i, 8 * len);
      memcpy(st.nan + p, c.ts_nanos + i, 4 * len);
    });
    if (!ok) key_ok = false;
    if (staged_sig) all_direct = false;
    if (tid < tdma.size()) tdma[tid].swap(mine);
  };
  parallel_ranges(m, nt, fill);
  if (!key_ok) return TMED_EINVAL;  // a key-set index past the key set (votes_enqueue's check)
  for (auto &v : tdma)  // thread ranges in order; a run cut at a thread boundary is joined again
    for (const tmed::VoteStage::Dma &r : v) {
      tmed::VoteStage::Dma *b = st.dma.empty() ? nullptr : &st.dma.back();
      if (b && b->dst + b->bytes == r.dst && (const uint8_t *)b->src + b->bytes == (const uint8_t *)r.src)
        b->bytes += r.bytes;
      else
        st.dma.push_back(r);
    }
  st.sig_direct = all_direct && m > 0;
  st.keys_checked = keyed;
  return TMED_OK;
}

static int bs_drain(tmed_ctx *ctx);
static void bs_reap(tmed_ctx *ctx);


// GPU verifier of one seam call: candidates of validator sets with a key-set handle go
// through the key-cached kernels, one launch sequence per distinct key set.
static int ctx_verify(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t n, const Cands &cands,
                      uint8_t *valid) {
  PhaseClock clk;
  thread_local Templates tmpl;
  bool fits = true;
  int rc = device_templates(reqs, n, cands, tmpl, &fits);
  if (rc != TMED_OK) return rc;
  if (!fits) return ctx_verify_host_msgs(ctx, reqs, n, cands, valid);
  clk.lap("templates");
  // group the runs by key set (usually a single group: then it is every run, in order)
  // (aliased candidates are left out: copy_aliases)
  std::vector<uint64_t> gkeys;
  std::vector<Group> groups;
  size_t ap = 0;
  bool one_set = !cands.runs.empty();
  for (size_t r = 1; r < cands.runs.size() && one_set; r++)
    one_set = reqs[cands.runs[r].req].vals->keyset == reqs[cands.runs[0].req].vals->keyset;
  if (one_set && !cands.alias.empty()) {
    gkeys.push_back(reqs[cands.runs[0].req].vals->keyset);
    groups.emplace_back();
    build_group(cands, groups[0]);
  }
  for (size_t r = 0; r < cands.runs.size() && !(one_set && !cands.alias.empty()); r++) {
    const uint64_t ks = reqs[cands.runs[r].req].vals->keyset;
    size_t g = 0;
    while (g < gkeys.size() && gkeys[g] != ks) g++;
    if (g == gkeys.size()) { gkeys.push_back(ks); groups.emplace_back(); groups.back().start(); }
    groups[g].add_run(cands, (uint32_t)r, cands.alias, ap);
  }
  if (groups.size() == 1 && cands.alias.empty()) groups[0] = Group();  // every run in order: the call's own offsets
  std::lock_guard<std::mutex> lk(ctx->mu);
  rc = bs_drain(ctx);  // batches of submitted blocksync windows hold the vote slots
  if (rc != TMED_OK) return rc;
  for (size_t g = 0; g < gkeys.size(); g++) {
    const Group &grp = groups[g];
    const uint32_t m = (uint32_t)grp.size(cands);
    if (m == 0) continue;
    tmed::VoteStage st;
    rc = stage_group(ctx, reqs, n, cands, grp, gkeys[g], tmpl, 0, st);
    clk.lap("stage");
    std::vector<uint8_t> out(m);
    if (rc == TMED_OK) rc = tmed::votes_launch(ctx, st, out.data());
    if (rc != TMED_OK) return rc;
    clk.lap("device");
    if (trace_on()) fprintf(stderr, "[tmed] group %zu: %u votes, assemble+verify kernels %.0fus\n", g, m,
                            1000.0 * ctx->last_ms);
    scatter_bits(reqs, cands, grp, out.data(), valid);
    clk.lap("scatter");
  }
  copy_aliases(cands, valid);
  clk.emit("ctx_verify", n, cands.size());
  return TMED_OK;
}

static int run_pipelined(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t nb, size_t bsz, uint64_t keyset,
                         tmed_commit_result *out, const KcCall *kc);

// ---- key-set cache (keycache.h / keycache.hip) -------------------------------
// The validator sets of one seam call that carry no handle, resolved through the context's cache:
// the call then runs on copies of its requests whose sets point into the cache's pool (keyset =
// the pool, keyset_index = the set's entry).  The call pins the pool from its first lookup until
// this object dies, after the call's last batch was collected; then the keys that generic sets of
// the call queued are built by the context's key-build worker (keycache.hip), off this call's
// critical path, in stream order ahead of later calls.
// Its buffers are the calling thread's, kept across calls: a light-client batch rewrites ~20k
// requests onto ~10k sets, and fresh pages cost a fault per 4 KB on every call.
struct KcStore {
  std::vector<tmed_commit_request> reqs;
  std::vector<tmed_valset> vals;           // copies of the resolved sets (reqs[q].vals points here)
  std::vector<const tmed::KcSet *> entry;  // the cache entry of vals[s] (nullptr: not keyed)
  // resolution scratch: distinct sets, request -> set, the pointer table
  struct SetRef {
    const tmed_valset *v;
    size_t sigs;
    const tmed::KcSet *e;
    uint64_t handle;
    bool hit, skip;
    tmed::KcKey key;
  };
  std::vector<SetRef> sets;
  std::vector<int32_t> set_of, tval;
  std::vector<const tmed_valset *> tkey;
  std::vector<uint32_t> slot;
  std::vector<uint8_t> is_first;
};
struct KcCall {
  tmed_ctx *c = nullptr;
  bool active = false;  // this call's requests were rewritten onto st.vals
  KcStore &st;
  KcCall() : st(store()) {}
  ~KcCall() {
    if (!c) return;
    std::lock_guard<std::mutex> lk(c->mu);
    tmed::keycache_unpin(c);  // entries dropped during the call are freed with the last pin
    tmed::keycache_after_call(c);  // the context's worker builds the queued keys
  }
  static KcStore &store() {
    thread_local KcStore s;
    return s;
  }
};

// The cached address index of a set this call resolved through the cache (nullptr otherwise, or
// when the request's addresses differ from the ones the entry's index was built from).
static const AddrIndex *kc_addr_index(const KcCall *kc, const tmed_valset &vs) {
  const std::vector<tmed_valset> &vals = kc->st.vals;
  if (!kc->active || !vs.addresses || &vs < vals.data() || &vs >= vals.data() + vals.size()) return nullptr;
  const tmed::KcSet *e = kc->st.entry[(size_t)(&vs - vals.data())];
  return e ? e->addr_index(vs.addresses, vs.n) : nullptr;
}

static const tmed_commit_request *keycache_resolve(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t n,
                                                   KcCall &kc) {
  if (!ctx->kc_on || n == 0 || !reqs) return reqs;
  PhaseClock clk;
  KcStore &S = kc.st;
  using SetRef = KcStore::SetRef;
  // distinct tmed_valset structs of the call (requests on one struct share its resolution), by a
  // flat open-addressing table of pointers filled by the host pool (a light-client batch: 20k
  // requests on 10k sets; serially the table's cache misses cost ~0.2 ms a call).  Sets are numbered
  // in the order of their first request (each slot keeps the smallest request index that names it),
  // so the set order — and the order keys are appended to the pool — does not depend on addresses.
  std::vector<SetRef> &sets = S.sets;
  sets.clear();
  S.set_of.resize(n);
  size_t cap = 16;
  while (cap < 2 * n) cap <<= 1;
  S.tkey.assign(cap, nullptr);
  S.tval.assign(cap, INT32_MAX);  // first request index per slot, then the set index
  S.slot.resize(n);
  S.is_first.resize(n);
  const tmed_valset **tkey = S.tkey.data();
  int32_t *tval = S.tval.data();
  uint32_t *slot = S.slot.data();
  const unsigned nt = host_threads(n >= 1024 ? ~(size_t)0 : n * 128);
  constexpr uint32_t kNoSet = 0xffffffffu;
  parallel_ranges(n, nt, [&](size_t lo, size_t hi, unsigned) {
    for (size_t q = lo; q < hi; q++) {
      const tmed_valset *v = reqs[q].vals;
      if (!v || !reqs[q].commit) {
        slot[q] = kNoSet;
        continue;
      }
      size_t h = (size_t)(((uintptr_t)v >> 4) * 0x9E3779B97F4A7C15ull >> 20) & (cap - 1);
      for (;;) {
        const tmed_valset *cur = __atomic_load_n(&tkey[h], __ATOMIC_ACQUIRE);
        if (cur == v) break;
        if (!cur) {
          const tmed_valset *expect = nullptr;
          if (__atomic_compare_exchange_n(&tkey[h], &expect, v, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) break;
          if (expect == v) break;
        }
        h = (h + 1) & (cap - 1);
      }
      slot[q] = (uint32_t)h;
      int32_t f = __atomic_load_n(&tval[h], __ATOMIC_RELAXED);  // the slot's smallest request index
      while ((int32_t)q < f && !__atomic_compare_exchange_n(&tval[h], &f, (int32_t)q, true, __ATOMIC_RELAXED,
                                                            __ATOMIC_RELAXED)) {
      }
    }
  });
  // a request opens a set when it is its slot's smallest index (read after the region: final)
  uint8_t *is_first = S.is_first.data();
  parallel_ranges(n, nt, [&](size_t lo, size_t hi, unsigned) {
    for (size_t q = lo; q < hi; q++) is_first[q] = slot[q] != kNoSet && tval[slot[q]] == (int32_t)q;
  });
  size_t nsets = 0;
  for (size_t q = 0; q < n; q++) nsets += is_first[q];
  if (nsets == 0) {
    for (size_t q = 0; q < n; q++) S.set_of[q] = -1;
    return reqs;
  }
  sets.resize(nsets);
  for (size_t q = 0, k = 0; q < n; q++)
    if (is_first[q]) {
      sets[k] = SetRef{reqs[q].vals, 0, nullptr, 0, false, false, tmed::KcKey()};
      tval[slot[q]] = -1 - (int32_t)k;  // slot -> set index (encoded negative: no request index collides)
      k++;
    }
  clk.lap("sets");
  // request -> set and signatures per set (the policy's amortisation and the counters)
  parallel_ranges(n, nt, [&](size_t lo, size_t hi, unsigned) {
    for (size_t q = lo; q < hi; q++) {
      const int32_t s_ = slot[q] == kNoSet ? -1 : -1 - tval[slot[q]];
      S.set_of[q] = s_;
      if (s_ >= 0) __atomic_fetch_add(&sets[s_].sigs, reqs[q].commit->n_sigs, __ATOMIC_RELAXED);
    }
  });
  clk.lap("sigs");
  bool any_keyed = false;
  size_t misses = 0;
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    kc.c = ctx;
    tmed::keycache_pin(ctx);
    tmed::keycache_touch(ctx);
    // one pass per set in parallel while this thread holds the lock (no writer can run): the
    // digest (or set_hash), the read-only find, the byte compare while the set's keys are in this
    // thread's cache, and the entry's LRU tick
    const uint64_t tick = tmed::keycache_call_tick(ctx);
    std::vector<size_t> thits(std::max(1u, nt), 0), tsigs(std::max(1u, nt), 0);
    parallel_ranges(sets.size(), nt, [&](size_t lo, size_t hi, unsigned t) {
      size_t h = 0, g = 0;  // this worker's hits and their signatures (stored once: shared lines)
      for (size_t s = lo; s < hi; s++) {  // keys and finds first: the compares below prefetch ahead
        SetRef &sr = sets[s];
        const tmed_valset &v = *sr.v;
        sr.skip = v.keyset || v.n == 0 || !v.pubkeys;
        if (sr.skip) continue;
        sr.key = tmed::kc_key(v.pubkeys, v.n, v.set_hash);
        sr.e = tmed::keycache_find(ctx, sr.key);
      }
      // the byte compares (~5.6 KB per set from the caller, cold, against the pool's key table through
      // the entry's indexes): the next set's keys and indexes are prefetched while this one is compared
      auto prefetch_set = [&](size_t s) {
        if (s >= hi || sets[s].skip || !sets[s].e) return;
        const tmed_valset &v = *sets[s].v;
        const uint8_t *a = v.pubkeys, *b = (const uint8_t *)sets[s].e->idx.data();
        const size_t nb = std::min(v.n, sets[s].e->idx.size());
        for (size_t o = 0; o < 32 * v.n; o += 64) __builtin_prefetch(a + o, 0, 0);
        for (size_t o = 0; o < 4 * nb; o += 64) __builtin_prefetch(b + o, 0, 0);
      };
      prefetch_set(lo);
      for (size_t s = lo; s < hi; s++) {
        SetRef &sr = sets[s];
        prefetch_set(s + 1);
        if (sr.skip) continue;
        const tmed_valset &v = *sr.v;
        sr.hit = sr.e && tmed::keycache_same_keys(ctx, *sr.e, v.pubkeys, v.n);
        if (sr.hit) {
          const_cast<tmed::KcSet *>(sr.e)->touch(tick);
          h++;
          g += sr.sigs;
        }
      }
      thits[t] = h;
      tsigs[t] = g;
    });
    clk.lap("find_compare");
    size_t nh = 0, ns = 0;
    for (size_t t = 0; t < thits.size(); t++) {
      nh += thits[t];
      ns += tsigs[t];
    }
    tmed::keycache_hits(ctx, nh, ns);
    any_keyed = nh > 0;
    const uint64_t pool = tmed::keycache_pool_handle(ctx);
    for (SetRef &sr : sets)
      if (sr.hit) sr.handle = pool;
      else if (!sr.skip) misses++;
    if (misses) {
      // the call's signatures against every key it lacks: a window / batch that pays for them all
      // builds them before its kernels (each set alone may carry too few signatures).  A call too
      // small to pay for even one key (a single commit: C1) counts nothing.
      size_t call_sigs = 0, call_missing = 0;
      for (SetRef &sr : sets)
        if (!sr.hit && !sr.skip) call_sigs += sr.sigs;
      if (call_sigs >= tmed::kKcAmortizeSigsPerKey) {
        std::unordered_set<tmed::Pub32, tmed::Pub32Hash> seen;
        for (SetRef &sr : sets)
          if (!sr.hit && !sr.skip) call_missing += tmed::keycache_missing(ctx, sr.v->pubkeys, sr.v->n, &seen);
      }
      const bool build_all = call_missing && call_sigs >= tmed::kKcAmortizeSigsPerKey * call_missing;
      for (SetRef &sr : sets) {
        if (sr.hit || sr.skip) continue;
        sr.e = nullptr;
        // too few signatures for even one key and not every key pooled: generic now, the keys are
        // sorted out by the worker after the call (the first commit of a new set)
        if (!build_all && sr.sigs < tmed::kKcAmortizeSigsPerKey &&
            !tmed::keycache_all_pooled(ctx, sr.v->pubkeys, sr.v->n)) {
          tmed::keycache_defer(ctx, sr.v->pubkeys, sr.v->n, sr.sigs);
          continue;
        }
        if (tmed::keycache_lookup(ctx, sr.v->pubkeys, sr.v->n, sr.key, sr.sigs, /*may_reset=*/!any_keyed, &sr.handle,
                                  sr.e, build_all)) {
          sr.hit = true;
          any_keyed = true;
        }
      }
    }
  }
  clk.lap("lookups");
  if (!any_keyed) {
    clk.emit("keycache_resolve (generic)", n, sets.size());
    return reqs;
  }
  // the call's requests, rewritten onto copies of the sets that resolved keyed
  S.vals.resize(sets.size());
  S.entry.resize(sets.size());
  S.reqs.resize(n);
  parallel_ranges(sets.size(), nt, [&](size_t lo, size_t hi, unsigned) {
    for (size_t s = lo; s < hi; s++) {
      const SetRef &sr = sets[s];
      S.entry[s] = sr.hit ? sr.e : nullptr;
      if (!sr.hit) continue;
      S.vals[s] = *sr.v;
      S.vals[s].keyset = sr.handle;
      S.vals[s].keyset_index = sr.e->idx.data();
    }
  });
  parallel_ranges(n, nt, [&](size_t lo, size_t hi, unsigned) {
    for (size_t q = lo; q < hi; q++) {
      S.reqs[q] = reqs[q];
      const int32_t s = S.set_of[q];
      if (s >= 0 && sets[s].hit) S.reqs[q].vals = &S.vals[s];
    }
  });
  kc.active = true;
  clk.lap("rewrite");
  clk.emit("keycache_resolve", n, sets.size());
  return S.reqs.data();
}

// A large call whose sets share one key set (a light-client or evidence backlog) goes through
// the two-slot pipeline in batches of ~2^19 signatures (env TMED_PIPE_SIGS), so the host
// planning, staging and replay of one batch overlap the device work of the next.
static size_t pipe_batch_sigs() {
  const char *e = getenv("TMED_PIPE_SIGS");
  return e ? std::max<size_t>(1, strtoull(e, nullptr, 10)) : (size_t)1 << 19;
}

static int verify_commits_impl(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t n, tmed_commit_result *out) {
  if (!ctx) return TMED_EINVAL;
  KcCall kc;
  reqs = keycache_resolve(ctx, reqs, n, kc);
  const size_t kPipeBatchSigs = pipe_batch_sigs();
  if (n > 1 && reqs && out) {
    // every request checked, one key set, the signature total (in parallel: a light-client call's
    // ~10k commit structs are cold in the cache)
    const uint64_t ks = reqs[0].vals ? reqs[0].vals->keyset : 0;
    std::atomic<bool> all_ok{true};
    std::atomic<size_t> sig_total{0};
    parallel_ranges(n, n >= 4096 ? host_threads(n * 64) : 1, [&](size_t lo, size_t hi, unsigned) {
      size_t sg = 0;
      bool good = true;
      for (size_t q = lo; q < hi && good; q++) {
        good = check_request(reqs[q]) == TMED_OK && reqs[q].vals->keyset == ks;
        if (good) sg += reqs[q].commit->n_sigs;
      }
      sig_total += sg;
      if (!good) all_ok = false;
    });
    const bool ok = all_ok.load();
    const size_t sigs = sig_total.load();
    if (ok && sigs >= 2 * kPipeBatchSigs) {
      const size_t bsz = std::max<size_t>(16, kPipeBatchSigs / std::max<size_t>(1, sigs / n));
      if (n > bsz) {
        const int rc = run_pipelined(ctx, reqs, n, bsz, ks, out, &kc);
        bs_reap(ctx);
        return rc;
      }
    }
  }
  const int rc = run_seam(
      reqs, n, out,
      [&](const tmed_commit_request *rq, size_t nr, const Cands &cands, uint8_t *valid) {
        return ctx_verify(ctx, rq, nr, cands, valid);
      },
      &kc);
  bs_reap(ctx);  // submitted windows this call collected (ctx_verify drained the stream) leave now
  return rc;
}

// ---- blocksync replay window (f4): pipelined LIGHT batches --------------------------------
// The context's batch stream: windows of requests whose sets share one key set (0 = generic keys)
// are cut into batches of up to bsz requests; batch b is planned, staged and queued while the
// device copies in and verifies the batches before it, which are then collected and replayed (f4).
// Same results as one run_seam over all requests.  The stream outlives a call: a replay that
// submits window w+1 before collecting window w (tmed_blocksync_submit) keeps the device busy
// across the windows' boundaries, where a call per window drains the pipeline at its end and
// refills it (the first batch's planning and copy-in) at the next start.
namespace {
struct BsWindow {
  const tmed_commit_request *rq = nullptr;  // the window's requests (checked: check_request)
  tmed_commit_result *out = nullptr;
  size_t n = 0, bsz = 0, next = 0;          // requests; per batch; the next one to batch
  uint64_t keyset = 0;
  const KcCall *kc = nullptr;  // planning's cached address indexes (a call-scoped window only)
  // a submitted window owns its requests, its resolved set and its key-set cache pin (held until
  // its last batch is collected; released outside ctx->mu: ~KcCall takes it)
  std::vector<tmed_commit_request> own_reqs;
  std::vector<tmed_block_id> own_bids;
  std::vector<tmed_commit> own_commits;
  tmed_valset own_set{}, own_vals{};  // the caller's set; its resolved copy
  std::string own_chain;
  std::unique_ptr<KcCall> own_kc;
  size_t inflight = 0;
  bool done() const { return next >= n && inflight == 0; }
};
struct BsBatch {
  BsWindow *win = nullptr;
  size_t lo = 0, n = 0;
  Plans plans;
  Cands cands;
  Templates tmpl;
  std::vector<uint8_t> bits, valid;
  Group grp;  // the staged segments when candidates are aliased (else every run, in order)
  tmed::VoteStage st;
  bool device = false;  // queued on a vote slot (else verified synchronously / nothing to verify)
  std::chrono::steady_clock::time_point enq;  // when it was queued (TMED_TRACE timeline)
};
}  // namespace

// Pipeline depth.  With the signatures staged (pageable caller memory) two slots: a third
// overlaps the host staging of batch b with the copy engine reading batch b-1 out of pinned
// memory, and both slow down (C4 166-172 against 181-191 M verifies/s, profiles/r03/c4_pipe/).
// With the signatures DMA'd from pinned caller memory the host's share per batch is ~1.5 ms
// against ~2.2 ms of kernels, and a third slot keeps the kernel stream busy (C4 280-307 against
// 258-282 M/s, profiles/r03/c4_direct/).  So the depth follows the stream's first batch: three
// slots when its signatures went direct (VoteStage::sig_direct), else two.  (A ramp of small first
// batches did not pay, in round 3 nor again in round 4 with direct DMA: the host's planning and
// staging of each larger batch outlasted the device work of the small one before it, leaving the
// device idle 0.6-1.6 ms per ramp step — profiles/r04/c4_ramp_rejected.txt.)
constexpr int kPipeSlots = 3;
static_assert(kPipeSlots <= (int)(sizeof(((tmed_ctx *)nullptr)->vslot) / sizeof(tmed::VoteSlot)),
              "one context vote slot per pipeline slot");

struct BsStream {
  BsBatch slots[kPipeSlots];
  int ns = 2;
  size_t idx = 0;    // batches queued since the stream was last empty (slot idx % ns)
  int rc = TMED_OK;  // the first error of a submitted window, reported by tmed_blocksync_wait
  std::deque<std::unique_ptr<BsWindow>> wins;
  bool empty() const {
    for (const BsBatch &b : slots)
      if (b.n) return false;
    return true;
  }
};

namespace tmed {
void bs_destroy(tmed_ctx *c) {  // tmed_destroy: nothing may still read the windows' buffers
  if (!c->bs) return;
  (void)hipStreamSynchronize(c->copy_stream);
  (void)hipStreamSynchronize(c->stream);
  if (c->lane1.s) (void)hipStreamSynchronize(c->lane1.s);  // key-cached batches alternate lanes
  delete c->bs;  // the windows' cache pins go with them (the cache is destroyed after this)
  c->bs = nullptr;
}
}  // namespace tmed

using BsClock = std::chrono::steady_clock;
static double bs_us(BsClock::time_point a, BsClock::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}

// TMED_DEBUG_ZERO=1 (diagnostics only): every staged candidate of a pipelined generic batch whose
// device bit is 0 is recorded with what the host staged (key, signature), what the device held
// (its copy of both, the assembled sign-bytes) and which request / signature it was, for
// tmed_debug_zero_bits.  It tells a false reject from the verification kernels apart from one
// in the staging, the copy or the assembly.
namespace {
struct ZeroRec {
  uint64_t req;  // request index in the call's window
  int32_t sig;   // signature index in its commit
  uint32_t pos, msg_len, batch_m;
  uint8_t key_host[32], sig_host[64], key_dev[32], sig_dev[64], msg[256];
};
std::mutex g_zero_mu;
std::vector<ZeroRec> g_zero;
bool debug_zero_on() {
  static const bool on = getenv("TMED_DEBUG_ZERO") != nullptr;
  return on;
}
}  // namespace

static void debug_record_zeros(tmed_ctx *ctx, const BsBatch &b) {
  if (b.st.ks || b.st.zc || b.st.sig_direct) return;  // generic staged batches only
  const tmed::VoteSlot &vs = ctx->vslot[b.st.slot];
  const size_t m = b.bits.size();
  std::vector<ZeroRec> recs;
  for_segments(b.cands, b.grp, 0, m, [&](size_t j, uint32_t u0, uint32_t u1, size_t p0) {
    const Run &run = b.cands.runs[b.grp.run(b.cands, j)];
    for (uint32_t u = u0; u < u1; u++) {
      const size_t p = p0 + (u - u0);
      if (b.bits[p]) continue;
      ZeroRec z{};
      z.req = b.lo + run.req;
      z.sig = run.sig + (int32_t)u;
      z.pos = (uint32_t)p;
      z.batch_m = (uint32_t)m;
      memcpy(z.key_host, b.st.key + 32 * p, 32);
      memcpy(z.sig_host, b.st.sig + 64 * p, 64);
      const uint8_t *d = (const uint8_t *)vs.d_votes.p;
      (void)hipMemcpy(z.key_dev, d + b.st.o_key + 32 * p, 32, hipMemcpyDeviceToHost);
      (void)hipMemcpy(z.sig_dev, d + b.st.o_sig + 64 * p, 64, hipMemcpyDeviceToHost);
      (void)hipMemcpy(z.msg, (const uint8_t *)vs.d_vmsg.p + (size_t)tmed::kVoteSlot * p, 256, hipMemcpyDeviceToHost);
      (void)hipMemcpy(&z.msg_len, (const uint32_t *)vs.d_off.p + p, 4, hipMemcpyDeviceToHost);
      recs.push_back(z);
    }
  });
  std::lock_guard<std::mutex> g(g_zero_mu);
  g_zero.insert(g_zero.end(), recs.begin(), recs.end());
}

// The recorded zero bits (TMED_DEBUG_ZERO), oldest first: copies up to cap records of
// sizeof(ZeroRec) bytes into out and removes them; *n = records copied.
extern "C" int tmed_debug_zero_bits(void *out, size_t cap, size_t *n) {
  std::lock_guard<std::mutex> g(g_zero_mu);
  const size_t k = std::min(cap, g_zero.size());
  if (k && out) memcpy(out, g_zero.data(), k * sizeof(ZeroRec));
  g_zero.erase(g_zero.begin(), g_zero.begin() + (ptrdiff_t)k);
  if (n) *n = k;
  return (int)sizeof(ZeroRec);
}

// Tests: every host-pool part starts up to max_us microseconds late (0: off), see host_pool.h.
extern "C" void tmed_test_pool_jitter(int max_us) { g_pool_jitter_us.store(max_us < 0 ? 0 : max_us); }

// Collect batch b (ctx->mu held): its bits, the alias copies, the replay into its window's results.
// ph: tmed_seam_phase_us — host plan + templates + staging, host time blocked on the device
// (enqueueing the copies and kernels, votes_collect), host replay.
static int bs_finish(tmed_ctx *ctx, BsBatch &b, double ph[3]) {
  if (b.n == 0) return TMED_OK;
  BsWindow &w = *b.win;
  const size_t m = b.cands.size();
  const bool aliased = b.device && !b.cands.alias.empty();
  int r = TMED_OK;
  if (b.device) {
    b.bits.resize(b.grp.size(b.cands));
    const auto t0 = BsClock::now();
    r = tmed::votes_collect(ctx, b.st, b.bits.data());
    ph[1] += bs_us(t0, BsClock::now());
    if (r == TMED_OK && debug_zero_on()) debug_record_zeros(ctx, b);
  }
  const auto t1 = BsClock::now();
  PhaseClock clk;
  const Cands &cd = b.cands;
  const size_t np = cd.preq.size() ? cd.preq.size() - 1 : 0;
  if (r == TMED_OK && aliased && np && !b.grp.rix.empty()) {
    // part by part (the planning workers' parts: each alias inside its part): the part's staged
    // bits -> by candidate, its aliased bits, then the replay of its requests — one fork-join
    b.valid.resize(m);
    r = finish_parts(w.rq + b.lo, cd, b.grp, b.bits.data(), b.valid.data(), b.plans, w.out + b.lo);
    clk.lap("scatter_aliases_replay");
  } else {
    if (r == TMED_OK && aliased) {  // bits by staged segment -> by candidate
      b.valid.resize(m);  // scatter_bits writes every staged candidate, copy_aliases the rest
      scatter_bits(w.rq + b.lo, b.cands, b.grp, b.bits.data(), b.valid.data());
      clk.lap("scatter");
      copy_aliases(b.cands, b.valid.data());
      clk.lap("aliases");
    }
    // the device bits are in candidate order: replay reads them directly (it applies the
    // signature-length rule itself)
    if (r == TMED_OK)
      r = seam_replay(w.rq + b.lo, b.n, w.out + b.lo, b.plans, b.device && !aliased ? b.bits.data() : b.valid.data());
    clk.lap("replay");
  }
  if (b.device) clk.emit("blocksync finish", b.n, m);
  ph[2] += bs_us(t1, BsClock::now());
  b.n = 0;
  b.device = false;
  b.win = nullptr;
  w.inflight--;
  return r;
}

// Collect every batch in flight, oldest first, except those of window `keep` (nullptr: all).
static int bs_collect(tmed_ctx *ctx, BsStream &S, const BsWindow *keep, double ph[3]) {
  int rc = TMED_OK;
  for (int k = 0; k < S.ns; k++) {
    BsBatch &b = S.slots[(S.idx + k) % S.ns];
    if (b.n && b.win != keep) {
      const int r = bs_finish(ctx, b, ph);
      if (rc == TMED_OK) rc = r;
    }
  }
  return rc;
}

// After an error: nothing queued may still read the callers' (pinned) buffers; the batches in
// flight are dropped (their windows' results are incomplete: the error is what the caller gets).
static void bs_abort(tmed_ctx *ctx, BsStream &S, int rc) {
  (void)hipStreamSynchronize(ctx->copy_stream);
  (void)hipStreamSynchronize(ctx->stream);
  // a dropped key-cached batch may run on the second lane: its slot (idx % ns) and its lane
  // (idx & 1) need not match the next batch's, so the lane must be idle before any slot is reused
  if (ctx->lane1.s) (void)hipStreamSynchronize(ctx->lane1.s);
  for (BsBatch &b : S.slots)
    if (b.n) {
      b.n = 0;
      b.device = false;
      if (b.win) b.win->inflight--;
      b.win = nullptr;
    }
  for (auto &w : S.wins) w->next = w->n;
  if (S.rc == TMED_OK) S.rc = rc;
}

// Queue window w's batches (ctx->mu held through lk), collecting older batches as their slots are
// reused; returns with up to S.ns - 1 of them... in flight.
static int bs_pump(tmed_ctx *ctx, BsStream &S, BsWindow &w, double ph[3], std::unique_lock<std::mutex> &lk) {
  int rc = TMED_OK;
  if (S.empty()) {
    S.idx = 0;
    S.ns = 2;  // raised to 3 after the stream's first batch when its signatures went direct
  }
  if (trace_on()) {  // origin of the per-batch device timeline in the trace
    if (!ctx->trace_t0) (void)hipEventCreate(&ctx->trace_t0);
    if (ctx->trace_t0) (void)hipEventRecord(ctx->trace_t0, ctx->stream);
  }
  const auto t_origin = BsClock::now();
  while (w.next < w.n && rc == TMED_OK) {
    PhaseClock clk;
    const size_t idx = S.idx++;
    const int ns = S.ns;
    BsBatch &b = S.slots[idx % ns];
    BsBatch &mid = S.slots[(idx + ns - 1) % ns];  // batch idx-1 (in flight; with two slots the same as old)
    BsBatch &old = S.slots[(idx + 1) % ns];       // batch idx-ns+1: collected once batch idx is queued
    if (b.n) rc = bs_finish(ctx, b, ph);          // the slot's previous batch (the depth changed)
    if (rc != TMED_OK) break;
    b.win = &w;
    b.lo = w.next;
    b.n = std::min(w.bsz, w.n - w.next);
    w.next += b.n;
    w.inflight++;
    const tmed_commit_request *rq = w.rq + b.lo;
    const auto tp = BsClock::now();
    // b.grp: the staging segments; b.tmpl: the template rows (when several workers planned)
    rc = seam_plan(rq, b.n, w.out + b.lo, b.plans, b.cands, w.kc, &b.grp, &b.tmpl);
    clk.lap("plan");
    const size_t m = b.cands.size();
    bool fits = b.tmpl.fits;
    if (rc == TMED_OK && m && !b.tmpl.ready) rc = device_templates(rq, b.n, b.cands, b.tmpl, &fits);
    clk.lap("templates");
    if (rc == TMED_OK && m) {
      if (fits && m <= 0xffffffffu) {
        rc = stage_group(ctx, rq, b.n, b.cands, b.grp, w.keyset, b.tmpl, (int)(idx % ns), b.st);
        // key-cached batches alternate between the two kernel lanes, so one batch's small kernels
        // (assembly, key order, prep, finish) run beside the other's main kernel
        b.st.lane = w.keyset && (idx & 1) && tmed::lanes_on() ? 1 : 0;
        clk.lap("stage");
        const auto te = BsClock::now();
        ph[0] += bs_us(tp, te);
        if (rc == TMED_OK) rc = tmed::votes_enqueue(ctx, b.st);
        b.enq = BsClock::now();
        if (idx == 0 && b.st.sig_direct) S.ns = 3;
        clk.lap("enqueue");
        ph[1] += bs_us(te, BsClock::now());  // queueing copies / launches can block behind a busy device
        b.device = rc == TMED_OK;
      } else {  // oversize template: host-assembled messages, synchronous (drain the pipeline first)
        if (old.n && &old != &b) rc = bs_finish(ctx, old, ph);
        if (rc == TMED_OK && mid.n && &mid != &b) rc = bs_finish(ctx, mid, ph);
        lk.unlock();
        b.valid.assign(m, 0);
        if (rc == TMED_OK) rc = ctx_verify_host_msgs(ctx, rq, b.n, b.cands, b.valid.data());
        lk.lock();
      }
    }
    const bool traced = trace_on() && old.n && old.st.m && &old != &b;
    if (rc == TMED_OK && &old != &b) rc = bs_finish(ctx, old, ph);  // overlaps the device work of batches idx-1 and idx
    clk.lap("finish_old");
    if (traced)
      fprintf(stderr,
              "[tmed] blocksync collected batch: kernels %.0fus copy-in %.0fus copy end -> kernels %.0fus"
              " | device us: copy %.0f-%.0f kernels %.0f-%.0f | host us: enqueued %.0f collected %.0f\n",
              1000.0 * ctx->last_ms, 1000.0 * ctx->last_copy_ms, 1000.0 * ctx->last_copy_gap_ms,
              1000.0 * ctx->last_at[0], 1000.0 * ctx->last_at[1], 1000.0 * ctx->last_at[2], 1000.0 * ctx->last_at[3],
              bs_us(t_origin, b.enq), bs_us(t_origin, BsClock::now()));
    clk.emit("pipelined batch", b.n, m);
  }
  return rc;
}

static BsStream &bs_stream(tmed_ctx *ctx) {
  if (!ctx->bs) ctx->bs = new BsStream();
  return *ctx->bs;
}

// Windows whose batches are all collected leave the stream (front first); they are destroyed by
// the caller after it released ctx->mu.
static void bs_pop_done(BsStream &S, std::vector<std::unique_ptr<BsWindow>> &gone) {
  while (!S.wins.empty() && S.wins.front()->done()) {
    gone.push_back(std::move(S.wins.front()));
    S.wins.pop_front();
  }
}

// Windows whose batches were collected by another seam call (bs_drain) are released here, outside
// ctx->mu (their key-set cache pins go with them: ~KcCall takes the lock).
static void bs_reap(tmed_ctx *ctx) {
  std::vector<std::unique_ptr<BsWindow>> gone;
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (ctx->bs) bs_pop_done(*ctx->bs, gone);
  }
}

// Every batch of the stream collected (ctx->mu held): before a seam call uses the vote slots.
static int bs_drain(tmed_ctx *ctx) {
  if (!ctx->bs || ctx->bs->empty()) return TMED_OK;
  double ph[3] = {0, 0, 0};
  int rc = bs_collect(ctx, *ctx->bs, nullptr, ph);
  if (rc != TMED_OK) bs_abort(ctx, *ctx->bs, rc);
  return rc;
}

// One window through the stream and back (every batch collected before returning).
static int run_pipelined(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t nb, size_t bsz, uint64_t keyset,
                         tmed_commit_result *out, const KcCall *kc) {
  std::vector<std::unique_ptr<BsWindow>> gone;
  int rc;
  {
    std::unique_lock<std::mutex> lk(ctx->mu);
    BsStream &S = bs_stream(ctx);
    double ph[3] = {0, 0, 0};
    rc = bs_collect(ctx, S, nullptr, ph);  // earlier submitted windows finish first
    if (rc != TMED_OK) bs_abort(ctx, S, rc);  // theirs: reported here and by tmed_blocksync_wait
    const int prev = S.rc;
    auto w = std::make_unique<BsWindow>();
    w->rq = reqs;
    w->out = out;
    w->n = nb;
    w->bsz = std::max<size_t>(1, bsz);
    w->keyset = keyset;
    w->kc = kc;
    BsWindow *wp = w.get();
    S.wins.push_back(std::move(w));
    if (rc == TMED_OK) {
      rc = bs_pump(ctx, S, *wp, ph, lk);
      if (rc == TMED_OK) rc = bs_collect(ctx, S, nullptr, ph);
      if (rc != TMED_OK) {
        bs_abort(ctx, S, rc);
        S.rc = prev;  // only this call's window was in flight: its error is reported here
      }
    }
    wp->next = wp->n;
    for (int k = 0; k < 3; k++) g_seam_us[k] = ph[k];
    bs_pop_done(S, gone);
    for (auto it = S.wins.begin(); it != S.wins.end(); ++it)  // this call's window (borrowed buffers) never stays
      if (it->get() == wp) {
        gone.push_back(std::move(*it));
        S.wins.erase(it);
        break;
      }
  }
  return rc;
}

// A blocksync window as LIGHT requests (blockchain/v0/reactor.go:366-367), resolved through the
// key-set cache, owned by the returned window.
static int bs_window(tmed_ctx *ctx, const tmed_blocksync_window *w, uint32_t batch_blocks, tmed_commit_result *out,
                     std::unique_ptr<BsWindow> &win) {
  if (!ctx || !w || (w->n_blocks && (!w->vals || !w->block_ids || !w->heights || !w->commits || !out)))
    return TMED_EINVAL;
  const size_t nb = w->n_blocks;
  win = std::make_unique<BsWindow>();
  BsWindow &W = *win;
  // the structs are copied (the caller may reuse them once submit returns); what they point to
  // (hashes, commit arrays, keys) is the caller's until the window's results are final
  W.own_reqs.resize(nb);
  W.own_bids.assign(w->block_ids, w->block_ids + nb);
  W.own_commits.assign(w->commits, w->commits + nb);
  if (nb) W.own_set = *w->vals;
  if (w->chain_id_len) W.own_chain.assign(w->chain_id, w->chain_id_len);
  for (size_t h = 0; h < nb; h++) {
    tmed_commit_request &r = W.own_reqs[h];
    memset(&r, 0, sizeof r);
    r.mode = TMED_MODE_LIGHT;
    r.chain_id = W.own_chain.data();
    r.chain_id_len = w->chain_id_len;
    r.vals = &W.own_set;
    r.block_id = &W.own_bids[h];
    r.height = w->heights[h];
    r.commit = &W.own_commits[h];
    if (check_request(r) != TMED_OK) return TMED_EINVAL;
  }
  W.own_kc = std::make_unique<KcCall>();  // one set for the whole window
  if (nb) {
    const tmed_commit_request *rq = keycache_resolve(ctx, W.own_reqs.data(), nb, *W.own_kc);
    if (rq != W.own_reqs.data()) {  // resolved onto the cache's pool: the window keeps its own copy
      W.own_vals = *rq[0].vals;
      for (tmed_commit_request &r : W.own_reqs) r.vals = &W.own_vals;
    }
  }
  W.rq = W.own_reqs.data();
  W.out = out;
  W.n = nb;
  W.bsz = batch_blocks ? batch_blocks : 128;
  W.keyset = nb ? W.own_reqs[0].vals->keyset : 0;
  return TMED_OK;
}

// The seam's C entry points: no C++ exception may cross into the caller (a cgo caller would abort).
// A host allocation that fails inside a call (the per-part plan vectors, a window's copies) returns
// TMED_ENOMEM, any other exception TMED_EINTERNAL (never TMED_EHIP: the device is fine).  When the
// context's blocksync stream still holds work (batches in flight, windows not collected), it is
// dropped (bs_abort), so no queued batch still reads the caller's buffers, and its windows' callers
// get the error from tmed_blocksync_wait; an idle stream is left alone, so the failure of one
// synchronous call is not reported to a later, unrelated window.
// The calling thread is bound to the context's device for the call and given its own device back
// on return: a cgo call may run on any OS thread (goroutines migrate), and the _multi entry points
// call in from fresh threads (device 0).
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(const tmed_ctx *ctx) {
    if (ctx && hipGetDevice(&prev) == hipSuccess && prev != ctx->device) (void)hipSetDevice(ctx->device);
    else prev = -1;
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <class F>
static int c_guard(tmed_ctx *ctx, F &&f) {
  int rc;
  DeviceScope dev(ctx);
  try {
    return f();
  } catch (const std::bad_alloc &) {
    rc = TMED_ENOMEM;
  } catch (...) {
    rc = TMED_EINTERNAL;
  }
  if (ctx) {
    try {
      std::lock_guard<std::mutex> lk(ctx->mu);
      if (ctx->bs && (!ctx->bs->empty() || !ctx->bs->wins.empty())) bs_abort(ctx, *ctx->bs, rc);
    } catch (...) {
    }
  }
  return rc;
}

extern "C" int tmed_verify_commits(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t n,
                                   tmed_commit_result *out) {
  return c_guard(ctx, [&] { return verify_commits_impl(ctx, reqs, n, out); });
}

extern "C" int tmed_blocksync_submit(tmed_ctx *ctx, const tmed_blocksync_window *w, uint32_t batch_blocks,
                                     tmed_commit_result *out) {
  return c_guard(ctx, [&] {
  std::unique_ptr<BsWindow> win;
  int rc = bs_window(ctx, w, batch_blocks, out, win);
  if (rc != TMED_OK) return rc;
  std::vector<std::unique_ptr<BsWindow>> gone;
  {
    std::unique_lock<std::mutex> lk(ctx->mu);
    BsStream &S = bs_stream(ctx);
    double ph[3] = {0, 0, 0};
    BsWindow *wp = win.get();
    S.wins.push_back(std::move(win));
    rc = bs_pump(ctx, S, *wp, ph, lk);
    // every EARLIER window's results final on return; this window's last batches stay in flight
    if (rc == TMED_OK) rc = bs_collect(ctx, S, wp, ph);
    if (rc != TMED_OK) bs_abort(ctx, S, rc);
    for (int k = 0; k < 3; k++) g_seam_us[k] = ph[k];
    bs_pop_done(S, gone);
  }
  return rc;
  });
}

extern "C" int tmed_blocksync_wait(tmed_ctx *ctx) {
  if (!ctx) return TMED_EINVAL;
  return c_guard(ctx, [&] {
  std::vector<std::unique_ptr<BsWindow>> gone;
  int rc;
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->bs) return TMED_OK;
    BsStream &S = *ctx->bs;
    double ph[3] = {0, 0, 0};
    rc = bs_collect(ctx, S, nullptr, ph);
    if (rc != TMED_OK) bs_abort(ctx, S, rc);
    rc = S.rc;
    S.rc = TMED_OK;
    for (int k = 0; k < 3; k++) g_seam_us[k] = ph[k];
    bs_pop_done(S, gone);
  }
  return rc;
  });
}

extern "C" int tmed_blocksync_verify(tmed_ctx *ctx, const tmed_blocksync_window *w, uint32_t batch_blocks,
                                     tmed_commit_result *out) {
  return c_guard(ctx, [&] {
    std::unique_ptr<BsWindow> win;
    int rc = bs_window(ctx, w, batch_blocks, out, win);
    if (rc != TMED_OK || win->n == 0) return rc;
    return run_pipelined(ctx, win->rq, win->n, win->bsz, win->keyset, out, nullptr);
  });
}

// ---- several GPUs in one process (§8e): contiguous shards balanced by signature count ----

// Shard boundaries over n items whose weights are w(i): shard t = [cut[t], cut[t+1]).
template <class W>
static std::vector<size_t> weighted_cuts(size_t n, size_t parts, W &&w) {
  size_t total = 0;
  for (size_t i = 0; i < n; i++) total += w(i);
  std::vector<size_t> cut(parts + 1, n);
  cut[0] = 0;
  size_t acc = 0, t = 1;
  for (size_t i = 0; i < n && t < parts; i++) {
    acc += w(i);
    while (t < parts && acc * parts >= total * t) cut[t++] = i + 1;
  }
  return cut;
}

template <class F>
static int run_shards(size_t n_ctx, const std::vector<size_t> &cut, F &&f) {
  std::vector<int> rcs(n_ctx, TMED_OK);
  std::vector<std::thread> th;
  for (size_t t = 0; t < n_ctx; t++)
    if (cut[t + 1] > cut[t]) th.emplace_back([&, t] { rcs[t] = f(t, cut[t], cut[t + 1]); });
  for (auto &x : th) x.join();
  for (int rc : rcs)
    if (rc != TMED_OK) return rc;
  return TMED_OK;
}

extern "C" int tmed_verify_commits_multi(tmed_ctx *const *ctxs, size_t n_ctx, const tmed_commit_request *reqs,
                                         size_t n, tmed_commit_result *out) {
  if (!ctxs || n_ctx == 0 || (n && (!reqs || !out))) return TMED_EINVAL;
  for (size_t t = 0; t < n_ctx; t++)
    if (!ctxs[t]) return TMED_EINVAL;
  for (size_t q = 0; q < n; q++)
    if (check_request(reqs[q]) != TMED_OK) return TMED_EINVAL;
  const auto cut = weighted_cuts(n, n_ctx, [&](size_t q) { return (size_t)reqs[q].commit->n_sigs + 1; });
  return run_shards(n_ctx, cut, [&](size_t t, size_t lo, size_t hi) {
    return tmed_verify_commits(ctxs[t], reqs + lo, hi - lo, out + lo);
  });
}

extern "C" int tmed_blocksync_verify_multi(tmed_ctx *const *ctxs, size_t n_ctx, const tmed_blocksync_window *w,
                                           uint32_t batch_blocks, tmed_commit_result *out) {
  if (!ctxs || n_ctx == 0 || !w) return TMED_EINVAL;
  for (size_t t = 0; t < n_ctx; t++)
    if (!ctxs[t]) return TMED_EINVAL;
  const size_t nb = w->n_blocks;
  if (nb && (!w->vals || !w->block_ids || !w->heights || !w->commits || !out)) return TMED_EINVAL;
  const auto cut = weighted_cuts(nb, n_ctx, [&](size_t h) { return (size_t)w->commits[h].n_sigs + 1; });
  return run_shards(n_ctx, cut, [&](size_t t, size_t lo, size_t hi) {
    tmed_blocksync_window s = *w;
    s.n_blocks = hi - lo;
    s.block_ids = w->block_ids + lo;
    s.heights = w->heights + lo;
    s.commits = w->commits + lo;
    return tmed_blocksync_verify(ctxs[t], &s, batch_blocks, out + lo);
  });
}
