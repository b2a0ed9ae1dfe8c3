// seam_host.h — the host half of the commit seam (commit.hip): planning (the reference
// prechecks and candidate selection), the parallel merge of the planning parts, candidate
// aliasing, staging groups, scatter and the replay of every reference loop.  Host C++ only (no
// HIP): commit.hip includes it, and tests/native/seam_race.cpp compiles the same code under
// ThreadSanitizer with the pool jitter on, so a read of what another part of the same parallel
// region writes is a reported race on the CPU suite, not a rare wrong bit on the GPU box.
//
// Parallel regions (parallel_ranges) and what each part reads from outside its own range — every
// such read is of data a PRIOR region (or the serial code before the region) wrote:
//   seam_plan plan_range   reqs (caller, read-only); writes part[t], plans[lo, hi), out[lo, hi)
//   seam_plan merge_part   part[t], pc / rbase / cbase (plan region + serial prefix sums);
//                          writes runs/off of its own run range, plans/tmpl_of/row_of of its
//                          own requests; pair_request and Group::add_run read only those
//   seam_plan join         ps.aparts / gparts / trows (merge region), abase / sbase / pbase /
//                          tbase (serial prefix sums)
//   build_group            c.off / c.runs / c.alias: complete before the call (seam_plan)
//   finish_parts           grp / cands / plans (planning, finished before the batch was staged);
//                          part t scatters, aliases and replays only its own requests' candidates
//                          (every alias lies inside its part: pair_request pairs within a part)
#pragma once

#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <memory>
#include <new>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/tmed25519.h"
#include "host_pool.h"
#include "keycache.h"
#include "signbytes.h"

namespace {

constexpr uint8_t kAbsent = 1, kCommit = 2, kNil = 3;
constexpr int64_t kMaxInt64 = 0x7fffffffffffffffLL;

bool block_id_equal(const tmed_block_id &a, const tmed_block_id &b) {  // types/block.go:1170-1173
  if (a.hash_len != b.hash_len || a.psh_total != b.psh_total || a.psh_hash_len != b.psh_hash_len) return false;
  if (a.hash_len && memcmp(a.hash, b.hash, a.hash_len) != 0) return false;
  if (a.psh_hash_len && memcmp(a.psh_hash, b.psh_hash, a.psh_hash_len) != 0) return false;
  return true;
}

// TMED_TRACE=1: per-phase wall times of every seam call on stderr (diagnostics only).
static bool trace_on() {
  static const bool on = getenv("TMED_TRACE") != nullptr;
  return on;
}
struct PhaseClock {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  char buf[512];
  int len = 0;
  void lap(const char *name) {
    if (!trace_on()) return;
    const auto now = std::chrono::steady_clock::now();
    const double us = std::chrono::duration<double, std::micro>(now - t).count();
    t = now;
    if (len < (int)sizeof(buf) - 48) len += snprintf(buf + len, sizeof(buf) - len, " %s=%.0fus", name, us);
  }
  void emit(const char *what, size_t n, size_t m) {
    if (trace_on()) fprintf(stderr, "[tmed] %s n=%zu m=%zu%.*s\n", what, n, m, len, buf);
  }
};

// safeMul (types/validator_set.go:1086-1105), Go-exact: Go's unary minus and product wrap, so
// -MinInt64 == MinInt64 (an int64(Numerator) of 2^63 gives |b| < 0 and MaxInt64 / |b| == 0).
// Two's-complement wrapping through uint64 (C++ -INT64_MIN is undefined); INT64_MAX / INT64_MIN
// is 0 in C++ as in Go (truncation), and |b| is never -1.
static inline int64_t go_neg(int64_t x) { return (int64_t)(0 - (uint64_t)x); }
bool safe_mul(int64_t a, int64_t b, int64_t *out) {
  if (a == 0 || b == 0) { *out = 0; return false; }
  const int64_t ab = b < 0 ? go_neg(b) : b, aa = a < 0 ? go_neg(a) : a;
  if (aa > kMaxInt64 / ab) { *out = 0; return true; }
  *out = (int64_t)((uint64_t)a * (uint64_t)b);
  return false;
}

// The signatures a seam call sends to the verifier, as runs: run r holds candidates
// off[r] .. off[r] + len - 1, the signatures sig .. sig + len - 1 of request req signed by
// validators val .. val + len - 1 of its set.  A VerifyCommit / Light request's candidates are
// one run per stretch of qualifying flags (C4: one run of ~6,667 per block), so planning, staging
// and scattering cost per run, not per signature; a Trusting request's runs break where the
// commit's order leaves the trusted set's.
struct Run {
  uint32_t req;
  int32_t sig, val;
  uint32_t len;
};
struct Cands {
  std::vector<Run> runs;
  std::vector<size_t> off;  // runs.size() + 1 candidate offsets
  // (candidate, the candidate whose bit it takes), ascending: see pair_request
  std::vector<std::pair<uint32_t, uint32_t>> alias;
  // request -> the request whose device template its candidates use (empty: its own); a
  // Trusting request shares the template of the Light request of the same commit (pair_request)
  std::vector<uint32_t> tmpl_of;
  // the planning workers' parts when the batch was aliased with a staging group (seam_plan):
  // part t holds requests [preq[t], preq[t+1]), aliases [pal[t], pal[t+1]) and group segments
  // [pseg[t], pseg[t+1]), every alias inside its part (bs_finish works part by part); else empty
  std::vector<size_t> preq, pal, pseg;
  size_t size() const { return off.empty() ? 0 : off.back(); }
  uint32_t tmpl_row(uint32_t q) const { return tmpl_of.empty() ? q : tmpl_of[q]; }
  void clear() {
    runs.clear();
    off.assign(1, 0);
    alias.clear();
    tmpl_of.clear();
    preq.clear();
    pal.clear();
    pseg.clear();
  }
};
// Append candidate (q, i, v) to a part's runs, extending the last run when it continues it.
inline void push_cand(std::vector<Run> &runs, uint32_t q, int32_t i, int32_t v) {
  if (!runs.empty()) {
    Run &b = runs.back();
    if (b.req == q && b.sig + (int32_t)b.len == i && b.val + (int32_t)b.len == v) {
      b.len++;
      return;
    }
  }
  runs.push_back(Run{q, i, v, 1u});
}

using tmed::AddrIndex;  // keycache.h

struct Plan {
  bool decided = false;
  int64_t needed = 0;
  int32_t panic_idx = -1;  // the loop panics on reaching this signature (TMED_COMMIT_PANIC)
  int32_t stop = 0;        // candidates were collected among signatures [0, stop)
  // Trusting only: sig idx -> validator index in the set, kNoValidator (the address is not in the
  // set), -1 (not reached by the plan).  Other modes: candidate k is the k-th qualifying
  // signature below stop (replay counts them), so nothing per signature is stored.
  int32_t *vof = nullptr;
  size_t cand_off = 0;  // the request's first candidate (in its part while planning, then global)
  uint32_t ncand = 0;
  size_t run_lo = 0, run_hi = 0;  // its runs (in its part while planning, then in the merged runs)
  // Trusting: the double vote the loop stops at (sig idx, validator, first sig idx), -1 = none
  int32_t dv_idx = -1, dv_val = -1, dv_first = -1;
};
constexpr int32_t kNoValidator = -2;

// Growable array without value-initialisation (every element is written before use).
template <class T>
struct RawBuf {
  std::unique_ptr<T[]> p;
  size_t cap = 0;
  T *ensure(size_t n) {
    if (n > cap) { p.reset(new T[n]); cap = n; }
    return p.get();
  }
};

// The run segments of one device group (one key set) and their staging positions: segment j is
// run rix[j]'s candidates from ub[j] on, staged at pos[j] .. pos[j + 1) (rix empty: every run
// whole, in order; ub empty: segments start at their run's first candidate).
struct Group {
  std::vector<uint32_t> rix, ub;
  std::vector<size_t> pos;
  size_t size(const Cands &c) const { return rix.empty() ? c.size() : pos.back(); }
  uint32_t run(const Cands &c, size_t j) const { (void)c; return rix.empty() ? (uint32_t)j : rix[j]; }
  uint32_t base(size_t j) const { return ub.empty() ? 0u : ub[j]; }
  size_t nruns(const Cands &c) const { return rix.empty() ? c.runs.size() : rix.size(); }
  const size_t *positions(const Cands &c) const { return rix.empty() ? c.off.data() : pos.data(); }
  void start() {
    rix.clear();
    ub.clear();
    pos.assign(1, 0);
  }
  // run r without its aliased candidates (al[ap..] ascending; ap advances past run r's).  The end
  // is off[r] + len, not off[r + 1]: seam_plan's merge calls this for a part's runs while the next
  // part's worker is still writing its offsets, and off[r + 1] of a part's last run is the next
  // part's first (read before it was written, it held the slot's previous batch's offset).
  void add_run(const Cands &c, uint32_t r, const std::vector<std::pair<uint32_t, uint32_t>> &al, size_t &ap) {
    const size_t c0 = c.off[r], c1 = c0 + c.runs[r].len;
    size_t k = c0;
    auto seg = [&](size_t a, size_t b) {
      if (a >= b) return;
      rix.push_back(r);
      ub.push_back((uint32_t)(a - c0));
      pos.push_back(pos.back() + (b - a));
    };
    for (; ap < al.size() && al[ap].first < c1; ap++) {
      seg(k, al[ap].first);
      k = (size_t)al[ap].first + 1;
    }
    seg(k, c1);
  }
};

// Device templates, one row per request whose candidates use its own (Cands::tmpl_row), rows
// packed in request order: row_of[q] is request q's row (kNoRow: none).
constexpr uint32_t kNoRow = 0xffffffffu;
struct Templates {
  std::vector<uint8_t> rows;
  std::vector<uint32_t> row_of;
  size_t nrows = 0;
  bool ready = false, fits = true;  // ready: built by seam_plan's merge pass (fits: all within the device assembler)
  uint32_t row(const Cands &c, uint32_t q) const { return row_of[c.tmpl_row(q)]; }
};

// The plans of one seam call and the planning workers' parts, kept between calls (blocksync
// plans batch after batch), so their pages are touched once.
// A planning worker's vof arrays: taken from chunks kept between calls (pointers stay valid
// until the next reset).
struct VofArena {
  std::vector<std::pair<std::unique_ptr<int32_t[]>, size_t>> chunks;
  size_t ci = 0, used = 0;
  void reset() { ci = 0; used = 0; }
  int32_t *take(size_t k) {
    while (ci < chunks.size() && chunks[ci].second - used < k) { ci++; used = 0; }
    if (ci == chunks.size()) {
      const size_t sz = std::max<size_t>((size_t)1 << 16, k);
      chunks.emplace_back(std::unique_ptr<int32_t[]>(new int32_t[sz]), sz);
      used = 0;
    }
    int32_t *p = chunks[ci].first.get() + used;
    used += k;
    return p;
  }
};

struct Plans {
  std::vector<Plan> v;
  std::vector<VofArena> tbits;  // per planning worker: its Trusting requests' vof arrays
  std::vector<std::vector<Run>> parts;
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> aparts;  // per worker: its aliases
  std::vector<Group> gparts;                                       // per worker: its group segments
  std::vector<std::vector<uint8_t>> trows;                         // per worker: its template rows
};


// Per-thread "seen" marks of the Trusting loops (first index of each validator), reset in
// O(1) per request by an epoch stamp instead of a fresh n-sized vector.
struct SeenMarks {
  std::vector<int32_t> idx;
  std::vector<uint32_t> stamp;
  uint32_t epoch = 0;
  void reset(size_t n) {
    if (++epoch == 0 || stamp.size() < n) {
      stamp.assign(std::max(n, stamp.size()), 0);
      idx.resize(stamp.size());
      epoch = 1;
    }
  }
  int32_t get(int32_t v) const { return stamp[v] == epoch ? idx[v] : -1; }
  void set(int32_t v, int32_t i) { stamp[v] = epoch; idx[v] = i; }
};

int check_request(const tmed_commit_request &r) {
  if (!r.vals || !r.commit) return TMED_EINVAL;
  const tmed_commit &c = *r.commit;
  if (c.n_sigs && (!c.flags || !c.ts_seconds || !c.ts_nanos || !c.sigs)) return TMED_EINVAL;
  if (r.vals->n && (!r.vals->pubkeys || !r.vals->powers)) return TMED_EINVAL;
  if (r.mode == TMED_MODE_LIGHT_TRUSTING && c.n_sigs && (!c.addresses || (r.vals->n && !r.vals->addresses)))
    return TMED_EINVAL;
  if (r.mode != TMED_MODE_LIGHT_TRUSTING && !r.block_id) return TMED_EINVAL;
  if (r.mode < TMED_MODE_COMMIT || r.mode > TMED_MODE_LIGHT_TRUSTING) return TMED_EINVAL;
  return TMED_OK;
}

// ValidateHash (types/validation.go:32-40): BlockIDFromProto, called by CanonicalizeBlockID
// (types/canonical.go:18-22) for every Commit-flag vote's sign-bytes, panics otherwise.
bool block_hashes_valid(const tmed_block_id &b) {
  return (b.hash_len == 0 || b.hash_len == 32) && (b.psh_hash_len == 0 || b.psh_hash_len == 32);
}

// GetByAddress(commitSig.ValidatorAddress) (types/validator_set.go:270-277): bytes.Equal against
// 20-byte validator addresses, so an address of any other length matches nothing.
int32_t lookup_address(const AddrIndex &ix, const tmed_commit &c, size_t i) {
  if (c.address_lens && c.address_lens[i] != 20) return -1;
  return ix.find(c.addresses + 20 * i);
}

}  // namespace



// Flattened candidates of one seam call.
struct CandBatch {
  size_t m = 0;
  std::vector<uint8_t> pubs, sigs, flags;
  std::vector<uint32_t> lens, val_idx, tmpl;
  std::vector<int64_t> ts_sec;
  std::vector<int32_t> ts_nanos;
  std::vector<uint64_t> keyset;
  std::vector<tmed::VoteEncoder> enc;  // per request
  // host-assembled sign-bytes (built on demand: callback verifiers, oversize templates)
  std::vector<uint8_t> msgs;
  std::vector<uint32_t> offs;
  int build_host_msgs() {
    if (!offs.empty()) return TMED_OK;
    offs.resize(m + 1);
    size_t total = 0;
    for (size_t k = 0; k < m; k++) {
      offs[k] = (uint32_t)total;
      total += enc[tmpl[k]].size(flags[k], ts_sec[k], ts_nanos[k]);
      if (total > 0xffffffffu) return TMED_EINVAL;
    }
    offs[m] = (uint32_t)total;
    msgs.resize(total + 16);
    for (size_t k = 0; k < m; k++) enc[tmpl[k]].write(msgs.data() + offs[k], flags[k], ts_sec[k], ts_nanos[k]);
    return TMED_OK;
  }
};
using BatchVerifier =
    std::function<int(const tmed_commit_request *reqs, size_t n, const Cands &cands, uint8_t *valid)>;

// Per-request CanonicalVote encoders for the requests that have candidates; then(q, enc)
// runs right after request q's encoder is built (false = failure).  Candidates are in request
// order, so the first candidate of each request marks it used (one writer per request).
template <class Then>
static int init_encoders(const tmed_commit_request *reqs, size_t n, const Cands &cands,
                         std::vector<tmed::VoteEncoder> &enc, std::vector<uint8_t> &used, Then &&then) {
  enc.assign(n, tmed::VoteEncoder());
  used.assign(n, 0);
  const size_t m = cands.size();
  for (const Run &r : cands.runs) used[r.req] = 1;
  std::atomic<int> bad{0};
  parallel_ranges(n, n >= 64 ? host_threads(m) : 1, [&](size_t lo, size_t hi, unsigned) {
  for (size_t q = lo; q < hi; q++) {
    if (!used[q]) continue;
    const tmed_commit &c = *reqs[q].commit;
    tmed_vote_template t;
    t.chain_id = reqs[q].chain_id;
    t.chain_id_len = reqs[q].chain_id_len;
    t.height = c.height;
    t.round = c.round;
    t.block_hash = c.block_id.hash;
    t.block_hash_len = c.block_id.hash_len;
    t.psh_total = c.block_id.psh_total;
    t.psh_hash = c.block_id.psh_hash;
    t.psh_hash_len = c.block_id.psh_hash_len;
    if (enc[q].init(&t) != TMED_OK || !then(q, enc[q])) bad = 1;
  }
  });
  return bad ? TMED_EINVAL : TMED_OK;
}

// Flatten candidates with host-assembled sign-bytes (callback verifiers; oversize templates).
static int build_cand_batch(const tmed_commit_request *reqs, size_t n, const Cands &cands, CandBatch &cb) {
  std::vector<uint8_t> used;
  int rc = init_encoders(reqs, n, cands, cb.enc, used, [](size_t, const tmed::VoteEncoder &) { return true; });
  if (rc != TMED_OK) return rc;
  const size_t m = cands.size();
  cb.m = m;
  cb.pubs.resize(m * 32);
  cb.sigs.assign(m * 64, 0);
  cb.lens.resize(m);
  cb.val_idx.resize(m);
  cb.keyset.resize(m);
  cb.tmpl.resize(m);
  cb.flags.resize(m);
  cb.ts_sec.resize(m);
  cb.ts_nanos.resize(m);
  for (size_t ri = 0; ri < cands.runs.size(); ri++) {
    const Run &run = cands.runs[ri];
    const tmed_commit_request &r = reqs[run.req];
    const tmed_commit &c = *r.commit;
    for (uint32_t u = 0; u < run.len; u++) {
      const size_t k = cands.off[ri] + u;
      const size_t i = (size_t)(run.sig + (int32_t)u);
      const int32_t v = run.val + (int32_t)u;
      memcpy(&cb.pubs[k * 32], r.vals->pubkeys + 32 * (size_t)v, 32);
      const uint32_t sl = c.sig_lens ? c.sig_lens[i] : 64;
      memcpy(&cb.sigs[k * 64], c.sigs + 64 * i, sl < 64 ? sl : 64);
      cb.lens[k] = sl;
      cb.val_idx[k] = r.vals->keyset_index ? r.vals->keyset_index[v] : (uint32_t)v;
      cb.keyset[k] = r.vals->keyset;
      cb.tmpl[k] = run.req;
      cb.flags[k] = c.flags[i];
      cb.ts_sec[k] = c.ts_seconds[i];
      cb.ts_nanos[k] = c.ts_nanos[i];
    }
  }
  return cb.build_host_msgs();
}

// ---- planning: prechecks + candidate selection, parallel over requests ----------------

// Address index of the Trusting set being planned, owned by one planning thread: rebuilt
// when that thread moves to a request on another set (within one seam call only, so a
// caller may rewrite its buffers between calls).  The plan records every lookup result the
// replay needs (the candidate's validator, kNoValidator, the double vote), so the index is
// never read after planning.
// Sets resolved through the key-set cache (KcCall, below) carry their entry's address index.
struct KcCall;
static const AddrIndex *kc_addr_index(const KcCall *kc, const tmed_valset &vs);
struct AddrScratch {
  AddrIndex ix;
  const tmed_valset *of = nullptr;
  const KcCall *kc = nullptr;
  const AddrIndex &get(const tmed_valset &vs) {
    if (kc)
      if (const AddrIndex *c = kc_addr_index(kc, vs)) return *c;
    if (of != &vs) { ix.build(vs.addresses, vs.n); of = &vs; }
    return ix;
  }
};

// Plan one request: its candidates are appended to `runs` (pl.cand_off = the part's candidate
// count before them, pl.ncand = how many).
static int plan_request(const tmed_commit_request *reqs, size_t q, tmed_commit_result &o, Plan &pl,
                        std::vector<Run> &runs, size_t &part_cands, AddrScratch &addr) {
  const tmed_commit_request &r = reqs[q];
  memset(&o, 0, sizeof o);
  int rc = check_request(r);
  if (rc != TMED_OK) return rc;
  const tmed_valset &vs = *r.vals;
  const tmed_commit &c = *r.commit;
  pl.cand_off = part_cands;
  pl.run_lo = runs.size();
  pl.stop = (int32_t)c.n_sigs;
  uint32_t nc = 0;
  const uint32_t qq = (uint32_t)q;
  const bool bid_ok = block_hashes_valid(c.block_id);
  if (r.mode != TMED_MODE_LIGHT_TRUSTING) {
    if (vs.n != c.n_sigs) {
      o.code = TMED_COMMIT_WRONG_SET_SIZE; o.expected = (int64_t)vs.n; o.actual = (int64_t)c.n_sigs;
      pl.decided = true; return TMED_OK;
    }
    if (r.height != c.height) {
      o.code = TMED_COMMIT_WRONG_HEIGHT; o.expected = r.height; o.actual = c.height;
      pl.decided = true; return TMED_OK;
    }
    if (!block_id_equal(*r.block_id, c.block_id)) {
      o.code = TMED_COMMIT_WRONG_BLOCK_ID; pl.decided = true; return TMED_OK;
    }
    pl.needed = vs.total_power * 2 / 3;
    if (r.mode == TMED_MODE_COMMIT) {
      for (size_t i = 0; i < c.n_sigs; i++) {
        const uint8_t f = c.flags[i];
        if (f == kAbsent) continue;
        // CommitSig.BlockID panics on an unknown flag (types/block.go:652-665), sign-bytes of a
        // Commit vote on a malformed hash: the loop stops there if it gets that far
        if ((f != kCommit && f != kNil) || (f == kCommit && !bid_ok)) { pl.panic_idx = (int32_t)i; pl.stop = (int32_t)i; break; }
        push_cand(runs, qq, (int32_t)i, (int32_t)i);
        nc++;
      }
    } else {
      int64_t tally = 0;
      for (size_t i = 0; i < c.n_sigs; i++) {
        if (c.flags[i] != kCommit) continue;
        if (!bid_ok) { pl.panic_idx = (int32_t)i; pl.stop = (int32_t)i; break; }
        push_cand(runs, qq, (int32_t)i, (int32_t)i);
        nc++;
        tally += vs.powers[i];
        if (tally > pl.needed) { pl.stop = (int32_t)i + 1; break; }
      }
    }
  } else {
    if (r.trust_den == 0) { o.code = TMED_COMMIT_ZERO_DENOMINATOR; pl.decided = true; return TMED_OK; }
    int64_t prod;
    if (safe_mul(vs.total_power, r.trust_num, &prod)) { o.code = TMED_COMMIT_OVERFLOW; pl.decided = true; return TMED_OK; }
    pl.needed = prod / r.trust_den;  // Go int64 division truncates toward zero, as C++ does
    std::fill(pl.vof, pl.vof + c.n_sigs, -1);
    const AddrIndex &ix = addr.get(vs);
    thread_local SeenMarks seen;
    seen.reset(vs.n);
    int64_t tally = 0;
    constexpr size_t kAhead = 8;
    bool hashed = false;  // the index is prefetched once a signature missed its position
    for (size_t i = 0; i < c.n_sigs; i++) {
      if (hashed) {
        if (i + kAhead < c.n_sigs) ix.prefetch_slot(c.addresses + 20 * (i + kAhead));
        if (i + kAhead / 2 < c.n_sigs) ix.prefetch_entry(c.addresses + 20 * (i + kAhead / 2));
      }
      if (c.flags[i] != kCommit) continue;
      int32_t v = c.address_lens && c.address_lens[i] != 20 ? -1 : ix.at(c.addresses + 20 * i, i);
      if (v == -2) {
        hashed = true;
        v = lookup_address(ix, c, i);
      }
      if (v < 0) { pl.vof[i] = kNoValidator; continue; }
      if (seen.get(v) >= 0) {  // the loop returns the double-vote error here
        pl.dv_idx = (int32_t)i; pl.dv_val = v; pl.dv_first = seen.get(v);
        pl.stop = (int32_t)i;
        break;
      }
      seen.set(v, (int32_t)i);
      if (!bid_ok) { pl.panic_idx = (int32_t)i; pl.stop = (int32_t)i; break; }
      pl.vof[i] = v;
      push_cand(runs, qq, (int32_t)i, v);
      nc++;
      tally += vs.powers[v];
      if (tally > pl.needed) { pl.stop = (int32_t)i + 1; break; }
    }
  }
  pl.ncand = nc;
  pl.run_hi = runs.size();
  part_cands += nc;
  return TMED_OK;
}

static size_t total_sigs(const tmed_commit_request *reqs, size_t n) {
  size_t s = 0;
  for (size_t q = 0; q < n; q++) s += reqs[q].commit ? reqs[q].commit->n_sigs : 0;
  return s;
}

static void pair_request(const tmed_commit_request *reqs, const std::vector<Plan> &plans, Cands &cands, size_t q,
                         size_t lo, size_t hi, std::vector<std::pair<uint32_t, uint32_t>> &mine);

// Candidates of requests [0, n) in request order (identical to a serial plan).
static bool template_row(const tmed_commit_request &rq, uint8_t *row, bool *fit);

static int seam_plan(const tmed_commit_request *reqs, size_t n, tmed_commit_result *out, Plans &ps, Cands &cands,
                     const KcCall *kc = nullptr, Group *grp = nullptr, Templates *tp = nullptr) {
  PhaseClock clk;
  std::vector<Plan> &plans = ps.v;
  plans.assign(n, Plan());
  cands.clear();
  // worker count: calls of 1,024+ requests fan out at once; smaller ones by their signature count
  // (a blocksync batch: 128 requests of 10k signatures).  Each worker checks its requests as it
  // plans them (plan_request) and keeps the vof arrays of its Trusting requests in a buffer of its
  // own, so no separate pass over the (cold) requests runs first.
  size_t sigs_est = 0;
  if (n < 1024)
    for (size_t q = 0; q < n; q++) sigs_est += reqs[q].commit ? reqs[q].commit->n_sigs : 0;
  const unsigned nt = n >= 1024 ? host_threads(~(size_t)0) : host_threads(sigs_est);
  const unsigned np = std::max(1u, nt);
  if (ps.parts.size() < np) ps.parts.resize(np);
  if (ps.tbits.size() < np) ps.tbits.resize(np);
  std::vector<std::vector<Run>> &part = ps.parts;
  // (parts that never run — parallel_ranges uses at most n of them — keep the empty range [n, n))
  std::vector<size_t> lo_of(np, n), hi_of(np, n), pc(np, 0);
  std::vector<int> rcs(np, TMED_OK);
  std::vector<uint8_t> trusting(np, 0);
  auto plan_range = [&](size_t lo, size_t hi, unsigned t) {
    lo_of[t] = lo; hi_of[t] = hi;
    AddrScratch addr;
    addr.kc = kc;
    size_t c = 0;
    VofArena &va = ps.tbits[t];
    va.reset();
    bool tr = false;
    std::vector<Run> mine;
    mine.swap(part[t]);
    int rc = TMED_OK;
    // the next request's arrays are cold (a light-client batch touches ~5 KB of flags, powers and
    // addresses per request, each request in arrays of its own): their first lines are fetched
    // while this request is planned
    auto prefetch_req = [&](size_t q) {
      if (q >= hi) return;
      const tmed_commit_request &r = reqs[q];
      if (!r.commit || !r.vals) return;
      const tmed_commit &cm = *r.commit;
      const size_t ns = std::min<size_t>(cm.n_sigs, 128);
      for (size_t o = 0; o < ns; o += 64) __builtin_prefetch(cm.flags + o, 0, 0);
      if (r.vals->powers)
        for (size_t o = 0; o < 8 * ns; o += 64) __builtin_prefetch((const uint8_t *)r.vals->powers + o, 0, 0);
      if (r.mode == TMED_MODE_LIGHT_TRUSTING && cm.addresses)
        for (size_t o = 0; o < 20 * ns; o += 64) __builtin_prefetch(cm.addresses + o, 0, 0);
    };
    for (size_t q = lo; q < lo + 4 && q < hi; q++) {  // the structs behind the requests are cold
      __builtin_prefetch(reqs[q].commit, 0, 0);
      __builtin_prefetch(reqs[q].vals, 0, 0);
    }
    prefetch_req(lo);
    for (size_t q = lo; q < hi && rc == TMED_OK; q++) {
      if (q + 4 < hi) {
        __builtin_prefetch(reqs[q + 4].commit, 0, 0);
        __builtin_prefetch(reqs[q + 4].vals, 0, 0);
      }
      prefetch_req(q + 1);
      if (reqs[q].mode == TMED_MODE_LIGHT_TRUSTING && reqs[q].commit) {
        plans[q].vof = va.take(std::max<size_t>(reqs[q].commit->n_sigs, 1));
        tr = true;
      }
      rc = plan_request(reqs, q, out[q], plans[q], mine, c, addr);
    }
    trusting[t] = tr;
    mine.swap(part[t]);
    rcs[t] = rc;
    pc[t] = c;
  };
  for (unsigned t = 0; t < np; t++) part[t].clear();
  if (nt <= 1) plan_range(0, n, 0);
  else parallel_ranges(n, nt, plan_range);
  for (int rc : rcs)
    if (rc != TMED_OK) return rc;
  clk.lap("plan_requests");
  // merge: the parts' runs in thread order (= request order), candidate offsets made global; in the
  // same pass each worker pairs its Trusting requests with their Light partners (pair_request)
  // and, for a device batch (grp), lays out its runs' staging segments without the aliased
  // candidates; one more pass joins the workers' aliases and segments
  std::vector<size_t> rbase(np + 1, 0), cbase(np + 1, 0);
  for (unsigned t = 0; t < np; t++) {
    rbase[t + 1] = rbase[t] + part[t].size();
    cbase[t + 1] = cbase[t] + pc[t];
  }
  const size_t nr = rbase[np], cb = cbase[np];
  cands.runs.resize(nr);
  cands.off.resize(nr + 1);
  cands.off[nr] = cb;
  bool any_trusting = false;
  for (unsigned t = 0; t < np; t++) any_trusting = any_trusting || trusting[t];
  const bool pair = any_trusting && cb <= 0xffffffffu;
  if (pair) {
    cands.tmpl_of.resize(n);
    if (ps.aparts.size() < np) ps.aparts.resize(np);
    if (grp && ps.gparts.size() < np) ps.gparts.resize(np);
  }
  // a device batch planned by several workers also gets its template rows here, each worker
  // encoding the requests of its part that own a row (row_of holds part-local rows until the join)
  const bool rows_here = tp && nt > 1;
  std::vector<uint8_t> tfit(np, 1), tbad(np, 0);
  if (tp) tp->ready = false;
  if (rows_here) {
    tp->row_of.resize(n);
    if (ps.trows.size() < np) ps.trows.resize(np);
  }
  // TMED_TEST_MERGE_SKEW=1 (tests): odd parts start their merge 2 ms late, so a part that read what
  // the next part's worker writes (add_run's end of a part's last run, before the fix) reads it
  // unwritten every time instead of rarely
  const bool skew = nt > 1 && getenv("TMED_TEST_MERGE_SKEW") != nullptr;
  auto merge_part = [&](size_t t) {
    if (skew && (t & 1)) std::this_thread::sleep_for(std::chrono::milliseconds(2));
    // reads from outside part t: part[t], pc, lo_of / hi_of (the planning region, finished), rbase /
    // cbase (the serial prefix sums above); everything else read below is part t's own output of
    // this same body (its runs, offsets and plans, written before pair_request / add_run read them)
    size_t c = cbase[t];
    Run *dst = cands.runs.data() + rbase[t];
    size_t *off = cands.off.data() + rbase[t];
    for (size_t r = 0; r < part[t].size(); r++) {
      dst[r] = part[t][r];
      off[r] = c;
      c += part[t][r].len;
    }
    for (size_t q = lo_of[t]; q < hi_of[t]; q++) {
      plans[q].cand_off += cbase[t];
      plans[q].run_lo += rbase[t];
      plans[q].run_hi += rbase[t];
    }
    auto rows_of_part = [&] {
      std::vector<uint8_t> rows;  // (a header of its own: see seam_plan)
      rows.swap(ps.trows[t]);
      rows.clear();
      uint32_t k = 0;
      bool fit = true;
      for (size_t q = lo_of[t]; q < hi_of[t]; q++) {
        const Plan &pl = plans[q];
        if (pl.run_lo == pl.run_hi || cands.tmpl_row((uint32_t)q) != q) {
          tp->row_of[q] = kNoRow;
          continue;
        }
        rows.resize((size_t)(k + 1) * tmed::kVoteTmplBytes);
        if (!template_row(reqs[q], rows.data() + (size_t)k * tmed::kVoteTmplBytes, &fit)) tbad[t] = 1;
        tp->row_of[q] = k++;
      }
      tfit[t] = fit;
      rows.swap(ps.trows[t]);
    };
    if (!pair) {
      if (rows_here) rows_of_part();
      return;
    }
    for (size_t q = lo_of[t]; q < hi_of[t]; q++) cands.tmpl_of[q] = (uint32_t)q;
    std::vector<std::pair<uint32_t, uint32_t>> mine;  // (a header of its own: see seam_plan)
    mine.swap(ps.aparts[t]);
    mine.clear();
    for (size_t q = lo_of[t]; q < hi_of[t]; q++) pair_request(reqs, plans, cands, q, lo_of[t], hi_of[t], mine);
    if (grp) {
      Group g;
      g.rix.swap(ps.gparts[t].rix);
      g.ub.swap(ps.gparts[t].ub);
      g.pos.swap(ps.gparts[t].pos);
      g.start();
      size_t ap = 0;
      for (size_t r = rbase[t]; r < rbase[t + 1]; r++) g.add_run(cands, (uint32_t)r, mine, ap);
      g.rix.swap(ps.gparts[t].rix);
      g.ub.swap(ps.gparts[t].ub);
      g.pos.swap(ps.gparts[t].pos);
    }
    mine.swap(ps.aparts[t]);
    if (rows_here) rows_of_part();  // after the pairing: tmpl_of of the part is final
  };
  if (nt <= 1) {
    for (unsigned t = 0; t < np; t++) merge_part(t);
  } else {
    parallel_ranges(np, np, [&](size_t lo, size_t hi, unsigned) {
      for (size_t t = lo; t < hi; t++) merge_part(t);
    });
  }
  clk.lap("merge");
  cands.alias.clear();
  if (grp) *grp = Group();  // no aliases: every run whole, in order
  std::vector<size_t> abase(np + 1, 0), sbase(np + 1, 0), pbase(np + 1, 0), tbase(np + 1, 0);
  bool rows_bad = false, rows_fit = true;
  for (unsigned t = 0; t < np; t++) {
    if (pair) {
      abase[t + 1] = abase[t] + ps.aparts[t].size();
      if (grp) {
        const Group &g = ps.gparts[t];
        sbase[t + 1] = sbase[t] + g.rix.size();
        pbase[t + 1] = pbase[t] + (g.rix.empty() ? 0 : g.pos.back());
      }
    }
    if (rows_here) {
      tbase[t + 1] = tbase[t] + ps.trows[t].size() / tmed::kVoteTmplBytes;
      rows_bad = rows_bad || tbad[t];
      rows_fit = rows_fit && tfit[t];
    }
  }
  if (rows_bad) return TMED_EINVAL;  // the encoder rejected a request (as device_templates does)
  const bool aliases = pair && abase[np] != 0;
  if (aliases) {
    cands.alias.resize(abase[np]);
    if (grp) {
      grp->rix.resize(sbase[np]);
      grp->ub.resize(sbase[np]);
      grp->pos.resize(sbase[np] + 1);
      grp->pos[0] = 0;
    }
  }
  if (rows_here) {
    tp->nrows = tbase[np];
    tp->rows.resize(std::max<size_t>(tp->nrows, 1) * tmed::kVoteTmplBytes);
  }
  if (aliases || rows_here) {
    auto join = [&](size_t t) {
      // reads ps.aparts / gparts / trows (the merge region, finished) and the prefix sums above;
      // writes only part t's slices of the joined arrays
      if (rows_here) {
        std::copy(ps.trows[t].begin(), ps.trows[t].end(), tp->rows.begin() + tbase[t] * tmed::kVoteTmplBytes);
        for (size_t q = lo_of[t]; q < hi_of[t]; q++)
          if (tp->row_of[q] != kNoRow) tp->row_of[q] += (uint32_t)tbase[t];
      }
      if (!aliases) return;
      std::copy(ps.aparts[t].begin(), ps.aparts[t].end(), cands.alias.begin() + abase[t]);
      if (!grp) return;
      const Group &g = ps.gparts[t];
      const size_t k = g.rix.size(), s0 = sbase[t], p0 = pbase[t];
      std::copy(g.rix.begin(), g.rix.end(), grp->rix.begin() + s0);
      std::copy(g.ub.begin(), g.ub.end(), grp->ub.begin() + s0);
      for (size_t j = 0; j < k; j++) grp->pos[s0 + j + 1] = p0 + g.pos[j + 1];
    };
    if (nt <= 1) {
      for (unsigned t = 0; t < np; t++) join(t);
    } else {
      parallel_ranges(np, np, [&](size_t lo, size_t hi, unsigned) {
        for (size_t t = lo; t < hi; t++) join(t);
      });
    }
    if (aliases && grp && nt > 1) {
      cands.preq.resize(np + 1);
      for (unsigned t = 0; t < np; t++) cands.preq[t] = lo_of[t];
      cands.preq[np] = n;
      cands.pal = abase;
      cands.pseg = sbase;
    }
  }
  if (rows_here) {
    tp->fits = rows_fit;
    tp->ready = true;
  }
  clk.lap("aliases");
  clk.emit("plan", n, cb);
  return TMED_OK;
}

// ---- candidates verified once for two requests ----------------------------------------
// The light client checks one commit twice, LightTrusting against the trusted set and Light
// against the untrusted one (light/verifier.go:58,73-76), and most validators sign for both
// sets: a Trusting candidate (signature i of a commit, key K) is the same verification as the
// Light / VerifyCommit candidate (signature i of the SAME commit — same_commit — same chain ID,
// same key K) of a neighbouring request.  Such a candidate is sent once; the other takes its bit (C3: ~59 of
// the ~176 candidates of each header).  alias: (candidate, the candidate whose bit it takes).
static bool same_key(const tmed_valset &a, int32_t va, const tmed_valset &b, int32_t vb) {
  if (a.keyset != b.keyset) return false;
  if (a.keyset) {
    const uint32_t ka = a.keyset_index ? a.keyset_index[va] : (uint32_t)va;
    const uint32_t kb = b.keyset_index ? b.keyset_index[vb] : (uint32_t)vb;
    return ka == kb;
  }
  return memcmp(a.pubkeys + 32 * (size_t)va, b.pubkeys + 32 * (size_t)vb, 32) == 0;
}

// One commit for both requests: the same struct, or structs over the same signature, flag and
// timestamp arrays with equal height, round and BlockID (marshallers that copy the struct per
// request).  Then signature i has the same sign-bytes and signature bytes in both.
static bool same_commit(const tmed_commit &a, const tmed_commit &b) {
  if (&a == &b) return true;
  return a.n_sigs == b.n_sigs && a.sigs == b.sigs && a.flags == b.flags && a.ts_seconds == b.ts_seconds &&
         a.ts_nanos == b.ts_nanos && a.sig_lens == b.sig_lens && a.height == b.height && a.round == b.round &&
         block_id_equal(a.block_id, b.block_id);
}

// The aliases of Trusting request q (its partner looked for at q + 1, q - 1 inside [lo, hi): the
// requests one planning worker merged; a pair split across two workers' ranges is not aliased,
// which costs a duplicate verification and nothing else) into `mine`, in candidate order;
// tmpl_of[q] set to the partner.  Runs and offsets of [lo, hi) must be global already.
static void pair_request(const tmed_commit_request *reqs, const std::vector<Plan> &plans, Cands &cands, size_t q,
                         size_t lo, size_t hi, std::vector<std::pair<uint32_t, uint32_t>> &mine) {
  const tmed_commit_request &r = reqs[q];
  const Plan &pl = plans[q];
  if (r.mode != TMED_MODE_LIGHT_TRUSTING || pl.decided || pl.ncand == 0) return;
  for (size_t pq : {q + 1, q - 1}) {  // the pair is adjacent in the light client's batches
    if (pq < lo || pq >= hi) continue;
    const tmed_commit_request &o = reqs[pq];
    const Plan &po = plans[pq];
    if (o.mode == TMED_MODE_LIGHT_TRUSTING || !same_commit(*o.commit, *r.commit) || po.decided || po.ncand == 0 ||
        o.chain_id_len != r.chain_id_len || memcmp(o.chain_id, r.chain_id, r.chain_id_len) != 0)
      continue;
    cands.tmpl_of[q] = (uint32_t)pq;  // one commit, one chain ID: the same sign-bytes template
    // the two sets' key identities (pool indexes, or the keys) are cold: fetch them at once
    // instead of one dependent miss per candidate
    for (const tmed_valset *vs : {r.vals, o.vals}) {
      const uint8_t *kp = vs->keyset ? (const uint8_t *)vs->keyset_index : vs->pubkeys;
      const size_t kb = vs->keyset ? 4 * vs->n : 32 * vs->n;
      if (kp)
        for (size_t b = 0; b < kb; b += 64) __builtin_prefetch(kp + b);
    }
    // o's candidates are its qualifying signatures in order, as runs sorted by signature.  pq lies in
    // [lo, hi), the calling merge part's own requests: plans[pq], its runs and their offsets were
    // written by this part's merge before this call, never by another part
    size_t ro = po.run_lo;
    for (size_t ri = pl.run_lo; ri < pl.run_hi; ri++) {
      const Run &run = cands.runs[ri];
      for (uint32_t u = 0; u < run.len; u++) {
        const int32_t i = run.sig + (int32_t)u;
        while (ro < po.run_hi && cands.runs[ro].sig + (int32_t)cands.runs[ro].len <= i) ro++;
        if (ro == po.run_hi) break;
        const Run &orun = cands.runs[ro];
        if (i < orun.sig || !same_key(*r.vals, run.val + (int32_t)u, *o.vals, orun.val + (i - orun.sig))) continue;
        mine.push_back({(uint32_t)(cands.off[ri] + u), (uint32_t)(cands.off[ro] + (size_t)(i - orun.sig))});
      }
    }
    return;
  }
}

// ---- replay of every reference loop over the validity bits (parallel over requests) ----

static int replay_request(const tmed_commit_request &r, tmed_commit_result &o, const Plan &pl, const uint8_t *valid) {
  const tmed_valset &vs = *r.vals;
  const tmed_commit &c = *r.commit;
  uint32_t k = 0;  // candidates consumed: the loop reaches them in the plan's order
  auto bit = [&](size_t i, bool *ok) -> bool {
    if ((int32_t)i >= pl.stop || k >= pl.ncand) { *ok = false; return false; }
    o.verified++;
    // a signature of any length but 64 is false (ed25519.go:150-152), whatever the verifier said
    return valid[pl.cand_off + k++] != 0 && (!c.sig_lens || c.sig_lens[i] == 64);
  };
  auto panics = [&](size_t i) -> bool {
    if ((int32_t)i != pl.panic_idx) return false;
    o.code = TMED_COMMIT_PANIC;
    o.idx = (int32_t)i;
    return true;
  };
  bool ok = true;
  int64_t tally = 0;
  o.code = -1;
  if (r.mode == TMED_MODE_COMMIT) {
    for (size_t i = 0; i < c.n_sigs && o.code < 0; i++) {
      if (c.flags[i] == kAbsent) continue;
      if (panics(i)) break;
      if (!bit(i, &ok)) { if (ok) { o.code = TMED_COMMIT_WRONG_SIGNATURE; o.idx = (int32_t)i; } break; }
      if (c.flags[i] == kCommit) tally += vs.powers[i];
    }
    if (o.code < 0 && ok) {
      if (tally <= pl.needed) { o.code = TMED_COMMIT_NOT_ENOUGH_POWER; o.got = tally; o.needed = pl.needed; }
      else o.code = TMED_COMMIT_OK;
    }
  } else if (r.mode == TMED_MODE_LIGHT) {
    for (size_t i = 0; i < c.n_sigs && o.code < 0; i++) {
      if (c.flags[i] != kCommit) continue;
      if (panics(i)) break;
      if (!bit(i, &ok)) { if (ok) { o.code = TMED_COMMIT_WRONG_SIGNATURE; o.idx = (int32_t)i; } break; }
      tally += vs.powers[i];
      if (tally > pl.needed) o.code = TMED_COMMIT_OK;
    }
    if (o.code < 0 && ok) { o.code = TMED_COMMIT_NOT_ENOUGH_POWER; o.got = tally; o.needed = pl.needed; }
  } else {
    // the plan resolved every address up to where its loop stopped, and the replay stops no later
    for (size_t i = 0; i < c.n_sigs && o.code < 0; i++) {
      if (c.flags[i] != kCommit || pl.vof[i] == kNoValidator) continue;
      if ((int32_t)i == pl.dv_idx) {
        o.code = TMED_COMMIT_DOUBLE_VOTE; o.val_idx = pl.dv_val; o.idx_first = pl.dv_first; o.idx = (int32_t)i;
        break;
      }
      if (panics(i)) break;
      const int32_t v = pl.vof[i];
      if (v < 0) { ok = false; break; }
      if (!bit(i, &ok)) { if (ok) { o.code = TMED_COMMIT_WRONG_SIGNATURE; o.idx = (int32_t)i; } break; }
      tally += vs.powers[v];
      if (tally > pl.needed) o.code = TMED_COMMIT_OK;
    }
    if (o.code < 0 && ok) { o.code = TMED_COMMIT_NOT_ENOUGH_POWER; o.got = tally; o.needed = pl.needed; }
  }
  return ok ? TMED_OK : TMED_EINVAL;  // replay reached a signature the plan did not send (cannot happen)
}

static int seam_replay(const tmed_commit_request *reqs, size_t n, tmed_commit_result *out, const Plans &ps,
                       const uint8_t *valid) {
  const std::vector<Plan> &plans = ps.v;
  const unsigned nt = host_threads(total_sigs(reqs, n));
  std::vector<int> rcs(std::max(1u, nt), TMED_OK);
  parallel_ranges(n, nt, [&](size_t lo, size_t hi, unsigned t) {
    for (size_t q = lo; q < hi; q++) {
      if (plans[q].decided) continue;
      if (replay_request(reqs[q], out[q], plans[q], valid) != TMED_OK) rcs[t] = TMED_EINVAL;
    }
  });
  for (int rc : rcs)
    if (rc != TMED_OK) return rc;
  return TMED_OK;
}

// Wall time of the three phases of the calling thread's last run_seam (tmed_seam_phase_us).
static thread_local double g_seam_us[3] = {0, 0, 0};

static int run_seam(const tmed_commit_request *reqs, size_t n, tmed_commit_result *out, const BatchVerifier &verify,
                    const KcCall *kc = nullptr) {
  if (n && (!reqs || !out)) return TMED_EINVAL;
  using clock = std::chrono::steady_clock;
  auto us = [](clock::time_point a, clock::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
  const auto t0 = clock::now();
  PhaseClock clk;
  // per-thread planning buffers kept across calls: a light-client batch plans ~1.8M candidates
  // (~60 MB of plans, parts and candidates), and fresh buffers cost a page fault per 4 KB on every
  // call — the planner's threads then serialise on the kernel's page-table lock
  thread_local Plans plans;
  thread_local Cands cands;
  thread_local std::vector<uint8_t> valid;
  int rc = seam_plan(reqs, n, out, plans, cands, kc);
  if (rc != TMED_OK) return rc;
  clk.lap("plan");
  const auto t1 = clock::now();
  // ---- one device batch for every candidate of every request
  const size_t m = cands.size();
  valid.assign(m, 0);
  if (m) {
    rc = verify(reqs, n, cands, valid.data());
    if (rc != TMED_OK) return rc;
  }
  clk.lap("verify");
  const auto t2 = clock::now();
  rc = seam_replay(reqs, n, out, plans, valid.data());
  clk.lap("replay");
  clk.emit("seam", n, m);
  const auto t3 = clock::now();
  g_seam_us[0] = us(t0, t1);
  g_seam_us[1] = us(t1, t2);
  g_seam_us[2] = us(t2, t3);
  return rc;
}

extern "C" int tmed_seam_phase_us(double out_us[3]) {
  if (!out_us) return TMED_EINVAL;
  for (int k = 0; k < 3; k++) out_us[k] = g_seam_us[k];
  return TMED_OK;
}

extern "C" int tmed_verify_commits_with(const tmed_commit_request *reqs, size_t n, tmed_commit_result *out,
                                        tmed_batch_verify_fn verify, void *user) {
  if (!verify) return TMED_EINVAL;
  try {  // no C++ exception crosses the C ABI (c_guard below does the same for the device seams)
    return run_seam(reqs, n, out,
                    [&](const tmed_commit_request *rq, size_t nr, const Cands &cands, uint8_t *valid) {
                      CandBatch cb;
                      int rc = build_cand_batch(rq, nr, cands, cb);
                      if (rc != TMED_OK) return rc;
                      return verify(user, cb.pubs.data(), cb.sigs.data(), cb.lens.data(), cb.msgs.data(),
                                    cb.offs.data(), cb.m, valid);
                    });
  } catch (const std::bad_alloc &) {
    return TMED_ENOMEM;
  }
}

// The group of every run without its aliased candidates: run ranges built in parallel (a
// light-client batch has ~90k aliases, one per Trusting vote), then joined.
static void build_group(const Cands &c, Group &g) {
  const size_t nr = c.runs.size();
  const unsigned nt = c.alias.size() >= 8192 ? host_threads(c.size()) : 1u;
  std::vector<Group> part(std::max(1u, std::min<unsigned>(nt, (unsigned)std::max<size_t>(nr, 1))));
  parallel_ranges(nr, nt, [&](size_t lo, size_t hi, unsigned t) {
    Group mine;  // (a header of its own: see seam_plan)
    mine.start();
    // c (runs, off, alias) is complete before this region (seam_plan returned): no part writes it
    const auto a0 = std::lower_bound(c.alias.begin(), c.alias.end(), std::make_pair((uint32_t)c.off[lo], 0u));
    size_t ap = (size_t)(a0 - c.alias.begin());
    for (size_t r = lo; r < hi; r++) mine.add_run(c, (uint32_t)r, c.alias, ap);
    part[t].rix.swap(mine.rix);
    part[t].ub.swap(mine.ub);
    part[t].pos.swap(mine.pos);
  });
  size_t ns = 0;
  std::vector<size_t> sbase(part.size() + 1, 0), pbase(part.size() + 1, 0);
  for (size_t t = 0; t < part.size(); t++) {
    const size_t k = part[t].rix.size();
    sbase[t + 1] = sbase[t] + k;
    pbase[t + 1] = pbase[t] + (k ? part[t].pos.back() : 0);
    ns += k;
  }
  g.rix.resize(ns);
  g.ub.resize(ns);
  g.pos.resize(ns + 1);
  g.pos[0] = 0;
  parallel_ranges(part.size(), (unsigned)part.size(), [&](size_t lo, size_t hi, unsigned) {
    for (size_t t = lo; t < hi; t++) {
      const Group &p = part[t];
      const size_t k = p.rix.size(), s = sbase[t], pb = pbase[t];
      std::copy(p.rix.begin(), p.rix.end(), g.rix.begin() + s);
      std::copy(p.ub.begin(), p.ub.end(), g.ub.begin() + s);
      for (size_t j = 0; j < k; j++) g.pos[s + j + 1] = pb + p.pos[j + 1];
    }
  });
}

// The verified bits of the aliased candidates (scatter_bits wrote their targets).
static void copy_aliases(const Cands &c, uint8_t *valid) {
  const size_t na = c.alias.size();
  parallel_ranges(na, na >= 8192 ? host_threads(c.size()) : 1u, [&](size_t lo, size_t hi, unsigned) {
    for (size_t k = lo; k < hi; k++) valid[c.alias[k].first] = valid[c.alias[k].second];
  });
}

// For f(j, u0, u1, p0): the segment u0 .. u1 - 1 of group run j, staged from position p0, for the
// positions [lo, hi) of a thread's share (runs split across threads are cut at the share edges).
template <class F>
static void for_segments(const Cands &c, const Group &g, size_t lo, size_t hi, F &&f) {
  const size_t *pos = g.positions(c);
  const size_t nr = g.nruns(c);
  size_t j = (size_t)(std::upper_bound(pos, pos + nr + 1, lo) - pos);
  j = j ? j - 1 : 0;
  for (; j < nr && pos[j] < hi; j++) {
    const size_t a = std::max(lo, pos[j]), b = std::min(hi, pos[j + 1]);
    const uint32_t u = g.base(j);
    if (a < b) f(j, u + (uint32_t)(a - pos[j]), u + (uint32_t)(b - pos[j]), a);
  }
}

// Request q's template row (kVoteTmplBytes at row); false: the encoder rejected the request
// (bad), or *fit = false when its template does not fit the device assembler.
static bool template_row(const tmed_commit_request &rq, uint8_t *row, bool *fit) {
  const tmed_commit &c = *rq.commit;
  tmed_vote_template t;
  t.chain_id = rq.chain_id;
  t.chain_id_len = rq.chain_id_len;
  t.height = c.height;
  t.round = c.round;
  t.block_hash = c.block_id.hash;
  t.block_hash_len = c.block_id.hash_len;
  t.psh_total = c.block_id.psh_total;
  t.psh_hash = c.block_id.psh_hash;
  t.psh_hash_len = c.block_id.psh_hash_len;
  tmed::VoteEncoder e;
  if (e.init(&t) != TMED_OK) return false;
  memset(row, 0, tmed::kVoteTmplBytes);
  if (!e.device_template(row, tmed::kVoteTmplBytes, tmed::kVoteSlot)) *fit = false;
  return true;
}

static int device_templates(const tmed_commit_request *reqs, size_t n, const Cands &cands, Templates &tp,
                            bool *fits) {
  tp.row_of.assign(n, kNoRow);
  for (const Run &r : cands.runs) tp.row_of[cands.tmpl_row(r.req)] = 0;
  size_t k = 0;
  for (size_t q = 0; q < n; q++)
    if (tp.row_of[q] != kNoRow) tp.row_of[q] = (uint32_t)k++;
  tp.nrows = k;
  tp.rows.resize(std::max<size_t>(k, 1) * tmed::kVoteTmplBytes);
  std::atomic<bool> ok{true}, bad{false};
  parallel_ranges(n, n >= 64 ? host_threads(cands.size()) : 1, [&](size_t lo, size_t hi, unsigned) {
    for (size_t q = lo; q < hi; q++) {
      if (tp.row_of[q] == kNoRow) continue;
      bool fit = true;
      if (!template_row(reqs[q], &tp.rows[(size_t)tp.row_of[q] * tmed::kVoteTmplBytes], &fit)) bad = true;
      if (!fit) ok = false;
    }
  });
  if (bad) return TMED_EINVAL;
  *fits = ok;
  return TMED_OK;
}

// Collected bits of a group -> valid[] by candidate (signatures of length != 64 are false:
// ed25519.go:150-152).
static void scatter_range(const tmed_commit_request *reqs, const Cands &cands, const Group &grp, const uint8_t *bits,
                          uint8_t *valid, size_t lo, size_t hi) {
  for_segments(cands, grp, lo, hi, [&](size_t j, uint32_t u0, uint32_t u1, size_t p) {
    const uint32_t ri = grp.run(cands, j);
    const Run &run = cands.runs[ri];
    const tmed_commit &c = *reqs[run.req].commit;
    uint8_t *dst = valid + cands.off[ri];
    for (uint32_t u = u0; u < u1; u++) {
      const uint32_t sl = c.sig_lens ? c.sig_lens[run.sig + (int32_t)u] : 64;
      dst[u] = sl == 64 ? bits[p + (u - u0)] : 0;
    }
  });
}
static void scatter_bits(const tmed_commit_request *reqs, const Cands &cands, const Group &grp, const uint8_t *bits,
                         uint8_t *valid) {
  const size_t m = grp.size(cands);
  parallel_ranges(m, host_threads(m), [&](size_t lo, size_t hi, unsigned) {
    scatter_range(reqs, cands, grp, bits, valid, lo, hi);
  });
}


// The part-wise finish of a pipelined batch (bs_finish): the planning workers' parts of an aliased
// batch, each in one fork-join — its staged bits -> valid[] by candidate, its aliased bits, then the
// replay of its requests.  Part t reads only candidates of its own requests: its staging segments
// [pseg[t], pseg[t+1]) hold exactly its runs, and every alias lies inside its part (pair_request
// pairs within the merging worker's range).  out: the results of requests [0, n) of the batch.
static int finish_parts(const tmed_commit_request *rq, const Cands &cd, const Group &grp, const uint8_t *bits,
                        uint8_t *valid, const Plans &ps, tmed_commit_result *out) {
  const size_t np = cd.preq.size() - 1;
  std::vector<int> rcs(np, TMED_OK);
  parallel_ranges(np, (unsigned)np, [&](size_t lo, size_t hi, unsigned) {
    for (size_t t = lo; t < hi; t++) {
      scatter_range(rq, cd, grp, bits, valid, grp.pos[cd.pseg[t]], grp.pos[cd.pseg[t + 1]]);
      for (size_t k = cd.pal[t]; k < cd.pal[t + 1]; k++) valid[cd.alias[k].first] = valid[cd.alias[k].second];
      for (size_t q = cd.preq[t]; q < cd.preq[t + 1]; q++)
        if (!ps.v[q].decided && replay_request(rq[q], out[q], ps.v[q], valid) != TMED_OK) rcs[t] = TMED_EINVAL;
    }
  });
  for (int rc : rcs)
    if (rc != TMED_OK) return rc;
  return TMED_OK;
}
