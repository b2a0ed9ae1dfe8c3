// go_marshal.cpp — the host-side marshal of the cgo shim (go/tmedgpu/tmedgpu.go)
// in compiled code, over the reference's objects as Go 1.18 holds them in memory (amd64).
//
// The reference's callers hold a commit as types.Commit (types/block.go:737-752) with a
// []CommitSig (types/block.go:595-600): per signature an 80-byte struct with the flag, the
// ValidatorAddress slice header (its 20 bytes a separate heap object), a time.Time and the
// Signature slice header (its 64 bytes another heap object); a validator set as
// types.ValidatorSet (types/validator_set.go:51-58) of []*Validator, each holding its PubKey as a
// crypto.PubKey interface whose data word points at the ed25519.PubKey slice header.  Go is not
// in this image, so this C++ stand-in reproduces those layouts (go_* builders, untimed) and the
// shim's flatten into the C ABI structs of include/tmed25519.h (gm_marshal_*, timed by the
// benches beside the seam): what a drop-in caller pays on the host before tmed_verify_commits /
// tmed_blocksync_submit run.
//
// The flatten follows the rewritten shim: every per-call array comes from buffers preallocated
// once and reused (no per-signature allocation), a validator set is flattened once per *ValSet
// seen (a replay reuses state.Validators window after window), the light client passes each
// set's ValidatorsHash as set_hash, and a VerifyCommitLight commit is marshalled only up to its
// 2/3 crossing — the reference loop (types/validator_set.go:739-761) returns there and never reads
// a later CommitSig; the tail's flags are written as BlockIDFlagAbsent (never reached either way),
// so the outcome is the reference's by construction.  Threads: OpenMP over commits.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "tmed25519.h"

namespace {

// ---- Go 1.18 amd64 layouts --------------------------------------------------------------------
struct GoSlice {
  uint8_t *p;
  int64_t len, cap;
};
struct GoTime {  // time.Time: wall (hasMonotonic bit 63 | 33-bit seconds | 30-bit nanoseconds), ext, loc
  uint64_t wall;
  int64_t ext;
  void *loc;
};
struct GoCommitSig {  // types.CommitSig
  uint8_t flag;
  uint8_t pad_[7];
  GoSlice address;
  GoTime ts;
  GoSlice sig;
};
static_assert(sizeof(GoCommitSig) == 80, "CommitSig is 80 bytes on amd64");
struct GoBlockID {  // types.BlockID{Hash []byte; PartSetHeader{Total uint32; Hash []byte}}
  GoSlice hash;
  uint32_t psh_total;
  uint32_t pad_;
  GoSlice psh_hash;
};
struct GoCommit {  // types.Commit
  int64_t height;
  int32_t round;
  int32_t pad_;
  GoBlockID block_id;
  GoSlice sigs;  // []CommitSig: p -> GoCommitSig[len]
  GoSlice hash;
  void *bit_array;
};
struct GoIface {
  void *itab;
  void *data;  // -> the ed25519.PubKey slice header (a heap copy: a slice is not pointer-shaped)
};
struct GoValidator {  // types.Validator
  GoSlice address;
  GoIface pub_key;
  int64_t voting_power;
  int64_t proposer_priority;
};
struct GoValSet {  // types.ValidatorSet
  GoSlice validators;  // []*Validator: p -> GoValidator*[len]
  GoValidator *proposer;
  int64_t total_voting_power;
};

constexpr int64_t kUnixToInternal = 62135596800LL;  // seconds from year 1 to 1970 (time.go)
constexpr int64_t kWallToInternal = 59453308800LL;  // seconds from year 1 to 1885 (time.go)

inline int64_t go_unix(const GoTime &t) {  // Time.Unix()
  const int64_t sec = (t.wall >> 63) ? kWallToInternal + (int64_t)((t.wall << 1) >> 31) : t.ext;
  return sec - kUnixToInternal;
}
inline int32_t go_nanos(const GoTime &t) { return (int32_t)(t.wall & ((1u << 30) - 1)); }  // Time.Nanosecond()

// Bump allocator standing in for Go's size-class spans (objects of one class laid out in order).
struct Bump {
  std::vector<uint8_t *> blocks;
  uint8_t *cur = nullptr;
  size_t left = 0;
  void *get(size_t n) {
    n = (n + 7) & ~(size_t)7;
    if (n > left) {
      const size_t sz = n > ((size_t)64 << 20) ? n : ((size_t)64 << 20);
      cur = (uint8_t *)malloc(sz);
      blocks.push_back(cur);
      left = sz;
    }
    void *p = cur;
    cur += n;
    left -= n;
    return p;
  }
  ~Bump() {
    for (uint8_t *b : blocks) free(b);
  }
};

}  // namespace

// ---- the Go heap (builders: untimed setup of the synthetic reference objects) --------------------
struct gm_heap {
  Bump structs, addr24, sig64, key32, misc;
  std::vector<GoCommit *> commits;
  std::vector<GoValSet *> sets;
};

// ---- the shim's reusable C memory --------------------------------------------------------------
// pointer -> index, open addressing (the shim's map[*ValSet] / map[*Commit], cleared per call
// without freeing)
struct PtrMap {
  std::vector<const void *> key;
  std::vector<size_t> val;
  size_t n = 0, mask = 0;
  void clear() {
    if (n) std::fill(key.begin(), key.end(), nullptr);
    n = 0;
  }
  void reserve(size_t want) {
    size_t cap = 64;
    while (cap < 2 * want) cap <<= 1;
    if (cap <= key.size()) return;
    std::vector<const void *> ok;
    std::vector<size_t> ov;
    ok.swap(key);
    ov.swap(val);
    key.assign(cap, nullptr);
    val.assign(cap, 0);
    mask = cap - 1;
    n = 0;
    for (size_t i = 0; i < ok.size(); i++)
      if (ok[i]) insert(ok[i], ov[i]);
  }
  static size_t slot(const void *p) { return (size_t)(((uintptr_t)p >> 3) * 0x9E3779B97F4A7C15ull >> 17); }
  // the index of p, or inserts v and returns it
  size_t find_or_insert(const void *p, size_t v, bool &fresh) {
    if (2 * (n + 1) > key.size()) reserve(n + 1);
    size_t h = slot(p) & mask;
    while (key[h] && key[h] != p) h = (h + 1) & mask;
    fresh = key[h] == nullptr;
    if (fresh) {
      key[h] = p;
      val[h] = v;
      n++;
    }
    return val[h];
  }
  void insert(const void *p, size_t v) {
    bool f;
    (void)find_or_insert(p, v, f);
  }
};

struct gm_ctx {
  int threads = 16;
  // per commit slot: the flat arrays of its tmed_commit (grown, never shrunk)
  struct CommitBuf {
    std::vector<uint8_t> flags, addrs;
    std::vector<int64_t> sec;
    std::vector<int32_t> nsec;
    std::vector<uint8_t> sigs;  // used when no pinned arena is given
    std::vector<uint32_t> slen, alen;
    std::vector<uint8_t> bid;   // hash + psh hash bytes
  };
  std::vector<CommitBuf> cb;
  std::vector<tmed_commit> commits;
  std::vector<tmed_block_id> bids;  // expected BlockIDs (requests / window)
  std::vector<std::vector<uint8_t>> bid_bytes;
  std::vector<int64_t> heights;
  // flattened validator sets, once per *ValSet (the shim's per-set cache)
  struct SetBuf {
    std::vector<uint8_t> pubs, addrs;
    std::vector<int64_t> powers;
    uint8_t hash[32];
    bool has_hash = false, has_addrs = false, flat = false;
  };
  PtrMap set_slot;             // *ValSet -> slot in sb
  std::vector<SetBuf> sb;      // slots [0, nsb) in use; the buffers of later slots are kept for reuse
  size_t nsb = 0;
  std::vector<tmed_valset> vals;
  std::vector<tmed_commit_request> reqs;
  std::vector<char> chain;
  // gm_marshal_requests scratch (kept across calls)
  PtrMap commit_slot;
  std::vector<const GoCommit *> cl;
  std::vector<uint8_t> c_trust;
  std::vector<size_t> rc, rs;
  std::vector<const GoValSet *> setp;  // slot -> *ValSet
  tmed_blocksync_window win{};
};

namespace {

void flatten_set(gm_ctx::SetBuf &s, const GoValSet *v, bool addresses) {
  const size_t n = (size_t)v->validators.len;
  GoValidator *const *vs = (GoValidator *const *)v->validators.p;
  s.pubs.resize(32 * n);
  s.powers.resize(n);
  if (addresses) s.addrs.resize(20 * n);
  constexpr size_t kAhead = 8;  // the *Validator -> PubKey -> bytes chain, prefetched a few validators ahead
  for (size_t i = 0; i < n && i < kAhead; i++) __builtin_prefetch(vs[i]);
  for (size_t i = 0; i < n; i++) {
    if (i + kAhead < n) __builtin_prefetch(vs[i + kAhead]);
    if (i + kAhead / 2 < n) __builtin_prefetch(vs[i + kAhead / 2]->pub_key.data);
    const GoValidator *x = vs[i];
    const GoSlice *pk = (const GoSlice *)x->pub_key.data;  // ed25519.PubKey
    memcpy(&s.pubs[32 * i], pk->p, 32);
    s.powers[i] = x->voting_power;
    if (addresses) memcpy(&s.addrs[20 * i], x->address.p, 20);
  }
  s.flat = true;
  s.has_addrs = s.has_addrs || addresses;
}

// The commit's arrays for the seam.  upto: CommitSigs [0, upto) are marshalled, the rest get the
// flag BlockIDFlagAbsent only (a Light commit past its crossing: never read by the loop).
void flatten_commit(gm_ctx::CommitBuf &b, tmed_commit &c, const GoCommit *g, size_t upto, bool addresses,
                    uint8_t *sig_dst) {
  const size_t n = (size_t)g->sigs.len;
  const GoCommitSig *cs = (const GoCommitSig *)g->sigs.p;
  if (b.flags.size() < n) {
    b.flags.resize(n);
    b.sec.resize(n);
    b.nsec.resize(n);
    b.slen.resize(n);
  }
  if (addresses && b.addrs.size() < 20 * n) {
    b.addrs.resize(20 * n);
    b.alen.resize(n);
  }
  if (!sig_dst) {
    if (b.sigs.size() < 64 * n) b.sigs.resize(64 * n);
    sig_dst = b.sigs.data();
  }
  for (size_t i = 0; i < upto; i++) {
    const GoCommitSig &s = cs[i];
    b.flags[i] = s.flag;
    b.sec[i] = go_unix(s.ts);
    b.nsec[i] = go_nanos(s.ts);
    const size_t sl = (size_t)s.sig.len;
    b.slen[i] = (uint32_t)sl;
    uint8_t *d = sig_dst + 64 * i;
    if (sl >= 64) {
      memcpy(d, s.sig.p, 64);
    } else {
      memset(d, 0, 64);
      if (sl) memcpy(d, s.sig.p, sl);
    }
    if (addresses) {
      const size_t al = (size_t)s.address.len;
      b.alen[i] = (uint32_t)al;
      if (al == 20) memcpy(&b.addrs[20 * i], s.address.p, 20);
      else memset(&b.addrs[20 * i], 0, 20);
    }
  }
  if (upto < n) memset(b.flags.data() + upto, 1, n - upto);
  const GoBlockID &id = g->block_id;
  const size_t hl = (size_t)id.hash.len, pl = (size_t)id.psh_hash.len;
  b.bid.resize(hl + pl + 1);
  if (hl) memcpy(b.bid.data(), id.hash.p, hl);
  if (pl) memcpy(b.bid.data() + hl, id.psh_hash.p, pl);
  c.height = g->height;
  c.round = g->round;
  c.block_id = tmed_block_id{b.bid.data(), (uint32_t)hl, id.psh_total, b.bid.data() + hl, (uint32_t)pl};
  c.n_sigs = n;
  c.flags = b.flags.data();
  c.addresses = addresses ? b.addrs.data() : nullptr;
  c.ts_seconds = b.sec.data();
  c.ts_nanos = b.nsec.data();
  c.sigs = sig_dst;
  c.sig_lens = b.slen.data();
  c.address_lens = addresses ? b.alen.data() : nullptr;
}

// CommitSigs a VerifyCommitLight loop reads: up to and including the one whose power crosses
// total * 2 / 3 (types/validator_set.go:739-761); all of them when it never crosses.
size_t light_prefix(const GoCommit *g, const int64_t *powers, int64_t total, size_t nvals) {
  const size_t n = (size_t)g->sigs.len;
  if (n != nvals) return n;  // the size check fails first: the seam reads nothing past it anyway
  const GoCommitSig *cs = (const GoCommitSig *)g->sigs.p;
  const int64_t needed = total * 2 / 3;
  int64_t tally = 0;
  for (size_t i = 0; i < n; i++) {
    if (cs[i].flag != 2) continue;  // ForBlock
    tally += powers[i];
    if (tally > needed) return i + 1;
  }
  return n;
}

void copy_bid(std::vector<uint8_t> &store, tmed_block_id &out, const GoBlockID &id) {
  const size_t hl = (size_t)id.hash.len, pl = (size_t)id.psh_hash.len;
  store.resize(hl + pl + 1);
  if (hl) memcpy(store.data(), id.hash.p, hl);
  if (pl) memcpy(store.data() + hl, id.psh_hash.p, pl);
  out = tmed_block_id{store.data(), (uint32_t)hl, id.psh_total, store.data() + hl, (uint32_t)pl};
}

}  // namespace

extern "C" {

// ---- builders ----------------------------------------------------------------------------------
gm_heap *gm_heap_new(void) { return new gm_heap(); }
void gm_heap_free(gm_heap *h) { delete h; }

// A commit as types.Commit from flat arrays (n signatures; ts as Unix seconds + nanoseconds,
// stored the way time.Unix(..).UTC() leaves them: no monotonic reading).  Returns its index.
int64_t go_commit_build(gm_heap *h, int64_t height, int32_t round, const uint8_t *hash, uint32_t hash_len,
                        uint32_t psh_total, const uint8_t *psh, uint32_t psh_len, size_t n, const uint8_t *flags,
                        const uint8_t *addrs,
                        const uint32_t *addr_lens, const int64_t *sec, const int32_t *nsec, const uint8_t *sigs,
                        const uint32_t *sig_lens) {
  GoCommit *c = (GoCommit *)h->structs.get(sizeof(GoCommit));
  memset(c, 0, sizeof *c);
  c->height = height;
  c->round = round;
  c->block_id.hash.p = (uint8_t *)h->misc.get(hash_len + 1);
  if (hash_len) memcpy(c->block_id.hash.p, hash, hash_len);
  c->block_id.hash.len = c->block_id.hash.cap = hash_len;
  c->block_id.psh_total = psh_total;
  c->block_id.psh_hash.p = (uint8_t *)h->misc.get(psh_len + 1);
  if (psh_len) memcpy(c->block_id.psh_hash.p, psh, psh_len);
  c->block_id.psh_hash.len = c->block_id.psh_hash.cap = psh_len;
  GoCommitSig *cs = (GoCommitSig *)h->structs.get(sizeof(GoCommitSig) * (n ? n : 1));
  for (size_t i = 0; i < n; i++) {
    GoCommitSig &s = cs[i];
    memset(&s, 0, sizeof s);
    s.flag = flags[i];
    const uint32_t al = addr_lens ? addr_lens[i] : (flags[i] == 1 ? 0u : 20u);
    if (al) {
      s.address.p = (uint8_t *)h->addr24.get(24);
      memcpy(s.address.p, addrs + 20 * i, al < 20 ? al : 20);
      s.address.len = s.address.cap = al;
    }
    s.ts.ext = sec[i] + kUnixToInternal;
    s.ts.wall = (uint64_t)(uint32_t)nsec[i];
    const uint32_t sl = sig_lens ? sig_lens[i] : 64u;
    if (sl) {
      s.sig.p = (uint8_t *)h->sig64.get(64);
      memcpy(s.sig.p, sigs + 64 * i, sl < 64 ? sl : 64);
      s.sig.len = s.sig.cap = sl;
    }
  }
  c->sigs.p = (uint8_t *)cs;
  c->sigs.len = c->sigs.cap = (int64_t)n;
  h->commits.push_back(c);
  return (int64_t)h->commits.size() - 1;
}

// A validator set as types.ValidatorSet (validators in set order).  Returns its index.
int64_t go_valset_build(gm_heap *h, size_t n, const uint8_t *pubs, const int64_t *powers, const uint8_t *addrs) {
  GoValSet *v = (GoValSet *)h->structs.get(sizeof(GoValSet));
  memset(v, 0, sizeof *v);
  GoValidator **arr = (GoValidator **)h->structs.get(sizeof(GoValidator *) * (n ? n : 1));
  int64_t total = 0;
  for (size_t i = 0; i < n; i++) {
    GoValidator *x = (GoValidator *)h->structs.get(sizeof(GoValidator));
    memset(x, 0, sizeof *x);
    x->address.p = (uint8_t *)h->addr24.get(24);
    memcpy(x->address.p, addrs + 20 * i, 20);
    x->address.len = x->address.cap = 20;
    GoSlice *pk = (GoSlice *)h->misc.get(sizeof(GoSlice));
    pk->p = (uint8_t *)h->key32.get(32);
    memcpy(pk->p, pubs + 32 * i, 32);
    pk->len = pk->cap = 32;
    x->pub_key.data = pk;
    x->voting_power = powers[i];
    total += powers[i];
    arr[i] = x;
  }
  v->validators.p = (uint8_t *)arr;
  v->validators.len = v->validators.cap = (int64_t)n;
  v->total_voting_power = total;
  h->sets.push_back(v);
  return (int64_t)h->sets.size() - 1;
}

// ---- the shim's marshal (timed) ------------------------------------------------------------------
gm_ctx *gm_ctx_new(int threads) {
  gm_ctx *c = new gm_ctx();
  c->threads = threads > 0 ? threads : 1;
  return c;
}
void gm_ctx_free(gm_ctx *c) { delete c; }
void gm_forget_sets(gm_ctx *c) {  // the per-*ValSet cache starts empty (its buffers are kept)
  c->set_slot.clear();
  c->nsb = 0;
}

// The slot of *ValSet v (new slots are flattened by the caller).
static size_t set_of(gm_ctx *c, const GoValSet *v, const uint8_t *hash) {
  bool fresh;
  const size_t k = c->set_slot.find_or_insert(v, c->nsb, fresh);
  if (!fresh) return k;
  if (c->nsb == c->sb.size()) c->sb.emplace_back();
  if (c->setp.size() <= k) c->setp.resize(k + 1);
  c->setp[k] = v;
  c->nsb++;
  gm_ctx::SetBuf &s = c->sb[k];
  s.flat = s.has_addrs = false;
  s.has_hash = hash != nullptr;
  if (hash) memcpy(s.hash, hash, 32);
  return k;
}

static tmed_valset valset_of(const gm_ctx::SetBuf &s, const GoValSet *v) {
  tmed_valset t{};
  t.n = s.powers.size();
  t.pubkeys = s.pubs.data();
  t.powers = s.powers.data();
  t.addresses = s.has_addrs ? s.addrs.data() : nullptr;
  t.total_power = v->total_voting_power;
  t.set_hash = s.has_hash ? s.hash : nullptr;
  return t;
}

// A blocksync window: block h = set.VerifyCommitLight(chain, expected[h], heights[h], commits[h])
// (blockchain/v0/reactor.go:366-367).  Fills and returns the tmed_blocksync_window (valid until
// the next gm_ call on this context); the signatures go to sig_arena (pinned, >= 64 x the
// window's signatures) when given.  set_hash: state.Validators' hash, or NULL.
const tmed_blocksync_window *gm_marshal_window(gm_ctx *c, gm_heap *h, int64_t set, const int64_t *commit_idx,
                                               const int64_t *heights, size_t n, const char *chain, uint32_t chain_len,
                                               const uint8_t *set_hash, uint8_t *sig_arena) {
  const GoValSet *v = h->sets[(size_t)set];
  const size_t sk = set_of(c, v, set_hash);
  gm_ctx::SetBuf &s = c->sb[sk];
  if (!s.flat) flatten_set(s, v, false);
  c->vals.resize(1);
  c->vals[0] = valset_of(s, v);
  if (c->cb.size() < n) c->cb.resize(n);
  c->commits.resize(n);
  c->bids.resize(n);
  c->bid_bytes.resize(n);
  c->heights.assign(heights, heights + n);
  // each commit's signature run goes to its own place in the arena: offsets by a prefix sum
  std::vector<size_t> off(n + 1, 0);
  for (size_t i = 0; i < n; i++) off[i + 1] = off[i] + 64 * (size_t)h->commits[(size_t)commit_idx[i]]->sigs.len;
  const int64_t *pw = s.powers.data();
  const int64_t total = v->total_voting_power;
  const size_t nv = s.powers.size();
#pragma omp parallel for schedule(dynamic, 4) num_threads(c->threads)
  for (size_t i = 0; i < n; i++) {
    const GoCommit *g = h->commits[(size_t)commit_idx[i]];
    const size_t upto = light_prefix(g, pw, total, nv);
    flatten_commit(c->cb[i], c->commits[i], g, upto, false, sig_arena ? sig_arena + off[i] : nullptr);
    copy_bid(c->bid_bytes[i], c->bids[i], g->block_id);  // the reactor's firstID: the block's own ID here
  }
  c->chain.assign(chain, chain + chain_len);
  c->chain.push_back(0);
  c->win = tmed_blocksync_window{c->chain.data(), chain_len, c->vals.data(), n, c->bids.data(), c->heights.data(),
                                 c->commits.data()};
  return &c->win;
}

// Light-client requests: request q = (mode[q], sets[set_idx[q]], commits[commit_idx[q]], expected
// BlockID = that commit's own ID for COMMIT / LIGHT, heights[q], trust num / den).  set_hashes:
// NULL or 32 bytes per set index (header.ValidatorsHash).  One C valset per distinct *ValSet and one
// C commit per distinct *Commit, as the shim's maps do.  Returns the request array (n entries).
const tmed_commit_request *gm_marshal_requests(gm_ctx *c, gm_heap *h, size_t n, const int32_t *mode,
                                               const int64_t *set_idx, const int64_t *commit_idx,
                                               const int64_t *heights, const int64_t *tnum, const int64_t *tden,
                                               const char *chain, uint32_t chain_len, const uint8_t *set_hashes) {
  // distinct sets / commits in first-seen order (the shim's map[*ValSet] / map[*Commit])
  PtrMap &cslot = c->commit_slot;
  cslot.clear();
  cslot.reserve(n);
  std::vector<const GoCommit *> &cl = c->cl;
  std::vector<uint8_t> &c_trust = c->c_trust;  // a commit checked by a Trusting request needs its addresses
  std::vector<size_t> &rc = c->rc, &rs = c->rs;
  std::vector<const GoValSet *> &setp = c->setp;
  cl.clear();
  c_trust.clear();
  rc.resize(n);
  rs.resize(n);
  c->set_slot.reserve(c->nsb + n);
  for (size_t q = 0; q < n; q++) {
    const GoValSet *v = h->sets[(size_t)set_idx[q]];
    rs[q] = set_of(c, v, set_hashes ? set_hashes + 32 * (size_t)set_idx[q] : nullptr);
    const GoCommit *g = h->commits[(size_t)commit_idx[q]];
    bool fresh;
    const size_t k = cslot.find_or_insert(g, cl.size(), fresh);
    if (fresh) {
      cl.push_back(g);
      c_trust.push_back(0);
    }
    rc[q] = k;
    if (mode[q] == TMED_MODE_LIGHT_TRUSTING) c_trust[k] = 1;
  }
  // sets not flattened yet (and those a Trusting request now needs the addresses of): in parallel
  std::vector<uint8_t> need_addr(c->nsb, 0);
  for (size_t q = 0; q < n; q++)
    if (mode[q] == TMED_MODE_LIGHT_TRUSTING) need_addr[rs[q]] = 1;
  std::vector<size_t> todo;
  for (size_t k = 0; k < c->nsb; k++)
    if (!c->sb[k].flat || (need_addr[k] && !c->sb[k].has_addrs)) todo.push_back(k);
#pragma omp parallel for schedule(dynamic, 16) num_threads(c->threads)
  for (size_t j = 0; j < todo.size(); j++) {
    const size_t sk = todo[j];
    flatten_set(c->sb[sk], setp[sk], need_addr[sk] != 0);
  }
  c->vals.resize(c->nsb);
  for (size_t k = 0; k < c->nsb; k++) c->vals[k] = valset_of(c->sb[k], setp[k]);
  const size_t nc = cl.size();
  if (c->cb.size() < nc) c->cb.resize(nc);
  c->commits.resize(nc);
#pragma omp parallel for schedule(dynamic, 16) num_threads(c->threads)
  for (size_t k = 0; k < nc; k++)
    flatten_commit(c->cb[k], c->commits[k], cl[k], (size_t)cl[k]->sigs.len, c_trust[k] != 0, nullptr);
  c->bids.resize(n);
  c->bid_bytes.resize(n);
  c->reqs.resize(n);
  c->chain.assign(chain, chain + chain_len);
  c->chain.push_back(0);
#pragma omp parallel for schedule(static) num_threads(c->threads)
  for (size_t q = 0; q < n; q++) {
    tmed_commit_request &r = c->reqs[q];
    memset(&r, 0, sizeof r);
    r.mode = mode[q];
    r.chain_id = c->chain.data();
    r.chain_id_len = chain_len;
    r.vals = &c->vals[rs[q]];
    r.commit = &c->commits[rc[q]];
    r.height = heights[q];
    r.trust_num = tnum[q];
    r.trust_den = tden[q];
    if (mode[q] != TMED_MODE_LIGHT_TRUSTING) {
      copy_bid(c->bid_bytes[q], c->bids[q], h->commits[(size_t)commit_idx[q]]->block_id);
      r.block_id = &c->bids[q];
    }
  }
  return c->reqs.data();
}

}  // extern "C"
