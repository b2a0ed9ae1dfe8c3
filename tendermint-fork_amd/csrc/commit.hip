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
#include <string.h>

#include <functional>
#include <memory>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/tmed25519.h"
#include "ctx.h"
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

// safeMul (types/validator_set.go:1086-1105)
bool safe_mul(int64_t a, int64_t b, int64_t *out) {
  if (a == 0 || b == 0) { *out = 0; return false; }
  const int64_t ab = b < 0 ? -b : b, aa = a < 0 ? -a : a;
  if (aa > kMaxInt64 / ab) { *out = 0; return true; }
  *out = a * b;
  return false;
}

struct Cand {
  size_t req;
  int32_t sig_idx;
  int32_t val_idx;
};

struct AddrKey {
  uint64_t a, b;
  uint32_t c;
  bool operator==(const AddrKey &o) const { return a == o.a && b == o.b && c == o.c; }
};
struct AddrHash {
  size_t operator()(const AddrKey &k) const { return k.a * 0x9E3779B97F4A7C15ull ^ k.b ^ ((uint64_t)k.c << 17); }
};
AddrKey addr_key(const uint8_t *p) {
  AddrKey k;
  memcpy(&k.a, p, 8);
  memcpy(&k.b, p + 8, 8);
  memcpy(&k.c, p + 16, 4);
  return k;
}

using AddrIndex = std::unordered_map<AddrKey, int32_t, AddrHash>;  // address -> first validator idx

struct Plan {
  bool decided = false;
  int64_t needed = 0;
  std::vector<int32_t> bit_of_sig;  // sig idx -> candidate slot (-1 = not sent)
  const AddrIndex *addr_index = nullptr;  // Trusting only (shared by requests on the same valset)
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
    std::function<int(const tmed_commit_request *reqs, size_t n, const std::vector<Cand> &cands, uint8_t *valid)>;

// Per-request CanonicalVote encoders for the requests that have candidates.
static int init_encoders(const tmed_commit_request *reqs, size_t n, const std::vector<Cand> &cands,
                         std::vector<tmed::VoteEncoder> &enc, std::vector<uint8_t> &used) {
  enc.assign(n, tmed::VoteEncoder());
  used.assign(n, 0);
  for (const Cand &cd : cands) used[cd.req] = 1;
  for (size_t q = 0; q < n; q++) {
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
    if (enc[q].init(&t) != TMED_OK) return TMED_EINVAL;
  }
  return TMED_OK;
}

// Flatten candidates with host-assembled sign-bytes (callback verifiers; oversize templates).
static int build_cand_batch(const tmed_commit_request *reqs, size_t n, const std::vector<Cand> &cands,
                            CandBatch &cb) {
  std::vector<uint8_t> used;
  int rc = init_encoders(reqs, n, cands, cb.enc, used);
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
  for (size_t k = 0; k < m; k++) {
    const Cand &cd = cands[k];
    const tmed_commit_request &r = reqs[cd.req];
    const tmed_commit &c = *r.commit;
    const size_t i = (size_t)cd.sig_idx;
    memcpy(&cb.pubs[k * 32], r.vals->pubkeys + 32 * (size_t)cd.val_idx, 32);
    const uint32_t sl = c.sig_lens ? c.sig_lens[i] : 64;
    memcpy(&cb.sigs[k * 64], c.sigs + 64 * i, sl < 64 ? sl : 64);
    cb.lens[k] = sl;
    cb.val_idx[k] = r.vals->keyset_index ? r.vals->keyset_index[cd.val_idx] : (uint32_t)cd.val_idx;
    cb.keyset[k] = r.vals->keyset;
    cb.tmpl[k] = (uint32_t)cd.req;
    cb.flags[k] = c.flags[i];
    cb.ts_sec[k] = c.ts_seconds[i];
    cb.ts_nanos[k] = c.ts_nanos[i];
  }
  return cb.build_host_msgs();
}

static int run_seam(const tmed_commit_request *reqs, size_t n, tmed_commit_result *out, const BatchVerifier &verify) {
  if (n && (!reqs || !out)) return TMED_EINVAL;
  std::vector<Plan> plans(n);
  std::vector<Cand> cands;
  std::unordered_map<const tmed_valset *, std::unique_ptr<AddrIndex>> addr_cache;
  for (size_t q = 0; q < n; q++) {
    const tmed_commit_request &r = reqs[q];
    tmed_commit_result &o = out[q];
    memset(&o, 0, sizeof o);
    int rc = check_request(r);
    if (rc != TMED_OK) return rc;
    const tmed_valset &vs = *r.vals;
    const tmed_commit &c = *r.commit;
    Plan &pl = plans[q];
    pl.bit_of_sig.assign(c.n_sigs, -1);
    if (r.mode != TMED_MODE_LIGHT_TRUSTING) {
      if (vs.n != c.n_sigs) {
        o.code = TMED_COMMIT_WRONG_SET_SIZE; o.expected = (int64_t)vs.n; o.actual = (int64_t)c.n_sigs;
        pl.decided = true; continue;
      }
      if (r.height != c.height) {
        o.code = TMED_COMMIT_WRONG_HEIGHT; o.expected = r.height; o.actual = c.height;
        pl.decided = true; continue;
      }
      if (!block_id_equal(*r.block_id, c.block_id)) {
        o.code = TMED_COMMIT_WRONG_BLOCK_ID; pl.decided = true; continue;
      }
      pl.needed = vs.total_power * 2 / 3;
      if (r.mode == TMED_MODE_COMMIT) {
        for (size_t i = 0; i < c.n_sigs; i++) {
          const uint8_t f = c.flags[i];
          if (f == kAbsent) continue;
          if (f != kCommit && f != kNil) return TMED_EINVAL;  // CommitSig.BlockID panics (types/block.go:663)
          pl.bit_of_sig[i] = (int32_t)cands.size();
          cands.push_back({q, (int32_t)i, (int32_t)i});
        }
      } else {
        int64_t tally = 0;
        for (size_t i = 0; i < c.n_sigs; i++) {
          if (c.flags[i] != kCommit) continue;
          pl.bit_of_sig[i] = (int32_t)cands.size();
          cands.push_back({q, (int32_t)i, (int32_t)i});
          tally += vs.powers[i];
          if (tally > pl.needed) break;
        }
      }
    } else {
      if (r.trust_den == 0) { o.code = TMED_COMMIT_ZERO_DENOMINATOR; pl.decided = true; continue; }
      int64_t prod;
      if (safe_mul(vs.total_power, r.trust_num, &prod)) { o.code = TMED_COMMIT_OVERFLOW; pl.decided = true; continue; }
      pl.needed = prod / r.trust_den;  // Go int64 division truncates toward zero, as C++ does
      auto &slot = addr_cache[r.vals];
      if (!slot) {
        slot.reset(new AddrIndex());
        slot->reserve(vs.n * 2);
        for (size_t v = 0; v < vs.n; v++) slot->emplace(addr_key(vs.addresses + 20 * v), (int32_t)v);  // first match wins
      }
      pl.addr_index = slot.get();
      std::vector<int32_t> seen(vs.n, -1);
      int64_t tally = 0;
      for (size_t i = 0; i < c.n_sigs; i++) {
        if (c.flags[i] != kCommit) continue;
        auto it = pl.addr_index->find(addr_key(c.addresses + 20 * i));
        if (it == pl.addr_index->end()) continue;
        const int32_t v = it->second;
        if (seen[v] >= 0) break;  // the loop returns the double-vote error here
        seen[v] = (int32_t)i;
        pl.bit_of_sig[i] = (int32_t)cands.size();
        cands.push_back({q, (int32_t)i, v});
        tally += vs.powers[v];
        if (tally > pl.needed) break;
      }
    }
  }

  // ---- one device batch for every candidate of every request
  const size_t m = cands.size();
  std::vector<uint8_t> valid(m, 0);
  if (m) {
    int rc = verify(reqs, n, cands, valid.data());
    if (rc != TMED_OK) return rc;
  }

  // ---- replay every reference loop over the bits
  for (size_t q = 0; q < n; q++) {
    Plan &pl = plans[q];
    if (pl.decided) continue;
    const tmed_commit_request &r = reqs[q];
    const tmed_valset &vs = *r.vals;
    const tmed_commit &c = *r.commit;
    tmed_commit_result &o = out[q];
    auto bit = [&](size_t i, bool *ok) -> bool {
      const int32_t k = pl.bit_of_sig[i];
      if (k < 0) { *ok = false; return false; }
      o.verified++;
      return valid[(size_t)k] != 0;
    };
    bool ok = true;
    int64_t tally = 0;
    o.code = -1;
    if (r.mode == TMED_MODE_COMMIT) {
      for (size_t i = 0; i < c.n_sigs && o.code < 0; i++) {
        if (c.flags[i] == kAbsent) continue;
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
        if (!bit(i, &ok)) { if (ok) { o.code = TMED_COMMIT_WRONG_SIGNATURE; o.idx = (int32_t)i; } break; }
        tally += vs.powers[i];
        if (tally > pl.needed) o.code = TMED_COMMIT_OK;
      }
      if (o.code < 0 && ok) { o.code = TMED_COMMIT_NOT_ENOUGH_POWER; o.got = tally; o.needed = pl.needed; }
    } else {
      std::vector<int32_t> seen(vs.n, -1);
      for (size_t i = 0; i < c.n_sigs && o.code < 0; i++) {
        if (c.flags[i] != kCommit) continue;
        auto it = pl.addr_index->find(addr_key(c.addresses + 20 * i));
        if (it == pl.addr_index->end()) continue;
        const int32_t v = it->second;
        if (seen[v] >= 0) {
          o.code = TMED_COMMIT_DOUBLE_VOTE; o.val_idx = v; o.idx_first = seen[v]; o.idx = (int32_t)i;
          break;
        }
        seen[v] = (int32_t)i;
        if (!bit(i, &ok)) { if (ok) { o.code = TMED_COMMIT_WRONG_SIGNATURE; o.idx = (int32_t)i; } break; }
        tally += vs.powers[v];
        if (tally > pl.needed) o.code = TMED_COMMIT_OK;
      }
      if (o.code < 0 && ok) { o.code = TMED_COMMIT_NOT_ENOUGH_POWER; o.got = tally; o.needed = pl.needed; }
    }
    if (!ok) return TMED_EINVAL;  // replay reached a signature the plan did not send (cannot happen)
  }
  return TMED_OK;
}

extern "C" int tmed_verify_commits_with(const tmed_commit_request *reqs, size_t n, tmed_commit_result *out,
                                        tmed_batch_verify_fn verify, void *user) {
  if (!verify) return TMED_EINVAL;
  return run_seam(reqs, n, out,
                  [&](const tmed_commit_request *rq, size_t nr, const std::vector<Cand> &cands, uint8_t *valid) {
                    CandBatch cb;
                    int rc = build_cand_batch(rq, nr, cands, cb);
                    if (rc != TMED_OK) return rc;
                    return verify(user, cb.pubs.data(), cb.sigs.data(), cb.lens.data(), cb.msgs.data(),
                                  cb.offs.data(), cb.m, valid);
                  });
}

// Host fallback of the GPU verifier for templates the device assembler cannot hold.
static int ctx_verify_host_msgs(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t n,
                                const std::vector<Cand> &cands, uint8_t *valid) {
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

// GPU verifier: sign-bytes are assembled on the device from per-commit templates
// (SURVEY.md §8f f1), so only key references, signatures, flags and timestamps cross
// PCIe; they are written straight from the request arrays into the pinned staging area
// (multi-threaded for large batches).  Candidates of validator sets with a key-set handle
// go through the key-cached kernels, one launch sequence per distinct key set.
static int ctx_verify(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t n, const std::vector<Cand> &cands,
                      uint8_t *valid) {
  std::vector<tmed::VoteEncoder> enc;
  std::vector<uint8_t> used;
  int rc = init_encoders(reqs, n, cands, enc, used);
  if (rc != TMED_OK) return rc;
  std::vector<uint8_t> tmpl(n * tmed::kVoteTmplBytes);
  for (size_t q = 0; q < n; q++)
    if (used[q] && !enc[q].device_template(&tmpl[q * tmed::kVoteTmplBytes], tmed::kVoteTmplBytes))
      return ctx_verify_host_msgs(ctx, reqs, n, cands, valid);
  // group by key set (usually a single group)
  std::vector<uint64_t> gkeys;
  std::vector<std::vector<uint32_t>> gidx;
  for (size_t k = 0; k < cands.size(); k++) {
    const uint64_t ks = reqs[cands[k].req].vals->keyset;
    size_t g = 0;
    while (g < gkeys.size() && gkeys[g] != ks) g++;
    if (g == gkeys.size()) { gkeys.push_back(ks); gidx.emplace_back(); }
    gidx[g].push_back((uint32_t)k);
  }
  for (size_t g = 0; g < gkeys.size(); g++) {
    const std::vector<uint32_t> &ix = gidx[g];
    const uint32_t m = (uint32_t)ix.size();
    const bool keyed = gkeys[g] != 0;
    tmed::VoteStage st;
    rc = tmed::votes_stage(ctx, gkeys[g], m, n, st);
    if (rc != TMED_OK) return rc;
    memcpy(st.tmpl, tmpl.data(), tmpl.size());
    auto fill = [&](uint32_t lo, uint32_t hi) {
      for (uint32_t j = lo; j < hi; j++) {
        const Cand &cd = cands[ix[j]];
        const tmed_commit_request &r = reqs[cd.req];
        const tmed_commit &c = *r.commit;
        const size_t i = (size_t)cd.sig_idx;
        if (keyed) {
          const uint32_t v = r.vals->keyset_index ? r.vals->keyset_index[cd.val_idx] : (uint32_t)cd.val_idx;
          memcpy(st.key + (size_t)j * 4, &v, 4);
        } else {
          memcpy(st.key + (size_t)j * 32, r.vals->pubkeys + 32 * (size_t)cd.val_idx, 32);
        }
        const uint32_t sl = c.sig_lens ? c.sig_lens[i] : 64;
        uint8_t *sd = st.sig + (size_t)j * 64;
        if (sl >= 64) memcpy(sd, c.sigs + 64 * i, 64);
        else { memset(sd, 0, 64); memcpy(sd, c.sigs + 64 * i, sl); }
        st.tidx[j] = (uint32_t)cd.req;
        st.flag[j] = c.flags[i];
        st.sec[j] = c.ts_seconds[i];
        st.nan[j] = c.ts_nanos[i];
      }
    };
    const uint32_t nthreads = m >= 65536 ? std::min<uint32_t>(16, std::max(1u, std::thread::hardware_concurrency())) : 1;
    if (nthreads > 1) {
      std::vector<std::thread> th;
      for (uint32_t t = 0; t < nthreads; t++)
        th.emplace_back(fill, (uint32_t)((uint64_t)m * t / nthreads), (uint32_t)((uint64_t)m * (t + 1) / nthreads));
      for (auto &x : th) x.join();
    } else {
      fill(0, m);
    }
    std::vector<uint8_t> out(m);
    rc = tmed::votes_launch(ctx, st, out.data());
    if (rc != TMED_OK) return rc;
    for (uint32_t j = 0; j < m; j++) {
      const Cand &cd = cands[ix[j]];
      const tmed_commit &c = *reqs[cd.req].commit;
      const uint32_t sl = c.sig_lens ? c.sig_lens[cd.sig_idx] : 64;
      valid[ix[j]] = sl == 64 ? out[j] : 0;  // crypto/ed25519/ed25519.go:150-152
    }
  }
  return TMED_OK;
}

extern "C" int tmed_verify_commits(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t n,
                                   tmed_commit_result *out) {
  if (!ctx) return TMED_EINVAL;
  return run_seam(reqs, n, out,
                  [&](const tmed_commit_request *rq, size_t nr, const std::vector<Cand> &cands, uint8_t *valid) {
                    return ctx_verify(ctx, rq, nr, cands, valid);
                  });
}
