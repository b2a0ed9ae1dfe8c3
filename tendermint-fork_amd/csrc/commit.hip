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
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/tmed25519.h"
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

struct Plan {
  bool decided = false;
  int64_t needed = 0;
  std::vector<int32_t> bit_of_sig;  // sig idx -> candidate slot (-1 = not sent)
  std::unordered_map<AddrKey, int32_t, AddrHash> addr_index;  // Trusting: address -> first validator idx
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
  std::vector<uint8_t> pubs, sigs, msgs;
  std::vector<uint32_t> lens, offs, val_idx;
  std::vector<uint64_t> keyset;
};
using BatchVerifier = std::function<int(const CandBatch &, uint8_t *valid)>;

static int run_seam(const tmed_commit_request *reqs, size_t n, tmed_commit_result *out, const BatchVerifier &verify) {
  if (n && (!reqs || !out)) return TMED_EINVAL;
  std::vector<Plan> plans(n);
  std::vector<Cand> cands;
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
      pl.addr_index.reserve(vs.n * 2);
      for (size_t v = 0; v < vs.n; v++) pl.addr_index.emplace(addr_key(vs.addresses + 20 * v), (int32_t)v);  // first match wins
      std::vector<int32_t> seen(vs.n, -1);
      int64_t tally = 0;
      for (size_t i = 0; i < c.n_sigs; i++) {
        if (c.flags[i] != kCommit) continue;
        auto it = pl.addr_index.find(addr_key(c.addresses + 20 * i));
        if (it == pl.addr_index.end()) continue;
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
    CandBatch cb;
    cb.m = m;
    cb.pubs.resize(m * 32);
    cb.sigs.resize(m * 64);
    cb.lens.resize(m);
    cb.offs.resize(m + 1);
    cb.val_idx.resize(m);
    cb.keyset.resize(m);
    std::vector<uint8_t> &pubs = cb.pubs, &sigs = cb.sigs;
    std::vector<uint32_t> &lens = cb.lens, &offs = cb.offs;
    std::vector<tmed::VoteEncoder> enc(n);
    for (size_t q = 0; q < n; q++) {
      if (plans[q].decided) continue;
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
    size_t total = 0;
    for (size_t k = 0; k < m; k++) {
      const Cand &cd = cands[k];
      const tmed_commit &c = *reqs[cd.req].commit;
      offs[k] = (uint32_t)total;
      total += enc[cd.req].size(c.flags[cd.sig_idx], c.ts_seconds[cd.sig_idx], c.ts_nanos[cd.sig_idx]);
      if (total > 0xffffffffu) return TMED_EINVAL;
    }
    offs[m] = (uint32_t)total;
    cb.msgs.resize(total + 16);
    std::vector<uint8_t> &msgs = cb.msgs;
    for (size_t k = 0; k < m; k++) {
      const Cand &cd = cands[k];
      const tmed_commit_request &r = reqs[cd.req];
      const tmed_commit &c = *r.commit;
      const size_t i = (size_t)cd.sig_idx;
      enc[cd.req].write(msgs.data() + offs[k], c.flags[i], c.ts_seconds[i], c.ts_nanos[i]);
      memcpy(&pubs[k * 32], r.vals->pubkeys + 32 * (size_t)cd.val_idx, 32);
      const uint32_t sl = c.sig_lens ? c.sig_lens[i] : 64;
      memcpy(&sigs[k * 64], c.sigs + 64 * i, sl < 64 ? sl : 64);
      lens[k] = sl;
      cb.val_idx[k] = r.vals->keyset_index ? r.vals->keyset_index[cd.val_idx] : (uint32_t)cd.val_idx;
      cb.keyset[k] = r.vals->keyset;
    }
    int rc = verify(cb, valid.data());
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
        auto it = pl.addr_index.find(addr_key(c.addresses + 20 * i));
        if (it == pl.addr_index.end()) continue;
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
  return run_seam(reqs, n, out, [&](const CandBatch &cb, uint8_t *valid) {
    return verify(user, cb.pubs.data(), cb.sigs.data(), cb.lens.data(), cb.msgs.data(), cb.offs.data(), cb.m, valid);
  });
}

// GPU verifier: candidates of validator sets with a key-set handle go through the
// key-cached kernel (one launch per distinct key set), the rest through the generic one.
static int ctx_verify(tmed_ctx *ctx, const CandBatch &cb, uint8_t *valid) {
  std::unordered_map<uint64_t, std::vector<uint32_t>> groups;
  for (size_t k = 0; k < cb.m; k++) groups[cb.keyset[k]].push_back((uint32_t)k);
  if (groups.size() == 1 && groups.begin()->first == 0)
    return tmed_verify_batch(ctx, cb.pubs.data(), cb.sigs.data(), cb.lens.data(), cb.msgs.data(), cb.offs.data(),
                             cb.m, valid);
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
    int rc = g.first == 0
                 ? tmed_verify_batch(ctx, pubs.data(), sigs.data(), lens.data(), msgs.data(), offs.data(), m, out.data())
                 : tmed_verify_batch_keyset(ctx, g.first, vidx.data(), sigs.data(), lens.data(), msgs.data(),
                                            offs.data(), m, out.data());
    if (rc != TMED_OK) return rc;
    for (size_t j = 0; j < m; j++) valid[ix[j]] = out[j];
  }
  return TMED_OK;
}

extern "C" int tmed_verify_commits(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t n,
                                   tmed_commit_result *out) {
  if (!ctx) return TMED_EINVAL;
  return run_seam(reqs, n, out, [&](const CandBatch &cb, uint8_t *valid) { return ctx_verify(ctx, cb, valid); });
}
