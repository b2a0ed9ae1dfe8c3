// seam_race.cpp — TEST-ONLY: the commit seam's host half (csrc/seam_host.h, the code commit.hip
// runs) on a light-client-shaped batch, driven as the pipelined seam drives it (bs_pump / bs_finish:
// seam_plan with a staging group and template rows, the staged bits produced in staging order by a
// stand-in verifier, then the part-wise finish), built with ThreadSanitizer by
// tests/test_native_sanitizers.py and run with the pool jitter on.  A part of a parallel region that
// reads what another part of the same region writes (round 5's Group::add_run read off[r + 1] of the
// next part) is a data race TSan reports on the first run, whatever the timing.
//
// Prints a digest of every request's outcome; the test compares it with a run on one host thread
// (TMED_HOST_THREADS=1: every region serial), so the parallel merge, aliasing and finish must also
// give exactly the serial plan's results.
//
// usage: seam_race HEADERS VALIDATORS ITERATIONS JITTER_US SEED
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "seam_host.h"

// no key-set cache in this harness: planning builds its own address indexes
struct KcCall {};
static const AddrIndex *kc_addr_index(const KcCall *, const tmed_valset &) { return nullptr; }

namespace {

// The stand-in verifier: a pseudo-random bit of (key, signature) — the same tuple always gets the
// same bit, so an alias (one verification serving two requests) reads exactly what its own
// verification would have said.
uint8_t fake_bit(const uint8_t *key, const uint8_t *sig) {
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < 32; i++) h = (h ^ key[i]) * 1099511628211ull;
  for (int i = 0; i < 64; i++) h = (h ^ sig[i]) * 1099511628211ull;
  return (h >> 7) % 53 != 0;  // ~2 % invalid
}

struct SetData {
  std::vector<uint8_t> pubs, addrs;
  std::vector<int64_t> powers;
  tmed_valset vs{};
  void make(size_t n, std::mt19937_64 &rng, const SetData *from, size_t change) {
    pubs.resize(32 * n);
    addrs.resize(20 * n);
    powers.resize(n);
    for (size_t v = 0; v < n; v++) {
      const bool fresh = !from || v == change;
      for (int b = 0; b < 32; b++) pubs[32 * v + b] = fresh ? (uint8_t)rng() : from->pubs[32 * v + b];
      for (int b = 0; b < 20; b++) addrs[20 * v + b] = fresh ? (uint8_t)rng() : from->addrs[20 * v + b];
      powers[v] = fresh ? 1 + (int64_t)(rng() % 100) : from->powers[v];
    }
    int64_t total = 0;
    for (int64_t p : powers) total += p;
    vs.n = n;
    vs.pubkeys = pubs.data();
    vs.powers = powers.data();
    vs.addresses = addrs.data();
    vs.total_power = total;
  }
};

struct CommitData {
  std::vector<uint8_t> flags, addrs, sigs, hash, psh;
  std::vector<int64_t> sec;
  std::vector<int32_t> nan;
  std::vector<uint32_t> slen;
  tmed_commit c{};
  void make(const SetData &signers, int64_t height, std::mt19937_64 &rng) {
    const size_t n = signers.vs.n;
    flags.resize(n);
    addrs = signers.addrs;
    sigs.resize(64 * n);
    sec.resize(n);
    nan.resize(n);
    slen.resize(n);
    hash.resize(32);
    psh.resize(32);
    for (auto &b : hash) b = (uint8_t)rng();
    for (auto &b : psh) b = (uint8_t)rng();
    for (size_t i = 0; i < n; i++) {
      const unsigned r = rng() % 100;
      flags[i] = r < 80 ? 2 : (r < 95 ? 1 : 3);  // Commit / Absent / Nil
      for (int b = 0; b < 64; b++) sigs[64 * i + b] = (uint8_t)rng();
      sec[i] = 1700000000 + height;
      nan[i] = (int32_t)(rng() % 1000000000);
      slen[i] = rng() % 211 == 0 ? 63 : 64;
    }
    c.height = height;
    c.round = 0;
    c.block_id = tmed_block_id{hash.data(), 32, 1, psh.data(), 32};
    c.n_sigs = n;
    c.flags = flags.data();
    c.addresses = addrs.data();
    c.ts_seconds = sec.data();
    c.ts_nanos = nan.data();
    c.sigs = sigs.data();
    c.sig_lens = slen.data();
    c.address_lens = nullptr;
  }
};

}  // namespace

int main(int argc, char **argv) {
  const size_t headers = argc > 1 ? (size_t)atol(argv[1]) : 600;
  const size_t nval = argc > 2 ? (size_t)atol(argv[2]) : 48;
  const int iters = argc > 3 ? atoi(argv[3]) : 3;
  const int jitter = argc > 4 ? atoi(argv[4]) : 0;
  const uint64_t seed = argc > 5 ? (uint64_t)atoll(argv[5]) : 7;
  g_pool_jitter_us.store(jitter);
  std::mt19937_64 rng(seed);
  // the light client's sets: set h + 1 is set h with one validator replaced (light/verifier.go)
  std::vector<SetData> sets(headers + 1);
  sets[0].make(nval, rng, nullptr, 0);
  for (size_t h = 1; h <= headers; h++) sets[h].make(nval, rng, &sets[h - 1], (size_t)(rng() % nval));
  std::vector<CommitData> commits(headers);
  for (size_t h = 0; h < headers; h++) commits[h].make(sets[h + 1], (int64_t)(h + 2), rng);
  const char chain[] = "test_chain_id";
  // per header: the Trusting request against the trusted set, then the Light request against the
  // untrusted set on the SAME commit (pair_request aliases their shared verifications)
  std::vector<tmed_commit_request> reqs;
  for (size_t h = 0; h < headers; h++) {
    tmed_commit_request t{};
    t.mode = TMED_MODE_LIGHT_TRUSTING;
    t.chain_id = chain;
    t.chain_id_len = sizeof(chain) - 1;
    t.vals = &sets[h].vs;
    t.commit = &commits[h].c;
    t.trust_num = 1;
    t.trust_den = 3;
    reqs.push_back(t);
    tmed_commit_request l{};
    l.mode = TMED_MODE_LIGHT;
    l.chain_id = chain;
    l.chain_id_len = sizeof(chain) - 1;
    l.vals = &sets[h + 1].vs;
    l.block_id = &commits[h].c.block_id;
    l.height = commits[h].c.height;
    l.commit = &commits[h].c;
    reqs.push_back(l);
  }
  const size_t n = reqs.size();
  uint64_t digest = 1469598103934665603ull;
  size_t aliases = 0, parts = 0, cands_total = 0;
  Plans ps;
  Cands cands;
  Group grp;
  Templates tp;
  for (int it = 0; it < iters; it++) {
    std::vector<tmed_commit_result> out(n);
    int rc = seam_plan(reqs.data(), n, out.data(), ps, cands, nullptr, &grp, &tp);
    if (rc != TMED_OK) { printf("seam_plan rc %d\n", rc); return 1; }
    bool fits = tp.fits;
    if (cands.size() && !tp.ready) rc = device_templates(reqs.data(), n, cands, tp, &fits);
    if (rc != TMED_OK) { printf("device_templates rc %d\n", rc); return 1; }
    // the device: one bit per staged position, in staging order (stage_group's layout)
    const size_t m = grp.size(cands);
    std::vector<uint8_t> bits(m, 0), valid(cands.size(), 0);
    for_segments(cands, grp, 0, m, [&](size_t j, uint32_t u0, uint32_t u1, size_t p) {
      const Run &run = cands.runs[grp.run(cands, j)];
      const tmed_commit_request &r = reqs[run.req];
      for (uint32_t u = u0; u < u1; u++) {
        const size_t i = (size_t)(run.sig + (int32_t)u), v = (size_t)(run.val + (int32_t)u);
        bits[p + (u - u0)] = fake_bit(r.vals->pubkeys + 32 * v, r.commit->sigs + 64 * i);
      }
    });
    // bs_finish
    const bool aliased = !cands.alias.empty();
    const size_t np = cands.preq.size() ? cands.preq.size() - 1 : 0;
    if (aliased && np && !grp.rix.empty()) {
      rc = finish_parts(reqs.data(), cands, grp, bits.data(), valid.data(), ps, out.data());
    } else {
      if (aliased) {
        scatter_bits(reqs.data(), cands, grp, bits.data(), valid.data());
        copy_aliases(cands, valid.data());
      }
      rc = seam_replay(reqs.data(), n, out.data(), ps, aliased ? valid.data() : bits.data());
    }
    if (rc != TMED_OK) { printf("finish rc %d\n", rc); return 1; }
    aliases = cands.alias.size();
    parts = np;
    cands_total = cands.size();
    for (size_t q = 0; q < n; q++) {
      const tmed_commit_result &o = out[q];
      const int64_t f[] = {o.code, o.got, o.needed, o.expected, o.actual, o.idx, o.idx_first, o.val_idx, o.verified};
      for (int64_t x : f) digest = (digest ^ (uint64_t)x) * 1099511628211ull;
    }
  }
  printf("requests %zu candidates %zu aliases %zu parts %zu digest %016llx\n", n, cands_total, aliases, parts,
         (unsigned long long)digest);
  return 0;
}
