// hostsim.cpp — TEST-ONLY host build of the device verify/sign code.
//
// Compiles tendermint-fork_amd/csrc/verify_core.h (the exact source the HIP
// kernels run) for the CPU with g++, so that the kernel arithmetic can be
// checked against the oracle in a container without a GPU.  Never part of the
// product: the product library (libtmed25519_hip.so) has no CPU path.
#include <stdint.h>
#include <string.h>

#include <vector>
#include "verify_core.h"
#include "verify_hs.h"
#include "sha256.h"

using namespace tmed;

namespace {
struct HostTab {
  ge_cached e[9];
  void store(int j, const ge_cached &c) { e[j] = c; }
  void load(int j, ge_cached &c) const { c = e[j]; }
  int pf = 0;
  bool sw = false;
  void prefetch(int j, bool swap = false) { pf = j; sw = swap; }
  void take(ge_cached &c) const {
    c = e[pf];
    if (sw) { const fe t = c.YpX; c.YpX = c.YmX; c.YmX = t; }
  }
};
struct HostBTab {
  ge_niels e[129];
};
HostBTab &btab() {
  static HostBTab t;
  static bool init = false;
  if (!init) { build_btab_niels(t.e); init = true; }
  return t;
}
// Per-lane view of a shared B table (prefetch/take state is the lane's own).
template <int BITS>
struct HostBRef {
  static constexpr int kBits = BITS;
  const ge_niels *e;
  int pf = 0;
  void prefetch(int j) { pf = j; }
  void take(ge_niels &n) const { n = e[pf]; }
};
// The radix-2^16 table of main-kernel variant 5 (j*B, j = 0..32768), built like the device's.
const std::vector<ge_niels> &b16tab() {
  static std::vector<ge_niels> t;
  static bool init = false;
  if (!init) {
    t.resize(32769);
    ge_p3 B;
    ge_base_point(B);
    ge_niels_0(t[0]);
#pragma omp parallel for schedule(dynamic, 64)
    for (long j = 1; j < 32769; j++) comb_entry(t[j], B, (uint32_t)j, 16);
    init = true;
  }
  return t;
}
// The device finish's accessor, on host arrays: lane l owns slots l, l + L, ... < m.
struct HostFin {
  const std::vector<ge_p2> *pts;
  std::vector<fe> *pre;
  const uint8_t *sig;
  uint8_t *out;
  uint32_t lane, L, m;
  int count() const { return lane < m ? (int)((m - lane + L - 1) / L) : 0; }
  uint32_t slot(int j) const { return lane + (uint32_t)j * L; }
  void load_z(int j, fe &z) const { z = (*pts)[slot(j)].Z; }
  void load_xy(int j, fe &X, fe &Y) const { X = (*pts)[slot(j)].X; Y = (*pts)[slot(j)].Y; }
  void store_pre(int j, const fe &p) const { (*pre)[(size_t)j * L + lane] = p; }
  void load_pre(int j, fe &p) const { p = (*pre)[(size_t)j * L + lane]; }
  void load_r(int j, uint32_t Rw[8]) const { load_words8(Rw, sig + 64 * (size_t)slot(j)); }
  void result(int j, bool ok) const { uint8_t &o = out[slot(j)]; o = (o && ok) ? 1 : 0; }
};

// Host twin of launch_finish: same group-size rule, but G is a parameter so tests can
// cover partial groups.
void host_finish(const std::vector<ge_p2> &pts, const uint8_t *sig, uint8_t *out, uint32_t m, uint32_t G) {
  if (m == 0) return;
  const uint32_t L = (m + G - 1) / G;
  std::vector<fe> pre((size_t)G * L);
#pragma omp parallel for schedule(dynamic, 8)
  for (long l = 0; l < (long)L; l++) {
    HostFin a{&pts, &pre, sig, out, (uint32_t)l, L, m};
    finish_group(a);
  }
}
}  // namespace

extern "C" {

// group = 0: per-signature encoding (verify_one); group >= 1: prep + main point per
// signature, then the batched finish with that group size (the device path).
static void verify_batch_impl(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                              size_t n, uint8_t *out, int group, int bbits) {
  const ge_niels *b8 = btab().e;
  const ge_niels *b16 = bbits == 16 ? b16tab().data() : nullptr;
  std::vector<ge_p2> pts(group > 0 ? n : 0);
#pragma omp parallel for schedule(dynamic, 16)
  for (long i = 0; i < (long)n; i++) {
    HostTab tab;
    HostBRef<8> bt{b8};
    HostBRef<16> bt16{b16};
    uint32_t pw[8], sw[16];
    load_words8(pw, pub + 32 * i);
    load_words8(sw, sig + 64 * i);
    load_words8(sw + 8, sig + 64 * i + 32);
    if (group <= 0) {
      out[i] = verify_one(pw, sw, msgs + off[i], off[i + 1] - off[i], tab, bt) ? 1 : 0;
    } else {
      uint32_t k[8], s[8];
      ge_p3 A;
      const bool ok = verify_prep(pw, sw, msgs + off[i], off[i + 1] - off[i], k, s, A);
      if (bbits == 16) verify_main_point(pts[i], k, s, A, tab, bt16);
      else verify_main_point(pts[i], k, s, A, tab, bt);
      out[i] = ok ? 1 : 0;
    }
  }
  if (group > 0) host_finish(pts, sig, out, (uint32_t)n, (uint32_t)group);
}

void hostsim_verify_batch_g(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                            size_t n, uint8_t *out, int group) {
  verify_batch_impl(pub, sig, msgs, off, n, out, group, 8);
}

// Main-kernel variant 5: radix-2^16 B windows (16 B additions) + the batched finish.
void hostsim_verify_batch_b16(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                              size_t n, uint8_t *out) {
  verify_batch_impl(pub, sig, msgs, off, n, out, 16, 16);
}

// Half-size-scalar path (verify_hs.h): prep_hs + main_hs per signature, B digits from the
// j*B and j*2^128*B tables (the device's radix-2^16 comb windows 0 and 8).
static const std::vector<ge_niels> &b16hi_tab() {
  static std::vector<ge_niels> t;
  static bool init = false;
  if (!init) {
    t.resize(32769);
    ge_p3 P;
    ge_base_point(P);
    for (int i = 0; i < 16; i++) ge_mul256(P);  // 2^128 B
    ge_niels_0(t[0]);
#pragma omp parallel for schedule(dynamic, 64)
    for (long j = 1; j < 32769; j++) comb_entry(t[j], P, (uint32_t)j, 16);
    init = true;
  }
  return t;
}

// The radix-2^26 B tables of the default main kernel (j * B, j * 2^128 B for j = 0..2^25, 8.6 GB
// on the device): entries computed on demand here (double-and-add, then the same affine niels
// conversion as the device's b26_fill_kernel).
struct HostB26Ref {
  static constexpr int kBits = 26;
  const ge_p3 *base;
  int pf = 0;
  void prefetch(int j) { pf = j; }
  void take(ge_niels &n) const {
    if (pf == 0) ge_niels_0(n);
    else comb_entry(n, *base, (uint32_t)pf, 26);
  }
};
static const ge_p3 *b26_bases() {
  static ge_p3 b[2];
  static bool init = false;
  if (!init) {
    ge_base_point(b[0]);
    b[1] = b[0];
    for (int i = 0; i < 16; i++) ge_mul256(b[1]);  // 2^128 B
    init = true;
  }
  return b;
}

// wmin (optional): run signature i's Straus over max(W_i, wmin[i]) windows — the device runs every
// lane of a wave over the wave's largest W, so a lane's top windows may lie above its own W.
// b16: the radix-2^16 B windows (the device's fallback when the 2^26 tables are unavailable).
static void verify_batch_hs_impl(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                                 size_t n, uint8_t *out, int32_t *wins, const int32_t *wmin, bool b16) {
  const ge_niels *lo = b16tab().data();
  const ge_niels *hi = b16hi_tab().data();
  const ge_p3 *b26 = b26_bases();
#pragma omp parallel for schedule(dynamic, 16)
  for (long i = 0; i < (long)n; i++) {
    HostTab ta, tr;
    HostBRef<16> bl{lo}, bh{hi};
    HostB26Ref bl26{&b26[0]}, bh26{&b26[1]};
    uint32_t pw[8], sw[16], er[8];
    load_words8(pw, pub + 32 * i);
    load_words8(sw, sig + 64 * i);
    load_words8(sw + 8, sig + 64 * i + 32);
    bool dneg;
    ge_p3 A;
    fe Rx, Ry;
    int W;
    HsDigits dg;
    const bool ok = verify_prep_hs(pw, sw, msgs + off[i], off[i + 1] - off[i], dg, er, dneg, A, Rx, Ry, W, !b16);
    const int Wrun = (wmin && wmin[i] > W) ? (wmin[i] > 64 ? 64 : wmin[i]) : W;
    const bool id = b16 ? verify_main_hs(dg, dneg, er, Wrun, A, Rx, Ry, ta, tr, bl, bh)
                        : verify_main_hs(dg, dneg, er, Wrun, A, Rx, Ry, ta, tr, bl26, bh26);
    out[i] = ok && id ? 1 : 0;
    if (wins) wins[i] = W;
  }
}

void hostsim_verify_batch_hs_w(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                               size_t n, uint8_t *out, int32_t *wins, const int32_t *wmin) {
  verify_batch_hs_impl(pub, sig, msgs, off, n, out, wins, wmin, false);
}

void hostsim_verify_batch_hs(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                             size_t n, uint8_t *out, int32_t *wins) {
  verify_batch_hs_impl(pub, sig, msgs, off, n, out, wins, nullptr, false);
}

void hostsim_verify_batch_hs16(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                               size_t n, uint8_t *out, int32_t *wins) {
  verify_batch_hs_impl(pub, sig, msgs, off, n, out, wins, nullptr, true);
}

// The lattice step alone: c, |d| (32-byte LE each), dneg, window count.
int hostsim_halfsize_impl(const uint8_t *k32, uint8_t *c32, uint8_t *d32, int *dneg, int fast) {
  uint32_t k[8], c[8], dm[8];
  load_words8(k, k32);
  bool neg;
  const int W = fast ? sc_halfsize<true>(c, dm, neg, k) : sc_halfsize<false>(c, dm, neg, k);
  for (int i = 0; i < 32; i++) {
    c32[i] = (uint8_t)(c[i / 4] >> (8 * (i % 4)));
    d32[i] = (uint8_t)(dm[i / 4] >> (8 * (i % 4)));
  }
  *dneg = neg ? 1 : 0;
  return W;
}

int hostsim_halfsize(const uint8_t *k32, uint8_t *c32, uint8_t *d32, int *dneg) {
  return hostsim_halfsize_impl(k32, c32, d32, dneg, 1);
}

int hostsim_halfsize_plain(const uint8_t *k32, uint8_t *c32, uint8_t *d32, int *dneg) {
  return hostsim_halfsize_impl(k32, c32, d32, dneg, 0);
}

void hostsim_verify_batch(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                          size_t n, uint8_t *out) {
  hostsim_verify_batch_g(pub, sig, msgs, off, n, out, 16);
}

void hostsim_sign_batch(const uint8_t *seeds, const uint8_t *msgs, const uint32_t *off, size_t n,
                        uint8_t *sig_out, uint8_t *pub_out) {
  const ge_niels *b8 = btab().e;
#pragma omp parallel for schedule(dynamic, 16)
  for (long i = 0; i < (long)n; i++) {
    HostTab tab;
    HostBRef<8> bt{b8};
    uint32_t seed[8], sg[16], pb[8];
    load_words8(seed, seeds + 32 * i);
    sign_one(sg, pb, seed, msgs + off[i], off[i + 1] - off[i], tab, bt);
    for (int w = 0; w < 16; w++) for (int b = 0; b < 4; b++) sig_out[64 * i + 4 * w + b] = (uint8_t)(sg[w] >> (8 * b));
    for (int w = 0; w < 8; w++) for (int b = 0; b < 4; b++) pub_out[32 * i + 4 * w + b] = (uint8_t)(pb[w] >> (8 * b));
  }
}

// Key-cached (comb) verification on the host: builds every comb with the kernel's
// comb_entry/ge_mul256 and runs verify_one_comb.
struct HostComb {
  static constexpr int kBits = 8;
  std::vector<ge_niels> e;  // 32 x 129
  void load(int w, int j, ge_niels &out) const { out = e[(size_t)w * 129 + j]; }
};
// The radix-2^16 comb of B (16 windows x 32769 entries): entries computed on demand with the
// device builder's comb_entry from the same bases (host_bcomb16_bases restated).
struct HostComb16 {
  static constexpr int kBits = 16;
  ge_p3 bases[16];
  HostComb16() {
    ge_p3 P;
    ge_base_point(P);
    for (int w = 0; w < 16; w++) { bases[w] = P; ge_mul256(P); ge_mul256(P); }
  }
  void load(int w, int j, ge_niels &out) const {
    if (j == 0) ge_niels_0(out);
    else comb_entry(out, bases[w], (uint32_t)j, 16);
  }
};

static void build_host_comb(HostComb &c, const uint32_t pw[8], bool negate, bool *ok) {
  ge_p3 P;
  *ok = ge_frombytes_go(P, pw);
  if (negate) { fe_neg(P.X, P.X); fe_neg(P.T, P.T); }
  c.e.resize(32 * 129);
  for (int w = 0; w < 32; w++) {
    ge_niels_0(c.e[(size_t)w * 129]);
#pragma omp parallel for
    for (int j = 1; j <= 128; j++) comb_entry(c.e[(size_t)w * 129 + j], P, (uint32_t)j);
    ge_mul256(P);
  }
}

static const HostComb &host_bcomb() {
  static HostComb bcomb;
  static bool binit = false;
  if (!binit) {
    uint32_t bw[8];
    const uint8_t by[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                            0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                            0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};
    load_words8(bw, by);
    bool ok;
    build_host_comb(bcomb, bw, false, &ok);
    binit = true;
  }
  return bcomb;
}

static void build_key_combs(const uint8_t *keys, size_t nkeys, std::vector<HostComb> &ac, std::vector<uint8_t> &kok) {
  ac.resize(nkeys);
  kok.resize(nkeys);
  for (size_t k = 0; k < nkeys; k++) {
    uint32_t pw[8];
    load_words8(pw, keys + 32 * k);
    bool ok;
    build_host_comb(ac[k], pw, true, &ok);
    kok[k] = ok;
  }
}

// Latency mode (verify_core.h): 8 partial comb sums, the device's cross-lane tree order,
// strict decode of R and the projective compare — no inversion.
void hostsim_verify_comb_lat(const uint8_t *keys, size_t nkeys, const uint32_t *key_idx, const uint8_t *sig,
                             const uint8_t *msgs, const uint32_t *off, size_t n, uint8_t *out) {
  const HostComb &bcomb = host_bcomb();
  std::vector<HostComb> ac;
  std::vector<uint8_t> kok;
  build_key_combs(keys, nkeys, ac, kok);
#pragma omp parallel for schedule(dynamic, 8)
  for (long i = 0; i < (long)n; i++) {
    uint32_t pw[8], sw[16], k[8], s[8], kr[8], sr[8];
    const uint32_t v = key_idx[i];
    load_words8(pw, keys + 32 * v);
    load_words8(sw, sig + 64 * i);
    load_words8(sw + 8, sig + 64 * i + 32);
    const bool ok = verify_prep_comb(pw, kok[v] != 0, sw, msgs + off[i], off[i + 1] - off[i], k, s);
    sc_recode256(kr, k);
    sc_recode256(sr, s);
    ge_p3 P[kLatLanes];
    for (int r = 0; r < kLatLanes; r++) comb_partial(P[r], kr, sr, r, ac[v], bcomb);
    for (int L = 1; L < kLatLanes; L <<= 1)
      for (int r = 0; r + L < kLatLanes; r += 2 * L) ge_p3_add(P[r], P[r + L]);
    fe xr, yr;
    const bool rok = r_decode_strict(xr, yr, sw);
    out[i] = (ok && rok && projective_matches(P[0].X, P[0].Y, P[0].Z, xr, yr)) ? 1 : 0;
  }
}

}  // extern "C"

template <class BC>
static void verify_comb_batch_impl(const uint8_t *keys, size_t nkeys, const uint32_t *key_idx, const uint8_t *sig,
                                   const uint8_t *msgs, const uint32_t *off, size_t n, uint8_t *out, const BC &bcomb) {
  std::vector<HostComb> ac;
  std::vector<uint8_t> kok;
  build_key_combs(keys, nkeys, ac, kok);
  std::vector<ge_p2> pts(n);
#pragma omp parallel for schedule(dynamic, 8)
  for (long i = 0; i < (long)n; i++) {
    uint32_t pw[8], sw[16], k[8], s[8];
    const uint32_t v = key_idx[i];
    load_words8(pw, keys + 32 * v);
    load_words8(sw, sig + 64 * i);
    load_words8(sw + 8, sig + 64 * i + 32);
    const bool ok = verify_prep_comb(pw, kok[v] != 0, sw, msgs + off[i], off[i + 1] - off[i], k, s);
    ge_p3 R;
    verify_main_comb_point(R, k, s, ac[v], bcomb);
    pts[i].X = R.X; pts[i].Y = R.Y; pts[i].Z = R.Z;
    out[i] = ok ? 1 : 0;
  }
  host_finish(pts, sig, out, (uint32_t)n, 3);
}

extern "C" {

void hostsim_verify_comb_batch(const uint8_t *keys, size_t nkeys, const uint32_t *key_idx, const uint8_t *sig,
                               const uint8_t *msgs, const uint32_t *off, size_t n, uint8_t *out) {
  verify_comb_batch_impl(keys, nkeys, key_idx, sig, msgs, off, n, out, host_bcomb());
}

// The key-cached throughput kernel's schedule: 32 A-comb + 16 radix-2^16 B-comb additions.
void hostsim_verify_comb_batch16(const uint8_t *keys, size_t nkeys, const uint32_t *key_idx, const uint8_t *sig,
                                 const uint8_t *msgs, const uint32_t *off, size_t n, uint8_t *out) {
  static const HostComb16 b16;
  verify_comb_batch_impl(keys, nkeys, key_idx, sig, msgs, off, n, out, b16);
}

// Field-level probes: inputs/outputs are 32-byte LE encodings.
static void to_bytes(uint8_t *o, const uint32_t w[8]) { for (int i = 0; i < 32; i++) o[i] = (uint8_t)(w[i / 4] >> (8 * (i % 4))); }

void hostsim_fe_op(int op, const uint8_t *a, const uint8_t *b, uint8_t *out) {
  uint32_t wa[8], wb[8], wo[8];
  load_words8(wa, a); load_words8(wb, b);
  fe fa, fb, fo;
  fe_from_words(fa, wa); fe_from_words(fb, wb);
  switch (op) {
    case 0: fe_mul(fo, fa, fb); break;
    case 1: fe_sq(fo, fa); break;
    case 2: fe_invert(fo, fa); break;
    case 3: fe_pow22523(fo, fa); break;
    case 4: fe_add(fo, fa, fb); fe_carry(fo, fo); break;
    case 5: fe_sub(fo, fa, fb); fe_carry(fo, fo); break;
    case 6: fe_sq2(fo, fa); break;
    case 7: { fe t; fe_add(t, fa, fb); fe_add(t, t, fa); fe_mul(fo, t, t); break; }  // 3-sum input
    case 8: { fe t; fe_add(t, fa, fb); fe_add(t, t, fa); fe_sq(fo, t); break; }
    case 9: fe_invert_bgcd(fo, fa); break;
    default: fe_copy(fo, fa);
  }
  fe_to_words(wo, fo);
  to_bytes(out, wo);
}

// mul / sq / sq2 on raw limbs (signed 32-bit; the caller keeps them inside the documented input
// bounds), the product's limbs and its canonical encoding out.
void hostsim_fe_raw(int op, const int32_t *a, const int32_t *b, int32_t *out_limbs, uint8_t *out) {
  fe fa, fb, fo;
  for (int i = 0; i < 10; i++) { fa.v[i] = a[i]; fb.v[i] = b[i]; }
  if (op == 0) fe_mul(fo, fa, fb);
  else if (op == 1) fe_sq(fo, fa);
  else fe_sq2(fo, fa);
  for (int i = 0; i < 10; i++) out_limbs[i] = fo.v[i];
  uint32_t wo[8];
  fe_to_words(wo, fo);
  to_bytes(out, wo);
}

// fe_pack256 / fe_unpack256 on raw limbs (the main kernel's table storage form): unpacked limbs
// out, and the product of the unpacked value with the carried g (32-byte LE) as a canonical encoding.
void hostsim_pack256(const int32_t *limbs, const uint8_t *g, int32_t *out_limbs, uint8_t *prod) {
  fe f, u, gf, o;
  for (int i = 0; i < 10; i++) f.v[i] = limbs[i];
  uint32_t w[8], wg[8], wo[8];
  fe_pack256(w, f);
  fe_unpack256(u, w);
  for (int i = 0; i < 10; i++) out_limbs[i] = u.v[i];
  load_words8(wg, g);
  fe_from_words(gf, wg);
  fe_mul(o, u, gf);
  fe_to_words(wo, o);
  to_bytes(prod, wo);
}

int hostsim_decode(const uint8_t *p, uint8_t *out_enc) {
  uint32_t w[8], e[8];
  load_words8(w, p);
  ge_p3 A;
  bool ok = ge_frombytes_go(A, w);
  ge_tobytes(e, A.X, A.Y, A.Z);
  to_bytes(out_enc, e);
  return ok ? 1 : 0;
}

void hostsim_sha512(const uint8_t *m, uint32_t n, uint8_t *out) {
  uint32_t z[8] = {0}, h[16];
  sha512_stream(h, z, z, 0, m, n);
  for (int i = 0; i < 64; i++) out[i] = (uint8_t)(h[i / 4] >> (8 * (i % 4)));
}

void hostsim_sc_reduce(const uint8_t *h64, uint8_t *out) {
  uint32_t x[16], r[8];
  for (int i = 0; i < 16; i++) x[i] = (uint32_t)h64[4 * i] | ((uint32_t)h64[4 * i + 1] << 8) | ((uint32_t)h64[4 * i + 2] << 16) | ((uint32_t)h64[4 * i + 3] << 24);
  sc_reduce512(r, x);
  to_bytes(out, r);
}

}  // extern "C"

// SHA-256 paths of the Merkle kernels (csrc/sha256.h), on the host.
extern "C" void hostsim_sha256(int npre, uint8_t prefix, const uint8_t *m, uint32_t mlen, uint8_t *out) {
  uint32_t st[8];
  sha256_prefixed(st, npre, prefix, m, mlen);
  for (int k = 0; k < 8; k++)
    for (int b = 0; b < 4; b++) out[4 * k + b] = (uint8_t)(st[k] >> (24 - 8 * b));
}
extern "C" void hostsim_sha256_inner(const uint8_t *l, const uint8_t *r, uint8_t *out) {
  uint32_t lw[8], rw[8], st[8];
  for (int k = 0; k < 8; k++) {
    lw[k] = ((uint32_t)l[4 * k] << 24) | ((uint32_t)l[4 * k + 1] << 16) | ((uint32_t)l[4 * k + 2] << 8) | l[4 * k + 3];
    rw[k] = ((uint32_t)r[4 * k] << 24) | ((uint32_t)r[4 * k + 1] << 16) | ((uint32_t)r[4 * k + 2] << 8) | r[4 * k + 3];
  }
  sha256_inner(st, lw, rw);
  for (int k = 0; k < 8; k++)
    for (int b = 0; b < 4; b++) out[4 * k + b] = (uint8_t)(st[k] >> (24 - 8 * b));
}
