// verify_core.h — one ed25519 verification (or signature) per lane.
//
// Restates, for the GPU, the decision procedure of the reference's hot path:
//   crypto/ed25519/ed25519.go:148-155 PubKey.VerifySignature
//   -> golang.org/x/crypto v0.1.0 (go.mod:44) -> Go 1.18 crypto/ed25519.Verify
// (SURVEY.md §8a row V0):
//   sig[63] & 0xE0 -> reject; A = SetBytes(pub) (permissive); k = SHA-512(R||A||M) mod L;
//   S >= L -> reject; R' = [k](-A) + [S]B (cofactorless); accept iff enc(R') == R bytes.
// (len(sig) != 64 is decided on the host, before a tuple reaches the device.)
//
// SIMT shape: the double-scalar multiplication is a Straus interleave with FIXED
// signed windows — radix 16 for k (64 windows: 4 doublings + one cached add from the
// per-lane table of -A) and radix 256 for S (32 niels adds from the shared LDS table of
// j*B, one per 8 doublings).  Unlike the reference's wNAF (whose data-dependent add
// positions would make every lane of a 64-wide wave pay for every other lane's adds),
// every lane runs exactly the same instruction stream; digit 0 adds the identity,
// which the complete formulas handle exactly.
#pragma once
#include "ge25519.h"
#include "sc25519.h"
#include "sha512.h"

namespace tmed {

// Signed radix-256 recoding: r = k + 0x8080...80; digit w = byte_w(r) - 128 (k < 2^255).
TMED_HD void sc_recode256(uint32_t r[8], const uint32_t k[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t t = (uint64_t)k[i] + 0x80808080u + c;
    r[i] = (uint32_t)t;
    c = t >> 32;
  }
}

// e <- sign(d) * entry(|d|): -(y+x, y-x, 2dxy) = (y-x, y+x, -2dxy)
TMED_HD void niels_apply_sign(ge_niels &e, bool neg) {
  fe t;
  fe_copy(t, e.YpX);
  fe_select(e.YpX, e.YpX, e.YmX, neg);
  fe_select(e.YmX, e.YmX, t, neg);
  fe_neg(t, e.XY2d);
  fe_select(e.XY2d, e.XY2d, t, neg);
}

// Per-lane variable-base table access.  T must provide
//   void store(int j, const ge_cached&), void prefetch(int j)  and  void take(ge_cached&)
// for j in [0, 8] (j = 0 is the identity): prefetch names the entry the next take
// returns, so a device table can start the fetch one window (four doublings) ahead.  The device implementation lives in a
// global-memory slab (per-lane tables are 1.4 KB: too large for LDS at useful
// occupancy); the host test build uses a local array.
template <class T>
TMED_HD void build_table_negA(T &tab, const ge_p3 &A) {
  ge_p3 nA;  // -A
  fe_neg(nA.X, A.X); fe_copy(nA.Y, A.Y); fe_copy(nA.Z, A.Z); fe_neg(nA.T, A.T);
  ge_cached c, c1;
  ge_cached_0(c);
  tab.store(0, c);
  ge_p3_to_cached(c1, nA);
  tab.store(1, c1);
  ge_p3 cur = nA;
  ge_p1p1 t;
#pragma unroll 1
  for (int j = 2; j <= 8; j++) {
    ge_add_cached(t, cur, c1, false);
    ge_p1p1_to_p3(cur, t);
    ge_p3_to_cached(c, cur);
    tab.store(j, c);
  }
}

// Per-lane table of j*P, j = 0..8, for an AFFINE P (Z = 1, T = xy: a decoded A or R).  P in
// niels form makes each step (j-1)P + P a mixed addition (3M + 4M to extended + 1M to cached)
// instead of a general cached one (4M + 4M + 1M): 58M per table against 64M for
// build_table_negA.  A loop, like build_table_negA: unrolled, the scheduler interleaves the seven
// steps and the main kernel spills (measured: 256 VGPRs + 61 spilled).
template <class T>
TMED_HD void build_table_affine(T &tab, const ge_p3 &P) {
  ge_cached c;
  ge_cached_0(c);
  tab.store(0, c);
  fe d2;
  fe_const_d2(d2);
  ge_niels n;  // P in niels form; as a cached point Z = 1
  fe_add(n.YpX, P.Y, P.X);
  fe_sub(n.YmX, P.Y, P.X);
  fe_mul(n.XY2d, P.T, d2);
  fe_copy(c.YpX, n.YpX);
  fe_copy(c.YmX, n.YmX);
  fe_1(c.Z);
  fe_copy(c.T2d, n.XY2d);
  tab.store(1, c);
  ge_p3 cur = P;
  ge_p1p1 t;
#pragma unroll 1
  for (int j = 2; j <= 8; j++) {
    ge_madd_niels(t, cur, n, false);
    ge_p1p1_to_p3(cur, t);
    ge_p3_to_cached(c, cur);
    tab.store(j, c);
  }
}

// out = [k](-A) + [S]B  (Straus, most-significant first).
// k: signed radix-16 digits (64 windows) from the per-lane table of j*(-A), j=0..8;
// S: signed radix-2^BBITS digits from a shared table of j*B (niels), added once per
// BBITS doublings:
//   BBITS = 8:  32 windows, j = 0..128 (the 15.5 KB table staged in LDS);
//   BBITS = 16: 16 windows, j = 0..32768 (a 4.2 MB table in HBM, L2/MALL-resident),
//               16 fewer mixed additions per signature.
// Both tables expose prefetch(j) / take(niels&): the next B digit is known one window
// ahead, so a global table's entry can be fetched while the doublings run.
template <int BBITS>
TMED_HD void sc_recode_b(uint32_t r[8], const uint32_t s[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t t = (uint64_t)s[i] + (BBITS == 8 ? 0x80808080u : 0x80008000u) + c;
    r[i] = (uint32_t)t;
    c = t >> 32;
  }
}

template <int BBITS, class T, class BT>
TMED_HD void double_scalarmult(ge_p2 &out, const uint32_t k[8], const uint32_t s[8], T &tab, BT &btab) {
  constexpr int kBias = 1 << (BBITS - 1);
  constexpr uint32_t kMask = (1u << BBITS) - 1u;
  uint32_t kr[8], sr[8];
  sc_recode16(kr, k);
  sc_recode_b<BBITS>(sr, s);
  ge_p2 q;
  ge_p2_0(q);
  ge_p1p1 t;
  ge_p3 r;
  ge_cached ca;
  ge_niels nb;
  {
    const int da0 = (int)(kr[7] >> 28) - 8;
    tab.prefetch(da0 < 0 ? -da0 : da0);
    const int db0 = (int)(sr[7] >> (32 - BBITS)) - kBias;
    btab.prefetch(db0 < 0 ? -db0 : db0);
  }
#pragma unroll 1
  for (int j = 0; j < 8; j++) {  // 32-bit word of the scalars, most significant first
    uint32_t kc = kr[7];
    const uint32_t sw = sr[7];
#pragma unroll
    for (int m = 7; m > 0; m--) { kr[m] = kr[m - 1]; sr[m] = sr[m - 1]; }
#pragma unroll 1
    for (int i = 0; i < 4; i++) {  // byte of the word: two radix-16 A windows
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int da = (int)(kc >> 28) - 8;
        kc <<= 4;
        // the window after this one (the next word's first digit after the last nibble;
        // past the final window any in-range index will do)
        const int dn = (int)(((h == 1 && i == 3) ? kr[7] : kc) >> 28) - 8;
        if (h == 0 && j == 0 && i == 0) {
          ge_p3_0(r);  // the first four doublings would double the identity: skipped
        } else {
#pragma unroll 1
          for (int d = 0; d < 3; d++) {
            ge_p2_dbl(t, q);
            ge_p1p1_to_p2(q, t);
          }
          ge_p2_dbl(t, q);
          ge_p1p1_to_p3(r, t);
        }
        tab.take(ca);
        ge_add_cached(t, r, ca, da < 0);
        tab.prefetch(dn < 0 ? -dn : dn);
        if (h == 0) ge_p1p1_to_p2(q, t);
      }
      const bool badd = BBITS == 8 || (i & 1);  // a B window ends after this byte
      if (badd) {
        // B digit of the window ending here: bits [32 - 8(i+1), 32 - 8(i+1) + BBITS) of sw
        const int sh = 32 - 8 * (i + 1);
        const int db = (int)((sw >> sh) & kMask) - kBias;
        // next B digit: same word, or the next word's first window after the last one
        const int dbn = (i == 3) ? (int)(sr[7] >> (32 - BBITS)) - kBias
                                 : (int)((sw >> (sh - BBITS)) & kMask) - kBias;
        ge_p1p1_to_p3(r, t);
        btab.take(nb);
        btab.prefetch(dbn < 0 ? -dbn : dbn);
        niels_apply_sign(nb, db < 0);
        ge_madd_niels(t, r, nb, false);
      }
      ge_p1p1_to_p2(q, t);
    }
  }
  out = q;
}

// Load 8 LE 32-bit words from 32 bytes.
TMED_HD void load_words8(uint32_t w[8], const uint8_t *p) {
#pragma unroll
  for (int i = 0; i < 8; i++)
    w[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
           ((uint32_t)p[4 * i + 3] << 24);
}

// Verification phase 1 (hash / scalar checks / decompression — the register-hungry
// part): returns ok and writes k = SHA-512(R||A||M) mod L, s (S, or 0 if rejected)
// and the decoded A (identity if rejected).
TMED_HD bool verify_prep(const uint32_t pubw[8], const uint32_t sigw[16], const uint8_t *msg, uint32_t mlen,
                         uint32_t k[8], uint32_t s[8], ge_p3 &A) {
  bool ok = (sigw[15] & 0xE0000000u) == 0;        // sig[63] & 0xE0
  const uint32_t *S = sigw + 8;
  ok = ok && sc_is_canonical(S);                  // Scalar.SetCanonicalBytes
  ok = ge_frombytes_go(A, pubw) && ok;            // Point.SetBytes (identity on failure)
  uint32_t h[16];
  sha512_stream(h, sigw, pubw, 64, msg, mlen);     // SHA-512(R || A || M)
  sc_reduce512(k, h);                              // Scalar.SetUniformBytes
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = ok ? S[i] : 0u;  // keep S < 2^255 for the recoding
  return ok;
}

// Verification phase 2 (point arithmetic): R' = [k](-A) + [s]B in projective form.  The
// canonical encoding of R' (one inversion) is left to the batched finish below.
template <class T, class BT>
TMED_HD void verify_main_point(ge_p2 &R, const uint32_t k[8], const uint32_t s[8], const ge_p3 &A, T &tab,
                               BT &btab) {
  build_table_negA(tab, A);
  double_scalarmult<BT::kBits>(R, k, s, tab, btab);
}

// enc(X/Z, Y/Z) == R bytes, given zi = 1/Z.
TMED_HD bool encoding_matches(const fe &X, const fe &Y, const fe &zi, const uint32_t Rw[8]) {
  fe x, y;
  fe_mul(x, X, zi);
  fe_mul(y, Y, zi);
  uint32_t enc[8];
  fe_to_words(enc, y);
  enc[7] |= (uint32_t)fe_isnegative(x) << 31;
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) diff |= enc[i] ^ Rw[i];
  return diff == 0;
}

// Unbatched phase 2 + compare (one inversion per signature).
template <class T, class BT>
TMED_HD bool verify_main(const uint32_t k[8], const uint32_t s[8], const ge_p3 &A, const uint32_t Rw[8], T &tab,
                         BT &btab) {
  ge_p2 R;
  verify_main_point(R, k, s, A, tab, btab);
  fe zi;
  fe_invert(zi, R.Z);
  return encoding_matches(R.X, R.Y, zi, Rw);
}

// Batched finish (Montgomery's simultaneous inversion): one lane owns the G' <= G
// signatures j = 0..count-1 of its group; with prefix products P_j = Z_0 ... Z_j,
// 1/Z_j = P_{j-1} / P_j, so the group costs one inversion + 3 multiplications per
// signature instead of one inversion per signature (the inversion is ~254 squarings).
// Acc provides: count(); load_z(j, fe&); load_xy(j, fe&, fe&); load_r(j, uint32_t[8]);
// store_pre(j, const fe&); load_pre(j, fe&); result(j, bool).
// Z = 0 cannot come out of the complete formulas for points on the curve; it is still
// guarded (replaced by 1 and the signature rejected) so one bad value cannot poison the
// inversion of its whole group.
#ifndef TMED_FIN_BGCD
#define TMED_FIN_BGCD 1  // the group's inversion by binary GCD (fe_invert_bgcd); 0: z^(p-2)
#endif
template <class Acc>
TMED_HD void finish_group(Acc &a) {
  const int cnt = a.count();
  if (cnt <= 0) return;
  // Each row is loaded one signature ahead of its use: a finish lane runs alone on its SIMD (one
  // wave per SIMD at 65,536 lanes), so a load issued right before its use exposes the whole memory
  // latency at every signature.
  fe acc, z, zn;
  uint32_t bad = 0;
  a.load_z(0, zn);
#pragma unroll 1
  for (int j = 0; j < cnt; j++) {
    fe_copy(z, zn);
    if (j + 1 < cnt) a.load_z(j + 1, zn);
    if (fe_iszero(z)) { fe_1(z); bad |= 1u << j; }
    if (j == 0) fe_copy(acc, z); else fe_mul(acc, acc, z);
    a.store_pre(j, acc);
  }
  fe inv;
#if TMED_FIN_BGCD
  fe_invert_bgcd(inv, acc);  // 1 / (Z_0 ... Z_{cnt-1})
#else
  fe_invert(inv, acc);
#endif
  fe pre, X, Y, pren, Xn, Yn;
  uint32_t Rw[8], Rn[8];
  auto load_row = [&](int j, fe &p, fe &zr, fe &x, fe &y, uint32_t r[8]) {
    if (j > 0) {
      a.load_pre(j - 1, p);
      a.load_z(j, zr);
    }
    a.load_xy(j, x, y);
    a.load_r(j, r);
  };
  load_row(cnt - 1, pren, zn, Xn, Yn, Rn);
#pragma unroll 1
  for (int j = cnt - 1; j >= 0; j--) {
    fe_copy(pre, pren);
    fe_copy(z, zn);
    fe_copy(X, Xn);
    fe_copy(Y, Yn);
#pragma unroll
    for (int i = 0; i < 8; i++) Rw[i] = Rn[i];
    if (j > 0) load_row(j - 1, pren, zn, Xn, Yn, Rn);
    fe zi;
    if (j > 0) {
      fe_mul(zi, pre, inv);  // 1 / Z_j
      if ((bad >> j) & 1u) fe_1(z);
      fe_mul(inv, inv, z);  // 1 / (Z_0 ... Z_{j-1})
    } else {
      fe_copy(zi, inv);
    }
    a.result(j, encoding_matches(X, Y, zi, Rw) && !((bad >> j) & 1u));
  }
}

// One verification.  pubw: 8 words of A; sigw: 16 words (R = 0..7, S = 8..15).
template <class T, class BT>
TMED_HD bool verify_one(const uint32_t pubw[8], const uint32_t sigw[16], const uint8_t *msg, uint32_t mlen,
                        T &tab, BT &btab) {
  uint32_t k[8], s[8];
  ge_p3 A;
  const bool ok = verify_prep(pubw, sigw, msg, mlen, k, s, A);
  return verify_main(k, s, A, sigw, tab, btab) && ok;
}

// [s]B for s < 2^255 via the same window schedule (k = 0 uses the identity
// table; used by the signer and key generation only).
template <class T, class BT>
TMED_HD void scalarmult_base(uint32_t enc[8], const uint32_t s[8], T &tab, BT &btab) {
  uint32_t zero[8];
#pragma unroll
  for (int i = 0; i < 8; i++) zero[i] = 0;
  ge_p3 id;
  ge_p3_0(id);
  build_table_negA(tab, id);
  ge_p2 R;
  double_scalarmult<BT::kBits>(R, zero, s, tab, btab);
  ge_tobytes(enc, R.X, R.Y, R.Z);
}

// RFC 8032 signing (crypto/ed25519/ed25519.go:57-60 -> Go ed25519.Sign):
//   h = SHA-512(seed); a = clamp(h[0:32]) mod L; A = [a]B;
//   r = SHA-512(h[32:64] || M) mod L; R = [r]B; k = SHA-512(R || A || M) mod L; S = r + k a.
// bm(enc, s) must write the canonical encoding of [s]B (s < L).
template <class BM>
TMED_HD void sign_one_bm(uint32_t sig[16], uint32_t pub[8], const uint32_t seed[8], const uint8_t *msg,
                         uint32_t mlen, const BM &bm) {
  uint32_t h[16], zero[8], a[8], x[16], r[8], k[8], s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) zero[i] = 0;
  sha512_stream(h, seed, zero, 32, msg, 0);
  h[0] &= 0xfffffff8u;
  h[7] &= 0x7fffffffu;
  h[7] |= 0x40000000u;
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = i < 8 ? h[i] : 0u;
  sc_reduce512(a, x);
  bm(pub, a);
  uint32_t prefix[8];
#pragma unroll
  for (int i = 0; i < 8; i++) prefix[i] = h[8 + i];
  sha512_stream(x, prefix, zero, 32, msg, mlen);
  sc_reduce512(r, x);
  bm(sig, r);
  sha512_stream(x, sig, pub, 64, msg, mlen);
  sc_reduce512(k, x);
  sc_muladd(s, k, a, r);
#pragma unroll
  for (int i = 0; i < 8; i++) sig[8 + i] = s[i];
}

// Signing with [s]B by the Straus schedule (k = 0) — the host test build's signer.
template <class T, class BT>
TMED_HD void sign_one(uint32_t sig[16], uint32_t pub[8], const uint32_t seed[8], const uint8_t *msg,
                      uint32_t mlen, T &tab, BT &btab) {
  sign_one_bm(sig, pub, seed, msg, mlen, [&](uint32_t enc[8], const uint32_t s[8]) {
    scalarmult_base(enc, s, tab, btab);
  });
}

// ------------------------------------------------------------------ combs
// Signed radix-256 comb (key cache): entry [w][j] = j * 256^w * P
// in affine niels form, j = 0..128.  [k]P = sum_w entry[w][d_w] with
// d_w = byte_w(k + 0x8080...80) - 128: 32 mixed additions, no doublings.

// P <- 256 * P
TMED_HD void ge_mul256(ge_p3 &P) {
  ge_p1p1 t;
  ge_p2 q;
  ge_p3_to_p2(q, P);
#pragma unroll 1
  for (int d = 0; d < 7; d++) { ge_p2_dbl(t, q); ge_p1p1_to_p2(q, t); }
  ge_p2_dbl(t, q);
  ge_p1p1_to_p3(P, t);
}

// Affine niels form (y + x, y - x, 2d x y) of a projective point: one inversion.
TMED_HD void ge_p3_to_niels(ge_niels &out, const ge_p3 &p) {
  fe zi, x, y, xy, d2;
  fe_const_d2(d2);
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_add(out.YpX, y, x); fe_carry(out.YpX, out.YpX);
  fe_sub(out.YmX, y, x); fe_carry(out.YmX, out.YmX);
  fe_mul(xy, x, y);
  fe_mul(out.XY2d, xy, d2);
}

// out = j * base (j in 1..255) in niels form; branch-free double-and-add.
TMED_HD void comb_entry(ge_niels &out, const ge_p3 &base, uint32_t j, int nbits = 8) {
  ge_cached cP;
  ge_p3_to_cached(cP, base);
  ge_p3 acc, sum;
  ge_p3_0(acc);
  ge_p1p1 t;
  ge_p2 q;
#pragma unroll 1
  for (int b = nbits - 1; b >= 0; b--) {
    ge_p3_to_p2(q, acc);
    ge_p2_dbl(t, q);
    ge_p1p1_to_p3(acc, t);
    ge_add_cached(t, acc, cP, false);
    ge_p1p1_to_p3(sum, t);
    const bool bit = (j >> b) & 1;
    fe_select(acc.X, acc.X, sum.X, bit);
    fe_select(acc.Y, acc.Y, sum.Y, bit);
    fe_select(acc.Z, acc.Z, sum.Z, bit);
    fe_select(acc.T, acc.T, sum.T, bit);
  }
  ge_p3_to_niels(out, acc);
}

// Key-cached verification, phase 1: k = SHA-512(R||A||M) mod L and the S checks (A is
// already decoded in the key set; key_ok carries Point.SetBytes' verdict).
TMED_HD bool verify_prep_comb(const uint32_t pubw[8], bool key_ok, const uint32_t sigw[16], const uint8_t *msg,
                              uint32_t mlen, uint32_t k[8], uint32_t s[8], bool slot = false) {
  bool ok = key_ok && (sigw[15] & 0xE0000000u) == 0;
  ok = ok && sc_is_canonical(sigw + 8);
  uint32_t h[16];
  if (slot) sha512_stream_slot(h, sigw, pubw, msg, mlen);  // msg: a 16-B aligned kVoteSlot slot
  else sha512_stream(h, sigw, pubw, 64, msg, mlen);
  sc_reduce512(k, h);
#pragma unroll
  for (int w = 0; w < 8; w++) s[w] = ok ? sigw[8 + w] : 0u;
  return ok;
}

// Key-cached verification, phase 2: [k](-A) from the key's comb, [s]B from the shared
// comb: 32 + 32 mixed additions (projective result; encoding by the batched finish).
// AC/BC provide  void load(int window, int j, ge_niels&) const  for j in 0..128.
// BC::kBits = 16 (the throughput kernel): [s]B from the radix-2^16 comb of B (16 windows of
// j * 2^(16w) * B, j = 0..32768), so 32 + 16 mixed additions; kBits = 8: 32 + 32.
template <class AC, class BC>
TMED_HD void verify_main_comb_point(ge_p3 &acc, const uint32_t k[8], const uint32_t s[8], const AC &acomb,
                                    const BC &bcomb) {
  if constexpr (BC::kBits == 16) {
    uint32_t kr[8], sr[8];
    sc_recode256(kr, k);
    sc_recode_b<16>(sr, s);
    ge_p3_0(acc);
    ge_p1p1 t;
    ge_niels e;
#pragma unroll 1
    for (int w = 0; w < 32; w++) {
      const int da = (int)((kr[w >> 2] >> (8 * (w & 3))) & 0xffu) - 128;
      acomb.load(w, da < 0 ? -da : da, e);
      niels_apply_sign(e, da < 0);
      ge_madd_niels(t, acc, e, false);
      ge_p1p1_to_p3(acc, t);
      if (w & 1) {  // B window w/2 (16 bits) after every second A window
        const int wb = w >> 1;
        const int db = (int)((sr[wb >> 1] >> (16 * (wb & 1))) & 0xffffu) - 32768;
        bcomb.load(wb, db < 0 ? -db : db, e);
        niels_apply_sign(e, db < 0);
        ge_madd_niels(t, acc, e, false);
        ge_p1p1_to_p3(acc, t);
      }
    }
    return;
  }
  uint32_t kr[8], sr[8];
  sc_recode256(kr, k);
  sc_recode256(sr, s);
  ge_p3_0(acc);
  ge_p1p1 t;
  ge_niels e;
#pragma unroll 1
  for (int wd = 0; wd < 8; wd++) {
    uint32_t kc = kr[0], scur = sr[0];
#pragma unroll
    for (int m = 0; m < 7; m++) { kr[m] = kr[m + 1]; sr[m] = sr[m + 1]; }
#pragma unroll 1
    for (int b = 0; b < 4; b++) {
      const int w = wd * 4 + b;
      const int da = (int)(kc & 0xffu) - 128;
      const int db = (int)(scur & 0xffu) - 128;
      kc >>= 8;
      scur >>= 8;
      acomb.load(w, da < 0 ? -da : da, e);
      niels_apply_sign(e, da < 0);
      ge_madd_niels(t, acc, e, false);
      ge_p1p1_to_p3(acc, t);
      bcomb.load(w, db < 0 ? -db : db, e);
      niels_apply_sign(e, db < 0);
      ge_madd_niels(t, acc, e, false);
      ge_p1p1_to_p3(acc, t);
    }
  }
}

// ------------------------------------------------------------------ latency mode
// A small batch (C1: one 175-validator commit) is bound by ONE lane's serial work — 64
// dependent comb additions, then one inversion — not by throughput.  Latency mode:
//  * splits a signature's 64 additions over kLatLanes = 8 lanes: lane r sums windows
//    r, r+8, r+16, r+24 of both combs (comb_partial), and three cross-lane additions
//    (level L = 1, 2, 4: lane r += lane r+L) combine the partial sums;
//  * replaces the inversion by a strict decode of R, run concurrently by other lanes:
//    encode(R') == R_bytes  iff  R_bytes is the canonical encoding of a curve point P_R
//    (y < p, x^2 = (y^2-1)/(dy^2+1) solvable, not x = 0 with the sign bit set) and
//    R' == P_R projectively (X' = x_R Z', Y' = y_R Z').  Both are exact.
constexpr int kLatLanes = 8;

// Partial comb sum of lane rr (0..7) of a signature: windows rr + 8t, t = 0..3.
template <class AC, class BC>
TMED_HD void comb_partial(ge_p3 &acc, const uint32_t kr[8], const uint32_t sr[8], int rr, const AC &acomb,
                          const BC &bcomb) {
  ge_p3_0(acc);
  ge_p1p1 t;
  ge_niels e;
  const int sh = 8 * (rr & 3);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int w = rr + 8 * q;  // byte w of the recoded scalars: word 2q + (rr >> 2)
    const uint32_t kw = (rr & 4) ? kr[2 * q + 1] : kr[2 * q];
    const uint32_t sw = (rr & 4) ? sr[2 * q + 1] : sr[2 * q];
    const int da = (int)((kw >> sh) & 0xffu) - 128;
    const int db = (int)((sw >> sh) & 0xffu) - 128;
    acomb.load(w, da < 0 ? -da : da, e);
    niels_apply_sign(e, da < 0);
    ge_madd_niels(t, acc, e, false);
    ge_p1p1_to_p3(acc, t);
    bcomb.load(w, db < 0 ? -db : db, e);
    niels_apply_sign(e, db < 0);
    ge_madd_niels(t, acc, e, false);
    ge_p1p1_to_p3(acc, t);
  }
}

// acc += o (both extended): one reduction step of the cross-lane tree.
TMED_HD void ge_p3_add(ge_p3 &acc, const ge_p3 &o) {
  ge_cached c;
  ge_p1p1 t;
  ge_p3_to_cached(c, o);
  ge_add_cached(t, acc, c, false);
  ge_p1p1_to_p3(acc, t);
}

// Strict decode of R (the set of byte strings Point.Bytes can produce): false unless R is
// a canonical encoding of a curve point; then (x, y) is that point.
// The checks strict decoding adds to Point.SetBytes for the encoding Rw of a decoded point
// with x-coordinate X: y < p, and not x = 0 with the sign bit set.
TMED_HD bool r_strict_extra(const fe &X, const uint32_t Rw[8]) {
  bool ones = (Rw[7] & 0x7fffffffu) == 0x7fffffffu;
#pragma unroll
  for (int i = 1; i < 7; i++) ones = ones && Rw[i] == 0xffffffffu;
  const bool canonical = !(ones && Rw[0] >= 0xffffffedu);  // y < p = 2^255 - 19
  return canonical && !(fe_iszero(X) && (Rw[7] >> 31) != 0);
}

TMED_HD bool r_decode_strict(fe &x, fe &y, const uint32_t Rw[8]) {
  ge_p3 P;
  bool ok = ge_frombytes_go(P, Rw);
  ok = ok && r_strict_extra(P.X, Rw);
  fe_copy(x, P.X);
  fe_copy(y, P.Y);
  return ok;
}

// (X : Y : Z) == (x, y)
TMED_HD bool projective_matches(const fe &X, const fe &Y, const fe &Z, const fe &x, const fe &y) {
  fe t;
  fe_mul(t, x, Z);
  const bool a = fe_equal(t, X);
  fe_mul(t, y, Z);
  const bool b = fe_equal(t, Y);
  return a && b && !fe_iszero(Z);
}

// enc([s]B) from the shared signed radix-256 comb of B (32 mixed additions; the device
// signer, which generates the synthetic commits of the benches).
template <class BC>
TMED_HD void comb_base_mult(uint32_t enc[8], const uint32_t s[8], const BC &bcomb) {
  uint32_t sr[8];
  sc_recode256(sr, s);
  ge_p3 acc;
  ge_p3_0(acc);
  ge_p1p1 t;
  ge_niels e;
#pragma unroll 1
  for (int w = 0; w < 32; w++) {
    const int d = (int)((sr[w >> 2] >> (8 * (w & 3))) & 0xffu) - 128;
    bcomb.load(w, d < 0 ? -d : d, e);
    niels_apply_sign(e, d < 0);
    ge_madd_niels(t, acc, e, false);
    ge_p1p1_to_p3(acc, t);
  }
  ge_tobytes(enc, acc.X, acc.Y, acc.Z);
}

template <class AC, class BC>
TMED_HD bool verify_main_comb(const uint32_t k[8], const uint32_t s[8], const uint32_t Rw[8], const AC &acomb,
                              const BC &bcomb) {
  ge_p3 acc;
  verify_main_comb_point(acc, k, s, acomb, bcomb);
  fe zi;
  fe_invert(zi, acc.Z);
  return encoding_matches(acc.X, acc.Y, zi, Rw);
}

template <class AC, class BC>
TMED_HD bool verify_one_comb(const uint32_t pubw[8], bool key_ok, const uint32_t sigw[16], const uint8_t *msg,
                             uint32_t mlen, const AC &acomb, const BC &bcomb) {
  uint32_t k[8], s[8];
  const bool ok = verify_prep_comb(pubw, key_ok, sigw, msg, mlen, k, s);
  return verify_main_comb(k, s, sigw, acomb, bcomb) && ok;
}

// The base point B = (x, 4/5), x even, from its encoding.
TMED_HD void ge_base_point(ge_p3 &B) {
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = 0x66666666u;
  w[0] = 0x66666658u;
  ge_frombytes_go(B, w);
}

// Construction of the shared B table: out[j] = j*B (niels, affine), j = 0..128.
TMED_HD void build_btab_niels(ge_niels out[129]) {
  // B = (x, 4/5), x even
  uint32_t byw[8];
  const uint8_t by[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                          0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                          0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};
  load_words8(byw, by);
  ge_p3 B;
  ge_frombytes_go(B, byw);
  ge_niels_0(out[0]);
  for (uint32_t j = 1; j <= 128; j++) comb_entry(out[j], B, j);
}

}  // namespace tmed
