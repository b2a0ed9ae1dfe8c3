// verify_hs.h — half-size-scalar verification (the generic throughput path).
//
// Same decision as verify_core.h's verify_one (crypto/ed25519/ed25519.go:148-155 ->
// Go 1.18 crypto/ed25519.Verify), with half the doublings:
//
//   Go accepts iff enc([S]B - [k]A) == R_bytes.  enc() is canonical, so this holds iff
//   R_bytes is the canonical encoding of a curve point R (strict decode: y < p, on the
//   curve, not x = 0 with the sign bit set) and D := [S]B - [k]A - R is the identity.
//
//   The curve group has order N = 8L and is cyclic, so [d] is injective for every odd d
//   with |d| < L.  Pick (c, d) with c = d*k (mod N), d odd and |c|, |d| ~ 2^128 (a short
//   vector of the lattice {(c, d) : c = d k mod N}); then
//       D = 0  <=>  [d]D = 0  <=>  [e]B - [c]A - [d]R = 0,   e = d*S mod L
//   exactly — for every A, including keys with a torsion component, because c = dk
//   holds modulo the full group order 8L, not only modulo L.  B has order L, so e can
//   be reduced mod L.
//
//   The check is then a 3-point Straus sum with ~130-bit scalars for A and R (4 doublings
//   and two cached additions per radix-16 window, ~33 windows instead of 64) and the full
//   scalar e for B from two radix-2^16 tables (j*B and j*2^128*B, 8 windows each), and
//   the comparison with the identity is projective (X = 0, Y = Z): no inversion.
//
// (c, d) comes from the extended Euclidean algorithm on (N, k): r_i = t_i k (mod N),
// stopped at the first r_i < 2^128, where |t_i| <= N / r_{i-1} <= 2^127.  If t_i is
// even (t_{i-1} and t_i are coprime, so t_{i-1} is odd), the vector
// (r_{i-1} - j r_i, t_{i-1} - j t_i) with j in [0, floor(r_{i-1}/r_i)] balancing the two
// magnitudes is taken instead (odd t, at most a few bits longer).  Quotients come from
// fp64 estimates corrected to the exact floor; any step the estimate cannot settle
// (quotient >= 2^32, or an estimate off by more than one) falls back to (c, d) = (k, 1),
// the unshortened equation — so the decision never depends on the lattice step, only
// the length of the loop does.  The loop length W (radix-16 windows) is per lane here and
// the wave maximum on the device.
#pragma once
#include <math.h>

#include "verify_core.h"

#ifndef TMED_SLAB_PF
#define TMED_SLAB_PF 1  // the default of kernels.hip (host builds follow the same order)
#endif
#ifndef TMED_B16_ONEBUF
#define TMED_B16_ONEBUF 0  // 1: BL and BH share one prefetch buffer (the high row is fetched after the
                           // low row is taken, the next low row after the high row is taken)
#endif

namespace tmed {

// N = 8L (little-endian words).
TMED_HD void sc_const_8L(uint32_t n[8]) {
  const uint32_t c[8] = {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u};
#pragma unroll
  for (int i = 0; i < 8; i++) n[i] = c[i];
}

TMED_HD int bitlen_words(const uint32_t *x, int n) {
  int b = 0;
#pragma unroll
  for (int i = 0; i < n; i++)
    if (x[i]) b = 32 * i + 32 - __builtin_clz(x[i]);
  return b;
}

TMED_HD double words_to_double(const uint32_t *x, int n) {
  double r = 0.0;
#pragma unroll
  for (int i = n - 1; i >= 0; i--) r = r * 4294967296.0 + (double)x[i];
  return r;
}

// r = a - q*b (8 words); returns true if the result went negative (wrapped mod 2^256).
// Two borrow chains: the low halves of q*b[i] and the high halves of q*b[i-1].
TMED_HD bool words8_submul(uint32_t r[8], const uint32_t a[8], uint32_t q, const uint32_t b[8]) {
  uint32_t b1 = 0, b2 = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t p = (uint64_t)q * b[i];
    const uint32_t t = subb32(a[i], (uint32_t)p, b1, b1);
    r[i] = subb32(t, hi, b2, b2);
    hi = (uint32_t)(p >> 32);
  }
  return (hi | b1 | b2) != 0;
}

// r += b; returns the carry out.
TMED_HD uint32_t words8_add(uint32_t r[8], const uint32_t b[8]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = addc32(r[i], b[i], c, c);
  return c;
}

// r -= b; returns the borrow out.
TMED_HD uint32_t words8_sub(uint32_t r[8], const uint32_t b[8]) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = subb32(r[i], b[i], borrow, borrow);
  return borrow;
}

// a >= b
TMED_HD bool words8_ge(const uint32_t a[8], const uint32_t b[8]) {
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = a[i];
  return words8_sub(t, b) == 0;
}

// Magnitudes of the cofactors t_i (< 2^160): r = a + q*b (5 words, carry out dropped).
constexpr int kHsTW = 5;
TMED_HD void words5_muladd(uint32_t r[kHsTW], const uint32_t a[kHsTW], uint32_t q, const uint32_t b[kHsTW]) {
  uint32_t c1 = 0, c2 = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < kHsTW; i++) {
    const uint64_t p = (uint64_t)q * b[i];
    const uint32_t t = addc32(a[i], (uint32_t)p, c1, c1);
    r[i] = addc32(t, hi, c2, c2);
    hi = (uint32_t)(p >> 32);
  }
}

// floor(x / y) to within one (x, y > 0, quotient < 2^32): on the device a reciprocal with one
// Newton step (relative error ~2^-50, against ~2^-52 for the IEEE division it replaces, whose
// scale / fixup sequence is twice as long); the caller corrects the floor exactly.
TMED_HD double quot_estimate(double x, double y) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(y);
  r = fma(r, fma(-y, r, 1.0), r);
  return floor(x * r);
#else
  return floor(x / y);
#endif
}

TMED_HD bool words8_high_zero(const uint32_t x[8]) { return (x[4] | x[5] | x[6] | x[7]) == 0; }  // x < 2^128

// One exact Euclid step in place: q = floor(x / y) (x > y), x <- x - q y, tx <- tx + q ty,
// fx <- double(x).  fx, fy approximate x, y to double precision, so the estimate floor(fx / fy)
// is off by at most one for q < 2^32; it is corrected exactly (the y-subtraction / comparison
// runs only when the remainder came out negative, or within 2^-30 of y).  Sets fail when q is
// out of range or the estimate was off by more.
TMED_HD void hs_euclid_step(uint32_t x[8], const uint32_t y[8], uint32_t tx[kHsTW], const uint32_t ty[kHsTW],
                            double &fx, double fy, bool &fail) {
  const double qd = quot_estimate(fx, fy);
  if (!(qd < 4294967294.0)) { fail = true; return; }
  const uint32_t q = (uint32_t)qd;
  const bool neg = words8_submul(x, x, q, y);  // x - q y (wrapped mod 2^256 when negative)
  words5_muladd(tx, tx, q, ty);
  if (neg) {  // q one too high
    if (words8_add(x, y) == 0) fail = true;    // still negative: the estimate was off by more
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < kHsTW; i++) tx[i] = subb32(tx[i], ty[i], borrow, borrow);  // tx -= ty
  }
  fx = words_to_double(x, 8);
  if (!neg && fx >= fy * (1.0 - 0x1p-30) && words8_ge(x, y)) {  // q one too low
    words8_sub(x, y);
    uint32_t cy = 0;
#pragma unroll
    for (int i = 0; i < kHsTW; i++) tx[i] = addc32(tx[i], ty[i], cy, cy);  // tx += ty
    if (words8_ge(x, y)) fail = true;
    fx = words_to_double(x, 8);
  }
}

// Half-size decomposition of k (< L): c >= 0, |d| = dm odd, dneg = (d < 0), c = d k mod 8L.
// Returns the radix-16 window count the pair needs (29..64; 64 for the (k, 1) fallback).
// The Euclid phase runs two in-place steps per iteration (the remainders and cofactors swap
// roles instead of being moved: the round-1 loop spent ~300 instructions a step, ~0.5 ms per
// 2^20 signatures, mostly register moves and control flow).  FAST = false: that round-1 loop,
// kept as the reference of tests/test_kernel_host.py.
// tight (optional): the window count when the top digit may take values up to 16 (x < 2^(4W):
// the throughput path, whose first window adds two table entries per scalar — hs_straus); the
// return value is the count for top digits up to 8 (x < 2^(4W-1): the latency kernels).
template <bool FAST = true>
TMED_HD int sc_halfsize(uint32_t c[8], uint32_t dm[8], bool &dneg, const uint32_t k[8], int *tight = nullptr) {
  uint32_t a[8], b[8], ta[kHsTW], tb[kHsTW], nb[8], nt[kHsTW];
  sc_const_8L(a);
#pragma unroll
  for (int i = 0; i < 8; i++) b[i] = k[i];
#pragma unroll
  for (int i = 0; i < kHsTW; i++) { ta[i] = 0; tb[i] = i == 0 ? 1u : 0u; }
  double fa = words_to_double(a, 8), fb = words_to_double(b, 8);
  bool fail = false, iodd = true;  // i = 1: b = r_1 = k, t_1 = +1
  if (FAST) {
    int steps = 0;
    bool swapped = false;  // the last step left r_i in a (roles of a/b and ta/tb exchanged)
#pragma unroll 1
    for (int it = 0; it < 96 && !fail; it++) {
      if (words8_high_zero(b)) break;
      hs_euclid_step(a, b, ta, tb, fa, fb, fail);  // a <- r_{i+1}
      steps++;
      if (fail || words8_high_zero(a)) { swapped = true; break; }
      hs_euclid_step(b, a, tb, ta, fb, fa, fail);  // b <- r_{i+2}
      steps++;
    }
    if (swapped) {
#pragma unroll
      for (int i = 0; i < 8; i++) { const uint32_t t = a[i]; a[i] = b[i]; b[i] = t; }
#pragma unroll
      for (int i = 0; i < kHsTW; i++) { const uint32_t t = ta[i]; ta[i] = tb[i]; tb[i] = t; }
      const double t = fa; fa = fb; fb = t;
    }
    if (steps & 1) iodd = !iodd;
  }
#pragma unroll 1
  for (int it = 0; it < (FAST ? 0 : 190); it++) {
    if ((b[4] | b[5] | b[6] | b[7]) == 0) break;  // r_i < 2^128
    const double qd = floor(fa / fb);
    if (!(qd < 4294967294.0)) { fail = true; break; }
    uint32_t q = (uint32_t)qd;
    if (words8_submul(nb, a, q, b)) {      // estimate one too high
      q -= 1;
      if (words8_add(nb, b) == 0) { fail = true; break; }
    } else if (words8_ge(nb, b)) {          // estimate one too low
      q += 1;
      words8_sub(nb, b);
      if (words8_ge(nb, b)) { fail = true; break; }
    }
    words5_muladd(nt, ta, q, tb);
#pragma unroll
    for (int i = 0; i < 8; i++) { a[i] = b[i]; b[i] = nb[i]; }
#pragma unroll
    for (int i = 0; i < kHsTW; i++) { ta[i] = tb[i]; tb[i] = nt[i]; }
    fa = fb;
    fb = words_to_double(b, 8);
    iodd = !iodd;
  }
  if ((b[4] | b[5] | b[6] | b[7]) != 0) fail = true;
  if (!fail && (tb[0] & 1u) == 0) {
    // t_i even: (r_{i-1} - j r_i, t_{i-1} - j t_i), sign of t_{i-1} (negative iff i odd)
    const double fta = words_to_double(ta, kHsTW), ftb = words_to_double(tb, kHsTW);
    const double qmax = floor(fa / fb);
    double j0 = floor((fa - fta) / (fb + ftb));
    if (!(qmax < 4294967294.0)) fail = true;
    if (j0 < 0.0) j0 = 0.0;
    if (j0 > qmax) j0 = qmax;
    const double j1 = j0 + 1.0 > qmax ? qmax : j0 + 1.0;
    const double m0 = fmax(fa - j0 * fb, fta + j0 * ftb), m1 = fmax(fa - j1 * fb, fta + j1 * ftb);
    const uint32_t j = fail ? 0u : (uint32_t)(m1 < m0 ? j1 : j0);
    if (words8_submul(nb, a, j, b)) fail = true;  // the estimate of floor(a/b) was high
    words5_muladd(nt, ta, j, tb);
#pragma unroll
    for (int i = 0; i < 8; i++) b[i] = nb[i];
#pragma unroll
    for (int i = 0; i < kHsTW; i++) tb[i] = nt[i];
    iodd = !iodd;  // sign(t_{i-1}) = -sign(t_i)
  }
  if (fail) {
#pragma unroll
    for (int i = 0; i < 8; i++) { c[i] = k[i]; dm[i] = i == 0 ? 1u : 0u; }
    dneg = false;
    if (tight) *tight = 64;
    return 64;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) { c[i] = b[i]; dm[i] = i < kHsTW ? tb[i] : 0u; }
  dneg = !iodd;  // t_i = (-1)^(i+1) |t_i|
  const int bc = bitlen_words(c, 8), bd = bitlen_words(dm, 8);
  if (bd > 150) {  // keeps the recoded |d| within five words (never seen: |d| ~ 2^128)
#pragma unroll
    for (int i = 0; i < 8; i++) { c[i] = k[i]; dm[i] = i == 0 ? 1u : 0u; }
    dneg = false;
    if (tight) *tight = 64;
    return 64;
  }
  const int bits = bc > bd ? bc : bd;
  // |x| < 2^(4W-1): the recoding's carry out of nibble W-1 is folded into the top digit
  // (hs_top_digit, digits 0..8), so 4W-1 bits suffice — one window less on a quarter of the lanes
  const int W = bits / 4 + 1;
  // |x| < 2^(4W): top digits 0..16 — one window less again for the half of the lanes whose
  // longer scalar has exactly 4W bits (128: c < 2^128 by the Euclid stop, |d| <= 2^127)
  const int Wt = (bits + 3) / 4;
  if (tight) *tight = Wt < 29 ? 29 : Wt;
  return W < 29 ? 29 : W;
}

// Top digit (window W-1) of a W-window signed radix-16 recoding (sc_recode16) of x: nibble W-1
// minus 8, plus 16 times the carry the recoding moved into nibble W (that nibble is 8 or 9; every
// nibble above it is 8).  In [0, 8] for x < 2^(4W-1) (the latency kernels' window count), in
// [0, 16] for x < 2^(4W) (the throughput path's tight count: hs_straus adds two table entries).
// w_top is the recoded word holding nibble W-1, w_next the one holding nibble W (W < 64; at
// W = 64 the (k, 1) fallback has x < 2^253 and no carry).
TMED_HD int hs_top_digit(uint32_t w_top, uint32_t w_next, int W) {
  const int n = W - 1;
  const int d = (int)((w_top >> (4 * (n & 7))) & 15u) - 8;
  return W < 64 ? d + 16 * (int)((w_next >> (4 * (W & 7))) & 1u) : d;
}

// The scalar half of phase 1b: the lattice step and e = d S mod L.  Writes the recoded
// scalars — cr, dr: signed radix-16 (sc_recode16; dr words 5..7 are 0x88888888, i.e. zero
// digits, since |d| < 2^150), er: signed radix-2^16 — and the window count W.
TMED_HD void hs_scalars(const uint32_t k[8], const uint32_t s[8], uint32_t cr[8], uint32_t dr[8], uint32_t er[8],
                        bool &dneg, int &W, bool raw_e = false, int *W_tight = nullptr) {
  uint32_t c[8], dm[8], e[8];
  W = sc_halfsize(c, dm, dneg, k, W_tight);
  uint32_t zero[8];
#pragma unroll
  for (int i = 0; i < 8; i++) zero[i] = 0;
  sc_muladd(e, dm, s, zero);  // |d| S mod L
  uint32_t L[8], ne[8];
  sc_const_L(L);
#pragma unroll
  for (int i = 0; i < 8; i++) ne[i] = L[i];
  words8_sub(ne, e);
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) nz |= e[i];
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = (dneg && nz) ? ne[i] : e[i];
  sc_recode16(cr, c);
  sc_recode16(dr, dm);
  if (raw_e) {  // the radix-2^26 B windows recode e themselves (hs_b26_digits)
#pragma unroll
    for (int i = 0; i < 8; i++) er[i] = e[i];
  } else {
    sc_recode_b<16>(er, e);
  }
}

// Phase 1b of the half-size path (after verify_prep's hash / S check / decode of A): strict
// decode of R (affine; the identity when it does not decode) and hs_scalars; returns the R
// verdict.
// permissive (the opt-in ZIP-215 rule): R decoded like A (Point.SetBytes: y >= p and x = 0 with
// the sign bit accepted) instead of strictly.
TMED_HD bool hs_prep_r(const uint32_t k[8], const uint32_t s[8], const uint32_t Rw[8], uint32_t cr[8],
                       uint32_t dr[8], uint32_t er[8], bool &dneg, fe &Rx, fe &Ry, int &W,
                       bool permissive = false, bool raw_e = false, int *W_tight = nullptr) {
  bool rok;
  if (permissive) {
    ge_p3 P;
    rok = ge_frombytes_go(P, Rw);
    fe_copy(Rx, P.X);
    fe_copy(Ry, P.Y);
  } else {
    rok = r_decode_strict(Rx, Ry, Rw);
  }
  if (!rok) { fe_0(Rx); fe_1(Ry); }
  hs_scalars(k, s, cr, dr, er, dneg, W, raw_e, W_tight);
  return rok;
}

// Host-side digit source over the recoded words (the device reads them from the hand-off).
struct HsDigits {
  uint32_t cr[8], dr[8];
  TMED_HDM uint32_t cword(int w) const { return cr[w]; }
  TMED_HDM uint32_t dword(int w) const { return dr[w]; }
};

// Both phases of the half-size prep (the host simulation's single pass of the throughput path):
// W is the tight window count (top digits up to 16), as verify_prep_r_kernel hands over.
TMED_HD bool verify_prep_hs(const uint32_t pubw[8], const uint32_t sigw[16], const uint8_t *msg, uint32_t mlen,
                            HsDigits &dg, uint32_t er[8], bool &dneg, ge_p3 &A, fe &Rx, fe &Ry, int &W,
                            bool raw_e = false) {
  uint32_t k[8], s[8];
  const bool ok = verify_prep(pubw, sigw, msg, mlen, k, s, A);
  int Wl;
  const bool rok = hs_prep_r(k, s, sigw, dg.cr, dg.dr, er, dneg, Rx, Ry, Wl, false, raw_e, &W);
  return ok && rok;
}

TMED_HD void words4_shl16(uint32_t x[4]) {
#pragma unroll
  for (int i = 3; i > 0; i--) x[i] = (x[i] << 16) | (x[i - 1] >> 16);
  x[0] <<= 16;
}

// Radix-2^26 B windows (BL::kBits == 26): e = e_lo + 2^128 e_hi, each half as five signed digits
// of 26 bits, d_m = bits [26m, 26m + 26) + bit (26m - 1) - 2^26 * bit (26m + 25), in [-2^25, 2^25]
// (every digit from the bits alone, no carry chain; the halves are < 2^128, so bits 128, 129
// are 0 and the top digit needs no carry out).  The tables hold j * B and j * 2^128 B for
// j = 0..2^25 (kernels.hip b26_fill_kernel, 8.6 GB).  Digit m is added when 26m doublings remain:
// at the end of windows 0, 13, 26 and after the second doubling of windows 6 and 19 — ten B
// additions instead of the sixteen of radix 2^16 (-42 field multiplications per signature).
TMED_HD int hs_b26_digit(const uint32_t x[4], int m) {
  const int o = 26 * m, q = o >> 5, r = o & 31;
  const uint64_t lo = x[q], hi = q + 1 < 4 ? x[q + 1] : 0u;
  const uint32_t u = (uint32_t)(((hi << 32) | lo) >> r) & 0x3ffffffu;
  const uint32_t below = m ? (x[(o - 1) >> 5] >> ((o - 1) & 31)) & 1u : 0u;
  return (int)(u + below) - (int)((u >> 25) << 26);
}
TMED_HD void hs_b26_digits(int dl[5], int dh[5], const uint32_t er[8]) {
  const uint32_t el[4] = {er[0], er[1], er[2], er[3]}, eh[4] = {er[4], er[5], er[6], er[7]};
#pragma unroll
  for (int m = 0; m < 5; m++) { dl[m] = hs_b26_digit(el, m); dh[m] = hs_b26_digit(eh, m); }
}

// The B step of position m (radix 2^26): r <- t (p1p1 -> p3) + digit lo + digit hi; leaves the sum
// in t (p1p1); the next position's rows are fetched into the buffers right after each take.
template <class BL, class BH>
TMED_HD void hs_b26_add(ge_p1p1 &t, ge_p3 &r, int m, const int dl[5], const int dh[5], BL &bl, BH &bh) {
  ge_niels nb;
  ge_p1p1_to_p3(r, t);
  bl.take(nb);
  if (m > 0) bl.prefetch(dl[m - 1] < 0 ? -dl[m - 1] : dl[m - 1]);
  niels_apply_sign(nb, dl[m] < 0);
  ge_madd_niels(t, r, nb, false);
  ge_p1p1_to_p3(r, t);
  bh.take(nb);
  if (m > 0) bh.prefetch(dh[m - 1] < 0 ? -dh[m - 1] : dh[m - 1]);
  niels_apply_sign(nb, dh[m] < 0);
  ge_madd_niels(t, r, nb, false);
}

// Q = [e]B + [c](-A) + [|d|](-sign(d) R) over W radix-16 windows (Straus, most significant
// first).  DS: cword(w) / dword(w), word w (0..7) of the recoded c / |d| — read once per
// eight windows, before the doublings that hide the read; the top window's digit also takes
// the recoding's carry from nibble W (hs_top_digit).  TA / TR: per-lane cached tables
// of j*(-A) and j*(-sign(d) R), j = 0..8 (build_table_affine), prefetch(j, neg) / take(ge_cached&):
// for neg the entry comes back with Y+X and Y-X exchanged (ge_add_cached_pre).
// BL / BH: niels tables of j*B and j*2^128*B, j = 0..32768, prefetch(j) / take(ge_niels&);
// the 16-bit digits of e (er, recoded) are added at windows 28, 24, ..., 0 (16 doublings
// apart): low-table digit m and high-table digit m + 8 at window 4m, each entry prefetched
// one B step ahead.  Needs 29 <= W <= 64.
template <class DS, class TA, class TR, class BL, class BH>
TMED_HD void hs_straus(ge_p2 &out, const DS &ds, const uint32_t er[8], int W, TA &ta, TR &tr, BL &bl, BH &bh) {
  constexpr bool b26 = BL::kBits == 26;
  static_assert(BL::kBits == 16 || BL::kBits == 26, "B windows of radix 2^16 or 2^26");
  uint32_t el[4] = {er[0], er[1], er[2], er[3]}, eh[4] = {er[4], er[5], er[6], er[7]};
  int d26l[5] = {0, 0, 0, 0, 0}, d26h[5] = {0, 0, 0, 0, 0};
  if (b26) {
    hs_b26_digits(d26l, d26h, er);
    bl.prefetch(d26l[4] < 0 ? -d26l[4] : d26l[4]);
    bh.prefetch(d26h[4] < 0 ? -d26h[4] : d26h[4]);
  } else {
    const int dl = (int)(el[3] >> 16) - 32768, dh = (int)(eh[3] >> 16) - 32768;
    bl.prefetch(dl < 0 ? -dl : dl);
    if (!TMED_B16_ONEBUF) bh.prefetch(dh < 0 ? -dh : dh);
  }
  ge_p2 q;
  ge_p1p1 t;
  ge_p3 r;
  ge_cached ca;
  ge_niels nb;
  uint32_t cw = 0, dw = 0;
#pragma unroll 1
  for (int n = W - 1; n >= 0; n--) {
    if (n == W - 1 || (n & 7) == 7) {
      cw = ds.cword(n >> 3);
      dw = ds.dword(n >> 3);
    }
    if (n == W - 1) {
      // The top window.  Its digits lie in [0, 16] (word W >> 3 holds nibble W; at W = 64, the
      // (k, 1) fallback, there is none and no carry): each is added as two table entries,
      // j1 = min(digit, 8) and digit - j1.  r starts as -A's first entry itself (cached ->
      // extended: one product) instead of an addition to the identity.
      const int dc = hs_top_digit(cw, W < 64 ? ((W & 7) ? cw : ds.cword(W >> 3)) : 0u, W);
      const int dd = hs_top_digit(dw, W < 64 ? ((W & 7) ? dw : ds.dword(W >> 3)) : 0u, W);
      const int c1 = dc < 8 ? dc : 8, d1 = dd < 8 ? dd : 8;
      ta.prefetch(c1, false);
      ta.take(ca);
      ta.prefetch(dc - c1, false);
      ge_cached_to_p3(r, ca);
      ta.take(ca);
      tr.prefetch(d1, false);
      ge_add_cached_pre(t, r, ca, false);
      ge_p1p1_to_p3(r, t);
      tr.take(ca);
      tr.prefetch(dd - d1, false);
      ge_add_cached_pre(t, r, ca, false);
      ge_p1p1_to_p3(r, t);
      tr.take(ca);
      ge_add_cached_pre(t, r, ca, false);
    } else {
      const int sh = 4 * (n & 7);
      const int dc = (int)((cw >> sh) & 15u) - 8, dd = (int)((dw >> sh) & 15u) - 8;
#pragma unroll 1
      for (int k = 0; k < 3; k++) {
        ge_p2_dbl(t, q);
        if (b26 && k == 1 && (n == 6 || n == 19)) hs_b26_add(t, r, n == 19 ? 3 : 1, d26l, d26h, bl, bh);  // 26m left
        ge_p1p1_to_p2(q, t);
      }
      if (TMED_SLAB_PF) ta.prefetch(dc < 0 ? -dc : dc, dc < 0);  // the row load overlaps the last doubling
      ge_p2_dbl(t, q);
      ge_p1p1_to_p3(r, t);
      if (!TMED_SLAB_PF) ta.prefetch(dc < 0 ? -dc : dc, dc < 0);
      ta.take(ca);
      if (TMED_SLAB_PF) tr.prefetch(dd < 0 ? -dd : dd, dd < 0);  // the row load overlaps the A addition
      ge_add_cached_pre(t, r, ca, dc < 0);
      ge_p1p1_to_p3(r, t);
      if (!TMED_SLAB_PF) tr.prefetch(dd < 0 ? -dd : dd, dd < 0);
      tr.take(ca);
      ge_add_cached_pre(t, r, ca, dd < 0);
    }
    if (b26) {
      if (n == 0 || n == 13 || n == 26) hs_b26_add(t, r, n / 13 * 2, d26l, d26h, bl, bh);
    } else if ((n & 3) == 0 && n <= 28) {
      const int dl = (int)(el[3] >> 16) - 32768, dh = (int)(eh[3] >> 16) - 32768;
      words4_shl16(el);
      words4_shl16(eh);
      ge_p1p1_to_p3(r, t);
      bl.take(nb);
      if (TMED_B16_ONEBUF) {  // one LDS row per wave: this window's high row goes where the low one was
        bh.prefetch(dh < 0 ? -dh : dh);
      } else {
        const int dn = (int)(el[3] >> 16) - 32768;
        bl.prefetch(dn < 0 ? -dn : dn);
      }
      niels_apply_sign(nb, dl < 0);
      ge_madd_niels(t, r, nb, false);
      ge_p1p1_to_p3(r, t);
      bh.take(nb);
      {
        const int dn = (int)((TMED_B16_ONEBUF ? el[3] : eh[3]) >> 16) - 32768;
        if (TMED_B16_ONEBUF) bl.prefetch(dn < 0 ? -dn : dn);
        else bh.prefetch(dn < 0 ? -dn : dn);
      }
      niels_apply_sign(nb, dh < 0);
      ge_madd_niels(t, r, nb, false);
    }
    ge_p1p1_to_p2(q, t);
  }
  out = q;
}

// (X : Y : Z) is the identity: X = 0 and Y = Z (Z != 0 for the complete formulas).
TMED_HD bool p2_is_identity(const ge_p2 &q) { return fe_iszero(q.X) && fe_equal(q.Y, q.Z) && !fe_iszero(q.Z); }

// [8] q (three doublings): the cofactored test of the opt-in ZIP-215 rule, [8][d](SB - kA - R) = O,
// exact by the same argument as the cofactorless one ([d] with d odd permutes E[8] and is
// injective on the order-L part).
TMED_HD void p2_mul8(ge_p2 &q) {
  ge_p1p1 t;
#pragma unroll 1
  for (int i = 0; i < 3; i++) {
    ge_p2_dbl(t, q);
    ge_p1p1_to_p2(q, t);
  }
}

// Phase 2 of the half-size path: tables of -A and -sign(d) R, the 3-point sum, the
// identity test (of [8] times the sum when cofactor8: ZIP-215).  A: affine extended (Z = 1,
// T set); R: affine (x, y).
template <class DS, class TA, class TR, class BL, class BH>
TMED_HD bool verify_main_hs(const DS &ds, bool dneg, const uint32_t er[8], int W, const ge_p3 &A, const fe &Rx,
                            const fe &Ry, TA &ta, TR &tr, BL &bl, BH &bh, bool cofactor8 = false) {
  ge_p3 P;  // -A (affine: the decoded key)
  fe_neg(P.X, A.X);
  fe_copy(P.Y, A.Y);
  fe_1(P.Z);
  fe_neg(P.T, A.T);
  build_table_affine(ta, P);
  if (dneg) fe_copy(P.X, Rx); else fe_neg(P.X, Rx);  // -sign(d) R (affine)
  fe_copy(P.Y, Ry);
  fe_mul(P.T, P.X, P.Y);
  build_table_affine(tr, P);
  ge_p2 q;
  hs_straus(q, ds, er, W, ta, tr, bl, bh);
  if (cofactor8) p2_mul8(q);
  return p2_is_identity(q);
}

}  // namespace tmed
