// ge25519.h — edwards25519 group operations for the CDNA4 verify kernels.
//
// Replaces the point layer of Go 1.18 crypto/internal/edwards25519 (Point.SetBytes,
// Point.Bytes, VarTimeDoubleScalarBaseMult's add/double steps), reached from
// crypto/ed25519/ed25519.go:154 in the reference.
//
// Coordinates (a = -1 twisted Edwards, complete HWCD formulas):
//   p2    (X:Y:Z)                x = X/Z, y = Y/Z
//   p3    (X:Y:Z:T)              extended, T = XY/Z
//   p1p1  (X:Y:Z:T) "completed"  x = X/Z, y = Y/T
//   cached (Y+X, Y-X, Z, 2dT)    variable-base table entries
//   niels  (y+x, y-x, 2dxy)      affine fixed-base table entries (Z = 1)
// The formulas are complete on the whole curve (d is a non-square), so the
// result of every add/double is the exact group element whatever the inputs
// (small-order and mixed-order points included) — which is what makes the
// GPU decision equal to Go's for every edge case.
#pragma once
#include "fe25519.h"

namespace tmed {

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z, T2d; };
struct ge_niels { fe YpX, YmX, XY2d; };

TMED_HD void ge_p2_0(ge_p2 &h) { fe_0(h.X); fe_1(h.Y); fe_1(h.Z); }
TMED_HD void ge_p3_0(ge_p3 &h) { fe_0(h.X); fe_1(h.Y); fe_1(h.Z); fe_0(h.T); }
TMED_HD void ge_cached_0(ge_cached &h) { fe_1(h.YpX); fe_1(h.YmX); fe_1(h.Z); fe_0(h.T2d); }
TMED_HD void ge_niels_0(ge_niels &h) { fe_1(h.YpX); fe_1(h.YmX); fe_0(h.XY2d); }

// (Independent products in pairs, fe_mul_x2; p1p1 -> p3 pairs only X, Y: a second pair spilled
// in verify_main_hs_kernel.)  fe_mul(h, f, g) premultiplies g by 19 (nine v_mul_lo_u32) and
// f's odd limbs by 2: the operands are ordered so that only T and Y are ever g (and X, Z f),
// and the compiler shares those copies between the products: 18 instead of 27 x19 copies in
// p1p1 -> p3, 10 instead of 15 x2 copies in p1p1 -> p2.
#ifndef TMED_P1P1_VC
#define TMED_P1P1_VC 1  // A/B knob: 0 = Y * Z with Y as f (the round-2 order)
#endif
TMED_HD void ge_p1p1_to_p2(ge_p2 &r, const ge_p1p1 &p) {
  if (TMED_P1P1_VC) fe_mul_x2(r.X, p.X, p.T, r.Y, p.Z, p.Y);
  else fe_mul_x2(r.X, p.X, p.T, r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
}
TMED_HD void ge_p1p1_to_p3(ge_p3 &r, const ge_p1p1 &p) {
  if (TMED_P1P1_VC) fe_mul_x2(r.X, p.X, p.T, r.Y, p.Z, p.Y);
  else fe_mul_x2(r.X, p.X, p.T, r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(r.T, p.X, p.Y);
}
TMED_HD void ge_p3_to_p2(ge_p2 &r, const ge_p3 &p) { fe_copy(r.X, p.X); fe_copy(r.Y, p.Y); fe_copy(r.Z, p.Z); }
// Cached (Y+X, Y-X, Z, 2dT) -> extended, every coordinate scaled by 2 (the same point):
// (Y+X) - (Y-X) = 2X, (Y+X) + (Y-X) = 2Y, 2Z, and 2T = 2dT * d^-1 — one product.  Outputs
// carried (the inputs may be unpacked table entries, limbs up to twice a carried limb).
TMED_HD void ge_cached_to_p3(ge_p3 &r, const ge_cached &c) {
  fe inv_d;  // d^-1 mod p, carried form
  const int32_t k[10] = {30013526, 3972531, -24787780, 12719051, 2979674, -4599962, -15693209, -3644061, 18959709, -16629253};
#pragma unroll
  for (int i = 0; i < 10; i++) inv_d.v[i] = k[i];
  fe_sub(r.X, c.YpX, c.YmX);
  fe_carry(r.X, r.X);
  fe_add(r.Y, c.YpX, c.YmX);
  fe_carry(r.Y, r.Y);
  fe_add(r.Z, c.Z, c.Z);
  fe_carry(r.Z, r.Z);
  fe_mul(r.T, c.T2d, inv_d);
}
TMED_HD void ge_p3_to_cached(ge_cached &r, const ge_p3 &p) {
  fe d2; fe_const_d2(d2);
  fe_add(r.YpX, p.Y, p.X);
  fe_sub(r.YmX, p.Y, p.X);
  fe_copy(r.Z, p.Z);
  fe_mul(r.T2d, p.T, d2);
}

// r = 2p.  4 squarings; outputs are <= 3-sums (see fe25519.h).
TMED_HD void ge_p2_dbl(ge_p1p1 &r, const ge_p2 &p) {
  fe xx, yy, b, a, t;
  fe_sqc_x2(xx, p.X, yy, p.Y);  // X, Y carried: product outputs, decoded or identity coordinates
  fe_add(t, p.X, p.Y);
  fe_sq2_sq(b, p.Z, a, t);
  fe_add(r.Y, yy, xx);
  fe_sub(r.Z, yy, xx);
  fe_sub(r.X, a, r.Y);
  fe_sub(r.T, b, r.Z);
}

// r = p + (neg ? -q : q)   with q cached.  -q = (Y-X, Y+X, Z, -2dT).
// r = p + (neg ? -q : q), with q's Y+X / Y-X already exchanged when neg (the per-lane tables
// swap them through the load addresses): only 2dT's sign is left.
TMED_HD void ge_add_cached_pre(ge_p1p1 &r, const ge_p3 &p, const ge_cached &q, bool neg) {
  fe a, b, c, d, t, t2;
  fe_add(t, p.Y, p.X);
  fe_sub(t2, p.Y, p.X);
  fe_mul_x2(a, t, q.YpX, b, t2, q.YmX);
  fe_mul_x2(c, q.T2d, p.T, d, p.Z, q.Z);
  fe_neg(t, c); fe_select(c, c, t, neg);
  fe_add(d, d, d);
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_add(r.Z, d, c);
  fe_sub(r.T, d, c);
}

TMED_HD void ge_add_cached(ge_p1p1 &r, const ge_p3 &p, const ge_cached &q, bool neg) {
  fe a, b, c, d, t, t2, qp, qm;
  fe_select(qp, q.YpX, q.YmX, neg);
  fe_select(qm, q.YmX, q.YpX, neg);
  fe_add(t, p.Y, p.X);
  fe_sub(t2, p.Y, p.X);
  fe_mul_x2(a, t, qp, b, t2, qm);
  fe_mul_x2(c, q.T2d, p.T, d, p.Z, q.Z);
  fe_neg(t, c); fe_select(c, c, t, neg);
  fe_add(d, d, d);
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_add(r.Z, d, c);
  fe_sub(r.T, d, c);
}

// r = p + (neg ? -q : q)   with q niels (affine, Z = 1).
TMED_HD void ge_madd_niels(ge_p1p1 &r, const ge_p3 &p, const ge_niels &q, bool neg) {
  fe a, b, c, d, t, t2, qp, qm;
  fe_select(qp, q.YpX, q.YmX, neg);
  fe_select(qm, q.YmX, q.YpX, neg);
  fe_add(t, p.Y, p.X);
  fe_sub(t2, p.Y, p.X);
  fe_mul_x2(a, t, qp, b, t2, qm);
  fe_mul(c, q.XY2d, p.T);
  fe_neg(t, c); fe_select(c, c, t, neg);
  fe_add(d, p.Z, p.Z);
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_add(r.Z, d, c);
  fe_sub(r.T, d, c);
}

// Go Point.SetBytes (permissive): y >= p accepted (reduced), bit 255 selects
// the sign of x, x = 0 with the sign bit set accepted, non-square rejected.
// Returns false on rejection (h is then the identity, so callers can keep
// computing branch-free and mask the decision).
TMED_HD bool ge_frombytes_go(ge_p3 &h, const uint32_t w[8]) {
  fe y, u, v, v3, uv7, r, chk, t, one, d, sqrtm1;
  fe_const_d(d); fe_const_sqrtm1(sqrtm1); fe_1(one);
  fe_from_words(y, w);
  fe_sqc(u, y);
  fe_mul(v, u, d);
  fe_sub(u, u, one); fe_carry(u, u);       // u = y^2 - 1
  fe_add(v, v, one); fe_carry(v, v);       // v = d y^2 + 1
  // SqrtRatio(u, v): r = (u v^3) (u v^7)^((p-5)/8)
  fe_sqc(t, v); fe_mul(v3, t, v);          // v^3
  fe_sqc(t, v3); fe_mul(uv7, t, v);        // v^7
  fe_mul(uv7, uv7, u);                     // u v^7
  fe_pow22523(t, uv7);
  fe_mul(r, u, v3);
  fe_mul(r, r, t);
  fe_sqc(t, r); fe_mul(chk, v, t);         // check = v r^2
  fe uneg; fe_neg(uneg, u);
  const bool correct = fe_equal(chk, u);
  const bool flipped = fe_equal(chk, uneg);
  fe_mul(t, uneg, sqrtm1);
  const bool flipped_i = fe_equal(chk, t);
  fe_mul(t, r, sqrtm1);
  fe_select(r, r, t, flipped || flipped_i);
  fe_neg(t, r);
  fe_select(r, r, t, fe_isnegative(r));    // Absolute(): non-negative root
  const bool ok = correct || flipped;
  fe_neg(t, r);
  fe_select(r, r, t, (w[7] >> 31) != 0);   // sign bit
  fe_copy(h.X, r); fe_copy(h.Y, y); fe_1(h.Z); fe_mul(h.T, r, y);
  if (!ok) ge_p3_0(h);
  return ok;
}

// Go Point.Bytes: canonical y with bit 255 = parity of x, as 8 LE words.
TMED_HD void ge_tobytes(uint32_t w[8], const fe &X, const fe &Y, const fe &Z) {
  fe zi, x, y;
  fe_invert(zi, Z);
  fe_mul(x, X, zi);
  fe_mul(y, Y, zi);
  fe_to_words(w, y);
  w[7] |= (uint32_t)fe_isnegative(x) << 31;
}

}  // namespace tmed
