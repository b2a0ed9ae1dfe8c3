// quad.h — 4-way split extended twisted-Edwards formulas: a quad of lanes (4q..4q+3) holds one
// point, one coordinate per lane (X, Y, Z, T), and runs the four field multiplications of each
// doubling / addition round in parallel; operands move inside the quad by DPP quad permutations.
// Used where one point operation's latency matters: the generic latency kernels (latency.hip,
// C1) and the ZIP-215 batch equation's final Horner chain (zip215.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "ge25519.h"
#include "kernels.h"

namespace tmed {

// ---- quad exchanges (DPP; lanes 4q..4q+3 form quad q) ---------------------------------------
template <int P0, int P1, int P2, int P3>
__device__ __forceinline__ void fe_qperm(fe &o, const fe &f) {
  constexpr int kCtrl = P0 | (P1 << 2) | (P2 << 4) | (P3 << 6);  // quad_perm
#pragma unroll
  for (int i = 0; i < 10; i++) o.v[i] = __builtin_amdgcn_mov_dpp(f.v[i], kCtrl, 0xf, 0xf, false);
}
__device__ __forceinline__ int32_t qbcast(int32_t v, int src) {  // lane src of each quad
  switch (src) {
    case 0: return __builtin_amdgcn_mov_dpp(v, 0x00, 0xf, 0xf, false);
    case 1: return __builtin_amdgcn_mov_dpp(v, 0x55, 0xf, 0xf, false);
    case 2: return __builtin_amdgcn_mov_dpp(v, 0xaa, 0xf, 0xf, false);
    default: return __builtin_amdgcn_mov_dpp(v, 0xff, 0xf, 0xf, false);
  }
}

// Per-lane constants of the quad formulas (r = lane & 3).
struct QuadK {
  int r;
  int32_t m1;    // -1 on r = 1 (the Y of a doubling's (X + Y)^2 operand)
  int32_t ky;    // doubling V: coefficient of the (S | C) operand: 1, -2, 0, 0
  int32_t mB;    // doubling V: -1 where B enters negated (r = 0, 3)
  int32_t s1;    // addition round 1: sign of the own coordinate: -1, +1, 0, 0
  int32_t m01;   // addition V: -1 where y enters negated (r = 0, 1)
  __device__ explicit QuadK(int lane) {
    r = lane & 3;
    m1 = r == 1 ? -1 : 0;
    ky = r == 0 ? 1 : (r == 1 ? -2 : 0);
    mB = (r == 0 || r == 3) ? -1 : 0;
    s1 = r == 0 ? -1 : (r == 1 ? 1 : 0);
    m01 = r < 2 ? -1 : 0;
  }
};

// Round 2 shared by doubling and addition: lanes hold V = (E, F, G, H); lane r gets
// (o1, o2) = (F, E), (G, H), (F, G), (E, H) and multiplies: X3 = EF, Y3 = GH, Z3 = FG, T3 = EH.
// o1 is the f operand of fe_mul (x2 copies only), so F may be the doubling's 4-sum.
__device__ __forceinline__ void quad_round2(fe &v, const fe &V) {
  fe o1, o2;
  fe_qperm<1, 2, 1, 0>(o1, V);
  fe_qperm<0, 3, 2, 3>(o2, V);
  fe_mul(v, o1, o2);
}

// v <- 2v (extended; T is not read).  Round 1: X^2, Y^2, Z^2, (X + Y)^2; then lane r forms
// E = S - A - B, F = B - A - 2C, G = B - A, H = -A - B  (dbl-2008-hwcd, a = -1; the result is
// the negation of ref10's (X', Y', Z', T') products, the same projective point).
__device__ __forceinline__ void quad_dbl(fe &v, const QuadK &K) {
  fe a, b, op, s;
  fe_qperm<0, 1, 2, 0>(a, v);  // lane 3 <- X
#pragma unroll
  for (int i = 0; i < 10; i++) op.v[i] = v.v[i] & K.m1;
  fe_qperm<0, 0, 0, 1>(b, op);  // lane 3 <- Y, lanes 0..2 <- 0
#pragma unroll
  for (int i = 0; i < 10; i++) op.v[i] = a.v[i] + b.v[i];
  fe_sq(s, op);
  fe V;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int32_t A = qbcast(s.v[i], 0), B = qbcast(s.v[i], 1);
    const int32_t y = __builtin_amdgcn_mov_dpp(s.v[i], 3 | (2 << 2) | (2 << 4) | (2 << 6), 0xf, 0xf, false);
    V.v[i] = y * K.ky + ((B ^ K.mB) - K.mB) - A;
  }
  quad_round2(v, V);
}

// v <- v + q, q cached on the quad (lane r: Y-X, Y+X, 2dT, 2Z of q).  Round 1:
// A = (Y1-X1)(Y2-X2), B = (Y1+X1)(Y2+X2), C = T1 * 2dT2, D = Z1 * 2Z2; then
// E = B - A, F = D - C, G = D + C, H = B + A (add-2008-hwcd-3).
__device__ __forceinline__ void quad_add(fe &v, const fe &q, const QuadK &K) {
  fe t, op, p;
  fe_qperm<1, 0, 3, 2>(t, v);  // Y, X, T, Z
#pragma unroll
  for (int i = 0; i < 10; i++) op.v[i] = t.v[i] + v.v[i] * K.s1;
  fe_mul(p, op, q);
  fe x, y, V;
  fe_qperm<1, 3, 3, 1>(x, p);  // B, D, D, B
  fe_qperm<0, 2, 2, 0>(y, p);  // A, C, C, A
#pragma unroll
  for (int i = 0; i < 10; i++) V.v[i] = x.v[i] + ((y.v[i] ^ K.m01) - K.m01);
  quad_round2(v, V);
}

// Lane r of the cached form of the quad's point: Y - X, Y + X, 2d T, 2Z.
__device__ __forceinline__ void quad_to_cached(fe &c, const fe &v, const QuadK &K) {
  fe t, m, d2;
  fe_qperm<1, 0, 3, 2>(t, v);  // Y, X, T, Z
  fe_const_d2(d2);
  fe_mul(m, t, d2);
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int32_t u = K.r == 3 ? t.v[i] : v.v[i] * K.s1;
    c.v[i] = K.r == 2 ? m.v[i] : t.v[i] + u;
  }
}

// Per-lane coordinate of the identity in extended / cached form.
__device__ __forceinline__ void quad_identity(fe &v, int r) {
  fe_0(v);
  v.v[0] = (r == 1 || r == 2) ? 1 : 0;
}
__device__ __forceinline__ void quad_identity_cached(fe &c, int r) {
  fe_0(c);
  c.v[0] = r < 2 ? 1 : (r == 2 ? 0 : 2);
}

// Entry |dg| of a radix-2^16 comb window as a cached point (Z = 1): lane r reads Y-X, Y+X,
// 2dxy from the 128-B niels row (YpX, YmX, XY2d), lane 3 the constant 2Z = 2.
__device__ __forceinline__ void comb_take(fe &c, const int4 *window, int dg, const QuadK &K) {
  const bool neg = dg < 0;
  const int j = neg ? -dg : dg;
  const int fidx = K.r == 0 ? (neg ? 0 : 1) : (K.r == 1 ? (neg ? 1 : 0) : 2);
  const int32_t *row = reinterpret_cast<const int32_t *>(window + (size_t)j * kCombEntryInt4) + fidx * 10;
  const int32_t m = (neg && K.r == 2) ? -1 : 0;
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = (row[i] ^ m) - m;
  if (K.r == 3) { fe_0(c); c.v[0] = 2; }
}

}  // namespace tmed
