// latency.hip — latency mode of the generic (uncached-key) path: one small batch (a single
// commit, C1) finishes in a few hundred microseconds instead of one lone lane per signature
// running the whole throughput pipeline.
//
// Callers: the first commit after a validator-set change, evidence/verify.go:130
// (ConflictingBlock.ValidatorSet, a fresh set per call) and the untrusted sets of
// light/verifier.go:73,126 — every VerifyCommit* on keys that are not in a key set
// (types/validator_set.go:667-826).  Same decision as the throughput path (verify_hs.h): Go's
// enc([S]B - [k]A) == R, as  R strictly decodes and [e]B - [c]A - [d]R is the identity.
//
// Two launches:
//  1. verify_glat_prep_kernel, wave-uniform roles by block (64-lane blocks):
//     * decode blocks: one lane per POINT, A_0..A_{n-1} then R_0..R_{n-1} (the same sqrt-ratio
//       chain; R also gets the strict checks) -> affine (x, y) and the verdict;
//     * hash blocks: one lane per signature: SHA-512(R||A||M) mod L, the S checks, the lattice
//       step and e = d S mod L (hs_scalars) -> recoded c, |d|, e, sign(d), W.
//     Both chains are ~the length of one sqrt-ratio chain and run side by side.
//  2. verify_glat_main_kernel: 8 lanes per signature, two quads.  A quad holds one point in
//     extended coordinates, one coordinate per lane (lane r of the quad: X, Y, Z, T), and runs
//     the four field multiplications of each doubling / addition round in parallel (the
//     4-way split of the extended twisted-Edwards formulas); operands move between the quad's
//     lanes with DPP quad permutations.  Quad 0 accumulates [c](-A) + [e_lo]B, quad 1
//     [|d|](-sign(d) R) + [e_hi] 2^128 B over the same W radix-16 windows (the Straus schedule
//     of hs_straus, verify_hs.h); the tables of j(-A), j(-sign(d) R) are built 4-way into LDS,
//     the B entries come from the radix-2^16 comb.  Quad 1's sum is moved onto quad 0 (DPP
//     row shift), added, and the identity test is projective.
#include "kernel_util.h"
#include "votes_dev.h"
#include "kernels.h"
#include "verify_core.h"
#include "verify_hs.h"
#include "quad.h"

namespace tmed {

namespace {

// LDS table of one 64-lane block: [entry 0..8][limb][lane], one coordinate per lane.
struct QuadTab {
  int32_t (*t)[10][64];
  int lane;
  __device__ void store(int j, const fe &c) const {
#pragma unroll
    for (int i = 0; i < 10; i++) t[j][i][lane] = c.v[i];
  }
  // digit dg in [-8, 8]: entry |dg|, negated (swap Y-X / Y+X between lanes 0 and 1, negate 2dT).
  __device__ void take(fe &c, int dg, const QuadK &K) const {
    const bool neg = dg < 0;
    const int j = neg ? -dg : dg;
    const int src = (neg && K.r < 2) ? (lane ^ 1) : lane;
    const int32_t m = (neg && K.r == 2) ? -1 : 0;
#pragma unroll
    for (int i = 0; i < 10; i++) c.v[i] = (t[j][i][src] ^ m) - m;
  }
};

// Table j * P, j = 0..8, of the affine point P = (x, y) (every lane of the quad holds x, y):
// entry 1 is P itself, entry j = entry j-1 + P by quad_add.
__device__ void quad_build_table(const QuadTab &tab, const fe &x, const fe &y, const QuadK &K) {
  fe c, v, t, d2;
  quad_identity_cached(c, K.r);
  tab.store(0, c);
  // cached P: y - x, y + x, 2d xy, 2
  fe_mul(t, x, y);
  fe_const_d2(d2);
  fe_mul(v, t, d2);
  fe p1;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int32_t a = K.r == 0 ? y.v[i] - x.v[i] : y.v[i] + x.v[i];
    p1.v[i] = K.r < 2 ? a : (K.r == 2 ? v.v[i] : (i == 0 ? 2 : 0));
  }
  tab.store(1, p1);
  // the quad's extended P: x, y, 1, xy
#pragma unroll
  for (int i = 0; i < 10; i++) v.v[i] = K.r == 0 ? x.v[i] : (K.r == 1 ? y.v[i] : (K.r == 2 ? (i == 0 ? 1 : 0) : t.v[i]));
#pragma unroll 1
  for (int j = 2; j <= 8; j++) {
    quad_add(v, p1, K);
    quad_to_cached(c, v, K);
    tab.store(j, c);
  }
}

// ---- hand-off layout (int4 [q][index]) -------------------------------------------------------
// decode region: 6 int4 per point (x[10], y[10], ok), points 0..cap-1 = A, cap..2cap-1 = R.
// scalar region: 7 int4 per signature (cr[8], dr[8], er[8], flags: ok | dneg << 1 | W << 8).
constexpr int kDecInt4 = 6;
constexpr int kScInt4 = 7;

}  // namespace

__global__ __launch_bounds__(64) void verify_glat_prep_kernel(const uint8_t *__restrict__ pub,
                                                              const uint8_t *__restrict__ sig, MsgSrc ms, uint32_t n,
                                                              uint32_t nD, int4 *__restrict__ hand, uint32_t cap,
                                                              VoteAsm va, int assemble) {
  __shared__ int4 tl[64][kVoteTmplBytes / 16];  // the hash lanes' vote templates (assemble_vote)
  const uint32_t t = threadIdx.x;
  if (blockIdx.x < nD) {  // decode role: point p = A_p (p < n) or R_{p-n}
    const uint32_t p = blockIdx.x * 64 + t;
    if (p >= 2 * n) return;
    const bool isR = p >= n;
    const uint32_t i = isR ? p - n : p;
    uint32_t w[8];
    if (isR)
      load_row_words(w, sig + 64 * (size_t)i, 2);
    else
      load_row_words(w, pub + 32 * (size_t)i, 2);
    ge_p3 P;
    bool ok = ge_frombytes_go(P, w);          // Point.SetBytes (A: permissive)
    if (isR) ok = ok && r_strict_extra(P.X, w);  // R: strict (r_decode_strict)
    fe x, y;
    fe_copy(x, P.X);
    fe_copy(y, P.Y);
    if (!ok) { fe_0(x); fe_1(y); }
    int32_t o[24];
#pragma unroll
    for (int k = 0; k < 10; k++) { o[k] = x.v[k]; o[10 + k] = y.v[k]; }
    o[20] = ok ? 1 : 0;
    o[21] = o[22] = o[23] = 0;
    const uint32_t slot = isR ? cap + i : i;
#pragma unroll
    for (int q = 0; q < kDecInt4; q++)
      hand[(size_t)q * 2 * cap + slot] = make_int4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    return;
  }
  const uint32_t i = (blockIdx.x - nD) * 64 + t;  // scalar role
  if (i >= n) return;
  if (assemble) assemble_vote(va, i, const_cast<uint8_t *>(ms.msgs), const_cast<uint32_t *>(ms.off), tl[t]);
  uint32_t pw[8], sw[16], k[8], s[8], cr[8], dr[8], er[8];
  load_row_words(pw, pub + 32 * (size_t)i, 2);
  load_row_words(sw, sig + 64 * (size_t)i, 4);
  const uint8_t *m;
  uint32_t mlen;
  ms.get(i, m, mlen);
  const bool ok = verify_prep_comb(pw, true, sw, m, mlen, k, s);  // hash, S checks (A: decode role)
  bool dneg;
  int W;
  hs_scalars(k, s, cr, dr, er, dneg, W);
  uint32_t o[28];
#pragma unroll
  for (int j = 0; j < 8; j++) { o[j] = cr[j]; o[8 + j] = dr[j]; o[16 + j] = er[j]; }
  o[24] = (ok ? 1u : 0u) | (dneg ? 2u : 0u) | ((uint32_t)W << 8);
  o[25] = o[26] = o[27] = 0;
  int4 *sc = hand + (size_t)kDecInt4 * 2 * cap;
#pragma unroll
  for (int q = 0; q < kScInt4; q++)
    sc[(size_t)q * cap + i] = make_int4((int)o[4 * q], (int)o[4 * q + 1], (int)o[4 * q + 2], (int)o[4 * q + 3]);
}

__global__ __launch_bounds__(64) void verify_glat_main_kernel(const int4 *__restrict__ hand, uint32_t n, uint32_t cap,
                                                              const int4 *__restrict__ comb16,
                                                              uint8_t *__restrict__ out) {
  __shared__ int32_t tabmem[9][10][64];
  const int lane = (int)threadIdx.x;
  const QuadK K(lane);
  const int quad = (lane >> 2) & 1;  // 0: -A, c, e_lo; 1: -sign(d) R, |d|, e_hi
  const uint32_t gi = blockIdx.x * 8 + (uint32_t)(lane >> 3);
  const bool active = gi < n;
  const uint32_t i = active ? gi : 0;  // idle groups replay signature 0 and store nothing
  // scalars and flags of signature i
  const int4 *sc = hand + (size_t)kDecInt4 * 2 * cap;
  uint32_t w[28];
#pragma unroll
  for (int q = 0; q < kScInt4; q++) {
    const int4 v = sc[(size_t)q * cap + i];
    w[4 * q] = (uint32_t)v.x; w[4 * q + 1] = (uint32_t)v.y; w[4 * q + 2] = (uint32_t)v.z; w[4 * q + 3] = (uint32_t)v.w;
  }
  const uint32_t flags = w[24];
  const bool dneg = (flags & 2u) != 0;
  int W = (int)(flags >> 8);
  uint32_t e4[4];
  const uint32_t dbase = quad ? 8u : 0u;  // the quad's digit words (c or |d|) in the scalar region
#pragma unroll
  for (int j = 0; j < 4; j++) e4[j] = quad ? w[20 + j] : w[16 + j];
  // the quad's point: -A (quad 0) or -sign(d) R (quad 1), affine
  const uint32_t slot = quad ? cap + i : i;
  int32_t pw[24];
#pragma unroll
  for (int q = 0; q < kDecInt4; q++) {
    const int4 v = hand[(size_t)q * 2 * cap + slot];
    pw[4 * q] = v.x; pw[4 * q + 1] = v.y; pw[4 * q + 2] = v.z; pw[4 * q + 3] = v.w;
  }
  const bool pok = pw[20] != 0;
  fe x, y;
#pragma unroll
  for (int k = 0; k < 10; k++) { x.v[k] = pw[k]; y.v[k] = pw[10 + k]; }
  if (quad == 0 || !dneg) fe_neg(x, x);
  // loop length: the largest W of the wave's eight signatures
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int v = __shfl_xor(W, o);
    W = v > W ? v : W;
  }
  W = __builtin_amdgcn_readfirstlane(W);
  if (W < 29) W = 29;
  if (W > 64) W = 64;

  const QuadTab tab{tabmem, lane};
  quad_build_table(tab, x, y, K);
  __syncthreads();  // the table's LDS writes before other lanes of the quad read them
  const int4 *bwin = comb16 + (quad ? (size_t)8 * kB16Entries * kCombEntryInt4 : 0);
  fe acc, c;
  quad_identity(acc, K.r);
  uint32_t cw = 0;
#pragma unroll 1
  for (int nw = W - 1; nw >= 0; nw--) {
    if (nw == W - 1 || (nw & 7) == 7) {  // word nw / 8 of the recoded scalar (re-read: no dynamic register index)
      const uint32_t wd = dbase + (uint32_t)(nw >> 3);
      cw = reinterpret_cast<const uint32_t *>(sc + (size_t)(wd >> 2) * cap + i)[wd & 3];
    }
    if (nw != W - 1) {
#pragma unroll 1
      for (int k = 0; k < 4; k++) quad_dbl(acc, K);
    }
    int dg = (int)((cw >> (4 * (nw & 7))) & 15u) - 8;
    if (nw == W - 1 && W < 64) {  // top window: the recoding's carry into nibble W (hs_top_digit)
      const uint32_t wn = dbase + (uint32_t)(W >> 3);
      const uint32_t cn = (W & 7) ? cw : reinterpret_cast<const uint32_t *>(sc + (size_t)(wn >> 2) * cap + i)[wn & 3];
      dg = hs_top_digit(cw, cn, W);
    }
    tab.take(c, dg, K);
    quad_add(acc, c, K);
    if ((nw & 3) == 0 && nw <= 28) {
      const int db = (int)(e4[3] >> 16) - 32768;
      words4_shl16(e4);
      comb_take(c, bwin, db, K);
      quad_add(acc, c, K);
    }
  }
  // quad 1's sum onto quad 0 (row shift by 4 lanes), one more addition, identity test
  quad_to_cached(c, acc, K);
  fe c1;
#pragma unroll
  for (int k = 0; k < 10; k++) c1.v[k] = __builtin_amdgcn_mov_dpp(c.v[k], 0x104, 0xf, 0xf, false);  // row_shl:4
  quad_add(acc, c1, K);
  fe zt, u;
  fe_qperm<0, 2, 2, 3>(zt, acc);  // lane 1 <- Z
#pragma unroll
  for (int k = 0; k < 10; k++) u.v[k] = K.r == 1 ? acc.v[k] - zt.v[k] : acc.v[k];
  fe_carry(u, u);
  const int z = fe_iszero(u) ? 1 : 0;  // lane 0: X = 0, lane 1: Y = Z, lane 2: Z = 0
  const int z0 = qbcast(z, 0), z1 = qbcast(z, 1), z2 = qbcast(z, 2);
  const int ok0 = qbcast(pok ? 1 : 0, 0);  // the A verdict (quad 0) and the R verdict (quad 1)
  const int okR = __builtin_amdgcn_mov_dpp(pok ? 1 : 0, 0x104, 0xf, 0xf, false);
  if (active && lane % 8 == 0)
    out[gi] = ((flags & 1u) && ok0 && okR && z0 && z1 && !z2) ? 1 : 0;
}

hipError_t launch_verify_glat(const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                              uint32_t n, uint8_t *out, const int4 *comb16, int4 *hand, hipStream_t stream,
                              bool msg_slots, KernelTimer *timer, const VoteAsm *va) {
  if (n == 0) return hipSuccess;
  if (n > kGLatMax) return hipErrorInvalidValue;  // the hand-off is sized for kGLatMax signatures
  const MsgSrc ms{msgs, off, msg_slots};
  const uint32_t nD = (2 * n + 63) / 64, nH = (n + 63) / 64;
  if (timer) timer->mark(stream, -1);
  if (va && !msg_slots) return hipErrorInvalidValue;
  hipLaunchKernelGGL(verify_glat_prep_kernel, dim3(nD + nH), dim3(64), 0, stream, pub, sig, ms, n, nD, hand,
                     kGLatMax, va ? *va : VoteAsm{}, va ? 1 : 0);
  if (timer) timer->mark(stream, 0);
  hipLaunchKernelGGL(verify_glat_main_kernel, dim3((n + 7) / 8), dim3(64), 0, stream, hand, n, kGLatMax, comb16, out);
  if (timer) timer->mark(stream, 1);
  return hipGetLastError();
}

}  // namespace tmed
