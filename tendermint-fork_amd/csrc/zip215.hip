// zip215.hip — opt-in ZIP-215 batch verification (BASELINE north_star: "Straus or Pippenger
// multi-scalar multiplication for the randomized batch equation, with wavefront-level bucket
// reductions and a bisecting fallback so per-signature accept/reject bits stay exact").
//
// The rule is ZIP-215 (spec/core/encoding.md:52-54 names it as the rule Tendermint adopts; the
// reference's code, crypto/ed25519/ed25519.go:148-155 -> Go 1.18 Verify, is cofactorless and stays
// the engine's default): A and R decoded permissively, S < L, k = SHA-512(R || A || M) mod L,
// accept iff [8]([S]B - R - [k]A) = O.  Restated in oracle/zip215.py; parity unpinned by the
// reference (it holds no ZIP-215 code or vectors).
//
// A chunk of N <= kZipMax signatures is checked as ONE equation with secret random 126-bit z_i
// (SHA-512 of a per-call 32-byte seed and the signature index):
//   [8]( [sum z_i S_i] B + sum_i [z_i k_i](-A_i) + sum_i [z_i](-R_i) ) = O,
// i.e. one multi-scalar multiplication over 2N points plus one fixed-base product.  Scalars mod L
// are exact here: the factor 8 removes every torsion component a reduction mod L could change.
// The MSM is Pippenger with signed radix-2^16 digits (16 windows for the A scalars, 8 for the
// 126-bit z), on the GPU:
//   zip_prep_r_kernel   decode R, z, z k mod L, z S mod L, niels rows of -A / -R, the digits
//   zip_bsum_*          sum z_i S_i mod L
//   zip_sort_*          per window, a stable two-pass LSD counting sort of (|digit|, point) by
//                       |digit| (8-bit passes; every tile is ranked by ONE wave with ballot
//                       matching into LDS and written out in bin order; no global atomics)
//   zip_accum_kernel    lane l of window w owns buckets 4l..4l+3: mixed additions of their
//                       points (sorted runs, next row prefetched), then the bucket-weighted
//                       running sums S_l = sum B_v, T_l = sum (v - 4l) B_v
//   zip_reduce*_kernel  wavefront-level bucket reduction: 64 items per wave by a suffix scan and
//                       two trees over shuffles, sum (d i S_i + T_i) -> one item; 3 levels in 2 launches
//   zip_final_kernel    Horner over the 16 windows, + [sum z S] B (radix-2^16 comb), x8, = O?
// A chunk whose equation fails is bisected (the same MSM over halves of its signatures, prep
// data reused); a group that still fails is decided signature by signature by the exact ZIP-215
// single check (the half-size kernels with a permissive R decode and a [8] before the identity
// test).  Every accepted group is all-valid with probability >= 1 - 2^-125 per failing signature
// (the z are secret); every rejected signature comes from the exact single check.
#include <hip/hip_runtime.h>
#include <string.h>
#include <sys/random.h>

#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "ctx.h"
#include "kernel_util.h"
#include "verify_core.h"
#include "verify_hs.h"
#include "quad.h"

namespace tmed {

constexpr int kZipWin = 16;       // radix-2^16 windows of the A scalars (z: windows 0..7)
constexpr int kZipZWin = 8;
constexpr uint32_t kZipRow = 8;   // int4 per niels point row (128 B)
// Accumulation lanes per window, balanced at ~cnt/8192 entries each: a lane owns g consecutive
// buckets |digit| = g l .. g l + g - 1 (and, for the top A window, h = 2 lanes split each group):
// windows 0..7 (A and R points, 2 cnt entries over 32768 buckets): g = 2, 16385 groups;
// windows 8..14 (A only): g = 4, 8193 groups; window 15 (the top 13 bits of a < L: digits 0..4097,
// 8x fewer buckets): g = 1, 4098 groups, h = 2.
constexpr uint32_t kZipItemsMax = 16385;
__host__ __device__ __forceinline__ int zip_glog(int w) { return w < 8 ? 1 : (w < 15 ? 2 : 0); }
__host__ __device__ __forceinline__ uint32_t zip_groups(int w) { return w < 8 ? 16385u : (w < 15 ? 8193u : 4098u); }
__host__ __device__ __forceinline__ uint32_t zip_h(int w) { return w == 15 ? 2u : 1u; }
__host__ __device__ __forceinline__ uint32_t zip_level_items(int w, int level) {
  uint32_t n = zip_groups(w);
  for (int L = 0; L < level; L++) n = (n + 63) / 64;
  return n;
}
constexpr uint32_t kSortTileE = 4096;  // entries per sort tile (one wave, 64 rounds of 64)
constexpr uint32_t kSortWaves = 4;

// ---------------------------------------------------------------- prep (after verify_prep)
__device__ __forceinline__ void niels_row_store(int4 *row, const fe &x, const fe &y) {
  // -P for the affine point (x, y): (y - x, y + x, -2d x y), each carried
  ge_niels e;
  fe t, d2;
  fe_const_d2(d2);
  fe_sub(e.YpX, y, x);
  fe_carry(e.YpX, e.YpX);
  fe_add(e.YmX, y, x);
  fe_carry(e.YmX, e.YmX);
  fe_mul(t, x, y);
  fe_mul(t, t, d2);
  fe_neg(e.XY2d, t);
  const fe *fs[3] = {&e.YpX, &e.YmX, &e.XY2d};
#pragma unroll
  for (int q = 0; q < (int)kZipRow; q++) {
    int32_t w[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int f = 4 * q + c;
      w[c] = f < 30 ? fs[f / 10]->v[f % 10] : 0;
    }
    row[q] = make_int4(w[0], w[1], w[2], w[3]);
  }
}

// z_i: SHA-512(seed || LE64(index)) (one block), 126 bits with bit 125 set: non-zero, and the
// signed radix-2^16 recoding of z stays within 8 windows (with 127 bits the top halfword 0x7fff
// plus the recoding's bias and carry overflowed into a ninth window about once per 2^16 z).
__device__ __forceinline__ void zip_scalar_z(uint32_t z[8], const uint32_t seed[8], uint64_t index) {
  uint64_t w[16];
#pragma unroll
  for (int i = 0; i < 4; i++) {  // big-endian 64-bit words of the 32 seed bytes
    const uint32_t lo = seed[2 * i], hi = seed[2 * i + 1];
    w[i] = ((uint64_t)bswap32(lo) << 32) | bswap32(hi);
  }
  uint64_t ix = 0;
#pragma unroll
  for (int b = 0; b < 8; b++) ix |= ((index >> (8 * b)) & 0xffull) << (56 - 8 * b);
  w[4] = ix;
  w[5] = 0x80ull << 56;
#pragma unroll
  for (int i = 6; i < 15; i++) w[i] = 0;
  w[15] = 40 * 8;
  uint64_t st[8];
  sha512_init(st);
  sha512_compress(st, w);
  z[0] = (uint32_t)st[0];
  z[1] = (uint32_t)(st[0] >> 32);
  z[2] = (uint32_t)st[1];
  z[3] = ((uint32_t)(st[1] >> 32) & 0x1fffffffu) | 0x20000000u;
  z[4] = z[5] = z[6] = z[7] = 0;
}

// One lane per signature of the chunk (after verify_prep_kernel wrote k, S, A, ok).  Point rows:
// [0, cnt) = -A_i, [cnt, 2 cnt) = -R_i; digits dig[w][row] (int16, signed radix 2^16); cs = z S.
// Invalid signatures (A or R not on the curve, S >= L) get z = 0: no contribution, out[i] = 0.
#ifndef TMED_ZIP_PREP_WAVES
#define TMED_ZIP_PREP_WAVES 2
#endif
__global__ __launch_bounds__(kThreadsPerBlock, TMED_ZIP_PREP_WAVES) void zip_prep_r_kernel(
    const uint8_t *__restrict__ sig, uint32_t base, uint32_t cnt, const int4 *__restrict__ prep, uint32_t stride,
    const uint32_t *__restrict__ seed, uint64_t index_base, int4 *__restrict__ pts, int16_t *__restrict__ dig,
    int4 *__restrict__ cs, uint32_t cs_stride, uint8_t *__restrict__ out) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= cnt) return;
  int32_t w[40];
#pragma unroll
  for (int q = 0; q < 10; q++) {
    const int4 v = prep[(size_t)q * stride + slot];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
  uint32_t k[8], s[8], Rw[8], sd[8];
#pragma unroll
  for (int j = 0; j < 8; j++) { k[j] = (uint32_t)w[j]; s[j] = (uint32_t)w[8 + j]; sd[j] = seed[j]; }
  fe Ax, Ay;
#pragma unroll
  for (int j = 0; j < 10; j++) { Ax.v[j] = w[16 + j]; Ay.v[j] = w[26 + j]; }
  const bool ok = w[36] != 0;
  load_row_words(Rw, sig + 64 * (size_t)(base + slot), 2);
  ge_p3 R;
  const bool rok = ge_frombytes_go(R, Rw);  // permissive decode (ZIP-215)
  const bool valid = ok && rok;
  uint32_t z[8], a[8], c[8], zero[8];
  zip_scalar_z(z, sd, index_base + slot);
#pragma unroll
  for (int j = 0; j < 8; j++) { zero[j] = 0; if (!valid) z[j] = 0; }
  sc_muladd(a, z, k, zero);
  sc_muladd(c, z, s, zero);
  niels_row_store(pts + (size_t)slot * kZipRow, Ax, Ay);
  niels_row_store(pts + ((size_t)cnt + slot) * kZipRow, R.X, R.Y);
  uint32_t ar[8], zr[8];
  sc_recode_b<16>(ar, a);
  sc_recode_b<16>(zr, z);
  const size_t rows = 2 * (size_t)cnt;
#pragma unroll
  for (int wi = 0; wi < kZipWin; wi++) {
    const int da = (int)((ar[wi >> 1] >> (16 * (wi & 1))) & 0xffffu) - 32768;
    const int dz = wi < kZipZWin ? (int)((zr[wi >> 1] >> (16 * (wi & 1))) & 0xffffu) - 32768 : 0;
    dig[(size_t)wi * rows + slot] = (int16_t)da;  // digits are in [-32768, 32767]
    dig[(size_t)wi * rows + cnt + slot] = (int16_t)dz;
  }
  cs[slot] = make_int4((int)c[0], (int)c[1], (int)c[2], (int)c[3]);
  cs[(size_t)cs_stride + slot] = make_int4((int)c[4], (int)c[5], (int)c[6], (int)c[7]);
  out[base + slot] = valid ? 1 : 0;
}

// ---------------------------------------------------------------- sum z_i S_i mod L
// Column sums of the 32-bit words as u64 (a block of 256 values per partial, < 2^40 per column).
__global__ __launch_bounds__(256) void zip_bsum_kernel(const int4 *__restrict__ cs, uint32_t stride, uint32_t lo,
                                                       uint32_t hi, uint64_t *__restrict__ partial) {
  __shared__ uint64_t col[8][256];
  const uint32_t i = lo + blockIdx.x * 256 + threadIdx.x;
  uint32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (i < hi) {
    const int4 a = cs[i], b = cs[(size_t)stride + i];
    c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w; c[4] = b.x; c[5] = b.y; c[6] = b.z; c[7] = b.w;
  }
#pragma unroll
  for (int q = 0; q < 8; q++) col[q][threadIdx.x] = c[q];
  __syncthreads();
  for (uint32_t o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
#pragma unroll
      for (int q = 0; q < 8; q++) col[q][threadIdx.x] += col[q][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 8) partial[(size_t)blockIdx.x * 8 + threadIdx.x] = col[threadIdx.x][0];
}

// One block: the column sums of all partials (< 2^52), carried into 512 bits, reduced mod L.
__global__ __launch_bounds__(256) void zip_bsum_final_kernel(const uint64_t *__restrict__ partial, uint32_t np,
                                                             uint32_t *__restrict__ ctot) {
  __shared__ uint64_t col[8][256];
  uint64_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t p = threadIdx.x; p < np; p += 256)
#pragma unroll
    for (int q = 0; q < 8; q++) c[q] += partial[(size_t)p * 8 + q];
#pragma unroll
  for (int q = 0; q < 8; q++) col[q][threadIdx.x] = c[q];
  __syncthreads();
  for (uint32_t o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
#pragma unroll
      for (int q = 0; q < 8; q++) col[q][threadIdx.x] += col[q][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    uint32_t x[16];
    uint64_t carry = 0;
    for (int q = 0; q < 16; q++) {
      const uint64_t v = (q < 8 ? col[q][0] : 0ull) + carry;
      x[q] = (uint32_t)v;
      carry = v >> 32;
    }
    uint32_t r[8];
    sc_reduce512(r, x);
    for (int q = 0; q < 8; q++) ctot[q] = r[q];
  }
}

// ---------------------------------------------------------------- per-window stable sort
// Window w's entries: e in [0, M_w) with M_w = 2 cnt (w < 8: A and R rows) or cnt (A rows only);
// entry e <-> point row j(e) = lo + e (e < cnt) or N + lo + (e - cnt), N = the chunk's row offset
// of R.  Pass 0 keys on the low byte of |digit| (read from dig), pass 1 on the high byte.
struct ZipSortArgs {
  const int16_t *dig;
  uint32_t rows;   // 2N: the row stride of dig
  uint32_t N, lo, cnt;
  uint16_t *keys[2];
  uint32_t *vals[2];
  uint32_t cap;    // per-window capacity of keys / vals (2N)
  uint32_t *hist;  // [w][tile + 1][bin]: counts, then offsets (zip_sort_scan_kernel)
  uint32_t tiles;  // tiles of this sort (row stride of hist: tiles + 1)
};

__device__ __forceinline__ uint32_t zip_m(const ZipSortArgs &a, int w) { return (w < kZipZWin ? 2u : 1u) * a.cnt; }

template <int PASS>
__device__ __forceinline__ void zip_entry(const ZipSortArgs &a, int w, uint32_t e, uint32_t &key, uint32_t &val) {
  if (PASS == 0) {
    const uint32_t j = e < a.cnt ? a.lo + e : a.N + a.lo + (e - a.cnt);
    const int d = a.dig[(size_t)w * a.rows + j];
    key = (uint32_t)(d < 0 ? -d : d);
    val = j | (d < 0 ? 0x80000000u : 0u);
  } else {
    key = a.keys[0][(size_t)w * a.cap + e];
    val = a.vals[0][(size_t)w * a.cap + e];
  }
}

template <int PASS>
__global__ __launch_bounds__(kSortWaves * 64) void zip_sort_hist_kernel(ZipSortArgs a) {
  __shared__ uint32_t h[kSortWaves][256];
  const int w = blockIdx.y;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t tile = blockIdx.x * kSortWaves + wave;
  for (uint32_t b = lane; b < 256; b += 64) h[wave][b] = 0;
  const uint32_t M = zip_m(a, w), e0 = tile * kSortTileE;
  for (uint32_t r = 0; r < kSortTileE / 64; r++) {
    const uint32_t e = e0 + r * 64 + lane;
    if (e < M) {
      uint32_t key, val;
      zip_entry<PASS>(a, w, e, key, val);
      atomicAdd(&h[wave][PASS == 0 ? (key & 0xffu) : (key >> 8)], 1u);
    }
  }
  if (tile < a.tiles)
    for (uint32_t b = lane; b < 256; b += 64) a.hist[((size_t)w * (a.tiles + 1) + tile) * 256 + b] = h[wave][b];
}

// Per window: hist[w] is [tile][bin] (+ one row of bin starts).  Thread (seg, b) of the 1024 sums
// its quarter of column b (coalesced: consecutive threads, consecutive bins), the quarters and the
// bin totals are scanned in LDS, then the thread rewrites its quarter as exclusive prefixes; tile
// t's range of bin b starts at row[tiles][b] + [t][b].
__global__ __launch_bounds__(1024) void zip_sort_scan_kernel(uint32_t *__restrict__ hist, uint32_t tiles) {
  __shared__ uint32_t part[4][256], tot[256], colsum[256];
  uint32_t *h = hist + (size_t)blockIdx.x * (tiles + 1) * 256;
  const uint32_t b = threadIdx.x & 255u, seg = threadIdx.x >> 8;
  const uint32_t per = (tiles + 3) / 4, t0 = seg * per < tiles ? seg * per : tiles;
  const uint32_t t1 = t0 + per < tiles ? t0 + per : tiles;
  uint32_t acc = 0;
  for (uint32_t t = t0; t < t1; t++) acc += h[(size_t)t * 256 + b];
  part[seg][b] = acc;
  __syncthreads();
  if (seg == 0) {
    uint32_t run = 0;
    for (int q = 0; q < 4; q++) { const uint32_t c = part[q][b]; part[q][b] = run; run += c; }
    colsum[b] = run;
    tot[b] = run;
  }
  __syncthreads();
  for (uint32_t o = 1; o < 256; o <<= 1) {  // inclusive scan of the bin totals
    const uint32_t x = (seg == 0 && b >= o) ? tot[b - o] : 0u;
    __syncthreads();
    if (seg == 0) tot[b] += x;
    __syncthreads();
  }
  uint32_t run = part[seg][b];
  for (uint32_t t = t0; t < t1; t++) {
    const uint32_t c = h[(size_t)t * 256 + b];
    h[(size_t)t * 256 + b] = run;
    run += c;
  }
  if (seg == 0) h[(size_t)tiles * 256 + b] = tot[b] - colsum[b];  // exclusive bin start
}

// Stable scatter: ONE wave (one workgroup) per tile.  The tile is first ranked into LDS in bin
// order — rounds of 64 consecutive entries; lanes with equal bins are ranked in lane order by
// ballot matching on the 8 bin bits, the bin's running position lives in LDS (read by all lanes,
// then advanced by the group's last lane) — and then written out in that order, so consecutive
// lanes store consecutive addresses of a bin's run (a direct scatter touched 64 lines per store
// instruction and was store-transaction bound: 0.5 ms per pass per 2^20 signatures).
template <int PASS>
__global__ __launch_bounds__(64) void zip_sort_scatter_kernel(ZipSortArgs a) {
  __shared__ uint16_t sk[kSortTileE];
  __shared__ uint32_t sv[kSortTileE];
  __shared__ uint32_t lstart[256], gbase[256], run[256];
  const int w = blockIdx.y;
  const uint32_t lane = threadIdx.x, tile = blockIdx.x;
  const uint32_t M = zip_m(a, w), e0 = tile * kSortTileE;
  if (tile >= a.tiles || e0 >= M) return;
  const uint32_t nt = M - e0 < kSortTileE ? M - e0 : kSortTileE;
  for (uint32_t b = lane; b < 256; b += 64) run[b] = 0;
  for (uint32_t j = lane; j < nt; j += 64) {  // the tile's own counts
    uint32_t key, val;
    zip_entry<PASS>(a, w, e0 + j, key, val);
    atomicAdd(&run[PASS == 0 ? (key & 0xffu) : (key >> 8)], 1u);
  }
  __builtin_amdgcn_wave_barrier();
  {  // exclusive scan of the 256 counts: 4 per lane, then a wave scan of the lane sums
    uint32_t c[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) { c[q] = run[4 * lane + q]; sum += c[q]; }
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = (uint32_t)__shfl_up((int)inc, (unsigned)o);
      if (lane >= (uint32_t)o) inc += x;
    }
    uint32_t ex = inc - sum;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t b = 4 * lane + q;
      lstart[b] = ex;
      run[b] = ex;
      const uint32_t *hw = a.hist + (size_t)w * (a.tiles + 1) * 256;
      gbase[b] = hw[(size_t)a.tiles * 256 + b] + hw[(size_t)tile * 256 + b];
      ex += c[q];
    }
  }
  __builtin_amdgcn_wave_barrier();
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (uint32_t r = 0; r * 64 < nt; r++) {
    const uint32_t j = r * 64 + lane;
    const bool act = j < nt;
    uint32_t key = 0, val = 0;
    if (act) zip_entry<PASS>(a, w, e0 + j, key, val);
    const uint32_t bin = PASS == 0 ? (key & 0xffu) : (key >> 8);
    uint64_t m = __ballot(act);
#pragma unroll
    for (int bit = 0; bit < 8; bit++) {
      const uint64_t bs = __ballot((bin >> bit) & 1u);
      m &= ((bin >> bit) & 1u) ? bs : ~bs;
    }
    const uint32_t pos = act ? run[bin] + (uint32_t)__builtin_popcountll(m & below) : 0u;
    __builtin_amdgcn_wave_barrier();
    if (act && (m >> lane) == 1ull) run[bin] += (uint32_t)__builtin_popcountll(m);  // the group's last lane
    __builtin_amdgcn_wave_barrier();
    if (act) {
      sk[pos] = (uint16_t)key;
      sv[pos] = val;
    }
  }
  __builtin_amdgcn_wave_barrier();
  uint16_t *ko = a.keys[PASS] + (size_t)w * a.cap;
  uint32_t *vo = a.vals[PASS] + (size_t)w * a.cap;
  for (uint32_t j = lane; j < nt; j += 64) {
    const uint32_t key = sk[j];
    const uint32_t b = PASS == 0 ? (key & 0xffu) : (key >> 8);
    const uint32_t gp = gbase[b] + (j - lstart[b]);
    ko[gp] = (uint16_t)key;
    vo[gp] = sv[j];
  }
}

// ---------------------------------------------------------------- bucket accumulation
__device__ __forceinline__ uint32_t lower_bound16(const uint16_t *k, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (k[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void p3_store_rows(int4 *dst, size_t stride, const ge_p3 &p) {
  const fe *fs[4] = {&p.X, &p.Y, &p.Z, &p.T};
#pragma unroll
  for (int q = 0; q < 10; q++) {
    int32_t w[4];
#pragma unroll
    for (int c = 0; c < 4; c++) w[c] = fs[(4 * q + c) / 10]->v[(4 * q + c) % 10];
    dst[(size_t)q * stride] = make_int4(w[0], w[1], w[2], w[3]);
  }
}
__device__ __forceinline__ void p3_load_rows(ge_p3 &p, const int4 *src, size_t stride) {
  fe *fs[4] = {&p.X, &p.Y, &p.Z, &p.T};
#pragma unroll
  for (int q = 0; q < 10; q++) {
    const int4 v = src[(size_t)q * stride];
    const int32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int c = 0; c < 4; c++) fs[(4 * q + c) / 10]->v[(4 * q + c) % 10] = w[c];
  }
}

// Items of a window level: item i holds points (S_i, T_i) — or the 4 bucket sums of an
// accumulation lane — as p3 (10 int4 each), stored [point][q][w][i]-major with stride istride per
// window so a wave's loads coalesce.
struct ZipItems {
  int4 *p;
  uint32_t istride;  // items per window slot
  __device__ __forceinline__ int4 *at(int w, uint32_t i, int which) const {
    return p + ((size_t)which * 10 * kZipWin + (size_t)w) * istride + i;  // q stride = kZipWin * istride
  }
  __device__ __forceinline__ size_t qstride() const { return (size_t)kZipWin * istride; }
};

struct ZipRowPf {
  int4 pv[8];
  bool neg;
  __device__ __forceinline__ void fetch(const int4 *row, bool n) {
#pragma unroll
    for (int q = 0; q < 8; q++) pv[q] = row[q];
    neg = n;
  }
  __device__ __forceinline__ void take(ge_niels &e) const {
    fe *fs[3] = {&e.YpX, &e.YmX, &e.XY2d};
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int32_t w[4] = {pv[q].x, pv[q].y, pv[q].z, pv[q].w};
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int f = 4 * q + c;
        if (f < 30) fs[f / 10]->v[f % 10] = w[c];
      }
    }
    niels_apply_sign(e, neg);
  }
};

#ifndef TMED_ZIP_ACC_WAVES
#define TMED_ZIP_ACC_WAVES 2
#endif
// The bucket sums of a lane go to bsum ([point][q][w][lane] rows) as each is finished, so the
// accumulation loop keeps only the accumulator, the prefetched row and the next entry live; the
// weighted sums S = sum_q B_q, T = sum_q q B_q of the lane's g buckets are formed afterwards.
// Row i + 1 and entry i + 2 are loaded while addition i runs.
__global__ __launch_bounds__(256, TMED_ZIP_ACC_WAVES) void zip_accum_kernel(const uint16_t *__restrict__ keys,
                                                           const uint32_t *__restrict__ vals, uint32_t cap,
                                                           uint32_t cnt, const int4 *__restrict__ pts,
                                                           ZipItems bsum, ZipItems out) {
  const int w = blockIdx.y;
  const uint32_t h = zip_h(w), g = 1u << zip_glog(w), ng = zip_groups(w), lanes = ng * h;
  if (blockIdx.x * blockDim.x >= lanes) return;  // the whole block past this window's lanes
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t grp = t / h, part = t % h;
  const uint32_t M = (w < kZipZWin ? 2u : 1u) * cnt;
  const uint16_t *k = keys + (size_t)w * cap;
  const uint32_t *v = vals + (size_t)w * cap;
  const bool lane_ok = t < lanes;
  const uint32_t v0 = g * grp;
  // bucket boundaries: [b[q], b[q+1]) holds |digit| = v0 + q (v = 0 skipped: weight 0); kept in
  // LDS (indexed by the rolled bucket loop without register-array indexing)
  __shared__ uint32_t bnd[5][256];
#pragma unroll
  for (int q = 0; q < 5; q++) {
    const uint32_t key = v0 + (uint32_t)q;
    bnd[q][threadIdx.x] = (lane_ok && (uint32_t)q <= g) ? lower_bound16(k, M, key == 0 ? 1u : key) : 0u;
  }
  ge_p3 acc;
  ge_p1p1 t1;
  ge_niels e;
  ZipRowPf pf;
#pragma unroll 1
  for (uint32_t q = 0; q < g; q++) {
    uint32_t lo = bnd[q][threadIdx.x], hi = bnd[q + 1][threadIdx.x];
    if (h == 2) {  // the two lanes of a group take the halves of each bucket's run
      const uint32_t mid = lo + (hi - lo) / 2;
      if (part == 0) hi = mid; else lo = mid;
    }
    const uint32_t nq = lane_ok ? hi - lo : 0u;
    uint32_t mx = nq;  // wave-uniform trip count: the largest run of the wave
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t x = (uint32_t)__shfl_xor((int)mx, o);
      mx = x > mx ? x : mx;
    }
    mx = __builtin_amdgcn_readfirstlane(mx);
    ge_p3_0(acc);
    uint32_t vn = 0;
    if (nq) {
      const uint32_t vv = v[lo];
      pf.fetch(pts + (size_t)(vv & 0x7fffffffu) * kZipRow, (vv >> 31) != 0);
      if (nq > 1) vn = v[lo + 1];
    }
#pragma unroll 1
    for (uint32_t i = 0; i < mx; i++) {
      if (i < nq) {
        pf.take(e);
        if (i + 1 < nq) pf.fetch(pts + (size_t)(vn & 0x7fffffffu) * kZipRow, (vn >> 31) != 0);
        if (i + 2 < nq) vn = v[lo + i + 2];
        ge_madd_niels(t1, acc, e, false);
        ge_p1p1_to_p3(acc, t1);
      }
    }
    if (lane_ok) p3_store_rows(bsum.at(w, t, (int)q), bsum.qstride(), acc);
  }
}

// S = sum B_q, T = sum q B_q = B_{g-1} + (B_{g-1} + B_{g-2}) + ... (running sums from the top) of
// each accumulation lane's g bucket sums -> item t.  With h = 2 the level-0 reduction adds the two
// halves of a group (items 2 grp, 2 grp + 1) before weighting: S and T are linear in the buckets.
__global__ __launch_bounds__(256) void zip_bucket_weights_kernel(ZipItems bsum, ZipItems out) {
  const int w = blockIdx.y;
  const uint32_t g = 1u << zip_glog(w), lanes = zip_groups(w) * zip_h(w);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= lanes) return;
  ge_p3 run, tsum, bq;
  p3_load_rows(run, bsum.at(w, t, (int)g - 1), bsum.qstride());
  if (g > 1) tsum = run; else ge_p3_0(tsum);
#pragma unroll 1
  for (int q = (int)g - 2; q >= 0; q--) {
    p3_load_rows(bq, bsum.at(w, t, q), bsum.qstride());
    ge_p3_add(run, bq);
    if (q > 0) ge_p3_add(tsum, run);
  }
  p3_store_rows(out.at(w, t, 0), out.qstride(), run);
  p3_store_rows(out.at(w, t, 1), out.qstride(), tsum);
}

// ---------------------------------------------------------------- wavefront bucket reduction
__device__ __forceinline__ void shfl_p3(ge_p3 &o, const ge_p3 &p, int src, bool down, int delta) {
  const fe *fi[4] = {&p.X, &p.Y, &p.Z, &p.T};
  fe *fo[4] = {&o.X, &o.Y, &o.Z, &o.T};
#pragma unroll
  for (int f = 0; f < 4; f++)
#pragma unroll
    for (int j = 0; j < 10; j++)
      fo[f]->v[j] = down ? __shfl_down(fi[f]->v[j], (unsigned)delta) : __shfl(fi[f]->v[j], src);
}

// One wave per 64 consecutive items of a window at reduction level `level`: (S', T') =
// (sum S_r, [2^dlog2] sum_r r S_r + sum T_r), with dlog2 = log2 of the items' weight step (g of the
// window at level 0, x64 per level).  sum_r r S_r = sum_{r >= 1} Suf_r, Suf_r = sum_{q >= r} S_q
// (Kogge-Stone suffix scan).
// The wave's 64 items (S_r, T_r) (lane r) -> on lane 0: Sout = sum S_r, Tout = [2^dlog2] sum_r r S_r
// + sum T_r.
__device__ __forceinline__ void zip_wave_reduce(ge_p3 &S, ge_p3 &T, int dlog2, uint32_t r, ge_p3 &Sout,
                                                ge_p3 &Tout) {
  ge_p3 o;
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {  // suffix sums
    shfl_p3(o, S, 0, true, d);
    if (r + d < 64) ge_p3_add(S, o);
  }
  shfl_p3(Sout, S, 0, false, 0);  // Suf_0 = sum S
  if (r == 0) ge_p3_0(S);         // U = sum_{r >= 1} Suf_r
#pragma unroll 1
  for (int d = 32; d > 0; d >>= 1) {  // two trees: U and sum T
    shfl_p3(o, S, 0, true, d);
    if (r < (uint32_t)d) ge_p3_add(S, o);
    shfl_p3(o, T, 0, true, d);
    if (r < (uint32_t)d) ge_p3_add(T, o);
  }
  Tout = S;
  if (r == 0 && dlog2 > 0) {  // (level 0 of the top window: g = 1, no doubling)
    ge_p2 q;
    ge_p1p1 t;
    ge_p3_to_p2(q, S);
#pragma unroll 1
    for (int k = 0; k < dlog2; k++) {
      ge_p2_dbl(t, q);
      if (k + 1 < dlog2) ge_p1p1_to_p2(q, t);
    }
    ge_p1p1_to_p3(Tout, t);
  }
  if (r == 0) ge_p3_add(Tout, T);
}

// Level 0: one wave per 64 items of a window (the top window's items are the sums of its two
// accumulation lanes per group).
__global__ __launch_bounds__(64) void zip_reduce_kernel(ZipItems in, ZipItems out) {
  const int w = blockIdx.y;
  const uint32_t n_items = zip_level_items(w, 0);
  if (blockIdx.x * 64 >= n_items) return;
  const uint32_t r = threadIdx.x, i = blockIdx.x * 64 + r;
  ge_p3 S, T;
  if (i < n_items && zip_h(w) == 2) {  // the two accumulation lanes of group i
    ge_p3 o;
    p3_load_rows(S, in.at(w, 2 * i, 0), in.qstride());
    p3_load_rows(o, in.at(w, 2 * i + 1, 0), in.qstride());
    ge_p3_add(S, o);
    p3_load_rows(T, in.at(w, 2 * i, 1), in.qstride());
    p3_load_rows(o, in.at(w, 2 * i + 1, 1), in.qstride());
    ge_p3_add(T, o);
  } else if (i < n_items) {
    p3_load_rows(S, in.at(w, i, 0), in.qstride());
    p3_load_rows(T, in.at(w, i, 1), in.qstride());
  } else {
    ge_p3_0(S);
    ge_p3_0(T);
  }
  ge_p3 So, To;
  zip_wave_reduce(S, T, zip_glog(w), r, So, To);
  if (r != 0) return;
  p3_store_rows(out.at(w, blockIdx.x, 0), out.qstride(), So);
  p3_store_rows(out.at(w, blockIdx.x, 1), out.qstride(), To);
}

// Levels 1 and 2 in one workgroup per window: wave j reduces level-1 items 64 j .. 64 j + 63 into
// LDS, then wave 0 reduces those (<= 5) into the window's value.
constexpr int kZipL1Waves = 5;  // ceil(ceil(kZipItemsMax / 64) / 64)
__global__ __launch_bounds__(64 * kZipL1Waves) void zip_reduce12_kernel(ZipItems in, ZipItems out) {
  __shared__ int32_t lds[kZipL1Waves][2][40];
  const int w = blockIdx.y;
  const uint32_t wave = threadIdx.x >> 6, r = threadIdx.x & 63u;
  const uint32_t n1 = zip_level_items(w, 1), n2 = zip_level_items(w, 2);
  const uint32_t i = wave * 64 + r;
  ge_p3 S, T, So, To;
  if (i < n1) {
    p3_load_rows(S, in.at(w, i, 0), in.qstride());
    p3_load_rows(T, in.at(w, i, 1), in.qstride());
  } else {
    ge_p3_0(S);
    ge_p3_0(T);
  }
  if (wave < n2) {  // (uniform per wave)
    zip_wave_reduce(S, T, zip_glog(w) + 6, r, So, To);
    if (r == 0) {
      const fe *fs[4] = {&So.X, &So.Y, &So.Z, &So.T}, *ft[4] = {&To.X, &To.Y, &To.Z, &To.T};
      for (int f = 0; f < 40; f++) { lds[wave][0][f] = fs[f / 10]->v[f % 10]; lds[wave][1][f] = ft[f / 10]->v[f % 10]; }
    }
  }
  __syncthreads();
  if (wave != 0) return;
  if (r < n2) {
    fe *fs[4] = {&S.X, &S.Y, &S.Z, &S.T}, *ft[4] = {&T.X, &T.Y, &T.Z, &T.T};
    for (int f = 0; f < 40; f++) { fs[f / 10]->v[f % 10] = lds[r][0][f]; ft[f / 10]->v[f % 10] = lds[r][1][f]; }
  } else {
    ge_p3_0(S);
    ge_p3_0(T);
  }
  zip_wave_reduce(S, T, zip_glog(w) + 12, r, So, To);
  if (r != 0) return;
  p3_store_rows(out.at(w, 0, 0), out.qstride(), So);
  p3_store_rows(out.at(w, 0, 1), out.qstride(), To);
}

// ---------------------------------------------------------------- final check
// total = sum_w 2^(16 w) W_w + [ctot] B; flag = ([8] total == O).  The 240 doublings of the Horner
// chain are serial, so ONE quad runs it with the 4-way split formulas (quad.h): each lane computes
// one coordinate's products of every doubling / addition (~3x less latency than one lane).
__global__ __launch_bounds__(64) void zip_final_kernel(ZipItems wins, const uint32_t *__restrict__ ctot,
                                                       const int4 *__restrict__ bcomb16, uint32_t *__restrict__ flag) {
  if (threadIdx.x >= 4) return;  // quad 0
  const QuadK K(threadIdx.x);
  auto coord = [&](int w, fe &c) {  // lane r: coordinate r (X, Y, Z, T) of W_w
    const int4 *src = wins.at(w, 0, 1);
    int32_t a[40];
#pragma unroll
    for (int q = 0; q < 10; q++) {
      const int4 x = src[(size_t)q * wins.qstride()];
      a[4 * q] = x.x; a[4 * q + 1] = x.y; a[4 * q + 2] = x.z; a[4 * q + 3] = x.w;
    }
#pragma unroll
    for (int j = 0; j < 10; j++) c.v[j] = a[10 * K.r + j];
  };
  fe v, wv, c;
  coord(kZipWin - 1, v);
#pragma unroll 1
  for (int w = kZipWin - 2; w >= 0; w--) {
#pragma unroll 1
    for (int d = 0; d < 16; d++) quad_dbl(v, K);
    coord(w, wv);
    quad_to_cached(c, wv, K);
    quad_add(v, c, K);
  }
  uint32_t cw[8], cr[8];
#pragma unroll
  for (int j = 0; j < 8; j++) cw[j] = ctot[j];
  sc_recode_b<16>(cr, cw);
#pragma unroll 1
  for (int w = 0; w < 16; w++) {
    const int d = (int)((cr[w >> 1] >> (16 * (w & 1))) & 0xffffu) - 32768;
    comb_take(c, bcomb16 + (size_t)w * kB16Entries * kCombEntryInt4, d, K);
    quad_add(v, c, K);
  }
#pragma unroll 1
  for (int d = 0; d < 3; d++) quad_dbl(v, K);  // [8]
  fe X, Y, Z;
#pragma unroll
  for (int j = 0; j < 10; j++) { X.v[j] = qbcast(v.v[j], 0); Y.v[j] = qbcast(v.v[j], 1); Z.v[j] = qbcast(v.v[j], 2); }
  if (threadIdx.x == 0) flag[0] = (fe_iszero(X) && fe_equal(Y, Z) && !fe_iszero(Z)) ? 1u : 0u;
}

// Failed verdicts (zero bytes) among n: 16 per lane, a wave sum, one atomic per wave (~1 MB per
// chunk, a few microseconds); the count steers the next chunk (zip215_verify_device).
__global__ __launch_bounds__(256) void zip_count_fail_kernel(const uint8_t *__restrict__ out, uint32_t n,
                                                             uint32_t *__restrict__ cnt) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x, i0 = 16 * t;
  uint32_t c = 0;
  if (i0 + 16 <= n && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
    const uint4 v = reinterpret_cast<const uint4 *>(out)[t];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 16; k++) c += ((w[k >> 2] >> (8 * (k & 3))) & 0xffu) == 0;
  } else {
    for (uint32_t i = i0; i < n && i < i0 + 16; i++) c += out[i] == 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, (unsigned)o);
  if ((threadIdx.x & 63u) == 0 && c) atomicAdd(cnt, c);
}

}  // namespace tmed

// ================================================================ host orchestration
using namespace tmed;

namespace {

struct ZipBufs {
  int4 *pts;
  int16_t *dig;
  int4 *cs;
  uint16_t *keys[2];
  uint32_t *vals[2];
  uint32_t *hist;
  uint64_t *partial;
  uint32_t *ctot;
  int4 *items[4];
  int4 *bsum;          // accumulation lanes' four bucket sums
  uint32_t *flag;      // device
  uint32_t *seed;      // device, 8 words
  uint32_t cap, tiles;
};

uint32_t zip_tiles(uint32_t cap) { return (cap + kSortTileE - 1) / kSortTileE; }

// Lay the chunk's scratch out in one device buffer (kZipMax signatures).
hipError_t zip_bufs(tmed_ctx *c, ZipBufs &z) {
  const size_t N = kZipMax, rows = 2 * N, cap = rows;
  const uint32_t tiles = zip_tiles((uint32_t)cap);
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
  const size_t o_pts = take(rows * kZipRow * 16), o_dig = take((size_t)kZipWin * rows * 2), o_cs = take(N * 32);
  size_t o_k[2], o_v[2];
  for (int p = 0; p < 2; p++) { o_k[p] = take((size_t)kZipWin * cap * 2); o_v[p] = take((size_t)kZipWin * cap * 4); }
  const size_t o_hist = take((size_t)kZipWin * 256 * (tiles + 1) * 4), o_part = take((N / 256 + 1) * 8 * 8);
  const size_t o_ctot = take(64);
  size_t o_it[4];
  uint32_t n_it[4] = {kZipItemsMax, (kZipItemsMax + 63) / 64, ((kZipItemsMax + 63) / 64 + 63) / 64, 1};
  for (int L = 0; L < 4; L++) o_it[L] = take((size_t)20 * kZipWin * n_it[L] * 16);
  const size_t o_bsum = take((size_t)40 * kZipWin * kZipItemsMax * 16);
  const size_t o_flag = take(16), o_seed = take(32);
  hipError_t e = c->d_zip.ensure(off);
  if (e != hipSuccess) return e;
  char *b = (char *)c->d_zip.p;
  z.pts = (int4 *)(b + o_pts);
  z.dig = (int16_t *)(b + o_dig);
  z.cs = (int4 *)(b + o_cs);
  for (int p = 0; p < 2; p++) { z.keys[p] = (uint16_t *)(b + o_k[p]); z.vals[p] = (uint32_t *)(b + o_v[p]); }
  z.hist = (uint32_t *)(b + o_hist);
  z.partial = (uint64_t *)(b + o_part);
  z.ctot = (uint32_t *)(b + o_ctot);
  for (int L = 0; L < 4; L++) z.items[L] = (int4 *)(b + o_it[L]);
  z.bsum = (int4 *)(b + o_bsum);
  z.flag = (uint32_t *)(b + o_flag);
  z.seed = (uint32_t *)(b + o_seed);
  z.cap = (uint32_t)cap;
  z.tiles = tiles;
  return hipSuccess;
}

// The batch equation over signatures [lo, lo + cnt) of the prepared chunk (rows at N).
hipError_t zip_msm(tmed_ctx *c, const ZipBufs &z, uint32_t N, uint32_t lo, uint32_t cnt, hipStream_t s) {
  const uint32_t np = (cnt + 255) / 256;
  hipLaunchKernelGGL(zip_bsum_kernel, dim3(np), dim3(256), 0, s, z.cs, kZipMax, lo, lo + cnt, z.partial);
  hipLaunchKernelGGL(zip_bsum_final_kernel, dim3(1), dim3(256), 0, s, z.partial, np, z.ctot);
  ZipSortArgs a;
  a.dig = z.dig;
  a.rows = 2 * N;
  a.N = N;
  a.lo = lo;
  a.cnt = cnt;
  a.keys[0] = z.keys[0]; a.keys[1] = z.keys[1];
  a.vals[0] = z.vals[0]; a.vals[1] = z.vals[1];
  a.cap = z.cap;
  a.hist = z.hist;
  a.tiles = zip_tiles(2 * cnt);
  const dim3 sg((a.tiles + kSortWaves - 1) / kSortWaves, kZipWin);
  hipLaunchKernelGGL(zip_sort_hist_kernel<0>, sg, dim3(kSortWaves * 64), 0, s, a);
  hipLaunchKernelGGL(zip_sort_scan_kernel, dim3(kZipWin), dim3(1024), 0, s, a.hist, a.tiles);
  const dim3 sc(a.tiles, kZipWin);
  hipLaunchKernelGGL(zip_sort_scatter_kernel<0>, sc, dim3(64), 0, s, a);
  hipLaunchKernelGGL(zip_sort_hist_kernel<1>, sg, dim3(kSortWaves * 64), 0, s, a);
  hipLaunchKernelGGL(zip_sort_scan_kernel, dim3(kZipWin), dim3(1024), 0, s, a.hist, a.tiles);
  hipLaunchKernelGGL(zip_sort_scatter_kernel<1>, sc, dim3(64), 0, s, a);
  uint32_t n_it[4] = {kZipItemsMax, (kZipItemsMax + 63) / 64, ((kZipItemsMax + 63) / 64 + 63) / 64, 1};
  ZipItems it[4];
  for (int L = 0; L < 4; L++) it[L] = ZipItems{z.items[L], n_it[L]};
  hipLaunchKernelGGL(zip_accum_kernel, dim3((kZipItemsMax + 255) / 256, kZipWin), dim3(256), 0, s, z.keys[1],
                     z.vals[1], z.cap, cnt, z.pts, ZipItems{z.bsum, kZipItemsMax}, it[0]);
  hipLaunchKernelGGL(zip_bucket_weights_kernel, dim3((kZipItemsMax + 255) / 256, kZipWin), dim3(256), 0, s,
                     ZipItems{z.bsum, kZipItemsMax}, it[0]);
  hipLaunchKernelGGL(zip_reduce_kernel, dim3((n_it[0] + 63) / 64, kZipWin), dim3(64), 0, s, it[0], it[1]);
  hipLaunchKernelGGL(zip_reduce12_kernel, dim3(1, kZipWin), dim3(64 * kZipL1Waves), 0, s, it[1], it[3]);
  hipLaunchKernelGGL(zip_final_kernel, dim3(1), dim3(64), 0, s, it[3], z.ctot, c->d_bcomb16, z.flag);
  return hipGetLastError();
}

int zip_read_flag(tmed_ctx *c, const ZipBufs &z, hipStream_t s, bool *ok) {
  uint32_t h = 0;
  hipError_t e = hipMemcpyAsync(&h, z.flag, 4, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  *ok = h == 1;
  return map_err(e);
}

}  // namespace

namespace tmed {

// Per-call state of tmed_zip215_set_seed (tests): a fixed seed instead of getrandom().
static thread_local bool g_zip_fixed = false;
static thread_local uint8_t g_zip_seed[32];
static thread_local uint32_t g_zip_stats[4];  // chunks, equations run, groups decided singly, signatures decided singly

// ZIP-215 verification of n device-resident tuples (generic keys).  The caller holds ctx->mu and
// has acquired the scratch on stream s.
int zip215_verify_device(tmed_ctx *c, const uint8_t *pub, const uint8_t *sig, const uint8_t *msgs, const uint32_t *off,
                         uint32_t n, uint8_t *out, hipStream_t s, bool msg_slots) {
  ZipBufs z;
  hipError_t e = zip_bufs(c, z);
  if (e != hipSuccess) return map_err(e);
  memset(g_zip_stats, 0, sizeof g_zip_stats);
  const uint32_t chunk = std::min<uint32_t>(kZipMax, c->slab_slots);  // the prep hand-off holds slab_slots
  for (uint32_t base = 0; base < n; base += chunk) {
    const uint32_t N = n - base < chunk ? n - base : chunk;
    uint8_t seed[32];
    if (g_zip_fixed) memcpy(seed, g_zip_seed, 32);
    else if (getrandom(seed, 32, 0) != 32) return TMED_EHIP;
    e = hipMemcpyAsync(z.seed, seed, 32, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return map_err(e);
    g_zip_stats[0]++;
    // Failure cut-off: a chunk of at least kZipSinglyMin signatures whose predecessor had failures
    // is decided signature by signature first, with no MSM: with even one invalid signature the
    // equation, its halves and the bisection down to kZipMinGroup cost more than the single checks
    // (2^20 signatures, one invalid: 13 equations, 24.5 ms; singly 10.3 ms; tools/zip_sparse.py,
    // profiles/r04/s19).  The failures of such a chunk are counted on the
    // device (zip_count_fail_kernel) and read when the next chunk starts: a chunk without any puts
    // the next one back on the batch equation.  The decision of every signature is the
    // single-check one either way.
    constexpr uint32_t kZipSinglyMin = 1u << 14;
    if (N >= kZipSinglyMin && c->zip_count_pending) {
      e = hipEventSynchronize(c->zip_ev);
      if (e != hipSuccess) return map_err(e);
      c->zip_count_pending = false;
      c->zip_dense = *static_cast<const uint32_t *>(c->h_zip.p) != 0;
    }
    if (c->zip_dense && N >= kZipSinglyMin) {
      g_zip_stats[2]++;
      g_zip_stats[3] += N;
      const uint8_t *gm = msg_slots ? msgs + (size_t)base * kVoteSlot : msgs;
      e = launch_verify(pub + 32 * (size_t)base, sig + 64 * (size_t)base, gm, off + base, N, out + base, c->d_slab,
                        c->slab_slots, BTabs{c->d_b16, c->d_bcomb16, c->d_b26}, c->d_prep, c->d_fin, c->d_fin_pre, s,
                        c->chunk, 6, msg_slots, nullptr, /*zip215=*/true);
      if (e == hipSuccess && !c->zip_ev) e = hipEventCreateWithFlags(&c->zip_ev, hipEventDisableTiming);
      if (e == hipSuccess) e = c->h_zip.ensure(4);
      if (e == hipSuccess) e = hipMemsetAsync(z.flag, 0, 4, s);
      if (e == hipSuccess)
        hipLaunchKernelGGL(zip_count_fail_kernel, dim3((N + 4095) / 4096), dim3(256), 0, s, out + base, N, z.flag);
      if (e == hipSuccess) e = hipGetLastError();
      if (e == hipSuccess) e = hipMemcpyAsync(c->h_zip.p, z.flag, 4, hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipEventRecord(c->zip_ev, s);
      if (e != hipSuccess) return map_err(e);
      c->zip_count_pending = true;
      continue;
    }
    // k, S checks, decode of A (the generic throughput path's prep), then the ZIP-215 prep
    const uint32_t blocks = (N + kThreadsPerBlock - 1) / kThreadsPerBlock;
    e = launch_verify_prep(pub, sig, msgs, off, msg_slots, base, N, c->d_prep, c->slab_slots, s);
    if (e != hipSuccess) return map_err(e);
    hipLaunchKernelGGL(zip_prep_r_kernel, dim3(blocks), dim3(kThreadsPerBlock), 0, s, sig, base, N, c->d_prep,
                       c->slab_slots, z.seed, (uint64_t)base, z.pts, z.dig, z.cs, kZipMax, out);
    // Groups [lo, lo + cnt) of the chunk: one equation each.  A failing group is split in halves
    // while the failures look sparse (at most half of a level's groups fail) and halves stay
    // >= kZipMinGroup; the remaining failing groups are decided signature by signature.
    constexpr uint32_t kZipMinGroup = 1u << 14;
    std::vector<std::pair<uint32_t, uint32_t>> level{{0u, N}}, single;
    while (!level.empty()) {
      std::vector<std::pair<uint32_t, uint32_t>> failed;
      for (auto &g : level) {
        e = zip_msm(c, z, N, g.first, g.second, s);
        if (e != hipSuccess) return map_err(e);
        bool ok = false;
        int rc = zip_read_flag(c, z, s, &ok);
        if (rc != TMED_OK) return rc;
        g_zip_stats[1]++;
        if (!ok) failed.push_back(g);
      }
      const bool dense = level.size() >= 2 && failed.size() * 2 > level.size();
      std::vector<std::pair<uint32_t, uint32_t>> next;
      for (auto &g : failed) {
        if (!dense && g.second >= 2 * kZipMinGroup) {
          const uint32_t h = g.second / 2;
          next.push_back({g.first, h});
          next.push_back({g.first + h, g.second - h});
        } else {
          single.push_back(g);
        }
      }
      level.swap(next);
    }
    if (N >= kZipSinglyMin) c->zip_dense = !single.empty();  // a failing group always ends in `single`
    for (auto &g : single) {  // the exact ZIP-215 single check on the group's signatures
      g_zip_stats[2]++;
      g_zip_stats[3] += g.second;
      const uint32_t lo = base + g.first;
      const uint8_t *gm = msg_slots ? msgs + (size_t)lo * kVoteSlot : msgs;
      e = launch_verify(pub + 32 * (size_t)lo, sig + 64 * (size_t)lo, gm, off + lo, g.second, out + lo, c->d_slab,
                        c->slab_slots, BTabs{c->d_b16, c->d_bcomb16, c->d_b26}, c->d_prep, c->d_fin, c->d_fin_pre, s, c->chunk,
                        6, msg_slots, nullptr, /*zip215=*/true);
      if (e != hipSuccess) return map_err(e);
    }
  }
  c->last_hs_count = 0;
  return TMED_OK;
}

}  // namespace tmed

extern "C" {

int tmed_zip215_set_seed(const uint8_t *seed32) {
  // Predictable weights let a forger cancel errors across a batch: only a process that declares
  // itself a test (TMED_ZIP215_TEST_SEED=1 in its environment) may fix them.
  const char *t = getenv("TMED_ZIP215_TEST_SEED");
  if (seed32 && !(t && t[0] == '1')) return TMED_EINVAL;
  if (seed32) {
    memcpy(g_zip_seed, seed32, 32);
    g_zip_fixed = true;
  } else {
    g_zip_fixed = false;
  }
  return TMED_OK;
}

int tmed_zip215_stats(uint32_t out[4]) {
  if (!out) return TMED_EINVAL;
  memcpy(out, g_zip_stats, sizeof g_zip_stats);
  return TMED_OK;
}

int tmed_verify_batch_zip215_device(tmed_ctx *c, const uint8_t *d_pub, const uint8_t *d_sig, const uint8_t *d_msgs,
                                    const uint32_t *d_off, size_t n, uint8_t *d_out, void *stream) {
  if (!c) return TMED_EINVAL;
  if (n == 0) return TMED_OK;
  if (!d_pub || !d_sig || !d_msgs || !d_off || !d_out || n > 0xffffffffu) return TMED_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  std::lock_guard<std::mutex> lk(c->mu);
  (void)hipSetDevice(c->device);
  hipError_t e = scratch_acquire(c, s);
  if (e != hipSuccess) return map_err(e);
  int rc = zip215_verify_device(c, d_pub, d_sig, d_msgs, d_off, (uint32_t)n, d_out, s, false);
  e = scratch_release(c, s);
  return rc != TMED_OK ? rc : map_err(e);
}

int tmed_verify_batch_zip215(tmed_ctx *c, const uint8_t *pubkeys, const uint8_t *sigs, const uint32_t *sig_lens,
                             const uint8_t *msgs, const uint32_t *msg_off, size_t n, uint8_t *out) {
  if (!c || !out) return TMED_EINVAL;
  if (n == 0) return TMED_OK;
  if (!pubkeys || !sigs || !msg_off || n > 0xffffffffu) return TMED_EINVAL;
  for (size_t i = 0; i < n; i++)
    if (msg_off[i + 1] < msg_off[i]) return TMED_EINVAL;
  const size_t mbytes = msg_off[n];
  if (mbytes && !msgs) return TMED_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  (void)hipSetDevice(c->device);
  hipError_t e = hipSuccess;
  const size_t moff = (n + 1) * 4;
  for (auto &pr : {std::make_pair(&c->d_a, n * 32), std::make_pair(&c->d_b, n * 64),
                   std::make_pair(&c->d_msg, mbytes + 16), std::make_pair(&c->d_off, moff),
                   std::make_pair(&c->d_out, n)})
    if (e == hipSuccess) e = pr.first->ensure(pr.second);
  if (e != hipSuccess) return map_err(e);
  hipStream_t s = c->stream;
  e = hipMemcpyAsync(c->d_a.p, pubkeys, n * 32, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->d_b.p, sigs, n * 64, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && mbytes) e = hipMemcpyAsync(c->d_msg.p, msgs, mbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->d_off.p, msg_off, moff, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = scratch_acquire(c, s);
  if (e != hipSuccess) return map_err(e);
  int rc = zip215_verify_device(c, (const uint8_t *)c->d_a.p, (const uint8_t *)c->d_b.p, (const uint8_t *)c->d_msg.p,
                                (const uint32_t *)c->d_off.p, (uint32_t)n, (uint8_t *)c->d_out.p, s, false);
  if (rc != TMED_OK) return rc;
  e = scratch_release(c, s);
  if (e == hipSuccess) e = hipMemcpyAsync(out, c->d_out.p, n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return map_err(e);
  if (sig_lens)
    for (size_t i = 0; i < n; i++)
      if (sig_lens[i] != 64) out[i] = 0;  // crypto/ed25519/ed25519.go:150-152
  return TMED_OK;
}

}  // extern "C"
