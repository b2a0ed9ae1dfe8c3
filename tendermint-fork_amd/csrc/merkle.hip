// merkle.hip — batched RFC-6962 Merkle roots on gfx950.
//
// Reference (all Go, restated here; oracle/merkle.py is the checker):
//   crypto/merkle/tree.go:9-22   HashFromByteSlices: 0 items -> emptyHash, 1 -> leafHash,
//                                else split at the largest power of two < n, recurse
//   crypto/merkle/hash.go:19-27  leafHash = SHA-256(0x00||x), innerHash = SHA-256(0x01||l||r)
//   types/validator_set.go:347-353  ValidatorSet.Hash = HashFromByteSlices(val.Bytes() ...)
//   types/validator.go:117-133      Validator.Bytes = SimpleValidator{PubKey, VotingPower} proto
//   types/block.go:440-475          Header.Hash = HashFromByteSlices(14 encoded fields)
//   types/part_set.go:166-194       PartSet root = ProofsFromByteSlices(part_size chunks) root
// Callers: light/verifier.go:183 (untrustedVals.Hash() per header), :237 (Header.Hash),
// blockchain/v0/reactor.go:359-361 (MakePartSet + first.Hash() per block).
//
// Device shape: one lane per leaf (SHA-256 of 0x00 || leaf), then one launch per tree level
// over ALL trees of the call (one lane per output node).  The split-point recursion of
// tree.go equals pairing adjacent nodes level by level and promoting an odd last node
// (HashFromByteSlicesIterative, tree.go:57-101, is asserted equal by tree_test.go:104-116),
// which is what the level kernel does.  Work per inner node: 2 SHA-256 blocks.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/tmed25519.h"
#include "ctx.h"
#include "sha256.h"

namespace tmed {

struct Digest { uint32_t w[8]; };

__device__ __forceinline__ void store_digest(Digest *d, const uint32_t st[8]) {
  uint4 *p = reinterpret_cast<uint4 *>(d);
  p[0] = make_uint4(st[0], st[1], st[2], st[3]);
  p[1] = make_uint4(st[4], st[5], st[6], st[7]);
}
__device__ __forceinline__ void load_digest(uint32_t st[8], const Digest *d) {
  const uint4 *p = reinterpret_cast<const uint4 *>(d);
  const uint4 a = p[0], b = p[1];
  st[0] = a.x; st[1] = a.y; st[2] = a.z; st[3] = a.w;
  st[4] = b.x; st[5] = b.y; st[6] = b.z; st[7] = b.w;
}

// leafHash of every leaf: leaf i = leaves[off[i] .. off[i+1]).
__global__ __launch_bounds__(256) void merkle_leaf_kernel(const uint8_t *__restrict__ leaves,
                                                          const uint64_t *__restrict__ off, uint32_t n,
                                                          Digest *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t o0 = off[i], o1 = off[i + 1];
  uint32_t st[8];
  sha256_prefixed(st, 1, 0x00, leaves + o0, (uint32_t)(o1 - o0));
  store_digest(out + i, st);
}

// leafHash(Validator.Bytes()) for ed25519 validators: the SimpleValidator encoding
//   0a 22 | 0a 20 <pubkey 32> | [10 varint(power) if power != 0]
// (types/validator.go:117-133; PublicKey oneof ed25519 = field 1) is built in registers:
// 1 + 36 + <= 11 bytes always fits one SHA-256 block.
__global__ __launch_bounds__(256) void valset_leaf_kernel(const uint8_t *__restrict__ pubkeys,
                                                          const int64_t *__restrict__ powers, uint32_t n,
                                                          Digest *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t b[64];
#pragma unroll
  for (int k = 0; k < 64; k++) b[k] = 0;
  b[0] = 0x00;  // leaf prefix
  b[1] = 0x0a; b[2] = 0x22; b[3] = 0x0a; b[4] = 0x20;
  const uint4 *pk = reinterpret_cast<const uint4 *>(pubkeys + 32 * (size_t)i);
  const uint4 p0 = pk[0], p1 = pk[1];
  const uint32_t pw[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
  for (int k = 0; k < 32; k++) b[5 + k] = (uint8_t)(pw[k >> 2] >> (8 * (k & 3)));
  uint32_t len = 37;
  uint64_t v = (uint64_t)powers[i];
  if (v != 0) {
    b[len++] = 0x10;
#pragma unroll
    for (int k = 0; k < 10; k++) {
      b[len++] = (uint8_t)((v & 0x7f) | (v >= 0x80 ? 0x80 : 0));
      v >>= 7;
      if (v == 0) break;
    }
  }
  b[len] = 0x80;
  uint32_t w[16];
#pragma unroll
  for (int t = 0; t < 14; t++)
    w[t] = ((uint32_t)b[4 * t] << 24) | ((uint32_t)b[4 * t + 1] << 16) | ((uint32_t)b[4 * t + 2] << 8) | b[4 * t + 3];
  w[14] = 0;
  w[15] = len * 8;
  uint32_t st[8];
  sha256_init(st);
  sha256_compress(st, w);
  store_digest(out + i, st);
}

// One tree level for every tree: tree t has c_t = in_base[t+1] - in_base[t] nodes at
// in[in_base[t] ..); output node k of tree t (k < ceil(c_t / 2)) goes to out[out_base[t] + k].
__global__ __launch_bounds__(256) void merkle_level_kernel(const Digest *__restrict__ in,
                                                           const uint32_t *__restrict__ in_base,
                                                           const uint32_t *__restrict__ out_base, uint32_t ntrees,
                                                           uint32_t nout, Digest *__restrict__ out) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nout) return;
  uint32_t lo = 0, hi = ntrees;  // last t with out_base[t] <= j (trees with no output are skipped)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (out_base[mid] <= j) lo = mid; else hi = mid;
  }
  const uint32_t t = lo;
  const uint32_t k = j - out_base[t];
  const uint32_t c = in_base[t + 1] - in_base[t];
  const uint32_t src = in_base[t] + 2 * k;
  uint32_t l[8];
  load_digest(l, in + src);
  if (2 * k + 1 < c) {
    uint32_t r[8], st[8];
    load_digest(r, in + src + 1);
    sha256_inner(st, l, r);
    store_digest(out + j, st);
  } else {
    store_digest(out + j, l);  // odd node promoted
  }
}

// roots[t] = digest bytes of tree t's single node, or emptyHash for an empty tree.
__global__ __launch_bounds__(256) void merkle_emit_kernel(const Digest *__restrict__ in,
                                                          const uint32_t *__restrict__ base, uint32_t ntrees,
                                                          uint8_t *__restrict__ roots) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntrees) return;
  uint32_t st[8];
  if (base[t + 1] == base[t]) sha256_prefixed(st, 0, 0, nullptr, 0);  // emptyHash
  else load_digest(st, in + base[t]);
  uint32_t *o = reinterpret_cast<uint32_t *>(roots + 32 * (size_t)t);
#pragma unroll
  for (int k = 0; k < 8; k++) o[k] = bswap32(st[k]);
}

static uint32_t blocks_for(size_t n) { return (uint32_t)((n + 255) / 256); }

// Reduce per-tree leaf digests (c->d_merkle_a: counts[t] nodes per tree, tree-contiguous)
// to roots (d_roots, 32 B each).  Host-side level bookkeeping (O(trees) per level); all
// hashing on the device.  Caller holds ctx->mu.
static int reduce_trees(tmed_ctx *c, std::vector<uint32_t> counts, size_t total_leaves, uint8_t *d_roots,
                        hipStream_t s) {
  const size_t T = counts.size();
  if (total_leaves > 0xffffffffu) return TMED_EINVAL;
  Digest *cur = (Digest *)c->d_merkle_a.p;
  hipError_t e = c->d_merkle_b.ensure(std::max<size_t>(total_leaves, 1) * sizeof(Digest));
  if (e != hipSuccess) return map_err(e);
  Digest *nxt = (Digest *)c->d_merkle_b.p;
  std::vector<uint32_t> in_base(T + 1), out_base(T + 1);
  e = c->d_merkle_idx.ensure((2 * T + 2) * sizeof(uint32_t));
  if (e != hipSuccess) return map_err(e);
  uint32_t *d_in = (uint32_t *)c->d_merkle_idx.p, *d_out = d_in + T + 1;
  for (;;) {
    in_base[0] = out_base[0] = 0;
    bool more = false;
    for (size_t t = 0; t < T; t++) {
      in_base[t + 1] = in_base[t] + counts[t];
      if (counts[t] > 1) more = true;
      counts[t] = (counts[t] + 1) / 2;  // 0 -> 0, 1 -> 1
      out_base[t + 1] = out_base[t] + counts[t];
    }
    if (!more) break;
    e = hipMemcpyAsync(d_in, in_base.data(), (T + 1) * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_out, out_base.data(), (T + 1) * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
      const uint32_t nout = out_base[T];
      hipLaunchKernelGGL(merkle_level_kernel, dim3(blocks_for(nout)), dim3(256), 0, s, cur, d_in, d_out,
                         (uint32_t)T, nout, nxt);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // the host index vectors are rewritten next level
    if (e != hipSuccess) return map_err(e);
    std::swap(cur, nxt);
  }
  e = hipMemcpyAsync(d_in, in_base.data(), (T + 1) * 4, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(merkle_emit_kernel, dim3(blocks_for(T)), dim3(256), 0, s, cur, d_in, (uint32_t)T, d_roots);
    e = hipGetLastError();
  }
  return map_err(e);
}

}  // namespace tmed

using namespace tmed;

namespace {

// gogoproto varint / field helpers for the header leaves (types/block.go:440-475)
void put_varint(std::vector<uint8_t> &o, uint64_t v) {
  while (v >= 0x80) { o.push_back((uint8_t)(v | 0x80)); v >>= 7; }
  o.push_back((uint8_t)v);
}
void put_bytes_field(std::vector<uint8_t> &o, uint8_t tag, const uint8_t *p, size_t n) {
  o.push_back(tag);
  put_varint(o, n);
  o.insert(o.end(), p, p + n);
}

// The 14 leaves of Header.Hash, appended to `leaves` with their offsets.
void header_leaves(const tmed_header &h, std::vector<uint8_t> &leaves, std::vector<uint64_t> &off) {
  std::vector<uint8_t> f;
  auto push = [&]() { leaves.insert(leaves.end(), f.begin(), f.end()); off.push_back(leaves.size()); f.clear(); };
  // 1. Version (tendermint.version.Consensus): block = 1, app = 2, zero fields omitted
  if (h.version_block) { f.push_back(0x08); put_varint(f, h.version_block); }
  if (h.version_app) { f.push_back(0x10); put_varint(f, h.version_app); }
  push();
  // 2. cdcEncode(ChainID): gogotypes.StringValue{1: value}
  if (h.chain_id_len) put_bytes_field(f, 0x0a, (const uint8_t *)h.chain_id, h.chain_id_len);
  push();
  // 3. cdcEncode(Height): gogotypes.Int64Value{1: value}
  if (h.height) { f.push_back(0x08); put_varint(f, (uint64_t)h.height); }
  push();
  // 4. gogotypes.StdTimeMarshal(Time): Timestamp{1: seconds, 2: nanos}
  if (h.time_seconds) { f.push_back(0x08); put_varint(f, (uint64_t)h.time_seconds); }
  if (h.time_nanos) { f.push_back(0x10); put_varint(f, (uint64_t)(int64_t)h.time_nanos); }
  push();
  // 5. LastBlockID.ToProto().Marshal(): BlockID{1: hash, 2: PartSetHeader (always present)}
  {
    std::vector<uint8_t> psh;
    if (h.last_block_id.psh_total) { psh.push_back(0x08); put_varint(psh, h.last_block_id.psh_total); }
    if (h.last_block_id.psh_hash_len)
      put_bytes_field(psh, 0x12, h.last_block_id.psh_hash, h.last_block_id.psh_hash_len);
    if (h.last_block_id.hash_len) put_bytes_field(f, 0x0a, h.last_block_id.hash, h.last_block_id.hash_len);
    put_bytes_field(f, 0x12, psh.data(), psh.size());
  }
  push();
  // 6..14. cdcEncode(HexBytes): gogotypes.BytesValue{1: value}
  for (int k = 0; k < 9; k++) {
    if (h.hash_lens[k]) put_bytes_field(f, 0x0a, h.hashes[k], h.hash_lens[k]);
    push();
  }
}

// Leaves on the host -> roots on the host: the common driver of the byte-slice APIs.
int roots_from_host_leaves(tmed_ctx *c, const uint8_t *leaves, const uint64_t *leaf_off, size_t L,
                           const std::vector<uint32_t> &counts, uint8_t *roots) {
  const size_t T = counts.size();
  const size_t bytes = leaf_off[L] - leaf_off[0];
  std::lock_guard<std::mutex> lk(c->mu);
  (void)hipSetDevice(c->device);
  hipStream_t s = c->stream;
  hipError_t e = c->d_msg.ensure(bytes + 16);
  if (e == hipSuccess) e = c->d_off.ensure((L + 1) * 8);
  if (e == hipSuccess) e = c->d_merkle_a.ensure(std::max<size_t>(L, 1) * sizeof(Digest));
  if (e == hipSuccess) e = c->d_out.ensure(std::max<size_t>(T, 1) * 32);
  if (e != hipSuccess) return map_err(e);
  std::vector<uint64_t> off(L + 1);
  for (size_t i = 0; i <= L; i++) off[i] = leaf_off[i] - leaf_off[0];
  if (bytes) e = hipMemcpyAsync(c->d_msg.p, leaves + leaf_off[0], bytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->d_off.p, off.data(), (L + 1) * 8, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && L) {
    hipLaunchKernelGGL(merkle_leaf_kernel, dim3(blocks_for(L)), dim3(256), 0, s, (const uint8_t *)c->d_msg.p,
                       (const uint64_t *)c->d_off.p, (uint32_t)L, (Digest *)c->d_merkle_a.p);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return map_err(e);
  int rc = reduce_trees(c, counts, L, (uint8_t *)c->d_out.p, s);
  if (rc != TMED_OK) return rc;
  e = hipMemcpyAsync(roots, c->d_out.p, T * 32, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return map_err(e);
}

}  // namespace

extern "C" {

int tmed_merkle_roots(tmed_ctx *c, const uint8_t *leaves, const uint64_t *leaf_off, const uint32_t *tree_off,
                      size_t n_trees, uint8_t *roots) {
  if (!c || (n_trees && (!tree_off || !roots || !leaf_off))) return TMED_EINVAL;
  if (n_trees == 0) return TMED_OK;
  const size_t L = tree_off[n_trees];
  if (tree_off[0] != 0 || L > 0xffffffffu) return TMED_EINVAL;
  std::vector<uint32_t> counts(n_trees);
  for (size_t t = 0; t < n_trees; t++) {
    if (tree_off[t + 1] < tree_off[t]) return TMED_EINVAL;
    counts[t] = tree_off[t + 1] - tree_off[t];
  }
  for (size_t i = 0; i < L; i++)
    if (leaf_off[i + 1] < leaf_off[i] || leaf_off[i + 1] - leaf_off[i] > 0xffffffffu - 64) return TMED_EINVAL;
  if (L && leaf_off[L] > leaf_off[0] && !leaves) return TMED_EINVAL;
  return roots_from_host_leaves(c, leaves, leaf_off, L, counts, roots);
}

int tmed_valset_hashes(tmed_ctx *c, const uint8_t *pubkeys, const int64_t *powers, const uint32_t *set_off,
                       size_t n_sets, uint8_t *out) {
  if (!c || (n_sets && (!set_off || !out))) return TMED_EINVAL;
  if (n_sets == 0) return TMED_OK;
  const size_t N = set_off[n_sets];
  if (set_off[0] != 0 || N > 0xffffffffu || (N && (!pubkeys || !powers))) return TMED_EINVAL;
  std::vector<uint32_t> counts(n_sets);
  for (size_t t = 0; t < n_sets; t++) {
    if (set_off[t + 1] < set_off[t]) return TMED_EINVAL;
    counts[t] = set_off[t + 1] - set_off[t];
  }
  std::lock_guard<std::mutex> lk(c->mu);
  (void)hipSetDevice(c->device);
  hipStream_t s = c->stream;
  hipError_t e = c->d_a.ensure(std::max<size_t>(N, 1) * 32);
  if (e == hipSuccess) e = c->d_b.ensure(std::max<size_t>(N, 1) * 8);
  if (e == hipSuccess) e = c->d_merkle_a.ensure(std::max<size_t>(N, 1) * sizeof(Digest));
  if (e == hipSuccess) e = c->d_out.ensure(n_sets * 32);
  if (e == hipSuccess && N) e = hipMemcpyAsync(c->d_a.p, pubkeys, N * 32, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && N) e = hipMemcpyAsync(c->d_b.p, powers, N * 8, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && N) {
    hipLaunchKernelGGL(valset_leaf_kernel, dim3(blocks_for(N)), dim3(256), 0, s, (const uint8_t *)c->d_a.p,
                       (const int64_t *)c->d_b.p, (uint32_t)N, (Digest *)c->d_merkle_a.p);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return map_err(e);
  int rc = reduce_trees(c, counts, N, (uint8_t *)c->d_out.p, s);
  if (rc != TMED_OK) return rc;
  e = hipMemcpyAsync(out, c->d_out.p, n_sets * 32, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return map_err(e);
}

int tmed_header_hashes(tmed_ctx *c, const tmed_header *headers, size_t n, uint8_t *out, uint8_t *ok) {
  if (!c || (n && (!headers || !out || !ok))) return TMED_EINVAL;
  if (n == 0) return TMED_OK;
  std::vector<uint8_t> leaves;
  std::vector<uint64_t> off;
  leaves.reserve(n * 200);
  off.reserve(n * 14 + 1);
  off.push_back(0);
  std::vector<uint32_t> counts(n, 14);
  for (size_t i = 0; i < n; i++) {
    const tmed_header &h = headers[i];
    for (int k = 0; k < 9; k++)
      if (h.hash_lens[k] && !h.hashes[k]) return TMED_EINVAL;
    if ((h.chain_id_len && !h.chain_id) || (h.last_block_id.hash_len && !h.last_block_id.hash) ||
        (h.last_block_id.psh_hash_len && !h.last_block_id.psh_hash))
      return TMED_EINVAL;
    header_leaves(h, leaves, off);
    ok[i] = h.hash_lens[2] != 0;  // Header.Hash returns nil without a ValidatorsHash (:441-443)
  }
  return roots_from_host_leaves(c, leaves.data(), off.data(), off.size() - 1, counts, out);
}

int tmed_partset_roots(tmed_ctx *c, const uint8_t *data, const uint64_t *data_off, size_t n_blocks,
                       uint32_t part_size, uint8_t *roots) {
  if (!c || part_size == 0 || (n_blocks && (!data_off || !roots))) return TMED_EINVAL;
  if (n_blocks == 0) return TMED_OK;
  std::vector<uint64_t> off;
  std::vector<uint32_t> counts(n_blocks);
  off.push_back(data_off[0]);
  for (size_t b = 0; b < n_blocks; b++) {
    if (data_off[b + 1] < data_off[b]) return TMED_EINVAL;
    const uint64_t len = data_off[b + 1] - data_off[b];
    const uint64_t parts = (len + part_size - 1) / part_size;  // types/part_set.go:168
    if (parts > 0xffffffffu) return TMED_EINVAL;
    counts[b] = (uint32_t)parts;
    for (uint64_t p = 0; p < parts; p++) off.push_back(std::min(data_off[b] + (p + 1) * part_size, data_off[b + 1]));
  }
  const size_t L = off.size() - 1;
  if (L > 0xffffffffu || (L && !data)) return TMED_EINVAL;
  return roots_from_host_leaves(c, data, off.data(), L, counts, roots);
}

}  // extern "C"
