// votes_dev.h — CanonicalVote sign-bytes assembly on the device, shared by
// assemble_votes_kernel (kernels.hip) and the hash lanes of the generic latency kernel
// (latency.hip), which assemble their own message instead of waiting for a separate launch.
//
// Per commit a template (signbytes.hip VoteEncoder): [pre_len, bid_len, cid_len, 0] then the
// pre bytes (type/height/round), the complete BlockID field (tag 0x22 + len + body) and the
// complete chain-id field (tag 0x32 + len + bytes).  Per vote only the flag and the timestamp
// vary (types/block.go:784-810): the message is
//   uvarint(body) || pre || [BlockID field if flag == Commit] || 0x2a len {0x08 sec}{0x10 nanos} || chain
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace tmed {

__device__ __forceinline__ int uvarint_len_dev(uint64_t v) {
  int n = 1;
  while (v >= 0x80) { v >>= 7; n++; }
  return n;
}
__device__ __forceinline__ uint32_t put_uvarint_dev(uint8_t *p, uint32_t pos, uint64_t v) {
  while (v >= 0x80) { p[pos++] = (uint8_t)(v | 0x80); v >>= 7; }
  p[pos++] = (uint8_t)v;
  return pos;
}

// Vote i into o (at most kVoteSlot bytes); returns its length.  tl: this lane's kVoteTmplBytes of
// LDS — the template is staged there with sixteen independent 16-B loads, so a template in pinned
// host memory (small batches, keyset.hip votes_enqueue) costs one bus round trip instead of one
// per byte of the copy loops.
__device__ __forceinline__ uint32_t assemble_vote_into(const VoteAsm &va, uint32_t i, uint8_t *__restrict__ o,
                                                       int4 *tl) {
  {
    const int4 *src = reinterpret_cast<const int4 *>(va.tmpl + (size_t)va.tmpl_idx[i] * kVoteTmplBytes);
    int4 v[kVoteTmplBytes / 16];
#pragma unroll
    for (int q = 0; q < (int)(kVoteTmplBytes / 16); q++) v[q] = src[q];
#pragma unroll
    for (int q = 0; q < (int)(kVoteTmplBytes / 16); q++) tl[q] = v[q];
  }
  const uint8_t *t = reinterpret_cast<const uint8_t *>(tl);
  const uint32_t pre_len = t[0], bid_len = t[1], cid_len = t[2];
  const bool with_bid = va.flags[i] == 2;
  const uint64_t s = (uint64_t)va.ts_sec[i], ns = (uint64_t)(int64_t)va.ts_nanos[i];
  const uint32_t ts_body = (s ? 1 + uvarint_len_dev(s) : 0) + (ns ? 1 + uvarint_len_dev(ns) : 0);
  const uint32_t body = pre_len + (with_bid ? bid_len : 0) + 1 + uvarint_len_dev(ts_body) + ts_body + cid_len;
  uint32_t p = put_uvarint_dev(o, 0, body);
  const uint8_t *src = t + 4;
  for (uint32_t j = 0; j < pre_len; j++) o[p++] = src[j];
  src += pre_len;
  if (with_bid)
    for (uint32_t j = 0; j < bid_len; j++) o[p++] = src[j];
  src += bid_len;
  o[p++] = 0x2a;
  p = put_uvarint_dev(o, p, ts_body);
  if (s) { o[p++] = 0x08; p = put_uvarint_dev(o, p, s); }
  if (ns) { o[p++] = 0x10; p = put_uvarint_dev(o, p, ns); }
  for (uint32_t j = 0; j < cid_len; j++) o[p++] = src[j];
  return p;
}

// Vote i into its kVoteSlot-byte slot of out, its length into out_len[i] (the latency kernels'
// hash lanes, which assemble their own message in place).
__device__ __forceinline__ void assemble_vote(const VoteAsm &va, uint32_t i, uint8_t *__restrict__ out,
                                              uint32_t *__restrict__ out_len, int4 *tl) {
  out_len[i] = assemble_vote_into(va, i, out + (size_t)i * kVoteSlot, tl);
}

}  // namespace tmed
