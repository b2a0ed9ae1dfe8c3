// signbytes.hip — CanonicalVote sign-bytes for the commit seam (host C++).
//
// Restates the byte layout the reference signs:
//   Commit.VoteSignBytes          types/block.go:807-810 (GetVote :784-796)
//   CommitSig.BlockID             types/block.go:652-665 (Commit -> commit BlockID; Absent/Nil -> zero)
//   VoteSignBytes                 types/vote.go:93-101 = protoio.MarshalDelimited(CanonicalizeVote)
//   CanonicalizeBlockID           types/canonical.go:18-34 (zero BlockID -> field omitted)
//   CanonicalVote marshal         proto/tendermint/types/canonical.pb.go:517-579 (field order,
//                                 zero-field omission, varints), CanonicalBlockID :370-393,
//                                 CanonicalPartSetHeader :410-428
//   length prefix                 libs/protoio/writer.go:54-100
//   Timestamp                     gogoproto StdTimeMarshalTo: {1: seconds, 2: nanos}, zeros omitted
// Only the timestamp (and the flag) differ between the votes of one commit, so
// the encoder writes a per-commit prefix/suffix once and splices each
// validator's timestamp between them.
#include <string.h>

#include "../../include/tmed25519.h"

namespace {

inline int uvarint_len(uint64_t v) {
  int n = 1;
  while (v >= 0x80) { v >>= 7; n++; }
  return n;
}
inline uint8_t *put_uvarint(uint8_t *p, uint64_t v) {
  while (v >= 0x80) { *p++ = (uint8_t)(v | 0x80); v >>= 7; }
  *p++ = (uint8_t)v;
  return p;
}
inline uint8_t *put_le64(uint8_t *p, uint64_t v) {
  for (int i = 0; i < 8; i++) *p++ = (uint8_t)(v >> (8 * i));
  return p;
}

// Encoded CanonicalBlockID body (without its tag/len); returns length or 0 when the BlockID is zero.
int block_id_body(const tmed_vote_template *t, uint8_t *buf) {
  const bool zero = t->block_hash_len == 0 && t->psh_total == 0 && t->psh_hash_len == 0;
  if (zero) return 0;
  uint8_t psh[64];
  uint8_t *q = psh;
  if (t->psh_total != 0) { *q++ = 0x08; q = put_uvarint(q, t->psh_total); }
  if (t->psh_hash_len > 0) { *q++ = 0x12; q = put_uvarint(q, t->psh_hash_len); memcpy(q, t->psh_hash, t->psh_hash_len); q += t->psh_hash_len; }
  const int psh_len = (int)(q - psh);
  uint8_t *p = buf;
  if (t->block_hash_len > 0) { *p++ = 0x0a; p = put_uvarint(p, t->block_hash_len); memcpy(p, t->block_hash, t->block_hash_len); p += t->block_hash_len; }
  *p++ = 0x12; p = put_uvarint(p, (uint64_t)psh_len); memcpy(p, psh, psh_len); p += psh_len;
  return (int)(p - buf);
}

}  // namespace

extern "C" int tmed_vote_sign_bytes(const tmed_vote_template *t, size_t n, const uint8_t *flags,
                                    const int64_t *ts_seconds, const int32_t *ts_nanos, uint8_t *out,
                                    size_t out_cap, uint32_t *out_off, size_t *out_len) {
  if (!t || (n && (!ts_seconds || !ts_nanos || !out_off))) return TMED_EINVAL;
  if ((t->block_hash_len != 0 && t->block_hash_len != 32) || (t->psh_hash_len != 0 && t->psh_hash_len != 32))
    return TMED_EINVAL;  // ValidateHash: BlockIDFromProto would panic (types/canonical.go:19-22)
  if (t->chain_id_len && !t->chain_id) return TMED_EINVAL;
  // prefix: type, height, round (identical for every vote of the commit)
  uint8_t pre[32];
  uint8_t *p = pre;
  *p++ = 0x08; *p++ = 0x02;  // SignedMsgType Precommit (GetVote, types/block.go:787)
  if (t->height != 0) { *p++ = 0x11; p = put_le64(p, (uint64_t)t->height); }
  if (t->round != 0) { *p++ = 0x19; p = put_le64(p, (uint64_t)(int64_t)t->round); }
  const int pre_len = (int)(p - pre);
  uint8_t bid[160];
  const int bid_body = block_id_body(t, bid);
  const int bid_field = bid_body ? 1 + uvarint_len((uint64_t)bid_body) + bid_body : 0;
  const int cid_field = t->chain_id_len ? 1 + uvarint_len(t->chain_id_len) + (int)t->chain_id_len : 0;
  size_t pos = 0;
  for (size_t i = 0; i < n; i++) {
    const uint8_t f = flags ? flags[i] : 2;
    if (f < 1 || f > 3) return TMED_EINVAL;  // CommitSig.BlockID panics on unknown flags (types/block.go:663)
    const bool with_bid = (f == 2);          // BlockIDFlagCommit -> commit BlockID, else zero BlockID
    const uint64_t sec = (uint64_t)ts_seconds[i];
    const uint64_t nan = (uint64_t)(int64_t)ts_nanos[i];
    const int ts_body = (sec ? 1 + uvarint_len(sec) : 0) + (nan ? 1 + uvarint_len(nan) : 0);
    const int body = pre_len + (with_bid ? bid_field : 0) + 1 + uvarint_len((uint64_t)ts_body) + ts_body + cid_field;
    const size_t total = (size_t)uvarint_len((uint64_t)body) + body;
    out_off[i] = (uint32_t)pos;
    if (out && pos + total <= out_cap) {
      uint8_t *w = out + pos;
      w = put_uvarint(w, (uint64_t)body);
      memcpy(w, pre, pre_len); w += pre_len;
      if (with_bid) { *w++ = 0x22; w = put_uvarint(w, (uint64_t)bid_body); memcpy(w, bid, bid_body); w += bid_body; }
      *w++ = 0x2a; w = put_uvarint(w, (uint64_t)ts_body);
      if (sec) { *w++ = 0x08; w = put_uvarint(w, sec); }
      if (nan) { *w++ = 0x10; w = put_uvarint(w, nan); }
      if (t->chain_id_len) { *w++ = 0x32; w = put_uvarint(w, t->chain_id_len); memcpy(w, t->chain_id, t->chain_id_len); w += t->chain_id_len; }
    }
    pos += total;
    if (pos > 0xffffffffu) return TMED_EINVAL;
  }
  if (n) out_off[n] = (uint32_t)pos;
  if (out_len) *out_len = pos;
  return (out && pos > out_cap) ? TMED_ENOMEM : TMED_OK;
}
