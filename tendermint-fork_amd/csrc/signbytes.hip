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
#include "signbytes.h"

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

}  // namespace

namespace tmed {

int VoteEncoder::init(const tmed_vote_template *t) {
  if (!t) return TMED_EINVAL;
  if (t->chain_id_len && !t->chain_id) return TMED_EINVAL;
  // ValidateHash: CanonicalizeBlockID panics on a malformed hash (types/canonical.go:18-22), which
  // only a Commit-flag vote reaches (Absent / Nil votes sign the zero BlockID): such a template
  // can still encode those, and write()/size() must never be asked for a Commit vote.
  bid_ok = (t->block_hash_len == 0 || t->block_hash_len == 32) && (t->psh_hash_len == 0 || t->psh_hash_len == 32);
  uint8_t *p = pre;
  *p++ = 0x08; *p++ = 0x02;  // SignedMsgType Precommit (Commit.GetVote, types/block.go:787)
  if (t->height != 0) { *p++ = 0x11; p = put_le64(p, (uint64_t)t->height); }
  if (t->round != 0) { *p++ = 0x19; p = put_le64(p, (uint64_t)(int64_t)t->round); }
  pre_len = (int)(p - pre);
  // CanonicalBlockID body; a zero BlockID is omitted (CanonicalizeBlockID -> nil)
  const bool zero = t->block_hash_len == 0 && t->psh_total == 0 && t->psh_hash_len == 0;
  bid_body = 0;
  if (!zero && bid_ok) {
    uint8_t psh[64];
    uint8_t *q = psh;
    if (t->psh_total != 0) { *q++ = 0x08; q = put_uvarint(q, t->psh_total); }
    if (t->psh_hash_len > 0) { *q++ = 0x12; q = put_uvarint(q, t->psh_hash_len); memcpy(q, t->psh_hash, t->psh_hash_len); q += t->psh_hash_len; }
    const int psh_len = (int)(q - psh);
    uint8_t *b = bid;
    if (t->block_hash_len > 0) { *b++ = 0x0a; b = put_uvarint(b, t->block_hash_len); memcpy(b, t->block_hash, t->block_hash_len); b += t->block_hash_len; }
    *b++ = 0x12; b = put_uvarint(b, (uint64_t)psh_len); memcpy(b, psh, psh_len); b += psh_len;
    bid_body = (int)(b - bid);
  }
  bid_field = bid_body ? 1 + uvarint_len((uint64_t)bid_body) + bid_body : 0;
  cid = t->chain_id;
  cid_len = t->chain_id_len;
  cid_field = cid_len ? 1 + uvarint_len(cid_len) + (int)cid_len : 0;
  return TMED_OK;
}

size_t VoteEncoder::size(int flag, int64_t sec, int32_t nanos) const {
  const uint64_t s = (uint64_t)sec, n = (uint64_t)(int64_t)nanos;
  const int ts_body = (s ? 1 + uvarint_len(s) : 0) + (n ? 1 + uvarint_len(n) : 0);
  const int body = pre_len + (flag == 2 ? bid_field : 0) + 1 + uvarint_len((uint64_t)ts_body) + ts_body + cid_field;
  return (size_t)uvarint_len((uint64_t)body) + body;
}

uint8_t *VoteEncoder::write(uint8_t *w, int flag, int64_t sec, int32_t nanos) const {
  const uint64_t s = (uint64_t)sec, n = (uint64_t)(int64_t)nanos;
  const int ts_body = (s ? 1 + uvarint_len(s) : 0) + (n ? 1 + uvarint_len(n) : 0);
  const bool with_bid = flag == 2;  // BlockIDFlagCommit -> commit BlockID; Absent/Nil -> zero BlockID
  const int body = pre_len + (with_bid ? bid_field : 0) + 1 + uvarint_len((uint64_t)ts_body) + ts_body + cid_field;
  w = put_uvarint(w, (uint64_t)body);
  memcpy(w, pre, pre_len); w += pre_len;
  if (with_bid && bid_body) { *w++ = 0x22; w = put_uvarint(w, (uint64_t)bid_body); memcpy(w, bid, bid_body); w += bid_body; }
  *w++ = 0x2a; w = put_uvarint(w, (uint64_t)ts_body);
  if (s) { *w++ = 0x08; w = put_uvarint(w, s); }
  if (n) { *w++ = 0x10; w = put_uvarint(w, n); }
  if (cid_len) { *w++ = 0x32; w = put_uvarint(w, cid_len); memcpy(w, cid, cid_len); w += cid_len; }
  return w;
}

bool VoteEncoder::device_template(uint8_t *out, size_t cap, size_t slot) const {
  const size_t need = 4 + (size_t)pre_len + (size_t)bid_field + (size_t)cid_field;
  if (need > cap || bid_field > 255 || cid_field > 255) return false;
  // the longest message of this template: a Commit-flag vote whose timestamp has a 10-byte seconds
  // varint and a 10-byte nanos varint (any int32 nanos crosses the ABI; negative ones are 10 bytes),
  // i.e. ts_body <= 22 and the timestamp field <= 24 bytes
  const size_t max_body = (size_t)pre_len + (size_t)bid_field + 24 + (size_t)cid_field;
  if ((size_t)uvarint_len(max_body) + max_body > slot) return false;
  out[0] = (uint8_t)pre_len;
  out[1] = (uint8_t)bid_field;
  out[2] = (uint8_t)cid_field;
  out[3] = 0;
  uint8_t *w = out + 4;
  memcpy(w, pre, pre_len); w += pre_len;
  if (bid_body) { *w++ = 0x22; w = put_uvarint(w, (uint64_t)bid_body); memcpy(w, bid, bid_body); w += bid_body; }
  if (cid_len) { *w++ = 0x32; w = put_uvarint(w, cid_len); memcpy(w, cid, cid_len); w += cid_len; }
  return true;
}

}  // namespace tmed

extern "C" int tmed_vote_sign_bytes(const tmed_vote_template *t, size_t n, const uint8_t *flags,
                                    const int64_t *ts_seconds, const int32_t *ts_nanos, uint8_t *out,
                                    size_t out_cap, uint32_t *out_off, size_t *out_len) {
  if (!t || (n && (!ts_seconds || !ts_nanos || !out_off))) return TMED_EINVAL;
  tmed::VoteEncoder enc;
  int rc = enc.init(t);
  if (rc != TMED_OK) return rc;
  size_t pos = 0;
  for (size_t i = 0; i < n; i++) {
    const int f = flags ? flags[i] : 2;
    if (f < 1 || f > 3) return TMED_EINVAL;  // CommitSig.BlockID panics on unknown flags (types/block.go:663)
    if (f == 2 && !enc.bid_ok) return TMED_EINVAL;  // CanonicalizeBlockID panics (types/canonical.go:18-22)
    const size_t total = enc.size(f, ts_seconds[i], ts_nanos[i]);
    out_off[i] = (uint32_t)pos;
    if (out && pos + total <= out_cap) enc.write(out + pos, f, ts_seconds[i], ts_nanos[i]);
    pos += total;
    if (pos > 0xffffffffu) return TMED_EINVAL;
  }
  if (n) out_off[n] = (uint32_t)pos;
  if (out_len) *out_len = pos;
  return (out && pos > out_cap) ? TMED_ENOMEM : TMED_OK;
}
