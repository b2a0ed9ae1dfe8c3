// signbytes.h — per-commit CanonicalVote encoder (see signbytes.hip for the layout + citations).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/tmed25519.h"

namespace tmed {

// f1: on-device CanonicalVote assembly (kernels.h launch_assemble_votes): templates are
// kVoteTmplBytes records, message i is written at i * kVoteSlot.
constexpr uint32_t kVoteTmplBytes = 256;
constexpr uint32_t kVoteSlot = 256;

// Everything but the per-vote flag/timestamp is encoded once per commit.
struct VoteEncoder {
  uint8_t pre[32];
  int pre_len = 0;
  uint8_t bid[160];
  int bid_body = 0, bid_field = 0;
  bool bid_ok = true;  // block/part-set hashes pass ValidateHash (else only Absent/Nil votes encode)
  const char *cid = nullptr;
  uint32_t cid_len = 0;
  int cid_field = 0;

  int init(const tmed_vote_template *t);
  size_t size(int flag, int64_t sec, int32_t nanos) const;
  uint8_t *write(uint8_t *out, int flag, int64_t sec, int32_t nanos) const;
  // Device template record for the on-device assembler (kernels.h kVoteTmplBytes):
  // [pre_len, bid_field_len, cid_field_len, 0] + pre + BlockID field + chain-id field.
  // Returns false if it does not fit in `cap` bytes, or if a vote's message could exceed `slot`
  // bytes (the device writes vote i at i * slot): long chain IDs take the host path.
  bool device_template(uint8_t *out, size_t cap, size_t slot) const;
};

}  // namespace tmed
