/*
 * tmed25519.h — C ABI of the MI355X batch ed25519 verification engine
 * (libtmed25519_hip.so, built from tendermint-fork_amd/csrc for gfx950).
 *
 * The reference (Tendermint Core v0.34.24, pure Go) has no native boundary on
 * this path: every signature goes through the Go interface method
 *     crypto.PubKey.VerifySignature(msg, sig []byte) bool      crypto/crypto.go:25
 *     -> ed25519.PubKey.VerifySignature                      crypto/ed25519/ed25519.go:148-155
 * called one at a time from the commit-verification loops
 *     ValidatorSet.VerifyCommit                              types/validator_set.go:667-714 (call :696)
 *     ValidatorSet.VerifyCommitLight                         types/validator_set.go:722-765 (call :752)
 *     ValidatorSet.VerifyCommitLightTrusting                 types/validator_set.go:775-826 (call :813)
 * This header is what a cgo shim at that seam binds: the
 * per-signature calls of one commit (or of many commits) become ONE call that
 * returns a validity byte per tuple, and the shim replays the reference loop
 * over those bytes, so early exits, error values and tallies are unchanged.
 *
 * Conventions
 *   - Plain pointers and sizes only; no allocation is handed across the ABI.
 *   - Return 0 on success, a negative TMED_E* code on failure.  On failure the
 *     caller must not use out_valid (the Go shim then calls the original Go
 *     method — never a guessed decision).  Nothing aborts or throws across the ABI.
 *   - out_valid[i] is 1 iff Go 1.18 crypto/ed25519.Verify would return true for
 *     (pub[i], msg[i], sig[i]) (and len(sig[i]) == 64): cofactorless, S < L
 *     strict, permissive A decoding, byte-compared R.
 *   - All host pointers are only read during the call (cgo pointer rules: the
 *     library copies what it needs before returning).  A context may be shared
 *     by concurrent callers: calls on one context are serialised internally.
 */
#ifndef TMED25519_H
#define TMED25519_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TMED_OK 0
#define TMED_EINVAL (-1)    /* bad argument (null pointer, offsets not monotone, ...) */
#define TMED_ENODEV (-2)    /* no usable gfx950 device */
#define TMED_EHIP (-3)      /* HIP runtime error (device lost, launch failure) */
#define TMED_ENOMEM (-4)    /* device or pinned-host allocation failed */
#define TMED_ENOKEYSET (-5) /* unknown key-set handle */
#define TMED_EINTERNAL (-6) /* internal error: a host-side exception inside the library (a bug, never a
                               decision); the call's outputs are unusable.  A seam call that fails this
                               way (or any other way) while blocksync windows are in flight on the
                               context drops those windows: their results are not final, and
                               tmed_blocksync_wait reports the error */

typedef struct tmed_ctx tmed_ctx;

/* Number of visible HIP devices (0 when none). */
int tmed_device_count(void);

/* Create a context bound to HIP device `device` (one process per GPU). */
int tmed_init(int device, tmed_ctx **out);
void tmed_destroy(tmed_ctx *ctx);
const char *tmed_strerror(int code);

/*
 * Batch verification, host buffers.  Replaces n calls of
 * ed25519.PubKey.VerifySignature (crypto/ed25519/ed25519.go:148-155).
 *   pubkeys   n x 32 bytes
 *   sigs      n x 64 bytes (slot i holds the first sig_lens[i] bytes when sig_lens != NULL)
 *   sig_lens  NULL (all 64) or n lengths; any length != 64 is rejected
 *             (ed25519.go:150-152) without touching the device
 *   msgs      concatenated messages; message i is msgs[msg_off[i] .. msg_off[i+1])
 *   msg_off   n + 1 non-decreasing offsets
 *   out_valid n bytes, 0/1
 */
int tmed_verify_batch(tmed_ctx *ctx, const uint8_t *pubkeys, const uint8_t *sigs, const uint32_t *sig_lens,
                      const uint8_t *msgs, const uint32_t *msg_off, size_t n, uint8_t *out_valid);

/*
 * Same, on device-resident buffers (all pointers are device pointers of the
 * context's device; stream = hipStream_t or NULL for the context stream).
 * Asynchronous: completion is ordered on `stream`.  Used when inputs already
 * live in HBM (bench, multi-commit pipelines).
 */
int tmed_verify_batch_device(tmed_ctx *ctx, const uint8_t *d_pubkeys, const uint8_t *d_sigs,
                             const uint8_t *d_msgs, const uint32_t *d_msg_off, size_t n, uint8_t *d_out_valid,
                             void *stream);

/*
 * RFC 8032 signing (crypto/ed25519/ed25519.go:57-60 semantics) used to build
 * synthetic commits at scale (SURVEY.md §7 "synthetic data volume").
 * seeds n x 32, outputs sigs n x 64 and pubkeys n x 32.
 */
int tmed_sign_batch(tmed_ctx *ctx, const uint8_t *seeds, const uint8_t *msgs, const uint32_t *msg_off, size_t n,
                    uint8_t *sigs_out, uint8_t *pubkeys_out);
int tmed_sign_batch_device(tmed_ctx *ctx, const uint8_t *d_seeds, const uint8_t *d_msgs, const uint32_t *d_msg_off,
                           size_t n, uint8_t *d_sigs_out, uint8_t *d_pubkeys_out, void *stream);

/*
 * Diagnostics of the default (half-size scalar) path: for the last chunk of the last
 * tmed_verify_batch / _device call, histograms of the radix-16 window count W the lattice step
 * gave each signature (lane_hist[W]) and of the per-wave maximum the main kernel ran
 * (wave_hist[W], 64 signatures per wave; W = 64 is the unshortened (k, 1) fallback).
 * All zero when the last call took another path.
 */
int tmed_window_stats(tmed_ctx *ctx, uint32_t lane_hist[65], uint32_t wave_hist[65]);

/*
 * Radix (in bits) of the fixed-base B windows of the default path on this context: 26 (two
 * tables of 2^25 + 1 affine multiples of B and 2^128 B, 8.6 GB per device, ten B additions per
 * signature) or 16 (windows of the context's radix-2^16 comb, sixteen additions: TMED_B26=0 or
 * when the large tables could not be allocated).  Diagnostic; decisions are identical.
 */
int tmed_b_window_bits(const tmed_ctx *ctx);
/*
 * The same for the key-cached throughput path: 24 (a shared radix-2^24 comb of B, 11 windows of
 * 2^23 + 1 multiples, 11.8 GB per device, acquired at the context's first tmed_keyset_load:
 * eleven B additions per signature) or 16 (the context's radix-2^16 comb, sixteen: before any
 * key-set load, with TMED_B24=0, or when the allocation failed).  Diagnostic; same decisions.
 */
int tmed_keyset_b_window_bits(const tmed_ctx *ctx);
/*
 * Radix (in bits) of the -A comb the key-cached throughput kernel reads for key set `handle`: 12
 * (21 windows of 2049 multiples, the top one 4225, 5.8 MB per key, built at the set's first
 * throughput batch with the radix-2^24 B comb in use: 32 comb rows per signature) or 8 (the
 * radix-256 comb every key set holds, also used by the latency kernels: TMED_KS_ACOMB=0, before
 * the first throughput batch, or no memory).  -1 for an unknown handle.  Diagnostic; decisions
 * are identical.
 */
int tmed_keyset_a_window_bits(tmed_ctx *ctx, uint64_t handle);
/*
 * Diagnostic (tests): entry j of window `window` of key `key`'s comb in key set `handle`, as the 30
 * int32 limbs (radix 2^25.5) the kernels read: y + x, y - x, 2d x y of the affine point
 * j * R^window * (-A_key), with R = 256 for radix_bits 8 (the comb every key set holds) or
 * R = 2^radix_bits for the throughput comb (radix_bits = tmed_keyset_a_window_bits(handle)).
 * Drains the device first.  TMED_EINVAL for an unknown handle, an index out of range or a comb
 * not built.
 */
int tmed_keyset_comb_entry(tmed_ctx *ctx, uint64_t handle, uint32_t key, int radix_bits, uint32_t window, uint32_t j,
                           int32_t out[30]);

/* Device time (ms) of the last verify/sign launch on this context (HIP events).  A commit batch
 * small enough for the zero-copy latency mode (a single commit), or a tmed_verify_batch of at most
 * 1024 signatures, reports 0 unless kernel timing is on (tmed_set_kernel_timing): its events would
 * add ~8 us to the call. */
float tmed_last_kernel_ms(tmed_ctx *ctx);

/*
 * Per-kernel timing of tmed_verify_batch_device (diagnostics, bench roofline): when on,
 * HIP events are recorded on the launch stream around each kernel of a call;
 * tmed_kernel_times returns, for the last call, the summed device time (ms) and the
 * launch count of each kernel kind: [0] prep (SHA-512, scalar checks, decompression),
 * [1] main (table + Straus), [2] finish (batched inversion + encode + compare).
 */
int tmed_set_kernel_timing(tmed_ctx *ctx, int on);
int tmed_kernel_times(tmed_ctx *ctx, float ms[3], int launches[3]);


/* ------------------------------------------------------- key-set cache */

/*
 * Decode a validator set's keys once (Point.SetBytes rule) and build a
 * signed radix-256 comb of -A per key in HBM.  Signatures
 * are then verified by key index: 64 mixed additions, no doublings, no per-
 * signature decompression.  Decisions are identical to tmed_verify_batch.
 * Callers key the handle by ValidatorSet.Hash() (types/validator_set.go:347-353).
 */
int tmed_keyset_load(tmed_ctx *ctx, const uint8_t *pubkeys, size_t n, uint64_t *handle);
int tmed_keyset_free(tmed_ctx *ctx, uint64_t handle);
/*
 * Append n keys to a loaded key set (its comb tables are built before the call returns).  The keys
 * already in the set keep their indexes; the new ones get first_index .. first_index + n - 1
 * (*first_index = the set's size before the call; may be NULL).  One pooled set can then serve
 * validator sets that change by a few keys per height (tmed_valset.keyset_index), as the light
 * client's do (light/verifier.go:58,73-76).
 */
int tmed_keyset_extend(tmed_ctx *ctx, uint64_t handle, const uint8_t *pubkeys, size_t n, uint32_t *first_index);
int tmed_verify_batch_keyset(tmed_ctx *ctx, uint64_t handle, const uint32_t *val_idx, const uint8_t *sigs,
                             const uint32_t *sig_lens, const uint8_t *msgs, const uint32_t *msg_off, size_t n,
                             uint8_t *out_valid);
int tmed_verify_batch_keyset_device(tmed_ctx *ctx, uint64_t handle, const uint32_t *d_val_idx, const uint8_t *d_sigs,
                                    const uint8_t *d_msgs, const uint32_t *d_msg_off, size_t n, uint8_t *d_out_valid,
                                    void *stream);

/* ---------------------------------------------------------------- ZIP-215 (opt-in) */

/*
 * The OPT-IN ZIP-215 rule (spec/core/encoding.md:52-54: "Tendermint adopted zip215 for verification
 * of ed25519 signatures ... released in 0.35"; the reference's own code, crypto/ed25519/ed25519.go:
 * 148-155, verifies with Go 1.18's cofactorless Verify, which tmed_verify_batch reproduces and which
 * stays the default).  Rule: A and R decoded permissively (y >= p and x = 0 with the sign bit
 * accepted), S < L, k = SHA-512(R || A || M) mod L, accept iff [8]([S]B - R - [k]A) = O.
 * Chunks of up to 2^20 signatures are checked as ONE randomized batch equation (Pippenger MSM with
 * secret 126-bit weights from getrandom); a failing chunk is bisected and the failing groups are
 * decided signature by signature by the exact single check, so out_valid[i] equals the ZIP-215
 * single-signature decision for every i.  sig_lens as in tmed_verify_batch.
 */
int tmed_verify_batch_zip215(tmed_ctx *ctx, const uint8_t *pubkeys, const uint8_t *sigs, const uint32_t *sig_lens,
                             const uint8_t *msgs, const uint32_t *msg_off, size_t n, uint8_t *out_valid);
int tmed_verify_batch_zip215_device(tmed_ctx *ctx, const uint8_t *d_pubkeys, const uint8_t *d_sigs,
                                    const uint8_t *d_msgs, const uint32_t *d_msg_off, size_t n, uint8_t *d_out_valid,
                                    void *stream);
/* Tests only: fix the batch weights' 32-byte seed for this thread's calls (NULL: getrandom again).
 * TMED_EINVAL unless the process environment has TMED_ZIP215_TEST_SEED=1 (known weights would let a
 * forger build invalid signatures whose errors cancel in the batch equation). */
int tmed_zip215_set_seed(const uint8_t *seed32);
/* This thread's last ZIP-215 call: chunks, batch equations evaluated, groups decided signature by
 * signature, signatures decided singly. */
int tmed_zip215_stats(uint32_t out[4]);

/* ---------------------------------------------------------------- commits */

/*
 * The per-commit part of a vote's CanonicalVote sign-bytes:
 * everything Commit.GetVote (types/block.go:784-796) copies from the commit.
 */
typedef struct {
  const char *chain_id;
  uint32_t chain_id_len;
  int64_t height;
  int32_t round;
  const uint8_t *block_hash; /* 0 or 32 bytes (ValidateHash) */
  uint32_t block_hash_len;
  uint32_t psh_total;
  const uint8_t *psh_hash;   /* 0 or 32 bytes */
  uint32_t psh_hash_len;
} tmed_vote_template;

/*
 * Commit.VoteSignBytes(chainID, idx) for n commit signatures
 * (types/block.go:807-810 -> types/vote.go:93-101): flags[i] in {1,2,3}
 * (BlockIDFlag; NULL = all Commit), per-signature timestamp (seconds, nanos).
 * Writes message i to out[out_off[i] .. out_off[i+1]) when out_cap suffices;
 * *out_len receives the total size (call with out = NULL to size the buffer,
 * TMED_ENOMEM when out_cap is too small).  Unknown flags -> TMED_EINVAL
 * (the reference panics, types/block.go:663).
 */
int tmed_vote_sign_bytes(const tmed_vote_template *t, size_t n, const uint8_t *flags, const int64_t *ts_seconds,
                         const int32_t *ts_nanos, uint8_t *out, size_t out_cap, uint32_t *out_off, size_t *out_len);

/* --------------------------------------------------------- diagnostics */

/*
 * Integer-VALU peak probe for the roofline: runs a
 * dependency-free stream of `kind` instructions on every lane of the device
 * (0 v_mad_i64_i32, 1 v_mad_u64_u32, 2 v_add_u32, 3 v_mul_lo_u32, 4 v_ashrrev_i64,
 * 5 v_lshl_add_u64, 6 v_lshl_add_u32, 7 v_add_co_u32+v_addc_co_u32, 8 v_lshrrev_b64,
 * 9 v_alignbit_b32, 10 v_and_b32, 11 v_bfe_i32, 12 v_and_or_b32, 13 v_cndmask_b32,
 * 14 v_ashrrev_i32, 15 v_cndmask_b32_e64 with an SGPR lane mask, 16 / 17 v_cmp_gt_u32 +
 * v_cndmask_b32 through vcc / an SGPR pair, counted as 2)
 * and returns the sustained rate in 1e9 instructions (lane-ops) per second.
 */
int tmed_valu_peak(tmed_ctx *ctx, int kind, double *giga_ops_per_s);

/*
 * Test hooks of the commit seam (process-wide, 0 = off, the product default; tests only):
 * tmed_test_pool_jitter — every part of the seam's host-parallel regions starts up to max_us
 * microseconds late (a part reading what another part of the same region writes then sees it
 * unwritten); tmed_test_stream_delay — a wave sleeping ~us microseconds is queued in front of every
 * batch copy on the copy stream and every key append on the context stream (a kernel lane that does
 * not wait for its producer then reads unfinished data).  tests/test_gpu_jitter.py,
 * tests/test_gpu_stream_delay.py.
 */
void tmed_test_pool_jitter(int max_us);
void tmed_test_stream_delay(int us);

/*
 * With TMED_DEBUG_ZERO set at the first pipelined generic batch: every staged candidate whose
 * device bit is 0 is recorded (request, signature, staging position, the staged and the device
 * copies of its key and signature, the assembled sign-bytes).  Copies up to cap records into out
 * and removes them; *n = records copied; returns the record size in bytes (tools/stress/c3_stress.py).
 */
int tmed_debug_zero_bits(void *out, size_t cap, size_t *n);

/* ------------------------------------------------------- commit seam (C++) */

/* BlockID as compared by BlockID.Equals (types/block.go:1170-1173). */
typedef struct {
  const uint8_t *hash;
  uint32_t hash_len;
  uint32_t psh_total;
  const uint8_t *psh_hash;
  uint32_t psh_hash_len;
} tmed_block_id;

/* ValidatorSet (types/validator_set.go:51-58), index order = commit order. */
typedef struct {
  size_t n;
  const uint8_t *pubkeys;   /* n x 32 (ed25519 keys; other key types stay on the Go path) */
  const int64_t *powers;    /* n voting powers */
  const uint8_t *addresses; /* n x 20, PubKey.Address(); needed by LightTrusting only (may be NULL otherwise).
                               Every validator address must be 20 bytes (Validator.ValidateBasic,
                               types/validator.go:49): a caller holding another length takes the Go path */
  int64_t total_power;      /* vals.TotalVotingPower() (its panics stay in Go, :298-321) */
  uint64_t keyset;          /* 0 (the context's key-set cache decides, see tmed_keycache_config), or a
                               tmed_keyset_load handle holding these pubkeys (key-cached path) */
  const uint32_t *keyset_index; /* NULL: validator i is key i of the key set; else its index there
                                   (one key set can then serve many validator sets, e.g. the light client) */
  const uint8_t *set_hash;  /* NULL, or ValidatorSet.Hash() of this set (32 bytes, types/validator_set.go:
                               347-353): the key-set cache's key for it (else a digest of the key bytes).
                               Either way a cached set is compared key by key before it is used. */
} tmed_valset;

/* Commit + CommitSigs (types/block.go:575-634, 737-752). */
typedef struct {
  int64_t height;
  int32_t round;
  tmed_block_id block_id;
  size_t n_sigs;
  const uint8_t *flags;       /* BlockIDFlag per signature: 1 Absent, 2 Commit, 3 Nil */
  const uint8_t *addresses;   /* n_sigs x 20 ValidatorAddress (LightTrusting only; may be NULL otherwise) */
  const int64_t *ts_seconds;  /* Timestamp.Unix() */
  const int32_t *ts_nanos;    /* Timestamp.Nanosecond() */
  const uint8_t *sigs;        /* n_sigs x 64 (first sig_lens[i] bytes meaningful) */
  const uint32_t *sig_lens;   /* NULL = all 64 */
  const uint32_t *address_lens; /* NULL = all 20; else len(ValidatorAddress) per signature.  GetByAddress
                                   compares with bytes.Equal (types/validator_set.go:270-277): an address
                                   whose length is not 20 matches no validator, so LightTrusting skips
                                   that signature (its 20-byte slot is then ignored) */
} tmed_commit;

#define TMED_MODE_COMMIT 0         /* ValidatorSet.VerifyCommit              :667-714 */
#define TMED_MODE_LIGHT 1          /* ValidatorSet.VerifyCommitLight         :722-765 */
#define TMED_MODE_LIGHT_TRUSTING 2 /* ValidatorSet.VerifyCommitLightTrusting :775-826 */

typedef struct {
  int mode;
  const char *chain_id;
  uint32_t chain_id_len;
  const tmed_valset *vals;
  const tmed_block_id *block_id; /* COMMIT / LIGHT: expected BlockID */
  int64_t height;                /* COMMIT / LIGHT: expected height */
  const tmed_commit *commit;
  int64_t trust_num, trust_den;  /* LIGHT_TRUSTING: tmmath.Fraction (libs/math/fraction.go:11-18) */
} tmed_commit_request;

/* ------------------------------------------------- key-set cache of the commit seam (f2) */

/*
 * tmed_verify_commits / tmed_blocksync_verify (and their _multi forms) give every validator set
 * that carries no handle (tmed_valset.keyset == 0) to the context's key-set cache, so the
 * reference's callers reach the key-cached kernels without managing handles: LastCommit against
 * LastValidators every block (state/validation.go:93-96), the blocksync window against
 * state.Validators (blockchain/v0/reactor.go:366-367), the light client's trusted / untrusted sets
 * (light/verifier.go:58,73-76).  The cache holds ONE pooled key set per context (a key held by many
 * sets is built once) and an entry per validator set, keyed by set_hash when given, else by a digest
 * of the ordered keys, and compared key by key on every hit.  On a miss: a set whose keys are all in
 * the pool is keyed at once; a call whose own signatures pay for building the missing keys (>= 2048
 * per key: a blocksync window, a light-client batch) builds them first and is keyed; otherwise the
 * call runs the generic kernels and the missing keys are built right after it by a worker thread of
 * the context (off the caller's critical path), so the next call against that set is keyed (C1: the first VerifyCommit after a set change is generic, the rest
 * are cache hits).  Decisions are identical either way.
 *   enabled: 1 on, 0 off (sets without a handle stay generic), -1 unchanged (default on; env
 *            TMED_KEYCACHE=0 turns it off at tmed_init);
 *   budget_bytes: 0 unchanged, else the pool's HBM budget (default 160 GiB, env TMED_KEYCACHE_GB;
 *            ~6.3 MB per key with the radix-2^12 comb): a set that does not fit empties the pool
 *            when no call is using it, else stays generic.
 */
int tmed_keycache_config(tmed_ctx *ctx, int enabled, size_t budget_bytes);
typedef struct {
  uint64_t enabled, budget_bytes;
  uint64_t lookups, hits;                 /* validator-set lookups by seam calls; hits on a cached entry */
  uint64_t keyed_sets, generic_sets;      /* lookups resolved to the key-cached / generic kernels */
  uint64_t keyed_sigs, generic_sigs;      /* signatures of the requests resolved each way */
  uint64_t keys_appended, keys_deferred;  /* keys built into the pool; of those, built after a generic call */
  uint64_t pool_resets, sets_evicted;     /* pool emptied to fit a set; entries dropped (LRU bound) */
  uint64_t pool_keys, pool_capacity_keys, pool_bytes, pool_a_window_bits;
  uint64_t sets_cached, pending_keys;
} tmed_keycache_counters;
int tmed_keycache_stats(tmed_ctx *ctx, tmed_keycache_counters *out);
/* Wait until the keys queued by generic calls are built (the context's build worker is idle and
 * the device has finished): the next call against those sets is keyed.  Tests and benches. */
int tmed_keycache_wait(tmed_ctx *ctx);
/* Drop every cached set and the pool (TMED_EINVAL while a call is using it). */
int tmed_keycache_flush(tmed_ctx *ctx);
/* Build a set's missing keys now (e.g. at a validator-set change, before its first commit), so
 * even its first call is keyed.  TMED_ENOMEM when it does not fit the budget. */
int tmed_keycache_warm(tmed_ctx *ctx, const tmed_valset *vals);

/* Outcome codes: the reference's return value, to be formatted by the caller exactly as Go does. */
#define TMED_COMMIT_OK 0
#define TMED_COMMIT_WRONG_SET_SIZE 1   /* ErrInvalidCommitSignatures{expected, actual} (types/errors.go:32-41) */
#define TMED_COMMIT_WRONG_HEIGHT 2     /* ErrInvalidCommitHeight{expected, actual} (types/errors.go:21-30) */
#define TMED_COMMIT_WRONG_BLOCK_ID 3   /* "invalid commit -- wrong block ID: want %v, got %v" */
#define TMED_COMMIT_WRONG_SIGNATURE 4  /* "wrong signature (#%d): %X" (idx) */
#define TMED_COMMIT_NOT_ENOUGH_POWER 5 /* ErrNotEnoughVotingPowerSigned{got, needed} (:856-863) */
#define TMED_COMMIT_DOUBLE_VOTE 6      /* "double vote from %v (%d and %d)" (val_idx, idx_first, idx) */
#define TMED_COMMIT_ZERO_DENOMINATOR 7 /* "trustLevel has zero Denominator" */
#define TMED_COMMIT_OVERFLOW 8         /* "int64 overflow while calculating voting power needed..." */
#define TMED_COMMIT_PANIC 9            /* the reference loop PANICS when it reaches signature idx: an unknown
                                          BlockIDFlag in VerifyCommit (CommitSig.BlockID, types/block.go:652-665)
                                          or a malformed BlockID hash in the sign-bytes of a Commit-flag vote
                                          (CanonicalizeBlockID, types/canonical.go:18-22).  Every earlier
                                          signature the loop reached was valid.  The caller runs the original
                                          Go method for this request, which panics exactly as before. */

typedef struct {
  int code;
  int64_t got, needed;     /* NOT_ENOUGH_POWER */
  int64_t expected, actual;/* WRONG_SET_SIZE / WRONG_HEIGHT */
  int32_t idx;             /* WRONG_SIGNATURE / PANIC index; DOUBLE_VOTE second index */
  int32_t idx_first;       /* DOUBLE_VOTE first index */
  int32_t val_idx;         /* DOUBLE_VOTE validator index */
  uint32_t verified;       /* signatures sent to the device for this request */
} tmed_commit_result;

/*
 * Verify n commit requests with ONE device batch: run the reference prechecks,
 * collect the signatures each loop would reach (all non-absent for COMMIT; the
 * ForBlock prefix up to the >2/3 (resp. trust-level) crossing for LIGHT /
 * LIGHT_TRUSTING, stopping at a double vote), build their CanonicalVote
 * sign-bytes, verify them on the GPU, then replay each reference loop over the
 * validity bits — same first-error index, same early exit, same Got/Needed.
 * Inputs on which the reference loop panics (unknown BlockIDFlag, malformed BlockID
 * hash) give that request the outcome TMED_COMMIT_PANIC at the index where the loop
 * would panic — only if the loop reaches it; the other requests are unaffected.
 * TMED_EINVAL is reserved for malformed calls (null pointers, unknown mode).
 */
int tmed_verify_commits(tmed_ctx *ctx, const tmed_commit_request *reqs, size_t n, tmed_commit_result *out);

/*
 * The same seam with the batch verifier supplied by the caller (same contract
 * as tmed_verify_batch; return 0 on success).  tmed_verify_commits is this
 * with the context's GPU verifier.  Lets a host integrate its own verifier
 * (e.g. the Go shim's fallback is the original Go method, not this) and lets
 * the CPU test-suite check the plan/replay logic against the oracle.
 */
typedef int (*tmed_batch_verify_fn)(void *user, const uint8_t *pubkeys, const uint8_t *sigs, const uint32_t *sig_lens,
                                    const uint8_t *msgs, const uint32_t *msg_off, size_t n, uint8_t *out_valid);
int tmed_verify_commits_with(const tmed_commit_request *reqs, size_t n, tmed_commit_result *out,
                             tmed_batch_verify_fn verify, void *user);

/*
 * Diagnostics: wall time in microseconds of the three phases of the calling thread's last
 * tmed_verify_commits / tmed_verify_commits_with / tmed_blocksync_verify call — [0] host plan
 * (prechecks, candidate collection), [1] verify (sign-bytes, staging, device, copy back),
 * [2] host replay.  For a call the seam pipelines (large batches: two vote slots), [0] is the
 * host plan + staging time, [1] the time the host is blocked waiting for the device and [2]
 * the host scatter + replay time; [0] and [2] overlap device work there.
 */
int tmed_seam_phase_us(double out_us[3]);

/* ------------------------------------------------ Merkle hashing (f3) */

/*
 * crypto/merkle.HashFromByteSlices (crypto/merkle/tree.go:9-22; RFC-6962 leaf 0x00 /
 * inner 0x01 prefixes, crypto/merkle/hash.go:19-27) for n_trees trees at once: tree t's
 * leaves are leaf indices [tree_off[t], tree_off[t+1]); leaf i is
 * leaves[leaf_off[i] .. leaf_off[i+1]).  roots: n_trees x 32 bytes.  An empty tree's root is
 * SHA-256("") as in the reference.  SHA-256 runs on the device (one lane per leaf, then one
 * launch per tree level across all trees).
 */
int tmed_merkle_roots(tmed_ctx *ctx, const uint8_t *leaves, const uint64_t *leaf_off, const uint32_t *tree_off,
                      size_t n_trees, uint8_t *roots);

/*
 * ValidatorSet.Hash (types/validator_set.go:347-353) for n_sets ed25519 validator sets:
 * set s = validators [set_off[s], set_off[s+1]) in set order; leaves are
 * Validator.Bytes() = SimpleValidator{PubKey ed25519, VotingPower} (types/validator.go:117-133),
 * encoded on the device.  out: n_sets x 32 bytes.
 */
int tmed_valset_hashes(tmed_ctx *ctx, const uint8_t *pubkeys, const int64_t *powers, const uint32_t *set_off,
                       size_t n_sets, uint8_t *out);

/* Header fields hashed by Header.Hash (types/block.go:440-475), in struct order. */
typedef struct {
  uint64_t version_block, version_app;  /* tmversion.Consensus */
  const char *chain_id;
  uint32_t chain_id_len;
  int64_t height;
  int64_t time_seconds;                 /* Time.Unix() */
  int32_t time_nanos;                   /* Time.Nanosecond() */
  tmed_block_id last_block_id;
  /* LastCommitHash, DataHash, ValidatorsHash, NextValidatorsHash, ConsensusHash, AppHash,
     LastResultsHash, EvidenceHash, ProposerAddress */
  const uint8_t *hashes[9];
  uint32_t hash_lens[9];
} tmed_header;

/*
 * Header.Hash for n headers: out[i] (32 bytes) with ok[i] = 1, or ok[i] = 0 where the
 * reference returns nil (empty ValidatorsHash, :441-443).  Leaves are encoded on the host
 * (gogoproto wrappers as cdcEncode, types/encoding_helper.go), hashed on the device.
 */
int tmed_header_hashes(tmed_ctx *ctx, const tmed_header *headers, size_t n, uint8_t *out, uint8_t *ok);

/*
 * PartSet root hash of n_blocks byte strings (NewPartSetFromData, types/part_set.go:166-194):
 * block b = data[data_off[b] .. data_off[b+1]) split into part_size chunks
 * (types.BlockPartSizeBytes = 65536 in the reference); roots: n_blocks x 32 bytes.
 */
int tmed_partset_roots(tmed_ctx *ctx, const uint8_t *data, const uint64_t *data_off, size_t n_blocks,
                       uint32_t part_size, uint8_t *roots);

/* ------------------------------------------------- blocksync replay (f4) */

/*
 * A window of blocks for the blocksync reactor: for each block h of the
 * window, the reactor's check  state.Validators.VerifyCommitLight(chainID, firstID,
 * first.Height, second.LastCommit)  (blockchain/v0/reactor.go:366-367, with first/second
 * from pool.PeekTwoBlocks, pool.go:193-205).  All blocks of a window are verified against
 * the same validator set (the state's set, predicted for the window; the reactor confirms
 * ValidatorsHash as it applies each block and re-verifies from there if the set changed).
 */
typedef struct {
  const char *chain_id;
  uint32_t chain_id_len;
  const tmed_valset *vals;          /* use a key-set handle for the key-cached kernels */
  size_t n_blocks;
  const tmed_block_id *block_ids;   /* firstID of each block */
  const int64_t *heights;           /* first.Height */
  const tmed_commit *commits;       /* second.LastCommit */
} tmed_blocksync_window;

/*
 * out[h] = the VerifyCommitLight outcome for block h — identical to tmed_verify_commits
 * over TMED_MODE_LIGHT requests — computed speculatively for the whole window, so the
 * caller applies blocks in order and stops at the first non-OK one (the reactor then
 * redoes that request, reactor.go:368-388).  The window is processed in device batches
 * of batch_blocks blocks (0 = 128, the measured best) through a pipeline of up to three batches:
 * while the device verifies batch b, the host plans and stages batch b+1 and replays batch b-2.
 */
int tmed_blocksync_verify(tmed_ctx *ctx, const tmed_blocksync_window *w, uint32_t batch_blocks,
                          tmed_commit_result *out);

/*
 * The same as a stream of windows: a replay that verifies its backlog window after window
 * (blockchain/v0/reactor.go:349-418 over the pool's pending blocks, pool.go:31-34) submits window
 * w+1 before it consumes window w.  tmed_blocksync_submit queues the window's batches behind the
 * context's batches in flight and returns once the results of every EARLIER submitted window are
 * final in their `out` arrays; the window's own last batches may still be in flight, so the device
 * is never drained between windows (a call per window drains the pipeline and refills it: the
 * first batch's planning and copy-in).  tmed_blocksync_wait collects everything submitted and
 * returns the first error of any submitted window (or TMED_OK).  Until the window's results are
 * final, `out` and the memory the window's structs point to (block hashes, the commits' arrays —
 * signatures in pinned memory are DMA'd from there — and the set's keys, powers and addresses)
 * must stay valid and unchanged; the structs themselves (the window, its block_ids / heights /
 * commits arrays, the tmed_valset, the chain ID) are copied by submit.  Any other seam call on the context
 * (tmed_verify_commits, tmed_blocksync_verify) first collects every submitted window.
 * Results are identical to tmed_blocksync_verify on each window.
 */
int tmed_blocksync_submit(tmed_ctx *ctx, const tmed_blocksync_window *w, uint32_t batch_blocks,
                          tmed_commit_result *out);
int tmed_blocksync_wait(tmed_ctx *ctx);

/*
 * Pinned (page-locked) host memory for the commit arrays a caller marshals its commits into
 * (the Go shim flattens every Commit into sigs / flags / timestamps arrays anyway).  When a
 * candidate run's signatures lie in such memory, a large seam batch (tmed_blocksync_verify,
 * tmed_verify_commits) DMAs them straight from the caller's array to the device instead of
 * copying them through the library's pinned staging area first: one pass over host memory
 * instead of three (read, staging write, DMA read) for 64 of the 85 bytes staged per vote.
 * Decisions are identical either way.  tmed_host_alloc: hipHostMalloc'd memory (*p, freed with
 * tmed_host_free); tmed_host_register: page-lock existing memory (hipHostRegister; undo with
 * tmed_host_unregister before freeing it).  Process-wide, any context.
 */
int tmed_host_alloc(size_t bytes, void **p);
int tmed_host_free(void *p);
int tmed_host_register(void *p, size_t bytes);
int tmed_host_unregister(void *p);

/* ------------------------------------------ several GPUs in ONE process (§8e) */

/*
 * A Tendermint node is one process: with one context per GPU (tmed_init(0..N-1)), these
 * split the work into contiguous shards balanced by signature count, run every shard on
 * its own context concurrently, and write each result in place — no collective is needed
 * because the host memory is shared.  Results are identical to the single-context calls.
 * A key-set handle in a request must be loaded on EVERY context under the same handle
 * value (load the set on each context in the same order).  Returns the first error.
 */
int tmed_verify_commits_multi(tmed_ctx *const *ctxs, size_t n_ctx, const tmed_commit_request *reqs, size_t n,
                              tmed_commit_result *out);
int tmed_blocksync_verify_multi(tmed_ctx *const *ctxs, size_t n_ctx, const tmed_blocksync_window *w,
                                uint32_t batch_blocks, tmed_commit_result *out);

#ifdef __cplusplus
}
#endif
#endif /* TMED25519_H */
