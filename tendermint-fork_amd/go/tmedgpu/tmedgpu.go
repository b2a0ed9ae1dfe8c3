// Package tmedgpu is the reference-side cgo binding of libtmed25519_hip.so
// (include/tmed25519.h) for Tendermint Core v0.34.24.
//
// It is NOT compiled in this repository (no Go toolchain in the build image); tools/go_cgo_check.py
// type-checks it statically against include/tmed25519.h instead (tests/test_go_binding.py).  It is
// the shim a maintainer adds under github.com/tendermint/tendermint/crypto/ to route the
// commit-verification loops to the GPU.  See INTEGRATION.md.
//
// Seam (SURVEY.md §8b): ValidatorSet.VerifyCommit / VerifyCommitLight /
// VerifyCommitLightTrusting (types/validator_set.go:667-826) call
// VerifyCommitsGPU instead of looping over crypto.PubKey.VerifySignature
// (crypto/ed25519/ed25519.go:148-155).  Any error returned here means "take the
// original Go path": the caller never guesses a decision.
package tmedgpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../lib -ltmed25519_hip -Wl,-rpath,${SRCDIR}/../../lib
#include <stdlib.h>
#include "tmed25519.h"
*/
import "C"

import (
	"errors"
	"sync"
	"unsafe"
)

// Engine wraps one tmed_ctx (one per GPU; safe for concurrent use: the
// library serialises calls on a context).
type Engine struct {
	ctx *C.tmed_ctx
	// page-locked arena the blocksync signatures are marshalled into (grow-only, kept across
	// calls): the library DMAs them from it instead of copying them through its staging area
	pinMu  sync.Mutex
	pin    unsafe.Pointer
	pinCap int
	arenas chan *arena // reusable C arenas (getArena / putArena)
}

func newEngine(ctx *C.tmed_ctx) *Engine { return &Engine{ctx: ctx, arenas: make(chan *arena, 8)} }

// pinnedSigs returns the engine's pinned arena grown to at least n bytes (nil if
// tmed_host_alloc fails: the caller then marshals into ordinary C memory).  Holds pinMu.
func (e *Engine) pinnedSigs(n int) unsafe.Pointer {
	if n > e.pinCap {
		if e.pin != nil {
			C.tmed_host_free(e.pin)
			e.pin, e.pinCap = nil, 0
		}
		var p unsafe.Pointer
		if C.tmed_host_alloc(C.size_t(n+n/4), &p) != 0 {
			return nil
		}
		e.pin, e.pinCap = p, n+n/4
	}
	return e.pin
}

var (
	once    sync.Once
	defEng  *Engine
	initErr error
)

// Default returns the process-wide engine on device 0 (or the init error).
func Default() (*Engine, error) {
	once.Do(func() {
		var ctx *C.tmed_ctx
		if rc := C.tmed_init(0, &ctx); rc != 0 {
			initErr = errors.New(C.GoString(C.tmed_strerror(rc)))
			return
		}
		defEng = newEngine(ctx)
	})
	return defEng, initErr
}

// Mode selects the reference loop being replaced.
type Mode int

const (
	ModeCommit         Mode = C.TMED_MODE_COMMIT
	ModeLight          Mode = C.TMED_MODE_LIGHT
	ModeLightTrusting  Mode = C.TMED_MODE_LIGHT_TRUSTING
)

// Outcome codes (see tmed25519.h); the caller formats the same errors Go does.
const (
	OK              = C.TMED_COMMIT_OK
	WrongSetSize    = C.TMED_COMMIT_WRONG_SET_SIZE
	WrongHeight     = C.TMED_COMMIT_WRONG_HEIGHT
	WrongBlockID    = C.TMED_COMMIT_WRONG_BLOCK_ID
	WrongSignature  = C.TMED_COMMIT_WRONG_SIGNATURE
	NotEnoughPower  = C.TMED_COMMIT_NOT_ENOUGH_POWER
	DoubleVote      = C.TMED_COMMIT_DOUBLE_VOTE
	ZeroDenominator = C.TMED_COMMIT_ZERO_DENOMINATOR
	Overflow        = C.TMED_COMMIT_OVERFLOW
	// Panic: the reference loop panics when it reaches signature Idx (unknown BlockIDFlag,
	// malformed BlockID hash); the caller runs the original Go method, which panics as before.
	Panic = C.TMED_COMMIT_PANIC
)

// ValSet / CommitData are flat copies of types.ValidatorSet / types.Commit
// (filled by the caller in package types, which owns those types).
type ValSet struct {
	PubKeys     []byte  // n x 32
	Powers      []int64 // n
	Addresses   []byte  // n x 20 (every Validator.Address is 20 bytes; see verifyCommitGPU)
	TotalPower  int64
	Keyset      uint64   // 0: the engine's key-set cache decides (the default); or a LoadKeyset handle
	KeysetIndex []uint32 // nil, or validator i -> index in the key set
	// nil, or ValidatorSet.Hash() (types/validator_set.go:347-353) when the caller has it at no cost
	// (a header's ValidatorsHash after its check): the key-set cache's key for this set.  Without it
	// the library keys the set by a digest of PubKeys; a hit is compared key by key either way.
	SetHash []byte
	cmem    bool // PubKeys / Powers / Addresses already live in C memory (Batch.NewValSet)
}

// valset builds the C struct of v (its slices copied into the arena).
func (a *arena) valset(v *ValSet) C.tmed_valset {
	var sh *C.uint8_t
	if len(v.SetHash) == 32 {
		sh = a.bytes(v.SetHash)
	}
	t := C.tmed_valset{n: C.size_t(len(v.Powers)), total_power: C.int64_t(v.TotalPower), keyset: C.uint64_t(v.Keyset),
		keyset_index: a.u32(v.KeysetIndex), set_hash: sh}
	if v.cmem {
		t.pubkeys, t.addresses = ptr8(v.PubKeys), ptr8(v.Addresses)
		if len(v.Powers) > 0 {
			t.powers = (*C.int64_t)(unsafe.Pointer(&v.Powers[0]))
		}
	} else {
		t.pubkeys, t.powers, t.addresses = a.bytes(v.PubKeys), a.i64(v.Powers), a.bytes(v.Addresses)
	}
	return t
}

type BlockID struct {
	Hash     []byte
	PSHTotal uint32
	PSHHash  []byte
}

type CommitData struct {
	Height    int64
	Round     int32
	BlockID   BlockID
	Flags     []byte  // BlockIDFlag per signature
	Addresses []byte  // n x 20 (zero-padded slots; AddrLens gives the real lengths)
	AddrLens  []uint32 // len(ValidatorAddress) per signature: only 20 can match (bytes.Equal)
	TsSeconds []int64
	TsNanos   []int32
	Sigs      []byte // n x 64 (zero padded)
	SigLens   []uint32
	cmem      bool // every array already lives in C memory (Batch.NewCommit / WindowBuilder.NewCommit)
}

// newCommitIn: a CommitData of n signatures whose arrays are allocated in C memory (the arena;
// Sigs at sigs when given: a pinned buffer) for the caller to fill in place — the shim then hands
// the library those pointers with no second copy.
func newCommitIn(a *arena, n int, sigs unsafe.Pointer) *CommitData {
	c := &CommitData{cmem: true}
	c.Flags = unsafe.Slice((*byte)(a.alloc(uintptr(n))), n)
	c.Addresses = unsafe.Slice((*byte)(a.alloc(uintptr(20*n))), 20*n)
	c.AddrLens = unsafe.Slice((*uint32)(a.alloc(uintptr(4*n))), n)
	c.TsSeconds = unsafe.Slice((*int64)(a.alloc(uintptr(8*n))), n)
	c.TsNanos = unsafe.Slice((*int32)(a.alloc(uintptr(4*n))), n)
	if sigs == nil {
		sigs = a.alloc(uintptr(64 * n))
	}
	c.Sigs = unsafe.Slice((*byte)(sigs), 64*n)
	c.SigLens = unsafe.Slice((*uint32)(a.alloc(uintptr(4*n))), n)
	return c
}

func newValSetIn(a *arena, n int) *ValSet {
	v := &ValSet{cmem: true}
	v.PubKeys = unsafe.Slice((*byte)(a.alloc(uintptr(32*n))), 32*n)
	v.Powers = unsafe.Slice((*int64)(a.alloc(uintptr(8*n))), n)
	v.Addresses = unsafe.Slice((*byte)(a.alloc(uintptr(20*n))), 20*n)
	return v
}

func ptr8(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// commitC: the C struct of c (its arrays passed as they are when they live in C memory, else
// copied into the arena once).  sigs: where the signatures go instead (nil: as above).
func (a *arena) commitC(c *CommitData, sigs *C.uint8_t) C.tmed_commit {
	t := C.tmed_commit{height: C.int64_t(c.Height), round: C.int32_t(c.Round), block_id: a.blockID(&c.BlockID),
		n_sigs: C.size_t(len(c.Flags))}
	if c.cmem {
		t.flags, t.addresses, t.sigs = ptr8(c.Flags), ptr8(c.Addresses), ptr8(c.Sigs)
		if len(c.Flags) > 0 {
			t.ts_seconds = (*C.int64_t)(unsafe.Pointer(&c.TsSeconds[0]))
			t.ts_nanos = (*C.int32_t)(unsafe.Pointer(&c.TsNanos[0]))
			t.sig_lens = (*C.uint32_t)(unsafe.Pointer(&c.SigLens[0]))
			t.address_lens = (*C.uint32_t)(unsafe.Pointer(&c.AddrLens[0]))
		}
	} else {
		t.flags, t.addresses, t.sigs = a.bytes(c.Flags), a.bytes(c.Addresses), a.bytes(c.Sigs)
		t.ts_seconds, t.ts_nanos = a.i64(c.TsSeconds), a.i32(c.TsNanos)
		t.sig_lens, t.address_lens = a.u32(c.SigLens), a.u32(c.AddrLens)
	}
	if sigs != nil {
		t.sigs = sigs
	}
	return t
}

type Request struct {
	Mode       Mode
	ChainID    string
	Vals       *ValSet
	BlockID    *BlockID
	Height     int64
	Commit     *CommitData
	TrustNum   int64
	TrustDen   int64
}

type Result struct {
	Code                   int
	Got, Needed            int64
	Expected, Actual       int64
	Idx, IdxFirst, ValIdx  int32
}

// cgo pointer rules (Go 1.18: no runtime.Pinner): C memory must not hold Go pointers, so every
// input the library reads lives in C memory for the duration of the call.  An arena is a bump
// allocator over C blocks that are KEPT across calls (Engine.getArena / putArena): a call costs no
// malloc per array and no fresh pages.  The flat arrays of a Batch's commits and validator sets
// are allocated in the arena first and filled by the caller in place (NewCommit / NewValSet: Go
// slices over C memory), so nothing is copied twice; slices the caller built in Go memory (the
// Request form) are copied in once.
type arena struct {
	blocks []unsafe.Pointer // C blocks, reused after reset
	sizes  []uintptr
	cur    int     // block being filled
	off    uintptr // offset in it
}

const arenaBlock = 8 << 20

func (a *arena) alloc(sz uintptr) unsafe.Pointer {
	sz = (sz + 15) &^ 15
	for a.cur < len(a.blocks) {
		if a.off+sz <= a.sizes[a.cur] {
			p := unsafe.Add(a.blocks[a.cur], a.off)
			a.off += sz
			return p
		}
		a.cur++
		a.off = 0
	}
	n := uintptr(arenaBlock)
	if sz > n {
		n = sz
	}
	p := C.malloc(C.size_t(n))
	a.blocks = append(a.blocks, p)
	a.sizes = append(a.sizes, n)
	a.cur, a.off = len(a.blocks)-1, sz
	return p
}

// inArena: b already lives in this arena's C memory (filled in place): pass it as is.
func (a *arena) inArena(b unsafe.Pointer) bool {
	for i, blk := range a.blocks {
		if uintptr(b) >= uintptr(blk) && uintptr(b) < uintptr(blk)+a.sizes[i] {
			return true
		}
	}
	return false
}

func (a *arena) bytes(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	if a.inArena(unsafe.Pointer(&b[0])) {
		return (*C.uint8_t)(unsafe.Pointer(&b[0]))
	}
	p := a.alloc(uintptr(len(b)))
	copy(unsafe.Slice((*byte)(p), len(b)), b)
	return (*C.uint8_t)(p)
}

func (a *arena) i64(v []int64) *C.int64_t {
	if len(v) == 0 {
		return nil
	}
	if a.inArena(unsafe.Pointer(&v[0])) {
		return (*C.int64_t)(unsafe.Pointer(&v[0]))
	}
	p := a.alloc(uintptr(len(v)) * 8)
	copy(unsafe.Slice((*int64)(p), len(v)), v)
	return (*C.int64_t)(p)
}

func (a *arena) i32(v []int32) *C.int32_t {
	if len(v) == 0 {
		return nil
	}
	if a.inArena(unsafe.Pointer(&v[0])) {
		return (*C.int32_t)(unsafe.Pointer(&v[0]))
	}
	p := a.alloc(uintptr(len(v)) * 4)
	copy(unsafe.Slice((*int32)(p), len(v)), v)
	return (*C.int32_t)(p)
}

func (a *arena) u32(v []uint32) *C.uint32_t {
	if len(v) == 0 {
		return nil
	}
	if a.inArena(unsafe.Pointer(&v[0])) {
		return (*C.uint32_t)(unsafe.Pointer(&v[0]))
	}
	p := a.alloc(uintptr(len(v)) * 4)
	copy(unsafe.Slice((*uint32)(p), len(v)), v)
	return (*C.uint32_t)(p)
}

func (a *arena) cstring(s string) *C.char {
	p := a.alloc(uintptr(len(s)) + 1)
	b := unsafe.Slice((*byte)(p), len(s)+1)
	copy(b, s)
	b[len(s)] = 0
	return (*C.char)(p)
}

// reset keeps the blocks for the next call; free returns them to C.
func (a *arena) reset() { a.cur, a.off = 0, 0 }

func (a *arena) free() {
	for _, p := range a.blocks {
		C.free(p)
	}
	a.blocks, a.sizes = nil, nil
	a.reset()
}

// getArena / putArena: a small free list of arenas per engine (calls may run concurrently).
func (e *Engine) getArena() *arena {
	select {
	case a := <-e.arenas:
		a.reset()
		return a
	default:
		return &arena{}
	}
}

func (e *Engine) putArena(a *arena) {
	select {
	case e.arenas <- a:
	default:
		a.free()
	}
}

func (a *arena) blockID(b *BlockID) C.tmed_block_id {
	return C.tmed_block_id{hash: a.bytes(b.Hash), hash_len: C.uint32_t(len(b.Hash)), psh_total: C.uint32_t(b.PSHTotal),
		psh_hash: a.bytes(b.PSHHash), psh_hash_len: C.uint32_t(len(b.PSHHash))}
}

// LoadKeyset decodes a validator set's keys once and builds their comb tables in HBM.
func (e *Engine) LoadKeyset(pubKeys []byte) (uint64, error) {
	a := e.getArena()
	defer e.putArena(a)
	var h C.uint64_t
	if rc := C.tmed_keyset_load(e.ctx, a.bytes(pubKeys), C.size_t(len(pubKeys)/32), &h); rc != 0 {
		return 0, errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	return uint64(h), nil
}

// FreeKeyset releases a key set.
func (e *Engine) FreeKeyset(h uint64) { C.tmed_keyset_free(e.ctx, C.uint64_t(h)) }

// ExtendKeyset appends keys to a key set; existing keys keep their indexes, the new ones start at
// the returned index (tmed_keyset_extend).
func (e *Engine) ExtendKeyset(h uint64, pubKeys []byte) (uint32, error) {
	a := e.getArena()
	defer e.putArena(a)
	var first C.uint32_t
	if rc := C.tmed_keyset_extend(e.ctx, C.uint64_t(h), a.bytes(pubKeys), C.size_t(len(pubKeys)/32), &first); rc != 0 {
		return 0, errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	return uint32(first), nil
}

// KeyCacheConfig turns the engine's key-set cache on or off (enabled < 0: unchanged) and sets its
// HBM budget (0: unchanged).  It is on by default: sets passed without a handle reach the
// key-cached kernels from their second call on (tmed_keycache_config).
func (e *Engine) KeyCacheConfig(enabled int, budgetBytes uint64) error {
	if rc := C.tmed_keycache_config(e.ctx, C.int(enabled), C.size_t(budgetBytes)); rc != 0 {
		return errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	return nil
}

// KeyCacheStats returns the cache's counters (tmed_keycache_counters).
func (e *Engine) KeyCacheStats() (C.tmed_keycache_counters, error) {
	var st C.tmed_keycache_counters
	if rc := C.tmed_keycache_stats(e.ctx, &st); rc != 0 {
		return st, errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	return st, nil
}

// WarmKeyCache builds a set's missing keys now — e.g. when EndBlock changes the validator set —
// so that even its first commit is keyed (tmed_keycache_warm).
func (e *Engine) WarmKeyCache(v *ValSet) error {
	a := e.getArena()
	defer e.putArena(a)
	cv := a.valset(v)
	if rc := C.tmed_keycache_warm(e.ctx, &cv); rc != 0 {
		return errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	return nil
}

// VerifyCommits verifies many commits with ONE device batch.
func (e *Engine) VerifyCommits(reqs []Request) ([]Result, error) {
	return e.verifyCommitsWith(reqs, func(a *arena, creqs *C.tmed_commit_request, n C.size_t,
		res *C.tmed_commit_result) C.int {
		return C.tmed_verify_commits(e.ctx, creqs, n, res)
	})
}

func (e *Engine) verifyCommitsWith(reqs []Request, call func(*arena, *C.tmed_commit_request, C.size_t,
	*C.tmed_commit_result) C.int) ([]Result, error) {
	a := e.getArena()
	defer e.putArena(a)
	return e.verifyIn(a, reqs, call)
}

func (e *Engine) verifyIn(a *arena, reqs []Request, call func(*arena, *C.tmed_commit_request, C.size_t,
	*C.tmed_commit_result) C.int) ([]Result, error) {
	n := len(reqs)
	if n == 0 {
		return nil, nil
	}
	creqs := (*[1 << 26]C.tmed_commit_request)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_commit_request{})))[:n:n]
	vs := (*[1 << 26]C.tmed_valset)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_valset{})))[:n:n]
	cs := (*[1 << 26]C.tmed_commit)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_commit{})))[:n:n]
	bids := (*[1 << 26]C.tmed_block_id)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_block_id{})))[:n:n]
	// one C copy per distinct *ValSet: requests on the same set share it (the library resolves each
	// set once per call; a light-client batch holds each set twice)
	seen := make(map[*ValSet]*C.tmed_valset, n)
	// one C copy per distinct *CommitData as well: the light client's Trusting + Light pair checks
	// one commit twice, and the library verifies a signature the two share once (same commit)
	seenC := make(map[*CommitData]*C.tmed_commit, n)
	for i := range reqs {
		r := &reqs[i]
		cv, ok := seen[r.Vals]
		if !ok {
			vs[i] = a.valset(r.Vals)
			cv = &vs[i]
			seen[r.Vals] = cv
		}
		c := r.Commit
		cc, ok := seenC[c]
		if !ok {
			cs[i] = a.commitC(c, nil)
			cc = &cs[i]
			seenC[c] = cc
		}
		bids[i] = C.tmed_block_id{}
		if r.BlockID != nil {
			bids[i] = a.blockID(r.BlockID)
		}
		cid := a.cstring(r.ChainID)
		creqs[i] = C.tmed_commit_request{mode: C.int(r.Mode), chain_id: cid, chain_id_len: C.uint32_t(len(r.ChainID)),
			vals: cv, block_id: &bids[i], height: C.int64_t(r.Height), commit: cc,
			trust_num: C.int64_t(r.TrustNum), trust_den: C.int64_t(r.TrustDen)}
	}
	res := make([]C.tmed_commit_result, n)
	if rc := call(a, &creqs[0], C.size_t(n), &res[0]); rc != 0 {
		return nil, errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	return toResults(res), nil
}

// Batch is one VerifyCommits call whose commits and validator sets are flattened by the caller
// straight into C memory (NewCommit / NewValSet), so the shim copies nothing: package types fills
// them from its Commit / ValidatorSet (INTEGRATION.md §2).  Verify, then Release.
type Batch struct {
	e    *Engine
	a    *arena
	reqs []Request
}

func (e *Engine) NewBatch() *Batch { return &Batch{e: e, a: e.getArena()} }

// NewCommit: a commit of n signatures to fill in place.
func (b *Batch) NewCommit(n int) *CommitData { return newCommitIn(b.a, n, nil) }

// NewValSet: a validator set of n validators to fill in place (TotalPower / SetHash set by the caller).
func (b *Batch) NewValSet(n int) *ValSet { return newValSetIn(b.a, n) }

func (b *Batch) Add(r Request) { b.reqs = append(b.reqs, r) }

func (b *Batch) Verify() ([]Result, error) {
	return b.e.verifyIn(b.a, b.reqs, func(a *arena, creqs *C.tmed_commit_request, n C.size_t,
		res *C.tmed_commit_result) C.int {
		return C.tmed_verify_commits(b.e.ctx, creqs, n, res)
	})
}

// Release returns the batch's C memory to the engine (the CommitData / ValSet it made are invalid after).
func (b *Batch) Release() {
	if b.a != nil {
		b.e.putArena(b.a)
		b.a, b.reqs = nil, nil
	}
}

func toResults(res []C.tmed_commit_result) []Result {
	out := make([]Result, len(res))
	for i := range res {
		out[i] = Result{Code: int(res[i].code), Got: int64(res[i].got), Needed: int64(res[i].needed),
			Expected: int64(res[i].expected), Actual: int64(res[i].actual), Idx: int32(res[i].idx),
			IdxFirst: int32(res[i].idx_first), ValIdx: int32(res[i].val_idx)}
	}
	return out
}

// BlocksyncWindow is a run of buffered blocks checked against one (predicted) validator
// set: block h is vals.VerifyCommitLight(ChainID, BlockIDs[h], Heights[h], Commits[h])
// (blockchain/v0/reactor.go:366-367).
type BlocksyncWindow struct {
	ChainID  string
	Vals     *ValSet
	BlockIDs []BlockID
	Heights  []int64
	Commits  []*CommitData
	builder  *WindowBuilder // set by WindowBuilder.Window: the commits already live in its C memory
}

// BlocksyncVerify returns the VerifyCommitLight outcome of every block of the window,
// computed speculatively through the pipelined device path (tmed_blocksync_verify).
// The reactor applies blocks in order and stops at the first non-OK result.
func (e *Engine) BlocksyncVerify(w *BlocksyncWindow, batchBlocks int) ([]Result, error) {
	n := len(w.Commits)
	if n == 0 {
		return nil, nil
	}
	a := e.getArena()
	defer e.putArena(a)
	vs := (*C.tmed_valset)(a.alloc(unsafe.Sizeof(C.tmed_valset{})))
	*vs = a.valset(w.Vals)
	cs := (*[1 << 26]C.tmed_commit)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_commit{})))[:n:n]
	bids := (*[1 << 26]C.tmed_block_id)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_block_id{})))[:n:n]
	// signatures into the pinned arena (direct DMA, include/tmed25519.h tmed_host_alloc)
	total := 0
	for _, c := range w.Commits {
		total += len(c.Sigs)
	}
	e.pinMu.Lock()
	defer e.pinMu.Unlock()
	arenaBase := e.pinnedSigs(total)
	off := 0
	for i, c := range w.Commits {
		sigs := (*C.uint8_t)(nil)
		if !c.cmem && arenaBase != nil && len(c.Sigs) > 0 {
			p := unsafe.Add(arenaBase, off)
			copy(unsafe.Slice((*byte)(p), len(c.Sigs)), c.Sigs)
			sigs, off = (*C.uint8_t)(p), off+len(c.Sigs)
		}
		cs[i] = a.commitC(c, sigs)
		bids[i] = a.blockID(&w.BlockIDs[i])
	}
	cid := a.cstring(w.ChainID)
	win := (*C.tmed_blocksync_window)(a.alloc(unsafe.Sizeof(C.tmed_blocksync_window{})))
	*win = C.tmed_blocksync_window{chain_id: cid, chain_id_len: C.uint32_t(len(w.ChainID)), vals: vs,
		n_blocks: C.size_t(n), block_ids: &bids[0], heights: a.i64(w.Heights), commits: &cs[0]}
	res := make([]C.tmed_commit_result, n)
	if rc := C.tmed_blocksync_verify(e.ctx, win, C.uint32_t(batchBlocks), &res[0]); rc != 0 {
		return nil, errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	return toResults(res), nil
}

// PendingWindow is a window queued by BlocksyncSubmit.  Its results are final once a LATER
// BlocksyncSubmit or BlocksyncWait on the same engine has returned; until then its C copies and
// its pinned signature buffer stay allocated (the library DMAs from them and writes the results
// into C memory: cgo forbids C retaining Go pointers after a call returns).
type PendingWindow struct {
	e   *Engine
	a   *arena
	pin unsafe.Pointer
	res *C.tmed_commit_result
	n   int
}

// BlocksyncSubmit queues a window behind the engine's windows in flight (tmed_blocksync_submit):
// the reactor's replay submits window w+1 before it applies window w, so the device is never
// drained between windows.  When it returns, every earlier submitted window's Results are final.
func (e *Engine) BlocksyncSubmit(w *BlocksyncWindow, batchBlocks int) (*PendingWindow, error) {
	n := len(w.Commits)
	if w.builder != nil { // built in place (NewWindow): its arena and pinned buffer travel with it
		return w.builder.submit(w, batchBlocks)
	}
	p := &PendingWindow{e: e, n: n, a: e.getArena()}
	if n == 0 {
		return p, nil
	}
	return p.submit(w, batchBlocks, true)
}

// submit marshals w into p's arena (signatures into p.pin when copyPin) and queues it.
func (p *PendingWindow) submit(w *BlocksyncWindow, batchBlocks int, copyPin bool) (*PendingWindow, error) {
	e, a, n := p.e, p.a, len(w.Commits)
	vs := (*C.tmed_valset)(a.alloc(unsafe.Sizeof(C.tmed_valset{})))
	*vs = a.valset(w.Vals)
	cs := (*[1 << 26]C.tmed_commit)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_commit{})))[:n:n]
	bids := (*[1 << 26]C.tmed_block_id)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_block_id{})))[:n:n]
	total := 0
	for _, c := range w.Commits {
		total += len(c.Sigs)
	}
	// a pinned buffer per window in flight (the engine's shared arena serves synchronous calls)
	if copyPin && total > 0 && C.tmed_host_alloc(C.size_t(total), &p.pin) != 0 {
		p.pin = nil
	}
	off := 0
	for i, c := range w.Commits {
		sigs := (*C.uint8_t)(nil)
		if copyPin && !c.cmem && p.pin != nil && len(c.Sigs) > 0 {
			q := unsafe.Add(p.pin, off)
			copy(unsafe.Slice((*byte)(q), len(c.Sigs)), c.Sigs)
			sigs, off = (*C.uint8_t)(q), off+len(c.Sigs)
		}
		cs[i] = a.commitC(c, sigs)
		bids[i] = a.blockID(&w.BlockIDs[i])
	}
	cid := a.cstring(w.ChainID)
	win := (*C.tmed_blocksync_window)(a.alloc(unsafe.Sizeof(C.tmed_blocksync_window{})))
	*win = C.tmed_blocksync_window{chain_id: cid, chain_id_len: C.uint32_t(len(w.ChainID)), vals: vs,
		n_blocks: C.size_t(n), block_ids: &bids[0], heights: a.i64(w.Heights), commits: &cs[0]}
	p.res = (*C.tmed_commit_result)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_commit_result{})))
	if rc := C.tmed_blocksync_submit(e.ctx, win, C.uint32_t(batchBlocks), p.res); rc != 0 {
		p.free()
		return nil, errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	return p, nil
}

// BlocksyncWait collects every window submitted on the engine (tmed_blocksync_wait).
func (e *Engine) BlocksyncWait() error {
	if rc := C.tmed_blocksync_wait(e.ctx); rc != 0 {
		return errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	return nil
}

// Results returns the window's outcomes and releases its memory.  Call it only after a later
// BlocksyncSubmit or BlocksyncWait returned without error.  A nil window (the one a failed
// BlocksyncSubmit returns) has no results.
func (p *PendingWindow) Results() []Result {
	if p == nil {
		return nil
	}
	var out []Result
	if p.n > 0 {
		out = toResults(unsafe.Slice(p.res, p.n))
	}
	p.free() // an empty window still holds its arena (and a builder's pinned buffer)
	return out
}

func (p *PendingWindow) free() {
	if p.pin != nil {
		C.tmed_host_free(p.pin)
		p.pin = nil
	}
	if p.a != nil {
		p.e.putArena(p.a)
		p.a = nil
	}
	p.n = 0
}

// WindowBuilder lays a blocksync window out in C memory as the reactor flattens its blocks: each
// commit's arrays in the window's arena, its signatures in the window's pinned buffer (the library
// DMAs them from there), filled in place by package types (INTEGRATION.md §3: up to the
// VerifyCommitLight crossing).  Submit with BlocksyncSubmit(w.Window(...)).
type WindowBuilder struct {
	p   *PendingWindow
	off uintptr
	cap uintptr
}

// NewWindow: room for maxSigs signatures over the window's commits.
func (e *Engine) NewWindow(maxSigs int) *WindowBuilder {
	b := &WindowBuilder{p: &PendingWindow{e: e, a: e.getArena()}}
	if maxSigs > 0 && C.tmed_host_alloc(C.size_t(64*maxSigs), &b.p.pin) != 0 {
		b.p.pin = nil // no page-locked memory: the signatures go to the arena (the library stages them)
	}
	if b.p.pin != nil {
		b.cap = uintptr(64 * maxSigs)
	}
	return b
}

// NewCommit: a commit of n signatures, its Sigs in the pinned buffer when room is left.
func (b *WindowBuilder) NewCommit(n int) *CommitData {
	var sigs unsafe.Pointer
	if b.p.pin != nil && b.off+uintptr(64*n) <= b.cap {
		sigs = unsafe.Add(b.p.pin, b.off)
		b.off += uintptr(64 * n)
	}
	return newCommitIn(b.p.a, n, sigs)
}

// Window wraps the built commits for BlocksyncSubmit.
func (b *WindowBuilder) Window(chainID string, vals *ValSet, blockIDs []BlockID, heights []int64,
	commits []*CommitData) *BlocksyncWindow {
	return &BlocksyncWindow{ChainID: chainID, Vals: vals, BlockIDs: blockIDs, Heights: heights, Commits: commits,
		builder: b}
}

func (b *WindowBuilder) submit(w *BlocksyncWindow, batchBlocks int) (*PendingWindow, error) {
	p := b.p
	p.n = len(w.Commits)
	if p.n == 0 {
		return p, nil
	}
	return p.submit(w, batchBlocks, false)
}

// ValsetHashes returns ValidatorSet.Hash() of every set: set s is validators
// [setOff[s], setOff[s+1]) of (pubKeys n x 32, powers n) in set order (tmed_valset_hashes).
func (e *Engine) ValsetHashes(pubKeys []byte, powers []int64, setOff []uint32) ([][32]byte, error) {
	ns := len(setOff) - 1
	if ns <= 0 {
		return nil, nil
	}
	a := e.getArena()
	defer e.putArena(a)
	out := (*[1 << 26][32]byte)(a.alloc(uintptr(ns) * 32))[:ns:ns]
	if rc := C.tmed_valset_hashes(e.ctx, a.bytes(pubKeys), a.i64(powers), a.u32(setOff), C.size_t(ns),
		(*C.uint8_t)(unsafe.Pointer(&out[0]))); rc != 0 {
		return nil, errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	return append([][32]byte(nil), out...), nil
}

// MerkleRoots returns merkle.HashFromByteSlices of every tree (tmed_merkle_roots).
func (e *Engine) MerkleRoots(trees [][][]byte) ([][32]byte, error) {
	nt := len(trees)
	if nt == 0 {
		return nil, nil
	}
	var flat []byte
	leafOff := []uint64{0}
	treeOff := []uint32{0}
	for _, t := range trees {
		for _, l := range t {
			flat = append(flat, l...)
			leafOff = append(leafOff, uint64(len(flat)))
		}
		treeOff = append(treeOff, uint32(len(leafOff)-1))
	}
	flat = append(flat, make([]byte, 8)...) // the device reader may touch the last dword
	a := e.getArena()
	defer e.putArena(a)
	lo := (*[1 << 26]C.uint64_t)(a.alloc(uintptr(len(leafOff)) * 8))[:len(leafOff):len(leafOff)]
	for i, v := range leafOff {
		lo[i] = C.uint64_t(v)
	}
	out := (*[1 << 26][32]byte)(a.alloc(uintptr(nt) * 32))[:nt:nt]
	if rc := C.tmed_merkle_roots(e.ctx, a.bytes(flat), &lo[0], a.u32(treeOff), C.size_t(nt),
		(*C.uint8_t)(unsafe.Pointer(&out[0]))); rc != 0 {
		return nil, errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	return append([][32]byte(nil), out...), nil
}

// VoteSignBytes returns Commit.VoteSignBytes for n votes of one commit (tmed_vote_sign_bytes;
// types/block.go:807-810 -> types/vote.go:93-101): vote i has flag flags[i] and timestamp
// (tsSec[i], tsNanos[i]).  The seam builds these itself (on the device); this is for callers and
// tests that sign synthetic commits.
func (e *Engine) VoteSignBytes(chainID string, height int64, round int32, bid *BlockID, flags []byte,
	tsSec []int64, tsNanos []int32) ([][]byte, error) {
	n := len(flags)
	if len(tsSec) != n || len(tsNanos) != n {
		return nil, errors.New("tmedgpu: one flag and one timestamp per vote")
	}
	if n == 0 {
		return nil, nil
	}
	a := e.getArena()
	defer e.putArena(a)
	t := (*C.tmed_vote_template)(a.alloc(unsafe.Sizeof(C.tmed_vote_template{})))
	*t = C.tmed_vote_template{chain_id: a.cstring(chainID), chain_id_len: C.uint32_t(len(chainID)),
		height: C.int64_t(height), round: C.int32_t(round), block_hash: a.bytes(bid.Hash),
		block_hash_len: C.uint32_t(len(bid.Hash)), psh_total: C.uint32_t(bid.PSHTotal), psh_hash: a.bytes(bid.PSHHash),
		psh_hash_len: C.uint32_t(len(bid.PSHHash))}
	fl, sec, ns := a.bytes(flags), a.i64(tsSec), a.i32(tsNanos)
	off := (*[1 << 26]C.uint32_t)(a.alloc(uintptr(n+1) * 4))[: n+1 : n+1]
	var total C.size_t
	if rc := C.tmed_vote_sign_bytes(t, C.size_t(n), fl, sec, ns, nil, 0, &off[0], &total); rc != 0 {
		return nil, errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	buf := (*C.uint8_t)(a.alloc(uintptr(total) + 1))
	if rc := C.tmed_vote_sign_bytes(t, C.size_t(n), fl, sec, ns, buf, total, &off[0], &total); rc != 0 {
		return nil, errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	flat := unsafe.Slice((*byte)(unsafe.Pointer(buf)), int(total))
	out := make([][]byte, n)
	for i := range out {
		out[i] = append([]byte(nil), flat[off[i]:off[i+1]]...)
	}
	return out, nil
}

// batchArgs packs n (pubkey, message, signature) tuples for tmed_verify_batch(_zip215):
// pubKeys n x 32, sigs as given (the lengths travel so a wrong-length signature is rejected
// exactly as ed25519.Verify rejects it), messages concatenated with offsets.
func batchArgs(a *arena, pubKeys []byte, msgs, sigs [][]byte) (pk, sg *C.uint8_t, sl *C.uint32_t,
	mg *C.uint8_t, mo *C.uint32_t) {
	n := len(msgs)
	sigBuf := make([]byte, 64*n)
	lens := make([]uint32, n)
	off := make([]uint32, n+1)
	var flat []byte
	for i := 0; i < n; i++ {
		copy(sigBuf[64*i:64*i+64], sigs[i])
		lens[i] = uint32(len(sigs[i]))
		flat = append(flat, msgs[i]...)
		off[i+1] = uint32(len(flat))
	}
	flat = append(flat, make([]byte, 16)...) // the device reader may touch past the last message
	return a.bytes(pubKeys), a.bytes(sigBuf), a.u32(lens), a.bytes(flat), a.u32(off)
}

// VerifyBatch returns ed25519.Verify (Go 1.18 rule, crypto/ed25519/ed25519.go:148-155) of every
// tuple (tmed_verify_batch).
func (e *Engine) VerifyBatch(pubKeys []byte, msgs, sigs [][]byte) ([]bool, error) {
	return e.batch(pubKeys, msgs, sigs, false)
}

// VerifyBatchZIP215 returns the ZIP-215 decision of every tuple (tmed_verify_batch_zip215):
// OPT-IN, for chains that adopt the rule of spec/core/encoding.md:52-54.
func (e *Engine) VerifyBatchZIP215(pubKeys []byte, msgs, sigs [][]byte) ([]bool, error) {
	return e.batch(pubKeys, msgs, sigs, true)
}

func (e *Engine) batch(pubKeys []byte, msgs, sigs [][]byte, zip215 bool) ([]bool, error) {
	n := len(msgs)
	if len(sigs) != n || len(pubKeys) != 32*n {
		return nil, errors.New("tmedgpu: want one 32-byte key and one signature per message")
	}
	if n == 0 {
		return nil, nil
	}
	a := e.getArena()
	defer e.putArena(a)
	pk, sg, sl, mg, mo := batchArgs(a, pubKeys, msgs, sigs)
	out := (*[1 << 28]C.uint8_t)(a.alloc(uintptr(n)))[:n:n]
	var rc C.int
	if zip215 {
		rc = C.tmed_verify_batch_zip215(e.ctx, pk, sg, sl, mg, mo, C.size_t(n), &out[0])
	} else {
		rc = C.tmed_verify_batch(e.ctx, pk, sg, sl, mg, mo, C.size_t(n), &out[0])
	}
	if rc != 0 {
		return nil, errors.New(C.GoString(C.tmed_strerror(rc)))
	}
	ok := make([]bool, n)
	for i := range ok {
		ok[i] = out[i] != 0
	}
	return ok, nil
}

// Pool is one engine per GPU of the node, used from ONE process (a Tendermint node):
// tmed_verify_commits_multi / tmed_blocksync_verify_multi shard the work over the contexts
// concurrently; no collective is needed since host memory is shared.
type Pool struct{ engines []*Engine }

// NewPool opens devices 0..n-1.
func NewPool(n int) (*Pool, error) {
	p := &Pool{}
	for d := 0; d < n; d++ {
		var ctx *C.tmed_ctx
		if rc := C.tmed_init(C.int(d), &ctx); rc != 0 {
			for _, e := range p.engines {
				C.tmed_destroy(e.ctx)
			}
			return nil, errors.New(C.GoString(C.tmed_strerror(rc)))
		}
		p.engines = append(p.engines, newEngine(ctx))
	}
	return p, nil
}

func (p *Pool) ctxs(a *arena) **C.tmed_ctx {
	arr := (*[1 << 10]*C.tmed_ctx)(a.alloc(uintptr(len(p.engines)) * unsafe.Sizeof((*C.tmed_ctx)(nil))))[:len(p.engines):len(p.engines)]
	for i, e := range p.engines {
		arr[i] = e.ctx
	}
	return &arr[0]
}

// LoadKeyset loads the same key set on every GPU; the handles agree when every pool
// member loads the same sets in the same order (the pool is the only loader).
func (p *Pool) LoadKeyset(pubKeys []byte) (uint64, error) {
	var h uint64
	for i, e := range p.engines {
		hi, err := e.LoadKeyset(pubKeys)
		if err != nil {
			return 0, err
		}
		if i > 0 && hi != h {
			return 0, errors.New("tmedgpu: key-set handles diverged across GPUs")
		}
		h = hi
	}
	return h, nil
}

// VerifyCommits is Engine.VerifyCommits sharded over the pool's GPUs.
func (p *Pool) VerifyCommits(reqs []Request) ([]Result, error) {
	if len(reqs) == 0 {
		return nil, nil
	}
	// the request structs are built exactly as Engine.VerifyCommits does
	return p.engines[0].verifyCommitsWith(reqs, func(a *arena, creqs *C.tmed_commit_request, n C.size_t,
		res *C.tmed_commit_result) C.int {
		return C.tmed_verify_commits_multi(p.ctxs(a), C.size_t(len(p.engines)), creqs, n, res)
	})
}
