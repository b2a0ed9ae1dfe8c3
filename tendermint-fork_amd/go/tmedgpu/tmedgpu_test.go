package tmedgpu

// Tests a maintainer runs on a GPU box after vendoring the binding (`go test ./crypto/tmedgpu`):
// the engine's decisions against Go's own crypto/ed25519.Verify — the function x/crypto v0.1.0
// forwards to (crypto/ed25519/ed25519.go:148-155) — and the commit seam's outcomes for a commit
// signed here.  Not run in this repository (no Go toolchain); tools/go_cgo_check.py type-checks it.
// (cgo is not allowed in _test.go files: everything below goes through the package's Go API.)

import (
	"crypto/ed25519"
	"crypto/rand"
	"testing"
)

func engineOrSkip(t *testing.T) *Engine {
	eng, err := Default()
	if err != nil {
		t.Skip("no usable gfx950 device: ", err)
	}
	return eng
}

func TestVerifyBatchMatchesStdlib(t *testing.T) {
	eng := engineOrSkip(t)
	n := 3000
	pubs := make([]byte, 0, 32*n)
	msgs := make([][]byte, n)
	sigs := make([][]byte, n)
	for i := 0; i < n; i++ {
		pub, priv, err := ed25519.GenerateKey(rand.Reader)
		if err != nil {
			t.Fatal(err)
		}
		msgs[i] = []byte{byte(i), byte(i >> 8), 0x2a}
		sigs[i] = ed25519.Sign(priv, msgs[i])
		switch i % 7 {
		case 1:
			sigs[i][5] ^= 0x20 // R bit flip
		case 2:
			sigs[i][40] ^= 0x01 // S bit flip
		case 3:
			sigs[i] = sigs[i][:63] // wrong length: rejected before the device (ed25519.go:150-152)
		case 4:
			msgs[i] = append(msgs[i], 0) // message changed
		}
		pubs = append(pubs, pub...)
	}
	got, err := eng.VerifyBatch(pubs, msgs, sigs)
	if err != nil {
		t.Fatal(err)
	}
	for i := 0; i < n; i++ {
		want := ed25519.Verify(ed25519.PublicKey(pubs[32*i:32*i+32]), msgs[i], sigs[i])
		if got[i] != want {
			t.Fatalf("signature %d: engine %v, crypto/ed25519 %v", i, got[i], want)
		}
	}
}

// A commit of nv validators (equal power 10) signed over the engine's own sign-bytes; validator bad
// signs a different message.  VerifyCommitLight stops at the 2/3 crossing, so a bad signature
// before it is "wrong signature (#bad)" and one after it is never reached
// (types/validator_set.go:722-765).
func signedCommit(t *testing.T, eng *Engine, b *Batch, nv, bad int) (*ValSet, *CommitData, BlockID) {
	bid := BlockID{Hash: make([]byte, 32), PSHTotal: 1, PSHHash: make([]byte, 32)}
	bid.Hash[0], bid.PSHHash[0] = 0xab, 0xcd
	vs := b.NewValSet(nv)
	c := b.NewCommit(nv)
	c.Height, c.Round, c.BlockID = 7, 0, bid
	privs := make([]ed25519.PrivateKey, nv)
	for i := 0; i < nv; i++ {
		pub, priv, err := ed25519.GenerateKey(rand.Reader)
		if err != nil {
			t.Fatal(err)
		}
		privs[i] = priv
		copy(vs.PubKeys[32*i:], pub)
		vs.Powers[i] = 10
		vs.Addresses[20*i] = byte(i)
		c.Flags[i] = 2 // BlockIDFlagCommit
		c.AddrLens[i] = 20
		copy(c.Addresses[20*i:20*i+20], vs.Addresses[20*i:20*i+20])
		c.TsSeconds[i] = 1672531200
		c.TsNanos[i] = int32(i) * 1000000
		c.SigLens[i] = 64
	}
	vs.TotalPower = int64(10 * nv)
	msgs, err := eng.VoteSignBytes("test_chain_id", c.Height, c.Round, &bid, c.Flags, c.TsSeconds, c.TsNanos)
	if err != nil {
		t.Fatal(err)
	}
	for i := 0; i < nv; i++ {
		m := msgs[i]
		if i == bad {
			m = append([]byte(nil), m...)
			m[len(m)-1] ^= 1
		}
		copy(c.Sigs[64*i:64*i+64], ed25519.Sign(privs[i], m))
	}
	return vs, c, bid
}

func TestVerifyCommitLightOutcomes(t *testing.T) {
	eng := engineOrSkip(t)
	for _, tc := range []struct {
		bad, code int
	}{{-1, OK}, {3, WrongSignature}, {170, OK}} {
		b := eng.NewBatch()
		vs, c, bid := signedCommit(t, eng, b, 175, tc.bad)
		b.Add(Request{Mode: ModeLight, ChainID: "test_chain_id", Vals: vs, BlockID: &bid, Height: 7, Commit: c})
		res, err := b.Verify()
		b.Release()
		if err != nil {
			t.Fatal(err)
		}
		if res[0].Code != tc.code || (tc.code == WrongSignature && int(res[0].Idx) != tc.bad) {
			t.Fatalf("bad signature at %d: got code %d idx %d, want code %d", tc.bad, res[0].Code, res[0].Idx, tc.code)
		}
	}
}

func TestFailedSubmitIsNilSafe(t *testing.T) {
	var p *PendingWindow // what BlocksyncSubmit returns with an error
	if p.Results() != nil {
		t.Fatal("a nil window has no results")
	}
}
