"""Static checks of the reference-side cgo binding (tendermint-fork_amd/go/tmedgpu/tmedgpu.go) and the
Go snippets of INTEGRATION.md against include/tmed25519.h (tools/go_cgo_check.py).

There is no Go toolchain in the image, so nothing else compiles this text.  Round 5 shipped a
binding that did not type-check (`batchArgs(&a, ...)` with `a` already an `*arena`).  These tests
keep the binding green and show that each class of mistake is caught, by mutating the real text.
Seam: types/validator_set.go:667-826 -> crypto/ed25519/ed25519.go:148-155."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import go_cgo_check as gc  # noqa: E402

with open(gc.GO_FILE) as _f:
    GO = _f.read()
with open(gc.INTEGRATION) as _f:
    MD = _f.read()
with open(gc.HEADER) as _f:
    HDR = _f.read()


@pytest.fixture(scope="module")
def header():
    try:
        return gc.Header()
    except RuntimeError as e:  # no clang: nothing to check against
        pytest.skip(str(e))


with open(gc.GO_FILE[:-3] + "_test.go") as _f:
    GOTEST = _f.read()


def check(header, go=GO, md=MD, gotest=GOTEST):
    errs, pkg = gc.check_binding(go, header, extra=[("tmedgpu_test.go", gotest)])
    return errs + gc.check_snippets(md, header, pkg)


def mutate(text, old, new):
    assert old in text, old
    return text.replace(old, new, 1)


def test_binding_and_snippets_clean(header):
    assert check(header) == []


def test_checker_types_almost_every_argument(header):
    """The checker must not pass the binding by failing to type it: nearly every argument of every
    C call and package call has an inferred type that was compared."""
    errs, _ = gc.check_binding(GO, header)
    st = gc.check_binding.stats
    assert st["c_calls"] >= 50 and st["go_calls"] >= 100
    assert st["c_args_typed"] >= 0.95 * st["c_args"]
    assert st["go_args_typed"] >= 0.95 * st["go_args"]


def test_header_parse(header):
    params, res = header.funcs["tmed_blocksync_submit"]
    assert params == ["*C.tmed_ctx", "*C.tmed_blocksync_window", "C.uint32_t", "*C.tmed_commit_result"]
    assert res == "C.int"
    assert header.funcs["tmed_verify_commits_multi"][0][0] == "**C.tmed_ctx"
    assert header.funcs["tmed_host_alloc"][0] == ["C.size_t", "*unsafe.Pointer"]
    assert header.structs["tmed_commit"]["block_id"] == "C.tmed_block_id"
    assert header.structs["tmed_header"]["hashes"] == "[9]*C.uint8_t"
    assert "TMED_COMMIT_PANIC" in header.macros


def test_round5_batchargs_break_is_caught(header):
    """The round-5 break: a **arena passed where batchArgs takes *arena (tmedgpu.go batch)."""
    go = mutate(GO, "batchArgs(a, pubKeys, msgs, sigs)", "batchArgs(&a, pubKeys, msgs, sigs)")
    errs = check(header, go=go)
    assert len(errs) == 1 and "batchArgs" in errs[0] and "**arena" in errs[0]


@pytest.mark.parametrize("old,new,expect", [
    # C1: argument count and cgo types of C calls
    ("C.tmed_verify_batch(e.ctx, pk, sg, sl, mg, mo, C.size_t(n), &out[0])",
     "C.tmed_verify_batch(e.ctx, pk, sg, sl, mg, mo, &out[0])", "takes 8 arguments"),
    ("C.tmed_blocksync_submit(e.ctx, win, C.uint32_t(batchBlocks), p.res)",
     "C.tmed_blocksync_submit(e.ctx, win, C.size_t(batchBlocks), p.res)", "C.uint32_t"),
    ("C.tmed_keyset_free(e.ctx, C.uint64_t(h))", "C.tmed_keyset_free(e.ctx, h)", "argument 2 of C.tmed_keyset_free"),
    ("C.tmed_verify_commits_multi(p.ctxs(a),", "C.tmed_verify_commits_multi(p.engines[0].ctx,", "**C.tmed_ctx"),
    ("C.tmed_keycache_warm(e.ctx, &cv)", "C.tmed_keycache_warm(e.ctx, cv)", "tmed_keycache_warm"),
    ("C.tmed_valset_hashes(", "C.tmed_valset_hash(", "not declared"),
    # C2: struct fields (literal keys, selectors, assigned types)
    ("n_sigs: C.size_t(len(c.Flags))", "nsigs: C.size_t(len(c.Flags))", "no field nsigs"),
    ("Expected: int64(res[i].expected)", "Expected: int64(res[i].expect)", "no field or method expect"),
    ("t.sig_lens = (*C.uint32_t)", "t.sig_lens = (*C.int32_t)", "assigning"),
    ("chain_id_len: C.uint32_t(len(r.ChainID))", "chain_id_len: C.int(len(r.ChainID))", "chain_id_len"),
    # C3: constants
    ("Panic = C.TMED_COMMIT_PANIC", "Panic = C.TMED_COMMIT_PANICKED", "TMED_COMMIT_PANICKED"),
    # C4: package calls, pointer depth, struct fields, unused locals, returns
    ("return e.verifyIn(a, reqs, call)", "return e.verifyIn(a, call)", "takes 3 arguments"),
    ("cs[i] = a.commitC(c, nil)", "cs[i] = a.commitC(&c, nil)", "**CommitData"),
    ("*vs = a.valset(w.Vals)\n\tcs := (*[1 << 26]C.tmed_commit)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_commit{})))[:n:n]\n\tbids := (*[1 << 26]C.tmed_block_id)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_block_id{})))[:n:n]\n\t// signatures",
     "*vs = a.valset(*w.Vals)\n\tcs := (*[1 << 26]C.tmed_commit)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_commit{})))[:n:n]\n\tbids := (*[1 << 26]C.tmed_block_id)(a.alloc(uintptr(n) * unsafe.Sizeof(C.tmed_block_id{})))[:n:n]\n\t// signatures",
     "method arena.valset"),
    ("p := &PendingWindow{e: e, n: n, a: e.getArena()}", "p := &PendingWindow{e: e, n: n, arena: e.getArena()}",
     "no field arena"),
    ("\tout := make([]Result, len(res))", "\tout := make([]Result, len(res))\n\tx := 1",
     "x declared and not used"),
    ("return uint64(h), nil", "return h, nil", "returns h"),
    ("return b.e.verifyIn(b.a, b.reqs, func(a *arena, creqs *C.tmed_commit_request, n C.size_t,",
     "return b.e.verifyIn(b.a, b.reqs, func(a *arena, creqs *C.tmed_commit_request, n C.uint32_t,", "argument 3"),
])
def test_binding_mutation_is_caught(header, old, new, expect):
    errs = check(header, go=mutate(GO, old, new))
    assert errs and any(expect in e for e in errs), errs


def test_header_change_is_caught(header):
    """A field the binding writes disappears from the header (the C side changed, the Go did not)."""
    h2 = gc.Header(text=mutate(HDR, "  const uint32_t *address_lens;", "  const uint32_t *addr_lens;"))
    errs = check(h2)
    assert any("address_lens" in e for e in errs), errs


@pytest.mark.parametrize("old,new,expect", [
    # C5: the round-5 INTEGRATION snippet: p.Results() after a failed BlocksyncSubmit (p == nil)
    ("if err != nil {\n\treturn err // p is nil when the submit failed: verify these blocks on the original path\n}\n",
     "", "p may be nil"),
    ("b := eng.NewBatch()", "b := eng.NewBatchFor()", "NewBatchFor"),
    ("vs.TotalPower = vals.TotalVotingPower() // TotalVotingPower", "vs.Total = vals.TotalVotingPower() // TotalVotingPower",
     "no field or method Total"),
    ("req := tmedgpu.Request{Mode: mode,", "req := tmedgpu.Request{Mod: mode,", "no field Mod"),
    ("case tmedgpu.ZeroDenominator:", "case tmedgpu.ZeroDenom:", "ZeroDenom"),
    ("b.Add(req)", "b.add(req)", "no field or method add"),
    ("vs := b.NewValSet(len(vals.Validators))\n\tvs.TotalPower", "vs := b.NewValSet(len(vals.Validators))\n\tvs.cmem = true\n\tvs.TotalPower", "unexported"),
    ("c := wb.NewCommit(len(lc.Signatures))", "c := wb.NewCommit(len(lc.Signatures), 0)", "takes 1 arguments"),
    ("_ = eng.WarmKeyCache(vs)", "_ = eng.WarmKeyCache(*vs)", "WarmKeyCache"),
])
def test_snippet_mutation_is_caught(header, old, new, expect):
    errs = check(header, md=mutate(MD, old, new))
    assert errs and any(expect in e for e in errs), errs


def test_cgo_preamble_paths():
    """The binding's #cgo -I / -L directories resolve from ${SRCDIR} to include/ (holding the header it
    includes) and to the library's build directory."""
    go_dir = os.path.dirname(gc.GO_FILE)
    assert gc.check_preamble(GO, go_dir) == []
    bad = GO.replace("-I${SRCDIR}/../../../include", "-I${SRCDIR}/../../include")
    assert any("tmed25519.h" in e or "does not exist" in e for e in gc.check_preamble(bad, go_dir))


@pytest.mark.parametrize("old,new,expect", [
    ("c.Height, c.Round, &bid, c.Flags", "c.Height, c.Round, bid, c.Flags", "argument 4 of method Engine.VoteSignBytes"),
    ("res, err := b.Verify()", "res, err := b.Verify(1)", "takes 0 arguments"),
    ("vs.Powers[i] = 10", "vs.Power[i] = 10", "no field or method Power"),
])
def test_go_test_file_mutation_is_caught(header, old, new, expect):
    """The binding's Go tests (tmedgpu_test.go, what a maintainer runs on a GPU box) are checked
    with the package's own declarations."""
    errs = check(header, gotest=mutate(GOTEST, old, new))
    assert errs and any(expect in e for e in errs), errs
