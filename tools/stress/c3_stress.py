"""Diagnostic (round 5): the C3-many-sets workload (tests/test_gpu_configs.py
test_c3_many_sets_through_the_cache[40-2050-70000]) through the GENERIC pipelined seam many times on
one cache-off context, for each batch size in TMED_PIPE_SIGS-like steps, counting outcome
mismatches against the oracle loops.  For every mismatch it prints the request, whether its
Trusting/Light pair was split across two planning parts (16 parts per batch) and what a repeat of
that request alone returns.  Usage: [C3_JITTER_US=us] [TMED_HOST_THREADS=k] python tools/stress/c3_stress.py [calls_per_size] [sizes...] [cache]"""
import ctypes
import os
import sys
import time

os.environ.setdefault("TMED_DEBUG_ZERO", "1")  # commit.hip debug_record_zeros

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from c3_flake import workload  # noqa: E402
from conftest import engine_with_env  # noqa: E402
from test_gpu_configs import CHAIN, _ocommit, _same  # noqa: E402
from oracle import port  # noqa: E402
import tmed.types as T  # noqa: E402
from tmed._native import lib  # noqa: E402


class ZeroRec(ctypes.Structure):  # commit.hip ZeroRec
    _fields_ = [("req", ctypes.c_uint64), ("sig", ctypes.c_int32), ("pos", ctypes.c_uint32),
                ("msg_len", ctypes.c_uint32), ("batch_m", ctypes.c_uint32),
                ("key_host", ctypes.c_uint8 * 32), ("sig_host", ctypes.c_uint8 * 64),
                ("key_dev", ctypes.c_uint8 * 32), ("sig_dev", ctypes.c_uint8 * 64), ("msg", ctypes.c_uint8 * 256)]


def zero_records():
    f = lib().tmed_debug_zero_bits
    f.restype = ctypes.c_int
    buf = (ZeroRec * 4096)()
    n = ctypes.c_size_t(0)
    size = f(buf, 4096, ctypes.byref(n))
    assert size == ctypes.sizeof(ZeroRec), (size, ctypes.sizeof(ZeroRec))
    return list(buf[:n.value])


def check_zeros(reqs, recs, ocache):
    """The zero bits whose signature is valid for the expected key and sign-bytes: each with what
    was wrong on its way to the device (host staging, the copy, the assembly) or nothing."""
    out = []
    for z in recs:
        q, i = int(z.req), int(z.sig)
        light = reqs[q | 1]
        pc = light[5]
        oc = ocache.setdefault(q | 1, _ocommit(pc))
        msg = oc.vote_sign_bytes(CHAIN, i)
        key = light[1].validators[i].pub_key
        sig = pc.sigs[i, :int(pc.sig_lens[i])].tobytes()
        if not port.verify(key, msg, sig):
            continue  # a bad signature of the workload: the zero is right
        kh, sh, kd, sd = bytes(z.key_host), bytes(z.sig_host), bytes(z.key_dev), bytes(z.sig_dev)
        m = bytes(z.msg)[:z.msg_len]
        out.append(dict(req=q, sig=i, pos=z.pos, batch_m=z.batch_m, key_host_ok=kh == key, sig_host_ok=sh == sig,
                        key_copy_ok=kd == kh, sig_copy_ok=sd == sh, msg_ok=m == msg, msg_len=z.msg_len,
                        want_len=len(msg), staged_verifies=port.verify(kd, m, sd)))
    return out


def split_points(n, bsz, parts=16):
    """Request indexes that start a planning part (seam_plan: part t = [m t / 16, m (t+1) / 16) of
    each batch of bsz requests)."""
    pts = set()
    for lo in range(0, n, bsz):
        m = min(bsz, n - lo)
        for t in range(1, parts):
            pts.add(lo + m * t // parts)
        pts.add(lo)
    return pts


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    cache = "cache" in sys.argv[2:]  # the key-set cache on: the first call generic, then keyed (lane 0 / 1)
    sizes = [int(x) for x in sys.argv[2:] if x != "cache"] or [70000, 40000]
    if os.environ.get("C3_JITTER_US"):  # host-pool jitter (tmed_test_pool_jitter) for the whole run
        lib().tmed_test_pool_jitter(int(os.environ["C3_JITTER_US"]))
    base = engine_with_env()
    reqs, exp = workload(base)
    base.close()
    n = len(reqs)
    sigs = 40 * n  # nv = 40 signatures per commit
    total = 0
    ocache = {}
    zero_rep = []
    for size in sizes:
        os.environ["TMED_PIPE_SIGS"] = str(size)
        bsz = max(16, size // max(1, sigs // n))
        pts = split_points(n, bsz)
        e = engine_with_env(TMED_KEYCACHE=1 if cache else 0)
        if cache:
            e.keycache_config(True, 16 << 30)
        t0 = time.perf_counter()
        bad_calls = 0
        for call in range(calls):
            got = T.verify_commits(e, reqs)
            if cache:
                e.keycache_wait()
            bad = [q for q in range(n) if not _same(got[q], exp[q])]
            zs = check_zeros(reqs, zero_records(), ocache)
            if zs:
                zero_rep += zs
                print("size %d call %d: false zero bits %s" % (size, call, zs), flush=True)
            if bad:
                bad_calls += 1
                total += len(bad)
                for q in bad[:4]:
                    pair_split = (q + 1) in pts if reqs[q][0] == T.MODE_LIGHT_TRUSTING else q in pts
                    lo = q - (q % 2)
                    alone = T.verify_commits(e, reqs[lo:lo + 2])
                    print("size %d call %d: request %d got %r want %r; pair split across parts: %s; "
                          "pair alone: %s" % (size, call, q, str(got[q])[:40], str(exp[q])[:40], pair_split,
                                              [_same(alone[k], exp[lo + k]) for k in range(2)]), flush=True)
            if call % 50 == 49:
                print("size %d: %d calls, %d with mismatches, %.1f s" % (size, call + 1, bad_calls,
                      time.perf_counter() - t0), flush=True)
        e.close()
    print("total mismatches", total, "false zero bits", len(zero_rep), flush=True)
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
