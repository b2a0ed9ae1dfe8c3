#!/usr/bin/env python3
"""Record OpenSSL 3's answers on the golden ed25519 vectors as DATA (TEST INFRASTRUCTURE ONLY).

SURVEY.md §8c: OpenSSL (EVP_PKEY_ED25519, EVP_DigestVerify) is an independent implementation,
not the reference; where it disagrees with the Go 1.18 rule (non-canonical A, small-order
points, ...) the disagreement is recorded, never used as a gate.  Writes
tests/golden/ed25519_openssl_answers.json: per vector class, how many vectors OpenSSL decides
like the oracle, and every disagreeing vector (index, class, oracle bit, OpenSSL bit).

Usage: python3 oracle/gen_openssl_answers.py   (needs libcrypto.so.3)
"""
import collections
import ctypes
import ctypes.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def openssl():
    lc = ctypes.CDLL(ctypes.util.find_library("crypto") or "libcrypto.so.3")
    P = ctypes.c_void_p
    lc.EVP_PKEY_new_raw_public_key.restype = P
    lc.EVP_PKEY_new_raw_public_key.argtypes = [ctypes.c_int, P, P, ctypes.c_size_t]
    lc.EVP_MD_CTX_new.restype = P
    lc.EVP_MD_CTX_free.argtypes = [P]
    lc.EVP_PKEY_free.argtypes = [P]
    lc.EVP_DigestVerifyInit.argtypes = [P, P, P, P, P]
    lc.EVP_DigestVerify.argtypes = [P, P, ctypes.c_size_t, P, ctypes.c_size_t]
    lc.OpenSSL_version.restype = ctypes.c_char_p
    lc.OpenSSL_version.argtypes = [ctypes.c_int]
    return lc


def ossl_verify(lc, pub, msg, sig):
    k = lc.EVP_PKEY_new_raw_public_key(1087, None, pub, 32)  # EVP_PKEY_ED25519
    if not k:
        return False
    c = lc.EVP_MD_CTX_new()
    lc.EVP_DigestVerifyInit(c, None, None, None, k)
    r = lc.EVP_DigestVerify(c, sig, len(sig), msg, len(msg))
    lc.EVP_MD_CTX_free(c)
    lc.EVP_PKEY_free(k)
    return r == 1


def answers(vectors, lc):
    per = collections.OrderedDict()
    diff = []
    for i, v in enumerate(vectors):
        pub, msg, sig = (bytes.fromhex(v[k]) for k in ("pub", "msg", "sig"))
        o = ossl_verify(lc, pub, msg, sig)
        c = per.setdefault(v["class"], {"n": 0, "agree": 0})
        c["n"] += 1
        if o == v["valid"]:
            c["agree"] += 1
        else:
            diff.append({"index": i, "class": v["class"], "oracle_go118": v["valid"], "openssl": o})
    return per, diff


def main():
    with open(os.path.join(ROOT, "tests", "golden", "ed25519_vectors.json")) as f:
        vectors = json.load(f)["vectors"]
    lc = openssl()
    per, diff = answers(vectors, lc)
    out = {
        "what": "OpenSSL EVP_DigestVerify(ED25519) answers on tests/golden/ed25519_vectors.json, recorded as "
                "data (SURVEY.md §8c): an independent implementation, NOT the reference's semantics",
        "generator": "oracle/gen_openssl_answers.py",
        "openssl": lc.OpenSSL_version(0).decode(),
        "vectors": len(vectors),
        "agree": sum(c["agree"] for c in per.values()),
        "per_class": per,
        "disagreements": diff,
    }
    path = os.path.join(ROOT, "tests", "golden", "ed25519_openssl_answers.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("%s: %d/%d agree, %d disagreements" % (out["openssl"], out["agree"], len(vectors), len(diff)))


if __name__ == "__main__":
    sys.exit(main())
