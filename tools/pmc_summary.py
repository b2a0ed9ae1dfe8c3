#!/usr/bin/env python3
"""Per-kernel average of every PMC counter in rocprofv3 counter-collection CSVs.
Usage: pmc_summary.py DIR_OR_CSV... -> JSON {kernel: {counter: mean per dispatch, "dispatches": n}}"""
import collections
import csv
import glob
import json
import os
import sys


def files(args):
    for a in args:
        if os.path.isdir(a):
            yield from glob.glob(os.path.join(a, "**", "*counter_collection.csv"), recursive=True)
        else:
            yield a


def short(name):
    for k in ("verify_main_kernel", "verify_prep_kernel", "verify_finish_kernel", "verify_keyset_main_kernel",
              "verify_keyset_prep_kernel", "sign_kernel", "sha256", "merkle"):
        if k in name:
            return k + (name[name.index("<"):name.index(">") + 1] if "<" in name and k == "verify_main_kernel" else "")
    return None


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files(sys.argv[1:]):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["dispatches"] = max(len(v) for v in cs.values())
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
