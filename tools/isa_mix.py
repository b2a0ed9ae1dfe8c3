#!/usr/bin/env python3
"""Instruction mix of one kernel in a gfx950 .s file (from `make isa`): totals per mnemonic,
and per basic block so the hot loops can be read off.  Usage: isa_mix.py FILE.s KERNEL_SUBSTR"""
import collections
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^[_A-Za-z0-9]+:\s*(;.*)?$", l) and name in l and not l.startswith(".L"):
            start = i
            break
    if start is None:
        sys.exit("kernel not found")
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    tot = collections.Counter()
    blocks = []
    cur = ("entry", collections.Counter())
    for l in body:
        s = l.strip()
        if s.startswith(".LBB"):
            blocks.append(cur)
            cur = (s.split(":")[0], collections.Counter())
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        tot[op] += 1
        cur[1][op] += 1
    blocks.append(cur)
    print("total instructions", sum(tot.values()))
    for op, c in tot.most_common(40):
        print("%6d %s" % (c, op))
    print("\nblocks (size >= 200):")
    for lab, c in blocks:
        n = sum(c.values())
        if n >= 200:
            top = ", ".join("%s %d" % kv for kv in c.most_common(8))
            print("%s  %d : %s" % (lab, n, top))


if __name__ == "__main__":
    main()
