#!/usr/bin/env python3
"""Per-batch device timeline of a blocksync (C4) run from a rocprofv3 kernel + memory-copy trace:
for every keyed batch (assemble_votes_kernel ... verify_finish_kernel) the kernel durations, the idle
gaps on the kernel stream and the copies overlapping it.  Usage: c4_timeline.py <prof dir> [run]"""
import csv
import os
import sys
from collections import defaultdict

d = sys.argv[1]
run = sys.argv[2] if len(sys.argv) > 2 else "run"
K = list(csv.DictReader(open(os.path.join(d, run + "_kernel_trace.csv"))))
M = list(csv.DictReader(open(os.path.join(d, run + "_memory_copy_trace.csv"))))


def short(n):
    n = n.split("(")[0].replace("tmed::", "").replace("void ", "")
    return n.split("<")[0] if "keyset_main" not in n else "keyset_main"


ks = sorted(((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), short(k["Kernel_Name"])) for k in K))
ms = sorted(((int(m["Start_Timestamp"]), int(m["End_Timestamp"]), m["Direction"].replace("MEMORY_COPY_", "")) for m in M))
# batches: from an assemble_votes_kernel to the next verify_finish_kernel
batches, cur = [], None
for s, e, n in ks:
    if n == "assemble_votes_kernel":
        cur = [(s, e, n)]
    elif cur is not None:
        cur.append((s, e, n))
        if n == "verify_finish_kernel":
            batches.append(cur)
            cur = None
print("batches:", len(batches))
tot = defaultdict(float)
rows = []
for b in batches:
    t0, t1 = b[0][0], b[-1][1]
    busy = sum(e - s for s, e, _ in b)
    per = defaultdict(float)
    for s, e, n in b:
        per[n] += (e - s) / 1e3
    cps = [(s, e, dr) for s, e, dr in ms if e > t0 and s < t1]
    rows.append((t0, (t1 - t0) / 1e3, busy / 1e3, per, cps))
for i, (t0, span, busy, per, cps) in enumerate(rows):
    gap_prev = (t0 - (rows[i - 1][0] + rows[i - 1][1] * 1e3)) / 1e3 if i else 0.0
    print("batch %2d span %7.1f us busy %7.1f us idle-before %7.1f us | %s | copies overlapping: %s" % (
        i, span, busy, gap_prev, " ".join("%s=%.0f" % (k.replace("_kernel", ""), v) for k, v in per.items()),
        ", ".join("%s %.0fus" % (dr, (e - s) / 1e3) for s, e, dr in cps)))
    for k, v in per.items():
        tot[k] += v
n = max(1, len(rows))
print("mean per batch:", {k: round(v / n, 1) for k, v in tot.items()}, "span %.1f us busy %.1f us" % (
    sum(r[1] for r in rows) / n, sum(r[2] for r in rows) / n))
# the whole timed part: first batch start -> last batch end, device kernel-stream occupancy
if rows:
    a, z = rows[0][0], rows[-1][0] + rows[-1][1] * 1e3
    print("timeline %.2f ms, kernel-busy %.2f ms (%.0f%%)" % ((z - a) / 1e6, sum(r[2] for r in rows) / 1e3,
                                                             100 * sum(r[2] for r in rows) * 1e3 / (z - a)))
    for dr in ("HOST_TO_DEVICE", "DEVICE_TO_HOST"):
        c = [(s, e) for s, e, x in ms if x == dr and s >= a and e <= z]
        print("  %s copies: %d, %.2f ms total, mean %.0f us, max %.0f us" % (
            dr, len(c), sum(e - s for s, e in c) / 1e6, sum(e - s for s, e in c) / max(1, len(c)) / 1e3,
            max([(e - s) for s, e in c] or [0]) / 1e3))
